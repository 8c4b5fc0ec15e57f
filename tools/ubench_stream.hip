// Streaming microbenchmarks that bound the fused fill + ACF tile kernel on MI355X:
//   * copy variants: per-thread unroll depth, contiguous per-workgroup spans (the tile
//     kernel's access shape), plain vs non-temporal loads / stores
//   * copy + FP64 MFMA: the same copy with M v_mfma_f64_16x16x4 per 64 copied doubles
//     (M = 5 is the ACF K = 60 load) -> the attainable ceiling of a fused stream + MFMA
//   * v_mfma_f64_4x4x4 (4-block) throughput, to price the alternative ACF decomposition
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/ubench_stream tools/ubench_stream.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
  fprintf(stderr, "HIP %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); exit(1);} } while (0)

typedef double d4 __attribute__((ext_vector_type(4)));

// Each workgroup owns SPAN contiguous double2; U double2 per thread in flight.
template <int U, bool NTL, bool NTS>
__global__ __launch_bounds__(256) void copy_span(const double2* __restrict__ in, double2* __restrict__ out,
                                                 size_t span) {
  const double2* src = in + blockIdx.x * span;
  double2* dst = out + blockIdx.x * span;
  for (size_t base = 0; base < span; base += 256 * U) {
    double2 r[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
      const double2* p = src + base + u * 256 + threadIdx.x;
      if (NTL) { r[u].x = __builtin_nontemporal_load(&p->x); r[u].y = __builtin_nontemporal_load(&p->y); }
      else r[u] = *p;
    }
#pragma unroll
    for (int u = 0; u < U; u++) {
      double2* p = dst + base + u * 256 + threadIdx.x;
      if (NTS) { __builtin_nontemporal_store(r[u].x, &p->x); __builtin_nontemporal_store(r[u].y, &p->y); }
      else *p = r[u];
    }
  }
}

// copy + M MFMAs per 64 doubles (per wave: per 32 double2 lanes... i.e. per wave-instruction
// pair of 64 double2 = 128 doubles -> 2*M MFMAs).  The MFMA operands depend on the data.
template <int U, int M>
__global__ __launch_bounds__(256) void copy_mfma(const double2* __restrict__ in, double2* __restrict__ out,
                                                 size_t span, double* sink) {
  const double2* src = in + blockIdx.x * span;
  double2* dst = out + blockIdx.x * span;
  d4 acc[M > 0 ? M : 1];
#pragma unroll
  for (int m = 0; m < (M > 0 ? M : 1); m++) acc[m] = d4{0, 0, 0, 0};
  for (size_t base = 0; base < span; base += 256 * U) {
    double2 r[U];
#pragma unroll
    for (int u = 0; u < U; u++) r[u] = src[base + u * 256 + threadIdx.x];
#pragma unroll
    for (int u = 0; u < U; u++) dst[base + u * 256 + threadIdx.x] = r[u];
#pragma unroll
    for (int u = 0; u < U; u++) {
#pragma unroll
      for (int m = 0; m < M; m++) {
        acc[m] = __builtin_amdgcn_mfma_f64_16x16x4f64(r[u].x, r[u].y, acc[m], 0, 0, 0);
        acc[m] = __builtin_amdgcn_mfma_f64_16x16x4f64(r[u].y, r[u].x, acc[m], 0, 0, 0);
      }
    }
  }
  double s = 0;
#pragma unroll
  for (int m = 0; m < (M > 0 ? M : 1); m++) s += acc[m][0] + acc[m][1] + acc[m][2] + acc[m][3];
  if (s == 1234.5) sink[0] = s;
}

template <int ACC>
__global__ void mfma4_k(double* out, int iters) {
  double acc[ACC];
#pragma unroll
  for (int c = 0; c < ACC; c++) acc[c] = 0;
  double a = threadIdx.x * 1e-3, b = 1.0 - threadIdx.x * 1e-4;
  for (int it = 0; it < iters; it++) {
#pragma unroll
    for (int c = 0; c < ACC; c++) acc[c] = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, acc[c], 0, 0, 0);
  }
  double s = 0;
#pragma unroll
  for (int c = 0; c < ACC; c++) s += acc[c];
  if (s == 1234.5) out[0] = s;
}

template <typename F>
static float time_ms(F f, int reps) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  f();
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(a));
  for (int r = 0; r < reps; r++) f();
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms; CK(hipEventElapsedTime(&ms, a, b));
  return ms / reps;
}

int main() {
  int cus = 0; CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const size_t bytes = (size_t)16 << 30;  // 16 GiB per buffer: far past the 256 MiB Infinity Cache
  double2 *in, *out; double* o;
  CK(hipMalloc(&in, bytes)); CK(hipMalloc(&out, bytes)); CK(hipMalloc(&o, 64));
  CK(hipMemset(in, 0, bytes));
  CK(hipMemset(out, 0, bytes));
  const size_t n2 = bytes / 16;
#define COPY(U, NTL, NTS, SPANK)                                                                           \
  {                                                                                                        \
    const size_t span = (size_t)(SPANK) * 1024 / 16;                                                       \
    const unsigned grid = (unsigned)(n2 / span);                                                           \
    float ms = time_ms([&] { copy_span<U, NTL, NTS><<<grid, 256>>>(in, out, span); }, 5);                   \
    printf("{\"test\":\"copy\",\"U\":%d,\"ntl\":%d,\"nts\":%d,\"span_KB\":%d,\"GBps\":%.1f}\n", U, NTL, NTS, \
           SPANK, 2.0 * grid * span * 16 / ms / 1e6);                                                      \
  }
  COPY(1, false, false, 64)
  COPY(2, false, false, 64)
  COPY(4, false, false, 64)
  COPY(8, false, false, 64)
  COPY(4, false, true, 64)
  COPY(4, true, true, 64)
  COPY(8, false, true, 64)
  COPY(4, false, false, 512)
  COPY(4, false, true, 512)
  COPY(8, false, true, 512)
  COPY(4, false, false, 1024)
#define CM(U, M)                                                                                           \
  {                                                                                                        \
    const size_t span = (size_t)512 * 1024 / 16;                                                           \
    const unsigned grid = (unsigned)(n2 / span);                                                           \
    float ms = time_ms([&] { copy_mfma<U, M><<<grid, 256>>>(in, out, span, o); }, 5);                       \
    double steps = (double)grid * span * 2;                                                                \
    printf("{\"test\":\"copy_mfma\",\"U\":%d,\"mfma_per_64_doubles\":%d,\"GBps\":%.1f,\"Gsteps\":%.1f,"   \
           "\"mfma_TF\":%.1f}\n", U, M, 2.0 * grid * span * 16 / ms / 1e6, steps / ms / 1e6,              \
           steps / 64.0 * M * 2048.0 / ms / 1e9);                                                          \
  }
  CM(4, 0)
  CM(4, 2)
  CM(4, 3)
  CM(4, 4)
  CM(4, 5)
  CM(8, 4)
  CM(8, 5)
  {
    const int iters = 4096, grid = cus * 8;
    float ms = time_ms([&] { mfma4_k<8><<<grid, 256>>>(o, iters); }, 5);
    double macs = 4.0 * 4 * 4 * 16 * 8.0 * iters * grid * 4;   // 16 blocks of 4x4x4 per instruction
    printf("{\"test\":\"mfma_f64_4x4x4\",\"TFps_if_16_blocks\":%.2f,\"cycles_per_instr_at_2.4GHz\":%.1f}\n",
           2 * macs / ms / 1e9, (ms * 1e-3 * 2.4e9) / ((double)8 * iters * grid * 4 / (cus * 4)));
  }
  return 0;
}
