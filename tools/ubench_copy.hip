// Read+write streaming ceiling on MI355X: which copy shape gets closest to HBM peak?
// The fused fill + ACF tile kernel moves 8 B in + 8 B out per step, so its ceiling is a
// 1:1 read:write copy, not a read-only stream.  Variants:
//   gs  : grid-stride, every wave-instruction 1 KiB contiguous (double2 per lane), U per
//         thread in flight, G workgroups per CU
//   span: each workgroup owns one contiguous span (the tile kernel's shape), U in flight
//   nt  : non-temporal stores (and loads)
//   rd / wr: read-only and write-only for reference
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/ubench_copy tools/ubench_copy.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
  fprintf(stderr, "HIP %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); exit(1);} } while (0)

template <int U, bool NT>
__global__ __launch_bounds__(256) void copy_gs(const double2* __restrict__ in, double2* __restrict__ out, size_t n2) {
  const size_t stride = (size_t)gridDim.x * 256 * U;
  for (size_t base = (size_t)blockIdx.x * 256 * U; base < n2; base += stride) {
    double2 r[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
      const double2* p = in + base + u * 256 + threadIdx.x;
      if (NT) { r[u].x = __builtin_nontemporal_load(&p->x); r[u].y = __builtin_nontemporal_load(&p->y); }
      else r[u] = *p;
    }
#pragma unroll
    for (int u = 0; u < U; u++) {
      double2* p = out + base + u * 256 + threadIdx.x;
      if (NT) { __builtin_nontemporal_store(r[u].x, &p->x); __builtin_nontemporal_store(r[u].y, &p->y); }
      else *p = r[u];
    }
  }
}

// span copy, software pipelined: loads of block i+1 in flight while block i is stored
template <int U, bool NT>
__global__ __launch_bounds__(256) void copy_span_pipe(const double2* __restrict__ in, double2* __restrict__ out,
                                                      size_t span) {
  const double2* src = in + blockIdx.x * span;
  double2* dst = out + blockIdx.x * span;
  double2 r[U];
#pragma unroll
  for (int u = 0; u < U; u++) r[u] = src[u * 256 + threadIdx.x];
  for (size_t base = 0; base < span; base += 256 * U) {
    double2 n[U];
    const size_t nb = base + 256 * U < span ? base + 256 * U : base;
#pragma unroll
    for (int u = 0; u < U; u++) n[u] = src[nb + u * 256 + threadIdx.x];
#pragma unroll
    for (int u = 0; u < U; u++) {
      double2* p = dst + base + u * 256 + threadIdx.x;
      if (NT) { __builtin_nontemporal_store(r[u].x, &p->x); __builtin_nontemporal_store(r[u].y, &p->y); }
      else *p = r[u];
    }
#pragma unroll
    for (int u = 0; u < U; u++) r[u] = n[u];
  }
}

template <int U>
__global__ __launch_bounds__(256) void read_gs(const double2* __restrict__ in, size_t n2, double* sink) {
  const size_t stride = (size_t)gridDim.x * 256 * U;
  double s = 0;
  for (size_t base = (size_t)blockIdx.x * 256 * U; base < n2; base += stride) {
#pragma unroll
    for (int u = 0; u < U; u++) { double2 v = in[base + u * 256 + threadIdx.x]; s += v.x + v.y; }
  }
  if (s == 1234.5) sink[0] = s;
}

template <int U>
__global__ __launch_bounds__(256) void write_gs(double2* __restrict__ out, size_t n2) {
  const size_t stride = (size_t)gridDim.x * 256 * U;
  for (size_t base = (size_t)blockIdx.x * 256 * U; base < n2; base += stride) {
#pragma unroll
    for (int u = 0; u < U; u++) out[base + u * 256 + threadIdx.x] = make_double2(1.0, 2.0);
  }
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
  const size_t bytes = (size_t)16 << 30;   // 16 GiB per buffer, far past the 256 MiB Infinity Cache
  double2 *in, *out; double* o;
  CK(hipMalloc(&in, bytes)); CK(hipMalloc(&out, bytes)); CK(hipMalloc(&o, 64));
  CK(hipMemset(in, 0, bytes));
  CK(hipMemset(out, 0, bytes));
  const size_t n2 = bytes / 16;
#define GS(U, NT, G)                                                                               \
  {                                                                                                \
    const unsigned grid = cus * (G);                                                               \
    float ms = time_ms([&] { copy_gs<U, NT><<<grid, 256>>>(in, out, n2); }, 4);                    \
    printf("{\"test\":\"copy_gs\",\"U\":%d,\"nt\":%d,\"wg_per_cu\":%d,\"GBps\":%.1f}\n", U, NT, G, \
           2.0 * bytes / ms / 1e6);                                                                \
    fflush(stdout);                                                                                \
  }
  GS(1, false, 4) GS(1, false, 8) GS(1, false, 16) GS(1, false, 32)
  GS(2, false, 4) GS(2, false, 8) GS(2, false, 16)
  GS(4, false, 2) GS(4, false, 4) GS(4, false, 8)
  GS(8, false, 2) GS(8, false, 4)
  GS(2, true, 8) GS(4, true, 4) GS(4, true, 8)
#define SP(U, NT, SPANK)                                                                           \
  {                                                                                                \
    const size_t span = (size_t)(SPANK) * 1024 / 16;                                               \
    const unsigned grid = (unsigned)(n2 / span);                                                   \
    float ms = time_ms([&] { copy_span_pipe<U, NT><<<grid, 256>>>(in, out, span); }, 4);           \
    printf("{\"test\":\"copy_span_pipe\",\"U\":%d,\"nt\":%d,\"span_KB\":%d,\"GBps\":%.1f}\n", U, NT, \
           SPANK, 2.0 * grid * span * 16 / ms / 1e6);                                              \
    fflush(stdout);                                                                                \
  }
  SP(2, false, 512) SP(4, false, 512) SP(8, false, 512) SP(4, true, 512) SP(8, true, 512)
  SP(4, false, 64) SP(8, false, 2048)
#define RD(U, G)                                                                                   \
  {                                                                                                \
    const unsigned grid = cus * (G);                                                               \
    float ms = time_ms([&] { read_gs<U><<<grid, 256>>>(in, n2, o); }, 4);                          \
    printf("{\"test\":\"read_gs\",\"U\":%d,\"wg_per_cu\":%d,\"GBps\":%.1f}\n", U, G, bytes / ms / 1e6); \
    fflush(stdout);                                                                                \
  }
  RD(2, 8) RD(4, 8) RD(4, 4)
#define WR(U, G)                                                                                   \
  {                                                                                                \
    const unsigned grid = cus * (G);                                                               \
    float ms = time_ms([&] { write_gs<U><<<grid, 256>>>(out, n2); }, 4);                           \
    printf("{\"test\":\"write_gs\",\"U\":%d,\"wg_per_cu\":%d,\"GBps\":%.1f}\n", U, G, bytes / ms / 1e6); \
    fflush(stdout);                                                                                \
  }
  WR(2, 8) WR(4, 8) WR(4, 4)
  return 0;
}
