// Issue-overlap microbenchmark: does FP64 MFMA overlap with integer VALU, FP64 VALU,
// SALU or LDS work issued by OTHER waves of the same SIMD?  (Sizes the fused fill + ACF
// kernels: how much non-MFMA work hides under the lag-product MFMAs.)
//   even waves: a chain of v_mfma_f64_16x16x4 on 2 accumulators
//   odd waves : int VALU / FP64 VALU / SALU / ds_read_b64 work of a chosen length
// time(mixed) vs time(each alone) -> overlap fraction.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/ubench_issue tools/ubench_issue.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
  fprintf(stderr, "HIP %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); exit(1);} } while (0)

typedef double d4 __attribute__((ext_vector_type(4)));

enum { kNone = 0, kMfma = 1, kIntValu = 2, kF64Valu = 3, kSalu = 4, kLds = 5 };

__device__ __forceinline__ void do_mfma(int iters, double* out) {
  d4 a0 = {0, 0, 0, 0}, a1 = {0, 0, 0, 0};
  double x = threadIdx.x * 1e-3, y = 1.0 - threadIdx.x * 1e-4;
  for (int it = 0; it < iters; it++) {
    a0 = __builtin_amdgcn_mfma_f64_16x16x4f64(x, y, a0, 0, 0, 0);
    a1 = __builtin_amdgcn_mfma_f64_16x16x4f64(y, x, a1, 0, 0, 0);
  }
  double s = a0[0] + a0[1] + a0[2] + a0[3] + a1[0] + a1[1] + a1[2] + a1[3];
  if (s == 1234.5) out[0] = s;
}

__device__ __forceinline__ void do_int(int iters, double* out) {
  unsigned v[8];
#pragma unroll
  for (int c = 0; c < 8; c++) v[c] = threadIdx.x + c;
  for (int it = 0; it < iters; it++) {
#pragma unroll
    for (int c = 0; c < 8; c++) v[c] = (v[c] ^ (v[c] << 3)) + 0x9e3779b9u;   // 3 VALU
  }
  unsigned s = 0;
#pragma unroll
  for (int c = 0; c < 8; c++) s += v[c];
  if (s == 12345u) out[0] = s;
}

__device__ __forceinline__ void do_f64(int iters, double* out) {
  double v[8];
#pragma unroll
  for (int c = 0; c < 8; c++) v[c] = threadIdx.x * 1e-3 + c;
  for (int it = 0; it < iters; it++) {
#pragma unroll
    for (int c = 0; c < 8; c++) v[c] = v[c] * 0.999 + 1e-9;   // 1 FP64 FMA-free pair (contract off) = 2 VALU
  }
  double s = 0;
#pragma unroll
  for (int c = 0; c < 8; c++) s += v[c];
  if (s == 1234.5) out[0] = s;
}

__device__ __forceinline__ void do_salu(int iters, double* out) {
  unsigned v = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), w = v + 7;
  for (int it = 0; it < iters; it++) {
    asm volatile("s_xor_b32 %0, %0, %1\n s_add_u32 %1, %1, %0\n s_lshl_b32 %0, %0, 1\n s_add_u32 %0, %0, %1\n"
                 "s_xor_b32 %0, %0, %1\n s_add_u32 %1, %1, %0\n s_lshl_b32 %0, %0, 1\n s_add_u32 %0, %0, %1\n"
                 : "+s"(v), "+s"(w));
  }
  if (v == 12345u) out[0] = v;
}

__device__ __forceinline__ void do_lds(int iters, double* out, double* sh) {
  const int lane = threadIdx.x & 63;
  double acc = 0;
  for (int it = 0; it < iters; it++) {
    const double* p = sh + ((it * 64 + lane) & 2047);
#pragma unroll
    for (int c = 0; c < 8; c++) acc += p[c * 64 & 2047];
  }
  if (acc == 1234.5) out[0] = acc;
}

__global__ __launch_bounds__(256) void mixed(int even_kind, int even_iters, int odd_kind, int odd_iters, double* out) {
  __shared__ double sh[2048];
  for (int i = threadIdx.x; i < 2048; i += 256) sh[i] = i * 1e-3;
  __syncthreads();
  const int wave = threadIdx.x >> 6;
  const int kind = (wave & 1) ? odd_kind : even_kind;
  const int iters = (wave & 1) ? odd_iters : even_iters;
  switch (kind) {
    case kMfma: do_mfma(iters, out); break;
    case kIntValu: do_int(iters, out); break;
    case kF64Valu: do_f64(iters, out); break;
    case kSalu: do_salu(iters, out); break;
    case kLds: do_lds(iters, out, sh); break;
    default: break;
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
  double* o; CK(hipMalloc(&o, 64));
  const int grid = cus * 4;   // 4 WGs x 4 waves per CU = 4 waves per SIMD (2 MFMA + 2 other)
  const int mi = 2000;
  const char* names[] = {"none", "mfma", "int_valu", "f64_valu", "salu", "lds_b64"};
  const int iters[] = {0, mi, 2000, 2000, 2000, 500};
  for (int k = 2; k <= 5; k++) {
    for (int scale : {1, 4}) {
      const int oi = iters[k] * scale;
      float tm = time_ms([&] { mixed<<<grid, 256>>>(kMfma, mi, kNone, 0, o); }, 3);
      float tk = time_ms([&] { mixed<<<grid, 256>>>(kNone, 0, k, oi, o); }, 3);
      float tb = time_ms([&] { mixed<<<grid, 256>>>(kMfma, mi, k, oi, o); }, 3);
      printf("{\"other\":\"%s\",\"other_iters\":%d,\"mfma_alone_ms\":%.3f,\"other_alone_ms\":%.3f,\"both_ms\":%.3f,"
             "\"overlap\":%.2f}\n", names[k], oi, tm, tk, tb, (tm + tk - tb) / (tm < tk ? tm : tk));
    }
  }
  return 0;
}
