// Microbenchmarks that size the design of the fp64 ACF kernel on MI355X:
//   * HBM streaming: read+write copy and read-only reduction (double2 per lane)
//   * FP64 VALU FMA throughput (v_fma_f64)
//   * FP64 MFMA throughput (v_mfma_f64_16x16x4_f64)
//   * both pipes at once (half the waves VALU, half MFMA)
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/ubench_fp64 tools/ubench_fp64.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
  fprintf(stderr, "HIP %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); exit(1);} } while (0)

typedef double d4 __attribute__((ext_vector_type(4)));

__global__ void copy_k(const double2* __restrict__ in, double2* __restrict__ out, size_t n2) {
  size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  size_t stride = (size_t)gridDim.x * blockDim.x;
  for (; i < n2; i += stride) out[i] = in[i];
}

__global__ void read_k(const double2* __restrict__ in, double* __restrict__ out, size_t n2) {
  size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  size_t stride = (size_t)gridDim.x * blockDim.x;
  double s = 0;
  for (; i < n2; i += stride) { double2 v = in[i]; s += v.x + v.y; }
  if (s == 1234.5) out[0] = s;
}

template <int CHAINS>
__global__ void valu_k(double* out, int iters, double a) {
  double acc[CHAINS];
#pragma unroll
  for (int c = 0; c < CHAINS; c++) acc[c] = threadIdx.x * 1e-3 + c;
  for (int it = 0; it < iters; it++) {
#pragma unroll
    for (int c = 0; c < CHAINS; c++) acc[c] = __builtin_fma(acc[c], a, 1e-9);
  }
  double s = 0;
#pragma unroll
  for (int c = 0; c < CHAINS; c++) s += acc[c];
  if (s == 1234.5) out[0] = s;
}

template <int ACC>
__global__ void mfma_k(double* out, int iters) {
  d4 acc[ACC];
#pragma unroll
  for (int c = 0; c < ACC; c++) acc[c] = d4{0, 0, 0, 0};
  double a = threadIdx.x * 1e-3, b = 1.0 - threadIdx.x * 1e-4;
  for (int it = 0; it < iters; it++) {
#pragma unroll
    for (int c = 0; c < ACC; c++) acc[c] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[c], 0, 0, 0);
  }
  double s = 0;
#pragma unroll
  for (int c = 0; c < ACC; c++) s += acc[c][0] + acc[c][1] + acc[c][2] + acc[c][3];
  if (s == 1234.5) out[0] = s;
}

// waves with (wave id & 1) == 0 do MFMA, others VALU
__global__ void mixed_k(double* out, int iters_m, int iters_v, double a) {
  int wave = threadIdx.x >> 6;
  double s = 0;
  if (wave & 1) {
    double acc[8];
#pragma unroll
    for (int c = 0; c < 8; c++) acc[c] = threadIdx.x * 1e-3 + c;
    for (int it = 0; it < iters_v; it++) {
#pragma unroll
      for (int c = 0; c < 8; c++) acc[c] = __builtin_fma(acc[c], a, 1e-9);
    }
#pragma unroll
    for (int c = 0; c < 8; c++) s += acc[c];
  } else {
    d4 acc[4];
#pragma unroll
    for (int c = 0; c < 4; c++) acc[c] = d4{0, 0, 0, 0};
    double x = threadIdx.x * 1e-3, y = 1.0 - threadIdx.x * 1e-4;
    for (int it = 0; it < iters_m; it++) {
#pragma unroll
      for (int c = 0; c < 4; c++) acc[c] = __builtin_amdgcn_mfma_f64_16x16x4f64(x, y, acc[c], 0, 0, 0);
    }
#pragma unroll
    for (int c = 0; c < 4; c++) s += acc[c][0] + acc[c][1] + acc[c][2] + acc[c][3];
  }
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
  size_t bytes = (size_t)4 << 30;  // 4 GiB per buffer
  double2 *in, *out; double* o;
  CK(hipMalloc(&in, bytes)); CK(hipMalloc(&out, bytes)); CK(hipMalloc(&o, 64));
  CK(hipMemset(in, 0, bytes));
  size_t n2 = bytes / 16;
  for (int grid : {2048, 4096, 8192, 16384}) {
    float ms = time_ms([&] { copy_k<<<grid, 256>>>(in, out, n2); }, 10);
    printf("{\"test\":\"copy\",\"grid\":%d,\"GBps\":%.1f}\n", grid, 2.0 * bytes / ms / 1e6);
    ms = time_ms([&] { read_k<<<grid, 256>>>(in, o, n2); }, 10);
    printf("{\"test\":\"read\",\"grid\":%d,\"GBps\":%.1f}\n", grid, 1.0 * bytes / ms / 1e6);
  }
  int iters = 4096;
  int grid = cus * 8;  // 8 WGs of 256 per CU = 32 waves/CU
  {
    float ms = time_ms([&] { valu_k<8><<<grid, 256>>>(o, iters, 0.999); }, 5);
    double flops = 2.0 * 8 * iters * (double)grid * 256;
    printf("{\"test\":\"valu_fma_f64\",\"TFps\":%.2f}\n", flops / ms / 1e9);
  }
  {
    float ms = time_ms([&] { mfma_k<4><<<grid, 256>>>(o, iters / 4); }, 5);
    double flops = 2.0 * 16 * 16 * 4 * 4 * (iters / 4) * (double)grid * 4;  // per wave
    printf("{\"test\":\"mfma_f64_16x16x4\",\"TFps\":%.2f,\"cycles_per_mfma_per_simd_at_2.4GHz\":%.1f}\n",
           flops / ms / 1e9, (ms * 1e-3 * 2.4e9) / ((double)4 * (iters / 4) * grid * 4 / (cus * 4)));
  }
  for (int ratio : {1, 2, 4, 8}) {
    int im = iters / 4, iv = iters * ratio / 4;
    float msm = time_ms([&] { mfma_k<4><<<grid, 256>>>(o, im); }, 3);
    float msv = time_ms([&] { valu_k<8><<<grid, 256>>>(o, iv, 0.999); }, 3);
    float ms = time_ms([&] { mixed_k<<<grid, 256>>>(o, im, iv, 0.999); }, 3);
    // mixed: half waves each, so alone each would take half the time of the full-grid kernels
    printf("{\"test\":\"mixed\",\"ratio\":%d,\"mfma_alone_half_ms\":%.3f,\"valu_alone_half_ms\":%.3f,"
           "\"mixed_ms\":%.3f}\n", ratio, msm / 2, msv / 2, ms);
  }
  return 0;
}
