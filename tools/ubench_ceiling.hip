// HBM ceilings on MI355X for the shapes the hot path moves (round 3):
//   copy4   : the guide's float4 copy (MI355X_MICROARCH.md: 6.29 TB/s) -- one 16-B load and one
//             16-B store per thread, one thread per float4, no grid stride
//   copy4x4 : the same with 4 float4 per thread (4 loads in flight before the stores)
//   rd4     : read-only stream (float4 per thread, sum kept live)
//   wr4     : write-only stream
//   r1w11   : the C5 mix -- 8 B read and 88 B written per element (fill + 10 lag columns),
//             every access 16 B per lane
// Buffers hold random data (DVFS: all-zero inputs clock differently, MI355X_MICROARCH.md) and
// are sized 4 GiB and 16 GiB per buffer, far past the 256 MiB Infinity Cache.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/ubench_ceiling tools/ubench_ceiling.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
  fprintf(stderr, "HIP %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); exit(1);} } while (0)

__global__ __launch_bounds__(256) void fill_rand(float4* p, size_t n) {
  size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  const size_t st = (size_t)gridDim.x * 256;
  for (; i < n; i += st) {
    unsigned h = (unsigned)i * 2654435761u ^ 0x9e3779b9u;
    h ^= h >> 15; h *= 0x2c1b3c6du; h ^= h >> 12;
    p[i] = make_float4((float)(h & 0xffff), (float)(h >> 16), (float)(h & 0xff), (float)(h >> 24));
  }
}

template <int U>
__global__ __launch_bounds__(256) void copy4(const float4* __restrict__ in, float4* __restrict__ out) {
  const size_t b = (size_t)blockIdx.x * 256 * U + threadIdx.x;
  float4 r[U];
#pragma unroll
  for (int u = 0; u < U; u++) r[u] = in[b + u * 256];
#pragma unroll
  for (int u = 0; u < U; u++) out[b + u * 256] = r[u];
}

__global__ __launch_bounds__(256) void rd4(const float4* __restrict__ in, float* sink) {
  const size_t b = (size_t)blockIdx.x * 1024 + threadIdx.x;
  float4 r[4];
#pragma unroll
  for (int u = 0; u < 4; u++) r[u] = in[b + u * 256];
  float s = 0.f;
#pragma unroll
  for (int u = 0; u < 4; u++) s += r[u].x + r[u].y + r[u].z + r[u].w;
  if (s == 1234.5f) sink[0] = s;   // keeps the loads live
}

__global__ __launch_bounds__(256) void wr4(float4* __restrict__ out) {
  const size_t b = (size_t)blockIdx.x * 1024 + threadIdx.x;
  const float4 v = make_float4(1.f, 2.f, 3.f, (float)threadIdx.x);
#pragma unroll
  for (int u = 0; u < 4; u++) out[b + u * 256] = v;
}

// C5 mix: a block reads 256 x 16 B and writes 11 x 256 x 16 B (the filled copy + 10 columns)
__global__ __launch_bounds__(256) void r1w11(const float4* __restrict__ in, float4* __restrict__ out, size_t n) {
  const size_t b = (size_t)blockIdx.x * 256 + threadIdx.x;
  const float4 v = in[b];
#pragma unroll
  for (int c = 0; c < 11; c++) out[(size_t)c * n + b] = v;
}

template <class F>
float time_ms(F f, int reps) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  f(); f();
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(a));
  for (int i = 0; i < reps; i++) f();
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms = 0.f;
  CK(hipEventElapsedTime(&ms, a, b));
  return ms / reps;
}

int main() {
  float4 *in, *out; float* sink;
  const size_t big = (size_t)16 << 30;
  CK(hipMalloc(&in, big)); CK(hipMalloc(&out, (size_t)44 << 30)); CK(hipMalloc(&sink, 64));
  fill_rand<<<4096, 256>>>(in, big / 16);
  fill_rand<<<4096, 256>>>(out, ((size_t)44 << 30) / 16);
  CK(hipDeviceSynchronize());
  for (size_t gib : {4, 16}) {
    const size_t bytes = gib << 30, n = bytes / 16;
    float ms = time_ms([&] { copy4<1><<<(unsigned)(n / 256), 256>>>(in, out); }, 5);
    printf("{\"test\":\"copy4\",\"GiB\":%zu,\"GBps\":%.1f}\n", gib, 2.0 * bytes / ms / 1e6);
    ms = time_ms([&] { copy4<4><<<(unsigned)(n / 1024), 256>>>(in, out); }, 5);
    printf("{\"test\":\"copy4x4\",\"GiB\":%zu,\"GBps\":%.1f}\n", gib, 2.0 * bytes / ms / 1e6);
    ms = time_ms([&] { rd4<<<(unsigned)(n / 1024), 256>>>(in, sink); }, 5);
    printf("{\"test\":\"rd4\",\"GiB\":%zu,\"GBps\":%.1f}\n", gib, 1.0 * bytes / ms / 1e6);
    ms = time_ms([&] { wr4<<<(unsigned)(n / 1024), 256>>>(out); }, 5);
    printf("{\"test\":\"wr4\",\"GiB\":%zu,\"GBps\":%.1f}\n", gib, 1.0 * bytes / ms / 1e6);
    const size_t n5 = n / 4;   // 12 x (bytes / 4) moved: in 1/4 of the buffer, out 11/4 of it
    ms = time_ms([&] { r1w11<<<(unsigned)(n5 / 256), 256>>>(in, out, n5); }, 5);
    printf("{\"test\":\"r1w11\",\"GiB\":%zu,\"GBps\":%.1f}\n", gib, 12.0 * n5 * 16 / ms / 1e6);
    fflush(stdout);
  }
  return 0;
}
