// sts_gen.hip -- synthetic NaN-riddled panels generated in HBM.
// Counter-based Philox4x32-10 keyed by (seed), counter = (t, s): any element of any
// shard is reproducible on the CPU (oracle/sts_oracle.c, orc_gen_*) bit for bit, so
// parity tests and the multi-GPU bench never ship panels around.
//   x[s,t] = ((100 + 10*u_s) + t/T) + (u_{s,t} - 0.5),  NaN with probability p
//   AR(p) panels: phi = base * (1 + 0.1*(u_s - 0.5)), c = 1, innovations u_{s,t} - 0.5,
//   built with ARModel.addTimeDependentEffects (S/models/Autoregression.scala:75-88).
#include "sts_internal.hpp"

#include <hip/hip_runtime.h>

namespace sts {
namespace {

__device__ __forceinline__ void philox(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t k0,
                                       uint32_t k1, uint32_t out[4]) {
#pragma unroll
    for (int r = 0; r < 10; r++) {
        const uint64_t p0 = (uint64_t)0xD2511F53u * c0;
        const uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
        const uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
        const uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
        const uint32_t n0 = hi1 ^ c1 ^ k0;
        const uint32_t n2 = hi0 ^ c3 ^ k1;
        c0 = n0;
        c1 = lo1;
        c2 = n2;
        c3 = lo0;
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
    out[0] = c0;
    out[1] = c1;
    out[2] = c2;
    out[3] = c3;
}

__device__ __forceinline__ double u53(uint32_t a, uint32_t b) {
    const uint64_t m = ((uint64_t)(a >> 5) << 26) | (uint64_t)(b >> 6);
    return (double)m * 0x1p-53;
}

__device__ __forceinline__ void words(uint64_t seed, int64_t s, uint64_t t, uint32_t w[4]) {
    philox((uint32_t)t, (uint32_t)(t >> 32), (uint32_t)(uint64_t)s, (uint32_t)((uint64_t)s >> 32),
           (uint32_t)seed, (uint32_t)(seed >> 32), w);
}

__device__ __forceinline__ double series_u(uint64_t seed, int64_t s) {
    uint32_t w[4];
    words(seed, s, ~(uint64_t)0, w);
    return u53(w[0], w[1]);
}

// mode 0: full panel value with NaN mask; mode 1: AR innovations u - 0.5
template <int MODE>
__global__ __launch_bounds__(256) void gen_kernel(double* out, int64_t s0, int64_t S, int64_t T, int64_t ld,
                                                  uint64_t seed, uint32_t thr) {
    const int64_t s = blockIdx.y + (int64_t)blockIdx.z * 65535;
    if (s >= S) return;
    const int64_t sg = s0 + s;
    __shared__ double us_sh;
    if (MODE == 0) {
        if (threadIdx.x == 0) us_sh = series_u(seed, sg);
        __syncthreads();
    }
    const double us = (MODE == 0) ? us_sh : 0.0;
    const double base = 100.0 + 10.0 * us;
    for (int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x; t < T; t += (int64_t)gridDim.x * 256) {
        uint32_t w[4];
        words(seed, sg, (uint64_t)t, w);
        const double u = u53(w[0], w[1]);
        double v;
        if (MODE == 0) {
            v = (base + (double)t / (double)T) + (u - 0.5);
            if (w[2] < thr) v = __builtin_nan("");
        } else {
            v = u - 0.5;
        }
        out[s * ld + t] = v;
    }
}

__global__ __launch_bounds__(256) void gen_ar_params_kernel(double* c, double* phi, int64_t s0, int64_t S,
                                                            uint64_t seed, int p) {
    const int64_t s = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (s >= S) return;
    const double base[8] = {0.3, -0.2, 0.1, 0.05, -0.05, 0.02, -0.02, 0.01};
    const double scale = 1.0 + 0.1 * (series_u(seed, s0 + s) - 0.5);
    c[s] = 1.0;
    for (int j = 0; j < p; j++) phi[s * p + j] = base[j & 7] * scale;
}

dim3 gen_grid(int64_t S, int64_t T) {
    unsigned gx = (unsigned)((T + 255) / 256);
    if (gx > 64) gx = 64;
    const unsigned gy = (unsigned)(S < 65535 ? S : 65535);
    const unsigned gz = (unsigned)((S + 65534) / 65535);
    return dim3(gx, gy, gz);
}

}  // namespace

hipError_t launch_gen_panel(double* out, int64_t s0, int64_t S, int64_t T, int64_t ld, uint64_t seed,
                            uint32_t thr, hipStream_t st) {
    if (S <= 0 || T <= 0) return hipSuccess;
    hipLaunchKernelGGL((gen_kernel<0>), gen_grid(S, T), dim3(256), 0, st, out, s0, S, T, ld, seed, thr);
    return hipGetLastError();
}

hipError_t launch_gen_ar(double* out, double* c, double* phi, int64_t s0, int64_t S, int64_t T, int64_t ld,
                         uint64_t seed, int p, hipStream_t st) {
    if (S <= 0 || T <= 0) return hipSuccess;
    hipLaunchKernelGGL((gen_kernel<1>), gen_grid(S, T), dim3(256), 0, st, out, s0, S, T, ld, seed, 0u);
    hipLaunchKernelGGL(gen_ar_params_kernel, dim3((unsigned)((S + 255) / 256)), dim3(256), 0, st, c, phi, s0, S,
                       seed, p);
    RecurArgs a{};
    a.in = out;
    a.out = out;
    a.S = S;
    a.T = T;
    a.ld_in = ld;
    a.ld_out = ld;
    a.c = c;
    a.coef = phi;
    a.p = p;
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    return launch_recur(kArAdd, a, st);
}

}  // namespace sts
