// sts_scan.hpp -- wave-wide searches of global memory for the nearest valid (non-NaN)
// step, used by the imputation kernels (sts_tile.hip, sts_seg.hip) when a NaN run is longer
// than what the kernel holds on chip, and the linear-fill chain threshold.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace sts {

// Wave-wide search of global memory for the last valid index < from (-1: none): 512 steps
// per iteration, eight coalesced loads in flight per lane.
__device__ inline int64_t scan_back(const double* src, int64_t from, int lane) {
    for (int64_t base = from - 512;; base -= 512) {
        double v[8];
#pragma unroll
        for (int j = 0; j < 8; j++) {
            const int64_t t = base + 64 * j + lane;
            v[j] = (t >= 0 && t < from) ? src[t] : __builtin_nan("");
        }
#pragma unroll
        for (int j = 7; j >= 0; j--) {
            const unsigned long long m = __ballot(!__builtin_isnan(v[j]));
            if (m) return base + 64 * j + 63 - __clzll(m);
        }
        if (base <= 0) return -1;
    }
}

// Wave-wide search for the first valid index >= from (T: none), 512 steps per iteration.
__device__ inline int64_t scan_fwd(const double* src, int64_t from, int64_t T, int lane) {
    for (int64_t base = from;; base += 512) {
        if (base >= T) return T;
        double v[8];
#pragma unroll
        for (int j = 0; j < 8; j++) {
            const int64_t t = base + 64 * j + lane;
            v[j] = (t < T) ? src[t] : __builtin_nan("");
        }
#pragma unroll
        for (int j = 0; j < 8; j++) {
            const unsigned long long m = __ballot(!__builtin_isnan(v[j]));
            if (m) return base + 64 * j + __ffsll(m) - 1;
        }
    }
}

// Linear fill: a NaN step more than kLongRun past its last valid index L is produced by the
// chain pass (one lane per run) instead of replaying t - L additions itself.
constexpr int kLongRun = 32;

}  // namespace sts
