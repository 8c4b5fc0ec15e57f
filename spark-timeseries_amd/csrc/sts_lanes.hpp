// sts_lanes.hpp -- cross-lane moves of doubles without the LDS crossbar, for the kernels whose
// reductions / broadcasts sit on dependency chains (sts_ar.hip, sts_seg.hip), and the XCD remap.
#pragma once
#include <hip/hip_runtime.h>

namespace sts {

// ds_bpermute (what __shfl / __shfl_xor compile to) costs an LDS round trip (~100+ cycles);
// DPP covers the in-row steps and the one-lane shift, v_readlane broadcasts from a known lane.
// Every lane is written: bound_ctrl makes a lane whose source is out of range (wave_shr's lane
// 0, row_shl past the row end) read 0, so no old value -- and no v_mov to zero it first (round 6:
// one VALU per DPP move; the C1 short kernel's ~350 such moves per series)
template <int CTRL>
__device__ __forceinline__ double dpp_d(double v) {
    const unsigned long long u = __builtin_bit_cast(unsigned long long, v);
    const int lo = __builtin_amdgcn_mov_dpp((int)(unsigned)u, CTRL, 0xf, 0xf, true);
    const int hi = __builtin_amdgcn_mov_dpp((int)(unsigned)(u >> 32), CTRL, 0xf, 0xf, true);
    return __builtin_bit_cast(double, ((unsigned long long)(unsigned)hi << 32) | (unsigned)lo);
}
__device__ __forceinline__ double lane_bcast(double v, int l) {
    const unsigned long long u = __builtin_bit_cast(unsigned long long, v);
    const unsigned lo = __builtin_amdgcn_readlane((unsigned)u, l);
    const unsigned hi = __builtin_amdgcn_readlane((unsigned)(u >> 32), l);
    return __builtin_bit_cast(double, ((unsigned long long)hi << 32) | lo);
}
// sum over the wave, the same bits in every lane: quad butterfly (quad_perm [1,0,3,2],
// [2,3,0,1]), row rotations by 4 and 8 (every lane then holds its row's sum), then the four
// row sums from lanes 0 / 16 / 32 / 48 in a fixed order
__device__ __forceinline__ double wave_sum_dpp(double v) {
    v = v + dpp_d<0xB1>(v);
    v = v + dpp_d<0x4E>(v);
    v = v + dpp_d<0x124>(v);
    v = v + dpp_d<0x128>(v);
    return (lane_bcast(v, 0) + lane_bcast(v, 16)) + (lane_bcast(v, 32) + lane_bcast(v, 48));
}
// sum over the lane's row of 16, the same bits in every lane of the row (wave_sum_dpp's first steps)
__device__ __forceinline__ double row_sum_dpp(double v) {
    v = v + dpp_d<0xB1>(v);
    v = v + dpp_d<0x4E>(v);
    v = v + dpp_d<0x124>(v);
    return v + dpp_d<0x128>(v);
}
// sum over the wave into lane 63 only, no SGPRs: row_sum_dpp, then DPP row_bcast:15 (rows 1 / 3
// add lane 15 / 47) and row_bcast:31 (rows 2 / 3 add lane 31): lane 63 = (r2 + r3) + (r0 + r1),
// wave_sum_dpp's bits (a + b = b + a exactly)
template <int CTRL, int ROWS>
__device__ __forceinline__ double dpp_rows_d(double v) {
    const unsigned long long u = __builtin_bit_cast(unsigned long long, v);
    const int lo = __builtin_amdgcn_update_dpp(0, (int)(unsigned)u, CTRL, ROWS, 0xf, false);
    const int hi = __builtin_amdgcn_update_dpp(0, (int)(unsigned)(u >> 32), CTRL, ROWS, 0xf, false);
    return __builtin_bit_cast(double, ((unsigned long long)(unsigned)hi << 32) | (unsigned)lo);
}
__device__ __forceinline__ double wave_sum_to_63(double v) {
    v = row_sum_dpp(v);
    v = v + dpp_rows_d<0x142, 0xa>(v);
    return v + dpp_rows_d<0x143, 0xc>(v);
}
// lane l - 1's value (wave_shr:1; lane 0 gets 0)
__device__ __forceinline__ double lane_prev(double v) { return dpp_d<0x138>(v); }
// lane l + 1's value (wave_shl:1; lane 63 gets 0)
__device__ __forceinline__ double lane_next(double v) { return dpp_d<0x130>(v); }
// inclusive suffix sum over lanes l .. 63: row_shl 1 / 2 / 4 / 8 inside the rows of 16 (lanes
// past the row end contribute 0), then the totals of the rows above from lanes 16 / 32 / 48
__device__ __forceinline__ double suffix_sum_dpp(double v, int lane) {
    v = v + dpp_d<0x101>(v);
    v = v + dpp_d<0x102>(v);
    v = v + dpp_d<0x104>(v);
    v = v + dpp_d<0x108>(v);
    const double r3 = lane_bcast(v, 48), r2 = lane_bcast(v, 32) + r3, r1 = lane_bcast(v, 16) + r2;
    const int row = lane >> 4;
    return row == 3 ? v : v + (row == 2 ? r3 : row == 1 ? r2 : r1);
}

// Bijective XCD-aware remap of a workgroup id (cdna_hip_programming.md §5 "XCD swizzle must be
// bijective"): workgroups go to the 8 XCDs round-robin (b % 8); this hands XCD x one contiguous
// range of ids, so each XCD streams one contiguous part of the panel (tile kernel: neighbour
// tiles of a series share the L2 that holds their overlapping halos; row kernels: C2 1.17 ->
// 1.07 ms, profiles/r04_v10_ab_c2_shape.jsonl).
__device__ __forceinline__ int64_t xcd_remap(int64_t b, int64_t n) {
    int64_t q = n / 8, r = n % 8, x = b % 8;
    return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + b / 8;
}

}  // namespace sts
