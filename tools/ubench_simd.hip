// Which SIMD does each wave of an 8-wave (512-thread) workgroup run on?  The role-split tile
// kernel (sts_tile.hip, STS_TILE_RS) gives waves 0-3 the fill and waves 4-7 the MFMA work and
// assumes one of each per SIMD.  This records HW_ID (SIMD id, CU id) per wave for 512-thread
// workgroups with the role-split kernel's LDS (two workgroups per CU), and prints how the MFMA
// waves of each workgroup spread over the four SIMDs.
//   hipcc --offload-arch=gfx950 -O2 tools/ubench_simd.hip -o /tmp/ubench_simd && /tmp/ubench_simd
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

__global__ __launch_bounds__(512, 2) void where(unsigned* out, int lds_bytes) {
    extern __shared__ double pad[];
    unsigned hw;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    const int wave = threadIdx.x >> 6;
    // hold the CU long enough that the dispatcher co-schedules workgroups
    double acc = threadIdx.x;
    for (int i = 0; i < 20000; i++) acc = acc * 1.0000001 + 1e-9;
    pad[threadIdx.x % (lds_bytes / 8)] = acc;
    __syncthreads();
    if ((threadIdx.x & 63) == 0) out[blockIdx.x * 8 + wave] = hw ^ (pad[(threadIdx.x + 64) % (lds_bytes / 8)] > 1e300 ? 1u : 0u);
}

int main() {
    const int nb = 4096, lds = 79176;
    unsigned* d;
    if (hipMalloc(&d, nb * 8 * sizeof(unsigned)) != hipSuccess) return 1;
    hipFuncSetAttribute((const void*)where, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    hipLaunchKernelGGL(where, dim3(nb), dim3(512), lds, 0, d, lds);
    if (hipDeviceSynchronize() != hipSuccess) return 2;
    std::vector<unsigned> h(nb * 8);
    hipMemcpy(h.data(), d, h.size() * sizeof(unsigned), hipMemcpyDeviceToHost);
    // gfx9 HW_ID: wave_id [3:0], simd_id [5:4], pipe [7:6], cu_id [11:8], sh_id [12], se_id [15:13]
    int pattern_count[256] = {0};
    int mfma_distinct[5] = {0};
    for (int b = 0; b < nb; b++) {
        unsigned pat = 0;
        int used = 0;
        for (int w = 0; w < 8; w++) {
            const unsigned simd = (h[b * 8 + w] >> 4) & 3;
            if (w < 4) pat |= simd << (2 * w);
            if (w >= 4) used |= 1 << simd;
        }
        pattern_count[pat & 255]++;
        mfma_distinct[__builtin_popcount(used)]++;
    }
    printf("{\"blocks\": %d, \"mfma_waves_distinct_simds\": [%d, %d, %d, %d, %d], \"first_blocks\": [", nb, mfma_distinct[0],
           mfma_distinct[1], mfma_distinct[2], mfma_distinct[3], mfma_distinct[4]);
    for (int b = 0; b < 4; b++) {
        printf("%s[", b ? ", " : "");
        for (int w = 0; w < 8; w++) printf("%s%u", w ? ", " : "", (h[b * 8 + w] >> 4) & 3);
        printf("]");
    }
    printf("]}\n");
    hipFree(d);
    return 0;
}
