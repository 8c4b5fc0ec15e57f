// Dependent-chain latency of FP64 VALU ops on MI355X (gfx950): the floor of every sequential
// recurrence the reference's bit-exact order imposes (rule 3's two-pass ACF loop, the GARCH /
// EWMA fit passes).  One wave per SIMD (grid = 1 workgroup of 64 threads, or `waves` one-wave
// workgroups), a chain of CH independent accumulators per lane, ITERS dependent steps each;
// s_memtime around the loop (100 MHz) -> cycles at the shader clock reported by the caller.
// Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -o tools/ubench_latency tools/ubench_latency.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                                  \
    do {                                                                                       \
        hipError_t e = (x);                                                                    \
        if (e != hipSuccess) {                                                                 \
            fprintf(stderr, "HIP %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__);    \
            exit(1);                                                                           \
        }                                                                                      \
    } while (0)

// OP 0: x = x + y (v_add_f64); 1: x = x * y (v_mul_f64); 2: x = u + b * x (mul then add, the
// GARCH / EWMA affine step); 3: x = fma(x, a, b)
template <int OP, int CH>
__global__ void chain_k(double* out, long long* clk, int iters, double y) {
    double x[CH];
#pragma unroll
    for (int c = 0; c < CH; c++) x[c] = threadIdx.x * 1e-6 + c;
    const long long t0 = wall_clock64();
    const long long c0 = clock64();
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int c = 0; c < CH; c++) {
            if (OP == 0) x[c] = x[c] + y;
            if (OP == 1) x[c] = x[c] * y;
            if (OP == 2) x[c] = 1e-3 + y * x[c];
            if (OP == 3) x[c] = __builtin_fma(x[c], y, 1e-3);
        }
    }
    const long long c1 = clock64();
    const long long t1 = wall_clock64();
    double s = 0;
#pragma unroll
    for (int c = 0; c < CH; c++) s += x[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    if (threadIdx.x == 0) {
        clk[2 * blockIdx.x] = c1 - c0;
        clk[2 * blockIdx.x + 1] = t1 - t0;
    }
}

template <int OP, int CH>
void run(const char* name, int waves, int iters) {
    double* out;
    long long* clk;
    CK(hipMalloc(&out, sizeof(double) * 64 * waves));
    CK(hipMalloc(&clk, sizeof(long long) * 2 * waves));
    hipLaunchKernelGGL((chain_k<OP, CH>), dim3(waves), dim3(64), 0, 0, out, clk, iters / 10, 0.999999);
    CK(hipDeviceSynchronize());
    hipLaunchKernelGGL((chain_k<OP, CH>), dim3(waves), dim3(64), 0, 0, out, clk, iters, 0.999999);
    CK(hipDeviceSynchronize());
    long long h[2];
    CK(hipMemcpy(h, clk, sizeof h, hipMemcpyDeviceToHost));
    // clock64 = s_memtime (shader clock on gfx9); wall_clock64 = 100 MHz constant clock
    const double steps = (double)iters;
    printf("{\"test\": \"%s\", \"chains_per_lane\": %d, \"waves\": %d, \"cycles_per_step\": %.2f, "
           "\"ns_per_step\": %.3f, \"clock_ghz\": %.3f}\n",
           name, CH, waves, (double)h[0] / steps, (double)h[1] * 10.0 / steps, (double)h[0] / ((double)h[1] * 10.0));
    CK(hipFree(out));
    CK(hipFree(clk));
}

int main() {
    const int it = 1 << 20;
    run<0, 1>("add_f64", 1, it);
    run<0, 2>("add_f64", 1, it);
    run<0, 4>("add_f64", 1, it);
    run<0, 8>("add_f64", 1, it);
    run<1, 1>("mul_f64", 1, it);
    run<2, 1>("mul_add_f64", 1, it);
    run<2, 4>("mul_add_f64", 1, it);
    run<3, 1>("fma_f64", 1, it);
    run<3, 8>("fma_f64", 1, it);
    return 0;
}
