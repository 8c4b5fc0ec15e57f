// Can the C3 shard's two loads -- the HBM stream of the fill (read + write every step) and the
// FP64 MFMA work of the lag products -- overlap on MI355X when they come from DIFFERENT waves?
// Kernel A is a float4-style copy (16 B per lane per access, in + out, no compute); kernel B
// runs v_mfma_f64_16x16x4_f64 chains on register operands (4 independent accumulators per wave,
// no memory).  Each is timed alone and both together on two streams (launched back to back,
// timed from the first event to the last).  Together ~= max(A, B): the hardware overlaps them
// and the C3 gap is the tile kernel's own coupling of the two inside its waves; together ~= A + B:
// the two compete for the same issue resources and more waves per SIMD cannot hide the MFMAs.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/ubench_overlap tools/ubench_overlap.hip
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

typedef double d4 __attribute__((ext_vector_type(4)));
typedef double d2 __attribute__((ext_vector_type(2)));

__global__ __launch_bounds__(256) void copy_k(const d2* __restrict__ in, d2* __restrict__ out, long n) {
    const long i = (long)blockIdx.x * 256 + threadIdx.x;
    if (i < n) __builtin_nontemporal_store(in[i], out + i);
}

__global__ __launch_bounds__(256) void mfma_k(double* out, int iters) {
    d4 acc0 = {0, 0, 0, 0}, acc1 = acc0, acc2 = acc0, acc3 = acc0;
    const double a = 1.0 + threadIdx.x * 1e-9, b = 1.0 - threadIdx.x * 1e-9;
    for (int it = 0; it < iters; it++) {
        acc0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc0, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f64_16x16x4f64(b, a, acc1, 0, 0, 0);
        acc2 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, a, acc2, 0, 0, 0);
        acc3 = __builtin_amdgcn_mfma_f64_16x16x4f64(b, b, acc3, 0, 0, 0);
    }
    const d4 s = acc0 + acc1 + acc2 + acc3;
    out[(long)blockIdx.x * 256 + threadIdx.x] = s[0] + s[1] + s[2] + s[3];
}

int main(int argc, char** argv) {
    const long bytes = (argc > 1 ? atol(argv[1]) : 8L) << 30;   // per buffer (in, out)
    const int copies = argc > 2 ? atoi(argv[2]) : 4;            // copy passes per launch set
    const int iters = argc > 3 ? atoi(argv[3]) : 4096;          // MFMA groups of 4 per wave
    const int blocksB = argc > 4 ? atoi(argv[4]) : 256 * 8;     // MFMA workgroups (4 waves each)
    const long n = bytes / 16;
    d2 *in, *out;
    double* sink;
    CK(hipMalloc(&in, bytes));
    CK(hipMalloc(&out, bytes));
    CK(hipMalloc(&sink, sizeof(double) * 256L * blocksB));
    CK(hipMemset(in, 0, bytes));
    hipStream_t sa, sb;
    CK(hipStreamCreateWithFlags(&sa, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&sb, hipStreamNonBlocking));
    hipEvent_t e0, ea, eb;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&ea));
    CK(hipEventCreate(&eb));
    const unsigned gridA = (unsigned)((n + 255) / 256);
    auto runA = [&](hipStream_t s) {
        for (int c = 0; c < copies; c++) hipLaunchKernelGGL(copy_k, dim3(gridA), dim3(256), 0, s, in, out, n);
    };
    auto runB = [&](hipStream_t s) { hipLaunchKernelGGL(mfma_k, dim3(blocksB), dim3(256), 0, s, sink, iters); };
    // warm-up
    runA(sa);
    runB(sb);
    CK(hipDeviceSynchronize());
    float tA = 0, tB = 0, tAB = 0, tA2 = 0, tB2 = 0;
    for (int rep = 0; rep < 3; rep++) {
        CK(hipEventRecord(e0, sa));
        runA(sa);
        CK(hipEventRecord(ea, sa));
        CK(hipEventSynchronize(ea));
        CK(hipEventElapsedTime(&tA, e0, ea));
        CK(hipEventRecord(e0, sb));
        runB(sb);
        CK(hipEventRecord(eb, sb));
        CK(hipEventSynchronize(eb));
        CK(hipEventElapsedTime(&tB, e0, eb));
        // together: B first (its waves resident), then A's stream
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(e0, sb));
        CK(hipStreamWaitEvent(sa, e0, 0));
        runB(sb);
        runA(sa);
        CK(hipEventRecord(ea, sa));
        CK(hipEventRecord(eb, sb));
        CK(hipEventSynchronize(ea));
        CK(hipEventSynchronize(eb));
        CK(hipEventElapsedTime(&tA2, e0, ea));
        CK(hipEventElapsedTime(&tB2, e0, eb));
        tAB = tA2 > tB2 ? tA2 : tB2;
        const double gb = 2.0 * bytes * copies / 1e9;
        const double mf = 4.0 * iters * 4.0 * blocksB * 1024.0 * 2.0 / 1e12;   // TFLOP (4 waves per WG)
        printf("{\"rep\": %d, \"copy_ms\": %.3f, \"copy_TBps\": %.3f, \"mfma_ms\": %.3f, \"mfma_TFps\": %.2f, "
               "\"together_ms\": %.3f, \"copy_end_ms\": %.3f, \"mfma_end_ms\": %.3f, \"sum_ms\": %.3f, \"max_ms\": %.3f}\n",
               rep, tA, gb / tA, tB, mf / (tB / 1e3), tAB, tA2, tB2, tA + tB, tA > tB ? tA : tB);
        fflush(stdout);
    }
    return 0;
}
