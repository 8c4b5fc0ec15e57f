// Exhaustive-style check of stats_fast_kernel's division (sts_instants.hip) against the
// library f64 division: q(delta, n) over ~4e9 random (delta, n) pairs, delta with random
// mantissas and exponents across [2^-900, 2^700] (the fast range) and n in [1, 2^24] plus
// n near 2^k and 3 * 2^k.  Prints the number of pairs whose bits differ (must be 0).
//   hipcc -O3 --offload-arch=gfx950 -ffp-contract=off tools/ubench_div.hip -o tools/ubench_div
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

__device__ __forceinline__ uint64_t mix(uint64_t x) {   // splitmix64
    x += 0x9e3779b97f4a7c15ull;
    x = (x ^ (x >> 30)) * 0xbf58476d1ce4e5b9ull;
    x = (x ^ (x >> 27)) * 0x94d049bb133111ebull;
    return x ^ (x >> 31);
}

__device__ __forceinline__ double newton_rcp(double b) {
    double y = __builtin_amdgcn_rcp(b);
    double e = __builtin_fma(-b, y, 1.0);
    y = __builtin_fma(y, e, y);
    e = __builtin_fma(-b, y, 1.0);
    return __builtin_fma(y, e, y);
}

__global__ void check(uint64_t seed, int iters, unsigned long long* bad, unsigned long long* first) {
    const uint64_t id = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    unsigned long long nbad = 0;
    for (int it = 0; it < iters; it++) {
        const uint64_t r1 = mix(seed ^ (id * 0x100000001b3ull + it));
        const uint64_t r2 = mix(r1);
        // delta: random sign and mantissa, exponent uniform over [-900, 700]
        const int e = -900 + (int)(r2 % 1601);
        const uint64_t bits = (r1 & 0x800fffffffffffffull) | ((uint64_t)(e + 1023) << 52);
        const double delta = __builtin_bit_cast(double, bits);
        uint64_t nn;
        switch ((r2 >> 20) & 3) {
        case 0: nn = 1 + ((r2 >> 24) & 0xffffff); break;          // [1, 2^24]
        case 1: nn = 1 + ((r2 >> 24) & 0x3ff); break;             // small n
        case 2: nn = (1ull << ((r2 >> 24) % 40)) + ((int)((r2 >> 40) % 5) - 2); break;   // near 2^k
        default: nn = 3ull * (1ull << ((r2 >> 24) % 38)) + ((int)((r2 >> 40) % 3) - 1); break;
        }
        if (nn == 0) nn = 1;
        const double n = (double)nn;
        const double y = newton_rcp(n), nb = -n;
        const double q0 = delta * y;
        const double rr = __builtin_fma(nb, q0, delta);
        const double q = __builtin_fma(rr, y, q0);
        const double ref = delta / n;
        if (__builtin_bit_cast(uint64_t, q) != __builtin_bit_cast(uint64_t, ref)) {
            if (nbad == 0 && atomicAdd(first + 2, 1ull) == 0) {
                first[0] = bits;
                first[1] = nn;
            }
            nbad++;
        }
    }
    if (nbad) atomicAdd(bad, nbad);
}

int main() {
    unsigned long long *bad, *first;
    hipMalloc(&bad, 8);
    hipMalloc(&first, 24);
    hipMemset(bad, 0, 8);
    hipMemset(first, 0, 24);
    const int blocks = 65536, threads = 256, iters = 256;
    for (int rep = 0; rep < 1; rep++) hipLaunchKernelGGL(check, dim3(blocks), dim3(threads), 0, 0, 12345ull + rep, iters, bad, first);
    unsigned long long h = 0, f[3] = {0, 0, 0};
    if (hipMemcpy(&h, bad, 8, hipMemcpyDeviceToHost) != hipSuccess) return 2;
    hipMemcpy(f, first, 24, hipMemcpyDeviceToHost);
    printf("{\"pairs\": %llu, \"mismatches\": %llu, \"first_delta_bits\": \"0x%016llx\", \"first_n\": %llu}\n",
           (unsigned long long)blocks * threads * iters, h, f[0], f[1]);
    return h ? 1 : 0;
}
