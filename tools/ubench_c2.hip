// Access-pattern ceilings for the C2 shape (1M series x 390 steps, fillPrevious -> diff(1)
// -> EWMA add, one lane per series, bit-exact sequential order):
//   chunkA<SPW, CH, COMPUTE> : the shipped recur_kernel shape -- SPW series x CH-step blocks
//                              through LDS, 16-B loads, next block in flight
//   rowsB<R, PF>             : R whole series per wave (R*T contiguous doubles), loaded in
//                              address order into LDS; lanes < R run the recurrence over the
//                              row; PF = the next block's loads in flight (persistent loop)
//   copy_gs                  : grid-stride 1:1 copy of the same bytes (ceiling)
// Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -o tools/ubench_c2 tools/ubench_c2.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstdint>
#include <vector>
#include <cstring>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
  fprintf(stderr, "HIP %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); exit(1);} } while (0)

__device__ __forceinline__ void step(double x, double& carry, double& hl, double& e, int t, double sm, double oms,
                                     double& y) {
    carry = (x != x) ? carry : x;
    const double f = carry;
    const double d = (t < 1) ? f : f - hl;
    e = (t == 0) ? d : sm * d + oms * e;
    hl = f;
    y = e;
}

template <int SPW, int CH, bool COMPUTE>
__global__ __launch_bounds__(64) void chunkA(const double* in, double* out, int64_t S, int64_t T, double sm) {
    constexpr int kRow = CH + 2;
    constexpr int NLD = SPW * CH / 128;
    __shared__ __attribute__((aligned(16))) double tile[SPW * kRow];
    const int lane = threadIdx.x;
    const int64_t s0 = (int64_t)blockIdx.x * SPW;
    const bool live = lane < SPW && s0 + lane < S;
    const int ns = (S - s0 < SPW) ? (int)(S - s0) : SPW;
    const double oms = 1.0 - sm;
    double carry = __builtin_nan(""), hl = 0.0, e = 0.0;
    double2 pre[NLD];
    auto fetch = [&](int64_t tc) {
        const int len = (T - tc < CH) ? (int)(T - tc) : CH;
#pragma unroll
        for (int i = 0; i < NLD; i++) {
            const int el = (i * 64 + lane) * 2;
            const int row = el / CH, col = el % CH;
            const double* src = in + (s0 + row) * T + tc + col;
            if (row < ns && col + 1 < len) pre[i] = *reinterpret_cast<const double2*>(src);
            else { pre[i].x = (row < ns && col < len) ? src[0] : 0.0; pre[i].y = 0.0; }
        }
    };
    fetch(0);
    for (int64_t tc = 0; tc < T; tc += CH) {
        const int len = (T - tc < CH) ? (int)(T - tc) : CH;
#pragma unroll
        for (int i = 0; i < NLD; i++) {
            const int el = (i * 64 + lane) * 2;
            const int row = el / CH, col = el % CH;
            if (row < ns && col < len) *reinterpret_cast<double2*>(&tile[row * kRow + col]) = pre[i];
        }
        if (tc + CH < T) fetch(tc + CH);
        __syncthreads();
        if (COMPUTE && live) {
            double* myrow = tile + lane * kRow;
            for (int c = 0; c < len; c++) {
                double y;
                step(myrow[c], carry, hl, e, (int)(tc + c), sm, oms, y);
                myrow[c] = y;
            }
        }
        __syncthreads();
#pragma unroll
        for (int i = 0; i < NLD; i++) {
            const int el = (i * 64 + lane) * 2;
            const int row = el / CH, col = el % CH;
            double* d = out + (s0 + row) * T + tc + col;
            if (row < ns && col + 1 < len) *reinterpret_cast<double2*>(d) = *reinterpret_cast<const double2*>(&tile[row * kRow + col]);
            else if (row < ns && col < len) d[0] = tile[row * kRow + col];
        }
        __syncthreads();
    }
}

// R whole rows per block; T <= TM; row stride in LDS TM + 1 (odd: the lanes' column reads
// spread over banks).  Persistent: wave w handles blocks w, w + G, ...
template <int R, int TM, bool PF>
__global__ __launch_bounds__(64) void rowsB(const double* in, double* out, int64_t S, int64_t T, double sm,
                                            int64_t nblk) {
    constexpr int kRow = TM + 1;
    constexpr int NL = (R * TM / 2 + 63) / 64;   // double2 loads per lane per block
    __shared__ double tile[R * kRow];
    const int lane = threadIdx.x;
    const double oms = 1.0 - sm;
    const int n2 = (int)(R * T / 2);              // T even: whole double2 per block
    double2 pre[NL];
    auto fetch = [&](int64_t b) {
        const double2* src = reinterpret_cast<const double2*>(in + b * R * T);
#pragma unroll
        for (int i = 0; i < NL; i++) {
            const int q = i * 64 + lane;
            if (q < n2) pre[i] = src[q];
        }
    };
    int64_t b = blockIdx.x;
    if (b < nblk) fetch(b);
    for (; b < nblk; b += gridDim.x) {
#pragma unroll
        for (int i = 0; i < NL; i++) {
            const int q = i * 64 + lane;
            if (q < n2) {
                const int el = 2 * q, row = el / (int)T, col = el - row * (int)T;
                tile[row * kRow + col] = pre[i].x;
                tile[row * kRow + col + 1] = pre[i].y;
            }
        }
        if (PF && b + gridDim.x < nblk) fetch(b + gridDim.x);
        __syncthreads();
        if (lane < R) {
            double carry = __builtin_nan(""), hl = 0.0, e = 0.0;
            double* myrow = tile + lane * kRow;
            for (int c = 0; c < T; c++) {
                double y;
                step(myrow[c], carry, hl, e, c, sm, oms, y);
                myrow[c] = y;
            }
        }
        __syncthreads();
        double2* dst = reinterpret_cast<double2*>(out + b * R * T);
#pragma unroll
        for (int i = 0; i < NL; i++) {
            const int q = i * 64 + lane;
            if (q < n2) {
                const int el = 2 * q, row = el / (int)T, col = el - row * (int)T;
                dst[q] = make_double2(tile[row * kRow + col], tile[row * kRow + col + 1]);
            }
        }
        if (!PF && b + gridDim.x < nblk) fetch(b + gridDim.x);
        __syncthreads();
    }
}


// R whole rows per wave, NW independent waves per workgroup; rows in LDS at an even stride
// KR (16-B aligned, conflict-free 16-B column reads for 8 lanes); the recurrence reads and
// writes 8 steps at a time from registers, the next 8 prefetched (software pipelined).
template <int R, int KR, int NW, int TT, bool COMPUTE = true>
__global__ __launch_bounds__(64 * NW) void rowsC(const double* in, double* out, int64_t S, int64_t T_, double sm) {
    __shared__ __attribute__((aligned(16))) double tile_all[NW * R * KR];
    constexpr int Ti = TT;
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    double* tile = tile_all + wave * R * KR;
    const int64_t b = (int64_t)blockIdx.x * NW + wave;
    if (b * R >= S) return;
    const double oms = 1.0 - sm;
    constexpr int n2 = R * Ti / 2;
    const double2* src = reinterpret_cast<const double2*>(in + b * R * Ti);
    constexpr int NL = (n2 + 63) / 64;
    double2 pre[NL];
#pragma unroll
    for (int i = 0; i < NL; i++) {
        const int q = i * 64 + lane;
        if (i * 64 + 64 <= n2 || q < n2) pre[i] = src[q];
    }
#pragma unroll
    for (int i = 0; i < NL; i++) {
        const int q = i * 64 + lane;
        if (i * 64 + 64 <= n2 || q < n2) {
            const int el = 2 * q, row = el / Ti, col = el - row * Ti;
            *reinterpret_cast<double2*>(&tile[row * KR + col]) = pre[i];
        }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront", "local");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront", "local");
    if (COMPUTE && lane < R) {
        double carry = __builtin_nan(""), hl = 0.0, e = 0.0;
        double* myrow = tile + lane * KR;
        double2 cur[4], nx[4];
#pragma unroll
        for (int j = 0; j < 4; j++) cur[j] = reinterpret_cast<const double2*>(myrow)[j];
        int c = 0;
        for (; c + 8 <= Ti; c += 8) {
#pragma unroll
            for (int j = 0; j < 4; j++) nx[j] = reinterpret_cast<const double2*>(myrow + c + 8)[j];   // KR >= Ti + 8
            double v[8] = {cur[0].x, cur[0].y, cur[1].x, cur[1].y, cur[2].x, cur[2].y, cur[3].x, cur[3].y};
#pragma unroll
            for (int j = 0; j < 8; j++) {
                double y;
                step(v[j], carry, hl, e, c + j, sm, oms, y);
                v[j] = y;
            }
#pragma unroll
            for (int j = 0; j < 4; j++) reinterpret_cast<double2*>(myrow + c)[j] = make_double2(v[2 * j], v[2 * j + 1]);
#pragma unroll
            for (int j = 0; j < 4; j++) cur[j] = nx[j];
        }
        for (; c < Ti; c++) {
            double y;
            step(myrow[c], carry, hl, e, c, sm, oms, y);
            myrow[c] = y;
        }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront", "local");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront", "local");
    double2* dst = reinterpret_cast<double2*>(out + b * R * Ti);
#pragma unroll
    for (int i = 0; i < NL; i++) {
        const int q = i * 64 + lane;
        if (i * 64 + 64 <= n2 || q < n2) {
            const int el = 2 * q, row = el / Ti, col = el - row * Ti;
            dst[q] = *reinterpret_cast<const double2*>(&tile[row * KR + col]);
        }
    }
}

typedef __attribute__((address_space(3))) void lds_void;
// recurrence over one LDS row (lane < R), 8 steps per batch through registers
template <int TT>
__device__ __forceinline__ void row_recur(double* myrow, double sm, double oms) {
    double carry = __builtin_nan(""), hl = 0.0, e = 0.0;
    static_assert(TT % 2 == 0, "16-B row reads");
    double2 cur[4], nx[4];
#pragma unroll
    for (int j = 0; j < 4; j++) cur[j] = reinterpret_cast<const double2*>(myrow)[j];
    int c = 0;
    for (; c + 16 <= TT; c += 8) {
#pragma unroll
        for (int j = 0; j < 4; j++) nx[j] = reinterpret_cast<const double2*>(myrow + c + 8)[j];
        double v[8] = {cur[0].x, cur[0].y, cur[1].x, cur[1].y, cur[2].x, cur[2].y, cur[3].x, cur[3].y};
#pragma unroll
        for (int j = 0; j < 8; j++) {
            double y;
            step(v[j], carry, hl, e, c + j, sm, oms, y);
            v[j] = y;
        }
#pragma unroll
        for (int j = 0; j < 4; j++) reinterpret_cast<double2*>(myrow + c)[j] = make_double2(v[2 * j], v[2 * j + 1]);
#pragma unroll
        for (int j = 0; j < 4; j++) cur[j] = nx[j];
    }
    for (; c < TT; c++) {
        double y;
        step(myrow[c], carry, hl, e, c, sm, oms, y);
        myrow[c] = y;
    }
}
__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront", "local");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront", "local");
}
// R whole rows per wave straight into LDS by LDS-DMA (global_load_lds_dwordx4: lane-linear,
// so the LDS image is the rows back to back); NW independent waves per workgroup
template <int R, int TT, int NW, bool COMPUTE = true>
__global__ __launch_bounds__(64 * NW) void rowsD(const double* in, double* out, int64_t S, double sm) {
    constexpr int NE = R * TT;                       // doubles per block
    constexpr int NI = (NE + 127) / 128;             // 1-KB DMA instructions
    __shared__ __attribute__((aligned(16))) double tile_all[NW * NI * 128];
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    double* tile = tile_all + wave * NI * 128;
    const int64_t b = (int64_t)blockIdx.x * NW + wave;
    if (b * R >= S) return;
    const double* src = in + b * NE;
#pragma unroll
    for (int i = 0; i < NI; i++) {
        int q = i * 128 + 2 * lane;
        if (q >= NE) q = 0;                          // tail lanes: a valid source, lands in the pad
        __builtin_amdgcn_global_load_lds(src + q, (lds_void*)(tile + i * 128), 16, 0, 0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    wave_lds_sync();
    if (COMPUTE && lane < R) row_recur<TT>(tile + lane * TT, sm, 1.0 - sm);
    wave_lds_sync();
    double2* dst = reinterpret_cast<double2*>(out + b * NE);
#pragma unroll
    for (int i = 0; i < NI; i++) {
        const int q2 = i * 64 + lane;
        if (2 * q2 < NE) dst[q2] = reinterpret_cast<const double2*>(tile)[q2];
    }
}
// persistent, two LDS buffers per wave: the next block's DMA in flight during this block's
// recurrence and stores
template <int R, int TT>
__global__ __launch_bounds__(64) void rowsE(const double* in, double* out, int64_t S, double sm, int64_t nblk) {
    constexpr int NE = R * TT;
    constexpr int NI = (NE + 127) / 128;
    __shared__ __attribute__((aligned(16))) double buf[2 * NI * 128];
    const int lane = threadIdx.x;
    auto issue = [&](int64_t bb, double* dstl) {
        const double* src = in + bb * NE;
#pragma unroll
        for (int i = 0; i < NI; i++) {
            int q = i * 128 + 2 * lane;
            if (q >= NE) q = 0;
            __builtin_amdgcn_global_load_lds(src + q, (lds_void*)(dstl + i * 128), 16, 0, 0);
        }
    };
    int64_t b = blockIdx.x;
    if (b >= nblk) return;
    issue(b, buf);
    int k = 0;
    for (; b < nblk; b += gridDim.x, k ^= 1) {
        double* cur = buf + k * NI * 128;
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        wave_lds_sync();
        if (b + gridDim.x < nblk) issue(b + gridDim.x, buf + (k ^ 1) * NI * 128);
        if (lane < R) row_recur<TT>(cur + lane * TT, sm, 1.0 - sm);
        wave_lds_sync();
        double2* dst = reinterpret_cast<double2*>(out + b * NE);
#pragma unroll
        for (int i = 0; i < NI; i++) {
            const int q2 = i * 64 + lane;
            if (2 * q2 < NE) dst[q2] = reinterpret_cast<const double2*>(cur)[q2];
        }
    }
}

__global__ __launch_bounds__(256) void copy_gs(const double2* __restrict__ in, double2* __restrict__ out, size_t n2) {
    const size_t stride = (size_t)gridDim.x * 256;
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n2; i += stride) out[i] = in[i];
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
    const int64_t S = 1000000, T = 390;
    const size_t n = (size_t)S * T, bytes = n * 8;
    std::vector<double> h(n);
    uint64_t st = 12345;
    for (size_t i = 0; i < n; i++) {
        st = st * 6364136223846793005ull + 1442695040888963407ull;
        const double u = (double)(st >> 11) / 9007199254740992.0;
        h[i] = (u < 0.05) ? __builtin_nan("") : u;
    }
    double *in, *out, *ref;
    CK(hipMalloc(&in, bytes)); CK(hipMalloc(&out, bytes)); CK(hipMalloc(&ref, bytes));
    CK(hipMemcpy(in, h.data(), bytes, hipMemcpyHostToDevice));
    const double sm = 0.3;
    chunkA<32, 64, true><<<(unsigned)((S + 31) / 32), 64>>>(in, ref, S, T, sm);
    CK(hipDeviceSynchronize());
    std::vector<double> hr(n), ho(n);
    CK(hipMemcpy(hr.data(), ref, bytes, hipMemcpyDeviceToHost));
    auto check = [&](const char* name) {
        CK(hipMemcpy(ho.data(), out, bytes, hipMemcpyDeviceToHost));
        if (memcmp(ho.data(), hr.data(), bytes) != 0) printf("{\"test\":\"%s\",\"MISMATCH\":1}\n", name);
        CK(hipMemset(out, 0, bytes));
    };
    const double alg = 2.0 * bytes;
#define PR(name, ms) printf("{\"test\":\"%s\",\"ms\":%.4f,\"GBps\":%.1f}\n", name, ms, alg / (ms) / 1e6), fflush(stdout)
    {
        float ms = time_ms([&] { copy_gs<<<cus * 8, 256>>>((const double2*)in, (double2*)out, n / 2); }, 10);
        PR("copy_gs_8", ms);
    }
    {
        float ms = time_ms([&] { chunkA<32, 64, false><<<(unsigned)((S + 31) / 32), 64>>>(in, out, S, T, sm); }, 10);
        PR("chunkA_32x64_copy", ms);
        ms = time_ms([&] { chunkA<32, 64, true><<<(unsigned)((S + 31) / 32), 64>>>(in, out, S, T, sm); }, 10);
        PR("chunkA_32x64_ewma", ms);
        check("chunkA_32x64_ewma");
        ms = time_ms([&] { chunkA<16, 64, true><<<(unsigned)((S + 15) / 16), 64>>>(in, out, S, T, sm); }, 10);
        PR("chunkA_16x64_ewma", ms);
        check("chunkA_16x64_ewma");
        ms = time_ms([&] { chunkA<32, 32, true><<<(unsigned)((S + 31) / 32), 64>>>(in, out, S, T, sm); }, 10);
        PR("chunkA_32x32_ewma", ms);
        check("chunkA_32x32_ewma");
    }
#define RB(R, PF, G)                                                                                      \
    {                                                                                                     \
        const int64_t nblk = S / R;                                                                       \
        const unsigned grid = (G) > 0 ? (unsigned)(cus * (G)) : (unsigned)nblk;                          \
        float ms = time_ms([&] { rowsB<R, 390, PF><<<grid, 64>>>(in, out, S, T, sm, nblk); }, 10);      \
        char nm[64]; snprintf(nm, 64, "rowsB_R%d_pf%d_g%d", R, (int)PF, G);                               \
        PR(nm, ms);                                                                                       \
        check(nm);                                                                                        \
    }
    RB(8, false, 0)
#define RC(R, KR, NW, CP)                                                                                 \
    {                                                                                                     \
        const unsigned grid = (unsigned)((S / R + NW - 1) / NW);                                          \
        float ms = time_ms([&] { rowsC<R, KR, NW, 390, CP><<<grid, 64 * NW>>>(in, out, S, T, sm); }, 10); \
        char nm[64]; snprintf(nm, 64, "rowsC_R%d_KR%d_nw%d_c%d", R, KR, NW, (int)CP);                    \
        PR(nm, ms);                                                                                       \
        if (CP) check(nm);                                                                                \
    }
#define RD(R, NW, CP)                                                                                     \
    {                                                                                                     \
        const unsigned grid = (unsigned)((S / R + NW - 1) / NW);                                          \
        float ms = time_ms([&] { rowsD<R, 390, NW, CP><<<grid, 64 * NW>>>(in, out, S, sm); }, 10);        \
        char nm[64]; snprintf(nm, 64, "rowsD_R%d_nw%d_c%d", R, NW, (int)CP);                              \
        PR(nm, ms);                                                                                       \
        if (CP) check(nm);                                                                                \
    }
#define RE(R, G)                                                                                          \
    {                                                                                                     \
        const int64_t nblk = S / R;                                                                       \
        const unsigned grid = (unsigned)(cus * (G));                                                      \
        float ms = time_ms([&] { rowsE<R, 390><<<grid, 64>>>(in, out, S, sm, nblk); }, 10);               \
        char nm[64]; snprintf(nm, 64, "rowsE_R%d_g%d", R, G);                                             \
        PR(nm, ms);                                                                                       \
        check(nm);                                                                                        \
    }
    RD(8, 1, false) RD(8, 1, true) RD(8, 2, true) RD(4, 1, false) RD(4, 1, true) RD(4, 4, true)
    RD(2, 1, true) RD(16, 1, true) RD(6, 1, true)
    RE(8, 3) RE(4, 6) RE(4, 8) RE(2, 12) RE(2, 16)
    return 0;
}
