// sts_dma.hpp -- LDS-DMA (global_load_lds_dwordx4) and wave-local LDS ordering, for the
// kernels that stage whole series through LDS (sts_ar.hip, sts_recur.hip, sts_short.hip).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace sts {

typedef __attribute__((address_space(3))) void lds_void;

__device__ __forceinline__ unsigned lds_addr(const void* p) {
    return (unsigned)(uintptr_t)(const lds_void*)p;
}

// One LDS-DMA instruction (global_load_lds_dwordx4): 64 lanes x 16 B from per-lane global
// addresses to LDS [lds_addr, lds_addr + 1 KB) in lane order.  Written as asm so that hipcc
// does not track it: with the builtin, hipcc treats every later vector-memory op as a
// possible pending LDS write and puts a vmcnt(0) before each LDS read of the store loop
// (one store round trip per 1-KB piece: measured 2.29 against 1.67 ms on the C2 shape).  The caller waits
// for the DMA itself (dma_wait).  M0 holds the LDS base; it is restored.
// NT: the non-temporal form (`nt`), per kernel as measured (profiles/r05_s20_ab_dma_store_policy.jsonl)
template <bool NT = false>
__device__ __forceinline__ void glds16(const double* gsrc, unsigned lds_byte_addr) {
    unsigned keep;
    lds_byte_addr = __builtin_amdgcn_readfirstlane(lds_byte_addr);   // wave-uniform: pin it to an SGPR
    if constexpr (NT)
        asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off nt\n\ts_mov_b32 m0, %0"
                     : "=&s"(keep)
                     : "v"(gsrc), "s"(lds_byte_addr)
                     : "memory");
    else
        asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                     : "=&s"(keep)
                     : "v"(gsrc), "s"(lds_byte_addr)
                     : "memory");
}

// the same from a wave-uniform base (SGPR pair) plus a per-lane byte offset (VGPR): no 64-bit
// address arithmetic per instruction
__device__ __forceinline__ void glds16_s(const double* sbase, unsigned voff, unsigned lds_byte_addr) {
    unsigned keep;
    lds_byte_addr = __builtin_amdgcn_readfirstlane(lds_byte_addr);
    // (readfirstlane returns int: through unsigned, or the low half sign-extends into the high one)
    const unsigned long long b =
        (unsigned long long)(unsigned)__builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)sbase) |
        ((unsigned long long)(unsigned)__builtin_amdgcn_readfirstlane((unsigned)((uintptr_t)sbase >> 32)) << 32);
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(voff), "s"(b), "s"(lds_byte_addr)
                 : "memory");
}

// one 16-B store of a staged result pair (NT: non-temporal)
template <bool NT = false>
__device__ __forceinline__ void store_pair16(double* p, const double* lds_src) {
    typedef double d2_t __attribute__((ext_vector_type(2)));
    const d2_t v = *reinterpret_cast<const d2_t*>(lds_src);
    if constexpr (NT) __builtin_nontemporal_store(v, reinterpret_cast<d2_t*>(p));
    else *reinterpret_cast<d2_t*>(p) = v;
}

__device__ __forceinline__ void dma_wait() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// order this wave's LDS accesses (no workgroup barrier: the buffers are per wave)
__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront", "local");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront", "local");
}

}  // namespace sts
