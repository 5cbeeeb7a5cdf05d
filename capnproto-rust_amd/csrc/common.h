// common.h — device helpers shared by the gfx950 packed-codec kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define CAPNP_WAVE 64

// Per-byte "is non-zero" flags of a 32-bit half, gathered into 4 tag bits.
// Byte k non-zero <=> bit 7 of ((b & 0x7f) + 0x7f) | b; the multiply by
// 0x01020408 moves bit 8k of (t >> 7) to bit 24 + k with no carries.
__host__ __device__ __forceinline__ uint32_t nz_nibble(uint32_t x) {
    uint32_t t = (((x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | x) & 0x80808080u;
    return ((t >> 7) * 0x01020408u) >> 24;
}

// The packed-encoding tag of a word: bit k set iff byte k is non-zero
// (PackedWrite::write_all, capnp/src/serialize_packed.rs:324-371).
__host__ __device__ __forceinline__ uint32_t word_tag(uint32_t lo, uint32_t hi) {
    return nz_nibble(lo) | (nz_nibble(hi) << 4);
}

// Byte k of the result is bit k of `tag` (0/1).  Done per nibble: the
// multiply by 0x00204081 puts bit j at 8j with no colliding terms.
__host__ __device__ __forceinline__ constexpr uint64_t spread_bits(uint32_t tag) {
    uint32_t lo = ((tag & 15u) * 0x00204081u) & 0x01010101u;
    uint32_t hi = (((tag >> 4) & 15u) * 0x00204081u) & 0x01010101u;
    return ((uint64_t)hi << 32) | lo;
}

// v_perm_b32 selector (two dwords, 8 bytes) that scatters the `pop` packed
// bytes of a tag back to their word positions: output byte k = bit k ?
// rank_k : 0x0C (zero), rank_k = number of set bits below k.
__host__ __device__ __forceinline__ constexpr uint64_t expand_selector(uint32_t tag) {
    uint64_t t8 = spread_bits(tag);
    uint64_t incl = t8 * 0x0101010101010101ull;     // inclusive prefix per byte
    uint64_t rank = incl - t8;                       // exclusive prefix
    uint64_t m = t8 * 0xFFull;                       // 0xFF where bit set
    return (rank & m) | (0x0C0C0C0C0C0C0C0Cull & ~m);
}

__device__ __forceinline__ uint32_t lane_id() {
    return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
}

// Number of set bits of a wave-uniform mask strictly below this lane.
__device__ __forceinline__ uint32_t mask_rank(uint64_t m) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                     __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

__device__ __forceinline__ uint64_t ballot64(bool p) { return __ballot(p); }

// Value of lane i - D of this lane's row of 16 lanes (DPP row_shr:D, a VALU
// op: no LDS round trip as __shfl_up's ds_bpermute); 0 for the row's first
// D lanes.  (0 is the identity of the row scans built from it, max and +.)
template <uint32_t D>
__device__ __forceinline__ uint32_t row_shr(uint32_t x) {
    static_assert(D >= 1 && D <= 15, "row_shr:1..15");
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x110 + D, 0xF, 0xF, false);
}

// Inclusive max over lanes 0..i of the wave (DPP: row_shr within each row of
// 16 lanes, then row_bcast:15 / row_bcast:31 carry the row maxima on; all
// VALU, no LDS round trip).
__device__ __forceinline__ uint32_t wave_max_scan(uint32_t x) {
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xf, 0xf, false));
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xf, 0xf, false));
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xf, 0xf, false));
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xf, 0xf, false));
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xa, 0xf, false));
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xc, 0xf, false));
    return x;
}

// The value of lane i - 1 (DPP wave_shr:1); 0 in lane 0.
__device__ __forceinline__ uint32_t wave_shr1(uint32_t x) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x138, 0xf, 0xf, false);
}

// Inclusive max / sum over lanes 0..i of this lane's row of 16 lanes.
__device__ __forceinline__ uint32_t row_max_scan(uint32_t x) {
    x = max(x, row_shr<1>(x));
    x = max(x, row_shr<2>(x));
    x = max(x, row_shr<4>(x));
    return max(x, row_shr<8>(x));
}
__device__ __forceinline__ uint32_t row_sum_scan(uint32_t x) {
    x += row_shr<1>(x);
    x += row_shr<2>(x);
    x += row_shr<4>(x);
    return x + row_shr<8>(x);
}

__host__ __device__ __forceinline__ uint64_t low_mask(uint32_t k) {
    return k >= 64 ? ~0ull : ((1ull << k) - 1ull);
}

__host__ __device__ __forceinline__ uint32_t ctz64(uint64_t x) {
    return x ? (uint32_t)__builtin_ctzll(x) : 64u;
}

__host__ __device__ __forceinline__ uint32_t popc64(uint64_t x) {
    return (uint32_t)__builtin_popcountll(x);
}

// Orders this wave's LDS writes before its later LDS reads (other lanes of
// the same wave): LDS ops of one wave execute in order, so a wait on the LGKM
// counter plus a compiler barrier suffices.
__device__ __forceinline__ void wave_lds_sync() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
}

template <typename T>
__device__ __forceinline__ T uniform(T v) {
    return (T)__builtin_amdgcn_readfirstlane((int)v);
}

__device__ __forceinline__ uint64_t uniform64(uint64_t v) {
    uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)v);
    uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(v >> 32));
    return ((uint64_t)hi << 32) | lo;
}

// Four 64-bit scalar loads in one round trip (uniform addresses).  The
// compiler otherwise waits after each load whose value a compare or branch
// uses before the next load is issued.
__device__ __forceinline__ void sload4(const uint64_t* p0, const uint64_t* p1, const uint64_t* p2,
                                       const uint64_t* p3, uint64_t& a, uint64_t& b, uint64_t& c,
                                       uint64_t& d) {
    asm volatile(
        "s_load_dwordx2 %0, %4, 0x0\n\t"
        "s_load_dwordx2 %1, %5, 0x0\n\t"
        "s_load_dwordx2 %2, %6, 0x0\n\t"
        "s_load_dwordx2 %3, %7, 0x0\n\t"
        "s_waitcnt lgkmcnt(0)"
        : "=&s"(a), "=&s"(b), "=&s"(c), "=&s"(d)
        : "s"(p0), "s"(p1), "s"(p2), "s"(p3));
}

__device__ __forceinline__ uint64_t readlane64(uint64_t v, uint32_t l) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, l);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), l);
    return ((uint64_t)hi << 32) | lo;
}

// Relaxed agent-scope 64-bit accesses (single global sc1 load/store): the
// look-back records are {flag, value} granules written by one store
// (MI355X_MICROARCH.md, "Valid forms", R2 granule).
__device__ __forceinline__ void store_relaxed_agent(uint64_t* p, uint64_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint64_t load_relaxed_agent(const uint64_t* p) {
    return __hip_atomic_load(const_cast<uint64_t*>(p), __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
}

// Cross-workgroup records (look-back): relaxed agent-scope 8-byte accesses
// to UNCACHED device memory (hipDeviceMallocUncached, capi.hip), so the
// reader and writer meet at memory.  In cached memory a relaxed agent load is
// served by the reader XCD's L2 (MI355X_MICROARCH.md: sc1 loads bypass L1
// only), where a line an earlier poll brought in stays stale after another
// XCD's store.
__device__ __forceinline__ uint64_t poll_agent(uint64_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void publish_agent(uint64_t* p, uint64_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
