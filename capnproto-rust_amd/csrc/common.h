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

// Inclusive sum over lanes 0..i of the wave (DPP, as wave_max_scan).
__device__ __forceinline__ uint32_t wave_sum_scan(uint32_t x) {
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xf, 0xf, false);
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xf, 0xf, false);
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xf, 0xf, false);
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xf, 0xf, false);
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xa, 0xf, false);
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xc, 0xf, false);
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

// ---- resident per-call service (capi.hip: the one-launch per-message calls
// without their launch).  One workgroup stays resident and polls one pinned
// 64-byte line: [0] the bell {gen << 32 | seq}, [1, 7) the request's
// arguments, [7] a check word (svc_mix of the other seven).  The host writes
// the arguments and the check, then the bell; a poll reads the whole line in
// one load, so a request costs no second round trip for its arguments, and a
// line read while the host was writing it fails the check and is read again.
// The workgroup serves every new seq of its own gen and exits on another gen
// (a newer service, or stop) or after `idle_ticks` of the 100 MHz real-time
// clock without a request, so it never outlives its last caller by more than
// that.
constexpr uint32_t kSvcArgs = 6;
// (one poll at a time: profiles/r06l_svc_ab.txt -- 2 or 4 polls in flight
// to the same line cost 1-3 us a call more than one)
#ifndef SVC_POLLS
#define SVC_POLLS 1
#endif
#ifndef SVC_POLL_GAP
#define SVC_POLL_GAP 1
#endif
constexpr uint32_t kSvcPolls = SVC_POLLS;  // poll loads in flight (spread over a PCIe round trip)
constexpr int kSvcPollGap = SVC_POLL_GAP;  // s_sleep between them (x 64 cycles)
#ifndef SVC_PROF
#define SVC_PROF 0  // diagnostic builds: per-request phase times (capnp_svc_prof)
#endif
#if SVC_PROF
// [0] requests, [2] bell seen -> body done (100 MHz ticks); msg_read_body:
// [3] table, [4] decode, [5] results landed, [6] - [7] staging (sums of
// stamps); [8] the body in shader clock cycles (s_memtime: [8] / [2] = the
// clock in units of 100 MHz); unpack_small: [9] selector table and init,
// [10] wave 0's walks, [11] expansion, [12] calls; within [10]: [16] spec
// walks, [17] rounds, [18] the last segment's walk, [19] descriptors, [20]
// rounds taken
__device__ unsigned long long g_svc_prof[24];
#endif
struct SvcCmd {
    uint64_t bell;
    uint64_t a[kSvcArgs];
#if SVC_PROF
    uint64_t t_args, c_args;
#endif
};

// The request line's arguments of each service, by name (host and device
// share these layouts): msg_read_service's and msg_pack_service's.
struct SvcReadReq {
    uint64_t in;      // the staged input (device memory written through the BAR, or pinned)
    uint64_t words;   // the body's words (pinned); {status, 0, consumed} at round16(8 cap) bytes on
    uint64_t flags;   // stage bytes | no_alloc << 32 | try_mode << 33 | has_limit << 34
    uint64_t limit, buffer_len, cap;
};
struct SvcPackReq {
    uint64_t words, off;  // the message's chunks and their offsets (as SvcReadReq::in)
    uint64_t out;         // the packed output (pinned); *total sits 16 bytes before it
    uint64_t counts;      // nchunks | nwords << 32
    uint64_t out_cap;
    uint64_t scratch;     // device scratch for the bytes before their copy out
};
static_assert(sizeof(SvcReadReq) == kSvcArgs * 8 && sizeof(SvcPackReq) == kSvcArgs * 8,
              "a request fills the line's arguments");

// The line's check word (host and device).
__host__ __device__ __forceinline__ uint64_t svc_mix(uint64_t b, const uint64_t* r) {
    uint64_t h = 0x9E3779B97F4A7C15ull ^ b;
    for (uint32_t i = 0; i < kSvcArgs; i++) {
        h ^= r[i];
        h *= 0xFF51AFD7ED558CCDull;
        h ^= h >> 33;
    }
    return h;
}

// Waits for the next request (wave 0 polls; the workgroup meets at a
// barrier).  false: exit.  On true, cmd.a holds the request's arguments and
// `last` its seq.
__device__ __forceinline__ bool svc_next(const uint64_t* line, SvcCmd& cmd, uint32_t gen,
                                         uint32_t& last, uint64_t idle_ticks, uint32_t wave,
                                         uint32_t lane) {
    if (wave == 0) {
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
        uint64_t* const p = const_cast<uint64_t*>(line) + (lane & 7u);
        uint64_t v[kSvcPolls];
#pragma unroll
        for (uint32_t k = 0; k < kSvcPolls; k++) {
            v[k] = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            if (k + 1 < kSvcPolls) __builtin_amdgcn_s_sleep(kSvcPollGap);
        }
        uint64_t b = 0, hit = 0;
        for (bool more = true; more;) {
#pragma unroll
            for (uint32_t k = 0; k < kSvcPolls && more; k++) {
                const uint64_t bk = readlane64(v[k], 0);
                if ((uint32_t)(bk >> 32) != gen) {
                    more = false;  // (b = 0: exit)
                } else if ((uint32_t)bk != last) {
                    uint64_t r[kSvcArgs];
#pragma unroll
                    for (uint32_t i = 0; i < kSvcArgs; i++) r[i] = readlane64(v[k], i + 1);
                    if (svc_mix(bk, r) == readlane64(v[k], 7)) {
                        b = bk;
                        hit = v[k];
                        more = false;
                    }
                }
                if (more) {
                    if (__builtin_amdgcn_s_memrealtime() - t0 > idle_ticks) {
                        more = false;
                    } else {
                        v[k] = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                        __builtin_amdgcn_s_sleep(kSvcPollGap);
                    }
                }
            }
        }
        if (b) {
#if SVC_PROF
            const uint64_t ta = __builtin_amdgcn_s_memrealtime();
            if (lane == 0) {
                atomicAdd(&g_svc_prof[0], 1ull);
                atomicAdd(&g_svc_prof[7], (unsigned long long)ta);
            }
            cmd.t_args = ta;  // (the body's start, for svc_prof_done)
            cmd.c_args = __builtin_amdgcn_s_memtime();
#endif
            // (system scope: the caches drop what earlier requests left, so the
            // payload the host wrote before the bell is seen)
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
            if (lane >= 1 && lane <= kSvcArgs) cmd.a[lane - 1] = hit;
        }
        if (lane == 0) cmd.bell = b;
    }
    __syncthreads();
    const uint64_t b = uniform64(cmd.bell);
    if (!b) return false;
    last = (uint32_t)b;
    return true;
}

// SVC_PROF: the body's time.
__device__ __forceinline__ void svc_prof_done(SvcCmd& cmd, uint32_t tid) {
#if SVC_PROF
    __syncthreads();
    if (tid == 0) {
        const uint64_t td = __builtin_amdgcn_s_memrealtime();
        atomicAdd(&g_svc_prof[2], (unsigned long long)(td - cmd.t_args));
        atomicAdd(&g_svc_prof[8], (unsigned long long)(__builtin_amdgcn_s_memtime() - cmd.c_args));
    }
#else
    (void)cmd;
    (void)tid;
#endif
}

// The service's exit mark for the host (process-exit path): {gen}, stored
// after the last request's results.
__device__ __forceinline__ void svc_exit(uint64_t* mark, uint32_t gen, uint32_t tid) {
    if (tid == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
        __hip_atomic_store(mark, (uint64_t)gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}
