// pack.hip — gfx950 PACK kernel: the batched body of PackedWrite::write_all
// (capnp/src/serialize_packed.rs:304-439).
//
// Work decomposition
//   * A tile = `tc` consecutive chunks; one 256-thread workgroup (4 waves)
//     per tile; tiles are claimed through an atomic ticket so a tile only
//     ever waits on tiles that were claimed before it (forward progress).
//   * A wave packs whole chunks, 64 words per step (lane = word).
//   * Pass A computes each chunk's packed size; the tile aggregate is
//     published and the tile's global byte offset found by a decoupled
//     look-back over {flag, value} 64-bit granules; pass B re-runs the chunk
//     (input re-read from L2 / Infinity Cache) and writes the bytes.
//
// Run segmentation without a serial loop
//   The reference walks words one at a time: a zero word absorbs up to 255
//   following zero words, a 0xFF word absorbs up to 255 following words with
//   at most one zero byte (serialize_packed.rs:375-427).  Here a step takes
//   three 64-bit ballots — Z (zero words), L (<= 1 zero byte), F (tag 0xFF)
//   — plus the run carried from the previous step (type, remaining
//   capacity) and derives the absorbed set with scalar bit arithmetic:
//     carried:  the first min(lead, rem) words of the matching class
//     Z runs:   Z' & (Z' << 1)             (every zero word after a zero)
//     F runs:   within each run of L', the words after its first F word:
//               filled = ((L' ^ (L' + F')) & L') | F';  filled & (filled<<1)
//   A head at lane h can absorb at most 63 words inside a step, so the
//   255 cap only matters through the carried capacity.  Heads = valid words
//   not absorbed; their bytes are [tag][non-zero bytes] (+ count), absorbed
//   literal words emit 8 raw bytes, absorbed zero words emit nothing.
//
// Output path
//   Each wave stages its chunk's bytes in a 4 KiB LDS ring (byte writes at
//   the wave-scanned offsets) and streams whole 16-byte blocks to HBM with
//   dwordx4 stores; only the first and last block of a chunk (shared with
//   the neighbouring chunks) are written byte by byte.  A run's count byte
//   is only known once the run ends, possibly several steps later, so the
//   ring holds back the block containing a pending count until it is
//   patched.
#include "common.h"

namespace {

constexpr int kWaves = 4;
constexpr int kThreads = kWaves * CAPNP_WAVE;
constexpr uint32_t kRing = 4096;           // per-wave staging ring (bytes)
constexpr uint32_t kRingMask = kRing - 1;
constexpr int kMaxTileChunks = 128;

constexpr uint64_t kFlagAgg = 1ull << 62;  // tile aggregate available
constexpr uint64_t kFlagInc = 2ull << 62;  // tile inclusive prefix available
constexpr uint64_t kValMask = (1ull << 62) - 1;

struct Smem {
    uint64_t sel[256];                  // compaction selectors per tag
    uint64_t chunk_size[kMaxTileChunks];
    uint64_t chunk_pos[kMaxTileChunks];
    uint64_t prefix;
    uint32_t tile;
    uint32_t pad;
    alignas(16) uint8_t ring[kWaves][kRing];
};

// Carried run state between 64-word steps of one chunk.
struct Carry {
    uint32_t type;  // 0 none, 1 zero run, 2 literal run
    uint32_t rem;   // words the open run may still absorb
};

struct StepMasks {
    uint64_t H;      // heads
    uint32_t absorbed_carry;  // words absorbed by the carried run
    Carry next;
};

__device__ __forceinline__ StepMasks resolve_step(uint64_t Zm, uint64_t Lm, uint64_t Fm,
                                                  uint32_t nvalid, Carry c) {
    StepMasks r;
    uint64_t AC = 0;
    uint32_t k = 0;
    if (c.type == 1) {
        uint32_t lead = ctz64(~Zm);
        k = lead < c.rem ? lead : c.rem;
        AC = low_mask(k);
    } else if (c.type == 2) {
        uint32_t lead = ctz64(~Lm);
        k = lead < c.rem ? lead : c.rem;
        AC = low_mask(k);
    }
    uint64_t Z2 = Zm & ~AC;
    uint64_t AZ = Z2 & (Z2 << 1);
    uint64_t L2 = Lm & ~AC;
    uint64_t F2 = Fm & ~AC;
    uint64_t filled = ((L2 ^ (L2 + F2)) & L2) | F2;
    uint64_t AF = filled & (filled << 1);
    uint64_t H = low_mask(nvalid) & ~(AC | AZ | AF);
    r.H = H;
    r.absorbed_carry = k;
    if (H == 0) {
        r.next.type = c.type;
        r.next.rem = c.rem - 64;  // only reachable when the carry covered the step
    } else {
        uint32_t h = 63u - (uint32_t)__builtin_clzll(H);
        uint64_t hb = 1ull << h;
        if (Zm & hb) { r.next.type = 1; r.next.rem = 255u - (63u - h); }
        else if (Fm & hb) { r.next.type = 2; r.next.rem = 255u - (63u - h); }
        else { r.next.type = 0; r.next.rem = 0; }
    }
    return r;
}

// Packs one chunk of `nwords` words starting at in[w0].  WRITE=false returns
// the packed size only; WRITE=true stages and stores the bytes at out[o_c..].
template <bool WRITE>
__device__ uint64_t pack_chunk(const uint64_t* __restrict__ in, uint64_t w0, uint64_t nwords,
                               uint8_t* __restrict__ out, uint64_t o_c, uint8_t* ring,
                               const uint64_t* sel, uint32_t lane) {
    Carry carry = {0, 0};
    uint64_t total = 0;
    bool pend = false;        // a run's count byte is not yet known
    uint64_t pend_pos = 0;    // absolute output position of that count byte
    uint32_t pend_cnt = 0;
    uint64_t flushed = o_c & ~15ull;

    uint64_t wnext = 0;
    if (nwords) wnext = lane < nwords ? in[w0 + lane] : 0;
    for (uint64_t base = 0; base < nwords; base += 64) {
        const uint32_t nvalid = (uint32_t)((nwords - base) < 64 ? (nwords - base) : 64);
        const bool last = base + 64 >= nwords;
        const bool valid = lane < nvalid;
        const uint64_t w = wnext;
        if (!last) {
            uint64_t nb = base + 64;
            wnext = (nb + lane < nwords) ? in[w0 + nb + lane] : 0;
        }
        const uint32_t lo = (uint32_t)w, hi = (uint32_t)(w >> 32);
        const uint32_t tag = word_tag(lo, hi);
        const uint32_t pop = __builtin_popcount(tag);
        const uint64_t Zm = ballot64(valid && tag == 0);
        const uint64_t Lm = ballot64(valid && pop >= 7);
        const uint64_t Fm = ballot64(valid && tag == 0xFF);
        const StepMasks sm = resolve_step(Zm, Lm, Fm, nvalid, carry);
        const bool head = (sm.H >> lane) & 1;
        uint32_t size;
        if (head) size = tag == 0 ? 2u : (tag == 0xFF ? 10u : 1u + pop);
        else size = (valid && tag != 0) ? 8u : 0u;
        const uint64_t B0 = ballot64(size & 1), B1 = ballot64(size & 2);
        const uint64_t B2 = ballot64(size & 4), B3 = ballot64(size & 8);
        const uint32_t step_bytes = popc64(B0) + 2 * popc64(B1) + 4 * popc64(B2) + 8 * popc64(B3);

        if (WRITE) {
            const uint32_t off = mask_rank(B0) + 2 * mask_rank(B1) + 4 * mask_rank(B2) +
                                 8 * mask_rank(B3);
            // count byte of a Z/F head whose run ends inside this step
            uint32_t cnt = 0;
            const uint64_t later = sm.H & ~low_mask(lane + 1);
            if (later) cnt = ctz64(later) - lane - 1;
            else cnt = nvalid - lane - 1;   // run reaches the step end
            const uint64_t pos = o_c + total + off;
            if (head || size) {
                uint32_t d0, d1 = 0, d2 = 0, len = size;
                if (head && tag == 0) {
                    d0 = cnt << 8;
                } else if (head) {
                    uint32_t clo = lo, chi = hi;
                    if (tag != 0xFF) {
                        const uint64_t s = sel[tag];
                        clo = __builtin_amdgcn_perm(hi, lo, (uint32_t)s);
                        chi = __builtin_amdgcn_perm(hi, lo, (uint32_t)(s >> 32));
                    }
                    d0 = tag | (clo << 8);
                    d1 = (clo >> 24) | (chi << 8);
                    d2 = (chi >> 24) | (cnt << 8);
                } else {
                    d0 = lo;
                    d1 = hi;
                }
#pragma unroll
                for (uint32_t k = 0; k < 10; k++) {
                    if (k < len) {
                        const uint32_t d = k < 4 ? d0 : (k < 8 ? d1 : d2);
                        ring[(pos + k) & kRingMask] = (uint8_t)(d >> (8 * (k & 3)));
                    }
                }
            }
            // Resolve the count carried in from earlier steps.
            if (pend) {
                pend_cnt += sm.absorbed_carry;
                if (sm.absorbed_carry < 64 || last) {
                    if (lane == 0) ring[pend_pos & kRingMask] = (uint8_t)pend_cnt;
                    pend = false;
                }
            }
            // A Z/F head whose run reaches the end of a non-final step: its
            // count continues into the next step.
            if (!last && nvalid == 64 && sm.H) {
                const uint32_t h = 63u - (uint32_t)__builtin_clzll(sm.H);
                const uint64_t hb = 1ull << h;
                if ((Zm | Fm) & hb) {
                    // the last head absorbs every later word of the step
                    pend = true;
                    pend_cnt = 63u - h;
                    // its output offset: bytes of lanes below h
                    const uint64_t below = low_mask(h);
                    const uint32_t hoff = popc64(B0 & below) + 2 * popc64(B1 & below) +
                                          4 * popc64(B2 & below) + 8 * popc64(B3 & below);
                    pend_pos = o_c + total + hoff + ((Zm & hb) ? 1u : 9u);
                }
            }
            total += step_bytes;
            wave_lds_sync();
            // Flush whole blocks that can no longer change.
            const uint64_t produced = o_c + total;
            uint64_t limit;
            if (last) limit = produced;
            else limit = (pend ? pend_pos : produced) & ~15ull;
            for (uint64_t b = flushed + 16ull * lane; b < limit; b += 16ull * CAPNP_WAVE) {
                const uint8_t* src = ring + (b & kRingMask);
                const uint64_t own_lo = b < o_c ? o_c : b;
                const uint64_t own_hi = (b + 16 < produced) ? b + 16 : produced;
                if (own_lo == b && own_hi == b + 16) {
                    *reinterpret_cast<uint4*>(out + b) = *reinterpret_cast<const uint4*>(src);
                } else {
                    for (uint64_t a = own_lo; a < own_hi; a++) out[a] = src[a - b];
                }
            }
            if (limit > flushed) flushed = (limit + 15) & ~15ull;
            wave_lds_sync();
        } else {
            total += step_bytes;
        }
        carry = sm.next;
    }
    return total;
}

__global__ void __launch_bounds__(kThreads)
pack_kernel(const uint64_t* __restrict__ in, const uint64_t* __restrict__ chunk_off,
            uint64_t nchunks, uint32_t tc, uint8_t* __restrict__ out, uint64_t out_cap,
            uint64_t* __restrict__ out_off, uint64_t* __restrict__ tile_state,
            uint32_t* __restrict__ ticket) {
    __shared__ Smem sm;
    const uint32_t tid = threadIdx.x;
    const uint32_t lane = tid & 63u;
    const uint32_t wave = tid >> 6;

    if (tid == 0) sm.tile = atomicAdd(ticket, 1u);
    // compaction selectors: byte r = index of the r-th set bit of the tag
    {
        uint64_t s = 0x0C0C0C0C0C0C0C0Cull;
        uint32_t r = 0;
        for (uint32_t k = 0; k < 8; k++) {
            if (tid & (1u << k)) {
                s = (s & ~(0xFFull << (8 * r))) | ((uint64_t)k << (8 * r));
                r++;
            }
        }
        sm.sel[tid] = s;
    }
    __syncthreads();
    const uint32_t tile = sm.tile;
    const uint64_t c0 = (uint64_t)tile * tc;
    const uint64_t c1 = (c0 + tc < nchunks) ? c0 + tc : nchunks;
    const uint32_t nc = (uint32_t)(c1 - c0);

    // ---- pass A: packed size of every chunk of the tile
    for (uint32_t i = wave; i < nc; i += kWaves) {
        const uint64_t a = chunk_off[c0 + i], b = chunk_off[c0 + i + 1];
        const uint64_t sz = pack_chunk<false>(in, a, b - a, out, 0, nullptr, sm.sel, lane);
        if (lane == 0) sm.chunk_size[i] = sz;
    }
    __syncthreads();

    // ---- tile scan + decoupled look-back (wave 0)
    if (wave == 0) {
        uint64_t v = lane < nc ? sm.chunk_size[lane] : 0;
        uint64_t v2 = (lane + 64 < nc) ? sm.chunk_size[lane + 64] : 0;
        // inclusive scan over 64 lanes (two halves of up to 128 chunks)
        uint64_t s = v, s2 = v2;
        for (uint32_t d = 1; d < 64; d <<= 1) {
            uint64_t t = __shfl_up(s, d, 64);
            uint64_t t2 = __shfl_up(s2, d, 64);
            if (lane >= d) { s += t; s2 += t2; }
        }
        const uint64_t half = __shfl(s, 63, 64);
        s2 += half;
        const uint64_t agg = __shfl(s2, 63, 64);
        uint64_t excl = 0;
        if (tile == 0) {
            if (lane == 0) store_relaxed_agent(&tile_state[0], kFlagInc | agg);
        } else {
            if (lane == 0) store_relaxed_agent(&tile_state[tile], kFlagAgg | agg);
            int64_t idx = (int64_t)tile - 1;
            for (;;) {
                const int64_t j = idx - (int64_t)lane;
                uint64_t st = j >= 0 ? load_relaxed_agent(&tile_state[j]) : kFlagInc;
                const uint64_t inc = ballot64((st & kFlagInc) != 0);
                const uint64_t none = ballot64((st >> 62) == 0);
                const uint32_t first_inc = ctz64(inc);
                const uint64_t need = first_inc < 64 ? low_mask(first_inc + 1) : ~0ull;
                if (none & need) {
                    __builtin_amdgcn_s_sleep(1);
                    continue;  // a predecessor has not published yet
                }
                uint64_t val = (lane <= first_inc) ? (st & kValMask) : 0;
                for (uint32_t d = 32; d >= 1; d >>= 1) val += __shfl_xor(val, d, 64);
                excl += val;
                if (first_inc < 64) break;
                idx -= 64;
            }
            if (lane == 0) store_relaxed_agent(&tile_state[tile], kFlagInc | (excl + agg));
        }
        if (lane < nc) sm.chunk_pos[lane] = excl + s - v;
        if (lane + 64 < nc) sm.chunk_pos[lane + 64] = excl + s2 - v2;
        if (lane == 0) sm.prefix = excl;
        if (c1 == nchunks && lane == 0) out_off[nchunks] = excl + agg;
    }
    __syncthreads();
    for (uint32_t i = tid; i < nc; i += kThreads) out_off[c0 + i] = sm.chunk_pos[i];

    // ---- pass B: write the bytes.  Block arithmetic runs on addresses
    // aligned to 16 in memory: positions are shifted by out's misalignment.
    const uint32_t mis = (uint32_t)(reinterpret_cast<uintptr_t>(out) & 15u);
    uint8_t* const outa = out - mis;
    for (uint32_t i = wave; i < nc; i += kWaves) {
        const uint64_t a = chunk_off[c0 + i], b = chunk_off[c0 + i + 1];
        const uint64_t pos = sm.chunk_pos[i];
        if (pos + sm.chunk_size[i] > out_cap) continue;  // does not fit: skip
        pack_chunk<true>(in, a, b - a, outa, pos + mis, sm.ring[wave], sm.sel, lane);
    }
}

}  // namespace

extern "C" hipError_t capnp_launch_pack(const uint64_t* d_in, const uint64_t* d_chunk_off,
                                        uint64_t nchunks, uint32_t tc, uint8_t* d_out,
                                        uint64_t out_cap, uint64_t* d_out_off,
                                        uint64_t* d_tile_state, uint32_t* d_ticket,
                                        size_t state_bytes, hipStream_t stream) {
    if (tc == 0 || tc > kMaxTileChunks) return hipErrorInvalidValue;
    const uint64_t ntiles = (nchunks + tc - 1) / tc;
    if (nchunks == 0) {
        return hipMemsetAsync(d_out_off, 0, sizeof(uint64_t), stream);
    }
    hipError_t e = hipMemsetAsync(d_ticket, 0, state_bytes, stream);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(pack_kernel, dim3((uint32_t)ntiles), dim3(kThreads), 0, stream, d_in,
                       d_chunk_off, nchunks, tc, d_out, out_cap, d_out_off, d_tile_state,
                       d_ticket);
    return hipGetLastError();
}
