// pack.hip — gfx950 PACK kernel: the batched body of PackedWrite::write_all
// (capnp/src/serialize_packed.rs:304-439).
//
// Work decomposition
//   * A tile = `tc` consecutive chunks; one 256-thread workgroup (4 waves)
//     per tile; tile = blockIdx.x (workgroups are dispatched in index
//     order), so a tile only ever waits on lower-numbered tiles, which were
//     dispatched before it (forward progress).
//   * Staged path (every wave's share fits kStageSteps 64-word steps): wave
//     w owns a contiguous run of the tile's chunks, loads all its words into
//     registers at once, packs them into its own zeroed LDS region (offsets
//     local to the wave need no look-back), and after the tile's global
//     offset is known copies the region out with aligned 16-byte stores.
//   * Streaming path (tiles with larger chunks): wave w owns chunks w, w+4,
//     ...; pass A computes sizes, pass B re-reads the words (L2 / MALL) and
//     flushes whole 16-byte blocks through a 4 KiB LDS ring.
//   * The tile offset comes from a decoupled look-back over {flag, value}
//     64-bit granules (one relaxed agent-scope store / load each).
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
// Byte compaction
//   Every lane ORs its (<= 10-byte) record, shifted to its byte offset, into
//   <= 4 dwords of a zeroed LDS buffer (ds_or_b32).  A run's count byte is
//   only known once the run ends, possibly several steps later; it is
//   patched in LDS (the ring holds back the block that contains it).
#include "common.h"
#include <stdlib.h>
#include "../../include/capnp_packed.h"



#ifndef PACK_PROF
#define PACK_PROF 0  // look-back counters (scripts/pack_prof.py); 0 = product
#endif
#if PACK_PROF
// [0] within-group spin rounds, [1] group-scan spin rounds, [2] tile
// fallbacks, [3] group fallbacks, [4] group windows scanned, [5] tiles,
// [6] s_memtime cycles in lookback (wave 0), [7] cycles in pass 2
__device__ unsigned long long g_prof[8];
// per-tile trace (set by capnp_pack_trace), 8 words per tile: [0] start,
// [1] published, [2] offset known, [3] end (s_memrealtime, 100 MHz),
// [4] XCC id << 32 | HW_ID, [5] within spins, [6] group spins, [7] windows
__device__ uint64_t* g_trace;
#define PROF_ADD(i, v) atomicAdd(&g_prof[i], (unsigned long long)(v))
#define TRACE(tile, k, v) do { if (g_trace) g_trace[(tile) * 8 + (k)] = (v); } while (0)
#define RT() __builtin_amdgcn_s_memrealtime()
#else
#define PROF_ADD(i, v) ((void)0)
#define TRACE(tile, k, v) ((void)0)
#define RT() 0ull
#endif

namespace {

constexpr int kWaves = 4;  // waves per workgroup (tile = kWaves x kStageSteps x 64 words)
constexpr int kThreads = kWaves * CAPNP_WAVE;
constexpr uint32_t kRing = 4096;           // streaming path: per-wave ring (bytes)
constexpr uint32_t kRingMask = kRing - 1;
constexpr int kMaxTileChunks = 64;
constexpr uint32_t kZeroAhead = 1024;      // ring bytes zeroed per refill
constexpr uint32_t kStepMax = 64 * 10 + 16;

// Staged path capacity: kStageSteps steps of 64 words per wave.
constexpr uint32_t kStageSteps = 8;
constexpr uint32_t kStageWords = 64 * kStageSteps;
// >= the packed bytes of a wave's range: at most 8.5 bytes per word (a 0xFF
// head of 10 bytes needs a word of <= 7 bytes before the next one) plus 1.5
// per chunk, and a range holds at most kStageSteps non-empty chunks
constexpr uint32_t kStageBytesMax = 8 * kStageWords + kStageWords / 2 + 2 * kStageSteps;
// Leading gaps (capnp_launch_pack_gap): a wave's range stays staged while
// its gaps total at most kGapSlack bytes.
constexpr uint32_t kGapSlack = 128;
// Word tiles (pack_wt_kernel): regions for the worst case, plus the 32
// bytes copy_out may read past the end.
constexpr uint32_t kRegion = (kStageBytesMax + kGapSlack + 32 + 15) & ~15u;
// Chunk tiles (pack_kernel): regions of kStageBytes (gaps included), 8.19
// bytes per word: incompressible words pack to 8.03, so only adversarial
// input (0xFF heads alternating with breakers, up to 8.5) overflows, and a
// tile whose ranges overflow after pass 1 takes the streaming path.  The
// smaller regions and the 8-byte selector entries fit 8 workgroups per CU
// (20.3 KB each) where the worst-case layout fit 6 (23.8 KB): 608 -> 570 us
// at config 2 in a trial build.
constexpr uint32_t kStageBytes = 4192;
static_assert(kStageBytes <= kStageBytesMax && kStageBytes % 16 == 0, "stage capacity");
constexpr uint32_t kStageRegion = (kStageBytes + 32 + 15) & ~15u;
// per-wave LDS region of the chunk tiles: the staged bytes, or the
// streaming path's flush ring
constexpr uint32_t kRegionBytes = kStageRegion > kRing ? kStageRegion : kRing;

// Record sync index (optional side-band): one entry per global word index
// m = kSyncWords * k (8k), for the chunk that holds word m: the chunk-relative packed offset of
// the record that covers word m (24 bits) and m minus that record's first
// word (8 bits; a run covers at most 255 words after its head, so it fits).  An
// unpack that has the index walks CAPNP_SYNC_WORDS-word segments in parallel and checks that
// consecutive segments meet (unpack.hip).  kSyncNone marks an entry the
// kernel does not provide (streaming path); the decoder then walks serially.
constexpr uint32_t kSyncWords = CAPNP_SYNC_WORDS;
constexpr uint32_t kSyncNone = 0xFFFFFFFFu;

constexpr uint64_t kFlagAgg = 1ull << 62;  // tile aggregate available
constexpr uint64_t kFlagInc = 2ull << 62;  // tile inclusive prefix available
constexpr uint64_t kValMask = (1ull << 62) - 1;

// Record assembly table, one entry per tag plus kSelCopy (a literal word
// inside a run, copied as is), so every lane runs the same four ops:
//   r0 = perm(hi, lo, s0) | ((cnt << 8 | tag) & m)
//   r1 = perm(hi, lo, s1),  r2 = perm(cnt, hi, s2)
// s0/s1 put a zero byte (the tag's slot) first and then the first seven
// non-zero bytes of the word; s2 places byte 7 and the count byte of a 0xFF
// word; m keeps the tag (0xFF), tag and count (0xFFFF, zero word) or nothing.
// Only s0/s1 live in the (LDS) table: s2 and m follow from the entry index
// (sel_s2 / sel_m), which halves the table to 2 KiB.
constexpr uint32_t kSelCopy = 256;
struct alignas(16) SelEntry {
    uint32_t s0, s1, s2, m;
};
struct alignas(8) Sel8 {
    uint32_t s0, s1;
};
__device__ __forceinline__ uint32_t sel_s2(uint32_t idx) {
    return idx == 0xFFu ? 0x0C0C0403u : 0x0C0C0C0Cu;
}
__device__ __forceinline__ uint32_t sel_m(uint32_t idx) {
    return idx == kSelCopy ? 0u : (idx == 0u ? 0xFFFFu : 0xFFu);
}

struct SelTable {
    SelEntry e[kSelCopy + 1];
};

// The table, built at compile time; each tile copies it to LDS (one 16-byte
// load and store per thread).
constexpr SelTable make_sel_table() {
    SelTable t{};
    for (uint32_t tag = 0; tag < 256; tag++) {
        uint64_t s = 0x0C0C0C0C0C0C0C0Cull;
        uint32_t r = 1;  // byte r + 1 = index of the r-th set bit (r < 7)
        for (uint32_t k = 0; k < 8; k++) {
            if (tag & (1u << k)) {
                if (r < 8) s = (s & ~(0xFFull << (8 * r))) | ((uint64_t)k << (8 * r));
                r++;
            }
        }
        t.e[tag].s0 = (uint32_t)s;
        t.e[tag].s1 = (uint32_t)(s >> 32);
        t.e[tag].s2 = tag == 0xFF ? 0x0C0C0403u : 0x0C0C0C0Cu;
        t.e[tag].m = tag == 0 ? 0xFFFFu : 0xFFu;
    }
    t.e[kSelCopy].s0 = 0x03020100u;
    t.e[kSelCopy].s1 = 0x07060504u;
    t.e[kSelCopy].s2 = 0x0C0C0C0Cu;
    t.e[kSelCopy].m = 0u;
    return t;
}
struct Sel8Table {
    Sel8 e[kSelCopy + 1];
};
constexpr Sel8Table make_sel8_table() {
    Sel8Table t{};
    const SelTable f = make_sel_table();
    for (uint32_t i = 0; i <= kSelCopy; i++) t.e[i] = Sel8{f.e[i].s0, f.e[i].s1};
    return t;
}
__device__ constexpr Sel8Table kSel8Table = make_sel8_table();

// (Reading the 16-byte entries from global memory instead, L1-resident, left
// 8 workgroups per CU but measured 1-2 % slower: the emit waits on the
// gather.)

template <bool GAP>
struct Smem {
    Sel8 sel[kSelCopy + 1];             // record assembly per tag (s0, s1)
    uint64_t chunk_size[kMaxTileChunks];
    uint64_t chunk_pos[kMaxTileChunks];
    uint64_t wave_bytes[kWaves];
    uint64_t wave_steps[kWaves];
    uint32_t chunk_oc[kMaxTileChunks];  // staged path: chunk start in its wave's region
    uint32_t chunk_gap[GAP ? kMaxTileChunks : 1];  // leading gap bytes of each chunk
    // per-wave staging region; the streaming path uses its first 4 KiB as
    // the flush ring.  emit_step ORs a zero into the dword before a record
    // that starts 4-aligned, hence the pad.
    alignas(16) uint32_t pad[4];
    alignas(16) uint8_t stage[kWaves][kRegionBytes];
};

// Carried run state between 64-word steps of one chunk.
struct Carry {
    uint32_t type;  // 0 none, 1 zero run, 2 literal run
    uint32_t rem;   // words the open run may still absorb
};

struct StepMasks {
    uint64_t H;               // heads
    uint32_t absorbed_carry;  // words absorbed by the carried run
    Carry next;
};

__device__ __forceinline__ StepMasks resolve_step(uint64_t Zm, uint64_t Lm, uint64_t Fm,
                                                  uint32_t nvalid, Carry c) {
    StepMasks r;
    uint64_t AC = 0;
    uint32_t k = 0;
    if (c.type != 0) {
        const uint32_t lead = ctz64(~(c.type == 1 ? Zm : Lm));
        k = lead < c.rem ? lead : c.rem;
        AC = low_mask(k);
    }
    const uint64_t Z2 = Zm & ~AC;
    const uint64_t AZ = Z2 & (Z2 << 1);
    const uint64_t L2 = Lm & ~AC;
    const uint64_t F2 = Fm & ~AC;
    const uint64_t filled = ((L2 ^ (L2 + F2)) & L2) | F2;
    const uint64_t AF = filled & (filled << 1);
    const uint64_t H = low_mask(nvalid) & ~(AC | AZ | AF);
    r.H = H;
    r.absorbed_carry = k;
    if (H == 0) {
        r.next.type = c.type;
        r.next.rem = c.rem - 64;  // only reachable when the carry covered the step
    } else {
        const uint32_t h = 63u - (uint32_t)__builtin_clzll(H);
        const uint64_t hb = 1ull << h;
        r.next.type = (Zm & hb) ? 1u : ((Fm & hb) ? 2u : 0u);
        r.next.rem = r.next.type ? 255u - (63u - h) : 0u;
    }
    return r;
}

// Stores output bytes [lo, hi) (16-aligned coordinates) from the ring: byte
// stores for the unaligned head and tail, dwordx4 for the rest.
__device__ __forceinline__ void flush_range(const uint8_t* ring, uint8_t* __restrict__ out,
                                            uint64_t lo, uint64_t hi, uint32_t lane) {
    if (hi <= lo) return;
    const uint64_t a = (lo + 15) & ~15ull, b = hi & ~15ull;
    if (a > b) {  // inside one block
        if (lane < hi - lo) out[lo + lane] = ring[(lo + lane) & kRingMask];
        return;
    }
    if (lane < a - lo) out[lo + lane] = ring[(lo + lane) & kRingMask];
    for (uint64_t blk = a + 16ull * lane; blk < b; blk += 16ull * CAPNP_WAVE)
        *reinterpret_cast<uint4*>(out + blk) =
            *reinterpret_cast<const uint4*>(ring + (blk & kRingMask));
    if (lane < hi - b) out[b + lane] = ring[(b + lane) & kRingMask];
}

// Where a step's bytes go.
enum StepMode {
    MODE_SIZE = 0,   // pass A of the streaming path: sizes only
    MODE_RING = 1,   // pass B of the streaming path: 4 KiB ring + flush
    MODE_STAGE = 2,  // staged path: wave-local LDS region, copied out later
};

// Per-wave packing state of the chunk in progress (wave-uniform).
struct Packer {
    Carry carry;
    uint64_t total;     // packed bytes of the chunk so far
    uint64_t o_c;       // chunk start (absolute for RING, region-local for STAGE)
    uint64_t flushed;   // RING: everything below is stored
    uint64_t zeroed;    // RING: ring zeroed up to here
    uint64_t pend_pos;  // position of a pending run count byte
    uint32_t pend_cnt;
    bool pend;

    __device__ __forceinline__ void begin(uint64_t oc) {
        carry.type = 0;
        carry.rem = 0;
        total = 0;
        o_c = oc;
        flushed = oc;
        zeroed = oc & ~15ull;
        pend = false;
        pend_pos = 0;
        pend_cnt = 0;
    }

    template <int MODE>
    __device__ __forceinline__ static uint32_t at(uint64_t p) {
        return MODE == MODE_RING ? (uint32_t)(p & kRingMask) : (uint32_t)p;
    }

    // One 64-word step.  ext (last step only): the words past the step the
    // run left open at its end goes on to absorb (a range that ends inside a
    // chunk: msg_pack_kernel's split segment), counted into its count byte.
    template <int MODE>
    __device__ __forceinline__ void step(uint64_t w, uint32_t nvalid, bool last, uint32_t lane,
                                         uint8_t* buf, uint8_t* __restrict__ out,
                                         const Sel8* sel, uint32_t ext = 0) {
        const bool valid = lane < nvalid;
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
        const uint32_t step_bytes =
            popc64(B0) + 2 * popc64(B1) + 4 * popc64(B2) + 8 * popc64(B3);
        carry = sm.next;
        if (MODE == MODE_SIZE) {
            total += step_bytes;
            return;
        }
        const uint64_t start = o_c + total;
        if (MODE == MODE_RING && zeroed < start + kStepMax) {  // zero the next KiB
            *reinterpret_cast<uint4*>(buf + ((zeroed + 16ull * lane) & kRingMask)) =
                make_uint4(0, 0, 0, 0);
            zeroed += kZeroAhead;
            wave_lds_sync();
        }
        const uint32_t off =
            mask_rank(B0) + 2 * mask_rank(B1) + 4 * mask_rank(B2) + 8 * mask_rank(B3);
        if (size) {
            // count byte of a Z/F head: words up to the next head (or step end)
            const uint64_t later = sm.H & ~low_mask(lane + 1);
            const uint32_t cnt = later ? ctz64(later) - lane - 1 : nvalid - lane - 1 + ext;
            uint32_t r0, r1 = 0, r2 = 0;
            if (head && tag == 0) {
                r0 = cnt << 8;
            } else if (head) {
                const Sel8 e = sel[tag];
                r0 = __builtin_amdgcn_perm(hi, lo, e.s0) | tag;
                r1 = __builtin_amdgcn_perm(hi, lo, e.s1);
                r2 = __builtin_amdgcn_perm(cnt, hi, sel_s2(tag));
            } else {
                r0 = lo;
                r1 = hi;
            }
            const uint64_t pos = start + off;
            const uint32_t sh = (uint32_t)(pos & 3) * 8;
            const uint32_t e0 = r0 << sh;
            const uint32_t e1 = (uint32_t)((((uint64_t)r1 << 32) | r0) >> (32 - sh));
            const uint32_t e2 = (uint32_t)((((uint64_t)r2 << 32) | r1) >> (32 - sh));
            const uint32_t e3 = (uint32_t)((uint64_t)r2 >> (32 - sh));
            const uint32_t nd = ((uint32_t)(pos & 3) + size + 3) >> 2;
            const uint64_t d = pos & ~3ull;
            uint32_t* b32 = reinterpret_cast<uint32_t*>(buf);
            __hip_atomic_fetch_or(b32 + (at<MODE>(d) >> 2), e0, __ATOMIC_RELAXED,
                                  __HIP_MEMORY_SCOPE_WAVEFRONT);
            if (nd > 1)
                __hip_atomic_fetch_or(b32 + (at<MODE>(d + 4) >> 2), e1, __ATOMIC_RELAXED,
                                      __HIP_MEMORY_SCOPE_WAVEFRONT);
            if (nd > 2)
                __hip_atomic_fetch_or(b32 + (at<MODE>(d + 8) >> 2), e2, __ATOMIC_RELAXED,
                                      __HIP_MEMORY_SCOPE_WAVEFRONT);
            if (nd > 3)
                __hip_atomic_fetch_or(b32 + (at<MODE>(d + 12) >> 2), e3, __ATOMIC_RELAXED,
                                      __HIP_MEMORY_SCOPE_WAVEFRONT);
        }
        // resolve a count carried in from earlier steps
        if (pend) {
            pend_cnt += sm.absorbed_carry + (sm.H == 0 ? ext : 0u);
            if (sm.absorbed_carry < 64 || last) {
                wave_lds_sync();
                if (lane == 0) buf[at<MODE>(pend_pos)] = (uint8_t)pend_cnt;
                pend = false;
            }
        }
        // a Z/F head whose run reaches the end of a non-final step
        if (!last && nvalid == 64 && sm.H) {
            const uint32_t h = 63u - (uint32_t)__builtin_clzll(sm.H);
            const uint64_t hb = 1ull << h;
            if ((Zm | Fm) & hb) {
                pend = true;
                pend_cnt = 63u - h;
                const uint64_t below = low_mask(h);
                const uint32_t hoff = popc64(B0 & below) + 2 * popc64(B1 & below) +
                                      4 * popc64(B2 & below) + 8 * popc64(B3 & below);
                pend_pos = start + hoff + ((Zm & hb) ? 1u : 9u);
            }
        }
        total += step_bytes;
        if (MODE == MODE_RING) {
            wave_lds_sync();
            const uint64_t produced = o_c + total;
            const uint64_t limit = last ? produced : ((pend ? pend_pos : produced) & ~15ull);
            if (limit > flushed) {
                flush_range(buf, out, flushed, limit, lane);
                flushed = limit;
            }
        }
    }
};

__device__ __forceinline__ uint64_t lds_u64(const uint64_t* p) { return uniform64(*p); }

// Wave-wide inclusive prefix sum with DPP (VALU only): Kogge-Stone inside
// each 16-lane row, then row_bcast:15 / row_bcast:31 carry the row totals.
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t x) {
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xf, 0xf, false);  // row_shr:1
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xf, 0xf, false);  // row_shr:2
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xf, 0xf, false);  // row_shr:4
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xf, 0xf, false);  // row_shr:8
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xa, 0xf, false);  // row_bcast:15
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xc, 0xf, false);  // row_bcast:31
    return x;
}

// Staged path, two passes over the register-cached words of a wave's range.
//
// Pass 1 (size): per 64-word step, the tag, the three ballots, the run
// segmentation (resolve_step) and a DPP scan of the record sizes give every
// lane its byte position inside the wave's region.  Only sizes are needed to
// publish the tile's aggregate, so the aggregate goes out before the bytes are
// assembled and the look-back latency overlaps pass 2.
//
// Pass 2 (emit): every lane ORs its record (<= 10 bytes) into the zeroed
// region.  The count byte of a Z/F head whose run crosses into later steps is
// completed from those steps' absorbed counts (ext), so nothing is patched.
struct StepInfo {
    uint64_t H;        // heads of the step
    uint32_t pos;      // this lane's byte position in the region (per lane)
    uint32_t tag;      // this lane's tag (per lane)
    uint32_t meta;     // nvalid | first << 7 | last << 8 | chunk << 9 | kin << 16,
                       // kin = words absorbed by the run carried into the step
};

// Per lane: bit `lane` of the wave-uniform mask m ? a : b.  One VOP3
// v_cndmask with the mask as its lane-select operand, instead of a 64-bit
// shift and compare the compiler would emit for ((m >> lane) & 1).
__device__ __forceinline__ uint32_t mask_sel(uint64_t m, uint32_t a, uint32_t b) {
    uint32_t r;
    asm("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(r) : "v"(b), "v"(a), "s"(m));
    return r;
}

// Index of the lowest set bit, 0xFFFFFFFF for zero (v_ffbl_b32 as is).
__device__ __forceinline__ uint32_t ffbl(uint32_t x) {
    uint32_t r;
    asm("v_ffbl_b32 %0, %1" : "=v"(r) : "v"(x));
    return r;
}

__device__ __forceinline__ uint32_t min3_u32(uint32_t a, uint32_t b, uint32_t c) {
    return min(min(a, b), c);  // v_min3_u32
}

// The tag of a word and its popcount.  Non-zero bytes flag bit 7 of each
// byte; v_dot4 with weights 1..128 gathers the eight flags (as tag << 7)
// at full rate, where the multiply gather needs two quarter-rate v_mul_lo.
__device__ __forceinline__ uint32_t word_tag_dot(uint32_t lo, uint32_t hi) {
    const uint32_t fl = (((lo & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | lo) & 0x80808080u;
    const uint32_t fh = (((hi & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | hi) & 0x80808080u;
    const uint32_t t = __builtin_amdgcn_udot4(fl, 0x08040201u,
                                              __builtin_amdgcn_udot4(fh, 0x80402010u, 0u, false),
                                              false);
    return t >> 7;
}

// Staged path: packing state of the chunk in progress (region-local, so
// 32 bits suffice).
struct StageState {
    Carry carry;
    uint32_t total;  // packed bytes of the chunk so far
    uint32_t o_c;    // chunk start in the wave's region
    __device__ __forceinline__ void begin(uint32_t oc) {
        carry.type = 0;
        carry.rem = 0;
        total = 0;
        o_c = oc;
    }
};

[[maybe_unused]] __device__ __forceinline__ void size_step(StageState& pk, uint64_t w,
                                                           uint32_t nvalid, uint32_t lane,
                                          StepInfo& si) {
    const uint32_t tag = word_tag_dot((uint32_t)w, (uint32_t)(w >> 32));
    const uint32_t pop = __builtin_popcount(tag);
    const bool isz = tag == 0, isf = tag == 0xFF;
    const uint64_t V = low_mask(nvalid);
    const uint64_t Zm = ballot64(isz) & V;
    const uint64_t Lm = ballot64(pop >= 7) & V;
    const uint64_t Fm = ballot64(isf) & V;
    const StepMasks sm = resolve_step(Zm, Lm, Fm, nvalid, pk.carry);
    // head: 2 (Z), 10 (F), else 1 + pop; other words: 8 unless zero (lanes
    // past nvalid hold zero words)
    const uint32_t hsize = 1u + pop + ((0x101u >> pop) & 1u);
    const uint32_t size = mask_sel(sm.H, hsize, isz ? 0u : 8u);
    const uint32_t incl = wave_incl_scan(size);
    si.H = sm.H;
    si.pos = pk.o_c + pk.total + incl - size;
    si.tag = tag;
    si.meta |= sm.absorbed_carry << 16;
    pk.carry = sm.next;
    pk.total += (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
}

// size_step with less scalar work.  The
// scalar unit (one per CU, shared by the four SIMDs) was the pack kernel's
// busiest pipe: ~95 SALU ops per 64-word step in pass 1, and one more SALU op
// per step cost ~2.1 us per launch against ~1.0 us for one more VALU op
// (PACK_SALU_PAD / PACK_VALU_PAD builds, config 2).  Here:
//   * validity is folded into the tag (lanes past nvalid get 0x100, no
//     class), so the three class ballots and V are bare v_cmp masks;
//   * the carried run's absorbed words are a v_cmp mask (lane < k);
//   * the next carry reads the last head's class with one v_readlane from
//     a per-lane class code instead of testing its bit in two masks;
//   * no branches.
__device__ __forceinline__ void size_step_lean(StageState& pk, uint64_t w, uint32_t nvalid,
                                               uint32_t lane, StepInfo& si) {
    const uint32_t tag = word_tag_dot((uint32_t)w, (uint32_t)(w >> 32));
    const uint32_t pop = __builtin_popcount(tag);
    const bool valid = lane < nvalid;
    const uint32_t tv = valid ? tag : 0x100u;
    const uint64_t V = ballot64(valid);
    const uint64_t Zm = ballot64(tv == 0);
    const uint64_t Lm = ballot64(valid && pop >= 7);
    const uint64_t Fm = ballot64(tv == 0xFF);
    const Carry c = pk.carry;
    // words of the carried run's class at the step start, at most rem
    uint32_t k = ctz64(~(c.type == 1 ? Zm : Lm));
    k = k < c.rem ? k : c.rem;
    k = c.type ? k : 0u;
    const uint64_t AC = ballot64(lane < k);
    const uint64_t Z2 = Zm & ~AC;
    const uint64_t AZ = Z2 & (Z2 << 1);
    const uint64_t L2 = Lm & ~AC;
    const uint64_t F2 = Fm & ~AC;
    const uint64_t filled = ((L2 ^ (L2 + F2)) & L2) | F2;
    const uint64_t AF = filled & (filled << 1);
    const uint64_t H = V & ~(AC | AZ | AF);
    // the run open at the step end: the last head's, or the carried one
    // when it covered the whole step
    const uint32_t code = tv == 0 ? 1u : (tv == 0xFF ? 2u : 0u);
    const uint32_t h = H ? 63u - (uint32_t)__builtin_clzll(H) : 0u;
    const uint32_t th = (uint32_t)__builtin_amdgcn_readlane((int)code, h);
    pk.carry.type = H ? th : c.type;
    pk.carry.rem = H ? (th ? 192u + h : 0u) : c.rem - 64u;
    const uint32_t hsize = 1u + pop + ((0x101u >> pop) & 1u);
    const uint32_t size = mask_sel(H, hsize, tag == 0 ? 0u : 8u);
    const uint32_t incl = wave_incl_scan(size);
    si.H = H;
    si.pos = pk.o_c + pk.total + incl - size;
    si.tag = tag;
    si.meta |= k << 16;
    pk.total += (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
}


// Pass 2 of one staged step.  With `tab` (record sync index), every head
// lane also writes the entries of the sync points its record covers: words
// g + lane .. + the run (t0 = the tile's first sync word, oc = the chunk's
// start in the region); usually none or one, more only for runs of > 16
// words.  The head lane knows its own position and run length, so this is
// a few VALU ops and a masked LDS store per step.
template <bool SYNC>
__device__ __forceinline__ void emit_step(uint64_t w, const StepInfo& si, uint32_t ext,
                                          uint32_t lane, uint8_t* region_m1, const Sel8* sel,
                                          uint8_t* __restrict__ tab, uint32_t t0, uint32_t g,
                                          uint32_t oc) {
    const uint32_t lo = (uint32_t)w, hi = (uint32_t)(w >> 32);
    const uint32_t tag = si.tag;
    const uint32_t nvalid = si.meta & 127u;
    // words after this lane's record up to the next head, else to the step
    // end plus what the run absorbs in later steps: the run count of a Z/F
    // head; 0 for any other head (every word no run absorbs is a head)
    const uint64_t nxt = (si.H >> 1) >> lane;
    const uint32_t cnt = min3_u32(ffbl((uint32_t)nxt), ffbl((uint32_t)(nxt >> 32)) | 32u,
                                  __builtin_elementwise_sub_sat(nvalid + ext, lane + 1u));
    // record dwords r2:r1:r0 = tag, compacted bytes, count byte; absorbed
    // zero words and lanes past nvalid hold w == 0 and emit nothing
    const uint32_t idx = mask_sel(si.H, tag, kSelCopy);
    const Sel8 se = sel[idx];
    const uint32_t r0 = __builtin_amdgcn_perm(hi, lo, se.s0) | (((cnt << 8) | tag) & sel_m(idx));
    const uint32_t r1 = __builtin_amdgcn_perm(hi, lo, se.s1);
    const uint32_t r2 = __builtin_amdgcn_perm(cnt, hi, sel_s2(idx));
    // OR (r << 8k), k = pos & 3, into the dwords from pos & ~3.  Written as
    // alignbyte by (-pos) & 3 from the dword before ceil(pos / 4): for k = 0
    // the first dword gets zero and the rest r0..r2 unshifted.
    const uint32_t pos = si.pos;
    const uint32_t s = 0u - pos;
    const uint32_t e0 = __builtin_amdgcn_alignbyte(r0, 0u, s);
    const uint32_t e1 = __builtin_amdgcn_alignbyte(r1, r0, s);
    const uint32_t e2 = __builtin_amdgcn_alignbyte(r2, r1, s);
    const uint32_t e3 = __builtin_amdgcn_alignbyte(0u, r2, s);
    // (region_m1 = region - 1, region 16-aligned: align_down(region - 1 + pos)
    // = region + ceil(pos / 4) * 4 - 4)
    uint32_t* b32 = reinterpret_cast<uint32_t*>(__builtin_align_down(region_m1 + pos, 4));
    // (the region is zeroed, so a zero dword needs no OR: absorbed zero words
    // and lanes past the step's words would otherwise all OR into the next
    // record's dword, same-address LDS atomics that serialise; long zero runs
    // made that the larger part of the emit)
    if (e0) __hip_atomic_fetch_or(b32 + 0, e0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
    if (e1) __hip_atomic_fetch_or(b32 + 1, e1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
    if (e2) __hip_atomic_fetch_or(b32 + 2, e2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
    if (e3) __hip_atomic_fetch_or(b32 + 3, e3, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
    if constexpr (SYNC) {
        // sync points m = hw + d, d = (t0 - hw) mod kSyncWords, d <= cnt, of
        // the record headed at word hw = g + lane; m - t0 is a multiple of
        // kSyncWords, so its entry is dword (m - t0) / kSyncWords of the
        // tile's part of the index.  Other lanes get d = ~0 > cnt.  Every
        // sync point is covered by exactly one record, so the entries go
        // straight to memory.
        const uint32_t c = t0 - g;
        const uint32_t d = (c - lane) & (kSyncWords - 1);
        const uint32_t dh = mask_sel(si.H, d, ~0u);
        if (dh <= cnt) {
            const uint32_t rel = pos - oc;
            // (lane + d - c is a multiple of kSyncWords)
            uint32_t b = (lane + d - c) / (kSyncWords / 4u);
            *reinterpret_cast<uint32_t*>(tab + b) = rel | (d << 24);
            // (runs longer than kSyncWords words: rare; a plain loop costs no registers)
#pragma clang loop unroll(disable) vectorize(disable)
            for (uint32_t dd = d + kSyncWords; dd <= cnt; dd += kSyncWords) {
                b += 4;
                *reinterpret_cast<uint32_t*>(tab + b) = rel | (dd << 24);
            }
        }
    }
}

// Copies region bytes [0, len) to out[D0 .. D0+len) (16-aligned coordinates),
// never writing at or past `cap`.
__device__ __forceinline__ void copy_out(const uint8_t* region, uint8_t* __restrict__ out,
                                         uint64_t D0, uint64_t len, uint64_t cap,
                                         uint32_t lane) {
    const uint64_t lo = D0;
    const uint64_t hi = (D0 + len < cap) ? D0 + len : cap;
    if (hi <= lo) return;
    const uint64_t a = (lo + 15) & ~15ull, b = hi & ~15ull;
    if (a > b) {
        if (lane < hi - lo) out[lo + lane] = region[lane];
        return;
    }
    if (lane < a - lo) out[lo + lane] = region[lane];
    const uint32_t m = (uint32_t)((a - D0) & 15);  // source misalignment (uniform)
    const uint32_t q = m >> 2, sb = m & 3;
    for (uint64_t blk = a + 16ull * lane; blk < b; blk += 16ull * CAPNP_WAVE) {
        const uint32_t s = (uint32_t)(blk - D0) & ~15u;
        const uint4 A = *reinterpret_cast<const uint4*>(region + s);
        const uint4 B = *reinterpret_cast<const uint4*>(region + s + 16);
        const uint32_t w[8] = {A.x, A.y, A.z, A.w, B.x, B.y, B.z, B.w};
        uint4 o;
        if (q == 0) {
            o = make_uint4(__builtin_amdgcn_alignbyte(w[1], w[0], sb),
                           __builtin_amdgcn_alignbyte(w[2], w[1], sb),
                           __builtin_amdgcn_alignbyte(w[3], w[2], sb),
                           __builtin_amdgcn_alignbyte(w[4], w[3], sb));
        } else if (q == 1) {
            o = make_uint4(__builtin_amdgcn_alignbyte(w[2], w[1], sb),
                           __builtin_amdgcn_alignbyte(w[3], w[2], sb),
                           __builtin_amdgcn_alignbyte(w[4], w[3], sb),
                           __builtin_amdgcn_alignbyte(w[5], w[4], sb));
        } else if (q == 2) {
            o = make_uint4(__builtin_amdgcn_alignbyte(w[3], w[2], sb),
                           __builtin_amdgcn_alignbyte(w[4], w[3], sb),
                           __builtin_amdgcn_alignbyte(w[5], w[4], sb),
                           __builtin_amdgcn_alignbyte(w[6], w[5], sb));
        } else {
            o = make_uint4(__builtin_amdgcn_alignbyte(w[4], w[3], sb),
                           __builtin_amdgcn_alignbyte(w[5], w[4], sb),
                           __builtin_amdgcn_alignbyte(w[6], w[5], sb),
                           __builtin_amdgcn_alignbyte(w[7], w[6], sb));
        }
        *reinterpret_cast<uint4*>(out + blk) = o;
    }
    if (lane < hi - b) out[b + lane] = region[(b - D0) + lane];
}

// The same for a whole tile whose waves' bytes lie back to back in LDS
// (PACK_TILECOPY): the tile's 16-byte output blocks are cut into one range
// per wave, and only the tile's two edges take byte stores.
__device__ __forceinline__ void copy_out_tile(const uint8_t* region, uint8_t* __restrict__ out,
                                              uint64_t D0, uint64_t len, uint64_t cap,
                                              uint32_t lane, uint32_t wave) {
    const uint64_t lo = D0;
    const uint64_t hi = (D0 + len < cap) ? D0 + len : cap;
    if (hi <= lo) return;
    const uint64_t a = (lo + 15) & ~15ull, b = hi & ~15ull;
    if (a > b) {
        if (wave == 0 && lane < hi - lo) out[lo + lane] = region[lane];
        return;
    }
    if (wave == 0 && lane < a - lo) out[lo + lane] = region[lane];
    if (wave == kWaves - 1 && lane < hi - b) out[b + lane] = region[(b - D0) + lane];
    const uint32_t nb = (uint32_t)((b - a) >> 4);
    const uint32_t k0 = nb * wave / kWaves, k1 = nb * (wave + 1) / kWaves;
    const uint32_t m = (uint32_t)((a - D0) & 15);  // source misalignment (uniform)
    const uint32_t q = m >> 2, sb = m & 3;
    for (uint32_t k = k0 + lane; k < k1; k += CAPNP_WAVE) {
        const uint64_t blk = a + 16ull * k;
        const uint32_t s = (uint32_t)(blk - D0) & ~15u;
        const uint4 A = *reinterpret_cast<const uint4*>(region + s);
        const uint4 B = *reinterpret_cast<const uint4*>(region + s + 16);
        const uint32_t w[8] = {A.x, A.y, A.z, A.w, B.x, B.y, B.z, B.w};
        uint4 o;
        if (q == 0) {
            o = make_uint4(__builtin_amdgcn_alignbyte(w[1], w[0], sb),
                           __builtin_amdgcn_alignbyte(w[2], w[1], sb),
                           __builtin_amdgcn_alignbyte(w[3], w[2], sb),
                           __builtin_amdgcn_alignbyte(w[4], w[3], sb));
        } else if (q == 1) {
            o = make_uint4(__builtin_amdgcn_alignbyte(w[2], w[1], sb),
                           __builtin_amdgcn_alignbyte(w[3], w[2], sb),
                           __builtin_amdgcn_alignbyte(w[4], w[3], sb),
                           __builtin_amdgcn_alignbyte(w[5], w[4], sb));
        } else if (q == 2) {
            o = make_uint4(__builtin_amdgcn_alignbyte(w[3], w[2], sb),
                           __builtin_amdgcn_alignbyte(w[4], w[3], sb),
                           __builtin_amdgcn_alignbyte(w[5], w[4], sb),
                           __builtin_amdgcn_alignbyte(w[6], w[5], sb));
        } else {
            o = make_uint4(__builtin_amdgcn_alignbyte(w[4], w[3], sb),
                           __builtin_amdgcn_alignbyte(w[5], w[4], sb),
                           __builtin_amdgcn_alignbyte(w[6], w[5], sb),
                           __builtin_amdgcn_alignbyte(w[7], w[6], sb));
        }
        *reinterpret_cast<uint4*>(out + blk) = o;
    }
}

// Streaming path: wave w owns chunks w, w+4, ...  MODE_SIZE fills
// chunk_size; MODE_RING re-reads and writes at chunk_pos.
template <int MODE, uint32_t NWV = kWaves>
__device__ void run_streaming(const uint64_t* __restrict__ in, const uint64_t* off,
                              uint64_t* chunk_size, const uint64_t* chunk_pos, uint32_t nc,
                              uint32_t wave, uint32_t lane, uint8_t* ring, const Sel8* sel,
                              uint8_t* out, uint32_t mis, uint64_t out_cap,
                              const uint32_t* cgap, uint64_t* last_size = nullptr) {
    Packer pk;
    for (uint32_t ci = wave; ci < nc; ci += NWV) {
        const uint64_t woff = uniform64(off[ci]);
        const uint64_t len = uniform64(off[ci + 1]) - woff;
        const uint32_t g = cgap ? uniform(cgap[ci]) : 0u;  // leading gap bytes
        if (len == 0) {
            if (MODE == MODE_SIZE && lane == 0) chunk_size[ci] = g;
            continue;
        }
        if (MODE == MODE_RING) {
            const uint64_t pos = lds_u64(&chunk_pos[ci]);
            if (pos + lds_u64(&chunk_size[ci]) > out_cap) continue;  // does not fit
            pk.begin(pos + g + mis);
        } else {
            pk.begin(0);
        }
        const uint64_t* src = in + woff;
        uint64_t wnext = lane < len ? src[lane] : 0;
        for (uint64_t base = 0;; base += 64) {
            const uint32_t nvalid = (uint32_t)((len - base) < 64 ? len - base : 64);
            const bool last = base + 64 >= len;
            const uint64_t w = wnext;
            if (!last) wnext = (base + 64 + lane < len) ? src[base + 64 + lane] : 0;
            pk.step<MODE>(w, nvalid, last, lane, ring, out, sel);
            if (last) break;
        }
        if (MODE == MODE_SIZE && lane == 0) chunk_size[ci] = pk.total + g;
        // (RING: the size of the last chunk, which its caller did not size)
        if (MODE == MODE_RING && last_size && ci + 1 == nc && lane == 0) *last_size = pk.total + g;
    }
}


// ---------------------------------------------------------------------------
// Word tiles (batches of long chunks): the batch is one word stream in which
// every chunk start is a forced record head, cut into tiles of kWtTile words
// and wave ranges of kWtRange words wherever those boundaries fall.  A range
// that starts inside a record needs the run state there (carry_into), and a
// run left open at its end needs the words it goes on to absorb (run_ext);
// both come from the words around the boundary.
constexpr uint32_t kWtRange = 64 * kStageSteps;  // words per wave range
constexpr uint32_t kWtTile = kWaves * kWtRange;  // words per tile

struct LookbackArgs {
    uint64_t* ts;
    uint64_t* gs;
    uint64_t ntiles;
    const uint64_t* in;
    const uint64_t* chunk_off;
    uint64_t nchunks;
    uint32_t tc;
    const uint32_t* gap;
    // word tiles: the batch's words [wlo, whi), tile t = global tile g0 + t
    uint32_t wt;
    uint64_t wlo, whi, g0;
    const uint64_t* map;  // first chunk starting at or after each wave range
};

// Run segmentation of one step with forced heads S (chunk starts) and
// `nvalid` valid words: the heads, the words the carried run absorbs, and
// the run state after the step's last valid word.  As resolve_step, plus:
// no run absorbs a chunk start (zero runs: Z' & (Z' << 1) & ~S; literal runs:
// the L runs are cut before every chunk start, and a 0xFF head at a chunk
// start opens its run at the next word).
__device__ __forceinline__ StepMasks resolve_step_s(uint64_t Zm, uint64_t Lm, uint64_t Fm,
                                                    uint64_t Sm, uint32_t nvalid, Carry c) {
    StepMasks r;
    uint64_t AC = 0;
    uint32_t k = 0;
    if (c.type != 0) {
        const uint32_t lead = ctz64(~(c.type == 1 ? Zm : Lm));
        const uint32_t cut = ctz64(Sm);
        k = min(min(lead, c.rem), cut);
        AC = low_mask(k);
    }
    const uint64_t Z2 = Zm & ~AC;
    const uint64_t AZ = Z2 & (Z2 << 1) & ~Sm;
    const uint64_t L2 = Lm & ~AC & ~Sm;
    const uint64_t F2 = Fm & ~AC;
    const uint64_t F3 = (F2 & ~Sm) | (((F2 & Sm) << 1) & L2);
    const uint64_t filled = ((L2 ^ (L2 + F3)) & L2) | F2;
    const uint64_t AF = filled & (filled << 1) & ~Sm;
    const uint64_t H = low_mask(nvalid) & ~(AC | AZ | AF);
    r.H = H;
    r.absorbed_carry = k;
    if (H == 0) {
        r.next.type = c.type;
        r.next.rem = c.rem - nvalid;  // the carry covered the valid words
    } else {
        const uint32_t h = 63u - (uint32_t)__builtin_clzll(H);
        const uint64_t hb = 1ull << h;
        r.next.type = (Zm & hb) ? 1u : ((Fm & hb) ? 2u : 0u);
        r.next.rem = r.next.type ? 255u - (nvalid - 1u - h) : 0u;
    }
    return r;
}

// Word i (after its chunk's first word) is a record head whatever came
// before when: it is zero after a non-zero word, or non-zero after a zero
// word (a zero run absorbs only zero words, a 0xFF run only words with at
// most one zero byte); it has 2..7 zero bytes (nothing absorbs it); or it has
// at most one zero byte after a word with 2..7 zero bytes (a head that opens
// no run).
__device__ __forceinline__ bool sure_head(uint32_t tag, uint32_t ptag) {
    const uint32_t pop = __builtin_popcount(tag), ppop = __builtin_popcount(ptag);
    const bool z = tag == 0, pz = ptag == 0;
    const bool brk = !z && pop <= 6, pbrk = !pz && ppop <= 6;
    return z != pz || brk || (pop >= 7 && pbrk);
}

__device__ __forceinline__ uint32_t tag_of(uint64_t w) {
    return word_tag_dot((uint32_t)w, (uint32_t)(w >> 32));
}

// Run state entering word R of the chunk starting at cs (cs < R): from the
// last sure head s before R, heads fall every 256 words while the words are
// all zero or all 0xFF-tagged; otherwise the steps from s are resolved.
__device__ Carry carry_into(const uint64_t* __restrict__ in, uint64_t cs, uint64_t R,
                            uint32_t lane) {
    uint64_t s = cs;
    bool allz = true, allf = true;  // over [s, R)
    for (uint64_t hi = R; hi > cs;) {
        const uint64_t lo = hi - cs > 64 ? hi - 64 : cs;
        const uint64_t i = lo + lane;
        const bool v = i < hi;
        const uint32_t tag = v ? tag_of(in[i]) : 0u;
        const uint32_t ptag = (v && i > cs) ? tag_of(in[i - 1]) : 0u;
        const uint64_t G = ballot64(v && (i == cs || sure_head(tag, ptag)));
        const uint32_t j = G ? 63u - (uint32_t)__builtin_clzll(G) : 0u;
        const bool mine = v && lane >= j;
        allz = allz && ballot64(mine && tag != 0) == 0;
        allf = allf && ballot64(mine && tag != 0xFF) == 0;
        if (G) {
            s = lo + j;
            break;
        }
        hi = lo;
    }
    if (allz || allf) {
        const uint64_t h = s + (R - 1 - s) / 256 * 256;  // the last head before R
        return Carry{allz ? 1u : 2u, (uint32_t)(255u - (R - 1 - h))};
    }
    Carry c{0, 0};
    for (uint64_t p = s; p < R; p += 64) {
        const uint32_t nv = (uint32_t)(R - p < 64 ? R - p : 64);
        const uint32_t tag = lane < nv ? tag_of(in[p + lane]) : 0u;
        const uint32_t pop = __builtin_popcount(tag);
        const uint64_t V = low_mask(nv);
        const StepMasks sm = resolve_step_s(ballot64(tag == 0) & V, ballot64(pop >= 7) & V,
                                            ballot64(tag == 0xFF) & V, 0, nv, c);
        c = sm.next;
    }
    return c;
}

// Chunk-start bits of a word-tile batch (pack_wt_bits): bit i & 63 of
// cb[1 + (i >> 6) - b64] is set when a chunk starts at word i (b64 = the
// batch's first word >> 6; cb[0] and a tail are zero guards).  The 64 bits
// for words p .. p + 63 (p >= 64 (b64 - 1)):
__device__ __forceinline__ uint64_t start_bits(const uint64_t* __restrict__ cb, uint64_t b64,
                                               uint64_t p) {
    const uint64_t q = 1 + (p >> 6) - b64;
    const uint32_t r = (uint32_t)(p & 63);
    const uint64_t lo = cb[q];
    return r ? (lo >> r) | (cb[q + 1] << (64 - r)) : lo;
}

// start_bits for a signed first word p > 64 (b64 - 1) - 64 (a window that
// may begin before word 0).
__device__ __forceinline__ uint64_t start_bits_s(const uint64_t* __restrict__ cb, uint64_t b64,
                                                 int64_t p) {
    const uint64_t q = (uint64_t)(1 + (p >> 6) - (int64_t)b64);  // (p >> 6: floor)
    const uint32_t r = (uint32_t)(p & 63);
    const uint64_t lo = cb[q];
    return r ? (lo >> r) | (cb[q + 1] << (64 - r)) : lo;
}

// The run state entering word R from the 64 words before it (w = word
// R - 64 + lane, wp = word R - 65, bits = their chunk-start bits): the last
// sure head or chunk start s before R, then heads every 256 words through an
// all-zero / all-0xFF stretch, or one resolved step.  Deeper stretches load
// eight windows (words and bits) per round.
// W: the words examined first are R - W .. R - 1 (lanes 64 - W ..; wp = word
// R - W - 1): with random data nearly every word is a sure head, so a short
// window decides almost every range and the deep search takes the rest.
// NW: windows loaded per round of the deep search (fewer: fewer registers,
// for a caller whose deep searches are rare).
template <uint32_t W = 64, int NW = 8>
__device__ __forceinline__ Carry carry_in_b(const uint64_t* __restrict__ in,
                                            const uint64_t* __restrict__ cb, uint64_t b64,
                                            uint64_t wlo, uint64_t R, uint32_t lane, uint64_t w,
                                            uint64_t wp, uint64_t bits) {
    // word R - 64 + lane is in the window and at or past wlo
    const bool v = (int)lane >= 64 - (int)W && R + lane >= 64 + wlo;
    const uint32_t tag = v ? tag_of(w) : 0u;
    const uint32_t up = (uint32_t)__shfl_up((int)tag, 1, 64);
    const uint32_t ptag = lane != 64u - W ? up : tag_of(wp);  // (W = 64: lane 0)
    const uint64_t G = ballot64(v && (((bits >> lane) & 1) || sure_head(tag, ptag)));
    if (G) {
        const uint32_t j = 63u - (uint32_t)__builtin_clzll(G);
        const uint64_t s = R - 64 + j;
        const bool mine = lane >= j;
        const bool allz = ballot64(mine && tag != 0) == 0, allf = ballot64(mine && tag != 0xFF) == 0;
        if (allz || allf) {
            const uint64_t h = s + (R - 1 - s) / 256 * 256;
            return Carry{allz ? 1u : 2u, (uint32_t)(255u - (R - 1 - h))};
        }
        const uint32_t pop = __builtin_popcount(tag);
        const uint64_t Vj = ~low_mask(j);
        return resolve_step_s(ballot64(tag == 0) & Vj, ballot64(pop >= 7) & Vj,
                              ballot64(tag == 0xFF) & Vj, 1ull << j, 64, Carry{0, 0}).next;
    }
    bool allz = ballot64(v && tag != 0) == 0, allf = ballot64(v && tag != 0xFF) == 0;
    constexpr uint64_t kSpan = 64ull * NW;
    for (uint64_t hi = R - W; hi > wlo; hi = hi > wlo + kSpan ? hi - kSpan : wlo) {
        uint32_t t[NW];
        uint64_t bk[NW];
        {
            uint64_t x[NW];
#pragma unroll
            for (int k = 0; k < NW; k++) {
                const uint64_t lo = hi - 64 * (k + 1);  // (may wrap below 0: then invalid)
                const bool inb = hi >= wlo + 64ull * (k + 1) - lane;  // lo + lane >= wlo
                x[k] = inb ? in[lo + lane] : 0ull;
                // (words lo .. lo + 63 reach the batch: lo >= 0 and lo + 64 > wlo)
                // (signed: with W < 64 the windows are not 64-aligned, so one
                // can start below word 0 and still hold valid words; cb[0]
                // is the zero guard for the 64 words before the batch's first
                // 64-word block, so any window overlapping the batch is
                // covered)
                const int64_t slo = (int64_t)hi - 64ll * (k + 1);
                bk[k] = slo + 64 <= (int64_t)wlo ? 0ull : start_bits_s(cb, b64, slo);
            }
#pragma unroll
            for (int k = 0; k < NW; k++) t[k] = tag_of(x[k]);
        }
        int kf = -1;
        uint64_t s = wlo;
#pragma unroll
        for (int k = 0; k < NW; k++) {
            const bool vk = hi >= wlo + 64ull * (k + 1) - lane;
            const uint32_t tk = vk ? t[k] : 0u;
            const uint32_t pt0 = (uint32_t)__shfl_up((int)tk, 1, 64);
            const uint32_t below = k < NW - 1 ? (uint32_t)__shfl((int)t[k < NW - 1 ? k + 1 : NW - 1], 63, 64) : 0u;
            const uint32_t pt = lane ? pt0 : below;
            const bool sure = vk && (((bk[k] >> lane) & 1) || ((lane || k < NW - 1) && sure_head(tk, pt)));
            const uint64_t Gk = ballot64(sure);
            if (kf < 0) {
                if (Gk) {
                    const uint32_t j = 63u - (uint32_t)__builtin_clzll(Gk);
                    kf = k;
                    s = hi - 64 * (k + 1) + j;
                    allz = allz && ballot64(lane >= j && tk != 0) == 0;
                    allf = allf && ballot64(lane >= j && tk != 0xFF) == 0;
                } else {
                    allz = allz && ballot64(tk != 0) == 0;
                    allf = allf && ballot64(tk != 0xFF) == 0;
                }
            }
        }
        if (kf >= 0) {
            if (allz || allf) {
                const uint64_t h = s + (R - 1 - s) / 256 * 256;
                return Carry{allz ? 1u : 2u, (uint32_t)(255u - (R - 1 - h))};
            }
            Carry c{0, 0};  // rare: resolve forward from s
            for (uint64_t p = s; p < R; p += 64) {
                const uint32_t nv = (uint32_t)(R - p < 64 ? R - p : 64);
                const uint32_t tt = lane < nv ? tag_of(in[p + lane]) : 0u;
                const uint32_t pop = __builtin_popcount(tt);
                const uint64_t V = low_mask(nv);
                c = resolve_step_s(ballot64(tt == 0) & V, ballot64(pop >= 7) & V,
                                   ballot64(tt == 0xFF) & V, start_bits(cb, b64, p) & V, nv, c)
                        .next;
            }
            return c;
        }
    }
    return Carry{0, 0};  // (not reached: the batch's first word is a chunk start)
}

// Words from R on that the open run c absorbs, up to the next chunk start
// or the batch end (w = word R + lane, bits = chunk-start bits of R ..).
__device__ __forceinline__ uint32_t run_ext_b(const uint64_t* __restrict__ in,
                                              const uint64_t* __restrict__ cb, uint64_t b64,
                                              uint64_t whi, uint64_t R, Carry c, uint32_t lane,
                                              uint64_t w, uint64_t bits) {
    if (c.type == 0 || c.rem == 0) return 0;
    uint32_t ext = 0;
    for (uint64_t p = R; p < whi; p += 64) {
        if (p != R) {
            w = p + lane < whi ? in[p + lane] : 0ull;
            bits = start_bits(cb, b64, p);
        }
        const uint32_t room = (uint32_t)(whi - p < 64 ? whi - p : 64);
        const uint32_t cut = ctz64(bits);
        const uint32_t nv = cut < room ? cut : room;
        const uint32_t tag = tag_of(w);
        const bool cls = c.type == 1 ? tag == 0 : __builtin_popcount(tag) >= 7;
        const uint32_t lead = ctz64(~ballot64(lane < nv && cls));
        ext += lead;
        if (lead < 64 || ext >= c.rem) break;
    }
    return ext < c.rem ? ext : c.rem;
}


__device__ __forceinline__ void wt_tile_bounds(const LookbackArgs& A, uint64_t t, uint64_t& Ta,
                                               uint64_t& Tb) {
    const uint64_t g = A.g0 + t;
    Ta = g * kWtTile > A.wlo ? g * kWtTile : A.wlo;
    Tb = (g + 1) * kWtTile < A.whi ? (g + 1) * kWtTile : A.whi;
}

// Packed bytes of words [R0, R1) (one wave; the look-back fallback).
__device__ uint64_t wt_range_size(const LookbackArgs& A, uint64_t R0, uint64_t R1, uint64_t cA,
                                  uint32_t lane) {
    const uint64_t* off = A.chunk_off;
    Carry c{0, 0};
    if (uniform64(off[cA]) != R0) c = carry_into(A.in, uniform64(off[cA - 1]), R0, lane);
    uint64_t total = 0, cp = cA;
    for (uint64_t p = R0; p < R1; p += 64) {
        const uint32_t nv = (uint32_t)(R1 - p < 64 ? R1 - p : 64);
        uint64_t S = 0;
        while (cp <= A.nchunks && uniform64(off[cp]) < p + nv) {
            S |= 1ull << (uniform64(off[cp]) - p);
            cp++;
        }
        const uint32_t tag = lane < nv ? tag_of(A.in[p + lane]) : 0u;
        const uint32_t pop = __builtin_popcount(tag);
        const uint64_t V = low_mask(nv);
        const StepMasks sm = resolve_step_s(ballot64(tag == 0) & V, ballot64(pop >= 7) & V,
                                            ballot64(tag == 0xFF) & V, S, nv, c);
        const bool head = (sm.H >> lane) & 1;
        const uint32_t size = lane >= nv ? 0u : head ? 1u + pop + ((0x101u >> pop) & 1u)
                                                     : (tag ? 8u : 0u);
        uint64_t v = size;
        for (uint32_t d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d, 64);
        total += v;
        c = sm.next;
    }
    return total;
}

__device__ uint64_t wt_tile_size(const LookbackArgs& A, uint64_t t, uint32_t lane) {
    uint64_t Ta, Tb, total = 0;
    wt_tile_bounds(A, t, Ta, Tb);
    for (uint32_t w = 0; w < kWaves; w++) {
        const uint64_t R0 = Ta + (uint64_t)w * kWtRange;
        if (R0 >= Tb) break;
        const uint64_t R1 = R0 + kWtRange < Tb ? R0 + kWtRange : Tb;
        total += wt_range_size(A, R0, R1, uniform64(A.map[t * kWaves + w]), lane);
    }
    return total;
}

// Packed size of tile j computed by one wave from the input (the look-back
// fallback below; normally never executed).
__device__ uint64_t tile_aggregate(const LookbackArgs& A, uint64_t j, uint32_t lane) {
    if (A.wt) return wt_tile_size(A, j, lane);
    const uint64_t* __restrict__ in = A.in;
    const uint64_t* __restrict__ chunk_off = A.chunk_off;
    const uint64_t nchunks = A.nchunks;
    const uint32_t tc = A.tc;
    const uint32_t* __restrict__ gap = A.gap;
    const uint64_t c0 = j * tc;
    const uint64_t c1 = (c0 + tc < nchunks) ? c0 + tc : nchunks;
    uint64_t total = 0;
    for (uint64_t ci = c0; ci < c1; ci++) {
        const uint64_t woff = uniform64(chunk_off[ci]);
        const uint64_t len = uniform64(chunk_off[ci + 1]) - woff;
        Packer pk;
        pk.begin(0);
        for (uint64_t base = 0; base < len; base += 64) {
            const uint32_t nvalid = (uint32_t)((len - base) < 64 ? len - base : 64);
            const uint64_t w = lane < nvalid ? in[woff + base + lane] : 0;
            pk.step<MODE_SIZE>(w, nvalid, base + 64 >= len, lane, nullptr, nullptr, nullptr);
        }
        total += pk.total + (gap ? gap[ci] : 0u);
    }
    return total;
}

// Two-level decoupled look-back.  Tile records ts[t] ({flag, value}
// granules) carry each tile's aggregate, published as soon as the tile's
// sizes are known (before its bytes are assembled, so the wait overlaps pass
// 2).  The last tile of each group of 64 publishes the group aggregate, and
// once known the group's inclusive prefix, in gs[g].  A tile's offset = its
// group's earlier tiles (one 64-record load) + the group's exclusive prefix
// (64 groups = 4096 tiles per load).
//
// The records live in uncached device memory (capi.hip), so relaxed
// agent-scope loads and stores meet at memory: in cached (hipMalloc) memory
// a poll is served by the reader XCD's L2 and can stay stale for tens of
// microseconds after another XCD's store.  Measured alternatives (round 1,
// config 2): hipMalloc'd records 1154 us/launch, uncached 748 us; adding
// per-group atomic totals (memory-side atomics) 2295 us; issuing the first
// polls before pass 2 822 us.  Round 3 (pack_cs_kernel, config 2): polling
// the group's tiles and the group window together, one round trip when all
// is published, 524 vs 506 us (the tile's wait is the group chain, not the
// polls); a persistent grid pipelining each tile's look-back behind the next
// tile's pass 1 (4 workgroups per CU) 1262 vs 472 us.  Round 5 (config 2,
// with the index): the first group window read in the same round trip as the
// group's tile records: 453.5 vs 442.7 us, carsales 476.7 vs 462.5; the
// look-back still takes 2.9 us because both polls fail about once a tile
// (scripts/pack_prof.py: 1.0 failed tile polls and 1.0 -> 1.7 failed window
// polls per tile; profiles/r05x_pack_lookback.txt).  A second copy of each
// poll issued 4 / 8 / 16 x 64 cycles after the first (used when the first
// misses, so a miss costs that delay instead of a round trip): 449 / 447 /
// 444 vs 434.5 us, carsales 480 / 479 / 472 vs 461 -- the extra uncached
// reads cost more than the round trips they save.  Groups of 31 / 47 tiles:
// 466 / 455 vs 444 us (config 2), 483 / 469 vs 461 (carsales); 63 stays.
//
// Every wait is bounded: on timeout the waiter computes the missing aggregate
// itself from the input (records are idempotent), so the kernel finishes with
// the right answer under any workgroup dispatch order.
#ifndef PACK_GROUP
#define PACK_GROUP 63
#endif
constexpr uint32_t kGroup = PACK_GROUP;  // tiles per look-back group (<= 64: one lane per tile)
constexpr int kSleep = 2;        // s_sleep between look-back polls (x 64 cycles)
// group records per poll; measured: 64 -> 564 us, 16 -> 552, 4 -> 555, 1 -> 603
constexpr uint32_t kGroupWindow = 16;
constexpr uint32_t kSpinLimit = 4096;

__device__ uint64_t group_aggregate(const LookbackArgs& A, uint64_t g, uint32_t lane) {
    uint64_t* __restrict__ ts = A.ts;
    const uint64_t ntiles = A.ntiles;
    const uint64_t t0 = g * kGroup;
    const uint64_t tn = (t0 + kGroup < ntiles) ? kGroup : ntiles - t0;
    uint64_t st = lane < tn ? poll_agent(&ts[t0 + lane]) : kFlagAgg;
    uint64_t miss = ballot64((st >> 62) == 0);
    while (miss) {
        const uint32_t k = ctz64(miss);
        const uint64_t a = tile_aggregate(A, t0 + k, lane);
        if (lane == 0) publish_agent(&ts[t0 + k], kFlagAgg | a);
        if (lane == k) st = kFlagAgg | a;
        miss &= miss - 1;
    }
    uint64_t v = st & kValMask;
    for (uint32_t d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d, 64);
    return v;
}

// Wave 0: publishes tile t's aggregate.
__device__ __forceinline__ void publish(const LookbackArgs& A, uint64_t t, uint64_t agg,
                                        uint32_t lane) {
    if (lane == 0) publish_agent(&A.ts[t], kFlagAgg | agg);
}

// Wave 0: global byte offset of tile t (aggregate already published).
__device__ uint64_t lookback(const LookbackArgs& A, uint64_t t, uint64_t agg, uint32_t lane,
                             bool early_group = false) {
    const uint64_t g = t / kGroup;
    const uint32_t r = (uint32_t)(t % kGroup);
#if PACK_PROF
    const uint64_t tp0 = __builtin_amdgcn_s_memtime();
    uint32_t n_ws = 0, n_gs = 0, n_win = 0;
#endif
    // aggregates of the group's earlier tiles
    uint64_t within;
    uint64_t st = lane < r ? poll_agent(&A.ts[g * kGroup + lane]) : kFlagAgg;
    for (uint32_t spins = 0;;) {
        const uint64_t miss = ballot64((st >> 62) == 0);
        if (!miss) break;
#if PACK_PROF
        n_ws++;
#endif
        if (++spins >= kSpinLimit) {
            if (lane == 0) PROF_ADD(2, 1);
            const uint64_t j = g * kGroup + ctz64(miss);
            const uint64_t a = tile_aggregate(A, j, lane);
            if (lane == 0) publish_agent(&A.ts[j], kFlagAgg | a);
        } else {
            __builtin_amdgcn_s_sleep(kSleep);
        }
        st = lane < r ? poll_agent(&A.ts[g * kGroup + lane]) : kFlagAgg;
    }
    {
        uint64_t v = st & kValMask;
        for (uint32_t d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d, 64);
        within = v;
    }
#if PACK_PROF == 3
    if (lane == 0) TRACE(t, 7, RT());  // (the group's earlier tiles are summed)
#endif
    const bool group_last = (r == kGroup - 1) || (t + 1 == A.ntiles);
    if (group_last && !early_group && lane == 0) publish_agent(&A.gs[g], kFlagAgg | (within + agg));
    // exclusive prefix of the group: 64 groups per round; a group contributes
    // its inclusive record (and ends the scan), else its aggregate
    uint64_t gexcl = 0;
    int64_t idx = (int64_t)g - 1;
    for (uint32_t spins = 0; idx >= 0;) {
        const int64_t j = idx - (int64_t)lane;
        const bool in_win = lane < kGroupWindow;
        const uint64_t rec =
            !in_win ? 0 : (j >= 0 ? poll_agent(&A.gs[j]) : kFlagInc);
        const uint64_t inc = ballot64((rec & kFlagInc) != 0);
        const uint32_t first_inc = ctz64(inc);
        const uint64_t need = first_inc < 64 ? low_mask(first_inc) : low_mask(kGroupWindow);
        const uint64_t missing = ballot64((rec >> 62) == 0) & need;
#if PACK_PROF
        n_win++;
#endif
        if (missing) {
#if PACK_PROF
            n_gs++;
#endif
            if (++spins >= kSpinLimit) {
                const uint64_t jg = (uint64_t)(idx - (int64_t)ctz64(missing));
                const uint64_t a = group_aggregate(A, jg, lane);
                if (lane == 0) publish_agent(&A.gs[jg], kFlagAgg | a);
            } else {
                __builtin_amdgcn_s_sleep(kSleep);
            }
            continue;
        }
        uint64_t val = (lane <= first_inc) ? (rec & kValMask) : 0;
        for (uint32_t d = 32; d >= 1; d >>= 1) val += __shfl_xor(val, d, 64);
        gexcl += val;
        if (first_inc < 64) break;
        idx -= kGroupWindow;
        spins = 0;
    }
    if (group_last && lane == 0) publish_agent(&A.gs[g], kFlagInc | (gexcl + within + agg));
#if PACK_PROF == 1
    if (lane == 0) {
        TRACE(t, 5, n_ws);
        TRACE(t, 6, n_gs);
        TRACE(t, 7, n_win);
    }
#endif
#if PACK_PROF
    (void)tp0;
    (void)n_ws;
    (void)n_gs;
    (void)n_win;
#endif
    return gexcl + within;
}

__device__ __forceinline__ uint64_t tile_offset(const LookbackArgs& A, uint64_t t, uint64_t agg,
                                                uint32_t lane, bool early_group = false) {
    return lookback(A, t, agg, lane, early_group);
}

// The group aggregate, published by the group's last tile from a wave that
// polls the group's earlier tile records right after pass 1:
// in `lookback` it is published by wave 0 only after its pass 2 and that
// poll, and the next group's tiles wait on it.  (A compare-and-swap from
// empty: it never overwrites the inclusive record wave 0 publishes later.)

__device__ void publish_group_early(const LookbackArgs& A, uint64_t t, uint64_t agg,
                                    uint32_t lane) {
    const uint64_t g = t / kGroup;
    const uint32_t r = (uint32_t)(t % kGroup);
    uint64_t st = lane < r ? poll_agent(&A.ts[g * kGroup + lane]) : kFlagAgg;
    for (uint32_t spins = 0;;) {
        const uint64_t miss = ballot64((st >> 62) == 0);
        if (!miss) break;
        if (++spins >= kSpinLimit) {
            const uint64_t j = g * kGroup + ctz64(miss);
            const uint64_t a = tile_aggregate(A, j, lane);
            if (lane == 0) publish_agent(&A.ts[j], kFlagAgg | a);
        } else {
            __builtin_amdgcn_s_sleep(kSleep);
        }
        st = lane < r ? poll_agent(&A.ts[g * kGroup + lane]) : kFlagAgg;
    }
    uint64_t v = st & kValMask;
    for (uint32_t d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d, 64);
    if (lane == 0) {
        uint64_t expected = 0;
        __hip_atomic_compare_exchange_strong(&A.gs[g], &expected, kFlagAgg | (v + agg),
                                             __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_AGENT);
    }
}

// Wave 0: exclusive scan of the tile's chunk sizes (<= 64) into chunk_pos
// (tile-relative); returns the tile aggregate.
// Staged path: the tile's packed bytes fit 32 bits (<= 4 regions), so the
// scan is the DPP wave scan.
template <class SM>
__device__ __forceinline__ uint64_t scan_chunks32(SM& sm, uint32_t nc, uint32_t lane) {
    const uint32_t v = lane < nc ? (uint32_t)sm.chunk_size[lane] : 0u;
    const uint32_t incl = wave_incl_scan(v);
    if (lane < nc) sm.chunk_pos[lane] = incl - v;
    return (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
}

template <class SM>
__device__ __forceinline__ uint64_t scan_chunks(SM& sm, uint32_t nc, uint32_t lane) {
    const uint64_t v = lane < nc ? sm.chunk_size[lane] : 0;
    uint64_t s = v;
    for (uint32_t d = 1; d < 64; d <<= 1) {
        const uint64_t t = __shfl_up(s, d, 64);
        if (lane >= d) s += t;
    }
    if (lane < nc) sm.chunk_pos[lane] = s - v;
    return __shfl(s, 63, 64);
}

// One workgroup per tile (tile = blockIdx.x), 4 waves.
// (8 waves per SIMD: LDS 19.7 KB, 8 workgroups per CU; 6 before the
// selector table left LDS)

// GAP: chunk c is preceded by gap[c] bytes of the output that the kernel
// leaves zero (out_off[c] is the gap's start; capnp_gpu_write_messages puts
// each message's segment table there).
template <bool SYNC, bool GAP>
__global__ void __launch_bounds__(kThreads, GAP ? 7 : 8)  // (GAP: 20.6 KB of LDS)
pack_kernel(const uint64_t* __restrict__ in, const uint64_t* __restrict__ chunk_off,
            uint64_t nchunks, uint32_t tc, uint8_t* __restrict__ out, uint64_t out_cap,
            uint64_t* __restrict__ out_off, uint64_t* __restrict__ ts,
            uint64_t* __restrict__ gs, uint32_t* __restrict__ sync,
            const uint32_t* __restrict__ gap, uint8_t* __restrict__ ovf) {
    static_assert(!(SYNC && GAP), "the sync index is not written with gaps");
    __shared__ Smem<GAP> sm;
    const uint32_t tid = threadIdx.x;
    const uint32_t lane = tid & 63u;
    const uint32_t wave = (uint32_t)__builtin_amdgcn_readfirstlane((int)(tid >> 6));
    const uint64_t ntiles = gridDim.x;  // = ceil(nchunks / tc), set by the launch
    const uint64_t tile = blockIdx.x;
    LookbackArgs LA;
    LA.ts = ts;
    LA.gs = gs;
    LA.ntiles = ntiles;
    LA.in = in;
    LA.chunk_off = chunk_off;
    LA.nchunks = nchunks;
    LA.tc = tc;
    LA.gap = GAP ? gap : nullptr;
    LA.wt = 0;
    LA.wlo = LA.whi = LA.g0 = 0;
    LA.map = nullptr;

    const uint64_t c0 = tile * tc;
    const uint64_t c1 = (c0 + tc < nchunks) ? c0 + tc : nchunks;
    const uint32_t nc = (uint32_t)(c1 - c0);
#if PACK_PROF
    if (tid == 0) {
        uint32_t xcc, hwid;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hwid));
        TRACE(tile, 0, RT());
        TRACE(tile, 4, ((uint64_t)xcc << 32) | hwid);
    }
#endif
    const uint64_t* __restrict__ toff = chunk_off + c0;  // the tile's chunk offsets
    // sync entries of the tile: k in [k0, k1), words kSyncWords * k in [W0, W1)
    const uint64_t TW0 = uniform64(chunk_off[c0]);
    const uint64_t TW1 = uniform64(chunk_off[c1]);
    const uint64_t k0 = (TW0 + kSyncWords - 1) / kSyncWords;
    const uint64_t k1 = (TW1 + kSyncWords - 1) / kSyncWords;
    const uint32_t t0 = (uint32_t)(k0 * kSyncWords - TW0);  // first sync word, tile-relative
    for (uint32_t i = tid; i < nc; i += kThreads) sm.chunk_size[i] = 0;
    if constexpr (GAP)
        for (uint32_t i = tid; i < nc; i += kThreads) sm.chunk_gap[i] = gap[c0 + i];
    // record assembly table: one 8-byte entry per thread (+ the copy entry)
    for (uint32_t i = tid; i <= kSelCopy; i += kThreads) sm.sel[i] = kSel8Table.e[i];
    uint8_t* region = sm.stage[wave];
    const uint32_t mis = (uint32_t)(reinterpret_cast<uintptr_t>(out) & 15u);
    uint8_t* const outa = out - mis;
    // (the ranges below read only chunk_off, so without gaps the barrier
    // after them also covers the table writes above)
    if (GAP) __syncthreads();
#if PACK_PROF == 2
    if (tid == 0) TRACE(tile, 5, RT());  // (2: prelude timeline instead of look-back counters)
#endif

    // contiguous chunk ranges per wave for the staged path.  Lane s of the
    // wave describes step s of the range: source word offset and
    // (nvalid | first << 7 | last << 8 | chunk << 9).
    const uint32_t q = (nc + kWaves - 1) / kWaves;
    const uint32_t wc0 = wave * q < nc ? wave * q : nc;
    const uint32_t wc1 = wc0 + q < nc ? wc0 + q : nc;
    // The range's words go out to registers before its steps are known:
    // step s loads the 64 words from the range start + 64 s.  That is the
    // staged layout exactly when every chunk of the range is a whole number
    // of steps (checked in the walk; otherwise the steps are loaded again),
    // and the load latency then overlaps the walk.  Interleaved A/B on three
    // boxes (us): config 2 583 / 584 vs 597 / 587 / 593, carsales 591 / 596
    // vs 610 / 609; equal chunks of 100 words pay 1.8-3 % (every step loaded
    // twice).
    const uint32_t tile_bytes = (uint32_t)((TW1 - TW0) * 8);
    const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<uint64_t*>(in + TW0), 0, (int)tile_bytes, 0x00020000);
    uint64_t cache[kStageSteps];
    // (messages with segment tables, GAP, have ragged segments: no speculation)
    constexpr bool kSpec = !GAP;
    uint64_t ragged = 63;  // OR of the range's chunk lengths (| 63: not speculated): low bits = load
    if (kSpec && wc1 > wc0) {
        const uint64_t a = uniform64(toff[wc0]);
        const uint32_t r0 = (uint32_t)(a - TW0);
        const uint32_t r1 = (uint32_t)(uniform64(toff[wc1]) - TW0);
        ragged = 0;
#pragma unroll
        for (uint32_t s = 0; s < kStageSteps; s++) {
            const uint32_t w = r0 + 64 * s + lane;
            const uint32_t vo = w < r1 ? w * 8u : 0x80000000u;
            const auto v = __builtin_amdgcn_raw_buffer_load_b64(rsrc, (int)vo, 0, 0);
            cache[s] = ((uint64_t)v[1] << 32) | v[0];
        }
    }

    uint64_t d_src = 0;
    uint32_t d_g = 0;  // tile-relative word of the step's lane 0
    uint32_t d_meta = 0;
    uint32_t nsteps = 0;
    uint32_t gsum = 0;  // GAP: the range's gap bytes; an empty chunk with a gap streams
    for (uint32_t ci = wc0; ci < wc1; ci++) {
        const uint64_t woff = uniform64(toff[ci]);
        const uint64_t len = uniform64(toff[ci + 1]) - woff;
        const uint32_t nst = (uint32_t)((len + 63) / 64);
        ragged |= len;
        if constexpr (GAP) {
            const uint32_t g = uniform(sm.chunk_gap[ci]);
            gsum += (len == 0 && g) ? kGapSlack + 1 : g;
        }
        const uint32_t k = lane - nsteps;
        if (lane >= nsteps && k < nst) {
            const uint64_t rest = len - 64ull * k;
            d_src = woff + 64ull * k;
            d_g = (uint32_t)(d_src - TW0);
            d_meta = (uint32_t)(rest < 64 ? rest : 64) | ((k == 0) << 7) |
                     ((k + 1 == nst) << 8) | ((ci - wc0) << 9);
        }
        nsteps += nst;
    }
    if (lane == 0) sm.wave_steps[wave] = (GAP && gsum > kGapSlack) ? kStageSteps + 1 : nsteps;
    __syncthreads();
    bool staged = true;
#pragma unroll
    for (int w = 0; w < kWaves; w++) staged &= sm.wave_steps[w] <= kStageSteps;
    staged = __builtin_amdgcn_readfirstlane((int)staged) != 0;
#if PACK_PROF == 2
    if (tid == 0) TRACE(tile, 6, RT());
#endif

    if (staged) {
        // Load every step of the range into registers and zero the region.
        // All kStageSteps steps run unconditionally: a step past nsteps has
        // meta 0 (no valid words, no chunk edges) and is a no-op, so the
        // compiler sees a straight line and counts the loads' waits exactly.
        // The loads go through a buffer descriptor over the tile's words (<=
        // 16 KiB here): a lane past nvalid reads out of range and gets 0.
        if (__builtin_amdgcn_readfirstlane((int)(uint32_t)(ragged & 63u)) != 0) {
#pragma unroll
            for (uint32_t s = 0; s < kStageSteps; s++) {
                const uint32_t g = (uint32_t)__builtin_amdgcn_readlane((int)d_g, s);
                const uint32_t nv = (uint32_t)__builtin_amdgcn_readlane((int)d_meta, s) & 127u;
                const uint32_t vo = lane < nv ? (g + lane) * 8u : 0x80000000u;
                const auto v = __builtin_amdgcn_raw_buffer_load_b64(rsrc, (int)vo, 0, 0);
                cache[s] = ((uint64_t)v[1] << 32) | v[0];
            }
        }
        for (uint32_t o = 16 * lane; o < kStageRegion; o += 16 * CAPNP_WAVE)
            *reinterpret_cast<uint4*>(region + o) = make_uint4(0, 0, 0, 0);
#if PACK_PROF == 2
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (tid == 0) TRACE(tile, 7, RT());
#endif
        // pass 1: sizes and positions
        StepInfo si[kStageSteps];
        uint32_t hbits = 0;  // bit s = this lane heads a record in step s
        {
            // (each step's chunk start and running size go to lane s of two
            // registers; the chunk tables are written once after the loop)
            StageState pk;
            pk.begin(0);
            uint32_t local = 0;
            uint32_t rec_oc = 0, rec_sz = 0;
#pragma unroll
            for (uint32_t s = 0; s < kStageSteps; s++) {
                const uint32_t meta = (uint32_t)__builtin_amdgcn_readlane((int)d_meta, s);
                si[s].meta = meta;
                (void)meta;
                if ((meta >> 7) & 1) {
                    if constexpr (GAP) local += uniform(sm.chunk_gap[wc0 + (meta >> 9)]);
                    pk.begin(local);
                }
                size_step_lean(pk, cache[s], meta & 127u, lane, si[s]);
                hbits |= mask_sel(si[s].H, 1u << s, 0u);
                rec_oc = lane == s ? pk.o_c : rec_oc;
                rec_sz = lane == s ? pk.total : rec_sz;
                if ((meta >> 8) & 1) local += pk.total;
            }
            if (lane < kStageSteps) {
                const uint32_t ci = wc0 + ((d_meta >> 9) & 63u);
                if ((d_meta >> 7) & 1) sm.chunk_oc[ci] = rec_oc;
                if ((d_meta >> 8) & 1) {
                    uint32_t g = 0;
                    if constexpr (GAP) g = sm.chunk_gap[ci];
                    sm.chunk_size[ci] = rec_sz + g;
                }
            }
            if (lane == 0) sm.wave_bytes[wave] = local;
        }
        __syncthreads();
        // every range's bytes (gaps included) must fit its region
        bool fits = true;
#pragma unroll
        for (int w = 0; w < kWaves; w++) fits &= sm.wave_bytes[w] <= kStageBytes;
        fits = __builtin_amdgcn_readfirstlane((int)fits) != 0;
        uint64_t agg = 0;
        if (wave == 0) {
            agg = scan_chunks32(sm, nc, lane);
            publish(LA, tile, agg, lane);
            if (lane == 0) TRACE(tile, 1, RT());
        }
        // pass 2: assemble the bytes (the look-back loads are in flight)
        uint8_t* const region_m1 = region - 1;
        wave_lds_sync();
        if (fits) {
            uint32_t ext = 0;  // words the run open at the step end absorbs later
#pragma unroll
            for (int s = (int)kStageSteps - 1; s >= 0; s--) {
                StepInfo sj = si[s];
                sj.H = ballot64(((hbits >> s) & 1u) != 0);
                const uint32_t meta = sj.meta;
                const uint32_t e = ((meta >> 8) & 1) ? 0u : ext;
                emit_step<SYNC>(cache[s], sj, e, lane, region_m1, sm.sel,
                          SYNC ? reinterpret_cast<uint8_t*>(sync + k0) : nullptr, t0,
                          (uint32_t)__builtin_amdgcn_readlane((int)d_g, s),
                          uniform(sm.chunk_oc[(wc0 + ((meta >> 9) & 63u)) & (kMaxTileChunks - 1)]));
                // ext for step s-1: absorbed here, plus later if the run
                // covered this whole step
                ext = ((meta >> 7) & 1) ? 0u : (meta >> 16) + (sj.H == 0 ? e : 0u);
            }
        }
        if (wave == 0) {
            const uint64_t excl = tile_offset(LA, tile, agg, lane);
            if (lane == 0) TRACE(tile, 2, RT());
            if (lane < nc) sm.chunk_pos[lane] += excl;
            if (c1 == nchunks && lane == 0) out_off[nchunks] = excl + agg;
        }
        __syncthreads();
        for (uint32_t i = tid; i < nc; i += kThreads) out_off[c0 + i] = sm.chunk_pos[i];
        if (fits) {
            if (wc1 > wc0) {
                const uint64_t D0 = lds_u64(&sm.chunk_pos[wc0]) + mis;
                copy_out(region, outa, D0, lds_u64(&sm.wave_bytes[wave]), out_cap + mis, lane);
            }
        } else {
            // a range overflowed its region (adversarial input, 8.19 to 8.5
            // bytes per word): the sizes and offsets stand; pack_ovf_kernel
            // writes the tile's bytes with the streaming path, and the tile
            // has no index entries.  (The streaming pass inlined here pushed
            // this kernel past 64 VGPRs; as a call it cost 3 % of every tile.)
            if constexpr (SYNC)
                for (uint32_t i = tid; i < (uint32_t)(k1 - k0); i += kThreads)
                    sync[k0 + i] = kSyncNone;
            if (tid == 0) ovf[tile] = 1;
        }
#if PACK_PROF
        __syncthreads();
        if (tid == 0) TRACE(tile, 3, RT());
#endif
    } else {
        if constexpr (SYNC)
            for (uint32_t i = tid; i < (uint32_t)(k1 - k0); i += kThreads) sync[k0 + i] = kSyncNone;
        run_streaming<MODE_SIZE>(in, toff, sm.chunk_size, sm.chunk_pos, nc, wave, lane,
                                 region, sm.sel, outa, mis, out_cap,
                                 GAP ? sm.chunk_gap : nullptr);
        __syncthreads();
        if (wave == 0) {
            const uint64_t agg = scan_chunks(sm, nc, lane);
            publish(LA, tile, agg, lane);
            const uint64_t excl = tile_offset(LA, tile, agg, lane);
            if (lane < nc) sm.chunk_pos[lane] += excl;
            if (c1 == nchunks && lane == 0) out_off[nchunks] = excl + agg;
        }
        __syncthreads();
        for (uint32_t i = tid; i < nc; i += kThreads) out_off[c0 + i] = sm.chunk_pos[i];
        run_streaming<MODE_RING>(in, toff, sm.chunk_size, sm.chunk_pos, nc, wave, lane,
                                 region, sm.sel, outa, mis, out_cap,
                                 GAP ? sm.chunk_gap : nullptr);
    }
}

// ---------------------------------------------------------------------------
// Lean chunk-tile pack kernel (the default for batches without gaps).
//
// The same tiles, wave ranges, look-back and copy-out as pack_kernel's staged
// path, with the two passes rebuilt for fewer instructions per 64-word step.
// pack_kernel's step issued ~158 VALU and ~109 SALU instructions per step
// (profiles/r02i_config2_pmc_summary.txt: 332 M VALU, 229 M SALU per
// 1 GiB launch): the scalar unit, one per CU and shared by its four SIMDs,
// was ~75 % busy and the per-tile chain of dependent phases could not be
// hidden.  Here:
//   * pass 1 does everything that needs the step's head mask H while H is
//     in scalar registers: byte positions (DPP scan), each head's run count
//     within the step and whether its run reaches the step end, and the
//     record sync index entries (written straight to memory, masked lanes
//     through an out-of-range buffer offset, no exec-mask branches);
//   * one 32-bit VGPR per step carries pass 1's result to pass 2:
//     pos (13 bits, in the wave's region) | idx (9: the record assembly
//     entry, the tag for a head, kSelCopy for a literal word inside a run)
//     << 13 | run count (6) << 22 | reaches step end << 28 | no bytes << 29;
//     the step's carried-run words and "no head" flag go to lane s of one
//     more VGPR, so no mask stays live across the passes (no SGPR spills);
//   * pass 2 is the record assembly and four LDS ORs under a single exec
//     mask (lanes with no bytes skip them), with the run count of the head
//     whose run crosses into later steps completed from those steps (ext).
// Tiles whose ranges do not fit the staged steps (chunks longer than the
// steps, or more chunks than steps) compute their chunk sizes with the
// streaming size pass, take part in the look-back, and leave their bytes to
// pack_ovf_kernel (as tiles whose staged bytes overflow their regions do).


struct LeanCarry {
    uint32_t type;   // run open at the step start: 0 none, 1 zero run, 2 literal run
    uint32_t rem;    // words it may still absorb
    uint32_t total;  // packed bytes of the chunk so far
};

constexpr uint32_t kInfoPosBits = 13;
static_assert(kStageRegion + 16 <= (1u << kInfoPosBits), "region positions fit 13 bits");

// Pass 1 of one step: the step's records sized and placed (chunk-relative
// `c.total`, wave-region start of the chunk `oc`), returned packed into one
// VGPR (see above); kin = words the carried run absorbs | no head << 8.
__device__ __forceinline__ uint32_t lean_size_step(uint64_t w, uint32_t nvalid, uint32_t lane,
                                                   LeanCarry& c, uint32_t oc, uint32_t& kin) {
    const uint32_t lo = (uint32_t)w, hi = (uint32_t)(w >> 32);
    const uint32_t tag = word_tag_dot(lo, hi);
    const uint32_t pop = __builtin_popcount(tag);
    // lanes past nvalid hold zero words (out-of-range loads): no class
    const bool valid = lane < nvalid;
    const uint32_t pv = valid ? pop : 64u;
    const uint64_t V = ballot64(valid);
    const uint64_t Zm = ballot64(pv == 0);
    const uint64_t Lm = ballot64(pop >= 7);
    const uint64_t Fm = ballot64(pop == 8);
    // words of the carried run's class at the step start, at most rem
    uint32_t k = ctz64(~(c.type == 1 ? Zm : Lm));
    k = k < c.rem ? k : c.rem;
    k = c.type ? k : 0u;
    const uint64_t AC = ballot64(lane < k);
    const uint64_t Z2 = Zm & ~AC;
    const uint64_t AZ = Z2 & (Z2 << 1);
    const uint64_t L2 = Lm & ~AC;
    const uint64_t F2 = Fm & ~AC;
    const uint64_t filled = ((L2 ^ (L2 + F2)) & L2) | F2;
    const uint64_t AF = filled & (filled << 1);
    const uint64_t H = V & ~(AC | AZ | AF);
    // record sizes and positions
    const uint32_t hsize = 1u + pop + ((0x101u >> pop) & 1u);
    const uint32_t size = mask_sel(H, hsize, tag == 0 ? 0u : 8u);
    const uint32_t incl = wave_incl_scan(size);
    const uint32_t prel = c.total + incl - size;  // chunk-relative
    // a head's run: the words up to the next head (none: to the step end)
    const uint64_t nxt = (H >> 1) >> lane;
    const uint32_t dn = min(ffbl((uint32_t)nxt), ffbl((uint32_t)(nxt >> 32)) | 32u);
    const uint32_t reach = dn > 63u ? 1u : 0u;
    const uint32_t cnt = min(dn, __builtin_elementwise_sub_sat(nvalid, lane + 1u));
    const uint32_t idx = mask_sel(H, tag, kSelCopy);
    const uint32_t skip = size == 0 ? 1u : 0u;
    uint32_t info = (oc + prel) | (idx << kInfoPosBits) | ((cnt & 63u) << 22) | (reach << 28) |
                    (skip << 29);
    // (materialised here: otherwise the compiler sinks the packing into pass
    // 2 and keeps its parts live across the steps, spilling)
    asm volatile("" : "+v"(info));
    // the run open at the step end: the last head's, or the carried one when
    // it covered the whole step
    const uint32_t code = pv == 0 ? 1u : (pv == 8 ? 2u : 0u);
    const uint32_t h = H ? 63u - (uint32_t)__builtin_clzll(H) : 0u;
    const uint32_t th = (uint32_t)__builtin_amdgcn_readlane((int)code, h);
    kin = k | (H ? 0u : 0x100u);
    c.type = H ? th : c.type;
    c.rem = H ? (th ? 192u + h : 0u) : c.rem - 64u;
    c.total += (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
    return info;
}

// Pass 2 of one step: the records of the step ORed into the wave's zeroed
// region (region_m1 = region - 1; see emit_step for the alignbyte placement).
// ext = words the run open at the step end absorbs in later steps.
// SYNC: every head writes the entries of the sync points its record covers
// (as emit_step; oc = the chunk's region start, g = tile-relative word of
// lane 0, t0 = the tile's first sync word, srs = the tile's entries).
template <bool SYNC>
__device__ __forceinline__ void lean_emit_step(uint64_t w, uint32_t info, uint32_t ext,
                                               uint32_t lane, uint8_t* region_m1, const Sel8* sel,
                                               __amdgpu_buffer_rsrc_t srs, uint32_t oc,
                                               uint32_t g, uint32_t t0) {
    if (info & (1u << 29)) return;  // no bytes (absorbed zero word, past the words)
    const uint32_t lo = (uint32_t)w, hi = (uint32_t)(w >> 32);
    const uint32_t pos = info & ((1u << kInfoPosBits) - 1u);
    const uint32_t idx = __builtin_amdgcn_ubfe(info, kInfoPosBits, 9);
    const uint32_t cnt = __builtin_amdgcn_ubfe(info, 22, 6) +
                         __builtin_amdgcn_ubfe(info, 28, 1) * ext;
    const Sel8 se = sel[idx];
    const uint32_t r0 = __builtin_amdgcn_perm(hi, lo, se.s0) | (((cnt << 8) | idx) & sel_m(idx));
    const uint32_t r1 = __builtin_amdgcn_perm(hi, lo, se.s1);
    const uint32_t r2 = __builtin_amdgcn_perm(cnt, hi, sel_s2(idx));
    const uint32_t s = 0u - pos;
    const uint32_t e0 = __builtin_amdgcn_alignbyte(r0, 0u, s);
    const uint32_t e1 = __builtin_amdgcn_alignbyte(r1, r0, s);
    const uint32_t e2 = __builtin_amdgcn_alignbyte(r2, r1, s);
    const uint32_t e3 = __builtin_amdgcn_alignbyte(0u, r2, s);
    uint32_t* b32 = reinterpret_cast<uint32_t*>(__builtin_align_down(region_m1 + pos, 4));
    __hip_atomic_fetch_or(b32 + 0, e0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
    __hip_atomic_fetch_or(b32 + 1, e1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
    __hip_atomic_fetch_or(b32 + 2, e2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
    __hip_atomic_fetch_or(b32 + 3, e3, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
    if constexpr (SYNC) {
        // sync points m = hw + d (d = (t0 - hw) mod kSyncWords, d <= cnt) of
        // the record headed at tile word hw = g + lane; entry (m - t0) / 8
        const uint32_t c = t0 - g;
        const uint32_t d = (c - lane) & (kSyncWords - 1);
        const uint32_t dh = idx < kSelCopy ? d : ~0u;
        const uint32_t rel = pos - oc;
        const uint32_t b = (lane + d - c) / (kSyncWords / 4u);
        __builtin_amdgcn_raw_buffer_store_b32(rel | (d << 24), srs,
                                              (int)(dh <= cnt ? b : 0x80000000u), 0, 0);
        // (runs longer than kSyncWords words: rare)
        if (dh < kSyncWords && dh + kSyncWords <= cnt) {  // (dh = ~0: not a head)
#pragma clang loop unroll(disable) vectorize(disable)
            for (uint32_t dd = d + kSyncWords, bb = b + 4; dd <= cnt; dd += kSyncWords, bb += 4)
                __builtin_amdgcn_raw_buffer_store_b32(rel | (dd << 24), srs, (int)bb, 0, 0);
        }
    }
}

template <bool SYNC>
__global__ void __launch_bounds__(kThreads, 8)
pack_lean_kernel(const uint64_t* __restrict__ in, const uint64_t* __restrict__ chunk_off,
                 uint64_t nchunks, uint32_t tc, uint8_t* __restrict__ out, uint64_t out_cap,
                 uint64_t* __restrict__ out_off, uint64_t* __restrict__ ts,
                 uint64_t* __restrict__ gs, uint32_t* __restrict__ sync,
                 uint8_t* __restrict__ ovf) {
    __shared__ Smem<false> sm;
    const uint32_t tid = threadIdx.x;
    const uint32_t lane = tid & 63u;
    const uint32_t wave = (uint32_t)__builtin_amdgcn_readfirstlane((int)(tid >> 6));
    const uint64_t ntiles = gridDim.x;
    const uint64_t tile = blockIdx.x;
    LookbackArgs LA;
    LA.ts = ts;
    LA.gs = gs;
    LA.ntiles = ntiles;
    LA.in = in;
    LA.chunk_off = chunk_off;
    LA.nchunks = nchunks;
    LA.tc = tc;
    LA.gap = nullptr;
    LA.wt = 0;
    LA.wlo = LA.whi = LA.g0 = 0;
    LA.map = nullptr;

    const uint64_t c0 = tile * tc;
    const uint64_t c1 = (c0 + tc < nchunks) ? c0 + tc : nchunks;
    const uint32_t nc = (uint32_t)(c1 - c0);
    const uint64_t* __restrict__ toff = chunk_off + c0;
    const uint64_t TW0 = uniform64(chunk_off[c0]);
    const uint64_t TW1 = uniform64(chunk_off[c1]);
    const uint64_t k0 = (TW0 + kSyncWords - 1) / kSyncWords;
    const uint64_t k1 = (TW1 + kSyncWords - 1) / kSyncWords;
    const uint32_t t0 = (uint32_t)(k0 * kSyncWords - TW0);
    for (uint32_t i = tid; i < nc; i += kThreads) sm.chunk_size[i] = 0;
    for (uint32_t i = tid; i <= kSelCopy; i += kThreads) sm.sel[i] = kSel8Table.e[i];
    uint8_t* region = sm.stage[wave];
    const uint32_t mis = (uint32_t)(reinterpret_cast<uintptr_t>(out) & 15u);
    uint8_t* const outa = out - mis;

    // contiguous chunk ranges per wave; lane s describes step s of the range
    const uint32_t q = (nc + kWaves - 1) / kWaves;
    const uint32_t wc0 = wave * q < nc ? wave * q : nc;
    const uint32_t wc1 = wc0 + q < nc ? wc0 + q : nc;
    const uint32_t tile_bytes = (uint32_t)((TW1 - TW0) * 8);
    const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<uint64_t*>(in + TW0), 0, (int)tile_bytes, 0x00020000);
    // speculative loads (see pack_kernel): step s = the 64 words from the
    // range start + 64 s, the staged layout when every chunk is whole steps
    uint64_t cache[kStageSteps];
    uint64_t ragged = 63;
    if (wc1 > wc0) {
        const uint32_t r0 = (uint32_t)(uniform64(toff[wc0]) - TW0);
        const uint32_t r1 = (uint32_t)(uniform64(toff[wc1]) - TW0);
        ragged = 0;
#pragma unroll
        for (uint32_t s = 0; s < kStageSteps; s++) {
            const uint32_t w = r0 + 64 * s + lane;
            const uint32_t vo = w < r1 ? w * 8u : 0x80000000u;
            const auto v = __builtin_amdgcn_raw_buffer_load_b64(rsrc, (int)vo, 0, 0);
            cache[s] = ((uint64_t)v[1] << 32) | v[0];
        }
    }
    uint32_t d_g = 0, d_meta = 0, nsteps = 0;
    for (uint32_t ci = wc0; ci < wc1; ci++) {
        const uint64_t woff = uniform64(toff[ci]);
        const uint64_t len = uniform64(toff[ci + 1]) - woff;
        const uint32_t nst = (uint32_t)((len + 63) / 64);
        ragged |= len;
        const uint32_t kk = lane - nsteps;
        if (lane >= nsteps && kk < nst) {
            const uint64_t rest = len - 64ull * kk;
            d_g = (uint32_t)(woff + 64ull * kk - TW0);
            d_meta = (uint32_t)(rest < 64 ? rest : 64) | ((kk == 0) << 7) |
                     ((kk + 1 == nst) << 8) | ((ci - wc0) << 9);
        }
        nsteps += nst;
    }
    if (lane == 0) sm.wave_steps[wave] = nsteps;
    __syncthreads();
    bool staged = true;
#pragma unroll
    for (int w = 0; w < kWaves; w++) staged &= sm.wave_steps[w] <= kStageSteps;
    staged = __builtin_amdgcn_readfirstlane((int)staged) != 0;

    if (!staged) {
        // sizes by the streaming size pass, offsets by the look-back; the
        // bytes come from pack_ovf_kernel
        if constexpr (SYNC)
            for (uint32_t i = tid; i < (uint32_t)(k1 - k0); i += kThreads) sync[k0 + i] = kSyncNone;
        run_streaming<MODE_SIZE>(in, toff, sm.chunk_size, sm.chunk_pos, nc, wave, lane, region,
                                 sm.sel, outa, mis, out_cap, nullptr);
        __syncthreads();
        if (wave == 0) {
            const uint64_t agg = scan_chunks(sm, nc, lane);
            publish(LA, tile, agg, lane);
            const uint64_t excl = tile_offset(LA, tile, agg, lane);
            if (lane < nc) sm.chunk_pos[lane] += excl;
            if (c1 == nchunks && lane == 0) out_off[nchunks] = excl + agg;
            if (lane == 0) ovf[tile] = 1;
        }
        __syncthreads();
        for (uint32_t i = tid; i < nc; i += kThreads) out_off[c0 + i] = sm.chunk_pos[i];
        return;
    }

    if (__builtin_amdgcn_readfirstlane((int)(uint32_t)(ragged & 63u)) != 0) {
#pragma unroll
        for (uint32_t s = 0; s < kStageSteps; s++) {
            const uint32_t g = (uint32_t)__builtin_amdgcn_readlane((int)d_g, s);
            const uint32_t nv = (uint32_t)__builtin_amdgcn_readlane((int)d_meta, s) & 127u;
            const uint32_t vo = lane < nv ? (g + lane) * 8u : 0x80000000u;
            const auto v = __builtin_amdgcn_raw_buffer_load_b64(rsrc, (int)vo, 0, 0);
            cache[s] = ((uint64_t)v[1] << 32) | v[0];
        }
    }
    for (uint32_t o = 16 * lane; o < kStageRegion; o += 16 * CAPNP_WAVE)
        *reinterpret_cast<uint4*>(region + o) = make_uint4(0, 0, 0, 0);

    // the tile's sync entries [k0, k1) as a buffer (out-of-range stores drop)
    const __amdgpu_buffer_rsrc_t srs = __builtin_amdgcn_make_buffer_rsrc(
        SYNC ? sync + k0 : nullptr, 0, SYNC ? (int)((k1 - k0) * 4) : 0, 0x00020000);

    // ---- pass 1: sizes, positions, run counts
    uint32_t info[kStageSteps];
    uint32_t kin_l = 0;  // lane s: step s's carried-run words | no head << 8
    uint32_t rec_oc = 0;  // lane s: region start of step s's chunk
    {
        LeanCarry c{0, 0, 0};
        uint32_t local = 0, oc = 0;
        uint32_t rec_sz = 0;
#pragma unroll
        for (uint32_t s = 0; s < kStageSteps; s++) {
            const uint32_t meta = (uint32_t)__builtin_amdgcn_readlane((int)d_meta, s);
            if ((meta >> 7) & 1) {
                c.type = 0;
                c.rem = 0;
                c.total = 0;
                oc = local;
            }
            uint32_t kin = 0;
            info[s] = lean_size_step(cache[s], meta & 127u, lane, c, oc, kin);
            kin_l = lane == s ? kin : kin_l;
            rec_oc = lane == s ? oc : rec_oc;
            rec_sz = lane == s ? c.total : rec_sz;
            if ((meta >> 8) & 1) local += c.total;
            __builtin_amdgcn_sched_barrier(0);  // one step at a time: registers
        }
        if (lane < kStageSteps && ((d_meta >> 8) & 1))
            sm.chunk_size[wc0 + ((d_meta >> 9) & 63u)] = rec_sz;
        if (lane == 0) sm.wave_bytes[wave] = local;
    }
    __syncthreads();
    bool fits = true;
#pragma unroll
    for (int w = 0; w < kWaves; w++) fits &= sm.wave_bytes[w] <= kStageBytes;
    fits = __builtin_amdgcn_readfirstlane((int)fits) != 0;
    uint64_t agg = 0;
    if (wave == 0) {
        agg = scan_chunks32(sm, nc, lane);
        publish(LA, tile, agg, lane);
    }
    // ---- pass 2: the bytes (the look-back loads are in flight)
    if (fits) {
        uint8_t* const region_m1 = region - 1;
        uint32_t ext = 0;
#pragma unroll
        for (int s = (int)kStageSteps - 1; s >= 0; s--) {
            const uint32_t meta = (uint32_t)__builtin_amdgcn_readlane((int)d_meta, s);
            const uint32_t kin = (uint32_t)__builtin_amdgcn_readlane((int)kin_l, s);
            const uint32_t e = ((meta >> 8) & 1) ? 0u : ext;
            lean_emit_step<SYNC>(cache[s], info[s], e, lane, region_m1, sm.sel, srs,
                                 (uint32_t)__builtin_amdgcn_readlane((int)rec_oc, s),
                                 (uint32_t)__builtin_amdgcn_readlane((int)d_g, s), t0);
            ext = ((meta >> 7) & 1) ? 0u : (kin & 0xFFu) + ((kin & 0x100u) ? e : 0u);
            __builtin_amdgcn_sched_barrier(0);
        }
    }
    if (wave == 0) {
        const uint64_t excl = tile_offset(LA, tile, agg, lane);
        if (lane < nc) sm.chunk_pos[lane] += excl;
        if (c1 == nchunks && lane == 0) out_off[nchunks] = excl + agg;
    }
    __syncthreads();
    for (uint32_t i = tid; i < nc; i += kThreads) out_off[c0 + i] = sm.chunk_pos[i];
    if (fits) {
        if (wc1 > wc0) {
            const uint64_t D0 = lds_u64(&sm.chunk_pos[wc0]) + mis;
            copy_out(region, outa, D0, lds_u64(&sm.wave_bytes[wave]), out_cap + mis, lane);
        }
    } else {
        // a range overflowed its region (adversarial input): the sizes and
        // offsets stand; pack_ovf_kernel writes the bytes; no index entries
        if constexpr (SYNC)
            for (uint32_t i = tid; i < (uint32_t)(k1 - k0); i += kThreads) sync[k0 + i] = kSyncNone;
        if (tid == 0) ovf[tile] = 1;
    }
}

// ---------------------------------------------------------------------------
// Chunk-step pack kernel (pack_cs_kernel): batches whose chunks hold at most
// 128 words (1 KiB segments: configs 2, 3, 5 and the carsales workload).
//
// A step is one whole chunk: lane l holds its words l and 64 + l, so the
// step's masks are 128-bit (lo = words 0-63, hi = words 64-127) and, since a
// run never crosses a write_all chunk (serialize_packed.rs:375-427 scan only
// the chunk) and a 128-word chunk cannot reach the 255-word cap, there is no
// run state carried between steps at all: no carry logic, no per-step chunk
// bookkeeping, one scalar segmentation per 128 words.  Each wave owns up to
// kCsSteps chunks of its tile.  Tiles with a longer chunk (or more chunks per
// wave) take the streaming size pass and leave their bytes to
// pack_ovf_kernel.
#ifndef PACK_TILECOPY
#define PACK_TILECOPY 1  // chunk-step tiles: the waves' bytes back to back in LDS, one tile copy-out
#endif
#ifndef PACK_ABL
#define PACK_ABL 0  // ablation builds (timing only, wrong bytes): 1 no LDS ORs, 2 no sync
                    // stores, 4 no look-back (a fixed tile offset), 8 no copy-out
#endif
constexpr uint32_t kCsSteps = 4;   // chunks (steps) per wave
constexpr uint32_t kCsWords = 128; // words per step

// 128-bit masks on the scalar unit: {lo, hi}.
struct M128 {
    uint64_t lo, hi;
};
__device__ __forceinline__ M128 shl1(M128 a) { return {a.lo << 1, (a.hi << 1) | (a.lo >> 63)}; }
__device__ __forceinline__ M128 operator&(M128 a, M128 b) { return {a.lo & b.lo, a.hi & b.hi}; }
__device__ __forceinline__ M128 operator|(M128 a, M128 b) { return {a.lo | b.lo, a.hi | b.hi}; }
__device__ __forceinline__ M128 operator^(M128 a, M128 b) { return {a.lo ^ b.lo, a.hi ^ b.hi}; }
__device__ __forceinline__ M128 andnot(M128 a, M128 b) { return {a.lo & ~b.lo, a.hi & ~b.hi}; }
// (an add-with-carry chain on the scalar unit; the C form compares in a VALU
// op and reads the carry back)
__device__ __forceinline__ M128 add128(M128 a, M128 b) {
    uint32_t r0, r1, r2, r3;
    asm("s_add_u32 %0, %4, %8\n\t"
        "s_addc_u32 %1, %5, %9\n\t"
        "s_addc_u32 %2, %6, %10\n\t"
        "s_addc_u32 %3, %7, %11"
        : "=&s"(r0), "=&s"(r1), "=&s"(r2), "=s"(r3)
        : "s"((uint32_t)a.lo), "s"((uint32_t)(a.lo >> 32)), "s"((uint32_t)a.hi),
          "s"((uint32_t)(a.hi >> 32)), "s"((uint32_t)b.lo), "s"((uint32_t)(b.lo >> 32)),
          "s"((uint32_t)b.hi), "s"((uint32_t)(b.hi >> 32))
        : "scc");
    return {((uint64_t)r1 << 32) | r0, ((uint64_t)r3 << 32) | r2};
}

// Index of the lowest set bit of a 64-bit lane value, >= 64 if none.
__device__ __forceinline__ uint32_t ffbl64(uint64_t x) {
    return min(ffbl((uint32_t)x), ffbl((uint32_t)(x >> 32)) | 32u);
}

// info of one word: pos (13) | idx (9) << 13 | run count (7) << 22 | no bytes << 29
constexpr uint32_t kCsSkip = 1u << 29;

__device__ __forceinline__ uint32_t cs_info(uint32_t pos, uint32_t idx, uint32_t cnt,
                                            uint32_t size) {
    uint32_t info = pos | (idx << kInfoPosBits) | (cnt << 22) | (size == 0 ? kCsSkip : 0u);
    asm volatile("" : "+v"(info));  // (materialised in pass 1: see lean_size_step)
    return info;
}

// Pass 1 of one chunk of n <= 128 words (lo = word lane, hi = word 64 +
// lane) placed at region position oc: both words' info; returns the chunk's
// packed size.  The two halves' record sizes (<= 10 bytes, <= 640 per half)
// share one 16:16 scan.
__device__ __forceinline__ uint32_t cs_size_step(uint64_t wlo, uint64_t whi, uint32_t n,
                                                 uint32_t lane, uint32_t oc, uint32_t& ilo,
                                                 uint32_t& ihi) {
    const uint32_t tlo = word_tag_dot((uint32_t)wlo, (uint32_t)(wlo >> 32));
    const uint32_t thi = word_tag_dot((uint32_t)whi, (uint32_t)(whi >> 32));
    const uint32_t plo = __builtin_popcount(tlo), phi = __builtin_popcount(thi);
    // (words past n are zero: out-of-range loads; only Z needs the bound)
    const M128 V{ballot64(lane < n), ballot64(lane + 64u < n)};
    const M128 Z = V & M128{ballot64(tlo == 0), ballot64(thi == 0)};
    const M128 L{ballot64(plo >= 7), ballot64(phi >= 7)};
    const M128 F{ballot64(plo == 8), ballot64(phi == 8)};
    const M128 AZ = Z & shl1(Z);
    const M128 filled = ((L ^ add128(L, F)) & L) | F;
    const M128 AF = filled & shl1(filled);
    const M128 H = andnot(V, AZ | AF);
    const uint32_t hs_lo = 1u + plo + ((0x101u >> plo) & 1u);
    const uint32_t hs_hi = 1u + phi + ((0x101u >> phi) & 1u);
    const uint32_t slo = mask_sel(H.lo, hs_lo, tlo == 0 ? 0u : 8u);
    const uint32_t shi = mask_sel(H.hi, hs_hi, thi == 0 ? 0u : 8u);
    const uint32_t x = slo | (shi << 16);
    const uint32_t incl = wave_incl_scan(x);
    const uint32_t tot = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
    const uint32_t tot_lo = tot & 0xFFFFu;
    const uint32_t excl = incl - x;  // (per half: no borrow crosses bit 16)
    // run counts: the words up to the next head within the chunk
    const uint64_t nlo = (H.lo >> 1) >> lane;         // heads after word lane, in lo
    const uint32_t dlo0 = ffbl64(nlo);
    const uint32_t dlo1 = H.hi ? (63u - lane) + ffbl64(H.hi) : ~0u;  // the first head in hi
    const uint32_t dlo = dlo0 < 64u ? dlo0 : dlo1;
    const uint32_t dhi = ffbl64((H.hi >> 1) >> lane);
    const uint32_t cnt_lo = min(dlo, __builtin_elementwise_sub_sat(n, lane + 1u));
    const uint32_t cnt_hi = min(dhi, __builtin_elementwise_sub_sat(n, lane + 65u));
    ilo = cs_info(oc + (excl & 0xFFFFu), mask_sel(H.lo, tlo, kSelCopy), cnt_lo & 127u, slo);
    ihi = cs_info(oc + tot_lo + (excl >> 16), mask_sel(H.hi, thi, kSelCopy), cnt_hi & 127u, shi);
    return tot_lo + (tot >> 16);
}

// Pass 2 of one word (cs info layout): the record from the selector table
// (s0, s1), with the header and the 0xFF head's tail computed here:
//   r0 = perm(hi, lo, s0) | (zero head ? cnt << 8 : tag), r2 = 0xFF head ?
//   byte 7 | cnt << 8 : 0,
// shifted to its byte position and ORed into the region.  SYNC: a head
// writes the entries of the sync points it covers, d, d + 8, ... <= cnt words
// after it (d = the distance to the next sync point, shared by both words of
// a lane; b = the entry's byte offset in the tile's index window).
template <bool SYNC>
__device__ __forceinline__ void cs_emit_word_sel(uint64_t w, uint32_t info, uint8_t* region_m1,
                                                 Sel8 se, __amdgpu_buffer_rsrc_t srs,
                                                 uint32_t oc, uint32_t d, uint32_t b,
                                                 uint32_t wof = 0) {
    if (info >= kCsSkip) return;  // (the skip flag is the top field)
    const uint32_t lo = (uint32_t)w, hi = (uint32_t)(w >> 32);
    const uint32_t idx = __builtin_amdgcn_ubfe(info, kInfoPosBits, 9);
    const uint32_t cnt = info >> 22;
    const uint32_t hdr = idx == 0 ? (cnt << 8) : (idx & 0xFFu);  // (copy words: 256 & 0xFF)
    const uint32_t r0 = __builtin_amdgcn_perm(hi, lo, se.s0) | hdr;
    const uint32_t r1 = __builtin_amdgcn_perm(hi, lo, se.s1);
    const uint32_t r2 = idx == 0xFFu ? ((hi >> 24) | (cnt << 8)) : 0u;
    // (alignbyte reads bits 1:0: -(wof + pos) mod 4; wof = the wave's start
    // in a tile-contiguous layout, PACK_TILECOPY)
    const uint32_t s = 0u - info - wof;
    const uint32_t e0 = __builtin_amdgcn_alignbyte(r0, 0u, s);
    const uint32_t e1 = __builtin_amdgcn_alignbyte(r1, r0, s);
    const uint32_t e2 = __builtin_amdgcn_alignbyte(r2, r1, s);
    const uint32_t e3 = __builtin_amdgcn_alignbyte(0u, r2, s);
    const uint32_t pos = info & ((1u << kInfoPosBits) - 1u);
    uint32_t* b32 = reinterpret_cast<uint32_t*>(__builtin_align_down(region_m1 + pos, 4));
    if (!(PACK_ABL & 1)) {
    __hip_atomic_fetch_or(b32 + 0, e0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
    __hip_atomic_fetch_or(b32 + 1, e1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
    __hip_atomic_fetch_or(b32 + 2, e2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
    __hip_atomic_fetch_or(b32 + 3, e3, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
    } else {
        asm volatile("" ::"v"(e0), "v"(e1), "v"(e2), "v"(e3), "v"(b32));
    }
    if constexpr (SYNC && !(PACK_ABL & 2)) {
        if (idx < kSelCopy && d <= cnt) {
            const uint32_t rel = pos - oc;
            __builtin_amdgcn_raw_buffer_store_b32(rel | (d << 24), srs, (int)b, 0, 0);
#pragma clang loop unroll(disable) vectorize(disable)
            for (uint32_t dd = d + kSyncWords, bb = b + 4; dd <= cnt; dd += kSyncWords, bb += 4)
                __builtin_amdgcn_raw_buffer_store_b32(rel | (dd << 24), srs, (int)bb, 0, 0);
        }
    }
}

// The selector of a word's record (pass 2 reads a step's selectors before
// its emission's LDS atomics).
__device__ __forceinline__ Sel8 cs_sel(const Sel8* sel, uint32_t info) {
    return sel[__builtin_amdgcn_ubfe(info, kInfoPosBits, 9)];
}

template <bool SYNC>
__device__ __forceinline__ void cs_emit_word(uint64_t w, uint32_t info, uint8_t* region_m1,
                                             const Sel8* sel, __amdgpu_buffer_rsrc_t srs,
                                             uint32_t oc, uint32_t d, uint32_t b,
                                             uint32_t wof = 0) {
    if (info >= kCsSkip) return;  // (the skip flag is the top field)
    cs_emit_word_sel<SYNC>(w, info, region_m1, cs_sel(sel, info), srs, oc, d, b, wof);
}

// GAP (capnp_gpu_write_messages): chunk c is preceded by gap[c] bytes that the
// kernel leaves zero (out_off[c] is the gap's start), as pack_kernel's GAP.
template <bool SYNC, bool GAP = false>
__global__ void __launch_bounds__(kThreads, 8)
pack_cs_kernel(const uint64_t* __restrict__ in, const uint64_t* __restrict__ chunk_off,
               uint64_t nchunks, uint32_t tc, uint8_t* __restrict__ out, uint64_t out_cap,
               uint64_t* __restrict__ out_off, uint64_t* __restrict__ ts,
               uint64_t* __restrict__ gs, uint32_t* __restrict__ sync,
               uint8_t* __restrict__ ovf, const uint32_t* __restrict__ gap = nullptr) {
    static_assert(!(SYNC && GAP), "the sync index is not written with gaps");
    __shared__ Smem<false> sm;
    const uint32_t tid = threadIdx.x;
    const uint32_t lane = tid & 63u;
    const uint32_t wave = (uint32_t)__builtin_amdgcn_readfirstlane((int)(tid >> 6));
    const uint64_t tile = blockIdx.x;
#if PACK_PROF == 3
    if (tid == 0) {
        uint32_t xcc, hwid;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hwid));
        TRACE(tile, 0, RT());
        TRACE(tile, 6, ((uint64_t)xcc << 32) | hwid);
    }
#endif
    const uint64_t c0 = tile * tc;
    const uint64_t c1 = (c0 + tc < nchunks) ? c0 + tc : nchunks;
    const uint32_t nc = (uint32_t)(c1 - c0);
    const uint64_t* __restrict__ toff = chunk_off + c0;
    uint8_t* region = sm.stage[wave];
    // wave w: chunks [wc0, wc1), one per step
    const uint32_t q = (nc + kWaves - 1) / kWaves;
    const uint32_t wc0 = wave * q < nc ? wave * q : nc;
    const uint32_t wc1 = wc0 + q < nc ? wc0 + q : nc;
    const uint32_t nw = wc1 - wc0;
    const uint64_t TW0 = uniform64(chunk_off[c0]);
    const uint64_t WS0 = uniform64(toff[wc0]);
    const uint64_t TW1 = uniform64(chunk_off[c1]);
    const uint32_t tile_bytes = (uint32_t)((TW1 - TW0) * 8);
    const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<uint64_t*>(in + TW0), 0, (int)tile_bytes, 0x00020000);
    uint64_t clo[kCsSteps], chi[kCsSteps];
    // Every load of the prologue is issued in one round trip: the scalar
    // offsets (TW0, TW1, the wave's first chunk WS0), the wave's chunk offsets
    // (one buffer load, lane l <= nw: toff[wc0 + l]; lanes past them read 0,
    // so no branch and no wait at its join), the selector table entry (written
    // to LDS after the word loads), and the words themselves, speculatively:
    // chunk s of the wave at WS0 + 128 s.  That is the step layout exactly
    // when every chunk of the wave but its last holds 128 words (1 KiB
    // segments); otherwise the steps load again once the offsets are in.
    // (The compiler had waited for the table entry, then for each of the two
    // offset loads, before the word loads: four round trips.)
    // (the offsets' low words: lengths and tile offsets fit 32 bits)
    const __amdgpu_buffer_rsrc_t crs = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<uint64_t*>(toff + wc0), 0, (int)((nw + 1) * 8), 0x00020000);
    const uint32_t o = __builtin_amdgcn_raw_buffer_load_b32(crs, (int)(lane * 8u), 0, 0);
    uint32_t gv = 0;  // GAP: lane s = the gap before the wave's chunk s
    if constexpr (GAP) {
        const __amdgpu_buffer_rsrc_t grs = __builtin_amdgcn_make_buffer_rsrc(
            const_cast<uint32_t*>(gap + c0 + wc0), 0, (int)(nw * 4), 0x00020000);
        gv = __builtin_amdgcn_raw_buffer_load_b32(grs, (int)(lane * 4u), 0, 0);
    }
    const Sel8 selv = kSel8Table.e[tid];
    const uint32_t sb = (uint32_t)(WS0 - TW0);
#pragma unroll
    for (uint32_t s = 0; s < kCsSteps; s++) {
        const uint32_t vlo = s < nw ? (sb + kCsWords * s + lane) * 8u : 0x80000000u;
        const uint32_t vhi = s < nw ? (sb + kCsWords * s + 64u + lane) * 8u : 0x80000000u;
        const auto x = __builtin_amdgcn_raw_buffer_load_b64(rsrc, (int)vlo, 0, 0);
        const auto y = __builtin_amdgcn_raw_buffer_load_b64(rsrc, (int)vhi, 0, 0);
        clo[s] = ((uint64_t)x[1] << 32) | x[0];
        chi[s] = ((uint64_t)y[1] << 32) | y[0];
    }
    const uint32_t onext = (uint32_t)__shfl_down((int)o, 1, 64);
    const uint32_t d_off = lane < nw ? o - (uint32_t)TW0 : 0u;
    const uint32_t d_len = lane < nw ? onext - o : 0u;
    const bool ok = nw <= kCsSteps && ballot64(lane < nw && d_len > kCsWords) == 0;
    if (lane == 0) sm.wave_steps[wave] = ok ? 0u : 1u;
    if (ballot64(lane + 1u < nw && d_len != kCsWords) != 0) {
        // (the speculative values enter the reloaded ones through an opaque
        // zero, so the compiler keeps their loads ahead of this branch)
        uint64_t z;
        asm volatile("s_mov_b64 %0, 0" : "=s"(z));
#pragma unroll
        for (uint32_t s = 0; s < kCsSteps; s++) {
            const uint32_t a = (uint32_t)__builtin_amdgcn_readlane((int)d_off, s);
            const uint32_t n = s < nw ? (uint32_t)__builtin_amdgcn_readlane((int)d_len, s) : 0u;
            const uint32_t vlo = lane < n ? (a + lane) * 8u : 0x80000000u;
            const uint32_t vhi = lane + 64u < n ? (a + lane + 64u) * 8u : 0x80000000u;
            const auto x = __builtin_amdgcn_raw_buffer_load_b64(rsrc, (int)vlo, 0, 0);
            const auto y = __builtin_amdgcn_raw_buffer_load_b64(rsrc, (int)vhi, 0, 0);
            clo[s] = (((uint64_t)x[1] << 32) | x[0]) | (clo[s] & z);
            chi[s] = (((uint64_t)y[1] << 32) | y[0]) | (chi[s] & z);
        }
    }
    else {
        // the wave's last chunk may be short: its step's words past it are
        // the next wave's (pass 1 takes words past n as zero)
        const uint32_t nl = nw ? (uint32_t)__builtin_amdgcn_readlane((int)d_len, nw - 1) : 0u;
#pragma unroll
        for (uint32_t s = 0; s < kCsSteps; s++) {
            if (s + 1 == nw) {
                clo[s] = lane < nl ? clo[s] : 0ull;
                chi[s] = lane + 64u < nl ? chi[s] : 0ull;
            }
        }
    }
    sm.sel[tid] = selv;
    if (tid == 0) sm.sel[kSelCopy] = kSel8Table.e[kSelCopy];
    for (uint32_t i = tid; i < nc; i += kThreads) sm.chunk_size[i] = 0;
    __syncthreads();
    bool staged = true;
#pragma unroll
    for (int w = 0; w < kWaves; w++) staged &= sm.wave_steps[w] == 0;
    staged = __builtin_amdgcn_readfirstlane((int)staged) != 0;

    LookbackArgs LA;
    LA.ts = ts;
    LA.gs = gs;
    LA.ntiles = gridDim.x;
    LA.in = in;
    LA.chunk_off = chunk_off;
    LA.nchunks = nchunks;
    LA.tc = tc;
    LA.gap = GAP ? gap : nullptr;
    LA.wt = 0;
    LA.wlo = LA.whi = LA.g0 = 0;
    LA.map = nullptr;
    const uint64_t k0 = (TW0 + kSyncWords - 1) / kSyncWords;
    const uint64_t k1 = (TW1 + kSyncWords - 1) / kSyncWords;

    if (!staged) {
        // a chunk longer than a step: sizes by the streaming size pass,
        // offsets by the look-back; the bytes come from pack_ovf_kernel
        if constexpr (SYNC)
            for (uint32_t i = tid; i < (uint32_t)(k1 - k0); i += kThreads) sync[k0 + i] = kSyncNone;
        const uint32_t mis = (uint32_t)(reinterpret_cast<uintptr_t>(out) & 15u);
        run_streaming<MODE_SIZE>(in, toff, sm.chunk_size, sm.chunk_pos, nc, wave, lane, region,
                                 sm.sel, out - mis, mis, out_cap, GAP ? gap + c0 : nullptr);
        __syncthreads();
        if (wave == 0) {
            const uint64_t agg = scan_chunks(sm, nc, lane);
            publish(LA, tile, agg, lane);
            const uint64_t excl = tile_offset(LA, tile, agg, lane);
            if (lane < nc) sm.chunk_pos[lane] += excl;
            if (c1 == nchunks && lane == 0) out_off[nchunks] = excl + agg;
            if (lane == 0) ovf[tile] = 1;
        }
        __syncthreads();
        for (uint32_t i = tid; i < nc; i += kThreads) out_off[c0 + i] = sm.chunk_pos[i];
        return;
    }

    for (uint32_t o = 16 * lane; o < kStageRegion; o += 16 * CAPNP_WAVE)
        *reinterpret_cast<uint4*>(region + o) = make_uint4(0, 0, 0, 0);
#if PACK_PROF == 3
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (tid == 0) TRACE(tile, 1, RT());
#endif

    // ---- pass 1: sizes and positions
    uint32_t ilo[kCsSteps], ihi[kCsSteps];
    uint32_t rec_oc = 0;  // lane s: region start of chunk s
    uint32_t local = 0;
#pragma unroll
    for (uint32_t s = 0; s < kCsSteps; s++) {
        const uint32_t n = s < nw ? (uint32_t)__builtin_amdgcn_readlane((int)d_len, s) : 0u;
        uint32_t g = 0;
        if constexpr (GAP) g = (uint32_t)__builtin_amdgcn_readlane((int)gv, s);
        local += g;  // (GAP: the chunk's bytes start after its gap)
        const uint32_t sz = cs_size_step(clo[s], chi[s], n, lane, local, ilo[s], ihi[s]);
        rec_oc = lane == s ? local : rec_oc;
        if (lane == s && s < nw) sm.chunk_size[wc0 + s] = sz + g;
        local += sz;
        __builtin_amdgcn_sched_barrier(0);
    }
    if (lane == 0) sm.wave_bytes[wave] = local;
    __syncthreads();
    bool fits = true;
    uint32_t woff = 0, tbytes = 0;  // (PACK_TILECOPY: this wave's start, the tile's bytes)
#pragma unroll
    for (int w = 0; w < kWaves; w++) {
        const uint32_t wb = (uint32_t)sm.wave_bytes[w];
        if (PACK_TILECOPY) {
            woff += (uint32_t)w < wave ? wb : 0u;
            tbytes += wb;
        } else {
            fits &= wb <= kStageBytes;
        }
    }
    if (PACK_TILECOPY) fits = tbytes <= kWaves * kStageBytes;
    fits = __builtin_amdgcn_readfirstlane((int)fits) != 0;
    woff = (uint32_t)__builtin_amdgcn_readfirstlane((int)woff);
    uint64_t agg = 0;
    if (wave == 0) {
        agg = scan_chunks32(sm, nc, lane);
        publish(LA, tile, agg, lane);
#if PACK_PROF == 3
        if (lane == 0) TRACE(tile, 2, RT());
#endif
    }
    const bool early_group = (tile % kGroup) == kGroup - 1;
    if (early_group && wave == kWaves - 1) {
        // (the same sum as wave 0's agg: wave w's local is the sum of the
        // sizes it stored for its chunks wc0 .. wc0 + nw - 1 (sz = 0 past nw),
        // and the waves' chunks partition the tile's nc; a mismatch would
        // shift every later tile's offsets, which the parity tests compare)
        uint32_t a = 0;
#pragma unroll
        for (int w = 0; w < kWaves; w++) a += (uint32_t)lds_u64(&sm.wave_bytes[w]);
        publish_group_early(LA, tile, a, lane);
    }
    // ---- pass 2: the bytes (the look-back loads are in flight)
    if (fits) {
        uint8_t* const region_m1 = (PACK_TILECOPY ? &sm.stage[0][0] + woff : region) - 1;
        const uint32_t t0 = (uint32_t)(k0 * kSyncWords - TW0);
        const __amdgpu_buffer_rsrc_t srs = __builtin_amdgcn_make_buffer_rsrc(
            SYNC ? sync + k0 : nullptr, 0, SYNC ? (int)((k1 - k0) * 4) : 0, 0x00020000);
#pragma unroll
        for (uint32_t s = 0; s < kCsSteps; s++) {
            const uint32_t oc = (uint32_t)__builtin_amdgcn_readlane((int)rec_oc, s);
            const uint32_t g = (uint32_t)__builtin_amdgcn_readlane((int)d_off, s);
            const uint32_t c = t0 - g;
            const uint32_t d = (c - lane) & (kSyncWords - 1);
            const uint32_t b = (lane + d - c) / (kSyncWords / 4u);
            cs_emit_word<SYNC>(clo[s], ilo[s], region_m1, sm.sel, srs, oc, d, b,
                               PACK_TILECOPY ? woff : 0u);
            cs_emit_word<SYNC>(chi[s], ihi[s], region_m1, sm.sel, srs, oc, d,
                               b + 64u / (kSyncWords / 4u), PACK_TILECOPY ? woff : 0u);
            __builtin_amdgcn_sched_barrier(0);
        }
    }
    if (wave == 0) {
#if PACK_PROF == 3
        wave_lds_sync();
        if (lane == 0) TRACE(tile, 3, RT());
#endif
#if PACK_ABL & 4
        const uint64_t excl = tile * 8800ull;
        (void)early_group;
#else
        const uint64_t excl = tile_offset(LA, tile, agg, lane, early_group);
#endif
#if PACK_PROF == 3
        if (lane == 0) TRACE(tile, 4, RT());
#endif
        if (lane < nc) sm.chunk_pos[lane] += excl;
        if (c1 == nchunks && lane == 0) out_off[nchunks] = excl + agg;
    }
    __syncthreads();
    for (uint32_t i = tid; i < nc; i += kThreads) out_off[c0 + i] = sm.chunk_pos[i];
    if (fits) {
        if (PACK_TILECOPY && !(PACK_ABL & 8)) {
            const uint32_t mis = (uint32_t)(reinterpret_cast<uintptr_t>(out) & 15u);
            const uint64_t D0 = lds_u64(&sm.chunk_pos[0]) + mis;
            copy_out_tile(&sm.stage[0][0], out - mis, D0, tbytes, out_cap + mis, lane, wave);
        } else if (nw && !(PACK_ABL & 8)) {
            const uint32_t mis = (uint32_t)(reinterpret_cast<uintptr_t>(out) & 15u);
            const uint64_t D0 = lds_u64(&sm.chunk_pos[wc0]) + mis;
            copy_out(region, out - mis, D0, lds_u64(&sm.wave_bytes[wave]), out_cap + mis, lane);
        }
#if PACK_PROF == 3
        __syncthreads();
        if (tid == 0) TRACE(tile, 5, RT());
#endif
    } else {
        if constexpr (SYNC)
            for (uint32_t i = tid; i < (uint32_t)(k1 - k0); i += kThreads) sync[k0 + i] = kSyncNone;
        if (tid == 0) ovf[tile] = 1;
    }
}

// Tiles whose staged ranges overflowed (ovf[t] set by pack_kernel, after its
// look-back wrote the chunks' offsets): the streaming path writes their
// bytes at those offsets.  One lane per tile finds them; a few workgroups.
template <bool GAP>
__global__ void __launch_bounds__(kThreads)
pack_ovf_kernel(const uint64_t* __restrict__ in, const uint64_t* __restrict__ chunk_off,
                uint64_t nchunks, uint32_t tc, uint8_t* __restrict__ out, uint64_t out_cap,
                const uint64_t* __restrict__ out_off, const uint8_t* __restrict__ ovf,
                uint64_t ntiles, const uint32_t* __restrict__ gap) {
    __shared__ Smem<GAP> sm;
    __shared__ uint32_t lst[kThreads];
    __shared__ uint32_t nl;
    const uint32_t tid = threadIdx.x;
    const uint32_t lane = tid & 63u;
    const uint32_t wave = (uint32_t)__builtin_amdgcn_readfirstlane((int)(tid >> 6));
    for (uint32_t i = tid; i <= kSelCopy; i += kThreads) sm.sel[i] = kSel8Table.e[i];
    const uint32_t mis = (uint32_t)(reinterpret_cast<uintptr_t>(out) & 15u);
    uint8_t* const outa = out - mis;
    uint8_t* region = sm.stage[wave];
    for (uint64_t base = (uint64_t)blockIdx.x * kThreads; base < ntiles;
         base += (uint64_t)gridDim.x * kThreads) {
        if (tid == 0) nl = 0;
        __syncthreads();
        if (base + tid < ntiles && ovf[base + tid]) lst[atomicAdd(&nl, 1u)] = tid;
        __syncthreads();
        const uint32_t n = nl;
        for (uint32_t k = 0; k < n; k++) {
            const uint64_t c0 = (base + lst[k]) * tc;
            const uint64_t c1 = c0 + tc < nchunks ? c0 + tc : nchunks;
            const uint32_t nc = (uint32_t)(c1 - c0);
            __syncthreads();  // the previous tile is done with the tables
            for (uint32_t j = tid; j < nc; j += kThreads) {
                sm.chunk_pos[j] = out_off[c0 + j];
                sm.chunk_size[j] = out_off[c0 + j + 1] - out_off[c0 + j];
                if constexpr (GAP) sm.chunk_gap[j] = gap[c0 + j];
            }
            __syncthreads();
            run_streaming<MODE_RING>(in, chunk_off + c0, sm.chunk_size, sm.chunk_pos, nc, wave,
                                     lane, region, sm.sel, outa, mis, out_cap,
                                     GAP ? sm.chunk_gap : nullptr);
        }
        __syncthreads();
    }
}

// ---------------------------------------------------------------------------
// Word-tile pack kernel.  Tile t = words [Ta, Tb) of the batch (kWtTile words
// at global multiples of kWtTile), wave w = range [Ta + w kWtRange, ...): the
// staged path of pack_kernel with steps of 64 consecutive words of the range,
// chunk starts as forced heads (resolve_step_s), the run state at the range
// start from carry_into and the words its last run goes on to absorb from
// run_ext.  Record bytes land as in the chunk tiles; a chunk's offset is the
// position of its first word's record.  Sync entries are written by the lane
// of the sync point's word: the covering record's position minus its
// chunk's, both tile-relative; for the chunk the tile starts inside of, the
// chunk's own start is unknown here, so the entry holds the record's position
// relative to the tile (24-bit two's complement) and pack_wt_fix_sync adds
// tile offset - chunk offset once every tile is placed.

#ifndef PACK_WT_OCC
#define PACK_WT_OCC 8
#endif

struct WtSmem {
    Sel8 sel[kSelCopy + 1];                // record assembly per tag (s0, s1)
    uint64_t wave_bytes[kWaves];
    uint32_t lastcs[kWaves];               // region position of the last chunk start
    uint64_t excl;
    uint32_t wcarry[kWaves];               // run state entering range w (w >= 1): type | rem << 2
    uint32_t wext[kWaves];                 // words from range w's start its open run absorbs
    alignas(16) uint32_t pad[4];           // (emit_step ORs a zero before a region)
    alignas(16) uint8_t stage[kWaves][kRegion];
    // (the region positions of the range's chunk-start words go into the
    // wave's region after its copy-out: a separate 4 KiB table had held the
    // kernel at 6 workgroups per CU)
};

__device__ __forceinline__ void size_step_s(StageState& pk, uint64_t w, uint32_t nvalid,
                                            uint64_t Sm, uint32_t lane, StepInfo& si) {
    const uint32_t tag = word_tag_dot((uint32_t)w, (uint32_t)(w >> 32));
    const uint32_t pop = __builtin_popcount(tag);
    const bool isz = tag == 0, isf = tag == 0xFF;
    const uint64_t V = low_mask(nvalid);
    const uint64_t Zm = ballot64(isz) & V;
    const uint64_t Lm = ballot64(pop >= 7) & V;
    const uint64_t Fm = ballot64(isf) & V;
    const StepMasks sm = resolve_step_s(Zm, Lm, Fm, Sm, nvalid, pk.carry);
    const uint32_t hsize = 1u + pop + ((0x101u >> pop) & 1u);
    const uint32_t size = mask_sel(sm.H, hsize, isz ? 0u : 8u);
    const uint32_t incl = wave_incl_scan(size);
    si.H = sm.H;
    si.pos = pk.o_c + pk.total + incl - size;
    si.tag = tag;
    si.meta = nvalid | (sm.absorbed_carry << 16);
    pk.carry = sm.next;
    pk.total += (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
}

// The run state at the end R1 = R0 + nw of a wave's range, from the range's
// own words (w[s] = word R0 + 64 s + lane, sb[s] = their chunk-start bits):
// the last sure head or chunk start in the range (word R0 itself counts
// only as a chunk start: its sureness needs word R0 - 1), then heads every
// 256 words through an all-zero / all-0xFF stretch, or the steps resolved
// forward from it.  homog = 1 / 2 when the range has none and is one
// all-zero / all-0xFF stretch (the state at R1 then follows from the state
// at R0: wt_compose), 3 when it has none and is neither (pop-7/8 words:
// the caller searches before R0).  No memory access: the in-kernel
// derivation's global searches (carry_in_b's deep windows, run_ext_b's
// forward loop) had made pack_wt_kernel 1194 us at config 4 (640 with a
// planned entry per range), its long zero / literal stretches sending most
// waves to them.
struct RangeExit {
    Carry c;
    uint32_t homog;
};
__device__ __forceinline__ RangeExit range_exit(const uint64_t (&w)[kStageSteps],
                                                uint32_t sbits, uint32_t nw, uint32_t lane) {
    uint32_t t[kStageSteps];
#pragma unroll
    for (uint32_t s = 0; s < kStageSteps; s++) t[s] = tag_of(w[s]);
    int ks = -1;
    uint32_t js = 0;
    bool allz = true, allf = true;  // over the words from the head found (or all)
#pragma unroll
    for (int s = kStageSteps - 1; s >= 0; s--) {
        const uint32_t nv = nw > 64u * s ? (nw - 64u * s < 64u ? nw - 64u * s : 64u) : 0u;
        const bool v = lane < nv;
        const uint32_t up = (uint32_t)__shfl_up((int)t[s], 1, 64);
        // (lane 63 of the step below by readlane, outside the select: a
        // shuffle under it would run with lane 63 masked off and read 0)
        const uint32_t below = s ? (uint32_t)__builtin_amdgcn_readlane((int)t[s > 0 ? s - 1 : 0], 63) : 0u;
        const uint32_t pt = lane ? up : below;
        const bool sure = v && (((sbits >> s) & 1u) || ((lane || s) && sure_head(t[s], pt)));
        if (ks < 0) {
            const uint64_t G = ballot64(sure);
            const uint32_t j = G ? 63u - (uint32_t)__builtin_clzll(G) : 0u;
            const bool mine = v && (!G || lane >= j);
            allz = allz && ballot64(mine && t[s] != 0) == 0;
            allf = allf && ballot64(mine && t[s] != 0xFF) == 0;
            if (G) {
                ks = s;
                js = j;
            }
        }
    }
    RangeExit r{{0u, 0u}, 0u};
    if (ks < 0) {
        r.homog = allz ? 1u : (allf ? 2u : 3u);
        return r;
    }
    const uint32_t sp = 64u * (uint32_t)ks + js;  // the last sure head, range-relative
    if (allz || allf) {
        r.c = Carry{allz ? 1u : 2u, 255u - (nw - 1u - sp) % 256u};
        return r;
    }
    Carry c{0, 0};  // resolve forward from the head (no sure head after it)
#pragma unroll
    for (int s = 0; s < kStageSteps; s++) {
        if (s < ks) continue;
        const uint32_t nv = nw > 64u * s ? (nw - 64u * s < 64u ? nw - 64u * s : 64u) : 0u;
        const uint64_t V = low_mask(nv) & (s == ks ? ~low_mask(js) : ~0ull);
        const uint32_t pop = __builtin_popcount(t[s]);
        c = resolve_step_s(ballot64(t[s] == 0) & V, ballot64(pop >= 7) & V,
                           ballot64(t[s] == 0xFF) & V, s == ks ? 1ull << js : 0ull,
                           s == ks ? 64u : nv, c)
                .next;
    }
    r.c = c;
    return r;
}

// The state after n words of one all-zero (T = 1) / all-0xFF (T = 2)
// stretch entered in state c: the open run of the same kind absorbs up to
// its remaining words, then a head every 256 words.
__device__ __forceinline__ Carry wt_compose(Carry c, uint32_t T, uint32_t n) {
    const uint32_t a = c.type == T ? c.rem : 0u;
    if (a >= n) return Carry{T, a - n};
    return Carry{T, 255u - (n - a - 1u) % 256u};
}

// Words from R0 on that the run open there (c) absorbs, from the range's
// own words: the leading words of its class (zero / at most one zero byte)
// before a chunk start, capped by the run's room.  *beyond = true when the
// whole range is such words and the run has room past it (the caller asks
// run_ext_b).
__device__ __forceinline__ uint32_t range_ext(const uint64_t (&w)[kStageSteps], uint32_t sbits,
                                              uint32_t nw, Carry c, uint32_t lane, bool& beyond) {
    beyond = false;
    if (c.type == 0 || c.rem == 0) return 0;
    uint32_t lead = 0;
    bool open = true;
#pragma unroll
    for (uint32_t s = 0; s < kStageSteps; s++) {
        const uint32_t nv = nw > 64u * s ? (nw - 64u * s < 64u ? nw - 64u * s : 64u) : 0u;
        const uint32_t tag = tag_of(w[s]);
        const bool cls = c.type == 1 ? tag == 0 : __builtin_popcount(tag) >= 7;
        const uint32_t cut = ctz64(ballot64(((sbits >> s) & 1u) != 0));
        const uint32_t lim = cut < nv ? cut : nv;
        const uint32_t l = ctz64(~ballot64(lane < lim && cls));
        if (open) {
            lead += l < lim ? l : lim;
            open = l >= lim && lim == 64u;
        }
    }
    beyond = open && lead < c.rem;
    return lead < c.rem ? lead : c.rem;
}

// (8 waves per SIMD: 64 VGPRs, LDS 20.2 KB)
template <bool SYNC>
__global__ void __launch_bounds__(kThreads, PACK_WT_OCC)
pack_wt_kernel(const uint64_t* __restrict__ in, const uint64_t* __restrict__ chunk_off,
               uint64_t nchunks, uint8_t* __restrict__ out, uint64_t out_cap,
               uint64_t* __restrict__ out_off, uint64_t* __restrict__ ts, uint64_t* __restrict__ gs,
               uint32_t* __restrict__ sync, const uint64_t* __restrict__ map,
               uint64_t* __restrict__ tile_off, const uint64_t* __restrict__ cbits,
               const uint32_t* __restrict__ plan, uint64_t wlo, uint64_t whi, uint64_t g0) {
    __shared__ WtSmem wm;
    WtSmem& sm = wm;
    const uint64_t b64 = wlo >> 6;
    const uint32_t tid = threadIdx.x;
    const uint32_t lane = tid & 63u;
    const uint32_t wave = (uint32_t)__builtin_amdgcn_readfirstlane((int)(tid >> 6));
    const uint64_t tile = blockIdx.x;
    LookbackArgs LA;
    LA.ts = ts;
    LA.gs = gs;
    LA.ntiles = gridDim.x;
    LA.in = in;
    LA.chunk_off = chunk_off;
    LA.nchunks = nchunks;
    LA.tc = 0;
    LA.gap = nullptr;
    LA.wt = 1;
    LA.wlo = wlo;
    LA.whi = whi;
    LA.g0 = g0;
    LA.map = map;
    uint64_t Ta, Tb;
    wt_tile_bounds(LA, tile, Ta, Tb);
    const uint64_t R0 = Ta + (uint64_t)wave * kWtRange;
    const bool have = R0 < Tb;
    const uint64_t R1 = !have ? R0 : (R0 + kWtRange < Tb ? R0 + kWtRange : Tb);
    const uint32_t nw = (uint32_t)(R1 - R0);
    const bool lastr = have && R1 == whi;
    const Sel8 selv = kSel8Table.e[tid];  // (written after the word loads are issued)
    uint8_t* region = sm.stage[wave];
    const uint32_t mis = (uint32_t)(reinterpret_cast<uintptr_t>(out) & 15u);
    uint8_t* const outa = out - mis;
    // the range's words (the run state at its ends comes from the plan
    // kernel, pack_wt_plan): every load goes out at once
    // (a buffer descriptor over the range: a lane past it reads 0, and the
    // unconditional loads let each step wait for its own load only)
    uint64_t cache[kStageSteps];
    {
        const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(
            const_cast<uint64_t*>(in + R0), 0, (int)(nw * 8u), 0x00020000);
#pragma unroll
        for (uint32_t s = 0; s < kStageSteps; s++) {
            const auto v = __builtin_amdgcn_raw_buffer_load_b64(rsrc, (int)((64u * s + lane) * 8u), 0, 0);
            cache[s] = ((uint64_t)v[1] << 32) | v[0];
        }
    }
    sm.sel[tid] = selv;
    if (tid == 0) sm.sel[kSelCopy] = kSel8Table.e[kSelCopy];
    // the range's first chunks (their offsets are written after the
    // look-back; loaded now, off that path)
    // (unconditional loads at in-bounds indexes, selected afterwards: map and
    // plan have an entry past the last range, and the steps' chunk-start
    // bits are one vector load; guarded loads had each waited at its join)
    const uint64_t r = tile * kWaves + wave;
    const uint64_t cAr = uniform64(map[r]);
    // the run states at the tile's ends (pack_wt_plan plans tile starts
    // only); between the tile's ranges they come from the neighbouring
    // waves' words (below), which this workgroup holds anyway
    const uint32_t pin0 = uniform(plan[tile * kWaves]), pnext = uniform(plan[(tile + 1) * kWaves]);
    const uint64_t q0 = have ? 1 + (R0 >> 6) - b64 : 0;
    const uint64_t cbv = cbits[q0 + (lane < kStageSteps ? lane : kStageSteps)];
    const uint64_t cA = have ? cAr : nchunks;
    // a full range followed by another range of this tile
    const bool succ = have && wave + 1 < (uint32_t)kWaves && R1 < Tb;
    const uint64_t stv = chunk_off[cA + lane < nchunks ? cA + lane : nchunks];
    const uint64_t st0 = cA + lane < nchunks ? stv : ~0ull;
    // chunk starts (forced heads) of the steps
    uint64_t smk[kStageSteps];
    const uint32_t rr = (uint32_t)(R0 & 63);
#pragma unroll
    for (uint32_t s = 0; s < kStageSteps; s++) {
        const uint32_t nv = nw > 64u * s ? (nw - 64u * s < 64u ? nw - 64u * s : 64u) : 0u;
        const uint64_t lo = readlane64(cbv, s), hi = readlane64(cbv, s + 1);
        const uint64_t bits = rr ? (lo >> rr) | (hi << (64 - rr)) : lo;
        smk[s] = nv ? bits & low_mask(nv) : 0ull;
    }
    // (per-lane bits from here on: bit s = this lane's word of step s starts
    // a chunk; each use rebuilds the step's mask with one compare, so no
    // 64-bit mask stays live in SGPRs across the kernel -- with the eight
    // masks and the eight steps' head masks live, it spilled 162 SGPRs to
    // VGPR lanes, a v_writelane / v_readlane pair per use)
    uint32_t sbits = 0;
#pragma unroll
    for (uint32_t s = 0; s < kStageSteps; s++) sbits |= mask_sel(smk[s], 1u << s, 0u);
    // the run state entering the next range (R1), from this range's own
    // words (range_exit): wcarry = type | rem << 2 | homog << 10
    if (succ) {
        uint32_t rec = 0;
        if (((readlane64(cbv, kStageSteps) >> rr) & 1) == 0) {  // R1 inside a chunk
            const RangeExit ex = range_exit(cache, sbits, nw, lane);
            Carry c = ex.c;
            uint32_t hg = ex.homog;
            if (hg == 3) {  // no sure head, pop-7/8 words: search before R0 (rare)
                c = carry_in_b<64, 2>(in, cbits, b64, wlo, R1, lane, cache[kStageSteps - 1],
                                   readlane64(cache[kStageSteps - 2], 63),
                                   ballot64(((sbits >> (kStageSteps - 1)) & 1u) != 0));
                hg = 0;
            }
            rec = c.type | (c.rem << 2) | (hg << 10);
        }
        if (lane == 0) wm.wcarry[wave + 1] = rec;
    }
    for (uint32_t o = 16 * lane; o < kRegion; o += 16 * CAPNP_WAVE)
        *reinterpret_cast<uint4*>(region + o) = make_uint4(0, 0, 0, 0);
    wave_lds_sync();
    // (pin the words here: nothing of pass 1 is computed ahead of the carry,
    // which would keep eight steps' worth of values live through it)
#pragma unroll
    for (uint32_t s = 0; s < kStageSteps; s++) asm volatile("" : "+v"(cache[s]));
    __syncthreads();
    // the state entering this range: the tile's planned entry, carried
    // through the earlier ranges (a homogeneous range composes: wt_compose)
    Carry cin{pin0 & 3u, (pin0 >> 2) & 0xFFu};
    for (uint32_t v = 1; v <= wave; v++) {
        const uint32_t e = uniform(wm.wcarry[v]);
        const uint32_t hg = e >> 10;
        cin = hg ? wt_compose(cin, hg, kWtRange) : Carry{e & 3u, (e >> 2) & 0xFFu};
    }
    if (!have) cin = Carry{0, 0};
#ifdef WT_CHECK
    if (have && wave > 0) {  // (diagnostic: the global search's state at R0)
        const uint64_t wq = in[R0 - 64 + lane];
        const uint64_t wpq = in[R0 - 65];
        const uint64_t bq = start_bits(cbits, b64, R0 - 64);
        const bool cs0 = (ballot64((sbits & 1u) != 0) & 1ull) != 0;
        const Carry oc = cs0 ? Carry{0, 0} : carry_in_b<64>(in, cbits, b64, wlo, R0, lane, wq, wpq, bq);
        if ((oc.type != cin.type || oc.rem != cin.rem) && lane == 0) {
            static __device__ unsigned int nprint;
            if (atomicAdd(&nprint, 1u) < 24u) {
                uint32_t es[4];
                for (uint32_t v = 0; v < 4; v++) es[v] = v ? wm.wcarry[v] : pin0;
                printf("WTCHK tile %lu wave %u R0 %lu old {%u,%u} new {%u,%u} tag0 %02x e %x %x %x %x\n",
                       (unsigned long)tile, wave, (unsigned long)R0, oc.type, oc.rem, cin.type, cin.rem,
                       tag_of(cache[0]), es[0], es[1], es[2], es[3]);
            }
        }
    }
#endif
    if (have && wave > 0) {
        // the words from R0 on that the run open at R0 absorbs: the previous
        // range's last record (its pass 2 needs them)
        bool beyond = false;
        uint32_t ext = range_ext(cache, sbits, nw, cin, lane, beyond);
        if (beyond)  // (the run reaches past this range: only a short last range)
            ext = run_ext_b(in, cbits, b64, whi, R0, cin, lane, cache[0],
                            rr ? (readlane64(cbv, 0) >> rr) | (readlane64(cbv, 1) << (64 - rr))
                               : readlane64(cbv, 0));
        if (lane == 0) wm.wext[wave] = ext;
    }
    // pass 1: sizes and positions
    StepInfo si[kStageSteps];
    StageState pk;
    pk.begin(0);
    pk.carry = cin;
    uint32_t lastcs = ~0u;
    uint32_t hbits = 0;  // bit s = this lane heads a record in step s
    uint32_t metav = 0;  // lane s = step s's meta (nvalid | absorbed << 16)

#pragma unroll
    for (uint32_t s = 0; s < kStageSteps; s++) {
        const uint32_t nv = nw > 64u * s ? (nw - 64u * s < 64u ? nw - 64u * s : 64u) : 0u;
        const uint64_t Sm = ballot64(((sbits >> s) & 1u) != 0);
        size_step_s(pk, cache[s], nv, Sm, lane, si[s]);
        hbits |= mask_sel(si[s].H, 1u << s, 0u);
        metav = lane == s ? si[s].meta : metav;
        if (Sm)
            lastcs = (uint32_t)__builtin_amdgcn_readlane((int)si[s].pos, 63 - __builtin_clzll(Sm));
    }
    if (lane == 0) {
        sm.wave_bytes[wave] = pk.total;
        wm.lastcs[wave] = lastcs;
    }
    __syncthreads();
    // (the run open at R1 is the next range's carry: the words it absorbs)
    const uint32_t rext = (!have || lastr) ? 0u : (succ ? uniform(wm.wext[wave + 1]) : pnext >> 10);
    uint32_t woff = 0, agg = 0;
#pragma unroll
    for (int w = 0; w < kWaves; w++) {
        const uint32_t b = (uint32_t)lds_u64(&sm.wave_bytes[w]);
        woff += w < (int)wave ? b : 0u;
        agg += b;
    }
    if (wave == 0) publish(LA, tile, agg, lane);
        // pass 2: the bytes
    wave_lds_sync();
    {
        uint8_t* const region_m1 = region - 1;
        uint32_t ext = rext;
#pragma unroll
        for (int s = (int)kStageSteps - 1; s >= 0; s--) {
            const uint32_t e = ext;
            StepInfo sj = si[s];
            sj.H = ballot64(((hbits >> s) & 1u) != 0);
            sj.meta = (uint32_t)__builtin_amdgcn_readlane((int)metav, s);
            emit_step<false>(cache[s], sj, e, lane, region_m1, sm.sel, nullptr, 0, 0, 0);
            ext = (sj.meta >> 16) + (sj.H == 0 ? e : 0u);
        }
    }
    if (SYNC) {
        // the chunk open at R0 started at tile position oc (0: before the tile)
        uint32_t oc = 0;
        for (int w = (int)wave - 1; w >= 0; w--) {
            const uint32_t l = uniform(wm.lastcs[w]);
            if (l != ~0u) {
                uint32_t o = 0;
                for (int v = 0; v < w; v++) o += (uint32_t)lds_u64(&sm.wave_bytes[v]);
                oc = o + l;
                break;
            }
        }
        // the record open at R0 (a run from before it): its head word and
        // tile position (its head bytes and literal words precede R0's bytes)
        const uint32_t before = cin.type == 2 ? 255u - cin.rem : 0u;
        uint32_t hp = woff - (cin.type == 1 ? 2u : 10u + 8u * before);
        uint64_t hw = R0 - (255u - cin.rem) - 1u;
#pragma unroll
        for (uint32_t s = 0; s < kStageSteps; s++) {
            const uint32_t nv = (uint32_t)__builtin_amdgcn_readlane((int)metav, s) & 127u;
            const uint64_t base = R0 + 64u * s;
            const uint64_t H = ballot64(((hbits >> s) & 1u) != 0);
            const uint64_t Sm = ballot64(((sbits >> s) & 1u) != 0);
            const uint32_t tpos = woff + si[s].pos;
            const uint64_t below = low_mask(lane + 1);
            const uint64_t sb = Sm & below, hb = H & below;
            const uint32_t js = sb ? 63u - (uint32_t)__builtin_clzll(sb) : 0u;
            const uint32_t jh = hb ? 63u - (uint32_t)__builtin_clzll(hb) : 0u;
            const uint32_t pjs = (uint32_t)__shfl((int)tpos, (int)js, 64);
            const uint32_t pjh = (uint32_t)__shfl((int)tpos, (int)jh, 64);
            const uint64_t gw = base + lane;
            if (lane < nv && (gw & (kSyncWords - 1)) == 0) {
                const uint32_t myoc = sb ? pjs : oc;
                const uint32_t myhp = hb ? pjh : hp;
                const uint32_t d = (uint32_t)(gw - (hb ? base + jh : hw));
                sync[gw / kSyncWords] = ((myhp - myoc) & 0xFFFFFFu) | (d << 24);
            }
            if (Sm) oc = (uint32_t)__builtin_amdgcn_readlane((int)tpos, 63 - __builtin_clzll(Sm));
            if (H) {
                const uint32_t h = 63u - (uint32_t)__builtin_clzll(H);
                hp = (uint32_t)__builtin_amdgcn_readlane((int)tpos, (int)h);
                hw = base + h;
            }
        }
    }
    if (wave == 0) {
        const uint64_t excl = tile_offset(LA, tile, agg, lane);
        if (lane == 0) {
            wm.excl = excl;
            tile_off[tile] = excl;
            if (Tb == whi) out_off[nchunks] = excl + agg;
        }
    }
    __syncthreads();
    const uint64_t excl = lds_u64(&wm.excl);
    if (!have) return;
    copy_out(region, outa, excl + woff + mis, lds_u64(&sm.wave_bytes[wave]), out_cap + mis, lane);
    // the chunk-start words' region positions, into the region just copied
    // out (LDS ops of a wave run in order: its reads are done)
    uint16_t* const wpos = reinterpret_cast<uint16_t*>(region);
#pragma unroll
    for (uint32_t s = 0; s < kStageSteps; s++)
        if ((sbits >> s) & 1u) wpos[64u * s + lane] = (uint16_t)si[s].pos;
    wave_lds_sync();
    // offsets of the chunks that start in the range (in the batch's last
    // range also the empty chunks at its end)
    for (uint64_t c0 = cA;; c0 += CAPNP_WAVE) {
        const uint64_t c = c0 + lane;
        const uint64_t st = c0 == cA ? st0 : (c < nchunks ? chunk_off[c] : ~0ull);
        const bool inr = c < nchunks && (st < R1 || (lastr && st == R1));
        if (inr) out_off[c] = st < R1 ? excl + woff + wpos[st - R0] : excl + agg;
        if (ballot64(inr) != ~0ull) break;
    }
}

// Zeroes a[0, na) and b[0, nb) (words).
__global__ void __launch_bounds__(256)
k_zero2(uint64_t* __restrict__ a, uint64_t na, uint64_t* __restrict__ b, uint64_t nb) {
    const uint64_t step = (uint64_t)gridDim.x * 256;
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < na + nb; i += step) {
        if (i < na) a[i] = 0;
        else b[i - na] = 0;
    }
}

// Chunk-start bits (start_bits); cb zeroed beforehand.
__global__ void __launch_bounds__(256)
pack_wt_bits(const uint64_t* __restrict__ chunk_off, uint64_t nchunks, uint64_t whi, uint64_t b64,
             unsigned long long* __restrict__ cb) {
    const uint64_t c = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (c >= nchunks) return;
    const uint64_t st = chunk_off[c];
    if (st < whi) atomicOr(&cb[1 + (st >> 6) - b64], 1ull << (st & 63));
}

// words before a range examined first (16: 254 vs 190 us, more deep searches)
constexpr uint32_t kPlanWin = 64;
static_assert(kPlanWin >= 2 && kPlanWin <= 64, "plan window");
// Run state at a wave range's first word, one wave per range: plan[r] =
// type | rem << 2 | ext << 10, ext = the words from R0 on that the run open
// there absorbs (run_ext_b).  Launched for the tiles' first ranges only
// (rstride = kWaves): inside a tile, range w's state comes from range w - 1's
// last 64 words and the ext from range w's first words, both held by the
// tile's own waves (round 4; planning every range read ~2 KiB around each
// 4 KiB range, 519 MB of config 4's 1 GiB).  The pack kernel
// reads its tile's entry and the next tile's.
__global__ void __launch_bounds__(256)
pack_wt_plan(const uint64_t* __restrict__ in, const uint64_t* __restrict__ cbits, uint64_t wlo,
             uint64_t whi, uint64_t g0, uint64_t nranges, uint32_t rstride,
             uint32_t* __restrict__ plan) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t i = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (i >= nranges) return;
    const uint64_t r = i * rstride;  // (rstride kWaves: the tiles' first ranges only)
    const uint64_t g = g0 + r / kWaves;
    const uint64_t Ta = g * kWtTile > wlo ? g * kWtTile : wlo;
    const uint64_t R = uniform64(Ta + (r % kWaves) * kWtRange);
    const uint64_t b64 = wlo >> 6;
    uint32_t rec = 0;
    if (R < whi && R > wlo) {
        // Every load in one round trip: clamped addresses and selects instead
        // of guarded loads (the compiler waited at each guard's join).  The
        // W words before R (lanes 64 - W ..) and the word before them; the
        // words after R only when the run state at R is an open run.
        constexpr uint32_t W = kPlanWin;
        // (a buffer load over words [B, R), B = max(R - W - 1, wlo): lanes
        // outside it read 0 without a fetch, and no branch means no wait at
        // a join before the scalar loads below)
        const uint64_t B = R - W - 1 >= wlo ? R - W - 1 : wlo;
        const __amdgpu_buffer_rsrc_t wrs = __builtin_amdgcn_make_buffer_rsrc(
            const_cast<uint64_t*>(in + B), 0, (int)((R - B) * 8), 0x00020000);
        const uint64_t wi = R - 64 + lane;
        const uint32_t vo = wi >= B ? (uint32_t)(wi - B) * 8u : 0x80000000u;
        const auto xv = __builtin_amdgcn_raw_buffer_load_b64(wrs, (int)vo, 0, 0);
        const uint64_t x = ((uint64_t)xv[1] << 32) | xv[0];
        // (the words after R: with the full window they load with the rest)
        const uint64_t xa = W == 64 ? in[R + lane < whi ? R + lane : whi - 1] : 0ull;
        const uint64_t qa = uniform64(1 + (R >> 6) - b64), qb = uniform64(R >= 64 ? qa - 1 : qa);
        const uint32_t rr = (uint32_t)(R & 63);
        uint64_t ca0, ca1, cb0, cb1;
        sload4(cbits + qa, cbits + qa + 1, cbits + qb, cbits + qb + 1, ca0, ca1, cb0, cb1);
        const uint64_t wb = R >= wlo + 64 - lane ? x : 0ull;
        const uint64_t xp = W < 64 ? readlane64(x, 63u - W) : in[R - 65 >= wlo ? R - 65 : wlo];
        const uint64_t wp = R >= wlo + W + 1 ? xp : 0ull;  // word R - W - 1
        const uint64_t bb = R >= 64 ? (rr ? (cb0 >> rr) | (cb1 << (64 - rr)) : cb0) : 0ull;
        const uint64_t ba = rr ? (ca0 >> rr) | (ca1 << (64 - rr)) : ca0;
        if (!(ba & 1)) {  // R inside a chunk
            const Carry c = carry_in_b<W>(in, cbits, b64, wlo, R, lane, wb, wp, bb);
            uint32_t ext = 0;
            if (c.type != 0 && c.rem != 0) {
                const uint64_t wa = R + lane < whi ? (W == 64 ? xa : in[R + lane]) : 0ull;
                ext = run_ext_b(in, cbits, b64, whi, R, c, lane, wa, ba);
            }
            rec = c.type | (c.rem << 2) | (ext << 10);
        }
    }
    if (lane == 0) plan[r] = rec;
}

// First chunk starting at or after each wave range's first word.
__global__ void __launch_bounds__(256)
pack_wt_map(const uint64_t* __restrict__ chunk_off, uint64_t nchunks, uint64_t wlo, uint64_t whi,
            uint64_t g0, uint64_t nranges, uint64_t* __restrict__ map) {
    const uint64_t r = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (r >= nranges) return;
    const uint64_t g = g0 + r / kWaves;
    const uint64_t Ta = g * kWtTile > wlo ? g * kWtTile : wlo;
    const uint64_t R0 = Ta + (r % kWaves) * kWtRange;
    uint64_t lo = 0, hi = nchunks;  // in [0, nchunks]
    while (lo < hi) {
        const uint64_t mid = (lo + hi) / 2;
        if (chunk_off[mid] < R0) lo = mid + 1;
        else hi = mid;
    }
    map[r] = R0 < whi ? lo : nchunks;
}

// Sync entries of each tile's first chunk when it started before the tile:
// tile-relative record positions become chunk-relative.
// (one wave per tile, four tiles per workgroup: one-wave workgroups left
// the CUs' workgroup slots, not their waves, as the limit)
__global__ void __launch_bounds__(256)
pack_wt_fix_sync(const uint64_t* __restrict__ chunk_off, const uint64_t* __restrict__ out_off,
                 const uint64_t* __restrict__ map, const uint64_t* __restrict__ tile_off,
                 uint32_t* __restrict__ sync, uint64_t wlo, uint64_t whi, uint64_t g0,
                 uint64_t ntiles) {
    const uint64_t t = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const uint32_t lane = threadIdx.x & 63u;
    if (t >= ntiles) return;
    const uint64_t g = g0 + t;
    const uint64_t Ta = g * kWtTile > wlo ? g * kWtTile : wlo;
    const uint64_t Tb = (g + 1) * kWtTile < whi ? (g + 1) * kWtTile : whi;
    const uint64_t cA = map[t * kWaves];
    if (chunk_off[cA] == Ta) return;  // the tile starts a chunk
    const uint64_t c = cA - 1;
    const int64_t delta = (int64_t)(tile_off[t] - out_off[c]);
    const uint64_t end = chunk_off[cA] < Tb ? chunk_off[cA] : Tb;
    const uint64_t k0 = (Ta + kSyncWords - 1) / kSyncWords, k1 = (end + kSyncWords - 1) / kSyncWords;
    for (uint64_t k = k0 + lane; k < k1; k += 64) {
        const uint32_t v = sync[k];
        const int32_t rel = (int32_t)(v << 8) >> 8;  // 24-bit two's complement
        const int64_t f = (int64_t)rel + delta;
        sync[k] = (f < 0 || f >= (1 << 24)) ? kSyncNone : ((uint32_t)f | (v & 0xFF000000u));
    }
}

// ---------------------------------------------------------------------------
// One write_message call in one launch (the drop-in at the reference's call
// granularity: serialize_packed::write_message once per message,
// serialize_packed.rs:446-453 -> serialize.rs:574-679, benchmark.rs:207-259).
// The host lays the message's write_all chunks out in pinned memory (word 0
// of the table, the rest of the table, each segment) with their word
// offsets; one workgroup stages the words into LDS in one round trip, sizes
// every chunk with the streaming path's pass A (wave w: chunks w, w + 16, ...),
// places them by a scan and writes their bytes with pass B into the pinned
// output.  No look-back state, no second launch, one wait on the host.
constexpr uint32_t kMsgWords = 8448;   // words staged in LDS (table + segments: 64 KiB and a table)
constexpr uint32_t kMsgChunks = 516;   // word 0, the table rest, <= 511 segments (+ pad)
constexpr uint32_t kMsgSplit = 256;    // a last chunk of this many words is split over the waves
// (64: a 128-word write 13.9 vs 13.1 us, 1500 words the same: r05z)
// messages of at most this many words flush straight to the output (the few
// 16-byte flushes cost less than the copy's device round trip: 128 words
// 12.8 vs 13.1 us, 256 13.9 vs 14.2; 512 and up the same, r05z)
constexpr uint32_t kMsgDirect = 512;
// 16 waves (4 per SIMD): a wave's steps are chains of dependent LDS and
// scalar work, and one wave per SIMD left each SIMD idle between them
constexpr uint32_t kMsgWaves = 16;
constexpr uint32_t kMsgThreads = kMsgWaves * CAPNP_WAVE;

// Words from R on (up to `end`, the chunk's end) that the open run c absorbs.
__device__ __forceinline__ uint32_t run_ext_at(const uint64_t* in, uint64_t R, uint64_t end,
                                               Carry c, uint32_t lane) {
    if (c.type == 0 || c.rem == 0) return 0;
    uint32_t ext = 0;
    for (uint64_t p = R; p < end; p += 64) {
        const uint32_t nv = (uint32_t)(end - p < 64 ? end - p : 64);
        const uint32_t tag = lane < nv ? tag_of(in[p + lane]) : 0u;
        const bool cls = lane < nv && (c.type == 1 ? tag == 0 : __builtin_popcount(tag) >= 7);
        const uint32_t lead = ctz64(~ballot64(cls));
        ext += lead;
        if (lead < 64 || ext >= c.rem) break;
    }
    return ext < c.rem ? ext : c.rem;
}

struct MsgPackSmem {
    Sel8 sel[kSelCopy + 1];
    uint64_t off[kMsgChunks + 1];
    uint64_t chunk_size[kMsgChunks];
    uint64_t chunk_pos[kMsgChunks];
    uint32_t wsum[kMsgWaves];
    uint32_t rsize[kMsgWaves];  // split segment: packed bytes of each wave's range
    alignas(16) uint32_t pad[4];  // (emit ORs a zero into the dword before a region)
    alignas(16) uint8_t ring[kMsgWaves][kRing];
    alignas(16) uint64_t words[kMsgWords];
};

__device__ __forceinline__ void msg_pack_body(MsgPackSmem& S, const uint64_t* words,
                                              const uint64_t* off, uint32_t nchunks,
                                              uint32_t nwords, uint8_t* out, uint64_t out_cap,
                                              uint64_t* total, uint32_t* flag, uint32_t seq,
                                              uint8_t* scratch) {
    const uint32_t tid = threadIdx.x;
    const uint32_t lane = tid & 63u;
    const uint32_t wave = (uint32_t)__builtin_amdgcn_readfirstlane((int)(tid >> 6));
    // stage: every load in flight at once (one round trip to host memory).
    // The offsets by buffer loads (lanes past them read 0: no branch, so no
    // wait at a join), the words by LDS DMA in whole 64-vector groups (the
    // host pads both regions to 16 bytes).  (Plain loops had waited for each
    // iteration's loads before the next: a 1500-word message took five PCIe
    // round trips to stage.)
    constexpr uint32_t kOffIt = (kMsgChunks + 1 + kMsgThreads - 1) / kMsgThreads;
    uint64_t ov[kOffIt];
    {
        const __amdgpu_buffer_rsrc_t ors = __builtin_amdgcn_make_buffer_rsrc(
            const_cast<uint64_t*>(off), 0, (int)((nchunks + 1) * 8), 0x00020000);
#pragma unroll
        for (uint32_t k = 0; k < kOffIt; k++) {
            const auto x = __builtin_amdgcn_raw_buffer_load_b64(ors, (int)((tid + k * kMsgThreads) * 8u), 0, 0);
            ov[k] = ((uint64_t)x[1] << 32) | x[0];
        }
        const uint4* w4 = reinterpret_cast<const uint4*>(words);
        uint4* s4 = reinterpret_cast<uint4*>(S.words);
        const uint32_t nvec = (nwords + 1) / 2;
        for (uint32_t i0 = wave * CAPNP_WAVE; i0 < nvec; i0 += kMsgThreads) {
            const uint32_t i = i0 + lane;
            if (i0 + CAPNP_WAVE <= nvec) {
                __builtin_amdgcn_global_load_lds(
                    (const __attribute__((address_space(1))) void*)(w4 + i),
                    (__attribute__((address_space(3))) void*)(s4 + i0), 16, 0, 0);
            } else if (i < nvec) {
                s4[i] = w4[i];
            }
        }
    }
    for (uint32_t i = tid; i <= kSelCopy; i += kMsgThreads) S.sel[i] = kSel8Table.e[i];
#pragma unroll
    for (uint32_t k = 0; k < kOffIt; k++)
        if (tid + k * kMsgThreads <= nchunks) S.off[tid + k * kMsgThreads] = ov[k];
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's words are in
    __syncthreads();
#if SVC_PROF
    const uint64_t tp0 = __builtin_amdgcn_s_memrealtime();
#endif
    uint8_t* ring = S.ring[wave];
    // (the last chunk -- a message's one segment, usually the longest -- is
    // placed without its size: pass B measures it)
    if (tid == 0) S.chunk_size[nchunks - 1] = 0;
    run_streaming<MODE_SIZE, kMsgWaves>(S.words, S.off, S.chunk_size, S.chunk_pos, nchunks - 1, wave, lane,
                             ring, S.sel, nullptr, 0, 0, nullptr);
    // A long last chunk is split into one range per wave (64-word multiples):
    // each wave takes the run state entering its range from the words before
    // it (carry_into), sizes its range here and writes it in pass B, with the
    // words its open run absorbs past the range end counted into the run's
    // count byte (serialize_packed.rs:375-427 walk the chunk as one; the
    // ranges reproduce that walk exactly).  One wave had walked it alone: 64
    // serial steps for a 4096-word segment.
    const uint32_t lc = nchunks - 1;
    const uint64_t la = uniform64(S.off[lc]), lb = uniform64(S.off[nchunks]);
    const bool split = lb - la >= kMsgSplit;
    const uint64_t q = ((lb - la + kMsgWaves - 1) / kMsgWaves + 63) & ~63ull;
    const uint64_t ra = la + wave * q < lb ? la + wave * q : lb;
    const uint64_t rb = ra + q < lb ? ra + q : lb;
    Carry rcarry{0, 0};
    uint32_t rext = 0;
    if (split) {
        uint32_t sz = 0;
        if (ra < rb) {
            if (ra > la) rcarry = carry_into(S.words, la, ra, lane);
            Packer pk;
            pk.begin(0);
            pk.carry = rcarry;
            for (uint64_t p = ra; p < rb; p += 64) {
                const uint32_t nv = (uint32_t)(rb - p < 64 ? rb - p : 64);
                const uint64_t w = lane < nv ? S.words[p + lane] : 0ull;
                pk.step<MODE_SIZE>(w, nv, p + 64 >= rb, lane, nullptr, nullptr, nullptr);
            }
            sz = (uint32_t)pk.total;
            rext = run_ext_at(S.words, rb, lb, pk.carry, lane);
        }
        if (lane == 0) S.rsize[wave] = sz;
    }
    __syncthreads();
#if SVC_PROF
    const uint64_t tp1 = __builtin_amdgcn_s_memrealtime();
#endif
    // chunk positions: exclusive scan of the sizes, up to 3 chunks per thread
    {
        constexpr uint32_t kPer = (kMsgChunks + kMsgThreads - 1) / kMsgThreads;
        uint32_t v[kPer], sum = 0;
        uint32_t rsum = 0;
#pragma unroll
        for (int k = 0; k < kMsgWaves; k++) rsum += split ? S.rsize[k] : 0u;
#pragma unroll
        for (uint32_t k = 0; k < kPer; k++) {
            const uint32_t i = tid * kPer + k;
            v[k] = i < nchunks ? (split && i == lc ? rsum : (uint32_t)S.chunk_size[i]) : 0u;
            sum += v[k];
        }
        if (split && tid == 0) S.chunk_size[lc] = rsum;
        const uint32_t inc = wave_incl_scan(sum);
        if (lane == CAPNP_WAVE - 1) S.wsum[wave] = inc;
        __syncthreads();
        uint32_t run = inc - sum, all = 0;
#pragma unroll
        for (uint32_t k = 0; k < (uint32_t)kMsgWaves; k++) {
            if (k < wave) run += S.wsum[k];
            all += S.wsum[k];
        }
#pragma unroll
        for (uint32_t k = 0; k < kPer; k++) {
            const uint32_t i = tid * kPer + k;
            if (i < nchunks) S.chunk_pos[i] = run;
            run += v[k];
        }
        if (tid == 0) S.wsum[0] = all;  // (the chunks before the last)
    }
    __syncthreads();
#if SVC_PROF
    const uint64_t tp2 = __builtin_amdgcn_s_memrealtime();
#endif
    // (pass B's flushes go to device memory -- a step's bytes in 16-byte
    // stores that a PCIe write path would take one at a time -- and the
    // packed bytes cross to the host output in one coalesced copy)
    // (a short message's few flushes go straight out: kMsgDirect)
    const bool via = scratch && nwords > kMsgDirect;
    uint8_t* const dst = via ? scratch : out;
    const uint32_t mis = (uint32_t)(reinterpret_cast<uintptr_t>(dst) & 15u);
    uint64_t* last = reinterpret_cast<uint64_t*>(S.chunk_size + nchunks - 1);
    run_streaming<MODE_RING, kMsgWaves>(S.words, S.off, S.chunk_size, S.chunk_pos, split ? lc : nchunks, wave,
                             lane, ring, S.sel, dst - mis, mis, out_cap, nullptr,
                             split ? nullptr : last);
    if (split && ra < rb) {
        const uint64_t cpos = lds_u64(&S.chunk_pos[lc]);
        if (cpos + lds_u64(&S.chunk_size[lc]) <= out_cap) {  // (as run_streaming: fits or none)
            uint32_t before = 0;
            for (uint32_t k = 0; k < wave; k++) before += S.rsize[k];
            Packer pk;
            pk.begin(cpos + before + mis);
            pk.carry = rcarry;
            for (uint64_t p = ra; p < rb; p += 64) {
                const uint32_t nv = (uint32_t)(rb - p < 64 ? rb - p : 64);
                const bool lst = p + 64 >= rb;
                const uint64_t w = lane < nv ? S.words[p + lane] : 0ull;
                pk.step<MODE_RING>(w, nv, lst, lane, ring, dst - mis, S.sel, lst ? rext : 0u);
            }
        }
    }
    __syncthreads();
#if SVC_PROF
    const uint64_t tp3 = __builtin_amdgcn_s_memrealtime();
#endif
    const uint64_t tot = S.chunk_pos[nchunks - 1] + S.chunk_size[nchunks - 1];
    if (via) {
        // (scratch and out both 16-byte aligned: whole vectors, the last one
        // padded -- out has the bound's room)
        const uint64_t nv = ((tot < out_cap ? tot : out_cap) + 15) / 16;
        const uint4* s4 = reinterpret_cast<const uint4*>(scratch);
        uint4* o4 = reinterpret_cast<uint4*>(out);
        for (uint64_t i = tid; i < nv; i += kMsgThreads) o4[i] = s4[i];
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // (this wave's stores have landed)
    __syncthreads();
#if SVC_PROF
    if (tid == 0) {  // (slots 3-6, 9: sizes, scan, pass B, copy-out; the stage's end)
        atomicAdd(&g_svc_prof[3], (unsigned long long)(tp1 - tp0));
        atomicAdd(&g_svc_prof[4], (unsigned long long)(tp2 - tp1));
        atomicAdd(&g_svc_prof[5], (unsigned long long)(tp3 - tp2));
        atomicAdd(&g_svc_prof[9], (unsigned long long)(__builtin_amdgcn_s_memrealtime() - tp3));
        atomicAdd(&g_svc_prof[6], (unsigned long long)tp0);
    }
#endif
    if (tid == 0) {
        total[0] = tot;
        if (flag) {  // (the host waits on this flag: everything above is visible first)
            __threadfence_system();
            __hip_atomic_store(flag, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
}

__global__ void __launch_bounds__(kMsgThreads)
msg_pack_kernel(const uint64_t* __restrict__ words, const uint64_t* __restrict__ off,
                uint32_t nchunks, uint32_t nwords, uint8_t* __restrict__ out, uint64_t out_cap,
                uint64_t* __restrict__ total, uint32_t* __restrict__ flag, uint32_t seq,
                uint8_t* __restrict__ scratch) {
    __shared__ MsgPackSmem S;
    msg_pack_body(S, words, off, nchunks, nwords, out, out_cap, total, flag, seq, scratch);
}

// The same call served by a resident workgroup (common.h, svc_next; the
// request's arguments: SvcPackReq).  The completion flag is the context's
// own.
__global__ void __launch_bounds__(kMsgThreads)
msg_pack_service(const uint64_t* line, uint64_t* mark, uint32_t gen, uint64_t idle_ticks,
                 uint32_t* flag) {
    __shared__ MsgPackSmem S;
    __shared__ SvcCmd cmd;
    const uint32_t tid = threadIdx.x;
    const uint32_t lane = tid & 63u;
    const uint32_t wave = (uint32_t)__builtin_amdgcn_readfirstlane((int)(tid >> 6));
    uint32_t last = 0;
    while (svc_next(line, cmd, gen, last, idle_ticks, wave, lane)) {
        const SvcPackReq& q = *reinterpret_cast<const SvcPackReq*>(cmd.a);
        const uint64_t nn = uniform64(q.counts);
        uint8_t* const out = reinterpret_cast<uint8_t*>(uniform64(q.out));
        msg_pack_body(S, reinterpret_cast<const uint64_t*>(uniform64(q.words)),
                      reinterpret_cast<const uint64_t*>(uniform64(q.off)), (uint32_t)nn,
                      (uint32_t)(nn >> 32), out, uniform64(q.out_cap),
                      reinterpret_cast<uint64_t*>(out - 16), flag, last,
                      reinterpret_cast<uint8_t*>(uniform64(q.scratch)));
        svc_prof_done(cmd, tid);
        __syncthreads();
    }
    svc_exit(mark, gen, tid);
}

}  // namespace

// Words per tile the staged path is sized for (kWaves waves x kStageSteps
// 64-word steps); the host picks chunks_per_tile ~ this / mean chunk words.
extern "C" uint32_t capnp_pack_tile_words(void) { return kWaves * 64 * kStageSteps; }

// Workspace layout (zeroed every call; uncached memory, capi.hip):
// ts[ntiles] tile records, then gs[ngroups] group records.
// Look-back records above the tiles': level 1 (groups of 64 tiles), then the
// deeper levels of lookback_ml (blocks of 64^k tiles) up to one record.
static uint64_t level_record_count(uint64_t ntiles) {
    uint64_t total = 0;
    for (uint64_t n = ntiles; n > 1;) {
        n = (n + kGroup - 1) / kGroup;
        total += n;
    }
    return total ? total : 1;
}

extern "C" size_t capnp_pack_state_bytes(uint64_t nchunks, uint32_t tc) {
    const uint64_t ntiles = (nchunks + tc - 1) / tc;
    return ((ntiles + level_record_count(ntiles)) * 8 + ntiles + 15) & ~size_t(15);  // + overflow flags
}

// The tiles' overflow flags follow the tile and level records in the state.
static uint8_t* pack_ovf_flags(uint64_t* d_state, uint64_t ntiles) {
    return reinterpret_cast<uint8_t*>(d_state + ntiles + level_record_count(ntiles));
}
static dim3 pack_ovf_grid(uint64_t ntiles) {
    const uint64_t g = (ntiles + kThreads - 1) / kThreads;
    return dim3((uint32_t)(g < 1024 ? g : 1024));
}

extern "C" hipError_t capnp_launch_pack(const uint64_t* d_in, const uint64_t* d_chunk_off,
                                        uint64_t nchunks, uint32_t tc, uint8_t* d_out,
                                        uint64_t out_cap, uint64_t* d_out_off,
                                        uint64_t* d_state, uint32_t* d_sync,
                                        hipStream_t stream) {
    if (tc == 0 || tc > kMaxTileChunks) return hipErrorInvalidValue;
    const uint64_t ntiles = (nchunks + tc - 1) / tc;
    if (nchunks == 0) {
        return hipMemsetAsync(d_out_off, 0, sizeof(uint64_t), stream);
    }
    hipError_t e = hipMemsetAsync(d_state, 0, capnp_pack_state_bytes(nchunks, tc), stream);
    if (e != hipSuccess) return e;
    uint8_t* ovf = pack_ovf_flags(d_state, ntiles);
    if (tc == kWaves * kCsSteps) {
        // chunks of at most 128 words (tc chosen for a mean of 65-128 words;
        // a tile with a longer chunk takes the streaming size pass)
        if (d_sync)
            hipLaunchKernelGGL((pack_cs_kernel<true>), dim3((uint32_t)ntiles), dim3(kThreads), 0,
                               stream, d_in, d_chunk_off, nchunks, tc, d_out, out_cap, d_out_off,
                               d_state, d_state + ntiles, d_sync, ovf);
        else
            hipLaunchKernelGGL((pack_cs_kernel<false>), dim3((uint32_t)ntiles), dim3(kThreads),
                               0, stream, d_in, d_chunk_off, nchunks, tc, d_out, out_cap,
                               d_out_off, d_state, d_state + ntiles, d_sync, ovf);
    } else if (d_sync) {
        hipLaunchKernelGGL((pack_lean_kernel<true>), dim3((uint32_t)ntiles), dim3(kThreads), 0,
                           stream, d_in, d_chunk_off, nchunks, tc, d_out, out_cap, d_out_off,
                           d_state, d_state + ntiles, d_sync, ovf);
    } else {
        hipLaunchKernelGGL((pack_lean_kernel<false>), dim3((uint32_t)ntiles), dim3(kThreads), 0,
                           stream, d_in, d_chunk_off, nchunks, tc, d_out, out_cap, d_out_off,
                           d_state, d_state + ntiles, d_sync, ovf);
    }
    hipLaunchKernelGGL((pack_ovf_kernel<false>), pack_ovf_grid(ntiles), dim3(kThreads), 0, stream,
                       d_in, d_chunk_off, nchunks, tc, d_out, out_cap, d_out_off, ovf, ntiles,
                       nullptr);
    return hipGetLastError();
}

// Pack with a leading gap of d_gap[c] bytes before every chunk c: out_off[c]
// is the gap's start, the chunk's bytes follow the gap, the gap bytes are
// written as zeros.
extern "C" hipError_t capnp_launch_pack_gap(const uint64_t* d_in, const uint64_t* d_chunk_off,
                                            uint64_t nchunks, uint32_t tc, uint8_t* d_out,
                                            uint64_t out_cap, uint64_t* d_out_off,
                                            uint64_t* d_state, const uint32_t* d_gap,
                                            hipStream_t stream) {
    if (tc == 0 || tc > kMaxTileChunks || !d_gap) return hipErrorInvalidValue;
    const uint64_t ntiles = (nchunks + tc - 1) / tc;
    if (nchunks == 0) return hipMemsetAsync(d_out_off, 0, sizeof(uint64_t), stream);
    hipError_t e = hipMemsetAsync(d_state, 0, capnp_pack_state_bytes(nchunks, tc), stream);
    if (e != hipSuccess) return e;
    uint8_t* ovf = pack_ovf_flags(d_state, ntiles);
    if (tc == kWaves * kCsSteps)  // (chunks of <= 128 words: the chunk-step kernel)
        hipLaunchKernelGGL((pack_cs_kernel<false, true>), dim3((uint32_t)ntiles), dim3(kThreads),
                           0, stream, d_in, d_chunk_off, nchunks, tc, d_out, out_cap, d_out_off,
                           d_state, d_state + ntiles, nullptr, ovf, d_gap);
    else
        hipLaunchKernelGGL((pack_kernel<false, true>), dim3((uint32_t)ntiles), dim3(kThreads), 0,
                           stream, d_in, d_chunk_off, nchunks, tc, d_out, out_cap, d_out_off,
                           d_state, d_state + ntiles, nullptr, d_gap, ovf);
    hipLaunchKernelGGL((pack_ovf_kernel<true>), pack_ovf_grid(ntiles), dim3(kThreads), 0, stream,
                       d_in, d_chunk_off, nchunks, tc, d_out, out_cap, d_out_off, ovf, ntiles,
                       d_gap);
    return hipGetLastError();
}

// Word tiles (batches of long chunks): workspace = map (first chunk of every
// wave range) + tile offsets; the look-back records live in d_state
// (capnp_pack_state_bytes(ntiles, 1), uncached).  [wlo, whi) = the batch's
// words, read by the caller (the grid is sized by them).
extern "C" uint64_t capnp_pack_wt_tiles(uint64_t wlo, uint64_t whi) {
    return whi > wlo ? (whi + kWtTile - 1) / kWtTile - wlo / kWtTile : 0;
}

static uint64_t wt_bits_words(uint64_t wlo, uint64_t whi) {
    return ((whi + 63) >> 6) - (wlo >> 6) + 16;
}

extern "C" size_t capnp_pack_wt_ws_bytes(uint64_t wlo, uint64_t whi) {
    const uint64_t nt = capnp_pack_wt_tiles(wlo, whi);
    return (nt * (kWaves + 1) + wt_bits_words(wlo, whi)) * 8 + (nt * kWaves + 1) * 4 + 64;
}

extern "C" uint32_t capnp_pack_wt_words(void) { return kWtTile; }

extern "C" int capnp_pack_wt_dbg(uint32_t* out) {
    (void)out;
    return -1;
}

extern "C" hipError_t capnp_launch_pack_wt(const uint64_t* d_in, const uint64_t* d_chunk_off,
                                           uint64_t nchunks, uint8_t* d_out, uint64_t out_cap,
                                           uint64_t* d_out_off, uint64_t* d_state, void* d_ws,
                                           size_t ws_bytes, uint32_t* d_sync, uint64_t wlo,
                                           uint64_t whi, hipStream_t stream) {
    const uint64_t ntiles = capnp_pack_wt_tiles(wlo, whi);
    if (nchunks == 0 || ntiles == 0 || ws_bytes < capnp_pack_wt_ws_bytes(wlo, whi))
        return hipErrorInvalidValue;
    const uint64_t g0 = wlo / kWtTile;
    uint64_t* map = reinterpret_cast<uint64_t*>(d_ws);
    uint64_t* toff = map + ntiles * kWaves;
    uint64_t* cbits = toff + ntiles;
    uint32_t* plan = reinterpret_cast<uint32_t*>(cbits + wt_bits_words(wlo, whi));
    {
        // the look-back state and the chunk-start bits cleared in one launch
        // (two runtime memsets were four fill kernels, ~20 us a call)
        const uint64_t na = (capnp_pack_state_bytes(ntiles, 1) + 7) / 8;
        const uint64_t nb = wt_bits_words(wlo, whi);
        const uint64_t nt = na + nb;
        const uint32_t blocks = (uint32_t)std::min<uint64_t>((nt + 255) / 256, 4096);
        hipLaunchKernelGGL(k_zero2, dim3(blocks), dim3(256), 0, stream, d_state, na, cbits, nb);
    }
    hipLaunchKernelGGL(pack_wt_bits, dim3((uint32_t)((nchunks + 255) / 256)), dim3(256), 0, stream,
                       d_chunk_off, nchunks, whi, wlo >> 6,
                       reinterpret_cast<unsigned long long*>(cbits));
    const uint64_t nr = ntiles * kWaves;
    hipLaunchKernelGGL(pack_wt_map, dim3((uint32_t)((nr + 255) / 256)), dim3(256), 0, stream,
                       d_chunk_off, nchunks, wlo, whi, g0, nr, map);
    // run states at the tiles' first ranges (and past the last tile); the
    // kernel derives the others from the words it holds
    hipLaunchKernelGGL(pack_wt_plan, dim3((uint32_t)((ntiles + 1 + 3) / 4)), dim3(256), 0, stream,
                       d_in, cbits, wlo, whi, g0, ntiles + 1, (uint32_t)kWaves, plan);
    if (d_sync) {
        hipLaunchKernelGGL(pack_wt_kernel<true>, dim3((uint32_t)ntiles), dim3(kThreads), 0, stream,
                           d_in, d_chunk_off, nchunks, d_out, out_cap, d_out_off, d_state,
                           d_state + ntiles, d_sync, map, toff, cbits, plan, wlo, whi, g0);
        hipLaunchKernelGGL(pack_wt_fix_sync, dim3((uint32_t)((ntiles + 3) / 4)), dim3(256), 0,
                           stream, d_chunk_off, d_out_off, map, toff, d_sync, wlo, whi, g0, ntiles);
    } else {
        hipLaunchKernelGGL(pack_wt_kernel<false>, dim3((uint32_t)ntiles), dim3(kThreads), 0, stream,
                           d_in, d_chunk_off, nchunks, d_out, out_cap, d_out_off, d_state,
                           d_state + ntiles, d_sync, map, toff, cbits, plan, wlo, whi, g0);
    }
    return hipGetLastError();
}

#if PACK_PROF
extern "C" hipError_t capnp_pack_trace(uint64_t* d_buf) {
    return hipMemcpyToSymbol(HIP_SYMBOL(g_trace), &d_buf, sizeof(d_buf));
}

extern "C" hipError_t capnp_pack_prof(unsigned long long* host8, int reset) {
    hipError_t e = hipMemcpyFromSymbol(host8, HIP_SYMBOL(g_prof), sizeof(g_prof));
    if (e == hipSuccess && reset) {
        static const unsigned long long z[8] = {};
        e = hipMemcpyToSymbol(HIP_SYMBOL(g_prof), z, sizeof(z));
    }
    return e;
}
#endif

// One write_message call in one launch (msg_pack_kernel): the message's
// chunks (nwords <= capnp_msg_pack_words(), nchunks <= 515) and offsets, the
// output and *total may be pinned host memory.  Bytes at or past out_cap are
// not written; *total is the size needed.
extern "C" uint32_t capnp_msg_pack_words(void) { return kMsgWords; }
#if SVC_PROF
extern "C" int capnp_svc_prof_w(unsigned long long* out8, int reset) {
    if (hipMemcpyFromSymbol(out8, HIP_SYMBOL(g_svc_prof), 192) != hipSuccess) return -1;
    if (reset) {
        static const unsigned long long z[24] = {};
        if (hipMemcpyToSymbol(HIP_SYMBOL(g_svc_prof), z, 192) != hipSuccess) return -1;
    }
    return 0;
}
#endif
extern "C" hipError_t capnp_launch_msg_pack_service(const uint64_t* line, uint64_t* mark,
                                                    uint32_t gen, uint64_t idle_ticks,
                                                    uint32_t* flag, hipStream_t stream) {
    hipLaunchKernelGGL(msg_pack_service, dim3(1), dim3(kMsgThreads), 0, stream, line, mark, gen,
                       idle_ticks, flag);
    return hipGetLastError();
}
extern "C" hipError_t capnp_launch_msg_pack(const uint64_t* words, const uint64_t* off,
                                            uint32_t nchunks, uint32_t nwords, uint8_t* out,
                                            uint64_t out_cap, uint64_t* total, uint32_t* flag,
                                            uint32_t seq, uint8_t* scratch, hipStream_t stream) {
    if (nwords > kMsgWords || nchunks + 1 > kMsgChunks || nchunks == 0)
        return hipErrorInvalidValue;
    hipLaunchKernelGGL(msg_pack_kernel, dim3(1), dim3(kMsgThreads), 0, stream, words, off, nchunks,
                       nwords, out, out_cap, total, flag, seq, scratch);
    return hipGetLastError();
}
