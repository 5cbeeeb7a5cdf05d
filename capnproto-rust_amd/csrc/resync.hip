// resync.hip — index-free parallel decode of long packed read units
// (SURVEY §8f row 2): the same transform and results as the batch UNPACK
// (PackedRead::read under read_exact, capnp/src/serialize_packed.rs:80-228,
// io.rs:16-31) for streams that carry no record sync index, where a chunk can
// be any length (a 64 KiB segment, or a whole multi-megabyte message body).
//
// The decode of a read unit is a serial tag chain: where record k+1 starts
// depends on record k's tag and run count.  The batch unpack without an index
// gives one lane per chunk, so a long chunk is one long dependent chain.
// Here each chunk's packed bytes are cut into kBlock-byte blocks and the
// chain is resynchronised speculatively, tile by tile (k_tile, below):
//
//   resolve  every block's entry (its first record start), exit (the first
//            record start at or past its end) and word count, from
//            speculative walks that meet the true chain (tag chains couple
//            within a few records: record lengths are 1..10 bytes), then
//            fix passes over the tiles whose entry was not their
//            predecessor's exit, until no exit changes.  At that fixed
//            point every block's entry is its predecessor's exit and the
//            first block's entry is the chunk start, so by induction every
//            exit is the one the serial walk produces.
//   scan     exclusive scan of the block word counts: each block's first
//            output word.
//   check    lane per chunk: the chain must end exactly at the chunk's packed
//            end with exactly the chunk's word count (then no record ran
//            short, and no run overran the output: the word count is
//            monotone).
//   decode   each resolved block is a read unit of its own (its records run
//            from its entry to its exit): the blocks go to the batch unpack
//            kernel as a batch of ~120-word units (staged LDS tiles,
//            coalesced stores).
//
// A chunk that fails the check (a malformed stream, or a valid unit followed
// by spare bytes in its range) is decoded serially as one unit of that same
// launch, so its status, consumed count and partial output are exactly
// capnp_gpu_unpack_batch's; the other chunks keep the block decode.
#include <mutex>
#include <vector>
#include <hipcub/hipcub.hpp>

#include "common.h"
#include "../../include/capnp_packed.h"


extern "C" hipError_t capnp_launch_unpack(const uint8_t* d_in, const uint64_t* d_in_off,
                                          size_t nchunks, uint32_t tc, uint64_t* d_out,
                                          const uint64_t* d_out_off, int32_t* d_status,
                                          uint64_t* d_consumed, const uint32_t* d_sync,
                                          hipStream_t stream);

namespace {

constexpr uint64_t kBlock = 512;  // packed bytes per block
constexpr uint32_t kThreads = 256;
constexpr int kMaxPasses = 512;  // fix passes before giving up to the serial path
constexpr int kPassBatch = 8;    // fix passes enqueued per flag read-back (after the first)
constexpr uint64_t kShortChunk = 2 * kBlock;  // mean packed bytes per chunk below which
                                              // the batch goes straight to the batch unpack

// One record hop from p (< b, the chunk's packed end): p moves past the
// record, w counts its words.  A record cut short by the chunk end leaves p
// at b + 1, which stops every walk and fails the chunk's check.
__device__ __forceinline__ void hop(const uint8_t* __restrict__ in, uint64_t& p, uint64_t& w,
                                    uint64_t b) {
    const uint32_t tag = in[p];
    uint64_t q = p + 1 + __builtin_popcount(tag);
    w += 1;
    if (tag == 0u || tag == 0xFFu) {
        if (q >= b) {
            p = b + 1;
            return;
        }
        const uint32_t r = in[q];
        q += 1;
        w += r;
        if (tag == 0xFFu) q += 8ull * r;
    }
    p = q > b ? b + 1 : q;
}

// Chunk of block `blk`: the last c with bstart[c] <= blk (chunks without
// blocks have equal starts, skipped by taking the last one).
__device__ __forceinline__ uint64_t chunk_of(const uint64_t* __restrict__ bstart, uint64_t n,
                                             uint64_t blk) {
    uint64_t lo = 0, hi = n;  // bstart[lo] <= blk < bstart[hi]
    while (hi - lo > 1) {
        const uint64_t mid = (lo + hi) >> 1;
        if (bstart[mid] <= blk) lo = mid;
        else hi = mid;
    }
    return lo;
}

struct Ws {
    uint64_t* nblk;        // [n+1] blocks per chunk
    uint64_t* bstart;      // [n+1] exclusive scan of nblk
    uint64_t* spec_exit;   // [nbb] (k_tile: each block's chunk; then decode units' starts)
    uint32_t* spec_words;  // [nbb] (the chunks' error marks; then the units' statuses)
    uint64_t* exit;        // [nbb]
    uint64_t* entry;       // [nbb] entry the current exit/words were derived from
    uint64_t* words;       // [nbb]
    uint64_t* wbase;       // [nbb] exclusive scan of words
    int32_t* ok;           // [n]
    int32_t* flags;        // [0] a tile hit the round cap, [1] chunk failed,
                           // [2 + i] fix pass i changed a tile's last exit
    uint64_t* trec;        // [ntiles] look-back records of k_tile ({final, last exit})
    uint32_t* ticket;      // k_tile's tile counter (zeroed with trec)
    void* tmp;
    size_t tmp_bytes;
};

// (a chunk with no packed bytes but a nonzero word count owns one empty
// block: it fails its check and is decoded as a unit of its own, below)
__global__ void __launch_bounds__(kThreads) k_count(const uint64_t* __restrict__ in_off, uint64_t n,
                                                    const uint64_t* __restrict__ out_off,
                                                    uint64_t* __restrict__ nblk) {
    const uint64_t c = (uint64_t)blockIdx.x * kThreads + threadIdx.x;
    if (c > n) return;
    if (c == n) {
        nblk[c] = 0;
        return;
    }
    const uint64_t len = in_off[c + 1] - in_off[c];
    nblk[c] = len == 0 ? (out_off[c + 1] != out_off[c] ? 1 : 0) : (len + kBlock - 1) / kBlock;
}

#ifndef RESYNC_DPP
#define RESYNC_DPP 1  // the rounds' wave scans by DPP (0: ds_bpermute shuffles, A/B)
#endif
#ifndef RESYNC_PROF
#define RESYNC_PROF 0  // diagnostic: per-tile phase timestamps of the spec launch (scripts/resync_prof.py)
#endif
#if RESYNC_PROF
__device__ uint64_t* g_rtrace;  // 8 per tile: start, staged, spec, rounds, look-back wait + re-run, end
#define RTRACE(k) do { if (tid == 0 && g_rtrace) g_rtrace[t * 8 + (k)] = __builtin_amdgcn_s_memrealtime(); } while (0)
#else
#define RTRACE(k) ((void)0)
#endif

// ---- tile resolution (k_tile) ----
// A 256-thread workgroup takes a tile of kTileBlocks consecutive blocks
// (contiguous packed bytes, <= 26 KiB), stages them in LDS by DMA, and each
// wave resolves kWaveBlocks blocks cut into kSegs segments of kSegBytes, one
// lane each:
//   spec   lane j walks from kLead bytes before its segment (or from its
//          chunk's start) to its first record start f >= s, then on to its
//          exit; the lead-in lets chains from different starts couple before
//          the segment begins, so f is usually the true start;
//   rounds entries are a prefix max over the lanes' own exits, across the
//          whole tile (shuffles within a wave, the waves' maxima through LDS):
//          a segment whose entry lies past its end -- inside a literal run --
//          owns none and passes the entry on, a walk that runs past its
//          chunk owns none either, the tile's first lane takes the tile's
//          entry and a chunk's first segment the chunk start.  A lane whose
//          entry is not the one its state derives from walks again from it,
//          in lockstep with its spec chain until they meet (then its exit
//          stands; the spec chain gives up after kCatchUp hops behind, and
//          the walk goes on alone); a lane whose entry lies below its
//          segment (a predecessor not settled yet) lets its spec chain stand
//          in for its successors.  At the fixed point every segment's entry
//          is its predecessor's exit;
//   blocks a block's entry is its first segment's, its exit its last
//          segment's (chunk end + 1 if any segment failed), its words the sum.
// (Round 2 walked each 512-byte block from global memory, one lane per block,
// and a literal-run region moved 8 blocks per fix pass: config 4 spent
// 0.9 ms in the spec walks and 1.95 ms in 24 fix passes; 2.4 ms in all now.)
// Segments of 128 bytes keep each walk short (a lane whose spec chain missed
// walks its whole segment; with one lane per 512-byte block that was the
// critical path, ~100 hops, and four waves share the tile's LDS).  Positions
// inside the tile are 32-bit offsets from the staged base.
// The tile's own entry is the previous tile's last exit.  Round 4 hands it
// over by look-back where that is cheap: tiles take their index from a
// ticket in start order; a tile whose last block's chunk starts inside it
// has a last exit that does not depend on its own entry, and publishes it
// right after its first rounds (one 8-byte granule {bit 63: final, exit},
// stored and polled with agent-scope atomics: memory-side, so no XCD's L2
// serves a stale copy).  A "near" tile -- its first block continues a chunk
// that starts at most kNearTiles tiles back -- polls that record once before its
// rounds (taking the true entry if it is there, else assuming its first
// lane's f), and after them waits for it if needed and re-runs the rounds
// from the true entry when it differs (the lanes' states stay in registers:
// only the cascade walks again), then publishes its own last exit: waits
// chain at most kNearTiles deep.  Deeper tiles of long units (more than
// kNearTiles tiles into a unit) keep their guess, and fix
// passes (fix = 1, host-driven) re-resolve
// the tiles whose stored entry is not their predecessor's exit, until no
// last exit moves; tiles later in a pass often read an exit their
// predecessor wrote in the same pass.  (Waiting in every tile chained the
// hand-offs through a long unit: one 256 MiB unit 8.1 ms against 0.5 with
// fix passes.)  Config 4 (segments <= 64 KiB): round 3's fix passes cost 302
// + 78 us for the two that moved exits, 6 x 7 us of no-op passes and two host
// read-backs per call.
// Segments per block re-checked in round 3 (2 / 4 / 8: 2574 / 2367 / 2497 us,
// config 4 index-free): 4.
constexpr uint32_t kSegs = 4;                               // segments per block
constexpr uint32_t kSegBytes = (uint32_t)kBlock / kSegs;    // 128
constexpr uint32_t kTileWaves = kSegs;                      // (a wave per 128-byte column)
// Blocks per wave (<= CAPNP_WAVE / kSegs): 13 leaves 12 of a wave's 64 lanes
// idle, but the tile's LDS (26.7 KB) lets 6 tiles share a CU instead of 4
// (73 VGPRs allow 6 waves per SIMD).  Round 4, config 4 index-free,
// interleaved: 16 / 15 / 13 / 12 blocks 1938 / 1788 / 1762 / 1798 us; 10 and
// 9 blocks at 8 waves per SIMD (57 VGPRs) 1816 / 1780; 11 at 7 (12 B spill)
// 1774.
#ifndef RESYNC_WAVE_BLOCKS
#define RESYNC_WAVE_BLOCKS 13
#endif
constexpr uint32_t kWaveBlocks = RESYNC_WAVE_BLOCKS;
static_assert(kWaveBlocks * kSegs <= CAPNP_WAVE, "a wave's segments fit its lanes");
constexpr uint32_t kTileBlocks = kTileWaves * kWaveBlocks;  // 52
constexpr uint32_t kTileThreads = kTileWaves * CAPNP_WAVE;
// spec walk lead-in (bytes); 48 -> 64: config 4 index-free -2.7 % on two
// boxes (32 / 80 / 96: 2478 / 2340 / 2295 us against 2311-2329)
#ifndef RESYNC_LEAD
#define RESYNC_LEAD 64
#endif
constexpr uint64_t kLead = RESYNC_LEAD;
// hops a re-walk lets its spec chain catch up per step (32: 2439 us, slower)
constexpr uint32_t kCatchUp = 16;
constexpr uint32_t kTileLds = (uint32_t)(kTileBlocks * kBlock + kLead + 64);
// look-back waits chain at most this many tiles from a chunk's first tile
// (config 4's 64 KiB segments span <= 3 tiles; 1: its third tiles went to a
// fix pass that moved exits, 9 passes a call, 1984 vs 1790 us)
constexpr uint64_t kNearTiles = 4;
constexpr uint32_t kRelCap = 0xF0000000u;  // chunk ends past this are "far" (tile offsets are < 40 K)
constexpr uint32_t kNone32 = 0xFFFFFFFFu;
static_assert(kBlock % kSegs == 0, "segments tile the block");

// hop() on the staged bytes, positions relative to the staged base.  The tag
// and both possible count bytes (p+1 for 0x00, p+9 for 0xFF) are read
// together, as unpack.hip's seg_hop does: one LDS latency per hop instead of
// two dependent ones (the staged range has slack past every segment end, so
// p+9 stays inside the buffer; a count byte past the chunk end is never used).
// hop() on the staged bytes, positions relative to the staged base.  (The
// tag and both possible count bytes read together, as unpack.hip's seg_hop
// does, measured slower here: config 4 index-free 2967 vs 2717 us, round 4;
// three byte reads per hop load the LDS more than the dependent read costs.)
__device__ __forceinline__ void hop32(const uint8_t* buf, uint32_t& p, uint32_t& w, uint32_t b) {
    const uint32_t tag = buf[p];
    uint32_t q = p + 1 + __builtin_popcount(tag);
    w += 1;
    if (tag == 0u || tag == 0xFFu) {
        if (q >= b) {
            p = b + 1;
            return;
        }
        const uint32_t r = buf[q];
        q += 1;
        w += r;
        if (tag == 0xFFu) q += 8u * r;
    }
    p = q > b ? b + 1 : q;
}

// One lane's segment state for the rounds.
struct SegState {
    uint32_t ss, se, b, a;  // segment [ss, se), chunk end, chunk start (relative)
    uint32_t f, sx, sw;     // spec chain: first start >= ss (kNone32: none), exit, words
    bool serr;
    uint32_t used, ex, own; // entry the state derives from, exit, owned exit (0: none)
    uint32_t wd;            // words from used to ex
};

// Rounds to the fixed point for the wave (in_j: lane 0's entry, a chunk's
// first segment's start, else 0).
// The prefix max runs over the whole tile: within the wave by shuffles,
// across waves through LDS (wmax: each wave's maximum), two barriers a round;
// the tile's rounds end together (wneed: whether a wave still has work).
// Termination: lane i's entry is a function of the owned exits of lanes < i
// only, and a lane's owned exit is a function of its entry.  So lane 0 (whose
// entry is fixed) is settled after round 1, and by induction lane i after
// round i + 1: the tile reaches its fixed point within kTileThreads + 1
// rounds.  kMaxRounds caps the loop anyway; a tile that reaches the cap (which
// the argument rules out) marks every segment with an error exit and returns
// false, and the caller flags the resolution as unreliable (the batch then
// takes the serial decode).
constexpr uint32_t kMaxRounds = kTileThreads + 2;
uint32_t g_max_rounds = kMaxRounds;  // (capnp_resync_max_passes: tests drive the fallbacks)
__device__ __forceinline__ bool seg_rounds(const uint8_t* buf, SegState& S, bool valid,
                                           uint32_t in_j, bool fixed_j, uint32_t lane,
                                           uint32_t wave, uint32_t* wmax, uint32_t* wneed,
                                           uint32_t max_rounds) {
    for (uint32_t round = 0;; round++) {
        if (round == max_rounds) {  // (uniform: every wave counts the same rounds)
            S.ex = S.b + 1;
            S.wd = 0;
            return false;
        }
        uint32_t v = S.own > in_j ? S.own : in_j;
        if (!valid) v = 0;
#if RESYNC_DPP
        const uint32_t x = wave_max_scan(v);  // (DPP: no LDS round trips)
        if (lane == CAPNP_WAVE - 1) wmax[wave] = x;
        uint32_t pm = wave_shr1(x);
#else
        uint32_t x = v;
#pragma unroll
        for (uint32_t d = 1; d < CAPNP_WAVE; d <<= 1) {
            const uint32_t y = (uint32_t)__shfl_up((int)x, d);
            if (lane >= d && y > x) x = y;
        }
        if (lane == CAPNP_WAVE - 1) wmax[wave] = x;
        uint32_t pm = (uint32_t)__shfl_up((int)x, 1);
        if (lane == 0) pm = 0;
#endif
        __syncthreads();
        for (uint32_t w2 = 0; w2 < wave; w2++) pm = wmax[w2] > pm ? wmax[w2] : pm;
        const uint32_t ent = fixed_j ? in_j : pm;
        const bool need = valid && ent != S.used;
        const bool wn = ballot64(need) != 0;
        if (lane == 0) wneed[wave] = wn;
        __syncthreads();
        uint32_t any = 0;
        for (uint32_t w2 = 0; w2 < kTileWaves; w2++) any |= wneed[w2];
        if (!any) return true;
        if (!need) continue;
        S.used = ent;
        if (ent < S.ss) {
            // no predecessor reaches this segment yet (one still stands on a
            // wrong entry, or its chunk failed): the spec chain stands in for
            // the successors (an error exit marks the segment until an entry
            // reaches it; at the fixed point of a valid chunk none is left)
            S.ex = S.b + 1;
            S.wd = 0;
            S.own = (S.f != kNone32 && S.f < S.se && !S.serr) ? S.sx : 0;
        } else if (ent > S.b) {  // past the chunk
            S.ex = S.b + 1;
            S.wd = 0;
            S.own = 0;
        } else if (ent >= S.se && S.se > S.ss) {  // inside a record that began earlier
            S.ex = ent;
            S.wd = 0;
            S.own = 0;
        } else if (S.se == S.ss) {  // an empty segment (a short block's tail) passes its entry on
            S.ex = ent;
            S.wd = 0;
            S.own = 0;
        } else {
            uint32_t pt = ent, wt = 0, ps = S.f, ws = 0, catchup = 0;
            bool spec = S.f != kNone32 && S.f < S.se, met = false;
            while (pt < S.se) {
                if (spec) {
                    while (ps < pt && ps < S.se && catchup < kCatchUp) {
                        hop32(buf, ps, ws, S.b);
                        catchup++;
                    }
                    if (ps == pt) {
                        met = true;
                        break;
                    }
                    if (ps < pt) spec = false;  // too far behind: walk alone
                }
                hop32(buf, pt, wt, S.b);
            }
            if (met) {
                S.ex = S.sx;
                S.wd = wt + S.sw - ws;
                S.own = S.serr ? 0 : S.sx;
            } else {
                S.ex = pt;
                S.wd = wt;
                S.own = pt > S.b ? 0 : pt;
            }
        }
    }
}

__global__ void __launch_bounds__(kTileThreads)
k_tile(const uint8_t* __restrict__ in, const uint64_t* __restrict__ in_off, uint64_t n,
       const uint64_t* __restrict__ bstart, uint64_t* __restrict__ exit,
       uint64_t* __restrict__ entry, uint64_t* __restrict__ words, uint64_t* __restrict__ blk_c,
       int32_t* flags, uint64_t* trec, uint32_t* ticket, uint32_t max_rounds, int fix, int pass) {
    extern __shared__ __align__(16) uint8_t tbuf[];
    __shared__ uint32_t wmax[kTileWaves], wneed[kTileWaves];
    __shared__ uint64_t s_t, s_e0;
    const uint32_t tid = threadIdx.x;
    const uint32_t lane = tid & (CAPNP_WAVE - 1);
    const uint32_t wave = (uint32_t)__builtin_amdgcn_readfirstlane((int)(tid / CAPNP_WAVE));
    // the tile index: in the first launch a ticket in start order (a tile's
    // predecessor has started before it, so waiting on it cannot deadlock);
    // in a fix pass the block index (fix passes never wait)
    if (fix && pass > 0 && __atomic_load_n(&flags[2 + pass - 1], __ATOMIC_RELAXED) == 0) return;
    if (tid == 0) {
        s_t = fix ? blockIdx.x
                  : __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        s_e0 = 0;
    }
    const uint64_t nb = uniform64(bstart[n]);
    __syncthreads();
    const uint64_t t = uniform64(s_t);
    const uint64_t k0 = t * kTileBlocks;
    if (k0 >= nb) return;
    if (fix) {
        if (k0 == 0) return;  // (block 0 starts chunk 0: exact since the first launch)
        // One read of the predecessor's exit for the whole workgroup (the
        // predecessor may rewrite it during this same pass: waves that read it
        // before and after the write disagreed on returning here and hung in
        // seg_rounds' barriers -- round 3).
        if (tid == 0) s_e0 = __atomic_load_n(&exit[k0 - 1], __ATOMIC_RELAXED);
        __syncthreads();
        if (uniform64(s_e0) == uniform64(entry[k0])) return;  // consistent
    }
    RTRACE(0);
    const uint64_t kn = nb - k0 < kTileBlocks ? nb - k0 : kTileBlocks;
    // c0 = the last chunk with bstart[c0] <= k0: a 64-way search (3 probes
    // deep for 10^5 chunks, where one lane's binary search was 17 dependent
    // loads)
    uint64_t clo = 0, chi = n;  // bstart[clo] <= k0 < bstart[chi]
    while (chi - clo > 1) {
        const uint64_t idx = clo + 1 + ((chi - clo - 1) * lane) / CAPNP_WAVE;
        const uint64_t m = ballot64(bstart[idx] <= k0);  // (monotone in the lane)
        const uint32_t nle = popc64(m);
        const uint64_t nlo = nle ? readlane64(idx, nle - 1) : clo;
        const uint64_t nhi = nle < CAPNP_WAVE ? readlane64(idx, nle) : chi;
        clo = nlo;
        chi = nhi;
    }
    const uint64_t c0 = clo;
    const uint64_t bs0 = uniform64(bstart[c0]), a0 = uniform64(in_off[c0]);
    // dep: the tile's first block continues a chunk from the previous tile;
    // near: that chunk starts at most kNearTiles tiles back, so the waits
    // chain at most that deep (the tile that holds the chunk start publishes
    // right after its first rounds, each near tile after its wait); a deeper
    // tile keeps its guess (fix passes follow)
    const bool dep = bs0 != k0;
    if (fix && !dep) return;  // a tile that starts a chunk is exact since the first launch
    const bool near = !fix && dep && bs0 + kNearTiles * kTileBlocks >= k0;
    if (near && tid == 0)  // one poll of the predecessor's record (0: not final yet)
        s_e0 = __hip_atomic_fetch_add(&trec[t - 1], 0ull, __ATOMIC_RELAXED,
                                      __HIP_MEMORY_SCOPE_AGENT);
    // stage [s0 - kLead, s0 + kTileBlocks * kBlock + 16) (clamped to the batch: the tile's
    // blocks are contiguous bytes, at most kBlock each) by LDS DMA, 16 bytes a
    // lane, every load in flight at once
    const uint64_t A = uniform64(in_off[0]), Z = uniform64(in_off[n]);
    const uint64_t s0 = a0 + (k0 - bs0) * kBlock;
    const uint64_t lo = s0 > A + kLead ? s0 - kLead : A;
    const uint64_t hi = s0 + kTileBlocks * kBlock + 16 < Z ? s0 + kTileBlocks * kBlock + 16 : Z;
    // (base: 16-byte aligned in memory; may lie below in_off[0] inside that vector)
    const uint64_t base = lo - (uint64_t)(reinterpret_cast<uintptr_t>(in + lo) & 15u);
    {
        const uint32_t nv = (uint32_t)((hi - base + 15) >> 4);
        const uint8_t* src = in + base;
        for (uint32_t i0 = wave * CAPNP_WAVE; i0 < nv; i0 += kTileThreads) {
            if (i0 + lane < nv)
                __builtin_amdgcn_global_load_lds(
                    (const __attribute__((address_space(1))) void*)(src + 16ull * (i0 + lane)),
                    (__attribute__((address_space(3))) void*)(tbuf + 16u * i0), 16, 0, 0);
        }
    }
    // this lane's block (offset jb in the tile) and segment q; its chunk: c0 +
    // the chunk starts in (k0, k0 + jb], counted over batches of 64 starts (a
    // lane's binary search over the batch by shuffles)
    const uint32_t jb = wave * kWaveBlocks + lane / kSegs, q = lane % kSegs;
    const bool valid = lane / kSegs < kWaveBlocks && jb < kn;
    const uint32_t jj = valid ? jb : (uint32_t)(kn - 1);
    const uint64_t k = k0 + jj;
    uint64_t c = c0;
    for (uint64_t cb = c0 + 1;; cb += CAPNP_WAVE) {
        const uint64_t idx = cb + lane;
        const uint64_t v = idx <= n ? bstart[idx] : ~0ull;
        const uint32_t d = v - k0 > CAPNP_WAVE ? CAPNP_WAVE + 1 : (uint32_t)(v - k0);
        uint32_t cnt = 0;
        for (uint32_t step = CAPNP_WAVE / 2; step; step >>= 1)
            if ((uint32_t)__shfl((int)d, (int)(cnt + step - 1)) <= jj) cnt += step;
        const uint32_t dlast = (uint32_t)__builtin_amdgcn_readlane((int)d, CAPNP_WAVE - 1);
        if (cnt == CAPNP_WAVE - 1 && dlast <= jj) cnt = CAPNP_WAVE;
        c += cnt;
        if (dlast >= CAPNP_WAVE) break;  // this batch reaches past the tile
    }
    const uint64_t a = in_off[c], b = in_off[c + 1], bsc = bstart[c];
    const uint64_t s = a + (k - bsc) * kBlock;
    const uint64_t e = s + kBlock < b ? s + kBlock : b;
    const uint64_t ssa = s + q * kSegBytes < e ? s + q * kSegBytes : e;
    const uint64_t sea = s + (q + 1) * kSegBytes < e ? s + (q + 1) * kSegBytes : e;
    const bool cfirst = k == bsc && q == 0;
    const uint64_t starta = ssa > a + kLead ? ssa - kLead : a;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's staged bytes are in
    __syncthreads();                                   // ... and every wave's
    RTRACE(1);
    SegState S;
    S.ss = (uint32_t)(ssa - base);
    S.se = (uint32_t)(sea - base);
    S.b = b - base < kRelCap ? (uint32_t)(b - base) : kRelCap;
    S.a = (uint32_t)(a > base ? a - base : 0);
    // spec walk (a chunk's first segment walks exactly from the chunk start)
    {
        uint32_t p = (uint32_t)(starta - base), w = 0;
        while (p < S.ss) hop32(tbuf, p, w, S.b);
        if (p > S.b) {  // the lead-in ran past the chunk: no spec chain
            S.f = kNone32;
            S.sx = S.b + 1;
            S.sw = 0;
            S.serr = true;
        } else {
            S.f = p;
            w = 0;
            while (p < S.se) hop32(tbuf, p, w, S.b);
            S.sx = p;
            S.sw = w;
            S.serr = p > S.b;
        }
    }
    if (S.f != kNone32 && (S.f >= S.se || S.se == S.ss)) {  // spec pass-through
        S.used = S.f;
        S.ex = S.f;
        S.wd = 0;
        S.own = 0;
    } else {
        S.used = S.f;
        S.ex = S.sx;
        S.wd = S.sw;
        S.own = S.serr ? 0 : S.sx;
    }
    RTRACE(2);
    // the tile's entry (lane 0 of wave 0): the previous tile's last exit if
    // its record is final already, else this lane's own f
    constexpr uint64_t kFinal = 1ull << 63;
    auto rel_entry = [&](uint64_t rec) -> uint32_t {
        const uint64_t e0 = rec & ~kFinal;
        const uint64_t r = e0 - base;
        return e0 < base ? 0u : (r < kRelCap ? (uint32_t)r : kRelCap + 1);
    };
    uint64_t rec = uniform64(s_e0);  // (written before the staging barrier)
    if (fix) rec |= kFinal;           // (a fix pass's entry: the predecessor's exit)
    uint32_t E0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)(S.f == kNone32 ? S.ss : S.f));
    if (rec & kFinal) E0 = rel_entry(rec);
    const bool tile_lane0 = wave == 0 && lane == 0;
    const bool fixed_j = cfirst || tile_lane0;
    bool settled = seg_rounds(tbuf, S, valid, cfirst ? S.ss : (tile_lane0 ? E0 : 0u), fixed_j,
                              lane, wave, wmax, wneed, max_rounds);
    RTRACE(3);
    // blocks: entry of segment 0, exit of segment 3, words summed
    // (a segment left with an error exit -- its walk ran past the chunk, or
    // no entry reached it -- marks the whole block, so the chunk fails its check)
    uint32_t wsum, berr, bx;
    auto block_result = [&]() {
        wsum = S.wd;
        berr = S.ex > S.b ? 1u : 0u;
#pragma unroll
        for (uint32_t m = 1; m < kSegs; m <<= 1) {
            wsum += (uint32_t)__shfl_xor((int)wsum, (int)m);
            berr |= (uint32_t)__shfl_xor((int)berr, (int)m);
        }
        bx = (uint32_t)__shfl((int)S.ex, (int)(lane | (kSegs - 1)));
    };
    auto block_exit = [&]() -> uint64_t { return (berr || bx > S.b) ? b + 1 : base + bx; };
    // the tile's last block: its exit is final already unless its chunk began
    // before this tile and the tile's entry is still a guess, so it goes to
    // the next tile now (only the waits within one chunk chain)
    const bool last = valid && q == 0 && (uint64_t)jb == kn - 1;
    const bool guess = dep && !(rec & kFinal);
    block_result();
    if (!fix && last && (!guess || bsc >= k0))
        __hip_atomic_exchange(&trec[t], kFinal | block_exit(), __ATOMIC_RELAXED,
                              __HIP_MEMORY_SCOPE_AGENT);
    if (guess && near) {
        // wait for the predecessor's last exit (it started before this tile
        // and waits, if at all, only on an earlier tile of the same chunk),
        // then re-run the rounds from it if the assumed entry was wrong
        if (tid == 0) {
            uint64_t v;
            while (!((v = __hip_atomic_fetch_add(&trec[t - 1], 0ull, __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_AGENT)) & kFinal))
                __builtin_amdgcn_s_sleep(2);
            s_e0 = v;
        }
        __syncthreads();
        rec = uniform64(s_e0);
        const uint32_t E1 = rel_entry(rec);
        if (E1 != E0 && settled) {
            settled = seg_rounds(tbuf, S, valid, cfirst ? S.ss : (tile_lane0 ? E1 : 0u), fixed_j,
                                 lane, wave, wmax, wneed, max_rounds);
            block_result();
        }
        if (last && bsc < k0)  // (for a near successor)
            __hip_atomic_exchange(&trec[t], kFinal | block_exit(), __ATOMIC_RELAXED,
                                  __HIP_MEMORY_SCOPE_AGENT);
    }
    if (!settled && tid == 0) flags[0] = 1;  // round cap: the segments carry error exits
    RTRACE(4);
    if (valid && q == 0) {
        const uint64_t xa = block_exit();
        const uint64_t old = fix ? exit[k] : 0;
        exit[k] = xa;
        entry[k] = S.used > S.b ? b + 1 : base + S.used;
        words[k] = wsum;
        if (!fix) blk_c[k] = c;
        if (fix && last && old != xa) flags[2 + pass] = 1;  // the next tile must look again
    }
    RTRACE(5);
}

// Chunks with a block whose resolved chain ran past the chunk end (the tile
// resolution marks such a block with exit b + 1; a segment that no entry
// reached keeps that mark): bad[c] = 1.  blk_c[k] = block k's chunk.
__global__ void __launch_bounds__(kThreads)
k_mark(const uint64_t* __restrict__ exit, const uint64_t* __restrict__ blk_c,
       const uint64_t* __restrict__ in_off, const uint64_t* __restrict__ bstart, uint64_t n,
       int32_t* __restrict__ bad) {
    const uint64_t k = (uint64_t)blockIdx.x * kThreads + threadIdx.x;
    if (k >= bstart[n]) return;
    const uint64_t c = blk_c[k];
    if (exit[k] > in_off[c + 1]) bad[c] = 1;
}

__global__ void __launch_bounds__(kThreads)
k_check(const uint64_t* __restrict__ in_off, uint64_t n, const uint64_t* __restrict__ out_off,
        const uint64_t* __restrict__ bstart, const uint64_t* __restrict__ exit,
        const uint64_t* __restrict__ words, const uint64_t* __restrict__ wbase,
        const int32_t* __restrict__ bad, int32_t* __restrict__ ok, int32_t* __restrict__ status,
        uint64_t* __restrict__ consumed, int32_t* __restrict__ flags) {
    const uint64_t c = (uint64_t)blockIdx.x * kThreads + threadIdx.x;
    if (c >= n) return;
    const uint64_t a = in_off[c], b = in_off[c + 1];
    const uint64_t nw = out_off[c + 1] - out_off[c];
    bool good;
    if (nw == 0) {
        good = true;  // read() of an empty buffer returns 0 and reads nothing
    } else if (a == b) {
        good = false;
    } else {
        const uint64_t f = bstart[c], l = bstart[c + 1] - 1;
        good = exit[l] == b && wbase[l] + words[l] - wbase[f] == nw && !(bad && bad[c]);
    }
    ok[c] = good;
    if (good) {
        status[c] = 0;
        if (consumed) consumed[c] = nw == 0 ? 0 : b - a;
    } else {
        flags[1] = 1;
    }
}

// Each block, resolved, is a read unit of its own: the records that start in
// it run from its entry to its exit and decode to exactly its word count.
// Lane k writes block k's packed start and first output word, so the blocks
// tile the batch's packed bytes and words contiguously (a block inside a
// literal run is an empty unit; a chunk of 0 words keeps its blocks empty,
// since read() of an empty buffer consumes nothing).  A chunk that failed its
// check (ok[c] = 0: malformed, or spare bytes in its range) becomes one unit:
// its blocks but the last are empty and the last spans the whole chunk, so
// the batch unpack decodes it exactly as capnp_gpu_unpack_batch would (status,
// consumed bytes and partial output; k_fail copies them to the chunk).
// ok = nullptr: every chunk passed.
__global__ void __launch_bounds__(kThreads)
k_blocks(const uint64_t* __restrict__ in_off, uint64_t n, const uint64_t* __restrict__ out_off,
         const uint64_t* __restrict__ bstart, const uint64_t* __restrict__ exit,
         const uint64_t* __restrict__ wbase, const int32_t* __restrict__ ok,
         uint64_t* __restrict__ blk_in, uint64_t* __restrict__ blk_out, uint64_t nbb) {
    const uint64_t k = (uint64_t)blockIdx.x * kThreads + threadIdx.x;
    const uint64_t nb = bstart[n];
    if (k > nbb) return;
    if (k >= nb) {  // (units nb .. nbb - 1: empty, past the batch end)
        blk_in[k] = in_off[n];
        blk_out[k] = out_off[n];
        return;
    }
    const uint64_t c = chunk_of(bstart, n, k);
    const uint64_t f = bstart[c];
    if (ok && !ok[c]) {
        blk_in[k] = in_off[c];
        blk_out[k] = out_off[c];
        return;
    }
    blk_in[k] = k == f ? in_off[c] : exit[k - 1];
    blk_out[k] = out_off[c] + (out_off[c + 1] == out_off[c] ? 0 : wbase[k] - wbase[f]);
}

// Status and consumed bytes of the chunks that failed their check: those of
// the unit that spans the chunk (its last block).
__global__ void __launch_bounds__(kThreads)
k_fail(uint64_t n, const uint64_t* __restrict__ bstart, const int32_t* __restrict__ ok,
       const int32_t* __restrict__ blk_status, const uint64_t* __restrict__ blk_consumed,
       int32_t* __restrict__ status, uint64_t* __restrict__ consumed) {
    const uint64_t c = (uint64_t)blockIdx.x * kThreads + threadIdx.x;
    if (c >= n || ok[c]) return;
    const uint64_t l = bstart[c + 1] - 1;  // (a failing chunk owns at least one block)
    status[c] = blk_status[l];
    if (consumed) consumed[c] = blk_consumed[l];
}

// k_tile's look-back records: one per tile (<= nbb / kTileBlocks + 1 tiles),
// then the ticket; resolve() zeroes them, with the flags before them, before its launches.
uint64_t trec_words(uint64_t nbb) { return nbb / kTileBlocks + 2; }

size_t carve(Ws* w, uint8_t* base, uint64_t n, uint64_t nbb, size_t tmp_bytes) {
    size_t off = 0;
    auto take = [&](size_t bytes) {
        uint8_t* p = base ? base + off : nullptr;
        off += (bytes + 255) & ~size_t(255);
        return p;
    };
    w->nblk = (uint64_t*)take(8 * (n + 1));
    w->bstart = (uint64_t*)take(8 * (n + 1));
    w->spec_exit = (uint64_t*)take(8 * (nbb + 1));  // (then the decode units' starts: nbb + 1)
    w->spec_words = (uint32_t*)take(4 * nbb);
    w->exit = (uint64_t*)take(8 * nbb);
    w->entry = (uint64_t*)take(8 * (nbb + 1));
    w->words = (uint64_t*)take(8 * nbb);
    w->wbase = (uint64_t*)take(8 * nbb);
    w->ok = (int32_t*)take(4 * n + 4);
    w->flags = (int32_t*)take(4 * (2 + kMaxPasses));
    w->trec = (uint64_t*)take(8 * trec_words(nbb));  // (the ticket in its last word)
    w->ticket = (uint32_t*)(w->trec ? w->trec + trec_words(nbb) - 1 : nullptr);
    w->tmp = take(tmp_bytes);
    w->tmp_bytes = tmp_bytes;
    return off;
}

size_t scan_tmp_bytes(uint64_t items) {
    size_t bytes = 0;
    (void)hipcub::DeviceScan::ExclusiveSum(nullptr, bytes, (const uint64_t*)nullptr, (uint64_t*)nullptr,
                                     (int)items);
    return bytes;
}

uint64_t blocks_bound(uint64_t n, uint64_t total_bytes) { return total_bytes / kBlock + n + 1; }

unsigned grid(uint64_t items) { return (unsigned)((items + kThreads - 1) / kThreads); }

// Tile resolution: the first k_tile launch (near tiles settled by
// look-back), then fix passes over the tiles whose entry is not their
// predecessor's exit (deep tiles of long units whose guess was wrong): one
// pass before the first flag read-back, then kPassBatch per read-back.
// *converged = false if the passes reach kMaxPasses; *capped = true if a
// tile hit the round cap (its segments carry error exits).  Blocking.
// Pinned flag buffers for resolve()'s read-back, shared by every thread: a
// call borrows one and returns it, so the pool holds at most as many buffers
// as calls that ever ran at once (they live until the process ends).  Null if
// pinned memory is unavailable (resolve then reads the flags through pageable
// copies).
struct PinnedFlags {
    int32_t* p = nullptr;
    static std::mutex& mu() {
        static std::mutex m;
        return m;
    }
    static std::vector<int32_t*>& pool() {
        static std::vector<int32_t*> v;
        return v;
    }
    PinnedFlags() {
        {
            std::lock_guard<std::mutex> g(mu());
            if (!pool().empty()) {
                p = pool().back();
                pool().pop_back();
                return;
            }
        }
        void* q = nullptr;
        if (hipHostMalloc(&q, 4 * (2 + kMaxPasses), 0) == hipSuccess) p = (int32_t*)q;
    }
    ~PinnedFlags() {
        if (!p) return;
        std::lock_guard<std::mutex> g(mu());
        pool().push_back(p);
    }
};

hipError_t resolve(const uint8_t* d_in, const uint64_t* in_off, uint64_t n, const Ws& w,
                   uint64_t nbb, hipStream_t s, bool* converged, bool* capped, int* passes) {
    hipError_t e;
    *converged = true;
    *capped = false;
    const unsigned ntiles = (unsigned)((nbb + kTileBlocks - 1) / kTileBlocks);
    // the flags (round cap, chunk failure, one per fix pass) and the tile
    // records with their ticket lie together in the workspace: one clear
    {
        const size_t zb = (size_t)(reinterpret_cast<uint8_t*>(w.trec + trec_words(nbb)) -
                                   reinterpret_cast<uint8_t*>(w.flags));
        if ((e = hipMemsetAsync(w.flags, 0, zb, s)) != hipSuccess) return e;
    }
    // (the flags come back through pinned memory: one DMA, no staged copy;
    // the buffer is borrowed from a process-wide pool for the call)
    PinnedFlags pf;
    int32_t* const t_hflags = pf.p;
    k_tile<<<ntiles, kTileThreads, kTileLds, s>>>(d_in, in_off, n, w.bstart, w.exit, w.entry,
                                                 w.words, w.spec_exit, w.flags, w.trec, w.ticket,
                                                 g_max_rounds, 0, 0);
    int pass = 0;
    for (int batch = 1;; batch = kPassBatch) {
        if (pass >= kMaxPasses) {
            *converged = false;
            break;
        }
        for (int i = 0; i < batch && pass < kMaxPasses; i++, pass++)
            k_tile<<<ntiles, kTileThreads, kTileLds, s>>>(d_in, in_off, n, w.bstart, w.exit,
                                                         w.entry, w.words, w.spec_exit, w.flags,
                                                         w.trec, w.ticket, g_max_rounds, 1, pass);
        int32_t last = 0, cap = 0;
        if (t_hflags) {
            if ((e = hipMemcpyAsync(t_hflags, w.flags, 4 * (2 + pass), hipMemcpyDeviceToHost, s)) !=
                hipSuccess)
                return e;
            if ((e = hipStreamSynchronize(s)) != hipSuccess) return e;
            cap = t_hflags[0];
            last = t_hflags[2 + pass - 1];
        } else {
            if ((e = hipMemcpyAsync(&last, w.flags + 2 + pass - 1, 4, hipMemcpyDeviceToHost, s)) !=
                hipSuccess)
                return e;
            if ((e = hipMemcpyAsync(&cap, w.flags, 4, hipMemcpyDeviceToHost, s)) != hipSuccess)
                return e;
            if ((e = hipStreamSynchronize(s)) != hipSuccess) return e;
        }
        if (cap) *capped = true;
        if (!last) break;
    }
    *passes = pass;
    return hipGetLastError();
}

}  // namespace

extern "C" uint32_t capnp_resync_block_bytes(void) { return (uint32_t)kBlock; }

// Test hook (the name predates the look-back): caps the rounds a tile may run
// (1 .. kMaxRounds; 0 restores the default), so tests reach the fallbacks.
extern "C" int capnp_resync_max_passes(int rounds) {
    const int old = (int)g_max_rounds;
    g_max_rounds = rounds <= 0 ? kMaxRounds
                               : ((uint32_t)rounds > kMaxRounds ? kMaxRounds : (uint32_t)rounds);
    return old == (int)kMaxRounds ? 0 : old;
}

// RESYNC_PROF builds: the per-tile trace buffer (8 words per tile), or null.
extern "C" int capnp_resync_trace(uint64_t* d_buf) {
#if RESYNC_PROF
    return hipMemcpyToSymbol(HIP_SYMBOL(g_rtrace), &d_buf, sizeof(d_buf)) == hipSuccess ? 0 : -1;
#else
    (void)d_buf;
    return -1;
#endif
}

// Workspace for capnp_resync_unpack over n chunks holding total_bytes packed bytes.
extern "C" size_t capnp_resync_ws_bytes(uint64_t n, uint64_t total_bytes) {
    const uint64_t nbb = blocks_bound(n, total_bytes);
    const uint64_t m = nbb > n + 1 ? nbb : n + 1;
    Ws w;
    return carve(&w, nullptr, n, nbb, scan_tmp_bytes(m)) + 256;
}

// Blocking until the resolution's fix passes settle (one flag read-back when
// none moves an exit), asynchronous after that.  On return, *passes = fix
// passes run, *serial = 1 if they did not converge (the batch went to the
// serial batch unpack), 2 if the chunks were short enough to go straight
// there; *failed_flag (device) turns nonzero if some chunks failed their
// check (those alone were decoded serially, each as one unit of the block
// decode: the caller reports serial = 3 from it, on demand).
extern "C" hipError_t capnp_resync_unpack(const uint8_t* d_in, const uint64_t* d_in_off, uint64_t n,
                                          uint64_t total_bytes, uint64_t* d_out,
                                          const uint64_t* d_out_off, int32_t* d_status,
                                          uint64_t* d_consumed, void* d_ws, size_t ws_bytes,
                                          hipStream_t s, int* passes, int* serial,
                                          const int32_t** failed_flag) {
    if (passes) *passes = 0;
    if (serial) *serial = 0;
    if (failed_flag) *failed_flag = nullptr;
    if (n == 0) return hipSuccess;
    hipError_t e;
    if (total_bytes < n * kShortChunk) {
        // chunks this short are parallel enough as they are: the batch unpack
        // (one walker per chunk) is faster than resolving blocks
        if (serial) *serial = 2;
        if ((e = capnp_launch_unpack(d_in, d_in_off, n, 0, d_out, d_out_off, d_status, d_consumed,
                                     nullptr, s)) != hipSuccess)
            return e;
        return hipStreamSynchronize(s);
    }
    const uint64_t nbb = blocks_bound(n, total_bytes);
    const uint64_t m = nbb > n + 1 ? nbb : n + 1;
    Ws w;
    uint8_t* base = (uint8_t*)(((uintptr_t)d_ws + 255) & ~uintptr_t(255));
    if (carve(&w, base, n, nbb, scan_tmp_bytes(m)) + (base - (uint8_t*)d_ws) >
        ws_bytes)
        return hipErrorInvalidValue;
    k_count<<<grid(n + 1), kThreads, 0, s>>>(d_in_off, n, d_out_off, w.nblk);
    size_t tb = w.tmp_bytes;
    if ((e = hipcub::DeviceScan::ExclusiveSum(w.tmp, tb, w.nblk, w.bstart, (int)(n + 1), s)) !=
        hipSuccess)
        return e;
    // (a tile that hits the round cap fails its chunks, which the block
    // decode below walks serially; fix passes that do not converge send the
    // batch to the serial batch unpack)
    bool conv = true, capped = false;
    int pass = 0;
    if ((e = resolve(d_in, d_in_off, n, w, nbb, s, &conv, &capped, &pass)) != hipSuccess) return e;
    if (passes) *passes = pass;
    if (!conv) {
        if (serial) *serial = 1;
        if ((e = capnp_launch_unpack(d_in, d_in_off, n, 0, d_out, d_out_off, d_status, d_consumed,
                                     nullptr, s)) != hipSuccess)
            return e;
        return hipStreamSynchronize(s);
    }
    tb = w.tmp_bytes;
    if ((e = hipcub::DeviceScan::ExclusiveSum(w.tmp, tb, w.words, w.wbase, (int)nbb, s)) !=
        hipSuccess)
        return e;
    // (blk_c in spec_exit, bad in spec_words: both dead until k_blocks)
    int32_t* bad = reinterpret_cast<int32_t*>(w.spec_words);
    if ((e = hipMemsetAsync(bad, 0, 4 * n, s)) != hipSuccess) return e;
    k_mark<<<grid(nbb), kThreads, 0, s>>>(w.exit, w.spec_exit, d_in_off, w.bstart, n, bad);
    k_check<<<grid(n), kThreads, 0, s>>>(d_in_off, n, d_out_off, w.bstart, w.exit, w.words,
                                         w.wbase, bad, w.ok, d_status, d_consumed, w.flags);
    // decode the blocks as independent read units with the batch unpack
    // (staged LDS tiles, coalesced stores); a chunk that failed its check
    // is one unit of its own, decoded serially in the same launch.  No
    // host read-back here: the decode runs over the nbb-unit bound (k_blocks
    // makes the units past the last block empty) and always returns the
    // units' consumed counts for k_fail, which only touches failed chunks
    // (one host round trip fewer per call; *failed_flag lets the caller
    // learn serial = 3 later, on demand).
    uint64_t* blk_in = w.spec_exit;  // (spec state is dead by now)
    uint64_t* blk_out = w.entry;
    int32_t* blk_status = reinterpret_cast<int32_t*>(w.spec_words);
    uint64_t* blk_consumed = w.words;  // (dead after the wbase scan and the check)
    k_blocks<<<grid(nbb + 1), kThreads, 0, s>>>(d_in_off, n, d_out_off, w.bstart, w.exit,
                                                w.wbase, w.ok, blk_in, blk_out, nbb);
    // (block units per tile: the unpack's 16; 4 / 8 / 32 measured 2576 / 2079
    // / 2618 vs 1906 us for config 4, round 4)
    if ((e = capnp_launch_unpack(d_in, blk_in, nbb, 0, d_out, blk_out, blk_status,
                                 blk_consumed, nullptr, s)) != hipSuccess)
        return e;
    k_fail<<<grid(n), kThreads, 0, s>>>(n, w.bstart, w.ok, blk_status, blk_consumed,
                                        d_status, d_consumed);
    if (failed_flag) *failed_flag = w.flags + 1;
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Message-boundary discovery in a concatenated packed stream (SURVEY §8f row
// 2): where successive try_read_message calls (serialize.rs:310-325,
// :448-524; serialize_packed.rs:246-255) would start each message, with no
// byte index.
//
//   1. the whole stream is resolved as one read unit (spec / fix / scan
//      above) and decoded block by block into words;
//   2. one lane follows the message chain in the word domain: message k
//      starts at word u_k, its table says 1 + nseg/2 + sum(lengths) words
//      (serialize.rs:467-510), so u_{k+1} = u_k + that; the walk stops at a
//      table that is invalid (segment count 0 or >= 512), at a message that
//      runs past the decoded words, or at max_msgs;
//   3. lane per message: the packed byte where word u_k's record starts
//      (binary search of the block word bases, then a walk from the block's
//      entry).  A u_k inside a run (the previous message's body ended inside
//      a record) is not a record start: the previous message is then the
//      failing one.
// A writer packs each message's table words and segments as separate chunks
// (serialize.rs:595-679), so records never cross message boundaries and the
// word-domain chain is the reference's.  For streams where they do (or that
// are malformed), the messages up to the first failing one are still
// exact, and the caller decodes the failing message's range to the end of
// the stream (capnp_gpu_read_messages gives the reference's status for it).

namespace {

// res[0] = words before the first block the walk may not trust: one whose
// entry is not its predecessor's exit (fix passes stopped before the fixed
// point; the blocks before it are exact) ...
__global__ void k_consistent(const uint64_t* __restrict__ entry, const uint64_t* __restrict__ exit_,
                             const uint64_t* __restrict__ wbase, uint64_t nb,
                             uint64_t* __restrict__ res) {
    const uint64_t k = (uint64_t)blockIdx.x * kThreads + threadIdx.x;
    if (k == 0 || k >= nb) return;
    if (entry[k] != exit_[k - 1]) atomicMin((unsigned long long*)res, (unsigned long long)wbase[k]);
}

// ... or one that failed to decode (a record cut by the stream end).
__global__ void k_valid_words(const int32_t* __restrict__ blk_status, uint64_t nb,
                              const uint64_t* __restrict__ wbase, uint64_t* __restrict__ res) {
    const uint64_t k = (uint64_t)blockIdx.x * kThreads + threadIdx.x;
    if (k >= nb) return;
    if (blk_status[k] != 0) atomicMin((unsigned long long*)res, (unsigned long long)wbase[k]);
}

// The last block may end in a record the stream cuts short: its unit then
// ends after its last complete record, and only those words count.
// tail[0] = that byte, tail[1] = the stream's complete words.
// The first block whose chain ran past the stream end (a record the stream
// cuts short): the blocks before it are exact and complete.  *kerr starts at nb.
__global__ void k_first_err(const uint64_t* __restrict__ exit_, uint64_t nb, uint64_t nbytes,
                            unsigned long long* __restrict__ kerr) {
    const uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k < nb && exit_[k] > nbytes) atomicMin(kerr, (unsigned long long)k);
}

// The longest prefix of complete records with at most max_words words:
// cut[0] = its bytes, cut[1] = its words, *cutk = the block it ends in.  The
// one block where the prefix ends (its words cross max_words, or it is the
// last trusted block) walks its records from its entry.
__global__ void k_cut(const uint8_t* __restrict__ in, uint64_t nbytes, uint64_t max_words,
                      const uint64_t* __restrict__ exit_, const uint64_t* __restrict__ wbase,
                      const uint64_t* __restrict__ words, uint64_t nb,
                      const unsigned long long* __restrict__ kerr, uint64_t* __restrict__ cut,
                      uint64_t* __restrict__ cutk) {
    const uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t ke = *kerr;
    if (k >= nb || k > ke) return;
    const uint64_t lo = wbase[k];
    if (lo > max_words) return;
    if (k != ke && k != nb - 1 && lo + words[k] <= max_words) return;
    uint64_t p = k == 0 ? 0 : exit_[k - 1], w = lo;
    while (p < nbytes) {
        uint64_t q = p, dw = 0;
        hop(in, q, dw, nbytes);
        if (q > nbytes || w + dw > max_words) break;
        p = q;
        w += dw;
    }
    cut[0] = p;
    cut[1] = w;
    *cutk = k;
}

// The same prefix by one lane walking from the stream start: the fallback
// when the resolution did not settle (fix passes past kMaxPasses, e.g. a
// literal-run region longer than kMaxPasses tiles, which no speculative chain
// couples with).
__global__ void k_cut_serial(const uint8_t* __restrict__ in, uint64_t nbytes, uint64_t max_words,
                             uint64_t* __restrict__ cut) {
    uint64_t p = 0, w = 0;
    while (p < nbytes) {
        uint64_t q = p, dw = 0;
        hop(in, q, dw, nbytes);
        if (q > nbytes || w + dw > max_words) break;
        p = q;
        w += dw;
    }
    cut[0] = p;
    cut[1] = w;
}

// Units after the cut's block are empty at the cut, so a decode of every
// block stops there (the blocks past a record the stream cuts short hold no
// trusted chain).
__global__ void k_set_cut(uint64_t* __restrict__ blk_in, uint64_t* __restrict__ blk_out,
                          uint64_t nb, const uint64_t* __restrict__ cut,
                          const uint64_t* __restrict__ cutk) {
    const uint64_t k = *cutk + 1 + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k > nb) return;
    blk_in[k] = cut[0];
    blk_out[k] = cut[1];
}

__global__ void k_msg_walk(const uint64_t* __restrict__ words, const uint64_t* __restrict__ res,
                           uint64_t max_msgs, uint64_t* __restrict__ ustart,
                           uint64_t* __restrict__ out) {
    // out[0] = messages found, out[1] = word where the walk stopped
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    const uint64_t W = res[0];
    uint64_t u = 0, k = 0;
    while (u < W && k < max_msgs) {
        const uint64_t w0 = words[u];
        const uint32_t nseg = (uint32_t)w0 + 1u;
        if (nseg == 0 || nseg >= 512) break;
        const uint64_t rest = nseg / 2;
        if (u + 1 + rest > W) break;
        uint64_t total = w0 >> 32;
        for (uint64_t i = 1; i < nseg; i++) {
            const uint64_t tw = words[u + 1 + (i - 1) / 2];
            total += ((i - 1) & 1) ? (tw >> 32) : (tw & 0xFFFFFFFFull);
        }
        const uint64_t next = u + 1 + rest + total;
        if (next > W || next < u) break;
        ustart[k++] = u;
        u = next;
    }
    ustart[k] = u;
    out[0] = k;
    out[1] = u;
}

// ---------------------------------------------------------------------------
// Message chain on the decoded words, in parallel (k_msg_walk's result).
// try_read_message's loop is a chain over the words: message k's table gives
// its length and so message k+1's start.  A 1 GiB stream of 12 KiB messages
// is ~87 k dependent loads for one thread (tens of ms); here the words are cut
// into ranges (msg_range_for), one wave each for the spec, one thread each
// after it:
//   spec   range t > 0 scans its words for the first that starts a
//          chain of kMsgVerify messages the loop would read (a body word
//          passes one header check easily, pointers have small low halves,
//          but not kMsgVerify in a row), then follows the chain to its first
//          start at or past the range end (its exit), counting messages.
//          Range 0 starts at word 0: its chain is the true one.  A chain that
//          stops inside the range (a table the loop rejects, or the end of
//          the words) exits kMsgStop | where it stopped.
//   fix    rounds, as the unpack's segment walk: the entry of range t is the
//          max of the ranges' own exits before it; a range whose spec start
//          is its entry keeps its exit and count, another walks from the
//          entry; an entry past the range end (a message longer than a
//          range) or a stop passes through (owns no exit).  Rounds repeat
//          until no entry changes; at that fixed point every exit is its
//          range's walk from its predecessor's exit, by induction the serial
//          chain's.
//   list   exclusive scan of the counts; each range writes its messages'
//          starts (ustart) as k_msg_walk does.
// Ranges of kMsgRange words, doubled up to kMsgRangeMax while a stream has
// more than kMsgRanges of them: each range's spec scan costs the same whatever
// its length (its first message start, ~a message's words in), so fewer,
// longer ranges do less of it; the chain follow inside them is the serial
// loop's work anyway.  A 1 GiB stream of 12 KiB messages, one pass: ranges
// of 4 Ki words 2.9 ms, 16 Ki 2.0, 64 Ki 1.9 (r05z).  Short streams (the
// tests) keep 4 Ki-word ranges, so their chains still cross many ranges.
constexpr uint64_t kMsgRange = 4096;
constexpr uint64_t kMsgRangeMax = 65536;
constexpr uint64_t kMsgRanges = 2048;
constexpr uint32_t kMsgVerify = 16;
constexpr uint64_t kMsgStop = 1ull << 63;
constexpr uint64_t kMsgBad = ~0ull;
constexpr int kMsgMaxRounds = 64;  // then the serial walk (k_msg_walk)

// The start of the message after the one at word u, or kMsgBad if the loop
// does not read a message at u (k_msg_walk's checks).
__device__ __forceinline__ uint64_t msg_next(const uint64_t* __restrict__ words, uint64_t W,
                                             uint64_t u) {
    if (u >= W) return kMsgBad;
    const uint64_t w0 = words[u];
    const uint32_t nseg = (uint32_t)w0 + 1u;
    if (nseg == 0 || nseg >= 512) return kMsgBad;
    const uint64_t rest = nseg / 2;
    if (u + 1 + rest > W) return kMsgBad;
    uint64_t total = w0 >> 32;
    for (uint64_t i = 1; i < nseg; i++) {
        const uint64_t tw = words[u + 1 + (i - 1) / 2];
        total += ((i - 1) & 1) ? (tw >> 32) : (tw & 0xFFFFFFFFull);
    }
    const uint64_t next = u + 1 + rest + total;
    return (next > W || next < u) ? kMsgBad : next;
}

// Follows the chain from x while x < b: -> exit (kMsgStop | x if it stopped
// first), *m = messages passed.
__device__ __forceinline__ uint64_t msg_follow(const uint64_t* __restrict__ words, uint64_t W,
                                               uint64_t x, uint64_t b, uint64_t* m) {
    uint64_t k = 0;
    while (x < b) {
        const uint64_t n = msg_next(words, W, x);
        if (n == kMsgBad) {
            *m = k;
            return kMsgStop | x;
        }
        x = n;
        k++;
    }
    *m = k;
    return x;
}

struct MsgRanges {
    uint64_t* s;     // spec start (kMsgBad: none found)
    uint64_t* xs;    // spec exit
    uint64_t* ms;    // spec messages
    uint64_t* own;   // exit from the entry used
    uint64_t* eu;    // entry used
    uint64_t* cnt;   // messages from the entry used
    uint64_t* xmax;  // inclusive max of own
    uint64_t* base;  // exclusive scan of cnt
    int32_t* flag;   // [0]: a round changed an entry
    void* tmp;
    size_t tmp_bytes;
};

// One wave per range: the lanes test 64 consecutive candidate words at a
// time and the lowest that starts a verified chain is the spec start.  (One
// thread per range had tested them one after another, each test at least
// one dependent load: a 1 GiB stream of 12 KiB messages took 13.1 ms here,
// ~750 candidates before a range's first message start.)
constexpr uint32_t kMsgSpecWaves = kThreads / CAPNP_WAVE;

__global__ void __launch_bounds__(kThreads)
k_msg_spec(const uint64_t* __restrict__ words, const uint64_t* __restrict__ res, uint64_t T,
           MsgRanges R, uint64_t rng) {
    const uint32_t lane = threadIdx.x & (CAPNP_WAVE - 1);
    const uint64_t t = (uint64_t)blockIdx.x * kMsgSpecWaves +
                       (uint32_t)__builtin_amdgcn_readfirstlane((int)(threadIdx.x / CAPNP_WAVE));
    if (t >= T) return;  // (uniform in the wave)
    const uint64_t W = res[0];
    const uint64_t a = t * rng, b = min(a + rng, W);
    uint64_t st = t == 0 ? 0 : kMsgBad;
    for (uint64_t u0 = a; t > 0 && u0 < b; u0 += CAPNP_WAVE) {
        const uint64_t u = u0 + lane;
        bool ok = false;
        if (u < b) {
            uint64_t v = u;
            uint32_t k = 0;
            for (; k < kMsgVerify && v < W; k++) {
                v = msg_next(words, W, v);
                if (v == kMsgBad) break;
            }
            ok = v != kMsgBad && (k == kMsgVerify || (v == W && k > 0));
        }
        const uint64_t m = ballot64(ok);
        if (m) {
            st = u0 + (uint64_t)__builtin_ctzll(m);
            break;
        }
    }
    if (lane != 0) return;
    uint64_t m = 0, x = 0;  // (no start found: owns no exit)
    if (st != kMsgBad && a < W) x = msg_follow(words, W, st, b, &m);
    R.s[t] = st;
    R.xs[t] = x;
    R.ms[t] = m;
    R.own[t] = x;
    R.eu[t] = kMsgBad;
    R.cnt[t] = m;
}

__global__ void __launch_bounds__(kThreads)
k_msg_round(const uint64_t* __restrict__ words, const uint64_t* __restrict__ res, uint64_t T,
            MsgRanges R, uint64_t rng) {
    const uint64_t t = (uint64_t)blockIdx.x * kThreads + threadIdx.x;
    if (t >= T) return;
    const uint64_t W = res[0];
    const uint64_t e = t == 0 ? 0 : R.xmax[t - 1];
    if (e == R.eu[t]) return;
    R.eu[t] = e;
    R.flag[0] = 1;
    const uint64_t a = t * rng, b = min(a + rng, W);
    uint64_t own = 0, m = 0;
    if ((e & kMsgStop) || e >= b || a >= W) {
        own = 0;  // passes its entry on
    } else if (e == R.s[t]) {
        own = R.xs[t];
        m = R.ms[t];
    } else {
        own = msg_follow(words, W, e, b, &m);
    }
    R.own[t] = own;
    R.cnt[t] = m;
}

__global__ void __launch_bounds__(kThreads)
k_msg_list(const uint64_t* __restrict__ words, const uint64_t* __restrict__ res, uint64_t T,
           MsgRanges R, uint64_t max_msgs, uint64_t* __restrict__ ustart, uint64_t rng) {
    const uint64_t t = (uint64_t)blockIdx.x * kThreads + threadIdx.x;
    if (t >= T) return;
    const uint64_t W = res[0];
    const uint64_t a = t * rng, b = min(a + rng, W);
    const uint64_t e = R.eu[t];
    uint64_t k = R.base[t];
    if (!(e & kMsgStop) && e < b && a < W) {
        // (k == max_msgs included: the start where a capped list stops)
        for (uint64_t x = e; x < b && k <= max_msgs; k++) {
            const uint64_t n = msg_next(words, W, x);
            if (n == kMsgBad) break;
            ustart[k] = x;
            x = n;
        }
    }
}

// The chain's end: its stop, or the last exit (>= W); capped at max_msgs
// messages as k_msg_walk.
__global__ void k_msg_end(const uint64_t* __restrict__ res, uint64_t T, MsgRanges R,
                          uint64_t max_msgs, uint64_t* __restrict__ ustart,
                          uint64_t* __restrict__ out, uint64_t* __restrict__ total_out) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    const uint64_t W = res[0];
    const uint64_t total = R.base[T - 1] + R.cnt[T - 1];
    const uint64_t xm = R.xmax[T - 1];
    uint64_t stop = (xm & kMsgStop) ? (xm & ~kMsgStop) : (xm < W ? xm : W);
    uint64_t n = total;
    if (n > max_msgs) {
        n = max_msgs;
        stop = ustart[max_msgs];
    }
    ustart[n] = stop;
    out[0] = n;
    out[1] = stop;
    total_out[0] = total;
}

struct MaxOp {
    __device__ __forceinline__ uint64_t operator()(uint64_t a, uint64_t b) const {
        return a > b ? a : b;
    }
};

size_t msg_chain_tmp_bytes(uint64_t T) {
    size_t a = 0, b = 0;
    (void)hipcub::DeviceScan::InclusiveScan(nullptr, a, (uint64_t*)nullptr, (uint64_t*)nullptr,
                                            MaxOp(), (int)T);
    (void)hipcub::DeviceScan::ExclusiveSum(nullptr, b, (uint64_t*)nullptr, (uint64_t*)nullptr,
                                           (int)T);
    return (a > b ? a : b) + 256;
}

size_t msg_chain_carve(MsgRanges* R, uint8_t* base, uint64_t T) {
    size_t off = 0;
    auto take = [&](size_t bytes) {
        uint8_t* p = base ? base + off : nullptr;
        off += (bytes + 255) & ~size_t(255);
        return p;
    };
    R->s = (uint64_t*)take(8 * T);
    R->xs = (uint64_t*)take(8 * T);
    R->ms = (uint64_t*)take(8 * T);
    R->own = (uint64_t*)take(8 * T);
    R->eu = (uint64_t*)take(8 * T);
    R->cnt = (uint64_t*)take(8 * T);
    R->xmax = (uint64_t*)take(8 * T);
    R->base = (uint64_t*)take(8 * T);
    R->flag = (int32_t*)take(16);
    R->tmp_bytes = msg_chain_tmp_bytes(T);
    R->tmp = take(R->tmp_bytes);
    return off;
}

// (the ranges' workspace for a decoded stream of at most W words: the most
// ranges any W' <= W takes)
uint64_t msg_ranges(uint64_t W) { return W / kMsgRange + 1; }
// the range length for a stream of W words
uint64_t msg_range_for(uint64_t W) {
    uint64_t r = kMsgRange;
    while (r < kMsgRangeMax && W / r > kMsgRanges) r <<= 1;
    return r;
}

size_t msg_chain_ws_bytes(uint64_t W) {
    MsgRanges R;
    return msg_chain_carve(&R, nullptr, msg_ranges(W)) + 256;
}

// The chain over W words (W = res[0], on the device; *W_host the same) into
// ustart / out as k_msg_walk.  d_chain: msg_chain_ws_bytes(W) bytes.
hipError_t msg_chain(const uint64_t* d_words, const uint64_t* res, uint64_t W_host,
                     uint64_t max_msgs, uint64_t* ustart, uint64_t* out, uint64_t* d_total,
                     void* d_chain, size_t chain_bytes, hipStream_t s) {
    const uint64_t rng = msg_range_for(W_host);
    const uint64_t T = W_host / rng + 1;
    MsgRanges R;
    uint8_t* base = (uint8_t*)(((uintptr_t)d_chain + 255) & ~uintptr_t(255));
    if (msg_chain_carve(&R, base, T) + (base - (uint8_t*)d_chain) > chain_bytes)
        return hipErrorInvalidValue;
    hipError_t e;
    const dim3 g((uint32_t)((T + kThreads - 1) / kThreads));
    k_msg_spec<<<dim3((uint32_t)((T + kMsgSpecWaves - 1) / kMsgSpecWaves)), kThreads, 0, s>>>(
        d_words, res, T, R, rng);
    bool done = false;
    for (int round = 0; round < kMsgMaxRounds; round++) {
        size_t tb = R.tmp_bytes;
        if ((e = hipcub::DeviceScan::InclusiveScan(R.tmp, tb, R.own, R.xmax, MaxOp(), (int)T, s)) !=
            hipSuccess)
            return e;
        if ((e = hipMemsetAsync(R.flag, 0, 4, s)) != hipSuccess) return e;
        k_msg_round<<<g, kThreads, 0, s>>>(d_words, res, T, R, rng);
        int32_t changed = 0;
        if ((e = hipMemcpyAsync(&changed, R.flag, 4, hipMemcpyDeviceToHost, s)) != hipSuccess)
            return e;
        if ((e = hipStreamSynchronize(s)) != hipSuccess) return e;
        if (!changed) {
            done = true;
            break;
        }
    }
    if (!done) {  // (not settled: the serial walk, exact; its count is capped)
        k_msg_walk<<<1, 64, 0, s>>>(d_words, res, max_msgs, ustart, out);
        return hipMemcpyAsync(d_total, out, 8, hipMemcpyDeviceToDevice, s);
    }
    size_t tb = R.tmp_bytes;
    if ((e = hipcub::DeviceScan::ExclusiveSum(R.tmp, tb, R.cnt, R.base, (int)T, s)) != hipSuccess)
        return e;
    k_msg_list<<<g, kThreads, 0, s>>>(d_words, res, T, R, max_msgs, ustart, rng);
    k_msg_end<<<1, 64, 0, s>>>(res, T, R, max_msgs, ustart, out, d_total);
    return hipGetLastError();
}

// Packed byte of the record that starts at word u (or ~0 if u is inside a
// record), from block j's entry.
__device__ uint64_t word_to_byte(const uint8_t* __restrict__ in, uint64_t nbytes,
                                 const uint64_t* __restrict__ exit_, const uint64_t* __restrict__ wbase,
                                 uint64_t nb, uint64_t u) {
    uint64_t lo = 0, hi = nb;  // last block with wbase <= u
    while (hi - lo > 1) {
        const uint64_t mid = (lo + hi) >> 1;
        if (wbase[mid] <= u) lo = mid;
        else hi = mid;
    }
    uint64_t p = lo == 0 ? 0 : exit_[lo - 1], w = wbase[lo];
    while (w < u && p < nbytes) hop(in, p, w, nbytes);
    return w == u ? p : ~0ull;
}

__global__ void __launch_bounds__(kThreads)
k_msg_pos(const uint8_t* __restrict__ in, uint64_t nbytes, const uint64_t* __restrict__ exit_,
          const uint64_t* __restrict__ wbase, uint64_t nb, const uint64_t* __restrict__ ustart,
          const uint64_t* __restrict__ out, uint64_t* __restrict__ pos,
          uint64_t* __restrict__ bad) {
    const uint64_t m = out[0];
    const uint64_t k = (uint64_t)blockIdx.x * kThreads + threadIdx.x;
    if (k > m) return;
    const uint64_t p = ustart[k] == 0 ? 0 : word_to_byte(in, nbytes, exit_, wbase, nb, ustart[k]);
    pos[k] = p;
    if (p == ~0ull) atomicMin((unsigned long long*)bad, (unsigned long long)k);
}

}  // namespace

namespace {

// capnp_gpu_read_message_stream: message m (word start ustart[m] in the
// decoded stream) -> its first segment's word, its segment count, and the
// first message whose words exceed the traversal limit (read_message's
// check, serialize.rs:494-501 via read_segment_table).
__global__ void __launch_bounds__(kThreads)
k_msg_meta(const uint64_t* __restrict__ words, const uint64_t* __restrict__ ustart, uint64_t n,
           uint64_t limit, int has_limit, uint64_t* __restrict__ body_off,
           uint64_t* __restrict__ nseg_out, unsigned long long* __restrict__ first_bad) {
    const uint64_t m = (uint64_t)blockIdx.x * kThreads + threadIdx.x;
    if (m >= n) return;
    const uint64_t u = ustart[m];
    const uint64_t w0 = words[u];
    const uint32_t nseg = (uint32_t)w0 + 1u;  // (the chain checked 1 <= nseg < 512)
    uint64_t total = w0 >> 32;
    for (uint32_t i = 1; i < nseg; i++) {
        const uint64_t tw = words[u + 1 + (i - 1) / 2];
        total += ((i - 1) & 1) ? (tw >> 32) : (tw & 0xFFFFFFFFull);
    }
    body_off[m] = u + 1 + nseg / 2;
    nseg_out[m] = nseg;
    if (has_limit && total > limit) atomicMin(first_bad, (unsigned long long)m);
}

__global__ void __launch_bounds__(kThreads)
k_msg_seglist(const uint64_t* __restrict__ words, const uint64_t* __restrict__ ustart, uint64_t n,
              const uint64_t* __restrict__ seg_off, uint64_t* __restrict__ seg_words) {
    const uint64_t m = (uint64_t)blockIdx.x * kThreads + threadIdx.x;
    if (m >= n) return;
    const uint64_t u = ustart[m];
    const uint64_t w0 = words[u];
    const uint32_t nseg = (uint32_t)w0 + 1u;
    uint64_t* out = seg_words + seg_off[m];
    out[0] = w0 >> 32;
    for (uint32_t i = 1; i < nseg; i++) {
        const uint64_t tw = words[u + 1 + (i - 1) / 2];
        out[i] = ((i - 1) & 1) ? (tw >> 32) : (tw & 0xFFFFFFFFull);
    }
}

}  // namespace

extern "C" hipError_t capnp_launch_msg_meta(const uint64_t* d_words, const uint64_t* d_ustart,
                                            uint64_t n, uint64_t limit, int has_limit,
                                            uint64_t* d_body_off, uint64_t* d_nseg,
                                            uint64_t* d_first_bad, hipStream_t s) {
    if (n == 0) return hipSuccess;
    k_msg_meta<<<dim3((uint32_t)((n + kThreads - 1) / kThreads)), kThreads, 0, s>>>(
        d_words, d_ustart, n, limit, has_limit, d_body_off, d_nseg,
        reinterpret_cast<unsigned long long*>(d_first_bad));
    return hipGetLastError();
}

extern "C" hipError_t capnp_launch_msg_seglist(const uint64_t* d_words, const uint64_t* d_ustart,
                                               uint64_t n, const uint64_t* d_seg_off,
                                               uint64_t* d_seg_words, hipStream_t s) {
    if (n == 0) return hipSuccess;
    k_msg_seglist<<<dim3((uint32_t)((n + kThreads - 1) / kThreads)), kThreads, 0, s>>>(
        d_words, d_ustart, n, d_seg_off, d_seg_words);
    return hipGetLastError();
}

// Exclusive scan of n counts into out[0..n] (out[n] = the total).
extern "C" hipError_t capnp_scan_counts(const uint64_t* d_in, uint64_t n, uint64_t* d_out,
                                        void* d_tmp, size_t tmp_bytes, hipStream_t s) {
    hipError_t e = hipMemsetAsync(d_out, 0, 8, s);
    if (e != hipSuccess || n == 0) return e;
    size_t tb = tmp_bytes;
    return hipcub::DeviceScan::InclusiveSum(d_tmp, tb, d_in, d_out + 1, (int)n, s);
}

extern "C" size_t capnp_scan_counts_tmp_bytes(uint64_t n) {
    size_t b = 0;
    (void)hipcub::DeviceScan::InclusiveSum(nullptr, b, (const uint64_t*)nullptr, (uint64_t*)nullptr,
                                           (int)(n ? n : 1));
    return b + 256;
}

// Workspace of the message chain for a decoded stream of up to words_cap
// words (capnp_resync_find_messages: on top of capnp_resync_ws_bytes).
extern "C" size_t capnp_msg_chain_ws_bytes(uint64_t words_cap) {
    return msg_chain_ws_bytes(words_cap) + 256;
}

// The longest prefix of complete records of nbytes packed bytes (which may
// end inside a record) with at most max_words words: *bytes = its packed
// length, *words = the words it decodes to (the resolution above, then the
// cut in the one block where the prefix ends), decoded into d_out[0, *words)
// unless d_out is null.  Blocking.  The stream reader takes its read units
// this way: whole records, so a unit never ends inside a run (the reference's
// read() fails there, serialize_packed.rs:166-185), and where its inner
// reader pends or ends it hands out every complete record first, as
// capnp-futures' PackedRead does (capnp-futures/src/serialize_packed.rs:
// 87-225).
extern "C" hipError_t capnp_resync_decode_prefix(const uint8_t* d_in, uint64_t nbytes,
                                                 uint64_t max_words, uint64_t* d_out, void* d_ws,
                                                 size_t ws_bytes, hipStream_t s, uint64_t* bytes,
                                                 uint64_t* words) {
    *bytes = *words = 0;
    if (nbytes == 0 || max_words == 0) return hipSuccess;
    hipError_t e;
    const uint64_t n = 1;
    const uint64_t nbb = blocks_bound(n, nbytes);
    Ws w;
    uint8_t* base = (uint8_t*)(((uintptr_t)d_ws + 255) & ~uintptr_t(255));
    size_t need = carve(&w, base, n, nbb, scan_tmp_bytes(nbb > 2 ? nbb : 2)) + (base - (uint8_t*)d_ws);
    uint64_t* aux = (uint64_t*)(base + ((need - (base - (uint8_t*)d_ws) + 255) & ~size_t(255)));
    need = (uint8_t*)(aux + 16) - (uint8_t*)d_ws;
    if (need > ws_bytes) return hipErrorInvalidValue;
    uint64_t* in_off = aux;   // [2]
    uint64_t* out_off = aux + 2;  // [2]
    uint64_t* kerr = aux + 4;     // [1]
    uint64_t* cut = aux + 8;      // [2]
    uint64_t* cutk = aux + 10;    // [1]
    const uint64_t h_in_off[2] = {0, nbytes};
    if ((e = hipMemcpyAsync(in_off, h_in_off, 16, hipMemcpyHostToDevice, s)) != hipSuccess) return e;
    k_count<<<grid(n + 1), kThreads, 0, s>>>(in_off, n, in_off, w.nblk);
    size_t tb = w.tmp_bytes;
    if ((e = hipcub::DeviceScan::ExclusiveSum(w.tmp, tb, w.nblk, w.bstart, (int)(n + 1), s)) !=
        hipSuccess)
        return e;
    bool conv = true, capped = false;
    int pass = 0;
    if ((e = resolve(d_in, in_off, n, w, nbb, s, &conv, &capped, &pass)) != hipSuccess) return e;
    if (!conv || capped) {  // exact serial walk for the cut, one unit for the decode
        k_cut_serial<<<1, 1, 0, s>>>(d_in, nbytes, max_words, cut);
        uint64_t hc[2] = {0, 0};
        if ((e = hipMemcpyAsync(hc, cut, 16, hipMemcpyDeviceToHost, s)) != hipSuccess) return e;
        if ((e = hipStreamSynchronize(s)) != hipSuccess) return e;
        *bytes = hc[0];
        *words = hc[1];
        if (!d_out || hc[1] == 0) return hipSuccess;
        const uint64_t h_off[4] = {0, hc[0], 0, hc[1]};
        if ((e = hipMemcpyAsync(in_off, h_off, 32, hipMemcpyHostToDevice, s)) != hipSuccess)
            return e;
        if ((e = capnp_launch_unpack(d_in, in_off, 1, 0, d_out, out_off, w.ok, nullptr, nullptr,
                                     s)) != hipSuccess)
            return e;
        return hipStreamSynchronize(s);
    }
    uint64_t nb = 0;
    if ((e = hipMemcpyAsync(&nb, w.bstart + n, 8, hipMemcpyDeviceToHost, s)) != hipSuccess) return e;
    if ((e = hipStreamSynchronize(s)) != hipSuccess) return e;
    tb = w.tmp_bytes;
    if ((e = hipcub::DeviceScan::ExclusiveSum(w.tmp, tb, w.words, w.wbase, (int)nb, s)) != hipSuccess)
        return e;
    if ((e = hipMemcpyAsync(kerr, &nb, 8, hipMemcpyHostToDevice, s)) != hipSuccess) return e;
    k_first_err<<<grid(nb), kThreads, 0, s>>>(w.exit, nb, nbytes, (unsigned long long*)kerr);
    k_cut<<<grid(nb), kThreads, 0, s>>>(d_in, nbytes, max_words, w.exit, w.wbase, w.words, nb,
                                        (const unsigned long long*)kerr, cut, cutk);
    uint64_t hcut[3] = {0, 0, 0};
    if ((e = hipMemcpyAsync(hcut, cut, 24, hipMemcpyDeviceToHost, s)) != hipSuccess) return e;
    if ((e = hipStreamSynchronize(s)) != hipSuccess) return e;
    *bytes = hcut[0];
    *words = hcut[1];
    if (!d_out || hcut[1] == 0) return hipSuccess;
    // decode blocks 0 .. cut[2] as units, the last one ending at the cut
    const uint64_t nu = hcut[2] + 1;
    const uint64_t h_out_off[2] = {0, hcut[1]};
    if ((e = hipMemcpyAsync(out_off, h_out_off, 16, hipMemcpyHostToDevice, s)) != hipSuccess)
        return e;
    uint64_t* blk_in = w.spec_exit;
    uint64_t* blk_out = w.entry;
    int32_t* blk_status = reinterpret_cast<int32_t*>(w.spec_words);
    k_blocks<<<grid(nb + 1), kThreads, 0, s>>>(in_off, n, out_off, w.bstart, w.exit, w.wbase,
                                               nullptr, blk_in, blk_out, nb);
    k_set_cut<<<1, 64, 0, s>>>(blk_in, blk_out, nu, cut, cutk);
    if ((e = capnp_launch_unpack(d_in, blk_in, nu, 0, d_out, blk_out, blk_status, nullptr, nullptr,
                                 s)) != hipSuccess)
        return e;
    return hipStreamSynchronize(s);
}

extern "C" hipError_t capnp_resync_prefix(const uint8_t* d_in, uint64_t nbytes, void* d_ws,
                                          size_t ws_bytes, hipStream_t s, uint64_t* bytes,
                                          uint64_t* words) {
    return capnp_resync_decode_prefix(d_in, nbytes, ~0ull, nullptr, d_ws, ws_bytes, s, bytes,
                                      words);
}

// The message discovery of capnp_resync_find_messages (below); for
// capnp_resync_read_stream also: the messages' word starts in d_words,
// d_ustart[0..nmsg], and *total_msgs = the messages the chain holds before
// any cap)
static hipError_t find_messages_impl(const uint8_t* d_in, uint64_t nbytes, uint64_t max_msgs,
                                     uint64_t* d_pos, uint64_t* d_words, uint64_t words_cap,
                                     uint64_t* nmsg, int* clean, void* d_ws, size_t ws_bytes,
                                     hipStream_t s, uint64_t* words_needed, uint64_t* d_ustart,
                                     uint64_t* total_msgs) {
    *nmsg = 0;
    *clean = nbytes == 0;
    if (words_needed) *words_needed = 0;
    if (total_msgs) *total_msgs = 0;
    if (nbytes == 0) {
        if (d_ustart) {
            hipError_t e = hipMemsetAsync(d_ustart, 0, 8, s);
            if (e != hipSuccess) return e;
        }
        return hipMemsetAsync(d_pos, 0, 8, s);
    }
    hipError_t e;
    const uint64_t n = 1;
    const uint64_t nbb = blocks_bound(n, nbytes);
    Ws w;
    uint8_t* base = (uint8_t*)(((uintptr_t)d_ws + 255) & ~uintptr_t(255));
    size_t need = carve(&w, base, n, nbb, scan_tmp_bytes(nbb > 2 ? nbb : 2)) + (base - (uint8_t*)d_ws);
    // + in_off[2], out_off[2], res[2], walk out[2], bad, ustart[max_msgs + 1]
    uint64_t* aux = (uint64_t*)(base + ((need - (base - (uint8_t*)d_ws) + 255) & ~size_t(255)));
    need = (uint8_t*)(aux + 12 + max_msgs + 1) - (uint8_t*)d_ws;
    if (need > ws_bytes) return hipErrorInvalidValue;
    uint64_t* in_off = aux;       // [2]
    uint64_t* out_off = aux + 2;  // [2]
    uint64_t* res = aux + 4;      // [1]
    uint64_t* wout = aux + 5;     // [2]
    uint64_t* bad = aux + 7;      // [1]
    uint64_t* dtotal = aux + 10;  // [1]
    uint64_t* ustart = aux + 12;  // [max_msgs + 1]
    // then the message chain's ranges (msg_chain_ws_bytes(words_cap))
    uint8_t* chain = (uint8_t*)(ustart + max_msgs + 1);
    const size_t chain_bytes = msg_chain_ws_bytes(words_cap);
    if ((size_t)(chain + chain_bytes - (uint8_t*)d_ws) > ws_bytes) return hipErrorInvalidValue;
    const uint64_t h_in_off[2] = {0, nbytes};
    if ((e = hipMemcpyAsync(in_off, h_in_off, 16, hipMemcpyHostToDevice, s)) != hipSuccess) return e;
    // (one chunk of nbytes > 0 bytes: k_count never reads its word offsets)
    k_count<<<grid(n + 1), kThreads, 0, s>>>(in_off, n, in_off, w.nblk);
    size_t tb = w.tmp_bytes;
    if ((e = hipcub::DeviceScan::ExclusiveSum(w.tmp, tb, w.nblk, w.bstart, (int)(n + 1), s)) !=
        hipSuccess)
        return e;
    // (not converged, or a capped tile: k_consistent bounds the walk to the
    // exact prefix)
    bool conv = true, capped = false;
    int pass = 0;
    if ((e = resolve(d_in, in_off, n, w, nbb, s, &conv, &capped, &pass)) != hipSuccess) return e;
    uint64_t nb = 0;
    if ((e = hipMemcpyAsync(&nb, w.bstart + n, 8, hipMemcpyDeviceToHost, s)) != hipSuccess) return e;
    if ((e = hipStreamSynchronize(s)) != hipSuccess) return e;
    tb = w.tmp_bytes;
    if ((e = hipcub::DeviceScan::ExclusiveSum(w.tmp, tb, w.words, w.wbase, (int)nb, s)) != hipSuccess)
        return e;
    // the complete-record prefix (a record the stream cuts short ends it)
    uint64_t* tail = aux + 8;  // [2]
    uint64_t* cutk = aux + 11;
    uint64_t* kerr = wout;     // (free until the message chain)
    if ((e = hipMemcpyAsync(kerr, &nb, 8, hipMemcpyHostToDevice, s)) != hipSuccess) return e;
    k_first_err<<<grid(nb), kThreads, 0, s>>>(w.exit, nb, nbytes, (unsigned long long*)kerr);
    k_cut<<<grid(nb), kThreads, 0, s>>>(d_in, nbytes, ~0ull, w.exit, w.wbase, w.words, nb,
                                        (const unsigned long long*)kerr, tail, cutk);
    uint64_t htail[2] = {0, 0};
    if ((e = hipMemcpyAsync(htail, tail, 16, hipMemcpyDeviceToHost, s)) != hipSuccess) return e;
    if ((e = hipStreamSynchronize(s)) != hipSuccess) return e;
    const uint64_t W = htail[1];
    if (words_needed) *words_needed = W;
    if (W > words_cap) return hipErrorInvalidValue;  // caller grows d_words and calls again
    // decode every block as its own unit; a block that fails (a record cut by
    // the stream end, or a chain the fix passes did not settle) bounds the
    // words the walk may use
    const uint64_t h_out_off[2] = {0, W};
    if ((e = hipMemcpyAsync(out_off, h_out_off, 16, hipMemcpyHostToDevice, s)) != hipSuccess)
        return e;
    if ((e = hipMemcpyAsync(res, &W, 8, hipMemcpyHostToDevice, s)) != hipSuccess) return e;
    const uint64_t none = ~0ull;
    if ((e = hipMemcpyAsync(bad, &none, 8, hipMemcpyHostToDevice, s)) != hipSuccess) return e;
    k_consistent<<<grid(nb), kThreads, 0, s>>>(w.entry, w.exit, w.wbase, nb, res);
    uint64_t* blk_in = w.spec_exit;
    uint64_t* blk_out = w.entry;
    int32_t* blk_status = reinterpret_cast<int32_t*>(w.spec_words);
    k_blocks<<<grid(nb + 1), kThreads, 0, s>>>(in_off, n, out_off, w.bstart, w.exit, w.wbase,
                                               nullptr, blk_in, blk_out, nb);
    k_set_cut<<<grid(nb + 1), kThreads, 0, s>>>(blk_in, blk_out, nb, tail, cutk);
    // (block units per decode tile: the unpack's 16; 8 / 12 / sized by the
    // mean words per block for ~1200-word tiles measured 2.10 / 1.96 / 1.97
    // vs 1.89 ms for a 1 GiB carsales stream, r05z)
    if ((e = capnp_launch_unpack(d_in, blk_in, nb, 0, d_words, blk_out, blk_status, nullptr,
                                 nullptr, s)) != hipSuccess)
        return e;
    k_valid_words<<<grid(nb), kThreads, 0, s>>>(blk_status, nb, w.wbase, res);
    if ((e = msg_chain(d_words, res, W, max_msgs, ustart, wout, dtotal, chain, chain_bytes, s)) !=
        hipSuccess)
        return e;
    k_msg_pos<<<grid(max_msgs + 1), kThreads, 0, s>>>(d_in, nbytes, w.exit, w.wbase, nb, ustart,
                                                      wout, d_pos, bad);
    uint64_t hout[2] = {0, 0}, hbad = 0, hres = 0;
    if ((e = hipMemcpyAsync(hout, wout, 16, hipMemcpyDeviceToHost, s)) != hipSuccess) return e;
    if (total_msgs &&
        (e = hipMemcpyAsync(total_msgs, dtotal, 8, hipMemcpyDeviceToHost, s)) != hipSuccess)
        return e;
    if ((e = hipMemcpyAsync(&hbad, bad, 8, hipMemcpyDeviceToHost, s)) != hipSuccess) return e;
    if ((e = hipMemcpyAsync(&hres, res, 8, hipMemcpyDeviceToHost, s)) != hipSuccess) return e;
    if ((e = hipStreamSynchronize(s)) != hipSuccess) return e;
    uint64_t m = hout[0];
    if (hbad != ~0ull) {
        // message hbad starts inside a record: message hbad - 1 is the one
        // that fails; report the messages before it, and its start as the end
        m = hbad == 0 ? 0 : hbad - 1;
    } else if (hres == W && hout[1] == W && m > 0) {
        // the walk consumed every word: clean end if the stream ends there
        uint64_t pend = 0;
        if ((e = hipMemcpyAsync(&pend, w.exit + nb - 1, 8, hipMemcpyDeviceToHost, s)) != hipSuccess)
            return e;
        if ((e = hipStreamSynchronize(s)) != hipSuccess) return e;
        if (pend == nbytes) {
            *clean = 1;
            if ((e = hipMemcpyAsync(d_pos + m, &nbytes, 8, hipMemcpyHostToDevice, s)) != hipSuccess)
                return e;
        }
    }
    *nmsg = m;
    if (d_ustart &&
        (e = hipMemcpyAsync(d_ustart, ustart, 8 * (m + 1), hipMemcpyDeviceToDevice, s)) != hipSuccess)
        return e;
    return hipStreamSynchronize(s);
}

// -> *nmsg complete messages with byte starts d_pos[0..nmsg) and
// d_pos[nmsg] = where the walk stopped (the next message's start, or the
// stream end); *clean = 1 if that is the end of the stream after the last
// message, i.e. the next try_read_message returns None.  A message whose
// start could not be placed truncates the list before the message that
// ended inside a record.  Blocking.
extern "C" hipError_t capnp_resync_find_messages(const uint8_t* d_in, uint64_t nbytes,
                                                 uint64_t max_msgs, uint64_t* d_pos,
                                                 uint64_t* d_words, uint64_t words_cap,
                                                 uint64_t* nmsg, int* clean, void* d_ws,
                                                 size_t ws_bytes, hipStream_t s,
                                                 uint64_t* words_needed) {
    return find_messages_impl(d_in, nbytes, max_msgs, d_pos, d_words, words_cap, nmsg, clean,
                              d_ws, ws_bytes, s, words_needed, nullptr, nullptr);
}

// As capnp_resync_find_messages, keeping the decode: d_words holds the
// stream's words, d_ustart[0..nmsg] the messages' word starts in it (and
// where the chain stopped), *total_msgs the messages the chain holds (more
// than max_msgs: the caller's lists are too short).
extern "C" hipError_t capnp_resync_read_stream(const uint8_t* d_in, uint64_t nbytes,
                                               uint64_t max_msgs, uint64_t* d_pos,
                                               uint64_t* d_words, uint64_t words_cap,
                                               uint64_t* d_ustart, uint64_t* nmsg,
                                               uint64_t* total_msgs, int* clean, void* d_ws,
                                               size_t ws_bytes, hipStream_t s,
                                               uint64_t* words_needed) {
    return find_messages_impl(d_in, nbytes, max_msgs, d_pos, d_words, words_cap, nmsg, clean,
                              d_ws, ws_bytes, s, words_needed, d_ustart, total_msgs);
}
