// unpack.hip — gfx950 UNPACK kernel: the batched body of PackedRead::read
// under read_exact (capnp/src/serialize_packed.rs:80-228, io.rs:16-31).
//
// The decode of one chunk is a serial chain: the position of tag k+1 depends
// on the value of tag k.  Parallelism comes from independent chunks (the
// batch carries a side-band index: each chunk's packed range and unpacked
// length, produced by the encoder's offsets).
//
// Staged path (one 256-thread workgroup per tile of `tc` consecutive chunks
// whose packed bytes and output words fit the LDS tables):
//   stage      the tile's packed bytes (one contiguous range) are copied into
//              LDS with aligned 16-byte loads;
//   walk       one thread per chunk follows the tag chain in LDS (~50-cycle
//              hops instead of L2/MALL round trips) and records, per output
//              word, a descriptor for every record head plus a continuation
//              entry wherever a run covers a 64-word group boundary;
//   expand     lane = output word of the tile (the tile's words are one
//              contiguous range): the covering descriptor is the highest entry
//              at or below the lane in its 64-word group (ballot + clz), the
//              word is rebuilt from LDS (v_perm with a SWAR rank selector) and
//              leaves in coalesced 512-byte stores.
// Global path (tiles that do not fit): lane = chunk walks the chain in
// global memory 64 output words at a time, then the wave expands chunk by
// chunk (the round-1 kernel).
//
// Status per chunk follows the reference exactly (first error in stream
// order): PrematureEndOfPackedInput when a tag, a tag's bytes or a run count
// is missing (:59-74, :109-145), DidNotEndCleanly when a run overruns the
// output (:166-170, :183-187; checked before copying), FailedToFill when a
// literal run's bytes are missing (:195-205 + io.rs:26-28) or the input is
// empty (read() returns 0, io.rs:26-28).
#include "common.h"
#include <stdlib.h>
#include "../../include/capnp_packed.h"
#include "frame.h"

#ifndef UNPACK_PROF
#define UNPACK_PROF 0  // phase timers (scripts/unpack_prof.py); 0 = product
#endif
#ifndef UNPACK_SEGREC
#define UNPACK_SEGREC 1
#endif
#if UNPACK_PROF
// per-tile trace (capnp_unpack_trace): s_memrealtime (100 MHz) at
// [0] start, [1] staged, [2] walked, [3] expanded; [4] 1 = global path
__device__ uint64_t* g_utrace;
__device__ unsigned long long g_uprof[16];  // (UNPACK_PROF: [0] serial chunk walks, [1..7] long-unit phases, [8] overflow tiles, [9] their cycles)
#define UPROF_T(v) const uint64_t v = __builtin_amdgcn_s_memrealtime()
// long-unit phases (unpack_long): g_uprof[1] windows, [2] rounds, [3..7]
// s_memrealtime ticks (10 ns) in stage, spec, rounds, words (+ the last
// segment's walk), descriptors + expansion; thread 0 of each workgroup adds
#define LUPROF_T(v) const uint64_t v = __builtin_amdgcn_s_memrealtime()
#define LUPROF_ADD(i, x) do { if (tid == 0) atomicAdd(&g_uprof[i], (unsigned long long)(x)); } while (0)
#else
#define UPROF_T(v)
#define LUPROF_T(v)
#define LUPROF_ADD(i, x)
#endif

namespace {

constexpr int kWaves = 4;
constexpr int kThreads = kWaves * CAPNP_WAVE;

enum : uint32_t {
    KIND_NONE = 0,
    KIND_NORMAL = 1,   // head word with tag not in {0x00, 0xFF}
    KIND_ZERO = 2,     // tag 0x00 head
    KIND_LIT = 3,      // tag 0xFF head
    KIND_ZERO_CONT = 4,  // zero run carried in from an earlier round
    KIND_LIT_CONT = 5,   // literal run carried in; position = its next raw word
};

enum : int32_t {
    ST_OK = 0,
    ST_PREMATURE = 2,
    ST_NOT_CLEAN = 3,
    ST_FAILED_FILL = 4,
};

// Loads `len` (1..8) bytes at byte position `pos` of `base` with aligned
// 8-byte loads, touching only qwords that hold a requested byte.
__device__ __forceinline__ uint64_t load_bytes(const uint8_t* __restrict__ base, uint64_t pos,
                                               uint32_t len) {
    const uint64_t a = pos & ~7ull;
    const uint32_t s = (uint32_t)(pos & 7);
    const uint64_t* q = reinterpret_cast<const uint64_t*>(base + a);
    uint64_t v = q[0] >> (8 * s);
    if (s + len > 8) v |= q[1] << (64 - 8 * s);
    return v;
}

__device__ __forceinline__ uint64_t expand_word(uint32_t tag, uint64_t packed) {
    const uint64_t sel = expand_selector(tag);
    const uint32_t lo = (uint32_t)packed, hi = (uint32_t)(packed >> 32);
    const uint32_t rlo = __builtin_amdgcn_perm(hi, lo, (uint32_t)sel);
    const uint32_t rhi = __builtin_amdgcn_perm(hi, lo, (uint32_t)(sel >> 32));
    return ((uint64_t)rhi << 32) | rlo;
}

// Global path: lane l < NL of the wave decodes chunk c0 + l (c < c_end);
// `desc` is this wave's NL x 64 descriptor table (NL * 128 bytes of LDS).
template <uint32_t NL>
__device__ void unpack_global(const uint8_t* __restrict__ in, const uint64_t* __restrict__ in_off,
                              uint64_t c0, uint64_t c_end, uint64_t* __restrict__ out,
                              const uint64_t* __restrict__ out_off, int32_t* __restrict__ status,
                              uint64_t* __restrict__ consumed, uint16_t (*desc)[CAPNP_WAVE],
                              uint32_t lane) {
    const uint64_t c = c0 + lane;
    const bool have = lane < NL && c < c_end;
    uint64_t p = 0, in_end = 0, n = 0, obase = 0;
    if (have) {
        p = in_off[c];
        in_end = in_off[c + 1];
        obase = out_off[c];
        n = out_off[c + 1] - obase;
    }
    const uint64_t p_start = p;
    int32_t st = ST_OK;
    uint64_t w = 0;  // words decoded so far
    bool active = have && n > 0;
    if (active && p == in_end) {  // read() returns Ok(0): read_exact fails
        st = ST_FAILED_FILL;
        active = false;
    }
    uint32_t pend_kind = KIND_NONE;  // carried run
    uint64_t pend_rem = 0, pend_src = 0;

    for (uint64_t wbeg = 0; ballot64(active); wbeg += CAPNP_WAVE) {
        // clear this wave's descriptor table (8 KiB, 16 B per lane-store)
        {
            uint4* d4 = reinterpret_cast<uint4*>(&desc[0][0]);
#pragma unroll
            for (uint32_t k = 0; k < NL / 8; k++) d4[k * CAPNP_WAVE + lane] = make_uint4(0, 0, 0, 0);
        }
        wave_lds_sync();

        // ---- walk: lane = chunk
        uint32_t cnt_round = 0;
        uint64_t pb = p;
        if (active) {
            const uint64_t wend = (wbeg + CAPNP_WAVE < n) ? wbeg + CAPNP_WAVE : n;
            if (pend_kind == KIND_LIT_CONT) pb = pend_src;
            if (pend_kind != KIND_NONE) {
                desc[lane][0] = (uint16_t)(pend_kind << 12);  // position = pb
                const uint64_t room = wend - w;
                const uint64_t take = pend_rem < room ? pend_rem : room;
                w += take;
                pend_rem -= take;
                if (pend_kind == KIND_LIT_CONT) pend_src += 8 * take;
                if (pend_rem == 0) pend_kind = KIND_NONE;
            }
            while (w < wend) {
                if (p >= in_end) { st = ST_PREMATURE; break; }
                const uint32_t tag = in[p];
                const uint32_t pop = __builtin_popcount(tag);
                if (p + 1 + pop > in_end) { st = ST_PREMATURE; break; }
                const uint32_t kind = tag == 0 ? KIND_ZERO : (tag == 0xFF ? KIND_LIT : KIND_NORMAL);
                desc[lane][w - wbeg] = (uint16_t)((kind << 12) | (uint32_t)(p - pb));
                uint64_t q = p + 1 + pop;
                w += 1;
                if (kind != KIND_NORMAL) {
                    if (q >= in_end) { st = ST_PREMATURE; break; }
                    const uint64_t cnt = in[q];
                    q += 1;
                    if (cnt > n - w) { st = ST_NOT_CLEAN; break; }
                    uint64_t src = q;
                    if (kind == KIND_LIT) {
                        if (in_end - q < 8 * cnt) { st = ST_FAILED_FILL; break; }
                        q += 8 * cnt;
                    }
                    const uint64_t room = wend - w;
                    const uint64_t take = cnt < room ? cnt : room;
                    w += take;
                    if (cnt > take) {
                        pend_kind = kind == KIND_LIT ? KIND_LIT_CONT : KIND_ZERO_CONT;
                        pend_rem = cnt - take;
                        pend_src = src + 8 * take;
                    }
                }
                p = q;
            }
            cnt_round = (uint32_t)(w - wbeg);
            if (st != ST_OK) { active = false; cnt_round = 0; }
            else if (w == n) active = false;
        }
        wave_lds_sync();

        // ---- expand: lane = word of one chunk at a time
        for (uint32_t s = 0; s < NL; s++) {
            const uint32_t cr = (uint32_t)__builtin_amdgcn_readlane((int)cnt_round, s);
            if (cr == 0) continue;
            const uint64_t pbs = readlane64(pb, s);
            const uint64_t ob = readlane64(obase, s);
            const bool valid = lane < cr;
            const uint32_t d = valid ? desc[s][lane] : 0u;
            const uint64_t heads = ballot64(d != 0);
            const uint64_t hm = heads & low_mask(lane + 1);
            const uint32_t h = hm ? 63u - (uint32_t)__builtin_clzll(hm) : 0u;
            const uint32_t dh = (h == lane) ? d : (uint32_t)desc[s][h];
            const uint32_t kind = dh >> 12;
            const uint64_t pos = pbs + (dh & 0xFFFu);
            uint64_t word = 0;
            if (valid) {
                if (kind == KIND_NORMAL) {
                    const uint32_t tag = in[pos];
                    const uint32_t pop = __builtin_popcount(tag);
                    const uint64_t pk = load_bytes(in, pos + 1, pop);
                    word = expand_word(tag, pk);
                } else if (kind == KIND_LIT) {
                    const uint64_t src = (h == lane) ? pos + 1 : pos + 10 + 8ull * (lane - h - 1);
                    word = load_bytes(in, src, 8);
                } else if (kind == KIND_LIT_CONT) {
                    word = load_bytes(in, pos + 8ull * (lane - h), 8);
                }
                out[ob + wbeg + lane] = word;
            }
        }
        wave_lds_sync();
    }
    if (have) {
        status[c] = st;
        // consumed = where the reference leaves a &[u8] reader: the bytes used
        // on success; all of them on PrematureEnd (refresh_buffer! consumes
        // the buffer first, serialize_packed.rs:59-74) and on FailedToFill
        // (consume + read_exact, :195-205); none on DidNotEndCleanly
        if (consumed)
            consumed[c] = st == ST_OK ? p - p_start : (st == ST_NOT_CLEAN ? 0 : in_end - p_start);
    }
}

// Global path for one chunk too large for the tile tables (unpack_tile_rest):
// the workgroup, windows of kG1Words output words, the descriptor table as one
// flat array.  Lane 0 of wave 0 walks the records from global memory, writing
// a descriptor at each record's first word and a continuation at each 64-word
// group a run enters (positions are 12-bit offsets from the group's first
// source byte, gpb[g]); then all waves expand the window's groups in turn
// with coalesced 512-byte stores.  (Round 4: wave 0 alone expanded, at ~370
// cycles a 512-byte store -- one wave's store throughput: a zero-run chunk of
// 8192 words took ~52 us, scripts/ovf_probe.py; config 4's index-free block
// decode and the drop-in read of long message bodies take this path.)  unpack_global's 64-word windows cost a walk round, an
// 8 KiB table clear and two waits per 64 words: a 512-byte block of zero runs
// (config 4's index-free block decode, ~600-word runs) spent ~1 us per 64 words.
// Statuses, consumed bytes and the words written before an error are
// unpack_global's rules (a window that fails writes nothing).
constexpr uint32_t kG1Words = CAPNP_WAVE * CAPNP_WAVE;

template <typename T>
__device__ void unpack_global1_t(const uint8_t* __restrict__ in_abs,
                               const uint64_t* __restrict__ in_off,
                               uint64_t c, uint64_t* __restrict__ out,
                               const uint64_t* __restrict__ out_off, int32_t* __restrict__ status,
                               uint64_t* __restrict__ consumed, uint16_t* desc, uint32_t* gpb,
                               uint64_t* shared3, uint8_t* bcache, uint32_t lane,
                               uint32_t wave) {
    // positions relative to the chunk start and words in T (32 bits where the
    // chunk allows: the walk's compares then stay scalar -- the SALU has no
    // 64-bit less-than, and each 64-bit compare went through a VALU compare
    // and a VCC branch)
    const uint64_t P0 = uniform64(in_off[c]);
    const uint8_t* __restrict__ in = in_abs + P0;
    const T p_start = 0, in_end = (T)(uniform64(in_off[c + 1]) - P0);
    // wave 0 walks with every lane in step (the same state on each), reading
    // tag and count bytes from a 1 KiB window of the packed bytes in LDS that
    // the wave refills with one coalesced load when a byte falls outside (a
    // lane-0 walk on global memory waited for two dependent loads a record)
    constexpr uint32_t kCache = 16 * CAPNP_WAVE;
    // (positions shifted by the chunk start's misalignment, so that the
    // window bases are aligned and never below the chunk's first vector)
    const uint32_t mis0 = (uint32_t)(reinterpret_cast<uintptr_t>(in) & 15u);
    const uint8_t* __restrict__ in16 = in - mis0;
    T cb0 = (T)~0ull;  // bcache holds shifted bytes [cb0, cb0 + kCache)
    auto byte_at = [&](T x) -> uint32_t {  // (x < in_end; uniform in wave 0)
        const T xs = x + mis0;
        if (xs < cb0 || xs - cb0 >= kCache) {  // (cb0 = ~0: empty)
            cb0 = xs & ~(T)15;
            const T v = cb0 + 16u * lane;
            // (an aligned vector starting before the chunk end stays in mapped memory)
            const uint4 d = v < in_end + mis0 ? *reinterpret_cast<const uint4*>(in16 + v)
                                              : make_uint4(0, 0, 0, 0);
            reinterpret_cast<uint4*>(bcache)[lane] = d;
            wave_lds_sync();
        }
        return bcache[xs - cb0];
    };
    const uint64_t obase = uniform64(out_off[c]);
    const T n = (T)(uniform64(out_off[c + 1]) - obase);
    T p = p_start, w = 0;
    int32_t st = ST_OK;
    bool active = n > 0;
    if (active && p == in_end) {  // read() returns Ok(0): read_exact fails
        st = ST_FAILED_FILL;
        active = false;
    }
    uint32_t pend_kind = KIND_NONE;
    T pend_rem = 0, pend_src = 0;
#if UNPACK_PROF
    const uint64_t gt0 = __builtin_amdgcn_s_memtime();
    uint64_t gwalk = 0, gexp = 0, gwin = 0;
#endif
    for (T wbeg = 0; active; wbeg += kG1Words) {
        __syncthreads();  // (the previous window's expansion is done with the tables)
#if UNPACK_PROF
        const uint64_t gw0 = __builtin_amdgcn_s_memtime();
        gwin++;
#endif
        if (wave == 0) {
            {
                uint4* d4 = reinterpret_cast<uint4*>(desc);
#pragma unroll
                for (uint32_t k = 0; k < kG1Words / 8 / CAPNP_WAVE; k++)
                    d4[k * CAPNP_WAVE + lane] = make_uint4(0, 0, 0, 0);
            }
            wave_lds_sync();
            {
                const T wend = (wbeg + kG1Words < n) ? wbeg + kG1Words : n;
                const T pbw = pend_kind == KIND_LIT_CONT ? pend_src : p;
                int32_t gcur = -1;
                uint32_t gbase = 0;  // gpb[gcur] (the table writes go from lane 0 only:
                                     // 64 lanes storing to one LDS address serialise)
                auto put = [&](T wi, uint32_t kind, T pos) {
                    const uint32_t i = (uint32_t)(wi - wbeg), g = i / CAPNP_WAVE;
                    if ((int32_t)g != gcur) {
                        gbase = (uint32_t)(pos - pbw);
                        if (lane == 0) gpb[g] = gbase;
                        gcur = (int32_t)g;
                    }
                    if (lane == 0)
                        desc[i] = (uint16_t)((kind << 12) | (uint32_t)(pos - pbw - gbase));
                };
                // run words [from, from + take): a continuation at each group start among them
                auto cont = [&](T from, T take, uint32_t kind, T src, T after) {
                    const T r = (from - wbeg) % CAPNP_WAVE;
                    for (T gs = r ? from + (CAPNP_WAVE - r) : from; gs < from + take;
                         gs += CAPNP_WAVE)
                        put(gs, kind, kind == KIND_LIT_CONT ? src + 8 * (gs - from) : after);
                };
                if (pend_kind != KIND_NONE) {  // the run carried in from the previous window
                    const T take = pend_rem < wend - w ? pend_rem : wend - w;
                    cont(w, take, pend_kind, pend_src, p);
                    w += take;
                    pend_rem -= take;
                    if (pend_kind == KIND_LIT_CONT) pend_src += 8 * take;
                    if (pend_rem == 0) pend_kind = KIND_NONE;
                }
                while (w < wend) {
                    if (p >= in_end) { st = ST_PREMATURE; break; }
                    const uint32_t tag = byte_at(p);
                    const uint32_t pop = __builtin_popcount(tag);
                    if (p + 1 + pop > in_end) { st = ST_PREMATURE; break; }
                    const uint32_t kind =
                        tag == 0 ? KIND_ZERO : (tag == 0xFF ? KIND_LIT : KIND_NORMAL);
                    put(w, kind, p);
                    T q = p + 1 + pop;
                    w += 1;
                    if (kind != KIND_NORMAL) {
                        if (q >= in_end) { st = ST_PREMATURE; break; }
                        const T cnt = byte_at(q);
                        q += 1;
                        if (cnt > n - w) { st = ST_NOT_CLEAN; break; }
                        const T src = q;
                        if (kind == KIND_LIT) {
                            if (in_end - q < 8 * cnt) { st = ST_FAILED_FILL; break; }
                            q += 8 * cnt;
                        }
                        const T take = cnt < wend - w ? cnt : wend - w;
                        const uint32_t ck = kind == KIND_LIT ? KIND_LIT_CONT : KIND_ZERO_CONT;
                        cont(w, take, ck, src, q);
                        w += take;
                        if (cnt > take) {
                            pend_kind = ck;
                            pend_rem = cnt - take;
                            pend_src = src + 8 * take;
                        }
                    }
                    p = q;
                }
                uint32_t cnt_round = (uint32_t)(w - wbeg);
                bool more = true;
                if (st != ST_OK) { more = false; cnt_round = 0; }
                else if (w == n) more = false;
                // the window for every wave: {more, words, the window's base byte}
                if (lane == 0) {
                    shared3[0] = more;
                    shared3[1] = cnt_round;
                    shared3[2] = P0 + pbw;  // (absolute: the expansion reads in_abs)
                }
            }
        }
        __syncthreads();
#if UNPACK_PROF
        const uint64_t gw1 = __builtin_amdgcn_s_memtime();
        gwalk += gw1 - gw0;
#endif
        active = uniform64(shared3[0]) != 0;
        const uint32_t cnt_round = (uint32_t)uniform64(shared3[1]);
        const uint64_t pbw = uniform64(shared3[2]);
        for (uint32_t g = wave; g * CAPNP_WAVE < cnt_round; g += kWaves) {
            const uint32_t i = g * CAPNP_WAVE + lane;
            const bool valid = i < cnt_round;
            const uint32_t d = valid ? desc[i] : 0u;
            const uint64_t heads = ballot64(d != 0);
            const uint64_t hm = heads & low_mask(lane + 1);
            const uint32_t h = hm ? 63u - (uint32_t)__builtin_clzll(hm) : 0u;
            const uint32_t dh = (h == lane) ? d : (uint32_t)desc[g * CAPNP_WAVE + h];
            const uint32_t kind = dh >> 12;
            const uint64_t pos = pbw + gpb[g] + (dh & 0xFFFu);  // (absolute)
            uint64_t word = 0;
            if (valid) {
                if (kind == KIND_NORMAL) {
                    const uint32_t tag = in_abs[pos];
                    word = expand_word(tag, load_bytes(in_abs, pos + 1, __builtin_popcount(tag)));
                } else if (kind == KIND_LIT) {
                    const uint64_t src = (h == lane) ? pos + 1 : pos + 10 + 8ull * (lane - h - 1);
                    word = load_bytes(in_abs, src, 8);
                } else if (kind == KIND_LIT_CONT) {
                    word = load_bytes(in_abs, pos + 8ull * (lane - h), 8);
                }
                out[obase + wbeg + i] = word;
            }
        }
#if UNPACK_PROF
        gexp += __builtin_amdgcn_s_memtime() - gw1;
#endif
    }
#if UNPACK_PROF
    if (wave == 0 && lane == 0 && g_utrace) {
        g_utrace[4 * c + 0] = __builtin_amdgcn_s_memtime() - gt0;
        g_utrace[4 * c + 1] = gwalk;
        g_utrace[4 * c + 2] = gexp;
        g_utrace[4 * c + 3] = gwin;
    }
#endif
    if (wave == 0 && lane == 0) {
        status[c] = st;
        if (consumed)
            consumed[c] = st == ST_OK ? p - p_start : (st == ST_NOT_CLEAN ? 0 : in_end - p_start);
    }
}

__device__ void unpack_global1(const uint8_t* __restrict__ in, const uint64_t* __restrict__ in_off,
                               uint64_t c, uint64_t* __restrict__ out,
                               const uint64_t* __restrict__ out_off, int32_t* __restrict__ status,
                               uint64_t* __restrict__ consumed, uint16_t* desc, uint32_t* gpb,
                               uint64_t* shared3, uint8_t* bcache, uint32_t lane,
                               uint32_t wave) {
    const uint64_t nb = uniform64(in_off[c + 1]) - uniform64(in_off[c]);
    const uint64_t nw = uniform64(out_off[c + 1]) - uniform64(out_off[c]);
    if (nb < (1ull << 31) && nw < (1ull << 31))
        unpack_global1_t<uint32_t>(in, in_off, c, out, out_off, status, consumed, desc, gpb,
                                   shared3, bcache, lane, wave);
    else
        unpack_global1_t<uint64_t>(in, in_off, c, out, out_off, status, consumed, desc, gpb,
                                   shared3, bcache, lane, wave);
}


constexpr uint32_t kMaxTileChunks = kWaves * CAPNP_WAVE;

// ---------------------------------------------------------------------------
// Staged path.

// Tile tables sized for kTileWords output words (~5.8 packed bytes per
// word of capacity: P/U up to 0.72; a tile with more is cut into sub-tiles).  The walk and the expansion are latency
// chains, so throughput scales with resident workgroups: smaller tiles, more
// of them per CU (2048 words: ~16 KB of LDS, 9 workgroups per CU).
constexpr uint32_t kTileWords = 2048;
constexpr uint32_t kGroups = 2;  // expansion groups in flight per wave   // descriptor capacity (output words)
// LDS capacity for packed bytes: 5.8 bytes per word of capacity (carsales
// segments pack to 5.6), what is left of 20 KiB per workgroup (8 per CU)
constexpr uint32_t kTileBytes = kTileWords * 93 / 16;
// The global path (tiles that do not fit) runs on as many waves as the
// staged tables' LDS can hold descriptor tables for (8 KiB each).
constexpr uint32_t kGlobalWaves = kTileWords >= 4096 ? 4 : 2;
constexpr uint32_t kStageChunks = 64;    // walkers: one lane of wave 0 per chunk

// Descriptor of an output word (u16), all the expansion needs for the word:
//   p < 0x8000       a record starts at the word, its tag is at LDS byte p
//                    (the tag gives the kind; the word's bytes follow it);
//   kRaw | p         the word is a raw word of a literal run, at LDS byte p;
//   kNone            the word is a word of a zero run (or of a chunk whose
//                    decode failed: output unspecified).
// The walkers write one entry per record plus one per literal-run word
// (rare), so the expansion is a plain per-word lookup: no head search.
constexpr uint16_t kNone = 0xFFFF;
constexpr uint16_t kRaw = 0x8000;

// Raw-word entries of a 0xFF record whose tag is at LDS byte p, head at word
// w, whose run covers words w+1 .. w+n (n <= 255).
template <class SM>
__device__ __forceinline__ void lit_entries(SM& S, uint32_t w, uint32_t p, uint32_t n) {
#pragma clang loop unroll(disable) vectorize(disable)
    for (uint32_t i = 0; i < n; i++) S.dpos[w + 1 + i] = (uint16_t)(kRaw | (p + 10 + 8 * i));
}

// expand_selector for every tag, built at compile time: each tile copies it
// into LDS with one 8-byte load and store per thread.
struct ExpandTable {
    uint64_t s[256];
};
constexpr ExpandTable make_expand_table() {
    ExpandTable t{};
    for (uint32_t tag = 0; tag < 256; tag++) t.s[tag] = expand_selector(tag);
    return t;
}
__device__ constexpr ExpandTable kExpandTable = make_expand_table();

// expand_selector(tag) in registers, a dword per half (byte k = its rank
// among the tag's set bits below k, or 0x0C for a zero byte): the nibble's
// bits spread to bytes by a 24-bit multiply, the ranks by shifted adds, the
// zero bytes by a bitfield insert.  ~20 VALU ops instead of an LDS table
// read (whose 2 KiB per workgroup decides the word tiles' occupancy).
__device__ __forceinline__ uint64_t sel_alu(uint32_t tag) {
    const uint32_t lo8 = __umul24(tag & 15u, 0x00204081u) & 0x01010101u;
    const uint32_t hi8 = __umul24((tag >> 4) & 15u, 0x00204081u) & 0x01010101u;
    const uint32_t loi = lo8 + (lo8 << 8) + (lo8 << 16) + (lo8 << 24);  // inclusive ranks
    // (+ the low nibble's popcount, loi's byte 3, in every byte: one v_perm)
    const uint32_t hii = hi8 + (hi8 << 8) + (hi8 << 16) + (hi8 << 24) +
                         __builtin_amdgcn_perm(0u, loi, 0x03030303u);
    const uint32_t mlo = (lo8 << 8) - lo8, mhi = (hi8 << 8) - hi8;  // 0xFF where set
    const uint32_t slo = ((loi - lo8) & mlo) | (0x0C0C0C0Cu & ~mlo);
    const uint32_t shi = ((hii - hi8) & mhi) | (0x0C0C0C0Cu & ~mhi);
    return ((uint64_t)shi << 32) | slo;
}

#ifndef FIT_SEL_ALU
#define FIT_SEL_ALU 0  // the chunk tiles' expansion computes its selectors
#endif

// Rebuilds one output word from its descriptor (sel = expand selectors).
template <bool ALU = false>
__device__ __forceinline__ uint64_t expand_desc(const uint8_t* B, const uint64_t* sel,
                                                uint32_t d) {
    const bool none = d == kNone, raw = !none && (d & kRaw);
    const uint32_t pos = none ? 0u : (d & 0x7FFFu);
    const uint32_t tag = B[pos];
    // (two naturally aligned 8-byte reads and a funnel shift: a ds_read_b64
    // off 8-byte alignment is replayed at 64 LDS cycles, MI355X_MICROARCH.md
    // §LDS, and was half the LDS time of this kernel)
    const uint32_t src = raw ? pos : pos + 1;
    // three naturally aligned dwords from src & ~3 (never misaligned) and a
    // funnel shift by src & 3 (alignbyte reads only the low two bits)
    const uint32_t* q4 = reinterpret_cast<const uint32_t*>(B + (src & ~3u));
    const uint32_t x0 = q4[0], x1 = q4[1], x2 = q4[2];
    const uint64_t v = ((uint64_t)__builtin_amdgcn_alignbyte(x2, x1, src) << 32) |
                       __builtin_amdgcn_alignbyte(x1, x0, src);
    const uint32_t t = none ? 0u : (raw ? 0xFFu : tag);
    const uint64_t sv = ALU ? sel_alu(t) : sel[t];
    const uint32_t lo = (uint32_t)v, hi = (uint32_t)(v >> 32);
    return ((uint64_t)__builtin_amdgcn_perm(hi, lo, (uint32_t)(sv >> 32)) << 32) |
           __builtin_amdgcn_perm(hi, lo, (uint32_t)sv);
}


// Record sync index (pack.hip): entry k describes global word kSyncWords * k.
constexpr uint32_t kSyncWords = CAPNP_SYNC_WORDS;
constexpr uint32_t kSyncNone = 0xFFFFFFFFu;

// The staged tables for tiles of up to TW output words and TB packed bytes
// (chunk tiles: kTileWords / kTileBytes; word tiles: kWtWords / kWtBytes).
// SEL = false: no selector table (the expansion computes the selectors).
// ENT = false: no sync-walk tables (tiles decoded without the index only).
template <uint32_t TW, uint32_t TB, bool SEL = true, bool ENT = true>
struct StageSmemT {
    static constexpr uint32_t kTW = TW, kTB = TB;
    static constexpr uint32_t kDummy = TW;  // dpos[kDummy + 2 lane]: dummy slots
    static constexpr uint32_t kSeg = ENT ? TW / kSyncWords + 2 : 1;
    union {
        uint64_t sel[SEL ? 256 : 1];  // expand_selector(tag): 0x00 -> zeros, 0xFF -> identity
    };
    uint8_t badc[kStageChunks];     // 1 = the chunk needs the exact walk
    uint32_t cw[kStageChunks + 1];  // chunk word offsets (tile-relative)
    uint32_t cp[kStageChunks + 1];  // chunk packed offsets (LDS positions)
    union {
        struct {
            uint32_t ent[kSeg];             // sync walk: entry of segment b (b >= 1)
            uint8_t segc[kSeg];             // sync walk: chunk that holds segment b's first word
        };
    };
    // word tiles (unpack_wt_kernel): walk start of segment 0 (position + 1,
    // word), the state the last walker must reach at the tile end when the
    // last chunk continues, words of the first chunk before the tile, flags
    uint32_t wt_q0, wt_w0, wt_qB, wt_wB, wt_pre, wt_pl;
    alignas(16) uint8_t bytes[TB + 16];
    alignas(16) uint16_t dpos[TW + 2 * CAPNP_WAVE];  // [TW + 2 lane]: dummy slots
};
using StageSmem = StageSmemT<kTileWords, kTileBytes>;
// The overflow kernels' staged sub-tiles without the index: their LDS holds
// the long-unit tables anyway, room for 4x the words of a tile, so a tile
// that overflows the fit kernel's tables by its words (zero-run units: the
// block decode of config 4) decodes in one or two staged passes instead of
// one per unit.
constexpr uint32_t kBigWords = 4 * kTileWords;
constexpr uint32_t kBigBytes = 16384;
using BigStageSmem = StageSmemT<kBigWords, kBigBytes, true, false>;
#ifndef OVF_BIG
#define OVF_BIG 1
#endif

// Long-unit decode (unpack_long): one chunk too large for the tile tables,
// decoded by the whole workgroup in windows of packed bytes.  Each window
// stages kLuWinBytes of record starts plus the tail of a record that starts
// in them (a literal run: <= 2050 bytes), cut into one kLuSeg-byte segment
// per thread; the decoded words leave in descriptor windows of kLuWords.
constexpr uint32_t kLuSeg = 64;
constexpr uint32_t kLuSegMin = 8;  // (a short last window: segments of at least this many bytes)
constexpr uint32_t kLuWinBytes = kLuSeg * kThreads;     // 16 KiB of record starts
#ifndef UNPACK_LU_LEAD
#define UNPACK_LU_LEAD 64
#endif
constexpr uint32_t kLuLead = UNPACK_LU_LEAD;             // spec lead-in (tests/emu_long.py: 64 > 48)
constexpr uint32_t kLuAvail = kLuWinBytes + 2080;        // bytes staged past the window start
constexpr uint32_t kLuStage = kLuAvail + 32;             // (+ misalignment and a hop's read-ahead)
constexpr uint32_t kLuWords = 8192;                      // descriptor window (output words)
constexpr uint32_t kLuMaxRounds = 64;                    // then the exact serial walk
static_assert(kLuStage + 16 < 0x8000, "LDS positions fit the descriptors' 15 bits");
struct LongSmem {
    uint64_t sel[256];  // (at the offset of StageSmem::sel: the copy serves both)
    alignas(16) uint8_t bytes[kLuStage];
    alignas(16) uint16_t dpos[kLuWords];
    uint32_t wsum[kWaves];
    uint32_t misc[4];
};

union USmem {
    StageSmem st;
    BigStageSmem big;  // (no larger than the long-unit tables: see below)
    uint16_t desc[kGlobalWaves][CAPNP_WAVE][CAPNP_WAVE];  // global path
    LongSmem lu;                                          // long-unit path
};
static_assert(sizeof(BigStageSmem) <= sizeof(LongSmem), "the big sub-tiles fit the long-unit LDS");
static_assert(offsetof(BigStageSmem, sel) == 0 && offsetof(StageSmem, sel) == 0 &&
                  offsetof(LongSmem, sel) == 0, "one selector table serves every view");


// The three bytes of the record whose tag is at LDS byte q-1: tag, q (zero
// run count) and q+8 (literal run count).  Left alone, the compiler merges
// the adjacent tag and count reads into one ds_read_u16, which at an odd
// address is a misaligned LDS access: replayed, and SQ_LDS_UNALIGNED_STALL
// was half of this kernel's LDS cycles.  b1's address goes through an opaque
// copy, so the three reads stay ds_read_u8 (never misaligned).  Round 4
// (interleaved A/B, config 2, settled clocks): byte reads 445 vs 490 us for
// the index-free decode and 297 vs 302 with the index, against the earlier
// form (the tag extracted from its aligned dword, which costs a dependent
// bit-field extract on every hop; round 1 measured that form faster, 403
// vs 427 us, on a walk with more VALU per hop).
__device__ __forceinline__ void rec_bytes(const uint8_t* B, uint32_t q, uint32_t& tag,
                                          uint32_t& b1, uint32_t& b9) {
    const uint32_t p = q - 1u;
    uint32_t p1 = p;
    asm("" : "+v"(p1));  // (b1's address, opaque: no merge with the tag into a u16 read)
    tag = B[p];
    b1 = B[p1 + 1u];
    b9 = B[q + 8];
}

// Exact status of a record that failed the fast check in walk_chunk, in the
// reference's order (serialize_packed.rs:109-145, :157-205).
__device__ __forceinline__ int32_t record_error(uint32_t p, uint32_t q, uint32_t pe, bool run,
                                                bool isf, uint32_t cnt, uint32_t left) {
    if (p >= pe || q > pe || (run && q >= pe)) return ST_PREMATURE;
    if (cnt > left) return ST_NOT_CLEAN;
    if (isf && pe - q - 1 < 8 * cnt) return ST_FAILED_FILL;
    return ST_OK;
}

// Walks one chunk: bytes [p, pe) of the staged tile, output words [wb, wb+n)
// of the tile.  One hop per record: the tag and both possible count bytes
// (p+1 for 0x00, p+9 for 0xFF) are read together, and one check
// (record end <= pe, run end <= chunk end) covers every error.  Status
// precedence and consumed bytes as in unpack_global.  (The exact path behind
// walk_wave: it only runs for chunks whose fast walk failed a check.)
template <class SM>
__device__ __forceinline__ void walk_chunk(SM& S, uint32_t p, uint32_t pe, uint32_t wb,
                                           uint32_t n, int32_t& st, uint32_t& used) {
    const uint32_t p0 = p;
    const uint32_t wend = wb + n;
    uint32_t w = wb;
    st = ST_OK;
    if (n > 0 && p == pe) st = ST_FAILED_FILL;  // read() returns Ok(0)
    bool go = n > 0 && st == ST_OK;
    // Software-pipelined: the next record's three bytes are requested as soon
    // as its position is known, before this record's checks, descriptor
    // write and loop control, which then overlap the LDS latency.  (The
    // empty asm statements pin the reads where they are written.)
    uint32_t tag = 0, b1 = 0, b9 = 0;
    if (go) {
        tag = S.bytes[p];
        b1 = S.bytes[p + 1];
        b9 = S.bytes[p + 9];
        asm volatile("" : "+v"(tag), "+v"(b1), "+v"(b9));
    }
    while (go) {
        const uint32_t q = p + 1 + __builtin_popcount(tag);
        const bool isz = tag == 0, isf = tag == 0xFF;
        const uint32_t cnt = isz ? b1 : (isf ? b9 : 0u);
        const uint32_t end = q + (uint32_t)(isz | isf) + (isf ? 8 * cnt : 0u);
        const uint32_t pn = end < pe ? end : p;  // stays inside the staged bytes
        const uint32_t ntag = S.bytes[pn];
        const uint32_t nb1 = S.bytes[pn + 1];
        const uint32_t nb9 = S.bytes[pn + 9];
        const uint32_t wn = w + 1 + cnt;
        if (end <= pe && wn <= wend) {
            S.dpos[w] = (uint16_t)p;
            if (isf) lit_entries(S, w, p, cnt);
            w = wn;
            p = end;
            go = w < wend;
        } else {
            st = record_error(p, q, pe, isz || isf, isf, cnt, wend - w - 1);
            go = false;
        }
        tag = ntag;
        b1 = nb1;
        b9 = nb9;
    }
    used = st == ST_OK ? p - p0 : (st == ST_NOT_CLEAN ? 0u : pe - p0);
}

// Branch-free walk of the walker wave: lane = chunk, same contract as
// walk_chunk.  Every lane runs every hop (the loop exits on a wave-uniform
// ballot), so there is no exec-mask bookkeeping per record: a lane that has
// finished keeps its state and sends its descriptor store to its own dummy
// slot (one dword per lane: same-address stores from many lanes serialise).
// The hop's dependent chain is the LDS read of the record's three bytes
// (tag, p+1, p+9) and four VALU ops to the next position (popcount with the
// position as accumulator, +isz, select of the 0xFF length, clamp); the
// next reads are issued before the descriptor store, the word count and the
// checks, which overlap their latency.  A record that would fail any check
// stops the lane and marks it bad; bad lanes re-walk with walk_chunk, which
// yields the exact status and consumed count.
template <class SM>
__device__ __forceinline__ void walk_wave(SM& S, uint32_t p, uint32_t pe, uint32_t wb,
                                          uint32_t n, int32_t& st, uint32_t& used) {
    const uint32_t p0 = p;
    const uint32_t wend = wb + n;
    // q = p + 1 (the position after the tag) is the loop state: the popcount
    // accumulates into it directly.  All selects are arithmetic (no branch).
    uint32_t q = p + 1u;
    uint32_t w = wb;
    bool act = n > 0 && p < pe;
    bool bad = n > 0 && p >= pe;
    const uint32_t dummy = SM::kDummy + 2u * lane_id();
    const uint8_t* B = S.bytes;
    uint32_t tag, b1, b9;
    rec_bytes(B, q, tag, b1, b9);
    while (ballot64(act)) {
        const bool isz = tag == 0, isf = tag == 0xFF;
        // end of the record + 1: q + popc + isz (+ 1 + 8 b9 for 0xFF)
        const uint32_t fx = isf ? 8u * b9 + 1u : 0u;
        const uint32_t qe = __builtin_popcount(tag) + q + (isz ? 1u : 0u) + fx + 1u;
        const uint32_t qn = qe < pe + 1u ? qe : pe + 1u;
        uint32_t ntag, nb1, nb9;
        rec_bytes(B, qn, ntag, nb1, nb9);
        const uint32_t cnt = isz ? b1 : (isf ? b9 : 0u);
        const uint32_t wn = w + 1u + cnt;
        const bool ok = act && qe <= pe + 1u && wn <= wend;
        bad = bad || (act && !ok);
        S.dpos[ok ? w : dummy] = (uint16_t)(q - 1u);
        if (ballot64(ok && isf && cnt)) {  // literal-run words (rare)
            if (ok && isf) lit_entries(S, w, q - 1u, cnt);
        }
        q = ok ? qe : q;
        w = ok ? wn : w;
        act = ok && wn < wend;
        tag = ntag;
        b1 = nb1;
        b9 = nb9;
    }
    if (bad) {
        walk_chunk(S, p0, pe, wb, n, st, used);
    } else {
        st = ST_OK;
        used = q - 1u - p0;
    }
}

// ---------------------------------------------------------------------------
// Sync walk: with the record sync index the tile's words split into segments
// at every multiple of kSyncWords (global word index); lane b of the walkers
// walks segment b from the record the index names, across chunk ends, until
// its word reaches the segment end.  The walks are exact if they meet: lane
// b's end state (position, word) must equal the start lane b+1 derives from
// the index, the first segment starts at the tile's first chunk, and every
// chunk must end exactly at its packed end.  Any mismatch, a failed record
// check or a missing entry marks the chunk bad, and bad chunks re-walk
// serially (walk_chunk) with exact status, so the index can only change the
// speed, never the result.

template <class SM>
__device__ __forceinline__ void mark_bad(SM& S, uint32_t c, bool& marked) {
    S.badc[c] = 1;
    marked = true;
}

// Start state of segment b (starting at tile word sb): chunk, position + 1,
// word.  The entry names the record that covers word sb; if that record
// started in an earlier segment (d > 0: a run), it belongs to that
// segment's walker and the segment starts after it.  An unusable entry
// yields the end of its chunk and marks it bad.
//
// WT (word tiles): segment 0 starts where the tile's plan put it (mid-chunk
// after the run that covers the tile's first word), and a run may have its
// head in the first chunk before the tile (wt_pre words of it lie there).
template <class SM, bool WT = false>
__device__ __forceinline__ void seg_start(SM& S, uint32_t nc, uint32_t b, uint32_t sb,
                                          uint32_t& c, uint32_t& q, uint32_t& w, bool mark,
                                          bool& marked) {
    c = S.segc[b];
    if (b == 0) {
        if constexpr (WT) {
            q = S.wt_q0;
            w = S.wt_w0;
        } else {
            q = S.cp[c] + 1u;
            w = 0;
        }
        return;
    }
    const uint32_t e = S.ent[b];
    const uint32_t off = e & 0xFFFFFFu, d = e >> 24;
    const uint32_t cpe1 = S.cp[c + 1] + 1u, cwe = S.cw[c + 1];
    // the run's head word sb - d must lie in chunk c
    uint32_t pre = 0;
    if constexpr (WT) pre = c == 0 ? S.wt_pre : 0u;
    bool ok = e != kSyncNone && off < S.cp[c + 1] - S.cp[c] && d <= sb - S.cw[c] + pre;
    q = S.cp[c] + off + 1u;
    w = sb;
    if (ok && d) {  // skip the run that covers sb
        uint32_t tag, b1, b9;
        rec_bytes(S.bytes, q, tag, b1, b9);
        const bool isz = tag == 0, isf = tag == 0xFF;
        const uint32_t qe = __builtin_popcount(tag) + q + (isz ? 1u : 0u) +
                            (isf ? 8u * b9 + 1u : 0u) + 1u;
        const uint32_t wn = sb - d + 1u + (isz ? b1 : (isf ? b9 : 0u));
        ok = (isz || isf) && wn > sb && wn <= cwe && qe <= cpe1;
        q = qe;
        w = wn;
    }
    if (!ok) {
        if (mark) mark_bad(S, c, marked);
        q = cpe1;
        w = cwe;
    }
}

// Returns true if it marked a chunk bad.
//
// The hop loop is kept short: a lane hops while w < stopw = min(segment
// end, chunk end), one compare per hop; lanes that reach stopw wait for the
// (rare, wave-uniform) stop branch, which moves a lane at a chunk end to the
// next chunk or retires it.  Record checks accumulate into a sticky error
// flag (a failed record ends its chunk; the chunk is re-walked exactly).
//
// WT: the last chunk may continue past the tile (wt_pl): its runs may reach
// past the tile end (their literal entries stop at wlim = the tile's words)
// and the last walker must end in the state the tile plan derived from the
// entry at the tile end.
template <class SM, bool WT = false>
__device__ __forceinline__ bool walk_segment(SM& S, uint32_t nc, uint32_t b, uint32_t sb,
                                             uint32_t eb, bool last, uint32_t wlim = 0) {
    bool marked = false;
    uint32_t c, q, w;
    seg_start<SM, WT>(S, nc, b, sb, c, q, w, true, marked);
    const uint8_t* B = S.bytes;
    const uint32_t dummy = SM::kDummy + 2u * lane_id();
    uint32_t cwe = S.cw[c + 1], cpe1 = S.cp[c + 1] + 1u;
    uint32_t stopw = cwe < eb ? cwe : eb;
    uint32_t tag, b1, b9;
    rec_bytes(B, q, tag, b1, b9);
    bool err = false;
    const uint64_t all = ballot64(true);
    uint64_t done = 0;
#if UNPACK_PROF
    const uint64_t lt0 = __builtin_amdgcn_s_memtime();
    uint32_t iters = 0;
#endif
    // Phase A: kSyncWords hops with no branch at all (a record covers >= 1
    // word, so a lane reaches stopw within kSyncWords hops; a lane already
    // there only sends its store to the dummy slot).  Phase B below handles
    // chunk ends and whatever is left.
    // (the hop runs under the exec mask of the lanes still
    // below stopw, so the state updates need no selects and the record
    // checks collect in a wave mask)
    // (the record checks as running maxima: cpe1 and cwe are fixed in phase
    // A, and a record past either bound is an error wherever it occurs)
    uint32_t qmx = 0, wmx = 0;
#pragma unroll 1  // (x2 / x4 / x8 measured within noise)
    for (uint32_t it = 0; it < kSyncWords; it++) {
        if (w < stopw) {
            const bool isz = tag == 0, isf = tag == 0xFF;
            const uint32_t fx = isf ? 8u * b9 + 1u : 0u;
            const uint32_t qe = __builtin_popcount(tag) + q + (isz ? 1u : 0u) + fx + 1u;
            const uint32_t qn = qe < cpe1 ? qe : cpe1;
            uint32_t ntag, nb1, nb9;
            rec_bytes(B, qn, ntag, nb1, nb9);
            const uint32_t cnt = isz ? b1 : (isf ? b9 : 0u);
            const uint32_t wn0 = w + 1u + cnt;
            qmx = max(qmx, qe);
            wmx = max(wmx, wn0);
            const uint32_t wn = wn0 < cwe ? wn0 : cwe;
            S.dpos[w] = (uint16_t)(q - 1u);
            if (isf && wn > w + 1)  // literal-run words (rare)
                lit_entries(S, w, q - 1u, (WT && wn > wlim ? wlim : wn) - w - 1);
            q = qn;
            w = wn;
            tag = ntag;
            b1 = nb1;
            b9 = nb9;
        }
    }
    err = qmx > cpe1 || wmx > cwe;
#if UNPACK_PROF
    const uint64_t lt1 = __builtin_amdgcn_s_memtime();
#endif
    // Fast end: when every lane reached its segment end within phase A (no
    // chunk ends inside a segment: aligned chunk sizes, the usual case) the
    // state "end of chunk c" already equals "start of chunk c + 1", so the
    // meet checks below cover the chunk-end checks (a failure marks both
    // chunks, which only costs an extra exact walk); only the last segment's
    // lane steps past the tile's last chunk.  Phase B's one bookkeeping
    // round cost ~2500 cycles per wave (UNPACK_PROF).
    const bool fastend = ballot64(!(w >= eb || c >= nc)) == 0;
    if (fastend) {
        if (last && c < nc && w == cwe) {
            if (err || (S.cw[c] < cwe && q != cpe1)) mark_bad(S, c, marked);
            err = false;
            c++;
            while (c < nc && S.cw[c + 1] == w) c++;
        }
    }
    for (; !fastend;) {
#if UNPACK_PROF
        iters++;
#endif
        const bool hop = w < stopw;
        const uint64_t pend = ballot64(!hop) & ~done;
        if (pend) {  // lanes at a chunk end or at their segment end
            if (!hop && !((done >> lane_id()) & 1)) {
                if (w == cwe) {
                    // a non-empty chunk must end exactly at its packed end
                    if (err || (S.cw[c] < cwe && q != cpe1)) {
                        mark_bad(S, c, marked);
                    }
                    err = false;
                    c++;
                    while (c < nc && S.cw[c + 1] == w) c++;  // empty chunks: status OK
                    if (c < nc) {
                        cwe = S.cw[c + 1];
                        cpe1 = S.cp[c + 1] + 1u;
                        q = S.cp[c] + 1u;
                        rec_bytes(B, q, tag, b1, b9);
                    }
                }
                stopw = (c < nc && cwe < eb) ? cwe : eb;
                if (c >= nc) stopw = 0;
            }
            done = ballot64(w >= eb || c >= nc);
            if (done == all) break;
            continue;
        }
        const bool isz = tag == 0, isf = tag == 0xFF;
        const uint32_t fx = isf ? 8u * b9 + 1u : 0u;
        const uint32_t qe = __builtin_popcount(tag) + q + (isz ? 1u : 0u) + fx + 1u;
        const uint32_t qn = qe < cpe1 ? qe : cpe1;
        uint32_t ntag, nb1, nb9;
        rec_bytes(B, qn, ntag, nb1, nb9);
        const uint32_t cnt = isz ? b1 : (isf ? b9 : 0u);
        const uint32_t wn0 = w + 1u + cnt;
        err = err || (hop && (qe > cpe1 || wn0 > cwe));
        const uint32_t wn = wn0 < cwe ? wn0 : cwe;  // (an overrun ends the chunk)
        S.dpos[hop ? w : dummy] = (uint16_t)(q - 1u);
        if (ballot64(hop && isf && wn > w + 1)) {  // literal-run words (rare)
            if (hop && isf) lit_entries(S, w, q - 1u, (WT && wn > wlim ? wlim : wn) - w - 1);
        }
        q = hop ? qn : q;
        w = hop ? wn : w;
        tag = ntag;
        b1 = nb1;
        b9 = nb9;
    }
#if UNPACK_PROF
    if (lane_id() == 0 && g_utrace) {
        g_utrace[blockIdx.x * 8 + 5] = iters;
        g_utrace[blockIdx.x * 8 + 6] = __builtin_amdgcn_s_memtime() - lt0;
        g_utrace[blockIdx.x * 8 + 7] = lt1 - lt0;
    }
#endif
    // the walks must meet
    if (last) {
        bool pl = false;
        if constexpr (WT) pl = S.wt_pl != 0;
        if (pl) {
            if constexpr (WT)
                // (c == nc: the walk reached the chunk's end exactly, just past
                // the tile, and passed its end check)
                if (c + 1 < nc || q != S.wt_qB || w != S.wt_wB || err) {
                    mark_bad(S, nc - 1, marked);
                }
        } else if (c < nc) {
            mark_bad(S, c, marked);
        }
    } else {
        uint32_t c2, q2, w2;
        seg_start<SM, WT>(S, nc, b + 1, eb, c2, q2, w2, false, marked);
        // (positions and words decide: "end of chunk c" and "start of chunk
        // c+1" are the same state)
        if (q2 != q || w2 != w || err) {
            if (c < nc) mark_bad(S, c, marked);
            mark_bad(S, c2, marked);
        }
    }
    return marked;
}

// Index-free walk of a staged tile on every thread (tiles of
// at most 16 chunks): each chunk's packed bytes are cut into S = 16 equal
// byte segments, one thread each, so a chunk's ~117-record
// chain becomes S chains of ~117 / S records and all four waves walk
// (the serial walker used 16 lanes of one wave for the whole chain).
//   1. spec: thread (c, j) walks from kSegOverlap bytes before its segment
//      start sb until it passes the segment end se, and keeps its first
//      record start at or past sb (f) and its exit.  Tag chains from
//      different starts couple within tens of bytes, so by sb the chain is
//      mostly the true one already.  j = 0 starts at the chunk start.
//   2. meet / repair: the true entry of segment j is the exit of segment
//      j - 1.  If the spec chain passes through it (f = entry), its exit and
//      words stand; otherwise the thread walks exactly from the entry.  A
//      segment whose exit changed makes its successor check again, round
//      after round within the wave, until no exit changes.  On config-2 data
//      4 % of the segments miss (16 % with no lead-in), so most waves need
//      one repair round.  A chunk is exact if its last exit is its packed
//      end with exactly its words and no record ran past the end; otherwise
//      (malformed input) it takes the exact serial walk for the status.
//   3. desc: word bases by a scan of the segment words; each thread writes
//      the descriptors of its records, from its entry to its exit.
// Speculation changes the speed only, never the result.
// spec walk lead-in (bytes); config 2 nosync: 0 -> 724 us, 16 -> 699,
// 32 -> 646, 48 -> 614, 64 -> 640 (re-checked in round 3: 40-64 within noise)
#ifndef UNPACK_SEG_OVERLAP
#define UNPACK_SEG_OVERLAP 48
#endif
constexpr uint32_t kSegOverlap = UNPACK_SEG_OVERLAP;
constexpr uint32_t kSegChunks = 16;  // tiles of at most this many chunks take the segment walk


// One record hop (the walk's loops stop once p >= the segment end, so a
// record running past the chunk end shows as p > pe at the stop).
__device__ __forceinline__ void seg_hop(const uint8_t* B, uint32_t& p, uint32_t& w) {
    uint32_t tag, b1, b9;
    rec_bytes(B, p + 1u, tag, b1, b9);
    asm("" : "+v"(tag));  // (tag's range unknown: no 16-bit arithmetic on it)
    const bool isz = tag == 0, isf = tag == 0xFF;
    const uint32_t cnt = isf ? b9 : (isz ? b1 : 0u);
    const uint32_t ext = isf ? 8u * b9 + 1u : (isz ? 1u : 0u);
    p += __builtin_popcount(tag) + ext + 1u;
    w += 1u + cnt;
}

#if UNPACK_SEGREC
// A segment walk that keeps its first kSegRecs records in registers
// (position | word offset from the walk start << 16), so that the
// descriptor pass writes them without walking the chain again; a walk of
// more records re-walks only the rest, from (qr, wr).
constexpr uint32_t kSegRecs = 12;
struct SegRecs {
    uint32_t r[kSegRecs];
    uint32_t nr, qr, wr;
};

// Walks from q (word 0) until q >= se -> exit q, words w.
__device__ __forceinline__ void seg_walk_rec(const uint8_t* B, uint32_t& q, uint32_t& w,
                                             uint32_t se, SegRecs& sr) {
    w = 0;
    sr.nr = 0;
#pragma unroll
    for (uint32_t k = 0; k < kSegRecs; k++) {
        if (q < se) {
            sr.r[k] = q | (w << 16);
            sr.nr = k + 1u;
            seg_hop(B, q, w);
        }
    }
    sr.qr = q;
    sr.wr = w;
    while (q < se) seg_hop(B, q, w);
}
#endif

// Inclusive max / sum over the lanes of this lane's group of NS (16: a DPP
// row; 8: half a row, j = the lane's index in its group).
template <uint32_t NS>
__device__ __forceinline__ uint32_t grp_max_scan(uint32_t x, uint32_t j) {
    if constexpr (NS == 16) {
        return row_max_scan(x);
    } else {
        static_assert(NS == 8, "groups of 8 or 16 lanes");
        uint32_t t = row_shr<1>(x);  // (unconditional: DPP reads need every lane)
        x = j >= 1 ? max(x, t) : x;
        t = row_shr<2>(x);
        x = j >= 2 ? max(x, t) : x;
        t = row_shr<4>(x);
        return j >= 4 ? max(x, t) : x;
    }
}
template <uint32_t NS>
__device__ __forceinline__ uint32_t grp_sum_scan(uint32_t x, uint32_t j) {
    if constexpr (NS == 16) {
        return row_sum_scan(x);
    } else {
        static_assert(NS == 8, "groups of 8 or 16 lanes");
        uint32_t t = row_shr<1>(x);
        x = j >= 1 ? x + t : x;
        t = row_shr<2>(x);
        x = j >= 2 ? x + t : x;
        t = row_shr<4>(x);
        return j >= 4 ? x + t : x;
    }
}

// Bit index of the k-th (from 0) set bit of m (k < popcount(m)).
__device__ __forceinline__ uint32_t nth_set_bit(uint64_t m, uint32_t k) {
    uint32_t pos = 0;
#pragma unroll
    for (uint32_t half = 32; half; half >>= 1) {
        const uint64_t lo = m & ((1ull << half) - 1ull);
        const uint32_t cnt = (uint32_t)__builtin_popcountll(lo);
        if (k >= cnt) {
            k -= cnt;
            m >>= half;
            pos += half;
        } else {
            m = lo;
        }
    }
    return pos;
}

// LG: 4 = 16 segments per chunk (tiles of <= 16 chunks), 3 = 8 segments per
// chunk (17..32 chunks: short-chunk batches; they had taken the
// one-lane-per-chunk walker).  MAP: the lane groups go to the chunks of
// `am` only (the chunks with words: read_messages interleaves each message's
// table chunk, which has none, with its body), in order; the others keep
// badc 0 and the per-chunk pass gives them OK with nothing consumed.
template <class SM, uint32_t LG = 4, bool MAP = false>
__device__ __forceinline__ void spec_seg_tile(SM& S, uint64_t ca, uint32_t nc,
                                              int32_t* __restrict__ status,
                                              uint64_t* __restrict__ consumed, uint32_t tid,
                                              uint32_t lane, uint64_t am = 0) {
    constexpr uint32_t lg = LG;
    constexpr uint32_t nseg = 1u << lg;
    const uint32_t j = tid & (nseg - 1u);
    uint32_t c = tid >> lg;
    if constexpr (MAP) c = c < (uint32_t)__builtin_popcountll(am) ? nth_set_bit(am, c) : nc;
    const bool act = c < nc;
    uint32_t cs = 0, pe = 0, n = 0, sb = 0, se = 0;
    if (act) {
        cs = S.cp[c];
        pe = S.cp[c + 1];
        n = S.cw[c + 1] - S.cw[c];
        const uint32_t len = pe - cs;
        sb = cs + (uint32_t)(((uint64_t)len * j) >> lg);
        se = cs + (uint32_t)(((uint64_t)len * (j + 1u)) >> lg);
    }
    // 1. spec walk from kSegOverlap bytes before the segment (the chain
    // couples with the true one on the way in, mostly): f = its first start
    // at or past sb and the words before it, x = its exit
    const uint32_t s0 = j == 0 ? sb : max(cs, sb >= kSegOverlap ? sb - kSegOverlap : 0u);
    uint32_t p = s0, w = 0;
    while (act && p < sb) seg_hop(S.bytes, p, w);
#if UNPACK_SEGREC
    // (inactive threads: sb = se = 0, no hops)
    const uint32_t f = p;
    SegRecs sr{};
    seg_walk_rec(S.bytes, p, w, se, sr);
    const bool serr = p > pe;
    const uint32_t xs = serr ? 0u : p, ws = w;
    uint32_t own = xs, wd = ws;
    bool err = j == 0 && serr, rep = false;  // rep: sr holds a repair walk's records
    uint32_t e_used = j == 0 ? sb : ~0u;
    uint32_t x = grp_max_scan<nseg>(xs, j);
    for (;;) {
        const uint32_t xu = row_shr<1>(x);
        const uint32_t e = j == 0 ? sb : xu;
        const bool need = act && e != e_used;
        if (ballot64(need) == 0) break;
        if (need) {
            e_used = e;
            if (e == f && !rep) {
                own = xs;
                wd = ws;
                err = serr;
            } else {
                uint32_t q = e, wt;
                seg_walk_rec(S.bytes, q, wt, se, sr);
                rep = true;
                err = q > pe;
                own = (err || e >= se) ? 0u : q;
                wd = wt;
            }
        }
        x = grp_max_scan<nseg>(own, j);
    }
    const uint32_t e = e_used;
    const uint32_t incl = grp_sum_scan<nseg>(wd, j);
    const uint64_t bad_m = ballot64(act && err);
    const uint32_t gl = lane & ~(nseg - 1u);
    const uint64_t gm = ((1ull << nseg) - 1ull) << gl;
    const uint32_t tot = (uint32_t)__shfl((int)incl, (int)(gl + nseg - 1u), 64);
    const uint32_t xl = (uint32_t)__shfl((int)x, (int)(gl + nseg - 1u), 64);
    const bool chunk_ok = act && (bad_m & gm) == 0 && tot == n && xl == pe && n > 0 && pe > cs;
    if (act && j == 0) S.badc[c] = chunk_ok ? 0 : 1;
    // 3. descriptors of the good chunks: the kept records (independent LDS
    // accesses, no chain), then a walk over the rest, if any
    if (chunk_ok) {
        const uint32_t ww = S.cw[c] + incl - wd;  // word of the entry e
        uint32_t lit = 0;
#pragma unroll
        for (uint32_t k = 0; k < kSegRecs; k++) {
            const uint32_t q = sr.r[k] & 0xFFFFu;
            if (k < sr.nr) {
                S.dpos[ww + (sr.r[k] >> 16)] = (uint16_t)q;
                if (S.bytes[q] == 0xFF) lit |= 1u << k;
            }
        }
        while (lit) {  // literal runs (rare)
            const uint32_t k = (uint32_t)__builtin_ctz(lit);
            lit &= lit - 1u;
            uint32_t rk = sr.r[0];
#pragma unroll
            for (uint32_t i = 1; i < kSegRecs; i++)
                if (i == k) rk = sr.r[i];
            const uint32_t q = rk & 0xFFFFu;
            const uint32_t cnt = S.bytes[q + 9];
            if (cnt) lit_entries(S, ww + (rk >> 16), q, cnt);
        }
        uint32_t q = sr.qr, wq = ww + sr.wr;
        (void)e;
        while (q < x) {
            uint32_t tag, b1, b9;
            rec_bytes(S.bytes, q + 1u, tag, b1, b9);
            const bool isz = tag == 0, isf = tag == 0xFF;
            const uint32_t cnt = isz ? b1 : (isf ? b9 : 0u);
            S.dpos[wq] = (uint16_t)q;
            if (isf && cnt) lit_entries(S, wq, q, cnt);
            wq += 1u + cnt;
            q += 1u + __builtin_popcount(tag) + ((isz || isf) ? 1u : 0u) + (isf ? 8u * cnt : 0u);
        }
    }
#else
    const uint32_t f = p, wf = w;
    while (act && p < se) seg_hop(S.bytes, p, w);
    const bool serr = p > pe;  // (a record past the chunk end: garbage, or j = 0's error)
    const uint32_t xs = serr ? 0u : p, ws = w - wf;
#if UNPACK_PROF
    if (tid == 0 && g_utrace) g_utrace[blockIdx.x * 8 + 5] = __builtin_amdgcn_s_memrealtime();
#endif
    // 2. meet and repair, in rounds within the wave (a chunk's segments are
    // nseg consecutive lanes).  A segment whose spec chain passes through
    // its entry (f = the previous exit) continues the true chain: its exit
    // and words stand.  Otherwise it walks exactly from the entry.  The
    // entries come from a prefix max of the segments' own exits (an exit is
    // never below its entry): a segment whose entry lies past its end owns
    // no exit (0) and passes its entry on, so a record covering several
    // segments settles them all in one round.  A walk that ran past the
    // chunk end owns no exit either (its error flag fails the chunk), so a
    // garbage spec chain cannot hold back the segments after it.  At the
    // fixed point every exit is its segment's walk from its predecessor's
    // exit, and every round settles at least one more segment: at most S + 1
    // rounds.
    uint32_t own = xs, x = xs, wd = ws;  // own: this segment's exit from e_used
    bool err = j == 0 && serr;
    uint32_t e_used = j == 0 ? sb : ~0u;
    for (uint32_t d = 1; d < nseg; d <<= 1) {
        const uint32_t t = (uint32_t)__shfl_up((int)x, d, 64);
        if (j >= d) x = max(x, t);
    }
    for (;;) {
        const uint32_t xu = (uint32_t)__shfl_up((int)x, 1, 64);
        const uint32_t e = j == 0 ? sb : xu;
        const bool need = act && e != e_used;
        if (ballot64(need) == 0) break;
        if (need) {
            e_used = e;
            if (e == f) {
                own = xs;
                wd = ws;
                err = serr;
            } else {
                uint32_t q = e, wt = 0;
                while (q < se) seg_hop(S.bytes, q, wt);
                err = q > pe;
                own = (err || e >= se) ? 0u : q;
                wd = wt;
            }
        }
        x = own;
        for (uint32_t d = 1; d < nseg; d <<= 1) {
            const uint32_t t = (uint32_t)__shfl_up((int)x, d, 64);
            if (j >= d) x = max(x, t);
        }
    }
    const uint32_t e = e_used;
#if UNPACK_PROF
    if (tid == 0 && g_utrace) g_utrace[blockIdx.x * 8 + 6] = __builtin_amdgcn_s_memrealtime();
#endif
    // chunk: segments (c, 0..S-1) are nseg consecutive threads of one wave
    // (S <= 16 divides 64): inclusive scan of wd within the group, no error,
    // and the last exit at the packed end
    uint32_t incl = wd;
    for (uint32_t d = 1; d < nseg; d <<= 1) {
        const uint32_t t = (uint32_t)__shfl_up((int)incl, d, 64);
        if (j >= d) incl += t;
    }
    const uint64_t bad_m = ballot64(act && err);
    const uint32_t gl = lane & ~(nseg - 1u);  // first lane of the group
    const uint64_t gm = ((nseg == 64u) ? ~0ull : ((1ull << nseg) - 1ull)) << gl;
    const uint32_t tot = (uint32_t)__shfl((int)incl, (int)(gl + nseg - 1u), 64);
    const uint32_t xl = (uint32_t)__shfl((int)x, (int)(gl + nseg - 1u), 64);
    const bool chunk_ok = act && (bad_m & gm) == 0 && tot == n && xl == pe && n > 0 && pe > cs;
    if (act && j == 0) S.badc[c] = chunk_ok ? 0 : 1;
    // 3. descriptors of the good chunks: records from the entry to the exit
    if (chunk_ok) {
        uint32_t q = e, ww = S.cw[c] + incl - wd;
        while (q < x) {
            uint32_t tag, b1, b9;
            rec_bytes(S.bytes, q + 1u, tag, b1, b9);
            const bool isz = tag == 0, isf = tag == 0xFF;
            const uint32_t cnt = isz ? b1 : (isf ? b9 : 0u);
            S.dpos[ww] = (uint16_t)q;
            if (isf && cnt) lit_entries(S, ww, q, cnt);
            ww += 1u + cnt;
            q += 1u + __builtin_popcount(tag) + ((isz || isf) ? 1u : 0u) + (isf ? 8u * cnt : 0u);
        }
    }
#endif
#if UNPACK_PROF
    if (tid == 0 && g_utrace) g_utrace[blockIdx.x * 8 + 7] = __builtin_amdgcn_s_memrealtime();
#endif
    __syncthreads();
    if (tid < nc) {
        const uint64_t cc = ca + tid;
        const uint32_t nn = S.cw[tid + 1] - S.cw[tid];
        if (S.badc[tid] && nn) {  // exact serial walk of the chunk
#if UNPACK_PROF
            atomicAdd(&g_uprof[0], 1ull);
#endif
            const uint32_t wa = S.cw[tid], wz = S.cw[tid + 1];
            for (uint32_t i = wa; i < wz; i++) S.dpos[i] = kNone;
            int32_t st;
            uint32_t used;
            walk_chunk(S, S.cp[tid], S.cp[tid + 1], wa, wz - wa, st, used);
            status[cc] = st;
            if (consumed) consumed[cc] = used;
        } else {
            status[cc] = ST_OK;
            if (consumed) consumed[cc] = nn ? S.cp[tid + 1] - S.cp[tid] : 0u;
        }
    }
}

// One staged sub-tile: chunks [ca, cb) whose packed bytes, output words and
// count fit the LDS tables (stage, walk, expand).  All threads of the
// workgroup call it; it ends after its last LDS access of the expansion.

// SELW: the selector table is written here too, its load issued with the
// staging loads (the caller's copy had waited for it before any of them).
// The tile [ca, cb) whose packed bytes are [B0, B1) and words [W0, W1).
template <bool SYNC, bool SELW = false, class SM = StageSmem>
__device__ __forceinline__ void unpack_staged_at(SM& S, const uint8_t* __restrict__ in,
                                                 const uint64_t* __restrict__ in_off, uint64_t ca,
                                                 uint64_t cb, uint64_t* __restrict__ out,
                                                 const uint64_t* __restrict__ out_off,
                                                 int32_t* __restrict__ status,
                                                 uint64_t* __restrict__ consumed,
                                                 const uint32_t* __restrict__ sync, uint32_t tid,
                                                 uint32_t lane, uint32_t wave, uint64_t B0,
                                                 uint64_t B1, uint64_t W0, uint64_t W1) {
    const uint32_t nc = (uint32_t)(cb - ca);
    const uint32_t off0 = (uint32_t)(reinterpret_cast<uintptr_t>(in + B0) & 15u);
    UPROF_T(t0);
    const uint32_t nbytes = (uint32_t)(B1 - B0) + off0;
    const uint32_t Wt = (uint32_t)(W1 - W0);
    // sync segments: [0, kSyncWords kf - W0), then kSyncWords-word blocks up to Wt
    const uint64_t kf = W0 / kSyncWords + 1;
    const uint32_t nseg =
        W1 > W0 ? 1u + (uint32_t)((W1 - 1) / kSyncWords + 1 - kf) : 0u;
    // stage the tile: every load in one round trip, then the LDS writes.  The
    // chunk tables and sync entries come by buffer loads (lanes past them
    // read 0: no branch, so no wait at a join), ahead of the byte loads, so
    // their LDS writes wait only for them (loads return in order); the
    // selector table entry likewise.  (Loads under `if (tid <= nc)` had each
    // waited for everything before them: with the table copy, ~4 dependent
    // round trips before the walk.)
    {
        constexpr uint32_t kLoads = (SM::kTB + 15 + 16 * kThreads - 1) / (16 * kThreads);
        const uint64_t selv = (SELW && !FIT_SEL_ALU) ? kExpandTable.s[tid] : 0;
        uint32_t e_a = 0, e_b = 0;
        const __amdgpu_buffer_rsrc_t ors = __builtin_amdgcn_make_buffer_rsrc(
            const_cast<uint64_t*>(out_off + ca), 0, (int)((nc + 1) * 8), 0x00020000);
        const __amdgpu_buffer_rsrc_t irs = __builtin_amdgcn_make_buffer_rsrc(
            const_cast<uint64_t*>(in_off + ca), 0, (int)((nc + 1) * 8), 0x00020000);
        // (low words: tile-relative offsets fit 32 bits)
        const uint32_t t_w = __builtin_amdgcn_raw_buffer_load_b32(ors, (int)(tid * 8u), 0, 0);
        const uint32_t t_wz = __builtin_amdgcn_raw_buffer_load_b32(ors, (int)(tid * 8u + 8u), 0, 0);
        const uint32_t t_p = __builtin_amdgcn_raw_buffer_load_b32(irs, (int)(tid * 8u), 0, 0);
        if constexpr (SYNC) {
            // entry of segment b >= 1 = sync[kf + b - 1]: b = tid and b = tid + 256
            const __amdgpu_buffer_rsrc_t srs = __builtin_amdgcn_make_buffer_rsrc(
                const_cast<uint32_t*>(sync + (kf - 1)), 0, (int)(nseg * 4), 0x00020000);
            e_a = __builtin_amdgcn_raw_buffer_load_b32(srs, (int)(tid * 4u), 0, 0);
            e_b = __builtin_amdgcn_raw_buffer_load_b32(srs, (int)((tid + kThreads) * 4u), 0, 0);
        }
        const uint4* src = reinterpret_cast<const uint4*>(in + B0 - off0);
        uint4* dst = reinterpret_cast<uint4*>(S.bytes);
        const uint32_t nblk = (nbytes + 15) / 16;
        uint4 r[kLoads];
#pragma unroll
        for (uint32_t k = 0; k < kLoads; k++) {
            const uint32_t idx = tid + k * kThreads;
            r[k] = nblk ? src[idx < nblk ? idx : nblk - 1] : make_uint4(0, 0, 0, 0);
        }
        uint4* dd = reinterpret_cast<uint4*>(S.dpos);
        const uint4 none = make_uint4(~0u, ~0u, ~0u, ~0u);
        for (uint32_t k = tid; k < (Wt + 7) / 8; k += kThreads) dd[k] = none;
        if (SELW && !FIT_SEL_ALU) S.sel[tid] = selv;
        if (tid <= nc) {
            const uint32_t wa = t_w - (uint32_t)W0;
            S.cw[tid] = wa;
            S.cp[tid] = t_p - (uint32_t)B0 + off0;
            if constexpr (SYNC) {
                // segments whose first word (max(0, b G - r0)) lies in this chunk
                const uint32_t wz = tid < nc ? t_wz - (uint32_t)W0 : wa;
                const uint32_t r0 = (uint32_t)(W0 % kSyncWords);
                if (wz > wa) {
                    const uint32_t blo = wa == 0 ? 0u : (wa + r0 + kSyncWords - 1) / kSyncWords;
                    const uint32_t bhi = (wz + r0 + kSyncWords - 1) / kSyncWords;
                    for (uint32_t bb = blo; bb < bhi; bb++) S.segc[bb] = (uint8_t)tid;
                }
            }
        }
        if (tid < kStageChunks) S.badc[tid] = 0;
        if constexpr (SYNC) {
            if (tid >= 1 && tid < nseg) S.ent[tid] = e_a;
            if (tid + kThreads < nseg) S.ent[tid + kThreads] = e_b;
        }
#pragma unroll
        for (uint32_t k = 0; k < kLoads; k++)
            if (tid + k * kThreads < nblk) dst[tid + k * kThreads] = r[k];
    }
    __syncthreads();
    UPROF_T(t1);
    // walk: lane j of one wave follows chunk j.  The walking wave rotates
    // with the tile so that the walks of the workgroups sharing a CU spread
    // over its four SIMDs instead of all landing on wave 0's.
    const uint32_t walker = (blockIdx.x + (uint32_t)ca) & (kWaves - 1);
    if constexpr (SYNC) {
        const uint32_t wrel = (wave - walker) & (kWaves - 1);
        bool marked = false;
        // (one pass unless the segments outnumber the threads: kSyncWords < 16)
        for (uint32_t b = wrel * CAPNP_WAVE + lane; b < nseg; b += kThreads) {
            const uint32_t sb = b == 0 ? 0u : (uint32_t)((kf + b - 1) * kSyncWords - W0);
            const bool last = b + 1 == nseg;
            const uint32_t eb = last ? Wt : (uint32_t)((kf + b) * kSyncWords - W0);
            marked |= walk_segment(S, nc, b, sb, eb, last);
        }
        const bool anybad = __syncthreads_or(marked);
        if (tid < nc) {
            const uint64_t c = ca + tid;
            if (anybad && S.badc[tid]) {  // exact serial walk of the chunk
                const uint32_t wa = S.cw[tid], wz = S.cw[tid + 1];
                for (uint32_t i = wa; i < wz; i++) S.dpos[i] = kNone;
                int32_t st;
                uint32_t used;
                walk_chunk(S, S.cp[tid], S.cp[tid + 1], wa, wz - wa, st, used);
                status[c] = st;
                if (consumed) consumed[c] = used;
            } else {
                status[c] = ST_OK;
                if (consumed)
                    consumed[c] = S.cw[tid + 1] > S.cw[tid] ? S.cp[tid + 1] - S.cp[tid] : 0u;
            }
        }
        if (anybad) __syncthreads();
    } else if (nc <= kSegChunks) {
        spec_seg_tile(S, ca, nc, status, consumed, tid, lane);
    } else if (nc <= 2 * kSegChunks) {
        // (8 segments a chunk: an index-free batch of 64-word chunks 0.30 ->
        // 0.23 ms; read_messages, whose table and body chunks interleave,
        // 1.117 -> 0.714 ms, and with the groups for the bodies only -- 16
        // segments each -- MAP; r05z)
        const uint64_t am = ballot64(lane < nc && S.cw[lane + 1u] > S.cw[lane]);
        const uint32_t na = (uint32_t)__builtin_popcountll(am);
        if (na <= kSegChunks)
            spec_seg_tile<SM, 4, true>(S, ca, nc, status, consumed, tid, lane, am);
        else
            spec_seg_tile<SM, 3>(S, ca, nc, status, consumed, tid, lane);
    } else if (wave == walker && lane < nc) {
        // (many short chunks -- the resync blocks, ~120 words -- keep 64
        // serial walkers busy; the segment walk is for few long chunks:
        // config 4 index-free 4.9 ms with this walk, 8.1 with 4 segments
        // per chunk)  // (idle lanes stay off: their LDS traffic counts)
        const uint64_t c = ca + lane;
        const uint64_t gp = in_off[c], ge = in_off[c + 1];
        const uint64_t ow = out_off[c], oe = out_off[c + 1];
        int32_t st;
        uint32_t used;
        walk_wave(S, (uint32_t)(gp - B0) + off0, (uint32_t)(ge - B0) + off0,
                  (uint32_t)(ow - W0), (uint32_t)(oe - ow), st, used);
        status[c] = st;
        if (consumed) consumed[c] = used;
    }
    if constexpr (!SYNC) __syncthreads();
    UPROF_T(t2);
    // expand: lane = output word (a plain descriptor lookup, no head
    // search); 64-word groups interleaved over waves, kGroups per iteration so
    // that their LDS round trips overlap; coalesced 512-byte stores.
    {
        const uint32_t ng = (Wt + CAPNP_WAVE - 1) / CAPNP_WAVE;
        for (uint32_t g0 = wave; g0 < ng; g0 += kGroups * kWaves) {
            uint32_t d[kGroups];
#pragma unroll
            for (int u = 0; u < kGroups; u++) {
                const uint32_t i = (g0 + u * kWaves) * CAPNP_WAVE + lane;
                d[u] = i < Wt ? S.dpos[i] : kNone;
            }
#pragma unroll
            for (int u = 0; u < kGroups; u++) {
                const uint32_t i = (g0 + u * kWaves) * CAPNP_WAVE + lane;
                const uint64_t word = expand_desc<FIT_SEL_ALU>(S.bytes, S.sel, d[u]);
                if (i < Wt) out[W0 + i] = word;
            }
        }
    }
#if UNPACK_PROF
    __syncthreads();
    UPROF_T(t3);
    if (tid == 0 && g_utrace) {
        uint64_t* tr = g_utrace + blockIdx.x * 8;
        tr[0] = t0;
        tr[1] = t1;
        tr[2] = t2;
        tr[3] = t3;
    }
#endif
}

template <bool SYNC, bool SELW = false, class SM = StageSmem>
__device__ __forceinline__ void unpack_staged(SM& S, const uint8_t* __restrict__ in,
                                              const uint64_t* __restrict__ in_off, uint64_t ca,
                                              uint64_t cb, uint64_t* __restrict__ out,
                                              const uint64_t* __restrict__ out_off,
                                              int32_t* __restrict__ status,
                                              uint64_t* __restrict__ consumed,
                                              const uint32_t* __restrict__ sync, uint32_t tid,
                                              uint32_t lane, uint32_t wave) {
    unpack_staged_at<SYNC, SELW, SM>(S, in, in_off, ca, cb, out, out_off, status, consumed, sync,
                                     tid, lane, wave, uniform64(in_off[ca]), uniform64(in_off[cb]),
                                     uniform64(out_off[ca]), uniform64(out_off[cb]));
}

// ---------------------------------------------------------------------------
// Long units: one chunk too large for the tile tables, decoded by the whole
// workgroup (round 5; it replaces the single-wave serial walk of
// unpack_global1, ~1000 cycles a record, as the overflow kernels' path).

// A segment walk from q (word 0) until q >= se -> exit q, words w, keeping
// its first kLuRecs records (position | word offset << 15) so that the
// descriptor pass writes them without walking the chain again.
constexpr uint32_t kLuRecs = 12;
struct LuRecs {
    uint32_t r[kLuRecs];
    uint32_t nr, from;
    bool full;  // every record of the walk is kept
};
__device__ __forceinline__ void lu_walk(const uint8_t* B, uint32_t& q, uint32_t se, uint32_t& w,
                                        LuRecs& rc) {
    rc.from = q;
    rc.nr = 0;
    w = 0;
#pragma unroll
    for (uint32_t k = 0; k < kLuRecs; k++) {
        if (q < se) {
            rc.r[k] = q | (w << 15);
            rc.nr = k + 1u;
            seg_hop(B, q, w);
        }
    }
    rc.full = q >= se;
    while (q < se) seg_hop(B, q, w);
}

// Exclusive max (MAX) or sum over the workgroup's threads in order; *total
// = the value over all of them.  One barrier inside; two uses of wsum need a
// barrier between them (the caller's).
template <bool MAX>
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t x, uint32_t* wsum, uint32_t wave,
                                                    uint32_t lane, uint32_t& total) {
    const uint32_t inc = MAX ? wave_max_scan(x) : wave_sum_scan(x);
    if (lane == CAPNP_WAVE - 1) wsum[wave] = inc;
    __syncthreads();
    uint32_t carry = 0, all = 0;
#pragma unroll
    for (uint32_t k = 0; k < (uint32_t)kWaves; k++) {
        const uint32_t v = wsum[k];
        if (k < wave) carry = MAX ? max(carry, v) : carry + v;
        all = MAX ? max(all, v) : all + v;
    }
    total = all;
    const uint32_t prev = wave_shr1(inc);
    return MAX ? max(prev, carry) : prev + carry;
}

// PackedRead::read_exact of chunk c (serialize_packed.rs:80-228, io.rs:16-31)
// by the whole workgroup, window by window.  A window starts at a record of
// the true chain (P) and stages kLuAvail packed bytes; its first kLuWinBytes
// are cut into one kLuSeg-byte segment per thread, and:
//   spec    each thread walks from kLuLead bytes before its segment (the tag
//           chains from different starts couple on the way in) to its first
//           record start f at or past the segment and on to its exit, the
//           first record start at or past the segment end, counting words;
//   rounds  a segment's entry is the previous segments' exit (an exclusive
//           max over the workgroup); a thread whose entry is not f walks
//           again from it, until no entry changes (spec_seg_tile's rounds,
//           across four waves; a segment inside a longer record owns no
//           exit and passes its entry on);
//   words   an exclusive sum of the segments' words places each segment's
//           records; where the chunk's words end inside the window, the
//           segment holding its last word walks to it with every check (the
//           decode stops right after the record that fills the buffer,
//           :222-225; a run past it is DidNotEndCleanly);
//   expand  in descriptor windows of kLuWords output words: each thread whose
//           words meet the window writes its records' descriptors, then every
//           thread expands words from LDS (expand_desc) in coalesced stores.
// The next window starts at the exit of the last segment.  Anything that is
// not a clean chain -- a record past the chunk's bytes, bytes that end before
// its words, a run past its words, rounds that do not settle -- sends the
// chunk to the exact serial walk (unpack_global1), which gives the status,
// the consumed count and the words written before the error; speculation
// changes the speed only.
__device__ __forceinline__ void unpack_long(USmem& sm, const uint8_t* __restrict__ in,
                            const uint64_t* __restrict__ in_off, uint64_t c,
                            uint64_t* __restrict__ out, const uint64_t* __restrict__ out_off,
                            int32_t* __restrict__ status, uint64_t* __restrict__ consumed,
                            uint32_t tid, uint32_t lane, uint32_t wave, uint32_t pre = 0) {
    // pre: the caller staged in[0, pre) at S.bytes[0, pre) (zeros after it,
    // to kLuStage): a first window inside those bytes is not loaded again
    LongSmem& S = sm.lu;
    const uint64_t P0 = uniform64(in_off[c]);
    const uint64_t E = uniform64(in_off[c + 1]) - P0;  // the chunk's packed bytes
    const uint64_t obase = uniform64(out_off[c]);
    const uint64_t n = uniform64(out_off[c + 1]) - obase;
    const uint8_t* __restrict__ u = in + P0;
    bool bad = n == 0 || E == 0;  // (empty units: the serial walk's rules)
    uint64_t P = 0, W = 0;        // the window's first byte (a true record start), words so far
    S.sel[tid] = kExpandTable.s[tid];
    while (!bad && W < n) {
        const uint64_t rem = E - P;
        const bool tail = rem <= kLuWinBytes;  // every remaining record start is in a segment
        const uint32_t L = rem < kLuAvail ? (uint32_t)rem : kLuAvail;  // bytes staged
        const uint32_t Lc = L < kLuWinBytes ? L : kLuWinBytes;        // record starts cut
        // ---- stage [P, P + L) (16-byte loads from the aligned base below P)
        const bool staged = W == 0 && P0 + L <= pre;  // (uniform; zeros follow `pre`)
        const uint32_t mis = staged ? (uint32_t)P0
                                    : (uint32_t)(reinterpret_cast<uintptr_t>(u + P) & 15u);
        const uint4* src = reinterpret_cast<const uint4*>(u + P - mis);
        const uint32_t nblk = (mis + L + 15) / 16;
        __syncthreads();  // (the previous window is done with the LDS)
        LUPROF_T(lt0);
        if (!staged) {
            // LDS DMA, 16 bytes a lane, every load in flight at once (no
            // registers held); the vectors past the chunk's bytes are zeroed
            constexpr uint32_t kVec = kLuStage / 16;
            for (uint32_t i0 = wave * CAPNP_WAVE; i0 < kVec; i0 += kThreads) {
                const uint32_t i = i0 + lane;
                if (i0 + CAPNP_WAVE <= nblk) {
                    __builtin_amdgcn_global_load_lds(
                        (const __attribute__((address_space(1))) void*)(src + i),
                        (__attribute__((address_space(3))) void*)(S.bytes + 16u * i0), 16, 0, 0);
                } else if (i < kVec) {
                    reinterpret_cast<uint4*>(S.bytes)[i] =
                        i < nblk ? src[i] : make_uint4(0, 0, 0, 0);
                }
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's bytes are in
        }
        __syncthreads();
        const uint8_t* B = S.bytes + mis;  // B[x] = the chunk's byte P + x
        LUPROF_T(lt1);
        // ---- spec walk (segments of kLuSeg bytes; a last window of fewer
        // bytes cuts shorter ones, down to kLuSegMin, so its walks are short)
        const uint32_t segb = Lc > kLuSegMin * kThreads ? (Lc + kThreads - 1) / kThreads : kLuSegMin;
        const uint32_t sb = tid * segb;
        const bool act = sb < Lc;
        const uint32_t se = act ? (sb + segb < Lc ? sb + segb : Lc) : 0u;
        uint32_t p = (tid == 0 || !act) ? sb : (sb > kLuLead ? sb - kLuLead : 0u);
        uint32_t w = 0;
        while (act && p < sb) seg_hop(B, p, w);
        const uint32_t f = p;
        LuRecs rc;
        lu_walk(B, p, se, w, rc);
        const bool serr = p > L;  // (a record past the staged bytes: past the chunk end)
        const uint32_t xs = serr ? 0u : p, ws = w;
        // (a spec walk that found no record start in its segment says "passes
        // through": it owns no exit; one past the staged bytes owns none)
        const uint32_t xsp = (serr || f >= se) ? 0u : xs;
        uint32_t own = act ? xsp : 0u, wd = act ? ws : 0u;
        bool err = act && serr;
        uint32_t e_used = tid == 0 ? 0u : ~0u, e = 0, xall = 0;
#if UNPACK_PROF
        __syncthreads();  // (the spec walks are done)
#endif
        LUPROF_T(lt2);
        // ---- rounds (resync.hip seg_rounds' rules).  At the fixed point
        // every entry is at or past its segment start: lane 0 walks from the
        // window start, and each later segment's entry is an earlier one's
        // exit (>= that segment's end) or a pass-through's entry -- unless a
        // walk ran past the staged bytes (err), which sends the chunk to the
        // exact walk.  So the rule for an entry below the segment (the spec
        // walk stands in, no walk) acts only on the way there: it keeps a
        // pass-through on a missed spec walk's far garbage exit from erasing
        // its successors' exits, which would send them walking from far back.
        for (uint32_t round = 0;; round++) {
            e = block_excl_scan<true>(own, S.wsum, wave, lane, xall);
            const bool need = act && e != e_used;
            if (!__syncthreads_or(need)) {
                LUPROF_ADD(2, round);
                break;
            }
            if (round == kLuMaxRounds) {
                bad = true;
                break;
            }
            if (need) {
                e_used = e;
                if (e < sb || e == f) {  // (below the segment: the spec walk stands in)
                    own = xsp;
                    wd = ws;
                    err = serr;
                } else if (e >= se) {  // a record covers the segment: pass through
                    own = 0;
                    wd = 0;
                    err = false;
                } else {
                    // from the entry, with the spec chain kept in step: where
                    // they meet the rest of the walk is the spec walk's
                    uint32_t pt = e, wt = 0, ps = f, wsp = 0;
                    bool met = false;
#if UNPACK_PROF == 2
                    atomicAdd(&g_uprof[3], 1ull);
#endif
                    while (pt < se) {
                        while (ps < pt && ps < se) seg_hop(B, ps, wsp);
                        if (ps == pt) {
                            met = true;
                            break;
                        }
                        seg_hop(B, pt, wt);
#if UNPACK_PROF == 2
                        atomicAdd(&g_uprof[4], 1ull);
#endif
                    }
                    rc.from = ~0u;  // (the descriptor pass walks from the entry)
                    if (met) {
                        own = xsp;
                        wd = wt + ws - wsp;
                        err = serr;
                    } else {
                        err = pt > L;
                        own = err ? 0u : pt;
                        wd = wt;
                    }
                }
            }
        }
        if (bad) break;
        LUPROF_T(lt3);
        // ---- words
        uint32_t wtot;
        const uint32_t base = block_excl_scan<false>(wd, S.wsum, wave, lane, wtot);
        const uint64_t nrem = n - W;
        const bool fin = (uint64_t)wtot >= nrem;
        uint32_t Wc, adv;
        if (!fin) {
            // the chunk's words go on past the window: its bytes must too
            if (__syncthreads_or(err) || tail || xall > L || xall < Lc) {
                bad = true;
                break;
            }
            Wc = wtot;
            adv = xall;
        } else {
            // the segment holding the last word walks to it with every check
            if (tid == 0) S.misc[0] = kThreads;
            __syncthreads();
            const uint32_t lim = (uint32_t)nrem;
            if (act && base < lim && lim <= base + wd) S.misc[0] = tid;
            __syncthreads();
            const uint32_t ts = S.misc[0];
            const bool errb = __syncthreads_or(err && tid < ts);
            if (tid == ts) {
                uint32_t q = e, wq = base;
                bool ok = true;
                while (wq < lim) {
                    uint32_t tag, b1, b9;
                    rec_bytes(B, q + 1u, tag, b1, b9);
                    const bool isz = tag == 0, isf = tag == 0xFF;
                    const uint32_t cnt = isz ? b1 : (isf ? b9 : 0u);
                    const uint32_t qe = q + 1u + __builtin_popcount(tag) + ((isz || isf) ? 1u : 0u) +
                                        (isf ? 8u * cnt : 0u);
                    const uint32_t wn = wq + 1u + cnt;
                    if (qe > L || wn > lim) {
                        ok = false;
                        break;
                    }
                    q = qe;
                    wq = wn;
                }
                S.misc[1] = q;
                S.misc[2] = ok ? 1u : 0u;
            }
            __syncthreads();
            if (ts >= kThreads || errb || S.misc[2] == 0) {
                bad = true;
                break;
            }
            Wc = lim;
            adv = S.misc[1];
        }
        LUPROF_T(lt4);
        // ---- descriptors and expansion, kLuWords output words at a time
        for (uint32_t sw = 0; sw < Wc; sw += kLuWords) {
            const uint32_t swe = Wc - sw < kLuWords ? Wc : sw + kLuWords;
            __syncthreads();  // (the previous descriptor window is expanded)
            {
                uint4* d4 = reinterpret_cast<uint4*>(S.dpos);
                const uint4 none = make_uint4(~0u, ~0u, ~0u, ~0u);
#pragma unroll
                for (uint32_t k = 0; k < kLuWords / 8 / kThreads; k++) d4[tid + k * kThreads] = none;
            }
            __syncthreads();
            if (act && wd > 0 && base < swe && base + wd > sw) {
                const uint32_t wlim = base + wd < swe ? base + wd : swe;
                if (rc.from == e && rc.full) {
                    // the records of the walk from the entry, kept in registers:
                    // independent LDS accesses, no chain; literal runs after
                    uint32_t lit = 0;
#pragma unroll
                    for (uint32_t k = 0; k < kLuRecs; k++) {
                        const uint32_t q = rc.r[k] & 0x7FFFu, wq = base + (rc.r[k] >> 15);
                        if (k < rc.nr && wq < wlim) {
                            if (wq >= sw) S.dpos[wq - sw] = (uint16_t)(q + mis);
                            if (B[q] == 0xFF) lit |= 1u << k;
                        }
                    }
                    while (lit) {  // literal runs (rare)
                        const uint32_t k = (uint32_t)__builtin_ctz(lit);
                        lit &= lit - 1u;
                        uint32_t rk = rc.r[0];
#pragma unroll
                        for (uint32_t i = 1; i < kLuRecs; i++)
                            if (i == k) rk = rc.r[i];
                        const uint32_t q = rk & 0x7FFFu, wq = base + (rk >> 15);
                        const uint32_t lp = q + mis, cnt = B[q + 9u];
                        const uint32_t lo = wq + 1u > sw ? wq + 1u : sw;
                        const uint32_t hi = wq + 1u + cnt < swe ? wq + 1u + cnt : swe;
                        for (uint32_t i = lo; i < hi; i++)
                            S.dpos[i - sw] = (uint16_t)(kRaw | (lp + 10u + 8u * (i - wq - 1u)));
                    }
                } else {
                uint32_t q = e, wq = base;
                while (wq < wlim) {
                    uint32_t tag, b1, b9;
                    rec_bytes(B, q + 1u, tag, b1, b9);
                    const bool isz = tag == 0, isf = tag == 0xFF;
                    const uint32_t cnt = isz ? b1 : (isf ? b9 : 0u);
                    const uint32_t lp = q + mis;  // (LDS position of the tag)
                    if (wq >= sw) S.dpos[wq - sw] = (uint16_t)lp;
                    if (isf && cnt) {  // literal-run words (raw, 8 bytes each after the count)
                        const uint32_t lo = wq + 1u > sw ? wq + 1u : sw;
                        const uint32_t hi = wq + 1u + cnt < swe ? wq + 1u + cnt : swe;
                        for (uint32_t i = lo; i < hi; i++)
                            S.dpos[i - sw] = (uint16_t)(kRaw | (lp + 10u + 8u * (i - wq - 1u)));
                    }
                    wq += 1u + cnt;
                    q += 1u + __builtin_popcount(tag) + ((isz || isf) ? 1u : 0u) +
                         (isf ? 8u * cnt : 0u);
                }
                }
            }
            __syncthreads();
            uint64_t* o = out + obase + W + sw;
            // (a zero-run word needs no LDS read past its descriptor: zero-run
            // windows -- config 4's index-free block decode -- expand at the
            // stores' rate)
#pragma unroll 4
            for (uint32_t i = tid; i < swe - sw; i += kThreads) {
                const uint32_t d = S.dpos[i];
                o[i] = d == kNone ? 0ull : expand_desc(S.bytes, S.sel, d);
            }
        }
        W += Wc;
        P += adv;
#if UNPACK_PROF
        __syncthreads();
        LUPROF_T(lt5);
        LUPROF_ADD(1, 1);
#if UNPACK_PROF != 2
        LUPROF_ADD(3, lt1 - lt0);
        LUPROF_ADD(4, lt2 - lt1);
#endif
        LUPROF_ADD(5, lt3 - lt2);
        LUPROF_ADD(6, lt4 - lt3);
        LUPROF_ADD(7, lt5 - lt4);
#endif
    }
    if (bad) {  // the exact serial walk, from the chunk start
        __syncthreads();
        unpack_global1(in, in_off, c, out, out_off, status, consumed, &sm.desc[0][0][0],
                       reinterpret_cast<uint32_t*>(&sm.desc[1][0][0]),
                       reinterpret_cast<uint64_t*>(&sm.desc[1][8][0]),
                       reinterpret_cast<uint8_t*>(&sm.desc[1][16][0]), lane, wave);
        return;
    }
    if (tid == 0) {
        status[c] = ST_OK;
        if (consumed) consumed[c] = P;
    }
}

// One workgroup per tile of `tc` chunks.  The tile is cut into sub-tiles
// that fit the LDS tables (normally one: the whole tile), each staged,
// walked and expanded in turn; a single chunk too large for the tables
// takes the global path.
// The tile's chunks [ca, cb) when they do not all fit at once: the longest
// prefixes that fit, staged in turn, and a chunk too large alone on the
// global path.
template <bool SYNC, bool G1 = false>
__device__ void unpack_tile_rest(USmem& sm, const uint8_t* __restrict__ in,
                                 const uint64_t* __restrict__ in_off, uint64_t ca, uint64_t cb,
                                 uint64_t* __restrict__ out, const uint64_t* __restrict__ out_off,
                                 int32_t* __restrict__ status, uint64_t* __restrict__ consumed,
                                 const uint32_t* __restrict__ sync, uint32_t tid, uint32_t lane,
                                 uint32_t wave) {
    bool first = true, resel = false;
    // (without the index the sub-tiles take the larger tables)
    constexpr bool kBig = !SYNC && OVF_BIG;
    constexpr uint64_t kTW = kBig ? kBigWords : kTileWords, kTB = kBig ? kBigBytes : kTileBytes;
    for (uint64_t lo = ca; lo < cb;) {
        // the longest prefix of [lo, cb) that fits: <= kStageChunks chunks,
        // <= kTW words, <= kTB bytes from lo's 16-byte block
        // (the fit is monotone in the prefix, so it is a ballot count)
        const uint64_t B0 = uniform64(in_off[lo]), W0 = uniform64(out_off[lo]);
        const uint32_t off0 = (uint32_t)(reinterpret_cast<uintptr_t>(in + B0) & 15u);
        uint32_t k;
        if (cb - lo <= kStageChunks && uniform64(in_off[cb]) - B0 <= kTB - off0 &&
            uniform64(out_off[cb]) - W0 <= kTW) {
            k = (uint32_t)(cb - lo);  // the usual case: the rest of the tile fits (scalar loads)
        } else {
            const uint64_t c = lo + 1 + lane;
            const bool fit = c <= cb && in_off[c < cb ? c : cb] - B0 <= kTB - off0 &&
                             out_off[c < cb ? c : cb] - W0 <= kTW;
            k = (uint32_t)__builtin_popcountll(ballot64(fit));
        }
        if (!first) __syncthreads();  // the previous sub-tile is done with LDS
        first = false;
        if (k == 0) {  // chunk lo alone does not fit: global walk (wave 0)
#if UNPACK_PROF
            if (tid == 0 && g_utrace) g_utrace[blockIdx.x * 8 + 4] = 1;
#endif
            if (G1)  // (the split overflow kernels; the combined kernels keep their registers)
                unpack_long(sm, in, in_off, lo, out, out_off, status, consumed,
                            lane + wave * CAPNP_WAVE, lane, wave);
            else if (wave == 0)
                unpack_global<CAPNP_WAVE>(in, in_off, lo, lo + 1, out, out_off, status,
                                          consumed, sm.desc[0], lane);
            resel = true;
            lo += 1;
            continue;
        }
        if (resel) {  // the global path's descriptor table overlaid the selectors
            sm.st.sel[tid] = kExpandTable.s[tid];
            resel = false;
        }
        if constexpr (!kBig)
            unpack_staged<SYNC>(sm.st, in, in_off, lo, lo + k, out, out_off, status, consumed,
                                sync, tid, lane, wave);
        else
            unpack_staged<SYNC, false, BigStageSmem>(sm.big, in, in_off, lo, lo + k, out, out_off,
                                                     status, consumed, sync, tid, lane, wave);
        lo += k;
    }
}

// Whether tile [ca, cb) fits the LDS tables at once (the overflow kernels'
// per-lane scan; unpack_fit_kernel makes the same test from its offsets).
__device__ __forceinline__ bool tile_fits_lane(const uint8_t* __restrict__ in,
                                               const uint64_t* __restrict__ in_off,
                                               const uint64_t* __restrict__ out_off, uint64_t ca,
                                               uint64_t cb) {
    const uint64_t B0 = in_off[ca];
    const uint32_t off0 = (uint32_t)(reinterpret_cast<uintptr_t>(in + B0) & 15u);
    return cb - ca <= kStageChunks && in_off[cb] - B0 <= kTileBytes - off0 &&
           out_off[cb] - out_off[ca] <= kTileWords;
}


// Split launch: unpack_fit_kernel stages the tiles that fit and returns on
// the others; unpack_ovf_kernel finds those by the same test (two offsets a
// tile, one lane each) and takes them.
// The fitting path alone needs no registers for the sub-tile loop and the
// global walk, so it does not spill at 8 waves per SIMD (the combined
// kernel spilled 44 B per lane).
template <bool SYNC>
__global__ void __launch_bounds__(kThreads, 8)
unpack_fit_kernel(const uint8_t* __restrict__ in, const uint64_t* __restrict__ in_off,
                  uint64_t nchunks, uint32_t tc, uint64_t* __restrict__ out,
                  const uint64_t* __restrict__ out_off, int32_t* __restrict__ status,
                  uint64_t* __restrict__ consumed, const uint32_t* __restrict__ sync) {
    __shared__ StageSmem S;
    const uint32_t tid = threadIdx.x;
    const uint32_t lane = tid & 63u;
    const uint32_t wave = (uint32_t)__builtin_amdgcn_readfirstlane((int)(tid >> 6));
    const uint64_t ca = (uint64_t)blockIdx.x * tc;
    const uint64_t cb = (ca + tc < nchunks) ? ca + tc : nchunks;
    uint64_t B0, B1, W0, W1;
    sload4(in_off + ca, in_off + cb, out_off + ca, out_off + cb, B0, B1, W0, W1);
    const uint32_t off0 = (uint32_t)(reinterpret_cast<uintptr_t>(in + B0) & 15u);
    if (cb - ca > kStageChunks || B1 - B0 > kTileBytes - off0 || W1 - W0 > kTileWords) {
        return;
    }
    unpack_staged_at<SYNC, true>(S, in, in_off, ca, cb, out, out_off, status, consumed, sync, tid,
                                 lane, wave, B0, B1, W0, W1);
}

template <bool SYNC>
__global__ void __launch_bounds__(kThreads, 4)
unpack_ovf_kernel(const uint8_t* __restrict__ in, const uint64_t* __restrict__ in_off,
                  uint64_t nchunks, uint32_t tc, uint64_t* __restrict__ out,
                  const uint64_t* __restrict__ out_off, int32_t* __restrict__ status,
                  uint64_t* __restrict__ consumed, const uint32_t* __restrict__ sync,
                  uint64_t ntiles) {
    __shared__ USmem sm;
    __shared__ uint32_t lst[kThreads];
    __shared__ uint32_t nl;
    const uint32_t tid = threadIdx.x;
    const uint32_t lane = tid & 63u;
    const uint32_t wave = (uint32_t)__builtin_amdgcn_readfirstlane((int)(tid >> 6));
    for (uint64_t base = (uint64_t)blockIdx.x * kThreads; base < ntiles;
         base += (uint64_t)gridDim.x * kThreads) {
        if (tid == 0) nl = 0;
        __syncthreads();
        if (base + tid < ntiles) {
            const uint64_t ca = (base + tid) * tc;
            const uint64_t cb = (ca + tc < nchunks) ? ca + tc : nchunks;
            if (!tile_fits_lane(in, in_off, out_off, ca, cb)) lst[atomicAdd(&nl, 1u)] = tid;
        }
        __syncthreads();
        const uint32_t n = nl;
        for (uint32_t i = 0; i < n; i++) {
            const uint64_t t = base + lst[i];
            const uint64_t ca = t * tc;
            const uint64_t cb = (ca + tc < nchunks) ? ca + tc : nchunks;
            __syncthreads();
            sm.st.sel[tid] = kExpandTable.s[tid];
            unpack_tile_rest<SYNC, true>(sm, in, in_off, ca, cb, out, out_off, status, consumed,
                                         sync, tid, lane, wave);
        }
        __syncthreads();
    }
}

// The overflow tiles of the index-free split launch.  Index-free batches
// can overflow in bulk -- the resync block decode of config 4 hands over
// ~10 % of its tiles expanding past the tables (zero-run blocks) -- so the
// tiles are checked in windows of kOvfWindow (one lane each) spread over up to 8192
// workgroups, where unpack_ovf_kernel's windows of 256 on at most 1024
// workgroups left a few hundred of them serialising the overflow tiles
// (config 4 index-free: 4.3 ms in the overflow kernel; one workgroup per
// tile instead cost config 2 0.13 ms of empty workgroups).
#ifndef OVF_WINDOW
#define OVF_WINDOW 32
#endif
#ifndef OVF_GRID
#define OVF_GRID 2048
#endif
// (round 5, with the 8192-word sub-tiles: windows of 32 on 2048 workgroups,
// config 2 index-free 451 vs 465 us, config 4 1553 vs 1542; 64 / 1024: 446
// and 1566)
constexpr uint32_t kOvfWindow = OVF_WINDOW;
constexpr uint64_t kOvfGrid = OVF_GRID;
static_assert(kOvfWindow <= CAPNP_WAVE, "one lane per tile of the window");

template <bool SYNC>
__global__ void __launch_bounds__(kThreads, 4)
unpack_ovf_win_kernel(const uint8_t* __restrict__ in, const uint64_t* __restrict__ in_off,
                      uint64_t nchunks, uint32_t tc, uint64_t* __restrict__ out,
                      const uint64_t* __restrict__ out_off, int32_t* __restrict__ status,
                      uint64_t* __restrict__ consumed, const uint32_t* __restrict__ sync,
                      uint64_t ntiles) {
    __shared__ USmem sm;
    __shared__ uint64_t ovf_mask;
    const uint32_t tid = threadIdx.x;
    const uint32_t lane = tid & 63u;
    const uint32_t wave = (uint32_t)__builtin_amdgcn_readfirstlane((int)(tid >> 6));
    bool sel_ok = false;
    // (tiles dealt round robin: workgroup g checks tiles g, g + G, g + 2G, ...
    // kOvfWindow at a time, so a batch whose tiles all overflow -- long
    // chunks one per tile -- spreads them over the whole grid instead of
    // kOvfWindow consecutive ones per workgroup)
    const uint64_t G = gridDim.x;
    for (uint64_t base = blockIdx.x; base < ntiles; base += G * kOvfWindow) {
        if (wave == 0) {
            const uint64_t t = base + lane * G;
            bool o = false;
            if (lane < kOvfWindow && t < ntiles) {
                const uint64_t ca = t * tc;
                const uint64_t cb = (ca + tc < nchunks) ? ca + tc : nchunks;
                o = !tile_fits_lane(in, in_off, out_off, ca, cb);
            }
            const uint64_t m = ballot64(o);
            if (lane == 0) ovf_mask = m;
        }
        __syncthreads();
        uint64_t m = ovf_mask;
        while (m) {
            const uint64_t t = base + ctz64(m) * G;
            m &= m - 1;
            const uint64_t ca = t * tc;
            const uint64_t cb = (ca + tc < nchunks) ? ca + tc : nchunks;
            __syncthreads();  // the previous tile is done with the tables
#if UNPACK_PROF
            const uint64_t tov0 = __builtin_amdgcn_s_memrealtime();
#endif
            if (!sel_ok) {
                sm.st.sel[tid] = kExpandTable.s[tid];
                sel_ok = true;
            }
            unpack_tile_rest<SYNC, true>(sm, in, in_off, ca, cb, out, out_off, status, consumed,
                                         sync, tid, lane, wave);
            sel_ok = false;  // (the global path may overlay the selectors)
#if UNPACK_PROF
            __syncthreads();
            LUPROF_ADD(8, 1);
            LUPROF_ADD(9, __builtin_amdgcn_s_memrealtime() - tov0);
#endif
        }
        __syncthreads();  // ovf_mask is rewritten next window
    }
}

// ---------------------------------------------------------------------------
// Word tiles: batches of long chunks with the record sync index.
//
// Chunk tiles (unpack_kernel) hold whole chunks, so a chunk longer than a
// tile falls to the lane-per-chunk global walk.  Word tiles cut the batch's
// output words at every multiple of kWtWords instead (a multiple of
// kSyncWords, so the index has an entry at every cut): tile s decodes words
// [Wa, Wb) whatever chunks they belong to.
//   * A chunk that starts before Wa (the tile's first chunk, "partial
//     first") is entered through the entry at Wa: its walk starts at the
//     record that covers Wa, or after it when that record is a run that began
//     earlier (a literal run's words in the tile are listed up front).
//   * A chunk that continues past Wb ("partial last") is walked up to Wb,
//     where the last walker must reach the state the entry at Wb names.
//   * Every segment boundary inside the tile is checked as in the chunk
//     tiles, so the pieces of a chunk are exact when every check passes.
// Chunks inside the tile get their status here.  A partial chunk's pieces
// report to flags[] (bit 0: the tile's first chunk failed, bit 1: its last),
// and unpack_wt_finish gives the chunk its status from all of them: OK, or an
// exact serial decode of the chunk when any piece failed or a tile could not
// be planned (an unusable index entry, more than kStageChunks chunks, or
// bytes beyond the LDS table).  unpack_wt_plan (one thread per tile) resolves
// the tile's chunks and both ends from global memory up front.
constexpr uint32_t kWtWords = 1536;
static_assert(kWtWords % kSyncWords == 0 && kWtWords <= kMaxTileChunks * CAPNP_WAVE,
              "word tile size");
// Packed bytes a word tile stages: 8.125 per word, so that runs of literal
// words (8.03 bytes per word) fit, plus 2064 for a literal run that began up
// to 255 words before the tile (staged from its head); only adversarial
// tiles (up to 8.5 bytes per word) exceed it and decode serially.
// Tile size (config 4, unpack µs): 1024 words in the chunk tiles' tables
// (half of the 256 walkers had no segment) 730; in their own tables 1280 ->
// 649, 1536 -> 632 (7 workgroups per CU), 1792 -> 660, 2048 -> 677 (5 per
// CU).
constexpr uint32_t kWtBytes = (kWtWords * 65 / 8 + 2064 + 15) & ~15u;
#ifndef WT_SEL_ALU
#define WT_SEL_ALU 1
#endif
using WtStageSmem = StageSmemT<kWtWords, kWtBytes, !WT_SEL_ALU>;
// (with the selector table the LDS, 21.8 KB at 1536 words, allowed 7
// workgroups per CU; computed selectors (WT_SEL_ALU) leave 19.7 KB: 8)
// plan flags
constexpr uint32_t kWtPf = 1, kWtPl = 2, kWtFallback = 4;

// Diagnostics (capnp_unpack_wt_stats): [0] tiles planned as fallback, [1]
// pieces that failed in a tile, [2] chunks the finish kernel decoded serially.
__device__ unsigned long long g_wt_stats[4];

struct alignas(16) WtPlan {
    uint64_t ca, cb;  // chunks [ca, cb) overlap the tile
    uint64_t bs;      // first staged byte (global)
    uint32_t span;    // staged bytes from bs
    uint32_t flags;   // kWtPf | kWtPl | kWtFallback
    uint32_t q0, w0;  // segment 0 start: position after bs + 1, tile word
    uint32_t qB, wB;  // state at the tile end (partial last): position after bs + 1, tile word
    uint32_t pre;     // words of the first chunk before the tile
    uint32_t litp;    // partial first inside a literal run: position after bs of
    uint32_t litn;    // tile word 0's raw word, and the tile words the run covers
    uint32_t pad;
};
static_assert(sizeof(WtPlan) == 64, "plan record");

__device__ __forceinline__ void wt_bounds(uint64_t s, uint64_t g0, uint64_t wlo, uint64_t whi,
                                          uint64_t& Wa, uint64_t& Wb) {
    const uint64_t g = g0 + s;
    Wa = g * kWtWords > wlo ? g * kWtWords : wlo;
    Wb = (g + 1) * kWtWords < whi ? (g + 1) * kWtWords : whi;
}

// The record that covers global word W of chunk c, from its sync entry:
// false if the entry is unusable.  h = the record's first byte; for a run that
// started before W (d > 0): its end (qe), its word count and whether literal.
__device__ bool wt_entry(const uint8_t* __restrict__ in, const uint64_t* __restrict__ in_off,
                         const uint64_t* __restrict__ out_off, const uint32_t* __restrict__ sync,
                         uint64_t c, uint64_t W, uint64_t& h, uint32_t& d, uint64_t& qe,
                         uint32_t& cnt, bool& lit) {
    const uint64_t cs = in_off[c], ce = in_off[c + 1];
    const uint32_t e = sync[W / kSyncWords];
    const uint32_t off = e & 0xFFFFFFu;
    d = e >> 24;
    if (e == kSyncNone || ce < cs || off >= ce - cs || d > W - out_off[c]) return false;
    h = cs + off;
    cnt = 0;
    lit = false;
    qe = h;
    if (d == 0) return true;
    const uint32_t tag = in[h];
    if (tag != 0 && tag != 0xFF) return false;
    lit = tag == 0xFF;
    const uint64_t cpos = h + (lit ? 9u : 1u);
    if (cpos >= ce) return false;
    cnt = in[cpos];
    qe = cpos + 1 + (lit ? 8ull * cnt : 0ull);
    return cnt >= d && qe <= ce;
}

__global__ void __launch_bounds__(256)
unpack_wt_plan(const uint8_t* __restrict__ in, const uint64_t* __restrict__ in_off, uint64_t n,
               const uint64_t* __restrict__ out_off, const uint32_t* __restrict__ sync,
               uint64_t wlo, uint64_t whi, uint64_t g0, uint64_t ntiles,
               WtPlan* __restrict__ plan) {
    const uint64_t s = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (s >= ntiles) return;
    uint64_t Wa, Wb;
    wt_bounds(s, g0, wlo, whi, Wa, Wb);
    const uint32_t Wt = (uint32_t)(Wb - Wa);
    // first chunk: the one holding Wa, else the first to start at Wa
    uint64_t lo = 0, hi = n;
    while (lo < hi) {
        const uint64_t mid = (lo + hi) / 2;
        if (out_off[mid] < Wa) lo = mid + 1;
        else hi = mid;
    }
    const uint64_t ca = (lo > 0 && out_off[lo] > Wa) ? lo - 1 : lo;
    uint64_t cb = ca + 1;
    if (Wb == whi) cb = n;  // the last tile takes the empty chunks at the end
    else
        while (cb < n && out_off[cb] < Wb) cb++;
    WtPlan P = {};
    P.ca = ca;
    P.cb = cb;
    const bool pf = out_off[ca] < Wa, pl = Wb < whi && out_off[cb] > Wb;
    bool ok = cb - ca <= kStageChunks;
    uint64_t bs = in_off[ca], be = in_off[cb];
    P.q0 = 1;
    if (ok && pf) {
        uint64_t h, qe;
        uint32_t d, cnt;
        bool lit;
        ok = wt_entry(in, in_off, out_off, sync, ca, Wa, h, d, qe, cnt, lit);
        if (ok) {
            bs = h;
            P.pre = (uint32_t)(Wa - out_off[ca]);
            if (d) {  // a run from before the tile covers its first words
                P.q0 = (uint32_t)(qe - h) + 1u;
                P.w0 = cnt - d + 1u;
                if (lit) {
                    P.litp = 10u + 8u * (d - 1u);
                    P.litn = P.w0 < Wt ? P.w0 : Wt;
                }
            }
        }
    }
    if (ok && pl) {
        const uint64_t cl = cb - 1;
        uint64_t h, qe;
        uint32_t d, cnt;
        bool lit;
        ok = wt_entry(in, in_off, out_off, sync, cl, Wb, h, d, qe, cnt, lit) && h >= bs;
        if (ok) {
            if (d == 0) {
                P.qB = (uint32_t)(h - bs) + 1u;
                P.wB = Wt;
                be = h;
            } else {
                P.qB = (uint32_t)(qe - bs) + 1u;
                P.wB = Wt - d + 1u + cnt;
                be = lit ? h + 10 + 8ull * (d - 1) : h + 2;
            }
        }
    }
    const uint32_t off0 = (uint32_t)(reinterpret_cast<uintptr_t>(in + bs) & 15u);
    ok = ok && be >= bs && be - bs <= kWtBytes - off0;
    P.bs = bs;
    P.span = ok ? (uint32_t)(be - bs) : 0u;
    P.flags = (pf ? kWtPf : 0u) | (pl ? kWtPl : 0u) | (ok ? 0u : kWtFallback);
    plan[s] = P;
}

// Exact decode of one chunk by one lane from global memory, the reference's
// order of checks (as unpack_global): the word-tile path's fallback.
__device__ void serial_chunk(const uint8_t* __restrict__ in, uint64_t p0, uint64_t pe,
                             uint64_t* __restrict__ out, uint64_t n, int32_t& st,
                             uint64_t& used) {
    uint64_t p = p0, w = 0;
    st = ST_OK;
    if (n > 0 && p == pe) st = ST_FAILED_FILL;
    while (st == ST_OK && w < n) {
        if (p >= pe) { st = ST_PREMATURE; break; }
        const uint32_t tag = in[p];
        const uint32_t pop = __builtin_popcount(tag);
        if (p + 1 + pop > pe) { st = ST_PREMATURE; break; }
        uint64_t word = 0;
        for (uint32_t k = 0, r = 0; k < 8; k++)
            if (tag & (1u << k)) word |= (uint64_t)in[p + 1 + r++] << (8 * k);
        out[w++] = word;
        uint64_t q = p + 1 + pop;
        if (tag == 0 || tag == 0xFF) {
            if (q >= pe) { st = ST_PREMATURE; break; }
            const uint64_t cnt = in[q++];
            if (cnt > n - w) { st = ST_NOT_CLEAN; break; }
            if (tag == 0) {
                for (uint64_t i = 0; i < cnt; i++) out[w++] = 0;
            } else {
                if (pe - q < 8 * cnt) { st = ST_FAILED_FILL; break; }
                for (uint64_t i = 0; i < cnt; i++, q += 8) out[w++] = load_bytes(in, q, 8);
            }
        }
        p = q;
    }
    used = st == ST_OK ? p - p0 : (st == ST_NOT_CLEAN ? 0 : pe - p0);
}

__device__ __forceinline__ void serial_chunk_at(const uint8_t* __restrict__ in,
                                                const uint64_t* __restrict__ in_off,
                                                uint64_t* __restrict__ out,
                                                const uint64_t* __restrict__ out_off,
                                                int32_t* __restrict__ status,
                                                uint64_t* __restrict__ consumed, uint64_t c) {
    int32_t st;
    uint64_t used;
    const uint64_t ow = out_off[c];
    serial_chunk(in, in_off[c], in_off[c + 1], out + ow, out_off[c + 1] - ow, st, used);
    status[c] = st;
    if (consumed) consumed[c] = used;
}

__global__ void __launch_bounds__(kThreads, WT_SEL_ALU ? 8 : 7)
unpack_wt_kernel(const uint8_t* __restrict__ in, const uint64_t* __restrict__ in_off,
                 uint64_t* __restrict__ out, const uint64_t* __restrict__ out_off,
                 int32_t* __restrict__ status, uint64_t* __restrict__ consumed,
                 const uint32_t* __restrict__ sync, const WtPlan* __restrict__ plan,
                 uint32_t* __restrict__ flags, uint64_t wlo, uint64_t whi, uint64_t g0) {
    __shared__ WtStageSmem S;
    const uint32_t tid = threadIdx.x;
    const uint64_t s = blockIdx.x;
    uint64_t Wa, Wb;
    wt_bounds(s, g0, wlo, whi, Wa, Wb);
    const uint32_t Wt = (uint32_t)(Wb - Wa);
    const WtPlan* Pp = plan + s;
    const uint64_t ca = uniform64(Pp->ca), cb = uniform64(Pp->cb);
    const uint32_t pf_ = uniform(Pp->flags);
    const bool pf = pf_ & kWtPf, pl = pf_ & kWtPl;
    if (pf_ & kWtFallback) {  // exact serial decode of the chunks inside the tile
        for (uint64_t c = ca + tid; c < cb; c += kThreads)
            if (!((pf && c == ca) || (pl && c + 1 == cb)))
                serial_chunk_at(in, in_off, out, out_off, status, consumed, c);
        if (tid == 0) {
            flags[s] = 3u;
            atomicAdd(&g_wt_stats[0], 1ull);
        }
        return;
    }
    const uint32_t nc = (uint32_t)(cb - ca);
    const uint64_t Bs = uniform64(Pp->bs);
    const uint32_t off0 = (uint32_t)(reinterpret_cast<uintptr_t>(in + Bs) & 15u);
    const uint32_t nbytes = uniform(Pp->span) + off0;
    // segments as in the chunk tiles: [0, kSyncWords kf - Wa), then blocks
    // at global multiples of kSyncWords (Wa is one except for a batch that
    // starts unaligned, whose first tile starts a chunk)
    const uint64_t kf = Wa / kSyncWords + 1;
    const uint32_t nseg = 1u + (uint32_t)((Wb - 1) / kSyncWords + 1 - kf);
    const uint32_t r0 = (uint32_t)(Wa % kSyncWords);
    // every staging load in one round trip (as unpack_staged_at): the chunk
    // tables and sync entries by buffer loads ahead of the byte loads, the
    // selector entry written after them
    {
        constexpr uint32_t kLoads = (kWtBytes + 15 + 16 * kThreads - 1) / (16 * kThreads);
        const uint64_t selv = WT_SEL_ALU ? 0 : kExpandTable.s[tid];
        const __amdgpu_buffer_rsrc_t ors = __builtin_amdgcn_make_buffer_rsrc(
            const_cast<uint64_t*>(out_off + ca), 0, (int)((nc + 1) * 8), 0x00020000);
        const __amdgpu_buffer_rsrc_t irs = __builtin_amdgcn_make_buffer_rsrc(
            const_cast<uint64_t*>(in_off + ca), 0, (int)((nc + 1) * 8), 0x00020000);
        const auto wov = __builtin_amdgcn_raw_buffer_load_b64(ors, (int)(tid * 8u), 0, 0);
        const auto wnv = __builtin_amdgcn_raw_buffer_load_b64(ors, (int)(tid * 8u + 8u), 0, 0);
        const uint32_t t_p = __builtin_amdgcn_raw_buffer_load_b32(irs, (int)(tid * 8u), 0, 0);
        const __amdgpu_buffer_rsrc_t srs = __builtin_amdgcn_make_buffer_rsrc(
            const_cast<uint32_t*>(sync + (kf - 1)), 0, (int)(nseg * 4), 0x00020000);
        const uint32_t e_a = __builtin_amdgcn_raw_buffer_load_b32(srs, (int)(tid * 4u), 0, 0);
        const uint32_t e_b = __builtin_amdgcn_raw_buffer_load_b32(srs, (int)((tid + kThreads) * 4u), 0, 0);
        const uint4* src = reinterpret_cast<const uint4*>(in + Bs - off0);
        uint4* dst = reinterpret_cast<uint4*>(S.bytes);
        const uint32_t nblk = (nbytes + 15) / 16;
        uint4 r[kLoads];
#pragma unroll
        for (uint32_t k = 0; k < kLoads; k++) {
            const uint32_t idx = tid + k * kThreads;
            r[k] = nblk ? src[idx < nblk ? idx : nblk - 1] : make_uint4(0, 0, 0, 0);
        }
        // descriptors: none, or the raw words of a literal run carried in
        const uint32_t litn = uniform(Pp->litn), litp = uniform(Pp->litp) + off0;
        if (litn == 0) {
            uint4* dd = reinterpret_cast<uint4*>(S.dpos);
            const uint4 none = make_uint4(~0u, ~0u, ~0u, ~0u);
            for (uint32_t k = tid; k < (Wt + 7) / 8; k += kThreads) dd[k] = none;
        } else {
            for (uint32_t i = tid; i < ((Wt + 7) & ~7u); i += kThreads)
                S.dpos[i] = i < litn ? (uint16_t)(kRaw | (litp + 8 * i)) : kNone;
        }
        if (!WT_SEL_ALU) S.sel[tid] = selv;
        if (tid <= nc) {
            const uint64_t wo = ((uint64_t)wov[1] << 32) | wov[0];
            const uint32_t wa = wo < Wa ? 0u : (uint32_t)(wo - Wa);
            S.cw[tid] = wa;  // (the end of a partial last chunk lies past Wt)
            S.cp[tid] = t_p - (uint32_t)Bs + off0;  // (wraps for a partial first)
            if (tid < nc) {
                const uint64_t wn = ((uint64_t)wnv[1] << 32) | wnv[0];
                const uint32_t wz = wn - Wa < Wt ? (uint32_t)(wn - Wa) : Wt;
                if (wz > wa) {
                    const uint32_t blo = wa == 0 ? 0u : (wa + r0 + kSyncWords - 1) / kSyncWords;
                    const uint32_t bhi = (wz + r0 + kSyncWords - 1) / kSyncWords;
                    for (uint32_t bb = blo; bb < bhi; bb++) S.segc[bb] = (uint8_t)tid;
                }
            }
        }
        if (tid >= 1 && tid < nseg) S.ent[tid] = e_a;
        if (tid + kThreads < nseg) S.ent[tid + kThreads] = e_b;
        if (tid < kStageChunks) S.badc[tid] = 0;
        if (tid == 0) {
            S.wt_q0 = uniform(Pp->q0) + off0;
            S.wt_w0 = uniform(Pp->w0);
            S.wt_qB = uniform(Pp->qB) + off0;
            S.wt_wB = uniform(Pp->wB);
            S.wt_pre = uniform(Pp->pre);
            S.wt_pl = pl ? 1u : 0u;
        }
#pragma unroll
        for (uint32_t k = 0; k < kLoads; k++)
            if (tid + k * kThreads < nblk) dst[tid + k * kThreads] = r[k];
    }
    __syncthreads();
    bool marked = false;
    for (uint32_t b = tid; b < nseg; b += kThreads) {
        const uint32_t sb = b == 0 ? 0u : (uint32_t)((kf + b - 1) * kSyncWords - Wa);
        const bool last = b + 1 == nseg;
        const uint32_t eb = last ? Wt : (uint32_t)((kf + b) * kSyncWords - Wa);
        marked |= walk_segment<WtStageSmem, true>(S, nc, b, sb, eb, last, Wt);
    }
    const bool anybad = __syncthreads_or(marked);
    if (tid < nc) {
        const uint64_t c = ca + tid;
        const bool part = (pf && tid == 0) || (pl && tid + 1 == nc);
        if (!part) {
            if (anybad && S.badc[tid]) {  // exact serial walk of the chunk
                const uint32_t wa = S.cw[tid], wz = S.cw[tid + 1];
                for (uint32_t i = wa; i < wz; i++) S.dpos[i] = kNone;
                int32_t st;
                uint32_t used;
                walk_chunk(S, S.cp[tid], S.cp[tid + 1], wa, wz - wa, st, used);
                status[c] = st;
                if (consumed) consumed[c] = used;
            } else {
                status[c] = ST_OK;
                if (consumed)
                    consumed[c] = S.cw[tid + 1] > S.cw[tid] ? S.cp[tid + 1] - S.cp[tid] : 0u;
            }
        }
    }
    if (tid == 0) {
        const uint32_t f = ((pf && S.badc[0]) ? 1u : 0u) | ((pl && S.badc[nc - 1]) ? 2u : 0u);
        flags[s] = f;
        if (f) atomicAdd(&g_wt_stats[1], 1ull);
    }
    if (anybad) __syncthreads();
    for (uint32_t i = tid; i < Wt; i += kThreads)
        out[Wa + i] = expand_desc<WT_SEL_ALU>(S.bytes, S.sel, S.dpos[i]);
}

// Status of every chunk that spans tiles, in the tile where it ends.
__global__ void __launch_bounds__(256)
unpack_wt_finish(const uint8_t* __restrict__ in, const uint64_t* __restrict__ in_off,
                 uint64_t* __restrict__ out, const uint64_t* __restrict__ out_off,
                 int32_t* __restrict__ status, uint64_t* __restrict__ consumed,
                 const WtPlan* __restrict__ plan, const uint32_t* __restrict__ flags,
                 uint64_t wlo, uint64_t whi, uint64_t g0, uint64_t ntiles) {
    const uint64_t s = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (s >= ntiles || !(plan[s].flags & kWtPf)) return;
    uint64_t Wa, Wb;
    wt_bounds(s, g0, wlo, whi, Wa, Wb);
    const uint64_t c = plan[s].ca;
    if (out_off[c + 1] > Wb) return;  // it goes on: the tile where it ends finishes it
    const uint64_t s0 = out_off[c] / kWtWords - g0;  // the tile of its first word
    uint32_t bad = flags[s] & 1u;
    for (uint64_t u = s - 1; u > s0; u--) bad |= flags[u];  // tiles it covers
    bad |= flags[s0] >> 1;
    if (!bad) {
        status[c] = ST_OK;
        if (consumed) consumed[c] = in_off[c + 1] - in_off[c];
    } else {
        atomicAdd(&g_wt_stats[2], 1ull);
        serial_chunk_at(in, in_off, out, out_off, status, consumed, c);
    }
}

// ---------------------------------------------------------------------------
// A short read unit already staged in the long-unit buffer (read_message's
// one-launch kernel): wave 0 decodes it alone with the in-tile segment walk's
// rules (spec_seg_tile) on 64 segments -- the spec walk with its lead-in, the
// meet / repair rounds by shuffles, the word scan, the segment holding word n
// walking to it with every check -- and writes the descriptors; then the
// four waves expand.  unpack_long's workgroup-wide scans and barriers cost
// about a microsecond a round at these sizes (a 1 KiB body: 6.6 us of its
// phases).  B = the unit's byte 0 (LDS position mis), L = the bytes the walks
// may use (staged, <= kSmallBytes), n = the words.  Returns false with
// nothing written to `out` when the unit does not check out within L bytes
// (malformed, truncated, or longer than L): the caller then takes
// unpack_long, which gives the exact status.
#ifndef UNPACK_SMALL_BYTES
// (r06n, DPP scans, before unpack_mid: 5120, a 4.4 KB body 24.0 vs 26.0 us
// on unpack_long; with unpack_mid, 2048: 500-1000-word reads 14.3-16.3 us
// against 16.4-20.6 at 5120, profiles/r06q_small_ab.txt)
#define UNPACK_SMALL_BYTES 2048
#endif
constexpr uint32_t kSmallBytes = UNPACK_SMALL_BYTES;
#ifndef UNPACK_SMALL_LEAD
#define UNPACK_SMALL_LEAD 96  // (48 as spec_seg_tile's kSegOverlap until r06q: a 1 KiB read 13.8 -> 12.4-12.6 us)
#endif
constexpr uint32_t kSmallLead = UNPACK_SMALL_LEAD;

__device__ bool unpack_small(LongSmem& S, uint32_t mis, uint32_t L, uint32_t n,
                             uint64_t* __restrict__ out, uint32_t tid, uint32_t lane,
                             uint32_t wave, uint32_t& used) {
    const uint8_t* B = S.bytes + mis;
#if SVC_PROF
    const uint64_t tq0 = __builtin_amdgcn_s_memrealtime();
#endif
    S.sel[tid] = kExpandTable.s[tid];
    {
        uint4* d4 = reinterpret_cast<uint4*>(S.dpos);
        const uint4 none = make_uint4(~0u, ~0u, ~0u, ~0u);
        for (uint32_t k = tid; k < (n + 7) / 8; k += kThreads) d4[k] = none;
    }
    __syncthreads();
#if SVC_PROF
    const uint64_t tq1 = __builtin_amdgcn_s_memrealtime();
#endif
    if (wave == 0) {
        const uint32_t j = lane;
        const uint32_t sb = (uint32_t)(((uint64_t)L * j) >> 6);
        const uint32_t se = (uint32_t)(((uint64_t)L * (j + 1u)) >> 6);
        // spec walk from kSmallLead bytes before the segment (lane 0: byte 0)
        uint32_t p = j == 0 ? 0u : (sb > kSmallLead ? sb - kSmallLead : 0u), w = 0;
        while (p < sb) seg_hop(B, p, w);
        const uint32_t f = p, wf = w;
        while (p < se) seg_hop(B, p, w);
#if SVC_PROF
        const uint64_t tw0 = __builtin_amdgcn_s_memrealtime();
#endif
        const bool serr = p > L;
        const uint32_t xs = serr ? 0u : p, ws = w - wf;
        // (a spec walk that found no record start in its segment owns no exit)
        const uint32_t xsp = (serr || f >= se) ? 0u : xs;
        // meet / repair rounds (unpack_long's rules on one wave of 64
        // segments): each round settles at least one more segment
        uint32_t own = xsp, x = xsp, wd = ws;
        bool err = j == 0 && serr;
        uint32_t e_used = j == 0 ? 0u : ~0u;
        // (the wave scans by DPP: VALU ops, where __shfl_up's ds_bpermute is an
        // LDS round trip each -- the rounds are chains of them)
        x = wave_max_scan(x);
        bool ok = true;
#if SVC_PROF
        uint32_t n_rounds = 0;
#endif
        for (uint32_t round = 0;; round++) {
#if SVC_PROF
            n_rounds++;
#endif
            const uint32_t e = wave_shr1(x);  // (0 in lane 0)
            const bool need = e != e_used;
            if (ballot64(need) == 0) break;
            if (round > CAPNP_WAVE + 1) {  // (not reached: lane i is settled after round i + 1)
                ok = false;
                break;
            }
            if (need) {
                e_used = e;
                if (e < sb || e == f) {
                    // (an entry below the segment -- a predecessor not settled
                    // yet -- lets the spec walk stand in: a far garbage exit
                    // of a missed spec walk then cannot send its successors
                    // walking from far back once it is repaired)
                    own = xsp;
                    wd = ws;
                    err = serr;
                } else {
                    // from the entry with the spec chain kept in step (unpack_long's
                    // meet rule): where they meet, the rest is the spec walk's, so
                    // a repair is short and the successors' entries stand
                    uint32_t pt = e, wt = 0, ps = f, wsp = 0;
                    bool met = false;
                    while (pt < se) {
                        while (ps < pt && ps < se) seg_hop(B, ps, wsp);
                        if (ps == pt) {
                            met = true;
                            break;
                        }
                        seg_hop(B, pt, wt);
                    }
                    if (met) {
                        own = xsp;
                        wd = wt + ws - wsp;
                        err = serr;
                    } else {
                        err = pt > L;
                        own = (err || e >= se) ? 0u : pt;
                        wd = wt;
                    }
                }
            }
            x = wave_max_scan(own);
        }
        const uint32_t e = e_used;
#if SVC_PROF
        const uint64_t tw1 = __builtin_amdgcn_s_memrealtime();
#endif
        // words: the segment holding word n walks to it with every check
        const uint32_t incl = wave_sum_scan(wd);
        const uint32_t base = incl - wd;
        const uint64_t hold = ballot64(wd > 0 && base < n && n <= incl);
        const uint32_t ts = hold ? (uint32_t)__builtin_ctzll(hold) : CAPNP_WAVE;
        ok = ok && ts < CAPNP_WAVE && ballot64(err && j <= ts) == 0;
        uint32_t q = e, wq = base;
        bool fine = true;
        if (ok && j == ts) {
            while (wq < n) {
                uint32_t tag, b1, b9;
                rec_bytes(B, q + 1u, tag, b1, b9);
                const bool isz = tag == 0, isf = tag == 0xFF;
                const uint32_t cnt = isz ? b1 : (isf ? b9 : 0u);
                const uint32_t qe = q + 1u + __builtin_popcount(tag) + ((isz || isf) ? 1u : 0u) +
                                    (isf ? 8u * cnt : 0u);
                const uint32_t wn = wq + 1u + cnt;
                if (qe > L || wn > n) {
                    fine = false;
                    break;
                }
                q = qe;
                wq = wn;
            }
        }
        ok = ok && ballot64(j == ts && !fine) == 0;
#if SVC_PROF
        const uint64_t tw2 = __builtin_amdgcn_s_memrealtime();
#endif
        used = (uint32_t)__builtin_amdgcn_readlane((int)q, (int)(ts < CAPNP_WAVE ? ts : 0u));
        // descriptors of the records from each entry (to word n in the last)
        if (ok && j <= ts) {
            uint32_t r = e, wr = base;
            const uint32_t wlim = j == ts ? n : incl;
            while (wr < wlim) {
                uint32_t tag, b1, b9;
                rec_bytes(B, r + 1u, tag, b1, b9);
                const bool isz = tag == 0, isf = tag == 0xFF;
                const uint32_t cnt = isz ? b1 : (isf ? b9 : 0u);
                const uint32_t lp = r + mis;  // (LDS position of the tag)
                S.dpos[wr] = (uint16_t)lp;
                if (isf)
                    for (uint32_t i = 0; i < cnt; i++)
                        S.dpos[wr + 1u + i] = (uint16_t)(kRaw | (lp + 10u + 8u * i));
                wr += 1u + cnt;
                r += 1u + __builtin_popcount(tag) + ((isz || isf) ? 1u : 0u) + (isf ? 8u * cnt : 0u);
            }
        }
        if (lane == 0) S.misc[0] = ok ? 1u : 0u;
#if SVC_PROF
        wave_lds_sync();
        const uint64_t tw3 = __builtin_amdgcn_s_memrealtime();
        if (lane == 0) {
            atomicAdd(&g_svc_prof[16], (unsigned long long)(tw0 - tq1));
            atomicAdd(&g_svc_prof[17], (unsigned long long)(tw1 - tw0));
            atomicAdd(&g_svc_prof[18], (unsigned long long)(tw2 - tw1));
            atomicAdd(&g_svc_prof[19], (unsigned long long)(tw3 - tw2));
            atomicAdd(&g_svc_prof[20], (unsigned long long)n_rounds);
        }
#endif
    }
    __syncthreads();
#if SVC_PROF
    const uint64_t tq2 = __builtin_amdgcn_s_memrealtime();
#endif
    if (S.misc[0] == 0) return false;
    for (uint32_t i = tid; i < n; i += kThreads) out[i] = expand_desc(S.bytes, S.sel, S.dpos[i]);
#if SVC_PROF
    __syncthreads();
    if (tid == 0) {
        atomicAdd(&g_svc_prof[9], (unsigned long long)(tq1 - tq0));
        atomicAdd(&g_svc_prof[10], (unsigned long long)(tq2 - tq1));
        atomicAdd(&g_svc_prof[11], (unsigned long long)(__builtin_amdgcn_s_memrealtime() - tq2));
        atomicAdd(&g_svc_prof[12], 1ull);
    }
#endif
    return true;
}

// ---------------------------------------------------------------------------
// A mid-size read unit staged in the long-unit buffer (bodies of more than
// kSmallBytes, up to kMidBytes, 2-18 KB): unpack_small's walk on all four waves, 256
// segments, each wave settling its 64 by DPP rounds of its own; the waves
// then meet once through LDS: wave w assumed its first segment's spec start
// as its entry, and is re-run from the true one (the running maximum of the
// earlier waves' exits) when that differs, until no entry changes.
// unpack_long's workgroup-wide rounds took two barriers each (a 1500-word
// body: 3 rounds, 5.7 of its 12.3 us; profiles/r06m_luprof_percall.txt).
// Returns false with nothing written to `out` when the unit does not check
// out (the caller then takes unpack_long, which gives the exact status).
#ifndef UNPACK_MID_BYTES
#define UNPACK_MID_BYTES 18432  // (the staged prefix's limit; a 4 Ki-word read 40.8 -> 30.7 us, r06p)
#endif
constexpr uint32_t kMidBytes = UNPACK_MID_BYTES;
#ifndef UNPACK_MID_LEAD
// spec walk lead-in (bytes) of the mid-size decode: 48 -> 96 took a
// 1500-word read 21.7 -> 17.2-17.9 us and the carsales pair 34.9 -> 32.1-33.5
// (profiles/r06q_midlead_ab*.txt; 128-160 are as good on carsales, worse on
// 2200- and 3000-word bodies; 320 worse everywhere)
#define UNPACK_MID_LEAD 96
#endif
constexpr uint32_t kMidLead = UNPACK_MID_LEAD;
static_assert(kMidBytes + 32 <= kLuStage, "a mid-size unit lies in the staged bytes");

__device__ bool unpack_mid(LongSmem& S, uint32_t mis, uint32_t L, uint32_t n,
                           uint64_t* __restrict__ out, uint32_t tid, uint32_t lane,
                           uint32_t wave, uint32_t& used) {
    __shared__ uint32_t wx[2][kWaves];   // each wave's last exit (the running max), per pass
    __shared__ uint32_t we[2][kWaves];   // the entry each wave assumed, per pass
    __shared__ uint32_t wok[2][kWaves];  // the wave's rounds settled
    __shared__ uint32_t wtot[kWaves];    // each wave's words
    __shared__ uint32_t wts[kWaves];     // the wave's segment holding word n (or kThreads)
    __shared__ uint32_t wbad[kWaves];
    const uint8_t* B = S.bytes + mis;
#if SVC_PROF
    const uint64_t tm0 = __builtin_amdgcn_s_memrealtime();
#endif
    S.sel[tid] = kExpandTable.s[tid];
    {
        uint4* d4 = reinterpret_cast<uint4*>(S.dpos);
        const uint4 none = make_uint4(~0u, ~0u, ~0u, ~0u);
        for (uint32_t k = tid; k < (n + 7) / 8; k += kThreads) d4[k] = none;
    }
    const uint32_t j = tid;
    const uint32_t sb = (uint32_t)(((uint64_t)L * j) / kThreads);
    const uint32_t se = (uint32_t)(((uint64_t)L * (j + 1u)) / kThreads);
    // spec walk from kMidLead bytes before the segment (segment 0: byte 0)
    uint32_t p = j == 0 ? 0u : (sb > kMidLead ? sb - kMidLead : 0u), w = 0;
    while (p < sb) seg_hop(B, p, w);
    const uint32_t f = p, wf = w;
    while (p < se) seg_hop(B, p, w);
    const bool serr = p > L;
    const uint32_t xs = serr ? 0u : p, ws = w - wf;
    const uint32_t xsp = (serr || f >= se) ? 0u : xs;
#if SVC_PROF
    const uint64_t tm1 = __builtin_amdgcn_s_memrealtime();
    uint32_t n_pass = 0;
#endif
    // the wave's entry: wave 0's is byte 0; the others assume their first
    // segment's spec start until the earlier waves have settled
    uint32_t E = wave == 0 ? 0u : (uint32_t)__builtin_amdgcn_readfirstlane((int)f);
    uint32_t own = xsp, wd = ws;
    bool err = j == 0 && serr;
    uint32_t e_used = ~0u, x = 0;
    bool ok = true, run = true;
    for (uint32_t pass = 0;; pass++) {
        if (run) {
            // rounds within the wave to its fixed point for entry E
            x = wave_max_scan(own);
            for (uint32_t round = 0;; round++) {
                // (the wave's entry E bounds every lane's: a record of an
                // earlier wave may cover this wave's first segments.  No
                // lane-dependent select around the DPP shift: the compiler
                // sank it into the select's branch, and lane 1 then read a
                // disabled lane 0 as 0 -- one word short, r06p)
                const uint32_t e = max(E, wave_shr1(x));  // (wave_shr1: 0 in lane 0)
                const bool need = e != e_used;
                if (ballot64(need) == 0) break;
                if (round > CAPNP_WAVE + 1) {  // (not reached: lane i is settled after round i + 1)
                    ok = false;
                    break;
                }
                if (need) {
                    e_used = e;
                    if (e < sb || e == f) {
                        own = xsp;
                        wd = ws;
                        err = serr;
                    } else {
                        uint32_t pt = e, wt = 0, ps = f, wsp = 0;
                        bool met = false;
                        while (pt < se) {
                            while (ps < pt && ps < se) seg_hop(B, ps, wsp);
                            if (ps == pt) {
                                met = true;
                                break;
                            }
                            seg_hop(B, pt, wt);
                        }
                        if (met) {
                            own = xsp;
                            wd = wt + ws - wsp;
                            err = serr;
                        } else {
                            err = pt > L;
                            own = (err || e >= se) ? 0u : pt;
                            wd = wt;
                        }
                    }
                }
                x = wave_max_scan(own);
            }
        }
        // the waves meet: wave v's true entry is the largest exit before it
        const uint32_t b = pass & 1u;
#if SVC_PROF
        n_pass++;
#endif
        if (lane == CAPNP_WAVE - 1) {
            wx[b][wave] = max(x, E);
            we[b][wave] = E;
            wok[b][wave] = ok ? 1u : 0u;
        }
        __syncthreads();
        // (every wave reads the same records: the decisions below are the
        // workgroup's, so the waves meet at the same barriers)
        bool any = false;
        uint32_t mine = E, m = 0, allok = 1;
#pragma unroll
        for (uint32_t v = 0; v < (uint32_t)kWaves; v++) {
            if (v > 0 && we[b][v] != m) any = true;
            if (v == wave) mine = v == 0 ? 0u : m;
            m = max(m, wx[b][v]);
            allok &= wok[b][v];
        }
        ok = allok != 0 && pass <= (uint32_t)kWaves;  // (each pass settles at least one more wave)
        if (!any || !ok) break;
        run = mine != E;
        E = mine;
    }
#if SVC_PROF
    const uint64_t tm2 = __builtin_amdgcn_s_memrealtime();
#endif
    // words: the waves' totals place each segment; the segment holding word
    // n walks to it with every check
    const uint32_t incl_w = wave_sum_scan(wd);
    if (lane == CAPNP_WAVE - 1) wtot[wave] = incl_w;
    __syncthreads();
    uint32_t before = 0;
#pragma unroll
    for (uint32_t v = 0; v < (uint32_t)kWaves; v++) before += v < wave ? wtot[v] : 0u;
    const uint32_t incl = before + incl_w, base = incl - wd;
    const uint64_t hold = ballot64(wd > 0 && base < n && n <= incl);
    if (lane == 0) wts[wave] = hold ? wave * CAPNP_WAVE + (uint32_t)__builtin_ctzll(hold) : kThreads;
    __syncthreads();
    uint32_t ts = kThreads;
#pragma unroll
    for (uint32_t v = 0; v < (uint32_t)kWaves; v++) ts = min(ts, wts[v]);
    const bool wave_bad = ballot64(err && j <= ts) != 0;  // (the ballot before the lane-0 store)
    if (lane == 0) wbad[wave] = wave_bad ? 1u : 0u;
    uint32_t q = e_used, wq = base;
    bool fine = true;
    if (ok && ts < kThreads && j == ts) {
        while (wq < n) {
            uint32_t tag, b1, b9;
            rec_bytes(B, q + 1u, tag, b1, b9);
            const bool isz = tag == 0, isf = tag == 0xFF;
            const uint32_t cnt = isz ? b1 : (isf ? b9 : 0u);
            const uint32_t qe = q + 1u + __builtin_popcount(tag) + ((isz || isf) ? 1u : 0u) +
                                (isf ? 8u * cnt : 0u);
            const uint32_t wn = wq + 1u + cnt;
            if (qe > L || wn > n) {
                fine = false;
                break;
            }
            q = qe;
            wq = wn;
        }
        S.misc[0] = fine ? 1u : 0u;
        S.misc[1] = q;
    }
    __syncthreads();
    bool bad = !ok || ts >= kThreads || S.misc[0] == 0;
#pragma unroll
    for (uint32_t v = 0; v < (uint32_t)kWaves; v++) bad |= wbad[v] != 0;
#ifdef MID_DEBUG
    if (tid == 0) printf("MID bad %d ts %u misc0 %u\n", (int)bad, ts, S.misc[0]);
#endif
    if (__builtin_amdgcn_readfirstlane((int)bad)) return false;  // (uniform: LDS after the barrier)
    used = S.misc[1];
#if SVC_PROF
    const uint64_t tm3 = __builtin_amdgcn_s_memrealtime();
#endif
#ifdef MID_DEBUG
    if (lane == 0) printf("MID wave %u E %u x63 %u tot %u ts %u L %u n %u\n", wave, E,
                          (uint32_t)__builtin_amdgcn_readlane((int)x, 63), wtot[wave], ts, L, n);
    if (j == ts) printf("MID ts %u e_used %u base %u wd %u used %u\n", ts, e_used, base, wd, S.misc[1]);
    if (err) printf("MID err lane %u e_used %u own %u wd %u\n", j, e_used, own, wd);
    if (lane == 0) printf("MID wbad %u %u %u %u ok %d\n", wbad[0], wbad[1], wbad[2], wbad[3], (int)ok);
#endif
    // descriptors of the records from each entry (to word n in the last)
    if (j <= ts) {
        uint32_t r = e_used, wr = base;
        const uint32_t wlim = j == ts ? n : incl;
        while (wr < wlim) {
            uint32_t tag, b1, b9;
            rec_bytes(B, r + 1u, tag, b1, b9);
            const bool isz = tag == 0, isf = tag == 0xFF;
            const uint32_t cnt = isz ? b1 : (isf ? b9 : 0u);
            const uint32_t lp = r + mis;  // (LDS position of the tag)
            S.dpos[wr] = (uint16_t)lp;
            if (isf)
                for (uint32_t i = 0; i < cnt; i++)
                    S.dpos[wr + 1u + i] = (uint16_t)(kRaw | (lp + 10u + 8u * i));
            wr += 1u + cnt;
            r += 1u + __builtin_popcount(tag) + ((isz || isf) ? 1u : 0u) + (isf ? 8u * cnt : 0u);
        }
    }
    __syncthreads();
#if SVC_PROF
    const uint64_t tm4 = __builtin_amdgcn_s_memrealtime();
#endif
    for (uint32_t i = tid; i < n; i += kThreads) out[i] = expand_desc(S.bytes, S.sel, S.dpos[i]);
#if SVC_PROF
    __syncthreads();
    if (tid == 0) {  // (slots 13-15, 21-23: spec, passes, words, descriptors, expand, count)
        atomicAdd(&g_svc_prof[13], (unsigned long long)(tm1 - tm0));
        atomicAdd(&g_svc_prof[14], (unsigned long long)(tm2 - tm1));
        atomicAdd(&g_svc_prof[15], (unsigned long long)(tm3 - tm2));
        atomicAdd(&g_svc_prof[21], (unsigned long long)(tm4 - tm3));
        atomicAdd(&g_svc_prof[22], (unsigned long long)(__builtin_amdgcn_s_memrealtime() - tm4));
        atomicAdd(&g_svc_prof[23], (unsigned long long)n_pass + (1ull << 32));
    }
#endif
    return true;
}

// ---------------------------------------------------------------------------
// One read_message call in one launch (the drop-in at the reference's call
// granularity: serialize_packed::read_message / try_read_message /
// read_message_no_alloc once per message, serialize_packed.rs:233-291,
// benchmark.rs:207-259).  The input prefix sits in pinned host memory and the
// kernel reads it there: the first kMsgPre bytes (more than any segment
// table's read units take, <= 10 bytes x 257 words) come into LDS in one
// round trip, lane 0 reads and checks the table from them (frame.h, the
// frame kernel's code), and the workgroup decodes the body unit with the
// long-unit decode (unpack_long) straight from the host bytes into the
// caller's pinned words.  The frame result and the body's status and
// consumed count are written to pinned memory too: the host waits once.
constexpr uint32_t kMsgPre = 4096;
static_assert(kMsgPre == 16 * kThreads, "one 16-byte load per thread");

struct MsgReadSmem {
    alignas(16) FrameResult fr;
    uint64_t offs[4];  // the body unit: packed range, words
    int32_t st;
    uint64_t used;
};

__device__ __forceinline__ void msg_read_body(USmem& sm, MsgReadSmem& M, const uint8_t* in,
                                              uint64_t in_len, uint32_t no_alloc, uint32_t try_mode,
                                              uint64_t limit, uint32_t has_limit,
                                              uint64_t buffer_len, uint64_t body_cap,
                                              FrameResult* fr_out, uint64_t* words, uint64_t* res,
                                              uint32_t* flag, uint32_t seq) {
    const uint32_t tid = threadIdx.x;
    const uint32_t lane = tid & 63u;
    const uint32_t wave = (uint32_t)__builtin_amdgcn_readfirstlane((int)(tid >> 6));
    const uint64_t npre = in_len < kMsgPre ? in_len : kMsgPre;
    // The input's first kLuStage - 16 bytes come into the long-unit decode's
    // staging buffer in one round trip (16-byte loads of whole vectors: the
    // host buffer is 16-byte aligned and padded; zeros past the input): the
    // table is read from there, and a body inside them is decoded without
    // loading its window again.
    constexpr uint32_t kPreVec = kLuStage / 16 - 1;
    const uint32_t pre = (uint32_t)(in_len < 16ull * kPreVec ? in_len : 16ull * kPreVec);
    {
        // (LDS DMA for whole 64-vector groups, as unpack_long's windows: every
        // load in flight at once.  The plain loop had waited for each
        // iteration's loads before the next: one PCIe round trip per 4 KiB)
        const uint4* src = reinterpret_cast<const uint4*>(in);
        uint4* dst = reinterpret_cast<uint4*>(sm.lu.bytes);
        const uint32_t nblk = (pre + 15) / 16;
        constexpr uint32_t kVec = kLuStage / 16;
        for (uint32_t i0 = wave * CAPNP_WAVE; i0 < kVec; i0 += kThreads) {
            const uint32_t i = i0 + lane;
            if (i0 + CAPNP_WAVE <= nblk) {
                __builtin_amdgcn_global_load_lds(
                    (const __attribute__((address_space(1))) void*)(src + i),
                    (__attribute__((address_space(3))) void*)(sm.lu.bytes + 16u * i0), 16, 0, 0);
            } else if (i < kVec) {
                dst[i] = i < nblk ? src[i] : make_uint4(0, 0, 0, 0);
            }
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's bytes are in
    }
    __syncthreads();
#if SVC_PROF
    const uint64_t tp0 = __builtin_amdgcn_s_memrealtime();
#endif
    // The common table -- one segment, a first read unit that is no run, a
    // body within the caps -- is decoded by every thread from the staged
    // bytes (the same LDS bytes, broadcast reads), and a short or mid-size
    // body's decode starts at once; the rest take lane 0's frame_table and
    // a barrier (0.75 us of a read, r06q_bar_svcprof).
    uint64_t w0 = 0, u0 = 0;
    const bool fw = !no_alloc && capnp_frame::first_word(sm.lu.bytes, npre, &w0, &u0);
    const uint64_t ftot = w0 >> 32;
    const bool fast = fw && (uint32_t)w0 == 0u && ftot > 0 && ftot <= body_cap &&
                      !(has_limit && ftot > limit);  // (uniform: the same bytes everywhere)
    if (fast) {
        if (tid == 0) {  // (frame_table's record for this table)
            M.fr.status = 0;
            M.fr.nseg = 1;
            M.fr.table_consumed = u0;
            M.fr.total_words = ftot;
            M.fr.table_bytes = 8;
            M.fr.body_in_off[0] = u0;
            M.fr.body_in_off[1] = in_len;
            M.fr.body_out_off[0] = 0;
            M.fr.body_out_off[1] = ftot;
            M.fr.seg_words[0] = (uint32_t)ftot;
            *reinterpret_cast<uint64_t*>(M.fr.table) = w0;
            M.offs[0] = u0;
            M.offs[1] = in_len;
            M.offs[2] = 0;
            M.offs[3] = ftot;
            M.st = 0;
            M.used = 0;
        }
    } else {
        if (tid == 0) {
            // (the table's read units end within kMsgPre bytes whenever the
            // input is longer: the staged prefix gives the same results as
            // the input)
            capnp_frame::frame_table(sm.lu.bytes, npre, no_alloc, try_mode, limit, has_limit,
                                     buffer_len, body_cap, &M.fr);
            if (M.fr.status == 0) M.fr.body_in_off[1] = in_len;  // (the unit runs to the input end)
            M.offs[0] = M.fr.body_in_off[0];
            M.offs[1] = M.fr.body_in_off[1];
            M.offs[2] = 0;
            M.offs[3] = M.fr.body_out_off[1];
            M.st = 0;
            M.used = 0;
        }
        __syncthreads();
    }
#if SVC_PROF
    const uint64_t tp1 = __builtin_amdgcn_s_memrealtime();
#endif
    // (uniform: registers, or LDS after the barrier)
    if (fast || (M.fr.status == 0 && M.offs[3] > 0)) {
        // a short body inside the staged prefix: wave 0 alone (unpack_small);
        // the rest, and any body it does not take, unpack_long
        const uint64_t P0 = fast ? u0 : M.offs[0], nw = fast ? ftot : M.offs[3];
        const uint64_t avail = (uint64_t)pre > P0 ? pre - P0 : 0;
        const uint64_t span = in_len - P0 < avail ? in_len - P0 : avail;
        const uint64_t Ls = span < 10 * nw + 16 ? span : 10 * nw + 16;
        bool done = false;
        if (Ls > 0 && Ls <= kMidBytes && nw <= kLuWords) {
            uint32_t used = 0;
            done = Ls <= kSmallBytes
                       ? unpack_small(sm.lu, (uint32_t)P0, (uint32_t)Ls, (uint32_t)nw, words, tid,
                                      lane, wave, used)
                       : unpack_mid(sm.lu, (uint32_t)P0, (uint32_t)Ls, (uint32_t)nw, words, tid,
                                    lane, wave, used);
            if (done && tid == 0) {
                M.st = 0;
                M.used = used;
            }
        }
        if (!done) {
            if (fast) __syncthreads();  // (lane 0's M.offs)
            unpack_long(sm, in, M.offs, 0, words, M.offs + 2, &M.st, &M.used, tid, lane, wave,
                        pre);
        }
    }
    __syncthreads();
#if SVC_PROF
    const uint64_t tp2 = __builtin_amdgcn_s_memrealtime();
#endif
    // results out: the frame record (whole 16-byte vectors) and {status, 0, consumed}
    {
        constexpr uint32_t kV = (uint32_t)(sizeof(FrameResult) / 16);
        const uint4* f4 = reinterpret_cast<const uint4*>(&M.fr);
        uint4* o4 = reinterpret_cast<uint4*>(fr_out);
        for (uint32_t i = tid; i < kV; i += kThreads) o4[i] = f4[i];
        if (tid == 0) {
            res[0] = (uint64_t)(uint32_t)M.st;
            res[1] = 0;
            res[2] = M.used;
        }
    }
    if (flag) {  // (the host waits on this flag: everything above is visible first)
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
#if SVC_PROF
        const uint64_t tp3 = __builtin_amdgcn_s_memrealtime();
        if (tid == 0) {
            atomicAdd(&g_svc_prof[3], (unsigned long long)(tp1 - tp0));
            atomicAdd(&g_svc_prof[4], (unsigned long long)(tp2 - tp1));
            atomicAdd(&g_svc_prof[5], (unsigned long long)(tp3 - tp2));
            atomicAdd(&g_svc_prof[6], (unsigned long long)tp0);
        }
#endif
        if (tid == 0) {
            __threadfence_system();
            __hip_atomic_store(flag, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
}

__global__ void __launch_bounds__(kThreads)  // (one workgroup: registers are free)
msg_read_kernel(const uint8_t* __restrict__ in, uint64_t in_len, uint32_t no_alloc,
                uint32_t try_mode, uint64_t limit, uint32_t has_limit, uint64_t buffer_len,
                uint64_t body_cap, FrameResult* __restrict__ fr_out, uint64_t* __restrict__ words,
                uint64_t* __restrict__ res, uint32_t* __restrict__ flag, uint32_t seq) {
    __shared__ USmem sm;
    __shared__ MsgReadSmem M;
    msg_read_body(sm, M, in, in_len, no_alloc, try_mode, limit, has_limit, buffer_len, body_cap,
                  fr_out, words, res, flag, seq);
}

// The same call served by a resident workgroup (common.h, svc_next; the
// request's arguments: SvcReadReq).  fr_out and the completion flag are the
// context's own.
__global__ void __launch_bounds__(kThreads)
msg_read_service(const uint64_t* line, uint64_t* mark, uint32_t gen, uint64_t idle_ticks,
                 FrameResult* fr_out, uint32_t* flag) {
    __shared__ USmem sm;
    __shared__ MsgReadSmem M;
    __shared__ SvcCmd cmd;
    const uint32_t tid = threadIdx.x;
    const uint32_t lane = tid & 63u;
    const uint32_t wave = (uint32_t)__builtin_amdgcn_readfirstlane((int)(tid >> 6));
    uint32_t last = 0;
    while (svc_next(line, cmd, gen, last, idle_ticks, wave, lane)) {
        const SvcReadReq& q = *reinterpret_cast<const SvcReadReq*>(cmd.a);
        const uint64_t f = uniform64(q.flags), cap = uniform64(q.cap);
        uint64_t* const words = reinterpret_cast<uint64_t*>(uniform64(q.words));
        msg_read_body(sm, M, reinterpret_cast<const uint8_t*>(uniform64(q.in)), (uint32_t)f,
                      (uint32_t)(f >> 32) & 1u, (uint32_t)(f >> 33) & 1u, uniform64(q.limit),
                      (uint32_t)(f >> 34) & 1u, uniform64(q.buffer_len), cap, fr_out, words,
                      words + ((8 * cap + 15) & ~15ull) / 8, flag, last);
        svc_prof_done(cmd, tid);
        __syncthreads();
    }
    svc_exit(mark, gen, tid);
}

}  // namespace

// Output words per unpack tile the staged path is sized for; the host picks
// chunks_per_tile ~ this / mean chunk words.
extern "C" uint32_t capnp_unpack_tile_words(void) { return kTileWords; }

// Output words per wave sub-tile of the sync kernel (chunks_per_tile for the
// record-sync-index calls ~ this / mean chunk words).
extern "C" uint32_t capnp_unpack_sync_tile_words(void) { return kTileWords; }

extern "C" hipError_t capnp_launch_unpack(const uint8_t* d_in, const uint64_t* d_in_off,
                                          uint64_t nchunks, uint32_t tc, uint64_t* d_out,
                                          const uint64_t* d_out_off, int32_t* d_status,
                                          uint64_t* d_consumed, const uint32_t* d_sync,
                                          hipStream_t stream) {
    if (nchunks == 0) return hipSuccess;
    if (tc == 0) tc = kTileWords / 128;
    if (tc > kMaxTileChunks) return hipErrorInvalidValue;  // global path: 4 waves x 64
    const uint64_t blocks = (nchunks + tc - 1) / tc;
    if (d_sync) {
        // fitting tiles and overflow tiles in two kernels (the global path's
        // registers spilled in the combined kernel)
        const uint64_t og = (blocks + kThreads - 1) / kThreads;
        hipLaunchKernelGGL(unpack_fit_kernel<true>, dim3((uint32_t)blocks), dim3(kThreads), 0,
                           stream, d_in, d_in_off, nchunks, tc, d_out, d_out_off, d_status,
                           d_consumed, d_sync);
        hipLaunchKernelGGL(unpack_ovf_kernel<true>, dim3((uint32_t)(og < 1024 ? og : 1024)),
                           dim3(kThreads), 0, stream, d_in, d_in_off, nchunks, tc, d_out,
                           d_out_off, d_status, d_consumed, d_sync, blocks);
    } else {
        // index-free with the segment walk: split as the sync path (the walk's
        // registers and the global path's no longer meet in one kernel)
        hipLaunchKernelGGL(unpack_fit_kernel<false>, dim3((uint32_t)blocks), dim3(kThreads), 0,
                           stream, d_in, d_in_off, nchunks, tc, d_out, d_out_off, d_status,
                           d_consumed, d_sync);
        // (one workgroup per tile up to kOvfGrid, tiles dealt round robin: a
        // batch of long chunks, one per tile, decodes them all at once)
        const uint64_t wg = blocks < kOvfGrid ? blocks : kOvfGrid;
        hipLaunchKernelGGL(unpack_ovf_win_kernel<false>, dim3((uint32_t)wg),
                           dim3(kThreads), 0, stream, d_in, d_in_off, nchunks, tc, d_out,
                           d_out_off, d_status, d_consumed, d_sync, blocks);
    }
    return hipGetLastError();
}

// Word tiles (long chunks, record sync index): workspace and launch.  The
// batch's output words are [wlo, whi) = [out_off[0], out_off[nchunks]), which
// the caller read (the grid is sized by them).
extern "C" size_t capnp_unpack_wt_ws_bytes(uint64_t wlo, uint64_t whi) {
    const uint64_t ntiles = whi > wlo ? (whi + kWtWords - 1) / kWtWords - wlo / kWtWords : 0;
    return ntiles * (sizeof(WtPlan) + 4) + 64;
}

extern "C" uint32_t capnp_unpack_wt_words(void) { return kWtWords; }

// Word-tile diagnostics since the last reset: fallback tiles, failed pieces,
// chunks decoded serially by the finish kernel (tests use them to check that
// a valid index keeps every piece on the fast path).
extern "C" int capnp_unpack_wt_stats(unsigned long long* out4, int reset) {
    if (hipMemcpyFromSymbol(out4, HIP_SYMBOL(g_wt_stats), sizeof(g_wt_stats)) != hipSuccess)
        return -1;
    if (reset) {
        static const unsigned long long z[4] = {};
        if (hipMemcpyToSymbol(HIP_SYMBOL(g_wt_stats), z, sizeof(z)) != hipSuccess) return -1;
    }
    return 0;
}

extern "C" hipError_t capnp_launch_unpack_wt(const uint8_t* d_in, const uint64_t* d_in_off,
                                             uint64_t nchunks, uint64_t* d_out,
                                             const uint64_t* d_out_off, int32_t* d_status,
                                             uint64_t* d_consumed, const uint32_t* d_sync,
                                             uint64_t wlo, uint64_t whi, void* d_ws,
                                             size_t ws_bytes, hipStream_t stream) {
    if (nchunks == 0 || whi <= wlo || !d_sync) return hipErrorInvalidValue;
    if (ws_bytes < capnp_unpack_wt_ws_bytes(wlo, whi)) return hipErrorInvalidValue;
    const uint64_t g0 = wlo / kWtWords;
    const uint64_t ntiles = (whi + kWtWords - 1) / kWtWords - g0;
    WtPlan* plan = reinterpret_cast<WtPlan*>((reinterpret_cast<uintptr_t>(d_ws) + 63) & ~uintptr_t(63));
    uint32_t* flags = reinterpret_cast<uint32_t*>(plan + ntiles);
    const uint32_t g256 = (uint32_t)((ntiles + 255) / 256);
    hipLaunchKernelGGL(unpack_wt_plan, dim3(g256), dim3(256), 0, stream, d_in, d_in_off, nchunks,
                       d_out_off, d_sync, wlo, whi, g0, ntiles, plan);
    hipLaunchKernelGGL(unpack_wt_kernel, dim3((uint32_t)ntiles), dim3(kThreads), 0, stream, d_in,
                       d_in_off, d_out, d_out_off, d_status, d_consumed, d_sync, plan, flags, wlo,
                       whi, g0);
    hipLaunchKernelGGL(unpack_wt_finish, dim3(g256), dim3(256), 0, stream, d_in, d_in_off, d_out,
                       d_out_off, d_status, d_consumed, plan, flags, wlo, whi, g0, ntiles);
    return hipGetLastError();
}

#if UNPACK_PROF
extern "C" hipError_t capnp_unpack_trace(uint64_t* d_buf) {
    return hipMemcpyToSymbol(HIP_SYMBOL(g_utrace), &d_buf, sizeof(d_buf));
}

extern "C" hipError_t capnp_unpack_prof(unsigned long long* host16, int reset) {
    hipError_t e = hipMemcpyFromSymbol(host16, HIP_SYMBOL(g_uprof), sizeof(g_uprof));
    if (e == hipSuccess && reset) {
        static const unsigned long long z[16] = {};
        e = hipMemcpyToSymbol(HIP_SYMBOL(g_uprof), z, sizeof(z));
    }
    return e;
}
#endif

// One read_message call in one launch (msg_read_kernel): `in` (in_len bytes,
// 16-byte aligned, readable to the next multiple of 16) and the three outputs
// may be pinned host memory.  res = {status of the body, 0, consumed bytes}.
#if SVC_PROF
extern "C" int capnp_svc_prof(unsigned long long* out8, int reset) {
    if (hipMemcpyFromSymbol(out8, HIP_SYMBOL(g_svc_prof), 192) != hipSuccess) return -1;
    if (reset) {
        static const unsigned long long z[24] = {};
        if (hipMemcpyToSymbol(HIP_SYMBOL(g_svc_prof), z, 192) != hipSuccess) return -1;
    }
    return 0;
}
#endif

extern "C" hipError_t capnp_launch_msg_read_service(const uint64_t* line, uint64_t* mark,
                                                    uint32_t gen, uint64_t idle_ticks,
                                                    FrameResult* fr_out, uint32_t* flag,
                                                    hipStream_t stream) {
    hipLaunchKernelGGL(msg_read_service, dim3(1), dim3(kThreads), 0, stream, line, mark, gen,
                       idle_ticks, fr_out, flag);
    return hipGetLastError();
}

extern "C" hipError_t capnp_launch_msg_read(const uint8_t* in, uint64_t in_len, uint32_t no_alloc,
                                            uint32_t try_mode, uint64_t limit, uint32_t has_limit,
                                            uint64_t buffer_len, uint64_t body_cap,
                                            FrameResult* fr_out, uint64_t* words, uint64_t* res,
                                            uint32_t* flag, uint32_t seq, hipStream_t stream) {
    hipLaunchKernelGGL(msg_read_kernel, dim3(1), dim3(kThreads), 0, stream, in, in_len, no_alloc,
                       try_mode, limit, has_limit, buffer_len, body_cap, fr_out, words, res, flag,
                       seq);
    return hipGetLastError();
}
