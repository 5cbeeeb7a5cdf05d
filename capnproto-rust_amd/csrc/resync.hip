// resync.hip — index-free parallel decode of long packed read units
// (SURVEY §8f row 2): the same transform and results as the batch UNPACK
// (PackedRead::read under read_exact, capnp/src/serialize_packed.rs:80-228,
// io.rs:16-31) for streams that carry no record sync index, where a chunk can
// be any length (a 64 KiB segment, or a whole multi-megabyte message body).
//
// The decode of a read unit is a serial tag chain: where record k+1 starts
// depends on record k's tag and run count.  The batch unpack without an index
// gives one lane per chunk, so a long chunk is one long dependent chain.
// Here each chunk's packed bytes are cut into kBlock-byte blocks, one lane
// per block, and the chain is resynchronised speculatively:
//
//   spec   lane k walks its block from the block's first byte as if a record
//          started there; its exit (first record position at or past the
//          block end) and word count are kept.  A chunk's first block starts
//          at a real record, so its walk is exact.
//   fix    lane k takes its true entry, the exit of block k-1, and walks from
//          it in lockstep with the speculative chain until both land on the
//          same byte (tag chains couple within a few records: record lengths
//          are 1..10 bytes).  From the meet on the speculative walk is exact,
//          so the exit stands and only the word count changes.  No meet (or an
//          entry past the block end, as inside a literal run that spans
//          blocks) means the block is re-walked from the entry and its exit
//          changes; the pass repeats until no exit changes.  A fix lane owns
//          8 consecutive blocks and fixes them in order, so inside a literal
//          run region (long records no speculative walk couples with) the
//          true chain advances 8 blocks per pass; passes are enqueued 8 at a
//          time and skip themselves after a pass that changed nothing.  At that fixed
//          point every block's entry is its predecessor's exit and the first
//          block's entry is the chunk start, so by induction every exit is
//          the one the serial walk produces.
//   scan   exclusive scan of the block word counts: each block's first
//          output word.
//   check  lane per chunk: the chain must end exactly at the chunk's packed
//          end with exactly the chunk's word count (then no record ran short,
//          and no run overran the output: the word count is monotone).
//   decode each resolved block is a read unit of its own (its records run
//          from its entry to its exit): the blocks go to the batch unpack
//          kernel as a batch of ~120-word units (staged LDS tiles, coalesced
//          stores).
//
// Any chunk that fails the check (a malformed stream, or a valid unit
// followed by spare bytes in its range) makes the call re-decode the batch
// with the serial batch unpack, so statuses, consumed counts and partial
// output are exactly capnp_gpu_unpack_batch's.
#include <hipcub/hipcub.hpp>

#include "common.h"
#include "../../include/capnp_packed.h"

#ifndef RESYNC_BLOCK
#define RESYNC_BLOCK 512
#endif

extern "C" hipError_t capnp_launch_unpack(const uint8_t* d_in, const uint64_t* d_in_off,
                                          size_t nchunks, uint32_t tc, uint64_t* d_out,
                                          const uint64_t* d_out_off, int32_t* d_status,
                                          uint64_t* d_consumed, const uint32_t* d_sync,
                                          hipStream_t stream);

namespace {

constexpr uint64_t kBlock = RESYNC_BLOCK;  // packed bytes per lane
constexpr uint32_t kThreads = 256;
constexpr uint64_t kGroup = 8;  // blocks per fix lane
constexpr int kMaxPasses = 512;  // fix passes before giving up to the serial path
constexpr int kPassBatch = 8;    // fix passes enqueued per flag read-back
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

// Chunk of block `blk`: the last c with bstart[c] <= blk (empty chunks own
// no blocks, so equal starts are skipped by taking the last one).
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
    uint64_t* spec_exit;   // [nbb]
    uint32_t* spec_words;  // [nbb]
    uint64_t* exit;        // [nbb]
    uint64_t* entry;       // [nbb] entry the current exit/words were derived from
    uint64_t* words;       // [nbb]
    uint64_t* wbase;       // [nbb] exclusive scan of words
    int32_t* ok;           // [n]
    int32_t* flags;        // [1] chunk failed, [2 + i] fix pass i changed an exit
    void* tmp;
    size_t tmp_bytes;
};

__global__ void __launch_bounds__(kThreads) k_count(const uint64_t* __restrict__ in_off, uint64_t n,
                                                    uint64_t* __restrict__ nblk) {
    const uint64_t c = (uint64_t)blockIdx.x * kThreads + threadIdx.x;
    if (c > n) return;
    nblk[c] = c == n ? 0 : (in_off[c + 1] - in_off[c] + kBlock - 1) / kBlock;
}

__global__ void __launch_bounds__(kThreads)
k_spec(const uint8_t* __restrict__ in, const uint64_t* __restrict__ in_off, uint64_t n,
       const uint64_t* __restrict__ bstart, uint64_t* __restrict__ spec_exit,
       uint32_t* __restrict__ spec_words, uint64_t* __restrict__ exit, uint64_t* __restrict__ entry,
       uint64_t* __restrict__ words) {
    const uint64_t k = (uint64_t)blockIdx.x * kThreads + threadIdx.x;
    if (k >= bstart[n]) return;
    const uint64_t c = chunk_of(bstart, n, k);
    const uint64_t b = in_off[c + 1];
    const uint64_t s = in_off[c] + (k - bstart[c]) * kBlock;
    const uint64_t end = s + kBlock < b ? s + kBlock : b;
    uint64_t p = s, w = 0;
    while (p < end) hop(in, p, w, b);
    spec_exit[k] = p;
    spec_words[k] = (uint32_t)w;
    exit[k] = p;
    entry[k] = s;
    words[k] = w;
}

// Fix pass `pass`: lane = group of kGroup consecutive blocks of the batch,
// fixed in order, so a lane's own blocks take their entries from exits it has
// just computed (a literal run that spans blocks, which no speculative walk
// couples with, then costs one pass per group rather than per block).  The
// group's first block reads its predecessor's exit as the last pass left it.
// The pass does nothing if the previous pass changed no exit.
__global__ void __launch_bounds__(kThreads)
k_fix(const uint8_t* __restrict__ in, const uint64_t* __restrict__ in_off, uint64_t n,
      const uint64_t* __restrict__ bstart, const uint64_t* __restrict__ spec_exit,
      const uint32_t* __restrict__ spec_words, uint64_t* exit, uint64_t* __restrict__ entry,
      uint64_t* __restrict__ words, int32_t* flags, int pass) {
    if (pass > 0 && __atomic_load_n(&flags[2 + pass - 1], __ATOMIC_RELAXED) == 0) return;
    const uint64_t k0 = ((uint64_t)blockIdx.x * kThreads + threadIdx.x) * kGroup;
    const uint64_t nb = bstart[n];
    if (k0 >= nb) return;
    uint64_t c = chunk_of(bstart, n, k0);
    bool changed = false;
    for (uint64_t k = k0; k < k0 + kGroup && k < nb; k++) {
        while (k >= bstart[c + 1]) c++;
        if (k == bstart[c]) continue;  // a chunk's first block starts at its first record
        // (a predecessor in another group may be rewritten by its own lane
        // during this pass; either value is fine, a later pass sees the last)
        const uint64_t e = __atomic_load_n(&exit[k - 1], __ATOMIC_RELAXED);
        if (e == entry[k]) continue;
        const uint64_t b = in_off[c + 1];
        const uint64_t s = in_off[c] + (k - bstart[c]) * kBlock;
        const uint64_t end = s + kBlock < b ? s + kBlock : b;
        uint64_t nx, nw;
        if (e >= end) {  // the block lies inside a record that began earlier
            nx = e;
            nw = 0;
        } else {
            uint64_t ps = s, ws = 0;  // speculative chain
            uint64_t pt = e, wt = 0;  // true chain
            bool met = false;
            while (pt < end) {
                while (ps < pt && ps < end) hop(in, ps, ws, b);
                if (ps == pt) {
                    met = true;
                    break;
                }
                hop(in, pt, wt, b);
            }
            if (met) {
                nx = spec_exit[k];
                nw = wt + spec_words[k] - ws;
            } else {
                nx = pt;
                nw = wt;
            }
        }
        entry[k] = e;
        words[k] = nw;
        if (nx != exit[k]) {
            __atomic_store_n(&exit[k], nx, __ATOMIC_RELAXED);
            changed = true;
        }
    }
    if (changed) flags[2 + pass] = 1;
}

__global__ void __launch_bounds__(kThreads)
k_check(const uint64_t* __restrict__ in_off, uint64_t n, const uint64_t* __restrict__ out_off,
        const uint64_t* __restrict__ bstart, const uint64_t* __restrict__ exit,
        const uint64_t* __restrict__ words, const uint64_t* __restrict__ wbase,
        int32_t* __restrict__ ok, int32_t* __restrict__ status, uint64_t* __restrict__ consumed,
        int32_t* __restrict__ flags) {
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
        good = exit[l] == b && wbase[l] + words[l] - wbase[f] == nw;
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
// since read() of an empty buffer consumes nothing).
__global__ void __launch_bounds__(kThreads)
k_blocks(const uint64_t* __restrict__ in_off, uint64_t n, const uint64_t* __restrict__ out_off,
         const uint64_t* __restrict__ bstart, const uint64_t* __restrict__ exit,
         const uint64_t* __restrict__ wbase, uint64_t* __restrict__ blk_in,
         uint64_t* __restrict__ blk_out) {
    const uint64_t k = (uint64_t)blockIdx.x * kThreads + threadIdx.x;
    const uint64_t nb = bstart[n];
    if (k > nb) return;
    if (k == nb) {
        blk_in[k] = in_off[n];
        blk_out[k] = out_off[n];
        return;
    }
    const uint64_t c = chunk_of(bstart, n, k);
    const uint64_t f = bstart[c];
    blk_in[k] = k == f ? in_off[c] : exit[k - 1];
    blk_out[k] = out_off[c] + (out_off[c + 1] == out_off[c] ? 0 : wbase[k] - wbase[f]);
}

size_t carve(Ws* w, uint8_t* base, uint64_t n, uint64_t nbb, size_t tmp_bytes) {
    size_t off = 0;
    auto take = [&](size_t bytes) {
        uint8_t* p = base ? base + off : nullptr;
        off += (bytes + 255) & ~size_t(255);
        return p;
    };
    w->nblk = (uint64_t*)take(8 * (n + 1));
    w->bstart = (uint64_t*)take(8 * (n + 1));
    w->spec_exit = (uint64_t*)take(8 * nbb);
    w->spec_words = (uint32_t*)take(4 * nbb);
    w->exit = (uint64_t*)take(8 * nbb);
    w->entry = (uint64_t*)take(8 * nbb);
    w->words = (uint64_t*)take(8 * nbb);
    w->wbase = (uint64_t*)take(8 * nbb);
    w->ok = (int32_t*)take(4 * n + 4);
    w->flags = (int32_t*)take(4 * (2 + kMaxPasses));
    w->tmp = take(tmp_bytes);
    w->tmp_bytes = tmp_bytes;
    return off;
}

size_t scan_tmp_bytes(uint64_t items) {
    size_t bytes = 0;
    hipcub::DeviceScan::ExclusiveSum(nullptr, bytes, (const uint64_t*)nullptr, (uint64_t*)nullptr,
                                     (int)items);
    return bytes;
}

uint64_t blocks_bound(uint64_t n, uint64_t total_bytes) { return total_bytes / kBlock + n + 1; }

unsigned grid(uint64_t items) { return (unsigned)((items + kThreads - 1) / kThreads); }

}  // namespace

extern "C" uint32_t capnp_resync_block_bytes(void) { return (uint32_t)kBlock; }

// Workspace for capnp_resync_unpack over n chunks holding total_bytes packed bytes.
extern "C" size_t capnp_resync_ws_bytes(uint64_t n, uint64_t total_bytes) {
    const uint64_t nbb = blocks_bound(n, total_bytes);
    const uint64_t m = nbb > n + 1 ? nbb : n + 1;
    Ws w;
    return carve(&w, nullptr, n, nbb, scan_tmp_bytes(m)) + 256;
}

// Blocking (the fix passes read a flag back).  On return, *passes = fix passes
// run and *serial = 1 if the batch was re-decoded by the serial batch unpack
// (a chunk failed its check), 2 if its chunks were short enough to go there
// directly.
extern "C" hipError_t capnp_resync_unpack(const uint8_t* d_in, const uint64_t* d_in_off, uint64_t n,
                                          uint64_t total_bytes, uint64_t* d_out,
                                          const uint64_t* d_out_off, int32_t* d_status,
                                          uint64_t* d_consumed, void* d_ws, size_t ws_bytes,
                                          hipStream_t s, int* passes, int* serial) {
    if (passes) *passes = 0;
    if (serial) *serial = 0;
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
    if (carve(&w, base, n, nbb, scan_tmp_bytes(m)) + (base - (uint8_t*)d_ws) > ws_bytes)
        return hipErrorInvalidValue;
    int32_t hflags[2] = {0, 0};
    if ((e = hipMemsetAsync(w.flags, 0, 4 * (2 + kMaxPasses), s)) != hipSuccess) return e;
    k_count<<<grid(n + 1), kThreads, 0, s>>>(d_in_off, n, w.nblk);
    size_t tb = w.tmp_bytes;
    if ((e = hipcub::DeviceScan::ExclusiveSum(w.tmp, tb, w.nblk, w.bstart, (int)(n + 1), s)) !=
        hipSuccess)
        return e;
    k_spec<<<grid(nbb), kThreads, 0, s>>>(d_in, d_in_off, n, w.bstart, w.spec_exit, w.spec_words,
                                          w.exit, w.entry, w.words);
    // fix passes, kPassBatch at a time; a pass after one that changed nothing
    // returns at once, so the flag of a batch's last pass says whether the
    // fixed point was reached
    int pass = 0;
    const uint64_t ngroups = (nbb + kGroup - 1) / kGroup;
    for (;;) {
        if (pass == kMaxPasses) {
            hflags[1] = 1;  // not converged: let the serial walk decide
            break;
        }
        for (int i = 0; i < kPassBatch; i++, pass++)
            k_fix<<<grid(ngroups), kThreads, 0, s>>>(d_in, d_in_off, n, w.bstart, w.spec_exit,
                                                     w.spec_words, w.exit, w.entry, w.words,
                                                     w.flags, pass);
        int32_t last = 0;
        if ((e = hipMemcpyAsync(&last, w.flags + 2 + pass - 1, 4, hipMemcpyDeviceToHost, s)) !=
            hipSuccess)
            return e;
        if ((e = hipStreamSynchronize(s)) != hipSuccess) return e;
        if (!last) break;
    }
    if (passes) *passes = pass;
    if (!hflags[1]) {
        tb = w.tmp_bytes;
        if ((e = hipcub::DeviceScan::ExclusiveSum(w.tmp, tb, w.words, w.wbase, (int)nbb, s)) !=
            hipSuccess)
            return e;
        k_check<<<grid(n), kThreads, 0, s>>>(d_in_off, n, d_out_off, w.bstart, w.exit, w.words,
                                             w.wbase, w.ok, d_status, d_consumed, w.flags);
        uint64_t nb = 0;
        if ((e = hipMemcpyAsync(hflags, w.flags, 8, hipMemcpyDeviceToHost, s)) != hipSuccess)
            return e;
        if ((e = hipMemcpyAsync(&nb, w.bstart + n, 8, hipMemcpyDeviceToHost, s)) != hipSuccess)
            return e;
        if ((e = hipStreamSynchronize(s)) != hipSuccess) return e;
        if (!hflags[1]) {
            // every chunk resolved: decode the blocks as independent read
            // units with the batch unpack (staged LDS tiles, coalesced stores)
            uint64_t* blk_in = w.spec_exit;  // (spec state is dead by now)
            uint64_t* blk_out = w.entry;
            int32_t* blk_status = reinterpret_cast<int32_t*>(w.spec_words);
            k_blocks<<<grid(nbb + 1), kThreads, 0, s>>>(d_in_off, n, d_out_off, w.bstart, w.exit,
                                                        w.wbase, blk_in, blk_out);
            if ((e = capnp_launch_unpack(d_in, blk_in, nb, 0, d_out, blk_out, blk_status, nullptr,
                                         nullptr, s)) != hipSuccess)
                return e;
        }
    }
    if (hflags[1]) {
        if (serial) *serial = 1;
        if ((e = capnp_launch_unpack(d_in, d_in_off, n, 0, d_out, d_out_off, d_status, d_consumed,
                                     nullptr, s)) != hipSuccess)
            return e;
        if ((e = hipStreamSynchronize(s)) != hipSuccess) return e;
    }
    return hipGetLastError();
}
