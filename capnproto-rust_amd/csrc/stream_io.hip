// stream_io.hip — streaming adaptors over caller-supplied byte streams (host
// C++ over the gfx950 kernels; no transform runs on the CPU here).
//
//   capnp_packed_writer   the async PackedWrite of capnp-futures
//                         (capnp-futures/src/serialize_packed.rs:330-521):
//                         bytes arrive in arbitrary pieces, partial words are
//                         carried between calls (:370-393)
//   capnp_packed_reader   the async PackedRead (:34-225) and a message reader
//                         on top of it (capnp-futures/src/serialize.rs
//                         read_message / try_read_message, :31-137), over a
//                         read function that may return short reads or
//                         "pending"
//
// Writer.  The async writer's output depends only on where the write calls
// split the input: in one poll_write, a word completed from the carried
// bytes and every whole word after it form one chunk whose runs are found in
// that call's bytes only (WriteWord stage, :407-452: "see how long of a run
// we can make" scans `inbuf`), and the bytes after the last whole word are
// carried.  So a write call is one PACK chunk, exactly as a sync write_all
// (serialize_packed.rs:300-440) of those words.  Chunks are collected and
// packed as one batch by the GPU pack kernel (on flush, or every kBatchWords
// words), and the packed bytes drain to the inner writer, which may accept
// them piecemeal or report pending.
//
// Reader.  Packed input is pulled from the inner reader into a staging
// buffer and decoded by the GPU unpack kernel in whole-word units
// (PackedRead::read semantics, serialize_packed.rs:80-228); decoded bytes
// wait in an output buffer, so reads of any size (down to one byte,
// :186-205 of the async twin) are served from it.  A unit that ends inside a
// run (DidNotEndCleanly) is retried larger; a unit that needs more input
// pulls more.  At the end of the stream with a partial record left the read
// fails with PrematureEndOfFile (the async reader's UnexpectedEof, :109-114,
// :164-168, :207-212, which capnp maps to PrematureEndOfFile, lib.rs:481-499).
// A literal run whose raw words have not all arrived (the inner reader pends
// or ends inside them) is handed out as the async reader's stages do: the
// run's head word once its 10 bytes (tag, 8 bytes, count) are in
// (BufferingWord -> DrainingBuffer, :139-185), then its raw bytes as they
// come in (WritingPassthrough, :186-220: copied from the inner reader, no
// transform), and UnexpectedEof if the stream ends first.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <condition_variable>
#include <cstring>
#include <functional>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/capnp_packed.h"

// capi.hip (internal): the longest prefix of complete records of n host
// bytes, resolved on the device.
extern "C" capnp_status capnp_stream_decode_prefix(capnp_ctx* ctx, const uint8_t* host, size_t n,
                                                   uint64_t max_words, uint64_t* out,
                                                   uint64_t* bytes, uint64_t* words);
extern "C" capnp_status capnp_stream_complete_prefix(capnp_ctx* ctx, const uint8_t* host,
                                                     size_t n, uint64_t* bytes, uint64_t* words);

namespace {

// The adaptors' bulk buffers live in pinned host memory, so the device
// copies of a unit or batch are direct DMAs (a copy from pageable memory is
// staged by the runtime through its own pinned buffers, and blocks), and
// resize() does not zero what the next copy overwrites anyway.
template <class T>
struct PinnedAlloc {
    using value_type = T;
    PinnedAlloc() = default;
    template <class U>
    PinnedAlloc(const PinnedAlloc<U>&) {}
    T* allocate(size_t n) {
        void* p = nullptr;
        if (hipHostMalloc(&p, n * sizeof(T), hipHostMallocPortable) != hipSuccess || !p)
            throw std::bad_alloc();
        return static_cast<T*>(p);
    }
    void deallocate(T* p, size_t) { (void)hipHostFree(p); }
    template <class U>
    void construct(U* p) noexcept {
        ::new (static_cast<void*>(p)) U;  // default-init: no zero fill
    }
    template <class U, class... A>
    void construct(U* p, A&&... a) {
        ::new (static_cast<void*>(p)) U(std::forward<A>(a)...);
    }
    template <class U>
    bool operator==(const PinnedAlloc<U>&) const { return true; }
    template <class U>
    bool operator!=(const PinnedAlloc<U>&) const { return false; }
};
using PBytes = std::vector<uint8_t, PinnedAlloc<uint8_t>>;
using PWords = std::vector<uint64_t, PinnedAlloc<uint64_t>>;

// writer: pack every 8 MiB of input (one device batch of many write_all
// chunks; 1 MiB batches measured 4.1 GiB/s at 1 MiB calls, each batch paying
// the launches and waits of one device call)
#ifndef STREAM_BATCH_LG
#define STREAM_BATCH_LG 20
#endif
constexpr size_t kBatchWords = size_t(1) << STREAM_BATCH_LG;
constexpr size_t kPull = size_t(1) << 16;        // reader: bytes asked of the inner reader
constexpr size_t kPullMax = size_t(1) << 24;     // ... at most, when a unit needs more

struct Drain {
    PBytes q;
    size_t pos = 0;
};

// A background thread that runs one job at a time: the adaptors' device work
// for the next read unit or the previous write batch, so that it overlaps
// the caller's copies and the inner stream's calls.  Jobs run on a private
// context (its own stream and staging buffers, never the caller's).
class Worker {
public:
    Worker() : th_([this] { loop(); }) {}
    ~Worker() {
        wait();
        {
            std::lock_guard<std::mutex> l(m_);
            quit_ = true;
        }
        cv_.notify_all();
        th_.join();
    }
    void run(std::function<void()> f) {
        std::lock_guard<std::mutex> l(m_);
        job_ = std::move(f);
        busy_ = true;
        cv_.notify_all();
    }
    void wait() {
        std::unique_lock<std::mutex> l(m_);
        cv_.wait(l, [this] { return !busy_; });
    }

private:
    void loop() {
        std::unique_lock<std::mutex> l(m_);
        for (;;) {
            cv_.wait(l, [this] { return quit_ || busy_; });
            if (quit_) return;
            std::function<void()> f = std::move(job_);
            l.unlock();
            f();
            l.lock();
            busy_ = false;
            cv_.notify_all();
        }
    }
    std::mutex m_;
    std::condition_variable cv_;
    std::function<void()> job_;
    bool busy_ = false, quit_ = false;
    std::thread th_;  // (last: starts once the members above exist)
};

// The private context and worker of one adaptor, created on first use.
struct Background {
    capnp_ctx* ctx = nullptr;
    std::unique_ptr<Worker> wk;
    ~Background() {
        wk.reset();  // (joins: no job runs past here)
        if (ctx) capnp_ctx_destroy(ctx);
    }
    capnp_status ensure(int device) {
        if (wk) return CAPNP_OK;
        capnp_status st = CAPNP_OK;
        ctx = capnp_ctx_create(device, &st);
        if (!ctx) return st == CAPNP_OK ? CAPNP_E_HIP : st;
        wk.reset(new Worker());
        return CAPNP_OK;
    }
};

}  // namespace

// capi.hip (internal): the device a context was created on.
extern "C" int capnp_ctx_device(const capnp_ctx* ctx);

namespace {

uint64_t get_u64(const uint8_t* p) {
    uint64_t v;
    memcpy(&v, p, 8);
    return v;
}

}  // namespace

struct capnp_packed_writer {
    capnp_ctx* ctx;
    capnp_write_fn fn;
    void* user;
    uint8_t part[8];
    size_t npart = 0;                   // carried bytes of an incomplete word
    PWords words;                       // chunks not yet packed, back to back
    std::vector<uint64_t> off{0};       // their word offsets
    Drain out;                          // packed bytes the inner writer has not taken
    // the full batch being packed in the background (bw, boff -> bout)
    Background bg;
    bool busy = false;
    PWords bw;
    std::vector<uint64_t> boff;
    PBytes bout;
    capnp_status bst = CAPNP_OK;
};

struct capnp_packed_reader {
    capnp_ctx* ctx;
    capnp_read_fn fn;
    void* user;
    PBytes in;                // staged packed input
    size_t ip = 0;            // bytes of `in` already decoded
    bool eof = false;
    // the last pull got every byte it asked for: the inner reader had more
    // ready than that, so pulling ahead of need is safe (a short read means
    // the source is drained for now, and a blocking reader would block)
    bool last_full = false;
    // bulk read-ahead allowed (capnp_packed_reader_set_readahead): pulls past
    // what the caller's current request can need, while pulls come back
    // full.  Off by default: then a read first decodes what is staged and
    // pulls only when no complete record is, as the reference reads no
    // further than the current request needs, so a blocking peer that sent
    // exactly one request's worth and awaits a reply is never read past it.
    bool readahead = false;
    PBytes dec;                // decoded bytes not yet handed out
    PBytes spare;              // the next decode's buffer (swapped with dec)
    size_t dp = 0;
    size_t pass_rem = 0;       // raw bytes of a literal run still to pass through
    capnp_status pull_err = CAPNP_OK;  // a read-ahead pull's error, for the next pull
    // read-ahead: the next whole-record unit (in[a_ip ..], a_nw words asked),
    // decoded in the background while the caller drains `dec`
    Background bg;
    bool ahead = false;
    size_t a_ip = 0, a_nw = 0;
    double bpw = 10.0;  // packed bytes per word of the last whole-record unit
    capnp_status a_st = CAPNP_OK;
    uint64_t a_pb = 0, a_pw = 0;
    PBytes a_out;
};

namespace {

// The background batch's packed bytes, once packed, go behind the queued
// ones (batches drain in order).
capnp_status writer_collect(capnp_packed_writer* w) {
    if (!w->busy) return CAPNP_OK;
    w->bg.wk->wait();
    w->busy = false;
    if (w->bst != CAPNP_OK) return w->bst;
    if (w->out.pos == w->out.q.size()) {
        w->out.q.swap(w->bout);
        w->out.pos = 0;
    } else {
        w->out.q.insert(w->out.q.end(), w->bout.begin(), w->bout.end());
    }
    w->bout.clear();
    return CAPNP_OK;
}

// Hands the collected chunks to the background (after the previous batch's
// bytes are queued): the caller's next writes fill a new batch meanwhile.
capnp_status writer_launch(capnp_packed_writer* w) {
    capnp_status st = writer_collect(w);
    if (st != CAPNP_OK) return st;
    if ((st = w->bg.ensure(capnp_ctx_device(w->ctx))) != CAPNP_OK) return st;
    w->bw.swap(w->words);
    w->boff.swap(w->off);
    w->words.clear();
    w->off.assign(1, 0);
    w->busy = true;
    w->bg.wk->run([w] {
        const size_t n = w->boff.size() - 1;
        const uint64_t nw = w->boff[n];
        const size_t cap = capnp_packed_batch_bound_bytes(nw, n);
        w->bout.resize(cap);
        std::vector<uint64_t> oo(n + 1);
        w->bst = capnp_pack_batch_host(w->bg.ctx, w->bw.data(), w->boff.data(), n, w->bout.data(),
                                       cap, oo.data());
        w->bout.resize(w->bst == CAPNP_OK ? oo[n] : 0);
    });
    return CAPNP_OK;
}

capnp_status writer_pack(capnp_packed_writer* w) {
    const size_t n = w->off.size() - 1;
    if (n == 0) return CAPNP_OK;
    const uint64_t nw = w->off[n];
    const size_t cap = capnp_packed_batch_bound_bytes(nw, n);
    const size_t base = w->out.q.size();
    w->out.q.resize(base + cap);
    std::vector<uint64_t> oo(n + 1);
    capnp_status st = capnp_pack_batch_host(w->ctx, w->words.data(), w->off.data(), n,
                                            w->out.q.data() + base, cap, oo.data());
    if (st != CAPNP_OK) {
        w->out.q.resize(base);
        return st;
    }
    w->out.q.resize(base + oo[n]);
    w->words.clear();
    w->off.assign(1, 0);
    return CAPNP_OK;
}

// Hands queued bytes to the inner writer until it is empty or pends.
capnp_status writer_drain(capnp_packed_writer* w) {
    while (w->out.pos < w->out.q.size()) {
        const ptrdiff_t r = w->fn(w->user, w->out.q.data() + w->out.pos,
                                  w->out.q.size() - w->out.pos);
        if (r == CAPNP_IO_PENDING) return CAPNP_PENDING;
        if (r <= 0) return CAPNP_E_IO;  // an error, or a writer that takes nothing
        w->out.pos += (size_t)r;
    }
    w->out.q.clear();
    w->out.pos = 0;
    return CAPNP_OK;
}

// Pulls more packed input; CAPNP_OK with bytes added, CAPNP_NONE at the end
// of the stream, CAPNP_PENDING, or an I/O error.
capnp_status reader_pull(capnp_packed_reader* r, size_t ask = kPull) {
    if (r->pull_err != CAPNP_OK) {  // (a read-ahead pull failed: the next pull reports it)
        const capnp_status e = r->pull_err;
        r->pull_err = CAPNP_OK;
        return e;
    }
    if (r->eof) return CAPNP_NONE;
    ask = std::min(std::max(ask, kPull), kPullMax);
    // drop the decoded prefix when the pull would otherwise grow the buffer
    // (a compaction moves what is staged ahead: only as often as needed)
    if (r->ip > 0 && r->in.size() + ask > r->in.capacity()) {
        r->in.erase(r->in.begin(), r->in.begin() + (ptrdiff_t)r->ip);
        r->ip = 0;
    }
    const size_t base = r->in.size();
    r->in.resize(base + ask);
    const ptrdiff_t got = r->fn(r->user, r->in.data() + base, ask);
    if (got == CAPNP_IO_PENDING) {
        r->in.resize(base);
        return CAPNP_PENDING;
    }
    if (got < 0) {
        r->in.resize(base);
        return CAPNP_E_IO;
    }
    r->in.resize(base + (size_t)got);
    r->last_full = (size_t)got == ask;
    if (got == 0) {
        r->eof = true;
        return CAPNP_NONE;
    }
    return CAPNP_OK;
}

// Whether a pull ahead of need may be made: nothing is staged, or the last
// pull was full.  The reference pulls only what the caller's words need
// (poll_read asks for a tag, a word, a run), so a reader over a blocking
// pipe or socket never waits for input beyond the current request; the
// adaptors pull in bulk (one decode per MiBs, not per record) but stop at the
// first short read, so with a blocking inner reader the same holds: every
// further pull is one the decode of the staged bytes showed it needs.
bool may_pull_ahead(const capnp_packed_reader* r) {
    return r->in.size() == r->ip || (r->readahead && r->last_full);
}

// One PackedRead::read of `nw` words at the current position, on the GPU.
// A stream decodes at most 10 input bytes per output word (tag, 8 bytes,
// count), so only that much of the staged input is handed to the kernel.
capnp_status reader_unit(capnp_packed_reader* r, size_t nw, PBytes& out,
                         size_t* used, int32_t* status, size_t max_bytes = ~size_t(0)) {
    const size_t avail = std::min(r->in.size() - r->ip, max_bytes);
    const size_t take = std::min(avail, nw * 10 + 16);
    out.resize(nw * 8);
    uint64_t io[2] = {0, take}, oo[2] = {0, nw};
    uint64_t cons = 0;
    capnp_status st = capnp_unpack_batch_host(r->ctx, r->in.data() + r->ip, io, 1,
                                              reinterpret_cast<uint64_t*>(out.data()), oo, status,
                                              &cons);
    *used = (size_t)cons;
    return st;
}

// WritingPassthrough (capnp-futures serialize_packed.rs:186-220): the raw
// bytes of a literal run go straight from the inner reader to the caller;
// the stream ending inside them is UnexpectedEof.
capnp_status reader_pass(capnp_packed_reader* r) {
    if (r->ip == r->in.size()) {
        capnp_status p = reader_pull(r);
        if (p == CAPNP_NONE) return CAPNP_E_PREMATURE_END_OF_FILE;
        if (p != CAPNP_OK) return p;
    }
    const size_t k = std::min(r->in.size() - r->ip, r->pass_rem);
    r->dec.assign(r->in.begin() + (ptrdiff_t)r->ip, r->in.begin() + (ptrdiff_t)(r->ip + k));
    r->dp = 0;
    r->ip += k;
    r->pass_rem -= k;
    return CAPNP_OK;
}

// The staged input starts with a record no unit decodes (the inner reader
// pends or has ended): if it is a literal run's head (tag 0xFF, 8 bytes,
// count) whose raw words are not all in, hand out the head word as the
// async reader's DrainingBuffer stage does, plus the raw bytes already
// staged, and pass the rest through (reader_pass).  The head word is decoded
// by the GPU unpack (a 1-word unit of the record with a zero count).
// CAPNP_NONE when the record is anything else.
capnp_status reader_lit_head(capnp_packed_reader* r) {
    const size_t avail = r->in.size() - r->ip;
    if (avail < 10 || r->in[r->ip] != 0xFF) return CAPNP_NONE;
    const size_t c8 = 8 * (size_t)r->in[r->ip + 9];
    uint8_t head[10];
    memcpy(head, r->in.data() + r->ip, 9);
    head[9] = 0;
    uint64_t io[2] = {0, 10}, oo[2] = {0, 1}, word = 0, cons = 0;
    int32_t st = 0;
    capnp_status e = capnp_unpack_batch_host(r->ctx, head, io, 1, &word, oo, &st, &cons);
    if (e != CAPNP_OK) return e;
    if (st != CAPNP_OK) return (capnp_status)st;
    const size_t k = std::min(avail - 10, c8);
    r->dec.resize(8 + k);
    memcpy(r->dec.data(), &word, 8);
    memcpy(r->dec.data() + 8, r->in.data() + r->ip + 10, k);
    r->dp = 0;
    r->ip += 10 + k;
    r->pass_rem = c8 - k;
    return CAPNP_OK;
}

// Decodes at least one word into r->dec (empty only at a clean end of the
// stream).  `want` = words the caller asked for; units are at least
// kMinUnit words (small reads are served from the decoded surplus), but an
// inner reader that pends while the caller's own words are staged gets
// those decoded rather than a pending answer.
constexpr size_t kMinUnit = 256;      // (>= the words of any one record: a run is 1 + 255)
constexpr size_t kWholeUnit = 8192;   // units this long are cut at whole records on the device
// a read of a whole-record unit decodes at least this many words (8 MiB):
// the surplus serves the next reads from `dec` while the unit after it
// decodes in the background (a 1 MiB unit paid ~18 launches and a few waits
// of the resync decode per 1 MiB read: 2.1 GiB/s; round 4, interleaved on
// one box, 1 MiB reads: 8 MiB units 8.1 / 8.3 / 8.6 GiB/s against 4 MiB
// units 5.6 / 6.7 / 6.4, profiles/r04af_adaptor_unit_ab.txt)
#ifndef STREAM_BIGUNIT_LG
#define STREAM_BIGUNIT_LG 20
#endif
constexpr size_t kBigUnit = size_t(1) << STREAM_BIGUNIT_LG;

// A long unit: the staged input is resolved on the device and cut after the
// last complete record that fits nw words (capnp_stream_decode_prefix), so
// the unit ends cleanly (no doubling when a run crosses its end) and its
// decode keeps the block walk (a unit with spare input bytes would take the
// serial walk).  The read returns at most nw words: whole records, at least
// nw - 255 of them unless the stream pends or ends.
// Read-ahead after a whole-record unit: stages the input the next unit of
// nw words consumes (as reader_fill_whole would, at its next call) and
// decodes it in the background.  Nothing changes what the reads hand out:
// the unit is the one the next call would decode, and a pull that pends or
// fails here leaves the next call to meet it.
void reader_ahead(capnp_packed_reader* r, size_t nw) {
    for (size_t need = nw * 10 + 16; r->in.size() - r->ip < need;) {
        // (never a pull the caller's request does not need; without bulk
        // read-ahead the next unit decodes only from what is staged)
        if (!r->last_full || !r->readahead) break;
        const capnp_status p = reader_pull(r, need - (r->in.size() - r->ip));
        if (p == CAPNP_OK) continue;
        if (p == CAPNP_NONE) break;      // end of stream: the rest is staged
        if (p != CAPNP_PENDING) r->pull_err = p;
        return;
    }
    if (r->in.size() == r->ip || r->bg.ensure(capnp_ctx_device(r->ctx)) != CAPNP_OK) return;
    r->ahead = true;
    r->a_ip = r->ip;
    r->a_nw = nw;
    const uint8_t* src = r->in.data() + r->ip;
    // the unit resolves only what it may consume: the last unit's bytes per
    // word with a margin (its records past nw words are resolved for
    // nothing); a unit that finds no complete record in that is decoded
    // again from everything staged by the next read (reader_fill_whole)
    const size_t est = (size_t)(r->bpw * 1.25 * 8.0 * (double)nw / 8.0) + (size_t(64) << 10);
    const size_t n = std::min(r->in.size() - r->ip, est);
    r->bg.wk->run([r, src, n, nw] {
        r->a_out.resize(nw * 8);
        r->a_pb = r->a_pw = 0;
        r->a_st = capnp_stream_decode_prefix(r->bg.ctx, src, n, nw,
                                             reinterpret_cast<uint64_t*>(r->a_out.data()),
                                             &r->a_pb, &r->a_pw);
        if (r->a_st == CAPNP_OK) r->a_out.resize(r->a_pw * 8);
    });
}

capnp_status reader_fill_whole(capnp_packed_reader* r, size_t nw) {
    PBytes& out = r->spare;
    if (r->ahead) {  // the unit decoded ahead, if it is this one
        r->bg.wk->wait();
        r->ahead = false;
        if (r->a_st == CAPNP_OK && r->a_pw > 0 && r->a_ip == r->ip && r->a_nw == nw) {
            r->bpw = (double)r->a_pb / (double)r->a_pw;
            r->ip += r->a_pb;
            r->dec.swap(r->a_out);
            r->dp = 0;
            reader_ahead(r, nw);
            return CAPNP_OK;
        }
    }
    for (;;) {
        if (r->ip == r->in.size()) {
            capnp_status p = reader_pull(r);
            if (p == CAPNP_NONE) return CAPNP_OK;  // clean end: nothing decoded
            if (p != CAPNP_OK) return p;
            continue;
        }
        capnp_status p = CAPNP_OK;
        for (size_t need = nw * 10 + 16; r->in.size() - r->ip < need && may_pull_ahead(r);)
            if ((p = reader_pull(r, need - (r->in.size() - r->ip))) != CAPNP_OK) break;
        out.resize(nw * 8);
        uint64_t pb = 0, pw = 0;
        capnp_status e = capnp_stream_decode_prefix(r->ctx, r->in.data() + r->ip,
                                                    r->in.size() - r->ip, nw,
                                                    reinterpret_cast<uint64_t*>(out.data()), &pb,
                                                    &pw);
        if (e != CAPNP_OK) return e;
        if (pw > 0) {
            out.resize(pw * 8);
            r->bpw = (double)pb / (double)pw;
            r->ip += pb;
            r->dec.swap(out);
            r->dp = 0;
            reader_ahead(r, nw);
            return CAPNP_OK;
        }
        // the first staged record is incomplete: more input, or pending / end
        if (p == CAPNP_OK) p = reader_pull(r);
        if (p == CAPNP_OK) continue;
        if (p != CAPNP_NONE && p != CAPNP_PENDING) return p;
        e = reader_lit_head(r);
        if (e != CAPNP_NONE) return e;
        return p == CAPNP_PENDING ? CAPNP_PENDING : CAPNP_E_PREMATURE_END_OF_FILE;  // UnexpectedEof
    }
}

capnp_status reader_fill(capnp_packed_reader* r, size_t want) {
    want = std::max<size_t>(want, 1);
    size_t nw = std::max(want, kMinUnit);
    PBytes& out = r->spare;
    if (r->ahead && (r->pass_rem || nw < kWholeUnit)) {
        // (not a whole-record unit: the one decoded ahead is not this one)
        r->bg.wk->wait();
        r->ahead = false;
    }
    if (r->pass_rem) return reader_pass(r);
    if (nw >= kWholeUnit) return reader_fill_whole(r, std::max(nw, kBigUnit));
    for (;;) {
        if (r->ip == r->in.size()) {
            capnp_status p = reader_pull(r);
            if (p == CAPNP_NONE) return CAPNP_OK;  // clean end: nothing decoded
            if (p != CAPNP_OK) return p;
            continue;
        }
        // stage what the unit can consume (<= 10 bytes a word) before the
        // decode, so one read costs one launch rather than one per pull; a
        // pull that stops short (pending, end, error) is met again below
        for (size_t need = nw * 10 + 16; r->in.size() - r->ip < need && may_pull_ahead(r);)
            if (reader_pull(r, need - (r->in.size() - r->ip)) != CAPNP_OK) break;
        size_t used = 0;
        int32_t st = 0;
        capnp_status e = reader_unit(r, nw, out, &used, &st);
        if (e != CAPNP_OK) return e;
        if (st == CAPNP_OK) {
            r->ip += used;
            r->dec.swap(out);
            r->dp = 0;
            return CAPNP_OK;
        }
        if (st == CAPNP_E_DID_NOT_END_CLEANLY) {  // a run crosses the unit end
            nw = nw * 2 + 256;
            continue;
        }
        // PrematureEnd / FailedToFill: the unit needs more input.  A bulk
        // source is pulled at once; from a drained one (the last pull was
        // short) the complete records already staged go out first, as the
        // reference's read returns what it has decoded, and a pull is made
        // only when there is none.
        capnp_status p = r->eof ? CAPNP_NONE : CAPNP_PENDING;
        const bool pulled = may_pull_ahead(r);
        if (pulled) {
            p = reader_pull(r);
            if (p == CAPNP_OK) continue;
            if (p != CAPNP_NONE && p != CAPNP_PENDING) return p;
        }
        // nothing more now (pending) or ever (end of stream): every complete
        // record staged (the device resolves where the last one ends), then
        // a literal run's head, else pending / a partial record
        uint64_t pb = 0, pw = 0;
        e = capnp_stream_complete_prefix(r->ctx, r->in.data() + r->ip, r->in.size() - r->ip, &pb,
                                         &pw);
        if (e != CAPNP_OK) return e;
        if (pw > 0) {
            // the unit is exactly the complete records
            e = reader_unit(r, pw, out, &used, &st, (size_t)pb);
            if (e != CAPNP_OK) return e;
            if (st != CAPNP_OK) return (capnp_status)st;
            r->ip += used;
            r->dec.swap(out);
            r->dp = 0;
            return CAPNP_OK;
        }
        if (!pulled && !r->eof) {  // nothing complete staged: the request needs input
            p = reader_pull(r);
            if (p == CAPNP_OK) continue;
            if (p != CAPNP_NONE && p != CAPNP_PENDING) return p;
        }
        e = reader_lit_head(r);
        if (e != CAPNP_NONE) return e;
        return p == CAPNP_PENDING ? CAPNP_PENDING : CAPNP_E_PREMATURE_END_OF_FILE;  // UnexpectedEof
    }
}

}  // namespace

extern "C" {

capnp_packed_writer* capnp_packed_writer_new(capnp_ctx* ctx, capnp_write_fn fn, void* user) {
    if (!ctx || !fn) return nullptr;
    auto* w = new capnp_packed_writer();
    w->ctx = ctx;
    w->fn = fn;
    w->user = user;
    return w;
}

void capnp_packed_writer_free(capnp_packed_writer* w) {
    if (w && w->bg.wk) w->bg.wk->wait();  // (the background batch uses w's buffers)
    delete w;
}

capnp_status capnp_packed_writer_write(capnp_packed_writer* w, const uint8_t* buf, size_t len) {
    if (!w || (len && !buf)) return CAPNP_E_INVALID_ARGUMENT;
    size_t k = 0;
    const size_t w0 = w->words.size();
    if (w->npart) {  // Start stage: complete the carried word (:370-393)
        const size_t t = std::min(8 - w->npart, len);
        memcpy(w->part + w->npart, buf, t);
        w->npart += t;
        k = t;
        if (w->npart == 8) {
            w->words.push_back(get_u64(w->part));
            w->npart = 0;
        }
    }
    const size_t m = (len - k) / 8;
    if (m) {
        const size_t b = w->words.size();
        w->words.resize(b + m);
        memcpy(w->words.data() + b, buf + k, m * 8);
        k += m * 8;
    }
    if (k < len) {  // carry the incomplete word
        memcpy(w->part + w->npart, buf + k, len - k);
        w->npart += len - k;
    }
    if (w->words.size() > w0) w->off.push_back(w->words.size());  // this call's chunk
    if (w->words.size() >= kBatchWords) {
        // the previous batch's bytes are queued and drained while this one
        // packs in the background
        capnp_status st = writer_launch(w);
        if (st != CAPNP_OK) return st;
        st = writer_drain(w);
        if (st != CAPNP_OK && st != CAPNP_PENDING) return st;
    }
    return CAPNP_OK;
}

capnp_status capnp_packed_writer_flush(capnp_packed_writer* w) {
    if (!w) return CAPNP_E_INVALID_ARGUMENT;
    capnp_status st = writer_collect(w);
    if (st != CAPNP_OK) return st;
    st = writer_pack(w);
    if (st != CAPNP_OK) return st;
    return writer_drain(w);
}

size_t capnp_packed_writer_carried(const capnp_packed_writer* w) { return w ? w->npart : 0; }

capnp_packed_reader* capnp_packed_reader_new(capnp_ctx* ctx, capnp_read_fn fn, void* user) {
    if (!ctx || !fn) return nullptr;
    auto* r = new capnp_packed_reader();
    r->ctx = ctx;
    r->fn = fn;
    r->user = user;
    return r;
}

void capnp_packed_reader_set_readahead(capnp_packed_reader* r, int on) {
    if (r) r->readahead = on != 0;
}

void capnp_packed_reader_free(capnp_packed_reader* r) {
    if (r && r->bg.wk) r->bg.wk->wait();  // (the read-ahead uses r's buffers)
    delete r;
}

capnp_status capnp_packed_reader_read(capnp_packed_reader* r, uint8_t* out, size_t len,
                                      size_t* nread) {
    if (!r || !nread || (len && !out)) return CAPNP_E_INVALID_ARGUMENT;
    *nread = 0;
    if (len == 0) return CAPNP_OK;
    if (r->dp == r->dec.size()) {
        capnp_status st = reader_fill(r, (len + 7) / 8);
        if (st != CAPNP_OK) return st;
        if (r->dec.empty()) return CAPNP_OK;  // clean end of stream: Ok(0)
    }
    const size_t n = std::min(len, r->dec.size() - r->dp);
    memcpy(out, r->dec.data() + r->dp, n);
    r->dp += n;
    if (r->dp == r->dec.size()) {
        r->dec.clear();
        r->dp = 0;
    }
    *nread = n;
    return CAPNP_OK;
}

// read_exact (futures AsyncReadExt::read_exact): loops over reads, retrying a
// pending inner reader; PrematureEndOfFile if the stream ends first.
// *got (optional) = bytes delivered before an error.
capnp_status capnp_packed_reader_read_exact(capnp_packed_reader* r, uint8_t* out, size_t len,
                                            size_t* got) {
    if (!r || (len && !out)) return CAPNP_E_INVALID_ARGUMENT;
    size_t k = 0;
    if (got) *got = 0;
    while (k < len) {
        size_t n = 0;
        capnp_status st = capnp_packed_reader_read(r, out + k, len - k, &n);
        if (st == CAPNP_PENDING) continue;
        if (got) *got = k;
        if (st != CAPNP_OK) return st;
        if (n == 0) return CAPNP_E_PREMATURE_END_OF_FILE;
        k += n;
    }
    if (got) *got = k;
    return CAPNP_OK;
}

// capnp-futures serialize::try_read_message / read_message over a
// PackedRead (capnp-futures/src/serialize_packed.rs:233-258 ->
// capnp-futures/src/serialize.rs:31-137): the segment table (a first word,
// then the rest of the table), then the body.  Checks as capnp's
// read_segment_table (serialize.rs:448-510): segment count 1..511, the
// traversal limit; the body goes to `body` (body_cap_words words; on
// BufferNotLargeEnough *body_words holds the words needed).
capnp_status capnp_packed_reader_read_message(capnp_packed_reader* r,
                                              const capnp_reader_options* opts, int try_mode,
                                              uint64_t* body, size_t body_cap_words,
                                              uint32_t* seg_words, uint32_t* nseg_out,
                                              uint64_t* body_words) {
    if (!r || !seg_words || !nseg_out) return CAPNP_E_INVALID_ARGUMENT;
    const capnp_reader_options o = opts ? *opts : capnp_default_reader_options();
    *nseg_out = 0;
    if (body_words) *body_words = 0;
    uint8_t w0[8];
    size_t got = 0;
    capnp_status st;
    do {  // the first read tells a clean end (Ok(0)) from a partial record
        st = capnp_packed_reader_read(r, w0, 8, &got);
    } while (st == CAPNP_PENDING);
    if (st != CAPNP_OK) return st;
    if (got == 0) return try_mode ? CAPNP_NONE : CAPNP_E_PREMATURE_END_OF_FILE;
    if (got < 8) {
        st = capnp_packed_reader_read_exact(r, w0 + got, 8 - got, nullptr);
        if (st != CAPNP_OK) return st;
    }
    uint32_t u0, l0;
    memcpy(&u0, w0, 4);
    memcpy(&l0, w0 + 4, 4);
    const uint32_t nseg = u0 + 1u;
    if (nseg == 0 || nseg >= 512) return CAPNP_E_INVALID_NUMBER_OF_SEGMENTS;
    seg_words[0] = l0;
    uint64_t total = l0;
    if (nseg > 1) {
        const size_t rest = nseg < 4 ? 8 : (size_t)(nseg & ~1u) * 4;
        uint8_t t[512 * 4];
        st = capnp_packed_reader_read_exact(r, t, rest, nullptr);
        if (st != CAPNP_OK) return st;
        for (uint32_t i = 1; i < nseg; i++) {
            uint32_t l;
            memcpy(&l, t + 4 * (i - 1), 4);
            seg_words[i] = l;
            total += l;
        }
    }
    *nseg_out = nseg;  // (the table is read: its lengths are valid from here on)
    if (o.has_traversal_limit && total > o.traversal_limit_in_words)
        return CAPNP_E_MESSAGE_TOO_LARGE;
    if (body_words) *body_words = total;
    if (total > body_cap_words || (total && !body)) return CAPNP_E_BUFFER_NOT_LARGE_ENOUGH;
    if (total) {
        st = capnp_packed_reader_read_exact(r, reinterpret_cast<uint8_t*>(body), total * 8,
                                            nullptr);
        if (st != CAPNP_OK) return st;
    }
    return CAPNP_OK;
}

// Bytes staged but not yet decoded, and decoded but not yet read.
size_t capnp_packed_reader_buffered(const capnp_packed_reader* r) {
    return r ? (r->in.size() - r->ip) + (r->dec.size() - r->dp) : 0;
}

}  // extern "C"
