// msgbatch.hip — device framing of many messages at once: the batched body of
// serialize_packed::write_message (serialize_packed.rs:446-453 ->
// serialize.rs:574-679), SURVEY §8f row 1.
//
// write_message packs a message as separate write_all calls: the segment
// table's first word, the rest of the table (when there is more than one
// segment), then every segment (serialize.rs:605-679), and a packed write_all
// never carries a run across calls.  So a batch of messages is a batch of
// chunks: msg_layout sizes each message (table words, chunk count), two
// exclusive scans place them, msg_assemble writes each message's table words
// and copies its segments into one staging array with the chunk offsets of
// the layout, and the regular batch pack kernel packs the chunks.  The
// message byte offsets are the chunk offsets of each message's first chunk.
#include "common.h"
#include "../../include/capnp_packed.h"
#include <hipcub/hipcub.hpp>

namespace {

constexpr int kThreads = 256;

// Per message: staging words (table + segments) and chunk count, into
// cw[m] / cc[m] (m < nmsg; entry nmsg is 0 so the exclusive scans end in the
// totals).  The table is 1 + nseg / 2 words: word 0 = (nseg - 1, len 0),
// then the other lengths as u32, padded to a word (serialize.rs:211-253).
__global__ void msg_layout(const uint64_t* __restrict__ seg_off,
                           const uint64_t* __restrict__ msg_seg_off, uint64_t nmsg,
                           uint64_t* __restrict__ cw, uint64_t* __restrict__ cc) {
    const uint64_t m = (uint64_t)blockIdx.x * kThreads + threadIdx.x;
    if (m > nmsg) return;
    if (m == nmsg) {
        cw[m] = 0;
        cc[m] = 0;
        return;
    }
    const uint64_t s0 = msg_seg_off[m], s1 = msg_seg_off[m + 1];
    const uint64_t nseg = s1 - s0;
    cw[m] = 1 + nseg / 2 + (seg_off[s1] - seg_off[s0]);
    cc[m] = 1 + (nseg > 1 ? 1 : 0) + nseg;
}

// One wave per message: table words, chunk offsets (staging-relative word
// offsets; chunk c ends where chunk c + 1 starts) and the segment words.
__global__ void msg_assemble(const uint64_t* __restrict__ words,
                             const uint64_t* __restrict__ seg_off,
                             const uint64_t* __restrict__ msg_seg_off, uint64_t nmsg,
                             const uint64_t* __restrict__ wofs, const uint64_t* __restrict__ cofs,
                             uint64_t* __restrict__ stage, uint64_t* __restrict__ chunk_off) {
    const uint64_t m = (uint64_t)blockIdx.x * (kThreads / CAPNP_WAVE) + (threadIdx.x >> 6);
    const uint32_t lane = threadIdx.x & 63u;
    if (m >= nmsg) return;
    const uint64_t s0 = msg_seg_off[m], s1 = msg_seg_off[m + 1];
    const uint64_t nseg = s1 - s0;
    const uint64_t w = wofs[m], c = cofs[m];
    const uint64_t t = 1 + nseg / 2;  // table words
    uint64_t* dst = stage + w;
    uint32_t* tab = reinterpret_cast<uint32_t*>(dst);
    // table: u32 [nseg - 1, len 0, len 1, ..., pad]
    for (uint64_t i = lane; i < 2 * t; i += CAPNP_WAVE) {
        uint32_t v;
        if (i == 0) v = (uint32_t)(nseg - 1);
        else if (i - 1 < nseg) v = (uint32_t)(seg_off[s0 + i] - seg_off[s0 + i - 1]);
        else v = 0;
        tab[i] = v;
    }
    // chunks: table word 0, the rest of the table, each segment
    if (lane == 0) {
        chunk_off[c] = w;
        if (nseg > 1) chunk_off[c + 1] = w + 1;
    }
    const uint64_t cs = c + 1 + (nseg > 1 ? 1 : 0);
    const uint64_t base = seg_off[s0];
    for (uint64_t j = lane; j < nseg; j += CAPNP_WAVE)
        chunk_off[cs + j] = w + t + (seg_off[s0 + j] - base);
    if (m + 1 == nmsg && lane == 0) chunk_off[cs + nseg] = w + t + (seg_off[s1] - base);
    // segment words (contiguous in the input from seg_off[s0] on)
    const uint64_t n = seg_off[s1] - base;
    const uint64_t* src = words + base;
    for (uint64_t i = lane; i < n; i += CAPNP_WAVE) dst[t + i] = src[i];
}

__global__ void msg_offsets(const uint64_t* __restrict__ cofs,
                            const uint64_t* __restrict__ chunk_byte_off, uint64_t nmsg,
                            uint64_t* __restrict__ msg_byte_off) {
    const uint64_t m = (uint64_t)blockIdx.x * kThreads + threadIdx.x;
    if (m <= nmsg) msg_byte_off[m] = chunk_byte_off[cofs[m]];
}

// ---- gap path: segments packed in place, tables written into the gaps ----
// Word i of message m's segment table (serialize.rs:211-253): word 0 =
// (nseg - 1, len 0), then the other lengths as u32 pairs, zero padded.
__device__ __forceinline__ uint64_t table_word(const uint64_t* __restrict__ seg_off, uint64_t s0,
                                               uint64_t nseg, uint64_t i) {
    auto len = [&](uint64_t k) -> uint64_t {
        return k < nseg ? (uint32_t)(seg_off[s0 + k + 1] - seg_off[s0 + k]) : 0u;
    };
    if (i == 0) return (uint64_t)(uint32_t)(nseg - 1) | (len(0) << 32);
    return len(2 * i - 1) | (len(2 * i) << 32);
}

// PackedWrite::write_all of table words [i0, i1) (serialize_packed.rs:
// 304-439, the oracle's pack_into): the bytes go to emit(byte) in order;
// returns their count.
template <class Emit>
__device__ uint32_t pack_table_words(const uint64_t* __restrict__ seg_off, uint64_t s0,
                                     uint64_t nseg, uint64_t i0, uint64_t i1, Emit emit) {
    uint32_t n = 0;
    uint64_t i = i0;
    while (i < i1) {
        const uint64_t w = table_word(seg_off, s0, nseg, i++);
        uint32_t tag = 0;
        for (int k = 0; k < 8; k++) tag |= (((w >> (8 * k)) & 0xFF) != 0) << k;
        emit(n++, tag);
        for (int k = 0; k < 8; k++)
            if ((w >> (8 * k)) & 0xFF) emit(n++, (uint32_t)(w >> (8 * k)) & 0xFF);
        if (tag == 0 || tag == 0xFF) {
            const uint64_t lim = (i1 - i) < 255 ? i1 - i : 255;
            uint64_t r = 0;
            while (r < lim) {
                const uint64_t v = table_word(seg_off, s0, nseg, i + r);
                if (tag == 0 ? v != 0 : __builtin_popcount(word_tag((uint32_t)v,
                                                                  (uint32_t)(v >> 32))) < 7)
                    break;
                r++;
            }
            emit(n++, (uint32_t)r);
            if (tag == 0xFF)
                for (uint64_t j = 0; j < r; j++) {
                    const uint64_t v = table_word(seg_off, s0, nseg, i + j);
                    for (int k = 0; k < 8; k++) emit(n++, (uint32_t)(v >> (8 * k)) & 0xFF);
                }
            i += r;
        }
    }
    return n;
}

// write_message packs the table as two write_all calls: word 0, then the
// rest (when nseg > 1; serialize.rs:605-679).
template <class Emit>
__device__ uint32_t pack_table(const uint64_t* __restrict__ seg_off, uint64_t s0, uint64_t nseg,
                               Emit emit) {
    const uint32_t a = pack_table_words(seg_off, s0, nseg, 0, 1, emit);
    if (nseg < 2) return a;
    return a + pack_table_words(seg_off, s0, nseg, 1, 1 + nseg / 2,
                                [&](uint32_t k, uint32_t b) { emit(a + k, b); });
}

// One thread per message: the packed table size into gap[first segment]
// (gap is zeroed beforehand).  flag bit 0: a message without segments, or
// message segment offsets that do not span [0, total_segs) -> staging path.
__global__ void msg_gap(const uint64_t* __restrict__ seg_off,
                        const uint64_t* __restrict__ msg_seg_off, uint64_t nmsg,
                        uint64_t total_segs, uint32_t* __restrict__ gap,
                        uint32_t* __restrict__ flag) {
    const uint64_t m = (uint64_t)blockIdx.x * kThreads + threadIdx.x;
    if (m >= nmsg) return;
    const uint64_t s0 = msg_seg_off[m], s1 = msg_seg_off[m + 1];
    bool bad = s1 <= s0 || s1 > total_segs;
    if (m == 0) bad |= s0 != 0;
    if (m + 1 == nmsg) bad |= s1 != total_segs;
    if (bad) {
        atomicOr(flag, 1u);
        return;
    }
    gap[s0] = pack_table(seg_off, s0, s1 - s0, [](uint32_t, uint32_t) {});
}

// After the gap pack: the table bytes into each message's gap and the
// message byte offsets (the gap starts).
__global__ void msg_tables(const uint64_t* __restrict__ seg_off,
                           const uint64_t* __restrict__ msg_seg_off, uint64_t nmsg,
                           const uint64_t* __restrict__ chunk_byte_off, uint8_t* __restrict__ out,
                           uint64_t out_cap, uint64_t* __restrict__ msg_byte_off) {
    const uint64_t m = (uint64_t)blockIdx.x * kThreads + threadIdx.x;
    if (m > nmsg) return;
    const uint64_t s0 = msg_seg_off[m];
    const uint64_t p = chunk_byte_off[s0];
    msg_byte_off[m] = p;
    if (m == nmsg) return;
    const uint64_t nseg = msg_seg_off[m + 1] - s0;
    const uint32_t g = pack_table(seg_off, s0, nseg, [](uint32_t, uint32_t) {});
    if (p + g > out_cap) return;  // the caller sees the size and reports it
    uint8_t* dst = out + p;
    pack_table(seg_off, s0, nseg, [&](uint32_t k, uint32_t b) { dst[k] = (uint8_t)b; });
}

}  // namespace

extern "C" hipError_t capnp_launch_msg_gap(const uint64_t* d_seg_off,
                                           const uint64_t* d_msg_seg_off, uint64_t nmsg,
                                           uint64_t total_segs, uint32_t* d_gap,
                                           uint32_t* d_flag, hipStream_t s) {
    hipError_t e = hipMemsetAsync(d_gap, 0, total_segs * 4, s);
    if (e != hipSuccess) return e;
    e = hipMemsetAsync(d_flag, 0, 4, s);
    if (e != hipSuccess) return e;
    const uint32_t g = (uint32_t)((nmsg + kThreads - 1) / kThreads);
    hipLaunchKernelGGL(msg_gap, dim3(g), dim3(kThreads), 0, s, d_seg_off, d_msg_seg_off, nmsg,
                       total_segs, d_gap, d_flag);
    return hipGetLastError();
}

extern "C" hipError_t capnp_launch_msg_tables(const uint64_t* d_seg_off,
                                              const uint64_t* d_msg_seg_off, uint64_t nmsg,
                                              const uint64_t* d_chunk_byte_off, uint8_t* d_out,
                                              uint64_t out_cap, uint64_t* d_msg_byte_off,
                                              hipStream_t s) {
    const uint32_t g = (uint32_t)((nmsg + 1 + kThreads - 1) / kThreads);
    hipLaunchKernelGGL(msg_tables, dim3(g), dim3(kThreads), 0, s, d_seg_off, d_msg_seg_off, nmsg,
                       d_chunk_byte_off, d_out, out_cap, d_msg_byte_off);
    return hipGetLastError();
}

extern "C" hipError_t capnp_msg_scan_bytes(uint64_t n, size_t* bytes) {
    *bytes = 0;
    return hipcub::DeviceScan::ExclusiveSum(nullptr, *bytes, (const uint64_t*)nullptr,
                                            (uint64_t*)nullptr, (int)n);
}

// Layout, scans and assembly; the caller reads the totals (wofs[nmsg],
// cofs[nmsg]) before packing.  tmp: capnp_msg_scan_bytes(nmsg + 1) bytes.
extern "C" hipError_t capnp_launch_msg_prepare(const uint64_t* d_words, const uint64_t* d_seg_off,
                                               const uint64_t* d_msg_seg_off, uint64_t nmsg,
                                               uint64_t* cw, uint64_t* cc, uint64_t* wofs,
                                               uint64_t* cofs, void* tmp, size_t tmp_bytes,
                                               uint64_t* stage, uint64_t* chunk_off,
                                               hipStream_t s) {
    const uint32_t g1 = (uint32_t)((nmsg + 1 + kThreads - 1) / kThreads);
    hipLaunchKernelGGL(msg_layout, dim3(g1), dim3(kThreads), 0, s, d_seg_off, d_msg_seg_off, nmsg,
                       cw, cc);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    size_t tb = tmp_bytes;
    e = hipcub::DeviceScan::ExclusiveSum(tmp, tb, cw, wofs, (int)(nmsg + 1), s);
    if (e != hipSuccess) return e;
    tb = tmp_bytes;
    e = hipcub::DeviceScan::ExclusiveSum(tmp, tb, cc, cofs, (int)(nmsg + 1), s);
    if (e != hipSuccess) return e;
    const uint32_t per = kThreads / CAPNP_WAVE;
    const uint32_t g2 = (uint32_t)((nmsg + per - 1) / per);
    if (g2)
        hipLaunchKernelGGL(msg_assemble, dim3(g2), dim3(kThreads), 0, s, d_words, d_seg_off,
                           d_msg_seg_off, nmsg, wofs, cofs, stage, chunk_off);
    return hipGetLastError();
}

extern "C" hipError_t capnp_launch_msg_offsets(const uint64_t* cofs,
                                               const uint64_t* chunk_byte_off, uint64_t nmsg,
                                               uint64_t* msg_byte_off, hipStream_t s) {
    const uint32_t g = (uint32_t)((nmsg + 1 + kThreads - 1) / kThreads);
    hipLaunchKernelGGL(msg_offsets, dim3(g), dim3(kThreads), 0, s, cofs, chunk_byte_off, nmsg,
                       msg_byte_off);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Batch read_message / try_read_message on the device (serialize_packed.rs:
// 233-255 -> serialize.rs:287-325, 448-524), messages delimited by a
// side-band byte index (as capnp_gpu_write_messages writes it).  Per
// message: the 8-byte first read unit, the rest of the table as one read
// unit (serialize.rs:476-496), then the body as one read_exact.  The table
// read units are decoded by one lane per message with PackedRead semantics
// (serialize_packed.rs:80-228), streaming the decoded bytes into a sink, so
// no per-message table buffer is needed; the bodies then go through the
// batch UNPACK kernel as chunks interleaved with zero-word "table" chunks
// (so that consecutive chunks stay contiguous in the packed stream).
namespace {

enum : int32_t {
    MST_OK = 0, MST_NONE = 1, MST_PREMATURE = 2, MST_NOT_CLEAN = 3, MST_FAILED_FILL = 4,
    MST_EOF = 5, MST_BAD_NSEG = 6, MST_TOO_LARGE = 8,
};

// One PackedRead::read of out_len bytes over in[0..in_len), the decoded
// bytes handed to sink(i, byte) in order (frame.hip serial_read with a sink).
template <class Sink>
__device__ int32_t read_unit(const uint8_t* in, uint64_t in_len, uint64_t out_len, Sink sink,
                             uint64_t* used, uint64_t* nread) {
    *used = 0;
    *nread = 0;
    if (out_len == 0 || in_len == 0) return MST_OK;
    uint64_t ip = 0, op = 0;
    while (op < out_len) {
        if (ip == in_len) return MST_PREMATURE;
        const uint32_t tag = in[ip++];
        for (int k = 0; k < 8; k++) {
            if (tag & (1u << k)) {
                if (ip == in_len) return MST_PREMATURE;
                sink(op++, in[ip++]);
            } else {
                sink(op++, 0);
            }
        }
        if (tag == 0 || tag == 0xFF) {
            if (ip == in_len) return MST_PREMATURE;
            const uint64_t run = 8ull * in[ip++];
            if (run > out_len - op) return MST_NOT_CLEAN;
            if (tag == 0) {
                for (uint64_t i = 0; i < run; i++) sink(op++, 0);
            } else {
                if (in_len - ip < run) { *used = in_len; return MST_FAILED_FILL; }
                for (uint64_t i = 0; i < run; i++) sink(op++, in[ip++]);
            }
        }
    }
    *used = ip;
    *nread = out_len;
    return MST_OK;
}

// The segment table of the message in in[0..in_len): status, segment count,
// body words and the packed bytes the table used; seg (may be null) receives
// the segment lengths.
__device__ int32_t read_table(const uint8_t* in, uint64_t in_len, int try_mode, uint64_t limit,
                              int has_limit, uint32_t* nseg_out, uint64_t* words_out,
                              uint64_t* used_out, uint64_t* seg) {
    *nseg_out = 0;
    *words_out = 0;
    *used_out = 0;
    uint32_t w0[2] = {0, 0};
    uint64_t used = 0, nread = 0;
    int32_t st = read_unit(in, in_len, 8,
                           [&](uint64_t i, uint32_t b) { w0[i >> 2] |= b << (8 * (i & 3)); },
                           &used, &nread);
    if (st != MST_OK) return st;
    if (nread == 0) return try_mode ? MST_NONE : MST_EOF;
    const uint32_t nseg = w0[0] + 1u;
    if (nseg >= 512u || nseg == 0) return MST_BAD_NSEG;
    uint64_t total = w0[1];
    if (seg) seg[0] = w0[1];
    uint64_t pos = used;
    if (nseg > 1) {
        const uint64_t rest = nseg < 4 ? 8 : (uint64_t)(nseg & ~1u) * 4;
        uint32_t acc = 0;
        st = read_unit(in + pos, in_len - pos, rest,
                       [&](uint64_t i, uint32_t b) {
                           acc |= b << (8 * (i & 3));
                           if ((i & 3) == 3) {
                               const uint64_t k = (i >> 2) + 1;  // segment index
                               if (k < nseg) {
                                   total += acc;
                                   if (seg) seg[k] = acc;
                               }
                               acc = 0;
                           }
                       },
                       &used, &nread);
        if (st == MST_OK && nread != rest) st = MST_FAILED_FILL;  // read_exact (io.rs:16-31)
        if (st != MST_OK) return st;
        pos += used;
    }
    if (has_limit && total > limit) return MST_TOO_LARGE;
    *nseg_out = nseg;
    *words_out = total;
    *used_out = pos;
    return MST_OK;
}

__global__ void msg_frame(const uint8_t* __restrict__ in, const uint64_t* __restrict__ msg_off,
                          uint64_t nmsg, int try_mode, uint64_t limit, int has_limit,
                          uint64_t* __restrict__ nseg, uint64_t* __restrict__ words,
                          int32_t* __restrict__ st, uint64_t* __restrict__ tused) {
    const uint64_t m = (uint64_t)blockIdx.x * kThreads + threadIdx.x;
    if (m > nmsg) return;
    if (m == nmsg) {
        nseg[m] = 0;
        words[m] = 0;
        return;
    }
    const uint64_t a = msg_off[m], b = msg_off[m + 1];
    uint32_t ns = 0;
    uint64_t w = 0, u = 0;
    const int32_t s = read_table(in + a, b - a, try_mode, limit, has_limit, &ns, &w, &u, nullptr);
    st[m] = s;
    nseg[m] = s == MST_OK ? ns : 0;
    words[m] = s == MST_OK ? w : 0;
    tused[m] = s == MST_OK ? u : 0;
}

// Segment lengths into seg[sofs[m] ..], and the interleaved chunk tables of
// the body unpack: chunk 2m = message m's table bytes (no output words),
// chunk 2m + 1 = its body (words[m] words; a failed table gets none).
__global__ void msg_segs(const uint8_t* __restrict__ in, const uint64_t* __restrict__ msg_off,
                         uint64_t nmsg, int try_mode, uint64_t limit, int has_limit,
                         const int32_t* __restrict__ st, const uint64_t* __restrict__ tused,
                         const uint64_t* __restrict__ sofs, const uint64_t* __restrict__ wofs,
                         uint64_t* __restrict__ seg, uint64_t* __restrict__ in_off,
                         uint64_t* __restrict__ out_off) {
    const uint64_t m = (uint64_t)blockIdx.x * kThreads + threadIdx.x;
    if (m > nmsg) return;
    if (m == nmsg) {
        in_off[2 * m] = msg_off[m];
        out_off[2 * m] = wofs[m];
        return;
    }
    const uint64_t a = msg_off[m], b = msg_off[m + 1];
    in_off[2 * m] = a;
    out_off[2 * m] = wofs[m];
    out_off[2 * m + 1] = wofs[m];
    if (st[m] == MST_OK) {
        uint32_t ns;
        uint64_t w, u;
        read_table(in + a, b - a, try_mode, limit, has_limit, &ns, &w, &u, seg + sofs[m]);
        in_off[2 * m + 1] = a + tused[m];
    } else {
        in_off[2 * m + 1] = b;  // the whole range is "table"; the body chunk is empty
    }
}

// Per message: the table's status, else the body's; bytes consumed.
__global__ void msg_status(uint64_t nmsg, const int32_t* __restrict__ tst,
                           const uint64_t* __restrict__ tused, const int32_t* __restrict__ cst,
                           const uint64_t* __restrict__ ccons, int32_t* __restrict__ status,
                           uint64_t* __restrict__ consumed) {
    const uint64_t m = (uint64_t)blockIdx.x * kThreads + threadIdx.x;
    if (m >= nmsg) return;
    const bool ok = tst[m] == MST_OK;
    status[m] = ok ? cst[2 * m + 1] : tst[m];
    if (consumed) consumed[m] = ok ? tused[m] + ccons[2 * m + 1] : 0;
}

// ---- unpacked flat-slice framing -------------------------
// One thread per message: the segment table is at most 2 KiB and almost
// always one word, so the pass is a handful of loads per message (the batch
// is bound by the 8-64 B of table each message reads plus its output rows).
// Status values are capnp_status codes.
enum : int32_t {
    FST_OK = 0, FST_FAILED_FILL = 4, FST_BAD_NSEG = 6, FST_TOO_LARGE = 8,
    FST_ENDS_PREMATURELY = 12, FST_EMPTY = 13, FST_NOT_ALIGNED = 14,
};

__device__ __forceinline__ uint32_t ld_u32(const uint8_t* p) {
    return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) |
           ((uint32_t)p[3] << 24);
}

// read_message_from_flat_slice (serialize.rs:53-78 over read_segment_table
// :448-510 on a &[u8]) or NoAllocSliceSegments::from_slice
// (no_alloc_buffer_segments.rs:22-92).  seg (nullable) receives the lengths.
__device__ int32_t flat_table(const uint8_t* p, uint64_t len, int no_alloc, uint64_t limit,
                              int has_limit, uint32_t* nseg_out, uint64_t* table_out,
                              uint64_t* words_out, uint32_t* seg) {
    // On FST_ENDS_PREMATURELY *table_out / *words_out carry the reference's
    // MessageEndsPrematurely(header, body) payload instead.
    uint64_t total = 0, pos, nseg;
#define ENDS_PREMATURELY(h, b) \
    do {                       \
        *table_out = (h);      \
        *words_out = (b);      \
        return FST_ENDS_PREMATURELY; \
    } while (0)
    if (!no_alloc) {
        if (len == 0) return FST_EMPTY;                       // serialize.rs:60-62
        if (len < 8) return FST_FAILED_FILL;                  // read_exact, :458-463
        const uint32_t n32 = ld_u32(p) + 1u;                  // wrapping_add(1)
        if (n32 >= 512u || n32 == 0) return FST_BAD_NSEG;     // :467-473
        nseg = n32;
        total = ld_u32(p + 4);
        if (seg) seg[0] = (uint32_t)total;
        pos = 8;
        if (nseg > 1) {
            const uint64_t rest = nseg < 4 ? 8 : (nseg & ~1ull) * 4;  // :476-496
            if (len - pos < rest) return FST_FAILED_FILL;
            for (uint64_t i = 0; i + 1 < nseg; i++) {
                const uint32_t l = ld_u32(p + pos + 4 * i);
                if (seg) seg[i + 1] = l;
                total += l;
            }
            pos += rest;
        }
        if (has_limit && total > limit) return FST_TOO_LARGE;           // :501-507
        if (total > (len - pos) / 8) ENDS_PREMATURELY(total, (len - pos) / 8);  // :66-70
    } else {
        if (((uintptr_t)p) & 7) return FST_NOT_ALIGNED;                 // :234-248
        if (len < 4) ENDS_PREMATURELY(4, len);                          // read_u32_le
        nseg = (uint64_t)ld_u32(p) + 1;                                 // :268-279
        if (nseg >= 512) return FST_BAD_NSEG;                           // :31-35
        pos = 4;
        for (uint64_t i = 0; i < nseg; i++) {                           // :38-45
            if (len - pos < 4) ENDS_PREMATURELY(4, len - pos);
            const uint32_t l = ld_u32(p + pos);
            if (seg) seg[i] = l;
            total += l;
            pos += 4;
        }
        if (has_limit && total > limit) return FST_TOO_LARGE;           // :50-57
        if (!(nseg & 1)) {                                              // padding :61-63
            if (len - pos < 4) ENDS_PREMATURELY(4, len - pos);
            pos += 4;
        }
        if (len - pos < total * 8) ENDS_PREMATURELY(total, (len - pos) / 8);  // :84-89
    }
#undef ENDS_PREMATURELY
    *nseg_out = (uint32_t)nseg;
    *table_out = pos;
    *words_out = total;
    return FST_OK;
}

__global__ void flat_frame(const uint8_t* __restrict__ buf, const uint64_t* __restrict__ off,
                           uint64_t nmsg, int no_alloc, uint64_t limit, int has_limit,
                           uint64_t* __restrict__ nseg, int32_t* __restrict__ status,
                           uint64_t* __restrict__ body_off, uint64_t* __restrict__ consumed) {
    const uint64_t m = (uint64_t)blockIdx.x * kThreads + threadIdx.x;
    if (m > nmsg) return;
    if (m == nmsg) {
        nseg[m] = 0;
        return;
    }
    const uint64_t a = off[m], b = off[m + 1];
    uint32_t ns = 0;
    uint64_t t = 0, w = 0;
    const int32_t s = flat_table(buf + a, b - a, no_alloc, limit, has_limit, &ns, &t, &w, nullptr);
    const bool ok = s == FST_OK, short_ = s == FST_ENDS_PREMATURELY;
    status[m] = s;
    nseg[m] = ok ? ns : 0;
    // MessageEndsPrematurely(header, body) rides in body_off / consumed
    if (body_off) body_off[m] = ok ? a + t : (short_ ? t : a);
    if (consumed) consumed[m] = ok ? t + 8 * w : (short_ ? w : 0);
}

__global__ void flat_segs(const uint8_t* __restrict__ buf, const uint64_t* __restrict__ off,
                          uint64_t nmsg, int no_alloc, uint64_t limit, int has_limit,
                          const int32_t* __restrict__ status, const uint64_t* __restrict__ sofs,
                          uint32_t* __restrict__ seg) {
    const uint64_t m = (uint64_t)blockIdx.x * kThreads + threadIdx.x;
    if (m >= nmsg || status[m] != FST_OK) return;
    const uint64_t a = off[m], b = off[m + 1];
    uint32_t ns;
    uint64_t t, w;
    flat_table(buf + a, b - a, no_alloc, limit, has_limit, &ns, &t, &w, seg + sofs[m]);
}

}  // namespace

extern "C" hipError_t capnp_launch_msg_frame(const uint8_t* in, const uint64_t* msg_off,
                                             uint64_t nmsg, int try_mode, uint64_t limit,
                                             int has_limit, uint64_t* nseg, uint64_t* words,
                                             int32_t* st, uint64_t* tused, void* tmp,
                                             size_t tmp_bytes, uint64_t* sofs, uint64_t* wofs,
                                             hipStream_t s) {
    const uint32_t g = (uint32_t)((nmsg + 1 + kThreads - 1) / kThreads);
    hipLaunchKernelGGL(msg_frame, dim3(g), dim3(kThreads), 0, s, in, msg_off, nmsg, try_mode,
                       limit, has_limit, nseg, words, st, tused);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    size_t tb = tmp_bytes;
    e = hipcub::DeviceScan::ExclusiveSum(tmp, tb, nseg, sofs, (int)(nmsg + 1), s);
    if (e != hipSuccess) return e;
    tb = tmp_bytes;
    return hipcub::DeviceScan::ExclusiveSum(tmp, tb, words, wofs, (int)(nmsg + 1), s);
}

extern "C" hipError_t capnp_launch_msg_segs(const uint8_t* in, const uint64_t* msg_off,
                                            uint64_t nmsg, int try_mode, uint64_t limit,
                                            int has_limit, const int32_t* st,
                                            const uint64_t* tused, const uint64_t* sofs,
                                            const uint64_t* wofs, uint64_t* seg,
                                            uint64_t* in_off, uint64_t* out_off, hipStream_t s) {
    const uint32_t g = (uint32_t)((nmsg + 1 + kThreads - 1) / kThreads);
    hipLaunchKernelGGL(msg_segs, dim3(g), dim3(kThreads), 0, s, in, msg_off, nmsg, try_mode,
                       limit, has_limit, st, tused, sofs, wofs, seg, in_off, out_off);
    return hipGetLastError();
}

extern "C" hipError_t capnp_launch_msg_status(uint64_t nmsg, const int32_t* tst,
                                              const uint64_t* tused, const int32_t* cst,
                                              const uint64_t* ccons, int32_t* status,
                                              uint64_t* consumed, hipStream_t s) {
    const uint32_t g = (uint32_t)((nmsg + kThreads - 1) / kThreads);
    if (g)
        hipLaunchKernelGGL(msg_status, dim3(g), dim3(kThreads), 0, s, nmsg, tst, tused, cst,
                           ccons, status, consumed);
    return hipGetLastError();
}

extern "C" hipError_t capnp_launch_flat_frame(const uint8_t* buf, const uint64_t* off,
                                              uint64_t nmsg, int no_alloc, uint64_t limit,
                                              int has_limit, uint64_t* nseg, int32_t* status,
                                              uint64_t* body_off, uint64_t* consumed, void* tmp,
                                              size_t tmp_bytes, uint64_t* sofs, hipStream_t s) {
    const uint32_t g = (uint32_t)((nmsg + 1 + kThreads - 1) / kThreads);
    hipLaunchKernelGGL(flat_frame, dim3(g), dim3(kThreads), 0, s, buf, off, nmsg, no_alloc,
                       limit, has_limit, nseg, status, body_off, consumed);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    size_t tb = tmp_bytes;
    return hipcub::DeviceScan::ExclusiveSum(tmp, tb, nseg, sofs, (int)(nmsg + 1), s);
}

extern "C" hipError_t capnp_launch_flat_segs(const uint8_t* buf, const uint64_t* off,
                                             uint64_t nmsg, int no_alloc, uint64_t limit,
                                             int has_limit, const int32_t* status,
                                             const uint64_t* sofs, uint32_t* seg,
                                             hipStream_t s) {
    const uint32_t g = (uint32_t)((nmsg + kThreads - 1) / kThreads);
    if (g)
        hipLaunchKernelGGL(flat_segs, dim3(g), dim3(kThreads), 0, s, buf, off, nmsg, no_alloc,
                           limit, has_limit, status, sofs, seg);
    return hipGetLastError();
}
