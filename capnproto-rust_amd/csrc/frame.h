// frame.h — result record of the device framing kernel (frame.hip).
#pragma once
#include <stdint.h>

struct FrameResult {
    int32_t status;
    uint32_t nseg;
    uint64_t table_consumed;   // packed bytes used by the table read units
    uint64_t total_words;      // body words
    uint64_t table_bytes;      // bytes of the decoded table (no-alloc layout)
    uint64_t body_in_off[2];   // packed range of the body unit (chunk index)
    uint64_t body_out_off[2];  // {0, total_words}
    uint32_t seg_words[512];
    uint8_t table[2064];       // decoded table bytes
};
static_assert(__builtin_offsetof(FrameResult, table) % 8 == 0, "first_unit's 8-byte store");

#ifdef __HIPCC__
// The segment-table read units of serialize_packed::{read_message,
// try_read_message, read_message_no_alloc, try_read_message_no_alloc}
// (serialize_packed.rs:233-291 -> serialize.rs:287-420, 448-510) for one
// lane: frame.hip's kernel, and the single-launch message read
// (unpack.hip msg_read_kernel) over a prefix of the input staged in LDS.
namespace capnp_frame {

enum : int32_t {
    ST_OK = 0, ST_NONE = 1, ST_PREMATURE = 2, ST_NOT_CLEAN = 3, ST_FAILED_FILL = 4,
    ST_EOF = 5, ST_BAD_NSEG = 6, ST_TOO_LARGE = 8, ST_BUF_SMALL = 9,
};

// One PackedRead::read call over in[0..in_len) into out[0..out_len)
// (serialize_packed.rs:80-228 on a slice).  *nread = out_len, or 0 when the
// input was empty at entry (:96-98).
__device__ inline int32_t serial_read(const uint8_t* in, uint64_t in_len, uint8_t* out,
                               uint64_t out_len, uint64_t* used, uint64_t* nread) {
    *used = 0;
    *nread = 0;
    if (out_len == 0) return ST_OK;
    if (in_len == 0) return ST_OK;
    uint64_t ip = 0, op = 0;
    while (op < out_len) {
        if (ip == in_len) return ST_PREMATURE;
        const uint32_t tag = in[ip++];
        for (int k = 0; k < 8; k++) {
            if (tag & (1u << k)) {
                if (ip == in_len) return ST_PREMATURE;
                out[op++] = in[ip++];
            } else {
                out[op++] = 0;
            }
        }
        if (tag == 0 || tag == 0xFF) {
            if (ip == in_len) return ST_PREMATURE;
            const uint64_t run = 8ull * in[ip++];
            if (run > out_len - op) return ST_NOT_CLEAN;
            if (tag == 0) {
                for (uint64_t i = 0; i < run; i++) out[op++] = 0;
            } else {
                if (in_len - ip < run) { *used = in_len; return ST_FAILED_FILL; }
                for (uint64_t i = 0; i < run; i++) out[op++] = in[ip++];
            }
        }
    }
    *used = ip;
    *nread = out_len;
    return ST_OK;
}

// serial_read of the table's first 8-byte unit into out (8-byte aligned) and
// *word, with every byte it may use read up front (independent loads and the
// word built in registers, instead of a dependent chain of byte reads and
// stores; a read_message call spent ~0.8 us in the table, r06q): a tag other
// than 0x00 / 0xFF takes 1 + popcount(tag) bytes and no run.  The others,
// and inputs shorter than 10 bytes, take serial_read.
// (first_word: that fast case alone, in registers; false for the others)
__device__ __forceinline__ bool first_word(const uint8_t* in, uint64_t in_len, uint64_t* word,
                                           uint64_t* used) {
    if (in_len < 10) return false;
    uint32_t b[10];
#pragma unroll
    for (int i = 0; i < 10; i++) b[i] = in[i];
    const uint32_t tag = b[0];
    if (tag == 0u || tag == 0xFFu) return false;
    uint64_t v = 0;  // the unit's non-zero bytes, in order
#pragma unroll
    for (int i = 8; i >= 1; i--) v = (v << 8) | b[i];
    uint64_t x = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) {
        const uint32_t k = __builtin_popcount(tag & ((1u << i) - 1u));
        if ((tag >> i) & 1u) x |= ((v >> (8 * k)) & 0xFFull) << (8 * i);
    }
    *word = x;
    *used = 1u + __builtin_popcount(tag);
    return true;
}

__device__ inline int32_t first_unit(const uint8_t* in, uint64_t in_len, uint8_t* out,
                                     uint64_t* word, uint64_t* used, uint64_t* nread) {
    if (first_word(in, in_len, word, used)) {
        *reinterpret_cast<uint64_t*>(out) = *word;
        *nread = 8;
        return ST_OK;
    }
    const int32_t st = serial_read(in, in_len, out, 8, used, nread);
    *word = *reinterpret_cast<const uint64_t*>(out);
    return st;
}

// read_exact over PackedRead (io.rs:16-31).
__device__ inline int32_t serial_read_exact(const uint8_t* in, uint64_t in_len, uint8_t* out,
                                     uint64_t out_len, uint64_t* used) {
    uint64_t nread = 0;
    const int32_t st = serial_read(in, in_len, out, out_len, used, &nread);
    if (st != ST_OK) return st;
    return nread == out_len ? ST_OK : ST_FAILED_FILL;
}

__device__ __forceinline__ uint32_t le32(const uint8_t* p) {
    return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) |
           ((uint32_t)p[3] << 24);
}

// Reads and validates the table of the message at in[0, in_len) into *r
// (any address space the caller's lane can write).
__device__ inline void frame_table(const uint8_t* __restrict__ in, uint64_t in_len,
                                   uint32_t no_alloc, uint32_t try_mode, uint64_t limit,
                                   uint32_t has_limit, uint64_t buffer_len, uint64_t body_cap,
                                   FrameResult* __restrict__ r) {
    uint8_t* t = r->table;
    // (a chained body unpack reads these: an empty unit unless the table is
    // read and its body fits body_cap words)
    r->body_in_off[0] = r->body_in_off[1] = 0;
    r->body_out_off[0] = r->body_out_off[1] = 0;
    uint64_t used = 0, nread = 0, pos = 0;
    r->nseg = 0;
    r->total_words = 0;
    r->table_bytes = 0;
    r->table_consumed = 0;
    uint64_t w0 = 0;
    int32_t st = first_unit(in, in_len, t, &w0, &used, &nread);
    if (st != ST_OK) { r->status = st; return; }
    if (nread == 0) { r->status = try_mode ? ST_NONE : ST_EOF; return; }
    pos += used;
    const uint32_t nseg = (uint32_t)w0 + 1u;
    if (nseg >= 512u || nseg == 0) { r->status = ST_BAD_NSEG; return; }
    uint64_t total = (uint32_t)(w0 >> 32);
    r->seg_words[0] = (uint32_t)(w0 >> 32);
    uint64_t start;
    if (!no_alloc) {
        // serialize.rs:476-496: the rest of the table is ONE read unit
        if (nseg > 1) {
            const uint64_t rest = nseg < 4 ? 8 : (uint64_t)(nseg & ~1u) * 4;
            st = serial_read_exact(in + pos, in_len - pos, t + 8, rest, &used);
            if (st != ST_OK) { r->status = st; return; }
            pos += used;
            for (uint32_t i = 0; i + 1 < nseg; i++) {
                const uint32_t l = le32(t + 8 + 4 * i);
                r->seg_words[i + 1] = l;
                total += l;
            }
        }
        start = 8;
    } else {
        // serialize.rs:371-395: 8 bytes at a time into buffer[(k+1)*4 ..]
        uint32_t k = 1;
        while (k < nseg) {
            const uint64_t s0 = (uint64_t)(k + 1) * 4, e0 = s0 + 8;
            if (buffer_len < e0) { r->status = ST_BUF_SMALL; return; }
            st = serial_read_exact(in + pos, in_len - pos, t + s0, 8, &used);
            if (st != ST_OK) { r->status = st; return; }
            pos += used;
            r->seg_words[k] = le32(t + s0);
            total += le32(t + s0);
            k++;
            if (k < nseg) { r->seg_words[k] = le32(t + s0 + 4); total += le32(t + s0 + 4); }
            k++;
        }
        start = (uint64_t)(k + 1) * 4;
    }
    if (has_limit && total > limit) { r->status = ST_TOO_LARGE; return; }
    if (no_alloc && buffer_len < start + total * 8) { r->status = ST_BUF_SMALL; return; }
    r->nseg = nseg;
    r->total_words = total;
    r->table_bytes = start;
    r->table_consumed = pos;
    r->body_in_off[0] = pos;
    r->body_in_off[1] = in_len;
    r->body_out_off[0] = 0;
    r->body_out_off[1] = total <= body_cap ? total : 0;
    r->status = ST_OK;
}

}  // namespace capnp_frame
#endif
