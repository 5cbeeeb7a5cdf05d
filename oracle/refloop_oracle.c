/*
 * refloop_oracle.c — the reference's CPU codec with its own loop shapes, for
 * timing (bench.py's cpu_baseline leg).
 *
 * TEST INFRASTRUCTURE ONLY, like packed_oracle.c: only tests/ and bench.py's
 * cpu_baseline leg load it.  The product library never links or calls it.
 *
 * packed_oracle.c is the parity oracle: it branches per byte, which is easy
 * to check against the reference's error paths but runs ~3x slower than the
 * reference's own loops.  This file restates the same transform the way the
 * reference executes it, so that the CPU baseline times the reference's
 * algorithm:
 *   - pack (PackedWrite::write_all, capnp/src/serialize_packed.rs:304-439):
 *     a 64-byte staging buffer flushed when fewer than 10 bytes are free
 *     (:313-319) and before a literal run's raw words (:429-432); per word,
 *     eight branch-free steps "store the byte, advance by its non-zero bit"
 *     (:324-362), the tag assembled from the bits (:364-373); a zero run
 *     counted by whole-word compares (:380-393); a literal run by counting
 *     zero bytes per word and un-reading the word with two (:403-423);
 *   - unpack (PackedRead::read, :80-228) over a `&[u8]` BufRead (io.rs:178-
 *     186: fill_buf returns every remaining byte): the fast path while >= 10
 *     input bytes remain (:146-156: eight masked stores, advance by the bit),
 *     the byte-checked slow path below that (:109-145), `write_bytes` for a
 *     zero run (:172) and `copy_nonoverlapping` for a literal run (:192);
 *   - write_message / read_message of one-segment messages for config 1
 *     (serialize.rs:574-679, :287-325, :448-524): read_message's
 *     allocate_zeroed_vec of the body (serialize.rs:248-254) is the memset
 *     before the body read.
 * Sinks are `&mut [u8]` (io.rs:127-139: a memcpy and a bounds check).
 * tests/test_refloop.py checks every output byte, status and consumed count
 * against packed_oracle.c (and so against the reference's golden vectors).
 */
#include <stdint.h>
#include <stddef.h>
#include <string.h>
#include <pthread.h>

#include "../include/capnp_packed.h"

typedef struct {
    uint8_t* p;
    size_t cap, len;
    int err;
} slice_w; /* impl Write for &mut [u8] (io.rs:127-139) */

static inline void sw_write(slice_w* s, const uint8_t* b, size_t n) {
    if (n > s->cap - s->len) { s->err = CAPNP_E_BUFFER_NOT_LARGE_ENOUGH; return; }
    memcpy(s->p + s->len, b, n);
    s->len += n;
}

/* serialize_packed.rs:304-439 */
static int ref_write_all(slice_w* s, const uint8_t* in, size_t len) {
    uint8_t buf[64 + 8];
    size_t bi = 0;
    const uint8_t* p = in;
    const uint8_t* end = in + len;
    while (p < end) {
        if (bi + 10 > 64) { /* :313-319 */
            sw_write(s, buf, bi);
            bi = 0;
        }
        const size_t tag_pos = bi++;
        uint8_t b, tag = 0;
#define STEP(k)                        \
        b = p[k];                      \
        buf[bi] = b;                   \
        bi += (b != 0);                \
        tag |= (uint8_t)((b != 0) << k);
        STEP(0) STEP(1) STEP(2) STEP(3) STEP(4) STEP(5) STEP(6) STEP(7)
#undef STEP
        p += 8;
        buf[tag_pos] = tag; /* :373 */
        if (tag == 0) { /* :375-393 */
            const uint8_t* w = p;
            const uint8_t* lim = (size_t)(end - w) / 8 > 255 ? w + 8 * 255 : end;
            while (w < lim) {
                uint64_t v;
                memcpy(&v, w, 8);
                if (v != 0) break;
                w += 8;
            }
            buf[bi++] = (uint8_t)((size_t)(w - p) / 8);
            p = w;
        } else if (tag == 0xFF) { /* :394-433 */
            const uint8_t* run = p;
            const uint8_t* lim = (size_t)(end - p) > 255 * 8 ? p + 255 * 8 : end;
            while (p < lim) {
                int c = 0;
                for (int k = 0; k < 8; k++) c += (p[k] == 0);
                p += 8;
                if (c >= 2) { p -= 8; break; }
            }
            const size_t count = (size_t)(p - run);
            buf[bi++] = (uint8_t)(count / 8);
            sw_write(s, buf, bi);
            bi = 0;
            sw_write(s, run, count);
        }
    }
    sw_write(s, buf, bi); /* :436 */
    return s->err;
}

/* PackedRead::read over a &[u8] (serialize_packed.rs:80-228).  Returns the
 * status; *consumed as packed_oracle.c's oracle_read reports it (the
 * reference's consume() calls on the slice). */
static int ref_read(const uint8_t* in, size_t in_len, size_t* consumed, uint8_t* outb,
                    size_t out_len, size_t* nread) {
    *nread = 0;
    *consumed = 0;
    if (out_len == 0) return CAPNP_OK;
    if (out_len % 8) return CAPNP_E_MISALIGNED_LEN;
    if (in_len == 0) return CAPNP_OK;
    const uint8_t* ip = in;
    const uint8_t* ie = in + in_len;
    uint8_t* out = outb;
    uint8_t* oe = outb + out_len;
    for (;;) {
        uint8_t tag;
        if ((size_t)(ie - ip) < 10) {
            if (ip == ie) { *consumed = in_len; return CAPNP_E_PREMATURE_END_OF_PACKED_INPUT; }
            tag = *ip++; /* :118-141 */
            for (int i = 0; i < 8; i++) {
                if (tag & (1u << i)) {
                    if (ip == ie) { *consumed = in_len; return CAPNP_E_PREMATURE_END_OF_PACKED_INPUT; }
                    *out++ = *ip++;
                } else {
                    *out++ = 0;
                }
            }
            if (ip == ie && (tag == 0 || tag == 0xFF)) { /* :143-145 */
                *consumed = in_len;
                return CAPNP_E_PREMATURE_END_OF_PACKED_INPUT;
            }
        } else {
            tag = *ip++; /* :147-155 */
            for (int n = 0; n < 8; n++) {
                const uint8_t nz = (uint8_t)((tag >> n) & 1u);
                *out++ = (uint8_t)(*ip & (uint8_t)(-(int8_t)nz));
                ip += nz;
            }
        }
        if (tag == 0) { /* :157-173 */
            const size_t run = (size_t)(*ip++) * 8;
            if (run > (size_t)(oe - out)) return CAPNP_E_DID_NOT_END_CLEANLY;
            memset(out, 0, run);
            out += run;
        } else if (tag == 0xFF) { /* :174-219 */
            const size_t run = (size_t)(*ip++) * 8;
            if (run > (size_t)(oe - out)) return CAPNP_E_DID_NOT_END_CLEANLY;
            const size_t rem = (size_t)(ie - ip);
            if (rem >= run) {
                memcpy(out, ip, run);
                out += run;
                ip += run;
            } else { /* the slice holds no more: read_exact fails (io.rs:26-28) */
                memcpy(out, ip, rem);
                *consumed = in_len;
                return CAPNP_E_FAILED_TO_FILL_WHOLE_BUFFER;
            }
        }
        if (out == oe) { /* :222-225 */
            *consumed = (size_t)(ip - in);
            *nread = out_len;
            return CAPNP_OK;
        }
    }
}

int refloop_pack(const uint8_t* in, size_t len, uint8_t* out, size_t cap, size_t* written) {
    if (len % 8) return CAPNP_E_MISALIGNED_LEN;
    slice_w s = {out, cap, 0, 0};
    int st = ref_write_all(&s, in, len);
    *written = s.len;
    return st;
}

int refloop_read_exact(const uint8_t* in, size_t in_len, size_t* consumed, uint8_t* out,
                       size_t out_len) {
    size_t nread = 0;
    int st = ref_read(in, in_len, consumed, out, out_len, &nread);
    if (st != CAPNP_OK) return st;
    return nread == out_len ? CAPNP_OK : CAPNP_E_FAILED_TO_FILL_WHOLE_BUFFER; /* io.rs:16-31 */
}

/* ---- batch drivers: contiguous chunk ranges on POSIX threads ---------------
 * Thread t packs chunks [c0, c1) back to back into its own region
 * out[region[t], region[t + 1]) (the caller sizes the regions with the bound
 * and maps their pages before timing); pos[c] / size[c] = where chunk c's
 * bytes went.  Unpack reads them back from pos / size. */
typedef struct {
    const uint64_t* words;
    const uint64_t* offs;
    uint8_t* out;
    const uint64_t* region;
    uint64_t* pos;
    uint64_t* size;
    const uint8_t* packed;
    uint64_t* back;
    int32_t* status;
    size_t c0, c1;
    int t, mode, err;
} job;

static void* worker(void* arg) {
    job* j = (job*)arg;
    if (j->mode == 0) {
        slice_w s = {j->out + j->region[j->t], j->region[j->t + 1] - j->region[j->t], 0, 0};
        for (size_t c = j->c0; c < j->c1; c++) {
            const size_t at = s.len;
            ref_write_all(&s, (const uint8_t*)(j->words + j->offs[c]),
                          (size_t)(j->offs[c + 1] - j->offs[c]) * 8);
            j->pos[c] = j->region[j->t] + at;
            j->size[c] = s.len - at;
        }
        j->err = s.err;
    } else {
        for (size_t c = j->c0; c < j->c1; c++) {
            size_t used = 0;
            j->status[c] = refloop_read_exact(j->packed + j->pos[c], (size_t)j->size[c], &used,
                                              (uint8_t*)(j->back + j->offs[c]),
                                              (size_t)(j->offs[c + 1] - j->offs[c]) * 8);
        }
    }
    return NULL;
}

static int run(job proto, size_t n, int threads) {
    if (threads < 1) threads = 1;
    if (threads > 256) threads = 256;
    pthread_t th[256];
    job jobs[256];
    int err = 0;
    for (int t = 0; t < threads; t++) {
        jobs[t] = proto;
        jobs[t].t = t;
        jobs[t].c0 = n * (size_t)t / (size_t)threads;
        jobs[t].c1 = n * (size_t)(t + 1) / (size_t)threads;
        if (threads == 1) worker(&jobs[t]);
        else pthread_create(&th[t], NULL, worker, &jobs[t]);
    }
    for (int t = 0; t < threads; t++) {
        if (threads > 1) pthread_join(th[t], NULL);
        if (jobs[t].err) err = jobs[t].err;
    }
    return err;
}

/* region[threads + 1]: thread t's output range (bound of its chunks). */
int refloop_pack_batch(const uint64_t* words, const uint64_t* offs, size_t n, uint8_t* out,
                       const uint64_t* region, uint64_t* pos, uint64_t* size, int threads) {
    job p;
    memset(&p, 0, sizeof p);
    p.words = words; p.offs = offs; p.out = out; p.region = region; p.pos = pos; p.size = size;
    p.mode = 0;
    return run(p, n, threads);
}

int refloop_unpack_batch(const uint8_t* packed, const uint64_t* pos, const uint64_t* size,
                         size_t n, uint64_t* back, const uint64_t* offs, int32_t* status,
                         int threads) {
    job p;
    memset(&p, 0, sizeof p);
    p.packed = packed; p.pos = (uint64_t*)pos; p.size = (uint64_t*)size; p.back = back;
    p.offs = offs; p.status = status; p.mode = 1;
    return run(p, n, threads);
}

/* ---- config 1: one-segment messages (benchmark.rs:235-241) ---------------- */
static void put_u32(uint8_t* p, uint32_t v) { memcpy(p, &v, 4); }

/* serialize_packed::write_message -> serialize::write_message (serialize.rs:
 * 574-679) for one segment: word 0 as one write_all, then the segment. */
int refloop_write_message1(const uint64_t* seg, uint32_t nwords, uint8_t* out, size_t cap,
                           size_t* written) {
    slice_w s = {out, cap, 0, 0};
    uint8_t w0[8];
    put_u32(w0, 0);
    put_u32(w0 + 4, nwords);
    ref_write_all(&s, w0, 8);
    ref_write_all(&s, (const uint8_t*)seg, (size_t)nwords * 8);
    *written = s.len;
    return s.err;
}

/* serialize_packed::read_message (serialize.rs:287-325, :448-524) of a
 * one-segment message: read(8), the table checks, the zeroed body
 * (allocate_zeroed_vec, :248-254), read_exact(body). */
int refloop_read_message1(const uint8_t* in, size_t in_len, uint64_t* body, size_t body_cap,
                          uint32_t* nwords) {
    uint8_t w0[8];
    size_t c = 0, nread = 0, used = 0;
    int st = ref_read(in, in_len, &c, w0, 8, &nread);
    if (st != CAPNP_OK) return st;
    if (nread == 0) return CAPNP_E_PREMATURE_END_OF_FILE;
    used = c;
    uint32_t u0, len;
    memcpy(&u0, w0, 4);
    memcpy(&len, w0 + 4, 4);
    if (u0 + 1u != 1u) return CAPNP_E_INVALID_ARGUMENT; /* (config 1 writes one segment) */
    if (len > (8u << 20)) return CAPNP_E_MESSAGE_TOO_LARGE; /* traversal limit, :501-507 */
    if (len > body_cap) return CAPNP_E_BUFFER_NOT_LARGE_ENOUGH;
    memset(body, 0, (size_t)len * 8);
    *nwords = len;
    return len ? refloop_read_exact(in + used, in_len - used, &c, (uint8_t*)body, (size_t)len * 8)
               : CAPNP_OK;
}

typedef struct {
    const uint64_t* words;
    const uint64_t* msg_off;
    uint8_t* out;
    const uint64_t* slot;
    uint64_t* sizes;
    uint64_t* body;
    int32_t* status;
    size_t m0, m1;
    int mode;
} mjob;

static void* mworker(void* arg) {
    mjob* j = (mjob*)arg;
    for (size_t m = j->m0; m < j->m1; m++) {
        const uint64_t a = j->msg_off[m], b = j->msg_off[m + 1];
        if (j->mode == 0) {
            size_t wr = 0;
            j->status[m] = refloop_write_message1(j->words + a, (uint32_t)(b - a),
                                                  j->out + j->slot[m],
                                                  (size_t)(j->slot[m + 1] - j->slot[m]), &wr);
            j->sizes[m] = wr;
        } else {
            uint32_t nw = 0;
            j->status[m] = refloop_read_message1(j->out + j->slot[m], (size_t)j->sizes[m],
                                                 j->body + a, (size_t)(b - a), &nw);
        }
    }
    return NULL;
}

static void mrun(mjob proto, size_t n, int threads) {
    if (threads < 1) threads = 1;
    if (threads > 256) threads = 256;
    pthread_t th[256];
    mjob jobs[256];
    for (int t = 0; t < threads; t++) {
        jobs[t] = proto;
        jobs[t].m0 = n * (size_t)t / (size_t)threads;
        jobs[t].m1 = n * (size_t)(t + 1) / (size_t)threads;
        if (threads == 1) mworker(&jobs[t]);
        else pthread_create(&th[t], NULL, mworker, &jobs[t]);
    }
    if (threads > 1)
        for (int t = 0; t < threads; t++) pthread_join(th[t], NULL);
}

int refloop_write_messages_mt(const uint64_t* words, const uint64_t* msg_off, size_t n,
                              uint8_t* out, const uint64_t* slot, uint64_t* sizes,
                              int32_t* status, int threads) {
    mjob p = {words, msg_off, out, slot, sizes, NULL, status, 0, 0, 0};
    mrun(p, n, threads);
    return CAPNP_OK;
}

int refloop_read_messages_mt(const uint8_t* packed, const uint64_t* slot, const uint64_t* sizes,
                             size_t n, uint64_t* body, const uint64_t* msg_off, int32_t* status,
                             int threads) {
    mjob p = {NULL, msg_off, (uint8_t*)packed, slot, (uint64_t*)sizes, body, status, 0, 0, 1};
    mrun(p, n, threads);
    return CAPNP_OK;
}
