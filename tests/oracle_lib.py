"""ctypes wrapper of the CPU oracle (oracle/build/liboracle.so).

Test infrastructure: imported only by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg.
"""
import ctypes as C
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")
LIB_PATH = os.path.join(ORACLE_DIR, "build", "liboracle.so")

STATUS = {
    "OK": 0, "NONE": 1, "PREMATURE_END_OF_PACKED_INPUT": 2, "DID_NOT_END_CLEANLY": 3,
    "FAILED_TO_FILL_WHOLE_BUFFER": 4, "PREMATURE_END_OF_FILE": 5,
    "INVALID_NUMBER_OF_SEGMENTS": 6, "MESSAGE_SIZE_OVERFLOW": 7, "MESSAGE_TOO_LARGE": 8,
    "BUFFER_NOT_LARGE_ENOUGH": 9, "UNALIGNED_SEGMENT": 10, "MISALIGNED_LEN": 11,
}
DEFAULT_TRAVERSAL_LIMIT = 8 * 1024 * 1024  # message.rs:117-120

_lib = None


def build():
    subprocess.check_call(["make", "-s", "-C", ORACLE_DIR])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = C.CDLL(LIB_PATH)
        u8p, u64p, szp = C.POINTER(C.c_uint8), C.POINTER(C.c_uint64), C.POINTER(C.c_size_t)
        L.oracle_pack.argtypes = [C.c_void_p, C.c_size_t, C.c_void_p, C.c_size_t, szp]
        L.oracle_read.argtypes = [C.c_void_p, C.c_size_t, szp, C.c_void_p, C.c_size_t, szp]
        L.oracle_read_exact.argtypes = [C.c_void_p, C.c_size_t, szp, C.c_void_p, C.c_size_t]
        L.oracle_bound.argtypes = [C.c_size_t]
        L.oracle_bound.restype = C.c_size_t
        L.oracle_write_message.argtypes = [C.c_void_p, C.c_void_p, C.c_uint32, C.c_void_p,
                                           C.c_size_t, szp]
        L.oracle_read_message.argtypes = [C.c_void_p, C.c_size_t, C.c_uint64, C.c_int, C.c_int,
                                          C.c_void_p, C.c_size_t, C.c_void_p,
                                          C.POINTER(C.c_uint32), szp]
        L.oracle_read_message_no_alloc.argtypes = [C.c_void_p, C.c_size_t, C.c_uint64, C.c_int,
                                                   C.c_int, C.c_void_p, C.c_size_t,
                                                   C.POINTER(C.c_uint32), szp, szp, szp]
        L.oracle_read_flat_message.argtypes = [C.c_void_p, C.c_size_t, C.c_uint64, C.c_int,
                                               C.c_int, C.c_void_p, C.POINTER(C.c_uint32),
                                               szp, szp]
        L.oracle_pack_batch.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p,
                                        C.c_size_t, C.c_void_p, C.c_int]
        L.oracle_unpack_batch.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p,
                                          C.c_void_p, C.c_void_p, C.c_void_p, C.c_int]
        L.oracle_sync_index.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_size_t,
                                        C.c_void_p]
        L.oracle_sync_words.restype = C.c_size_t
        L.gen_word.argtypes = [C.c_int, C.c_uint32, C.c_uint64, C.c_uint64]
        L.gen_word.restype = C.c_uint64
        L.gen_fill.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_size_t, C.c_uint64,
                               C.c_void_p, C.c_int, C.c_uint32]
        L.oracle_write_messages_mt.argtypes = [
            C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
            C.c_int]
        L.oracle_read_messages_mt.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_size_t,
                                              C.c_void_p, C.c_void_p, C.c_void_p, C.c_int]
        L.carsales_seed.argtypes = [C.c_void_p]
        L.carsales_request.argtypes = [C.c_void_p, C.c_void_p, C.POINTER(C.c_uint64)]
        L.carsales_request.restype = C.c_size_t
        L.carsales_value.argtypes = [C.c_void_p, C.c_size_t]
        L.carsales_value.restype = C.c_uint64
        L.carsales_stream.argtypes = [C.c_void_p, C.c_uint64, C.c_void_p, C.c_uint64,
                                      C.c_void_p, C.c_size_t]
        L.carsales_stream.restype = C.c_size_t
        # oracle/refloop_oracle.c: the reference's own loop shapes (timing)
        L.refloop_pack.argtypes = [C.c_void_p, C.c_size_t, C.c_void_p, C.c_size_t, szp]
        L.refloop_read_exact.argtypes = [C.c_void_p, C.c_size_t, szp, C.c_void_p, C.c_size_t]
        L.refloop_pack_batch.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p,
                                         C.c_void_p, C.c_void_p, C.c_void_p, C.c_int]
        L.refloop_unpack_batch.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_size_t,
                                           C.c_void_p, C.c_void_p, C.c_void_p, C.c_int]
        L.refloop_write_messages_mt.argtypes = L.oracle_write_messages_mt.argtypes
        L.refloop_read_messages_mt.argtypes = L.oracle_read_messages_mt.argtypes
        _lib = L
    return _lib


def _buf(b):
    a = np.frombuffer(bytes(b), dtype=np.uint8) if not isinstance(b, np.ndarray) else b
    return np.ascontiguousarray(a)


def pack(data):
    """PackedWrite::write_all of one chunk -> (status, bytes)."""
    a = _buf(data)
    cap = lib().oracle_bound(len(a) // 8) + 16
    out = np.zeros(cap, np.uint8)
    n = C.c_size_t(0)
    st = lib().oracle_pack(a.ctypes.data, len(a), out.ctypes.data, cap, C.byref(n))
    return st, out[:n.value].tobytes()


def read_exact(packed, out_len):
    """read_exact over PackedRead -> (status, bytes, consumed)."""
    a = _buf(packed)
    out = np.zeros(max(out_len, 1), np.uint8)
    used = C.c_size_t(0)
    st = lib().oracle_read_exact(a.ctypes.data if len(a) else None, len(a), C.byref(used),
                                 out.ctypes.data, out_len)
    return st, out[:out_len].tobytes(), used.value


def read(packed, out_len):
    a = _buf(packed)
    out = np.zeros(max(out_len, 1), np.uint8)
    used, nread = C.c_size_t(0), C.c_size_t(0)
    st = lib().oracle_read(a.ctypes.data if len(a) else None, len(a), C.byref(used),
                           out.ctypes.data, out_len, C.byref(nread))
    return st, out[:out_len].tobytes(), used.value, nread.value


def write_message(segments):
    """segments: list of np.uint64 arrays -> (status, packed bytes)."""
    words = np.concatenate([np.asarray(s, np.uint64) for s in segments]) if segments else \
        np.zeros(0, np.uint64)
    words = np.ascontiguousarray(words)
    lens = np.array([len(s) for s in segments], np.uint32)
    cap = 16 + sum(lib().oracle_bound(int(n)) for n in lens) + lib().oracle_bound(
        len(segments) // 2 + 1)
    out = np.zeros(cap, np.uint8)
    n = C.c_size_t(0)
    st = lib().oracle_write_message(words.ctypes.data if len(words) else None,
                                    lens.ctypes.data, len(segments), out.ctypes.data, cap,
                                    C.byref(n))
    return st, out[:n.value].tobytes()


def read_message(packed, try_mode=False, limit=DEFAULT_TRAVERSAL_LIMIT, body_cap=None):
    """-> (status, [segments as np.uint64 arrays], consumed)."""
    a = _buf(packed)
    grow = body_cap is None  # (a packed byte can stand for up to 128 words)
    if body_cap is None:
        body_cap = max(8 * len(a) + 8, 1)
    while True:
        body = np.zeros(body_cap, np.uint64)
        seg = np.zeros(512, np.uint32)
        nseg, used = C.c_uint32(0), C.c_size_t(0)
        st = lib().oracle_read_message(a.ctypes.data if len(a) else None, len(a),
                                       limit if limit is not None else 0, limit is not None,
                                       int(try_mode), body.ctypes.data, body_cap,
                                       seg.ctypes.data, C.byref(nseg), C.byref(used))
        if st == 9 and grow and body_cap < 128 * len(a) + 8:
            body_cap = min(4 * body_cap, 128 * len(a) + 8)
            continue
        break
    segs = []
    if st == 0:
        o = 0
        for i in range(nseg.value):
            segs.append(body[o:o + seg[i]].copy())
            o += int(seg[i])
    return st, segs, used.value


def read_message_no_alloc(packed, buffer_words, try_mode=False, limit=DEFAULT_TRAVERSAL_LIMIT):
    a = _buf(packed)
    buf = np.zeros(max(buffer_words, 1), np.uint64)
    nseg, tb, bb, used = C.c_uint32(0), C.c_size_t(0), C.c_size_t(0), C.c_size_t(0)
    st = lib().oracle_read_message_no_alloc(a.ctypes.data if len(a) else None, len(a),
                                            limit if limit is not None else 0,
                                            limit is not None, int(try_mode), buf.ctypes.data,
                                            buffer_words * 8, C.byref(nseg), C.byref(tb),
                                            C.byref(bb), C.byref(used))
    return st, buf.view(np.uint8), nseg.value, tb.value, bb.value, used.value


def pack_batch(words, offs, threads=1):
    words = np.ascontiguousarray(words, np.uint64)
    offs = np.ascontiguousarray(offs, np.uint64)
    n = len(offs) - 1
    cap = int(sum(lib().oracle_bound(int(x)) for x in np.diff(offs))) if n < 4096 else \
        int(8 * int(offs[-1]) + (int(offs[-1]) + 1) // 2 + 2 * n + 64)
    out = np.zeros(max(cap, 1), np.uint8)
    out_offs = np.zeros(n + 1, np.uint64)
    st = lib().oracle_pack_batch(words.ctypes.data, offs.ctypes.data, n, out.ctypes.data, cap,
                                 out_offs.ctypes.data, threads)
    return st, out[:int(out_offs[-1])], out_offs


def unpack_batch(packed, in_offs, out_offs, threads=1):
    packed = np.ascontiguousarray(packed, np.uint8)
    in_offs = np.ascontiguousarray(in_offs, np.uint64)
    out_offs = np.ascontiguousarray(out_offs, np.uint64)
    n = len(in_offs) - 1
    words = np.zeros(max(int(out_offs[-1]), 1), np.uint64)
    status = np.zeros(n, np.int32)
    consumed = np.zeros(n, np.uint64)
    lib().oracle_unpack_batch(packed.ctypes.data, in_offs.ctypes.data, n, words.ctypes.data,
                              out_offs.ctypes.data, status.ctypes.data, consumed.ctypes.data,
                              threads)
    return words[:int(out_offs[-1])], status, consumed


def sync_index(packed, in_offs, out_offs):
    """Record sync index of a cleanly packed batch (oracle_sync_index)."""
    packed = np.ascontiguousarray(packed, np.uint8)
    in_offs = np.ascontiguousarray(in_offs, np.uint64)
    out_offs = np.ascontiguousarray(out_offs, np.uint64)
    n = len(in_offs) - 1
    ne = -(-int(out_offs[-1]) // sync_words())
    sync = np.full(max(ne, 1), 0xFFFFFFFF, np.uint32)
    r = lib().oracle_sync_index(packed.ctypes.data, in_offs.ctypes.data, out_offs.ctypes.data,
                                n, sync.ctypes.data)
    assert r == 0, "batch does not decode cleanly"
    return sync[:ne]


def sync_words():
    return int(lib().oracle_sync_words())


PZ30 = 1288490189  # round(0.30 * 2**32)
PZ80 = 3435973837  # round(0.80 * 2**32)


def gen_fill(offs, kinds=None, kind0=0, pz=PZ30, id0=0):
    offs = np.ascontiguousarray(offs, np.uint64)
    n = len(offs) - 1
    words = np.zeros(max(int(offs[-1]), 1), np.uint64)
    k = None
    if kinds is not None:
        k = np.ascontiguousarray(kinds, np.uint8)
    lib().gen_fill(words.ctypes.data, offs.ctypes.data, 0, n, id0,
                   k.ctypes.data if k is not None else None, kind0, pz)
    return words[:int(offs[-1])]


def read_flat_message(buf, off, length, no_alloc=False, limit=DEFAULT_TRAVERSAL_LIMIT):
    """serialize::read_message_from_flat_slice(_no_alloc) on buf[off:off+length]
    (buf an 8-byte aligned np.uint8 array, so off % 8 is the slice's
    alignment).  -> (status, [segment lengths], table_bytes, consumed)."""
    seg = np.zeros(512, np.uint32)
    nseg, tb, used = C.c_uint32(0), C.c_size_t(0), C.c_size_t(0)
    st = lib().oracle_read_flat_message(buf.ctypes.data + off, length,
                                        limit if limit is not None else 0, limit is not None,
                                        int(no_alloc), seg.ctypes.data, C.byref(nseg),
                                        C.byref(tb), C.byref(used))
    return st, [int(x) for x in seg[:nseg.value]], tb.value, used.value


# ---- carsales (oracle/carsales_oracle.c; BASELINE.json configs[0]) --------

CARSALES_MAX_WORDS = 3 + 15 * 199


def carsales_seed():
    """FastRand's default state (benchmark/common.rs:30-39) as uint32[4]."""
    st = np.zeros(4, np.uint32)
    lib().carsales_seed(st.ctypes.data)
    return st


def carsales_request(st):
    """setup_request on the chain state `st` (advanced in place) ->
    (request segment words, expected total value)."""
    seg = np.zeros(CARSALES_MAX_WORDS, np.uint64)
    exp = C.c_uint64(0)
    nw = lib().carsales_request(st.ctypes.data, seg.ctypes.data, C.byref(exp))
    return seg[:nw].copy(), exp.value


def carsales_value(seg):
    seg = np.ascontiguousarray(seg, np.uint64)
    return int(lib().carsales_value(seg.ctypes.data, len(seg)))


def carsales_stream(target_words, skip=0, st=None, max_msgs=None):
    """Request segments of the benchmark's chain back to back, cut at
    target_words -> (words, msg_off[nmsgs + 1], state after)."""
    if st is None:
        st = carsales_seed()
    if max_msgs is None:
        max_msgs = target_words // 3 + 2
    words = np.zeros(max(target_words, 1), np.uint64)
    offs = np.zeros(max_msgs + 1, np.uint64)
    m = lib().carsales_stream(st.ctypes.data, skip, words.ctypes.data, target_words,
                              offs.ctypes.data, max_msgs)
    return words[:target_words], offs[:m + 1], st


def messages_roundtrip_mt(words, msg_off, threads=1):
    """One-segment messages words[msg_off[m]:msg_off[m+1]] through
    write_message then read_message (the carsales benchmark's codec calls) on
    `threads` threads -> (seconds write, seconds read, packed bytes, ok)."""
    import time
    words = np.ascontiguousarray(words, np.uint64)
    msg_off = np.ascontiguousarray(msg_off, np.uint64)
    n = len(msg_off) - 1
    lens = np.diff(msg_off).astype(np.int64)
    slot = np.zeros(n + 1, np.uint64)
    slot[1:] = np.cumsum(8 * lens + (lens + 1) // 2 + 48)
    out = np.zeros(int(slot[-1]) + 16, np.uint8)
    sizes = np.zeros(n, np.uint64)
    st = np.zeros(n, np.int32)
    body = np.zeros(max(int(msg_off[-1]), 1), np.uint64)
    out.fill(1)   # map the pages before the timed region
    body.fill(1)
    t0 = time.perf_counter()
    lib().oracle_write_messages_mt(words.ctypes.data, msg_off.ctypes.data, n, out.ctypes.data,
                                   slot.ctypes.data, sizes.ctypes.data, st.ctypes.data, threads)
    t1 = time.perf_counter()
    ok = bool((st == 0).all())
    lib().oracle_read_messages_mt(out.ctypes.data, slot.ctypes.data, sizes.ctypes.data, n,
                                  body.ctypes.data, msg_off.ctypes.data, st.ctypes.data, threads)
    t2 = time.perf_counter()
    ok = ok and bool((st == 0).all()) and np.array_equal(body[:len(words)], words)
    return t1 - t0, t2 - t1, int(sizes.sum()), ok


# ---- the reference's loop shapes (oracle/refloop_oracle.c): the timed CPU
# baseline.  Outputs are allocated and their pages mapped before the clock
# starts; bytes are checked against the parity oracle by the caller.

def refloop_pack(data):
    a = _buf(data)
    cap = lib().oracle_bound(len(a) // 8) + 16
    out = np.zeros(cap, np.uint8)
    n = C.c_size_t(0)
    st = lib().refloop_pack(a.ctypes.data, len(a), out.ctypes.data, cap, C.byref(n))
    return st, out[:n.value].tobytes()


def refloop_read_exact(packed, out_len):
    a = _buf(packed)
    out = np.zeros(max(out_len, 1), np.uint8)
    used = C.c_size_t(0)
    st = lib().refloop_read_exact(a.ctypes.data if len(a) else None, len(a), C.byref(used),
                                  out.ctypes.data, out_len)
    return st, out[:out_len].tobytes(), used.value


class RefloopBatch:
    """Chunk-level pack + unpack of one batch on `threads` threads with the
    reference's loops: each thread packs its contiguous chunk range into its
    own output region (one independent write_all per chunk, as the
    reference's callers do per segment), then reads every chunk back with
    read_exact.  All buffers are allocated and mapped here, outside any timed
    region; pack() and unpack() are what the caller times."""

    def __init__(self, words, offs, threads):
        self.words = np.ascontiguousarray(words, np.uint64)
        self.offs = np.ascontiguousarray(offs, np.uint64)
        self.n = len(self.offs) - 1
        self.threads = max(1, int(threads))
        t = self.threads
        cuts = [self.n * i // t for i in range(t + 1)]
        w = self.offs[cuts].astype(np.int64)
        nw = np.diff(w)
        nc = np.diff(np.array(cuts, np.int64))
        bound = 8 * nw + (nw + 1) // 2 + 2 * nc + 64  # >= the sum of the chunks' bounds
        self.region = np.concatenate([[0], np.cumsum(bound)]).astype(np.uint64)
        self.out = np.ones(int(self.region[-1]) + 16, np.uint8)  # (ones: pages mapped)
        self.pos = np.ones(self.n, np.uint64)
        self.size = np.ones(self.n, np.uint64)
        self.back = np.ones(max(int(self.offs[-1]), 1), np.uint64)
        self.status = np.ones(self.n, np.int32)

    def pack(self):
        return lib().refloop_pack_batch(self.words.ctypes.data, self.offs.ctypes.data, self.n,
                                        self.out.ctypes.data, self.region.ctypes.data,
                                        self.pos.ctypes.data, self.size.ctypes.data,
                                        self.threads)

    def unpack(self):
        return lib().refloop_unpack_batch(self.out.ctypes.data, self.pos.ctypes.data,
                                          self.size.ctypes.data, self.n, self.back.ctypes.data,
                                          self.offs.ctypes.data, self.status.ctypes.data,
                                          self.threads)

    def packed_stream(self):
        """The chunks' packed bytes concatenated in chunk order (the stream
        successive write_all calls produce) and its byte offsets."""
        parts = [self.out[int(p):int(p) + int(s)] for p, s in zip(self.pos, self.size)]
        stream = np.concatenate(parts) if parts else np.zeros(0, np.uint8)
        offs = np.concatenate([[0], np.cumsum(self.size)]).astype(np.uint64)
        return stream, offs


def refloop_messages_roundtrip_mt(words, msg_off, threads=1):
    """messages_roundtrip_mt with the reference's loops (write_message +
    read_message of one-segment messages, read_message zeroing the body as
    allocate_zeroed_vec does) -> (seconds write, seconds read, packed bytes,
    ok)."""
    import time
    words = np.ascontiguousarray(words, np.uint64)
    msg_off = np.ascontiguousarray(msg_off, np.uint64)
    n = len(msg_off) - 1
    lens = np.diff(msg_off).astype(np.int64)
    slot = np.zeros(n + 1, np.uint64)
    slot[1:] = np.cumsum(8 * lens + (lens + 1) // 2 + 48)
    out = np.ones(int(slot[-1]) + 16, np.uint8)
    sizes = np.zeros(n, np.uint64)
    st = np.ones(n, np.int32)
    body = np.ones(max(int(msg_off[-1]), 1), np.uint64)
    t0 = time.perf_counter()
    lib().refloop_write_messages_mt(words.ctypes.data, msg_off.ctypes.data, n, out.ctypes.data,
                                    slot.ctypes.data, sizes.ctypes.data, st.ctypes.data, threads)
    t1 = time.perf_counter()
    ok = bool((st == 0).all())
    lib().refloop_read_messages_mt(out.ctypes.data, slot.ctypes.data, sizes.ctypes.data, n,
                                   body.ctypes.data, msg_off.ctypes.data, st.ctypes.data, threads)
    t2 = time.perf_counter()
    ok = ok and bool((st == 0).all()) and np.array_equal(body[:len(words)], words)
    return t1 - t0, t2 - t1, int(sizes.sum()), ok
