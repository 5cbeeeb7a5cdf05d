"""Host-side mirror of capnp::serialize_packed (capnp/src/serialize_packed.rs)
on top of the gfx950 codec.

Same names, argument meaning and error behaviour as the reference:

    write_message(write, segments)                   serialize_packed.rs:446-453
    read_message(read, options)                      serialize_packed.rs:233-242
    try_read_message(read, options)                  serialize_packed.rs:246-255
    read_message_no_alloc(read, buffer, options)     serialize_packed.rs:263-273
    try_read_message_no_alloc(read, buffer, options) serialize_packed.rs:281-291
    PackedWrite(inner).write_all(buf)                serialize_packed.rs:300-440
    PackedRead(inner).read(n) / read_exact(n)        serialize_packed.rs:76-229

`read` is a BufRead (io.rs:35-38): `SliceRead` (the `&[u8]` impl), or
`BufReader` over any raw reader, whose fill_buf() hands out one buffer at a
time and refills after consume() — as PackedRead's refresh_buffer!
(serialize_packed.rs:59-74) does, a read unit that runs past the current
buffer consumes it and continues in the next one.  A successful read
consumes exactly the bytes the message used, so a stream of messages is
read by calling try_read_message until it returns None; a failed one leaves
the reader where the reference leaves it (every buffer it had to look past
consumed).  Errors raise CapnpError whose `.kind` is the capnp::ErrorKind
name.  Every transform runs in the HIP kernels; nothing here touches bytes.
"""
import ctypes as C
from dataclasses import dataclass
from typing import Optional

import numpy as np

from . import _lib
from ._lib import CapnpError
from .codec import default_context

SEGMENTS_COUNT_LIMIT = 512  # serialize.rs:39


@dataclass
class ReaderOptions:
    """capnp::message::ReaderOptions (message.rs:85-148)."""
    traversal_limit_in_words: Optional[int] = 8 * 1024 * 1024
    nesting_limit: int = 64

    def _c(self):
        o = _lib.ReaderOptionsC()
        o.has_traversal_limit = self.traversal_limit_in_words is not None
        o.traversal_limit_in_words = self.traversal_limit_in_words or 0
        o.nesting_limit = self.nesting_limit
        return o


DEFAULT_READER_OPTIONS = ReaderOptions()


class SliceRead:
    """BufRead over an in-memory byte slice (io.rs:165-186)."""

    def __init__(self, data):
        self.data = memoryview(bytes(data)) if not isinstance(data, memoryview) else data
        self.pos = 0

    def fill_buf(self):
        return self.data[self.pos:]

    def consume(self, n):
        self.pos += n

    def is_empty(self):
        return self.pos >= len(self.data)


class BufReader:
    """std::io::BufReader over a raw reader (`.read(n) -> bytes`, b"" at the
    end): fill_buf() returns the current buffer of up to `capacity` bytes,
    reading the next one only once it is consumed.  `unread(bufs)` puts
    whole buffers back in front (in order), so _refilling can look ahead and
    still leave the reader exactly where the reference's PackedRead would."""

    def __init__(self, raw, capacity=8192):
        self.raw = raw
        self.capacity = capacity
        self.buf = b""
        self.pos = 0
        self.back = []  # buffers put back by unread, next first

    def fill_buf(self):
        if self.pos >= len(self.buf):
            self.buf = self.back.pop() if self.back else bytes(self.raw.read(self.capacity))
            self.pos = 0
        return memoryview(self.buf)[self.pos:]

    def consume(self, n):
        self.pos = min(self.pos + n, len(self.buf))

    def unread(self, bufs):
        """Puts `bufs` back; the current buffer's unconsumed rest follows them."""
        rest = self.buf[self.pos:]
        if rest:
            self.back.append(rest)
        self.back.extend(reversed([b for b in bufs if b]))
        self.buf, self.pos = b"", 0


# statuses that mean "the unit ran past the bytes in hand"
_NEEDS_MORE = (2, 4, 5)  # PrematureEndOfPackedInput, FailedToFill, PrematureEndOfFile


def _refilling(r, attempt):
    """Runs attempt(data) on the reader's current buffer; while it fails for
    lack of input and the reader has more, consumes that buffer (the
    reference's refresh_buffer!, serialize_packed.rs:59-74) and retries over
    everything seen so far.  On success consumes exactly the bytes used:
    `attempt` returns (status, used, result).

    The reference streams, so the result is the outcome at the first buffer
    boundary where the unit stops needing input.  Retrying at every boundary
    re-decodes everything seen each time (O(k^2) for a unit spanning k
    buffers); with a reader that can put buffers back (`unread`) the retries
    happen only once the bytes in hand have doubled, and the first boundary
    whose outcome is final is then found by bisection over the buffers taken
    since the last retry (a decode is left to right, so once the outcome over
    a prefix is final it is the same over every longer prefix); the buffers
    past that boundary are put back."""
    bufs = []           # buffers taken so far; all consumed but maybe the last
    plen = [0]          # plen[j] = bytes in bufs[:j]
    lookahead = hasattr(r, "unread")
    tried = 0           # the outcome over bufs[:tried] is known to need more
    last = None
    while True:
        cur = bytes(r.fill_buf())
        if not cur:  # the reader has nothing more (or was empty at entry)
            if not bufs:
                st, used, res = attempt(b"")
                return st, res
            if len(bufs) == tried:
                return last  # the failure stands over all the bytes seen, all consumed
            j, cur_taken = len(bufs), True
            st, used, res = attempt(b"".join(bufs))
            if st in _NEEDS_MORE:
                return st, res
            break
        bufs.append(cur)
        plen.append(plen[-1] + len(cur))
        j = len(bufs)
        if lookahead and tried and plen[j] < 2 * plen[tried]:
            r.consume(len(cur))  # not worth a retry yet: take the next buffer too
            continue
        st, used, res = attempt(b"".join(bufs))
        if st in _NEEDS_MORE:
            r.consume(len(cur))
            tried, last = j, (st, res)
            continue
        cur_taken = False
        break
    # the outcome over bufs[:j] is final; the reference stopped at the first
    # such boundary in (tried, j], with that boundary's buffer current
    lo, hi = tried, j
    while hi - lo > 1:
        mid = (lo + hi) // 2
        s2, u2, r2 = attempt(b"".join(bufs[:mid]))
        if s2 in _NEEDS_MORE:
            lo = mid
        else:
            hi, st, used, res = mid, s2, u2, r2
    if cur_taken or hi < j:
        r.unread(bufs[hi - 1:j] if cur_taken else bufs[hi - 1:j - 1])
        r.fill_buf()
    if st == _lib.OK:
        r.consume(used - plen[hi - 1])
    return st, res


class OwnedSegments:
    """Segments of a read message (serialize.rs:170-211): one contiguous
    8-byte-aligned buffer plus (start, end) word indices."""

    def __init__(self, body, seg_words):
        self.body = body
        self.indices = []
        o = 0
        for n in seg_words:
            self.indices.append((o, o + int(n)))
            o += int(n)

    def __len__(self):
        return len(self.indices)

    def get_segment(self, i):
        if i >= len(self.indices):
            return None
        a, b = self.indices[i]
        return self.body[a:b]

    def segments(self):
        return [self.get_segment(i) for i in range(len(self))]


def _as_reader(read):
    return read if hasattr(read, "fill_buf") else SliceRead(read)


def _np_u8(buf):
    return np.frombuffer(buf, dtype=np.uint8) if len(buf) else np.zeros(1, np.uint8)


def _check(st, ctx):
    if st != _lib.OK:
        raise CapnpError(st, (_lib.lib().capnp_ctx_last_error(ctx.handle) or b"").decode())


class PackedWrite:
    """Write adaptor that packs every write_all chunk independently
    (serialize_packed.rs:293-440)."""

    def __init__(self, inner, ctx=None):
        self.inner = inner
        self.ctx = ctx or default_context()

    def write_all(self, buf):
        data = bytes(buf)
        if len(data) % 8:
            raise CapnpError(11, "packed writes must be word-aligned")
        cap = _lib.lib().capnp_packed_bound_bytes(len(data) // 8) + 16
        out = np.empty(cap, np.uint8)
        n = C.c_size_t(0)
        a = _np_u8(data)
        st = _lib.lib().capnp_pack(self.ctx.handle, a.ctypes.data, len(data), out.ctypes.data,
                                   cap, C.byref(n))
        _check(st, self.ctx)
        _write(self.inner, out[:n.value].tobytes())


class PackedRead:
    """Read adaptor that unpacks (serialize_packed.rs:37-229).  read(n)
    returns n unpacked bytes, or b"" when the input is empty at entry."""

    def __init__(self, inner, ctx=None):
        self.inner = _as_reader(inner)
        self.ctx = ctx or default_context()

    def read(self, n):
        if n == 0:
            return b""
        if n % 8:
            raise CapnpError(11, "PackedRead reads must be word-aligned.")
        buf = self.inner.fill_buf()
        if len(buf) == 0:
            return b""
        return self._read_exact(n)

    def read_exact(self, n):
        """io::Read::read_exact (io.rs:16-31)."""
        if n == 0:
            return b""
        if n % 8:
            raise CapnpError(11, "PackedRead reads must be word-aligned.")
        return self._read_exact(n)

    def _read_exact(self, n):
        out = np.empty(n, np.uint8)

        def attempt(data):
            used = C.c_size_t(0)
            a = _np_u8(data)
            st = _lib.lib().capnp_unpack(self.ctx.handle, a.ctypes.data, len(data),
                                         C.byref(used), out.ctypes.data, n)
            return st, used.value, None

        st, _ = _refilling(self.inner, attempt)
        _check(st, self.ctx)
        return out.tobytes()


def _write(w, data):
    if hasattr(w, "write_all"):
        w.write_all(data)
    elif isinstance(w, (bytearray,)):
        w.extend(data)
    else:
        w.write(data)


def _segments_to_words(segments):
    arrs = []
    for s in segments:
        if isinstance(s, (bytes, bytearray, memoryview)):
            if len(s) % 8:
                raise ValueError("segments must be whole words")
            arrs.append(np.frombuffer(bytes(s), dtype=np.uint64))
        else:
            arrs.append(np.ascontiguousarray(np.asarray(s).view(np.uint64)))
    return arrs


def write_message(write, segments, ctx=None):
    """serialize_packed::write_message: packs the segment table and each
    segment as separate chunks (serialize.rs:574-582, 605-679) and writes the
    packed stream to `write` (bytearray, file-like or an object with
    write_all)."""
    ctx = ctx or default_context()
    arrs = _segments_to_words(segments)
    if not arrs:
        raise ValueError("a message has at least one segment")
    nseg = len(arrs)
    ptrs = (C.c_void_p * nseg)(*[a.ctypes.data if len(a) else None for a in arrs])
    lens = (C.c_uint32 * nseg)(*[len(a) for a in arrs])
    total = sum(len(a) for a in arrs)
    cap = _lib.lib().capnp_packed_batch_bound_bytes(total + nseg // 2 + 1, nseg + 2)
    out = np.empty(cap, np.uint8)
    n = C.c_size_t(0)
    st = _lib.lib().capnp_packed_write_message(ctx.handle, ptrs, lens, nseg, out.ctypes.data,
                                               cap, C.byref(n))
    _check(st, ctx)
    _write(write, out[:n.value].tobytes())


def _read(read, options, try_mode, ctx):
    ctx = ctx or default_context()
    r = _as_reader(read)
    opts = (options or DEFAULT_READER_OPTIONS)._c()

    def attempt(data):
        a = _np_u8(data)
        cap = 1 << 12
        while True:
            body = np.empty(cap, np.uint64)
            segs = np.empty(SEGMENTS_COUNT_LIMIT, np.uint32)
            nseg, used = C.c_uint32(0), C.c_size_t(0)
            st = _lib.lib().capnp_packed_read_message(ctx.handle, a.ctypes.data, len(data),
                                                      C.byref(opts), int(try_mode),
                                                      body.ctypes.data, cap, segs.ctypes.data,
                                                      C.byref(nseg), C.byref(used))
            if st == 9:  # BufferNotLargeEnough: the table says how many words
                need = int(segs[:nseg.value].astype(np.uint64).sum())
                if need > cap:
                    cap = need
                    continue
            return st, used.value, (body, segs, nseg.value)

    st, res = _refilling(r, attempt)
    if st == _lib.NONE:
        return None
    _check(st, ctx)
    body, segs, nseg = res
    total = int(segs[:nseg].astype(np.uint64).sum())
    return OwnedSegments(body[:total], segs[:nseg])


def read_message(read, options=None, ctx=None):
    """serialize_packed::read_message -> OwnedSegments (PrematureEndOfFile on
    an empty input)."""
    return _read(read, options, False, ctx)


def try_read_message(read, options=None, ctx=None):
    """serialize_packed::try_read_message -> OwnedSegments or None."""
    return _read(read, options, True, ctx)


def _read_no_alloc(read, buffer, options, try_mode, ctx):
    ctx = ctx or default_context()
    r = _as_reader(read)
    nb = np.frombuffer(buffer, dtype=np.uint8) if not isinstance(buffer, np.ndarray) else \
        buffer.view(np.uint8)
    nseg, tb, bb = C.c_uint32(0), C.c_size_t(0), C.c_size_t(0)
    opts = (options or DEFAULT_READER_OPTIONS)._c()

    def attempt(data):
        a = _np_u8(data)
        used = C.c_size_t(0)
        st = _lib.lib().capnp_packed_read_message_no_alloc(
            ctx.handle, a.ctypes.data, len(data), C.byref(opts), int(try_mode), nb.ctypes.data,
            nb.nbytes, C.byref(nseg), C.byref(tb), C.byref(bb), C.byref(used))
        return st, used.value, None

    st, _ = _refilling(r, attempt)
    if st == _lib.NONE:
        return None
    _check(st, ctx)
    body = nb[tb.value:tb.value + bb.value].view(np.uint64)
    lens = []
    t = nb[:tb.value].view(np.uint32)
    for i in range(nseg.value):
        lens.append(int(t[1 + i]))
    return OwnedSegments(body, lens)


def read_message_no_alloc(read, buffer, options=None, ctx=None):
    """serialize_packed::read_message_no_alloc: the message lands in
    `buffer` (writable, 8-byte aligned)."""
    return _read_no_alloc(read, buffer, options, False, ctx)


def try_read_message_no_alloc(read, buffer, options=None, ctx=None):
    return _read_no_alloc(read, buffer, options, True, ctx)
