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
buffer consumes it and continues in the next one (_read_unit: each buffer is
decoded once; only an incomplete record is carried to the next).  A
successful read consumes exactly the bytes the message used, so a stream of
messages is read by calling try_read_message until it returns None; a
failed one leaves the reader where the reference leaves it (every buffer it
had to look past consumed).  Errors raise CapnpError whose `.kind` is the capnp::ErrorKind
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
    reading the next one only once it is consumed."""

    def __init__(self, raw, capacity=8192):
        self.raw = raw
        self.capacity = capacity
        self.buf = b""
        self.pos = 0

    def fill_buf(self):
        if self.pos >= len(self.buf):
            self.buf = bytes(self.raw.read(self.capacity))
            self.pos = 0
        return memoryview(self.buf)[self.pos:]

    def consume(self, n):
        self.pos = min(self.pos + n, len(self.buf))


# statuses that mean "the unit ran past the bytes in hand"
_NEEDS_MORE = (2, 4, 5)  # PrematureEndOfPackedInput, FailedToFill, PrematureEndOfFile
_EMPTY = -1              # _read_unit: read() found the input empty at entry (Ok(0))


def _unpack(ctx, data, out):
    """capnp_unpack: PackedRead::read_exact of len(out) bytes (a np.uint8
    view) from the slice `data` -> (status, consumed)."""
    a = _np_u8(data)
    used = C.c_size_t(0)
    st = _lib.lib().capnp_unpack(ctx.handle, a.ctypes.data, len(data), C.byref(used),
                                 out.ctypes.data if len(out) else None, len(out))
    return st, used.value


def _prefix(ctx, data, max_words, out):
    """capnp_unpack_prefix: the whole records of `data` decoding to at most
    max_words words, decoded into `out` -> (bytes, words)."""
    a = _np_u8(data)
    nb, nw = C.c_size_t(0), C.c_uint64(0)
    _check(_lib.lib().capnp_unpack_prefix(ctx.handle, a.ctypes.data, len(data), max_words,
                                          out.ctypes.data, C.byref(nb), C.byref(nw)), ctx)
    return nb.value, nw.value


def _read_unit(r, ctx, out, exact):
    """One PackedRead::read (exact False) or read_exact (exact True) of
    len(out) bytes into `out` (np.uint8, a word multiple) from the BufRead
    `r`, streaming over its buffers as the reference does
    (serialize_packed.rs:80-228; refresh_buffer!, :59-74: a unit that runs
    past the current buffer consumes it and continues in the next).

    Each buffer is decoded once: the input in hand is the current buffer
    plus `tail`, the bytes of the one record the previous buffer ended in.
    If the unit completes, exactly the bytes it used are consumed.  If it
    fails for a reason the bytes in hand already decide (a run past the
    unit's end), the current buffer stays unconsumed, as in the reference.
    If it needs more input, its whole records are final (the decode is left
    to right), so they are kept in `out`, only the incomplete record is
    carried, and the buffer is consumed.  At the end of the input the
    failure over what was seen stands.  Returns the status, or _EMPTY for a
    read() at an empty input (Ok(0), :96-98)."""
    n = len(out)
    if n == 0:
        return _lib.OK
    tail, done, first = b"", 0, True
    while True:
        cur = bytes(r.fill_buf())
        if not cur:
            if first:  # read() of an empty input is Ok(0); read_exact fails (io.rs:26-28)
                return 4 if exact else _EMPTY
            if not tail:  # the next record's tag: refresh_buffer! finds nothing (:59-74)
                return 2
            st, _ = _unpack(ctx, tail, out[done:])  # the record cut short stands
            return st
        first = False
        data = tail + cur if tail else cur
        st, used = _unpack(ctx, data, out[done:])
        if st == _lib.OK:
            r.consume(used - len(tail))
            return st
        if st not in _NEEDS_MORE:
            return st
        nb, nw = _prefix(ctx, data, (n - done) // 8, out[done:].view(np.uint64))
        done += 8 * nw
        tail = data[nb:]
        r.consume(len(cur))


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
        st = _read_unit(self.inner, self.ctx, out, exact=True)
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


def _fast(r, attempt):
    """The message within the reader's current buffer, in one device call:
    (status, result) when it is there whole (or the input is at a clean
    end), else None, and the caller reads the message unit by unit
    (nothing has been consumed): a message past the buffer, and every
    failure, whose stream position then comes out as the reference leaves
    it (the units before the failing one consumed)."""
    cur = bytes(r.fill_buf())
    st, used, res = attempt(cur)
    if st == _lib.OK:
        r.consume(used)
        return st, res
    if st == _lib.NONE:
        return st, res
    return None


def _u32(b, i):
    return int.from_bytes(bytes(b[i:i + 4]), "little")


def _read(read, options, try_mode, ctx):
    ctx = ctx or default_context()
    r = _as_reader(read)
    options = options or DEFAULT_READER_OPTIONS
    opts = options._c()

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
            return st, used.value, (body, segs[:nseg.value])

    fast = _fast(r, attempt)
    if fast is not None:
        st, res = fast
        if st == _lib.NONE:
            return None
        _check(st, ctx)
        body, segs = res
        return OwnedSegments(body[:int(segs.astype(np.uint64).sum())], segs)
    # read_segment_table + read_segments unit by unit (serialize.rs:448-524)
    w0 = np.empty(8, np.uint8)
    st = _read_unit(r, ctx, w0, exact=False)
    if st == _EMPTY:  # :456-462
        if try_mode:
            return None
        raise CapnpError(5, "PrematureEndOfFile")
    _check(st, ctx)
    nseg = (_u32(w0, 0) + 1) & 0xFFFFFFFF
    if nseg == 0 or nseg >= SEGMENTS_COUNT_LIMIT:  # :467-473
        raise CapnpError(6)
    lens = [_u32(w0, 4)]
    if nseg > 1:  # :476-496
        t = np.empty(8 if nseg < 4 else (nseg & ~1) * 4, np.uint8)
        _check(_read_unit(r, ctx, t, exact=True), ctx)
        lens += [_u32(t, 4 * i) for i in range(nseg - 1)]
    total = sum(lens)
    limit = options.traversal_limit_in_words
    if limit is not None and total > limit:  # :501-507
        raise CapnpError(8)
    body = np.empty(max(total, 1), np.uint64)
    _check(_read_unit(r, ctx, body.view(np.uint8)[:8 * total], exact=True), ctx)  # :514-524
    return OwnedSegments(body[:total], np.array(lens, np.uint32))


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
    options = options or DEFAULT_READER_OPTIONS
    opts = options._c()

    def attempt(data):
        a = _np_u8(data)
        used = C.c_size_t(0)
        st = _lib.lib().capnp_packed_read_message_no_alloc(
            ctx.handle, a.ctypes.data, len(data), C.byref(opts), int(try_mode), nb.ctypes.data,
            nb.nbytes, C.byref(nseg), C.byref(tb), C.byref(bb), C.byref(used))
        return st, used.value, None

    def result(table_bytes, body_bytes, n):
        t = nb[:table_bytes].view(np.uint32)
        return OwnedSegments(nb[table_bytes:table_bytes + body_bytes].view(np.uint64),
                             [int(t[1 + i]) for i in range(n)])

    fast = _fast(r, attempt)
    if fast is not None:
        st, _ = fast
        if st == _lib.NONE:
            return None
        _check(st, ctx)
        return result(tb.value, bb.value, nseg.value)
    # serialize.rs:333-420 unit by unit: read(8), the table rest 8 bytes at
    # a time into the buffer (:371-395), then the body after the table
    if nb.ctypes.data % 8:  # :341-343
        raise CapnpError(10)
    if nb.nbytes < 8:  # :345-347
        raise CapnpError(9)
    st = _read_unit(r, ctx, nb[:8], exact=False)
    if st == _EMPTY:
        if try_mode:
            return None
        raise CapnpError(5, "PrematureEndOfFile")
    _check(st, ctx)
    n = (_u32(nb, 0) + 1) & 0xFFFFFFFF
    if n == 0 or n >= SEGMENTS_COUNT_LIMIT:
        raise CapnpError(6)
    total = _u32(nb, 4)
    got = 1
    while got < n:
        start = (got + 1) * 4
        if nb.nbytes < start + 8:  # :374-376
            raise CapnpError(9)
        _check(_read_unit(r, ctx, nb[start:start + 8], exact=True), ctx)
        total += _u32(nb, start)
        got += 1
        if got < n:
            total += _u32(nb, start + 4)
        got += 1
    limit = options.traversal_limit_in_words
    if limit is not None and total > limit:
        raise CapnpError(8)
    start = (got + 1) * 4
    if nb.nbytes < start + 8 * total:  # :407-409
        raise CapnpError(9)
    _check(_read_unit(r, ctx, nb[start:start + 8 * total], exact=True), ctx)
    return result(start, 8 * total, n)


def read_message_no_alloc(read, buffer, options=None, ctx=None):
    """serialize_packed::read_message_no_alloc: the message lands in
    `buffer` (writable, 8-byte aligned)."""
    return _read_no_alloc(read, buffer, options, False, ctx)


def try_read_message_no_alloc(read, buffer, options=None, ctx=None):
    return _read_no_alloc(read, buffer, options, True, ctx)
