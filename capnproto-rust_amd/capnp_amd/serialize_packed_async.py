"""Host-side mirror of capnp_futures::serialize_packed
(capnp-futures/src/serialize_packed.rs) on the gfx950 codec: byte streams
split at any byte, inner streams that return short reads, partial writes or
"pending".

    PackedWrite(inner).write(buf) / .flush()     serialize_packed.rs:330-521
    PackedRead(inner).read(n) / .read_exact(n)   serialize_packed.rs:34-225
    write_message(writer, segments)              serialize_packed.rs:317-328
    try_read_message(reader, options)            serialize_packed.rs:233-245
    read_message(reader, options)                serialize_packed.rs:248-258

An inner stream is any object with
    read(n)  -> bytes (b"" at the end of the stream) or None (pending),
    write(b) -> bytes accepted (>= 1) or None (pending).
The transform runs in the HIP kernels behind the C adaptors of
include/capnp_packed.h (capnp_packed_writer_* / capnp_packed_reader_*).
Errors raise CapnpError; Pending surfaces as CapnpError(15) from a single
poll (PackedWrite.flush, PackedRead.read), while read_exact and the message
functions retry until the inner stream moves, as a future driven by
block_on does.
"""
import ctypes as C
import io
import os
import stat
import socket

import numpy as np

from . import _lib
from ._lib import CapnpError
from .codec import default_context
from .serialize_packed import OwnedSegments, ReaderOptions, DEFAULT_READER_OPTIONS

SEGMENTS_COUNT_LIMIT = 512


def _as_u8(buf):
    """A uint8 view of a bytes-like object (no copy for contiguous buffers)."""
    try:
        return np.frombuffer(memoryview(buf).cast("B"), np.uint8)
    except (TypeError, ValueError):
        return np.frombuffer(bytes(buf), np.uint8)


def _check(st, ctx):
    if st != _lib.OK:
        raise CapnpError(st, (_lib.lib().capnp_ctx_last_error(ctx.handle) or b"").decode())


class PackedWrite:
    """An AsyncWrite wrapper that packs any data passed into it."""

    def __init__(self, inner, ctx=None, inner_copies=None):
        """`inner_copies`: whether `inner.write(b)` copies the bytes of `b`
        before it returns (io objects and sockets do).  Such a writer is
        handed a view of the adaptor's queue, valid during the call only, as
        the reference's poll_write(&[u8]) hands a borrow; the view is
        released afterwards, so a writer that kept it gets an error on use
        instead of bytes the queue has since overwritten.  Any other writer
        (a list sink that keeps what it is given, a buffered transport) gets
        a bytes copy.  None = decide by type."""
        self.inner = inner
        self.ctx = ctx or default_context()
        self._err = None
        if inner_copies is None:
            inner_copies = isinstance(inner, (io.IOBase, socket.socket))
        self._view = bool(inner_copies)

        def write_cb(_user, buf, n):
            mv = None
            err = None
            try:
                addr = C.cast(buf, C.c_void_p).value
                mv = memoryview((C.c_ubyte * n).from_address(addr)).cast("B")
                r = self.inner.write(mv if self._view else bytes(mv))
            except Exception as e:  # surfaced as CAPNP_E_IO
                err = e
            if mv is not None:
                try:
                    mv.release()
                except BufferError as e:  # the writer exported the view and kept it
                    err = err or e
            if err is not None:
                self._err = err
                return -2
            return _lib.IO_PENDING if r is None else int(r)

        self._cb = _lib.WRITE_FN(write_cb)
        self._h = _lib.lib().capnp_packed_writer_new(self.ctx.handle, self._cb, None)
        if not self._h:
            raise CapnpError(64, "capnp_packed_writer_new")

    def write(self, buf):
        """poll_write: takes every byte of `buf` (packed bytes are queued).
        `buf` is any bytes-like object; it is read in place (no copy)."""
        a = _as_u8(buf)
        n = a.size
        if n == 0:
            a = np.zeros(1, np.uint8)
        _check(_lib.lib().capnp_packed_writer_write(self._h, a.ctypes.data, n), self.ctx)
        return n

    def write_all(self, buf):
        self.write(buf)

    def flush(self):
        """poll_flush: raises CapnpError(15) (Pending) if the inner writer
        pends; call again."""
        st = _lib.lib().capnp_packed_writer_flush(self._h)
        if st == 68 and self._err is not None:
            raise self._err
        _check(st, self.ctx)

    def flush_blocking(self):
        while True:
            try:
                return self.flush()
            except CapnpError as e:
                if e.status != _lib.PENDING:
                    raise

    @property
    def carried(self):
        """Bytes of an incomplete word carried to the next write (0..7)."""
        return _lib.lib().capnp_packed_writer_carried(self._h)

    def __del__(self):
        if getattr(self, "_h", None):
            _lib.lib().capnp_packed_writer_free(self._h)
            self._h = None


def _bulk_source(inner):
    """Whether `inner` is a source whose reads never wait on a peer."""
    if isinstance(inner, io.BytesIO):
        return True
    try:
        return stat.S_ISREG(os.fstat(inner.fileno()).st_mode)
    except (AttributeError, OSError, ValueError, io.UnsupportedOperation):
        return False


class PackedRead:
    """An AsyncRead wrapper that unpacks packed data."""

    def __init__(self, inner, ctx=None, readahead=None):
        """`readahead`: pull the inner reader in MiB units past what the
        current read needs while it returns every byte asked (a file, an
        in-memory stream).  Off, reads pull no further than the current
        request can need, as the reference does, so a blocking pipe or socket
        whose peer awaits a reply is never read past the request.  None =
        on for `io.BytesIO` and regular files, off otherwise."""
        self.inner = inner
        self.ctx = ctx or default_context()
        self._err = None
        self._extra = None  # bytes an inner reader returned beyond what was asked
        if readahead is None:
            readahead = _bulk_source(inner)

        def read_cb(_user, buf, n):
            if self._extra is not None and self._extra.size:
                r = self._extra
            else:
                try:
                    r = self.inner.read(n)
                except Exception as e:
                    self._err = e
                    return -2
                if r is None:
                    return _lib.IO_PENDING
                # (read in place: no copy; but an object the reader may reuse
                # -- a bytearray, a view of its buffer -- is copied before any
                # of it is carried to the next call)
                keep = isinstance(r, bytes) or (isinstance(r, memoryview) and r.readonly)
                r = _as_u8(r)
                if not keep and r.size > n:
                    r = r.copy()
            # never more than n into the adaptor's n-byte staging slot
            k = min(r.size, n)
            self._extra = r[k:]
            if k:
                C.memmove(buf, r.ctypes.data, k)
            return k

        self._cb = _lib.READ_FN(read_cb)
        self._h = _lib.lib().capnp_packed_reader_new(self.ctx.handle, self._cb, None)
        if not self._h:
            raise CapnpError(64, "capnp_packed_reader_new")
        _lib.lib().capnp_packed_reader_set_readahead(self._h, 1 if readahead else 0)

    def _raise(self, st):
        if st == 68 and self._err is not None:
            raise self._err
        _check(st, self.ctx)

    def read(self, n):
        """poll_read: 1..n unpacked bytes, b"" at a clean end of the stream;
        CapnpError(15) if the inner reader pends, PrematureEndOfFile if the
        stream ends inside a record (the reference's UnexpectedEof)."""
        out = np.empty(max(n, 1), np.uint8)
        got = C.c_size_t(0)
        self._raise(_lib.lib().capnp_packed_reader_read(self._h, out.ctypes.data, n,
                                                        C.byref(got)))
        return out[:got.value].tobytes()

    def readinto(self, b):
        """poll_read into a caller's writable buffer (the reference's
        `poll_read(buf: &mut [u8])`): the unpacked bytes go straight into
        `b`; returns how many (1..len(b), 0 at a clean end of the stream)."""
        out = np.frombuffer(memoryview(b).cast("B"), np.uint8)
        if out.size == 0:
            return 0
        got = C.c_size_t(0)
        self._raise(_lib.lib().capnp_packed_reader_read(self._h, out.ctypes.data, out.size,
                                                        C.byref(got)))
        return got.value

    def read_exact(self, n):
        out = np.empty(max(n, 1), np.uint8)
        got = C.c_size_t(0)
        self._raise(_lib.lib().capnp_packed_reader_read_exact(self._h, out.ctypes.data, n,
                                                              C.byref(got)))
        return out[:n].tobytes()

    def read_to_end(self):
        parts = []
        while True:
            try:
                b = self.read(1 << 16)
            except CapnpError as e:
                if e.status == _lib.PENDING:
                    continue
                raise
            if not b:
                return b"".join(parts)
            parts.append(b)

    @property
    def buffered(self):
        return _lib.lib().capnp_packed_reader_buffered(self._h)

    def __del__(self):
        if getattr(self, "_h", None):
            _lib.lib().capnp_packed_reader_free(self._h)
            self._h = None


def write_message(writer, segments, ctx=None):
    """Packs the segment table and the segments as the capnp-futures writer
    does (one write per table part and per segment,
    capnp-futures/src/serialize.rs:211-263) and finishes pending writes."""
    pw = writer if isinstance(writer, PackedWrite) else PackedWrite(writer, ctx)
    segs = []
    for s in segments:
        b = bytes(s) if isinstance(s, (bytes, bytearray, memoryview)) else \
            np.ascontiguousarray(np.asarray(s).view(np.uint64)).tobytes()
        if len(b) % 8:
            raise ValueError("segments must be whole words")
        segs.append(b)
    if not segs:
        raise ValueError("a message has at least one segment")
    n = len(segs)
    t = np.zeros(2 * (n // 2 + 1), np.uint32)
    t[0] = n - 1
    for i, s in enumerate(segs):
        t[1 + i] = len(s) // 8
    tb = t.tobytes()
    pw.write(tb[:8])
    if n > 1:
        pw.write(tb[8:])
    for s in segs:
        pw.write(s)
    pw.flush_blocking()


def _read(reader, options, try_mode, ctx):
    pr = reader if isinstance(reader, PackedRead) else PackedRead(reader, ctx)
    L = _lib.lib()
    opts = (options or DEFAULT_READER_OPTIONS)._c()
    segs = np.zeros(SEGMENTS_COUNT_LIMIT, np.uint32)
    nseg, need = C.c_uint32(0), C.c_uint64(0)
    cap = 1 << 12
    body = np.empty(cap, np.uint64)
    st = L.capnp_packed_reader_read_message(pr._h, C.byref(opts), int(try_mode), body.ctypes.data,
                                            cap, segs.ctypes.data, C.byref(nseg), C.byref(need))
    if st == 9 and need.value > cap:  # BufferNotLargeEnough: the table is read; read the body
        body = np.empty(need.value, np.uint64)
        got = C.c_size_t(0)
        st = L.capnp_packed_reader_read_exact(pr._h, body.ctypes.data, need.value * 8,
                                              C.byref(got))
    if st == _lib.NONE:
        return None
    pr._raise(st)
    total = int(segs[:nseg.value].astype(np.uint64).sum())
    return OwnedSegments(body[:total], segs[:nseg.value])


def try_read_message(reader, options=None, ctx=None):
    """-> OwnedSegments, or None at a clean end of the stream."""
    return _read(reader, options, True, ctx)


def read_message(reader, options=None, ctx=None):
    """-> OwnedSegments; PrematureEndOfFile at a clean end of the stream."""
    return _read(reader, options, False, ctx)


class BlockingRead:
    """Test stream of capnp-futures/src/serialize.rs:536-586: pends once every
    `blocking_period` bytes, then reads at most that many."""

    def __init__(self, data, blocking_period):
        self.data = memoryview(bytes(data))
        self.pos = 0
        self.period = blocking_period
        self.idx = 0

    def read(self, n):
        if self.idx == 0:
            self.idx = self.period
            return None
        k = min(self.idx, n, len(self.data) - self.pos)
        b = bytes(self.data[self.pos:self.pos + k])
        self.pos += k
        self.idx -= k
        return b

    def is_empty(self):
        return self.pos >= len(self.data)


class BlockingWrite:
    """Test stream of capnp-futures/src/serialize.rs:588-640: pends once every
    `blocking_period` bytes, then accepts at most that many."""

    def __init__(self, blocking_period, cap=None):
        self.buf = bytearray()
        self.period = blocking_period
        self.idx = 0
        self.cap = cap

    def write(self, b):
        if self.idx == 0:
            self.idx = self.period
            return None
        k = min(self.idx, len(b))
        if self.cap is not None:
            k = min(k, self.cap - len(self.buf))
            if k <= 0:
                return 0
        self.buf.extend(b[:k])
        self.idx -= k
        return k
