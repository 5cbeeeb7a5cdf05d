"""Device context and the batched GPU codec (the hot path).

`Context` owns a capnp_ctx (HIP stream + workspace).  The batch methods take
torch tensors that already live in HBM (int64 views of the words / offsets)
and enqueue the gfx950 kernels on the current torch stream:

    pack_batch(words, chunk_word_off)            -> (packed u8, out_byte_off)
    unpack_batch(packed, in_byte_off, out_word_off) -> (words, status, consumed)

which are the batched bodies of PackedWrite::write_all and
PackedRead::read_exact (capnp/src/serialize_packed.rs:304-439, :80-228).
"""
import ctypes as C

import numpy as np

from . import _lib
from ._lib import CapnpError


def _check(st, ctx=None):
    if st != _lib.OK:
        msg = ""
        if ctx is not None:
            msg = (_lib.lib().capnp_ctx_last_error(ctx) or b"").decode()
        raise CapnpError(st, msg)


def _ptr(t):
    return C.c_void_p(t.data_ptr()) if t is not None else None


def seg_words_u32(segs):
    """Segment lengths returned in int32 storage read as the ABI's uint32
    (a segment of 2^31 words or more would otherwise read negative)."""
    import torch
    return segs.to(torch.int64) & 0xFFFFFFFF


class Context:
    """A device context bound to one gfx950 GPU."""

    def __init__(self, device=0):
        L = _lib.lib()
        st = C.c_int(0)
        h = L.capnp_ctx_create(int(device), C.byref(st))
        if not h:
            raise CapnpError(st.value, f"no gfx950 device {device} available")
        self._h = C.c_void_p(h)
        self.device = device

    @property
    def handle(self):
        return self._h

    def close(self):
        if getattr(self, "_h", None):
            _lib.lib().capnp_ctx_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    # ------------------------------------------------------------------
    @staticmethod
    def bound_bytes(words):
        return _lib.lib().capnp_packed_bound_bytes(int(words))

    @staticmethod
    def batch_bound_bytes(total_words, nchunks):
        return _lib.lib().capnp_packed_batch_bound_bytes(int(total_words), int(nchunks))

    def reserve(self, max_chunks):
        _check(_lib.lib().capnp_ctx_reserve(self._h, int(max_chunks)), self._h)

    @staticmethod
    def _stream(stream):
        if stream is not None:
            return C.c_void_p(stream)
        import torch
        return C.c_void_p(torch.cuda.current_stream().cuda_stream)

    # ---- device batch API (torch tensors in HBM) -----------------------
    @staticmethod
    def sync_entries(total_words):
        """Entries of the record sync index for a batch of total_words words
        (int32 tensor of this length; include/capnp_packed.h)."""
        return _lib.lib().capnp_sync_index_entries(int(total_words))

    def pack_batch_into(self, words, chunk_word_off, out, out_off, chunks_per_tile=0,
                        stream=None, sync=None):
        """Enqueue PACK; `out` (uint8) and `out_off` (int64, n+1) are
        preallocated; `sync` (int32, sync_entries(total words)) receives the
        record sync index when given."""
        n = chunk_word_off.numel() - 1
        L = _lib.lib()
        if sync is None:
            st = L.capnp_gpu_pack_batch_tuned(self._h, _ptr(words), _ptr(chunk_word_off), n,
                                              _ptr(out), out.numel(), _ptr(out_off),
                                              int(chunks_per_tile), self._stream(stream))
        else:
            st = L.capnp_gpu_pack_batch_sync_tuned(self._h, _ptr(words), _ptr(chunk_word_off),
                                                   n, _ptr(out), out.numel(), _ptr(out_off),
                                                   _ptr(sync), int(chunks_per_tile),
                                                   self._stream(stream))
        _check(st, self._h)

    def unpack_batch_into(self, packed, in_byte_off, out_word_off, words, status,
                          consumed=None, chunks_per_tile=0, stream=None, sync=None):
        """Enqueue UNPACK; chunks_per_tile 0 = library default; `sync` = the
        record sync index from pack_batch_into (same word offsets), optional."""
        n = in_byte_off.numel() - 1
        L = _lib.lib()
        if sync is None:
            st = L.capnp_gpu_unpack_batch_tuned(
                self._h, _ptr(packed), _ptr(in_byte_off), n, _ptr(words), _ptr(out_word_off),
                _ptr(status), _ptr(consumed), int(chunks_per_tile), self._stream(stream))
        else:
            st = L.capnp_gpu_unpack_batch_sync_tuned(
                self._h, _ptr(packed), _ptr(in_byte_off), n, _ptr(words), _ptr(out_word_off),
                _ptr(sync), _ptr(status), _ptr(consumed), int(chunks_per_tile),
                self._stream(stream))
        _check(st, self._h)

    def unpack_batch_resync_into(self, packed, in_byte_off, out_word_off, words, status,
                                 consumed=None, stream=None, stats=True):
        """Index-free UNPACK of chunks of any length (capnp_gpu_unpack_batch_resync):
        results identical to unpack_batch_into.  With stats (the default) it
        blocks until done and returns (fix passes; serial: 1 the batch went to
        the serial batch unpack, 2 short chunks went there directly, 3 only the
        chunks that failed their check were decoded serially); stats=False
        returns None with the decode only enqueued (ordered on the stream)."""
        import ctypes as C
        n = in_byte_off.numel() - 1
        L = _lib.lib()
        st = L.capnp_gpu_unpack_batch_resync(
            self._h, _ptr(packed), _ptr(in_byte_off), n, _ptr(words), _ptr(out_word_off),
            _ptr(status), _ptr(consumed), self._stream(stream))
        _check(st, self._h)
        if not stats:
            return None
        passes, serial = C.c_int(0), C.c_int(0)
        _check(L.capnp_resync_stats(self._h, C.byref(passes), C.byref(serial)), self._h)
        return passes.value, serial.value

    def pack_batch(self, words, chunk_word_off, chunks_per_tile=0):
        """Returns (packed uint8 tensor trimmed to size, out_byte_off int64).
        Synchronises the stream once to read the total size."""
        import torch
        n = chunk_word_off.numel() - 1
        total_words = int(chunk_word_off[-1].item() - chunk_word_off[0].item()) if n else 0
        cap = self.batch_bound_bytes(total_words, n)
        out = torch.empty(cap, dtype=torch.uint8, device=words.device)
        out_off = torch.empty(n + 1, dtype=torch.int64, device=words.device)
        if chunks_per_tile == 0 and n:
            chunks_per_tile = tile_chunks_for(total_words, n)
        self.pack_batch_into(words, chunk_word_off, out, out_off, chunks_per_tile)
        total = int(out_off[-1].item())
        return out[:total], out_off

    def unpack_batch(self, packed, in_byte_off, out_word_off, chunks_per_tile=0):
        import torch
        n = in_byte_off.numel() - 1
        total = int(out_word_off[-1].item()) if n else 0
        dev = in_byte_off.device
        words = torch.empty(max(total, 1), dtype=torch.int64, device=dev)
        status = torch.empty(max(n, 1), dtype=torch.int32, device=dev)
        consumed = torch.empty(max(n, 1), dtype=torch.int64, device=dev)
        self.unpack_batch_into(packed, in_byte_off, out_word_off, words, status, consumed,
                               chunks_per_tile)
        return words[:total], status[:n], consumed[:n]

    def write_messages(self, words, seg_word_off, msg_seg_off, out=None, stream=None):
        """serialize_packed::write_message for a batch of messages on the
        device (capnp_gpu_write_messages): int64 device tensors `words`
        (segments back to back), `seg_word_off` (segments + 1) and
        `msg_seg_off` (messages + 1).  Returns (packed uint8 trimmed,
        msg_byte_off int64)."""
        import torch
        nmsg = msg_seg_off.numel() - 1
        nseg = seg_word_off.numel() - 1
        # (the words `words` holds up to the last segment: the bound the
        # library checks every segment offset against)
        total_words = int(seg_word_off[-1].item()) if nseg else 0
        if out is None:
            cap = self.batch_bound_bytes(total_words + 2 * nmsg + nseg // 2, 2 * nmsg + nseg)
            out = torch.empty(max(cap, 1), dtype=torch.uint8, device=words.device)
        mo = torch.empty(nmsg + 1, dtype=torch.int64, device=words.device)
        st = _lib.lib().capnp_gpu_write_messages(self._h, _ptr(words), _ptr(seg_word_off),
                                                 _ptr(msg_seg_off), nmsg, nseg, total_words,
                                                 _ptr(out), out.numel(), _ptr(mo),
                                                 self._stream(stream))
        _check(st, self._h)
        total = int(mo[-1].item())
        return out[:total], mo

    def read_messages(self, packed, msg_byte_off, words_cap=None, segs_cap=None, try_mode=False,
                      limit=8 * 1024 * 1024, stream=None):
        """serialize_packed::read_message for a batch of messages on the
        device (capnp_gpu_read_messages).  Returns (words, msg_word_off,
        seg_words, msg_seg_off, status, consumed) as device tensors; limit
        None = no traversal limit.  words_cap / segs_cap None size the
        outputs in two phases: a first guess, then exactly the totals the
        library reports with CAPNP_E_BUFFER_NOT_LARGE_ENOUGH (a packed zero
        run expands 2 bytes into up to 256 words, so no fixed ratio to the
        packed size is safe)."""
        import torch
        nmsg = msg_byte_off.numel() - 1
        dev = msg_byte_off.device
        wc = int(words_cap) if words_cap is not None else \
            int(msg_byte_off[-1].item() - msg_byte_off[0].item()) + 64 if nmsg else 1
        sc = int(segs_cap) if segs_cap is not None else 4 * max(nmsg, 1)
        mwo = torch.empty(nmsg + 1, dtype=torch.int64, device=dev)
        mso = torch.empty(nmsg + 1, dtype=torch.int64, device=dev)
        status = torch.empty(max(nmsg, 1), dtype=torch.int32, device=dev)
        consumed = torch.empty(max(nmsg, 1), dtype=torch.int64, device=dev)
        o = _lib.ReaderOptionsC(int(limit or 0), 1 if limit is not None else 0, 64)
        for phase in range(2):
            words = torch.empty(max(wc, 1), dtype=torch.int64, device=dev)
            segs = torch.empty(max(sc, 1), dtype=torch.int64, device=dev)
            st = _lib.lib().capnp_gpu_read_messages(
                self._h, _ptr(packed), _ptr(msg_byte_off), nmsg, C.byref(o),
                int(bool(try_mode)), _ptr(words), wc, _ptr(mwo), _ptr(segs), sc, _ptr(mso),
                _ptr(status), _ptr(consumed), self._stream(stream))
            if st == 9 and phase == 0 and (words_cap is None or segs_cap is None):
                need_w, need_s = int(mwo[nmsg].item()), int(mso[nmsg].item())
                if (need_w > wc and words_cap is not None) or (need_s > sc and segs_cap is not None):
                    break  # a caller-given capacity is too small: report it
                wc, sc = max(wc, need_w), max(sc, need_s)
                continue
            break
        _check(st, self._h)
        return words, mwo, segs, mso, status[:nmsg], consumed[:nmsg]

    def find_messages(self, packed, nbytes=None, max_msgs=None, stream=None):
        """Message starts of a concatenated packed stream with no byte index
        (capnp_gpu_find_messages).  -> (offs int64 device tensor of nmsg + 1
        entries, nmsg): messages [offs[k], offs[k+1]) read completely;
        offs[nmsg] is where the next try_read_message starts (== nbytes: a
        clean end).  At most max_msgs are returned (default nbytes // 8 + 1);
        nmsg == max_msgs with offs[nmsg] < nbytes means the walk stopped at
        the cap and goes on from offs[nmsg] (a packed message can be as short
        as 2 bytes, so the default does not cover every stream)."""
        import torch
        nb = int(packed.numel() if nbytes is None else nbytes)
        cap = int(max_msgs if max_msgs is not None else nb // 8 + 1)
        offs = torch.empty(cap + 1, dtype=torch.int64, device=packed.device)
        n = C.c_size_t(0)
        st = _lib.lib().capnp_gpu_find_messages(self._h, _ptr(packed) if nb else None, nb, cap,
                                                _ptr(offs), C.byref(n), self._stream(stream))
        _check(st, self._h)
        return offs[:n.value + 1], n.value

    def _read_ranges(self, packed, ranges, limit, stream):
        """read_messages in try mode over byte ranges of `packed` -> (list of
        (segments, consumed) up to the first failing message, its status or
        0 when every one read)."""
        m = ranges.numel() - 1
        words, mwo, segs, mso, status, consumed = self.read_messages(
            packed, ranges, try_mode=True, limit=limit, stream=stream)
        st = status.cpu().tolist()
        mwo_h, mso_h = mwo.cpu().tolist(), mso.cpu().tolist()
        seg_h = segs.cpu().numpy().view(np.uint64) if segs.numel() else np.zeros(0, np.uint64)
        cons = consumed.cpu().tolist()
        out = []
        for k in range(m):
            if st[k] != 0:
                return out, st[k]
            a, p = mwo_h[k], []
            for j in range(mso_h[k], mso_h[k + 1]):
                ln = int(seg_h[j]) & 0xFFFFFFFF
                p.append(words[a:a + ln])
                a += ln
            out.append((p, cons[k]))
        return out, 0

    def decode_stream(self, packed, limit=8 * 1024 * 1024, words_cap=None, msgs_cap=None,
                      segs_cap=None, stream=None):
        """try_read_message's loop over one device stream in one pass
        (capnp_gpu_read_message_stream): the stream is decoded once and its
        messages described in place.  -> (words, msg_byte_off, body_word_off,
        seg_words, msg_seg_off, nmsg, clean) as device tensors (nmsg + 1
        entries for the offset lists): message m's segments start at word
        body_word_off[m] of words, with lengths seg_words[msg_seg_off[m]:
        msg_seg_off[m + 1]]; clean = the loop ended at the end of the stream.
        Capacities None are guessed (decoded words: twice the packed words)
        and grown to what the library reports on
        CAPNP_E_BUFFER_NOT_LARGE_ENOUGH (each retry decodes again)."""
        import torch
        dev = packed.device
        nb = int(packed.numel())
        wc = int(words_cap if words_cap is not None else nb // 4 + 64)
        mc = int(msgs_cap if msgs_cap is not None else nb // 1024 + 64)
        sc = int(segs_cap if segs_cap is not None else mc)
        o = _lib.ReaderOptionsC(int(limit or 0), 1 if limit is not None else 0, 64)
        for _ in range(4):
            words = torch.empty(max(wc, 1), dtype=torch.int64, device=dev)
            mbo = torch.empty(mc + 1, dtype=torch.int64, device=dev)
            bwo = torch.empty(max(mc, 1), dtype=torch.int64, device=dev)
            segw = torch.empty(max(sc, 1), dtype=torch.int64, device=dev)
            mso = torch.empty(mc + 1, dtype=torch.int64, device=dev)
            n, cl = C.c_size_t(0), C.c_int32(0)
            wn, mn, sn = C.c_size_t(0), C.c_size_t(0), C.c_size_t(0)
            st = _lib.lib().capnp_gpu_read_message_stream(
                self._h, _ptr(packed) if nb else None, nb, C.byref(o), _ptr(words), wc,
                _ptr(mbo), _ptr(bwo), mc, _ptr(segw), sc, _ptr(mso), C.byref(n), C.byref(cl),
                C.byref(wn), C.byref(mn), C.byref(sn), self._stream(stream))
            if st == 9:  # CAPNP_E_BUFFER_NOT_LARGE_ENOUGH: grow and decode again
                wc, mc, sc = max(wc, wn.value), max(mc, mn.value), max(sc, sn.value)
                continue
            _check(st, self._h)
            k = n.value
            return (words, mbo[:k + 1], bwo[:k], segw[:int(mso[k].item()) if k else 0],
                    mso[:k + 1], k, bool(cl.value))
        raise _lib.CapnpError(9, "read_message_stream: capacities did not settle")

    def read_message_stream(self, packed, limit=8 * 1024 * 1024, stream=None, max_msgs=None):
        """serialize_packed::try_read_message in a loop over one device
        stream until it returns None or fails (serialize.rs:310-325).
        -> (messages, end): messages = list of (segment word arrays as device
        tensors, consumed bytes) in stream order; end = CAPNP_NONE (1) after
        a clean end, else the status of the try_read_message that failed.
        One pass (decode_stream) finds and describes the messages; where it
        stops short of a clean end, the next message is read as the loop's
        next try_read_message (capnp_gpu_read_messages), which fails as the
        reference does, or succeeds and the loop goes on after it.
        max_msgs caps the messages one pass lists (None: no cap): a pass that
        finds more hands out the first max_msgs and the next pass decodes the
        stream again from the message after them."""
        import torch
        nb = int(packed.numel())
        out, start = [], 0
        while start < nb:
            view = packed[start:]
            rest = nb - start
            words, mbo, bwo, segw, mso, n, clean = self.decode_stream(
                view, limit=limit, msgs_cap=max_msgs, stream=stream)
            mbo_h, bwo_h, mso_h = mbo.cpu().tolist(), bwo.cpu().tolist(), mso.cpu().tolist()
            seg_h = segw.cpu().tolist()
            take = n if max_msgs is None else min(n, int(max_msgs))
            for k in range(take):
                a, p = bwo_h[k], []
                for j in range(mso_h[k], mso_h[k + 1]):
                    ln = seg_h[j]
                    p.append(words[a:a + ln])
                    a += ln
                out.append((p, mbo_h[k + 1] - mbo_h[k]))
            if take < n:  # the cap: the next pass starts at message `take`
                start += mbo_h[take]
                continue
            stop = mbo_h[n]
            if clean or stop >= rest:
                break
            # the loop's next try_read_message, from `stop`
            tail = torch.tensor([stop, rest], dtype=torch.int64, device=packed.device)
            msgs, bad = self._read_ranges(view, tail, limit, stream)
            if bad:
                return out, bad
            out += msgs
            start += stop + int(msgs[0][1])
        return out, 1

    def read_flat_messages(self, buf, slice_off, segs_cap=None, no_alloc=False,
                           limit=8 * 1024 * 1024, stream=None):
        """serialize::read_message_from_flat_slice (or its _no_alloc twin)
        for a batch of unpacked messages on the device
        (capnp_gpu_read_flat_messages): message m is read from the slice
        buf[slice_off[m]:slice_off[m+1]].  Returns (seg_words, msg_seg_off,
        status, body_off, consumed) as device tensors; seg_words holds the
        ABI's uint32 lengths in int32 storage (read them through
        `seg_words_u32`).  limit None = no traversal limit.  segs_cap None
        sizes the segment array in two phases: one entry per message first,
        then exactly msg_seg_off[nmsg] on CAPNP_E_BUFFER_NOT_LARGE_ENOUGH.
        slice_off must be non-decreasing and end within buf (checked by the
        library on the device, CapnpError 64 otherwise)."""
        import torch
        if buf.dtype != torch.uint8 or buf.dim() != 1 or not buf.is_contiguous():
            raise CapnpError(64, "buf must be a contiguous 1-D uint8 tensor")
        nmsg = slice_off.numel() - 1
        dev = slice_off.device
        slice_off = slice_off.to(torch.int64).contiguous()
        mso = torch.empty(nmsg + 1, dtype=torch.int64, device=dev)
        status = torch.empty(max(nmsg, 1), dtype=torch.int32, device=dev)
        body_off = torch.empty(max(nmsg, 1), dtype=torch.int64, device=dev)
        consumed = torch.empty(max(nmsg, 1), dtype=torch.int64, device=dev)
        o = _lib.ReaderOptionsC(int(limit or 0), 1 if limit is not None else 0, 64)
        cap = int(segs_cap) if segs_cap is not None else max(nmsg, 1)
        for phase in range(2):
            segs = torch.empty(max(cap, 1), dtype=torch.int32, device=dev)
            st = _lib.lib().capnp_gpu_read_flat_messages(
                self._h, _ptr(buf), buf.numel(), _ptr(slice_off), nmsg, C.byref(o),
                int(bool(no_alloc)),
                _ptr(segs), cap, _ptr(mso), _ptr(status), _ptr(body_off), _ptr(consumed),
                self._stream(stream))
            if st == 9 and segs_cap is None and phase == 0:
                cap = int(mso[nmsg])
                continue
            break
        _check(st, self._h)
        return segs, mso, status[:nmsg], body_off[:nmsg], consumed[:nmsg]

    # ---- streaming host batch (host buffers; pinned for overlap) ---------
    def stream_pack(self, words, chunk_word_off, out, out_off, slice_words=0):
        """capnp_stream_pack_batch on host tensors (CPU torch tensors, ideally
        pinned): words int64, chunk_word_off int64[n+1], out uint8,
        out_off int64[n+1].  Returns the packed total."""
        n = chunk_word_off.numel() - 1
        st = _lib.lib().capnp_stream_pack_batch(self._h, _ptr(words), _ptr(chunk_word_off), n,
                                                _ptr(out), out.numel(), _ptr(out_off),
                                                int(slice_words))
        _check(st, self._h)
        return int(out_off[n]) if n else 0

    def stream_unpack(self, packed, in_byte_off, out_word_off, words, status, consumed=None,
                      slice_words=0):
        """capnp_stream_unpack_batch on host tensors (see stream_pack)."""
        n = in_byte_off.numel() - 1
        st = _lib.lib().capnp_stream_unpack_batch(self._h, _ptr(packed), _ptr(in_byte_off), n,
                                                  _ptr(words), _ptr(out_word_off), _ptr(status),
                                                  _ptr(consumed), int(slice_words))
        _check(st, self._h)

    def gen_batch(self, words, offs, kind=0, pz_thresh=0, kinds=None, id0=0, stream=None):
        n = offs.numel() - 1
        st = _lib.lib().capnp_gpu_gen_batch(self._h, _ptr(words), _ptr(offs), n, int(id0),
                                            _ptr(kinds), int(kind), int(pz_thresh),
                                            self._stream(stream))
        _check(st, self._h)

    def gen_carsales(self, words, skip_requests=0, stream=None):
        """Fill `words` (int64, HBM) with the reference benchmark's carsales
        request stream (capnp_gpu_gen_carsales) -> host list of request word
        offsets (nreq + 1 entries).  The last request is cut at
        words.numel(), but its end offset is the uncut request's (it may
        exceed words.numel(): use the first nreq - 1 requests as whole
        messages)."""
        import numpy as np
        total = words.numel()
        cap = total // 3 + 2
        offs = np.zeros(cap + 1, np.uint64)
        nreq = C.c_size_t(0)
        st = _lib.lib().capnp_gpu_gen_carsales(
            self._h, _ptr(words), total, int(skip_requests),
            C.c_void_p(offs.ctypes.data), cap, C.byref(nreq), self._stream(stream))
        _check(st, self._h)
        return offs[:nreq.value + 1]


def carsales_plan(total_words, skip_requests=0):
    """Host walk of the carsales FastRand chain (no device needed):
    -> (states uint32[nreq, 4], request word offsets uint64[nreq + 1])."""
    import numpy as np
    cap = total_words // 3 + 2
    seed = np.array([0x1d2acd47, 0x58ca3e14, 0xf563f232, 0x0bc76199], np.uint32)
    states = np.zeros((cap, 4), np.uint32)
    offs = np.zeros(cap + 1, np.uint64)
    m = _lib.lib().capnp_carsales_plan(seed.ctypes.data, int(skip_requests), int(total_words),
                                       states.ctypes.data, offs.ctypes.data, cap)
    return states[:m], offs[:m + 1]


WORD_TILE_MEAN = 512  # capi.hip kWordTileMean


def tile_chunks_for(total_words, nchunks, lib=None):
    """Chunks per pack workgroup: the staged path holds
    capnp_pack_tile_words() / 64 steps of 64 words per tile and a chunk
    takes whole steps, so the budget is counted in steps of the mean chunk
    (pack.hip kStageSteps; the same rule as capi.hip)."""
    import math
    if nchunks <= 0:
        return 16
    if total_words / nchunks >= WORD_TILE_MEAN:
        return 0  # word tiles (pack.hip pack_wt_kernel): chunks of any length
    tw = (lib or _lib.lib()).capnp_pack_tile_words()
    steps = max(1, math.ceil(total_words / nchunks / 64.0))
    return int(max(1, min(64, (tw // 64) // steps)))


def unpack_tile_chunks_for(total_words, nchunks, lib=None, sync=False):
    """Chunks per unpack tile: about capnp_unpack_tile_words() output words
    per 256-thread tile (the staged path's descriptor capacity, unpack.hip),
    or capnp_unpack_sync_tile_words() per wave sub-tile when the record sync
    index is used.  For a mean chunk of WORD_TILE_MEAN words or more: 0, the
    library's long-chunk path (word tiles through the index, unpack.hip
    unpack_wt_kernel; without it the speculative block walk, resync.hip)."""
    L = lib or _lib.lib()
    tw = L.capnp_unpack_sync_tile_words() if sync else L.capnp_unpack_tile_words()
    if nchunks <= 0:
        return max(1, tw // 128)
    mean = max(total_words / nchunks, 1.0)
    if mean >= WORD_TILE_MEAN:
        return 0  # the library's long-chunk path: word tiles, or resync with no index
    return int(max(1, min(64, tw // mean)))


_default = {}


def default_context(device=0):
    ctx = _default.get(device)
    if ctx is None:
        ctx = Context(device)
        _default[device] = ctx
    return ctx
