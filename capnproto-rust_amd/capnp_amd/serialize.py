"""Host mirror of the unpacked flat-slice readers of capnp::serialize
(SURVEY §8f row 4), over device-resident bytes:

  read_message_from_flat_slice          serialize.rs:53-78
  read_message_from_flat_slice_no_alloc serialize.rs:88-96 ->
                                        no_alloc_buffer_segments.rs:152-162

Both take a 1-D uint8 CUDA tensor (`slice`, may extend past the message, as
in the reference) and return (segments, remaining): the segments are
zero-copy views of the slice (the BufferSegments / NoAllocSliceSegments
get_segment results), `remaining` the rest of the slice (the reference's
`*slice` advance).  Errors raise CapnpError with the reference's kind.  The
framing runs in capnp_gpu_read_flat_messages; `read_flat_messages` is its
batch form (many slices of one buffer per call)."""
from . import _lib
from ._lib import CapnpError
from .codec import default_context, seg_words_u32
from .serialize_packed import DEFAULT_READER_OPTIONS


def read_flat_messages(buf, slice_off, options=None, no_alloc=False, segs_cap=None, ctx=None):
    """Batch form: message m read from buf[slice_off[m]:slice_off[m+1]].
    -> (seg_words, msg_seg_off, status, body_off, consumed) device tensors
    (seg_words: uint32 lengths in int32 storage, see codec.seg_words_u32).
    segs_cap None sizes the segment array exactly (two-phase call)."""
    o = options or DEFAULT_READER_OPTIONS
    ctx = ctx or default_context(buf.device.index or 0)
    return ctx.read_flat_messages(buf, slice_off, segs_cap, no_alloc=no_alloc,
                                  limit=o.traversal_limit_in_words)


def _read_one(slice_, options, no_alloc, ctx):
    import torch
    if (slice_.dtype != torch.uint8 or slice_.dim() != 1 or not slice_.is_cuda
            or not slice_.is_contiguous()):
        raise CapnpError(64, "slice must be a contiguous 1-D uint8 CUDA tensor")
    off = torch.tensor([0, slice_.numel()], dtype=torch.int64, device=slice_.device)
    segs, mso, st, body, used = read_flat_messages(slice_, off, options, no_alloc, 511, ctx)
    st, body, used = int(st[0]), int(body[0]), int(used[0])
    if st != 0:
        raise CapnpError(st)
    lens = seg_words_u32(segs[:int(mso[1])]).tolist()
    out, p = [], body
    for n in lens:
        out.append(slice_[p:p + 8 * n])
        p += 8 * n
    return out, slice_[used:]


def read_message_from_flat_slice(slice_, options=None, ctx=None):
    """serialize::read_message_from_flat_slice (serialize.rs:53-78)."""
    return _read_one(slice_, options, False, ctx)


def read_message_from_flat_slice_no_alloc(slice_, options=None, ctx=None):
    """serialize::read_message_from_flat_slice_no_alloc (serialize.rs:88-96)."""
    return _read_one(slice_, options, True, ctx)
