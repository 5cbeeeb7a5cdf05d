"""capnp_amd — MI355X-native Cap'n Proto packed-stream codec.

The hot path (batched PACK / UNPACK of word-aligned segments) runs in
hand-written gfx950 HIP kernels behind a C ABI (include/capnp_packed.h);
this package is the host-side mirror of capnp::serialize_packed.
"""
from ._lib import CapnpError, STATUS_NAMES  # noqa: F401
from .codec import Context, default_context, tile_chunks_for, unpack_tile_chunks_for  # noqa: F401
from . import serialize_packed  # noqa: F401
from . import serialize  # noqa: F401
from . import serialize_packed_async  # noqa: F401

__all__ = ["CapnpError", "Context", "default_context", "serialize", "serialize_packed", "serialize_packed_async", "tile_chunks_for",
           "unpack_tile_chunks_for"]
