"""ctypes binding of the gfx950 codec library (libcapnp_packed.so, C ABI in
include/capnp_packed.h).  No CPU fallback exists: a missing library or a
missing gfx950 device raises."""
import ctypes as C
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
PKG_ROOT = os.path.dirname(HERE)
# (CAPNP_PACKED_LIB: another build of the same library, e.g. a diagnostic
# variant from the Makefile's uvariant/pvariant rules, for A/B parity runs)
LIB_PATH = os.environ.get("CAPNP_PACKED_LIB") or os.path.join(HERE, "libcapnp_packed.so")

OK = 0
NONE = 1
STATUS_NAMES = {
    0: "OK", 1: "NONE", 2: "PrematureEndOfPackedInput",
    3: "PackedInputDidNotEndCleanlyOnASegmentBoundary", 4: "FailedToFillTheWholeBuffer",
    5: "PrematureEndOfFile", 6: "InvalidNumberOfSegments", 7: "MessageSizeOverflow",
    8: "MessageTooLarge", 9: "BufferNotLargeEnough", 10: "UnalignedSegment",
    11: "MisalignedLength", 12: "MessageEndsPrematurely", 13: "EmptySlice",
    14: "MessageNotAlignedBy8BytesBoundary", 15: "Pending", 64: "InvalidArgument", 65: "NoDevice", 66: "HipError",
    67: "OutOfMemory", 68: "Io",
}
PENDING = 15
IO_PENDING = -1  # CAPNP_IO_PENDING: an inner stream callback has nothing now

# inner-stream callbacks of the streaming adaptors (capnp_read_fn / capnp_write_fn)
READ_FN = C.CFUNCTYPE(C.c_ssize_t, C.c_void_p, C.POINTER(C.c_uint8), C.c_size_t)
WRITE_FN = C.CFUNCTYPE(C.c_ssize_t, C.c_void_p, C.POINTER(C.c_uint8), C.c_size_t)

EXPORTS = [
    "capnp_ctx_create", "capnp_ctx_destroy", "capnp_ctx_stream", "capnp_ctx_last_error",
    "capnp_version", "capnp_default_reader_options", "capnp_packed_bound_bytes",
    "capnp_packed_batch_bound_bytes", "capnp_gpu_pack_batch", "capnp_gpu_unpack_batch",
    "capnp_pack", "capnp_unpack", "capnp_pack_batch_host", "capnp_unpack_batch_host",
    "capnp_packed_write_message", "capnp_packed_read_message",
    "capnp_packed_read_message_no_alloc", "capnp_gpu_gen_batch", "capnp_gpu_pack_batch_tuned",
    "capnp_ctx_reserve", "capnp_pack_tile_words", "capnp_gpu_unpack_batch_tuned",
    "capnp_unpack_tile_words", "capnp_sync_index_entries", "capnp_gpu_pack_batch_sync",
    "capnp_gpu_unpack_batch_sync", "capnp_gpu_pack_batch_sync_tuned",
    "capnp_gpu_unpack_batch_sync_tuned", "capnp_unpack_sync_tile_words",
    "capnp_stream_pack_batch", "capnp_stream_unpack_batch", "capnp_gpu_write_messages",
    "capnp_gpu_read_messages", "capnp_gpu_unpack_batch_resync", "capnp_resync_stats",
    "capnp_resync_block_bytes", "capnp_gpu_read_flat_messages", "capnp_gpu_gen_carsales",
    "capnp_packed_writer_new", "capnp_packed_writer_free", "capnp_packed_writer_write",
    "capnp_packed_writer_flush", "capnp_packed_writer_carried", "capnp_packed_reader_new",
    "capnp_packed_reader_free", "capnp_packed_reader_read", "capnp_packed_reader_read_exact",
    "capnp_packed_reader_set_readahead",
    "capnp_packed_reader_read_message", "capnp_packed_reader_buffered",
    "capnp_gpu_find_messages",
    "capnp_gpu_read_message_stream", "capnp_abi_version", "capnp_resync_max_passes",
    "capnp_unpack_prefix",
]
ABI_VERSION = 6  # include/capnp_packed.h CAPNP_ABI_VERSION


class ReaderOptionsC(C.Structure):
    _fields_ = [("traversal_limit_in_words", C.c_uint64), ("has_traversal_limit", C.c_int32),
                ("nesting_limit", C.c_int32)]


class CapnpError(Exception):
    """An error carrying a capnp::ErrorKind-style status."""

    def __init__(self, status, msg=""):
        self.status = status
        self.kind = STATUS_NAMES.get(status, str(status))
        super().__init__(f"{self.kind}{': ' + msg if msg else ''}")


_lib = None


def build():
    subprocess.check_call(["make", "-s", "-C", PKG_ROOT])


def lib():
    """Loads the library (building it in-tree if absent and hipcc exists)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        build()
    L = C.CDLL(LIB_PATH)
    vp, sz, u64, u32, i32 = C.c_void_p, C.c_size_t, C.c_uint64, C.c_uint32, C.c_int
    L.capnp_abi_version.restype = u32
    if L.capnp_abi_version() != ABI_VERSION:  # (signatures below are this revision's)
        raise ImportError(f"{LIB_PATH}: ABI {L.capnp_abi_version()}, binding expects "
                          f"{ABI_VERSION}")
    L.capnp_resync_max_passes.argtypes = [C.c_int]
    L.capnp_resync_max_passes.restype = C.c_int
    L.capnp_ctx_create.argtypes = [C.c_int, C.POINTER(C.c_int)]
    L.capnp_ctx_create.restype = vp
    L.capnp_ctx_destroy.argtypes = [vp]
    L.capnp_ctx_stream.argtypes = [vp]
    L.capnp_ctx_stream.restype = vp
    L.capnp_ctx_last_error.argtypes = [vp]
    L.capnp_ctx_last_error.restype = C.c_char_p
    L.capnp_version.restype = C.c_char_p
    L.capnp_default_reader_options.restype = ReaderOptionsC
    L.capnp_packed_bound_bytes.argtypes = [sz]
    L.capnp_packed_bound_bytes.restype = sz
    L.capnp_packed_batch_bound_bytes.argtypes = [sz, sz]
    L.capnp_packed_batch_bound_bytes.restype = sz
    L.capnp_gpu_pack_batch.argtypes = [vp, vp, vp, sz, vp, sz, vp, vp]
    L.capnp_gpu_pack_batch_tuned.argtypes = [vp, vp, vp, sz, vp, sz, vp, u32, vp]
    L.capnp_gpu_unpack_batch.argtypes = [vp, vp, vp, sz, vp, vp, vp, vp, vp]
    L.capnp_gpu_unpack_batch_tuned.argtypes = [vp, vp, vp, sz, vp, vp, vp, vp, C.c_uint32, vp]
    L.capnp_gpu_gen_batch.argtypes = [vp, vp, vp, sz, u64, vp, u32, u32, vp]
    L.capnp_gpu_gen_carsales.argtypes = [vp, vp, u64, u64, vp, sz, C.POINTER(C.c_size_t), vp]
    L.capnp_carsales_plan.argtypes = [vp, u64, u64, vp, vp, u64]
    L.capnp_carsales_plan.restype = u64
    L.capnp_unpack_sync_tile_words.argtypes = []
    L.capnp_unpack_sync_tile_words.restype = u32
    L.capnp_sync_index_entries.argtypes = [sz]
    L.capnp_sync_index_entries.restype = sz
    L.capnp_gpu_pack_batch_sync.argtypes = [vp, vp, vp, sz, vp, sz, vp, vp, vp]
    L.capnp_gpu_unpack_batch_sync.argtypes = [vp, vp, vp, sz, vp, vp, vp, vp, vp, vp]
    L.capnp_gpu_pack_batch_sync_tuned.argtypes = [vp, vp, vp, sz, vp, sz, vp, vp, u32, vp]
    L.capnp_gpu_unpack_batch_sync_tuned.argtypes = [vp, vp, vp, sz, vp, vp, vp, vp, vp, u32, vp]
    L.capnp_ctx_reserve.argtypes = [vp, sz]
    L.capnp_gpu_unpack_batch_resync.argtypes = [vp, vp, vp, sz, vp, vp, vp, vp, vp]
    L.capnp_resync_stats.argtypes = [vp, C.POINTER(C.c_int), C.POINTER(C.c_int)]
    L.capnp_resync_block_bytes.argtypes = []
    L.capnp_resync_block_bytes.restype = u32
    L.capnp_pack_tile_words.argtypes = []
    L.capnp_pack_tile_words.restype = C.c_uint32
    L.capnp_unpack_tile_words.argtypes = []
    L.capnp_unpack_tile_words.restype = C.c_uint32
    L.capnp_pack.argtypes = [vp, vp, sz, vp, sz, C.POINTER(C.c_size_t)]
    L.capnp_unpack.argtypes = [vp, vp, sz, C.POINTER(C.c_size_t), vp, sz]
    L.capnp_unpack_prefix.argtypes = [vp, vp, sz, u64, vp, C.POINTER(C.c_size_t),
                                      C.POINTER(C.c_uint64)]
    L.capnp_pack_batch_host.argtypes = [vp, vp, vp, sz, vp, sz, vp]
    L.capnp_unpack_batch_host.argtypes = [vp, vp, vp, sz, vp, vp, vp, vp]
    L.capnp_stream_pack_batch.argtypes = [vp, vp, vp, sz, vp, sz, vp, sz]
    L.capnp_stream_unpack_batch.argtypes = [vp, vp, vp, sz, vp, vp, vp, vp, sz]
    L.capnp_gpu_write_messages.argtypes = [vp, vp, vp, vp, sz, sz, sz, vp, sz, vp, vp]
    L.capnp_gpu_read_messages.argtypes = [vp, vp, vp, sz, C.POINTER(ReaderOptionsC), i32, vp, sz,
                                          vp, vp, sz, vp, vp, vp, vp]
    L.capnp_gpu_read_flat_messages.argtypes = [vp, vp, sz, vp, sz, C.POINTER(ReaderOptionsC), i32,
                                               vp, sz, vp, vp, vp, vp, vp]
    L.capnp_packed_write_message.argtypes = [vp, vp, vp, u32, vp, sz, C.POINTER(C.c_size_t)]
    L.capnp_packed_read_message.argtypes = [vp, vp, sz, C.POINTER(ReaderOptionsC), i32, vp, sz,
                                            vp, C.POINTER(C.c_uint32), C.POINTER(C.c_size_t)]
    L.capnp_packed_read_message_no_alloc.argtypes = [
        vp, vp, sz, C.POINTER(ReaderOptionsC), i32, vp, sz, C.POINTER(C.c_uint32),
        C.POINTER(C.c_size_t), C.POINTER(C.c_size_t), C.POINTER(C.c_size_t)]
    L.capnp_packed_writer_new.argtypes = [vp, WRITE_FN, vp]
    L.capnp_packed_writer_new.restype = vp
    L.capnp_packed_writer_free.argtypes = [vp]
    L.capnp_packed_writer_write.argtypes = [vp, vp, sz]
    L.capnp_packed_writer_flush.argtypes = [vp]
    L.capnp_packed_writer_carried.argtypes = [vp]
    L.capnp_packed_writer_carried.restype = sz
    L.capnp_packed_reader_new.argtypes = [vp, READ_FN, vp]
    L.capnp_packed_reader_new.restype = vp
    L.capnp_packed_reader_free.argtypes = [vp]
    L.capnp_packed_reader_set_readahead.argtypes = [vp, i32]
    L.capnp_packed_reader_read.argtypes = [vp, vp, sz, C.POINTER(C.c_size_t)]
    L.capnp_packed_reader_read_exact.argtypes = [vp, vp, sz, C.POINTER(C.c_size_t)]
    L.capnp_packed_reader_read_message.argtypes = [vp, C.POINTER(ReaderOptionsC), i32, vp, sz,
                                                   vp, C.POINTER(C.c_uint32),
                                                   C.POINTER(C.c_uint64)]
    L.capnp_gpu_find_messages.argtypes = [vp, vp, sz, sz, vp, C.POINTER(C.c_size_t), vp]
    L.capnp_gpu_read_message_stream.argtypes = [
        vp, vp, sz, C.POINTER(ReaderOptionsC), vp, sz, vp, vp, sz, vp, sz, vp,
        C.POINTER(C.c_size_t), C.POINTER(C.c_int32), C.POINTER(C.c_size_t),
        C.POINTER(C.c_size_t), C.POINTER(C.c_size_t), vp]
    L.capnp_unpack_wt_stats.argtypes = [C.POINTER(C.c_ulonglong), C.c_int]
    L.capnp_unpack_wt_stats.restype = C.c_int
    L.capnp_packed_reader_buffered.argtypes = [vp]
    L.capnp_packed_reader_buffered.restype = sz
    _lib = L
    return L


def exported_symbols():
    """Names of the C ABI entry points the library exports (checked against
    include/*.h by the CPU test-suite)."""
    L = lib()
    return [n for n in EXPORTS if hasattr(L, n)]
