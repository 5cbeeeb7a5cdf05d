"""CPU checks of the drop-in boundary: the gfx950 library builds, loads
without a GPU, exports every entry point include/*.h declares, and refuses
to run without a device (no CPU fallback)."""
import ctypes as C
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADERS = [os.path.join(ROOT, "include", h) for h in ("capnp_packed.h", "capnp_packed_bench.h")]


def declared_functions():
    names = []
    for h in HEADERS:
        src = open(h).read()
        src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
        names += re.findall(r"\b(capnp_[a-z0-9_]+)\s*\(", src)
    return sorted(set(names))


def test_headers_declare_the_boundary():
    names = declared_functions()
    for must in ("capnp_gpu_pack_batch", "capnp_gpu_unpack_batch", "capnp_pack", "capnp_unpack",
                 "capnp_packed_write_message", "capnp_packed_read_message",
                 "capnp_packed_read_message_no_alloc"):
        assert must in names


def test_library_exports_every_declared_symbol():
    from capnp_amd import _lib
    L = _lib.lib()
    missing = [n for n in declared_functions() if not hasattr(L, n)]
    assert not missing, missing
    assert set(_lib.EXPORTS) == set(declared_functions())


def test_library_is_gfx950_code():
    from capnp_amd import _lib
    data = open(_lib.LIB_PATH, "rb").read()
    assert b"gfx950" in data
    assert _lib.lib().capnp_version().startswith(b"capnp-packed-mi355x")


def test_bounds_match_survey_formula():
    from capnp_amd import _lib
    L = _lib.lib()
    for n in (0, 1, 2, 7, 128, 1000):
        assert L.capnp_packed_bound_bytes(n) == (8 * n + (n + 1) // 2 + 2 if n else 0)


def test_default_reader_options():
    from capnp_amd import _lib
    o = _lib.lib().capnp_default_reader_options()
    assert o.traversal_limit_in_words == 8 * 1024 * 1024 and o.has_traversal_limit == 1
    assert o.nesting_limit == 64


def test_no_cpu_fallback_without_device():
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    from capnp_amd import _lib, Context, CapnpError
    with pytest.raises(CapnpError) as e:
        Context(0)
    assert e.value.kind == "NoDevice"
    # the host single-unit API also refuses without a context
    n = C.c_size_t(0)
    assert _lib.lib().capnp_pack(None, None, 0, None, 0, C.byref(n)) == 64


def test_seg_words_read_unsigned():
    """Segment lengths are uint32 in the ABI but land in int32 storage: a
    2^31-word segment must read back as 2^31, not negative."""
    import torch
    from capnp_amd.codec import seg_words_u32
    raw = torch.tensor([1, -1, -(2**31), 2**31 - 1], dtype=torch.int32)
    assert seg_words_u32(raw).tolist() == [1, 2**32 - 1, 2**31, 2**31 - 1]
