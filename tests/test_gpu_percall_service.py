"""The per-message calls' resident services (csrc/capi.hip CallSvc, common.h
svc_next): a write_message / read_message within 1 ms of the previous
per-message call is served by a resident workgroup polling a pinned doorbell
instead of a launch.  Every path of that protocol against the oracle
(serialize.rs:574-679 write, :448-524 read; serialize_packed.rs:233-255,
446-453):

* back-to-back calls (a live service rung directly), alternating kinds;
* gaps around the trust window (150 us), the service's idle exit (250 us)
  and the warm window (1 ms): a new generation, or the one-launch kernel;
* a device-wide synchronisation between calls (it waits for the resident
  workgroup's idle exit and must not hang);
* a pinned-buffer growth between calls (services stopped before it moves);
* a context destroyed while its services are resident, then a new one;
* malformed inputs (statuses) through the service.
"""
import random
import time

import numpy as np
import pytest

import oracle_lib as O
from test_gpu_long_units import _read_message_call
from test_gpu_parity import _rand_segment, _runs_segment

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


def _ctx():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from capnp_amd import Context
    return Context(0)


def _messages(seed, n):
    rng = random.Random(seed)
    out = []
    for i in range(n):
        nseg = rng.choice([1, 1, 2, 3, 7])
        gen = rng.choice([_rand_segment, _runs_segment])
        segs = [gen(rng, rng.choice([0, 1, 5, 64, 127, 128, 700, 1500]))
                for _ in range(nseg)]
        if sum(len(s) for s in segs) > 8000:
            segs = segs[:1]
        st, ref = O.write_message(segs)
        assert st == 0
        out.append((segs, ref))
    return out


def _write(ctx, segs):
    from capnp_amd import serialize_packed as sp
    out = bytearray()
    sp.write_message(out, segs, ctx=ctx)
    return bytes(out)


def _read_check(ctx, data, what):
    rst, rsegs, rused = O.read_message(bytes(data))
    r, body, used = _read_message_call(ctx.handle, data)
    assert r == rst, what
    if rst == 0:
        assert used == rused, what
        flat = np.concatenate([np.asarray(s, np.uint64) for s in rsegs]) if rsegs else \
            np.zeros(0, np.uint64)
        assert np.array_equal(body[:len(flat)], flat), what


def test_back_to_back_alternating():
    ctx = _ctx()
    try:
        for k, (segs, ref) in enumerate(_messages(1, 300)):
            assert _write(ctx, segs) == ref, k
            _read_check(ctx, ref, k)
    finally:
        ctx.close()


@pytest.mark.parametrize("gap_us", [0, 100, 200, 300, 600, 1200, 3000])
def test_gaps_between_calls(gap_us):
    """Each gap a few times, so that both kinds see it as the time since
    their own last request and since the previous per-message call."""
    ctx = _ctx()
    try:
        for k, (segs, ref) in enumerate(_messages(100 + gap_us, 40)):
            assert _write(ctx, segs) == ref, (gap_us, k)
            time.sleep(gap_us * 1e-6)
            _read_check(ctx, ref, (gap_us, k))
            time.sleep(gap_us * 1e-6)
    finally:
        ctx.close()


def test_device_synchronize_between_calls():
    ctx = _ctx()
    try:
        for k, (segs, ref) in enumerate(_messages(7, 30)):
            assert _write(ctx, segs) == ref, k
            t0 = time.perf_counter()
            torch.cuda.synchronize()
            assert time.perf_counter() - t0 < 0.5  # (the idle exit is 250 us)
            _read_check(ctx, ref, k)
    finally:
        ctx.close()


def test_pinned_growth_between_calls():
    """Small calls (resident services), then a message whose staging grows
    the pinned buffer, then small calls again."""
    ctx = _ctx()
    rng = random.Random(9)
    try:
        small = _messages(3, 6)
        for segs, ref in small:
            assert _write(ctx, segs) == ref
            _read_check(ctx, ref, "small")
        big = [_rand_segment(rng, 8400)]
        st, ref = O.write_message(big)
        assert _write(ctx, big) == ref
        _read_check(ctx, ref, "big")
        for segs, ref in small:
            assert _write(ctx, segs) == ref
            _read_check(ctx, ref, "small again")
    finally:
        ctx.close()


def test_close_with_resident_services():
    for round_ in range(3):
        ctx = _ctx()
        for segs, ref in _messages(20 + round_, 5):
            assert _write(ctx, segs) == ref
            _read_check(ctx, ref, round_)
        ctx.close()  # (both services resident: stopped and waited for)


def test_malformed_inputs_through_service():
    """Truncated, corrupted and oversized inputs, each right after a good call
    (so the service serves them), statuses against the oracle."""
    ctx = _ctx()
    rng = np.random.default_rng(12)
    try:
        for k, (segs, ref) in enumerate(_messages(44, 40)):
            _read_check(ctx, ref, ("good", k))
            cut = ref[:int(rng.integers(0, len(ref)))] if len(ref) else ref
            _read_check(ctx, cut, ("cut", k))
            bad = bytearray(ref)
            if bad:
                bad[int(rng.integers(0, len(bad)))] ^= 0xFF
            _read_check(ctx, bytes(bad), ("flip", k))
    finally:
        ctx.close()


@pytest.mark.parametrize("env", [{"CAPNP_PERCALL_BAR": "0"}, {"CAPNP_SVC_LINE_BAR": "1"},
                                 {"CAPNP_PERCALL_SERVICE": "0"}])
def test_staging_variants(env):
    """The inputs staged in pinned memory (no BAR path), the request line in
    device memory, and one launch per call: each in its own process (the
    switches are read once)."""
    import os
    import subprocess
    import sys
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    here = os.path.dirname(os.path.abspath(__file__))
    r = subprocess.run([sys.executable, os.path.join(here, "_percall_worker.py"), "31"],
                       env={**os.environ, **env}, capture_output=True, text=True, timeout=100)
    assert r.returncode == 0 and r.stdout.strip().endswith("ok"), (r.stdout[-2000:],
                                                                   r.stderr[-2000:])
