"""CPU check of the read_message mid-size body decode's logic (tests/emu_mid.py
restates csrc/unpack.hip unpack_mid): on bodies the oracle packs (every fill
kind, runs across the waves' quarter cuts) and on garbage after a valid table,
an accepted decode consumes exactly what the reference's read_exact consumes
(oracle) with a successful status, and every segment's descriptors start on
the true record chain; valid bodies are accepted."""
import numpy as np

import emu_mid as M
import oracle_lib as O


def _run(data, k):
    tab = O.pack(np.array([k << 32], np.uint64).tobytes())[1]
    P0 = len(tab)
    assert data[:P0] == tab
    B = list(np.frombuffer(bytes(data) + bytes(2100), np.uint8).astype(np.int64)[P0:])
    L = min(len(data) - P0, 10 * k + 16)
    acc, used, entries = M.mid(B, L, k)
    rst, _, rused = O.read_message(bytes(data))
    if acc:
        assert rst == 0 and rused == P0 + used, (len(data), rst, rused, used)
        starts = M.true_starts(B, L)
        assert all(e in starts for e in entries)
    return acc, rst


def test_mid_valid_bodies_accepted():
    for k in (600, 1024, 1500):
        for kind in (0, 1, 2):
            w = O.gen_fill(np.array([0, k], np.uint64), kinds=np.array([kind], np.uint8),
                           pz=O.PZ30, id0=70 + k + kind)
            msg = O.write_message([w])[1]
            acc, rst = _run(msg, k)
            assert rst == 0 and acc, (k, kind)
            acc, rst = _run(msg + O.write_message([w[:3]])[1], k)
            assert rst == 0 and acc
            _run(msg[:-1], k)  # (truncated: accepted only if the oracle agrees)


def test_mid_runs_across_quarters_and_garbage():
    rng = np.random.default_rng(8)
    for k in (800, 1500):
        w = np.zeros(k, np.uint64)
        w[:k // 4 - 7] = 0x0102030405060708
        w[k // 2 + 5:] = 0x1112131415161718
        msg = O.write_message([w])[1]
        acc, rst = _run(msg, k)
        assert rst == 0 and acc
    for _ in range(12):
        k = int(rng.integers(500, 1500))
        body = rng.integers(0, 256, int(rng.integers(5200, 9000))).astype(np.uint8).tobytes()
        data = O.pack(np.array([k << 32], np.uint64).tobytes())[1] + body
        _run(data, k)  # an accepted garbage body must be the oracle's valid read
