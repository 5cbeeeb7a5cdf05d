"""CPU check of the index-free segment walk's logic (tests/emu_unpack.py
restates csrc/unpack.hip spec_seg_tile): on packed chunks from the oracle
(config-2 data, zero-heavy, literal-run-heavy, adversarial literal runs
across segments) every chunk resolves with exact segment exits and the
chunk's word count, in a few rounds, and the descriptor pass (records kept
from the walks plus a walk over the rest) yields exactly the true chain's
(word, record start) pairs."""
import numpy as np

import emu_unpack as E
import oracle_lib as O


def _chunks(words, offs):
    st, packed, poff = O.pack_batch(words, offs)
    assert st == 0
    B0 = bytes(packed) + bytes(2100)
    for c in range(len(offs) - 1):
        a, b = int(poff[c]), int(poff[c + 1])
        yield B0[a:b + 2100], b - a, int(offs[c + 1] - offs[c])


def _check(words, offs, max_rounds, ov=32, k=12):
    worst = 0
    for B, L, n in _chunks(words, offs):
        if L == 0:
            continue
        x, wd, err, rounds, descs = E.seg_walk(B, L, OV=ov, K=k, descs=True)
        assert not any(err) and sum(wd) == n and x[-1] == L
        assert x == E.true_exits(B, L)
        assert descs == E.true_records(B, L)
        worst = max(worst, rounds)
    assert worst <= max_rounds, worst


def test_segment_walk_config2_kinds():
    n, cw = 150, 128
    offs = np.arange(0, (n + 1) * cw, cw, dtype=np.uint64)
    for kind in (0, 1, 2):
        for ov in (0, 32):
            _check(O.gen_fill(offs, kind0=kind, pz=O.PZ30), offs, 16, ov)
        _check(O.gen_fill(offs, kind0=kind, pz=O.PZ30), offs, 16, 48, 2)  # (records past K)


def test_segment_walk_literal_and_zero_runs():
    n, cw = 100, 128
    offs = np.arange(0, (n + 1) * cw, cw, dtype=np.uint64)
    rng = np.random.default_rng(1)
    lit = rng.integers(1 << 56, 1 << 63, n * cw, dtype=np.uint64) * 2 + 1
    _check(lit, offs, 16)
    _check(lit, offs, 16, 0)
    _check(lit, offs, 16, 48, 1)
    z = np.zeros(n * cw, np.uint64)
    z[::37] = 5
    _check(z, offs, 16)
    _check(z, offs, 16, 0)
    # literal runs of every length placed across segment boundaries
    w = np.zeros(n * cw, np.uint64)
    for c in range(n):
        k = c % 120
        w[c * cw + 3:c * cw + 3 + k] = 0x1112131415161718
        w[c * cw + 3 + k::7][:4] = 0x0000000100000001
    _check(w, offs, 16)
    _check(w, offs, 16, 0)
    _check(w, offs, 16, 48, 3)
