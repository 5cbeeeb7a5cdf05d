"""CPU check of the long-unit decode's window logic (tests/emu_long.py
restates csrc/unpack.hip unpack_long's spec walks and rounds): at the fixed
point every segment's entry is the first record start of the true chain at
or past the segment start, the words of the segments add up to the true
chain's, and the rounds' repair walks stay short (the rule that lets a spec
walk stand in for an entry below its segment)."""
import bisect

import numpy as np
import pytest

import emu_long as E
import oracle_lib as O
from emu_unpack import record_hop


def _window(kind, pz, seed, words=8192):
    offs = np.array([0, words], np.uint64)
    w = O.gen_fill(offs, kinds=np.array([kind], np.uint8), pz=pz, id0=100 + seed)
    st, p = O.pack(w.tobytes())
    assert st == 0
    L = min(len(p), E.WIN + 2080)
    return bytes(p[:L]) + bytes(64), L


@pytest.mark.parametrize("kind,pz", [(0, O.PZ30), (0, O.PZ80), (1, O.PZ30), (2, O.PZ30)])
def test_long_unit_window_exact(kind, pz):
    for seed in range(4):
        B, L = _window(kind, pz, seed)
        own, wd, e, rounds, hops = E.window(B, L)
        starts, _ = E.true_starts(B, L)
        Lc = min(L, E.WIN)
        segb = (Lc + E.THREADS - 1) // E.THREADS if Lc > E.SEG_MIN * E.THREADS else E.SEG_MIN
        nact = (Lc + segb - 1) // segb
        for t in range(1, nact):
            i = bisect.bisect_left(starts, t * segb)
            if i < len(starts):
                assert e[t] == starts[i], (seed, t)
        # words of the segments = words of the true chain up to the last exit
        x = max(own[:nact])
        q, wt = 0, 0
        while q < x:
            q, dw, _ = record_hop(B, q, L)
            wt += dw
        assert q == x and sum(wd[:nact]) == wt, seed
        assert rounds <= 20 and sum(hops) < 8 * E.THREADS, (seed, rounds, hops)
