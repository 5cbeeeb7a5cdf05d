"""CPU check of the pack kernels' step formulas (tests/emu_pack.py, a
bit-level emulation of pack_cs_kernel / pack_lean_kernel's masks, sizes and
run counts) against the oracle: the arithmetic is pinned here before the
GPU parity tests run the kernels themselves."""
import random

import numpy as np

import emu_pack as E
import oracle_lib as O


def _cases():
    sizes = [0, 1, 2, 7, 8, 63, 64, 65, 127, 128, 129, 191, 192, 255, 256, 257, 320, 511, 512]
    for kind in (0, 1, 2):
        offs = np.concatenate([[0], np.cumsum(sizes)]).astype(np.uint64)
        words = O.gen_fill(offs, kind0=kind, pz=O.PZ30)
        for i in range(len(sizes)):
            yield words[int(offs[i]):int(offs[i + 1])]
    rng = random.Random(1)
    for _ in range(200):
        n = rng.choice([1, 5, 64, 100, 128, 200, 300, 512])
        yield np.array([rng.choice([0, 0, 0xFFFFFFFFFFFFFFFF, 0x0101010101010100,
                                    rng.getrandbits(64)]) for _ in range(n)], np.uint64)


def test_step_formulas_match_oracle():
    for c in _cases():
        st, ref = O.pack(c.tobytes())
        assert st == 0
        if len(c) <= 128:
            assert E.cs_chunk(c) == ref, len(c)
        assert E.lean_chunk(c) == ref, len(c)
