"""CPU restatement of read_message's short-body decode (csrc/unpack.hip
unpack_small: 64 segments, a 96-byte spec lead-in, meet / repair rounds with
unpack_long's rules) checked against the true record chain: the rounds reach
their fixed point within 65, every settled entry is a true record start (or
passes through inside a record), and the words before the segment holding
word n add up to the chain's.  Without the below-segment rule a missed spec
walk's far garbage exit sent runs of successors walking from far back
(profiles/r05z_small_read_ab.txt); the repair-hop bound pins that."""
import numpy as np
import pytest

import oracle_lib as O


def _hop(B, p, w):
    tag = B[p]
    isz, isf = tag == 0, tag == 0xFF
    cnt = B[p + 9] if isf else (B[p + 1] if isz else 0)
    ext = 8 * B[p + 9] + 1 if isf else (1 if isz else 0)
    return p + bin(tag).count("1") + ext + 1, w + 1 + cnt


def _emulate(body, n, lead=96, ns=64):  # (unpack.hip UNPACK_SMALL_LEAD)
    L = len(body)
    B = list(body) + [0] * 4200
    sb = [L * j // ns for j in range(ns)]
    se = [L * (j + 1) // ns for j in range(ns)]
    f, xs, ws, xsp, serr = [0] * ns, [0] * ns, [0] * ns, [0] * ns, [False] * ns
    for j in range(ns):
        p, w = (0 if j == 0 else max(sb[j] - lead, 0)), 0
        while p < sb[j]:
            p, w = _hop(B, p, w)
        f[j], wf = p, w
        while p < se[j]:
            p, w = _hop(B, p, w)
        serr[j] = p > L
        xs[j], ws[j] = (0 if serr[j] else p), w - wf
        xsp[j] = 0 if (serr[j] or f[j] >= se[j]) else xs[j]
    own, wd, used = xsp[:], ws[:], [0] + [None] * (ns - 1)
    rounds = max_hops = 0
    while True:
        x = np.maximum.accumulate(own).tolist()
        e = [0] + x[:-1]
        need = [e[j] != used[j] for j in range(ns)]
        if not any(need):
            break
        rounds += 1
        assert rounds <= ns + 1
        for j in range(ns):
            if not need[j]:
                continue
            used[j] = e[j]
            if e[j] < sb[j] or e[j] == f[j]:
                own[j], wd[j] = xsp[j], ws[j]
                continue
            pt, wt, ps, wsp, met, h = e[j], 0, f[j], 0, False, 0
            while pt < se[j]:
                while ps < pt and ps < se[j]:
                    ps, wsp = _hop(B, ps, wsp)
                    h += 1
                if ps == pt:
                    met = True
                    break
                pt, wt = _hop(B, pt, wt)
                h += 1
            max_hops = max(max_hops, h)
            if met:
                own[j], wd[j] = xsp[j], wt + ws[j] - wsp
            else:
                own[j] = 0 if (pt > L or e[j] >= se[j]) else pt
                wd[j] = wt
    return used, wd, rounds, max_hops, B


@pytest.mark.parametrize("kind", [0, 1, 2])
@pytest.mark.parametrize("words", [64, 128, 300, 511, 640, 896])
def test_small_rounds_match_true_chain(kind, words):
    w = O.gen_fill(np.array([0, words], np.uint64), kinds=np.array([kind], np.uint8),
                   pz=O.PZ30, id0=77 + words + kind)
    st, body = O.pack(w.tobytes())
    assert st == 0
    if len(body) > 3072:  # (kSmallBytes is 2048 now; the emulator's logic holds past it)
        pytest.skip("past the short-body limit")
    used, wd, rounds, max_hops, B = _emulate(body, words)
    # the true chain's record starts and the words before each
    starts, p, acc = {}, 0, 0
    while p < len(body):
        starts[p] = acc
        p, acc = _hop(B, p, acc)
    assert acc == words
    seg_end = [len(body) * (j + 1) // 64 for j in range(64)]
    for j, e in enumerate(used):
        if e < seg_end[j]:
            assert e in starts, (j, e)   # a settled entry is a true record start
            assert starts[e] == sum(wd[:j]), j
    assert sum(wd) == words
    assert max_hops <= 64   # repairs stay short (the meet and below-segment rules)
