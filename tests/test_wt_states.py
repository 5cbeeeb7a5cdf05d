"""CPU restatement of how pack_wt_kernel (csrc/pack.hip) gets the run state
entering each 512-word range of a word tile without global searches
(range_exit / wt_compose, round 4), checked against the reference's own
sequential scan (PackedWrite::write_all, serialize_packed.rs:375-427: a
0x00 tag absorbs up to 255 following zero words, a 0xFF tag up to 255
following words with at most one zero byte; a write_all chunk start is
always a head).

State = (type, rem): the open run entering a word (0 none, 1 zero run,
2 literal run) and how many more words it may absorb.  Two states are
equivalent at word i when both do (or neither does) absorb word i."""
import random

import numpy as np
import pytest

import oracle_lib as O


def tags(words):
    b = words.view(np.uint8).reshape(-1, 8)
    return ((b != 0) * (1 << np.arange(8))).sum(1).astype(np.int64)


def pop(x):
    return bin(int(x)).count("1")


def in_class(T, tag):
    return tag == 0 if T == 1 else pop(tag) >= 7


def reference_states(t, starts):
    """State entering every word, by the reference's scan."""
    ent, typ, rem = [], 0, 0
    for i in range(len(t)):
        ent.append((typ, rem))
        if typ and rem > 0 and i not in starts and in_class(typ, t[i]):
            rem -= 1
            continue
        typ, rem = (1, 255) if t[i] == 0 else (2, 255) if t[i] == 0xFF else (0, 0)
    ent.append((typ, rem))
    return ent


def canon(s, i, t, starts):
    if i >= len(t):
        return s
    absorbs = s[0] and s[1] > 0 and i not in starts and in_class(s[0], t[i])
    return s if absorbs else (0, 0)


def sure_head(tag, ptag):
    """pack.hip sure_head: a head whatever state precedes it."""
    p, pp = pop(tag), pop(ptag)
    z, pz = tag == 0, ptag == 0
    brk, pbrk = (not z) and p <= 6, (not pz) and pp <= 6
    return z != pz or brk or (p >= 7 and pbrk)


def scan_from(t, s, R, starts):
    typ, rem = 0, 0
    for i in range(s, R):
        if i != s and typ and rem > 0 and i not in starts and in_class(typ, t[i]):
            rem -= 1
            continue
        typ, rem = (1, 255) if t[i] == 0 else (2, 255) if t[i] == 0xFF else (0, 0)
    return typ, rem


def range_exit(t, R0, nw, starts):
    """pack.hip range_exit: (state at R0 + nw, None) from the range's words, or
    (None, T) when the range holds no sure head and is one all-zero (T = 1) /
    all-0xFF (T = 2) stretch, or (None, 3) otherwise."""
    ks = None
    for i in range(R0 + nw - 1, R0 - 1, -1):
        if i in starts or (i > R0 and sure_head(t[i], t[i - 1])):
            ks = i
            break
    seg = t[(ks if ks is not None else R0):R0 + nw]
    allz, allf = all(x == 0 for x in seg), all(x == 0xFF for x in seg)
    if ks is None:
        return None, (1 if allz else 2 if allf else 3)
    if allz or allf:
        return ((1 if allz else 2), 255 - (R0 + nw - 1 - ks) % 256), None
    return scan_from(t, ks, R0 + nw, starts), None


def wt_compose(c, T, n):
    """pack.hip wt_compose: the state after n words of one T stretch."""
    a = c[1] if c[0] == T else 0
    if a >= n:
        return (T, a - n)
    return (T, 255 - (n - a - 1) % 256)


@pytest.mark.parametrize("kind", [0, 1, 2])
def test_range_states_match_reference_scan(kind):
    rng = random.Random(70 + kind)
    for trial in range(12):
        sizes = [rng.choice([9, 300, 700, 2500, 5000]) for _ in range(6)]
        offs = np.concatenate([[0], np.cumsum(sizes)]).astype(np.uint64)
        w = O.gen_fill(offs, kind0=kind, pz=O.PZ30, id0=trial * 13 + kind)
        t = tags(w)
        starts = set(int(x) for x in offs[:-1])
        ent = reference_states(t, starts)
        n = len(t)
        for T0 in range(0, n, 2048):  # tiles: the plan kernel's entry at T0
            c = ent[T0]
            for wv in range(4):
                R0 = T0 + 512 * wv
                if R0 >= n:
                    break
                assert canon(c, R0, t, starts) == canon(ent[R0], R0, t, starts), (trial, R0)
                nw = min(512, n - R0)
                if R0 + nw >= min(T0 + 2048, n):
                    break
                ex, hg = range_exit(t, R0, nw, starts)
                if hg in (1, 2):
                    c = wt_compose(c, hg, nw)
                elif hg == 3:
                    c = ent[R0 + nw]  # (the kernel searches before R0: exact)
                else:
                    c = ex


def test_compose_long_stretches():
    """All-zero and all-0xFF stretches far longer than a run, entered in every
    phase: composition over 512-word ranges equals the scan."""
    for fill in (0, 0xFF):
        t = np.array([7] + [fill] * 5000, np.int64)  # a head that opens no run, then the stretch
        ent = reference_states(t, {0})
        for R0 in range(1, 4000, 37):
            got = wt_compose(ent[R0], 1 if fill == 0 else 2, 512)
            assert canon(got, R0 + 512, t, {0}) == canon(ent[R0 + 512], R0 + 512, t, {0})
