"""Emulation of one window of the long-unit decode (csrc/unpack.hip
unpack_long) on the CPU: test infrastructure that checks the window's
round logic (led-in spec walks over kLuSeg-byte segments, an exclusive max
of the owned exits as each segment's entry, repair walks from entries that
differ from the spec walk's first record) against the true record chain,
and counts the repair walks each round costs.  Not a decoder."""
from emu_unpack import record_hop

THREADS = 256
SEG = 64
WIN = SEG * THREADS
LEAD = 64
SEG_MIN = 8


def window(B, L, lead=LEAD):
    """Window bytes B[0:L] (zero padded), the true chain starting at 0:
    -> (exits, words, entries, rounds, repair hops per round)."""
    Lc = min(L, WIN)
    segb = (Lc + THREADS - 1) // THREADS if Lc > SEG_MIN * THREADS else SEG_MIN
    sb = [t * segb for t in range(THREADS)]
    act = [s < Lc for s in sb]
    se = [min(s + segb, Lc) if a else 0 for s, a in zip(sb, act)]
    f, xs, ws, serr = [], [], [], []
    for t in range(THREADS):
        if not act[t]:
            f.append(sb[t]); xs.append(0); ws.append(0); serr.append(False)
            continue
        p = sb[t] if t == 0 else max(0, sb[t] - lead)
        w = 0
        while p < sb[t]:
            p, dw, _ = record_hop(B, p, L)
        f.append(p)
        w = 0
        while p < se[t]:
            p, dw, _ = record_hop(B, p, L)
            w += dw
        serr.append(p > L)
        xs.append(0 if p > L else p)
        ws.append(w)
    # a spec walk that found no record start in its segment says "passes
    # through" (owns no exit); one that ran past the staged bytes owns none
    own = [(0 if (serr[t] or f[t] >= se[t]) else xs[t]) if act[t] else 0 for t in range(THREADS)]
    wd = [ws[t] if act[t] else 0 for t in range(THREADS)]
    used = [0] + [None] * (THREADS - 1)
    err = [False] * THREADS
    rewalks = []
    rounds = 0
    while True:
        e, m = [0] * THREADS, 0
        for t in range(THREADS):
            e[t] = m
            m = max(m, own[t])
        need = [act[t] and e[t] != used[t] for t in range(THREADS)]
        if not any(need):
            break
        n = 0
        for t in range(THREADS):
            if not need[t]:
                continue
            ent = used[t] = e[t]
            if ent < sb[t]:
                # not reached yet (an earlier segment passed through on a
                # wrong entry): the spec walk stands in for the successors
                own[t] = 0 if (serr[t] or f[t] >= se[t]) else xs[t]
                wd[t], err[t] = ws[t], serr[t]
            elif ent >= se[t]:
                own[t], wd[t], err[t] = 0, 0, False
            elif ent == f[t]:
                own[t], wd[t], err[t] = (0 if serr[t] else xs[t]), ws[t], serr[t]
            else:
                # from the entry, the spec chain kept in step: where they meet
                # the rest of the walk is the spec walk's
                pt, wt, ps, wsp, met = ent, 0, f[t], 0, False
                while pt < se[t]:
                    while ps < pt and ps < se[t]:
                        ps, dw, _ = record_hop(B, ps, L)
                        wsp += dw
                        n += 1
                    if ps == pt:
                        met = True
                        break
                    pt, dw, _ = record_hop(B, pt, L)
                    wt += dw
                    n += 1
                if met:
                    own[t], wd[t], err[t] = (0 if serr[t] else xs[t]), wt + ws[t] - wsp, serr[t]
                else:
                    err[t] = pt > L
                    own[t], wd[t] = (0 if err[t] else pt), wt
        rounds += 1
        rewalks.append(n)
    return own, wd, e, rounds, rewalks


def true_starts(B, L):
    """Record starts of the true chain from 0 up to L."""
    p, s = 0, []
    while p < L:
        s.append(p)
        p, _, _ = record_hop(B, p, L)
    return s, p
