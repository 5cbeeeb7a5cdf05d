"""CPU restatement of csrc/unpack.hip unpack_mid (the read_message
mid-size body decode: 4 waves x 64 segments, each wave settled by its own
rounds, the waves meeting through LDS), for tests/test_emu_mid.py.  Test
infrastructure only: the oracle (serialize_packed.rs:80-228) is the
reference; this checks the decode's logic on many inputs on the CPU."""

LEAD = 96  # unpack.hip kMidLead (UNPACK_MID_LEAD)


def hop(B, p, w):
    tag = B[p]
    isz, isf = tag == 0, tag == 0xFF
    cnt = B[p + 9] if isf else (B[p + 1] if isz else 0)
    ext = 8 * B[p + 9] + 1 if isf else (1 if isz else 0)
    return p + bin(tag).count("1") + ext + 1, w + 1 + cnt


def mid(B, L, n, NT=256, W=64):
    """-> (accepted, used, entries): B = the unit's bytes (readable past L),
    L = bytes the walks may use, n = words.  entries: the records each
    segment's descriptors start from (j <= ts, words > 0)."""
    NW = NT // W
    sb = [L * j // NT for j in range(NT)]
    se = [L * (j + 1) // NT for j in range(NT)]
    f, xs, ws, serr, xsp = [0] * NT, [0] * NT, [0] * NT, [False] * NT, [0] * NT
    for j in range(NT):
        p = 0 if j == 0 else max(sb[j] - LEAD, 0)
        w = 0
        while p < sb[j]:
            p, w = hop(B, p, w)
        f[j], wf = p, w
        while p < se[j]:
            p, w = hop(B, p, w)
        serr[j] = p > L
        xs[j] = 0 if serr[j] else p
        ws[j] = w - wf
        xsp[j] = 0 if (serr[j] or f[j] >= se[j]) else xs[j]
    own, wd = xsp[:], ws[:]
    err = [j == 0 and serr[j] for j in range(NT)]
    e_used = [None] * NT
    E = [0] + [f[W * v] for v in range(1, NW)]
    run = [True] * NW
    for _ in range(NW + 1):
        for v in range(NW):
            if not run[v]:
                continue
            lanes = list(range(W * v, W * v + W))
            while True:
                x, m = [], 0
                for j in lanes:
                    m = max(m, own[j])
                    x.append(m)
                es = [E[v] if i == 0 else max(E[v], x[i - 1]) for i in range(W)]
                need = [es[i] != e_used[j] for i, j in enumerate(lanes)]
                if not any(need):
                    break
                for i, j in enumerate(lanes):
                    if not need[i]:
                        continue
                    e = e_used[j] = es[i]
                    if e < sb[j] or e == f[j]:
                        own[j], wd[j], err[j] = xsp[j], ws[j], serr[j]
                        continue
                    pt, wt, ps, wsp, met = e, 0, f[j], 0, False
                    while pt < se[j]:
                        while ps < pt and ps < se[j]:
                            ps, wsp = hop(B, ps, wsp)
                        if ps == pt:
                            met = True
                            break
                        pt, wt = hop(B, pt, wt)
                    if met:
                        own[j], wd[j], err[j] = xsp[j], wt + ws[j] - wsp, serr[j]
                    else:
                        err[j] = pt > L
                        own[j] = 0 if (err[j] or e >= se[j]) else pt
                        wd[j] = wt
        wx = [max(max(own[W * v:W * v + W]), E[v]) for v in range(NW)]
        newE, m, changed = E[:], 0, False
        for v in range(NW):
            newE[v] = 0 if v == 0 else m
            changed |= v > 0 and E[v] != m
            m = max(m, wx[v])
        if not changed:
            break
        run = [newE[v] != E[v] for v in range(NW)]
        E = newE
    else:
        return False, 0, []
    base, acc = [], 0
    for j in range(NT):
        base.append(acc)
        acc += wd[j]
    ts = next((j for j in range(NT) if wd[j] > 0 and base[j] < n <= base[j] + wd[j]), None)
    if ts is None or any(err[j] for j in range(ts + 1)):
        return False, 0, []
    q, wq = e_used[ts], base[ts]
    while wq < n:
        tag = B[q]
        isz, isf = tag == 0, tag == 0xFF
        cnt = B[q + 1] if isz else (B[q + 9] if isf else 0)
        qe = q + 1 + bin(tag).count("1") + (1 if isz or isf else 0) + (8 * cnt if isf else 0)
        if qe > L or wq + 1 + cnt > n:
            return False, 0, []
        q, wq = qe, wq + 1 + cnt
    return True, q, [e_used[j] for j in range(ts + 1) if wd[j] > 0]


def true_starts(B, L):
    """Record starts of the serial walk from byte 0 within L bytes."""
    s, p = set(), 0
    while p < L:
        s.add(p)
        p, _ = hop(B, p, 0)
    return s
