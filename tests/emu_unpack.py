"""Emulation of the index-free segment walk (csrc/unpack.hip spec_seg_tile)
on the CPU: test infrastructure that checks the walk's round logic (spec
walk, coupling walks, prefix max of owned exits, pass-through segments)
against the true record chain, before any GPU run.  Not a decoder: it
returns each segment's exit and words, which the kernel turns into
descriptors."""


def record_hop(B, p, pe):
    """One record at byte p of a chunk ending at pe: next start, words, past end."""
    tag = B[p]
    isz, isf = tag == 0, tag == 0xFF
    cnt = B[p + 1] if isz else (B[p + 9] if isf else 0)
    q = p + 1 + bin(tag).count("1") + (1 if (isz or isf) else 0) + (8 * cnt if isf else 0)
    return q, 1 + cnt, q > pe


def seg_walk(B, L, S=16, M=16, couple=True):
    """Chunk bytes B[0:L] (zero padded past L), S byte segments: returns
    (exits, words, err, rounds) as the kernel computes them (couple: the
    UNPACK_SEG_COUPLE build, whose exact walks stop on a kept spec start)."""
    NONE = 0xFFFF
    sb = [(L * j) // S for j in range(S)]
    se = [(L * (j + 1)) // S for j in range(S)]
    kept, xs, ws, serr = [], [], [], []
    for j in range(S):  # 1. spec walks
        p, w, e, kl = sb[j], 0, False, []
        while p < se[j] and not e:
            if len(kl) < M:
                kl.append((p, w))
            p, dw, er = record_hop(B, p, L)
            w += dw
            e = e or er
        kept.append(kl)
        xs.append(NONE if e else p)
        ws.append(w)
        serr.append(e)
    own, x, wd = list(xs), list(xs), list(ws)
    err = [serr[0]] + [False] * (S - 1)
    used = [sb[0]] + [None] * (S - 1)
    rounds = 0
    while True:  # 2. coupling rounds
        ent = [sb[0]] + x[:-1]
        need = [j > 0 and ent[j] != used[j] for j in range(S)]
        if not any(need):
            break
        rounds += 1
        for j in range(1, S):
            if not need[j]:
                continue
            e = used[j] = ent[j]
            q, wt, terr, coupled, wc = e, 0, False, False, 0
            while q < se[j] and not terr:
                hit = [w for (pp, w) in kept[j] if pp == q] if couple else []
                if hit:
                    coupled, wc = True, hit[0]
                    break
                q, dw, er = record_hop(B, q, L)
                wt += dw
                terr = terr or er
            own[j] = xs[j] if coupled else (NONE if terr else (0 if e >= se[j] else q))
            wd[j] = wt + (ws[j] - wc) if coupled else wt
            err[j] = terr or (coupled and serr[j]) or e == NONE
        x, m = [], 0
        for v in own:
            m = max(m, v)
            x.append(m)
    return x, wd, err, rounds


def true_exits(B, L, S=16):
    """The exact chain: first record start at or past each segment end."""
    starts, p = [], 0
    while p < L:
        starts.append(p)
        p, _, _ = record_hop(B, p, L)
    out = []
    for j in range(S):
        se = (L * (j + 1)) // S
        out.append(min([t for t in starts if t >= se] + [p]))
    return out
