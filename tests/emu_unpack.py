"""Emulation of the index-free segment walk (csrc/unpack.hip spec_seg_tile)
on the CPU: test infrastructure that checks the walk's round logic (led-in
spec walk, meet check, repair walks, prefix max of owned exits,
pass-through segments)
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


def seg_walk(B, L, S=16, OV=32):
    """Chunk bytes B[0:L] (zero padded past L), S byte segments, spec walks
    led in by OV bytes: returns (exits, words, err, rounds) as the kernel
    computes them."""
    sb = [(L * j) // S for j in range(S)]
    se = [(L * (j + 1)) // S for j in range(S)]
    f, xs, ws, serr = [], [], [], []
    for j in range(S):  # 1. spec walks
        p, w = (sb[j] if j == 0 else max(0, sb[j] - OV)), 0
        while p < sb[j]:
            p, dw, _ = record_hop(B, p, L)
            w += dw
        fj, wf = p, w
        while p < se[j]:
            p, dw, _ = record_hop(B, p, L)
            w += dw
        f.append(fj)
        serr.append(p > L)
        xs.append(0 if p > L else p)
        ws.append(w - wf)
    own, x, wd = list(xs), [max(xs[:j + 1]) for j in range(S)], list(ws)
    err = [serr[0]] + [False] * (S - 1)
    used = [sb[0]] + [None] * (S - 1)
    rounds = 0
    while True:  # 2. meet / repair rounds
        ent = [sb[0]] + x[:-1]
        need = [j > 0 and ent[j] != used[j] for j in range(S)]
        if not any(need):
            break
        rounds += 1
        for j in range(1, S):
            if not need[j]:
                continue
            e = used[j] = ent[j]
            if e == f[j]:
                own[j], wd[j], err[j] = xs[j], ws[j], serr[j]
            else:
                q, wt = e, 0
                while q < se[j]:
                    q, dw, _ = record_hop(B, q, L)
                    wt += dw
                err[j] = q > L
                own[j] = 0 if (err[j] or e >= se[j]) else q
                wd[j] = wt
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
