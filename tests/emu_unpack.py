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


def walk_rec(B, q, se, L, K):
    """Walk from q until q >= se keeping the first K records (position, word
    offset): -> (exit, words, kept records, state after them)."""
    w, recs = 0, []
    while q < se and len(recs) < K:
        recs.append((q, w))
        q, dw, _ = record_hop(B, q, L)
        w += dw
    qr, wr = q, w
    while q < se:
        q, dw, _ = record_hop(B, q, L)
        w += dw
    return q, w, recs, (qr, wr)


def seg_walk(B, L, S=16, OV=32, K=12, descs=False):
    """Chunk bytes B[0:L] (zero padded past L), S byte segments, spec walks
    led in by OV bytes, K records kept per walk: returns (exits, words, err,
    rounds) as the kernel computes them, plus with descs=True the
    descriptor pass's (word, record start) pairs of the chunk."""
    sb = [(L * j) // S for j in range(S)]
    se = [(L * (j + 1)) // S for j in range(S)]
    f, xs, ws, serr, recs, rest = [], [], [], [], [], []
    for j in range(S):  # 1. spec walks
        p, w = (sb[j] if j == 0 else max(0, sb[j] - OV)), 0
        while p < sb[j]:
            p, dw, _ = record_hop(B, p, L)
            w += dw
        fj = p
        p, w, rj, sj = walk_rec(B, p, se[j], L, K)
        f.append(fj)
        serr.append(p > L)
        xs.append(0 if p > L else p)
        ws.append(w)
        recs.append(rj)
        rest.append(sj)
    rep = [False] * S
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
            if e == f[j] and not rep[j]:
                own[j], wd[j], err[j] = xs[j], ws[j], serr[j]
            else:
                q, wt, recs[j], rest[j] = walk_rec(B, e, se[j], L, K)
                rep[j] = True
                err[j] = q > L
                own[j] = 0 if (err[j] or e >= se[j]) else q
                wd[j] = wt
        x, m = [], 0
        for v in own:
            m = max(m, v)
            x.append(m)
    if not descs:
        return x, wd, err, rounds
    # 3. descriptors: word base of each segment's entry by a scan of wd, the
    # kept records, then a walk from the state after them to the exit
    out, base = [], 0
    for j in range(S):
        out += [(base + w, q) for q, w in recs[j]]
        q, w = rest[j]
        w += base
        while q < x[j]:
            out.append((w, q))
            q, dw, _ = record_hop(B, q, L)
            w += dw
        base += wd[j]
    return x, wd, err, rounds, out


def true_records(B, L):
    """The exact chain's (word, record start) pairs."""
    out, p, w = [], 0, 0
    while p < L:
        out.append((w, p))
        p, dw, _ = record_hop(B, p, L)
        w += dw
    return out


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
