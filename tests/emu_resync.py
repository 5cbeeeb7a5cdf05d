"""Emulation of the resync tile resolution (csrc/resync.hip k_tile: blocks
cut into segments, spec walks led in by kLead bytes, per-wave rounds of a
prefix max over owned exits across the tile with lockstep meet walks, fix
passes over tiles) on the CPU: test infrastructure
that checks its logic against the true record chain before any GPU run.  Not
a decoder: it returns each block's (entry, exit, words) as the kernel stores
them (k_spec + k_fix's contract)."""


def hop(B, p, w, b):
    """resync.hip hop(): one record from p (< b); a record cut short by the
    chunk end leaves p at b + 1."""
    tag = B[p]
    q = p + 1 + bin(tag).count("1")
    w += 1
    if tag in (0, 0xFF):
        if q >= b:
            return b + 1, w
        r = B[q]
        q += 1
        w += r
        if tag == 0xFF:
            q += 8 * r
    return (b + 1 if q > b else q), w


def blocks_of(in_off, blk):
    """(chunk, s, e, chunk-first) per block, as k_count + chunk_of lay them out."""
    out = []
    for c in range(len(in_off) - 1):
        a, b = in_off[c], in_off[c + 1]
        nb = (b - a + blk - 1) // blk
        for i in range(nb):
            s = a + i * blk
            out.append((c, s, min(s + blk, b), i == 0))
    return out


def _rounds(B, st, E0, catchup):
    """seg_rounds(): the wave's rounds to the fixed point (st: its lanes)."""
    NONE = -1
    rounds = 0
    while True:
        ins = [E0 if j == 0 else (L["a"] if L["first"] else 0) for j, L in enumerate(st)]
        pm, ents = 0, []
        for j, L in enumerate(st):
            ents.append(ins[j] if (j == 0 or L["first"]) else pm)
            if L["valid"]:
                pm = max(pm, L["own"], ins[j])
        need = [L["valid"] and ents[j] != L["used"] for j, L in enumerate(st)]
        if not any(need):
            return rounds
        rounds += 1
        for j, L in enumerate(st):
            if not need[j]:
                continue
            ent = L["used"] = ents[j]
            s, e, b, f = L["s"], L["e"], L["b"], L["f"]
            if ent < s:  # not reached yet: the spec chain stands in for the successors
                L["ex"], L["wd"] = b + 1, 0
                L["own"] = L["sx"] if (f != NONE and f < e and not L["serr"]) else 0
            elif ent > b:
                L["ex"], L["wd"], L["own"] = b + 1, 0, 0
            elif ent >= e or e == s:
                L["ex"], L["wd"], L["own"] = ent, 0, 0
            else:
                pt, wt, ps, ws, met, cu = ent, 0, f, 0, False, 0
                spec = f != NONE and f < e
                while pt < e:
                    if spec:
                        while ps < pt and ps < e and cu < catchup:
                            ps, ws = hop(B, ps, ws, b)
                            cu += 1
                        if ps == pt:
                            met = True
                            break
                        if ps < pt:
                            spec = False
                    pt, wt = hop(B, pt, wt, b)
                if met:
                    L["ex"], L["wd"] = L["sx"], wt + L["sw"] - ws
                    L["own"] = 0 if L["serr"] else L["sx"]
                else:
                    L["ex"], L["wd"], L["own"] = pt, wt, (0 if pt > b else pt)


def tile(B, in_off, bl, k0, T, lead, E0=None, segs=4, waves=4, catchup=16):
    """One k_tile launch for the tile at block k0 (E0 None: the spec launch):
    T blocks, waves x (T / waves) blocks, `segs` segments a block."""
    NONE = -1
    kn = min(T, len(bl) - k0)
    lanes = []
    for jb in range(T):
        jj = min(jb, kn - 1)
        c, s, e, first = bl[k0 + jj]
        a, b = in_off[c], in_off[c + 1]
        for q in range(segs):
            lanes.append((jb < kn, c, a, b, s, e, first and q == 0, q))
    st = []
    for (valid, c, a, b, s, e, first, q) in lanes:
        seg = SEG  # kSegBytes
        ss, se = min(s + q * seg, e), min(s + (q + 1) * seg, e)
        p, w = (ss - lead if ss > a + lead else a), 0
        while p < ss:
            p, w = hop(B, p, w, b)
        if p > b:
            f, sx, sw, serr = NONE, b + 1, 0, True
        else:
            f, w = p, 0
            while p < se:
                p, w = hop(B, p, w, b)
            sx, sw, serr = p, w, p > b
        L = dict(valid=valid, a=a, b=b, s=ss, e=se, first=first, f=f, sx=sx, sw=sw, serr=serr)
        if f != NONE and (f >= se or se == ss):
            L.update(used=f, ex=f, wd=0, own=0)
        else:
            L.update(used=f, ex=sx, wd=sw, own=(0 if serr else sx))
        st.append(L)
    # rounds over the whole tile (the kernel's prefix max spans its waves)
    L0 = st[0]
    e = E0 if E0 is not None else (L0["f"] if L0["f"] != NONE else L0["s"])
    if L0["first"]:
        e = L0["s"]
    rounds = _rounds(B, st, e, catchup)
    out = []
    for jb in range(kn):
        g = st[jb * segs:(jb + 1) * segs]
        err = any(x["ex"] > x["b"] for x in g)  # any segment's error marks the block
        out.append((g[0]["used"], g[0]["b"] + 1 if err else g[-1]["ex"], sum(x["wd"] for x in g)))
    return out, rounds


SEG = 128


def resolve(B, in_off, blk=512, T=64, lead=48, max_passes=512, snapshot=True, segs=4, waves=4):
    """Spec launch + fix passes: per block (entry, exit, words), passes, max rounds.
    snapshot: a pass reads its predecessors' exits as the previous pass left
    them (the GPU's concurrent tiles, the slow case); else in tile order."""
    global SEG
    SEG = blk // segs
    bl = blocks_of(in_off, blk)
    nb = len(bl)
    res = [None] * nb
    worst = 0
    for k0 in range(0, nb, T):
        r, rounds = tile(B, in_off, bl, k0, T, lead, None, segs, waves)
        res[k0:k0 + T] = r
        worst = max(worst, rounds)
    passes = 0
    while passes < max_passes:
        changed = False
        passes += 1
        prev = list(res)
        for k0 in range(T, nb, T):
            if bl[k0][3]:
                continue
            E0 = (prev if snapshot else res)[k0 - 1][1]
            if E0 == res[k0][0]:
                continue
            old = res[min(k0 + T, nb) - 1][1]
            r, rounds = tile(B, in_off, bl, k0, T, lead, E0, segs, waves)
            res[k0:k0 + T] = r
            worst = max(worst, rounds)
            changed |= r[-1][1] != old
        if not changed:
            break
    return bl, res, passes, worst


def true_blocks(B, in_off, bl):
    """The exact chain per block: entry = first record start >= s, exit = first
    >= e, words between (None for a chunk whose chain runs past its end)."""
    out = []
    chains = {}
    for (c, s, e, first) in bl:
        if c not in chains:
            a, b = in_off[c], in_off[c + 1]
            starts, wbefore, p, w = [], [], a, 0
            while p < b:
                starts.append(p)
                wbefore.append(w)
                p, w = hop(B, p, w, b)
            chains[c] = None if p != b else (starts + [b], wbefore + [w])
        ch = chains[c]
        if ch is None:
            out.append(None)
            continue
        st, wb = ch
        i = next(i for i, t in enumerate(st) if t >= s)
        j = next(j for j, t in enumerate(st) if t >= e)
        out.append((st[i], st[j], wb[j] - wb[i]))
    return out
