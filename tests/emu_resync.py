"""Emulation of the resync tile resolution (csrc/resync.hip k_tile: spec
walks led in by kLead bytes, rounds of a prefix max over owned exits with
lockstep meet walks, fix passes over tiles) on the CPU: test infrastructure
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


def tile(B, in_off, bl, k0, T, lead, E0=None):
    """One k_tile launch for the tile at block k0 (E0 None: the spec launch)."""
    NONE = -1
    lanes = bl[k0:k0 + T]
    st = []
    for (c, s, e, first) in lanes:
        a, b = in_off[c], in_off[c + 1]
        p, w = (s - lead if s > a + lead else a), 0
        while p < s:
            p, w = hop(B, p, w, b)
        if p > b:
            f, sx, sw, serr = NONE, b + 1, 0, True
        else:
            f, w = p, 0
            while p < e:
                p, w = hop(B, p, w, b)
            sx, sw, serr = p, w, p > b
        if f != NONE and f >= e:
            used, ex, wd, own = f, f, 0, 0
        else:
            used, ex, wd, own = f, sx, sw, (0 if serr else sx)
        st.append(dict(c=c, a=a, b=b, s=s, e=e, first=first, f=f, sx=sx, sw=sw, serr=serr,
                       used=used, ex=ex, wd=wd, own=own))
    if E0 is None:
        E0 = st[0]["f"] if st[0]["f"] != NONE else st[0]["s"]
    rounds = 0
    while True:
        ins = [E0 if j == 0 else (L["a"] if L["first"] else 0) for j, L in enumerate(st)]
        pm, ents = 0, []
        for j, L in enumerate(st):
            ents.append(E0 if j == 0 else (L["a"] if L["first"] else pm))
            pm = max(pm, L["own"], ins[j])
        need = [ents[j] != L["used"] for j, L in enumerate(st)]
        if not any(need):
            break
        rounds += 1
        for j, L in enumerate(st):
            if not need[j]:
                continue
            ent = L["used"] = ents[j]
            s, e, b, f = L["s"], L["e"], L["b"], L["f"]
            if ent < s or ent > b:
                L["ex"], L["wd"], L["own"] = b + 1, 0, 0
            elif ent >= e:
                L["ex"], L["wd"], L["own"] = ent, 0, 0
            else:
                pt, wt, ps, ws, met = ent, 0, f, 0, False
                if f != NONE and f < e:
                    while pt < e:
                        while ps < pt and ps < e:
                            ps, ws = hop(B, ps, ws, b)
                        if ps == pt:
                            met = True
                            break
                        pt, wt = hop(B, pt, wt, b)
                else:
                    while pt < e:
                        pt, wt = hop(B, pt, wt, b)
                if met:
                    L["ex"], L["wd"] = L["sx"], wt + L["sw"] - ws
                    L["own"] = 0 if L["serr"] else L["sx"]
                else:
                    L["ex"], L["wd"], L["own"] = pt, wt, (0 if pt > b else pt)
    return [(L["used"], L["ex"], L["wd"]) for L in st], rounds


def resolve(B, in_off, blk=512, T=64, lead=48, max_passes=512, snapshot=True):
    """Spec launch + fix passes: per block (entry, exit, words), passes, max rounds.
    snapshot: a pass reads its predecessors' exits as the previous pass left
    them (the GPU's concurrent tiles, the slow case); else in tile order."""
    bl = blocks_of(in_off, blk)
    nb = len(bl)
    res = [None] * nb
    worst = 0
    for k0 in range(0, nb, T):
        r, rounds = tile(B, in_off, bl, k0, T, lead)
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
            r, rounds = tile(B, in_off, bl, k0, T, lead, E0)
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
