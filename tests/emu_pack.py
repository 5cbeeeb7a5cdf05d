"""Bit-level emulation of the pack kernels' per-step arithmetic (test
infrastructure: checks the formulas of csrc/pack.hip's lean and chunk-step
kernels against the oracle on the CPU, before any GPU run).  Not a codec: it
re-derives record heads, sizes, positions and run counts from the masks the
kernels compute, and assembles the bytes the way pass 2 places them."""
import numpy as np

M64 = (1 << 64) - 1


def _tags(ws):
    tags = []
    for w in ws:
        w = int(w)
        tags.append(sum(1 << k for k in range(8) if (w >> (8 * k)) & 0xFF))
    return tags


def _ballot(bits):
    m = 0
    for i, b in enumerate(bits):
        if b:
            m |= 1 << i
    return m


def _ffbl(x):
    return (x & -x).bit_length() - 1 if x else 0xFFFFFFFF


def _ffbl64(x):
    lo, hi = x & 0xFFFFFFFF, (x >> 32) & 0xFFFFFFFF
    return min(_ffbl(lo), _ffbl(hi) | 32)


def _record(w, tag, head, cnt):
    b = int(w).to_bytes(8, "little")
    if not head:
        return b if tag else b""
    out = bytes([tag]) + bytes(x for x in b if x)
    if tag in (0, 0xFF):
        out += bytes([cnt])
    return out


def cs_chunk(words):
    """pack_cs_kernel's pass 1 + pass 2 for one chunk of <= 128 words."""
    n = len(words)
    assert n <= 128
    ws = list(words) + [0] * (128 - n)
    tags = _tags(ws)
    pops = [bin(t).count("1") for t in tags]
    V = _ballot([i < n for i in range(128)])
    Z = _ballot([(pops[i] if i < n else 64) == 0 for i in range(128)])
    L = _ballot([p >= 7 for p in pops])
    F = _ballot([p == 8 for p in pops])
    M = (1 << 128) - 1
    AZ = Z & ((Z << 1) & M)
    filled = ((L ^ ((L + F) & M)) & L) | F
    AF = filled & ((filled << 1) & M)
    H = V & ~(AZ | AF) & M
    Hlo, Hhi = H & M64, H >> 64
    out = b""
    for half in (0, 1):
        for lane in range(64):
            i = 64 * half + lane
            head = (H >> i) & 1
            if half == 0:
                d0 = _ffbl64(((Hlo >> 1) >> lane) & M64)
                d1 = (63 - lane) + _ffbl64(Hhi) if Hhi else 0xFFFFFFFF
                dn = d0 if d0 < 64 else d1
            else:
                dn = _ffbl64(((Hhi >> 1) >> lane) & M64)
            cnt = min(dn, max(n - (i + 1), 0)) & 127
            out += _record(ws[i], tags[i], head, cnt) if i < n else b""
    return out


def lean_chunk(words):
    """pack_lean_kernel's steps (64 words each, carried run) for one chunk."""
    n = len(words)
    steps = max(1, (n + 63) // 64) if n else 0
    ctype, crem = 0, 0
    recs = []  # per step: list of (word, tag, head, cnt_in, reach), kin, H == 0
    for s in range(steps):
        ws = list(words[64 * s:64 * s + 64])
        nv = len(ws)
        ws += [0] * (64 - nv)
        tags = _tags(ws)
        pops = [bin(t).count("1") for t in tags]
        V = _ballot([i < nv for i in range(64)])
        Z = _ballot([(pops[i] if i < nv else 64) == 0 for i in range(64)])
        L = _ballot([p >= 7 for p in pops])
        F = _ballot([p == 8 for p in pops])
        cm = Z if ctype == 1 else L
        inv = ~cm & M64
        k = _ffbl64(inv) if inv else 64
        k = min(k, crem) if ctype else 0
        AC = (1 << k) - 1
        Z2 = Z & ~AC
        AZ = Z2 & ((Z2 << 1) & M64)
        L2, F2 = L & ~AC, F & ~AC
        filled = ((L2 ^ ((L2 + F2) & M64)) & L2) | F2
        AF = filled & ((filled << 1) & M64)
        H = V & ~(AC | AZ | AF) & M64
        row = []
        for lane in range(64):
            dn = _ffbl64(((H >> 1) >> lane) & M64)
            reach = 1 if dn > 63 else 0
            cnt = min(dn, max(nv - (lane + 1), 0)) & 63
            row.append((ws[lane], tags[lane], (H >> lane) & 1, cnt, reach, lane < nv))
        recs.append((row, k, H == 0))
        code = [1 if (pops[i] if i < nv else 64) == 0 else (2 if (pops[i] if i < nv else 64) == 8 else 0)
                for i in range(64)]
        if H:
            h = H.bit_length() - 1
            ctype = code[h]
            crem = 192 + h if ctype else 0
        else:
            crem -= 64
    # pass 2 (reverse): ext
    out_steps = [b""] * steps
    ext = 0
    for s in range(steps - 1, -1, -1):
        row, kin, nohead = recs[s]
        e = 0 if s == steps - 1 else ext
        b = b""
        for (w, tag, head, cnt, reach, valid) in row:
            if valid:
                b += _record(w, tag, head, cnt + reach * e)
        out_steps[s] = b
        ext = 0 if s == 0 else kin + (e if nohead else 0)
    return b"".join(out_steps)
