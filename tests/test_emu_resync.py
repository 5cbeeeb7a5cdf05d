"""CPU check of the resync tile resolution's logic (tests/emu_resync.py
restates csrc/resync.hip k_tile): on packed batches from the oracle (config-4
kinds: ~30 %-zero words, long zero runs, long literal runs; mixed chunk
sizes) every block resolves to the true chain's entry, exit and words, and a
literal-run region costs one fix pass per tile it spans."""
import numpy as np

import emu_resync as E
import oracle_lib as O


def _batch(words, offs):
    st, packed, poff = O.pack_batch(words, offs)
    assert st == 0
    return bytes(packed) + bytes(2100), [int(x) for x in poff]


def _check(words, offs, blk, T, max_passes):
    B, in_off = _batch(words, offs)
    bl, res, passes, rounds = E.resolve(B, in_off, blk=blk, T=T)
    truth = E.true_blocks(B, in_off, bl)
    for k, (r, t) in enumerate(zip(res, truth)):
        assert t is not None
        assert r == t, (k, bl[k], r, t)
    assert passes <= max_passes, passes
    return passes, rounds


def test_tile_resolution_kinds():
    rng = np.random.default_rng(4)
    sizes = np.exp(rng.uniform(np.log(8), np.log(1500), 60)).astype(np.int64)
    offs = np.concatenate([[0], np.cumsum(sizes)]).astype(np.uint64)
    for kind in (0, 1, 2):
        words = O.gen_fill(offs, kind0=kind, pz=O.PZ30)
        _check(words, offs, blk=128, T=16, max_passes=8)
        _check(words, offs, blk=512, T=64, max_passes=8)


def test_tile_resolution_literal_region_passes():
    # one long literal chunk: 4 KiB tiles (16 blocks of 256 B), ~200 KiB of
    # 0xFF records: the spec chains never couple, each pass settles a tile
    n = 25000
    lit = np.random.default_rng(2).integers(1 << 56, 1 << 63, n, dtype=np.uint64) * 2 + 1
    offs = np.array([0, n], np.uint64)
    passes, _ = _check(lit, offs, blk=256, T=16, max_passes=64)
    assert passes >= 2


def test_tile_resolution_runs_across_blocks():
    n, cw = 40, 300
    offs = np.arange(0, (n + 1) * cw, cw, dtype=np.uint64)
    w = np.zeros(n * cw, np.uint64)
    for c in range(n):
        k = (c * 37) % 280
        w[c * cw + 3:c * cw + 3 + k] = 0x1112131415161718
        w[c * cw + 3 + k::7][:4] = 0x0000000100000001
    _check(w, offs, blk=64, T=8, max_passes=64)
    z = np.zeros(n * cw, np.uint64)
    z[::97] = 5
    _check(z, offs, blk=64, T=8, max_passes=64)


def test_tile_resolution_malformed_chunks():
    """Truncated, corrupted and mis-sized chunks: a chunk passes the check
    (last exit at its end, its word count, no block marked) only if the
    oracle decodes it cleanly (a failing one must leave for the serial walk;
    a segment that no entry reached marks its block)."""
    import random
    rng = random.Random(23)
    chunks, lens = [], []
    for _ in range(200):
        n = rng.choice([1, 7, 64, 130, 700])
        w = np.array([rng.getrandbits(64) if rng.random() < 0.6 else 0 for _ in range(n)],
                     np.uint64)
        if rng.random() < 0.3:
            w |= np.uint64(0x0101010101010101)
        st, k = O.pack(w.tobytes())
        k = bytearray(k)
        r = rng.random()
        if r < 0.15 and len(k) > 1:
            k = k[:rng.randrange(len(k))]
        elif r < 0.3 and len(k):
            k[rng.randrange(len(k))] = rng.choice([0, 0xFF, rng.randrange(256)])
        elif r < 0.4:
            n = max(1, n + rng.choice([-3, -1, 1, 4]))
        chunks.append(bytes(k))
        lens.append(n)
    in_offs = np.concatenate([[0], np.cumsum([len(k) for k in chunks])]).astype(np.uint64)
    out_offs = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
    packed = np.frombuffer(b"".join(chunks), np.uint8)
    _, rst, _ = O.unpack_batch(packed, in_offs, out_offs)
    B = bytes(packed) + bytes(4096)
    in_off = [int(x) for x in in_offs]
    bl, res, _, _ = E.resolve(B, in_off, blk=512, T=64)
    byc = {}
    for k, (c, s, e, f) in enumerate(bl):
        byc.setdefault(c, []).append(k)
    passed = 0
    for c, ks in byc.items():
        b = in_off[c + 1]
        good = (res[ks[-1]][1] == b and sum(res[k][2] for k in ks) == lens[c]
                and all(res[k][1] <= b for k in ks))
        assert not (good and rst[c] != 0), c
        passed += good
    assert passed > 50 and (rst != 0).sum() > 20


def test_tile_rounds_bounded():
    """seg_rounds' termination argument (csrc/resync.hip): lane i's entry
    depends only on the owned exits of lanes < i, so lane i is settled after
    round i + 1 and a tile needs at most lanes + 1 rounds (the kernel caps
    them at kTileThreads + 2 and sends a capped tile to the serial decode).
    Checked on garbage byte streams, literal regions and malformed chunks,
    where the spec chains couple least."""
    rng = np.random.default_rng(11)
    T, segs = 16, 4
    worst = 0
    for trial in range(12):
        n = int(rng.integers(2000, 9000))
        if trial % 3 == 0:  # random bytes: no record structure at all
            B = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        elif trial % 3 == 1:  # 0xFF-heavy garbage: long fake literal runs
            b = rng.integers(0, 256, n, dtype=np.uint8)
            b[rng.random(n) < 0.3] = 0xFF
            B = b.tobytes()
        else:  # a real literal region with corrupted bytes
            lit = rng.integers(1 << 56, 1 << 63, n // 8, dtype=np.uint64) * 2 + 1
            st, k = O.pack(lit.tobytes())
            k = bytearray(k)
            for i in rng.integers(0, len(k), 20):
                k[int(i)] = int(rng.integers(0, 256))
            B = bytes(k)
        cut = sorted(set(int(x) for x in rng.integers(1, len(B), 5)))
        in_off = [0] + cut + [len(B)]
        _, _, _, rounds = E.resolve(B + bytes(4096), in_off, blk=128, T=T, segs=segs)
        assert rounds <= T * segs + 1, (trial, rounds)
        worst = max(worst, rounds)
    assert worst >= 2
