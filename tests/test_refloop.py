"""The timed CPU baseline (oracle/refloop_oracle.c: the reference's own
branch-free loops, serialize_packed.rs:304-439 and :80-228) gives the parity
oracle's bytes, statuses and consumed counts: on the reference's golden
vectors, on random and adversarial chunks, on truncated and corrupted
input, and through the threaded batch and message drivers bench.py times."""
import json
import os
import random

import numpy as np

import oracle_lib as O

GOLD = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "golden_packing.json")))


def test_golden_vectors():
    for v in GOLD["packing"]:
        u, k = bytes(v["unpacked"]), bytes(v["packed"])
        assert O.refloop_pack(u) == (0, k)
        assert O.refloop_read_exact(k, len(u)) == (0, u, len(k))
    for v in GOLD["unpack_errors"]:
        st, _, _ = O.refloop_read_exact(bytes(v["packed"]), v["out_len"])
        assert st == O.STATUS[v["status"]], v
    for v in GOLD["unpacks_to"]:
        assert O.refloop_read_exact(bytes(v["packed"]), len(v["unpacked"])) == (
            0, bytes(v["unpacked"]), len(v["packed"]))


def _rand_words(rng, n):
    kind = rng.random()
    w = []
    for _ in range(n):
        r = rng.random()
        if kind < 0.3:
            w.append(0 if r < 0.5 else rng.getrandbits(64))
        elif kind < 0.6:
            w.append(rng.getrandbits(64) | 0x0101010101010101 if r < 0.9 else 0)
        else:
            b = [0 if rng.random() < 0.45 else rng.randrange(1, 256) for _ in range(8)]
            w.append(int.from_bytes(bytes(b), "little"))
    return np.array(w, np.uint64)


def test_random_chunks_match_oracle():
    rng = random.Random(9)
    for _ in range(400):
        n = rng.choice([0, 1, 2, 9, 64, 255, 256, 300, 700])
        u = _rand_words(rng, n).tobytes()
        st, k = O.pack(u)
        assert O.refloop_pack(u) == (st, k)
        assert O.refloop_read_exact(k, len(u)) == O.read_exact(k, len(u))
        # truncated, corrupted, and wrong-length reads: the same status and consumed
        for cut in {0, len(k) // 2, max(len(k) - 1, 0)}:
            assert O.refloop_read_exact(k[:cut], len(u)) == O.read_exact(k[:cut], len(u))
        if k:
            kb = bytearray(k)
            kb[rng.randrange(len(kb))] = rng.choice([0, 0xFF, rng.randrange(256)])
            for ol in (len(u), len(u) + 8, max(len(u) - 8, 0)):
                assert O.refloop_read_exact(bytes(kb), ol) == O.read_exact(bytes(kb), ol)


def test_random_byte_strings_match_oracle():
    rng = random.Random(10)
    for _ in range(2000):
        k = bytes(rng.randrange(256) if rng.random() < 0.7 else rng.choice([0, 0xFF])
                  for _ in range(rng.randrange(0, 40)))
        ol = 8 * rng.randrange(0, 12)
        assert O.refloop_read_exact(k, ol) == O.read_exact(k, ol), (k, ol)


def test_batch_drivers_match_oracle():
    sizes = np.random.default_rng(2).integers(0, 400, 3000)
    offs = np.concatenate([[0], np.cumsum(sizes)]).astype(np.uint64)
    words = O.gen_fill(offs, kind0=0, pz=O.PZ30)
    st, ref, ref_offs = O.pack_batch(words, offs)
    assert st == 0
    for threads in (1, 3, 8):
        b = O.RefloopBatch(words, offs, threads)
        assert b.pack() == 0
        stream, soffs = b.packed_stream()
        assert np.array_equal(stream, ref) and np.array_equal(soffs, ref_offs)
        assert b.unpack() == 0
        assert (b.status == 0).all()
        assert np.array_equal(b.back[:len(words)], words)


def test_message_drivers_match_oracle():
    words, msg_off, _ = O.carsales_stream(60_000)
    mo = msg_off[:-1]  # complete requests only
    ww = words[:int(mo[-1])]
    for threads in (1, 4):
        tw, tr, pbytes, ok = O.refloop_messages_roundtrip_mt(ww, mo, threads)
        assert ok
        _, _, pb2, ok2 = O.messages_roundtrip_mt(ww, mo, threads)
        assert ok2 and pb2 == pbytes
