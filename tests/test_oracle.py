"""Pins the CPU oracle: every known-answer vector the reference's tests hold
(tests/golden/golden_packing.json) plus cross-checks against the independent
Python restatement (oracle/packed_ref.py) and round-trip properties mirroring
the reference's quickcheck tests (serialize_packed.rs:568-594)."""
import json
import os
import random

import numpy as np
import pytest

import oracle_lib as O
import packed_ref as R

GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "golden_packing.json")


@pytest.fixture(scope="module")
def golden():
    with open(GOLDEN) as f:
        return json.load(f)


def test_golden_json_is_regenerable(tmp_path, golden):
    import importlib.util
    spec = importlib.util.spec_from_file_location(
        "make_golden", os.path.join(os.path.dirname(__file__), "golden", "make_golden.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    pairs = m.packing_pairs()
    assert [(p["unpacked"], p["packed"]) for p in golden["packing"]] == [
        (list(u), list(k)) for u, k in pairs]


def test_simple_packing(golden):
    # check_packing (serialize_packed.rs:487-504): pack == packed, then unpack round-trips
    for v in golden["packing"]:
        u, k = bytes(v["unpacked"]), bytes(v["packed"])
        st, got = O.pack(u)
        assert st == 0 and got == k, (v, got)
        st, out, used = O.read_exact(k, len(u))
        assert st == 0 and out == u and used == len(k)
        assert R.pack(u) == k
        st, out, used = R.read_exact(k, len(u))
        assert st == 0 and out == u and used == len(k)


def test_unpack_errors(golden):
    for v in golden["unpack_errors"]:
        st, _, _ = O.read_exact(bytes(v["packed"]), v["out_len"])
        assert st == O.STATUS[v["status"]], v
        st2, _, _ = R.read_exact(bytes(v["packed"]), v["out_len"])
        assert st2 == st


def test_unpacks_to(golden):
    for v in golden["unpacks_to"]:
        st, out, used = O.read_exact(bytes(v["packed"]), len(v["unpacked"]))
        assert st == 0 and out == bytes(v["unpacked"]) and used == len(v["packed"])


def test_read_message_kats(golden):
    for v in golden["read_message"]:
        st, segs, used = O.read_message(bytes(v["packed"]))
        assert st == O.STATUS[v["status"]], v
        if st == 0:
            assert [len(s) for s in segs] == v["seg_words"]
            assert used == len(v["packed"])
        if "try_status" in v:
            st, _, _ = O.read_message(bytes(v["packed"]), try_mode=True)
            assert st == O.STATUS[v["try_status"]]


def _pack_stream_of_table(table):
    """A packed stream whose first read units unpack to `table`: pack the table
    as one chunk (padded to a word) — the read side then sees the same words."""
    t = bytes(table) + b"\0" * (-len(table) % 8)
    st, k = O.pack(t)
    assert st == 0
    return k


def test_segment_tables(golden):
    # test_read_segment_table (serialize.rs:742-831) through the packed reader:
    # the body is absent, so a non-empty body must fail to fill; empty body is OK.
    for v in golden["segment_tables"]:
        total = sum(v["seg_words"])
        body = np.arange(1, total + 1, dtype=np.uint64)
        stream = _pack_stream_of_table(v["table"])
        st, k = O.pack(body.tobytes())
        st, segs, used = O.read_message(stream + k)
        assert st == 0, v
        assert [len(s) for s in segs] == v["seg_words"]
        assert np.array_equal(np.concatenate(segs) if segs else np.zeros(0, np.uint64), body)


def test_invalid_segment_tables(golden):
    for v in golden["invalid_segment_tables"]:
        stream = _pack_stream_of_table(v["table"])
        if len(v["table"]) % 8:
            # a table cut mid-word (serialize.rs:912-918) has no packed form;
            # its packed counterpart is a stream cut before the word ends
            stream = stream[:-1]
        st, _, _ = O.read_message(stream)
        assert st != 0, v
        if v["status"] != "ANY_ERROR":
            assert st == O.STATUS[v["status"]]


def test_write_segment_tables(golden):
    # test_write_segment_table (serialize.rs:937-1028): the table is the
    # first one or two write_all chunks of write_message (serialize.rs:605-664).
    for v in golden["write_segment_tables"]:
        segs = [np.full(n, 0x0101010101010101, np.uint64) for n in v["seg_words"]]
        st, packed = O.write_message(segs)
        assert st == 0
        table = bytes(v["table"])
        exp = R.pack(table[:8]) + (R.pack(table[8:]) if len(table) > 8 else b"")
        assert packed.startswith(exp)
        st, back, used = O.read_message(packed)
        assert st == 0 and used == len(packed)
        assert [len(s) for s in back] == v["seg_words"]


def test_overflow_literal_runs():
    # capnp-futures/test/overflow_test.rs:63-78: 100 000 non-zero bytes pack to
    # literal runs capped at 255 words and round-trip.
    data = b"A" * 100000
    data += b"\0" * (-len(data) % 8)
    st, k = O.pack(data)
    assert st == 0 and k == R.pack(data)
    # first run: 0xFF tag, 8 bytes, count 255
    assert k[0] == 0xFF and k[9] == 255
    st, out, used = O.read_exact(k, len(data))
    assert st == 0 and out == data and used == len(k)


def _rand_words(rng, n):
    out = bytearray()
    for _ in range(n):
        kind = rng.random()
        if kind < 0.3:
            out += b"\0" * 8
        elif kind < 0.5:
            out += bytes(rng.randrange(1, 256) for _ in range(8))
        elif kind < 0.6:
            w = [rng.randrange(1, 256) for _ in range(8)]
            w[rng.randrange(8)] = 0
            out += bytes(w)
        else:
            out += bytes(rng.randrange(256) if rng.random() < 0.6 else 0 for _ in range(8))
    return bytes(out)


def test_random_vs_python_restatement():
    rng = random.Random(1234)
    for _ in range(300):
        n = rng.choice([0, 1, 2, 5, 63, 64, 65, 127, 128, 255, 256, 257, 300])
        d = _rand_words(rng, n)
        st, k = O.pack(d)
        assert st == 0 and k == R.pack(d)
        assert len(k) <= O.lib().oracle_bound(n)
        st, out, used = O.read_exact(k, len(d))
        assert st == 0 and out == d and used == len(k)


def test_long_runs_cap_255():
    for n in (255, 256, 257, 511, 512, 513, 1000):
        z = b"\0" * (8 * n)
        assert O.pack(z)[1] == R.pack(z)
        lit = b"\x11" * (8 * n)
        assert O.pack(lit)[1] == R.pack(lit)
        st, out, _ = O.read_exact(O.pack(lit)[1], 8 * n)
        assert st == 0 and out == lit


def test_unpack_garbage_never_crashes_and_matches_python():
    # test_unpack (serialize_packed.rs:584-593): arbitrary bytes must not crash.
    rng = random.Random(99)
    for _ in range(2000):
        n = rng.randrange(0, 40)
        d = bytes(rng.choice([0, 0xFF, 1, 2, 0x81, rng.randrange(256)]) for _ in range(n))
        out_len = 8 * rng.randrange(0, 12)
        a = O.read_exact(d, out_len)
        b = R.read_exact(d, out_len)
        assert a[0] == b[0], (d, out_len)
        assert a[2] == b[2], (d, out_len, a, b)  # consumed, every status
        if a[0] == 0:
            assert a[1] == b[1]


def test_consumed_on_errors_follows_refresh_buffer():
    # Where the reference leaves a &[u8] reader after a failed read_exact:
    # PrematureEndOfPackedInput consumes the whole buffer (refresh_buffer!,
    # serialize_packed.rs:59-74, then fill_buf() is empty); FailedToFill
    # consumes everything (consume + read_exact of the rest, :195-205, io.rs
    # :16-31); DidNotEndCleanly returns before any consume (:166-170, :183-187);
    # an empty input reads nothing (read() = Ok(0), :96-98).
    cases = [
        (bytes([0xf0, 1, 2]), 200 // 8 * 8, O.STATUS["PREMATURE_END_OF_PACKED_INPUT"], 3),
        (bytes([0]), 8, O.STATUS["PREMATURE_END_OF_PACKED_INPUT"], 1),
        (bytes([0xff, 1, 2, 3, 4, 5, 6, 7, 8]), 200 // 8 * 8,
         O.STATUS["PREMATURE_END_OF_PACKED_INPUT"], 9),
        (bytes([1, 1]), 200 // 8 * 8, O.STATUS["PREMATURE_END_OF_PACKED_INPUT"], 2),
        (bytes([0xff, 1, 2, 3, 4, 5, 6, 7, 8, 37, 1, 2]), 8 * 2,
         O.STATUS["DID_NOT_END_CLEANLY"], 0),
        (bytes([0xff, 1, 2, 3, 4, 5, 6, 7, 8, 3, 1, 2, 3]), 8 * 4,
         O.STATUS["FAILED_TO_FILL_WHOLE_BUFFER"], 13),
        (b"", 8, O.STATUS["FAILED_TO_FILL_WHOLE_BUFFER"], 0),
    ]
    for data, out_len, st, used in cases:
        for impl in (O, R):
            got = impl.read_exact(data, out_len)
            assert got[0] == st and got[2] == used, (impl.__name__, data, got)


def test_message_round_trip_quickcheck_style():
    # test_round_trip (serialize_packed.rs:568-582): arbitrary segments ->
    # write_message_segments -> read_message.
    rng = random.Random(7)
    for _ in range(200):
        nseg = rng.randrange(1, 9)
        segs = [np.frombuffer(_rand_words(rng, rng.randrange(0, 40)), np.uint64)
                for _ in range(nseg)]
        st, packed = O.write_message(segs)
        assert st == 0
        st, back, used = O.read_message(packed)
        assert st == 0 and used == len(packed)
        assert len(back) == nseg
        for a, b in zip(segs, back):
            assert np.array_equal(a, b)
        # no-alloc variant (serialize.rs:333-420) agrees
        st, buf, n2, tb, bb, used2 = O.read_message_no_alloc(packed, 4096)
        if nseg >= 3 and all(len(s) == 0 for s in segs[1:]):
            continue  # multi-word zero run in the table: see test below
        assert st == 0 and n2 == nseg and used2 == used
        body = buf[tb:tb + bb].view(np.uint64)
        assert np.array_equal(body, np.concatenate(segs) if segs else body[:0])


def test_no_alloc_reads_table_8_bytes_at_a_time():
    # 5 segments [1,0,0,0,0] -> the packed table rest is a
    # 2-word zero run; the alloc path reads it in one unit (OK), the no-alloc
    # path reads 8 bytes at a time and the run overruns that unit.
    packed = bytes([0x11, 4, 1, 0, 1, 0, 0])
    st, segs, _ = O.read_message(packed)
    assert st == 0
    st, *_ = O.read_message_no_alloc(packed, 64)
    assert st == O.STATUS["DID_NOT_END_CLEANLY"]


def test_try_read_message_stream():
    # try_read_message loop over a stream of messages ends with NONE.
    rng = random.Random(3)
    msgs = [[np.frombuffer(_rand_words(rng, rng.randrange(0, 20)), np.uint64)
             for _ in range(rng.randrange(1, 4))] for _ in range(10)]
    stream = b"".join(O.write_message(m)[1] for m in msgs)
    pos = 0
    for m in msgs:
        st, segs, used = O.read_message(stream[pos:], try_mode=True)
        assert st == 0
        assert all(np.array_equal(a, b) for a, b in zip(m, segs))
        pos += used
    assert O.read_message(stream[pos:], try_mode=True)[0] == O.STATUS["NONE"]
    assert O.read_message(stream[pos:])[0] == O.STATUS["PREMATURE_END_OF_FILE"]


def test_traversal_limit():
    segs = [np.ones(100, np.uint64)]
    st, packed = O.write_message(segs)
    assert O.read_message(packed, limit=99)[0] == O.STATUS["MESSAGE_TOO_LARGE"]
    assert O.read_message(packed, limit=100)[0] == 0
    assert O.read_message(packed, limit=None)[0] == 0


def test_batch_matches_single_and_threads():
    rng = np.random.default_rng(5)
    sizes = rng.integers(0, 300, 200)
    offs = np.concatenate([[0], np.cumsum(sizes)]).astype(np.uint64)
    words = O.gen_fill(offs, kind0=0, pz=O.PZ30)
    st, packed, poffs = O.pack_batch(words, offs, threads=1)
    st4, packed4, poffs4 = O.pack_batch(words, offs, threads=4)
    assert st == 0 and st4 == 0
    assert np.array_equal(poffs, poffs4) and packed.tobytes() == packed4.tobytes()
    for c in range(len(sizes)):
        seg = words[int(offs[c]):int(offs[c + 1])].tobytes()
        assert packed[int(poffs[c]):int(poffs[c + 1])].tobytes() == R.pack(seg)
    back, status, consumed = O.unpack_batch(packed, poffs, offs, threads=3)
    assert (status == 0).all()
    assert np.array_equal(back, words)
    assert np.array_equal(consumed, np.diff(poffs))


def test_generator_statistics():
    offs = np.arange(0, 129 * 2000, 128, dtype=np.uint64)[:2001]
    w = O.gen_fill(offs, kind0=0, pz=O.PZ30)
    zero_words = (w == 0).mean()
    assert abs(zero_words - 0.30) < 0.01
    b = w[w != 0].view(np.uint8)
    assert abs((b == 0).mean() - 111 / 256) < 0.01
    st, packed, poffs = O.pack_batch(w, offs)
    ratio = len(packed) / (8 * len(w))
    assert 0.50 < ratio < 0.58, ratio


# ---- the async PackedRead restatement, pinned by the reference's own tests
def test_async_poll_reads_golden_blocking_periods():
    """capnp-futures serialize_packed.rs:603-671: every packing vector read
    back through readers that return at most 1..9 bytes a read, with reads
    of 1..9 bytes (check_packing's blocking periods)."""
    with open(GOLDEN) as f:
        g = json.load(f)
    for v in g["packing"]:
        u, p = bytes(v["unpacked"]), bytes(v["packed"])
        for inner_max in range(1, 10):
            for size in range(1, 10):
                got, end = R.async_poll_reads(p, size, inner_max)
                assert got == u and end == b"", (v["ref"], inner_max, size)


def test_async_poll_reads_reference_cases():
    """The reference's async edge tests (capnp-futures
    serialize_packed.rs:747-814)."""
    # unpacks_across_partial_output_buffers (:748-760)
    assert R.async_poll_reads(bytes([0x81, 42, 99]), 1) == (bytes([42, 0, 0, 0, 0, 0, 0, 99]), b"")
    assert R.async_poll_reads(
        bytes([0xff, 1, 3, 2, 4, 5, 7, 6, 8, 1, 8, 6, 7, 4, 5, 2, 3, 1]), 3) == (
        bytes([1, 3, 2, 4, 5, 7, 6, 8, 8, 6, 7, 4, 5, 2, 3, 1]), b"")
    # eof_mid_tag_word (:762-773): one byte of a tag word, then the end
    assert R.async_poll_reads(bytes([0x81]), 8)[1] == "EOF"
    # eof_mid_passthrough_run (:775-790): two raw words promised, four bytes there
    got, end = R.async_poll_reads(bytes([0xff, 1, 2, 3, 4, 5, 6, 7, 8, 2, 10, 11, 12, 13]), 64)
    assert end == "EOF" and got == bytes([1, 2, 3, 4, 5, 6, 7, 8, 10, 11, 12, 13])
    # read_empty (:792-800): a clean end at once
    assert R.async_poll_reads(b"", 8) == (b"", b"")
    # eof_mid_message (:802-813): the first table word's tag wants 7 bytes, 2 are there
    assert R.async_poll_reads(bytes([0xfe, 3, 3]), 8)[1] == "EOF"
