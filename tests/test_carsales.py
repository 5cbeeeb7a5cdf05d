"""Config 1 (BASELINE.json configs[0]): the carsales request restated in
oracle/carsales_oracle.c (benchmark/common.rs:22-70, carsales.rs:84-150).

CPU only.  Pins what can be pinned without running the Rust reference:
  * every request re-reads through its own pointers to setup_request's
    expectation (handle_request / car_value, carsales.rs:32-72, :152-163);
  * the stream's size and packing statistics agree with the reference
    benchmark's published totals (blog/_posts/2013-11-16-benchmark.md:38-41:
    ~125 MB unpacked, ~81 MB packed per 10 000 carsales iterations, which
    include the small responses);
  * the product library's host walk of the FastRand chain
    (capnp_carsales_plan, used by the device generator) agrees with the
    oracle request by request.
Byte identity with the Rust builder itself is parity-unpinned (no cargo)."""
import numpy as np

import oracle_lib as O


def test_fastrand_first_outputs():
    # xorshift128 from the default seed (common.rs:30-54), restated in Python
    x, y, z, w = 0x1d2acd47, 0x58ca3e14, 0xf563f232, 0x0bc76199
    out = []
    for _ in range(5):
        t = (x ^ (x << 11)) & 0xFFFFFFFF
        x, y, z = y, z, w
        w = (w ^ (w >> 19) ^ t ^ (t >> 8)) & 0xFFFFFFFF
        out.append(w)
    st = O.carsales_seed()
    seg, _ = O.carsales_request(st)
    assert (len(seg) - 3) // 15 == out[0] % 200


def test_requests_reread_to_expectation():
    st = O.carsales_seed()
    sizes = []
    for i in range(3000):
        seg, exp = O.carsales_request(st)
        assert O.carsales_value(seg) == exp, i
        assert len(seg) % 15 == 3
        sizes.append(len(seg))
    assert max(sizes) <= O.CARSALES_MAX_WORDS and min(sizes) >= 3


def test_request_text_fields():
    st = O.carsales_seed()
    seg, _ = O.carsales_request(st)
    n = (len(seg) - 3) // 15
    assert n > 0
    makes = {b"Toyota", b"GM", b"Ford", b"Honda", b"Tesla"}
    models = {b"Camry", b"Prius", b"Volt", b"Accord", b"Leaf", b"Model S"}
    for i in range(n):
        c = 3 + 7 * i
        for k, names in ((3, makes), (4, models)):
            p = int(seg[c + k])
            assert p & 3 == 1 and (p >> 32) & 7 == 2  # byte list
            tgt = c + k + 1 + (np.int32(np.uint32(p & 0xFFFFFFFF)) >> 2)
            count = p >> 35
            txt = int(seg[tgt]).to_bytes(8, "little")[:count]
            assert txt.endswith(b"\0") and txt[:-1] in names


def test_stream_statistics_match_published_totals():
    st = O.carsales_seed()
    U = P = 0
    zero_words = words = 0
    for _ in range(10000):
        seg, _ = O.carsales_request(st)
        _, pk = O.write_message([seg])
        U += 8 + 8 * len(seg)
        P += len(pk)
        zero_words += int((seg == 0).sum())
        words += len(seg)
    # published: ~125 MB unpacked / ~81 MB packed (read off a chart)
    assert 0.9 * 125e6 < U < 1.05 * 125e6
    assert 0.9 * 81e6 < P < 1.1 * 81e6
    assert zero_words / words < 1e-3          # ~0 % zero words
    assert 0.65 < P / U < 0.75


def test_stream_cut_and_offsets():
    words, offs, _ = O.carsales_stream(100_000)
    assert offs[0] == 0 and offs[-1] >= 100_000 > offs[-2]
    st = O.carsales_seed()
    for i in range(len(offs) - 1):
        seg, _ = O.carsales_request(st)
        a, b = int(offs[i]), min(int(offs[i + 1]), 100_000)
        assert np.array_equal(words[a:b], seg[:b - a])


def test_library_plan_matches_oracle_chain():
    """capnp_carsales_plan (host code of the product library) walks the same
    chain: same request boundaries, and each recorded state regenerates the
    oracle's request (skip honoured)."""
    from capnp_amd.codec import carsales_plan
    states, offs = carsales_plan(200_000, skip_requests=7)
    _, ooffs, _ = O.carsales_stream(200_000, skip=7)
    assert np.array_equal(offs, ooffs)
    st = O.carsales_seed()
    for _ in range(7):
        O.carsales_request(st)
    for i in range(len(states)):
        assert np.array_equal(states[i], st)
        O.carsales_request(st)
