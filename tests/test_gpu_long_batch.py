"""Batches of one or two very long read units through the public batch
decode (capnp_gpu_unpack_batch, csrc/capi.hip unpack_batch_dev): a unit of
1-8 Mi words is one `read_exact` of a whole message body in the reference
(serialize.rs:512-524; bodies reach 8 Mi words at the default traversal
limit, message.rs:116-119).  Such a batch is decoded by the index-free block
decode (resync.hip), which spreads one unit over the whole chip; a malformed
unit takes the exact serial walk on its own.  Words, statuses and consumed
byte counts equal the oracle's (PackedRead::read_exact,
serialize_packed.rs:80-228, io.rs:16-31), including a truncated unit, a
corrupted unit and a unit whose word count overruns its bytes.
"""
import numpy as np
import pytest

import oracle_lib as O

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

MI = 1 << 20


@pytest.fixture(scope="module")
def ctx():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from capnp_amd import Context
    c = Context(0)
    yield c
    c.close()


def _units(sizes, kinds, seed):
    offs = np.concatenate([[0], np.cumsum(sizes)]).astype(np.uint64)
    words = O.gen_fill(offs, kinds=np.array(kinds, np.uint8), pz=O.PZ30, id0=seed)
    st, packed, poffs = O.pack_batch(words, offs)
    assert st == 0
    return words, offs, np.frombuffer(packed, np.uint8).copy(), poffs.astype(np.uint64)


def _check(ctx, packed, in_offs, out_offs):
    rw, rst, rcons = O.unpack_batch(packed, in_offs, out_offs)
    d = lambda a: torch.from_numpy(np.ascontiguousarray(a).view(np.int64)).cuda()
    dp = torch.from_numpy(packed).cuda()
    w, st, cons = ctx.unpack_batch(dp, d(in_offs), d(out_offs))
    torch.cuda.synchronize()
    st = st.cpu().numpy()
    cons = cons.cpu().numpy().view(np.uint64)
    w = w.cpu().numpy().view(np.uint64)
    assert np.array_equal(st, rst), (st, rst)
    for c in range(len(st)):
        if rst[c] == 0:
            a, b = int(out_offs[c]), int(out_offs[c + 1])
            assert cons[c] == rcons[c], (c, cons[c], rcons[c])
            assert np.array_equal(w[a:b], rw[a:b]), c
    return rst


@pytest.mark.parametrize("sizes,kinds", [([MI], [0]), ([MI, 3 * MI], [0, 2]),
                                         ([8 * MI], [0]), ([2 * MI, MI], [1, 0])])
def test_long_units_vs_oracle(ctx, sizes, kinds):
    words, offs, packed, poffs = _units(sizes, kinds, 4242 + len(sizes))
    rst = _check(ctx, packed, poffs, offs)
    assert (rst == 0).all()


def test_long_units_malformed_vs_oracle(ctx):
    """Two units of 1 and 2 Mi words: the last truncated by 7 bytes; the first
    with a byte flipped mid-stream; the first claiming 64 words more than its
    bytes hold (its bytes then run into the second unit's)."""
    words, offs, packed, poffs = _units([MI, 2 * MI], [0, 0], 777)
    cut = poffs.copy()
    cut[-1] -= 7
    rst = _check(ctx, packed, cut, offs)
    assert rst[1] != 0 and rst[0] == 0
    bad = packed.copy()
    rng = np.random.default_rng(5)
    pos = int(poffs[1]) // 2 + int(rng.integers(0, 1000))
    bad[pos] ^= 0xFF
    _check(ctx, bad, poffs, offs)
    more = offs.copy()
    more[1] += 64
    more[2] += 64
    _check(ctx, packed, poffs, more)
