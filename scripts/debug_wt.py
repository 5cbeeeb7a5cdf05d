"""Word-tile diagnostics on the config-4 workload: how many tiles/pieces
leave the fast path with the GPU's own sync index."""
import ctypes as C
import sys
import os
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "capnproto-rust_amd"))
import bench
import torch
from capnp_amd import _lib
_v = os.path.join(os.path.dirname(__file__), "..", "capnproto-rust_amd", "build", "abl",
                  "libcapnp_packed_u_wtdbg.so")
if os.path.exists(_v):
    _lib.LIB_PATH = _v
from capnp_amd import Context

args = bench.parse(["--workload", "config4"])
ctx = Context(0)
dev = torch.device("cuda", 0)
words, offs, n, desc = bench.make_workload(args, ctx, torch, dev, 0)
total = words.numel()
L = _lib.lib()
st = (C.c_ulonglong * 4)()
L.capnp_unpack_wt_stats(st, 1)
cap = ctx.batch_bound_bytes(total, n)
packed = torch.empty(cap, dtype=torch.uint8, device=dev)
poffs = torch.empty(n + 1, dtype=torch.int64, device=dev)
sync = torch.empty(ctx.sync_entries(total), dtype=torch.int32, device=dev)
ctx.pack_batch_into(words, offs, packed, poffs, chunks_per_tile=0, sync=sync)
torch.cuda.synchronize()
s = sync.cpu().numpy().view("uint32")
print("sync none entries:", int((s == 0xFFFFFFFF).sum()), "of", len(s))
back = torch.empty_like(words)
status = torch.empty(n, dtype=torch.int32, device=dev)
consumed = torch.empty(n, dtype=torch.int64, device=dev)
ctx.unpack_batch_into(packed, poffs, offs, back, status, consumed, chunks_per_tile=0, sync=sync)
torch.cuda.synchronize()
L.capnp_unpack_wt_stats(st, 1)
print("stats fallback tiles, bad pieces, serial chunks:", list(st))
print("status nonzero:", int((status != 0).sum()), "equal:", bool(torch.equal(back, words)))
# which tiles fail: compare with oracle index on the first 200 chunks
import numpy as np
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
import oracle_lib as O
k = 300
o = offs[:k + 1].cpu().numpy().view(np.uint64)
w = words[:int(o[-1])].cpu().numpy().view(np.uint64)
stt, ref, ref_offs = O.pack_batch(w, o)
rs = O.sync_index(ref, ref_offs, o)
gs = s[:len(rs)]
bad = np.nonzero(gs != rs)[0]
print("sync mismatches in first", k, "chunks:", len(bad), bad[:10], [hex(x) for x in gs[bad[:5]]], [hex(x) for x in rs[bad[:5]]])
po = poffs[:k + 1].cpu().numpy().view(np.uint64)
print("offsets equal:", np.array_equal(po, ref_offs))
# failing tiles
dbg = (C.c_ulonglong * 512)()
L.capnp_unpack_wt_dbg.argtypes = [C.POINTER(C.c_ulonglong)]
L.capnp_unpack_wt_stats(st, 1)
ctx.unpack_batch_into(packed, poffs, offs, back, status, consumed, chunks_per_tile=0, sync=sync)
torch.cuda.synchronize()
L.capnp_unpack_wt_dbg(dbg)
oo = offs.cpu().numpy().view(np.uint64)
kinds = np.random.default_rng(4).choice(3, size=n, p=[0.8, 0.1, 0.1])  # same as bench (rank 0)
T = 1024
for i in range(12):
    t, m = dbg[2 * i], dbg[2 * i + 1]
    Wa, Wb = t * T, min((t + 1) * T, total)
    ca = int(np.searchsorted(oo, Wa, side="right") - 1)
    cb = int(np.searchsorted(oo, Wb, side="left"))
    chunks = [(c, int(oo[c]), int(oo[c + 1] - oo[c]), int(kinds[c])) for c in range(ca, min(cb, ca + 6))]
    print("tile", t, "Wa", Wa, "bad mask", bin(m), "chunks(c,start,len,kind)", chunks)
    ww = words[Wa:Wb].cpu().numpy().view(np.uint64)
    e0 = s[Wa // 8]; eb = s[Wb // 8] if Wb // 8 < len(s) else None
    print("   entry@Wa", hex(e0), "entry@Wb", hex(eb) if eb is not None else None,
          "zero words", int((ww == 0).sum()), "first words", [hex(x) for x in ww[:3]])

ev = (C.c_uint32 * 768)()
if L.capnp_unpack_wt_events(ev) == 0:
    names = {1: "last!=B", 2: "last c<nc", 3: "no-meet", 4: "seg_start bad", 5: "chunk end"}
    for i in range(40):
        e = list(ev[12 * i:12 * i + 12])
        if e[1] == 0:
            break
        print("tile", e[0], names.get(e[1]), "b", e[2], "c", e[3], "q", e[4], "w", e[5],
              "| c2/q2/w2", e[6], e[7], e[8], "err", e[9], "x", e[10], "y", e[11])
