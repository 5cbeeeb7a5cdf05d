"""Reproduce test_word_tile_pack[1] and show the first differing bytes."""
import os
import random
import sys
import numpy as np
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "capnproto-rust_amd"))
import torch
import oracle_lib as O
from capnp_amd import _lib
if len(sys.argv) > 1:
    _lib.LIB_PATH = sys.argv[1]
from capnp_amd import Context
import test_gpu_wordtiles as T

ctx = Context(0)
kind = 1
rng = random.Random(200 + kind)
sizes = T._sizes_long(rng, 300)
offs = np.concatenate([[0], np.cumsum(sizes)]).astype(np.uint64)
words = O.gen_fill(offs, kind0=kind, pz=O.PZ30, id0=kind * 77)
st, ref, ref_offs = O.pack_batch(words, offs)
n, total = len(offs) - 1, int(offs[-1])
dw = torch.from_numpy(words.view(np.int64).copy()).cuda()
do = T.dev(offs)
out = torch.empty(ctx.batch_bound_bytes(total, n), dtype=torch.uint8, device="cuda")
oo = torch.empty(n + 1, dtype=torch.int64, device="cuda")
sync = torch.empty(ctx.sync_entries(total), dtype=torch.int32, device="cuda")
ctx.pack_batch_into(dw, do, out, oo, chunks_per_tile=0, sync=sync)
torch.cuda.synchronize()
got = out[:len(ref)].cpu().numpy()
bad = np.nonzero(got != ref)[0]
print("sizes[:5]", sizes[:5], "n bad bytes", len(bad), "first", bad[:10])
for b in bad[:6]:
    c = int(np.searchsorted(ref_offs, b, side="right") - 1)
    print("byte", b, "chunk", c, "chunk byte", b - int(ref_offs[c]), "got", got[b], "ref", ref[b],
          "ctx ref", list(ref[max(0, b - 4):b + 4]), "got", list(got[max(0, b - 4):b + 4]))
print("words 262..292:", [hex(int(x)) for x in words[262:292]])
print("ref 0..60", list(ref[:60]))
print("got 0..60", list(got[:60]))
import ctypes as C
buf = (C.c_uint32 * (4096 * 8))()
if _lib.lib().capnp_pack_wt_dbg(buf) == 0:
    for r in range(6):
        print("range", r, "cin", buf[8*r], buf[8*r+1], "rext", buf[8*r+2], "carry out", buf[8*r+3], buf[8*r+4], "R0/R1", buf[8*r+5], buf[8*r+6], "bytes", buf[8*r+7])
sys.exit(0)
# walk the oracle records of the chunk to find which word the byte belongs to
c = int(np.searchsorted(ref_offs, bad[0], side="right") - 1)
p, w = int(ref_offs[c]), int(offs[c])
while p <= bad[0]:
    tag = ref[p]
    pop = bin(tag).count("1")
    ln = 1 + pop
    cnt = 0
    if tag in (0, 255):
        cnt = ref[p + ln]
        ln += 1 + (8 * cnt if tag == 255 else 0)
    if p + ln > bad[0]:
        print("record at byte", p, "tag", tag, "head word", w, "count", cnt, "(range", w // 512, ")")
        break
    p += ln
    w += 1 + cnt
