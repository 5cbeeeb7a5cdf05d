import sys, random, os
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "capnproto-rust_amd")); sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np, torch
import oracle_lib as O
import test_gpu_find_messages as T
from capnp_amd import Context
ctx = Context(0)
rng = random.Random(2)
for trial in range(40):
    s = T._stream(rng, rng.choice([1, 3, 20])); r = rng.random()
    if r < 0.4: s = s[:rng.randrange(1, len(s))]
    elif r < 0.7: s = s + bytes(rng.randrange(256) for _ in range(rng.randrange(1, 40)))
    else:
        k = rng.randrange(len(s)); s = s[:k] + bytes([rng.choice([0, 0xFF, rng.randrange(256)])]) + s[k + 1:]
    ref, ref_end = T._oracle_loop(s)
    dev = torch.from_numpy(np.frombuffer(s, np.uint8).copy()).cuda()
    offs, n = ctx.find_messages(dev)
    got, end = ctx.read_message_stream(dev)
    pos = [0]
    for segs, used in ref: pos.append(pos[-1] + used)
    print(trial, len(s), "ref", len(ref), ref_end, pos[-3:], "| find", n, offs.cpu().tolist()[-3:], "stream", len(got), end, flush=True)
