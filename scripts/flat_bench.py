"""Diagnostic: device flat-slice framing rate (capnp_gpu_read_flat_messages)
on N single-segment 1 KiB flat messages (messages/s and table bytes read)."""
import sys
import time

import numpy as np
import torch

sys.path.insert(0, "capnproto-rust_amd")
from capnp_amd import Context  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 20
words = 127
starts = np.arange(n + 1, dtype=np.int64) * (8 * (words + 1))
buf = torch.zeros(int(starts[-1]) // 8, dtype=torch.int64)
buf[0::words + 1] = words << 32  # word 0: nseg-1 = 0, len0 = words
d_buf = buf.cuda().view(torch.uint8)
d_off = torch.from_numpy(starts).cuda()
ctx = Context(0)
for na in (False, True):
    for _ in range(3):
        ctx.read_flat_messages(d_buf, d_off, segs_cap=n, no_alloc=na)
    torch.cuda.synchronize()
    t = time.perf_counter()
    reps = 20
    for _ in range(reps):
        segs, mso, st, body, used = ctx.read_flat_messages(d_buf, d_off, segs_cap=n, no_alloc=na)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t) / reps
    assert bool((st == 0).all()) and int(mso[-1]) == n
    print(f"no_alloc={int(na)} n={n} {dt * 1e3:.3f} ms/batch  {n / dt / 1e6:.1f} M msg/s  "
          f"{n * (8 + 8 + 4 + 8 + 8 + 8 + 4) / dt / 1e9:.1f} GB/s framing bytes", flush=True)
