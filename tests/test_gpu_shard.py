"""Multi-rank assembly on the GPU: two ranks pack their
word-balanced shards with the device codec (side by side on a one-GPU box),
exchange shard totals, and the concatenated stream equals the oracle's pack
of the whole batch; and bench.py launched through torch.distributed.run with
the RCCL ("nccl") backend runs its rank path end to end."""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

import oracle_lib as O

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_two_rank_gpu_shard_concat(tmp_path):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import torch.multiprocessing as mp
    import _dist_worker as W
    world = 2
    mp.spawn(W.pack_concat_worker_gpu, args=(world, _free_port(), str(tmp_path)), nprocs=world,
             join=True)
    words, offs = W.batch(seed=23, n=3000)
    st, ref, ref_offs = O.pack_batch(words, offs)
    assert st == 0
    packed = np.concatenate([np.load(tmp_path / f"packed{r}.npy") for r in range(world)])
    assert packed.tobytes() == ref.tobytes()
    for r in range(world):
        c0, c1, _, total = (int(x) for x in open(tmp_path / f"meta{r}.txt").read().split())
        assert np.array_equal(np.load(tmp_path / f"offs{r}.npy"), ref_offs[c0:c1 + 1])
        assert total == len(ref)


def test_bench_through_torchrun_rccl():
    """bench.py --gpus 1 under torch.distributed.run (RCCL backend, one
    rank): the launcher's rank path -- process group, per-rank shard, the
    max-over-ranks all-reduce -- runs and prints one valid JSON line."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    env = dict(os.environ)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(ROOT, "bench.py"), "--gpus", "1", "--steps", "3", "--warmup", "1",
           "--no-cpu", "--chunks", "65536"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    line = [x for x in r.stdout.splitlines() if x.startswith("{")][-1]
    d = json.loads(line)
    assert d["n_gpus"] == 1 and d["value"] > 0 and d["config"]["parallelism"] == "shard1"
    assert d["process_group"] == "nccl" and d["roundtrip_ok"]
