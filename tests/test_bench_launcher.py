"""bench.py --gpus N (N > 1) from a plain process re-launches itself under
torch.distributed.run with N ranks; checked here without a GPU through
--dry-run (gloo rendezvous on 127.0.0.1, max-over-ranks, rank-0 report)."""
import json
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_two_rank_launch_reports_two_gpus():
    env = dict(os.environ, OMP_NUM_THREADS="1")
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2",
                        "--dry-run", "--steps", "3"], capture_output=True, text=True,
                       timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1 and lines[0]["n_gpus"] == 2 and lines[0]["steps"] == 3
    assert abs(lines[0]["max_elapsed"] - 0.02) < 1e-9   # max over ranks of 0.01 (r + 1)
    # (the ranks share stderr, so their lines may interleave)
    ranks = sorted(int(m) for m in re.findall(r'"dry_run": true, "rank": (\d+)', r.stderr))
    assert ranks == [0, 1]
