"""bench.py's multi-rank path end to end on one GPU.

`python bench.py --gpus 2 --share-gpu` (ranks as processes on GPU 0, libfs2's
shared-memory transport, the bench's own barrier / max-over-ranks timing over
gloo) runs exactly the code the driver's N-GPU run takes with RCCL: the
launcher's children, per-rank shards and initial state, the sharded scans with
their resamples and migrations, the timing reduction and rank 0's JSON line.
"""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_two_ranks_on_one_gpu():
    env = dict(os.environ)
    for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    n = 40000
    out = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--share-gpu",
                          "--particles", str(n), "--landmarks", "60", "--steps", "8", "--warmup", "2",
                          "--no-extras", "--no-cpu-baseline"],
                         env=env, capture_output=True, text=True, timeout=140)
    assert out.returncode == 0, out.stderr[-4000:]
    lines = [l for l in out.stdout.strip().splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout            # rank 0 alone prints the result line
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["steps"] == 8 and d["value"] > 0
    assert d["config"]["particles_total"] == 2 * n and d["config"]["particles_per_gpu"] == n
    assert d["config"]["transport"] == "shm" and d["config"]["ranks_share_gpu"] is True
    assert d["config"]["parallelism"] == "particle-shard2"
    mig = d["extra"]["migration"]
    assert mig is not None and mig["resamples"] >= 1
    assert d["cpu_baseline"] is None               # rank 0 at N = 1 only
