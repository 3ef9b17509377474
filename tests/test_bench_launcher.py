"""bench.py --gpus N starts its N ranks itself (CPU test, nothing touches a GPU).

The driver runs `python3 bench.py --gpus N` without torch.distributed.run; the
parent must start one child per GPU with the rank environment torchrun would
give (RANK, LOCAL_RANK, WORLD_SIZE, LOCAL_WORLD_SIZE, MASTER_ADDR=127.0.0.1,
MASTER_PORT) before it initialises HIP, and refuse loudly to time fewer ranks
than asked.
"""
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(REPO, "bench.py")


def _env():
    e = dict(os.environ)
    for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT"):
        e.pop(k, None)
    return e


def test_dry_run_prints_rank_environments():
    out = subprocess.run([sys.executable, BENCH, "--gpus", "8", "--steps", "3", "--dry-run"], env=_env(),
                         capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr
    envs = json.loads(out.stdout.strip().splitlines()[-1])
    assert [e["RANK"] for e in envs] == [str(r) for r in range(8)]
    assert [e["LOCAL_RANK"] for e in envs] == [str(r) for r in range(8)]
    assert {e["WORLD_SIZE"] for e in envs} == {"8"} and {e["LOCAL_WORLD_SIZE"] for e in envs} == {"8"}
    assert {e["MASTER_ADDR"] for e in envs} == {"127.0.0.1"}
    ports = {e["MASTER_PORT"] for e in envs}
    assert len(ports) == 1 and 0 < int(ports.pop()) < 65536


def test_rank_envs_keep_the_callers_environment():
    sys.path.insert(0, REPO)
    import bench
    envs = bench.rank_envs(3, 29500, base={"PATH": "/bin", "HSA_ENABLE_IPC_MODE_LEGACY": "0", "X": "1"})
    assert len(envs) == 3
    for r, e in enumerate(envs):
        assert e["PATH"] == "/bin" and e["X"] == "1" and e["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"
        assert e["RANK"] == e["LOCAL_RANK"] == str(r) and e["MASTER_PORT"] == "29500"
    assert bench.rank_envs(1, 1, base={})[0]["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"


def test_too_few_gpus_fails_loudly():
    # this container has no GPU: --gpus 2 must exit non-zero and say why, without
    # timing a single rank and printing a result line
    out = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--steps", "1", "--warmup", "0"], env=_env(),
                         capture_output=True, text=True, timeout=300)
    assert out.returncode != 0
    assert "needs 2 visible GPUs" in out.stderr
    assert '"metric"' not in out.stdout
