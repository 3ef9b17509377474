#!/usr/bin/env python3
"""Same-box A/B of libfs2 builds on the headline bench (config 3): runs
`bench.py --no-extras --no-cpu-baseline` once per library per round, alternating,
and prints ms/scan and the per-kernel event times of each run.

  python scripts/ab_lib.py --rounds 3 base=fast-slam_amd/lib/libfs2.so nomove=fast-slam_amd/lib/libfs2_nomove.so
"""
import argparse
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs="+", help="name=path")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--out", default=None)
    ap.add_argument("--bench-args", default="")
    a = ap.parse_args()
    rows = []
    for r in range(a.rounds):
        for spec in a.libs:
            name, path = spec.split("=", 1)
            env = dict(os.environ, FS2_LIB=os.path.abspath(path))
            cmd = [sys.executable, os.path.join(REPO, "bench.py"), "--no-extras", "--no-cpu-baseline",
                   "--steps", str(a.steps), *a.bench_args.split()]
            p = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=600)
            line = next((l for l in p.stdout.splitlines() if l.startswith("{")), None)
            if p.returncode or line is None:
                print(f"{name}: failed rc={p.returncode}\n{p.stderr[-3000:]}", flush=True)
                sys.exit(1)
            d = json.loads(line)
            e = d.get("extra", {})
            k = e.get("kernels", {})
            row = {"round": r, "lib": name, "ms_per_scan": d["ms_per_step"], "value": d["value"],
                   "k_candidates_ms": k.get("k_candidates", {}).get("ms_per_launch"),
                   "k_update_ms": k.get("k_update", {}).get("ms_per_launch"),
                   "tail_ms": e.get("reduce_and_resample_ms"), "resamples": e.get("resamples"),
                   "pages_opened": e.get("pages_opened_per_particle_scan")}
            rows.append(row)
            print(json.dumps(row), flush=True)
    if a.out:
        with open(a.out, "w") as fh:
            json.dump(rows, fh, indent=1)


if __name__ == "__main__":
    main()
