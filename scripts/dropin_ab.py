"""A/B of the drop-in iterate() (numpy's legacy RNG drawn on the GPU) with and
without the speculative draw (fs2.h fs2_debug_mt_speculate): the bench's
dropin() at the headline size, alternating, `reps` times each, in one process.

    python scripts/dropin_ab.py [--reps 3] [--n 1000000] > gpurun_out/dropin_ab.json
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "fast-slam_amd"))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--n", type=int, default=1_000_000)
    ap.add_argument("--L", type=int, default=500)
    ap.add_argument("--seed", type=int, default=0)
    a = ap.parse_args()
    import torch  # noqa: F401  (the wheel's HIP runtime first, as bench.py)
    import bench
    args = argparse.Namespace(seed=a.seed)
    rows = []
    for r in range(a.reps):
        for spec in (True, False):
            d = bench.dropin(args, a.L, a.n, spec=spec)
            row = {"rep": r, "speculate": spec, "ms_per_scan": d["ms_per_scan"],
                   "ms_per_scan_median": d["ms_per_scan_median"], "resamples": d["resamples"], "ms_each": d["ms_each"],
                   "speculative_draws": d["speculative_draws"], "numpy_state_sha1": d["numpy_state_sha1"]}
            rows.append(row)
            print(json.dumps(row), file=sys.stderr, flush=True)
    digests = {r["numpy_state_sha1"] for r in rows}
    out = {"n": a.n, "L": a.L, "rows": rows, "same_numpy_state": len(digests) == 1}
    for spec in (True, False):
        ms = sorted(r["ms_per_scan"] for r in rows if r["speculate"] == spec)
        md = sorted(r["ms_per_scan_median"] for r in rows if r["speculate"] == spec)
        out["spec" if spec else "nospec"] = {"ms_per_scan": ms, "ms_per_scan_median": md}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
