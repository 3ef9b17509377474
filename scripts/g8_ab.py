"""A/B of the in-process G = 8 sharded path with page references against the
page transfer over a longer window than the bench's 6 scans: bench.sharded_local()
at 10^6 particles in all, L = 500, `scans` scans (3 untimed), alternating,
`reps` times each, in one process.

    python scripts/g8_ab.py [--reps 2] [--scans 23] > gpurun_out/g8_ab.json
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
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--scans", type=int, default=23)
    ap.add_argument("--n", type=int, default=1_000_000)
    ap.add_argument("--L", type=int, default=500)
    ap.add_argument("--G", type=int, default=8)
    a = ap.parse_args()
    import torch  # noqa: F401  (the wheel's HIP runtime first, as bench.py)
    import bench
    args = argparse.Namespace(seed=0)
    rows = []
    for r in range(a.reps):
        for refs in ("on", "off"):
            d = bench.sharded_local(args, a.L, a.n, G=a.G, scans=a.scans, page_refs=refs)
            d.pop("note", None)
            d["rep"] = r
            d["page_refs_asked"] = refs
            rows.append(d)
            print(json.dumps({k: d[k] for k in ("rep", "page_refs_asked", "ms_per_scan", "scan_device_ms",
                                                "comm_ms_per_scan", "resamples", "scan_ms_each")}),
                  file=sys.stderr, flush=True)
    out = {"n": a.n, "L": a.L, "G": a.G, "scans": a.scans, "rows": rows}
    for refs in ("on", "off"):
        sel = [r for r in rows if r["page_refs_asked"] == refs]
        out["refs" if refs == "on" else "pages"] = {
            "ms_per_scan": sorted(r["ms_per_scan"] for r in sel),
            "scan_device_ms": sorted(r["scan_device_ms"] for r in sel),
            "median_scan_ms": sorted(sorted(r["scan_ms_each"])[len(r["scan_ms_each"]) // 2] for r in sel)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
