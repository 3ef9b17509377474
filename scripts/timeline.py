#!/usr/bin/env python3
"""Kernel timeline of the last scans of a rocprofv3 --kernel-trace run.

  python3 scripts/timeline.py gpurun_out/prof/run_results.db [scans]
Prints each dispatch of the last `scans` scans (start relative to the first
k_candidates shown, duration, gap to the previous dispatch) in microseconds.
"""
import glob
import re
import sqlite3
import sys


def main():
    db = sys.argv[1] if len(sys.argv) > 1 else glob.glob("gpurun_out/prof/*.db")[0]
    scans = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    con = sqlite3.connect(db)
    rows = con.execute("select name, start, end from kernels order by start").fetchall()
    idx = [i for i, r in enumerate(rows) if "k_candidates" in r[0]]
    first = idx[-scans]
    t0 = rows[first][1]
    prev = None
    for r in rows[first:]:
        nm = re.sub(r"void |fs2::|<.*|\(.*", "", r[0])[:30]
        gap = (r[1] - prev) / 1000 if prev is not None else 0.0
        print(f"{nm:32s} {(r[1] - t0) / 1000:9.1f} {(r[2] - r[1]) / 1000:8.1f}  gap {gap:6.1f}")
        prev = r[2]


if __name__ == "__main__":
    main()
