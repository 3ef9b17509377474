#!/usr/bin/env python3
"""Host time between scans from a rocprofv3 --kernel-trace --hip-trace database:
for the last scans, every HIP API call the host makes between the end of a scan's
last kernel (k_tail_single / k_publish) and the start of the next k_candidates.

  python3 scripts/host_gap.py gpurun_out/hprof/run_results.db [scans]
"""
import glob
import re
import sqlite3
import sys


def main():
    db = sys.argv[1] if len(sys.argv) > 1 else glob.glob("gpurun_out/hprof/**/*.db", recursive=True)[0]
    scans = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    con = sqlite3.connect(db)
    views = [r[0] for r in con.execute("select name from sqlite_master where type in ('table','view')")]
    print("views:", [v for v in views if not v.startswith("rocpd_info")][:40])
    kern = con.execute("select name, start, end from kernels order by start").fetchall()
    api_view = next((v for v in ("regions", "rocpd_region", "regions_and_samples") if v in views), None)
    cols = [r[1] for r in con.execute(f"pragma table_info({api_view})")]
    print("api view:", api_view, cols)
    name_col = "name" if "name" in cols else cols[0]
    api = con.execute(f"select {name_col}, start, end from {api_view} order by start").fetchall()
    cand = [i for i, k in enumerate(kern) if "k_candidates" in k[0]]
    for j in cand[-scans:]:
        t1 = kern[j][1]
        prev_end = max(k[2] for k in kern[:j]) if j else t1
        print(f"--- gap {((t1 - prev_end) / 1000):.1f} us before k_candidates at {t1}")
        for nm, s, e in api:
            if prev_end - 2000 <= s <= t1:
                short = re.sub(r"\(.*", "", str(nm))[:40]
                print(f"  {short:40s} start {(s - prev_end) / 1000:8.1f}  dur {(e - s) / 1000:7.1f}")


if __name__ == "__main__":
    main()
