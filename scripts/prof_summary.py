#!/usr/bin/env python3
"""Summarise a rocprofv3 --kernel-trace --stats database into a small text table.

usage: prof_summary.py <results.db> <out.txt> [title]
"""
import glob
import sqlite3
import sys


def main():
    db = sys.argv[1]
    if not db.endswith(".db"):
        db = glob.glob(db.rstrip("/") + "/**/*.db", recursive=True)[0]
    out = sys.argv[2]
    title = sys.argv[3] if len(sys.argv) > 3 else ""
    c = sqlite3.connect(db)
    rows = list(c.execute("select name, total_calls, total_duration, average, percentage "
                          "from top_kernels"))
    with open(out, "w") as f:
        f.write(f"# rocprofv3 --kernel-trace --stats summary {title}\n")
        f.write("# durations in microseconds; names shortened\n")
        f.write(f"{'kernel':60s} {'calls':>6s} {'total_us':>12s} {'avg_us':>11s} {'pct':>6s}\n")
        for name, calls, tot, avg, pct in rows:
            short = name.replace("(anonymous namespace)::", "")
            short = short.split("(")[0][:60] if short.startswith(("fs2", "void fs2")) else short[:60]
            f.write(f"{short:60s} {calls:6d} {tot:12.1f} {avg:11.1f} {pct:6.2f}\n")
    print(open(out).read())


if __name__ == "__main__":
    main()
