#!/usr/bin/env python3
"""Summarise the PMC passes of scripts/pmc_round.sh into profiles/.

HBM bytes per launch = 2 x FETCH_SIZE + WRITE_SIZE (both in KiB), the gfx950
corrections of MI355X_MICROARCH.md (HBM section): FETCH_SIZE tallies a wide
coalesced streaming read at half its bytes (re-checked every run on the layout
microbenchmark, whose byte count is known), WRITE_SIZE is exact.

  python3 scripts/pmc_summary.py gpurun_out <workload> <tag>
writes profiles/pmc_<workload>.json and profiles/<tag>_pmc_<workload>.txt
"""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def short(name):
    m = re.search(r"(k_\w+)", name)
    return m.group(1) if m else name


def read(pattern, counter):
    vals = defaultdict(list)
    durs = defaultdict(list)
    for path in glob.glob(pattern, recursive=True):
        for row in csv.DictReader(open(path)):
            if row["Counter_Name"] != counter:
                continue
            k = short(row["Kernel_Name"])
            vals[k].append(float(row["Counter_Value"]))
            durs[k].append((int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) * 1e-6)
    return vals, durs


def main():
    out_dir, workload, tag = sys.argv[1], sys.argv[2], sys.argv[3]
    cal, _ = read(f"{out_dir}/pmc_cal/**/*counter_collection.csv", "FETCH_SIZE")
    # known bytes per launch (scripts/ubench_layout.hip): k_soa streams 2^20 x 512 x 16 B
    # (16 B/lane), k_desc8 2^20 x 512 x 8 B (8 B/lane: the descriptor stream), k_lines128
    # 2^23 distinct random 128-B lines read 16 B/lane (page opens)
    known = {"k_soa": 2.0 ** 33, "k_desc8": 2.0 ** 32, "k_lines128": 2.0 ** 30}
    factors = {k: known[k] / (sum(v) / len(v) * 1024) for k, v in cal.items() if k in known and v}
    fetch_factor = factors.get("k_soa", 2.0)
    fetch, fdur = read(f"{out_dir}/pmc_fetch/**/*counter_collection.csv", "FETCH_SIZE")
    write, _ = read(f"{out_dir}/pmc_write/**/*counter_collection.csv", "WRITE_SIZE")
    sys.path.insert(0, os.path.join(REPO, "fast-slam_amd"))
    import build
    import subprocess
    head = subprocess.run(["git", "-C", REPO, "rev-parse", "--short", "HEAD"], capture_output=True,
                          text=True).stdout.strip()
    res = {"workload": workload, "source_id": build.source_id(), "source": f"{tag} (HEAD {head})",
           "fetch_factor_measured": fetch_factor, "fetch_factors": factors, "fetch_factor_used": 2.0}
    lines = [f"PMC summary {tag} workload={workload} (HEAD {head}, libfs2 {build.source_id()})",
             "FETCH_SIZE calibration (known bytes / FETCH_SIZE bytes): " +
             ", ".join(f"{k} {v:.4f}" for k, v in sorted(factors.items())) +
             " (guide: 2.0 for 16 B/lane streaming reads)",
             f"{'kernel':<22}{'launches':>9}{'fetch GB':>11}{'write GB':>11}{'hbm GB':>10}{'avg ms':>9}"]
    for k in sorted(set(fetch) | set(write)):
        f = sum(fetch.get(k, [0])) / max(len(fetch.get(k, [])), 1) * 1024 * 2.0
        w = sum(write.get(k, [0])) / max(len(write.get(k, [])), 1) * 1024
        ms = sum(fdur.get(k, [0])) / max(len(fdur.get(k, [])), 1)
        res[k] = {"launches": len(fetch.get(k, [])), "fetch_bytes_per_launch": f,
                  "write_bytes_per_launch": w, "hbm_bytes_per_launch": f + w,
                  "avg_ms_under_pmc": ms}
        lines.append(f"{k:<22}{len(fetch.get(k, [])):>9}{f / 1e9:>11.3f}{w / 1e9:>11.3f}"
                     f"{(f + w) / 1e9:>10.3f}{ms:>9.3f}")
    os.makedirs(os.path.join(REPO, "profiles"), exist_ok=True)
    json.dump(res, open(os.path.join(REPO, "profiles", f"pmc_{workload}.json"), "w"), indent=1)
    txt = "\n".join(lines) + "\n"
    open(os.path.join(REPO, "profiles", f"{tag}_pmc_{workload}.txt"), "w").write(txt)
    print(txt)


if __name__ == "__main__":
    main()
