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
    soa = cal.get("k_soa", [])
    # k_soa streams 2^20 particles x 512 slots x 16 B = 2^33 B per launch
    cal_bytes = float(os.environ.get("PMC_CAL_BYTES", 8589934592))
    fetch_factor = cal_bytes / (sum(soa) / len(soa) * 1024) if soa else 2.0
    fetch, fdur = read(f"{out_dir}/pmc_fetch/**/*counter_collection.csv", "FETCH_SIZE")
    write, _ = read(f"{out_dir}/pmc_write/**/*counter_collection.csv", "WRITE_SIZE")
    res = {"workload": workload, "fetch_factor_measured": fetch_factor, "fetch_factor_used": 2.0}
    lines = [f"PMC summary {tag} workload={workload}",
             f"FETCH_SIZE calibration on k_soa (known {cal_bytes:.3e} B): factor {fetch_factor:.4f} "
             f"(guide: 2.0 for 16 B/lane streaming reads)",
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
