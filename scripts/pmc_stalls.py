#!/usr/bin/env python3
"""Summarise scripts/pmc_stalls.sh: per kernel, the mean per dispatch of every SQ
counter and the ratios that say where wave time goes.

  python3 scripts/pmc_stalls.py gpurun_out/pmc_stalls > profiles/<tag>_pmc_stalls.txt

  waves/SIMD   SQ_LEVEL_WAVES / SQ_BUSY_CYCLES / 4 SIMDs ... (resident waves per SIMD
               while the SQ is busy; the counters are summed over the SEs, so the
               ratios, not the absolutes, are read)
  wait         SQ_WAIT_ANY / SQ_WAVE_CYCLES   (wave-cycles waiting on anything)
  issue-wait   SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES (waiting for an instruction to issue)
  valu         SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES
  vmem lat     SQ_INST_LEVEL_VMEM / (SQ_INSTS_VMEM_RD + SQ_INSTS_VMEM_WR) (mean cycles a
               vector memory instruction is in flight, Little's law)
"""
import csv
import glob
import re
import sys
from collections import defaultdict


def short(name):
    m = re.search(r"(k_\w+)", name)
    return m.group(1) if m else name


def main():
    d = sys.argv[1]
    vals = defaultdict(lambda: defaultdict(list))
    for path in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for row in csv.DictReader(open(path)):
            vals[short(row["Kernel_Name"])][row["Counter_Name"]].append(float(row["Counter_Value"]))
    print("# SQ counters per dispatch (means; scripts/pmc_stalls.sh, default bench, config 3)")
    for k in sorted(vals):
        m = {c: sum(v) / len(v) for c, v in vals[k].items()}
        print(f"\n{k} ({len(next(iter(vals[k].values())))} dispatches)")
        for c in sorted(m):
            print(f"  {c:28s} {m[c]:16.4g}")
        g = m.get
        wc = g("SQ_WAVE_CYCLES")
        if wc:
            print(f"  -> wait {g('SQ_WAIT_ANY', 0) / wc:.3f}  issue-wait {g('SQ_WAIT_INST_ANY', 0) / wc:.3f}"
                  f"  active-any {g('SQ_ACTIVE_INST_ANY', 0) / wc:.3f}  valu {g('SQ_ACTIVE_INST_VALU', 0) / wc:.3f}"
                  f"  vmem {g('SQ_ACTIVE_INST_VMEM', 0) / wc:.3f}")
        nv = g("SQ_INSTS_VMEM_RD", 0) + g("SQ_INSTS_VMEM_WR", 0)
        if nv and g("SQ_INST_LEVEL_VMEM"):
            print(f"  -> vmem instructions {nv:.4g}, mean in flight {g('SQ_INST_LEVEL_VMEM') / nv:.1f} cycles each")
        if g("SQ_BUSY_CYCLES") and g("SQ_LEVEL_WAVES"):
            print(f"  -> mean resident waves per busy cycle {g('SQ_LEVEL_WAVES') / g('SQ_BUSY_CYCLES'):.1f}")
        if g("SQ_WAVES"):
            print(f"  -> per wave: valu {g('SQ_INSTS_VALU', 0) / g('SQ_WAVES'):.0f}  vmem {nv / g('SQ_WAVES'):.0f}"
                  f"  salu {g('SQ_INSTS_SALU', 0) / g('SQ_WAVES'):.0f}  lds {g('SQ_INSTS_LDS', 0) / g('SQ_WAVES'):.0f}"
                  f"  fp64 flops {g('SQ_INSTS_VALU_FLOPS_FP64', 0) / g('SQ_WAVES'):.0f}"
                  f"  fp64 trans {g('SQ_INSTS_VALU_TRANS_F64', 0) / g('SQ_WAVES'):.0f}")


if __name__ == "__main__":
    main()
