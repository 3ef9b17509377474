#!/usr/bin/env python3
"""Time the Python reference itself at BASELINE config 1 on THIS container's host
(SURVEY.md §8d "CPU baseline, in this container"), beside the C oracle on the
same inputs.

Config 1: N = 100 particles, L = 20 landmarks (6 m grid), M = 4 measurements per
scan (3 hits + 1 miss), the odometry pattern of jde_robots_main.py:25-31,
NUM_THREAD = 1 (the reference's pool runs the particles in index order).
The reference is imported from /root/reference exactly as tests/golden/gen_golden.py
does (HAL / cv2 stubbed, config knobs patched by name); only its wall time over
FastSLAM2.iterate (fast_slam_2/algorithms/fast_slam_2.py:33-67) is measured.
Container-only: /root/reference does not exist on the GPU box.

  python scripts/time_reference_cfg1.py [scans]   -> profiles/r04_reference_cfg1_container.json
"""
import json
import os
import platform
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, os.path.join(REPO, "tests", "golden"))
sys.path.insert(0, REPO)


def main():
    scans = int(sys.argv[1]) if len(sys.argv) > 1 else 40
    import gen_golden as gg            # imports the reference (container only)
    from fast_slam_2 import FastSLAM2, Measurement  # the reference's package (gen_golden put it on sys.path)
    syn = gg.syn
    N, L = 100, 20
    gg.configure(N)
    np.random.seed(0)
    fs = FastSLAM2()
    init = gg.grid_init(N, L, 0, cap=L + 4 * scans + 8)
    gg.populate(fs, *init)
    wl = syn.Workload(N, L, 0)
    meas = [[Measurement(float(d), float(b)) for d, b in wl.measurements(s)] for s in range(scans)]
    times = []
    for s in range(scans):
        r, t = syn.odometry(s)
        t0 = time.perf_counter()
        fs.iterate(r, t, meas[s])
        times.append(time.perf_counter() - t0)
    warm = 3
    ref_s = float(np.median(times[warm:]))
    ref_mean = float(np.mean(times[warm:]))

    # the C oracle (oracle/fs2_oracle.c) on the same inputs, one thread
    from oracle import oracle as orc
    orc.set_threads(1)
    o = orc.OracleFilter(N, L + 4 * scans + 8)
    x, y, yaw, w, cnt, lm = init
    o.set_state(x, y, yaw, w, cnt, lm)
    rng = np.random.default_rng(0)
    ot = []
    for s in range(scans):
        r, t = syn.odometry(s)
        ms = wl.measurements(s)
        nz = rng.normal(0, 0.001 if r else 0.0055, N)
        u0 = rng.uniform(0, 1.0 / N)
        t0 = time.perf_counter()
        o.iterate(r, t, ms, nz, u0)
        ot.append(time.perf_counter() - t0)
    oracle_s = float(np.median(ot[warm:]))
    model = next((ln.split(":", 1)[1].strip() for ln in open("/proc/cpuinfo") if ln.startswith("model name")),
                 platform.processor())
    rec = {
        "what": "Python reference FastSLAM2.iterate at BASELINE config 1 (N=100, L=20, M=4, NUM_THREAD=1)",
        "host": f"this build container (not the GPU box): {model}, {os.cpu_count()} CPUs",
        "scans_timed": scans - warm,
        "reference_ms_per_scan_median": ref_s * 1e3,
        "reference_ms_per_scan_mean": ref_mean * 1e3,
        "reference_particle_updates_per_s": N / ref_s,
        "oracle_c_ms_per_scan_median": oracle_s * 1e3,
        "oracle_c_particle_updates_per_s": N / oracle_s,
        "numpy": np.__version__, "python": platform.python_version(),
        "note": "reference: the pure-Python object path (per-particle deepcopy on resample, Python loops "
                "over landmarks); oracle: its C restatement, same inputs and draws pattern",
    }
    out = os.path.join(REPO, "profiles", "r04_reference_cfg1_container.json")
    json.dump(rec, open(out, "w"), indent=1)
    print(json.dumps(rec, indent=1))


if __name__ == "__main__":
    main()
