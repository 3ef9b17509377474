"""Host side of a scan at config 3 (N=1e6, L=500, M=4): how long fs2_iterate_submit
and fs2_iterate_wait hold the calling thread, and how much of a scan's wall time
the GPU waits for the host.  Run on the GPU box (python scripts/host_turnaround.py);
with rocprofv3 --kernel-trace the gaps between a scan's last kernel and the next
scan's first one are the host's share.  Prints one JSON line."""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "fast-slam_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    import torch
    import bench
    import fast_slam_2
    import fs2_synthetic as syn
    N = int(os.environ.get("N", "1000000"))
    L = int(os.environ.get("L", "500"))
    scans = 3 + 20
    torch.cuda.init()
    f = fast_slam_2.FastSLAM2(N, rng="device", seed=0, landmark_capacity=L + 3 * scans + 8, verbose=False)
    bench.populate(f, N, L, 0, 0)
    meas = [np.ascontiguousarray(syn.scan_measurements(L, s, 0), dtype=np.float64) for s in range(3 * scans)]
    out = {}
    # A: step() per scan (the bench loop)
    for s in range(3):
        f.step(*syn.odometry(s), meas[s])
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for s in range(3, scans):
        f.step(*syn.odometry(s), meas[s])
    out["step_ms"] = (time.perf_counter() - t0) / (scans - 3) * 1e3
    # B: submit / wait, timed apart
    sub, wt, res = [], [], []
    for s in range(scans, 2 * scans):
        a = time.perf_counter()
        f.step_submit(*syn.odometry(s), meas[s])
        b = time.perf_counter()
        _, st = f.step_wait()
        c = time.perf_counter()
        sub.append((b - a) * 1e3)
        wt.append((c - b) * 1e3)
        res.append(int(st.resampled))
    out["submit_ms"] = float(np.median(sub))
    out["wait_ms"] = float(np.median(wt))
    out["submit_ms_resampling"] = [round(x, 4) for x, r in zip(sub, res) if r]
    out["submit_ms_each"] = [round(x, 4) for x in sub]
    out["wait_ms_each"] = [round(x, 4) for x in wt]
    # C: the C entry point alone (no Python argument handling)
    lib = f._lib
    import ctypes as C
    pose = np.empty(3)
    from fast_slam_2 import _native as nat
    st = nat.fs2_iter_stats()
    t0 = time.perf_counter()
    for s in range(2 * scans, 3 * scans):
        rot, tr = syn.odometry(s)
        m = meas[s]
        rc = lib.fs2_iterate(f._h, rot, tr, nat.ptr(m), None, m.shape[0], None, None, nat.dptr(pose), C.byref(st))
        assert rc == 0
    out["c_iterate_ms"] = (time.perf_counter() - t0) / scans * 1e3
    f.close()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
