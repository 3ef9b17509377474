"""The bench's sharded_local_g8 (page references on, 8 ranks as threads on one GPU,
1e6 particles in all, L = 500) with FS2_TRACE=1: each scan's wall time with its
monotonic start on stdout, libfs2's per-rank trace (same clock) on stderr, so a
multi-second scan can be placed in the sharing / collective / growth steps.
Run on the GPU box:  FS2_TRACE=1 python3 scripts/g8_refs_probe.py [reps [pause_s]]"""
import os
import sys
import threading
import time

import numpy as np

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "fast-slam_amd"))
import torch  # noqa: F401,E402
import bench  # noqa: E402
import fast_slam_2  # noqa: E402
import fs2_synthetic as syn  # noqa: E402

G, N, L, scans = 8, 1000000, 500, 9


def one(rep):
    key = os.urandom(128)
    hs = [fast_slam_2.FastSLAM2(N, rng="device", seed=0, landmark_capacity=L + scans + 8, rank=g, world_size=G,
                                comm_id=key, comm_mode="local", verbose=False, page_refs="on") for g in range(G)]
    for g, h in enumerate(hs):
        bench.populate(h, h.n_local, L, 0, g)
    meas = {s: np.ascontiguousarray(syn.scan_measurements(L, s, 0), dtype=np.float64) for s in range(scans)}
    for h in hs:
        h.set_profiling(True)
    for s in range(scans):
        err = []
        res = [0] * G

        def run(g):
            try:
                _, st = hs[g].step(*syn.odometry(s), meas[s])
                res[g] = st.resampled
            except Exception as e:  # surfaced below
                err.append(e)
        t0 = time.monotonic()
        th = [threading.Thread(target=run, args=(g,)) for g in range(G)]
        for t in th:
            t.start()
        for t in th:
            t.join()
        print(f"rep {rep} scan {s} start {t0:.3f} ms {(time.monotonic() - t0) * 1e3:.3f} resampled {res[0]}",
              flush=True)
        if err:
            raise err[0]
    p = hs[0].profile()
    print(f"rep {rep} profile rank0 " + " ".join(f"{k}={p[k]}" for k in sorted(p) if "grow" in k or "collect" in k
                                               or k in ("comm_ms", "page_refs", "scans")), flush=True)
    for h in hs:
        h.close()


# optional pause (seconds) between one set of handles' close and the next set's creation
PAUSE = float(sys.argv[2]) if len(sys.argv) > 2 else 0.0
for r in range(int(sys.argv[1]) if len(sys.argv) > 1 else 3):
    if r and PAUSE:
        torch.cuda.synchronize()
        time.sleep(PAUSE)
    one(r)
