#!/usr/bin/env python3
"""Mid-run state round trip: two identical config-3-like handles (device RNG),
S scans; handle B re-imports every map (fs2_get_state -> fs2_set_state, host
buffers) and both continue; report where they differ."""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "fast-slam_amd")]


def main():
    import torch
    import bench
    import fast_slam_2
    import fs2_synthetic as syn
    torch.cuda.set_device(0)
    N, L, S = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
    cap = L + S + 30
    hs = [fast_slam_2.FastSLAM2(N, rng="device", seed=0, reduce="auto", landmark_capacity=cap, verbose=False)
          for _ in range(2)]
    for h in hs:
        bench.populate(h, N, L, 0, 0)
    meas = lambda s: np.ascontiguousarray(syn.scan_measurements(L, s, 0), dtype=np.float64)
    for s in range(S):
        for h in hs:
            h.step(*syn.odometry(s), meas(s))
    a = hs[1].get_state(lm_cap=cap)
    x, y, yaw, w, cnt, lm = a
    P = lm[:, :, 2:6]
    det = P[..., 0] * P[..., 3] - P[..., 1] * P[..., 2]
    live = np.arange(cap)[None, :] < cnt[:, None]
    print("exported: det<=0 live slots", int(((det <= 0) & live).sum()), "min det", det[live].min(),
          "nonfinite", int((~np.isfinite(lm[live])).sum()), flush=True)
    if len(sys.argv) > 4:       # device buffers, chunks of K particles (fs2_get_state / fs2_set_state FS2_DEVICE)
        from fast_slam_2 import _native as nat
        K = int(sys.argv[4])
        f = hs[1]
        for o in range(0, N, K):
            k = min(K, N - o)
            dl = torch.empty((k, cap, 6), dtype=torch.float64, device="cuda")
            dc = torch.empty(k, dtype=torch.int32, device="cuda")
            nat.check(f._lib.fs2_get_state(f._h, o, k, None, None, None, None, dc.data_ptr(), dl.data_ptr(), cap,
                                           nat.FS2_DEVICE), f._h)
            torch.cuda.synchronize()
            nat.check(f._lib.fs2_set_state(f._h, o, k, None, None, None, None, dc.data_ptr(), dl.data_ptr(), cap,
                                           nat.FS2_DEVICE), f._h)
            del dl, dc
    else:
        hs[1].set_state(x, y, yaw, w, cnt, lm)
    b = hs[1].get_state(lm_cap=cap)
    for k, nm in enumerate(("x", "y", "yaw", "w", "cnt")):
        print(nm, "roundtrip equal", np.array_equal(a[k], b[k]), flush=True)
    eq = (a[5] == b[5]) | ~live[:, :, None]
    bad = ~eq.all(axis=2)
    print("lm roundtrip equal", bool(eq.all()), "bad slots", int(bad.sum()), flush=True)
    if bad.any():
        pi, sj = np.nonzero(bad)
        print("first bad (particle, slot)", list(zip(pi[:5].tolist(), sj[:5].tolist())), "cnt", cnt[pi[:5]].tolist(),
              flush=True)
        print("  before", a[5][pi[0], sj[0]].tolist(), "\n  after ", b[5][pi[0], sj[0]].tolist(), flush=True)
    for s in range(S, S + 5):
        out = []
        for i, h in enumerate(hs):
            try:
                out.append(h.step(*syn.odometry(s), meas(s)))
            except Exception as e:
                out.append(e)
        print("scan", s, [o if isinstance(o, Exception) else (o[0].tolist(), o[1].resampled) for o in out], flush=True)
        if any(isinstance(o, Exception) for o in out):
            break
    for h in hs:
        h.close()


if __name__ == "__main__":
    main()
