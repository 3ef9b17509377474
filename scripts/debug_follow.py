"""Debug: the G=4 sharded case of test_gpu_sharded.py, printing where the sharded
state departs from the single handle (shard moves, differing particles)."""
import os, sys, threading
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tests")); sys.path.insert(0, os.path.join(REPO, "fast-slam_amd"))
import numpy as np


def main():
    import torch  # noqa
    import fast_slam_2
    import fs2_synthetic as syn
    from gpu_util import configure
    configure()
    G, N, L = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
    wl = syn.Workload(N, L, seed=21)
    x, y, yaw = wl.poses(); lm = wl.maps(); lm[:, :, 2] = lm[:, :, 5] = 0.01
    w = np.full(N, 1.0 / N); cnt = np.full(N, L, np.int32); cap = L + 40
    single = fast_slam_2.FastSLAM2(N, reduce="parallel", record_assoc=True, seed=5, landmark_capacity=cap, verbose=False)
    single.set_state(x, y, yaw, w, cnt, lm)
    key = os.urandom(128)
    sh = [fast_slam_2.FastSLAM2(N, reduce="parallel", record_assoc=True, seed=5, landmark_capacity=cap, rank=g,
                                world_size=G, comm_id=key, comm_mode="local", verbose=False) for g in range(G)]
    for h in sh:
        a, b = h.first_global, h.first_global + h.n_local
        h.set_state(x[a:b], y[a:b], yaw[a:b], w[a:b], cnt[a:b], lm[a:b])
    for s in range(8):
        rot, tr = syn.odometry(s); ms = wl.measurements(s)
        p1, st1 = single.step(rot, tr, ms)
        out = [None] * G
        th = [threading.Thread(target=lambda g=g: out.__setitem__(g, sh[g].step(rot, tr, ms))) for g in range(G)]
        [t.start() for t in th]; [t.join() for t in th]
        order = sorted(sh, key=lambda h: h.first_global)
        print("scan", s, "resampled", st1.resampled, "firsts", [h.first_global for h in sh], flush=True)
        a1 = single.associations(); ag = np.concatenate([h.associations() for h in order], axis=1)
        s1 = single.get_state(lm_cap=cap)
        parts = [h.get_state(lm_cap=cap) for h in order]
        sg = [np.concatenate([p[k] for p in parts]) for k in range(6)]
        bad = np.nonzero((a1 != ag).any(axis=0))[0]
        dpose = np.nonzero((s1[0] != sg[0]) | (s1[1] != sg[1]) | (s1[2] != sg[2]))[0]
        dcnt = np.nonzero(s1[4] != sg[4])[0]
        dlm = np.nonzero((s1[5] != sg[5]).any(axis=(1, 2)))[0]
        print("  assoc diff", len(bad), bad[:10], "pose bitdiff", len(dpose), dpose[:10], "cnt diff", len(dcnt),
              "lm bitdiff", len(dlm), dlm[:10], flush=True)
        if len(bad):
            i = bad[0]
            print("  particle", i, "single assoc", a1[:, i], "sharded", ag[:, i], "pose", s1[0][i], sg[0][i], s1[1][i], sg[1][i], flush=True)
            print("  maxdiff lm", np.abs(s1[5] - sg[5]).max(), "pose", np.abs(s1[0] - sg[0]).max())


if __name__ == "__main__":
    main()
