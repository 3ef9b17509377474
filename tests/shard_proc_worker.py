"""One rank of the multi-process sharded scan (tests/test_gpu_sharded_procs.py).

  python shard_proc_worker.py G RANK N L SEED SCANS KEYHEX OUT.npz

Runs FastSLAM2 rank RANK of G with the stream-ordered shared-memory transport
(FS2_COMM_SHM) on cuda:0 over the workload of test_gpu_sharded.py, and saves
per scan what the parent compares with a single handle: decisions, estimates,
N_eff, reduce_ambiguous, associations, and the final local state.
"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "fast-slam_amd"))

import numpy as np  # noqa: E402


def workload(N, L, seed, mode="peaked", G=1):
    """mode "peaked": peaked likelihoods, so resampling moves particles across
    shards ("refs": the same with page references, the rank processes' pools
    mapped into each other as VMM chunks); "follow": only rank 0's particles carry weight (its first 100 ten
    times more), so the first scan (no measurements) resamples and rank 0 keeps
    a higher shard (equal shards follow their sources); "numpy":
    "peaked" through iterate() with numpy's global stream drawn on the device
    (fs2_mt_draw: every rank draws all N normals and keeps its shard's)."""
    import fs2_synthetic as syn
    wl = syn.Workload(N, L, seed=seed)
    x, y, yaw = wl.poses()
    lm = wl.maps()
    w = np.full(N, 1.0 / N)
    if mode == "follow":
        w = np.zeros(N)
        w[:N // G] = 1e-3
        w[:100] = 1e-2
    else:
        lm[:, :, 2] = lm[:, :, 5] = 0.01
    return wl, x, y, yaw, w, np.full(N, L, np.int32), lm


def measurements(wl, s, mode):
    return np.zeros((0, 2)) if (mode == "follow" and s == 0) else wl.measurements(s)


def main(argv):
    G, rank, N, L, seed, scans = (int(a) for a in argv[:6])
    key = bytes.fromhex(argv[6])
    out = argv[7]
    mode = argv[8] if len(argv) > 8 else "peaked"
    if os.environ.get("FS2_HIP_RUNTIME", "").lower() != "system":
        import torch  # noqa: F401  -- one HIP runtime in the process
    # (FS2_HIP_RUNTIME=system: this process never imports torch; libfs2 and RCCL run
    # on the system ROCm runtime they were built against)
    import fast_slam_2
    from fast_slam_2 import _native as nat
    import fs2_synthetic as syn
    from gpu_util import configure
    configure()
    wl, x, y, yaw, w, cnt, lm = workload(N, L, seed, mode, G)
    cap = L + 4 * scans + 8
    h = fast_slam_2.FastSLAM2(N, reduce="parallel", record_assoc=True, seed=5, landmark_capacity=cap, rank=rank,
                              world_size=G, comm_id=key, comm_mode="shm", verbose=False,
                              rng="numpy" if mode == "numpy" else "device",
                              page_refs="on" if mode == "refs" else "auto")
    np.random.seed(77)
    a, b = h.first_global, h.first_global + h.n_local
    h.set_state(x[a:b], y[a:b], yaw[a:b], w[a:b], cnt[a:b], lm[a:b])
    h.set_profiling(True)
    rec = {k: [] for k in ("resampled", "best_index", "pose", "n_eff", "reduce_amb", "firsts", "firsts_pre")}
    assoc = []
    if mode == "stall":
        # the last rank arrives late at scan 1: with FS2_SHM_TIMEOUT_S below the
        # delay every rank's scan must fail with FS2_ERR_COMM, nothing stale used
        import time
        from fast_slam_2._native import FS2Error
        err = (0, -1, "")
        for s in range(scans):
            if s == 1 and rank == G - 1:
                time.sleep(float(os.environ.get("FS2_TEST_STALL_S", "8")))
            rot, tr = syn.odometry(s)
            try:
                h.step(rot, tr, measurements(wl, s, mode))
            except FS2Error as e:
                err = (e.code, s, str(e))
                break
        h.close()
        np.savez(out, err_code=err[0], err_scan=err[1], err_msg=err[2])
        print(f"rank {rank} error {err}", flush=True)
        return 0
    for s in range(scans):
        rot, tr = syn.odometry(s)
        rec["firsts_pre"].append(h.first_global)    # the shard whose particles the associations describe
        if mode == "numpy":
            ms = [fast_slam_2.Measurement(float(d), float(b)) for d, b in measurements(wl, s, mode)]
            pose = np.array(h.iterate(rot, tr, ms))
            st = h.last_stats
        else:
            pose, st = h.step(rot, tr, measurements(wl, s, mode))
        rec["resampled"].append(st.resampled)
        rec["best_index"].append(st.best_index)
        rec["pose"].append(pose)
        rec["n_eff"].append(st.n_eff)
        rec["reduce_amb"].append(st.reduce_ambiguous)
        a = h.associations()
        pad = np.full((4, h.n_local), -2, np.int32)      # scans without measurements: 0 rows
        pad[:a.shape[0]] = a
        assoc.append(pad)
        rec["firsts"].append(h.first_global)        # a resample may hand this rank another shard
        print(f"rank {rank} scan {s} resampled {st.resampled}", flush=True)
    xs, ys, yaws, ws, cnts, lms = h.get_state(lm_cap=cap)
    a, b = h.first_global, h.first_global + h.n_local
    prof = h.profile()
    h.close()
    np.savez(out, first=a, count=b - a, assoc=np.stack(assoc), x=xs, y=ys, yaw=yaws, w=ws, cnt=cnts, lm=lms,
             sent_particles=prof["sent_particles"], sent_rows=prof["sent_rows"], sent_pages=prof["sent_pages"],
             migrations=prof["migrations"], scan_allocs=prof["scan_allocs"], page_refs=prof["page_refs"],
             localized_pages=prof["localized_pages"], hip_runtime=str(nat.HIP_RUNTIME[0]),
             torch_imported=("torch" in sys.modules),
             np_key=np.random.get_state()[1], np_pos=np.random.get_state()[2],
             **{k: np.array(v) for k, v in rec.items()})
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
