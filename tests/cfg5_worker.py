"""One rank of the config-5-shape run (tests/test_gpu_config5_shape.py).

  python cfg5_worker.py G RANK N L SCANS KEYHEX OUTDIR

Rank RANK of G processes on cuda:0, the stream-ordered shared-memory transport
(FS2_COMM_SHM), exact reductions across the shards (reduce="auto" -> EXACT).
Its slice of the initial state is generated here (the same generators and seeds
as the parent's oracle, fs2_synthetic.particle_maps by index range), the motion
normals and resample starts are the parent's (one global stream, every rank
takes its shard's slice), so the parent can compare each scan with the C
oracle.  Saves, per scan, the decisions, estimate, N_eff, total, associations,
the particle scalars, one window of whole maps and a per-particle map checksum.
"""
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "fast-slam_amd"))

import numpy as np  # noqa: E402

from cfg5_common import (CAP, WINDOW, draws, initial_scalars, map_checksum,  # noqa: E402
                         window_start)


def main(argv):
    G, rank, N, L, scans = (int(a) for a in argv[:5])
    key = bytes.fromhex(argv[5])
    outdir = argv[6]
    import torch  # noqa: F401  -- one HIP runtime in the process
    import fast_slam_2
    import fs2_synthetic as syn
    from gpu_util import configure
    configure()
    t0 = time.time()
    cap = CAP(L, scans)
    h = fast_slam_2.FastSLAM2(N, reduce="auto", record_assoc=True, seed=5, landmark_capacity=cap, rank=rank,
                              world_size=G, comm_id=key, comm_mode="shm", verbose=False, rng="device",
                              page_refs=os.environ.get("FS2_CFG5_PAGE_REFS", "auto"))
    a, b = h.first_global, h.first_global + h.n_local
    x, y, yaw, w = initial_scalars(N)
    lm = syn.particle_maps(N, L, 0, a, b - a)
    h.set_state(x[a:b], y[a:b], yaw[a:b], w[a:b], np.full(b - a, L, np.int32), lm)
    h.set_profiling(True)
    del lm
    print(f"rank {rank} ready in {time.time() - t0:.1f} s", flush=True)
    rec = {k: [] for k in ("resampled", "best_index", "pose", "n_eff", "total", "reduce_amb", "error_flags",
                           "firsts", "firsts_pre", "collections")}
    assoc, scal, wins, sums = [], [], [], []
    for s, (rot, tr, ms, nz, u0) in enumerate(draws(N, L, scans)):
        a = h.first_global
        rec["firsts_pre"].append(a)
        pose, st = h.step(rot, tr, ms, None, nz[a:a + h.n_local], u0)
        rec["resampled"].append(st.resampled)
        rec["best_index"].append(st.best_index)
        rec["pose"].append(pose)
        rec["n_eff"].append(st.n_eff)
        rec["total"].append(st.total_weight)
        rec["reduce_amb"].append(st.reduce_ambiguous)
        rec["error_flags"].append(st.error_flags)
        rec["collections"].append(st.collections)
        assoc.append(h.associations().copy())
        a = h.first_global
        rec["firsts"].append(a)
        xs, ys, yaws, ws, cnts, _ = h.get_state(lm_cap=0)
        scal.append(np.stack([xs, ys, yaws, ws, cnts.astype(np.float64)]))
        # one window of whole maps (global indices [w0, w0 + WINDOW)) if this shard holds it
        w0 = window_start(N, s)
        if a <= w0 and w0 + WINDOW <= a + h.n_local:
            wins.append(h.get_state(first=w0 - a, count=WINDOW, lm_cap=cap)[5])
        else:
            wins.append(np.zeros((0, cap, 6)))
        print(f"rank {rank} scan {s} resampled {st.resampled} n_eff {st.n_eff:.6g}", flush=True)
    # every particle's map, as a checksum (chunks of the export)
    cs = []
    for o in range(0, h.n_local, 8192):
        k = min(8192, h.n_local - o)
        cs.append(map_checksum(h.get_state(first=o, count=k, lm_cap=cap)[5]))
    prof = h.profile()
    n_local = h.n_local
    h.close()
    np.savez(os.path.join(outdir, f"rank{rank}.npz"), first=rec["firsts"][-1], count=n_local,
             assoc=np.stack(assoc), scal=np.stack(scal), checksum=np.concatenate(cs),
             migrations=prof["migrations"], sent_particles=prof["sent_particles"],
             sent_bytes=prof["sent_bytes"], scan_allocs=prof["scan_allocs"], page_refs=prof["page_refs"],
             localized_pages=prof["localized_pages"],
             **{f"win{s}": wv for s, wv in enumerate(wins)}, **{k: np.array(v) for k, v in rec.items()})
    print(f"rank {rank} done in {time.time() - t0:.1f} s", flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
