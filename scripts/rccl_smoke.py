#!/usr/bin/env python3
"""RCCL transport check: G processes (torchrun) run the sharded filter and rank 0
compares every scan with a single-GPU handle.  On a one-GPU box all ranks share
device 0 (FS2_DEVICE_OVERRIDE=0).

  torchrun --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 scripts/rccl_smoke.py
"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "fast-slam_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))


def main():
    import torch
    import torch.distributed as dist
    world = int(os.environ["WORLD_SIZE"])
    rank = int(os.environ["RANK"])
    dev = int(os.environ.get("FS2_DEVICE_OVERRIDE", os.environ.get("LOCAL_RANK", "0")))
    torch.cuda.set_device(dev)
    dist.init_process_group("gloo")
    import fast_slam_2
    import fs2_synthetic as syn
    from fast_slam_2 import _native as nat
    obj = [nat.comm_unique_id() if rank == 0 else None]
    dist.broadcast_object_list(obj, src=0)
    N, L = 20000, 30
    wl = syn.Workload(N, L, seed=31)
    x, y, yaw = wl.poses()
    lm = wl.maps()
    lm[:, :, 2] = lm[:, :, 5] = 0.01
    w = np.full(N, 1.0 / N)
    cnt = np.full(N, L, np.int32)
    cap = L + 32
    f = fast_slam_2.FastSLAM2(N, device=dev, reduce="parallel", record_assoc=True, seed=9,
                              landmark_capacity=cap, rank=rank, world_size=world,
                              comm_id=obj[0], verbose=False)
    a, b = f.first_global, f.first_global + f.n_local
    f.set_state(x[a:b], y[a:b], yaw[a:b], w[a:b], cnt[a:b], lm[a:b])
    single = None
    if rank == 0:
        single = fast_slam_2.FastSLAM2(N, device=dev, reduce="parallel", record_assoc=True, seed=9,
                                       landmark_capacity=cap, verbose=False)
        single.set_state(x, y, yaw, w, cnt, lm)
    resamples = 0
    for s in range(6):
        rot, tr = syn.odometry(s)
        ms = wl.measurements(s)
        pose, st = f.step(rot, tr, ms)
        state = f.get_state(lm_cap=cap)
        parts = [None] * world
        dist.all_gather_object(parts, (pose.tolist(), int(st.resampled), state))
        if rank == 0:
            p1, s1 = single.step(rot, tr, ms)
            ref = single.get_state(lm_cap=cap)
            resamples += s1.resampled
            for pp, rs, _ in parts:
                assert rs == s1.resampled and np.allclose(pp, p1, rtol=1e-9, atol=1e-12), s
            for k in range(6):
                got = np.concatenate([q[2][k] for q in parts])
                assert np.allclose(got, ref[k], rtol=1e-9, atol=1e-12), (s, k)
    if rank == 0:
        print(f"rccl smoke ok: world={world} scans=6 resamples={resamples}", flush=True)
    f.close()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
