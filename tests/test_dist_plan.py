"""Sharded resample plan across processes (torch.distributed gloo, CPU).

Restates, in numpy, the per-shard plan that libfs2 runs on the GPU
(fast-slam_amd/csrc/fs2_resample.hip): every rank knows only its own
particles' normalised weights, all-gathers its shard total, and derives from
its local prefix plus the offset of the ranks before it the contiguous output
range each of its particles fills; then it lists what it must send to each
peer.  Checked against the CPU oracle's sequential low-variance resample
(reference fast_slam_2.py:177-199): the union of all shards' plans must give
exactly the oracle's source of every output, every output must be covered once,
and a receiver must get exactly the remote sources of its outputs.
"""
import os

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp


def shard(N, G, r):
    return N * r // G, N * (r + 1) // G


def u_of(u0, m, N):
    return u0 + m * (1.0 / N)


def first_above(v, u0, N):
    lo, hi = 0, N
    while lo < hi:
        mid = (lo + hi) // 2
        if u_of(u0, mid, N) > v:
            hi = mid
        else:
            lo = mid + 1
    return lo


def local_plan(w_local, a, N, offset, u0):
    """Output range [mlo, mhi] of each local particle (empty when mlo > mhi)."""
    c = np.cumsum(w_local)       # order differs from the device scan only by rounding
    n = len(w_local)
    mlo = np.empty(n, dtype=np.int64)
    mhi = np.empty(n, dtype=np.int64)
    for i in range(n):
        g = a + i
        cur = c[i] if a == 0 else offset + c[i]
        if g == 0:
            lo = 0
        else:
            prev = offset if i == 0 else (c[i - 1] if a == 0 else offset + c[i - 1])
            lo = first_above(prev, u0, N)
        hi = N - 1 if g == N - 1 else first_above(cur, u0, N) - 1
        mlo[i], mhi[i] = lo, hi
    return mlo, mhi, float(c[-1])


def _worker(rank, G, N, seed, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=G)
    rng = np.random.default_rng(seed)
    w = rng.random(N) ** 6
    w /= w.sum()
    w[rng.integers(0, N, N // 10)] = 0.0          # dropped-weight particles
    u0 = rng.uniform(0, 1.0 / N)
    a, b = shard(N, G, rank)
    wl = w[a:b]
    # local prefix end, all-gathered; offset = sum of the totals of earlier ranks
    t_local = float(np.cumsum(wl)[-1])
    totals = [None] * G
    dist.all_gather_object(totals, t_local)
    off = 0.0
    for g in range(rank):
        off = totals[0] if g == 0 else off + totals[g]
    mlo, mhi, _ = local_plan(wl, a, N, off, u0)
    sends = {}
    for p in range(G):
        pa, pb = shard(N, G, p)
        if p == rank:
            continue
        sel = [(a + i, max(mlo[i], pa), min(mhi[i], pb - 1)) for i in range(len(wl))
               if mlo[i] <= mhi[i] and mlo[i] < pb and mhi[i] >= pa]
        if sel:
            sends[p] = sel
    allp = [None] * G
    dist.all_gather_object(allp, (a, b, mlo.tolist(), mhi.tolist(), sends))
    if rank == 0:
        q.put((w, u0, allp))
    dist.destroy_process_group()


@pytest.mark.parametrize("G,N", [(2, 3001), (3, 4000)])
def test_sharded_plan_matches_oracle(G, N):
    from oracle import oracle as orc
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29600 + G
    procs = [ctx.Process(target=_worker, args=(r, G, N, 7 + G, port, q)) for r in range(G)]
    for p in procs:
        p.start()
    w, u0, allp = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    src_ref = orc.resample_src(w, u0)
    src = np.full(N, -1)
    for a, b, mlo, mhi, _ in allp:
        for i in range(b - a):
            if mlo[i] <= mhi[i]:
                assert (src[mlo[i]:mhi[i] + 1] == -1).all()      # covered once
                src[mlo[i]:mhi[i] + 1] = a + i
    assert (src >= 0).all()
    assert np.array_equal(src, src_ref)
    # every rank receives exactly the remote sources of its outputs
    for r in range(G):
        ra, rb = shard(N, G, r)
        need = {int(s) for s in src_ref[ra:rb] if not (ra <= s < rb)}
        got = set()
        for g, (a, b, mlo, mhi, sends) in enumerate(allp):
            for gsrc, lo, hi in sends.get(r, []):
                got.add(gsrc)
                assert np.all(src_ref[lo:hi + 1] == gsrc)
        assert got == need
