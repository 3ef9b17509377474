"""Sharded resample plan across processes (torch.distributed gloo, CPU).

Every rank runs libfs2's own plan code (fs2_plan_ranges / fs2_plan_sends:
csrc/fs2_plan.hpp, the arithmetic the device kernels k_ranges and
k_pack_bounds run) on its shard: it knows only its particles' normalised
weights, all-gathers its shard total, derives from its local prefix plus the
offset of the ranks before it the contiguous output range of each particle,
and plans what it sends to each peer.  Checked against the CPU oracle's
sequential low-variance resample (reference fast_slam_2.py:177-199): the union
of all shards' plans gives exactly the oracle's source of every output, every
output is covered once, and a receiver gets exactly the remote sources of its
outputs, with the slot counts of their maps.
"""
import ctypes as C
import os

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp


def shard(N, G, r):
    return N * r // G, N * (r + 1) // G


def _plan_lib():
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, os.path.join(os.path.dirname(here), "fast-slam_amd"))
    from fast_slam_2 import _native
    return _native.load()


def _worker(rank, G, N, seed, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=G)
    lib = _plan_lib()
    rng = np.random.default_rng(seed)
    w = rng.random(N) ** 6
    w /= w.sum()
    w[rng.integers(0, N, N // 10)] = 0.0          # dropped-weight particles
    cnt_all = rng.integers(0, 40, N).astype(np.int32)
    u0 = rng.uniform(0, 1.0 / N)
    a, b = shard(N, G, rank)
    wl = w[a:b]
    c = np.cumsum(wl)
    # local prefix end, all-gathered; offset = sum of the totals of earlier ranks
    totals = [None] * G
    dist.all_gather_object(totals, float(c[-1]))
    off = 0.0
    for g in range(rank):
        off = totals[0] if g == 0 else off + totals[g]
    n = b - a
    mlo = np.empty(n, np.int32)
    mhi = np.empty(n, np.int32)
    assert lib.fs2_plan_ranges(c.ctypes.data, n, a, N, off, u0, mlo.ctypes.data, mhi.ctypes.data) == 0
    cnt = np.ascontiguousarray(cnt_all[a:b])
    run = np.empty(2 * G, np.int64)
    K = np.empty(G, np.int64)
    S = np.empty(G, np.int64)
    assert lib.fs2_plan_sends(mlo.ctypes.data, mhi.ctypes.data, cnt.ctypes.data, n, N, G, rank,
                              run.ctypes.data, K.ctypes.data, S.ctypes.data) == 0
    sends = {}
    for p in range(G):
        if p == rank:
            assert K[p] == 0 and S[p] == 0
            continue
        pa, pb = shard(N, G, p)
        sel = [(a + i, max(int(mlo[i]), pa), min(int(mhi[i]), pb - 1), int(cnt[i]))
               for i in range(run[2 * p], run[2 * p + 1]) if mlo[i] <= mhi[i]]
        # the run holds every particle whose range reaches p, and only those
        direct = [i for i in range(n) if mlo[i] <= mhi[i] and mlo[i] < pb and mhi[i] >= pa]
        assert [g - a for g, _, _, _ in sel] == direct
        assert K[p] == len(sel) and S[p] == sum(x[3] for x in sel)
        if sel:
            sends[p] = sel
    allp = [None] * G
    dist.all_gather_object(allp, (a, b, mlo.tolist(), mhi.tolist(), sends))
    if rank == 0:
        q.put((w, cnt_all, u0, allp))
    dist.destroy_process_group()


@pytest.mark.parametrize("G,N", [(2, 3001), (3, 4000), (5, 997)])
def test_sharded_plan_matches_oracle(G, N):
    from oracle import oracle as orc
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29600 + G
    procs = [ctx.Process(target=_worker, args=(r, G, N, 7 + G, port, q)) for r in range(G)]
    for p in procs:
        p.start()
    w, cnt_all, u0, allp = q.get(timeout=240)
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
            for gsrc, lo, hi, nslots in sends.get(r, []):
                got.add(gsrc)
                assert np.all(src_ref[lo:hi + 1] == gsrc)
                assert nslots == cnt_all[gsrc]
        assert got == need
