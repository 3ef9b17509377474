"""Pools that grow in place (reference fast_slam_2.py:111, where
maps grow by one landmark per append).

The page and record pools are virtual ranges reserved at creation, grown by
mapping physical chunks at their end (hipMemCreate / hipMemMap), so a growth
copies nothing: a scan that grows the record pool costs a collection and a
mapping, not an allocate-and-copy of the whole pool (round 3: ~20 ms for 35 GB).
A handle whose record pool starts just above its maps grows it within the run:
every measurement is a miss far from the maps (four new landmarks per particle
and scan, no weight change, no resample to share records), so the live records
grow by 4 N per scan and the pool must grow several times.  Every scan is
compared with the C oracle, and no scan takes more than 1 ms longer than the
median of its neighbours.
"""
import os
import time

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.mark.timeout(300)
@pytest.mark.parametrize("fail_relocate", [False, True])
def test_record_pool_grows_in_place(fail_relocate):
    """fail_relocate: the first growth that must move its reserved
    range fails right after the move (fs2_debug_vm_fail_after_relocate), so the
    allocate-and-copy fallback copies from the moved mapping; every scan must
    still match the oracle, with pool_copies > 0."""
    import fast_slam_2
    from fast_slam_2 import _native as nat
    import fs2_synthetic as syn
    from gpu_util import configure
    from oracle import oracle as orc
    configure()
    N, L, S = 200_000, 64, 24
    cap = L + 4 * S + 8
    wl = syn.Workload(N, L, seed=3)
    x, y, yaw = wl.poses()
    lm = wl.maps()
    w = np.full(N, 1.0 / N)
    cnt = np.full(N, L, np.int32)
    # records just above the maps: a few scans of writes, then collections, then growth
    f = fast_slam_2.FastSLAM2(N, rng="device", seed=4, landmark_capacity=cap, verbose=False, reduce="exact",
                              record_assoc=True, record_pool=N * L + 12 * N)
    f.set_state(x, y, yaw, w, cnt, lm)
    f.set_profiling(True)                   # (the collections' and growths' host time)
    nat.check(nat.load().fs2_debug_vm_fail_after_relocate(1 if fail_relocate else 0))
    o = orc.OracleFilter(N, cap)
    o.set_state(x, y, yaw, w, cnt, lm)
    rng = np.random.default_rng(12)
    ms_each, recs = [], []
    for s in range(S):
        rot, tr = syn.odometry(s)
        # four misses, 20+ m from the maps and from each other
        ms = np.array([[100.0 + 10.0 * s + 20.0 * k, 0.25 * k + 0.01 * s] for k in range(4)])
        nz = rng.normal(0, 0.001 if rot else 0.0055, N)
        u0 = rng.uniform(0, 1.0 / N)
        t0 = time.perf_counter()
        pose, st = f.step(rot, tr, ms, None, nz, u0)
        ms_each.append((time.perf_counter() - t0) * 1e3)
        recs.append(st.pool_records)
        opose, oassoc, ors, one = o.iterate(rot, tr, ms, nz, u0)
        assert np.array_equal(f.associations(), oassoc), s
        assert bool(st.resampled) == ors, s
        assert np.allclose(pose, opose, rtol=1e-9, atol=1e-12), s
    nat.load().fs2_debug_vm_fail_after_relocate(0)
    prof = f.profile()
    pool = {k: prof[k] for k in ("pool_collections", "collect_ms", "pool_grows", "grow_ms")}
    fx, fy, fyaw, fw, fc, flm = f.get_state(lm_cap=cap)
    assert np.array_equal(fc, o.cnt)
    assert np.allclose(flm, o.lm, rtol=1e-9, atol=1e-12)
    f.close()
    grew = [s for s in range(1, S) if recs[s] > recs[s - 1]]
    assert len(grew) >= 2, (recs, pool)                 # the record pool grew inside the run
    if fail_relocate:
        assert st.pool_copies > 0, st.pool_copies       # the fallback ran (and the scans matched)
        return
    assert st.pool_copies == 0, st.pool_copies          # in place: nothing moved
    for s in grew:
        nb = [ms_each[k] for k in range(max(1, s - 3), min(S, s + 4)) if k != s and k not in grew]
        assert ms_each[s] - float(np.median(nb)) < 1.0, (s, ms_each[s], nb, ms_each, pool)


@pytest.mark.timeout(300)
def test_growth_after_close_is_fast():
    """a set of handles closed, a new set created in
    the same process, and its first pool growth waited ~4 s for the runtime's
    deferred release of the closed handles' VMM chunks (profiles/
    r04_g8_refs_growth_probe.txt: 8 ranks as threads, page references on, 1e6
    particles, L = 500; the growth at the collective regrow after the resamples).
    fs2_destroy now drains the device around the releases.  Two sets of the same
    handles, one after the other: every set grows, and no growth takes 50 ms."""
    import threading

    import torch  # noqa: F401  -- (bench.populate fills the maps on the GPU)
    import bench
    import fast_slam_2
    import fs2_synthetic as syn
    G, N, L, S = 8, 1_000_000, 500, 9
    # the chunk cache is opt-in (by default a closed handle's memory
    # goes back to the device); this process closes and re-creates large handles
    old = os.environ.get("FS2_VMM_CACHE_MB")
    os.environ["FS2_VMM_CACHE_MB"] = "131072"
    try:
        _two_sets(G, N, L, S, bench, fast_slam_2, syn, threading)
    finally:
        if old is None:
            os.environ.pop("FS2_VMM_CACHE_MB", None)
        else:
            os.environ["FS2_VMM_CACHE_MB"] = old
        released = fast_slam_2.release_cached_memory()
        print(f"released {released >> 20} MiB of cached chunks")


def _two_sets(G, N, L, S, bench, fast_slam_2, syn, threading):
    for rep in range(2):
        key = b"grow" + bytes([rep]) * 124
        # (a record pool just above the maps: the records the scans write make
        # every set grow it -- the growth the stall was in)
        hs = [fast_slam_2.FastSLAM2(N, rng="device", seed=0, landmark_capacity=L + S + 8, rank=g, world_size=G,
                                    comm_id=key, comm_mode="local", verbose=False, page_refs="on",
                                    record_pool=(N // G) * (L + 12))
              for g in range(G)]
        for g, h in enumerate(hs):
            bench.populate(h, h.n_local, L, 0, g)
            h.set_profiling(True)
        meas = {s: np.ascontiguousarray(syn.scan_measurements(L, s, 0), dtype=np.float64) for s in range(S)}
        ms_each = []
        for s in range(S):
            err = []

            def run(g):
                try:
                    hs[g].step(*syn.odometry(s), meas[s])
                except Exception as e:    # re-raised below
                    err.append(e)
            t0 = time.perf_counter()
            th = [threading.Thread(target=run, args=(g,)) for g in range(G)]
            for t in th:
                t.start()
            for t in th:
                t.join()
            ms_each.append((time.perf_counter() - t0) * 1e3)
            if err:
                raise err[0]
        profs = [h.profile() for h in hs]
        for h in hs:
            h.close()
        grows = sum(p["pool_grows"] for p in profs)
        worst = max(p["grow_ms"] / max(p["pool_grows"], 1) for p in profs)
        print(f"rep {rep}: grows {grows} worst grow_ms {worst:.2f} scans {[round(m, 2) for m in ms_each]}")
        assert grows >= 1, (rep, profs[0])
        assert worst < 50.0, (rep, worst, ms_each)
