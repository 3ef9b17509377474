"""Sharded (multi-rank) particle filter on one GPU.

G ranks run as threads of this process with the in-process transport
(FS2_COMM_LOCAL): every sharded code path -- cross-rank weight totals and
records, the range-based resample plan, packing, the grouped exchange and the
unpacking of received particles -- runs exactly as with RCCL, only the bytes
move by device copies.  Each scan is compared with a single-GPU handle on the
same inputs (device Philox noise is keyed by the global particle index, so both
draw identical noise): same resample decisions, estimates and associations;
states within 1e-9 relative (the weight total and the prefix are summed in a
different order across shards).
"""
import os
import threading

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _step_all(handles, rot, tr, ms):
    out = [None] * len(handles)
    err = [None] * len(handles)

    def run(g):
        try:
            out[g] = handles[g].step(rot, tr, ms)
        except Exception as e:  # pragma: no cover - surfaced below
            err[g] = e

    th = [threading.Thread(target=run, args=(g,)) for g in range(len(handles))]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=300)
    for e in err:
        if e is not None:
            raise e
    return out


def _ordered(handles):
    """Handles in the order of the shards they hold (equal shards change hands at
    resamples: a rank keeps the shard its sources fill most)."""
    return sorted(handles, key=lambda h: h.first_global)


def _gather(handles, cap):
    parts = [h.get_state(lm_cap=cap) for h in _ordered(handles)]
    return [np.concatenate([p[k] for p in parts]) for k in range(6)]


@pytest.mark.parametrize("G,N,L", [(2, 6000, 40), (3, 10007, 30), (4, 8192, 24), (8, 16384, 20)])
def test_sharded_matches_single(G, N, L):
    import torch  # noqa: F401
    import fast_slam_2
    import fs2_synthetic as syn
    from gpu_util import configure
    configure()
    wl = syn.Workload(N, L, seed=21)
    x, y, yaw = wl.poses()
    lm = wl.maps()
    # peaked likelihoods so that resampling fires and particles cross shard boundaries
    lm[:, :, 2] = lm[:, :, 5] = 0.01
    w = np.full(N, 1.0 / N)
    cnt = np.full(N, L, np.int32)
    cap = L + 40
    single = fast_slam_2.FastSLAM2(N, reduce="parallel", record_assoc=True, seed=5,
                                   landmark_capacity=cap, verbose=False)
    single.set_state(x, y, yaw, w, cnt, lm)
    key = os.urandom(128)
    shards = [fast_slam_2.FastSLAM2(N, reduce="parallel", record_assoc=True, seed=5,
                                    landmark_capacity=cap, rank=g, world_size=G, comm_id=key,
                                    comm_mode="local", verbose=False) for g in range(G)]
    for h in shards:
        a, b = h.first_global, h.first_global + h.n_local
        h.set_state(x[a:b], y[a:b], yaw[a:b], w[a:b], cnt[a:b], lm[a:b])
        h.set_profiling(True)
    resamples = 0
    moved = 0
    firsts = {g: {h.first_global} for g, h in enumerate(shards)}
    for s in range(8):
        rot, tr = syn.odometry(s)
        ms = wl.measurements(s)
        pre = _ordered(shards)       # the update pass's associations are of the shards held before the scan
        pose1, st1 = single.step(rot, tr, ms)
        outs = _step_all(shards, rot, tr, ms)
        for pose, st in outs:
            assert st.resampled == st1.resampled, s
            assert st.best_index == st1.best_index, s
            assert np.allclose(pose, pose1, rtol=1e-9, atol=1e-12), s
            assert np.isclose(st.n_eff, st1.n_eff, rtol=1e-9), s
            assert st.reduce_ambiguous == 0, s          # no decision the shard order could flip
        resamples += st1.resampled
        moved += sum(sh.last_stats.resample_slots for sh in shards)
        for g, h in enumerate(shards):
            firsts[g].add(h.first_global)
        assert sorted(h.first_global for h in shards) == [N * g // G for g in range(G)], s
        a1 = single.associations()
        ag = np.concatenate([h.associations() for h in pre], axis=1)
        assert np.array_equal(a1, ag), s
        s1 = single.get_state(lm_cap=cap)
        sg = _gather(shards, cap)
        assert np.array_equal(s1[4], sg[4]), s                     # map sizes
        for k in range(4):
            assert np.allclose(s1[k], sg[k], rtol=1e-9, atol=1e-15), (s, k)
        assert np.allclose(s1[5], sg[5], rtol=1e-9, atol=1e-12), s
    assert resamples >= 2
    # transfers: each destination gets each distinct page once, so once particles
    # share ancestors the pages sent are fewer than the rows they fill
    prof = [h.profile() for h in shards]
    assert sum(p["migrations"] for p in prof) >= 2, "the case must move particles across shards twice"
    assert sum(p["sent_particles"] for p in prof) > 0
    assert sum(p["sent_pages"] for p in prof) < sum(p["sent_rows"] for p in prof)
    for h in shards + [single]:
        h.close()


@pytest.mark.parametrize("G,N,L", [(2, 20000, 24), (3, 30011, 20), (4, 40000, 16), (8, 70001, 12)])
def test_sharded_exact_is_bitwise(G, N, L):
    """EXACT reductions across shards: Python's sum of the weights
    and the resample's running sum over the global order (every rank folds all
    shards' chain ops), numpy's sum(w'^2) over the global 8192-chunks (the chunks a
    shard boundary cuts completed from both neighbours' edges).  Every scan equals
    a single GPU handle in exact mode -- itself bit-exact with the reference's
    orders -- bit for bit: decisions, estimates, N_eff, every weight and pose, every
    landmark; reduce_ambiguous is 0 (no tree anywhere).  Weights spread over many
    binades (lognormal) so that the chains cross binades inside and across shards."""
    import torch  # noqa: F401
    import fast_slam_2
    import fs2_synthetic as syn
    from gpu_util import configure
    configure()
    wl = syn.Workload(N, L, seed=23)
    x, y, yaw = wl.poses()
    lm = wl.maps()
    lm[:, :, 2] = lm[:, :, 5] = 0.01
    wh = np.random.default_rng(5).lognormal(0.0, 2.0, N)
    w = wh / wh.sum()
    cnt = np.full(N, L, np.int32)
    cap = L + 40
    single = fast_slam_2.FastSLAM2(N, reduce="exact", record_assoc=True, seed=5, landmark_capacity=cap,
                                   verbose=False)
    single.set_state(x, y, yaw, w, cnt, lm)
    key = os.urandom(128)
    shards = [fast_slam_2.FastSLAM2(N, reduce="auto", record_assoc=True, seed=5, landmark_capacity=cap, rank=g,
                                    world_size=G, comm_id=key, comm_mode="local", verbose=False) for g in range(G)]
    for h in shards:
        a, b = h.first_global, h.first_global + h.n_local
        h.set_state(x[a:b], y[a:b], yaw[a:b], w[a:b], cnt[a:b], lm[a:b])
    resamples = 0
    for s in range(8):
        rot, tr = syn.odometry(s)
        ms = wl.measurements(s)
        pre = _ordered(shards)
        pose1, st1 = single.step(rot, tr, ms)
        outs = _step_all(shards, rot, tr, ms)
        for pose, st in outs:
            assert st.reduce_ambiguous == 0 and st.error_flags == 0, s
            assert st.resampled == st1.resampled, s
            assert st.best_index == st1.best_index, s
            assert st.n_eff == st1.n_eff, (s, st.n_eff, st1.n_eff)
            assert st.total_weight == st1.total_weight, (s, st.total_weight, st1.total_weight)
            assert np.array_equal(pose, pose1), s
        resamples += st1.resampled
        a1 = single.associations()
        assert np.array_equal(a1, np.concatenate([h.associations() for h in pre], axis=1)), s
        s1 = single.get_state(lm_cap=cap)
        sg = _gather(shards, cap)
        for k in range(6):
            assert np.array_equal(s1[k], sg[k]), (s, k)
    assert resamples >= 2
    for h in shards + [single]:
        h.close()


@pytest.mark.parametrize("G", [2, 4])
def test_sharded_exact_straddle(G):
    """(round 6) The exact chain across shards on tests/chain_cases.straddle_runs:
    long runs of identity units whose estimate straddles 2^0, on both sides of the
    crossing (translations by 0 in an inherited binade, chain_export's runs), a
    crossing inside one shard and heavy sources feeding every rank.  One scan
    without measurements (the tail alone) equals the single exact handle bit for
    bit."""
    import torch  # noqa: F401
    import fast_slam_2
    from chain_cases import straddle_runs
    from gpu_util import configure
    configure()
    N, L = 200_003, 4
    rng = np.random.default_rng(9)
    w = straddle_runs(N, rng)
    x, y, yaw = rng.normal(0, 1, N), rng.normal(0, 1, N), rng.normal(0, 0.1, N)
    lm = np.zeros((N, L, 6))
    lm[:, :, 0] = rng.normal(0, 5, (N, L))
    lm[:, :, 1] = rng.normal(0, 5, (N, L))
    lm[:, :, 2] = lm[:, :, 5] = 0.01
    cnt = np.full(N, L, np.int32)
    single = fast_slam_2.FastSLAM2(N, reduce="exact", seed=5, landmark_capacity=L, verbose=False)
    single.set_state(x, y, yaw, w, cnt, lm)
    key = os.urandom(128)
    shards = [fast_slam_2.FastSLAM2(N, reduce="auto", seed=5, landmark_capacity=L, rank=g, world_size=G,
                                    comm_id=key, comm_mode="local", verbose=False) for g in range(G)]
    for h in shards:
        a, b = h.first_global, h.first_global + h.n_local
        h.set_state(x[a:b], y[a:b], yaw[a:b], w[a:b], cnt[a:b], lm[a:b])
    ms = np.zeros((0, 2))
    pose1, st1 = single.step(0.0, 0.0, ms)
    assert st1.resampled
    for pose, st in _step_all(shards, 0.0, 0.0, ms):
        assert st.reduce_ambiguous == 0 and st.error_flags == 0
        assert st.total_weight == st1.total_weight and st.n_eff == st1.n_eff
        assert st.best_index == st1.best_index
        assert np.array_equal(pose, pose1)
    s1 = single.get_state(lm_cap=L)
    sg = _gather(shards, L)
    for k in range(6):
        assert np.array_equal(s1[k], sg[k]), k
    for h in shards + [single]:
        h.close()


def _run_sharded(G, N, L, scans, page_refs, seed=21, page_pool=0, record_pool=0, refuse=()):
    """G local ranks over the peaked workload, each scan checked against a single
    handle (decisions, estimates, associations; states within 1e-9); returns the
    ranks' profiles and last stats."""
    import fast_slam_2
    import fs2_synthetic as syn
    wl = syn.Workload(N, L, seed=seed)
    x, y, yaw = wl.poses()
    lm = wl.maps()
    lm[:, :, 2] = lm[:, :, 5] = 0.01
    w = np.full(N, 1.0 / N)
    cnt = np.full(N, L, np.int32)
    cap = L + 4 * scans + 8
    single = fast_slam_2.FastSLAM2(N, reduce="parallel", record_assoc=True, seed=5, landmark_capacity=cap,
                                   verbose=False)
    single.set_state(x, y, yaw, w, cnt, lm)
    key = os.urandom(128)
    shards = [fast_slam_2.FastSLAM2(N, reduce="parallel", record_assoc=True, seed=5, landmark_capacity=cap, rank=g,
                                    world_size=G, comm_id=key, comm_mode="local", verbose=False, page_refs=page_refs,
                                    page_pool=page_pool, record_pool=record_pool) for g in range(G)]
    for h in shards:
        a, b = h.first_global, h.first_global + h.n_local
        h.set_state(x[a:b], y[a:b], yaw[a:b], w[a:b], cnt[a:b], lm[a:b])
        h.set_profiling(True)
    from fast_slam_2 import _native as nat
    for g in refuse:
        nat.check(shards[g]._lib.fs2_debug_refuse_peer_maps(shards[g]._h), shards[g]._h)
    resamples = 0
    for s in range(scans):
        rot, tr = syn.odometry(s)
        ms = wl.measurements(s)
        pre = _ordered(shards)
        pose1, st1 = single.step(rot, tr, ms)
        outs = _step_all(shards, rot, tr, ms)
        for pose, st in outs:
            assert st.error_flags == 0, s
            assert st.resampled == st1.resampled and st.best_index == st1.best_index, s
            assert np.allclose(pose, pose1, rtol=1e-9, atol=1e-12), s
            assert st.reduce_ambiguous == 0, s
        resamples += st1.resampled
        assert np.array_equal(single.associations(), np.concatenate([h.associations() for h in pre], axis=1)), s
        if s % 4 == 3 or s == scans - 1:
            s1 = single.get_state(lm_cap=cap)
            sg = _gather(shards, cap)
            assert np.array_equal(s1[4], sg[4]), s
            for k in range(4):
                assert np.allclose(s1[k], sg[k], rtol=1e-9, atol=1e-15), (s, k)
            assert np.allclose(s1[5], sg[5], rtol=1e-9, atol=1e-12), s
    profs = [h.profile() for h in shards]
    last = [h.last_stats for h in shards]
    for h in shards + [single]:
        h.close()
    return resamples, profs, last


@pytest.mark.parametrize("G,N,L", [(2, 6000, 40), (8, 16384, 20)])
def test_page_refs_vs_whole_pages(G, N, L):
    """The sharded resample sending page-table rows of references (page_refs, the
    default) against sending each distinct page's content: both equal the single
    handle every scan; references move far fewer bytes at the resamples, and the
    update passes localise the remote pages they open (k_localize)."""
    from gpu_util import configure
    configure()
    r1, on, _ = _run_sharded(G, N, L, 10, "on")
    r0, off, _ = _run_sharded(G, N, L, 10, "off")
    assert r1 == r0 >= 2
    b_on, b_off = sum(p["sent_bytes"] for p in on), sum(p["sent_bytes"] for p in off)
    assert sum(p["migrations"] for p in on) >= 2
    assert 0 < b_on * 4 < b_off, (b_on, b_off)
    assert sum(p["localized_pages"] for p in on) > 0
    assert sum(p["localized_pages"] for p in off) == 0


def test_page_refs_fall_back_when_a_rank_cannot_map():
    """A rank that cannot map its peers' pools at the first scan (no peer access
    between devices; fs2_debug_refuse_peer_maps) turns page_refs off on every rank:
    the resamples send pages, every scan still equals the single handle."""
    from gpu_util import configure
    configure()
    G, N, L = 3, 6000, 40
    r1, fb, _ = _run_sharded(G, N, L, 8, "on", refuse=(1,))
    assert r1 >= 2
    assert [p["page_refs"] for p in fb] == [-1] * G
    assert sum(p["localized_pages"] for p in fb) == 0 and sum(p["migrations"] for p in fb) >= 2


def test_page_refs_collective_collections():
    """page_refs with pools just above the maps: after references cross ranks no
    rank may collect alone (another rank's rows name its pages), so every
    collection is collective (DevStats.collect_next from the all-gathered records);
    30 scans with collections and growing maps still equal the single handle."""
    from gpu_util import configure
    configure()
    G, N, L = 3, 4500, 12
    n = N // G
    rows = (L + 4 * 30 + 8 + 7) // 8
    resamples, profs, last = _run_sharded(G, N, L, 30, "on", seed=77, page_pool=n * rows * 2 + 16 * n,
                                          record_pool=n * rows * 8 * 2 + 64 * n)
    assert resamples >= 3
    cols = [st.collections for st in last]
    # (the imports' record shortfalls grow the fresh pools without collecting:
    # nothing could be freed) then, after references cross ranks, collective
    # collections, together (since round 5 the room bound counts distinct remote
    # pages, not remote row entries, so fewer collections are needed)
    assert min(cols) >= 2 and len(set(cols)) == 1, cols
    assert sum(p["localized_pages"] for p in profs) > 0


def _follow_case(G, N, L, seed):
    """Rank 0's particles alone carry weight, its first 100 ten times more than
    the rest: its sources fill shard 0 with few (heavy) particles and the other
    shards with many, so with shards following their sources rank 0 keeps a
    higher shard and the other ranks take the rest (all received)."""
    import fs2_synthetic as syn
    wl = syn.Workload(N, L, seed=seed)
    x, y, yaw = wl.poses()
    lm = wl.maps()
    n0 = N // G
    w = np.zeros(N)
    w[:n0] = 1e-3
    w[:100] = 1e-2
    return wl, x, y, yaw, w, np.full(N, L, np.int32), lm


@pytest.mark.parametrize("G,N", [(2, 6000), (4, 8192)])
def test_shards_follow_sources(G, N, monkeypatch):
    """A resample hands a rank the shard its own sources fill most (DESIGN §5,
    "output shards follow their sources"): every scan still equals a single handle,
    the shards stay a partition of the global order, and fewer particles move than
    with shard r pinned to rank r (FS2_SHARD_FOLLOW=0, the A/B)."""
    import fast_slam_2
    import fs2_synthetic as syn
    from gpu_util import configure
    configure()
    L = 16
    wl, x, y, yaw, w, cnt, lm = _follow_case(G, N, L, 5)
    cap = L + 24
    single = fast_slam_2.FastSLAM2(N, reduce="parallel", record_assoc=True, seed=9, landmark_capacity=cap,
                                   verbose=False)
    single.set_state(x, y, yaw, w, cnt, lm)
    sent = {}
    for follow in ("1", "0"):
        monkeypatch.setenv("FS2_SHARD_FOLLOW", follow)
        key = os.urandom(128)
        shards = [fast_slam_2.FastSLAM2(N, reduce="parallel", record_assoc=True, seed=9, landmark_capacity=cap,
                                        rank=g, world_size=G, comm_id=key, comm_mode="local", verbose=False)
                  for g in range(G)]
        for h in shards:
            a, b = h.first_global, h.first_global + h.n_local
            h.set_state(x[a:b], y[a:b], yaw[a:b], w[a:b], cnt[a:b], lm[a:b])
            h.set_profiling(True)
        if follow == "0":
            single.close()
            single = fast_slam_2.FastSLAM2(N, reduce="parallel", record_assoc=True, seed=9, landmark_capacity=cap,
                                           verbose=False)
            single.set_state(x, y, yaw, w, cnt, lm)
        for s in range(3):
            ms = np.zeros((0, 2)) if s == 0 else wl.measurements(s)
            pre = _ordered(shards)
            pose1, st1 = single.step(0.0, 0.03, ms)
            outs = _step_all(shards, 0.0, 0.03, ms)
            if s == 0:
                assert st1.resampled == 1
            for pose, st in outs:
                assert st.resampled == st1.resampled and st.best_index == st1.best_index, s
                assert np.allclose(pose, pose1, rtol=1e-9, atol=1e-12), s
                assert st.reduce_ambiguous == 0, s
            assert sorted(h.first_global for h in shards) == [N * g // G for g in range(G)], s
            assert np.array_equal(single.associations(),
                                  np.concatenate([h.associations() for h in pre], axis=1)), s
            s1 = single.get_state(lm_cap=cap)
            sg = _gather(shards, cap)
            assert np.array_equal(s1[4], sg[4]), s
            for k in range(4):
                assert np.allclose(s1[k], sg[k], rtol=1e-9, atol=1e-15), (s, k)
            assert np.allclose(s1[5], sg[5], rtol=1e-9, atol=1e-12), s
        if follow == "1":
            assert shards[0].first_global > 0, "rank 0 keeps the higher shard its sources fill most"
        else:
            assert [h.first_global for h in shards] == [N * g // G for g in range(G)]
        sent[follow] = sum(h.profile()["sent_particles"] for h in shards)
        for h in shards:
            h.close()
    single.close()
    assert 0 < sent["1"] < sent["0"], sent


@pytest.mark.parametrize("mode", ["rccl", "local"])
def test_sharded_path_one_rank(mode):
    """The sharded path with world_size 1 (sharded_path=True): the transport is
    created and every collective runs (RCCL: ncclCommInitRank, ncclAllGather, an
    empty grouped send/recv), so the RCCL transport is exercised on a one-GPU box.
    Results equal a plain handle."""
    import fast_slam_2
    import fs2_synthetic as syn
    from fast_slam_2 import _native as nat
    from gpu_util import configure
    configure()
    N, L = 5000, 30
    wl = syn.Workload(N, L, seed=41)
    x, y, yaw = wl.poses()
    lm = wl.maps()
    lm[:, :, 2] = lm[:, :, 5] = 0.01
    key = nat.comm_unique_id() if mode == "rccl" else os.urandom(128)
    hs = [fast_slam_2.FastSLAM2(N, reduce="parallel", record_assoc=True, seed=3, landmark_capacity=L + 40,
                                verbose=False, **kw)
          for kw in ({}, dict(sharded_path=True, comm_mode=mode, comm_id=key))]
    for h in hs:
        h.set_state(x, y, yaw, np.full(N, 1.0 / N), np.full(N, L, np.int32), lm)
    resamples = 0
    for s in range(6):
        rot, tr = syn.odometry(s)
        ms = wl.measurements(s)
        (p0, s0), (p1, s1) = [h.step(rot, tr, ms) for h in hs]
        assert s0.resampled == s1.resampled and s0.best_index == s1.best_index, s
        assert np.allclose(p0, p1, rtol=1e-12, atol=1e-15), s
        assert np.array_equal(hs[0].associations(), hs[1].associations()), s
        resamples += s0.resampled
    a, b = hs[0].get_state(lm_cap=L + 40), hs[1].get_state(lm_cap=L + 40)
    for u, v in zip(a, b):
        assert np.allclose(u, v, rtol=1e-12, atol=1e-15)
    assert resamples >= 1
    for h in hs:
        h.close()


def test_sharded_long_run_with_collections():
    """30 scans, 3 ranks, small initial capacity: maps grow past several page rows,
    resampling moves shared pages across shards and every rank's pool is collected
    more than once; each scan equals the single-handle run."""
    import fast_slam_2
    import fs2_synthetic as syn
    from gpu_util import configure
    configure()
    G, N, L = 3, 4500, 12
    wl = syn.Workload(N, L, seed=77)
    x, y, yaw = wl.poses()
    lm = wl.maps()
    lm[:, :, 2] = lm[:, :, 5] = 0.01
    w = np.full(N, 1.0 / N)
    cnt = np.full(N, L, np.int32)
    single = fast_slam_2.FastSLAM2(N, reduce="parallel", record_assoc=True, seed=11, landmark_capacity=16,
                                   verbose=False)
    single.set_state(x, y, yaw, w, cnt, lm)
    key = os.urandom(128)
    shards = [fast_slam_2.FastSLAM2(N, reduce="parallel", record_assoc=True, seed=11, landmark_capacity=16,
                                    rank=g, world_size=G, comm_id=key, comm_mode="local", verbose=False)
              for g in range(G)]
    for h in shards:
        a, b = h.first_global, h.first_global + h.n_local
        h.set_state(x[a:b], y[a:b], yaw[a:b], w[a:b], cnt[a:b], lm[a:b])
    resamples = 0
    for s in range(30):
        rot, tr = syn.odometry(s)
        ms = wl.measurements(s)
        pre = _ordered(shards)
        pose1, st1 = single.step(rot, tr, ms)
        outs = _step_all(shards, rot, tr, ms)
        for pose, st in outs:
            assert st.resampled == st1.resampled and st.best_index == st1.best_index, s
            assert np.allclose(pose, pose1, rtol=1e-9, atol=1e-12), s
        assert np.array_equal(single.associations(),
                              np.concatenate([h.associations() for h in pre], axis=1)), s
        resamples += st1.resampled
    cap = L + 30 * 4
    s1 = single.get_state(lm_cap=cap)
    sg = _gather(shards, cap)
    assert np.array_equal(s1[4], sg[4])
    assert np.allclose(s1[5], sg[5], rtol=1e-9, atol=1e-12)
    assert resamples >= 5
    assert max(h.last_stats.collections for h in shards) >= 2
    for h in shards + [single]:
        h.close()


def test_received_maps_longer_than_local_rows():
    """Rank 0's particles carry 40 landmarks (5 page rows), rank 1's only 4 (one
    row); peaked weights at the end of rank 0 make every output of rank 1 a copy
    of a rank-0 particle.  Rank 1 must size its page table for the received maps
    (the largest map over all ranks), and the result equals a single handle."""
    import fast_slam_2
    import fs2_synthetic as syn
    from gpu_util import configure
    configure()
    G, N, L = 2, 4000, 40
    wl = syn.Workload(N, L, seed=13)
    x, y, yaw = wl.poses()
    lm = wl.maps()
    cnt = np.full(N, L, np.int32)
    cnt[N // 2:] = 4
    lm[N // 2:, 4:] = 0.0
    w = np.full(N, 1e-9)
    w[N // 2 - 100:N // 2] = 1.0
    single = fast_slam_2.FastSLAM2(N, reduce="parallel", record_assoc=True, seed=2, landmark_capacity=8,
                                   verbose=False)
    single.set_state(x, y, yaw, w, cnt, lm)
    key = os.urandom(128)
    shards = [fast_slam_2.FastSLAM2(N, reduce="parallel", record_assoc=True, seed=2, landmark_capacity=8,
                                    rank=g, world_size=G, comm_id=key, comm_mode="local", verbose=False)
              for g in range(G)]
    for h in shards:
        a, b = h.first_global, h.first_global + h.n_local
        h.set_state(x[a:b], y[a:b], yaw[a:b], w[a:b], cnt[a:b], lm[a:b])
    for s in range(3):
        ms = np.zeros((0, 2)) if s == 0 else wl.measurements(s)
        pose1, st1 = single.step(0.0, 0.03, ms)
        outs = _step_all(shards, 0.0, 0.03, ms)
        if s == 0:
            assert st1.resampled == 1
        for pose, st in outs:
            assert st.resampled == st1.resampled and st.best_index == st1.best_index, s
            assert np.allclose(pose, pose1, rtol=1e-9, atol=1e-12), s
    cap = L + 16
    s1 = single.get_state(lm_cap=cap)
    sg = _gather(shards, cap)
    assert np.array_equal(s1[4], sg[4])
    assert int(sg[4][N // 2:].min()) >= L          # rank 1 now holds rank 0's long maps
    assert np.allclose(s1[5], sg[5], rtol=1e-9, atol=1e-12)
    for h in shards + [single]:
        h.close()
