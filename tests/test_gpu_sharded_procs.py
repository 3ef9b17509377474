"""The whole sharded scan across processes (one GPU, G = 2 and 3 processes).

Each rank is its own process (tests/shard_proc_worker.py) with the
stream-ordered shared-memory transport (FS2_COMM_SHM): its collectives are a
copy to pinned staging, one host function on the stream behind a process
barrier, and a copy back -- no host-side stream sync, so the scan's kernels,
mid-scan posts and host waits follow the stream ordering RCCL ranks rely on
(the in-process transport of test_gpu_sharded.py synchronises around every
collective and hides it).  Reference semantics at stake: normalise, N_eff and
the low-variance resample across shards (fast_slam_2.py:161-199,212-223).

The parent compares every scan with a single handle in this process on the same
inputs: resample decisions, estimate index and pose, N_eff, associations, and at
the end every particle's state within 1e-9; reduce_ambiguous is 0 on every rank
and scan (no decision the shard order could flip), at least two resamples move
particles across shards.  The "numpy" case runs the drop-in iterate() with
numpy's global stream drawn on the device (fs2_mt_draw) on every rank, shards
that move included, and checks numpy's final state too.  The "refs" case sends
page references instead of pages: every rank maps the other processes' pools (VMM
chunks exported as file descriptors over Unix sockets, fs2_comm.hpp share_vm).
"refs_system" is the same on the system ROCm 7.2 runtime (FS2_HIP_RUNTIME=system,
rank processes that never import torch): the import branch that passes the
descriptor by value (fs2_comm.hpp import_fd), which the wheel's HIP 7.0 never takes.
"""
import os
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.mark.parametrize("G,N,L,scans,mode", [(2, 6000, 40, 8, "peaked"), (3, 10007, 30, 8, "peaked"),
                                               (2, 6000, 24, 4, "follow"), (2, 6000, 40, 8, "numpy"),
                                               (3, 9000, 40, 8, "refs"), (3, 9000, 40, 8, "refs_system")])
def test_sharded_processes_match_single(G, N, L, scans, mode, tmp_path):
    import torch  # noqa: F401
    import fast_slam_2
    import fs2_synthetic as syn
    from gpu_util import configure
    from shard_proc_worker import measurements, workload
    configure()
    key = os.urandom(128).hex()
    env = dict(os.environ, FS2_SHM_CHUNK=str(64 << 10), FS2_SHM_TIMEOUT_S="40")   # small mailboxes: rounds
    wmode = mode
    if mode == "refs_system":
        env["FS2_HIP_RUNTIME"] = "system"
        wmode = mode = "refs"
        system_rt = True
    else:
        system_rt = False
    outs = [str(tmp_path / f"rank{r}.npz") for r in range(G)]
    procs = [subprocess.Popen([sys.executable, "-u", os.path.join(HERE, "shard_proc_worker.py"), str(G), str(r),
                               str(N), str(L), "21", str(scans), key, outs[r], wmode],
                              env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
             for r in range(G)]
    logs = []
    for p in procs:
        try:
            logs.append(p.communicate(timeout=100)[0])
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
    for r, p in enumerate(procs):
        assert p.returncode == 0, f"rank {r} failed:\n{logs[r][-4000:]}"
    ranks = [np.load(o) for o in outs]
    for d in ranks:
        if system_rt:
            assert str(d["hip_runtime"]) == "system" and not bool(d["torch_imported"])
        else:
            assert bool(d["torch_imported"])

    wl, x, y, yaw, w, cnt, lm = workload(N, L, 21, mode, G)
    cap = L + 4 * scans + 8
    single = fast_slam_2.FastSLAM2(N, reduce="parallel", record_assoc=True, seed=5, landmark_capacity=cap,
                                   verbose=False, rng="numpy" if mode == "numpy" else "device")
    single.set_state(x, y, yaw, w, cnt, lm)
    np.random.seed(77)
    resamples = 0
    for s in range(scans):
        rot, tr = syn.odometry(s)
        if mode == "numpy":
            ms = [fast_slam_2.Measurement(float(d), float(b)) for d, b in measurements(wl, s, mode)]
            pose1 = np.array(single.iterate(rot, tr, ms))
            st1 = single.last_stats
        else:
            pose1, st1 = single.step(rot, tr, measurements(wl, s, mode))
        for r, d in enumerate(ranks):
            assert d["resampled"][s] == st1.resampled, (r, s)
            assert d["best_index"][s] == st1.best_index, (r, s)
            assert np.allclose(d["pose"][s], pose1, rtol=1e-9, atol=1e-12), (r, s)
            assert np.isclose(d["n_eff"][s], st1.n_eff, rtol=1e-9), (r, s)
            assert d["reduce_amb"][s] == 0, (r, s)
        # ranks in the order of the shards they held during scan s's update pass (the
        # associations' particles; a resample may then hand a rank another shard)
        order = sorted(ranks, key=lambda d: int(d["firsts_pre"][s]))
        a1 = single.associations()
        assert np.array_equal(a1, np.concatenate([d["assoc"][s][:a1.shape[0]] for d in order], axis=1)), s
        resamples += st1.resampled
    s1 = single.get_state(lm_cap=cap)
    for d in ranks:
        a, b = int(d["first"]), int(d["first"]) + int(d["count"])
        assert np.array_equal(s1[4][a:b], d["cnt"])
        for k, name in enumerate(("x", "y", "yaw", "w")):
            assert np.allclose(s1[k][a:b], d[name], rtol=1e-9, atol=1e-15), name
        assert np.allclose(s1[5][a:b], d["lm"], rtol=1e-9, atol=1e-12)
    single.close()
    if mode == "numpy":      # every rank left numpy's stream where the single handle did
        key, pos = np.random.get_state()[1], np.random.get_state()[2]
        for d in ranks:
            assert np.array_equal(d["np_key"], key) and int(d["np_pos"]) == pos
    need = 1 if mode == "follow" else 2
    assert resamples >= need
    assert sum(int(d["migrations"]) for d in ranks) >= need, "particles must cross shards"
    pages, rows = sum(int(d["sent_pages"]) for d in ranks), sum(int(d["sent_rows"]) for d in ranks)
    # siblings share pages once particles have resampled ancestors ("follow" moves
    # each particle's own initial map once: nothing shared yet)
    assert pages < rows if mode == "peaked" else pages <= rows
    if mode == "refs":       # page references between processes (VMM chunks over Unix sockets)
        assert all(int(d["page_refs"]) == 1 for d in ranks), [int(d["page_refs"]) for d in ranks]
        assert sum(int(d["localized_pages"]) for d in ranks) > 0
    if mode != "follow":     #  no buffer was reallocated inside a scan
        # ("follow" hands a whole shard over at once, beyond the half shard the
        # transfer arenas are sized for at creation)
        assert all(int(d["scan_allocs"]) == 0 for d in ranks), [int(d["scan_allocs"]) for d in ranks]
    if mode == "follow":     # rank 0 took the higher shard its sources fill most
        assert int(ranks[0]["firsts"][0]) > 0 and int(ranks[0]["first"]) > 0



def test_shm_timeout_is_a_clean_comm_error(tmp_path):
    """A rank that never reaches a collective: the others' stream-ordered
    collectives time out, and the scan reports FS2_ERR_COMM before any stale
    staging bytes could size the resample (post_and_wait checks the
    transport status); the late rank fails at once on the marked segment."""
    G = 2
    key = os.urandom(128).hex()
    env = dict(os.environ, FS2_SHM_TIMEOUT_S="2", FS2_TEST_STALL_S="8")
    outs = [str(tmp_path / f"rank{r}.npz") for r in range(G)]
    procs = [subprocess.Popen([sys.executable, "-u", os.path.join(HERE, "shard_proc_worker.py"), str(G), str(r),
                               "4000", "24", "21", "4", key, outs[r], "stall"],
                              env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
             for r in range(G)]
    logs = []
    for p in procs:
        try:
            logs.append(p.communicate(timeout=100)[0])
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
    for r, p in enumerate(procs):
        assert p.returncode == 0, f"rank {r} failed:\n{logs[r][-4000:]}"
    for r in range(G):
        d = np.load(outs[r])
        assert int(d["err_code"]) == -6, (r, str(d["err_msg"]))      # FS2_ERR_COMM
        assert int(d["err_scan"]) == 1, r
        assert "shm transport" in str(d["err_msg"]), str(d["err_msg"])
