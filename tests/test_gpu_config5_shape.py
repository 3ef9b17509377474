"""BASELINE config 5's shape on one GPU, checked against the C oracle every scan.

Config 5 is 8 ranks x 1e6 particles, L = 500, 180-beam scans, the resample
across ranks.  Here: 8 rank processes on cuda:0 (tests/cfg5_worker.py, the
stream-ordered shared-memory transport standing in for RCCL), 1e6 particles in
all (125 000 per rank), L = 500, M = 4 measurements per scan, 8 scans with
resamples that move particles across the shards, EXACT reductions across the
ranks (Python's sum and the running sum over the global order, numpy's
sum(w'^2) over the global chunks).  The parent runs the reference's algorithm
(oracle/fs2_oracle.c: first-match association, deep-copied maps, sequential
sums; fast_slam_2/algorithms/fast_slam_2.py:33-223, landmark_utils.py:92-117)
on the same inputs and draws, and requires, every scan and on every rank:
  * associations (N x M) bit-exact;
  * the resample decision and the estimate's index equal;
  * N_eff, the estimate's pose, every weight and pose within 1e-9, map sizes equal;
  * reduce_ambiguous == 0 (no decision left to a tree's rounding);
and a window of whole maps per scan within 1e-9, every particle's final map
through a per-particle checksum within 1e-9.
"""
import os
import subprocess
import sys
import time

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
G, N, L, S = 8, 1_000_000, 500, 8
RTOL = 1e-9


def _threads(pid):
    """Every thread's name, wait channel and (where readable) kernel stack: what a
    stuck rank waits on (read-only /proc)."""
    import glob
    out = []
    for t in sorted(glob.glob(f"/proc/{pid}/task/*")):
        row = [os.path.basename(t)]
        for k in ("comm", "wchan", "stack"):
            try:
                row.append(open(os.path.join(t, k)).read().strip().replace("\n", " | ")[:400])
            except OSError as e:
                row.append(f"<{e.strerror}>")
        out.append("  ".join(row))
    return "\n".join(out)


def _progress(msg):
    """A line into gpurun_out/ on the GPU box (the harness watches it for progress)."""
    root = os.environ.get("GRAFT_REPO_ROOT")
    if root and os.path.isdir(os.path.join(root, "gpurun_out")):
        with open(os.path.join(root, "gpurun_out", "test_progress.log"), "a") as f:
            f.write(f"{time.strftime('%H:%M:%S')} config5 {msg}\n")


@pytest.mark.timeout(900)
@pytest.mark.parametrize("page_refs", ["auto", "on"])
def test_config5_shape_eight_ranks_vs_oracle(tmp_path, page_refs):
    """page_refs "on": a migrating particle travels as references to pages on the
    rank that holds them; the rank processes map each other's pools (VMM chunks
    exported as file descriptors over Unix sockets -- hipIpcOpenMemHandle did not
    return here in round 4, profiles/r05_ipc_probe.txt) and grow them in place."""
    import fs2_synthetic as syn
    from cfg5_common import CAP, WINDOW, draws, initial_scalars, map_checksum, window_start
    from oracle import oracle as orc
    cap = CAP(L, S)
    key = os.urandom(128).hex()
    env = dict(os.environ, FS2_SHM_TIMEOUT_S="90", OMP_NUM_THREADS="2", FS2_TRACE="1",
               FS2_CFG5_PAGE_REFS=os.environ.get("FS2_CFG5_PAGE_REFS", page_refs))
    # the ranks' logs under gpurun_out/ on the GPU box (they come back with the call)
    root = os.environ.get("GRAFT_REPO_ROOT")
    logdir = os.path.join(root, "gpurun_out") if root and os.path.isdir(os.path.join(root, "gpurun_out")) \
        else str(tmp_path)
    logpaths = [os.path.join(logdir, f"cfg5_rank{r}.log") for r in range(G)]
    logs = [open(q, "w") for q in logpaths]
    procs = [subprocess.Popen([sys.executable, "-u", os.path.join(HERE, "cfg5_worker.py"), str(G), str(r), str(N),
                               str(L), str(S), key, str(tmp_path)], env=env, stdout=logs[r],
                              stderr=subprocess.STDOUT)
             for r in range(G)]
    try:
        # the oracle meanwhile (host): the same initial state and draws
        t0 = time.time()
        o = orc.OracleFilter(N, cap)
        x, y, yaw, w = initial_scalars(N)
        o.x[:], o.y[:], o.yaw[:], o.w[:] = x, y, yaw, w
        o.cnt[:] = L
        for a in range(0, N, 50_000):
            o.lm[a:a + 50_000, :L] = syn.particle_maps(N, L, 0, a, 50_000)
        _progress(f"oracle state ready {time.time() - t0:.0f} s")
        ref = []
        for s, (rot, tr, ms, nz, u0) in enumerate(draws(N, L, S)):
            pose, assoc, rs, ne = o.iterate(rot, tr, ms, nz, u0)
            w0 = window_start(N, s)
            ref.append(dict(pose=pose, assoc=assoc, resampled=rs, n_eff=ne, x=o.x.copy(), y=o.y.copy(),
                            yaw=o.yaw.copy(), w=o.w.copy(), cnt=o.cnt.copy(), win=o.lm[w0:w0 + WINDOW].copy()))
            _progress(f"oracle scan {s} resampled {rs} ({time.time() - t0:.0f} s)")
        checksum = np.concatenate([map_checksum(o.lm[a:a + 8192]) for a in range(0, N, 8192)])
        del o
        # a rank whose log has not grown for 240 s is taken to be stuck: every rank
        # is stopped and the test fails with their logs
        last, sizes = time.time(), [0] * G
        for r, p in enumerate(procs):
            while True:
                try:
                    p.wait(timeout=30)
                    break
                except subprocess.TimeoutExpired:
                    now = [os.path.getsize(q) for q in logpaths]
                    if now != sizes:
                        sizes, last = now, time.time()
                    _progress(f"waiting for rank {r}")
                    if time.time() - last > float(os.environ.get("FS2_CFG5_STUCK_S", "240")):
                        dump = "\n".join(f"rank {q} pid {procs[q].pid}:\n{_threads(procs[q].pid)}" for q in range(G)
                                         if procs[q].poll() is None)
                        with open(os.path.join(logdir, "cfg5_stuck_threads.txt"), "w") as f:
                            f.write(dump)
                        tails = "\n".join(f"rank {q}: " + open(logpaths[q]).read()[-600:] for q in range(G))
                        pytest.fail("ranks stuck (no log line for 240 s):\n" + tails)
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
        for f in logs:
            f.close()
    for r, p in enumerate(procs):
        assert p.returncode == 0, f"rank {r}:\n" + open(logpaths[r]).read()[-4000:]
    ranks = [np.load(tmp_path / f"rank{r}.npz") for r in range(G)]
    resamples = 0
    for s in range(S):
        R = ref[s]
        for r, d in enumerate(ranks):
            tag = (s, r)
            assert d["reduce_amb"][s] == 0 and d["error_flags"][s] == 0, tag
            assert bool(d["resampled"][s]) == R["resampled"], tag
            assert np.isclose(d["n_eff"][s], R["n_eff"], rtol=RTOL), tag
            assert np.allclose(d["pose"][s], R["pose"], rtol=RTOL, atol=1e-12), tag
        # the estimate's index is the one the oracle's pose belongs to
        bi = int(ranks[0]["best_index"][s])
        assert all(int(d["best_index"][s]) == bi for d in ranks), s
        assert np.allclose([R["x"][bi], R["y"][bi], R["yaw"][bi]], R["pose"], rtol=0, atol=0), s
        # associations: the shards held during the update pass, in global order
        order = sorted(ranks, key=lambda d: int(d["firsts_pre"][s]))
        assert np.array_equal(np.concatenate([d["assoc"][s] for d in order], axis=1), R["assoc"]), s
        # state after the scan: the shards held after it
        for d in ranks:
            a = int(d["firsts"][s])
            n = int(d["count"])
            sc = d["scal"][s]
            assert np.array_equal(sc[4].astype(np.int32), R["cnt"][a:a + n]), (s, a)
            for k, name in enumerate(("x", "y", "yaw")):
                assert np.allclose(sc[k], R[name][a:a + n], rtol=RTOL, atol=1e-12), (s, a, name)
            assert np.allclose(sc[3], R["w"][a:a + n], rtol=RTOL, atol=1e-300), (s, a)
        wins = [d[f"win{s}"] for d in ranks if d[f"win{s}"].shape[0]]
        assert len(wins) == 1, s
        assert np.allclose(wins[0], R["win"], rtol=RTOL, atol=1e-12), s
        resamples += int(R["resampled"])
    last = sorted(ranks, key=lambda d: int(d["firsts"][S - 1]))
    got = np.concatenate([d["checksum"] for d in last])
    assert np.allclose(got, checksum, rtol=RTOL, atol=1e-9)
    assert resamples >= 2, resamples
    assert sum(int(d["migrations"]) for d in ranks) >= 2, "particles must cross shards at two resamples"
    # no buffer reallocated inside a scan (received rows / pages are
    # sized for a whole shard at creation, the transfer arenas for half of one)
    assert all(int(d["scan_allocs"]) == 0 for d in ranks), [int(d["scan_allocs"]) for d in ranks]
    if env["FS2_CFG5_PAGE_REFS"] == "on":     # in effect on every rank, remote pages localised
        assert all(int(d["page_refs"]) == 1 for d in ranks), [int(d["page_refs"]) for d in ranks]
        assert sum(int(d["localized_pages"]) for d in ranks) > 0
