#!/usr/bin/env python3
"""Benchmark of the FastSLAM 2.0 particle update (BASELINE.json metric).

One step = one FastSLAM2.iterate (reference fast_slam_2/algorithms/fast_slam_2.py:33-67)
over every particle: motion sample, M = 4 measurement updates (3 associating,
1 new landmark), normalise, N_eff, resample when N_eff < N/2, estimate.
Synthetic workload of SURVEY.md §8(d); particle state resident in HBM before
the timed region starts.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--config 3]
  torchrun --nproc-per-node N bench.py --gpus N ...   (one rank per GPU, particles sharded)

`python bench.py --gpus N` (N > 1) without WORLD_SIZE in the environment starts
the N ranks itself: one child process per GPU with RANK / LOCAL_RANK /
WORLD_SIZE / MASTER_ADDR / MASTER_PORT, spawned before this process touches the
GPU (no exec); it fails loudly when fewer than N GPUs are visible.  Rank 0
prints the JSON line.  `--dry-run` prints the children's environments instead.

Default workload: BASELINE config 3, 1e6 particles per GPU x 500 landmarks.
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
# libfs2 keeps closed handles' VMM chunks for later growths only when asked (default
# off); this process closes and re-creates handle sets of the headline's size, whose
# first growth otherwise waits for the driver's deferred release
os.environ.setdefault("FS2_VMM_CACHE_MB", "131072")
sys.path.insert(0, os.path.join(REPO, "fast-slam_amd"))
sys.path.insert(0, REPO)

CONFIGS = {
    "1": dict(N=100, L=20, P=180, icp=False, name="cfg1_N100_L20_180beam"),
    "2": dict(N=100_000, L=200, P=180, icp=False, name="cfg2_N1e5_L200_180beam"),
    "3": dict(N=1_000_000, L=500, P=180, icp=False, name="cfg3_N1e6_L500_180beam"),
    "4": dict(N=1_000_000, L=500, P=720, icp=True, name="cfg4_N1e6_L500_720beam_icp"),
}
HBM_PEAK_GBS = 8000.0        # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
PROFILE_EVERY = 4            # timed scans per profiled scan (libfs2 fs2_set_profiling)


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="3", choices=sorted(CONFIGS))
    ap.add_argument("--particles", type=int, default=0, help="override particles per GPU")
    ap.add_argument("--landmarks", type=int, default=0, help="override landmarks per particle")
    ap.add_argument("--map", choices=("grid", "dense"), default="grid",
                    help="dense: the robustness dense-map workload as the timed one (its PMC record)")
    ap.add_argument("--profile-every", type=int, default=PROFILE_EVERY,
                    help="timed scans per scan with kernel events (0: none; the line then lacks kernel times)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--no-gate-filter", action="store_true",
                    help="A/B: read every visited slot's fp64 data (no fp32 gate mirror)")
    ap.add_argument("--no-extras", action="store_true",
                    help="skip the workload-robustness runs (60-scan continuation, dense map, no gate filter)")
    ap.add_argument("--serial-icp", action="store_true",
                    help="A/B (config 4): align each scan just before its update instead of "
                         "beside the previous scan's update")
    ap.add_argument("--comm", choices=("rccl", "shm"), default="rccl",
                    help="libfs2 transport between ranks (shm: POSIX shared memory, any GPUs)")
    ap.add_argument("--share-gpu", action="store_true",
                    help="testing: every rank on GPU 0 (implies --comm shm; the bench's own barrier and "
                         "timing reduction over gloo)")
    ap.add_argument("--dry-run", action="store_true",
                    help="with --gpus N > 1 and no WORLD_SIZE: print the ranks' environments, start nothing")
    ap.add_argument("--icp-offline", action="store_true",
                    help="A/B (config 4): align every scan before the timed loop and feed the same odometry, "
                         "so the timed scans run config 4's workload without an alignment beside them")
    ap.add_argument("--probe-side-kernels", type=int, default=0,
                    help="A/B (config 4 interference): launch this many tiny kernels on a second stream "
                         "before each scan, as the ICP hand-off does")
    ap.add_argument("--pipelined", action="store_true",
                    help="time the headline through step_submit / step_wait with two submits outstanding "
                         "(fs2.h fs2_iterate_submit: the second completes the first; round 5's overlapped "
                         "variant measured no faster, profiles/r05_ab_pipelined.txt, and was removed)")
    ap.add_argument("--dropin", action="store_true",
                    help="time the drop-in FastSLAM2.iterate() (numpy RNG) beside the device-RNG step")
    return ap.parse_args(argv)


RANK_ENV = ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")


def rank_envs(n, port, base=None):
    """The environment of each of the n rank processes bench.py starts itself
    (the variables torch.distributed.run would set; 127.0.0.1 rendezvous)."""
    base = dict(os.environ if base is None else base)
    base.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")      # RCCL over dmabuf IPC on this pool
    return [dict(base, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                 MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port)) for r in range(n)]


def free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


def visible_gpus():
    """GPUs this process could use, counted without initialising HIP
    (torch.cuda.device_count() reads the device list only, on this image)."""
    import torch
    return torch.cuda.device_count()


def launch_ranks(args, argv):
    """--gpus N > 1 outside torch.distributed.run: start N rank processes (children,
    this process never touches the GPU), wait for all, exit with the worst status.
    A rank that fails ends the others (their collectives would wait forever)."""
    import signal
    import subprocess
    n = args.gpus
    envs = rank_envs(n, free_port())
    if args.dry_run:
        print(json.dumps([{k: e[k] for k in RANK_ENV} for e in envs]), flush=True)
        return 0
    have = visible_gpus()
    need = 1 if args.share_gpu else n
    if have < need:
        print(f"bench.py: --gpus {n} needs {need} visible GPUs, this process sees {have}; "
              f"refusing to time fewer ranks than asked", file=sys.stderr, flush=True)
        return 2
    procs = [subprocess.Popen([sys.executable, os.path.abspath(__file__), *argv], env=e) for e in envs]
    rcs = [None] * n
    try:
        while any(rc is None for rc in rcs):
            for r, p in enumerate(procs):
                if rcs[r] is None:
                    rcs[r] = p.poll()
            bad = [r for r, rc in enumerate(rcs) if rc not in (None, 0)]
            if bad:
                time.sleep(5)                   # a failing rank's peers get a moment to report
                for r, p in enumerate(procs):
                    if p.poll() is None:
                        print(f"bench.py: rank {bad[0]} exited with {rcs[bad[0]]}; stopping rank {r}",
                              file=sys.stderr, flush=True)
                        p.send_signal(signal.SIGTERM)
                for r, p in enumerate(procs):
                    try:
                        rcs[r] = p.wait(timeout=30)
                    except subprocess.TimeoutExpired:
                        p.kill()
                        rcs[r] = p.wait()
                break
            time.sleep(0.2)
    except KeyboardInterrupt:
        for p in procs:
            if p.poll() is None:
                p.kill()
        raise
    worst = max((abs(rc) for rc in rcs), default=0)
    return 0 if worst == 0 else (worst if worst < 256 else 1)


def populate(f, n_local, L, seed, rank, base_map=None):
    """Synthetic initial state generated on the GPU in chunks; base_map
    [L][2] replaces the 6 m landmark grid (dense-map variant)."""
    import torch
    import fs2_synthetic as syn
    from fast_slam_2 import _native as nat
    dev = torch.device("cuda", torch.cuda.current_device())
    g = torch.Generator(device=dev)
    g.manual_seed(1_000_003 * (seed + 1) + rank)
    base = torch.tensor(syn.common_landmarks(L, seed) if base_map is None else base_map, dtype=torch.float64,
                        device=dev)
    x = torch.randn(n_local, generator=g, dtype=torch.float64, device=dev) * 0.05
    y = torch.randn(n_local, generator=g, dtype=torch.float64, device=dev) * 0.05
    yaw = torch.randn(n_local, generator=g, dtype=torch.float64, device=dev) * 0.01
    w = torch.full((n_local,), 1.0 / f.num_particles, dtype=torch.float64, device=dev)
    torch.cuda.synchronize()
    nat.check(f._lib.fs2_set_state(f._h, 0, n_local, x.data_ptr(), y.data_ptr(), yaw.data_ptr(),
                                   w.data_ptr(), None, None, 0, nat.FS2_DEVICE), f._h)
    chunk = max(1, (512 << 20) // (L * 48))
    for o in range(0, n_local, chunk):
        k = min(chunk, n_local - o)
        lm = torch.empty((k, L, 6), dtype=torch.float64, device=dev)
        lm[:, :, 0:2] = base + syn.MAP_JITTER * torch.randn((k, L, 2), generator=g,
                                                            dtype=torch.float64, device=dev)
        lm[:, :, 2] = syn.INIT_COV
        lm[:, :, 3] = 0.0
        lm[:, :, 4] = 0.0
        lm[:, :, 5] = syn.INIT_COV
        cnt = torch.full((k,), L, dtype=torch.int32, device=dev)
        torch.cuda.synchronize()
        nat.check(f._lib.fs2_set_state(f._h, o, k, None, None, None, None, cnt.data_ptr(),
                                       lm.data_ptr(), L, nat.FS2_DEVICE), f._h)
        del lm, cnt
    torch.cuda.synchronize()


def cpu_baseline(L, P, budget_s, seed):
    """The C oracle (oracle/fs2_oracle.c, reference semantics) on a sample of the
    workload: with every host thread OpenMP gives it (the reference's NUM_THREAD
    particle pool), and with one thread."""
    import fs2_synthetic as syn
    from oracle import oracle as orc

    def run(n, threads, budget):
        orc.set_threads(threads)
        wl = syn.Workload(n, L, seed)
        x, y, yaw = wl.poses()
        o = orc.OracleFilter(n, L + 4 * 61)
        o.set_state(x, y, yaw, np.full(n, 1.0 / n), np.full(n, L), wl.maps())
        rng = np.random.default_rng(seed)
        t_work, scans = 0.0, 0
        while t_work < budget and scans < 60:
            rot, tr = syn.odometry(scans)
            ms = wl.measurements(scans)
            nz = rng.normal(0, 0.001 if rot else 0.0055, n)
            u0 = rng.uniform(0, 1.0 / n)
            t0 = time.perf_counter()
            o.iterate(rot, tr, ms, nz, u0)
            t_work += time.perf_counter() - t0
            scans += 1
        del o
        return n * scans / t_work, scans, t_work

    threads = orc.threads()
    try:
        affinity = len(os.sched_getaffinity(0))
    except Exception:
        affinity = None
    quota = None                  # the cgroup's CPU quota (cpu.max), in CPUs
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        quota = None if q == "max" else int(q) / int(per)
    except Exception:
        pass
    model = "unknown"
    try:
        model = next(l.split(":", 1)[1].strip() for l in open("/proc/cpuinfo") if l.startswith("model name"))
    except Exception:
        pass
    one, s1, t1 = run(6000, 1, budget_s / 2)
    n = 6000 * max(1, min(threads, 32))
    many, sm, tm = run(n, threads, budget_s / 2)
    orc.set_threads(threads)
    return dict(value=many, unit="particle-updates/s", cores=threads, kind="port",
                cpu_model=model, host_cpus=os.cpu_count(), affinity_cpus=affinity, cgroup_cpu_quota=quota,
                single_thread_value=one,
                affinity_linear_projection=(one * affinity if affinity else None),
                threads_note=("threads = OMP_NUM_THREADS, the CPU share a one-GPU job gets on the GPU pool "
                              "(its rules fix worker pools at that share although the affinity mask lists "
                              "every host CPU); affinity_linear_projection = single_thread_value x "
                              "affinity_cpus, a projection to every CPU of the host, not a measurement"),
                python_reference_config1=python_reference_record(),
                sample=f"{n} particles x {L} landmarks, M=4, {sm} scans on {threads} OpenMP threads "
                       f"(OMP_NUM_THREADS; {affinity} CPUs in this process's affinity mask of "
                       f"{os.cpu_count()} on the host) ({tm:.1f} s); 1 thread: 6000 particles, {s1} scans "
                       f"({t1:.1f} s); "
                       f"C oracle, reference semantics and reference algorithm (first-match linear "
                       f"scan of every map, deep-copied maps on resample): the ratio to the GPU "
                       f"value mixes algorithm (pruning, page sharing) with hardware")


def python_reference_record():
    """The Python reference itself timed at config 1 in the build container
    (scripts/time_reference_cfg1.py; /root/reference is not on the GPU box)."""
    p = os.path.join(REPO, "profiles", "r04_reference_cfg1_container.json")
    try:
        rec = json.load(open(p))
    except Exception:
        return None
    return {k: rec.get(k) for k in ("host", "reference_ms_per_scan_median", "reference_particle_updates_per_s",
                                    "oracle_c_particle_updates_per_s")}


def pmc_record(workload):
    """The committed PMC summary of `workload` (scripts/pmc_round.sh ->
    scripts/pmc_summary.py -> profiles/pmc_{workload}.json) if it was measured on a
    library built from these sources (its source_id equals the build's), else None."""
    import build
    p = os.path.join(REPO, "profiles", f"pmc_{workload}.json")
    if not os.path.exists(p):
        return None
    try:
        rec = json.load(open(p))
    except Exception:
        return None
    return rec if rec.get("source_id") == build.source_id() else None


def pmc_traffic(rec, kernel):
    return None if rec is None else rec.get(kernel, {}).get("hbm_bytes_per_launch")


def timed_scans(f, scans, meas_of, odo_of, warmup):
    """Warm-up then timed scans of handle f; (particle-updates/s, ms/scan, stats sums)."""
    import torch
    for s in scans[:warmup]:
        f.step(*odo_of(s), meas_of(s))
    torch.cuda.synchronize()
    sums = dict(visited=0, opened=0, appends=0, resamples=0, cow=0)
    t0 = time.perf_counter()
    for s in scans[warmup:]:
        _, st = f.step(*odo_of(s), meas_of(s))
        sums["visited"] += st.slots_visited
        sums["opened"] += st.pages_opened
        sums["appends"] += st.appends
        sums["resamples"] += st.resampled
        sums["cow"] += st.cow_pages
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    k = len(scans) - warmup
    n = f.n_local
    return {"value": n * k / dt, "ms_per_scan": dt / k * 1e3, "scans": k,
            "slots_visited_per_particle_scan": sums["visited"] / (n * k),
            "pages_opened_per_particle_scan": sums["opened"] / (n * k),
            "appends_per_particle_scan": sums["appends"] / (n * k),
            "cow_pages_per_particle_scan": sums["cow"] / (n * k), "resamples": sums["resamples"]}


def dense_workload(L, seed):
    """The dense-map variant: L landmarks uniform over the room, each scan's hits
    near random ones and a miss 30 m outside.  Returns (map [L][2], meas_of)."""
    import fs2_synthetic as syn
    rng = np.random.default_rng(seed + 17)
    hw, hh = syn.ROOM[0] / 2, syn.ROOM[1] / 2
    dense = np.column_stack([rng.uniform(-hw, hw, L), rng.uniform(-hh, hh, L)])

    def dense_meas(s):
        r = np.random.default_rng([seed, 900 + s])
        ks = r.integers(0, L, 3)
        pts = [dense[k] + r.uniform(-0.3, 0.3, 2) for k in ks] + [np.array([30.0 + s, -30.0])]
        return np.array([syn.encode(*p) for p in pts])

    return dense, dense_meas


def robustness(args, f, L, first_scan):
    """How much of the headline depends on the synthetic map's sparsity and on the
    run length: the same handle 40 scans further (60 in all), a dense
    map (L landmarks uniform over the 20 x 15 m room, several inside every gate),
    and the grid map without the fp32 gate filter.  Not part of `value`."""
    import fast_slam_2
    import fs2_synthetic as syn
    out = {}
    steps = 40
    meas = {s: np.ascontiguousarray(syn.scan_measurements(L, s, args.seed), dtype=np.float64)
            for s in range(first_scan, first_scan + steps)}
    out["long_run_60"] = timed_scans(f, list(range(first_scan, first_scan + steps)), meas.__getitem__,
                                     syn.odometry, 0)
    out["long_run_60"]["note"] = f"scans {first_scan}..{first_scan + steps - 1} of the headline handle"
    n = f.n_local
    dense, dense_meas = dense_workload(L, args.seed)
    scans = list(range(13))
    g = fast_slam_2.FastSLAM2(n, rng="device", seed=args.seed, landmark_capacity=L + 24, verbose=False)
    populate(g, n, L, args.seed, 0, base_map=dense)
    out["dense_map"] = timed_scans(g, scans, dense_meas, syn.odometry, 3)
    out["dense_map"]["note"] = f"{L} landmarks uniform in the room (grid: 6 m spacing)"
    g.close()
    g = fast_slam_2.FastSLAM2(n, rng="device", seed=args.seed, landmark_capacity=L + 24, verbose=False,
                              gate_filter=False)
    populate(g, n, L, args.seed, 0)
    gm = {s: np.ascontiguousarray(syn.scan_measurements(L, s, args.seed), dtype=np.float64) for s in scans}
    out["no_gate_filter"] = timed_scans(g, scans, gm.__getitem__, syn.odometry, 3)
    out["no_gate_filter"]["note"] = "grid map, every slot's fp64 record read (no mirrors, no page boxes)"
    g.close()
    out["appended_maps"] = appended_maps(args, L, n)
    out["sharded_local_g2"] = sharded_local(args, L, n)
    out["sharded_local_g8"] = sharded_local(args, L, n, G=8, page_refs="on")
    # the same with whole pages sent (round 3's transfer; A/B of the page references)
    out["sharded_local_g8_pages"] = sharded_local(args, L, n, G=8, page_refs="off")
    out["dropin_iterate"] = dropin(args, L, n)
    out["dropin_iterate_host_rng"] = dropin(args, L, n, rng="numpy-host")
    return out


def appended_maps(args, L, n, per_scan=8):
    """The reference's own operating mode: maps grown by appends
    from fs2_create's empty maps (fast_slam_2.py:20-31 -- every particle at the
    origin, no landmark) through the misses of a robot discovering the L grid
    landmarks in observation order (a lawnmower sweep, fs2_synthetic.
    buildup_measurements: 8 new landmarks and 2 re-observations per scan, standing
    still), so pages hold landmarks in the order they were seen and no import
    layout is involved; then the headline's 3 warm-up + 20 timed scans of
    measurements on those maps."""
    import fast_slam_2
    import fs2_synthetic as syn
    import torch
    nb = syn.buildup_scans(L, per_scan)
    cap = L + 40
    g = fast_slam_2.FastSLAM2(n, rng="device", seed=args.seed, landmark_capacity=cap, verbose=False)
    t0 = time.perf_counter()
    res_b = 0
    for s in range(nb):
        _, st = g.step(0.0, 0.0, np.ascontiguousarray(syn.buildup_measurements(L, s, args.seed, per_scan)))
        res_b += st.resampled
    torch.cuda.synchronize()
    t_build = time.perf_counter() - t0
    cnt = g.get_state(lm_cap=0)[4] if n <= 2_000_000 else None
    meas = {s: np.ascontiguousarray(syn.scan_measurements(L, s, args.seed), dtype=np.float64) for s in range(23)}
    g.set_profiling(True, every=PROFILE_EVERY)
    r = timed_scans(g, list(range(23)), meas.__getitem__, syn.odometry, 3)
    pr = g.profile()
    g.close()
    r["kernel_ms"] = {"k_candidates": pr["filter_ms"] / max(pr["filter_launches"], 1),
                      "k_update": pr["exact_ms"] / max(pr["exact_launches"], 1),
                      "reduce_and_resample": pr["reduce_ms"] / max(pr["scans"], 1)}
    # pool upkeep inside the 23 scans (the maps grew to L by appends: the pools hold
    # what the build-up wrote, so collections / growths come sooner than after an import)
    r["pool"] = {"collections": pr["pool_collections"], "collect_ms": pr["collect_ms"],
                 "grows": pr["pool_grows"], "grow_ms": pr["grow_ms"]}
    r.update(buildup_scans=nb, buildup_s=t_build, buildup_resamples=res_b,
             map_size_after_buildup=(None if cnt is None else [int(cnt.min()), int(cnt.max())]),
             note=f"maps grown from empty by appends in observation order ({nb} scans of {per_scan} new "
                  f"landmarks + 2 re-observations, lawnmower discovery order), then the headline's "
                  f"measurement stream; compare pages_opened_per_particle_scan with the imported layout's")
    return r


def dropin(args, L, n, scans=23, warm=3, rng="numpy"):
    """What a reference caller gets: FastSLAM2.iterate(rotation, translation,
    list[Measurement]) (fast_slam_2.py:33, called at jde_robots_main.py:38) with
    numpy's global legacy RNG -- N normals per scan and the resample start,
    exactly as the reference draws them (Q4/Q5) -- on a handle of the headline
    size.  rng="numpy": drawn on the GPU from np.random's state (fs2_mt_draw);
    "numpy-host": drawn by numpy on the host.  host_rng_ms: np.random.normal of N
    values alone.  The numpy state after the run is the same either way."""
    import fast_slam_2
    import fs2_synthetic as syn
    from fast_slam_2.models.measurement import Measurement
    import ctypes
    from fast_slam_2 import _native as nat
    np.random.seed(args.seed)
    f = fast_slam_2.FastSLAM2(n, rng=rng, seed=args.seed, landmark_capacity=L + scans + 8, verbose=False)
    populate(f, n, L, args.seed, 0)
    meas = [[Measurement(float(d), float(b)) for d, b in syn.scan_measurements(L, s, args.seed)]
            for s in range(scans)]
    for s in range(warm):
        f.iterate(*syn.odometry(s), meas[s])
    f.set_profiling(True)          # every scan's device time (events), to split host from device
    t0 = time.perf_counter()
    res = 0
    each, rs_each = [], []
    for s in range(warm, scans):
        t1 = time.perf_counter()
        f.iterate(*syn.odometry(s), meas[s])
        each.append(time.perf_counter() - t1)
        res += f.last_stats.resampled
        rs_each.append(int(f.last_stats.resampled))
    dt = time.perf_counter() - t0
    pr = f.profile()
    f.close()
    state_digest = hashlib.sha1(np.random.get_state()[1].tobytes()).hexdigest()[:12]
    t1 = time.perf_counter()
    for _ in range(3):
        np.random.normal(0, 0.0055, size=n)
    rng_ms = (time.perf_counter() - t1) / 3 * 1e3
    k = scans - warm
    note = ("FastSLAM2.iterate() with numpy's legacy RNG (the reference's draws, bit for bit); "
            + ("drawn on the GPU from np.random's state (MT19937 + polar method, fs2_mt_draw)" if rng == "numpy"
               else "drawn by numpy on one host core (host-RNG bound)"))
    ms_rs = [e * 1e3 for e, r in zip(each, rs_each) if r]
    ms_ot = [e * 1e3 for e, r in zip(each, rs_each) if not r]
    return {"value": n * k / dt, "ms_per_scan": dt / k * 1e3, "scans": k, "resamples": res,
            "ms_per_scan_median": float(np.median(each)) * 1e3,
            "ms_each": [round(e * 1e3, 3) for e in each],
            "resampled_each": rs_each,
            # scan by scan against the headline (extra.scan_ms_by_kind): the same kinds of scan
            "ms_resampling_scan_mean": float(np.mean(ms_rs)) if ms_rs else None,
            "ms_other_scan_mean": float(np.mean(ms_ot)) if ms_ot else None,
            # the scans' device time (first kernel to publication) against the wall time per
            # iterate(): the rest is the host's share (measurement objects, numpy's state
            # read and written, the draw's host half: counts, listed logs)
            "scan_device_ms_mean": pr["scan_ms"] / max(pr["scans"], 1),
            "host_share_ms_per_scan": dt / k * 1e3 - pr["scan_ms"] / max(pr["scans"], 1),
            "window": f"scans {warm}..{scans - 1} (the headline's)",
            "host_rng_ms": rng_ms, "rng": rng, "numpy_state_sha1": state_digest, "note": note}


def sharded_local(args, L, n_total, G=2, scans=9, warm=3, page_refs="auto"):
    """The sharded path (fs2_comm.hpp) with G ranks as threads of this process on
    this GPU (in-process transport: device copies + host barriers), n_total
    particles in all: the per-scan time and the host time inside the transport
    calls and mid-scan waits (libfs2 profile comm_ms).  Not an RCCL figure."""
    import threading
    import fast_slam_2
    import fs2_synthetic as syn
    key = os.urandom(128)
    hs = [fast_slam_2.FastSLAM2(n_total, rng="device", seed=args.seed, landmark_capacity=L + scans + 8, rank=g,
                                world_size=G, comm_id=key, comm_mode="local", verbose=False, page_refs=page_refs)
          for g in range(G)]
    for g, h in enumerate(hs):
        populate(h, h.n_local, L, args.seed, g)
    meas = {s: np.ascontiguousarray(syn.scan_measurements(L, s, args.seed), dtype=np.float64) for s in range(scans)}
    res = [0] * G

    def step_all(s):
        err = []

        def run(g):
            try:
                _, st = hs[g].step(*syn.odometry(s), meas[s])
                res[g] += st.resampled
            except Exception as e:  # surfaced below
                err.append(e)
        th = [threading.Thread(target=run, args=(g,)) for g in range(G)]
        for t in th:
            t.start()
        for t in th:
            t.join()
        if err:
            raise err[0]
    for s in range(warm):
        step_all(s)
    for h in hs:
        h.set_profiling(True)
    res = [0] * G
    per = []
    t0 = time.perf_counter()
    for s in range(warm, scans):
        t1 = time.perf_counter()
        step_all(s)
        per.append((time.perf_counter() - t1) * 1e3)
    dt = time.perf_counter() - t0
    k = scans - warm
    profs = [h.profile() for h in hs]
    for h in hs:
        h.close()
    return {"value": n_total * k / dt, "ms_per_scan": dt / k * 1e3, "scans": k, "ranks": G, "resamples": res[0],
            "comm_ms_per_scan": max(p["comm_ms"] for p in profs) / k,
            "comm_calls_per_scan": profs[0]["comm_calls"] / k,
            "scan_device_ms": max(p["scan_ms"] / max(p["scans"], 1) for p in profs),
            "scan_ms_each": [round(v, 3) for v in per],
            "bytes_sent_per_resample": sum(p["sent_bytes"] for p in profs) / max(res[0], 1),
            "particles_sent_per_resample": sum(p["sent_particles"] for p in profs) / max(res[0], 1),
            "page_dedup_ratio": (sum(p["sent_rows"] for p in profs) / sum(p["sent_pages"] for p in profs)
                                 if sum(p["sent_pages"] for p in profs) else None),
            "pages_sent_before_fraction": (sum(p["sent_pages_repeat"] for p in profs) /
                                           sum(p["sent_pages"] for p in profs)
                                           if sum(p["sent_pages"] for p in profs) else None),
            "recv_bytes_per_rank_scan_max": max(p["recv_bytes"] for p in profs) / k,
            "exchange_ms_per_scan_rank_max": max(p["exchange_ms"] for p in profs) / k,
            "page_refs": profs[0]["page_refs"] == 1,     # (in effect: fs2_profile.page_refs)
            # page_refs: remote pages the update passes copied (each with its 8 records)
            "localized_pages_per_scan": sum(p["localized_pages"] for p in profs) / k,
            "localized_bytes_per_scan": sum(p["localized_pages"] for p in profs) * (128 + 8 * 48) / k,
            "note": f"{G} ranks as threads on one GPU, in-process transport, {n_total} particles in all; "
                    "comm: host time in transport calls and mid-scan waits (a wait includes the collectives "
                    "queued before it)"}


def main(argv=None):
    argv = sys.argv[1:] if argv is None else list(argv)
    args = parse(argv)
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args, argv))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}; timing {world} ranks",
              file=sys.stderr, flush=True)
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.share_gpu:
        args.comm = "shm"
    dev = 0 if args.share_gpu else local
    import torch
    import torch.distributed as dist
    torch.cuda.set_device(dev)
    # the bench's own barrier and timing reduction: RCCL with one GPU per rank, gloo
    # when ranks share a GPU (RCCL refuses two ranks on one device)
    host_coll = args.share_gpu
    tdev = "cpu" if host_coll else "cuda"
    if world > 1:
        if host_coll:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    import fast_slam_2
    import fs2_synthetic as syn
    from fast_slam_2 import _native as nat

    cfg = dict(CONFIGS[args.config])
    if args.map == "dense":
        cfg["name"] += "_dense"          # (its own PMC record, profiles/pmc_<name>.json)
    n_per_gpu = args.particles or cfg["N"]
    L = args.landmarks or cfg["L"]
    comm_id = None
    if world > 1:
        obj = [(nat.comm_unique_id() if args.comm == "rccl" else os.urandom(128)) if rank == 0 else None]
        dist.broadcast_object_list(obj, src=0)
        comm_id = obj[0]

    def barrier():
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()

    R = run_config(args, cfg, n_per_gpu, L, world, rank, dev, comm_id, barrier, args.steps, args.warmup)
    f, dt, prof, st = R["handle"], R["dt"], R["prof"], R["st"]
    N = n_per_gpu * world
    if world > 1:
        tt = torch.tensor([dt], dtype=torch.float64, device=tdev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt = float(tt.item())
    migration = None
    if world > 1:
        # the sharded resample's transfers, summed over the ranks
        keys = ("migrations", "sent_particles", "sent_rows", "sent_pages", "sent_bytes", "migrate_ms", "comm_ms",
                "recv_bytes", "exchange_ms")
        mt = torch.tensor([float(prof[k]) for k in keys], dtype=torch.float64, device=tdev)
        mx = mt.clone()
        dist.all_reduce(mt, op=dist.ReduceOp.SUM)
        dist.all_reduce(mx, op=dist.ReduceOp.MAX)
        tot = dict(zip(keys, mt.tolist()))
        top = dict(zip(keys, mx.tolist()))
        resamples = R["sums"]["resamples"]
        per = max(resamples, 1)
        rs_ms = sorted(m for m, r in R["step_ms"] if r)
        ot_ms = sorted(m for m, r in R["step_ms"] if not r)
        migration = {
            "resamples": resamples,
            "particles_sent_per_resample": tot["sent_particles"] / per,
            "rows_sent_per_resample": tot["sent_rows"] / per,
            "pages_sent_per_resample": tot["sent_pages"] / per,
            "bytes_sent_per_resample": tot["sent_bytes"] / per,
            "page_dedup_ratio": tot["sent_rows"] / tot["sent_pages"] if tot["sent_pages"] else None,
            "host_ms_per_resample_rank_mean": tot["migrate_ms"] / world / per,
            "comm_ms_per_scan_rank_mean": tot["comm_ms"] / world / args.steps,
            # what must arrive before a rank's next update pass, and the device time the
            # exchanges hold the scan's stream (nothing overlaps them): per rank and scan,
            # the largest rank's
            "recv_bytes_per_rank_scan_max": top["recv_bytes"] / args.steps,
            "recv_bytes_per_rank_resample_max": top["recv_bytes"] / per,
            "exchange_ms_per_scan_rank_max": top["exchange_ms"] / args.steps,
            "exchange_ms_per_resample_rank_max": top["exchange_ms"] / per,
            "scan_ms_resample_median_rank0": rs_ms[len(rs_ms) // 2] if rs_ms else None,
            "scan_ms_other_median_rank0": ot_ms[len(ot_ms) // 2] if ot_ms else None,
            "note": "every resample moves the particles whose outputs land on another rank's shard, "
                    "each destination's distinct pages once; Q6/Q8 (sum of weights > 1) shift "
                    "outputs toward lower global indices, so the flow is mostly rank p -> p+1.."}

    if rank == 0:
        K = kernel_summary(prof, cfg, n_per_gpu, L)
        cpu = None
        if not args.no_cpu_baseline and world == 1:
            cpu = cpu_baseline(L, cfg["P"], args.cpu_seconds, args.seed)
        scan_ms = dt / args.steps * 1e3
        units = f.n_local * args.steps
        sums = R["sums"]
        # SURVEY §8(d)'s accounting: the reference layout's bytes (48 B per landmark
        # its first-match scan reads, 48 B per updated / appended landmark, 104 B of
        # particle scalars) at this run's scan rate -- a work rate, not a bandwidth
        ref_bytes = 48.0 * sums["ref_visits"] + 48.0 * sums["hits_appends"] + 104.0 * units
        out = {
            "metric": "particle-updates/s",
            "value": N * args.steps / dt,
            "unit": "particle-updates/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": scan_ms,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (SURVEY.md §8d: 6 m landmark grid, 3 hits + 1 miss per scan, "
                    "odometry 4x0.03 m then 0.05 rad; device Philox motion noise)",
            "config": {"workload": cfg["name"], "particles_per_gpu": n_per_gpu,
                       "particles_total": N, "landmarks": L, "beams": cfg["P"],
                       "measurements_per_scan": 4, "icp": cfg["icp"],
                       "icp_pipelined": bool(cfg["icp"] and not args.serial_icp),
                       "gate_filter": not args.no_gate_filter, "reduce": "exact" if N > 4096 and world == 1
                       else ("parallel" if world > 1 else "sequential"),
                       "parallelism": f"particle-shard{world}",
                       "scans_in_flight": 2 if R["pipelined"] else 1,
                       "transport": args.comm if world > 1 else None,
                       "ranks_share_gpu": bool(args.share_gpu and world > 1)},
            "roofline": K["roofline"],
            "cpu_baseline": cpu,
            "extra": {"scan_device_ms": prof["scan_ms"] / max(prof["scans"], 1),
                      "update_pass_ms": K["update_pass_ms"],
                      "kernels": K["kernels"],
                      "byte_model": K["byte_model"],
                      "reference_equivalent": {
                          "bytes_per_scan": ref_bytes / args.steps,
                          "work_rate_GBs": ref_bytes / dt / 1e9,
                          "landmark_reads_per_particle_scan": sums["ref_visits"] / units,
                          "note": "SURVEY §8d bytes of the reference's layout and linear scan at this "
                                  "run's scan rate; not a bandwidth (pruning and page sharing skip them)"},
                      "update_pass_bytes": prof["update_bytes"] / max(prof["update_launches"], 1),
                      "reduce_and_resample_ms": prof["reduce_ms"] / max(prof["scans"], 1),
                      "resamples": sums["resamples"],
                      # host wall time per scan by kind (the drop-in line reports the same split)
                      "scan_ms_by_kind": {
                          "resampling_mean": (float(np.mean([m for m, r in R["step_ms"] if r]))
                                              if any(r for _, r in R["step_ms"]) else None),
                          "other_mean": (float(np.mean([m for m, r in R["step_ms"] if not r]))
                                         if any(not r for _, r in R["step_ms"]) else None)},
                      "resample_shared_slots": sums["copied_slots"],
                      "cow_pages_per_particle_scan": sums["cow"] / units,
                      "pool_collections": st.collections,
                      "pool_collections_timed": st.collections - R["coll0"],
                      "pool_pages": st.pool_pages,
                      "pages_opened_per_particle_scan": sums["opened"] / units,
                      "slots_visited_per_particle_scan": sums["visited"] / units,
                      "exact_slots_per_particle_scan": sums["exact"] / units,
                      "icp_us": R["icp_us"],
                      "icp_host_ms_per_scan": R["icp_host"]},
        }
        if migration is not None:
            out["extra"]["migration"] = migration
        extras = not args.no_extras and world == 1
        if extras and not cfg["icp"]:
            out["extra"]["robustness"] = robustness(args, f, L, args.warmup + args.steps)
        f.close()
        if extras and args.config == "3" and not (args.particles or args.landmarks):
            # the other single-GPU BASELINE configs, each on a fresh handle
            out["extra"]["configs"] = {k: config_line(args, k, world, rank, dev, barrier) for k in ("2", "4")}
        print(json.dumps(out), flush=True)
    else:
        f.close()
    if world > 1:
        dist.destroy_process_group()


def run_config(args, cfg, n_per_gpu, L, world, rank, dev, comm_id, barrier, steps, warmup):
    """Create and populate a handle for one workload, run `warmup` untimed and
    `steps` timed scans (config 4: each scan's odometry from the ICP alignment of
    the next scan pair, run beside the previous scan's update); returns the
    handle, the timed wall time and the per-scan sums."""
    import torch
    import fast_slam_2
    import fs2_synthetic as syn
    N = n_per_gpu * world
    total_scans = warmup + steps
    f = fast_slam_2.FastSLAM2(N, device=dev, rng="device", seed=args.seed, reduce="auto",
                              landmark_capacity=L + total_scans + 8, rank=rank,
                              world_size=world, comm_id=comm_id, verbose=False,
                              gate_filter=not args.no_gate_filter, comm_mode=args.comm)
    dense = dense_workload(L, args.seed) if args.map == "dense" else None
    populate(f, f.n_local, L, args.seed, rank, base_map=None if dense is None else dense[0])
    scans_pts = None
    fast_slam_2.ICP.device = dev
    if cfg["icp"]:
        scans_pts = [syn.room_scan((0.03 * s, 0.0, 0.0), cfg["P"], args.seed, s)
                     for s in range(total_scans + 1)]

    # the scans' measurements are inputs (the front-end's output), made before timing
    meas = [np.ascontiguousarray(syn.scan_measurements(L, s, args.seed) if dense is None else dense[1](s),
                                 dtype=np.float64)
            for s in range(total_scans)]

    # ICP of scan s+1 runs beside scan s's filter update: the scan is enqueued
    # (step_submit: fs2_iterate_submit), then this thread hands the next alignment
    # to the ICP stream, waits for it and turns it into odometry
    # (Robot.get_transformation_icp, robot.py:108-120) while the GPU runs the scan,
    # then completes the scan (step_wait).  The hand-off's host time (~0.1 ms of HIP
    # calls, event wait, numpy) stays off the GPU's critical path.  The timed
    # region's first scan prepares its own alignment, so exactly one alignment per
    # timed scan runs inside the timing.
    icp_odo = {}
    icp_host = {"wait_ms": 0.0, "prep_ms": 0.0, "scans": 0}

    def icp_prepare(s):
        """Odometry of scan s from the alignment of scans s -> s+1 (and its host time)."""
        t0 = time.perf_counter()
        Rm, t, _ = fast_slam_2.ICP.submit(scans_pts[s], scans_pts[s + 1]).result()
        # the commanded linear velocity is nonzero on the driving scans of the pattern
        v = 0.3 if syn.odometry(s)[1] != 0 else 0.0
        rot, tr = (float(q) for q in fast_slam_2.Robot.icp_odometry(Rm, t, v))
        return rot, tr, (time.perf_counter() - t0) * 1e3

    offline_odo = ({s: icp_prepare(s)[:2] for s in range(total_scans)}
                   if (scans_pts is not None and args.icp_offline) else None)
    side = torch.cuda.Stream() if args.probe_side_kernels else None
    side_x = torch.zeros(64, device="cuda") if side is not None else None

    def one_scan(s):
        rot, tr = syn.odometry(s)
        if side is not None:
            with torch.cuda.stream(side):
                for _ in range(args.probe_side_kernels):
                    side_x.add_(1.0)
        if scans_pts is None:
            return f.step(rot, tr, meas[s])
        if args.icp_offline:
            return f.step(*offline_odo[s], meas[s])
        t0 = time.perf_counter()
        ready = icp_odo.pop(s, None)
        rot, tr, prep = ready if ready is not None else icp_prepare(s)
        t1 = time.perf_counter()
        f.step_submit(rot, tr, meas[s])
        nxt = None
        if s + 1 != warmup and s + 1 < total_scans and not args.serial_icp:
            nxt = icp_prepare(s + 1)
            icp_odo[s + 1] = nxt
        out = f.step_wait()
        if s >= warmup:
            icp_host["wait_ms"] += (t1 - t0) * 1e3       # alignment work before this scan could start
            icp_host["prep_ms"] += nxt[2] if nxt is not None else prep
            icp_host["scans"] += 1
        return out

    coll0 = 0
    for s in range(warmup):
        _, st0 = one_scan(s)
        coll0 = st0.collections
    # kernel events on every 4th timed scan: a dispatch's start / end events delay
    # the next dispatch by ~4.5 us, which the other scans do not pay
    if args.profile_every > 0:
        f.set_profiling(True, every=args.profile_every)
    sums = dict(resamples=0, visited=0, copied_slots=0, cow=0, exact=0, opened=0, ref_visits=0, hits_appends=0)
    step_ms = []                 # (host ms, resampled) of each timed scan on this rank
    def account(st):
        sums["resamples"] += st.resampled
        sums["visited"] += st.slots_visited
        sums["copied_slots"] += st.resample_slots
        sums["cow"] += st.cow_pages
        sums["exact"] += st.candidates
        sums["opened"] += st.pages_opened
        sums["ref_visits"] += st.reference_visits
        sums["hits_appends"] += st.hits + st.appends

    # two scans in flight (one GPU, no ICP hand-off): scan s+1 is submitted before
    # scan s is waited for, so its candidate pass runs beside scan s's tail
    # (fs2_iterate_submit); the results are the same bits as step()'s
    pipelined = scans_pts is None and world == 1 and args.pipelined
    barrier()
    t0 = time.perf_counter()
    if pipelined:
        t1 = t0
        for s in range(warmup, total_scans):
            f.step_submit(*syn.odometry(s), meas[s])
            if s > warmup:
                _, st = f.step_wait()
                step_ms.append(((time.perf_counter() - t1) * 1e3, st.resampled))
                t1 = time.perf_counter()
                account(st)
        _, st = f.step_wait()
        step_ms.append(((time.perf_counter() - t1) * 1e3, st.resampled))
        account(st)
    else:
        for s in range(warmup, total_scans):
            t1 = time.perf_counter()
            _, st = one_scan(s)
            step_ms.append(((time.perf_counter() - t1) * 1e3, st.resampled))
            account(st)
    barrier()
    dt = time.perf_counter() - t0
    prof = f.profile()
    icp_us = None
    if scans_pts is not None:
        # one alignment through the synchronous call, warm (its stream and scratch
        # are first touched here; the timed loop used ICP.submit)
        fast_slam_2.ICP.get_transformation(scans_pts[0], scans_pts[1])
        t1 = time.perf_counter()
        for s in range(5):
            fast_slam_2.ICP.get_transformation(scans_pts[s], scans_pts[s + 1])
        icp_us = (time.perf_counter() - t1) / 5 * 1e6
    host = ({"before_scan": icp_host["wait_ms"] / max(icp_host["scans"], 1),
             "hand_off": icp_host["prep_ms"] / max(icp_host["scans"], 1),
             "note": "hand_off: submission + alignment + odometry of the next scan, done between "
                     "step_submit and step_wait; before_scan: alignment work ahead of a scan's submission"}
            if scans_pts is not None else None)
    return {"handle": f, "dt": dt, "prof": prof, "st": st, "coll0": coll0, "sums": sums, "step_ms": step_ms,
            "icp_us": icp_us, "icp_host": host, "pipelined": pipelined}


# Algorithmic byte model of the two update kernels (include/fs2.h
# fs2_profile): bytes per unit the counters count
BYTE_MODEL = {
    "k_candidates": {"descriptor_streamed": 4, "page_opened": 128, "list_entry": 8,
                     "particle_pass (cnt read, count write)": 8, "row_box_read": 4},
    "k_update": {"fixed (scalars, free-list ids, counts; per particle, summed)": 1, "list_entry": 8,
                 "candidate_record": 48, "slot_written (record 48, mirror 16, descriptor read 4)": 68,
                 "page_copied (128 read + 128 write, descriptor write 4)": 260, "row_box_read_and_written": 8},
}


def kernel_summary(prof, cfg, n_per_gpu, L):
    """Per-kernel times (HIP events of the dispatches), the algorithmic byte model
    evaluated from the profile's counters, the PMC HBM bytes of this build when a
    record exists, and the roofline line of the dominant kernel on both bases."""
    launches = max(prof["update_launches"], 1)
    upd_ms = prof["update_ms"] / launches
    kern = {}
    fl = prof["filter_launches"]
    if fl > 0:
        kern["k_candidates"] = (prof["filter_ms"] / fl, prof["filter_bytes"] / fl)
        kern["k_update"] = (prof["exact_ms"] / max(prof["exact_launches"], 1),
                            (prof["update_bytes"] - prof["filter_bytes"]) / fl)
    else:
        kern["k_update"] = (upd_ms, prof["update_bytes"] / launches)
    pmc = pmc_record(cfg["name"]) if n_per_gpu == cfg["N"] and L == cfg["L"] else None
    model = None
    if fl > 0:
        c = {k: prof[f"model_{k}"] / fl for k in ("groups", "opened", "words", "candidates", "written", "cow",
                                                  "fixed_bytes", "box_bytes")}
        model = {"units": BYTE_MODEL, "counts_per_launch": c,
                 "k_candidates_bytes": kern["k_candidates"][1], "k_update_bytes": kern["k_update"][1],
                 "note": "k_candidates = 4 groups + 128 opened + 8 words + 8 n + 4/12 box_bytes; "
                         "k_update = fixed_bytes + 8 words + 48 candidates + 68 written + 260 cow + 8/12 box_bytes; "
                         "reuse = model bytes / PMC HBM bytes (> 1: L2 / MALL hits, e.g. siblings' shared pages)"}
        for k in ("k_candidates", "k_update"):
            t = pmc_traffic(pmc, k)
            model[f"{k}_reuse_vs_pmc"] = (kern[k][1] / t) if t else None
    kernels = {}
    for k, v in kern.items():
        t = pmc_traffic(pmc, k)
        kernels[k] = {"ms_per_launch": v[0], "algorithmic_bytes_per_launch": v[1],
                      "algorithmic_GBs": v[1] / (v[0] * 1e-3) / 1e9 if v[0] > 0 else 0.0,
                      "hbm_bytes_per_launch": t,
                      "hbm_GBs": (t / (v[0] * 1e-3) / 1e9 if t and v[0] > 0 else None)}
    # the roofline line is for the dominant (longest) kernel: HBM bytes per launch
    # from the PMC passes on this build (profiles/pmc_<workload>.json), over the
    # launch's live duration (HIP events on the library's stream, this run)
    kernel = max(kern, key=lambda k: kern[k][0])
    ms_launch, alg_bytes = kern[kernel]
    traffic = pmc_traffic(pmc, kernel)
    alg_GBs = alg_bytes / (ms_launch * 1e-3) / 1e9 if ms_launch > 0 else 0.0
    if traffic is not None and ms_launch > 0:
        achieved, basis = traffic / (ms_launch * 1e-3) / 1e9, "pmc_hbm_bytes"
    else:
        achieved, basis = alg_GBs, "algorithmic_bytes (no PMC record for this build)"
    roof = {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "basis": basis,
            "kernel": kernel, "ms_per_launch": ms_launch,
            "pmc_source": None if pmc is None else pmc.get("source"),
            "algorithmic_bytes_per_launch": alg_bytes, "algorithmic_GBs": alg_GBs,
            "frac_algorithmic": alg_GBs / HBM_PEAK_GBS}
    return {"roofline": roof, "kernels": kernels, "byte_model": model, "update_pass_ms": upd_ms}


def config_line(args, key, world, rank, dev, barrier, steps=20, warmup=3):
    """BASELINE config `key` (2: 1e5 x 200; 4: 1e6 x 500 with the 720-beam ICP
    beside each update) on a fresh handle: ms per scan, value, the dominant
    kernel's event time and roofline (PMC basis when this build has a record)."""
    cfg = dict(CONFIGS[key])
    R = run_config(args, cfg, cfg["N"], cfg["L"], 1, 0, dev, None, barrier, steps, warmup)
    R["handle"].close()
    K = kernel_summary(R["prof"], cfg, cfg["N"], cfg["L"])
    sums = R["sums"]
    units = cfg["N"] * steps
    return {"workload": cfg["name"], "value": cfg["N"] * steps / R["dt"], "ms_per_scan": R["dt"] / steps * 1e3,
            "steps": steps, "warmup": warmup, "roofline": K["roofline"], "kernels": K["kernels"],
            "reduce_and_resample_ms": R["prof"]["reduce_ms"] / max(R["prof"]["scans"], 1),
            "resamples": sums["resamples"], "pages_opened_per_particle_scan": sums["opened"] / units,
            "cow_pages_per_particle_scan": sums["cow"] / units, "icp_us": R["icp_us"],
            "icp_host_ms_per_scan": R["icp_host"], "scans_in_flight": 2 if R["pipelined"] else 1}

if __name__ == "__main__":
    main()
