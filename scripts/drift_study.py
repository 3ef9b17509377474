#!/usr/bin/env python3
"""Where the config-5 migration comes from, and what shard policy minimises it
(VERDICT r05 "do this" #1; reference fast_slam_2.py:177-199).

Systematic resampling keeps the global particle order, so a run's whole
resampling history is the sequence of out_src arrays of one GPU (output m ->
global source), and every sharded run of the same stream resamples identically
(exact-order reductions span the shards).  So the migration any shard
policy would cause at G ranks can be replayed offline from one GPU's history:

  dump  (GPU)  run the bench's synthetic stream on one handle of N particles and
               save every resample's out_src (fs2_debug_out_src) to an .npz;
  sim   (CPU)  replay the history at G ranks under the policies
                 pinned   shard q on rank q, equal shards (round 2)
                 follow   equal shards, each rank takes the shard its sources
                          fill most (round 3, today's default; keep_shards)
                 movable  contiguous shards of any length <= cap * N / G, cut and
                          assigned to keep the most outputs local (fs2_shard.hpp
                          plan_movable, the same DP libfs2 runs);
               and print, per resample, the outputs and the distinct sources that
               change ranks and the largest shard.

  python scripts/drift_study.py dump --particles 1000000 --landmarks 500 --scans 30 --out gpurun_out/drift.npz
  python scripts/drift_study.py sim gpurun_out/drift.npz --ranks 8 --cap 1.15
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "fast-slam_amd"))
sys.path.insert(0, REPO)


def dump(args):
    import torch
    import bench
    import fast_slam_2
    import fs2_synthetic as syn
    from fast_slam_2 import _native as nat
    torch.cuda.set_device(0)
    N, L = args.particles, args.landmarks
    if args.guard:
        os.environ["FS2_GUARD"] = "1"       # buffers followed by a checked pattern (fs2_debug_check_guards)
    f = fast_slam_2.FastSLAM2(N, rng="device", seed=args.seed, landmark_capacity=L + args.scans + 8, verbose=False)
    os.environ.pop("FS2_GUARD", None)
    t0 = time.time()
    bench.populate(f, N, L, args.seed, 0)
    print(f"populated N={N} L={L} in {time.time() - t0:.1f} s", flush=True)
    lib = nat.load()
    buf = np.empty(N, dtype=np.int32)
    diffs, scans, sums = [], [], []
    for s in range(args.scans):
        meas = np.ascontiguousarray(syn.scan_measurements(L, s, args.seed), dtype=np.float64)
        _, st = f.step(*syn.odometry(s), meas)
        if st.resampled:
            n = lib.fs2_debug_out_src(f._h, buf.ctypes.data, N)
            if n != N:
                raise RuntimeError(f"fs2_debug_out_src returned {n}")
            assert buf[0] >= 0 and np.all(np.diff(buf) >= 0), "out_src must be non-decreasing"
            diffs.append(np.diff(buf, prepend=0).astype(np.int32))
            scans.append(s)
            sums.append(float(st.n_eff))
        if args.guard:
            name = C.create_string_buffer(128)
            bad = lib.fs2_debug_check_guards(f._h, name, 128)
            if bad:
                raise RuntimeError(f"scan {s}: {bad} guard bytes overwritten after {name.value.decode()}")
        print(f"scan {s}: resampled {int(st.resampled)} n_eff {st.n_eff:.1f}", flush=True)
    f.close()
    np.savez_compressed(args.out, N=N, L=L, seed=args.seed, scans=np.array(scans),
                        n_eff=np.array(sums), diffs=np.stack(diffs) if diffs else np.zeros((0, N), np.int32))
    print(f"wrote {args.out}: {len(scans)} resamples", flush=True)


# ---------------------------------------------------------------- simulation --

def natural(src, starts, order):
    """Natural output interval of each position: outputs whose source lies in the
    position's interval [starts[q], starts[q+1]).  Returns lo[q], hi[q] (outputs)."""
    lo = np.searchsorted(src, starts[:-1], side="left")
    hi = np.searchsorted(src, starts[1:], side="left")
    return lo, hi


def moved(src, starts, new_starts, new_order, order):
    """Outputs and distinct (source, destination) pairs that change ranks: output m
    is held at the resample by the rank holding its source; afterwards by the rank
    whose new interval contains m."""
    N = len(src)
    pos_src = np.searchsorted(starts, src, side="right") - 1          # position of the source
    rank_src = np.asarray(order)[pos_src]
    m = np.arange(N)
    pos_new = np.searchsorted(new_starts, m, side="right") - 1
    rank_new = np.asarray(new_order)[pos_new]
    mv = rank_src != rank_new
    outs = int(mv.sum())
    # distinct sources sent, per destination (a source whose outputs go to two ranks counts twice)
    pairs = np.unique(src[mv].astype(np.int64) * 64 + rank_new[mv]) if outs else np.zeros(0)
    recv = np.bincount(rank_new[mv], minlength=len(order)) if outs else np.zeros(len(order), int)
    return outs, len(pairs), recv


def equal_starts(N, G):
    return np.array([N * q // G for q in range(G + 1)], dtype=np.int64)


def follow(src, starts, order, N, G):
    """Round 3's keep_shards: equal shards, the assignment of shards to ranks that
    keeps the most outputs local (exact, DP over subsets)."""
    lo, hi = natural(src, starts, order)
    eq = equal_starts(N, G)
    rank_pos = {r: q for q, r in enumerate(order)}
    keep = np.zeros((G, G), dtype=np.int64)                 # keep[rank][shard]
    for r in range(G):
        q = rank_pos[r]
        for p in range(G):
            keep[r, p] = max(0, min(hi[q], eq[p + 1]) - max(lo[q], eq[p]))
    full = (1 << G) - 1
    dp = np.full(full + 1, -1, dtype=np.int64)
    pick = np.zeros(full + 1, dtype=np.int64)
    dp[0] = 0
    for msk in range(full):
        if dp[msk] < 0:
            continue
        r = bin(msk).count("1")
        for p in range(G):
            if msk >> p & 1:
                continue
            v = dp[msk] + 2 * keep[r, p] + (1 if p == rank_pos[r] else 0)
            if v > dp[msk | 1 << p]:
                dp[msk | 1 << p] = v
                pick[msk | 1 << p] = p
    owner = [0] * G
    msk = full
    while msk:
        p = int(pick[msk])
        owner[p] = bin(msk).count("1") - 1
        msk &= ~(1 << p)
    return eq, owner


def movable(src, starts, order, N, G, cap, units_per_shard=64):
    """Movable boundaries (the DP of fs2_shard.hpp, restated in numpy): positions are
    cut on a grid of U = G * units_per_shard units; ranks whose sources have outputs
    ("busy") keep their order, ranks without ("free") may go anywhere; every
    interval holds at most cap * N / G outputs; maximise the outputs kept local."""
    lo, hi = natural(src, starts, order)
    U = G * units_per_shard
    edge = np.array([N * k // U for k in range(U + 1)], dtype=np.int64)
    capu = int(np.floor(cap * units_per_shard + 1e-9))
    busy = [q for q in range(G) if hi[q] > lo[q]]
    free = [q for q in range(G) if hi[q] <= lo[q]]
    k, F = len(busy), len(free)
    NEG = -1 << 60
    # best[j][f][u]: outputs kept with j busy and f free positions placed, boundary at unit u
    best = np.full((k + 1, F + 1, U + 1), NEG, dtype=np.int64)
    arg = np.zeros((k + 1, F + 1, U + 1, 3), dtype=np.int64)     # (prev j, prev f, prev u)
    best[0, 0, 0] = 0
    for j in range(k + 1):
        for f in range(F + 1):
            row = best[j, f]
            for u in np.nonzero(row > NEG)[0]:
                base = row[u]
                vmax = min(U, u + capu)
                vs = np.arange(u, vmax + 1)
                if j < k:
                    q = busy[j]
                    gain = np.maximum(0, np.minimum(hi[q], edge[vs]) - np.maximum(lo[q], edge[u]))
                    cand = base + gain
                    tgt = best[j + 1, f]
                    upd = cand > tgt[vs]
                    tgt[vs[upd]] = cand[upd]
                    arg[j + 1, f, vs[upd]] = (j, f, u)
                if f < F:
                    vs2 = vs[1:]
                    tgt = best[j, f + 1]
                    upd = base > tgt[vs2]
                    tgt[vs2[upd]] = base
                    arg[j, f + 1, vs2[upd]] = (j, f, u)
    fbest = max(range(F + 1), key=lambda f: best[k, f, U])
    assert best[k, fbest, U] > NEG, "infeasible cap"
    # walk back: the sequence of (position kind, end unit)
    seq = []
    j, f, u = k, fbest, U
    while (j, f, u) != (0, 0, 0):
        pj, pf, pu = arg[j, f, u]
        seq.append(("busy", busy[pj]) if pj != j else ("free", free[pf]))
        seq[-1] = seq[-1] + (pu, u)
        j, f, u = pj, pf, pu
    seq.reverse()
    new_order, cuts = [], [0]
    for kind, q, pu, u in seq:
        new_order.append(order[q])
        cuts.append(int(edge[u]))
    for q in free[fbest:]:                       # unused free ranks: empty intervals at the end
        new_order.append(order[q])
        cuts.append(N)
    return np.array(cuts, dtype=np.int64), new_order


def sim(args):
    d = np.load(args.npz)
    N = int(d["N"])
    src_all = np.cumsum(d["diffs"], axis=1)
    G = args.ranks
    out = {"N": N, "L": int(d["L"]), "G": G, "cap": args.cap, "resamples": int(len(src_all)),
           "scans": d["scans"].tolist(), "policies": {}}
    # the least any balanced placement must move: rank r's sources have c_r outputs,
    # at most cap * N / G of them can stay (contiguous shards or not)
    starts, order = equal_starts(N, G), list(range(G))
    forced = []
    for src in src_all:
        lo, hi = natural(src, starts, order)
        forced.append(int(np.maximum(0, (hi - lo) - int(args.cap * N / G)).sum()))
        starts, order = movable(src, starts, order, N, G, args.cap)
    out["forced_outputs_frac_mean"] = float(np.mean(forced)) / N if forced else 0.0
    print(f"lower bound (movable placements, cap {args.cap}): {out['forced_outputs_frac_mean'] * 100:.2f} % of N "
          f"per resample must change ranks", flush=True)
    for pol in ("pinned", "follow", "movable"):
        starts = equal_starts(N, G)
        order = list(range(G))
        rows = []
        for src in src_all:
            if pol == "pinned":
                ns, no = equal_starts(N, G), list(range(G))
            elif pol == "follow":
                ns, no = follow(src, starts, order, N, G)
            else:
                ns, no = movable(src, starts, order, N, G, args.cap)
            outs, pairs, recv = moved(src, starts, ns, no, order)
            sizes = np.diff(ns)
            rows.append({"outputs_moved": outs, "sources_sent": pairs, "max_recv": int(recv.max()),
                         "max_shard": int(sizes.max()), "empty_ranks": int((sizes == 0).sum())})
            starts, order = ns, no
        tot = sum(r["outputs_moved"] for r in rows)
        out["policies"][pol] = {
            "per_resample": rows,
            "outputs_moved_frac_mean": tot / (N * max(len(rows), 1)),
            "sources_sent_mean": float(np.mean([r["sources_sent"] for r in rows])) if rows else 0.0,
            "max_recv_per_rank_mean": float(np.mean([r["max_recv"] for r in rows])) if rows else 0.0,
            "max_shard_over_fair": max((r["max_shard"] for r in rows), default=0) / (N / G),
        }
        p = out["policies"][pol]
        print(f"{pol:8s} G={G}: outputs moved {p['outputs_moved_frac_mean'] * 100:6.2f} % of N per resample, "
              f"sources sent {p['sources_sent_mean']:.0f}, worst receiver {p['max_recv_per_rank_mean']:.0f} outputs, "
              f"largest shard {p['max_shard_over_fair']:.3f} x N/G", flush=True)
        for s, r in zip(out["scans"], rows):
            print(f"    scan {s:3d}: moved {r['outputs_moved']:9d}  sources {r['sources_sent']:9d}  "
                  f"max recv {r['max_recv']:9d}  max shard {r['max_shard']:9d}  empty {r['empty_ranks']}")
    if args.json:
        with open(args.json, "w") as fh:
            json.dump(out, fh, indent=1)


def main():
    ap = argparse.ArgumentParser()
    sub = ap.add_subparsers(dest="cmd", required=True)
    a = sub.add_parser("dump")
    a.add_argument("--particles", type=int, default=1_000_000)
    a.add_argument("--landmarks", type=int, default=500)
    a.add_argument("--scans", type=int, default=30)
    a.add_argument("--seed", type=int, default=0)
    a.add_argument("--out", required=True)
    a.add_argument("--guard", action="store_true", help="FS2_GUARD: check every buffer's end after each scan")
    b = sub.add_parser("sim")
    b.add_argument("npz")
    b.add_argument("--ranks", type=int, default=8)
    b.add_argument("--cap", type=float, default=1.15)
    b.add_argument("--json")
    args = ap.parse_args()
    dump(args) if args.cmd == "dump" else sim(args)


if __name__ == "__main__":
    main()
