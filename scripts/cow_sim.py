"""How many of k_update's copy-on-write page copies a sharer count could save, on
the bench's workload shape (CPU model, numpy).

Model: N particles, each map a row of R pages; every scan each particle writes W
slots on distinct random pages of its row, then the particles are resampled
systematically (fast_slam_2.py:177-199) from lognormal weights whose N_eff / N is
about `neff` (the headline resamples every scan).  Three ownership rules for a
write to a page:
  bit     libfs2 today: a row entry is owned (written in place) only when its
          particle made the page and every resample since kept it with a source of
          exactly one output; otherwise the write copies the page;
  owned   + a count on the pages a source owned when it was resampled (the k
          outputs share them; a copying output decrements; the output that sees 1
          takes the page in place) -- VERDICT r04's proposal restricted to what
          the gather knows;
  exact   every page's reference count kept exactly (a resample adds the
          outputs' references and drops the dead sources'); a write copies only
          while another reference exists.
Prints copies per particle and scan under each rule, and the reference-count
updates the exact rule needs per resample.

    python scripts/cow_sim.py [--n 20000] [--rows 63] [--writes 3] [--scans 40]
"""
import argparse

import numpy as np


def systematic(w, rng):
    n = len(w)
    c = np.cumsum(w / w.sum())
    u = (rng.random() + np.arange(n)) / n
    return np.minimum(np.searchsorted(c, u), n - 1)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=20000)
    ap.add_argument("--rows", type=int, default=63)
    ap.add_argument("--writes", type=int, default=3)
    ap.add_argument("--scans", type=int, default=30)
    ap.add_argument("--warm", type=int, default=10)
    ap.add_argument("--neff", type=float, default=0.45)
    ap.add_argument("--seed", type=int, default=0)
    a = ap.parse_args()
    rng = np.random.default_rng(a.seed)
    N, R, W = a.n, a.rows, a.writes
    sig = np.sqrt(-np.log(a.neff))          # lognormal: N_eff / N = exp(-sigma^2)
    out = {}
    for rule in ("bit", "owned", "exact"):
        rng = np.random.default_rng(a.seed)
        rows = np.arange(N * R, dtype=np.int64).reshape(N, R)     # fresh, all owned
        nxt = N * R
        ref = np.ones(N * R + a.scans * N * W + 1, dtype=np.int32)  # exact counts (by page id)
        own = np.ones((N, R), dtype=bool)                        # bit rule
        cnt = {}                                                 # owned rule: page -> sharers
        copies, updates, scans = 0, 0, 0
        for s in range(a.scans):
            timed = s >= a.warm
            for i in range(N):
                for r in rng.choice(R, W, replace=False):
                    p = rows[i, r]
                    if rule == "bit":
                        inplace = own[i, r]
                    elif rule == "owned":
                        inplace = own[i, r]
                        if not inplace and p in cnt:
                            if cnt[p] == 1:          # the last sharer: in place
                                inplace = True
                                del cnt[p]
                            else:
                                cnt[p] -= 1
                    else:
                        inplace = ref[p] == 1
                    if inplace:
                        own[i, r] = True
                    else:
                        if rule == "exact":
                            ref[p] -= 1
                        rows[i, r] = nxt
                        ref[nxt] = 1
                        nxt += 1
                        own[i, r] = True
                        copies += timed
            scans += timed
            w = rng.lognormal(0.0, sig, N)
            src = systematic(w, rng)
            k = np.bincount(src, minlength=N)
            if rule == "exact":
                # every output row references its source's pages; dead sources drop theirs
                d = (k - 1)[:, None] * np.ones((1, R), dtype=np.int64)
                np.add.at(ref, rows.ravel(), d.ravel().astype(np.int32))
                if timed:
                    updates += int(np.count_nonzero(k != 1)) * R
            if rule == "owned":
                # pages a source owned now have k sharers (the first k - 1 writers copy)
                cnt = {}
                for i in np.flatnonzero(k >= 2):
                    for r in np.flatnonzero(own[i]):
                        cnt[rows[i, r]] = int(k[i])
            keep = (k[src] == 1)[:, None]
            rows = rows[src]
            own = own[src] & keep
        out[rule] = copies / (scans * N)
        if rule == "exact":
            out["exact_count_updates_per_resample_per_particle"] = updates / (scans * N)
    print({k: round(v, 4) for k, v in out.items()})
    b = out["bit"]
    print(f"copies saved vs bit: owned {1 - out['owned'] / b:.1%}, exact {1 - out['exact'] / b:.1%}")


if __name__ == "__main__":
    main()
