#!/usr/bin/env python3
"""Pages the candidate stream opens per particle and scan on the config-3 map
(500 landmarks on a 6 m grid, pages of 8 consecutive landmarks),
under different page summaries; CPU only, numpy.

  python3 scripts/page_open_sim.py
box       the 8-bit-code box on the 1 m summary grid with the measurement bands
          (what k_candidates does)
box_fine  the same box on a 1/8 m grid
half      two boxes per page (slots 0-3, 4-7)
exact     pages holding a slot within the gate radius (the floor)
"""
import math
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "fast-slam_amd"))
import fs2_synthetic as syn  # noqa: E402


def box_open(sl, fx, fy, R, cell, org=-127.0):
    xlo = org + np.floor((sl[:, 0].min() - org) / cell) * cell
    xhi = org + np.ceil((sl[:, 0].max() - org) / cell) * cell
    ylo = org + np.floor((sl[:, 1].min() - org) / cell) * cell
    yhi = org + np.ceil((sl[:, 1].max() - org) / cell) * cell
    return not (xlo >= fx + R or xhi <= fx - R or ylo >= fy + R or yhi <= fy - R)


def main(N=200, L=500, scans=10):
    base = syn.common_landmarks(L, 0)
    rng = np.random.default_rng(5)
    maps = base[None] + rng.normal(0, syn.MAP_JITTER, (N, L, 2))
    R = math.sqrt(64 / 10)           # gate 8, covariance 0.1 I -> s = 10
    meas = []
    for s in range(scans):
        ms = syn.scan_measurements(L, s, 0)
        meas.append(np.stack([ms[:, 0] * np.cos(ms[:, 1]), ms[:, 0] * np.sin(ms[:, 1])], 1))
    tot = dict(box=0, box_fine=0, half=0, exact=0)
    for p in range(N):
        m = maps[p]
        for pts in meas:
            for fx, fy in pts:
                for pg in range(0, L, 8):
                    sl = m[pg:pg + 8]
                    tot["box"] += box_open(sl, fx, fy, R, 1.0)
                    tot["box_fine"] += box_open(sl, fx, fy, R, 0.125)
                    tot["half"] += box_open(sl[:4], fx, fy, R, 1.0) or (len(sl) > 4 and box_open(sl[4:], fx, fy, R, 1.0))
                    tot["exact"] += bool((((sl[:, 0] - fx) ** 2 + (sl[:, 1] - fy) ** 2) < R * R).any())
    for k, v in tot.items():
        print(f"{k:9s} {v / (N * scans):6.2f} pages per particle and scan")


if __name__ == "__main__":
    main()
