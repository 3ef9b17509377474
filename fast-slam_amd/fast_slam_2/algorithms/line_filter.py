"""LineFilter on the GPU (reference: fast_slam_2/algorithms/line_filter.py:12-21).

Per-column Gaussian smoothing equal to scipy.ndimage.gaussian_filter1d
(mode='reflect', truncate=4).  The taps are built on the host with numpy
exactly as scipy builds them; the correlation runs in libfs2.  At the default
sigma = 0.1 the kernel has one tap of 1.0 and the filter is an identity
(SURVEY.md Q13).
"""
from __future__ import annotations

import numpy as np

from .. import _native as nat


def gaussian_taps(sigma: float, truncate: float = 4.0):
    """scipy.ndimage._gaussian_kernel1d(sigma, 0, radius)[::-1] and its radius."""
    sd = float(sigma)
    radius = int(truncate * sd + 0.5)
    x = np.arange(-radius, radius + 1)
    phi = np.exp(-0.5 / (sigma * sigma) * x ** 2)
    phi = phi / phi.sum()
    return np.ascontiguousarray(phi[::-1]), radius


class LineFilter:
    device = 0

    @staticmethod
    def filter(points: np.ndarray, sigma=0.1):
        pts = nat.f64(points, (-1, 2))
        taps, r = gaussian_taps(sigma)
        out = np.empty_like(pts)
        nat.check(nat.load().fs2_line_filter(LineFilter.device, nat.dptr(pts), len(pts),
                                             nat.dptr(taps), r, nat.dptr(out)))
        return out
