"""HoughTransformation on the GPU (reference: fast_slam_2/algorithms/hough_transformation.py).

The reference draws the points (x100, padding 20) into a uint8 image with
cv2.circle(radius 2, filled), runs cv2.HoughLines(img, 1, pi/180, 80),
intersects every pair of lines at least 45 degrees apart in numpy float32
arithmetic and converts the intersections back to metres.  libfs2 does all of
it on the device (fs2_frontend.hip): the image is a per-scan bitmap of lit
pixels, the vote runs one workgroup per angle with the accumulator row in LDS,
and the numpy float32 sin/cos are restated bit for bit.
"""
from __future__ import annotations

import numpy as np

from . import _frontend


class HoughTransformation:

    @staticmethod
    def detect_line_intersections(points: np.ndarray) -> list:
        """Intersection points (x, y) in the points' frame, in the reference's order
        (hough_transformation.py:14-41); numpy float32 scalars (float64 with
        config.FRONTEND_NUMPY1_PROMOTION), like the reference under that numpy."""
        from .. import config
        r = _frontend.run([points], sigma=None, want=("intersections",))["intersections"][0]
        t = np.float64 if config.FRONTEND_NUMPY1_PROMOTION else np.float32
        return [(t(x), t(y)) for x, y in r]

    @staticmethod
    def hough_lines(points: np.ndarray) -> np.ndarray | None:
        """What cv2.HoughLines returns inside detect_line_intersections: [K][1][2]
        float32 (rho, theta) in OpenCV's order, or None."""
        r = _frontend.run([points], sigma=None, want=("lines",))["lines"][0]
        return r.reshape(-1, 1, 2) if len(r) else None
