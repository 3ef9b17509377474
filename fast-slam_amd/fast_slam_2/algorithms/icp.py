"""ICP scan matcher on the GPU (reference: fast_slam_2/algorithms/icp.py:13-90).

One workgroup per alignment holds both clouds in LDS for the whole loop;
exact nearest neighbours through a uniform grid over the target cloud (ring
search with a conservative bound; lowest index on exact ties, as brute force
and a KD-tree query on non-degenerate clouds give), rotation by the closed-form
2-D Kabsch angle (equal to the reference's SVD + reflection fix).
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from .. import _native as nat


class ICP:
    device = 0

    @staticmethod
    def get_transformation(source_points: np.ndarray, target_points: np.ndarray,
                           max_iterations=100, threshold=1e-5) -> tuple[np.ndarray, np.ndarray]:
        R, t, _ = ICP.get_transformation_ex(source_points, target_points, max_iterations,
                                            threshold)
        return R, t

    @staticmethod
    def get_transformation_ex(source_points, target_points, max_iterations=100, threshold=1e-5):
        """As get_transformation, plus the number of iterations run."""
        src = nat.f64(source_points, (-1, 2))
        tgt = nat.f64(target_points, (-1, 2))
        R = np.empty(4)
        t = np.empty(2)
        it = C.c_int32()
        nat.check(nat.load().fs2_icp(ICP.device, nat.dptr(src), len(src), nat.dptr(tgt), len(tgt),
                                     int(max_iterations), float(threshold), nat.dptr(R),
                                     nat.dptr(t), C.byref(it)))
        return R.reshape(2, 2), t, int(it.value)

    @staticmethod
    def submit(source_points, target_points, max_iterations=100, threshold=1e-5) -> "IcpTicket":
        """Enqueue get_transformation on the device's ICP stream and return at once;
        ``.result()`` gives (R, t, iterations).  Lets the alignment of scan s+1 run
        beside the filter update of scan s (fs2_icp_submit in include/fs2.h)."""
        src = nat.f64(source_points, (-1, 2))
        tgt = nat.f64(target_points, (-1, 2))
        tk = C.c_int64()
        nat.check(nat.load().fs2_icp_submit(ICP.device, nat.dptr(src), len(src), nat.dptr(tgt),
                                            len(tgt), int(max_iterations), float(threshold),
                                            C.byref(tk)))
        return IcpTicket(ICP.device, tk.value)

    @staticmethod
    def get_transformation_batched(sources, targets, max_iterations=100, threshold=1e-5):
        """B independent alignments: sources/targets [B][P][2] -> R [B][2][2], t [B][2], iters [B]."""
        src = nat.f64(sources)
        tgt = nat.f64(targets)
        B, P = src.shape[0], src.shape[1]
        R = np.empty((B, 4))
        t = np.empty((B, 2))
        it = np.empty(B, dtype=np.int32)
        nat.check(nat.load().fs2_icp_batched(ICP.device, B, P, nat.ptr(src), nat.ptr(tgt),
                                             int(max_iterations), float(threshold), nat.ptr(R),
                                             nat.ptr(t), nat.ptr(it), nat.FS2_HOST))
        return R.reshape(B, 2, 2), t, it

    @staticmethod
    def best_fit_transform(source_points, target_points):
        src = nat.f64(source_points, (-1, 2))
        tgt = nat.f64(target_points, (-1, 2))
        R = np.empty(4)
        t = np.empty(2)
        nat.check(nat.load().fs2_best_fit_transform(ICP.device, nat.dptr(src), nat.dptr(tgt),
                                                    len(src), nat.dptr(R), nat.dptr(t)))
        return R.reshape(2, 2), t


class IcpTicket:
    """An alignment enqueued by ICP.submit; result() waits for it once."""

    def __init__(self, device, ticket):
        self.device = device
        self.ticket = ticket
        self._out = None

    def result(self):
        if self._out is None:
            R = np.empty(4)
            t = np.empty(2)
            it = C.c_int32()
            nat.check(nat.load().fs2_icp_wait(self.device, self.ticket, nat.dptr(R), nat.dptr(t),
                                              C.byref(it)))
            self._out = (R.reshape(2, 2), t, int(it.value))
        return self._out
