"""Seeded synthetic workload for the FastSLAM 2.0 particle-update hot path.

Implements the canonical generator of SURVEY.md §8(d).  It is shared by the
golden-fixture script (tests/golden/gen_golden.py), the parity tests and
bench.py, so every consumer sees the same scans, odometry, maps and
measurements for a given (seed, config).  Nothing here touches the GPU or the
reference; it is plain numpy.

Geometry conventions follow the reference:
  * laser beams: angle = radians(i - 90) for the 180-beam scanner
    (fast_slam_2/models/robot.py:42-55); the 720-beam variant uses 0.25 deg;
  * measurement encoding (distance, bearing) = (sqrt(x^2 + y^2), atan2(y, x))
    (fast_slam_2/utils/geometry_utils.py:65-74);
  * odometry pattern of jde_robots_main.py:25-31: translate, or rotate in place.
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import numpy as np

GRID_SPACING = 6.0          # > 2 x default gate radius 8*sqrt(0.1) = 2.53 m
GRID_JITTER = 0.25          # common landmark jitter U(-0.25, 0.25)
MAP_JITTER = 0.02           # per-particle copy jitter N(0, 0.02^2)
HIT_RADIUS = 0.3            # hit measurement within 0.3 m of its landmark
INIT_COV = 0.1              # landmark.py:13 default covariance 0.1*I
ROOM = (20.0, 15.0)         # rectangular room, centred at the origin
RANGE_NOISE = 0.01


def substream(seed: int, k: int) -> np.random.Generator:
    """Independent substream `k` of master seed `seed`."""
    return np.random.default_rng([seed, k])


def grid_shape(L: int) -> tuple[int, int]:
    cols = max(1, int(math.ceil(math.sqrt(L))))
    rows = max(1, int(math.ceil(L / cols)))
    return rows, cols


def common_landmarks(L: int, seed: int = 0) -> np.ndarray:
    """L landmark positions on a 6 m grid centred at the origin, jittered."""
    rows, cols = grid_shape(L)
    rng = substream(seed, 1)
    out = np.empty((L, 2))
    for n in range(L):
        r, c = divmod(n, cols)
        out[n, 0] = (c - (cols - 1) / 2.0) * GRID_SPACING
        out[n, 1] = (r - (rows - 1) / 2.0) * GRID_SPACING
    out += rng.uniform(-GRID_JITTER, GRID_JITTER, size=(L, 2))
    return out


def miss_point(L: int, scan: int) -> np.ndarray:
    """Centre of a grid cell (>= 3.9 m from every landmark); a distinct cell per scan."""
    rows, cols = grid_shape(L)
    rows_c, cols_c = max(rows - 1, 1) + 2, max(cols - 1, 1) + 2
    n = scan % (rows_c * cols_c)
    r, c = divmod(n, cols_c)
    x = (c - 1 + 0.5 - (cols - 1) / 2.0) * GRID_SPACING
    y = (r - 1 + 0.5 - (rows - 1) / 2.0) * GRID_SPACING
    return np.array([x, y])


def particle_poses(N: int, seed: int = 0) -> tuple[np.ndarray, np.ndarray, np.ndarray]:
    rng = substream(seed, 2)
    x = rng.normal(0.0, 0.05, N)
    y = rng.normal(0.0, 0.05, N)
    yaw = rng.normal(0.0, 0.01, N)
    return x, y, yaw


def particle_maps(N: int, L: int, seed: int = 0, first: int = 0,
                  count: int | None = None) -> np.ndarray:
    """Per-particle landmark copies [count][L][6] = (x, y, P00, P01, P10, P11).

    Particle `first + i` gets the common grid plus its own N(0, 0.02^2) jitter
    drawn from substream (seed, 1000 + particle index // 4096) so any range of
    particles can be generated independently (bench uploads in chunks).
    """
    count = N - first if count is None else count
    base = common_landmarks(L, seed)
    out = np.empty((count, L, 6))
    out[:, :, 2] = INIT_COV
    out[:, :, 3] = 0.0
    out[:, :, 4] = 0.0
    out[:, :, 5] = INIT_COV
    blk = 4096
    i = 0
    while i < count:
        g = first + i
        b = g // blk
        lo = b * blk
        rng = substream(seed, 1000 + b)
        jit = rng.normal(0.0, MAP_JITTER, size=(blk, L, 2))
        take = min(count - i, lo + blk - g)
        out[i:i + take, :, 0:2] = base[None, :, :] + jit[g - lo:g - lo + take]
        i += take
    return out


def odometry(scan: int) -> tuple[float, float]:
    """(rotation, translation): 4 translations of 0.03 m, then a 0.05 rad turn."""
    if scan % 5 == 4:
        return 0.05, 0.0
    return 0.0, 0.03


def encode(px: float, py: float) -> tuple[float, float]:
    """GeometryUtils.calculate_distance_and_angle (geometry_utils.py:65-74)."""
    return math.sqrt(px ** 2 + py ** 2), math.atan2(py, px)


def scan_measurements(L: int, scan: int, seed: int = 0, n_hits: int = 3,
                      with_miss: bool = True) -> np.ndarray:
    """M x 2 (distance, bearing): n_hits near common landmarks, then one miss."""
    base = common_landmarks(L, seed)
    rng = substream(seed, 100000 + scan)
    rows = []
    for _ in range(n_hits):
        j = int(rng.integers(0, L))
        r = HIT_RADIUS * math.sqrt(rng.uniform())
        a = rng.uniform(-math.pi, math.pi)
        p = base[j] + np.array([r * math.cos(a), r * math.sin(a)])
        rows.append(encode(float(p[0]), float(p[1])))
    if with_miss:
        p = miss_point(L, scan)
        rows.append(encode(float(p[0]), float(p[1])))
    return np.array(rows, dtype=np.float64).reshape(-1, 2)


def discovery_order(L: int) -> np.ndarray:
    """The order in which a robot sweeping the landmark grid row by row, turning at
    each row's end (a lawnmower path), first sees the L landmarks of
    common_landmarks: the order its map grows in by appends (fast_slam_2.py:108-111)."""
    rows, cols = grid_shape(L)
    order = []
    for r in range(rows):
        for c in (range(cols) if r % 2 == 0 else range(cols - 1, -1, -1)):
            if r * cols + c < L:
                order.append(r * cols + c)
    return np.array(order, dtype=np.int64)


def buildup_scans(L: int, per_scan: int = 8) -> int:
    """Scans of the map build-up (buildup_measurements) that discover all L landmarks."""
    return (L + per_scan - 1) // per_scan


def buildup_measurements(L: int, scan: int, seed: int = 0, per_scan: int = 8, rehits: int = 2,
                         recent: int = 24) -> np.ndarray:
    """Scan `scan` of the reference's own operating mode, maps grown by appends from
    empty (fast_slam_2.py:20-31, :108-111): the next `per_scan` landmarks in
    discovery order (each a miss for every particle, so each is appended, in
    observation order), then `rehits` observations of landmarks discovered in the
    scans before (within `recent` landmarks of the front: what the robot still
    sees), which associate, update the maps and move the weights.  Points within
    HIT_RADIUS of the true landmark, encoded like scan_measurements."""
    base = common_landmarks(L, seed)
    order = discovery_order(L)
    rng = substream(seed, 300000 + scan)
    lo = scan * per_scan
    rows = []
    for j in order[lo:lo + per_scan]:
        r = HIT_RADIUS * math.sqrt(rng.uniform())
        a = rng.uniform(-math.pi, math.pi)
        p = base[j] + np.array([r * math.cos(a), r * math.sin(a)])
        rows.append(encode(float(p[0]), float(p[1])))
    if lo > 0:
        for _ in range(rehits):
            j = order[int(rng.integers(max(0, lo - recent), min(lo, L)))]
            r = HIT_RADIUS * math.sqrt(rng.uniform())
            a = rng.uniform(-math.pi, math.pi)
            p = base[j] + np.array([r * math.cos(a), r * math.sin(a)])
            rows.append(encode(float(p[0]), float(p[1])))
    return np.array(rows, dtype=np.float64).reshape(-1, 2)


def beam_angles(P: int) -> np.ndarray:
    if P == 180:
        return np.radians(np.arange(180) - 90.0)
    step = 180.0 / P
    return np.radians(np.arange(P) * step - 90.0)


def room_scan(pose: tuple[float, float, float], P: int = 180, seed: int = 0,
              scan: int = 0, noise: float = RANGE_NOISE) -> np.ndarray:
    """Ray-cast a P-beam scan of the 20 x 15 m room; points in the robot frame."""
    px, py, pyaw = pose
    hw, hh = ROOM[0] / 2.0, ROOM[1] / 2.0
    ang = beam_angles(P)
    wa = ang + pyaw
    c, s = np.cos(wa), np.sin(wa)
    with np.errstate(divide="ignore", invalid="ignore"):
        tx = np.where(c > 0, (hw - px) / c, np.where(c < 0, (-hw - px) / c, np.inf))
        ty = np.where(s > 0, (hh - py) / s, np.where(s < 0, (-hh - py) / s, np.inf))
    r = np.minimum(tx, ty)
    rng = substream(seed, 200000 + scan)
    r = r + rng.normal(0.0, noise, size=P)
    return np.column_stack((r * np.cos(ang), r * np.sin(ang)))


@dataclass
class Workload:
    """Initial state of a benchmark/parity configuration."""
    N: int
    L: int
    seed: int = 0

    def poses(self):
        return particle_poses(self.N, self.seed)

    def maps(self, first: int = 0, count: int | None = None):
        return particle_maps(self.N, self.L, self.seed, first, count)

    def measurements(self, scan: int) -> np.ndarray:
        return scan_measurements(self.L, scan, self.seed)

    @staticmethod
    def odometry(scan: int):
        return odometry(scan)


def room_corners() -> np.ndarray:
    hw, hh = ROOM[0] / 2.0, ROOM[1] / 2.0
    return np.array([[hw, hh], [-hw, hh], [-hw, -hh], [hw, -hh]])


def corner_measurements(pose, scan: int, seed: int = 0, noise: float = 0.02,
                        max_range: float = 12.0) -> np.ndarray:
    """Room-corner observations from `pose` (robot frame), as the front-end emits."""
    px, py, pyaw = pose
    rng = substream(seed, 300000 + scan)
    rows = []
    for cx, cy in room_corners():
        dx, dy = cx - px, cy - py
        lx = math.cos(-pyaw) * dx - math.sin(-pyaw) * dy
        ly = math.sin(-pyaw) * dx + math.cos(-pyaw) * dy
        if math.hypot(lx, ly) > max_range or lx < -1.0:
            continue
        lx += rng.normal(0.0, noise)
        ly += rng.normal(0.0, noise)
        rows.append(encode(lx, ly))
    return np.array(rows, dtype=np.float64).reshape(-1, 2)


# --------------------------------------------------------------- front-end ---
# Scenes for LandmarkUtils.get_measurements_to_landmarks (landmark_utils.py:21-89):
# closed polygons (walls), ray-cast like Robot.scan_environment (robot.py:32-58):
# beams outside [min_range, max_range] are dropped.

L_ROOM = np.array([[-6.0, -4.0], [6.0, -4.0], [6.0, 1.0], [2.0, 1.0], [2.0, 5.0], [-6.0, 5.0]])
BOX_ROOM = np.array([[-ROOM[0] / 2, -ROOM[1] / 2], [ROOM[0] / 2, -ROOM[1] / 2],
                     [ROOM[0] / 2, ROOM[1] / 2], [-ROOM[0] / 2, ROOM[1] / 2]])


def polygon_scan(vertices: np.ndarray, pose: tuple[float, float, float], P: int = 180,
                 rng: np.random.Generator | None = None, noise: float = RANGE_NOISE,
                 min_range: float = 0.1, max_range: float = 10.0) -> np.ndarray:
    """Robot-frame points (x, y) of a P-beam scan over -90..90 deg of a polygon."""
    px, py, pyaw = pose
    ang = beam_angles(P)
    dx, dy = np.cos(ang + pyaw), np.sin(ang + pyaw)
    v0 = np.asarray(vertices, dtype=np.float64)
    v1 = np.roll(v0, -1, axis=0)
    ex, ey = (v1 - v0)[:, 0], (v1 - v0)[:, 1]
    wx, wy = v0[:, 0] - px, v0[:, 1] - py
    den = dx[:, None] * ey[None, :] - dy[:, None] * ex[None, :]
    with np.errstate(divide="ignore", invalid="ignore"):
        t = (wx[None, :] * ey[None, :] - wy[None, :] * ex[None, :]) / den
        u = (wx[None, :] * dy[:, None] - wy[None, :] * dx[:, None]) / den
    ok = (np.abs(den) > 1e-12) & (t > 0) & (u >= 0) & (u <= 1)
    r = np.where(ok, t, np.inf).min(axis=1)
    if rng is not None and noise > 0:
        r = r + rng.normal(0.0, noise, size=P)
    keep = (r >= min_range) & (r <= max_range)
    return np.column_stack((r[keep] * np.cos(ang[keep]), r[keep] * np.sin(ang[keep])))
