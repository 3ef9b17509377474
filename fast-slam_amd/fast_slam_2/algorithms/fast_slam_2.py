"""FastSLAM2: drop-in for the reference's fast_slam_2.algorithms.FastSLAM2.

The per-scan hot path -- motion sample, association, EKF, likelihood,
normalisation, N_eff, low-variance resample, estimate
(reference fast_slam_2/algorithms/fast_slam_2.py:33-223) -- runs in libfs2.so on
the GPU; particle state stays resident in HBM between scans.

Randomness.  By default the motion noise and the resample starting point are
drawn from numpy's global legacy RandomState exactly as the reference draws
them (N normals in particle order, then one uniform only if resampling fires,
SURVEY.md Q4/Q5), so a seeded run reproduces the reference's stream.  The
draws are made on the GPU from np.random.get_state() (fs2_mt_draw: MT19937 and
the polar method bit for bit, a few logs near a rounding midpoint recomputed
with the host's libm) and numpy's state is advanced to where the reference's
draws leave it: past the normals, and past the uniform only when resampling
fired.  rng="numpy-host" draws them with numpy on the host instead (the same
values, ~10 ms per 1e6 particles); rng="device" draws both with Philox on the
GPU (not numpy's stream; used by bench.py).
"""
from __future__ import annotations

import ctypes as C
from collections.abc import Sequence

import numpy as np

from .. import _native as nat
from .. import _npstate
from .. import config
from ..models.landmark import Landmark
from ..models.measurement import Measurement
from ..models.particle import Particle

_REDUCE = {"auto": nat.FS2_REDUCE_AUTO, "sequential": nat.FS2_REDUCE_SEQUENTIAL,
           "parallel": nat.FS2_REDUCE_PARALLEL, "exact": nat.FS2_REDUCE_EXACT}


class FastSLAM2:
    """FastSLAM 2.0 particle filter (reference fast_slam_2.py:15-31)."""

    def __init__(self, num_particles: int | None = None, *, device: int = 0, rng: str = "numpy",
                 seed: int | None = None, reduce: str = "auto", record_assoc: bool = False,
                 landmark_capacity: int = 64, rank: int = 0, world_size: int = 1,
                 comm_id: bytes | None = None, verbose: bool = True, gate_filter: bool = True,
                 comm_mode: str = "rccl", sharded_path: bool = False, page_pool: int = 0,
                 record_pool: int = 0, page_refs: str = "auto"):
        lib = nat.load()
        cfg = nat.default_config()
        cfg.num_particles = int(config.NUM_PARTICLES if num_particles is None else num_particles)
        cfg.translation_noise = float(config.TRANSLATION_NOISE)
        cfg.rotation_noise = float(config.ROTATION_NOISE)
        R = np.asarray(config.MEASUREMENT_NOISE, dtype=np.float64).reshape(4)
        for k in range(4):
            cfg.measurement_noise[k] = R[k]
        cfg.max_landmark_distance = float(config.MAXIMUM_LANDMARK_DISTANCE)
        cfg.landmark_capacity = int(landmark_capacity)
        cfg.device = int(device)
        cfg.reduce_mode = _REDUCE[reduce]
        if seed is not None:
            cfg.seed = int(seed) & 0xFFFFFFFFFFFFFFFF
        cfg.record_assoc = 1 if record_assoc else 0
        cfg.gate_filter = 1 if gate_filter else 0
        cfg.rank = int(rank)
        cfg.world_size = int(world_size)
        if comm_id is not None:
            C.memmove(cfg.comm_id, comm_id, 128)
        cfg.comm_mode = {"rccl": nat.FS2_COMM_RCCL, "local": nat.FS2_COMM_LOCAL,
                         "shm": nat.FS2_COMM_SHM}[comm_mode]
        cfg.sharded_path = 1 if sharded_path else 0
        cfg.page_pool = int(page_pool)          # initial pool sizes (0: defaults; fs2.h)
        cfg.record_pool = int(record_pool)
        # sharded resample: pages by reference ("on"), by content ("off"); fs2.h page_refs
        cfg.page_refs = {"auto": 0, "on": 1, "off": -1}[page_refs]
        if rng not in ("numpy", "numpy-host", "device"):
            raise ValueError("rng must be 'numpy', 'numpy-host' or 'device'")
        self._rng = rng
        self._verbose = verbose
        h = C.c_void_p()
        nat.check(lib.fs2_create(C.byref(cfg), C.byref(h)))
        self._lib = lib
        self._h = h
        self._cfg = cfg
        n_local, first, cap = C.c_int64(), C.c_int64(), C.c_int32()
        nat.check(lib.fs2_shard_info(h, C.byref(n_local), C.byref(first), C.byref(cap)), h)
        self.num_particles = int(cfg.num_particles)
        self.n_local = int(n_local.value)
        self._particles = None
        self.last_stats = None
        # step(): fs2_iterate through a prototype of plain addresses and buffers
        # made once (ndarray.ctypes conversions cost ~3 us each, a scan ~500 us)
        proto = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_double, C.c_double, C.c_void_p, C.c_void_p, C.c_int32,
                            C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p)
        self._iterate_raw = proto(C.cast(lib.fs2_iterate, C.c_void_p).value)
        sproto = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_double, C.c_double, C.c_void_p, C.c_void_p, C.c_int32,
                             C.c_void_p, C.c_void_p)
        self._submit_raw = sproto(C.cast(lib.fs2_iterate_submit, C.c_void_p).value)
        wproto = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, C.c_void_p)
        self._wait_raw = wproto(C.cast(lib.fs2_iterate_wait, C.c_void_p).value)
        self._hv = h.value
        self._mcap = 0
        self._grow_meas(8)                      # measurement / observed-point buffers
        self._pose = np.empty(3)
        self._pose_addr = self._pose.ctypes.data
        self._st = nat.fs2_iter_stats()
        self._st_addr = C.addressof(self._st)
        self._u0 = np.empty(1)
        self._u0_addr = self._u0.ctypes.data
        self._mt = [nat.fs2_mt_state() for _ in range(3)]     # in, after the normals, after u0
        self._mt_addr = [C.addressof(m) for m in self._mt]
        dproto = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, C.c_double, C.c_void_p, C.c_void_p, C.c_void_p)
        self._draw_raw = dproto(C.cast(lib.fs2_mt_draw_deferred, C.c_void_p).value)

    @property
    def first_global(self) -> int:
        """Global index of local particle 0.  Sharded handles with equal shards may
        take another shard at a resample (the one their sources fill most; DESIGN.md
        §5), so this is read from libfs2 each time."""
        if self._h is None:
            raise nat.FS2Error(nat.FS2_ERR_ARG, "first_global of a closed FastSLAM2 handle")
        n_local, first, cap = C.c_int64(), C.c_int64(), C.c_int32()
        nat.check(self._lib.fs2_shard_info(self._h, C.byref(n_local), C.byref(first), C.byref(cap)), self._h)
        return int(first.value)

    # ------------------------------------------------------------------ core
    def iterate(self, rotation: float, translation: float,
                measurements: list[Measurement]) -> tuple[float, float, float]:
        """One FastSLAM step (reference fast_slam_2.py:33-67); returns the estimate pose."""
        if not getattr(self, "_h", None) or not self._hv:
            raise nat.FS2Error(nat.FS2_ERR_ARG, "iterate on a closed FastSLAM2 handle")
        M = len(measurements)
        if M > self._mcap:
            self._grow_meas(M)
        mb, ob = self._mbuf, self._obuf
        for k, m in enumerate(measurements):
            d, b = m.distance, m.yaw
            mb[k, 0] = d
            mb[k, 1] = b
            # observed robot-frame point, computed as the reference does (:100-103)
            ob[k, 0] = d * np.cos(b)
            ob[k, 1] = d * np.sin(b)
        noise = u0 = None
        state = None
        sigma = config.ROTATION_NOISE if rotation != 0 else config.TRANSLATION_NOISE
        if self._rng == "numpy":
            mt_in = self._mt[0]
            npv = _npstate.view()                # numpy's state in place (get_state: ~40-70 us)
            if npv is not None:
                npv.read(mt_in)
            else:
                C.pointer(mt_in)[0] = nat.fs2_mt_state.from_numpy(np.random.get_state())
            # ended by fs2_iterate below, while its candidate pass runs (mt_after / mt_u0 written then)
            rc = self._draw_raw(self._hv, self._mt_addr[0], float(sigma), self._mt_addr[1], self._mt_addr[2], None)
            if rc == nat.FS2_ERR_STATE and "libm" in nat.last_error(self._h):
                self._rng = "numpy-host"        # another libm: numpy draws on the host, still exact
            else:
                nat.check(rc, self._h)
        if self._rng == "numpy-host":
            noise = np.random.normal(0, sigma, size=self.num_particles)
            noise = np.ascontiguousarray(noise[self.first_global:self.first_global + self.n_local])
            state = np.random.get_state()
            self._u0[0] = np.random.uniform(0, 1 / self.num_particles)
            u0 = self._u0_addr
        rc = self._iterate_raw(self._hv, float(rotation), float(translation), self._mbuf_addr if M else None,
                               self._obuf_addr if M else None, M, None if noise is None else noise.ctypes.data, u0,
                               self._pose_addr, self._st_addr)
        self._particles = None
        st = nat.fs2_iter_stats.from_buffer_copy(self._st)
        self.last_stats = st
        if self._rng == "numpy":
            # the normals are drawn by the move, u0 only when resampling (fast_slam_2.py:79,81,183)
            chosen = self._mt[2] if (rc == 0 and st.resampled) else self._mt[1]
            npv = _npstate.view()
            if npv is not None:
                npv.write(chosen)
            else:
                np.random.set_state(chosen.to_numpy())
        elif state is not None and not st.resampled:
            np.random.set_state(state)          # the reference draws u0 only when resampling
        nat.check(rc, self._h)
        if st.resampled and self._verbose:
            print("\nRESAMPLING")               # reference fast_slam_2.py:63
        pose = self._pose
        return float(pose[0]), float(pose[1]), float(pose[2])

    def _grow_meas(self, M):
        self._mcap = max(M, 2 * self._mcap, 8)
        self._mbuf = np.empty((self._mcap, 2))
        self._obuf = np.empty((self._mcap, 2))
        self._mbuf_addr = self._mbuf.ctypes.data
        self._obuf_addr = self._obuf.ctypes.data

    def step(self, rotation: float, translation: float, meas, observed=None, noise=None,
             u0=None):
        """iterate() with explicit inputs: meas [M][2] (distance, yaw); observed [M][2]
        robot-frame points (None: computed in libfs2); noise [N_local] motion draws and
        u0 the resample start (None: Philox on the device).  Returns (pose, stats)."""
        return self._step(rotation, translation, meas, observed, noise, u0, split=False)

    def step_submit(self, rotation: float, translation: float, meas, observed=None, noise=None, u0=None):
        """The first half of step(): enqueue the scan and return while the GPU works
        (libfs2 fs2_iterate_submit).  Finish it with step_wait()."""
        self._step(rotation, translation, meas, observed, noise, u0, split=True)

    def step_wait(self):
        """Complete the scan step_submit() enqueued; returns (pose, stats) like step()."""
        if not getattr(self, "_h", None) or not self._hv:
            raise nat.FS2Error(nat.FS2_ERR_ARG, "step_wait() on a closed FastSLAM2 handle")
        rc = self._wait_raw(self._hv, self._pose_addr, self._st_addr)
        self._particles = None
        st = nat.fs2_iter_stats.from_buffer_copy(self._st)
        self.last_stats = st
        nat.check(rc, self._h)
        return self._pose.copy(), st

    def _step(self, rotation, translation, meas, observed, noise, u0, split):
        if not getattr(self, "_h", None) or not self._hv:
            raise nat.FS2Error(nat.FS2_ERR_ARG, "step() on a closed FastSLAM2 handle")
        meas = nat.f64(meas).reshape(-1, 2)
        M = meas.shape[0]
        obs = None
        if observed is not None:
            obs = nat.f64(observed).reshape(-1, 2)
            if obs.shape[0] != M:
                raise ValueError(f"observed has {obs.shape[0]} points for {M} measurements")
        if M > self._mcap:
            self._grow_meas(M)
        oa = None
        if M:
            self._mbuf[:M] = meas
            if obs is not None:
                self._obuf[:M] = obs
                oa = self._obuf_addr
        nz = None
        if noise is not None:
            nz = nat.f64(noise)
            if nz.size != self.n_local:
                raise ValueError(f"noise must have {self.n_local} values")
        ua = None
        if u0 is not None:
            self._u0[0] = float(u0)
            ua = self._u0_addr
        if split:
            rc = self._submit_raw(self._hv, float(rotation), float(translation), self._mbuf_addr if M else None, oa,
                                  M, None if nz is None else nz.ctypes.data, ua)
            self._particles = None
            nat.check(rc, self._h)
            return None
        rc = self._iterate_raw(self._hv, float(rotation), float(translation), self._mbuf_addr if M else None, oa,
                               M, None if nz is None else nz.ctypes.data, ua, self._pose_addr, self._st_addr)
        self._particles = None
        st = nat.fs2_iter_stats.from_buffer_copy(self._st)
        self.last_stats = st
        nat.check(rc, self._h)
        return self._pose.copy(), st

    # ------------------------------------------------------------ particles
    def get_state(self, first: int = 0, count: int | None = None, lm_cap: int | None = None):
        """Local particles [first, first+count) as arrays (x, y, yaw, w, cnt, lm[count][cap][6])."""
        count = self.n_local - first if count is None else count
        x, y, yaw, w = (np.empty(count) for _ in range(4))
        cnt = np.empty(count, dtype=np.int32)
        nat.check(self._lib.fs2_get_state(self._h, first, count, nat.ptr(x), nat.ptr(y),
                                          nat.ptr(yaw), nat.ptr(w), nat.ptr(cnt), None, 0,
                                          nat.FS2_HOST), self._h)
        cap = int(cnt.max()) if (lm_cap is None and count) else (lm_cap or 0)
        lm = np.zeros((count, max(cap, 1), 6))
        if cap:
            nat.check(self._lib.fs2_get_state(self._h, first, count, None, None, None, None,
                                              None, nat.ptr(lm), max(cap, 1), nat.FS2_HOST),
                      self._h)
        return x, y, yaw, w, cnt, lm

    def set_state(self, x=None, y=None, yaw=None, w=None, cnt=None, lm=None, first: int = 0):
        """Upload local particles starting at `first`; lm is [count][cap][6] with cnt."""
        arrs = [None if a is None else nat.f64(a) for a in (x, y, yaw, w)]
        count = next((len(a) for a in arrs + [cnt] if a is not None), 0)
        lmh = None
        cap = 0
        cnth = None
        if cnt is not None:
            cnth = np.ascontiguousarray(cnt, dtype=np.int32)
            lmh = nat.f64(lm)
            cap = lmh.shape[1]
        nat.check(self._lib.fs2_set_state(self._h, first, count, *(nat.ptr(a) for a in arrs),
                                          nat.ptr(cnth), nat.ptr(lmh), cap, nat.FS2_HOST),
                  self._h)
        self._particles = None

    @property
    def particles(self) -> "ParticleView":
        """This rank's particles (reference attribute `particles`), materialised lazily in
        chunks; LandmarkUtils.update_known_landmarks given this view clusters on the device."""
        if self._particles is None:
            self._particles = ParticleView(self)
        return self._particles

    def poses(self):
        """(x, y, yaw) arrays of this rank's particles (one structure-of-arrays download)."""
        x, y, yaw = (np.empty(self.n_local) for _ in range(3))
        nat.check(self._lib.fs2_get_state(self._h, 0, self.n_local, nat.ptr(x), nat.ptr(y), nat.ptr(yaw),
                                          None, None, None, 0, nat.FS2_HOST), self._h)
        return x, y, yaw

    def cluster_landmarks(self, eps: float = 0.5, min_fraction: float = 0.7):
        """Centres [K][2] of DBSCAN over every particle's landmarks, on the device
        (update_known_landmarks, landmark_utils.py:120-144); None when min_samples < 1."""
        cap = 256
        while True:
            cen = np.empty((cap, 2))
            k = C.c_int64()
            rc = self._lib.fs2_update_known_landmarks(self._h, float(eps), float(min_fraction),
                                                      nat.dptr(cen), cap, C.byref(k))
            if rc == nat.FS2_ERR_ARG and k.value > cap:
                cap = int(k.value)
                continue
            nat.check(rc, self._h)
            return None if k.value < 0 else cen[:k.value].copy()

    @particles.setter
    def particles(self, plist: list[Particle]):
        if len(plist) != self.n_local:
            raise ValueError(f"expected {self.n_local} particles, got {len(plist)}")
        cnt = np.array([len(p.landmarks) for p in plist], dtype=np.int32)
        cap = max(int(cnt.max()) if len(cnt) else 0, 1)
        lm = np.zeros((len(plist), cap, 6))
        for i, p in enumerate(plist):
            for j, l in enumerate(p.landmarks):
                c = np.asarray(l.cov, dtype=np.float64).reshape(4)
                lm[i, j] = (l.x, l.y, c[0], c[1], c[2], c[3])
        self.set_state([p.x for p in plist], [p.y for p in plist], [p.yaw for p in plist],
                       [p.weight for p in plist], cnt, lm)

    # ------------------------------------------------------------ extras
    def associations(self) -> np.ndarray:
        """[M][N_local] association indices of the last scan (-1 = appended)."""
        m = C.c_int32()
        buf = np.empty(max(self.n_local * 64, 1), dtype=np.int32)
        nat.check(self._lib.fs2_get_assoc(self._h, buf.ctypes.data_as(C.POINTER(C.c_int32)),
                                          buf.size, C.byref(m)), self._h)
        return buf[:m.value * self.n_local].reshape(m.value, self.n_local).copy()

    def set_profiling(self, enable: bool = True, every: int = 1):
        """Device-event timing of the update kernels on every `every`-th scan (libfs2
        fs2_set_profiling; resets the profile)."""
        nat.check(self._lib.fs2_set_profiling(self._h, max(1, int(every)) if enable else 0), self._h)

    def profile(self) -> dict:
        p = nat.fs2_profile()
        nat.check(self._lib.fs2_get_profile(self._h, C.byref(p)), self._h)
        return p.as_dict()

    def synchronize(self):
        nat.check(self._lib.fs2_synchronize(self._h), self._h)

    def close(self):
        self._hv = None                         # step()'s raw address: never reused once freed
        if getattr(self, "_h", None):
            self._lib.fs2_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class ParticleView(Sequence):
    """Lazy, read-only sequence of Particle objects over a FastSLAM2's device state
    (downloaded 4096 particles at a time on first access)."""

    _CHUNK = 4096

    def __init__(self, filt: FastSLAM2):
        self._filter = filt
        self._n = filt.n_local
        self._chunks: dict[int, list[Particle]] = {}

    def __len__(self):
        return self._n

    def _chunk(self, c: int) -> list[Particle]:
        if c not in self._chunks:
            first = c * self._CHUNK
            count = min(self._CHUNK, self._n - first)
            x, y, yaw, w, cnt, lm = self._filter.get_state(first, count)
            out = []
            for i in range(count):
                p = Particle.__new__(Particle)
                p.x, p.y, p.yaw, p.weight = float(x[i]), float(y[i]), float(yaw[i]), float(w[i])
                p.landmarks = [Landmark(float(lm[i, j, 0]), float(lm[i, j, 1]),
                                        lm[i, j, 2:6].reshape(2, 2).copy())
                               for j in range(int(cnt[i]))]
                out.append(p)
            self._chunks[c] = out
        return self._chunks[c]

    def __getitem__(self, i):
        if isinstance(i, slice):
            return [self[k] for k in range(*i.indices(self._n))]
        if i < 0:
            i += self._n
        if not 0 <= i < self._n:
            raise IndexError("particle index out of range")
        return self._chunk(i // self._CHUNK)[i % self._CHUNK]
