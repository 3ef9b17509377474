"""ctypes binding of libfs2.so (include/fs2.h).

There is no CPU fallback: if the library or a HIP device is missing, every
entry point raises.  Build the library with `python fast-slam_amd/build.py`.
"""
from __future__ import annotations

import ctypes as C
import os
import sys

import numpy as np

_PKG = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("FS2_LIB", os.path.join(os.path.dirname(_PKG), "lib", "libfs2.so"))

FS2_OK = 0
FS2_ERR_ARG = -1
FS2_ERR_HIP = -2
FS2_ERR_OOM = -3
FS2_ERR_LINALG = -4
FS2_ERR_STATE = -5
FS2_ERR_COMM = -6
FS2_ERR_CAPACITY = -7

FS2_REDUCE_AUTO = 0
FS2_REDUCE_SEQUENTIAL = 1
FS2_REDUCE_PARALLEL = 2
FS2_REDUCE_EXACT = 3
FS2_HOST = 0
FS2_DEVICE = 1
FS2_COMM_RCCL = 0
FS2_COMM_LOCAL = 1
FS2_COMM_SHM = 2


class fs2_config(C.Structure):
    _fields_ = [
        ("num_particles", C.c_int64),
        ("translation_noise", C.c_double),
        ("rotation_noise", C.c_double),
        ("measurement_noise", C.c_double * 4),
        ("max_landmark_distance", C.c_double),
        ("init_landmark_cov", C.c_double * 4),
        ("weight_floor", C.c_double),
        ("landmark_capacity", C.c_int32),
        ("max_landmark_capacity", C.c_int32),
        ("device", C.c_int32),
        ("reduce_mode", C.c_int32),
        ("seed", C.c_uint64),
        ("record_assoc", C.c_int32),
        ("gate_filter", C.c_int32),
        ("rank", C.c_int32),
        ("world_size", C.c_int32),
        ("comm_id", C.c_uint8 * 128),
        ("comm_mode", C.c_int32),
        ("sharded_path", C.c_int32),
        ("page_pool", C.c_int64),
        ("record_pool", C.c_int64),
        ("page_refs", C.c_int32),
        ("reserved0", C.c_int32),
    ]


class fs2_iter_stats(C.Structure):
    _fields_ = [
        ("resampled", C.c_int32),
        ("max_count", C.c_int32),
        ("n_eff", C.c_double),
        ("total_weight", C.c_double),
        ("best_index", C.c_int64),
        ("slots_visited", C.c_uint64),
        ("candidates", C.c_uint64),
        ("hits", C.c_uint64),
        ("appends", C.c_uint64),
        ("slots_written", C.c_uint64),
        ("ambiguous", C.c_uint64),
        ("resample_slots", C.c_uint64),
        ("error_flags", C.c_int32),
        ("reduce_ambiguous", C.c_int32),
        ("cow_pages", C.c_uint64),
        ("new_pages", C.c_uint64),
        ("collections", C.c_uint64),
        ("pool_pages", C.c_uint64),
        ("pages_opened", C.c_uint64),
        ("reference_visits", C.c_uint64),
        ("pool_records", C.c_uint64),
        ("pool_copies", C.c_uint64),
    ]

    def as_dict(self):
        return {name: getattr(self, name) for name, _ in self._fields_}


class fs2_profile(C.Structure):
    _fields_ = [
        ("scans", C.c_int64),
        ("update_launches", C.c_int64),
        ("update_ms", C.c_double),
        ("reduce_ms", C.c_double),
        ("resample_ms", C.c_double),
        ("scan_ms", C.c_double),
        ("update_bytes", C.c_uint64),
        ("resample_bytes", C.c_uint64),
        ("filter_launches", C.c_int64),
        ("filter_ms", C.c_double),
        ("filter_bytes", C.c_uint64),
        ("exact_launches", C.c_int64),
        ("exact_ms", C.c_double),
        ("comm_calls", C.c_int64),
        ("comm_ms", C.c_double),
        ("migrations", C.c_int64),
        ("sent_particles", C.c_uint64),
        ("sent_rows", C.c_uint64),
        ("sent_pages", C.c_uint64),
        ("sent_bytes", C.c_uint64),
        ("migrate_ms", C.c_double),
        ("sent_pages_repeat", C.c_uint64),
        ("model_groups", C.c_uint64),
        ("model_opened", C.c_uint64),
        ("model_words", C.c_uint64),
        ("model_candidates", C.c_uint64),
        ("model_written", C.c_uint64),
        ("model_cow", C.c_uint64),
        ("model_fixed_bytes", C.c_uint64),
        ("model_box_bytes", C.c_uint64),
        ("localized_pages", C.c_uint64),
        ("page_refs", C.c_int64),
        ("pool_collections", C.c_int64),
        ("collect_ms", C.c_double),
        ("pool_grows", C.c_int64),
        ("grow_ms", C.c_double),
        ("scan_allocs", C.c_int64),
        ("recv_bytes", C.c_uint64),
        ("exchange_ms", C.c_double),
    ]

    def as_dict(self):
        return {name: getattr(self, name) for name, _ in self._fields_}


class fs2_frontend_out(C.Structure):
    _fields_ = [("cap", C.c_int32), ("lines", C.c_void_p), ("intersections", C.c_void_p),
                ("clusters", C.c_void_p), ("corners", C.c_void_p), ("measurements", C.c_void_p),
                ("counts", C.c_void_p)]


class fs2_mt_state(C.Structure):
    """np.random.get_state()'s ('MT19937', key, pos, has_gauss, cached_gaussian)."""
    _fields_ = [("key", C.c_uint32 * 624), ("pos", C.c_int32), ("has_gauss", C.c_int32),
                ("gauss", C.c_double)]

    @classmethod
    def from_numpy(cls, st):
        name, key, pos, has_gauss, gauss = st
        if name != "MT19937":
            raise ValueError(f"numpy bit generator {name!r} is not MT19937")
        out = cls()
        C.memmove(out.key, np.ascontiguousarray(key, dtype=np.uint32).ctypes.data, 624 * 4)
        out.pos, out.has_gauss, out.gauss = int(pos), int(has_gauss), float(gauss)
        return out

    def to_numpy(self):
        return ("MT19937", np.frombuffer(bytes(self.key), dtype=np.uint32).copy(), int(self.pos),
                int(self.has_gauss), float(self.gauss))


class FS2Error(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"libfs2 error {code}: {msg}")
        self.code = code


_dp = C.POINTER(C.c_double)
_ip = C.POINTER(C.c_int32)
_vp = C.c_void_p
_H = C.c_void_p

# (name, restype, argtypes) for every entry point declared in include/fs2.h
SIGNATURES = [
    ("fs2_abi_version", C.c_int32, []),
    ("fs2_build_id", C.c_char_p, []),
    ("fs2_config_default", None, [C.POINTER(fs2_config)]),
    ("fs2_create", C.c_int, [C.POINTER(fs2_config), C.POINTER(_H)]),
    ("fs2_destroy", None, [_H]),
    ("fs2_last_error", C.c_char_p, [_H]),
    ("fs2_iterate", C.c_int, [_H, C.c_double, C.c_double, _vp, _vp, C.c_int32, _vp, _vp, _dp,
                              C.POINTER(fs2_iter_stats)]),
    ("fs2_iterate_submit", C.c_int, [_H, C.c_double, C.c_double, _vp, _vp, C.c_int32, _vp, _vp]),
    ("fs2_iterate_wait", C.c_int, [_H, _dp, C.POINTER(fs2_iter_stats)]),
    ("fs2_mt_draw", C.c_int, [_H, C.POINTER(fs2_mt_state), C.c_double, C.POINTER(fs2_mt_state),
                              C.POINTER(fs2_mt_state), _dp]),
    ("fs2_mt_draw_deferred", C.c_int, [_H, C.POINTER(fs2_mt_state), C.c_double, C.POINTER(fs2_mt_state),
                                       C.POINTER(fs2_mt_state), _dp]),
    ("fs2_get_state", C.c_int, [_H, C.c_int64, C.c_int64, _vp, _vp, _vp, _vp, _vp, _vp, C.c_int32,
                                C.c_int32]),
    ("fs2_set_state", C.c_int, [_H, C.c_int64, C.c_int64, _vp, _vp, _vp, _vp, _vp, _vp, C.c_int32,
                                C.c_int32]),
    ("fs2_get_assoc", C.c_int, [_H, _ip, C.c_int64, _ip]),
    ("fs2_shard_info", C.c_int, [_H, C.POINTER(C.c_int64), C.POINTER(C.c_int64),
                                 C.POINTER(C.c_int32)]),
    ("fs2_synchronize", C.c_int, [_H]),
    ("fs2_set_profiling", C.c_int, [_H, C.c_int32]),
    ("fs2_get_profile", C.c_int, [_H, C.POINTER(fs2_profile)]),
    ("fs2_icp", C.c_int, [C.c_int32, _dp, C.c_int32, _dp, C.c_int32, C.c_int32, C.c_double, _dp,
                          _dp, _ip]),
    ("fs2_icp_submit", C.c_int, [C.c_int32, _dp, C.c_int32, _dp, C.c_int32, C.c_int32, C.c_double,
                                 C.POINTER(C.c_int64)]),
    ("fs2_icp_wait", C.c_int, [C.c_int32, C.c_int64, _dp, _dp, _ip]),
    ("fs2_icp_batched", C.c_int, [C.c_int32, C.c_int32, C.c_int32, _vp, _vp, C.c_int32,
                                  C.c_double, _vp, _vp, _vp, C.c_int32]),
    ("fs2_best_fit_transform", C.c_int, [C.c_int32, _dp, _dp, C.c_int32, _dp, _dp]),
    ("fs2_line_filter", C.c_int, [C.c_int32, _dp, C.c_int32, _dp, C.c_int32, _dp]),
    ("fs2_gaussian_taps", C.c_int32, [C.c_double, C.c_double, _dp, C.c_int32]),
    ("fs2_associate", C.c_int, [C.c_int32, _dp, _dp, C.c_int32, C.c_double, _ip]),
    ("fs2_mahalanobis", C.c_int, [C.c_int32, _dp, _dp, _dp, C.c_int32, _dp]),
    ("fs2_cluster_points", C.c_int, [C.c_int32, _vp, C.c_int64, C.c_double, C.c_int64, _vp, C.c_int64,
                                     C.POINTER(C.c_int64), _vp, C.c_int32]),
    ("fs2_update_known_landmarks", C.c_int, [_H, C.c_double, C.c_double, _dp, C.c_int64,
                                             C.POINTER(C.c_int64)]),
    ("fs2_frontend", C.c_int, [C.c_int32, C.c_int32, _vp, _vp, C.c_int32, _dp, C.c_int32, C.c_int32,
                               C.POINTER(fs2_frontend_out)]),
    ("fs2_debug_philox", C.c_int, [C.c_int32, C.c_int64, _vp, _vp, _vp]),
    ("fs2_debug_normals", C.c_int, [C.c_int32, C.c_uint64, C.c_uint64, C.c_uint64, C.c_int64, _vp]),
    ("fs2_debug_mt_log", C.c_int, [C.c_int32, _vp, C.c_int64, _vp, _vp, C.c_int32]),
    ("fs2_debug_refuse_peer_maps", C.c_int, [_H]),
    ("fs2_debug_vm_fail_after_relocate", C.c_int, [C.c_int32]),
    ("fs2_release_cached_memory", C.c_int64, []),
    ("fs2_debug_noise", C.c_int, [_H, _vp]),
    ("fs2_debug_out_src", C.c_int64, [_H, _vp, C.c_int64]),
    ("fs2_debug_weights", C.c_int, [_H, C.c_int32, _vp]),
    ("fs2_debug_check_guards", C.c_int64, [_H, C.c_char_p, C.c_int64]),
    ("fs2_debug_mt_jump", C.c_int, [_vp, C.c_uint64, _vp]),
    ("fs2_comm_unique_id", C.c_int, [C.POINTER(C.c_uint8)]),
    ("fs2_plan_ranges", C.c_int, [_vp, C.c_int64, C.c_int64, C.c_int64, C.c_double, C.c_double, _vp, _vp]),
    ("fs2_plan_sends", C.c_int, [_vp, _vp, _vp, C.c_int64, C.c_int64, C.c_int32, C.c_int32, _vp, _vp, _vp]),
]

_lib = None


HIP_RUNTIME = None   # which HIP runtime libfs2 runs on: ("torch-wheel" | "system", path, version)


def _wheel_hip_version(torch_dir):
    """The HIP version a PyTorch wheel was built with, read from torch/version.py
    as text (no torch import)."""
    try:
        for line in open(os.path.join(torch_dir, "version.py")):
            if line.startswith("hip"):
                v = line.split("=", 1)[1].strip().strip("'\"")
                return None if v in ("None", "") else v
    except OSError:
        pass
    return None


def _system_hip_version():
    try:
        return open(os.path.join(os.environ.get("ROCM_PATH", "/opt/rocm"), ".info", "version")).read().strip()
    except OSError:
        return None


def _share_torch_hip_runtime():
    """One HIP runtime per process.  A PyTorch-ROCm wheel ships its own
    libamdhip64.so (and HSA runtime), which its libraries name without the ".7"
    (NEEDED libamdhip64.so, RPATH $ORIGIN); libfs2 names the system runtime's
    soname, libamdhip64.so.7.  Loaded first, libfs2 brings in /opt/rocm's runtime,
    and a later `import torch` loads the wheel's copy beside it -- two HSA runtimes,
    and PyTorch then finds no GPU (tests/test_gpu_torch_coexist.py).  Loaded after
    the wheel's copy, libfs2's soname matches it and both share it -- which is what
    happens whenever torch is imported first.

    FS2_HIP_RUNTIME chooses: "system" never loads the wheel's runtime (libfs2 and
    /opt/rocm's RCCL on the runtime they were built against; a later `import
    torch` in the same process then sees no GPU), "torch" always does.  Unset:
    the wheel's runtime when torch is already imported (it is loaded anyway) or a
    wheel is installed, so a later `import torch` works.  The choice and both
    versions are recorded in HIP_RUNTIME; a version mismatch is reported once
    (FS2_VERBOSE=1 prints the choice)."""
    global HIP_RUNTIME
    want = os.environ.get("FS2_HIP_RUNTIME", "").strip().lower()
    sysv = _system_hip_version()
    HIP_RUNTIME = ("system", None, sysv)
    if want == "system":
        return
    torch_dirs = []
    if "torch" in sys.modules and getattr(sys.modules["torch"], "__file__", None):
        torch_dirs = [os.path.dirname(sys.modules["torch"].__file__)]
    else:
        try:
            import importlib.util
            spec = importlib.util.find_spec("torch")
        except Exception:
            spec = None
        if spec is not None and spec.submodule_search_locations:
            torch_dirs = list(spec.submodule_search_locations)
    for d in torch_dirs:
        p = os.path.join(d, "lib", "libamdhip64.so")
        if not os.path.exists(p):
            continue
        try:
            C.CDLL(p, mode=C.RTLD_GLOBAL)
        except OSError:
            return
        wv = _wheel_hip_version(d)
        HIP_RUNTIME = ("torch-wheel", p, wv)
        if wv and sysv and wv.split(".")[:2] != sysv.split(".")[:2]:
            import warnings
            warnings.warn(f"libfs2 runs on PyTorch's HIP runtime {wv} ({p}), not the system ROCm {sysv} it "
                          f"was compiled against (one runtime per process; FS2_HIP_RUNTIME=system opts out)",
                          RuntimeWarning, stacklevel=3)
        break
    if os.environ.get("FS2_VERBOSE"):
        print(f"[fs2] HIP runtime: {HIP_RUNTIME}", file=sys.stderr)


def load():
    """Load libfs2.so (raises ImportError when it has not been built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"libfs2.so not found at {LIB_PATH}; build it with "
                          f"`python fast-slam_amd/build.py` (there is no CPU fallback)")
    _share_torch_hip_runtime()
    lib = C.CDLL(LIB_PATH)
    for name, res, args in SIGNATURES:
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if lib.fs2_abi_version() != 2:
        raise ImportError(f"libfs2 ABI {lib.fs2_abi_version()} != 2")
    _lib = lib
    return lib


def last_error(h=None) -> str:
    msg = load().fs2_last_error(h)
    return msg.decode() if msg else ""


def check(rc, h=None):
    if rc == FS2_OK:
        return
    msg = last_error(h)
    if rc == FS2_ERR_LINALG:
        raise np.linalg.LinAlgError(msg or "Singular matrix")
    if rc == FS2_ERR_ARG:
        raise ValueError(msg)
    if rc == FS2_ERR_OOM:
        raise MemoryError(msg)
    raise FS2Error(rc, msg)


def ptr(a):
    return None if a is None else a.ctypes.data_as(C.c_void_p)


def dptr(a):
    return a.ctypes.data_as(_dp)


def f64(a, shape=None):
    a = np.ascontiguousarray(a, dtype=np.float64)
    return a if shape is None else a.reshape(shape)


def default_config() -> fs2_config:
    cfg = fs2_config()
    load().fs2_config_default(C.byref(cfg))
    return cfg


def comm_unique_id() -> bytes:
    buf = (C.c_uint8 * 128)()
    check(load().fs2_comm_unique_id(buf))
    return bytes(buf)
