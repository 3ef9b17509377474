#!/usr/bin/env python3
"""Build libfs2.so for gfx950 in-tree (fast-slam_amd/lib/libfs2.so).

hipcc cross-compiles without a GPU.  -ffp-contract=off: the kernels place
every FMA explicitly to follow the reference's numpy/OpenBLAS operation order.
"""
from __future__ import annotations

import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
LIB_DIR = os.path.join(HERE, "lib")
LIB = os.path.join(LIB_DIR, "libfs2.so")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
ARCH = os.environ.get("FS2_OFFLOAD_ARCH", "gfx950")
SOURCES = ["fs2_api.hip", "fs2_update.hip", "fs2_resample.hip", "fs2_exact.hip", "fs2_pages.hip", "fs2_cluster.hip",
           "fs2_geometry.hip", "fs2_frontend.hip"]
HEADERS = ["fs2_device.hpp", "fs2_kernels.hpp", "fs2_comm.hpp", "fs2_reduce.hpp", "fs2_frontend.hpp"]


def _stale() -> bool:
    if not os.path.exists(LIB):
        return True
    t = os.path.getmtime(LIB)
    deps = [os.path.join(CSRC, f) for f in SOURCES + HEADERS]
    deps.append(os.path.join(os.path.dirname(HERE), "include", "fs2.h"))
    deps.append(os.path.abspath(__file__))
    return any(os.path.getmtime(d) > t for d in deps if os.path.exists(d))


def build(force: bool = False, verbose: bool = False, defines=(), out: str | None = None) -> str:
    """defines / out: an A/B variant (-D flags) written to `out` instead of libfs2.so."""
    lib = out or LIB
    if not force and not defines and out is None and not _stale():
        return LIB
    os.makedirs(LIB_DIR, exist_ok=True)
    hipcc = os.path.join(ROCM, "bin", "hipcc")
    cmd = [hipcc, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared",
           "-ffp-contract=off", "-Wall", "-Wno-unused-function", "-Wno-unused-value",
           "-I", os.path.join(ROCM, "include"), *defines,
           *[os.path.join(CSRC, s) for s in SOURCES],
           "-o", lib + ".tmp", "-L", os.path.join(ROCM, "lib"), "-lrccl",
           "-Wl,-rpath," + os.path.join(ROCM, "lib")]
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    os.replace(lib + ".tmp", lib)
    return lib


HOOKS = os.path.join(LIB_DIR, "libfs2_hooks.so")


def build_hooks(verbose: bool = False) -> str:
    """libfs2_hooks.so: fs2_pages.hip alone with -DFS2_TEST_HOOKS (test entry points
    of single kernels; the GPU tests load it beside libfs2.so)."""
    src = os.path.join(CSRC, "fs2_pages.hip")
    deps = [src] + [os.path.join(CSRC, h) for h in os.listdir(CSRC) if h.endswith(".hpp")]
    if os.path.exists(HOOKS) and os.path.getmtime(HOOKS) >= max(os.path.getmtime(d) for d in deps):
        return HOOKS
    cmd = [os.path.join(ROCM, "bin", "hipcc"), f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC",
           "-shared", "-ffp-contract=off", "-DFS2_TEST_HOOKS", "-I", os.path.join(ROCM, "include"),
           src, "-o", HOOKS + ".tmp"]
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    os.replace(HOOKS + ".tmp", HOOKS)
    return HOOKS


if __name__ == "__main__":
    # python build.py [--force] [--variant TAG -DNAME=V ...]  (variant -> lib/libfs2_TAG.so)
    args = sys.argv[1:]
    tag = args[args.index("--variant") + 1] if "--variant" in args else None
    defs = [a for a in args if a.startswith("-D")]
    out = os.path.join(LIB_DIR, f"libfs2_{tag}.so") if tag else None
    print(build(force="--force" in args, verbose=True, defines=defs, out=out))
    if not tag:
        print(build_hooks(verbose=True))
