#!/usr/bin/env python3
"""Build libfs2.so for gfx950 in-tree (fast-slam_amd/lib/libfs2.so).

hipcc cross-compiles without a GPU.  -ffp-contract=off: the kernels place
every FMA explicitly to follow the reference's numpy/OpenBLAS operation order.
"""
from __future__ import annotations

import hashlib
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
           "fs2_geometry.hip", "fs2_frontend.hip", "fs2_mtrng.hip"]
# every header in csrc/ (a header left out of the hash would let a stale library pass)
HEADERS = sorted(f for f in os.listdir(CSRC) if f.endswith(".hpp"))


FLAGS = ["-O3", "-std=c++17", "-fPIC", "-shared", "-ffp-contract=off", "-Wall", "-Wno-unused-function",
         "-Wno-unused-value"]


def source_id(defines=()) -> str:
    """Hash of every source and header libfs2.so is built from, the build flags and
    the target: compiled into the library (fs2_build_id) and checked by the tests,
    so a library built from other sources is rebuilt here and refused on the GPU box."""
    h = hashlib.sha256()
    for f in sorted(SOURCES + HEADERS):
        h.update(f.encode() + b"\0" + open(os.path.join(CSRC, f), "rb").read())
    h.update(open(os.path.join(os.path.dirname(HERE), "include", "fs2.h"), "rb").read())
    h.update(" ".join([ARCH, *FLAGS, *defines]).encode())
    return h.hexdigest()[:20]


def built_id(lib: str = LIB) -> str | None:
    """The fs2_build_id the library at `lib` was compiled with (read from its
    sidecar file, written with the library)."""
    p = lib + ".id"
    return open(p).read().strip() if os.path.exists(p) and os.path.exists(lib) else None


def _stale() -> bool:
    return built_id() != source_id()


def build(force: bool = False, verbose: bool = False, defines=(), out: str | None = None) -> str:
    """defines / out: an A/B variant (-D flags) written to `out` instead of libfs2.so."""
    lib = out or LIB
    if not force and not defines and out is None and not _stale():
        return LIB
    os.makedirs(LIB_DIR, exist_ok=True)
    hipcc = os.path.join(ROCM, "bin", "hipcc")
    sid = source_id(defines)
    # one object per source, compiled in parallel, then linked (no -fgpu-rdc: each
    # translation unit's device code is self-contained, as in a one-command build)
    objdir = os.path.join(LIB_DIR, "obj", os.path.basename(lib))
    os.makedirs(objdir, exist_ok=True)
    cflags = [f"--offload-arch={ARCH}", *[f for f in FLAGS if f != "-shared"], f'-DFS2_BUILD_ID="{sid}"',
              "-I", os.path.join(ROCM, "include"), *defines]
    objs = [os.path.join(objdir, os.path.splitext(src)[0] + ".o") for src in SOURCES]
    cmds = [[hipcc, *cflags, "-c", os.path.join(CSRC, src), "-o", o] for src, o in zip(SOURCES, objs)]
    if verbose:
        for c in cmds:
            print(" ".join(c), flush=True)
    from concurrent.futures import ThreadPoolExecutor
    jobs = max(1, min(len(cmds), int(os.environ.get("MAX_JOBS", os.cpu_count() or 1)), 16))
    with ThreadPoolExecutor(jobs) as ex:
        res = list(ex.map(lambda c: subprocess.run(c, capture_output=True, text=True), cmds))
    for c, r in zip(cmds, res):
        if r.stdout or r.stderr:
            print(r.stdout + r.stderr, file=sys.stderr, flush=True)
        if r.returncode:
            raise subprocess.CalledProcessError(r.returncode, c)
    cmd = [hipcc, f"--offload-arch={ARCH}", "-shared", "-fPIC", *objs, "-o", lib + ".tmp",
           "-L", os.path.join(ROCM, "lib"), "-lrccl", "-Wl,-rpath," + os.path.join(ROCM, "lib")]
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    os.replace(lib + ".tmp", lib)
    with open(lib + ".id", "w") as fh:
        fh.write(sid + "\n")
    return lib


HOOKS = os.path.join(LIB_DIR, "libfs2_hooks.so")


def build_hooks(verbose: bool = False) -> str:
    """libfs2_hooks.so: fs2_pages.hip alone with -DFS2_TEST_HOOKS (test entry points
    of single kernels; the GPU tests load it beside libfs2.so)."""
    src = os.path.join(CSRC, "fs2_pages.hip")
    hid = hashlib.sha256(b"".join(open(os.path.join(CSRC, f), "rb").read()
                                  for f in ["fs2_pages.hip"] + sorted(HEADERS))).hexdigest()[:20]
    if os.path.exists(HOOKS) and built_id(HOOKS) == hid:
        return HOOKS
    cmd = [os.path.join(ROCM, "bin", "hipcc"), f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC",
           "-shared", "-ffp-contract=off", "-DFS2_TEST_HOOKS", "-I", os.path.join(ROCM, "include"),
           src, "-o", HOOKS + ".tmp"]
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    os.replace(HOOKS + ".tmp", HOOKS)
    with open(HOOKS + ".id", "w") as fh:
        fh.write(hid + "\n")
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
