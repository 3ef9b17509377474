"""CPU checks of the C ABI boundary: libfs2.so builds, loads without a GPU and
exports every entry point include/fs2.h declares; the ctypes structs match the
header layout; the library refuses to run without a device (no CPU path)."""
import ctypes as C
import os
import re

import numpy as np
import pytest

from conftest import REPO


def header_functions():
    src = open(os.path.join(REPO, "include", "fs2.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(fs2_[a-z0-9_]+)\s*\(", src)))


def test_build_and_exports():
    import build
    lib_path = build.build()
    lib = C.CDLL(lib_path)
    names = header_functions()
    assert len(names) >= 20
    for n in names:
        assert hasattr(lib, n), n


def test_ctypes_signatures_cover_header():
    from fast_slam_2 import _native
    assert sorted(n for n, _, _ in _native.SIGNATURES) == header_functions()


def test_struct_layout_matches_header():
    from fast_slam_2 import _native
    src = open(os.path.join(REPO, "include", "fs2.h")).read()
    for cname, py in [("fs2_config", _native.fs2_config), ("fs2_iter_stats", _native.fs2_iter_stats),
                      ("fs2_profile", _native.fs2_profile),
                      ("fs2_frontend_out", _native.fs2_frontend_out), ("fs2_mt_state", _native.fs2_mt_state)]:
        body = re.search(r"typedef struct %s \{(.*?)\} %s;" % (cname, cname), src, re.S).group(1)
        body = re.sub(r"/\*.*?\*/", "", body, flags=re.S)
        fields = []
        for decl in body.split(";"):
            decl = decl.strip()
            if not decl:
                continue
            names = decl.split(None, 1)[1]
            for nm in names.split(","):
                fields.append(re.sub(r"\[.*\]", "", nm).strip().lstrip("*"))
        assert [f for f, _ in py._fields_] == fields, cname


def test_defaults_are_reference_config():
    from fast_slam_2 import _native
    cfg = _native.default_config()
    assert cfg.num_particles == 20 and cfg.translation_noise == 0.0055
    assert cfg.rotation_noise == 0.001 and cfg.max_landmark_distance == 8.0
    assert list(cfg.measurement_noise) == [0.001, 0.0, 0.0, 0.001]
    assert list(cfg.init_landmark_cov) == [0.1, 0.0, 0.0, 0.1]
    assert cfg.weight_floor == 1e-5 and cfg.world_size == 1


def test_gaussian_taps_match_scipy_builder():
    from fast_slam_2 import _native
    from fast_slam_2.algorithms.line_filter import gaussian_taps
    lib = _native.load()
    for s in [0.1, 0.3, 1.0, 2.5]:
        ref, r = gaussian_taps(s)
        out = np.empty(64)
        rr = lib.fs2_gaussian_taps(s, 4.0, _native.dptr(out), 64)
        assert rr == r
        assert np.allclose(out[:2 * r + 1], ref, rtol=1e-14)


@pytest.mark.skipif(os.path.exists("/dev/kfd") and os.access("/dev/kfd", os.R_OK),
                    reason="a GPU is present")
def test_no_cpu_fallback():
    import fast_slam_2
    from fast_slam_2._native import FS2Error
    with pytest.raises(FS2Error):
        fast_slam_2.FastSLAM2(10)
    with pytest.raises(FS2Error):
        fast_slam_2.LineFilter.filter(np.zeros((4, 2)))


def test_build_id_is_source_hash():
    """fs2_build_id names the sources the library was built from (build.source_id)."""
    import build
    from fast_slam_2 import _native
    build.build()
    assert _native.load().fs2_build_id().decode() == build.source_id()


def test_struct_sizes_match_c_compiler():
    """sizeof / offsetof of the ABI structs as gcc lays out include/fs2.h equal the
    ctypes mirrors (a field added on one side only would shift everything after it)."""
    import subprocess
    import tempfile
    from fast_slam_2 import _native
    structs = [("fs2_config", _native.fs2_config), ("fs2_iter_stats", _native.fs2_iter_stats),
               ("fs2_profile", _native.fs2_profile), ("fs2_frontend_out", _native.fs2_frontend_out),
               ("fs2_mt_state", _native.fs2_mt_state)]
    lines = ['#include <stdio.h>', '#include <stddef.h>', '#include "fs2.h"', "int main(void) {"]
    for cname, py in structs:
        lines.append(f'printf("{cname} %zu\\n", sizeof({cname}));')
        for f, _ in py._fields_:
            lines.append(f'printf("{cname}.{f} %zu\\n", offsetof({cname}, {f}));')
    lines.append("return 0; }")
    with tempfile.TemporaryDirectory() as d:
        src, exe = os.path.join(d, "l.c"), os.path.join(d, "l")
        open(src, "w").write("\n".join(lines))
        subprocess.run(["gcc", "-I", os.path.join(REPO, "include"), src, "-o", exe], check=True)
        out = dict(l.rsplit(" ", 1) for l in subprocess.run([exe], capture_output=True, text=True,
                                                             check=True).stdout.splitlines())
    for cname, py in structs:
        assert int(out[cname]) == C.sizeof(py), cname
        for f, _ in py._fields_:
            assert int(out[f"{cname}.{f}"]) == getattr(py, f).offset, (cname, f)
