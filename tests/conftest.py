import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "fast-slam_amd")
GOLDEN = os.path.join(REPO, "tests", "golden")
for p in (REPO, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libfs2 on cuda:0)")
    config.addinivalue_line("markers", "slow: longer CPU test")

# fast-slam_amd/build.py is importable as `build`
if os.path.join(REPO, "fast-slam_amd") not in sys.path:
    sys.path.insert(0, os.path.join(REPO, "fast-slam_amd"))


def pytest_sessionstart(session):
    """Refuse a libfs2.so built from other sources than this tree's (the GPU box
    runs the prebuilt library that travels with the snapshot)."""
    import build
    lib = os.path.join(PKG, "lib", "libfs2.so")
    if not os.path.exists(lib):
        return                      # test_abi builds it; GPU tests fail loudly without it
    want = build.source_id()
    # the id is a string constant of the library (fs2_build_id); look for it in the
    # file rather than loading the library before torch's HIP runtime
    if want.encode() not in open(lib, "rb").read():
        import pytest
        pytest.exit(f"libfs2.so was not built from this tree's sources (id {want} not in it): "
                    f"run `python fast-slam_amd/build.py`", returncode=3)
