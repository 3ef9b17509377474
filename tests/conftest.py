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
