"""The oracle under AddressSanitizer + UndefinedBehaviorSanitizer: the golden
tests of the C restatement (tests/test_oracle_golden.py) run against
oracle/_build/liboracle_san.so (`make -C oracle sanitize`) in a python with
libasan preloaded; any out-of-bounds access, use-after-free or undefined
behaviour aborts the run."""
import os
import subprocess
import sys

import pytest

from conftest import REPO


def test_oracle_golden_under_asan_ubsan():
    r = subprocess.run(["make", "-s", "-C", os.path.join(REPO, "oracle"), "sanitize"], capture_output=True,
                       text=True)
    if r.returncode != 0:
        pytest.skip(f"sanitizer build unavailable: {r.stderr[-400:]}")
    asan = subprocess.run(["gcc", "-print-file-name=libasan.so"], capture_output=True, text=True).stdout.strip()
    ubsan = subprocess.run(["gcc", "-print-file-name=libubsan.so"], capture_output=True, text=True).stdout.strip()
    env = dict(os.environ, LD_PRELOAD=f"{asan} {ubsan}",
               ASAN_OPTIONS="detect_leaks=0:abort_on_error=1:halt_on_error=1",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1",
               ORACLE_LIB=os.path.join(REPO, "oracle", "_build", "liboracle_san.so"), OMP_NUM_THREADS="2")
    r = subprocess.run([sys.executable, "-m", "pytest", "-q", "-x", "-p", "no:cacheprovider",
                        os.path.join(REPO, "tests", "test_oracle_golden.py"),
                        os.path.join(REPO, "tests", "test_frontend_oracle.py")],
                       capture_output=True, text=True, env=env, cwd=REPO, timeout=900)
    assert r.returncode == 0, (r.stdout[-3000:], r.stderr[-3000:])
    assert "passed" in r.stdout
