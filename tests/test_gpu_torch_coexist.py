"""One HIP runtime per process (fast_slam_2/_native.py _share_torch_hip_runtime).
A PyTorch-ROCm wheel ships its own HIP and HSA runtimes; libfs2 links the system
one.  Loaded first, libfs2 used to bring /opt/rocm's runtime in and a later
`import torch` then loaded the wheel's copy beside it, after which PyTorch found
no GPU ("No HIP GPUs are available").  In a fresh process (the order matters, so
not in this test process): the shim, a handle whose record pool grows in place,
then PyTorch's first CUDA call and a tensor op."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SCRIPT = r"""
import sys
import numpy as np
import fast_slam_2
assert "torch" not in sys.modules
N, L = 100000, 32
f = fast_slam_2.FastSLAM2(N, rng="device", seed=1, landmark_capacity=L + 40, verbose=False,
                          record_pool=N * L + 2 * N)
x = np.zeros(N); w = np.full(N, 1.0 / N)
lm = np.zeros((N, L, 6)); lm[:, :, 0] = np.arange(L) * 7.0; lm[:, :, 2] = lm[:, :, 5] = 0.1
f.set_state(x, x, x, w, np.full(N, L, np.int32), lm)
for s in range(6):
    ms = np.array([[100.0 + 10.0 * s + 20.0 * k, 0.25 * k] for k in range(4)])
    pose, st = f.step(0.0, 0.03, ms)
assert st.pool_records > N * L + 2 * N, st.pool_records      # grew in place
import torch
assert torch.cuda.is_available() and torch.cuda.device_count() >= 1
t = torch.arange(1 << 20, device="cuda", dtype=torch.float64)
assert float(t.sum()) == float((1 << 20) * ((1 << 20) - 1) / 2)
f.close()
print("ok", st.pool_records, st.pool_copies)
"""


@pytest.mark.timeout(180)
def test_torch_initialises_after_a_growing_handle():
    env = dict(os.environ)
    env["PYTHONPATH"] = os.pathsep.join([os.path.join(ROOT, "fast-slam_amd"), env.get("PYTHONPATH", "")])
    r = subprocess.run([sys.executable, "-c", SCRIPT], cwd=ROOT, env=env, capture_output=True, text=True,
                       timeout=170)
    assert r.returncode == 0 and r.stdout.startswith("ok"), (r.returncode, r.stdout[-2000:], r.stderr[-4000:])
