"""Which libfs2 / HIP use before PyTorch's first CUDA call keeps PyTorch from
starting in the same process?  Each variant runs in a fresh process:
  torch_first   torch.cuda.init(), then a libfs2 handle (what bench.py does)
  philox        a plain libfs2 HIP call (fs2_debug_philox: malloc, kernel, copy), then torch
  handle        a libfs2 handle (pools in reserved ranges), then torch
  reserve       hipMemAddressReserve / Free through ctypes on libamdhip64, then torch
  create        hipMemCreate / Release through ctypes, then torch
Prints one line per variant.  Run on the GPU box."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PRE = "import sys; sys.path.insert(0, %r)\n" % os.path.join(ROOT, "fast-slam_amd")
TORCH = ("import torch\nok = torch.cuda.is_available() and torch.cuda.device_count() > 0\n"
         "t = torch.ones(4, device='cuda') if ok else None\nprint('torch_ok' if ok else 'torch_FAIL')\n")
HIP = ("import ctypes as C\nhip = C.CDLL('libamdhip64.so')\n")
V = {
    "torch_first": "import torch\ntorch.cuda.init()\nimport fast_slam_2\nf = fast_slam_2.FastSLAM2(1000, rng='device', verbose=False)\nf.close()\n" + TORCH,
    "philox": "import numpy as np, ctypes as C\nfrom fast_slam_2 import _native as nat\nlib = nat.load()\n"
              "ctr = np.zeros(16, np.uint32); key = np.zeros(8, np.uint32); out = np.zeros(16, np.uint32)\n"
              "assert lib.fs2_debug_philox(0, 4, ctr.ctypes.data, key.ctypes.data, out.ctypes.data) == 0\n" + TORCH,
    "handle": "import fast_slam_2\nf = fast_slam_2.FastSLAM2(1000, rng='device', verbose=False)\nf.close()\n" + TORCH,
    "reserve": HIP + "p = C.c_void_p()\nassert hip.hipMemAddressReserve(C.byref(p), C.c_size_t(1 << 30), C.c_size_t(0), None, C.c_ulonglong(0)) == 0\n"
               "assert hip.hipMemAddressFree(p, C.c_size_t(1 << 30)) == 0\n" + TORCH,
    "malloc": HIP + "p = C.c_void_p()\nassert hip.hipMalloc(C.byref(p), C.c_size_t(1 << 20)) == 0\nhip.hipFree(p)\n" + TORCH,
}
for name, code in V.items():
    r = subprocess.run([sys.executable, "-c", PRE + code], capture_output=True, text=True, timeout=120)
    last = (r.stdout.strip().splitlines() or [""])[-1]
    err = [l for l in r.stderr.strip().splitlines() if "amdgpu.ids" not in l][-1:]
    print(f"{name:12s} rc={r.returncode} {last} {err[0][:160] if err else ''}", flush=True)
