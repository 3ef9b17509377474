import sys, os, json, types
sys.path.insert(0, os.getcwd()); sys.path.insert(0, os.path.join(os.getcwd(), "fast-slam_amd"))
import torch
torch.cuda.set_device(0)
import bench
args = types.SimpleNamespace(seed=0)
r = bench.appended_maps(args, 500, 1_000_000)
print(json.dumps({k: r[k] for k in ("value", "ms_per_scan", "resamples", "kernel_ms", "pool", "pages_opened_per_particle_scan")}))
