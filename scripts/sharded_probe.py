#!/usr/bin/env python3
"""The sharded path at config-3 size with G ranks as threads on one GPU (in-process
transport), for rocprofv3 --kernel-trace: python3 scripts/sharded_probe.py [G] [scans]"""
import os
import sys
import types

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "fast-slam_amd"))


def main():
    import torch
    import bench
    G = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    scans = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    torch.cuda.set_device(0)
    args = types.SimpleNamespace(seed=0)
    out = bench.sharded_local(args, 500, 1_000_000, G=G, scans=scans, warm=2)
    print(out, flush=True)


if __name__ == "__main__":
    main()
