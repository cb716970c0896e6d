#!/usr/bin/env python3
"""bench.py's hbm_kernels table alone (diagnostic; GPU): achieved GB/s of the HBM-bound kernels
at a workload's shapes.  usage: python tools/hbm_micro.py [WORKLOAD] [reps]  (RGAN_LIB for variants)"""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from relativisticgan_amd import kernels as K  # noqa: E402

if __name__ == "__main__":
    wl = sys.argv[1] if len(sys.argv) > 1 else "C3"
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    torch.cuda.set_device(0)
    for k in bench.hbm_kernels(wl, K, reps=reps)["kernels"]:
        print(f"{k['kernel'][:60]:60s} {k['us']:9.1f} us {k['GB_s']:8.1f} GB/s")
