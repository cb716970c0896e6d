"""Drift probe (diagnostic, GPU): free-running iterations of a small config on the GPU and in
the oracle at fp32 and fp64; prints per-step relative errD/errG gaps to the fp64 run."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tests.test_drift_gpu import CFGS, gpu_traj, oracle_traj  # noqa: E402


def main():
    names = sys.argv[1:] or list(CFGS)
    for name in names:
        o64 = oracle_traj(name, torch.float64, 8)
        o32 = oracle_traj(name, torch.float32, 8)
        g = gpu_traj(name)
        den = np.abs(o64) + 1e-3
        do, dg = np.abs(o32 - o64) / den, np.abs(g - o64) / den
        print(name)
        for i in range(12):
            print(f"  it{i:3d} oracle32 {do[i, 0]:.2e} {do[i, 1]:.2e}   gpu {dg[i, 0]:.2e} {dg[i, 1]:.2e}")
        print(f"  mean oracle32 {do.mean():.2e} gpu {dg.mean():.2e}", flush=True)


if __name__ == "__main__":
    main()
