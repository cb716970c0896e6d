"""Spectral-norm power iteration micro-benchmark at the C5 D's layer shapes (diagnostic; GPU).

usage: python tools/sn_micro.py [reps]   (RGAN_LIB selects an experiment build)
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from relativisticgan_amd import kernels as K  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    torch.manual_seed(0)
    chans = [3, 128, 256, 512, 1024]
    layers = []
    nbytes = 0
    for cin, cout in zip(chans[:-1], chans[1:]):
        w = torch.randn(cout, cin, 4, 4, device="cuda") * 0.02
        layers.append((w, torch.randn(cout, device="cuda"), torch.randn(cin * 16, device="cuda"), False))
        nbytes += w.numel() * 4
    w = torch.randn(1, 1024, 4, 4, device="cuda") * 0.02
    layers.append((w, torch.randn(1, device="cuda"), torch.randn(1024 * 16, device="cuda"), False))
    nbytes += w.numel() * 4
    K.spectral_power_batch(layers)
    torch.cuda.synchronize()
    # cold: a 512 MB write between calls evicts W from L2 and the MALL, as in a training step
    flush = torch.empty(128 * 1024 * 1024, device="cuda")
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for e0, e1 in ev:
        flush.fill_(1.0)
        e0.record()
        K.spectral_power_batch(layers)
        e1.record()
    torch.cuda.synchronize()
    us = sum(e0.elapsed_time(e1) for e0, e1 in ev) / reps * 1000
    print(f"spectral power batch (C5 D, {nbytes / 1e6:.1f} MB of W): {us:8.1f} us  {2 * nbytes / us / 1e3:7.1f} GB/s",
          flush=True)


if __name__ == "__main__":
    main()
