"""Image-layer (narrow) kernel micro-benchmark at the C3 shard's shapes (diagnostic; GPU).

D's image conv (3 -> 128, k4 s2 p1, 256^2 -> 128^2, conv_narrow_in_mfma), G's image convT
(128 -> 3, 128^2 -> 256^2, convt2_narrow_mfma) and their data gradients, B = 32.  Prints
time per launch (library HIP events) and HBM-side algorithmic GB/s (image + 128-channel side
once each).  usage: python tools/narrow_micro.py [reps] [B]
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from relativisticgan_amd import kernels as K  # noqa: E402


def run(name, fn, reps, nbytes):
    fn()
    torch.cuda.synchronize()
    K.profile_begin(reps + 8)
    for _ in range(reps):
        fn()
    pr = K.profile_end()
    us = pr["ms"] / reps * 1000
    print(f"{name:28s} {us:8.1f} us  {nbytes / us / 1e3:7.1f} GB/s  {pr['flops'] / pr['ms'] / 1e9:6.1f} TF/s",
          flush=True)


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    B = int(sys.argv[2]) if len(sys.argv) > 2 else 32
    S, C = 256, 128
    g = K.ConvGeom(4, 2, 1, False)
    gt = K.ConvGeom(4, 2, 1, True)
    img = torch.rand(B, 3, S, S, device="cuda") * 2 - 1
    wd = torch.nn.Parameter(torch.randn(C, 3, 4, 4, device="cuda") * 0.02)
    wg = torch.nn.Parameter(torch.randn(C, 3, 4, 4, device="cuda") * 0.02)
    h = torch.randn(B, C, S // 2, S // 2, device="cuda").contiguous(memory_format=torch.channels_last)
    nb = 4 * (B * 3 * S * S + B * C * (S // 2) ** 2)
    run("D image conv fwd", lambda: K.conv_fwd(img, wd, g, act="lrelu", alpha=0.2, cache=True), reps, nb)
    run("D image conv dgrad", lambda: K.conv_dgrad(h, wd, g, tuple(img.shape), like=img, cache=True), reps, nb)
    run("G image convT fwd", lambda: K.conv_fwd(h, wg, gt, act="tanh", nchw_out=True, cache=True), reps, nb)
    run("G image convT dgrad", lambda: K.conv_dgrad(img, wg, gt, tuple(h.shape), cache=True), reps, nb)


if __name__ == "__main__":
    main()
