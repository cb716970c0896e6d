"""GEMM micro-benchmark on the C1 (RaLSGAN 64², B=32 per step, h=128) layer shapes (diagnostic; GPU).

Every GEMM call of a C1 iteration at its own shape (the batched D pass at 2B = 64), timed by
the library's HIP events around the GEMM launch (split-K reduces excluded), `reps` times.
Run against variant builds (RGAN_LIB=tools/variants/librgan_X.so) to A/B a GEMM parameter.

usage: python tools/c1_gemm_micro.py [reps]
"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from relativisticgan_amd import kernels as K  # noqa: E402

G = K.ConvGeom(4, 2, 1, False)
GT = K.ConvGeom(4, 2, 1, True)


def nhwc(*s):
    return torch.randn(*s, device="cuda").contiguous(memory_format=torch.channels_last)


def run(name, fn, reps):
    fn()
    torch.cuda.synchronize()
    K.profile_begin(reps + 8)
    for _ in range(reps):
        fn()
    pr = K.profile_end()
    ks = ",".join(k["name"].split("<")[1].split(">")[0] if "<" in k["name"] else k["name"] for k in pr["kernels"])
    us = pr["ms"] / reps * 1000
    print(f"{name:40s} {us:8.1f} us  {pr['flops'] / pr['ms'] / 1e9:7.1f} TF/s  [{ks}]", flush=True)
    return us


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    tot = 0.0
    for B in (64, 32):
        for cin, cout, H in ((128, 256, 32), (256, 512, 16), (512, 1024, 8)):  # D middle convs
            x = nhwc(B, cin, H, H)
            w = torch.nn.Parameter(torch.randn(cout, cin, 4, 4, device="cuda") * 0.02)
            dy = nhwc(B, cout, H // 2, H // 2)
            tot += run(f"D fwd   {cin}->{cout} @{H} B{B}", lambda: K.conv_fwd(x, w, G, cache=True), reps)
            tot += run(f"D dgrad {cin}->{cout} @{H} B{B}", lambda: K.conv_dgrad(dy, w, G, tuple(x.shape), cache=True),
                       reps)
            if B == 64:
                tot += run(f"D wgrad {cin}->{cout} @{H} B{B}", lambda: K.conv_wgrad(x, dy, G, tuple(w.shape)), reps)
    B = 32
    for cin, cout, H in ((1024, 512, 4), (512, 256, 8), (256, 128, 16)):  # G middle ConvTs
        x = nhwc(B, cin, H, H)
        w = torch.nn.Parameter(torch.randn(cin, cout, 4, 4, device="cuda") * 0.02)
        dy = nhwc(B, cout, 2 * H, 2 * H)
        tot += run(f"G fwd   {cin}->{cout} @{H} B{B}", lambda: K.conv_fwd(x, w, GT, cache=True), reps)
        tot += run(f"G dgrad {cin}->{cout} @{H} B{B}", lambda: K.conv_dgrad(dy, w, GT, tuple(x.shape), cache=True),
                   reps)
        tot += run(f"G wgrad {cin}->{cout} @{H} B{B}", lambda: K.conv_wgrad(x, dy, GT, tuple(w.shape)), reps)
    print(f"sum of the shapes above: {tot:.1f} us", flush=True)


if __name__ == "__main__":
    main()
