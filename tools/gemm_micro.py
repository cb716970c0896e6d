"""GEMM micro-benchmark on C2 layer shapes (diagnostic; GPU).

Runs conv fwd / dgrad / wgrad of a few representative C2 layers `reps` times each
(packed weights cached) and prints TF/s from the library's HIP-event timing.
Meant to be run under rocprofv3 (--kernel-trace / --pmc) as a clean target.

usage: python tools/gemm_micro.py [reps] [ops]   ops: comma list of fwd,dgrad,wgrad,convt,convtd,convtw,small
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
    ks = ",".join(k["name"].split("<")[1].split(">")[0] for k in pr["kernels"])
    print(f"{name:34s} {pr['ms'] / reps * 1000:9.1f} us  {pr['flops'] / pr['ms'] / 1e9:7.1f} TF/s  [{ks}]", flush=True)


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    ops = (sys.argv[2] if len(sys.argv) > 2 else "fwd,dgrad,wgrad,convt,convtd,convtw,small").split(",")
    B = 64
    layers = [(128, 256, 64), (512, 1024, 16)]  # (cin, cout, H_in) of D convs k4s2p1
    if "deep" in ops:
        layers = [(1024, 2048, 8)]
    for cin, cout, H in layers:
        x = nhwc(B, cin, H, H)
        w = torch.nn.Parameter(torch.randn(cout, cin, 4, 4, device="cuda") * 0.02)
        dy = nhwc(B, cout, H // 2, H // 2)
        if "fwd" in ops:
            run(f"conv fwd   {cin}->{cout} @{H}", lambda: K.conv_fwd(x, w, G, cache=True), reps)
        if "dgrad" in ops:
            run(f"conv dgrad {cin}->{cout} @{H}", lambda: K.conv_dgrad(dy, w, G, tuple(x.shape), cache=True), reps)
        if "wgrad" in ops:
            run(f"conv wgrad {cin}->{cout} @{H}", lambda: K.conv_wgrad(x, dy, G, tuple(w.shape)), reps)
    for cin, cout, H in ([(2048, 1024, 4)] if "deep" in ops else [(256, 128, 32), (1024, 512, 8)]):  # G ConvT
        x = nhwc(B, cin, H, H)
        w = torch.nn.Parameter(torch.randn(cin, cout, 4, 4, device="cuda") * 0.02)
        dy = nhwc(B, cout, 2 * H, 2 * H)
        if "convt" in ops:
            run(f"convT fwd   {cin}->{cout} @{H}", lambda: K.conv_fwd(x, w, GT, cache=True), reps)
        if "convtd" in ops:
            run(f"convT dgrad {cin}->{cout} @{H}", lambda: K.conv_dgrad(dy, w, GT, tuple(x.shape), cache=True), reps)
        if "convtw" in ops:
            run(f"convT wgrad {cin}->{cout} @{H}", lambda: K.conv_wgrad(x, dy, GT, tuple(w.shape)), reps)
    if "small" in ops:
        x = nhwc(B, 128, 64, 64)
        w = torch.nn.Parameter(torch.randn(128, 3, 4, 4, device="cuda") * 0.02)
        run("convT fwd   128->3 @64 (G out)", lambda: K.conv_fwd(x, w, GT, nchw_out=True, cache=True), reps)
        img = torch.randn(B, 3, 128, 128, device="cuda")
        wd = torch.nn.Parameter(torch.randn(128, 3, 4, 4, device="cuda") * 0.02)
        dyd = nhwc(B, 128, 64, 64)
        run("conv fwd   3->128 @128 (D in)", lambda: K.conv_fwd(img, wd, G, cache=True), reps)
        run("conv dgrad 3->128 @128 (D in)",
            lambda: K.conv_dgrad(dyd, wd, G, tuple(img.shape), like=img, cache=True), reps)
        run("conv wgrad 3->128 @128 (D in)", lambda: K.conv_wgrad(img, dyd, G, tuple(wd.shape)), reps)


if __name__ == "__main__":
    main()
