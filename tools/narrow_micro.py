"""Narrow ConvTranspose2d micro-benchmark (diagnostic; GPU): G's image layer (128 -> 3,
32x32 -> 64x64, tanh) and D's image-layer data gradient (the same ConvT shape, no act) at
C1 / C2 batch sizes (NARROW_SHAPE=C3: the 256^2 shard's), each launch sequence (narrow kernel + split reduce) timed alone with
HIP events.  Run against variant builds (RGAN_LIB=..., tools/build_variant.py).

usage: python tools/narrow_micro.py [reps]
"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from relativisticgan_amd import kernels as K  # noqa: E402

SHAPES = [(32, 128, 32, 32), (64, 128, 32, 32), (64, 128, 64, 64), (32, 64, 32, 32)]
if os.environ.get("NARROW_SHAPE") == "C3":  # G's 256^2 image layer at the C3 shard (32 x 128 x 128^2)
    SHAPES = [(32, 128, 128, 128)]


def one(fn, reps):
    fn()
    torch.cuda.synchronize()
    tot = 0.0
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        torch.cuda.synchronize()
        tot += a.elapsed_time(b)
    return tot / reps * 1000.0


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 30
    gt = K.ConvGeom(4, 2, 1, True)
    tot = 0.0
    for B, C, H, W in SHAPES:
        x = K.empty_nhwc(B, C, H, W, "cuda").normal_()
        w = torch.randn(C, 3, 4, 4, device="cuda") * 0.05
        t1 = one(lambda: K.conv_fwd(x, w, gt, act="tanh", cache=True), reps)
        ref = torch.nn.functional.conv_transpose2d(x.double(), w.double(), stride=2, padding=1).tanh()
        err = (K.conv_fwd(x, w, gt, act="tanh", cache=True).double() - ref).abs().max().item()
        tot += t1
        print(f"{str((B, C, H, W)):20s} convT->3 {t1:6.1f} us  max err {err:.2e}", flush=True)
    print(f"sum {tot:.1f} us")


if __name__ == "__main__":
    main()
