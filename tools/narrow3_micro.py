#!/usr/bin/env python3
"""conv3_narrow_out at C4's shapes (diagnostic; GPU): G's image layer (64 -> 3 channels, 3x3,
32 x 32, NCHW tanh out) and D's input layer's data gradient (64-channel dy -> 3-channel image),
batch 32, plus D's input layer forward (3 -> C), each timed as HIP-graph replays of REPS calls (GPU time per call, launch gaps
included).  Run against variant builds (RGAN_LIB=..., tools/build_variant.py).

usage: [N3_EAGER=1] python tools/narrow3_micro.py [reps]   (N3_EAGER: eager launches, no timing)
"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from relativisticgan_amd import kernels as K  # noqa: E402

sys.path.insert(0, os.path.join(ROOT, "tools"))
from bn_small_micro import graph_time  # noqa: E402

DEV = "cuda"


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 50
    torch.manual_seed(0)
    g = K.ConvGeom(3, 1, 1, False)
    s = torch.tensor([0.5], device=DEV)
    for B, C, H in ((32, 64, 32), (64, 64, 32), (32, 128, 32)):
        x = K.empty_nhwc(B, C, H, H, DEV).normal_()
        w = torch.randn(3, C, 3, 3, device=DEV) * 0.1
        b = torch.randn(3, device=DEV)
        y = torch.empty(B, 3, H, H, device=DEV)
        w_in = torch.randn(C, 3, 3, 3, device=DEV) * 0.1
        dy = K.empty_nhwc(B, C, H, H, DEV).normal_()
        dx = K.empty_nhwc(B, 3, H, H, DEV)

        def fwd():
            K.conv_fwd(x, w, g, bias=b, act="tanh", wscale=s, nchw_out=True, out=y)

        def dgrad():
            K.conv_dgrad(dy, w_in, g, (B, 3, H, H), wscale=s, out=dx)

        img = torch.randn(B, 3, H, H, device=DEV)
        yin = K.empty_nhwc(B, C, H, H, DEV)
        bin_ = torch.randn(C, device=DEV)

        def infwd():  # D's input layer forward (3 -> C channels over the NCHW image)
            K.conv_fwd(img, w_in, g, bias=bin_, act="lrelu", alpha=0.2, wscale=s, out=yin, cache=True)
        if os.environ.get("N3_EAGER"):  # plain launches, for rocprofv3 --pmc
            for _ in range(reps):
                fwd()
                dgrad()
                infwd()
            torch.cuda.synchronize()
            continue
        mb = B * H * H * C * 4 / 1e6
        tf, td, ti = graph_time(fwd, reps), graph_time(dgrad, reps), graph_time(infwd, reps)
        print(f"B={B} C={C} H={H}: fwd {tf:7.2f} us ({mb / tf * 1e3:6.0f} GB/s of x)  dgrad {td:7.2f} us  "
              f"input-layer fwd {ti:7.2f} us", flush=True)


if __name__ == "__main__":
    main()
