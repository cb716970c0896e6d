#!/usr/bin/env python3
"""Wide dense layer (arch 1's G input Linear as a 1x1 conv over a 1x1 map) at C4's shape:
forward and weight + bias gradient, each timed as HIP-graph replays (diagnostic; GPU).  Run
against variant builds (RGAN_LIB=..., tools/build_variant.py).

usage: [N3_EAGER=1] python tools/dense_micro.py [reps]   (N3_EAGER: eager launches, no timing)
"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
from relativisticgan_amd import kernels as K  # noqa: E402
from bn_small_micro import graph_time  # noqa: E402

DEV = "cuda"


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 50
    torch.manual_seed(0)
    g = K.ConvGeom(1, 1, 0, False)
    for B, C, N in ((32, 128, 8192), (64, 128, 8192)):
        x = torch.randn(B, C, 1, 1, device=DEV)
        w = torch.randn(N, C, 1, 1, device=DEV) * 0.05
        b = torch.randn(N, device=DEV)
        y = torch.empty(B, N, 1, 1, device=DEV)
        dy = torch.randn(B, N, 1, 1, device=DEV)
        dw, db = torch.zeros(N, C, 1, 1, device=DEV), torch.zeros(N, device=DEV)

        def fwd():
            K.conv_fwd(x, w, g, bias=b, act="none", out=y, cache=True)

        def wgrad():
            K.conv_wgrad(x, dy, g, w.shape, with_bias=True, out=dw, out_bias=db)
        if os.environ.get("N3_EAGER"):  # plain launches, for rocprofv3 --pmc
            for _ in range(reps):
                fwd()
                wgrad()
            torch.cuda.synchronize()
            continue
        print(f"B={B} C={C} N={N}: fwd {graph_time(fwd, reps):7.2f} us  wgrad+bias {graph_time(wgrad, reps):7.2f} us",
              flush=True)


if __name__ == "__main__":
    main()
