"""BatchNorm apply / backward-apply micro-benchmark on the C1 (64², B=32 per step, h=128)
activation shapes, each launch timed alone (diagnostic; GPU): HIP events around single
launches separated by a device sync, so the number is one launch's latency as a training step
sees it, not back-to-back throughput.  Run against variant builds (RGAN_LIB=..., a patch of the
apply grid constants in bn_act.hip built by tools/build_variant.py).

usage: python tools/bn_c1_micro.py [reps]
"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from relativisticgan_amd import kernels as K  # noqa: E402

SHAPES = [(64, 256, 16, 16), (64, 512, 8, 8), (64, 1024, 4, 4), (32, 1024, 4, 4), (32, 512, 8, 8),
          (32, 256, 16, 16), (32, 128, 32, 32)]


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
    tot = 0.0
    for B, C, H, W in SHAPES:
        y = K.empty_nhwc(B, C, H, W, "cuda").normal_()
        g = K.empty_nhwc(B, C, H, W, "cuda").normal_()
        gam, bet = torch.ones(C, device="cuda"), torch.zeros(C, device="cuda")
        st2 = torch.cat([torch.zeros(2, C, device="cuda"), torch.ones(2, C, device="cuda")], 1)
        out = torch.empty_like(y)
        t1 = one(lambda: K.bn_apply(y, st2[0], gam, bet, "lrelu", 0.2, out=out), reps)
        t2 = one(lambda: K.bn_apply_segments(y, st2, gam, bet, "lrelu", 0.2, out=out), reps)
        sums = torch.zeros(2 * C, dtype=torch.float64, device="cuda")
        t3 = one(lambda: K.bn_backward_apply(g, y, st2[0], gam, bet, "none", 0.0, sums, B * H * W, out=out), reps)
        tot += t1 + t2 + t3
        print(f"{str((B, C, H, W)):20s} apply {t1:6.1f} us  apply2 {t2:6.1f} us  bwd_apply {t3:6.1f} us", flush=True)
    print(f"sum {tot:.1f} us")


if __name__ == "__main__":
    main()
