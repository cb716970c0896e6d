"""G's first layer: the fused kernels (rgan_g1_fwd_bn, rgan_g1_wgrad) vs the GEMM + BatchNorm
launches they replace, per call at the BASELINE shapes, HIP events around single calls after a
sync (diagnostic; GPU).  usage: python tools/g1_micro.py [reps]"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from relativisticgan_amd import kernels as K  # noqa: E402


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
    g = K.ConvGeom(4, 1, 0, True)
    for name, B, cout in (("C1", 32, 1024), ("C2", 64, 2048), ("C3", 32, 4096)):
        z = torch.randn(B, 128, 1, 1, device="cuda")
        w = torch.nn.Parameter(torch.randn(128, cout, 4, 4, device="cuda") * 0.05)
        gam, bet = torch.ones(cout, device="cuda"), torch.zeros(cout, device="cuda")
        rm, rv = torch.zeros(cout, device="cuda"), torch.ones(cout, device="cuda")
        dy = K.empty_nhwc(B, cout, 4, 4, "cuda").normal_()

        def fused():
            K.g1_fwd_bn(z, w, gam, bet, 1e-5, 0.1, rm, rv, None, "relu", 0.0)

        def gemm():
            y = K.conv_fwd(z, w, g, cache=True)
            st = K.bn_stats(y, 1e-5, 0.1, rm, rv)
            K.bn_apply(y, st, gam, bet, "relu", 0.0)

        tf, tg = one(fused, reps), one(gemm, reps)
        wf = one(lambda: K.g1_wgrad(z, dy, tuple(w.shape)), reps)
        wg = one(lambda: K.conv_wgrad(z, dy, g, tuple(w.shape)), reps)
        print(f"{name} B{B} Cout {cout}: fwd+BN fused {tf:6.1f} us vs GEMM+BN {tg:6.1f} us | wgrad {wf:6.1f} vs {wg:6.1f} us",
              flush=True)


if __name__ == "__main__":
    main()
