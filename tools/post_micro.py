"""Micro-benchmark of the producer post-ops (kernels.Post / rgan_conv_post) on the C1 and C3
shapes that use them: the GEMM with the post-op vs the GEMM alone + the separate pass it
replaces (act_backward / bn_backward_sums), HIP-event timed (diagnostic; GPU).

usage: python tools/post_micro.py [reps]
"""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from relativisticgan_amd import kernels as K  # noqa: E402


def nhwc(*s):
    return torch.randn(*s, device="cuda").contiguous(memory_format=torch.channels_last)


def timed(fn, reps):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1000.0


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    G = K.ConvGeom(4, 2, 1, False)
    GT = K.ConvGeom(4, 2, 1, True)
    for B, H, name in ((32, 32, "C1"), (32, 128, "C3")):
        # G's image-layer data gradient as a 1x1 GEMM over the patch matrix, post = G's last BN (mode 2)
        C = 128
        dimg = torch.randn(B, 3, 2 * H, 2 * H, device="cuda")
        w = torch.randn(C, 3, 4, 4, device="cuda") * 0.05
        Xg = K.patches_k4s2(dimg)
        Wp = K.PATCHW.get(torch.nn.Parameter(w), True)
        y = nhwc(B, C, H, H)
        stats = torch.cat([torch.zeros(1, C, device="cuda"), torch.ones(1, C, device="cuda")], 1)
        gam, bet = torch.ones(C, device="cuda"), torch.zeros(C, device="cuda")

        def plain():
            da = K.conv_fwd(Xg, Wp, K.G1X1, cache=False)
            K.bn_backward_sums(da, y, stats[0], gam, bet, "relu", 0.0)

        def fused():
            p = K.Post(2, "relu", 0.0, y, stats=stats, gamma=gam, beta=bet)
            K.conv_fwd(Xg, Wp, K.G1X1, cache=False, post=p)
            assert p.fused

        print(f"{name} G image dgrad + BN sums: plain {timed(plain, reps):8.1f} us   fused {timed(fused, reps):8.1f} us",
              flush=True)
        # D's second conv's data gradient, post = D's first-layer LeakyReLU (mode 1)
        x1 = nhwc(2 * B, 128, H, H)
        w2 = torch.nn.Parameter(torch.randn(256, 128, 4, 4, device="cuda") * 0.02)
        dy2 = nhwc(2 * B, 256, H // 2, H // 2)
        a1 = nhwc(2 * B, 128, H, H)

        def plain1():
            da = K.conv_dgrad(dy2, w2, G, tuple(x1.shape), cache=True)
            K.act_backward(da, a1, "lrelu", 0.2)

        def fused1():
            p = K.Post(1, "lrelu", 0.2, a1)
            K.conv_dgrad(dy2, w2, G, tuple(x1.shape), cache=True, post=p)
            assert p.fused

        print(f"{name} D conv2 dgrad + lrelu': plain {timed(plain1, reps):8.1f} us   fused {timed(fused1, reps):8.1f} us",
              flush=True)
        # G's middle ConvT data gradient, post = the BN of the layer below (mode 2)
        cin, cout, h = (512, 256, H // 8)
        x = nhwc(B, cin, h, h)
        wt = torch.nn.Parameter(torch.randn(cin, cout, 4, 4, device="cuda") * 0.02)
        dyt = nhwc(B, cout, 2 * h, 2 * h)
        yb = nhwc(B, cin, h, h)
        st = torch.cat([torch.zeros(1, cin, device="cuda"), torch.ones(1, cin, device="cuda")], 1)
        g2, b2 = torch.ones(cin, device="cuda"), torch.zeros(cin, device="cuda")

        def plain2():
            da = K.conv_dgrad(dyt, wt, GT, tuple(x.shape), cache=True)
            K.bn_backward_sums(da, yb, st[0], g2, b2, "relu", 0.0)

        def fused2():
            p = K.Post(2, "relu", 0.0, yb, stats=st, gamma=g2, beta=b2)
            K.conv_dgrad(dyt, wt, GT, tuple(x.shape), cache=True, post=p)
            assert p.fused

        print(f"{name} G ConvT {cin}->{cout} dgrad + BN sums: plain {timed(plain2, reps):8.1f} us   "
              f"fused {timed(fused2, reps):8.1f} us", flush=True)


if __name__ == "__main__":
    main()
