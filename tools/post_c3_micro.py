"""Micro-benchmark of D's data-gradient GEMMs at the C3 shapes (RaLSGAN 256^2, h=128, the
batched D step: 2B = 64 rows of the batch) with and without the producer post-op in the
epilogue (gemm_post<1>: mode 1 = D's first-layer LeakyReLU', mode 2 = the lower layer's
BatchNorm backward sums).  Prints per shape: plain dgrad GEMM, dgrad + post, their TF/s
(algorithmic conv FLOPs), and the epilogue's extra time.  HIP-event timed (diagnostic; GPU).

usage: python tools/post_c3_micro.py [reps] [B2]
"""
import os
import sys

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
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    B2 = int(sys.argv[2]) if len(sys.argv) > 2 else 64
    G = K.ConvGeom(4, 2, 1, False)
    h, S = 128, 256
    tot_plain = tot_post = 0.0
    # D layer k: cin = h 2^(k-1) at S / 2^k -> cout = 2 cin at S / 2^(k+1); its dgrad writes the
    # layer-below activation gradient (cin channels at S / 2^k), post = that layer's act' / BN
    for k in range(1, 6):
        cin, H = h << (k - 1), S >> k
        cout = 2 * cin
        x = nhwc(B2, cin, H, H)
        w = torch.nn.Parameter(torch.randn(cout, cin, 4, 4, device="cuda") * 0.02)
        dy = nhwc(B2, cout, H // 2, H // 2)
        a = nhwc(B2, cin, H, H)
        flops = 2.0 * B2 * cin * cout * 16 * (H // 2) ** 2
        if k == 1:
            post = lambda: K.Post(1, "lrelu", 0.2, a)  # noqa: E731
        else:
            st = torch.cat([torch.zeros(1, cin, device="cuda"), torch.ones(1, cin, device="cuda")], 1)
            gam, bet = torch.ones(cin, device="cuda"), torch.zeros(cin, device="cuda")
            post = lambda: K.Post(2, "lrelu", 0.2, a, stats=st, gamma=gam, beta=bet)  # noqa: E731

        def plain():
            K.conv_dgrad(dy, w, G, tuple(x.shape), cache=True)

        def fused():
            p = post()
            K.conv_dgrad(dy, w, G, tuple(x.shape), cache=True, post=p)
            assert p.fused

        tp, tf = timed(plain, reps), timed(fused, reps)
        tot_plain += tp
        tot_post += tf
        print(f"D dgrad {cin:5d}->{cout:5d} @ {H:3d}: plain {tp:8.1f} us {flops / tp / 1e6:6.1f} TF/s   "
              f"post {tf:8.1f} us {flops / tf / 1e6:6.1f} TF/s   epilogue +{tf - tp:6.1f} us", flush=True)
        del x, w, dy, a
    print(f"total: plain {tot_plain:.1f} us, with post {tot_post:.1f} us", flush=True)


if __name__ == "__main__":
    main()
