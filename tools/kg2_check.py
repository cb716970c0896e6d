"""Quick check of the k-group GEMMs (gemm_kernel_kg2 / gemm_post_kg2) on the C1 / C3 layer shapes
that split K: forward, data gradient and weight gradient of each against torch float64 (MIOpen
off), and the HIP-event time per call.  Diagnostic; GPU.

usage: python tools/kg2_check.py [reps]
"""
import os
import sys

import torch
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from relativisticgan_amd import kernels as K  # noqa: E402


def nhwc(t):
    return t.contiguous(memory_format=torch.channels_last)


def rel(a, b):
    a, b = a.double().reshape(-1), b.double().reshape(-1)
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


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


# (B, cin, cout, H_in, transposed): C1's D (2B = 64) and G (B = 32) layers that split K, and the
# deepest C3 layers
SHAPES = [(64, 128, 256, 32, False), (64, 256, 512, 16, False), (64, 512, 1024, 8, False),
          (32, 1024, 512, 4, True), (32, 512, 256, 8, True), (32, 256, 128, 16, True),
          (32, 2048, 4096, 8, False), (32, 4096, 2048, 4, True)]


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    torch.manual_seed(0)
    worst = 0.0
    for B, cin, cout, H, tr in SHAPES:
        g = K.ConvGeom(4, 2, 1, tr)
        x = nhwc(torch.randn(B, cin, H, H, device="cuda"))
        w = torch.randn((cin, cout, 4, 4) if tr else (cout, cin, 4, 4), device="cuda") * 0.02
        with torch.backends.cudnn.flags(enabled=False):
            xr = x.detach().double().requires_grad_(True)
            wr = w.detach().double().requires_grad_(True)
            ref = (F.conv_transpose2d if tr else F.conv2d)(xr, wr, stride=2, padding=1)
            dy = torch.randn(ref.shape, device="cuda")
            ref.backward(dy.double())
        dyk = nhwc(dy)
        y = K.conv_fwd(x, w, g)
        dx = K.conv_dgrad(dyk, w, g, x.shape, like=x)
        dw = K.conv_wgrad(x, dyk, g, w.shape)[0]
        e = (rel(y, ref.detach()), rel(dx, xr.grad), rel(dw, wr.grad))
        worst = max(worst, *e)
        pix = (H * H) if tr else (H // 2) ** 2
        flops = 2.0 * B * cin * cout * 16 * pix
        t = (timed(lambda: K.conv_fwd(x, w, g), reps), timed(lambda: K.conv_dgrad(dyk, w, g, x.shape, like=x), reps),
             timed(lambda: K.conv_wgrad(x, dyk, g, w.shape), reps))
        print(f"B{B} {cin:5d}->{cout:5d} @{H:3d} {'T' if tr else 'C'}: rel fwd {e[0]:.1e} dgrad {e[1]:.1e} "
              f"wgrad {e[2]:.1e} | us fwd {t[0]:7.1f} dgrad {t[1]:7.1f} wgrad {t[2]:7.1f} | "
              f"TF/s {flops / t[0] / 1e6:5.1f} {flops / t[1] / 1e6:5.1f} {flops / t[2] / 1e6:5.1f}", flush=True)
        del x, w, xr, wr, ref, dy, dyk, y, dx, dw
    print(f"worst rel {worst:.2e}", flush=True)
    assert worst < 1e-5, worst


if __name__ == "__main__":
    main()
