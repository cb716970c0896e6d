"""BatchNorm kernel micro-benchmark on the C2 activation shapes (diagnostic; GPU):
achieved HBM-side bandwidth of bn_stats / bn_apply / bn_backward / act_backward per shape.
usage: python tools/bn_micro.py [reps]"""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from relativisticgan_amd import kernels as K  # noqa: E402

SHAPES = [(128, 256, 32, 32), (128, 512, 16, 16), (128, 1024, 8, 8), (128, 2048, 4, 4),
          (64, 128, 64, 64), (64, 256, 32, 32), (64, 2048, 4, 4)]


def timeit(fn, reps):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps * 1000.0  # us


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 50
    for shp in SHAPES:
        B, C, H, W = shp
        y = K.empty_nhwc(B, C, H, W, "cuda").normal_()
        da = K.empty_nhwc(B, C, H, W, "cuda").normal_()
        g = torch.ones(C, device="cuda")
        bta = torch.zeros(C, device="cuda")
        rm, rv = torch.zeros(C, device="cuda"), torch.ones(C, device="cuda")
        st = K.bn_stats(y, 1e-5, 0.1, rm, rv)
        out = torch.empty_like(y)
        n = y.numel() * 4
        t_st = timeit(lambda: K.bn_stats(y, 1e-5, 0.1, rm, rv), reps)
        t_ap = timeit(lambda: K.bn_apply(y, st, g, bta, "lrelu", 0.2, out=out), reps)
        t_bw = timeit(lambda: K.bn_backward(da, y, st, g, bta, "lrelu", 0.2), reps)
        t_ab = timeit(lambda: K.act_backward(da, y, "lrelu", 0.2), reps)
        print(f"{str(shp):22s} stats {t_st:7.1f} us {n / t_st / 1e6:5.2f} TB/s | apply {t_ap:7.1f} us "
              f"{2 * n / t_ap / 1e6:5.2f} TB/s | bwd {t_bw:7.1f} us {5 * n / t_bw / 1e6:5.2f} TB/s | "
              f"act_bwd {t_ab:6.1f} us {3 * n / t_ab / 1e6:5.2f} TB/s", flush=True)


if __name__ == "__main__":
    main()
