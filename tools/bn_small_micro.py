#!/usr/bin/env python3
"""Small-layer BatchNorm paths on C4's shapes, timed as HIP-graph replays (diagnostic; GPU).

The arch-1 layers are 512-4096 rows: every BN kernel there is a few microseconds, so the
per-call Python/ctypes cost would dominate an eager loop.  Each case captures REPS calls in a
graph and times replays with HIP events: GPU time per call, launch gaps included (as in the
bench's graph-mode step).
  fwd  : rgan_bn_segment_stats_n + rgan_bn_apply_segments (two launches) vs rgan_bn_segment_apply
  bwd  : rgan_bn_backward_sums + rgan_bn_backward_apply_ex vs rgan_bn_backward (bn_bwd_small
         where it applies) vs rgan_bn_backward_sums_apply
usage: python tools/bn_small_micro.py [reps]
"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from relativisticgan_amd import kernels as K  # noqa: E402

DEV = "cuda"


def graph_time(fn, reps):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            for _ in range(reps):
                fn()
    torch.cuda.synchronize()
    g.replay()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(5):
        g.replay()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / (5 * reps) * 1000.0  # us per call


def nhwc_rows(P, C):
    return K.empty_nhwc(P // 64, C, 8, 8, DEV).normal_()  # P rows as [P/64, C, 8, 8]


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 100
    torch.manual_seed(0)
    print("forward: rows, C, nseg | stats_n + apply_segments | segment_apply (us per call)")
    for P, C, nseg in ((512, 256, 1), (2048, 128, 1), (2048, 256, 1), (1024, 256, 2), (4096, 128, 2),
                       (4096, 256, 2), (8192, 128, 1), (16384, 64, 2)):
        y = nhwc_rows(P, C)
        S = P // 64
        yv = y.permute(0, 2, 3, 1).reshape(S, 64, C).double()  # NHWC rows, 64 per segment
        part = torch.stack([yv.sum(1), (yv * yv).sum(1)], 1).contiguous()  # [S][2][C]
        gamma, beta = torch.rand(C, device=DEV) + 0.5, torch.randn(C, device=DEV)
        rm, rv, nbt = torch.zeros(C, device=DEV), torch.ones(C, device=DEV), torch.zeros((), dtype=torch.long,
                                                                                          device=DEV)
        st = torch.empty(nseg, 2 * C, device=DEV)
        a = torch.empty_like(y)

        def two():
            K.bn_segment_stats_n(part, S, nseg, C, 1e-5, 0.1, rm, rv, nbt, out=st)
            K.bn_apply_segments(y, st, gamma, beta, "lrelu", 0.1, out=a)

        def one():
            K.bn_segment_apply(part, S, y, 1e-5, 0.1, rm, rv, nbt, gamma, beta, "lrelu", 0.1, st, a)
        print(f"  {P:6d} {C:5d} {nseg} | {graph_time(two, reps):7.2f} | {graph_time(one, reps):7.2f}", flush=True)
    print("backward: rows, C | sums + apply_ex | bn_backward | sums_apply (us per call)")
    for P, C in ((512, 256), (2048, 128), (2048, 256), (1024, 1024), (8192, 64), (8192, 128)):
        y, da = nhwc_rows(P, C), nhwc_rows(P, C)
        stats = torch.cat([torch.randn(C, device=DEV), torch.rand(C, device=DEV) + 0.5])
        gamma, beta = torch.rand(C, device=DEV) + 0.5, torch.randn(C, device=DEV)
        dy = torch.empty_like(y)
        dg, db = torch.zeros(C, device=DEV), torch.zeros(C, device=DEV)

        def sep():
            sums, dac = K.bn_backward_sums(da, y, stats, gamma, beta, "lrelu", 0.1)
            K.bn_backward_apply_ex(dac, y, stats, gamma, beta, "lrelu", 0.1, sums, P, out=dy, dgamma=dg, dbeta=db)

        def bwd():
            K.bn_backward(da, y, stats, gamma, beta, "lrelu", 0.1, out=dy)

        def fused():
            K.bn_backward_sums_apply(da, y, stats, gamma, beta, "lrelu", 0.1, out=dy, dgamma=dg, dbeta=db)
        print(f"  {P:6d} {C:5d} | {graph_time(sep, reps):7.2f} | {graph_time(bwd, reps):7.2f} | "
              f"{graph_time(fused, reps):7.2f}", flush=True)


if __name__ == "__main__":
    main()
