"""Per-call GEMM breakdown of one training iteration (diagnostic; GPU).

Wraps kernels.conv_fwd/conv_dgrad/conv_wgrad during a real iteration of a bench
workload and records, per call, the library's HIP-event GEMM time and algorithmic
FLOPs (profile_begin/profile_end around the call).  Prints a table aggregated by
(op, shapes, kernel) sorted by total time.

usage: python tools/conv_breakdown.py [C1|C2|C3|C4|C4p|C5] [iters]
"""
import collections
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from bench import ARCH, WORKLOADS  # noqa: E402
from relativisticgan_amd import kernels as K  # noqa: E402
from relativisticgan_amd.config import make_param  # noqa: E402
from relativisticgan_amd.train import Trainer, synthetic_images  # noqa: E402

REC = collections.defaultdict(lambda: [0, 0.0, 0.0, ""])
ACTIVE = [False]


def wrap(name, fn, shape_of):
    def f(*a, **kw):
        if not ACTIVE[0]:
            return fn(*a, **kw)
        K.profile_begin(64)
        out = fn(*a, **kw)
        pr = K.profile_end()
        key = (name,) + shape_of(*a, **kw)
        r = REC[key]
        r[0] += 1
        r[1] += pr["ms"]
        r[2] += pr["flops"]
        r[3] = ",".join((k["name"].split("<")[1].split(">")[0] if "<" in k["name"] else k["name"].split("(")[0])
                        for k in pr["kernels"])
        return out
    return f


def g(geom):
    return f"k{geom.k}s{geom.stride}p{geom.pad}{'T' if geom.transposed else ''}"


def main():
    wl = sys.argv[1] if len(sys.argv) > 1 else "C2"
    iters = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    loss_D, size, bpg, h = WORKLOADS[wl]
    p = make_param(loss_D=loss_D, image_size=size, batch_size=bpg, G_h_size=h, D_h_size=h, seed=1,
                   print_every=10 ** 9, spectral=wl == "C5", rgan_rng="device", arch=ARCH.get(wl, 0))
    t = Trainer(p, synthetic_images(1024, size, device="cuda"))
    K.conv_fwd = wrap("fwd", K.conv_fwd, lambda x, w, geom, *a, **kw: (tuple(x.shape), tuple(w.shape), g(geom)))
    K.conv_fwd_bn = wrap("fwd_bn", K.conv_fwd_bn, lambda x, w, geom, *a, **kw: (tuple(x.shape), tuple(w.shape),
                                                                              g(geom)))
    K.conv_dgrad = wrap("dgrad", K.conv_dgrad, lambda dy, w, geom, xs, *a, **kw: (tuple(xs), tuple(w.shape), g(geom)))
    K.conv_wgrad = wrap("wgrad", K.conv_wgrad, lambda x, dy, geom, ws, *a, **kw: (tuple(x.shape), tuple(ws), g(geom)))
    for i in range(2):
        t.iteration(i + 1)
    torch.cuda.synchronize()
    ACTIVE[0] = True
    for i in range(iters):
        t.iteration(3 + i)
    torch.cuda.synchronize()
    tot_ms = sum(r[1] for r in REC.values()) / iters
    tot_fl = sum(r[2] for r in REC.values()) / iters
    print(f"workload {wl}: GEMM {tot_ms:.2f} ms/iter, {tot_fl / 1e12:.3f} TFLOP/iter, "
          f"{tot_fl / tot_ms / 1e9:.1f} TF/s")
    rows = sorted(REC.items(), key=lambda kv: -kv[1][1])
    print(f"{'op':6s} {'x / dx shape':22s} {'w shape':22s} {'geom':9s} {'n/it':>4s} {'ms/it':>7s} {'TF/s':>6s}  kernel")
    for key, (n, ms, fl, kern) in rows:
        print(f"{key[0]:6s} {str(key[1]):22s} {str(key[2]):22s} {key[3]:9s} {n / iters:4.0f} {ms / iters:7.3f} "
              f"{fl / ms / 1e9 if ms else 0:6.1f}  {kern}")


if __name__ == "__main__":
    main()
