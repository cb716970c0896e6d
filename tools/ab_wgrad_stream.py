"""A/B of the weight-gradient stream (autograd.owning_grads.side_stream: the weight-gradient
GEMMs written into .grad run on a second stream, overlapping the data-gradient chain) in one
process on one box: bench.py's timed steps of a workload, alternating on / off.  First checks
that both settings give bit-identical weights after 3 eager iterations.

usage: python tools/ab_wgrad_stream.py [workload=C1] [rounds=3] [steps=20] [graph=auto|off]
"""
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from relativisticgan_amd import autograd as AG  # noqa: E402
from relativisticgan_amd import kernels as K  # noqa: E402
from relativisticgan_amd.config import make_param  # noqa: E402
from relativisticgan_amd.train import Trainer, synthetic_images  # noqa: E402


def weights(name, on):
    AG.owning_grads.side_stream = on
    loss_D, size, bpg, h = bench.WORKLOADS[name]
    p = make_param(loss_D=loss_D, image_size=size, batch_size=bpg, G_h_size=h, D_h_size=h, seed=1,
                   print_every=10 ** 9, spectral=name == "C5", rgan_rng="device", arch=bench.ARCH.get(name, 0))
    t = Trainer(p, synthetic_images(256, size, device="cuda"))
    for i in range(3):
        t.iteration(i + 1)
    t.flush()
    torch.cuda.synchronize()
    return [q.detach().clone() for q in list(t.G.parameters()) + list(t.D.parameters())]


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "C1"
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    steps = int(sys.argv[3]) if len(sys.argv) > 3 else 20
    graph = sys.argv[4] if len(sys.argv) > 4 else "auto"
    a, b = weights(name, False), weights(name, True)
    same = all(torch.equal(x, y) for x, y in zip(a, b))
    print(f"{name} weights after 3 iterations, stream on vs off: {'bit-identical' if same else 'DIFFER'}", flush=True)
    del a, b
    args = argparse.Namespace(batch_d="auto", graph=graph, sync_bn=False)
    res = {True: [], False: []}
    for r in range(rounds):
        for on in (True, False) if r % 2 == 0 else (False, True):
            AG.owning_grads.side_stream = on
            out = bench.run_workload(name, steps, 5, 1, args, K)
            res[on].append(out["value"])
            print(f"{name} wgrad-stream={'on ' if on else 'off'} {out['value']:9.1f} img/s  "
                  f"{out['ms_per_step']:.3f} ms/step ({out['mode']})", flush=True)
    for on in (True, False):
        v = sorted(res[on])
        print(f"{name} wgrad-stream={'on ' if on else 'off'} median {v[len(v) // 2]:.1f} img/s  "
              f"all {[round(x, 1) for x in v]}")
    if not same:
        sys.exit(1)


if __name__ == "__main__":
    main()
