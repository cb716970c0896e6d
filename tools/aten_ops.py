#!/usr/bin/env python3
"""List the ATen ops one training iteration dispatches (diagnostic, GPU box).

Every op that launches device work outside librgan.so shows up here; allocation, views
and metadata ops are filtered.  usage: python tools/aten_ops.py [bench workload] [iters]
"""
import collections
import os
import sys
import traceback

import torch
from torch.utils._python_dispatch import TorchDispatchMode

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

SKIP = ("empty", "view", "_unsafe_view", "as_strided", "detach", "t.default", "alias", "slice", "select",
        "reshape", "expand", "unsqueeze", "squeeze", "permute", "transpose", "split", "lift_fresh",
        "_local_scalar_dense", "is_same_size", "set_", "resize_", "unbind", "_to_copy", "result_type")


class Log(TorchDispatchMode):
    def __init__(self):
        super().__init__()
        self.ops = collections.Counter()
        self.where = {}

    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        name = str(func)
        if not any(name.startswith("aten." + s) for s in SKIP):
            self.ops[name] += 1
            if name not in self.where:
                st = [f for f in traceback.extract_stack() if "relativisticgan_amd" in f.filename or
                      "bench.py" in f.filename]
                self.where[name] = " <- ".join(f"{os.path.basename(f.filename)}:{f.lineno}" for f in st[-3:][::-1])
        return func(*args, **(kwargs or {}))


def main():
    w = sys.argv[1] if len(sys.argv) > 1 else "C1"
    iters = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    from relativisticgan_amd.config import make_param
    from relativisticgan_amd.train import Trainer, synthetic_images
    loss_D, size, bpg, h = bench.WORKLOADS[w]
    p = make_param(loss_D=loss_D, image_size=size, batch_size=bpg, G_h_size=h, D_h_size=h, seed=1,
                   print_every=10 ** 9, spectral=w == "C5", rgan_rng="device", arch=bench.ARCH.get(w, 0))
    t = Trainer(p, synthetic_images(1024, size, device="cuda"))
    for i in range(2):
        t.iteration(i + 1)
    torch.cuda.synchronize()
    log = Log()
    with log:
        for i in range(iters):
            t.iteration(3 + i)
    torch.cuda.synchronize()
    print(f"{w}: ATen ops per {iters} iterations")
    for name, n in log.ops.most_common():
        print(f"{n:6d}  {name:55s} {log.where[name]}")


if __name__ == "__main__":
    main()
