#!/usr/bin/env python3
"""C-ABI call trace of one eager training iteration: every rgan_* call the host makes, in
order, with its scalar arguments, the RganConv descriptor decoded, and the Python caller
chain (kernels.* -> autograd / gp / nets).  Diagnostic only (GPU box).

usage: python tools/abi_trace.py [WORKLOAD] [ITERS_WARMUP]   (workloads of bench.py)
"""
import ctypes
import os
import sys
import traceback

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from bench import ARCH, WORKLOADS  # noqa: E402
from relativisticgan_amd import _lib as L  # noqa: E402

SKIP = {"rgan_conv_workspace", "rgan_bn_partial_bytes", "rgan_bn_dd_partial_bytes", "rgan_conv_bn_segments",
        "rgan_conv_post_segments", "rgan_spectral_batch_ws_bytes", "rgan_spectral_ws_bytes", "rgan_profile_kernel"}


def _fmt(a):
    if isinstance(a, (int, float)):
        return repr(a)
    if isinstance(a, ctypes.c_void_p) or a is None:
        return "p" if a is not None and a.value else "0"
    try:
        obj = a._obj  # byref(...)
    except AttributeError:
        return type(a).__name__
    if isinstance(obj, L.RganConv):
        return (f"conv[B{obj.batch} {obj.cin}x{obj.hin}x{obj.win}->{obj.cout}x{obj.hout}x{obj.wout} "
                f"k{obj.kh} s{obj.stride} p{obj.pad} T{obj.transposed}]")
    if isinstance(obj, L.RganPost):
        return f"post[mode{obj.mode} nseg{obj.nseg} S{obj.part_segments}]"
    return type(obj).__name__


class Proxy:
    def __init__(self, lib, log):
        self._lib, self._log = lib, log

    def __getattr__(self, name):
        fn = getattr(self._lib, name)
        if not name.startswith("rgan_") or name in SKIP:
            return fn
        log = self._log

        def wrapped(*args):
            if log.on:
                st = [f.name for f in traceback.extract_stack(limit=9)[:-1]
                      if f.filename.startswith(os.path.join(ROOT, "relativisticgan_amd"))]
                log.rows.append(f"{name}({', '.join(_fmt(a) for a in args)})  <- {'/'.join(st[-4:])}")
            return fn(*args)
        return wrapped


class Log:
    on = False
    rows = []


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "C4"
    warm = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    from relativisticgan_amd.config import make_param
    from relativisticgan_amd.train import Trainer, synthetic_images
    loss_D, size, bpg, h = WORKLOADS[name]
    p = make_param(loss_D=loss_D, image_size=size, batch_size=bpg, G_h_size=h, D_h_size=h, seed=1,
                   print_every=10 ** 9, spectral=name == "C5", rgan_rng="device", arch=ARCH.get(name, 0))
    t = Trainer(p, synthetic_images(1024, size, device="cuda"))
    for i in range(warm):
        t.iteration(i + 1)
    torch.cuda.synchronize()
    log = Log()
    L._LIB = Proxy(L.lib(), log)
    log.on = True
    t.iteration(warm + 1)
    torch.cuda.synchronize()
    log.on = False
    for r in log.rows:
        print(r)
    print(f"# {len(log.rows)} rgan_* calls in one {name} iteration")


if __name__ == "__main__":
    main()
