"""Census of weight-layout packs per training iteration (GPU box): which layouts miss the
pack cache (a pack_tiled / pack_weights launch) after the first iteration, and why.

usage: python tools/pack_census.py [workload] [iterations]   (bench.py workload names)
"""
import collections
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from relativisticgan_amd import kernels as K  # noqa: E402
from relativisticgan_amd.config import make_param  # noqa: E402
from relativisticgan_amd.train import Trainer, synthetic_images  # noqa: E402


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "C4"
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    loss_D, size, bpg, h = bench.WORKLOADS[name]
    p = make_param(loss_D=loss_D, image_size=size, batch_size=bpg, G_h_size=h, D_h_size=h, seed=1,
                   print_every=10 ** 9, spectral=name == "C5", rgan_rng="device", arch=bench.ARCH.get(name, 0))
    t = Trainer(p, synthetic_images(1024, size, device="cuda"))
    log = []
    orig_get = K.PACKS.get

    def get(w, which, geom, d):
        base = w._base if w._base is not None else w
        key = (id(base), which, geom, d.cin, d.cout, d.hin, d.win, d.hout, d.wout)
        ent = K.PACKS.entries.get(key)
        hit = ent is not None and ent[0]() is base and ent[1] == w._version and ent[3] == w.data_ptr()
        why = "hit" if hit else ("new" if ent is None else ("version" if ent[1] != w._version else "other"))
        log.append((tuple(w.shape), "view" if w._base is not None else "param", which, why))
        return orig_get(w, which, geom, d)
    K.PACKS.get = get
    wrapped = {}
    for fn in ("conv_fwd", "conv_dgrad", "conv_fwd_bn"):
        orig = getattr(K, fn)

        def wrap(*a, _orig=orig, _fn=fn, **k):
            if not k.get("cache", False):
                log.append((tuple(a[1].shape), "uncached", _fn, "workspace-pack"))
            return _orig(*a, **k)
        wrapped[fn] = wrap
        setattr(K, fn, wrap)
    for i in range(n):
        log.clear()
        t.iteration(i + 1)
        torch.cuda.synchronize()
        c = collections.Counter(e for e in log if e[3] != "hit")
        print(f"iteration {i + 1}: {sum(c.values())} pack-cache misses / workspace packs")
        for k, v in sorted(c.items(), key=lambda kv: -kv[1]):
            print("   ", v, k)


if __name__ == "__main__":
    main()
