"""Diagnostic: per-tensor GPU-vs-oracle report of one fixture config (prints every tensor).

Usage: python tools/debug_parity.py CONFIG [--nocache]
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from tests import test_parity_gpu as T  # noqa: E402
from tests.golden.configs import CONFIGS  # noqa: E402
from tests.oracle_replay import dataset_for  # noqa: E402


def main():
    name = sys.argv[1]
    if "--nocache" in sys.argv:
        from relativisticgan_amd import kernels as K
        orig = K.conv_fwd

        def nocache(*a, **k):
            k["cache"] = False
            return orig(*a, **k)
        K.conv_fwd = nocache
    from relativisticgan_amd.train import Trainer
    n_iter = CONFIGS[name]["args"].get("n_iter", 3)
    p, init, steps = T.oracle_steps(name, n_iter)
    p.rgan_rng = "host"
    t = Trainer(p, dataset_for(name).to(T.DEV))
    for st in steps:
        got = T.gpu_step(t, st)
        exact = T.oracle_exact_step(name, st)
        go, ex = T.per_net(got["masks"]), T.per_net(exact["masks"])
        per = [int((a != b).sum()) for tag in ("G", "D") for a, b in zip(go[tag], ex[tag])]
        print(f"== it{st['i']} flips per activation call: {per}")
        report = []
        errs = T.compare(p, st, got, exact, report, sum(per))
        for label, e, env in report:
            if e > 1e-5:
                print(f"  {label:60s} {e:.3e} {env}")
        for e in errs:
            print("  ERR", e)


if __name__ == "__main__":
    main()
