"""A/B of arch 1's dense output copied channels-last (nets.VIEW_OUT_CHANNELS_LAST) in one
process on one box: bench.py's timed graph replays of a workload, alternating on / off.

usage: python tools/ab_dense_cl.py [workload=C4] [rounds=3] [steps=20]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from relativisticgan_amd import nets as NETS  # noqa: E402
from relativisticgan_amd import kernels as K  # noqa: E402


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "C4"
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    steps = int(sys.argv[3]) if len(sys.argv) > 3 else 20
    args = argparse.Namespace(batch_d="auto", graph="auto", sync_bn=False)
    res = {True: [], False: []}
    for r in range(rounds):
        for on in (True, False) if r % 2 == 0 else (False, True):
            NETS.VIEW_OUT_CHANNELS_LAST = on
            out = bench.run_workload(name, steps, 5, 1, args, K)
            res[on].append(out["value"])
            print(f"{name} dense-cl={'on ' if on else 'off'} {out['value']:9.1f} img/s  {out['ms_per_step']:.3f} ms/step",
                  flush=True)
    for on in (True, False):
        v = sorted(res[on])
        print(f"{name} dense-cl={'on ' if on else 'off'} median {v[len(v) // 2]:.1f} img/s  all {[round(x, 1) for x in v]}")


if __name__ == "__main__":
    main()
