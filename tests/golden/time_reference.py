#!/usr/bin/env python3
"""SURVEY §8(d) cross-check: the oracle (CPU restatement) must time within +-10 % of the
unmodified reference script on the same host, so the oracle's GPU-box CPU baseline stands in
for the reference's own CPU path.  Runs here only (the reference does not travel): GLI via
runpy (make_golden.py's stubs) and the oracle, same config and thread count, per-iteration
wall time from consecutive optimizerG steps (iteration 0 and the warm-up excluded).

usage: python tests/golden/time_reference.py [config] [iterations] [threads] [both|reference|oracle] [out.json]
(the reference prints its nets to stdout: the result goes to out.json, default stdout's last line)
"""
import json
import os
import platform
import runpy
import sys
import tempfile
import time

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
from tests.golden.configs import CONFIGS  # noqa: E402
from tests.golden.make_golden import REF_SCRIPT, install_stubs, synthetic_dataset, _script_globals  # noqa: E402


def time_reference(name, n_iter, threads):
    cfg = CONFIGS[name]
    torch.set_num_threads(threads)
    args = dict(cfg["args"])
    install_stubs(synthetic_dataset(cfg.get("n_images", 64), args.get("image_size", 64)))
    stamps = []
    orig = torch.optim.Adam.step

    def step(self, *a, **k):
        out = orig(self, *a, **k)
        g = _script_globals()
        if self is g["optimizerG"]:
            stamps.append(time.perf_counter())
        return out
    torch.optim.Adam.step = step
    tmp = tempfile.mkdtemp(prefix="rgan_time_")
    os.makedirs(os.path.join(tmp, "extra"))
    argv = [REF_SCRIPT, "--cuda", "False", "--seed", "1", "--n_iter", str(n_iter), "--gen_extra_images", "0",
            "--print_every", "100000", "--output_folder", tmp, "--extra_folder", tmp + "/extra", "--input_folder", tmp]
    for k, v in args.items():
        if k != "n_iter":
            argv += ["--" + k, str(v)]
    old, cwd = sys.argv, os.getcwd()
    sys.argv = argv
    os.chdir(tmp)
    try:
        runpy.run_path(REF_SCRIPT, run_name="__main__")
    finally:
        sys.argv, _ = old, os.chdir(cwd)
        torch.optim.Adam.step = orig
    d = [b - a for a, b in zip(stamps[1:], stamps[2:])]  # iterations 2.. (0 and 1 warm)
    return sum(d) / len(d), len(d)


def time_oracle(name, n_iter, threads):
    from tests.oracle_replay import dataset_for, param_for
    from oracle.reference_cpu import Trainer
    torch.set_num_threads(threads)
    p = param_for(name, print_every=100000)
    t = Trainer(p, dataset_for(name))
    stamps = []
    for i in range(n_iter):
        t.iteration(i)
        stamps.append(time.perf_counter())
    d = [b - a for a, b in zip(stamps[1:], stamps[2:])]
    return sum(d) / len(d), len(d)


if __name__ == "__main__":
    name = sys.argv[1] if len(sys.argv) > 1 else "ralsgan_c1"
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 12
    th = int(sys.argv[3]) if len(sys.argv) > 3 else 8
    which = sys.argv[4] if len(sys.argv) > 4 else "both"
    res = {"config": name, "threads": th, "host": platform.processor() or platform.machine(),
           "torch": torch.__version__}
    if which in ("both", "reference"):
        res["reference_s_per_iter"], res["reference_iters"] = time_reference(name, n, th)
    if which in ("both", "oracle"):
        res["oracle_s_per_iter"], res["oracle_iters"] = time_oracle(name, n, th)
    if "reference_s_per_iter" in res and "oracle_s_per_iter" in res:
        res["oracle_over_reference"] = res["oracle_s_per_iter"] / res["reference_s_per_iter"]
        res["within_10pct"] = abs(res["oracle_over_reference"] - 1.0) <= 0.10
    if len(sys.argv) > 5:
        with open(sys.argv[5], "w") as f:
            json.dump(res, f, indent=1)
    print(json.dumps(res))
