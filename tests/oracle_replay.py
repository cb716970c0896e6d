"""Replay a fixture config through the ORACLE and record it in the golden key format.

Test infrastructure (imports ``oracle/``).  Used by the CPU pin tests (oracle vs the
reference's fixtures, bitwise) and by the GPU parity tests (teacher-forcing states).
"""
import json

import numpy as np
import torch

from oracle.reference_cpu import Trainer, make_param, optimizer_state, synthetic_images
from tests.golden.configs import CONFIGS, Recorder

import os

GOLDEN_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load_golden(name):
    d = np.load(os.path.join(GOLDEN_DIR, f"{name}.npz"), allow_pickle=False)
    return {k: d[k] for k in d.files}


def golden_meta(g):
    return json.loads(bytes(g["meta.json"]).decode())


def param_for(name, **extra):
    cfg = CONFIGS[name]
    kw = dict(cfg["args"])
    kw.update(seed=cfg.get("seed", 1), cuda=False, gen_extra_images=0, print_every=1000, pac=cfg.get("pac", 1))
    kw.update(extra)
    return make_param(**kw)


def dataset_for(name):
    cfg = CONFIGS[name]
    return synthetic_images(cfg.get("n_images", 64), cfg["args"].get("image_size", 64))


def replay(name, n_iter=None, threads=1):
    """Run the oracle on a fixture config; return (recorded dict, trainer)."""
    torch.set_num_threads(threads)
    p = param_for(name)
    n_iter = n_iter or CONFIGS[name]["args"].get("n_iter", 3)
    rec = Recorder()
    state = {"i": 0}
    holder = {}

    def hooks(tag, r):
        t = holder["t"]
        i = state["i"]
        if tag == "D":
            base = f"it{i}.D"
            for k in ("x", "z", "u"):
                if k in r:
                    rec.put(f"{base}.{k}", r[k])
            if "gp" in r:
                rec.put(f"{base}.gp", r["gp"].reshape(1))
            rec.put(f"{base}.y_pred", r["y_pred"])
            rec.put(f"{base}.y_pred_fake", r["y_pred_fake"])
            rec.put(f"{base}.errD", r["errD"].reshape(1))
            for n, q in t.D.named_parameters():
                rec.put(f"{base}.grad.{n}", q.grad)
        elif tag == "D.post":
            base = f"it{i}.D"
            rec.state(base + ".post", t.D)
            rec.state(base + ".postG", t.G)
            rec.optim(base + ".adam", t.optD, t.D)
        elif tag == "G":
            base = f"it{i}.G"
            rec.put(base + ".z", r["z"])
            if "x" in r:
                rec.put(base + ".x", r["x"])
                rec.put(base + ".y_pred", r["y_pred"])
            rec.put(base + ".y_pred_fake", r["y_pred_fake"])
            rec.put(base + ".errG", r["errG"].reshape(1))
            for n, q in t.G.named_parameters():
                rec.put(f"{base}.grad.{n}", q.grad)
        elif tag == "G.post":
            base = f"it{i}.G"
            rec.state(base + ".post", t.G)
            rec.state(base + ".postD", t.D)
            rec.optim(base + ".adam", t.optG, t.G)

    t = Trainer(p, dataset_for(name), hooks=hooks)
    holder["t"] = t
    rec.state("init.G", t.G)
    rec.state("init.D", t.D)
    rec.put("init.z_test", t.z_test)
    for i in range(n_iter):
        state["i"] = i
        t.iteration(i)
    return rec.store, t


def trainer_state(t):
    """Full teacher-forcing state of an oracle trainer (CPU tensors, cloned)."""
    return {
        "G": {k: v.clone() for k, v in t.G.state_dict().items()},
        "D": {k: v.clone() for k, v in t.D.state_dict().items()},
        "optG": {k: tuple(x.clone() if torch.is_tensor(x) else x for x in v)
                 for k, v in optimizer_state(t.optG, t.G).items()},
        "optD": {k: tuple(x.clone() if torch.is_tensor(x) else x for x in v)
                 for k, v in optimizer_state(t.optD, t.D).items()},
        "z_test": t.z_test.clone(),
        "lrD": t.optD.param_groups[0]["lr"], "lrG": t.optG.param_groups[0]["lr"],
    }
