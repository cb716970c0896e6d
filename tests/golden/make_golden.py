#!/usr/bin/env python3
"""Golden-vector generator: runs the UNMODIFIED reference training script on CPU.

Test infrastructure only (runs in the build container, never on the GPU box, never
imported by the product).  It executes ``/root/reference/code/GAN_losses_iter.py``
(referred to as GLI below) with ``runpy`` after injecting stub modules for the
third-party packages the script imports but this image lacks (torchvision,
IPython, fid, pytorch_visualize; GLI:121-143).  The stubs only replace I/O:

* ``torchvision.datasets.ImageFolder`` -> a synthetic uint8 image set mapped by
  ``(u8/255 - 0.5)/0.5`` (what ToTensor+Normalize does, GLI:160-166);
* ``torchvision.utils.save_image`` -> no-op (GLI:565, 768);
* ``fid.calculate_fid_given_paths`` / ``pytorch_visualize`` / ``IPython`` -> unused.

Capture points: ``torch.optim.Adam.__init__`` (state after ``weights_init``,
GLI:476-477, and ``z_test``, GLI:497) and ``torch.optim.Adam.step`` (GLI:659 and
GLI:712).  At each step the harness reads the loop's module-level variables
(``x``, ``z``, ``u``, ``y_pred``, ``y_pred_fake``, ``errD``, ``errG``) from the
script's frame, the parameter gradients before the update and the full module and
optimizer state after it.

Output: one ``.npz`` per config under ``tests/golden/`` (``allow_pickle=False``
loadable).  Tensors above ``FULL_LIMIT`` elements are stored as a summary
(sampled elements at seeded positions + sum + sum of squares + sha1) so the arch-1
fixtures stay small.

Usage:  python tests/golden/make_golden.py [config-name ...]
"""
import json
import os
import runpy
import sys
import tempfile
import types

import numpy as np
import torch

REF_SCRIPT = "/root/reference/code/GAN_losses_iter.py"
REF_SCRIPT_PAC = "/root/reference/code/GAN_losses_iter_PAC.py"  # PacGAN-2 variant (config key "pac": 2)
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
from tests.golden.configs import CONFIGS, PINNED, Recorder  # noqa: E402

THREADS = 1


def synthetic_dataset(n, size, seed=1234, n_colors=3):
    """uint8 images -> float in [-1,1] on the 1/127.5 grid."""
    g = torch.Generator().manual_seed(seed)
    u8 = torch.randint(0, 256, (n, n_colors, size, size), generator=g, dtype=torch.uint8)
    return (u8.float() / 255.0 - 0.5) / 0.5


def install_stubs(dataset):
    tv = types.ModuleType("torchvision")
    dset = types.ModuleType("torchvision.datasets")
    transf = types.ModuleType("torchvision.transforms")
    models = types.ModuleType("torchvision.models")
    vutils = types.ModuleType("torchvision.utils")

    class _Folder:
        def __init__(self, *a, **k):
            self.images = dataset

        def __len__(self):
            return self.images.shape[0]

        def __getitem__(self, i):
            return self.images[i], 0

    dset.ImageFolder = _Folder
    dset.CIFAR10 = _Folder

    class _Identity:
        def __init__(self, *a, **k):
            pass

        def __call__(self, x):
            return x

    for name in ("Compose", "Resize", "ToTensor", "Normalize", "ToPILImage"):
        setattr(transf, name, _Identity)
    vutils.save_image = lambda *a, **k: None
    tv.datasets, tv.transforms, tv.models, tv.utils = dset, transf, models, vutils
    sys.modules.update({"torchvision": tv, "torchvision.datasets": dset,
                        "torchvision.transforms": transf, "torchvision.models": models,
                        "torchvision.utils": vutils})
    ipy = types.ModuleType("IPython")
    ipyd = types.ModuleType("IPython.display")
    ipyd.Image = lambda *a, **k: None
    ipy.display = ipyd
    sys.modules.update({"IPython": ipy, "IPython.display": ipyd})
    pv = types.ModuleType("pytorch_visualize")
    pv.make_dot = lambda *a, **k: None
    sys.modules["pytorch_visualize"] = pv
    fid = types.ModuleType("fid")
    fid.calculate_fid_given_paths = lambda *a, **k: 0.0
    sys.modules["fid"] = fid


def _script_globals():
    f = sys._getframe(1)
    while f is not None:
        if "optimizerD" in f.f_globals and "param" in f.f_globals:
            return f.f_globals
        f = f.f_back
    return None


def run_config(name, cfg):
    threads = cfg.get("threads", THREADS)
    torch.set_num_threads(threads)
    args = cfg["args"]
    S = args.get("image_size", 64)
    dataset = synthetic_dataset(cfg.get("n_images", 64), S)
    install_stubs(dataset)
    rec = Recorder()
    n_iter = args.get("n_iter", 3)

    orig_init = torch.optim.Adam.__init__
    orig_step = torch.optim.Adam.step
    n_init = [0]

    def init_hook(self, params, *a, **k):
        orig_init(self, params, *a, **k)
        n_init[0] += 1
        if n_init[0] == 2:  # optimizerG: G and D fully initialised (GLI:529-530)
            g = sys._getframe(1).f_globals
            rec.state("init.G", g["G"])
            rec.state("init.D", g["D"])
            rec.put("init.z_test", g["z_test"])

    def step_hook(self, *a, **k):
        g = _script_globals()
        i = g["i"]
        if self is g["optimizerD"]:
            tag = f"it{i}.D"
            rec.put(tag + ".x", g["x"])
            rec.put(tag + ".z", g["z"])
            if g["param"].loss_D == 3 or g["param"].grad_penalty:
                rec.put(tag + ".u", g["u"])
                rec.put(tag + ".gp", g["grad_penalty"].reshape(1))
            rec.put(tag + ".y_pred", g["y_pred"])
            rec.put(tag + ".y_pred_fake", g["y_pred_fake"])
            rec.put(tag + ".errD", g["errD"].reshape(1))
            for n, p in g["D"].named_parameters():
                rec.put(f"{tag}.grad.{n}", p.grad)
            out = orig_step(self, *a, **k)
            rec.state(tag + ".post", g["D"])
            rec.state(tag + ".postG", g["G"])
            rec.optim(tag + ".adam", self, g["D"])
        else:
            tag = f"it{i}.G"
            rec.put(tag + ".z", g["z"])
            if g["param"].loss_D not in (1, 2, 3, 4):
                rec.put(tag + ".x", g["x"])
                rec.put(tag + ".y_pred", g["y_pred"])
            rec.put(tag + ".y_pred_fake", g["y_pred_fake"])
            rec.put(tag + ".errG", g["errG"].reshape(1))
            for n, p in g["G"].named_parameters():
                rec.put(f"{tag}.grad.{n}", p.grad)
            out = orig_step(self, *a, **k)
            rec.state(tag + ".post", g["G"])
            rec.state(tag + ".postD", g["D"])
            rec.optim(tag + ".adam", self, g["G"])
        return out

    torch.optim.Adam.__init__ = init_hook
    torch.optim.Adam.step = step_hook
    tmp = tempfile.mkdtemp(prefix="rgan_golden_")
    os.makedirs(os.path.join(tmp, "extra"))  # GLI:103-104 only creates it when gen_extra_images > 0
    script = REF_SCRIPT_PAC if cfg.get("pac", 1) == 2 else REF_SCRIPT
    argv = [script, "--cuda", "False", "--seed", str(cfg.get("seed", 1)),
            "--n_iter", str(n_iter), "--gen_extra_images", "0", "--print_every", "1000",
            "--output_folder", tmp, "--extra_folder", tmp + "/extra", "--input_folder", tmp]
    for k, v in args.items():
        if k == "n_iter":
            continue
        argv += ["--" + k, str(v)]
    if cfg.get("save_every"):  # the reference writes its own checkpoint (GLI:729-747)
        argv += ["--gen_every", str(cfg["save_every"]), "--save", "True"]
    old_argv, old_cwd = sys.argv, os.getcwd()
    sys.argv = argv
    os.chdir(tmp)
    try:
        runpy.run_path(script, run_name="__main__")
    finally:
        sys.argv = old_argv
        os.chdir(old_cwd)
        torch.optim.Adam.__init__ = orig_init
        torch.optim.Adam.step = orig_step
    rec.store["meta.json"] = np.frombuffer(json.dumps({
        "config": name, "args": args, "seed": cfg.get("seed", 1), "n_iter": n_iter, "pac": cfg.get("pac", 1),
        "n_images": cfg.get("n_images", 64), "threads": threads,
        "torch": torch.__version__}).encode(), dtype=np.uint8).copy()
    out = os.path.join(HERE, f"{name}.npz")
    np.savez_compressed(out, **rec.store)
    if cfg.get("save_every"):
        import shutil
        for f in sorted(os.listdir(os.path.join(tmp, "extra", "models"))):
            shutil.copy(os.path.join(tmp, "extra", "models", f), os.path.join(HERE, f"{name}_{f}"))
    return out


TRAJ_KEYS = ("errD", "errG", "D.y_pred", "D.y_pred_fake", "G.y_pred", "G.y_pred_fake",
             "D.x", "D.z", "G.z", "G.x", "D.wsum", "G.wsum")


def run_trajectory(name, threads, n_iter):
    """Scalar trajectory of the unmodified reference: per iteration the
    losses, the means of D's outputs in both steps, the sums of the drawn inputs (draw order)
    and the sums of each net's parameters after its step, at ``threads`` intra-op threads.
    Written to tests/golden/traj_<name>_t<threads>.npz."""
    cfg = CONFIGS[name]
    torch.set_num_threads(threads)
    args = dict(cfg["args"])
    S = args.get("image_size", 64)
    install_stubs(synthetic_dataset(cfg.get("n_images", 64), S))
    out = {k: np.full(n_iter, np.nan) for k in TRAJ_KEYS}
    orig_step = torch.optim.Adam.step

    def wsum(net):
        return float(sum(p.detach().double().sum() for p in net.parameters()))

    def step_hook(self, *a, **k):
        g = _script_globals()
        i = g["i"]
        side = "D" if self is g["optimizerD"] else "G"
        res = orig_step(self, *a, **k)
        if side == "D":
            out["errD"][i] = float(g["errD"])
            out["D.y_pred"][i] = float(g["y_pred"].detach().double().mean())
            out["D.y_pred_fake"][i] = float(g["y_pred_fake"].detach().double().mean())
            out["D.x"][i] = float(g["x"].double().sum())
            out["D.z"][i] = float(g["z"].double().sum())
        else:
            out["errG"][i] = float(g["errG"])
            if g["param"].loss_D not in (1, 2, 3, 4):
                out["G.y_pred"][i] = float(g["y_pred"].detach().double().mean())
                out["G.x"][i] = float(g["x"].double().sum())
            out["G.y_pred_fake"][i] = float(g["y_pred_fake"].detach().double().mean())
            out["G.z"][i] = float(g["z"].double().sum())
        out[side + ".wsum"][i] = wsum(g[side])
        return res

    torch.optim.Adam.step = step_hook
    tmp = tempfile.mkdtemp(prefix="rgan_traj_")
    os.makedirs(os.path.join(tmp, "extra"))
    argv = [REF_SCRIPT, "--cuda", "False", "--seed", str(cfg.get("seed", 1)), "--n_iter", str(n_iter),
            "--gen_extra_images", "0", "--print_every", "1000", "--output_folder", tmp,
            "--extra_folder", tmp + "/extra", "--input_folder", tmp]
    for k, v in args.items():
        if k != "n_iter":
            argv += ["--" + k, str(v)]
    old_argv, old_cwd = sys.argv, os.getcwd()
    sys.argv = argv
    os.chdir(tmp)
    try:
        runpy.run_path(REF_SCRIPT, run_name="__main__")
    finally:
        sys.argv = old_argv
        os.chdir(old_cwd)
        torch.optim.Adam.step = orig_step
    out["meta.json"] = np.frombuffer(json.dumps({
        "config": name, "args": args, "seed": cfg.get("seed", 1), "n_iter": n_iter, "threads": threads,
        "n_images": cfg.get("n_images", 64), "torch": torch.__version__}).encode(), dtype=np.uint8).copy()
    path = os.path.join(HERE, f"traj_{name}_t{threads}.npz")
    np.savez_compressed(path, **out)
    return path


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "--trajectory":
        # --trajectory NAME [THREADS ...]: one fresh interpreter per thread count
        from tests.golden.configs import TRAJECTORIES, traj_iters
        name = sys.argv[2]
        threads = [int(t) for t in sys.argv[3:]] or list(TRAJECTORIES[name])
        if len(threads) == 1:
            print(name, threads[0], "->", run_trajectory(name, threads[0], traj_iters(name)), flush=True)
        else:
            import subprocess
            for th in threads:
                r = subprocess.run([sys.executable, os.path.abspath(__file__), "--trajectory", name, str(th)],
                                   capture_output=True, text=True)
                print(name, th, "ok" if r.returncode == 0 else "FAILED\n" + r.stderr[-2000:], flush=True)
        sys.exit(0)
    names = sys.argv[1:] or PINNED
    if len(names) == 1:
        print(names[0], "->", run_config(names[0], CONFIGS[names[0]]), flush=True)
    else:  # one fresh interpreter per config: the reference mutates global torch state
        import subprocess
        for n in names:
            r = subprocess.run([sys.executable, os.path.abspath(__file__), n],
                               capture_output=True, text=True)
            print(n, "ok" if r.returncode == 0 else "FAILED\n" + r.stderr[-2000:], flush=True)
