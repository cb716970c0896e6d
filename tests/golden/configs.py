"""Fixture configurations shared by the golden generator and the parity tests.

Each entry is a set of reference CLI flags (GLI:17-62).  Sizes are reduced (h=8,
z=16, B=8, S=32) so the oracle replays them in seconds.  Large tensors are stored
as sha1 + sums + sampled elements: the sha1 pins the oracle bitwise (CPU tests),
the samples/sums let a GPU result be compared within tolerance.  The full-size
configs of BASELINE.json are covered by size-independent property tests.
"""
import hashlib

import numpy as np
import torch

FULL_LIMIT = 1024  # tensors above this many elements are stored as summaries (sha1 + stats + samples)

_SMALL = {"image_size": 32, "batch_size": 8, "z_size": 16, "G_h_size": 8, "D_h_size": 8,
          "n_iter": 3}


def _cfg(**kw):
    args = dict(_SMALL)
    args.update(kw)
    return {"args": args, "seed": 1, "n_images": 64}


CONFIGS = {
    "sgan": _cfg(loss_D=1),
    "lsgan": _cfg(loss_D=2),
    "wgangp": _cfg(loss_D=3),
    "hinge": _cfg(loss_D=4),
    "rsgan": _cfg(loss_D=5),
    "rasgan": _cfg(loss_D=6),
    "ralsgan": _cfg(loss_D=7),
    "rahinge": _cfg(loss_D=8),
    "ralsgan64": _cfg(loss_D=7, image_size=64),
    "rahinge_spectral": _cfg(loss_D=8, spectral="True"),
    "ralsgan_gp": _cfg(loss_D=7, grad_penalty="True"),
    "rasgan_spectralG": _cfg(loss_D=6, spectral_G="True"),
    "ralsgan_nobn": _cfg(loss_D=7, no_batch_norm_G="True", no_batch_norm_D="True"),
    "ralsgan_tanh": _cfg(loss_D=7, Tanh_GD="True"),
    "ralsgan_selu": _cfg(loss_D=7, SELU="True"),
    "ralsgan_wd": _cfg(loss_D=7, weight_decay=0.01, decay=0.1),
    "ralsgan_nnconv": _cfg(loss_D=7, NN_conv="True"),
    "rasgan_nnconv_spectralG": _cfg(loss_D=6, NN_conv="True", spectral_G="True"),
    # PacGAN-2 (code/GAN_losses_iter_PAC.py): no reference fixture -- the script fails at
    # PAC:609 on the pinned torch (`z.data.resize_(2B)` no longer reshapes the Variable z, so
    # G(z) returns B samples and the channel-wise packing of fake[B:2B] is empty).  The oracle
    # restates the script's torch-0.4 semantics (2B z per step, stale D-step fake reused by
    # the G step at PAC:674); parity of these configs is GPU-vs-oracle only ("unpinned").
    "ralsgan_pac2": dict(_cfg(loss_D=7), pac=2, golden=False),
    "sgan_pac2_gp": dict(_cfg(loss_D=1, grad_penalty="True"), pac=2, golden=False),
    "rahinge_pac2_arch1": {"args": {"image_size": 32, "batch_size": 8, "z_size": 16, "loss_D": 8, "arch": 1,
                                    "n_iter": 2}, "seed": 1, "n_images": 64, "pac": 2, "golden": False},
    # the north-star target at FULL size: RaLSGAN DCGAN 64x64, batch 32, h = z = 128 (the
    # reference defaults, GLI:20-25) = BASELINE configs[0]; 2 iterations
    "ralsgan_c1": {"args": {"image_size": 64, "batch_size": 32, "z_size": 128, "G_h_size": 128,
                            "D_h_size": 128, "loss_D": 7, "n_iter": 2}, "seed": 1, "n_images": 64},
    # WGAN-GP at 64x64 on the DCGAN nets (SURVEY C4'; GLI:646-658), reduced width
    "wgangp64": {"args": {"image_size": 64, "batch_size": 16, "z_size": 32, "G_h_size": 16, "D_h_size": 16,
                          "loss_D": 3, "n_iter": 3}, "seed": 1, "n_images": 64},
    "wgangp_arch1": {"args": {"image_size": 32, "batch_size": 8, "z_size": 16, "loss_D": 3,
                              "arch": 1, "n_iter": 2}, "seed": 1, "n_images": 64},
    "rahinge_arch1": {"args": {"image_size": 32, "batch_size": 8, "z_size": 16, "loss_D": 8,
                               "arch": 1, "n_iter": 2}, "seed": 1, "n_images": 64},
    # the reference writes state_01.pth itself after iteration 1 (--gen_every 2 --save True,
    # GLI:729-747); the file is kept as tests/golden/ralsgan_ckpt_state_01.pth
    "ralsgan_ckpt": dict(_cfg(loss_D=7, n_iter=2), save_every=2),
    # the other single-GPU BASELINE configs at FULL size (h = z = 128), 2 iterations each,
    # captured at 8 threads (the reference is bitwise deterministic at a fixed thread count)
    # C2 = configs[1]: RaSGAN DCGAN 128x128, batch 64 (GLI:636-637, 699-702)
    "rasgan_c2": {"args": {"image_size": 128, "batch_size": 64, "z_size": 128, "G_h_size": 128,
                           "D_h_size": 128, "loss_D": 6, "n_iter": 2}, "seed": 1, "n_images": 128,
                  "threads": 8},
    # C4' = configs[3] on the DCGAN nets at 64x64, h = 128, batch 32 (GLI:646-658)
    "wgangp_c4p": {"args": {"image_size": 64, "batch_size": 32, "z_size": 128, "G_h_size": 128,
                            "D_h_size": 128, "loss_D": 3, "n_iter": 2}, "seed": 1, "n_images": 64,
                   "threads": 8},
    # C5 = configs[4]: spectral-norm RaHingeGAN 128x128, batch 32 (GLI:408-446, 641, 709)
    "rahinge_spectral_c5": {"args": {"image_size": 128, "batch_size": 32, "z_size": 128, "G_h_size": 128,
                                     "D_h_size": 128, "loss_D": 8, "spectral": "True", "n_iter": 2},
                            "seed": 1, "n_images": 64, "threads": 8},
    # C4 = configs[3] on the reference's "standard CNN" (arch 1, 32x32 only: GLI:186-319) at the
    # bench's batch 32, z = 128 -- the bench's C4 workload at full size (round 5; the arch-1
    # configs above run B = 8)
    "wgangp_c4": {"args": {"image_size": 32, "batch_size": 32, "z_size": 128, "loss_D": 3, "arch": 1,
                           "n_iter": 2}, "seed": 1, "n_images": 64, "threads": 8},
    # C3 = the per-GPU shard of configs[2] (the bench's headline workload): RaLSGAN DCGAN
    # 256x256, batch 32, h = z = 128 (GLI:329 mult = S/8 -> 5 middle layers per net; heads
    # GLI:639, 705).  ~2.5 min of reference CPU time per iteration at 8 threads.
    "ralsgan_c3": {"args": {"image_size": 256, "batch_size": 32, "z_size": 128, "G_h_size": 128,
                            "D_h_size": 128, "loss_D": 7, "n_iter": 2}, "seed": 1, "n_images": 64,
                   "threads": 8},
}

# full-size configs: minutes of CPU oracle time each (GPU parity runs them with all host cores)
FULL_SIZE = ("ralsgan_c1", "rasgan_c2", "wgangp_c4p", "wgangp_c4", "rahinge_spectral_c5", "ralsgan_c3")
# configs too slow for the default CPU suite's bitwise oracle pin (RGAN_SLOW=1 runs them)
SLOW_PIN = ("ralsgan_c3",)

# 100-iteration scalar trajectories of the unmodified reference at several thread counts
# (SURVEY §8(c)(iii)): the spread between thread counts is the drift envelope.  Keys of
# TRAJECTORIES name a config of CONFIGS whose args are used with n_iter = traj_iters(name)
# (TRAJ_ITERS, or the reduced count of TRAJ_ITERS_OF: C2 costs ~6 s per reference iteration at
# 8 threads and ~40 s at 1).
TRAJ_ITERS = 100
TRAJECTORIES = {
    "ralsgan_c1": (1, 2, 4, 8),           # north-star RaLSGAN 64^2 (GLI:639, 705)
    "wgangp_c4": (1, 2, 4, 8),            # arch-1 WGAN-GP 32^2 (GLI:183-319, 646-658)
    "rasgan_c2": (1, 4, 8),               # RaSGAN 128^2 B64 (GLI:636-637, 699-702), reduced iterations
    "rahinge_spectral_c5": (1, 4, 8),     # spectral RaHinge 128^2 (GLI:408-446, 641, 709)
}
TRAJ_ITERS_OF = {"rasgan_c2": 30}


def traj_iters(name):
    return TRAJ_ITERS_OF.get(name, TRAJ_ITERS)


# configs with a reference fixture (tests/golden/<name>.npz) pinning the oracle bitwise
PINNED = [n for n, c in CONFIGS.items() if c.get("golden", True)]


def summarize_indices(numel, count=64, seed=97):
    """Positions sampled from a large tensor (same on every machine)."""
    rng = np.random.default_rng(seed + numel)
    return np.sort(rng.choice(numel, size=min(count, numel), replace=False))


class Recorder:
    def __init__(self):
        self.store = {}

    def put(self, key, t):
        t = t.detach().to(torch.float32).contiguous().cpu() if t.is_floating_point() else t.detach().cpu()
        arr = t.numpy()
        if arr.size <= FULL_LIMIT:
            self.store[key] = arr.copy()
        else:
            flat = arr.reshape(-1).astype(np.float32)
            idx = summarize_indices(flat.size)
            self.store[key + "@sample"] = flat[idx].copy()
            self.store[key + "@shape"] = np.array(arr.shape, dtype=np.int64)
            self.store[key + "@sum"] = np.array([flat.astype(np.float64).sum(),
                                                 (flat.astype(np.float64) ** 2).sum()])
            self.store[key + "@sha1"] = np.frombuffer(
                hashlib.sha1(flat.tobytes()).hexdigest().encode(), dtype=np.uint8).copy()

    def state(self, prefix, module):
        for k, v in module.state_dict().items():
            self.put(f"{prefix}.{k}", v)

    def optim(self, prefix, opt, module):
        names = [n for n, _ in module.named_parameters()]
        for p, n in zip(module.parameters(), names):
            st = opt.state.get(p, {})
            if st:
                self.put(f"{prefix}.{n}.exp_avg", st["exp_avg"])
                self.put(f"{prefix}.{n}.exp_avg_sq", st["exp_avg_sq"])
                self.store[f"{prefix}.{n}.step"] = np.array([float(st["step"])])
