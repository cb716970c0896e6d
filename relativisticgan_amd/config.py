"""The reference's command-line surface (GLI:14-62): same flag names, types, defaults.

Plus this build's own switches (prefixed ``--rgan_``), which the reference lacks:
``--rgan_rng`` (``host``: draw z/u/batches from the CPU generators in the reference's
order, bit-compatible inputs; ``device``: draw on the GPU, for throughput runs) and
``--rgan_sync_bn`` (BatchNorm statistics under data parallelism: default off = the
reference's DataParallel, each rank normalises with its own shard; on = SyncBN over the
global batch), ``--rgan_pac 2`` (the PacGAN-2 script,
code/GAN_losses_iter_PAC.py, which shares this CLI) and ``--rgan_script`` (the defaults of
GAN_losses_iter / GAN_losses_iter_art / GAN_losses_iter_PAC).
"""
import argparse


def str_to_bool(s):
    """GLI:14-15."""
    return s.lower() in ("true", "yes", "on", "t", "1")


_FLAGS = [
    ("image_size", int, 64), ("batch_size", int, 32), ("n_colors", int, 3), ("z_size", int, 128),
    ("G_h_size", int, 128), ("D_h_size", int, 128), ("lr_D", float, .0001), ("lr_G", float, .0001),
    ("n_iter", int, 100000), ("beta1", float, 0.5), ("beta2", float, 0.999), ("decay", float, 0),
    ("SELU", "bool", False), ("NN_conv", "bool", False), ("seed", int, None),
    ("input_folder", str, "/home/alexia/Datasets/Meow_64x64"),
    ("output_folder", str, "/home/alexia/Dropbox/Ubuntu_ML/Output/GANlosses"),
    ("inception_folder", str, "/home/alexia/Inception"), ("load", str, None), ("cuda", "bool", True),
    ("n_gpu", int, 1), ("loss_D", int, 1), ("Diters", int, 1), ("Giters", int, 1), ("penalty", float, 10),
    ("spectral", "bool", False), ("spectral_G", "bool", False), ("weight_decay", float, 0),
    ("gen_extra_images", int, 50000), ("gen_every", int, 100000), ("extra_folder", str, "/home/alexia/Output/Extra"),
    ("show_graph", "bool", False), ("no_batch_norm_G", "bool", False), ("no_batch_norm_D", "bool", False),
    ("Tanh_GD", "bool", False), ("grad_penalty", "bool", False), ("arch", int, 0), ("print_every", int, 1000),
    ("save", "bool", True), ("CIFAR10", "bool", False), ("CIFAR10_input_folder", str, "/home/alexia/Datasets/CIFAR10"),
]


# code/GAN_losses_iter_art.py is GLI with these defaults (its only differences, art:20-60)
ART_DEFAULTS = {
    "image_size": 128, "loss_D": 7, "gen_extra_images": 2000, "gen_every": 2000,
    "input_folder": "/home/ubuntu/datasets/meow_128x128", "output_folder": "/home/ubuntu/RelativisticGAN/output",
    "inception_folder": "/home/ubuntu/models/Inception", "extra_folder": "/home/ubuntu/RelativisticGAN/extra",
    "CIFAR10_input_folder": "/home/ubuntu/datasets/CIFAR10",
}
SCRIPTS = ("GAN_losses_iter", "GAN_losses_iter_art", "GAN_losses_iter_PAC")


def make_parser(script="GAN_losses_iter"):
    """The CLI of one of the reference's three training scripts (same flags; the art script
    changes defaults, the PAC script packs 2 samples for D)."""
    p = argparse.ArgumentParser(description="RelativisticGAN training (MI355X build)")
    p.register("type", "bool", str_to_bool)
    for name, typ, default in _FLAGS:
        if script == "GAN_losses_iter_art":
            default = ART_DEFAULTS.get(name, default)
        if typ is str:
            p.add_argument("--" + name, default=default)
        else:
            p.add_argument("--" + name, type=typ, default=default)
    p.add_argument("--rgan_script", choices=SCRIPTS, default=script,
                   help="which reference script's defaults/behaviour to follow")
    p.add_argument("--rgan_rng", choices=("host", "device"), default="host")
    p.add_argument("--rgan_sync_bn", type="bool", default=False)
    p.add_argument("--rgan_batch_D", type="bool", default=None,
                   help="run the D step's D(x) and D(x_fake) as one batched pass (per-call BN kept); "
                        "default: on (one process and data parallel)")
    p.add_argument("--rgan_batch_G", type="bool", default=None,
                   help="run the G step's D(G(z)) and D(x) (heads 5-8) as one batched pass (per-call BN "
                        "kept, gradient through the D(G(z)) half only); default: on")
    p.add_argument("--rgan_pac", dest="pac", type=int, default=2 if script == "GAN_losses_iter_PAC" else 1,
                   choices=(1, 2),
                   help="2 = PacGAN-2, the reference's code/GAN_losses_iter_PAC.py (D sees 2 samples packed "
                        "channel-wise)")
    p.add_argument("--rgan_perf_log", type="bool", default=True,
                   help="after each reference log line, a line with img/s and MFMA%% of the training "
                        "iterations since the previous one (sample PNGs, checkpoints and extra images excluded)")
    p.add_argument("--rgan_synthetic", type=int, default=0,
                   help="use N synthetic images instead of an image folder (no torchvision here)")
    return p


def parse(argv=None):
    pre = argparse.ArgumentParser(add_help=False)
    pre.add_argument("--rgan_script", choices=SCRIPTS, default="GAN_losses_iter")
    script = pre.parse_known_args(argv)[0].rgan_script
    return make_parser(script).parse_args(argv)


def make_param(**overrides):
    """Namespace with the reference defaults, then ``overrides``."""
    ns = make_parser().parse_args([])
    for k, v in overrides.items():
        cur = getattr(ns, k, None)
        if isinstance(v, str) and isinstance(cur, bool):
            v = str_to_bool(v)
        setattr(ns, k, v)
    return ns


TITLES = {1: "GAN_", 2: "LSGAN_", 3: "WGANGP_", 4: "HingeGAN_", 5: "RSGAN_", 6: "RaSGAN_", 7: "RaLSGAN_",
          8: "RaHingeGAN_"}
