"""Generate FID / sample images from a checkpoint (code/inference_art.py; GLI:752-768).

``python -m relativisticgan_amd.generate --load state_NN.pth [reference G flags]
--gen_extra_images N --extra_folder DIR`` rebuilds G from the same flags as training,
loads ``G_state`` from the reference-format checkpoint (GLI:737-747 keys), and writes N
images as ``DIR/<current_set_images>/fake_samples_%05d.png`` -- 100 per G forward in train
mode, ``fake*.5+.5`` quantised like torchvision.save_image (relativisticgan_amd.images).

inference_art.py itself swaps G's last layer for an ``End-ConvTranspose2dNew`` (k2 s2 p1)
that no checkpoint holds and loads with ``strict=False`` (it stays randomly initialised);
this tool keeps the trained G's own last layer instead.
"""
import sys

import torch

from .config import parse
from .nets import DCGAN_G
from .train import generate_extra_images


def main(argv=None):
    p = parse(argv)
    if not p.load:
        raise SystemExit("--load <checkpoint> is required")
    if not torch.cuda.is_available():
        raise SystemExit("image generation runs on the MI355X only")
    if p.seed is not None:
        torch.manual_seed(p.seed)
    G = DCGAN_G(p)
    ck = torch.load(p.load, map_location="cpu", weights_only=True)
    G.load_state_dict(ck["G_state"])
    G.to("cuda")
    folder = "%s/%01d/" % (p.extra_folder, ck.get("current_set_images", 0))
    generate_extra_images(G, p, folder)
    return folder


if __name__ == "__main__":
    print(main(sys.argv[1:]))
