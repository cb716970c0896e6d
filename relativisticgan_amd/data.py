"""Real-image dataset (GLI:159-179): ImageFolder + Resize((S, S)) + ToTensor + Normalize(0.5, 0.5).

The reference decodes and resizes every sampled image again for every batch, synchronously
in the training loop (``[data[i][0] for i in random_indexes]``, GLI:177), which would starve
a GPU.  Here the whole folder is decoded and resized ONCE, on host threads, into a uint8
[N, C, S, S] tensor that stays resident in HBM (a 64x64 RGB image is 12 KiB: 10^5 images are
1.2 GB of the 288 GB); each batch is then a device gather fused with ToTensor + Normalize
(``kernels.gather_images`` -> ``rgan_gather_images_u8``).  The numpy RNG draws the batch
indices exactly as the reference (``numpy.random.choice(N, B, replace=False)``).

File discovery and order follow torchvision.datasets.ImageFolder (classes = sorted
sub-directories, files walked in sorted order, torchvision's IMG_EXTENSIONS), decoding
follows its default ``pil_loader`` (``Image.open(f).convert('RGB')``) and Resize on a PIL
image is ``img.resize((S, S), Image.BILINEAR)``.  torchvision itself is not installed here
(and is unpinned by the reference), so this restates those published behaviours.
"""
import os
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import torch

IMG_EXTENSIONS = (".jpg", ".jpeg", ".png", ".ppm", ".bmp", ".pgm", ".tif", ".tiff", ".webp")


def find_images(root):
    """[(path, class_index)] in ImageFolder order."""
    classes = sorted(e.name for e in os.scandir(root) if e.is_dir())
    if not classes:
        raise FileNotFoundError(f"no class folders under {root} (ImageFolder expects root/<class>/<image>)")
    out = []
    for ci, cls in enumerate(classes):
        for dirpath, _dirs, files in sorted(os.walk(os.path.join(root, cls), followlinks=True)):
            for f in sorted(files):
                if f.lower().endswith(IMG_EXTENSIONS):
                    out.append((os.path.join(dirpath, f), ci))
    if not out:
        raise FileNotFoundError(f"no images with extensions {IMG_EXTENSIONS} under {root}")
    return out


def _load(path, size, n_colors):
    from PIL import Image
    with open(path, "rb") as f:
        img = Image.open(f)
        img = img.convert("RGB" if n_colors == 3 else "L")
    img = img.resize((size, size), Image.BILINEAR)
    a = np.asarray(img, dtype=np.uint8)
    return a[:, :, None] if a.ndim == 2 else a


def load_image_folder(root, size, n_colors=3, device="cuda", workers=None):
    """Decode + resize every image under ``root`` -> uint8 [N, C, S, S] on ``device``."""
    paths = [p for p, _ in find_images(root)]
    workers = workers or min(16, os.cpu_count() or 1)
    out = np.empty((len(paths), size, size, n_colors), dtype=np.uint8)

    def work(i):
        out[i] = _load(paths[i], size, n_colors)
    with ThreadPoolExecutor(max_workers=workers) as ex:
        list(ex.map(work, range(len(paths))))
    t = torch.from_numpy(out).permute(0, 3, 1, 2).contiguous()
    return t.to(device) if device is not None else t
