"""Real-image pipeline (GLI:159-179): ImageFolder order, decode/resize once into a uint8 HBM
tensor, device gather + ToTensor/Normalize vs the CPU restatement of torchvision's transform
(oracle/image_folder.py; parity unpinned: torchvision is absent)."""
import os
import tempfile

import numpy as np
import pytest
import torch
from PIL import Image


def _make_folder(root):
    rng = np.random.default_rng(5)
    specs = [("cats", "b.png", (40, 30), "RGB"), ("cats", "a.jpg", (64, 64), "RGB"),
             ("cats", "sub/c.png", (20, 50), "L"), ("dogs", "z.bmp", (33, 33), "RGB"),
             ("dogs", "y.png", (16, 16), "RGBA"), ("dogs", "notes.txt", None, None)]
    for cls, name, size, mode in specs:
        path = os.path.join(root, cls, name)
        os.makedirs(os.path.dirname(path), exist_ok=True)
        if size is None:
            open(path, "w").write("x")
            continue
        ch = {"RGB": 3, "L": 1, "RGBA": 4}[mode]
        a = rng.integers(0, 256, size=(size[1], size[0], ch), dtype=np.uint8)
        Image.fromarray(a[:, :, 0] if ch == 1 else a, mode).save(path)
    return root


def test_imagefolder_order_and_decode_cpu():
    from relativisticgan_amd.data import find_images, load_image_folder
    root = _make_folder(tempfile.mkdtemp())
    rel = [(os.path.relpath(p, root), c) for p, c in find_images(root)]
    assert rel == [("cats/a.jpg", 0), ("cats/b.png", 0), ("cats/sub/c.png", 0), ("dogs/y.png", 1),
                   ("dogs/z.bmp", 1)]
    u8 = load_image_folder(root, 24, device=None)
    assert u8.dtype == torch.uint8 and tuple(u8.shape) == (5, 3, 24, 24)


@pytest.mark.gpu
def test_device_batches_match_torchvision_transform():
    from oracle.image_folder import batch
    from relativisticgan_amd import kernels as K
    from relativisticgan_amd.data import find_images, load_image_folder
    root = _make_folder(tempfile.mkdtemp())
    paths = [p for p, _ in find_images(root)]
    images = load_image_folder(root, 24)
    np.random.seed(1)
    for _ in range(3):
        idx = np.random.choice(len(paths), size=4, replace=False)  # GLI:176
        got = K.gather_images(images, torch.from_numpy(idx.astype(np.int64)).cuda()).cpu()
        want = batch(paths, idx, 24)
        assert torch.equal(got, want)
