"""Sample / FID image export (GLI:563-565, 752-768): device quantisation vs the CPU
restatement of torchvision's make_grid/save_image (oracle/save_image.py; parity unpinned:
torchvision is absent), and the PNG encoder vs PIL's decoder."""
import os
import tempfile

import numpy as np
import pytest
import torch

from oracle.save_image import save_image_pixels


def test_png_encoder_roundtrip_pil():
    from PIL import Image
    from relativisticgan_amd.images import write_png
    rng = np.random.default_rng(0)
    for shape in ((5, 7, 3), (16, 9, 1), (1, 1, 3)):
        a = rng.integers(0, 256, size=shape, dtype=np.uint8)
        path = os.path.join(tempfile.mkdtemp(), "x.png")
        write_png(path, a)
        b = np.asarray(Image.open(path))
        assert np.array_equal(b.reshape(shape), a)


def test_oracle_grid_layout():
    t = torch.arange(5 * 3 * 2 * 2, dtype=torch.float32).view(5, 3, 2, 2) / 60.0
    px = save_image_pixels(t, nrow=2, padding=1)
    assert tuple(px.shape) == (3 * 3 + 1, 2 * 3 + 1, 3)
    assert px[0].sum() == 0 and px[:, 0].sum() == 0  # padding is pad value 0


@pytest.mark.gpu
@pytest.mark.parametrize("B,normalize,nrow,padding", [(64, True, 8, 2), (10, True, 8, 2), (7, False, 3, 1),
                                                      (1, True, 8, 2), (33, False, 8, 2)])
def test_device_grid_matches_torchvision_semantics(B, normalize, nrow, padding):
    from relativisticgan_amd.images import to_u8
    torch.manual_seed(B)
    x = torch.tanh(torch.randn(B, 3, 16, 12) * 2)
    x[0, 0, 0, 0] = 1.0  # exact extremes
    got = to_u8(x.cuda(), normalize=normalize, grid=True, nrow=nrow, padding=padding).cpu()
    want = save_image_pixels(x, nrow=nrow, padding=padding, normalize=normalize)
    assert got.shape == want.shape
    assert torch.equal(got, want)


@pytest.mark.gpu
def test_device_extra_images_match_reference_expression():
    """GLI:766: save_image(fake[i]*.50+.50, normalize=False, padding=0), one file per image."""
    from PIL import Image
    from relativisticgan_amd.images import save_images
    torch.manual_seed(3)
    x = torch.tanh(torch.randn(6, 3, 20, 20) * 3).cuda().contiguous(memory_format=torch.channels_last)
    d = tempfile.mkdtemp()
    paths = [os.path.join(d, "fake_samples_%05d.png" % i) for i in range(6)]
    save_images(x, paths)
    for i, p in enumerate(paths):
        want = save_image_pixels(x[i].cpu() * .50 + .50, padding=0)
        assert np.array_equal(np.asarray(Image.open(p)), want.numpy())
