"""CPU restatement of torchvision.utils.make_grid + save_image's pixel pipeline.

TEST INFRASTRUCTURE ONLY (imported by tests/, never by the product).  The reference writes
its sample grid with ``vutils.save_image(fake_test.data, path, normalize=True)`` (GLI:565)
and its FID images with ``vutils.save_image(fake[i].data*.50+.50, path, normalize=False,
padding=0)`` (GLI:766-768).  torchvision is not installed here and is unpinned by the
reference (README.md:11 "conda install pytorch torchvision"), so this follows the
torchvision >= 0.8 source of make_grid / save_image (normalize: clamp to [min, max],
sub_(min).div_(max(max - min, 1e-5)); grid nrow=8, padding=2, pad_value=0; quantise
mul(255).add_(0.5).clamp_(0, 255).to(uint8)) -- parity unpinned: no reference fixture
covers these bytes.
"""
import math

import torch


def make_grid(tensor, nrow=8, padding=2, normalize=False, pad_value=0.0):
    t = tensor.detach().float().cpu().clone()
    if t.dim() == 3:
        t = t.unsqueeze(0)
    if normalize:
        low, high = float(t.min()), float(t.max())
        t.clamp_(min=low, max=high)
        t.sub_(low).div_(max(high - low, 1e-5))
    if t.size(0) == 1:
        return t.squeeze(0)
    nmaps = t.size(0)
    xmaps = min(nrow, nmaps)
    ymaps = int(math.ceil(float(nmaps) / xmaps))
    height, width = int(t.size(2) + padding), int(t.size(3) + padding)
    grid = t.new_full((t.size(1), height * ymaps + padding, width * xmaps + padding), pad_value)
    k = 0
    for y in range(ymaps):
        for x in range(xmaps):
            if k >= nmaps:
                break
            grid.narrow(1, y * height + padding, height - padding).narrow(
                2, x * width + padding, width - padding).copy_(t[k])
            k += 1
    return grid


def save_image_pixels(tensor, nrow=8, padding=2, normalize=False):
    """The uint8 HWC array save_image would hand to PIL."""
    grid = make_grid(tensor, nrow=nrow, padding=padding, normalize=normalize)
    return grid.mul(255).add_(0.5).clamp_(0, 255).permute(1, 2, 0).to(torch.uint8)
