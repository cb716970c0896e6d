"""CPU restatement of the reference's data transform (GLI:160-166, 169, 176-177).

TEST INFRASTRUCTURE ONLY.  torchvision (absent here, unpinned by the reference) would run,
per sampled index: ImageFolder's pil_loader (Image.open(f).convert('RGB')), Resize((S, S))
on the PIL image (img.resize((S, S), BILINEAR)), ToTensor (HWC uint8 -> CHW float / 255) and
Normalize(mean 0.5, std 0.5) (sub_(0.5).div_(0.5)).  Parity unpinned: no reference fixture.
"""
import numpy as np
import torch
from PIL import Image


def load_sample(path, size):
    with open(path, "rb") as f:
        img = Image.open(f).convert("RGB")
    img = img.resize((size, size), Image.BILINEAR)
    t = torch.from_numpy(np.array(img, dtype=np.uint8)).permute(2, 0, 1).contiguous()
    t = t.to(torch.float32).div(255)
    return t.sub_(0.5).div_(0.5)


def batch(paths, indexes, size):
    return torch.stack([load_sample(paths[i], size) for i in indexes], 0)
