"""Sample / FID image export (GLI:563-565, GLI:752-768; code/inference_art.py:118-127).

The reference writes images with ``torchvision.utils.save_image`` (absent from this image):
``make_grid`` tiling (nrow 8, padding 2, pad value 0), optional min/max normalisation over
the batch, ``mul(255).add_(0.5).clamp_(0, 255).to(uint8)``, then PIL's PNG encoder.  Here the
float -> uint8 step (tiling and normalisation fused) runs on the MI355X
(``rgan_images_to_u8``), only the uint8 pixels cross PCIe, and PNG encoding (zlib, RGB/grey
8-bit, filter 0) runs on host threads -- zlib releases the GIL, so a batch of 100 extra
images encodes in parallel.  Pixel values equal torchvision's; the PNG byte streams need not.
"""
import ctypes
import os
import struct
import zlib
from concurrent.futures import ThreadPoolExecutor

import torch

from . import _lib as L


def to_u8(x, scale=1.0, shift=0.0, normalize=False, grid=False, nrow=8, padding=2):
    """[B,C,H,W] float (CUDA) -> uint8 CUDA tensor: [B,H,W,C] (grid=False) or the
    make_grid image [Hg,Wg,C] (grid=True; a single image is returned unpadded, like
    make_grid for B == 1)."""
    L.require_cuda(x)
    if x.dim() == 3:
        x = x.unsqueeze(0)
    x = x.float()
    B, C, H, W = x.shape
    single = grid and B == 1  # make_grid returns a lone image unpadded
    if single:
        grid, padding = False, 0
    lib = L.lib()
    rng = None
    if normalize:
        rng = torch.empty(2, dtype=torch.float32, device=x.device)
        src = x.contiguous()
        ws = L.workspace(lib.rgan_minmax_ws_bytes(src.numel()), x.device)
        L.check(lib.rgan_minmax(L.ptr(src), src.numel(), L.ptr(rng), L.ptr(ws), L.stream()), "rgan_minmax")
    if grid:
        xmaps = min(nrow, B)
        ymaps = (B + xmaps - 1) // xmaps
        out = torch.empty(((H + padding) * ymaps + padding, (W + padding) * xmaps + padding, C), dtype=torch.uint8,
                          device=x.device)
    else:
        out = torch.empty((B, H, W, C), dtype=torch.uint8, device=x.device)
    strides = (ctypes.c_longlong * 4)(*x.stride())
    L.check(lib.rgan_images_to_u8(L.ptr(x), B, C, H, W, strides, float(scale), float(shift), L.ptr(rng),
                                  int(grid), int(nrow), int(padding), L.ptr(out), L.stream()),
            "rgan_images_to_u8")
    return out[0] if single else out


def encode_png(u8_hwc):
    """PNG bytes of an [H, W, C] (C = 1 or 3) uint8 array (numpy or CPU tensor)."""
    a = u8_hwc.numpy() if torch.is_tensor(u8_hwc) else u8_hwc
    if a.ndim == 2:
        a = a[:, :, None]
    H, W, C = a.shape
    if C not in (1, 3, 4):
        raise ValueError(f"PNG export supports 1, 3 or 4 channels, got {C}")
    color = {1: 0, 3: 2, 4: 6}[C]
    raw = bytearray()
    rows = a.reshape(H, W * C)
    for r in range(H):
        raw.append(0)  # filter type 0 (none)
        raw += rows[r].tobytes()

    def chunk(tag, data):
        return struct.pack(">I", len(data)) + tag + data + struct.pack(">I", zlib.crc32(tag + data) & 0xFFFFFFFF)
    return (b"\x89PNG\r\n\x1a\n" + chunk(b"IHDR", struct.pack(">IIBBBBB", W, H, 8, color, 0, 0, 0))
            + chunk(b"IDAT", zlib.compress(bytes(raw), 6)) + chunk(b"IEND", b""))


def write_png(path, u8_hwc):
    with open(path, "wb") as f:
        f.write(encode_png(u8_hwc))


_POOL = None


def _pool():
    global _POOL
    if _POOL is None:
        _POOL = ThreadPoolExecutor(max_workers=min(16, os.cpu_count() or 1))
    return _POOL


def save_image(x, path, normalize=False, nrow=8, padding=2, scale=1.0, shift=0.0):
    """torchvision.utils.save_image(x*scale+shift, path, normalize=..., nrow=..., padding=...)
    for a [B,C,H,W] or [C,H,W] CUDA tensor (GLI:565: normalize=True, default grid)."""
    img = to_u8(x, scale, shift, normalize=normalize, grid=True, nrow=nrow, padding=padding)
    write_png(path, img.cpu())


def save_images(x, paths, scale=0.5, shift=0.5):
    """One PNG per image of x [B,C,H,W] (CUDA) -- the reference's extra-image loop
    ``save_image(fake[i]*.50+.50, path_i, normalize=False, padding=0)`` (GLI:766-768).
    Encoding runs on a thread pool; returns when every file is written."""
    if len(paths) != x.shape[0]:
        raise ValueError(f"{x.shape[0]} images but {len(paths)} paths")
    u8 = to_u8(x, scale, shift, normalize=False, grid=False).cpu()
    list(_pool().map(lambda a: write_png(a[1], u8[a[0]]), enumerate(paths)))
