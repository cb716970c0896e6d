"""D image-layer conv (conv_img_in) at full batch sizes vs MIOpen fp32 (GPU diagnostic).

usage: python tools/img_in_check.py  (RGAN_LIB=... to load a variant library)
Prints per shape the worst per-sample relative error and, for a bad sample, where the
bad outputs lie (channels, rows, columns)."""
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from relativisticgan_amd import kernels as K  # noqa: E402


def main():
    g = K.ConvGeom(4, 2, 1, False)
    for B, S, C in ((32, 128, 128), (64, 128, 128), (128, 128, 128), (8, 256, 128), (32, 256, 128), (64, 256, 128),
                    (32, 64, 128), (64, 64, 128), (32, 256, 32), (32, 128, 256)):
        torch.manual_seed(B + S)
        img = torch.rand(B, 3, S, S, device="cuda") * 2 - 1
        w = torch.nn.Parameter(torch.randn(C, 3, 4, 4, device="cuda") * 0.05)
        y = K.conv_fwd(img, w, g, act="lrelu", alpha=0.2)
        ref = F.leaky_relu(F.conv2d(img.double(), w.detach().double(), stride=2, padding=1), 0.2)
        d = (y.double() - ref).abs()
        per = d.flatten(1).amax(1) / ref.abs().amax()
        bad = (per > 1e-5).nonzero().flatten().tolist()
        print(f"B={B} S={S} C={C}: worst sample err {per.max():.2e}; bad samples {bad[:16]}{'...' if len(bad) > 16 else ''} "
              f"({len(bad)})", flush=True)
        if bad:
            n = bad[0]
            m = d[n] > 1e-5 * ref.abs().amax()
            cs = m.any(2).any(1).nonzero().flatten().tolist()
            hs = m.any(0).any(1).nonzero().flatten().tolist()
            ws = m.any(0).any(0).nonzero().flatten().tolist()
            print(f"   sample {n}: {int(m.sum())} bad; channels {cs[:40]}; rows {hs[:40]}; cols {ws[:40]}", flush=True)


if __name__ == "__main__":
    main()
