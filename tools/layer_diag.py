"""Per-layer forward diagnosis (GPU box): run a fixture config's G or D layer by layer on
the HIP path and compare each fused layer's output with the same layer computed in
float64 on the CPU from the GPU layer's own (upcast) input -- the local error of every
layer, independent of what the layers before it did.

usage: python tools/layer_diag.py CONFIG [D|G] [segments]
"""
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, ".")
from tests.golden.configs import CONFIGS  # noqa: E402
from tests.oracle_replay import dataset_for, param_for  # noqa: E402


def ref_layer(layer, h, segs, u, v):
    spec, conv, bn = layer.spec, layer.conv, layer.bn
    w = layer.weight().detach().double().cpu()
    x = h.detach().double().cpu()
    if spec.spectral:
        W = w.permute(1, 0, 2, 3) if spec.geom.transposed else w
        Wm = W.reshape(W.shape[0], -1)
        v1 = F.normalize(Wm.t() @ u.double().cpu(), dim=0, eps=1e-12)
        u1 = F.normalize(Wm @ v1, dim=0, eps=1e-12)
        w = w / torch.dot(u1, Wm @ v1)
    b = conv.bias.detach().double().cpu() if conv.bias is not None else None
    g = spec.geom
    if getattr(g, "upsample", 1) == 2:
        x = F.interpolate(x, scale_factor=2, mode="nearest")
    if g.transposed:
        y = F.conv_transpose2d(x, w, b, stride=g.stride, padding=g.pad)
    else:
        y = F.conv2d(x, w, b, stride=g.stride, padding=g.pad)
    if bn is not None:
        parts = []
        for s in y.chunk(segs):
            m = s.mean((0, 2, 3), keepdim=True)
            var = s.var((0, 2, 3), unbiased=False, keepdim=True)
            parts.append((s - m) / torch.sqrt(var + bn.eps) * bn.weight.detach().double().cpu().view(1, -1, 1, 1)
                         + bn.bias.detach().double().cpu().view(1, -1, 1, 1))
        y = torch.cat(parts)
    act = spec.act
    if act == "relu":
        y = F.relu(y)
    elif act == "lrelu":
        y = F.leaky_relu(y, spec.alpha)
    elif act == "tanh":
        y = torch.tanh(y)
    elif act == "sigmoid":
        y = torch.sigmoid(y)
    elif act == "selu":
        y = F.selu(y)
    return y


def main():
    name = sys.argv[1]
    net_tag = sys.argv[2] if len(sys.argv) > 2 else "D"
    segs = int(sys.argv[3]) if len(sys.argv) > 3 else 1
    from relativisticgan_amd.train import Trainer
    p = param_for(name)
    p.rgan_rng = "host"
    torch.manual_seed(5)
    t = Trainer(p, dataset_for(name).cuda())
    net = t.D if net_tag == "D" else t.G
    B = p.batch_size
    if net_tag == "D":
        h = torch.cat([dataset_for(name)[:B], dataset_for(name)[B:2 * B] if segs > 1 else dataset_for(name)[:0]])
        h = h[:B * segs].cuda()
    else:
        h = torch.randn(B * segs, p.z_size, 1, 1).cuda()
    with torch.no_grad():
        for li, layer in enumerate(net._plan):
            conv = layer.conv
            u = conv.weight_u.detach().clone() if layer.spec.spectral else None
            v = conv.weight_v.detach().clone() if layer.spec.spectral else None
            out = layer.run(h, True, segs)
            torch.cuda.synchronize()
            ref = ref_layer(layer, h, segs, u, v)
            got = out.detach().double().cpu().reshape(ref.shape)
            err = (got - ref).norm() / ref.norm()
            mx = (got - ref).abs().max()
            bad = ((got - ref).abs() > 1e-4 * ref.abs().max()).sum().item()
            print(f"{net_tag} layer {li} {tuple(ref.shape)} act={layer.spec.act} bn={layer.bn is not None} "
                  f"rel {err:.3e} maxabs {mx:.3e} (ref max {ref.abs().max():.3e}) n_bad {bad}", flush=True)
            if bad:
                d = ((got - ref).abs() > 1e-4 * ref.abs().max())
                idx = d.nonzero()[:8].tolist()
                print("   first bad (n,c,h,w):", idx)
                per_n = d.flatten(1).sum(1)
                print("   bad per sample:", per_n.tolist()[:40])
            h = out


if __name__ == "__main__":
    main()
