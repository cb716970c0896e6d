"""The rgan:: operator namespace (relativisticgan_amd/ops.py, SURVEY §8(b) "Op registration")
on CPU: every op is registered with a fake implementation, and torch.export traces the
reference's nets (arch 0 / 1, spectral D, NN_conv, SELU) into graphs whose compute nodes are
rgan:: operators only (plus views) -- fake CUDA tensors, no GPU needed."""
import pytest
import torch
from torch._subclasses.fake_tensor import FakeTensorMode

from relativisticgan_amd import ops
from relativisticgan_amd.config import make_param
from relativisticgan_amd.nets import DCGAN_D, DCGAN_G

ALLOWED = {"aten.view.default", "aten.reshape.default", "aten.detach.default", "<built-in function getitem>"}


def test_ops_registered():
    for name in ops.OPS:
        assert hasattr(torch.ops.rgan, name), name
        assert torch.ops.rgan.__getattr__(name).default._schema.name == f"rgan::{name}"


@pytest.mark.parametrize("kw", [dict(loss_D=7), dict(loss_D=8, spectral=True), dict(loss_D=6, spectral_G=True),
                                dict(loss_D=3, arch=1), dict(loss_D=7, NN_conv=True), dict(loss_D=1, SELU=True),
                                dict(loss_D=7, Tanh_GD=True), dict(loss_D=7, image_size=64)],
                         ids=lambda kw: "-".join(f"{k}={v}" for k, v in kw.items()))
def test_export_nets_through_rgan_ops(kw):
    kw = dict(kw)
    S = kw.pop("image_size", 32)
    p = make_param(batch_size=8, z_size=16, G_h_size=8, D_h_size=8, seed=1, image_size=S, **kw)
    torch.manual_seed(1)
    for net, shape, out_shape in ((DCGAN_G(p), (8, 16, 1, 1), (8, 3, 32 if p.arch == 1 else S, 32 if p.arch == 1 else S)),
                                  (DCGAN_D(p), (8, 3, 32 if p.arch == 1 else S, 32 if p.arch == 1 else S), (8,))):
        with FakeTensorMode(allow_non_fake_inputs=True):
            net = net.to("cuda")
            ep = torch.export.export(net, (torch.empty(shape, device="cuda"),))
        targets = {str(n.target) for n in ep.graph.nodes if n.op == "call_function"}
        compute = {t for t in targets if t not in ALLOWED}
        assert compute and all(t.startswith("rgan.") for t in compute), compute
        out = [n for n in ep.graph.nodes if n.op == "output"][0].args[0]
        assert tuple(out[-1].meta["val"].shape) == out_shape


def test_fake_conv_shapes_and_nhwc_strides():
    with FakeTensorMode():
        x = torch.empty(4, 16, 8, 8, device="cuda").contiguous(memory_format=torch.channels_last)
        w = torch.empty(16, 32, 4, 4, device="cuda")          # ConvTranspose2d [cin][cout][k][k]
        y = torch.ops.rgan.conv2d(x, w, None, 4, 2, 1, True, 1, "relu", 0.0, False)
        assert tuple(y.shape) == (4, 32, 16, 16) and y.stride() == (16 * 16 * 32, 1, 16 * 32, 32)
        dx = torch.ops.rgan.conv2d_dgrad(y, w, [4, 16, 8, 8], 4, 2, 1, True, 1)
        assert tuple(dx.shape) == (4, 16, 8, 8) and dx.stride()[1] == 1
        dw = torch.ops.rgan.conv2d_wgrad(x, y, [16, 32, 4, 4], 4, 2, 1, True, 1)
        assert tuple(dw.shape) == (16, 32, 4, 4)
        img = torch.ops.rgan.conv2d(y, torch.empty(32, 3, 4, 4, device="cuda"), None, 4, 2, 1, True, 1, "tanh", 0.0,
                                    True)
        assert tuple(img.shape) == (4, 3, 32, 32) and img.is_contiguous()
