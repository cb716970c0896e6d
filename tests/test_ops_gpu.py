"""The rgan:: operators on the MI355X (relativisticgan_amd/ops.py): torch.library.opcheck
(schema, autograd registration, fake tensors), an exported D / G run on the GPU against the
fused eager nets, first derivatives against torch fp64 (CPU), and the double backward of a
conv chain (the WGAN-GP shape) differentiated on the HIP kernels against torch fp64.
Tolerances: rel-L2 1e-5 for single ops (fp32 MFMA sums vs fp64), 1e-4 through BatchNorm."""
import pytest
import torch
import torch.nn.functional as F

from relativisticgan_amd import ops  # noqa: F401  (registers rgan::)

pytestmark = pytest.mark.gpu
DEV = "cuda"
OPCHECK = ("test_schema", "test_autograd_registration", "test_faketensor")


def _rel(a, b):
    a, b = a.detach().double().cpu().reshape(-1), b.detach().double().cpu().reshape(-1)
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


def _nhwc(t):
    return t.contiguous(memory_format=torch.channels_last)


def test_opcheck_conv_family():
    torch.manual_seed(0)
    x = _nhwc(torch.randn(2, 32, 8, 8, device=DEV)).requires_grad_(True)
    w = (torch.randn(64, 32, 4, 4, device=DEV) * 0.05).requires_grad_(True)
    b = torch.randn(64, device=DEV).requires_grad_(True)
    torch.library.opcheck(torch.ops.rgan.conv2d.default, (x, w, b, 4, 2, 1, False, 1, "lrelu", 0.2, False),
                          test_utils=OPCHECK)
    dy = _nhwc(torch.randn(2, 64, 4, 4, device=DEV))
    torch.library.opcheck(torch.ops.rgan.conv2d_dgrad.default, (dy, w.detach(), [2, 32, 8, 8], 4, 2, 1, False, 1),
                          test_utils=OPCHECK)
    torch.library.opcheck(torch.ops.rgan.conv2d_wgrad.default, (x.detach(), dy, [64, 32, 4, 4], 4, 2, 1, False, 1),
                          test_utils=OPCHECK)
    torch.library.opcheck(torch.ops.rgan.channel_sum.default, (dy,), test_utils=("test_schema", "test_faketensor"))


def test_opcheck_bn_heads_penalty_spectral_adam():
    torch.manual_seed(1)
    y = _nhwc(torch.randn(4, 32, 8, 8, device=DEV)).requires_grad_(True)
    rm, rv, nbt = torch.zeros(32, device=DEV), torch.ones(32, device=DEV), torch.zeros((), dtype=torch.long, device=DEV)
    torch.library.opcheck(torch.ops.rgan.batch_norm_stats_.default, (y.detach(), rm, rv, nbt, 1e-5, 0.1),
                          test_utils=("test_schema", "test_faketensor"))
    stats = torch.ops.rgan.batch_norm_stats_(y.detach(), rm, rv, nbt, 1e-5, 0.1)
    g, bt = (torch.rand(32, device=DEV) + 0.5).requires_grad_(True), torch.randn(32, device=DEV).requires_grad_(True)
    torch.library.opcheck(torch.ops.rgan.batch_norm_apply.default, (y, stats, g, bt, "relu", 0.0), test_utils=OPCHECK)
    r, f = torch.randn(16, device=DEV).requires_grad_(True), torch.randn(16, device=DEV).requires_grad_(True)
    for kind in (1, 2, 3, 4, 5, 6, 7, 8):
        torch.library.opcheck(torch.ops.rgan.loss_head.default, (kind, 2, r if kind > 4 else None, f),
                              test_utils=OPCHECK)
    gr = torch.randn(4, 3, 8, 8, device=DEV).requires_grad_(True)
    torch.library.opcheck(torch.ops.rgan.gp_penalty.default, (gr, 10.0, 4), test_utils=OPCHECK)
    w = (torch.randn(64, 32, 4, 4, device=DEV) * 0.05)
    u = F.normalize(torch.randn(64, device=DEV), dim=0)
    v = F.normalize(torch.randn(512, device=DEV), dim=0)
    uc, vc, inv = torch.ops.rgan.spectral_power_(w, u, v, False, 1e-12, True)
    torch.library.opcheck(torch.ops.rgan.spectral_scale.default, (w.requires_grad_(True), uc, vc, inv, False),
                          test_utils=OPCHECK)
    ps = [torch.randn(33, device=DEV), torch.randn(4, 8, device=DEV)]
    torch.library.opcheck(torch.ops.rgan.adam_.default,
                          (ps, [torch.randn_like(p) for p in ps], [torch.zeros_like(p) for p in ps],
                           [torch.zeros_like(p) for p in ps],
                           torch.tensor([1e-4, 0.5, 0.999, 1e-8, 0, 0, 0, 0], dtype=torch.float64, device=DEV),
                           torch.zeros(1, device=DEV)), test_utils=("test_schema", "test_faketensor"))


@pytest.mark.parametrize("kw", [dict(loss_D=7), dict(loss_D=8, spectral=True), dict(loss_D=3, arch=1)],
                         ids=["ralsgan", "rahinge_spectral", "wgangp_arch1"])
def test_exported_nets_match_fused_eager(kw):
    """An exported G / D (graphs of rgan:: ops, unfused: conv, then BatchNorm) on the GPU == the
    fused eager nets (GEMM-epilogue statistics): outputs and BN running statistics / spectral
    u, v after the call, rel-L2 1e-5."""
    import copy
    from relativisticgan_amd.config import make_param
    from relativisticgan_amd.nets import DCGAN_D, DCGAN_G
    p = make_param(batch_size=8, z_size=16, G_h_size=8, D_h_size=8, seed=1, image_size=32, **kw)
    torch.manual_seed(1)
    for net, x in ((DCGAN_G(p).to(DEV), torch.randn(8, 16, 1, 1, device=DEV)),
                   (DCGAN_D(p).to(DEV), torch.randn(8, 3, 32, 32, device=DEV))):
        twin = copy.deepcopy(net)
        ep = torch.export.export(twin, (x,))
        prog = ep.module()
        want = net(x)
        got = prog(x)
        assert _rel(got, want) <= 1e-5, (type(net).__name__, _rel(got, want))
        sd_e = dict(ep.state_dict)
        sd_e.update({k: v for k, v in prog.state_dict().items()})
        for k, v in net.state_dict().items():
            if ("running" in k or k.endswith("weight_u") or k.endswith("weight_v")) and k in sd_e:
                assert _rel(sd_e[k], v) <= 1e-5, k


def test_conv_autograd_first_and_second_order_vs_fp64():
    """L = sum((d/dx sum(lrelu(conv(x, W)) * c))^2): its gradient w.r.t. W runs the double
    backward of the conv chain on rgan:: ops (conv2d -> dgrad -> wgrad / conv2d) -- compared
    with torch fp64 on the CPU."""
    torch.manual_seed(3)
    xc = torch.randn(2, 32, 8, 8, dtype=torch.float64)
    wc = torch.randn(64, 32, 4, 4, dtype=torch.float64) * 0.05
    cc = torch.randn(2, 64, 4, 4, dtype=torch.float64)

    def ref():
        x, w = xc.clone().requires_grad_(True), wc.clone().requires_grad_(True)
        y = F.leaky_relu(F.conv2d(x, w, stride=2, padding=1), 0.2)
        g, = torch.autograd.grad((y * cc).sum(), x, create_graph=True)
        L = (g * g).sum()
        gw, gx = torch.autograd.grad(L, (w, x))
        return g.detach(), gw, gx

    x = _nhwc(xc.float().to(DEV)).requires_grad_(True)
    w = wc.float().to(DEV).requires_grad_(True)
    c = _nhwc(cc.float().to(DEV))
    y = torch.ops.rgan.conv2d(x, w, None, 4, 2, 1, False, 1, "lrelu", 0.2, False)
    g, = torch.autograd.grad((y * c).sum(), x, create_graph=True)
    L = (g * g).sum()
    gw, gx = torch.autograd.grad(L, (w, x))
    rg, rgw, rgx = ref()
    assert _rel(g, rg) <= 1e-5 and _rel(gw, rgw) <= 1e-5 and _rel(gx, rgx) <= 1e-5, (_rel(g, rg), _rel(gw, rgw),
                                                                                     _rel(gx, rgx))


def test_bn_head_penalty_autograd_vs_fp64():
    """conv -> BatchNorm (train) -> LReLU -> head 7 (RaLSGAN D side) gradients on rgan:: ops
    vs torch fp64."""
    torch.manual_seed(4)
    xc = torch.randn(8, 16, 8, 8, dtype=torch.float64)
    wc = torch.randn(32, 16, 4, 4, dtype=torch.float64) * 0.05
    gc, bc = torch.rand(32, dtype=torch.float64) + 0.5, torch.randn(32, dtype=torch.float64)
    w2 = torch.randn(1, 32, 4, 4, dtype=torch.float64) * 0.05

    def ref():
        w, g, b = wc.clone().requires_grad_(True), gc.clone().requires_grad_(True), bc.clone().requires_grad_(True)
        y = F.conv2d(xc, w, stride=2, padding=1)
        a = F.leaky_relu(F.batch_norm(y, None, None, g, b, training=True, eps=1e-5), 0.2)
        o = F.conv2d(a, w2).view(-1)
        r, f = o[:4], o[4:]
        L = 0.5 * (((r - f.mean() - 1) ** 2).mean() + ((f - r.mean() + 1) ** 2).mean())
        return L.detach(), torch.autograd.grad(L, (w, g, b))

    w = wc.float().to(DEV).requires_grad_(True)
    g, b = gc.float().to(DEV).requires_grad_(True), bc.float().to(DEV).requires_grad_(True)
    x = _nhwc(xc.float().to(DEV))
    rm, rv, nbt = torch.zeros(32, device=DEV), torch.ones(32, device=DEV), torch.zeros((), dtype=torch.long, device=DEV)
    y = torch.ops.rgan.conv2d(x, w, None, 4, 2, 1, False, 1, "none", 0.0, False)
    st = torch.ops.rgan.batch_norm_stats_(y.detach(), rm, rv, nbt, 1e-5, 0.1)
    a = torch.ops.rgan.batch_norm_apply(y, st, g, b, "lrelu", 0.2)
    o = torch.ops.rgan.conv2d(a, w2.float().to(DEV), None, 4, 1, 0, False, 1, "none", 0.0, False).reshape(-1)
    L = torch.ops.rgan.loss_head(7, 0, o[:4].contiguous(), o[4:].contiguous())
    grads = torch.autograd.grad(L, (w, g, b))
    rL, rgrads = ref()
    assert _rel(L, rL) <= 1e-5
    for a_, b_ in zip(grads, rgrads):
        assert _rel(a_, b_) <= 1e-4, _rel(a_, b_)
