"""WGAN-GP double backward (GLI:646-658): the native engine (relativisticgan_amd/gp.py,
explicit sweeps over the HIP kernels) against the autograd composite of the same layers
(ConvLayerFn's create-graph backward, itself parity-tested against the oracle), and
gradient accumulation in the weight-gradient kernels.

The engine ADDS into existing .grad tensors (the errD backward has filled them), so every
case starts from random gradients.  Tolerance: rel L2 <= 2e-5 (fp32, two summation orders
of the same algebra; observed ~1e-6).
"""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"

CASES = {
    "arch0_bn_lrelu": dict(loss_D=3, image_size=32, D_h_size=8),
    "arch0_64": dict(loss_D=3, image_size=64, D_h_size=16),
    "arch0_tanh": dict(loss_D=3, image_size=32, D_h_size=8, Tanh_GD="True"),
    "arch0_selu": dict(loss_D=3, image_size=32, D_h_size=8, SELU="True"),
    "arch0_spectral": dict(loss_D=3, image_size=32, D_h_size=8, spectral="True"),
    "arch0_nobn": dict(loss_D=3, image_size=32, D_h_size=8, no_batch_norm_D="True"),
    "arch0_sigmoid_end": dict(loss_D=1, image_size=32, D_h_size=8, grad_penalty="True"),
    "arch1": dict(loss_D=3, image_size=32, arch=1),
}


def _rel(a, b):
    a, b = a.double().cpu().reshape(-1), b.double().cpu().reshape(-1)
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


def _run(D, x, xf, u, fn, grads0):
    for q, g in zip(D.parameters(), grads0):
        q.grad = g.clone()
    gp = fn(D, x, xf, u, 10.0)
    gp.backward()
    torch.cuda.synchronize()
    return gp.detach().clone(), [q.grad.detach().clone() for q in D.parameters()], \
        {k: v.detach().clone() for k, v in D.state_dict().items()}


@pytest.mark.parametrize("case", sorted(CASES))
def test_native_gp_matches_composite(case):
    from relativisticgan_amd import losses
    from relativisticgan_amd.config import make_param
    from relativisticgan_amd.nets import DCGAN_D, weights_init
    torch.manual_seed(7)
    p = make_param(batch_size=6, seed=1, **CASES[case])
    D = DCGAN_D(p)
    D.apply(weights_init)
    D = D.to(DEV)
    S = p.image_size
    x = torch.rand(6, 3, S, S, device=DEV) * 2 - 1
    xf = torch.rand(6, 3, S, S, device=DEV) * 2 - 1
    u = torch.rand(6, 1, 1, 1, device=DEV)
    grads0 = [torch.randn_like(q) * 1e-2 for q in D.parameters()]
    state0 = {k: v.clone() for k, v in D.state_dict().items()}
    gp_n, g_n, st_n = _run(D, x, xf, u, losses.gradient_penalty, grads0)
    D.load_state_dict(state0)
    gp_c, g_c, st_c = _run(D, x, xf, u, losses.gradient_penalty_composite, grads0)
    assert abs(gp_n.item() - gp_c.item()) <= 2e-5 * abs(gp_c.item())
    names = [n for n, _ in D.named_parameters()]
    for n, a, b, g0 in zip(names, g_n, g_c, grads0):
        # compare the GP's own contribution (the accumulated base cancels exactly)
        # (a conv bias feeding BatchNorm has an exact GP gradient of 0: both are roundoff)
        assert _rel(a - g0, b - g0) < 2e-5 or (a - b).abs().max() < 1e-7, (case, n, _rel(a - g0, b - g0))
    for k in st_c:  # BN running stats and spectral u/v move exactly as in one D(x_hat) call
        if st_c[k].is_floating_point():
            assert _rel(st_n[k], st_c[k]) < 1e-6, (case, k)
        else:
            assert torch.equal(st_n[k], st_c[k]), (case, k)


# (B, cin, cout, H, k, s, p, transposed): unsplit tap-staged, split-K, dense end, arch-1 3x3, convT
ACC_CASES = [
    (64, 128, 256, 32, 4, 2, 1, False),
    (4, 256, 512, 8, 4, 2, 1, False),
    (6, 64, 1, 4, 4, 1, 0, False),
    (4, 32, 48, 8, 3, 1, 1, False),
    (4, 64, 32, 8, 4, 2, 1, True),
]


@pytest.mark.parametrize("case", ACC_CASES)
def test_wgrad_accumulate(case):
    """rgan_conv_wgrad(accumulate=1): dw += wgrad and dbias += sum dy, in every epilogue
    (scalar stores, tap transpose, split-K reduce, dense one-output kernel)."""
    from relativisticgan_amd import kernels as K
    B, cin, cout, H, k, s, p, tr = case
    g = K.ConvGeom(k, s, p, tr)
    torch.manual_seed(5)
    x = torch.randn(B, cin, H, H, device=DEV).contiguous(memory_format=torch.channels_last)
    Ho, Wo = g.out_hw(H, H)
    dy = torch.randn(B, cout, Ho, Wo, device=DEV).contiguous(memory_format=torch.channels_last)
    wshape = (cin, cout, k, k) if tr else (cout, cin, k, k)
    dw, db = K.conv_wgrad(x, dy, g, wshape, with_bias=True)
    base_w = torch.randn(wshape, device=DEV)
    base_b = torch.randn(cout, device=DEV)
    acc_w, acc_b = base_w.clone(), base_b.clone()
    K.conv_wgrad(x, dy, g, wshape, with_bias=True, out=acc_w, out_bias=acc_b)
    assert _rel(acc_w - base_w, dw) < 1e-6
    assert _rel(acc_b - base_b, db) < 1e-6
