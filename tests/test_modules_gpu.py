"""Module-level numerics: DCGAN_G / DCGAN_D on the HIP kernels vs the oracle's torch
modules evaluated in float64 with the same state (forward, input and parameter grads).

Tolerance: fp32 kernels vs an fp64 reference of the same modules, rel-L2 <= 2e-5 on
outputs and gradients, or -- where fp32 itself is ill-conditioned -- no more than 4x the
error of torch's own fp32 CPU modules vs fp64 (BN-preceded conv biases excluded: their
exact gradient is 0).
"""
import copy

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _rel(a, b):
    a = a.detach().double().cpu().reshape(-1)
    b = b.detach().double().cpu().reshape(-1)
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


CASES = [
    dict(arch=0, image_size=32, batch_size=8, z_size=16, G_h_size=8, D_h_size=8, loss_D=7),
    dict(arch=0, image_size=64, batch_size=4, z_size=32, G_h_size=16, D_h_size=16, loss_D=1),
    dict(arch=0, image_size=32, batch_size=8, z_size=16, G_h_size=8, D_h_size=8, loss_D=8, spectral=True),
    dict(arch=0, image_size=32, batch_size=8, z_size=16, G_h_size=8, D_h_size=8, loss_D=7, SELU=True),
    dict(arch=1, image_size=32, batch_size=8, z_size=16, loss_D=8),
    dict(arch=1, image_size=32, batch_size=8, z_size=16, loss_D=1, no_batch_norm_D=True),
]


def _biases_before_bn(net):
    names = set()
    prev = None
    for n, m in net.named_modules():
        if "BatchNorm" in type(m).__name__ and prev is not None:
            names.add(prev + ".bias")
        if hasattr(m, "bias") and isinstance(getattr(m, "bias", None), torch.nn.Parameter) and \
                "BatchNorm" not in type(m).__name__:
            prev = n
    return names


@pytest.mark.parametrize("case", CASES, ids=lambda c: "-".join(f"{k}{v}" for k, v in c.items()))
def test_nets_vs_fp64_torch(case):
    from oracle.reference_cpu import build_D, build_G, make_param as oparam, weights_init as owi
    from relativisticgan_amd.config import make_param
    from relativisticgan_amd.nets import DCGAN_D, DCGAN_G, weights_init
    torch.manual_seed(3)
    po = oparam(cuda=False, **case)
    Go, Do = build_G(po), build_D(po)
    Go.apply(owi)
    Do.apply(owi)
    p = make_param(**case)
    G, D = DCGAN_G(p), DCGAN_D(p)
    G.load_state_dict(Go.state_dict())
    D.load_state_dict(Do.state_dict())
    G.to(DEV)
    D.to(DEV)
    Go64, Do64 = copy.deepcopy(Go).double(), copy.deepcopy(Do).double()
    Go32, Do32 = copy.deepcopy(Go), copy.deepcopy(Do)
    B = case["batch_size"]
    z = torch.randn(B, case["z_size"], 1, 1)
    # G forward (activation signs traced on both sides: ReLU'/LeakyReLU'/SELU' jump at 0)
    from relativisticgan_amd import autograd
    masks64 = []
    hooks = [m.register_forward_hook(lambda mod, i, o: masks64.append((o.detach() > 0).clone()))
             for net in (Go64, Do64) for m in net.modules()
             if isinstance(m, (torch.nn.ReLU, torch.nn.LeakyReLU, torch.nn.SELU))]
    autograd.ACT_TRACE = []
    out64 = Go64(z.double())
    out32 = Go32(z)
    fake = G(z.to(DEV))
    flips = [0]

    def env(label, ours, ref32, ref64, tol=2e-5):
        e, e32 = _rel(ours, ref64), _rel(ref32, ref64)
        bound = max(tol, 4 * e32, 5e-2 if flips[0] else 0.0)
        assert e < bound, f"{label}: {e:.2e} vs fp64 (torch fp32: {e32:.2e}, flips {flips[0]})"

    env("G out", fake, out32, out64)
    # D on the same image with input grad (the G-step path) and param grads (D-step path)
    img = out64.detach()
    x = img.float().to(DEV).requires_grad_(True)
    x32 = img.float().clone().requires_grad_(True)
    x64 = img.clone().requires_grad_(True)
    y, y32, y64 = D(x), Do32(x32), Do64(x64)
    ours_masks, autograd.ACT_TRACE = autograd.ACT_TRACE, None
    for h in hooks:
        h.remove()
    assert len(ours_masks) == len(masks64)
    flips[0] = sum(int((a != b).sum()) for a, b in zip(ours_masks, masks64))
    print(f"activation-sign flips vs fp64: {flips[0]}")
    env("D out", y, y32, y64)
    gy = torch.randn(B)
    y.backward(gy.to(DEV))
    y32.backward(gy)
    y64.backward(gy.double())
    env("D input grad", x.grad, x32.grad, x64.grad)
    skip = _biases_before_bn(Do64)
    for (n, q), (_, q32), (n64, q64) in zip(D.named_parameters(), Do32.named_parameters(), Do64.named_parameters()):
        assert n == n64
        if n in skip:  # exact gradient is 0: both fp32 results are roundoff
            assert q.grad.abs().max().item() <= 10 * q32.grad.abs().max().item() + 1e-7, n
            continue
        env(f"D grad {n}", q.grad, q32.grad, q64.grad)
    # G backward from one shared upstream gradient (the fp64 one, rounded to fp32)
    gfake = x64.grad.detach()
    fake.backward(gfake.float().to(DEV))
    out32.backward(gfake.float())
    out64.backward(gfake)
    skipg = _biases_before_bn(Go64)
    for (n, q), (_, q32), (_, q64) in zip(G.named_parameters(), Go32.named_parameters(), Go64.named_parameters()):
        if n in skipg:
            continue
        env(f"G grad {n}", q.grad, q32.grad, q64.grad)
    # BN running statistics after the train-mode forwards
    for (n, b), (_, b32), (_, b64) in zip(D.named_buffers(), Do32.named_buffers(), Do64.named_buffers()):
        if "running" in n:
            env(n, b, b32, b64, 1e-5)


def test_weight_hooks_fire_in_trainer_backward():
    """A fused layer writes its weight gradient into .grad itself inside the trainer's
    backward (autograd.owning_grads) -- unless the weight carries a tensor hook or a
    post-accumulate-grad hook, which only autograd's AccumulateGrad would fire: then the
    gradient goes through autograd and the hooks run (and the result is the same)."""
    from relativisticgan_amd.config import make_param
    from relativisticgan_amd.train import Trainer
    from oracle.reference_cpu import synthetic_images
    kw = dict(loss_D=7, image_size=32, batch_size=8, z_size=16, G_h_size=8, D_h_size=8, seed=1, print_every=1000)
    fired = {"post": 0, "tensor": 0}
    nets = []
    for with_hooks in (False, True):  # each trainer re-seeds at construction: the same draws
        t = Trainer(make_param(**kw), synthetic_images(64, 32).cuda())
        if with_hooks:
            t.D.main[0].weight.register_post_accumulate_grad_hook(
                lambda p: fired.__setitem__("post", fired["post"] + 1))
            t.G.main[0].weight.register_hook(lambda g: fired.__setitem__("tensor", fired["tensor"] + 1))
        t.iteration(0)
        torch.cuda.synchronize()
        nets.append(t)
    plain, hooked = nets
    assert fired["post"] >= 1 and fired["tensor"] >= 1
    # the two accumulation paths round differently (one vs two roundings of grad + dw), and
    # Adam's first step is a sign step: parameters agree to 2 lr, buffers closely
    for a, b in ((plain.D, hooked.D), (plain.G, hooked.G)):
        for (n, x), (_, y) in zip(a.state_dict().items(), b.state_dict().items()):
            assert torch.allclose(x.float(), y.float(), rtol=1e-5, atol=2.02e-4), n
