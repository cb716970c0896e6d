"""ORACLE — CPU restatement of the RelativisticGAN training step.  TEST INFRASTRUCTURE.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg
may import this module, and only as the checker / CPU baseline.  The product
(``relativisticgan_amd``) never imports it.

What it restates (``GLI`` = ``code/GAN_losses_iter.py`` of the reference):

* configuration surface: the 40 CLI flags and their defaults (GLI:17-62);
* seeding and RNG consumption order (GLI:147-157);
* random real-batch sampler: ``numpy.random.choice(N, B, replace=False)`` (GLI:173-179);
* DCGAN G/D, arch 0 (GLI:321-460) and the "standard CNN" arch 1 (GLI:183-319), built
  from torch CPU modules with the reference's module names (state_dict keys);
* ``weights_init`` (GLI:466-477);
* persistent buffers and ``z_test`` (GLI:486-499), Adam x2 + ExponentialLR x2 (GLI:526-534);
* the training iteration (GLI:560-714): D step with the eight ``--loss_D`` heads,
  the WGAN-GP gradient penalty (GLI:646-658), the G step, LR decay.

Everything runs on the torch CPU backend with fp32, like the reference with
``--cuda False``.  Pinned: ``tests/test_oracle_golden.py`` replays every fixture
in ``tests/golden/`` (captured from the unmodified reference) and requires
bitwise-identical tensors at the fixture's thread count.
"""
from __future__ import annotations

import argparse
import math
import random
from dataclasses import dataclass, field

import numpy
import torch
import torch.nn as nn
from torch.nn.utils import spectral_norm

HEAD_NAMES = {1: "GAN", 2: "LSGAN", 3: "WGANGP", 4: "HingeGAN", 5: "RSGAN",
              6: "RaSGAN", 7: "RaLSGAN", 8: "RaHingeGAN"}


def _str2bool(s):
    return s.lower() in ("true", "yes", "on", "t", "1")


def make_parser():
    """The reference CLI (GLI:17-62), same names, types and defaults."""
    p = argparse.ArgumentParser()
    p.register("type", "bool", _str2bool)
    a = p.add_argument
    a("--image_size", type=int, default=64)
    a("--batch_size", type=int, default=32)
    a("--n_colors", type=int, default=3)
    a("--z_size", type=int, default=128)
    a("--G_h_size", type=int, default=128)
    a("--D_h_size", type=int, default=128)
    a("--lr_D", type=float, default=.0001)
    a("--lr_G", type=float, default=.0001)
    a("--n_iter", type=int, default=100000)
    a("--beta1", type=float, default=0.5)
    a("--beta2", type=float, default=0.999)
    a("--decay", type=float, default=0)
    a("--SELU", type="bool", default=False)
    a("--NN_conv", type="bool", default=False)
    a("--seed", type=int)
    a("--input_folder", default="")
    a("--output_folder", default="")
    a("--inception_folder", default="")
    a("--load", default=None)
    a("--cuda", type="bool", default=True)
    a("--n_gpu", type=int, default=1)
    a("--loss_D", type=int, default=1)
    a("--Diters", type=int, default=1)
    a("--Giters", type=int, default=1)
    a("--penalty", type=float, default=10)
    a("--spectral", type="bool", default=False)
    a("--spectral_G", type="bool", default=False)
    a("--weight_decay", type=float, default=0)
    a("--gen_extra_images", type=int, default=50000)
    a("--gen_every", type=int, default=100000)
    a("--extra_folder", default="")
    a("--show_graph", type="bool", default=False)
    a("--no_batch_norm_G", type="bool", default=False)
    a("--no_batch_norm_D", type="bool", default=False)
    a("--Tanh_GD", type="bool", default=False)
    a("--grad_penalty", type="bool", default=False)
    a("--arch", type=int, default=0)
    a("--print_every", type=int, default=1000)
    a("--save", type="bool", default=True)
    a("--CIFAR10", type="bool", default=False)
    a("--CIFAR10_input_folder", default="")
    return p


def make_param(**overrides):
    """Namespace with the reference defaults, then ``overrides`` (strings ok for bools)."""
    ns = make_parser().parse_args([])
    for k, v in overrides.items():
        if isinstance(v, str) and isinstance(getattr(ns, k, None), bool):
            v = _str2bool(v)
        elif isinstance(v, str) and isinstance(getattr(ns, k, None), (int, float)) \
                and not isinstance(getattr(ns, k, None), bool):
            v = type(getattr(ns, k))(v)
        setattr(ns, k, v)
    return ns


def synthetic_images(n, size, n_colors=3, seed=1234):
    """The benchmark / fixture image set: uint8 -> (u8/255-0.5)/0.5."""
    g = torch.Generator().manual_seed(seed)
    u8 = torch.randint(0, 256, (n, n_colors, size, size), generator=g, dtype=torch.uint8)
    return (u8.float() / 255.0 - 0.5) / 0.5


# --------------------------------------------------------------------------- models
def _pac(p):
    """PacGAN packing degree: 1 for GLI, 2 for code/GAN_losses_iter_PAC.py (D sees
    n_colors*2 channels: PAC:242,260,408,410)."""
    return getattr(p, "pac", 1)


def pack(t, B, pac):
    """[pac*B, C, ...] -> [B, pac*C, ...]: torch.cat([t[0:B], t[B:2B]], 1) (PAC:582,609,682)."""
    if pac == 1:
        return t
    return torch.cat([t[k * B:(k + 1) * B] for k in range(pac)], 1)


def _dp_shards(p):
    """Replicas of the reference's ``data_parallel`` forward (GLI:393, GLI:455: arch 0 with
    ``--n_gpu > 1`` on CUDA); the CPU oracle emulates it when ``p.dp_shards > 1``."""
    return int(getattr(p, "dp_shards", 1) or 1)


def data_parallel_emulated(main, x, n):
    """torch.nn.parallel.data_parallel(main, x, range(n)) restated on one CPU device:
    scatter = ``x.chunk(n)``, one replica per chunk, gather = ``cat`` on dim 0, gradients of
    the shared parameters summed over replicas.  Buffers: replica 0 shares the module's
    buffers (broadcast_coalesced hands the source device its own tensors), so only its
    BatchNorm running-stat and spectral-norm u/v updates persist; every other replica starts
    from the pre-forward buffers and its updates are discarded."""
    if n <= 1:
        return main(x)
    chunks = x.chunk(n)
    bufs = list(main.buffers())
    with torch.no_grad():
        pre = [b.clone() for b in bufs]
    outs = [main(chunks[0])]
    with torch.no_grad():
        post = [b.clone() for b in bufs]
    for c in chunks[1:]:
        for b, v in zip(bufs, pre):
            b.data.copy_(v)  # .data: the autograd graph keeps the buffers' version counters
        outs.append(main(c))
    for b, v in zip(bufs, post):
        b.data.copy_(v)
    return torch.cat(outs)


def _maybe_sn(mod, on):
    return spectral_norm(mod) if on else mod


class _G0(nn.Module):
    """DCGAN generator, arch 0 (GLI:323-397)."""

    def __init__(self, p):
        super().__init__()
        seq = nn.Sequential()
        mult = p.image_size // 8
        sn = p.spectral_G
        head = "Start-SpectralConvTranspose2d" if sn else "Start-ConvTranspose2d"
        seq.add_module(head, _maybe_sn(nn.ConvTranspose2d(p.z_size, p.G_h_size * mult, 4, 1, 0,
                                                          bias=False), sn))
        self._act_block(seq, p, "Start", "", p.G_h_size * mult)
        i = 1
        while mult > 1:
            cin, cout = p.G_h_size * mult, p.G_h_size * (mult // 2)
            if p.NN_conv:
                seq.add_module("Middle-UpSample [%d]" % i, nn.Upsample(scale_factor=2))
                nm = ("Middle-SpectralConv2d [%d]" if sn else "Middle-Conv2d [%d]") % i
                seq.add_module(nm, _maybe_sn(nn.Conv2d(cin, cout, 3, 1, 1), sn))
            else:
                nm = ("Middle-SpectralConvTranspose2d [%d]" if sn else "Middle-ConvTranspose2d [%d]") % i
                seq.add_module(nm, _maybe_sn(nn.ConvTranspose2d(cin, cout, 4, 2, 1, bias=False), sn))
            self._act_block(seq, p, "Middle", " [%d]" % i, cout)
            mult //= 2
            i += 1
        if p.NN_conv:
            seq.add_module("End-UpSample", nn.Upsample(scale_factor=2))
            nm = "End-SpectralConv2d" if sn else "End-Conv2d"
            seq.add_module(nm, _maybe_sn(nn.Conv2d(p.G_h_size, p.n_colors, 3, 1, 1), sn))
        else:
            nm = "End-SpectralConvTranspose2d" if sn else "End-ConvTranspose2d"
            seq.add_module(nm, _maybe_sn(nn.ConvTranspose2d(p.G_h_size, p.n_colors, 4, 2, 1,
                                                            bias=False), sn))
        seq.add_module("End-Tanh", nn.Tanh())
        self.main = seq
        self.dp = _dp_shards(p)

    @staticmethod
    def _act_block(seq, p, part, suffix, ch):
        if p.SELU:
            seq.add_module(part + "-SELU" + suffix, nn.SELU(inplace=True))
            return
        if not p.no_batch_norm_G and not p.spectral_G:
            seq.add_module(part + "-BatchNorm2d" + suffix, nn.BatchNorm2d(ch))
        if p.Tanh_GD:
            seq.add_module(part + "-Tanh" + suffix, nn.Tanh())
        else:
            seq.add_module(part + "-ReLU" + suffix, nn.ReLU())

    def forward(self, z):
        return data_parallel_emulated(self.main, z, self.dp)


class _D0(nn.Module):
    """DCGAN discriminator, arch 0 (GLI:400-460)."""

    def __init__(self, p):
        super().__init__()
        seq = nn.Sequential()
        sn = p.spectral
        seq.add_module("Start-SpectralConv2d" if sn else "Start-Conv2d",
                       _maybe_sn(nn.Conv2d(p.n_colors * _pac(p), p.D_h_size, 4, 2, 1, bias=False), sn))
        if p.SELU:
            seq.add_module("Start-SELU", nn.SELU(inplace=True))
        elif p.Tanh_GD:
            seq.add_module("Start-Tanh", nn.Tanh())
        else:
            seq.add_module("Start-LeakyReLU", nn.LeakyReLU(0.2, inplace=True))
        size, mult, i = p.image_size // 2, 1, 0
        while size > 4:
            cin, cout = p.D_h_size * mult, p.D_h_size * 2 * mult
            nm = ("Middle-SpectralConv2d [%d]" if sn else "Middle-Conv2d [%d]") % i
            seq.add_module(nm, _maybe_sn(nn.Conv2d(cin, cout, 4, 2, 1, bias=False), sn))
            if p.SELU:
                seq.add_module("Middle-SELU [%d]" % i, nn.SELU(inplace=True))
            else:
                if not p.no_batch_norm_D and not sn:
                    seq.add_module("Middle-BatchNorm2d [%d]" % i, nn.BatchNorm2d(cout))
                if p.Tanh_GD:
                    # the reference names this activation 'Start-Tanh [i]' (GLI:435)
                    seq.add_module("Start-Tanh [%d]" % i, nn.Tanh())
                else:
                    seq.add_module("Middle-LeakyReLU [%d]" % i, nn.LeakyReLU(0.2, inplace=True))
            size //= 2
            mult *= 2
            i += 1
        seq.add_module("End-SpectralConv2d" if sn else "End-Conv2d",
                       _maybe_sn(nn.Conv2d(p.D_h_size * mult, 1, 4, 1, 0, bias=False), sn))
        if p.loss_D == 1:
            seq.add_module("End-Sigmoid", nn.Sigmoid())
        self.main = seq
        self.dp = _dp_shards(p)

    def forward(self, x):
        return data_parallel_emulated(self.main, x, self.dp).view(-1)


def _act1(p, slope):
    return nn.Tanh() if p.Tanh_GD else nn.LeakyReLU(slope, inplace=True)


class _G1(nn.Module):
    """'Standard CNN' generator, arch 1 (GLI:186-233); 32x32 output only."""

    def __init__(self, p):
        super().__init__()
        self.z_size = p.z_size
        self.dense = nn.Linear(p.z_size, 512 * 4 * 4)
        layers = []
        chans = [(512, 256), (256, 128), (128, 64)]
        for cin, cout in chans:
            layers.append(_maybe_sn(nn.ConvTranspose2d(cin, cout, 4, 2, 1, bias=True), p.spectral_G))
            if p.spectral_G:
                layers.append(nn.ReLU(True))
                continue
            if not p.no_batch_norm_G:
                layers.append(nn.BatchNorm2d(cout))
            layers.append(nn.Tanh() if p.Tanh_GD else nn.ReLU(True))
        layers.append(_maybe_sn(nn.Conv2d(64, p.n_colors, 3, 1, 1, bias=True), p.spectral_G))
        layers.append(nn.Tanh())
        self.model = nn.Sequential(*layers)

    def forward(self, z):
        return self.model(self.dense(z.view(-1, self.z_size)).view(-1, 512, 4, 4))


class _D1(nn.Module):
    """'Standard CNN' discriminator, arch 1 (GLI:235-319)."""

    SPEC = [(None, 64, 3, 1), (64, 64, 4, 2), (64, 128, 3, 1), (128, 128, 4, 2),
            (128, 256, 3, 1), (256, 256, 4, 2), (256, 512, 3, 1)]

    def __init__(self, p):
        super().__init__()
        self.loss_D = p.loss_D
        self.dense = nn.Linear(512 * 4 * 4, 1)
        layers = []
        for idx, (cin, cout, k, s) in enumerate(self.SPEC):
            cin = p.n_colors * _pac(p) if cin is None else cin
            layers.append(_maybe_sn(nn.Conv2d(cin, cout, k, s, 1, bias=True), p.spectral))
            last = idx == len(self.SPEC) - 1
            if p.spectral:
                layers.append(nn.LeakyReLU(0.1, inplace=True))
                continue
            if not p.no_batch_norm_D and not last:
                layers.append(nn.BatchNorm2d(cout))
            layers.append(_act1(p, 0.1))
        self.model = nn.Sequential(*layers)
        self.sig = nn.Sigmoid()

    def forward(self, x):
        out = self.dense(self.model(x).view(-1, 512 * 4 * 4)).view(-1)
        if self.loss_D == 1:
            out = self.sig(out)
        return out


def build_G(p):
    return _G1(p) if p.arch == 1 else _G0(p)


def build_D(p):
    return _D1(p) if p.arch == 1 else _D0(p)


def weights_init(m):
    """GLI:467-475: N(0,0.02) for every *Conv* weight, BN gamma~N(1,0.02), beta=0."""
    kind = type(m).__name__
    if "Conv" in kind:
        m.weight.data.normal_(0.0, 0.02)
    elif "BatchNorm" in kind:
        m.weight.data.normal_(1.0, 0.02)
        m.bias.data.fill_(0)


# --------------------------------------------------------------------------- losses
_bce = nn.BCELoss()
_bce_logits = nn.BCEWithLogitsLoss()


def head_real(kind, r, y):
    """D loss on real outputs for heads 1-4 (GLI:595-604)."""
    if kind == 1:
        return _bce(r, y)
    if kind == 2:
        return torch.mean((r - y) ** 2)
    if kind == 3:
        return -torch.mean(r)
    return torch.mean(torch.nn.ReLU()(1.0 - r))


def head_fake(kind, f, y):
    """D loss on fake outputs for heads 1-4 (GLI:614-623)."""
    if kind == 1:
        return _bce(f, y)
    if kind == 2:
        return torch.mean(f ** 2)
    if kind == 3:
        return torch.mean(f)
    return torch.mean(torch.nn.ReLU()(1.0 + f))


def head_relativistic_D(kind, r, f, y, y2):
    """D loss for heads 5-8 (GLI:634-641)."""
    if kind == 5:
        return _bce_logits(r - f, y)
    if kind == 6:
        return (_bce_logits(r - torch.mean(f), y) + _bce_logits(f - torch.mean(r), y2)) / 2
    if kind == 7:
        return (torch.mean((r - torch.mean(f) - y) ** 2) + torch.mean((f - torch.mean(r) + y) ** 2)) / 2
    return (torch.mean(torch.nn.ReLU()(1.0 - (r - torch.mean(f))))
            + torch.mean(torch.nn.ReLU()(1.0 + (f - torch.mean(r))))) / 2


def head_G(kind, f, r, y, y2):
    """G loss, all heads (GLI:686-709); ``r`` is None for heads 1-4."""
    if kind == 1:
        return _bce(f, y)
    if kind == 2:
        return torch.mean((f - y) ** 2)
    if kind in (3, 4):
        return -torch.mean(f)
    if kind == 5:
        return _bce_logits(f - r, y)
    if kind == 6:
        return (_bce_logits(r - torch.mean(f), y2) + _bce_logits(f - torch.mean(r), y)) / 2
    if kind == 7:
        return (torch.mean((r - torch.mean(f) + y) ** 2) + torch.mean((f - torch.mean(r) - y) ** 2)) / 2
    return (torch.mean(torch.nn.ReLU()(1.0 + (r - torch.mean(f))))
            + torch.mean(torch.nn.ReLU()(1.0 - (f - torch.mean(r))))) / 2


def gradient_penalty(D, x, x_fake, u, penalty, grad_outputs):
    """WGAN-GP term (GLI:648-657): returns (penalty, interpolates)."""
    x_both = x.data * u + x_fake.data * (1 - u)
    x_both = x_both.detach().requires_grad_(True)
    g = torch.autograd.grad(outputs=D(x_both), inputs=x_both, grad_outputs=grad_outputs,
                            retain_graph=True, create_graph=True, only_inputs=True)[0]
    return penalty * ((g.norm(2, 1).norm(2, 1).norm(2, 1) - 1) ** 2).mean()


# --------------------------------------------------------------------------- trainer
@dataclass
class StepRecord:
    """What one iteration exposes to the parity tests."""
    D: dict = field(default_factory=dict)
    G: dict = field(default_factory=dict)


class Trainer:
    """The reference's module-level script as an object (GLI:147-714).

    ``images`` is the dataset tensor [N, C, S, S] (CPU float).  ``hooks`` receives
    ``hooks(tag, record)`` right before each optimizer step and ``hooks(tag+'.post', ...)``
    right after it, mirroring the golden capture points.
    """

    def __init__(self, param, images, hooks=None, seed_all=True, dtype=torch.float32, device=None):
        """``dtype`` != float32 (test envelope only): modules and buffers are cast after the
        fp32 initialisation, so the same initial values are used at higher precision.
        ``device`` (test envelope only, with a ``feed``: the float64 judge steps of the GPU
        parity tests) moves modules and buffers after that cast; the fp32 replay that is
        pinned to the reference always stays on the CPU."""
        self.p = p = param
        self.hooks = hooks
        if seed_all:
            if p.seed is None:
                p.seed = random.randint(1, 10000)
            random.seed(p.seed)
            numpy.random.seed(p.seed)
            torch.manual_seed(p.seed)
        self.images = images
        self.G = build_G(p)
        self.D = build_D(p)
        self.G.apply(weights_init)
        self.D.apply(weights_init)
        B, C, S = p.batch_size, p.n_colors * _pac(p), p.image_size
        self.pac = _pac(p)
        self.x = torch.FloatTensor(B, C, S, S)
        self.x_fake = torch.FloatTensor(B, C, S, S)
        self.y = torch.FloatTensor(B)
        self.y2 = torch.FloatTensor(B)
        # PacGAN draws 2B z per step: the reference resizes z's .data (PAC:607), which
        # reshaped the Variable on the torch it was written for; allocate it 2B here
        self.z = torch.FloatTensor(B * self.pac, p.z_size, 1, 1)
        self.u = torch.FloatTensor(B, 1, 1, 1)
        self.z_test = torch.FloatTensor(B, p.z_size, 1, 1).normal_(0, 1)
        self.grad_outputs = torch.ones(B)
        if dtype != torch.float32:
            self.G.to(dtype)
            self.D.to(dtype)
            for name in ("x", "x_fake", "y", "y2", "z", "u", "z_test", "grad_outputs"):
                setattr(self, name, getattr(self, name).to(dtype))
        if device is not None:
            self.G.to(device)
            self.D.to(device)
            for name in ("x", "x_fake", "y", "y2", "z", "u", "z_test", "grad_outputs"):
                setattr(self, name, getattr(self, name).to(device))
        self.optD = torch.optim.Adam(self.D.parameters(), lr=p.lr_D, betas=(p.beta1, p.beta2),
                                     weight_decay=p.weight_decay)
        self.optG = torch.optim.Adam(self.G.parameters(), lr=p.lr_G, betas=(p.beta1, p.beta2),
                                     weight_decay=p.weight_decay)
        self.decayD = torch.optim.lr_scheduler.ExponentialLR(self.optD, gamma=1 - p.decay)
        self.decayG = torch.optim.lr_scheduler.ExponentialLR(self.optG, gamma=1 - p.decay)
        self.errD = self.errG = None

    # -- data
    def next_real(self):
        """GLI:176-177 (PAC:176: 2B indices, packed channel-wise at PAC:582/682)."""
        B = self.p.batch_size
        idx = numpy.random.choice(self.images.shape[0], size=B * self.pac, replace=False)
        return pack(torch.stack([self.images[i] for i in idx], 0), B, self.pac)

    def _set_D_grad(self, flag):
        for q in self.D.parameters():
            q.requires_grad = flag

    # -- one iteration (GLI:560-714)
    def iteration(self, i, feed=None):
        """One reference iteration.  ``feed`` (test teacher-forcing only) supplies the
        random inputs {x_D, z_D, u, z_G, x_G} instead of drawing them."""
        p, D, G = self.p, self.D, self.G
        draw_real = (lambda key: feed[key]) if feed else (lambda key: self.next_real())
        rec = StepRecord()
        if i % p.print_every == 0:
            G(self.z_test)  # sample image; mutates G's BN running statistics (GLI:564)
        self._set_D_grad(True)
        for _ in range(p.Diters):
            D.zero_grad()
            real = draw_real("x_D")
            B = real.size(0)
            self.x.data.resize_as_(real).copy_(real)
            y_pred = D(self.x)
            if p.loss_D in (1, 2, 3, 4):
                self.y.data.resize_(B).fill_(1)
                err_real = head_real(p.loss_D, y_pred, self.y)
                err_real.backward()
                self._draw_z(B * self.pac, feed, "z_D")
                fake = G(self.z)
                self.x_fake.data.resize_(pack(fake, B, self.pac).size()).copy_(pack(fake.data, B, self.pac))
                self.y.data.resize_(B).fill_(0)
                y_pred_fake = D(self.x_fake.detach())
                err_fake = head_fake(p.loss_D, y_pred_fake, self.y)
                err_fake.backward()
                errD = err_real + err_fake
            else:
                self.y.data.resize_(B).fill_(1)
                self.y2.data.resize_(B).fill_(0)
                self._draw_z(B * self.pac, feed, "z_D")
                fake = G(self.z)
                self.x_fake.data.resize_(pack(fake, B, self.pac).size()).copy_(pack(fake.data, B, self.pac))
                y_pred_fake = D(self.x_fake.detach())
                errD = head_relativistic_D(p.loss_D, y_pred, y_pred_fake, self.y, self.y2)
                errD.backward()
            rec.D.update(x=self.x.clone(), z=self.z.clone(), y_pred=y_pred.detach(),
                         y_pred_fake=y_pred_fake.detach(), errD=errD.detach())
            if p.loss_D == 3 or p.grad_penalty:
                self.u.data.resize_(B, 1, 1, 1)
                if feed:
                    self.u.data.copy_(feed["u"])
                elif self.u.dtype != torch.float32:
                    self.u.data.copy_(torch.empty(B, 1, 1, 1).uniform_(0, 1))
                else:
                    self.u.uniform_(0, 1)
                gp = gradient_penalty(D, self.x, self.x_fake, self.u, p.penalty, self.grad_outputs)
                gp.backward()
                rec.D.update(u=self.u.clone(), gp=gp.detach())
            if self.hooks:
                self.hooks("D", rec.D)
            self.optD.step()
            if self.hooks:
                self.hooks("D.post", rec.D)
        self.errD = errD
        self._set_D_grad(False)
        for _ in range(p.Giters):
            G.zero_grad()
            self.y.data.resize_(B).fill_(1)
            self._draw_z(B * self.pac, feed, "z_G")
            if self.pac == 1:
                fake = G(self.z)
            else:
                # PAC:673-674: the fresh z is drawn but unused; the G step reuses the D step's
                # G(z) output (graph included) -- G's weights have not moved since
                fake = pack(fake, B, self.pac)
            y_pred_fake = D(fake)
            y_pred = None
            if p.loss_D not in (1, 2, 3, 4):
                real = draw_real("x_G")
                B = real.size(0)
                self.x.data.resize_as_(real).copy_(real)
                if p.loss_D == 6:
                    y_pred = D(self.x)
                    self.y2.data.resize_(B).fill_(0)
                else:
                    y_pred = D(self.x)
            errG = head_G(p.loss_D, y_pred_fake, y_pred, self.y, self.y2)
            errG.backward()
            rec.G.update(z=self.z.clone(), y_pred_fake=y_pred_fake.detach(), errG=errG.detach())
            if y_pred is not None:
                rec.G.update(x=self.x.clone(), y_pred=y_pred.detach())
            if self.hooks:
                self.hooks("G", rec.G)
            self.optG.step()
            if self.hooks:
                self.hooks("G.post", rec.G)
        self.errG = errG
        self.decayD.step()
        self.decayG.step()
        return rec

    def _draw_z(self, B, feed, key):
        if feed:
            self.z.data.resize_(B, self.p.z_size, 1, 1).copy_(feed[key])
        elif self.z.dtype != torch.float32:  # envelope runs: the fp32 draws, cast
            self.z.data.resize_(B, self.p.z_size, 1, 1).copy_(torch.empty(B, self.p.z_size, 1, 1).normal_(0, 1))
        else:
            self.z.data.resize_(B, self.p.z_size, 1, 1).normal_(0, 1)

    def log_line(self, i, elapsed):
        """The reference's progress line format (GLI:723)."""
        d, g = self.errD.data.item(), self.errG.data.item()
        return '[%d] Diff: %.4f loss_D: %.4f loss_G: %.4f time:%.4f' % (i, -d + g, d, g, elapsed)


def optimizer_state(opt, module):
    """{param-name: (exp_avg, exp_avg_sq, step)} for the module's parameters."""
    out = {}
    for (n, q) in module.named_parameters():
        st = opt.state.get(q, {})
        if st:
            out[n] = (st["exp_avg"], st["exp_avg_sq"], float(st["step"]))
    return out


def checkpoint(t, i, current_set_images):
    """The reference's checkpoint dict (GLI:737-747; saved with torch.save at GLI:737)."""
    return {"i": i, "current_set_images": current_set_images, "G_state": t.G.state_dict(),
            "D_state": t.D.state_dict(), "G_optimizer": t.optG.state_dict(), "D_optimizer": t.optD.state_dict(),
            "G_scheduler": t.decayG.state_dict(), "D_scheduler": t.decayD.state_dict(), "z_test": t.z_test}


def load_checkpoint(t, ck):
    """GLI:537-549: restore modules, optimizers, schedulers and z_test into a freshly built
    (and seeded) trainer; returns (iter_offset, current_set_images)."""
    t.G.load_state_dict(ck["G_state"])
    t.D.load_state_dict(ck["D_state"])
    t.optG.load_state_dict(ck["G_optimizer"])
    t.optD.load_state_dict(ck["D_optimizer"])
    t.decayG.load_state_dict(ck["G_scheduler"])
    t.decayD.load_state_dict(ck["D_scheduler"])
    t.z_test.copy_(ck["z_test"])
    return ck["i"], ck["current_set_images"]
