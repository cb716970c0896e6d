"""DCGAN_G / DCGAN_D with the reference's surface, running on the HIP kernels.

The reference builds its nets from ``param`` globals (GLI:183-460).  Here the classes
take ``param`` explicitly (any namespace with the GLI:17-62 flag names) and keep:

* the module tree and ``add_module`` names, hence every ``state_dict`` key (SURVEY
  Appendix C), so reference checkpoints load unchanged;
* the parameter-initialisation RNG stream: each conv/linear/spectral-norm layer is
  initialised by the same torch CPU init calls in the same order as the reference's
  constructors (kaiming-uniform, bias uniform, spectral u/v normal draws), and
  ``weights_init`` (GLI:466-477) matches the same class-name patterns;
* forward semantics: train-mode BatchNorm with running-stat updates, one spectral
  power iteration per train-mode forward, ``D(x).view(-1)`` outputs.

Forward runs the layers as fused ``ConvLayerFn`` calls (conv + bias + BN + activation)
rather than module-by-module: the activation modules are name placeholders only.
Activations between layers are NHWC; G's output image is NCHW-contiguous like the
reference's, and D accepts images in any layout.
"""
import math

import torch
import torch.nn as nn

from . import autograd as AG
from . import ops
from .autograd import ConvLayerFn, LayerSpec
from .kernels import ConvGeom, spectral_power, spectral_power_batch


# ---------------------------------------------------------------- parameter holders
class _ConvBase(nn.Module):
    transposed = False

    def __init__(self, cin, cout, k, stride, pad, bias, spectral, upsample=1):
        super().__init__()
        self.cin, self.cout, self.k, self.stride, self.pad = cin, cout, k, stride, pad
        self.spectral = spectral
        ctor = torch.nn.ConvTranspose2d if self.transposed else torch.nn.Conv2d
        tmp = ctor(cin, cout, k, stride, pad, bias=bias)  # same RNG draws as the reference
        if spectral:
            tmp = torch.nn.utils.spectral_norm(tmp)       # draws u then v (spectral_norm.py:168-169)
            # torch's spectral_norm deletes `weight` and registers `weight_orig` AFTER `bias`:
            # parameter order = optimizer state order (Adam.state_dict is positional)
            self.bias = nn.Parameter(tmp.bias.detach().clone()) if bias else None
            self.weight_orig = nn.Parameter(tmp.weight_orig.detach().clone())
            self.register_buffer("weight_u", tmp.weight_u.detach().clone())
            self.register_buffer("weight_v", tmp.weight_v.detach().clone())
        else:
            self.weight = nn.Parameter(tmp.weight.detach().clone())
            self.bias = nn.Parameter(tmp.bias.detach().clone()) if bias else None
        self.geom = ConvGeom(k, stride, pad, self.transposed, upsample)

    @property
    def w(self):
        return self.weight_orig if self.spectral else self.weight

    def extra_repr(self):
        return (f"{self.cin}, {self.cout}, kernel_size=({self.k}, {self.k}), stride=({self.stride}, {self.stride}),"
                f" padding=({self.pad}, {self.pad}), bias={self.bias is not None}, spectral={self.spectral}")


class Conv2d(_ConvBase):
    """Conv2d parameters (torch layout [cout][cin][k][k])."""

    def __init__(self, cin, cout, k, stride=1, pad=0, bias=True, spectral=False, upsample=1):
        super().__init__(cin, cout, k, stride, pad, bias, spectral, upsample)


class ConvTranspose2d(_ConvBase):
    """ConvTranspose2d parameters (torch layout [cin][cout][k][k])."""
    transposed = True

    def __init__(self, cin, cout, k, stride=1, pad=0, bias=True, spectral=False):
        super().__init__(cin, cout, k, stride, pad, bias, spectral)


class SpectralConv2d(Conv2d):
    """Spectral-norm Conv2d: state_dict weight_orig / weight_u / weight_v; ``.weight``
    aliases weight_orig like torch's hook-based attribute (so weights_init hits it)."""

    def __init__(self, *a, **k):
        super().__init__(*a, spectral=True, **k)

    @property
    def weight(self):
        return self.weight_orig


class SpectralConvTranspose2d(ConvTranspose2d):
    def __init__(self, *a, **k):
        super().__init__(*a, spectral=True, **k)

    @property
    def weight(self):
        return self.weight_orig


class Linear(nn.Module):
    """Linear parameters; run as a 1x1 (arch-1 G) or k4 (arch-1 D) convolution."""

    def __init__(self, fin, fout):
        super().__init__()
        tmp = torch.nn.Linear(fin, fout)
        self.weight = nn.Parameter(tmp.weight.detach().clone())
        self.bias = nn.Parameter(tmp.bias.detach().clone())
        self.in_features, self.out_features = fin, fout

    def extra_repr(self):
        return f"in_features={self.in_features}, out_features={self.out_features}, bias=True"


class BatchNorm2d(nn.Module):
    """BatchNorm2d parameters and running buffers (torch.nn.BatchNorm2d's names/defaults)."""

    def __init__(self, c, eps=1e-5, momentum=0.1):
        super().__init__()
        self.num_features, self.eps, self.momentum = c, eps, momentum
        self.weight = nn.Parameter(torch.ones(c))
        self.bias = nn.Parameter(torch.zeros(c))
        self.register_buffer("running_mean", torch.zeros(c))
        self.register_buffer("running_var", torch.ones(c))
        self.register_buffer("num_batches_tracked", torch.tensor(0, dtype=torch.long))

    def extra_repr(self):
        return f"{self.num_features}, eps={self.eps}, momentum={self.momentum}, affine=True, track_running_stats=True"


class _Act(nn.Module):
    """Name placeholder for an activation module (the math is fused into the kernels)."""

    def __init__(self, kind, alpha=0.0):
        super().__init__()
        self.kind, self.alpha = kind, alpha

    def extra_repr(self):
        return f"{self.kind}" + (f", {self.alpha}" if self.kind == "lrelu" else "")


class _Upsample(nn.Module):
    def __init__(self):
        super().__init__()


def weights_init(m):
    """GLI:467-475: N(0,0.02) for *Conv* weights, N(1,0.02)/0 for *BatchNorm* affine."""
    name = m.__class__.__name__
    if name.find("Conv") != -1:
        m.weight.data.normal_(0.0, 0.02)
    elif name.find("BatchNorm") != -1:
        m.weight.data.normal_(1.0, 0.02)
        m.bias.data.fill_(0)


# ---------------------------------------------------------------- fused layer plan
VIEW_OUT_CHANNELS_LAST = True  # C4 3.850 -> 3.800 ms/step (tools/ab_dense_cl.py, run r4ac)


class _Layer:
    """One fused step: conv module (+ bn module) + activation."""

    __slots__ = ("conv", "bn", "spec", "w_view", "in_view", "out_view")

    def __init__(self, conv, bn, act, alpha=0.0, nchw_out=False, w_view=None, in_view=None, out_view=None):
        self.conv, self.bn = conv, bn
        geom = conv.geom if isinstance(conv, _ConvBase) else None
        self.spec = (LayerSpec(geom, act, alpha, bn is not None, spectral=getattr(conv, "spectral", False),
                               nchw_out=nchw_out) if geom is not None else None)
        self.w_view, self.in_view, self.out_view = w_view, in_view, out_view

    def weight(self):
        conv = self.conv
        w = conv.w if isinstance(conv, _ConvBase) else conv.weight
        return w.view(*self.w_view) if self.w_view is not None else w

    def run(self, h, training, segs=1, out=None, sn=None, gsegs=None, link_in=None, link_out=None):
        """``sn``: this call's (u, v, inv_sigma) when the net already ran the power
        iteration of all its spectral layers (_Net._spectral); ``gsegs``: leading segments
        that carry an output gradient (ConvLayerFn); ``link_in`` / ``link_out``: the
        autograd.LayerLink to the layer below / above in the same chain call."""
        conv, bn = self.conv, self.bn
        if self.in_view is not None:
            h = h.reshape(h.shape[0], *self.in_view)
        if ops.tracing(h):
            # traced (torch.export / torch.compile): the layer as rgan:: operators (ops.py)
            if segs != 1 or out is not None:
                raise NotImplementedError("traced nets: one forward call per net (no batched segments)")
            res = ops.layer_forward(self, h, training)
            return res.reshape(res.shape[0], *self.out_view) if self.out_view is not None else res
        w = self.weight()
        if self.spec.spectral and sn is None:
            with torch.no_grad():
                inv_sigma = spectral_power(w.detach(), conv.weight_u, conv.weight_v, conv.geom.transposed,
                                           do_iter=training)
            sn = (conv.weight_u.clone(), conv.weight_v.clone(), inv_sigma)
        bufs = (bn.running_mean, bn.running_var, bn.num_batches_tracked, training) if bn is not None else None
        if out is not None and self.out_view is not None:
            raise ValueError("an output buffer for a reshaped layer")
        res = ConvLayerFn.apply(h, w, conv.bias, bn.weight if bn is not None else None,
                                bn.bias if bn is not None else None, self.spec, bufs, sn, segs, out, gsegs,
                                link_in, link_out)
        if self.out_view is not None:
            res = res.reshape(res.shape[0], *self.out_view)
            if VIEW_OUT_CHANNELS_LAST and res.dim() == 4 and res.shape[2] * res.shape[3] > 1:
                # arch 1's dense output viewed as G's NCHW 4x4 map: one channels-last copy so
                # the next ConvT and its weight gradient read it with vector loads
                res = res.contiguous(memory_format=torch.channels_last)
        return res


def _lin_spec(layer, geom, act, alpha=0.0, nchw_out=False):
    layer.spec = LayerSpec(geom, act, alpha, False, nchw_out=nchw_out)
    return layer


class _Net(nn.Module):
    @property
    def _tag(self):
        return type(self).__name__[1]  # "G" / "D": activation-trace tag (parity tests)

    def _spectral(self):
        """One power iteration for every spectral layer of this call, all in four launches
        (torch's spectral_norm pre-hook runs one per layer per train-mode call,
        spectral_norm.py:97-116; u and v of different layers are independent)."""
        idx = [li for li, l in enumerate(self._plan) if l.spec is not None and l.spec.spectral]
        if not idx or not self.training:
            return {}
        with torch.no_grad():
            outs = spectral_power_batch([(self._plan[li].weight().detach(), self._plan[li].conv.weight_u,
                                          self._plan[li].conv.weight_v, self._plan[li].conv.geom.transposed)
                                         for li in idx])
        return dict(zip(idx, outs))

    def _links(self):
        """One autograd.LayerLink per boundary between consecutive layers whose output feeds
        the next layer directly (no reshape between them), else None: the upper layer's
        data-gradient GEMM then applies the lower layer's activation / BatchNorm backward pass
        in its epilogue."""
        plan = self._plan
        return [AG.LayerLink() if plan[i].out_view is None and plan[i + 1].in_view is None else None
                for i in range(len(plan) - 1)] + [None]

    def _run(self, x, out=None):
        """``out``: a buffer for the last layer's output (e.g. half of a batched D input)."""
        AG.TRACE_NET = self._tag
        h = x
        last = len(self._plan) - 1
        if ops.tracing(x):  # rgan:: operators per layer (ops.layer_forward): no fused hand-offs
            for layer in self._plan:
                h = layer.run(h, self.training)
            return h
        sns = self._spectral()
        links = self._links()
        for li, layer in enumerate(self._plan):
            AG.TRACE_LAYER = li
            h = layer.run(h, self.training, out=out if li == last else None, sn=sns.get(li),
                          link_in=links[li - 1] if li else None, link_out=links[li])
        return h

    @property
    def segmentable(self):
        """Several forward calls can share one batched pass (no spectral layer: the
        reference runs one power iteration per call, so each call has its own sigma)."""
        return not any(layer.spec is not None and layer.spec.spectral for layer in self._plan)

    def forward_segments(self, xs, cat=None, flat=False, grad_segs=None):
        """``[self(x) for x in xs]`` as ONE pass over the concatenated batch: every layer's
        GEMMs run once over all segments, BatchNorm normalises (and updates its running
        statistics) per segment in list order, exactly as the separate calls would.
        ``cat``: the segments already laid out back to back in one tensor (no copy; inputs
        that require grad get it back through _Joined);
        ``flat``: return the joint output (segments back to back) instead of a list;
        ``grad_segs``: only the leading segments' outputs get a gradient (the rest is used
        as a constant, e.g. the G step's no-graph D(x)): the backward runs over their rows."""
        if not self.segmentable:
            raise ValueError("forward_segments: a spectral-norm layer needs one call per forward")
        n = len(xs)
        B = xs[0].shape[0]
        if any(x.shape != xs[0].shape for x in xs):
            raise ValueError("forward_segments: segments must have equal shapes")
        trace0 = len(AG.ACT_TRACE) if AG.ACT_TRACE is not None else 0
        AG.TRACE_NET = self._tag
        if grad_segs is not None and any(x.requires_grad for x in xs[grad_segs:]):
            raise ValueError("forward_segments: an input past grad_segs requires grad")
        if cat is None:
            h = torch.cat(xs)
        elif any(x.requires_grad for x in xs):
            h = _Joined.apply(cat, *xs)
        else:
            h = cat
        links = self._links()
        for li, layer in enumerate(self._plan):
            AG.TRACE_LAYER = li
            h = layer.run(h, self.training, n, gsegs=grad_segs, link_in=links[li - 1] if li else None,
                          link_out=links[li])
        if AG.ACT_TRACE is not None:  # activation masks in the separate calls' order
            masks = AG.ACT_TRACE[trace0:]
            layers = AG.ACT_LAYERS[trace0:]
            del AG.ACT_TRACE[trace0:]
            del AG.ACT_TAGS[trace0:]
            del AG.ACT_LAYERS[trace0:]
            for s_ in range(n):
                AG.ACT_TRACE.extend(m[s_ * B:(s_ + 1) * B] for m in masks)
                AG.ACT_TAGS.extend(self._tag for _ in masks)
                AG.ACT_LAYERS.extend(layers)
        return h if flat else list(h.split(B))

    def forward_pair_G(self, fake, x, cat=None):
        """[D(G(z)); D(x)] of the G step (GLI:674, 695-707) as one batched pass: BatchNorm
        per call in the reference's call order (fake first), gradient through the fake half
        only (the reference's D(x) there has no graph: D's parameters are frozen, x is data)."""
        return self.forward_segments([fake, x], cat, flat=True, grad_segs=1).reshape(-1)


class _Joined(torch.autograd.Function):
    """The segments ``xs`` already written back to back into ``cat`` (e.g. G's output
    written into the first half of the batched D input): a view of ``cat`` whose gradient
    goes back to each segment's producer as its rows (no concatenation either way)."""

    @staticmethod
    def forward(ctx, cat, *xs):
        ctx.B = xs[0].shape[0]
        ctx.need = [x.requires_grad for x in xs]
        return cat.view_as(cat)

    @staticmethod
    def backward(ctx, g):
        B = ctx.B
        return (None,) + tuple(g[k * B:(k + 1) * B] if need else None for k, need in enumerate(ctx.need))


# ---------------------------------------------------------------- arch 0 (DCGAN)
class _G0(_Net):
    """DCGAN generator (GLI:323-397)."""

    def __init__(self, p):
        super().__init__()
        self.param = p
        main = nn.Sequential()
        plan = []
        mult = p.image_size // 8
        sn = p.spectral_G

        def block(part, suffix, conv, ch):
            main.add_module(conv[0], conv[1])
            if p.SELU:
                main.add_module(f"{part}-SELU{suffix}", _Act("selu"))
                plan.append(_Layer(conv[1], None, "selu"))
                return
            bn = None
            if not p.no_batch_norm_G and not sn:
                bn = BatchNorm2d(ch)
                main.add_module(f"{part}-BatchNorm2d{suffix}", bn)
            act = "tanh" if p.Tanh_GD else "relu"
            main.add_module(f"{part}-{'Tanh' if p.Tanh_GD else 'ReLU'}{suffix}", _Act(act))
            plan.append(_Layer(conv[1], bn, act))

        cls = SpectralConvTranspose2d if sn else ConvTranspose2d
        start = cls(p.z_size, p.G_h_size * mult, 4, 1, 0, bias=False)
        block("Start", "", ("Start-SpectralConvTranspose2d" if sn else "Start-ConvTranspose2d", start),
              p.G_h_size * mult)
        i = 1
        while mult > 1:
            cin, cout = p.G_h_size * mult, p.G_h_size * (mult // 2)
            if p.NN_conv:
                main.add_module("Middle-UpSample [%d]" % i, _Upsample())
                ccls = SpectralConv2d if sn else Conv2d
                conv = ccls(cin, cout, 3, 1, 1, bias=True, upsample=2)  # Upsample folded into the conv
                name = ("Middle-SpectralConv2d [%d]" if sn else "Middle-Conv2d [%d]") % i
            else:
                conv = cls(cin, cout, 4, 2, 1, bias=False)
                name = ("Middle-SpectralConvTranspose2d [%d]" if sn else "Middle-ConvTranspose2d [%d]") % i
            block("Middle", " [%d]" % i, (name, conv), cout)
            mult //= 2
            i += 1
        if p.NN_conv:
            main.add_module("End-UpSample", _Upsample())
            ccls = SpectralConv2d if sn else Conv2d
            end = ccls(p.G_h_size, p.n_colors, 3, 1, 1, bias=True, upsample=2)
            main.add_module("End-SpectralConv2d" if sn else "End-Conv2d", end)
        else:
            end = cls(p.G_h_size, p.n_colors, 4, 2, 1, bias=False)
            main.add_module("End-SpectralConvTranspose2d" if sn else "End-ConvTranspose2d", end)
        main.add_module("End-Tanh", _Act("tanh"))
        plan.append(_Layer(end, None, "tanh", nchw_out=True))
        self.main = main
        self._plan = plan

    def forward(self, z, out=None):
        return self._run(z, out)


class _D0(_Net):
    """DCGAN discriminator (GLI:400-460)."""

    def __init__(self, p):
        super().__init__()
        self.param = p
        main = nn.Sequential()
        plan = []
        sn = p.spectral
        cls = SpectralConv2d if sn else Conv2d
        start = cls(p.n_colors * getattr(p, "pac", 1), p.D_h_size, 4, 2, 1, bias=False)  # PAC:408-410
        main.add_module("Start-SpectralConv2d" if sn else "Start-Conv2d", start)
        if p.SELU:
            main.add_module("Start-SELU", _Act("selu"))
            plan.append(_Layer(start, None, "selu"))
        elif p.Tanh_GD:
            main.add_module("Start-Tanh", _Act("tanh"))
            plan.append(_Layer(start, None, "tanh"))
        else:
            main.add_module("Start-LeakyReLU", _Act("lrelu", 0.2))
            plan.append(_Layer(start, None, "lrelu", 0.2))
        size, mult, i = p.image_size // 2, 1, 0
        while size > 4:
            cin, cout = p.D_h_size * mult, p.D_h_size * 2 * mult
            conv = cls(cin, cout, 4, 2, 1, bias=False)
            main.add_module(("Middle-SpectralConv2d [%d]" if sn else "Middle-Conv2d [%d]") % i, conv)
            if p.SELU:
                main.add_module("Middle-SELU [%d]" % i, _Act("selu"))
                plan.append(_Layer(conv, None, "selu"))
            else:
                bn = None
                if not p.no_batch_norm_D and not sn:
                    bn = BatchNorm2d(cout)
                    main.add_module("Middle-BatchNorm2d [%d]" % i, bn)
                if p.Tanh_GD:
                    main.add_module("Start-Tanh [%d]" % i, _Act("tanh"))  # the reference's name (GLI:435)
                    plan.append(_Layer(conv, bn, "tanh"))
                else:
                    main.add_module("Middle-LeakyReLU [%d]" % i, _Act("lrelu", 0.2))
                    plan.append(_Layer(conv, bn, "lrelu", 0.2))
            size //= 2
            mult *= 2
            i += 1
        end = cls(p.D_h_size * mult, 1, 4, 1, 0, bias=False)
        main.add_module("End-SpectralConv2d" if sn else "End-Conv2d", end)
        act = "none"
        if p.loss_D == 1:
            main.add_module("End-Sigmoid", _Act("sigmoid"))
            act = "sigmoid"
        plan.append(_Layer(end, None, act))
        self.main = main
        self._plan = plan

    def forward(self, x):
        return self._run(x).view(-1)

    def forward_pair(self, x, x_fake, cat=None):
        """[D(x); D(x_fake)] as one [2B] vector from one batched pass (``forward_segments``):
        the loss heads read both halves of it (losses.loss_D_cat), so autograd sees one
        output and the backward needs no concatenation of two gradients."""
        return self.forward_segments([x, x_fake], cat, flat=True).reshape(-1)


# ---------------------------------------------------------------- arch 1 ("standard CNN", 32x32)
class _G1(_Net):
    """Standard-CNN generator (GLI:186-233)."""

    def __init__(self, p):
        super().__init__()
        self.param = p
        self.z_size = p.z_size
        self.dense = Linear(p.z_size, 512 * 4 * 4)
        layers, plan = [], []
        # dense as a 1x1 conv on [B, z, 1, 1]; its [B, 8192] output is the NCHW [B,512,4,4]
        plan.append(_lin_spec(_Layer(self.dense, None, "none", w_view=(8192, p.z_size, 1, 1),
                                     in_view=(p.z_size, 1, 1), out_view=(512, 4, 4)),
                              ConvGeom(1, 1, 0, False), "none"))
        self.dense.geom = ConvGeom(1, 1, 0, False)
        sn = p.spectral_G
        for cin, cout in ((512, 256), (256, 128), (128, 64)):
            conv = (SpectralConvTranspose2d if sn else ConvTranspose2d)(cin, cout, 4, 2, 1, bias=True)
            layers.append(conv)
            if sn:
                layers.append(_Act("relu"))
                plan.append(_Layer(conv, None, "relu"))
                continue
            bn = None
            if not p.no_batch_norm_G:
                bn = BatchNorm2d(cout)
                layers.append(bn)
            act = "tanh" if p.Tanh_GD else "relu"
            layers.append(_Act(act))
            plan.append(_Layer(conv, bn, act))
        end = (SpectralConv2d if sn else Conv2d)(64, p.n_colors, 3, 1, 1, bias=True)
        layers += [end, _Act("tanh")]
        plan.append(_Layer(end, None, "tanh", nchw_out=True))
        self.model = nn.Sequential(*layers)
        self._plan = plan

    def forward(self, z, out=None):
        return self._run(z, out)


class _D1(_Net):
    """Standard-CNN discriminator (GLI:235-319)."""

    SPEC = ((None, 64, 3, 1), (64, 64, 4, 2), (64, 128, 3, 1), (128, 128, 4, 2),
            (128, 256, 3, 1), (256, 256, 4, 2), (256, 512, 3, 1))

    def __init__(self, p):
        super().__init__()
        self.param = p
        self.dense = Linear(512 * 4 * 4, 1)
        layers, plan = [], []
        sn = p.spectral
        for idx, (cin, cout, k, s) in enumerate(self.SPEC):
            cin = p.n_colors * getattr(p, "pac", 1) if cin is None else cin  # PAC:242,260
            conv = (SpectralConv2d if sn else Conv2d)(cin, cout, k, s, 1, bias=True)
            layers.append(conv)
            if sn:
                layers.append(_Act("lrelu", 0.1))
                plan.append(_Layer(conv, None, "lrelu", 0.1))
                continue
            bn = None
            if not p.no_batch_norm_D and idx < len(self.SPEC) - 1:
                bn = BatchNorm2d(cout)
                layers.append(bn)
            act = "tanh" if p.Tanh_GD else "lrelu"
            layers.append(_Act(act, 0.1))
            plan.append(_Layer(conv, bn, act, 0.1))
        self.model = nn.Sequential(*layers)
        self.sig = _Act("sigmoid")
        # dense(view(-1, 512*4*4)) == a k4 conv over the [B,512,4,4] map with W viewed [1,512,4,4]
        act = "sigmoid" if p.loss_D == 1 else "none"
        plan.append(_lin_spec(_Layer(self.dense, None, act, w_view=(1, 512, 4, 4)), ConvGeom(4, 1, 0, False), act))
        self.dense.geom = ConvGeom(4, 1, 0, False)
        self._plan = plan

    def forward(self, x):
        return self._run(x).view(-1)

    def forward_pair(self, x, x_fake, cat=None):
        return self.forward_segments([x, x_fake], cat, flat=True).reshape(-1)


def DCGAN_G(param):
    """Generator for ``param.arch`` (0: DCGAN, 1: standard CNN), like GLI's DCGAN_G()."""
    return _G1(param) if param.arch == 1 else _G0(param)


def DCGAN_D(param):
    """Discriminator for ``param.arch``, like GLI's DCGAN_D()."""
    return _D1(param) if param.arch == 1 else _D0(param)
