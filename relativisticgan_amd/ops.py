"""torch.library registration of the HIP kernels: the ``rgan::`` operator namespace.

SURVEY §8(b) "Op registration": every hot-path kernel family is a registered operator with a
fake (meta) implementation -- output shapes *and* the NHWC strides the kernels produce -- and
an autograd formula built only from other ``rgan::`` operators, so ``torch.export`` and the
dispatcher-level tracers see the MI355X kernels as graph nodes (not opaque Python), and
``create_graph`` backward differentiates the convolutions on the same kernels:

  rgan::conv2d           Conv2d / ConvTranspose2d (+ bias + activation) forward   GLI:336-448
  rgan::conv2d_dgrad     its data gradient
  rgan::conv2d_wgrad     its weight gradient
  rgan::channel_sum      bias gradient (sum over pixels)
  rgan::act_backward     activation backward from the activation output
  rgan::batch_norm_stats_ train-mode batch statistics, running stats updated    GLI:341,366,433
  rgan::batch_norm_apply normalise + activation (train-mode BatchNorm2d derivative)
  rgan::batch_norm_backward
  rgan::spectral_power_  spectral_norm's power iteration (u, v in place)          GLI:334-446
  rgan::spectral_scale   W / sigma (u, v constant in the derivative)
  rgan::spectral_backward
  rgan::loss_head        the eight --loss_D heads (D side 0/1, G side 2)           GLI:592-709
  rgan::loss_head_grad
  rgan::gp_penalty       lam * mean((||g_b|| - 1)^2)                               GLI:646-658
  rgan::gp_penalty_backward
  rgan::adam_            torch.optim.Adam's single-tensor step (mutating)          GLI:659,712

Differentiability: every op above has a first-order formula; conv2d / conv2d_dgrad /
conv2d_wgrad and act_backward of the piecewise-linear activations (ReLU, LeakyReLU, none) are
differentiable to any order (the WGAN-GP double backward of a conv chain).  The second
derivative of BatchNorm and of the curved activations is the native GP engine's (gp.py) and
raises here.  The training step itself runs the fused layers (autograd.ConvLayerFn: GEMM
epilogue statistics, producer post-ops, batched passes); ``nets`` routes through these ops
when it is traced (torch.export / torch.compile), so an exported D or G is a graph of
``rgan::`` nodes on the same kernels.
"""
from typing import List, Optional, Tuple

import torch

from . import kernels as K
from .kernels import ConvGeom

_LIB = "rgan"
_DEV = "cuda"

# activations whose derivative is piecewise constant (act'' = 0 away from the kink)
_PL_ACTS = ("none", "relu", "lrelu")


def _geom(k, stride, pad, transposed, upsample):
    return ConvGeom(int(k), int(stride), int(pad), bool(transposed), int(upsample))


def _nhwc_like(shape, device):
    B, C, H, W = shape
    return torch.empty_strided((B, C, H, W), (H * W * C, 1, W * C, C), dtype=torch.float32, device=device)


def _out_shape(x_shape, w_shape, geom):
    B, _, H, W = x_shape
    cout = w_shape[1] if geom.transposed else w_shape[0]
    if geom.upsample != 1:  # --NN_conv: the weight is the 3x3 Conv2d's [cout][cin][3][3]
        cout = w_shape[0]
    Ho, Wo = geom.out_hw(H, W)
    return (B, cout, Ho, Wo)


# ------------------------------------------------------------------ convolution
@torch.library.custom_op("rgan::conv2d", mutates_args=(), device_types=_DEV)
def conv2d(x: torch.Tensor, w: torch.Tensor, bias: Optional[torch.Tensor], k: int, stride: int, pad: int,
           transposed: bool, upsample: int, act: str, alpha: float, nchw_out: bool) -> torch.Tensor:
    """act(conv(x, w) + bias), NHWC output (NCHW when nchw_out: the image G emits)."""
    return K.conv_fwd(x, w, _geom(k, stride, pad, transposed, upsample), bias=bias, act=act, alpha=alpha,
                      nchw_out=nchw_out)


@conv2d.register_fake
def _(x, w, bias, k, stride, pad, transposed, upsample, act, alpha, nchw_out):
    shape = _out_shape(x.shape, w.shape, _geom(k, stride, pad, transposed, upsample))
    if nchw_out:
        return torch.empty(shape, dtype=torch.float32, device=x.device)
    return _nhwc_like(shape, x.device)


def _conv2d_setup(ctx, inputs, output):
    x, w, bias, k, stride, pad, transposed, upsample, act, alpha, nchw_out = inputs
    ctx.args = (k, stride, pad, transposed, upsample)
    ctx.act, ctx.alpha, ctx.has_bias = act, alpha, bias is not None
    ctx.x_shape, ctx.w_shape = tuple(x.shape), tuple(w.shape)
    ctx.save_for_backward(x, w, output if act != "none" else None)


def _conv2d_backward(ctx, g):
    x, w, out = ctx.saved_tensors
    k, stride, pad, transposed, upsample = ctx.args
    if ctx.act != "none":
        g = torch.ops.rgan.act_backward(g, out, ctx.act, ctx.alpha)
    elif not K.is_nhwc(g) and g.dim() == 4:
        g = g.contiguous(memory_format=torch.channels_last)
    nx, nw, nb = ctx.needs_input_grad[:3]
    dx = torch.ops.rgan.conv2d_dgrad(g, w, list(ctx.x_shape), k, stride, pad, transposed, upsample) if nx else None
    dw = torch.ops.rgan.conv2d_wgrad(x, g, list(ctx.w_shape), k, stride, pad, transposed, upsample) if nw else None
    db = torch.ops.rgan.channel_sum(g) if (nb and ctx.has_bias) else None
    return dx, dw, db, None, None, None, None, None, None, None, None


conv2d.register_autograd(_conv2d_backward, setup_context=_conv2d_setup)


@torch.library.custom_op("rgan::conv2d_dgrad", mutates_args=(), device_types=_DEV)
def conv2d_dgrad(dy: torch.Tensor, w: torch.Tensor, x_shape: List[int], k: int, stride: int, pad: int,
                 transposed: bool, upsample: int) -> torch.Tensor:
    return K.conv_dgrad(dy, w, _geom(k, stride, pad, transposed, upsample), tuple(x_shape))


@conv2d_dgrad.register_fake
def _(dy, w, x_shape, k, stride, pad, transposed, upsample):
    return _nhwc_like(tuple(x_shape), dy.device)


def _dgrad_setup(ctx, inputs, output):
    dy, w, x_shape, k, stride, pad, transposed, upsample = inputs
    ctx.args = (k, stride, pad, transposed, upsample)
    ctx.w_shape = tuple(w.shape)
    ctx.save_for_backward(dy, w)


def _dgrad_backward(ctx, ddx):
    dy, w = ctx.saved_tensors
    k, stride, pad, transposed, upsample = ctx.args
    if not K.is_nhwc(ddx):
        ddx = ddx.contiguous(memory_format=torch.channels_last)
    d_dy = (torch.ops.rgan.conv2d(ddx, w, None, k, stride, pad, transposed, upsample, "none", 0.0, False)
            if ctx.needs_input_grad[0] else None)
    d_w = (torch.ops.rgan.conv2d_wgrad(ddx, dy, list(ctx.w_shape), k, stride, pad, transposed, upsample)
           if ctx.needs_input_grad[1] else None)
    return d_dy, d_w, None, None, None, None, None, None


conv2d_dgrad.register_autograd(_dgrad_backward, setup_context=_dgrad_setup)


@torch.library.custom_op("rgan::conv2d_wgrad", mutates_args=(), device_types=_DEV)
def conv2d_wgrad(x: torch.Tensor, dy: torch.Tensor, w_shape: List[int], k: int, stride: int, pad: int,
                 transposed: bool, upsample: int) -> torch.Tensor:
    return K.conv_wgrad(x, dy, _geom(k, stride, pad, transposed, upsample), tuple(w_shape))[0]


@conv2d_wgrad.register_fake
def _(x, dy, w_shape, k, stride, pad, transposed, upsample):
    return torch.empty(tuple(w_shape), dtype=torch.float32, device=x.device)


def _wgrad_setup(ctx, inputs, output):
    x, dy, w_shape, k, stride, pad, transposed, upsample = inputs
    ctx.args = (k, stride, pad, transposed, upsample)
    ctx.x_shape = tuple(x.shape)
    ctx.save_for_backward(x, dy)


def _wgrad_backward(ctx, ddw):
    x, dy = ctx.saved_tensors
    k, stride, pad, transposed, upsample = ctx.args
    ddw = ddw.contiguous()
    d_x = (torch.ops.rgan.conv2d_dgrad(dy, ddw, list(ctx.x_shape), k, stride, pad, transposed, upsample)
           if ctx.needs_input_grad[0] else None)
    d_dy = (torch.ops.rgan.conv2d(x, ddw, None, k, stride, pad, transposed, upsample, "none", 0.0, False)
            if ctx.needs_input_grad[1] else None)
    return d_x, d_dy, None, None, None, None, None, None


conv2d_wgrad.register_autograd(_wgrad_backward, setup_context=_wgrad_setup)


@torch.library.custom_op("rgan::channel_sum", mutates_args=(), device_types=_DEV)
def channel_sum(t: torch.Tensor) -> torch.Tensor:
    """sum over (b, h, w) per channel of an NHWC tensor (a conv bias gradient)."""
    if not K.is_nhwc(t):
        t = t.contiguous(memory_format=torch.channels_last)
    return K.channel_sum(t, torch.empty(t.shape[1], dtype=torch.float32, device=t.device))


@channel_sum.register_fake
def _(t):
    return torch.empty(t.shape[1], dtype=torch.float32, device=t.device)


def _no_double(name):
    def bwd(ctx, *g):
        raise NotImplementedError(f"rgan::{name}: no derivative registered (second order: gp.py's native engine)")
    return bwd


channel_sum.register_autograd(_no_double("channel_sum"), setup_context=lambda ctx, inputs, output: None)


@torch.library.custom_op("rgan::act_backward", mutates_args=(), device_types=_DEV)
def act_backward(g: torch.Tensor, a: torch.Tensor, act: str, alpha: float) -> torch.Tensor:
    """g * act'(x), act' read from the activation output a (g gets a's strides)."""
    if g.stride() != a.stride():
        g = g.contiguous(memory_format=torch.channels_last) if K.is_nhwc(a) else g.contiguous()
    return K.act_backward(g, a, act, alpha)


@act_backward.register_fake
def _(g, a, act, alpha):
    return torch.empty_like(a)


def _actb_setup(ctx, inputs, output):
    g, a, act, alpha = inputs
    ctx.act, ctx.alpha = act, alpha
    ctx.save_for_backward(a)


def _actb_backward(ctx, gg):
    a, = ctx.saved_tensors
    if ctx.needs_input_grad[1] and ctx.act not in _PL_ACTS:
        raise NotImplementedError(f"rgan::act_backward: d/da of {ctx.act} (act'') is gp.py's native engine")
    d_g = torch.ops.rgan.act_backward(gg, a, ctx.act, ctx.alpha) if ctx.needs_input_grad[0] else None
    # piecewise-linear activations: act' is constant away from the kink, d/da = 0
    d_a = torch.zeros_like(a) if ctx.needs_input_grad[1] else None
    return d_g, d_a, None, None


act_backward.register_autograd(_actb_backward, setup_context=_actb_setup)


# ------------------------------------------------------------------ BatchNorm (train mode)
# A mutating operator cannot carry an autograd formula, so train-mode BatchNorm is two ops:
# batch_norm_stats_ (the batch statistics; updates the running statistics in place) and the
# functional batch_norm_apply, whose derivative is train-mode BatchNorm's -- it treats ``stats``
# as the batch statistics of ``y`` (what batch_norm_stats_ returned for it), as torch does.
@torch.library.custom_op("rgan::batch_norm_stats_",
                         mutates_args=("running_mean", "running_var", "num_batches_tracked"), device_types=_DEV)
def batch_norm_stats_(y: torch.Tensor, running_mean: torch.Tensor, running_var: torch.Tensor,
                      num_batches_tracked: torch.Tensor, eps: float, momentum: float) -> torch.Tensor:
    """[mean; invstd] (float[2C]) of y over (b, h, w); running statistics updated as torch's
    train-mode BatchNorm2d does (unbiased variance, momentum, num_batches_tracked += 1)."""
    if not K.is_nhwc(y):
        y = y.contiguous(memory_format=torch.channels_last)
    return K.bn_stats(y, eps, momentum, running_mean, running_var, num_batches_tracked)


@batch_norm_stats_.register_fake
def _(y, running_mean, running_var, num_batches_tracked, eps, momentum):
    return torch.empty(2 * y.shape[1], dtype=torch.float32, device=y.device)


@torch.library.custom_op("rgan::batch_norm_apply", mutates_args=(), device_types=_DEV)
def batch_norm_apply(y: torch.Tensor, stats: torch.Tensor, gamma: Optional[torch.Tensor],
                     beta: Optional[torch.Tensor], act: str, alpha: float) -> torch.Tensor:
    """act(gamma * (y - mean) * invstd + beta), NHWC."""
    if not K.is_nhwc(y):
        y = y.contiguous(memory_format=torch.channels_last)
    return K.bn_apply(y, stats, gamma, beta, act, alpha)


@batch_norm_apply.register_fake
def _(y, stats, gamma, beta, act, alpha):
    return _nhwc_like(tuple(y.shape), y.device)


def _bn_setup(ctx, inputs, output):
    y, stats, gamma, beta, act, alpha = inputs
    ctx.act, ctx.alpha = act, alpha
    ctx.save_for_backward(y, stats, gamma, beta)


def _bn_backward(ctx, da):
    y, stats, gamma, beta = ctx.saved_tensors
    dy, dgamma, dbeta = torch.ops.rgan.batch_norm_backward(da, y, stats, gamma, beta, ctx.act, ctx.alpha)
    ng, nb = ctx.needs_input_grad[2:4]
    return dy, None, (dgamma if ng else None), (dbeta if nb else None), None, None


batch_norm_apply.register_autograd(_bn_backward, setup_context=_bn_setup)


@torch.library.custom_op("rgan::batch_norm_backward", mutates_args=(), device_types=_DEV)
def batch_norm_backward(da: torch.Tensor, y: torch.Tensor, stats: torch.Tensor, gamma: Optional[torch.Tensor],
                        beta: Optional[torch.Tensor], act: str, alpha: float
                        ) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
    if not K.is_nhwc(y):
        y = y.contiguous(memory_format=torch.channels_last)
    dy, dg, db = K.bn_backward(da, y, stats, gamma, beta, act, alpha, need_affine=True)
    C = y.shape[1]
    dg = dg if dg is not None else torch.zeros(C, dtype=torch.float32, device=y.device)
    db = db if db is not None else torch.zeros(C, dtype=torch.float32, device=y.device)
    return dy, dg, db


@batch_norm_backward.register_fake
def _(da, y, stats, gamma, beta, act, alpha):
    C = y.shape[1]
    return (_nhwc_like(tuple(y.shape), y.device), torch.empty(C, dtype=torch.float32, device=y.device),
            torch.empty(C, dtype=torch.float32, device=y.device))


batch_norm_backward.register_autograd(_no_double("batch_norm_backward"),
                                      setup_context=lambda ctx, inputs, output: None)


# ------------------------------------------------------------------ spectral norm
# spectral_power_ (mutating: u, v updated in place, returns their copies and 1/sigma) and the
# functional spectral_scale (W / sigma with u, v constant -- torch spectral_norm's autograd).
@torch.library.custom_op("rgan::spectral_power_", mutates_args=("u", "v"), device_types=_DEV)
def spectral_power_(w: torch.Tensor, u: torch.Tensor, v: torch.Tensor, transposed: bool, eps: float,
                    do_iter: bool) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
    """One power iteration (train mode: do_iter) of torch spectral_norm's forward pre-hook,
    dim 1 for ConvTranspose2d: (u copy, v copy, 1 / sigma)."""
    inv = K.spectral_power(w, u, v, transposed, eps=eps, do_iter=do_iter)
    return u.clone(), v.clone(), inv


@spectral_power_.register_fake
def _(w, u, v, transposed, eps, do_iter):
    return torch.empty_like(u), torch.empty_like(v), torch.empty(1, dtype=torch.float32, device=w.device)


@torch.library.custom_op("rgan::spectral_scale", mutates_args=(), device_types=_DEV)
def spectral_scale(w: torch.Tensor, u: torch.Tensor, v: torch.Tensor, inv_sigma: torch.Tensor,
                   transposed: bool) -> torch.Tensor:
    """W * (1 / sigma)."""
    return K.scale(w.contiguous(), inv_sigma)


@spectral_scale.register_fake
def _(w, u, v, inv_sigma, transposed):
    return torch.empty_like(w, memory_format=torch.contiguous_format)


def _sn_setup(ctx, inputs, output):
    w, u, v, inv, transposed = inputs
    ctx.transposed = transposed
    ctx.save_for_backward(w, u, v, inv)


def _sn_backward(ctx, dw_eff):
    w, u, v, inv = ctx.saved_tensors
    dw = torch.ops.rgan.spectral_backward(w, dw_eff.contiguous(), u, v, inv, ctx.transposed)
    return dw, None, None, None, None


spectral_scale.register_autograd(_sn_backward, setup_context=_sn_setup)


@torch.library.custom_op("rgan::spectral_backward", mutates_args=(), device_types=_DEV)
def spectral_backward(w: torch.Tensor, dw_eff: torch.Tensor, u: torch.Tensor, v: torch.Tensor,
                      inv_sigma: torch.Tensor, transposed: bool) -> torch.Tensor:
    """dW_orig of W_eff = W / sigma(W) with u, v constant (torch spectral_norm's autograd)."""
    return K.spectral_backward(w, dw_eff, u, v, inv_sigma, transposed)


@spectral_backward.register_fake
def _(w, dw_eff, u, v, inv_sigma, transposed):
    return torch.empty_like(w)


spectral_backward.register_autograd(_no_double("spectral_backward"), setup_context=lambda ctx, inputs, output: None)


# ------------------------------------------------------------------ loss heads / penalty
@torch.library.custom_op("rgan::loss_head", mutates_args=(), device_types=_DEV)
def loss_head(kind: int, side: int, r: Optional[torch.Tensor], f: Optional[torch.Tensor]) -> torch.Tensor:
    """The --loss_D head (1-8) on D's outputs: side 0 = D (heads 5-8) / D-real (1-4), 1 =
    D-fake (1-4), 2 = G (include/rgan.h rgan_loss_head)."""
    loss, _, _ = K.loss_head(kind, side, r, f, need_dr=False, need_df=False)
    return loss


@loss_head.register_fake
def _(kind, side, r, f):
    t = r if r is not None else f
    return torch.empty((), dtype=torch.float32, device=t.device)


def _head_setup(ctx, inputs, output):
    kind, side, r, f = inputs
    ctx.kind, ctx.side = kind, side
    ctx.save_for_backward(r, f)


def _head_backward(ctx, g):
    r, f = ctx.saved_tensors
    dr, df = torch.ops.rgan.loss_head_grad(ctx.kind, ctx.side, r, f, g)
    return None, None, (dr if r is not None and ctx.needs_input_grad[2] else None), \
        (df if f is not None and ctx.needs_input_grad[3] else None)


loss_head.register_autograd(_head_backward, setup_context=_head_setup)


@torch.library.custom_op("rgan::loss_head_grad", mutates_args=(), device_types=_DEV)
def loss_head_grad(kind: int, side: int, r: Optional[torch.Tensor], f: Optional[torch.Tensor],
                   g: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
    """(g * d loss / d r, g * d loss / d f); an absent input's gradient is an empty tensor."""
    _, dr, df = K.loss_head(kind, side, r, f, need_dr=r is not None, need_df=f is not None)
    g = g.reshape(1).contiguous()
    e = torch.empty(0, dtype=torch.float32, device=g.device)
    return (K.scale(dr, g) if dr is not None else e), (K.scale(df, g) if df is not None else e)


@loss_head_grad.register_fake
def _(kind, side, r, f, g):
    e = torch.empty(0, dtype=torch.float32, device=g.device)
    return (torch.empty_like(r) if r is not None else e), (torch.empty_like(f) if f is not None else e)


loss_head_grad.register_autograd(_no_double("loss_head_grad"), setup_context=lambda ctx, inputs, output: None)


@torch.library.custom_op("rgan::gp_penalty", mutates_args=(), device_types=_DEV)
def gp_penalty(g: torch.Tensor, lam: float, n_global: int) -> Tuple[torch.Tensor, torch.Tensor]:
    """(lam * mean_b (||g_b||_2 - 1)^2 over n_global samples, the per-sample norms)."""
    loss, norms, _ = K.gp_penalty(g, lam, n_global)
    return loss, norms


@gp_penalty.register_fake
def _(g, lam, n_global):
    return torch.empty((), dtype=torch.float32, device=g.device), torch.empty(g.shape[0], dtype=torch.float32,
                                                                              device=g.device)


def _gp_setup(ctx, inputs, output):
    g, lam, n_global = inputs
    ctx.lam, ctx.n_global = lam, n_global
    ctx.save_for_backward(g, output[1])


def _gp_backward(ctx, gl, gnorms):
    g, norms = ctx.saved_tensors
    return torch.ops.rgan.gp_penalty_backward(g, norms, ctx.lam, ctx.n_global, gl), None, None


gp_penalty.register_autograd(_gp_backward, setup_context=_gp_setup)


@torch.library.custom_op("rgan::gp_penalty_backward", mutates_args=(), device_types=_DEV)
def gp_penalty_backward(g: torch.Tensor, norms: torch.Tensor, lam: float, n_global: int,
                        gl: torch.Tensor) -> torch.Tensor:
    return K.gp_penalty_backward(g.contiguous(), norms, lam, n_global, gl.reshape(1).contiguous())


@gp_penalty_backward.register_fake
def _(g, norms, lam, n_global, gl):
    return torch.empty(g.shape, dtype=torch.float32, device=g.device)


gp_penalty_backward.register_autograd(_no_double("gp_penalty_backward"),
                                      setup_context=lambda ctx, inputs, output: None)


# ------------------------------------------------------------------ optimizer
@torch.library.custom_op("rgan::adam_", mutates_args=("params", "exp_avgs", "exp_avg_sqs", "step"),
                         device_types=_DEV)
def adam_(params: List[torch.Tensor], grads: List[torch.Tensor], exp_avgs: List[torch.Tensor],
          exp_avg_sqs: List[torch.Tensor], hyper: torch.Tensor, step: torch.Tensor) -> None:
    """torch.optim.Adam's step over the tensors (hyper = double[8] {lr, beta1, beta2, eps,
    weight_decay, 0, 0, 0}, step = float[1] incremented first; include/rgan.h rgan_adam)."""
    K.adam(params, grads, exp_avgs, exp_avg_sqs, hyper, step)


@adam_.register_fake
def _(params, grads, exp_avgs, exp_avg_sqs, hyper, step):
    return None


# ------------------------------------------------------------------ traced layers (nets)
def tracing(t):
    """A trace (torch.export / torch.compile / fake-tensor propagation) rather than a run."""
    from torch._subclasses.fake_tensor import FakeTensor
    return (isinstance(t, FakeTensor) or torch.compiler.is_compiling()
            or getattr(torch.compiler, "is_exporting", lambda: False)())


def layer_forward(layer, h, training):
    """One nets._Layer as rgan:: ops (unfused: conv, then BatchNorm + act), for traces."""
    conv, bn, spec = layer.conv, layer.bn, layer.spec
    w = layer.weight()
    geom = spec.geom
    if spec.spectral:
        u, v, inv = torch.ops.rgan.spectral_power_(w.detach(), conv.weight_u, conv.weight_v, geom.transposed, 1e-12,
                                                   training)
        w = torch.ops.rgan.spectral_scale(w, u, v, inv, geom.transposed)
    if bn is not None:
        if not training:
            raise NotImplementedError("rgan:: ops: eval-mode BatchNorm is not on the reference's path (GLI:560-714)")
        y = torch.ops.rgan.conv2d(h, w, conv.bias, geom.k, geom.stride, geom.pad, geom.transposed, geom.upsample,
                                  "none", 0.0, False)
        stats = torch.ops.rgan.batch_norm_stats_(y.detach(), bn.running_mean, bn.running_var, bn.num_batches_tracked,
                                                 spec.eps, spec.momentum)
        return torch.ops.rgan.batch_norm_apply(y, stats, bn.weight, bn.bias, spec.act, spec.alpha)
    return torch.ops.rgan.conv2d(h, w, conv.bias, geom.k, geom.stride, geom.pad, geom.transposed, geom.upsample,
                                 spec.act, spec.alpha, spec.nchw_out)


OPS = ("conv2d", "conv2d_dgrad", "conv2d_wgrad", "channel_sum", "act_backward", "batch_norm_stats_",
       "batch_norm_apply", "batch_norm_backward", "spectral_power_", "spectral_scale", "spectral_backward", "loss_head",
       "loss_head_grad", "gp_penalty", "gp_penalty_backward", "adam_")
