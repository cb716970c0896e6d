"""The eight --loss_D heads and the WGAN-GP penalty as autograd ops on the HIP kernels.

Heads (GLI:481-484 criteria; D side GLI:592-644; G side GLI:686-709):
  1 SGAN (BCE on D's sigmoid), 2 LSGAN, 3 WGAN(-GP), 4 HingeGAN: real and fake terms
  are separate losses backpropagated separately (GLI:605, 624), G loss per GLI:686-693;
  5 RSGAN, 6 RaSGAN, 7 RaLSGAN, 8 RaHingeGAN: one loss over (y_pred, y_pred_fake).
Each head is ONE kernel launch computing the loss and both input gradients; the
backward only scales them by the upstream gradient.  Under data parallelism the
batch means are global: the head runs in three phases with two tiny
all-reduces in between.
"""
import weakref

import torch

from . import dp
from . import kernels as K


# data_ptr -> tensor: device scalars 1.0 used as backward seeds (Trainer._backward); weak, so a
# dead seed's entry goes with it (its address may be reused by another tensor)
_UNIT_SEEDS = weakref.WeakValueDictionary()


def unit_seed(device, dtype=torch.float32):
    """A device scalar 1.0 for ``loss.backward(seed)``: the heads' backward recognises it and
    hands its saved gradients on as they are (x * 1.0 == x: no scale launch)."""
    one = torch.ones((), dtype=dtype, device=device)
    _UNIT_SEEDS[one.data_ptr()] = one
    return one


def _is_unit(g):
    u = _UNIT_SEEDS.get(g.data_ptr())
    return u is not None and g.numel() == 1 and g.dtype == u.dtype and g.device == u.device


def _times(t, g):
    """t * g (g the upstream scalar gradient)."""
    if t is None:
        return None
    return t if _is_unit(g) else K.scale(t, g.contiguous())


class _Head(torch.autograd.Function):
    @staticmethod
    def forward(ctx, r, f, kind, side):
        need_r = r is not None and ctx.needs_input_grad[0]
        need_f = f is not None and ctx.needs_input_grad[1]
        if dp.active():
            loss, dr, df = _head_dist(kind, side, r, f, need_r, need_f)
        else:
            loss, dr, df = K.loss_head(kind, side, r, f, need_dr=need_r, need_df=need_f)
        ctx.save_for_backward(dr, df)
        return loss

    @staticmethod
    def backward(ctx, g):
        dr, df = ctx.saved_tensors
        return _times(dr, g), _times(df, g), None, None


def _head_dist(kind, side, r, f, need_r, need_f):
    t = r if r is not None else f
    n_global = t.numel() * dp.world()
    if kind >= 6:
        s0, _, _, _ = K.loss_head_dist(kind, side, 0, r, f, n_global)
        g = dp.all_reduce_sum(s0[:2].clone())
        s1, _, _, _ = K.loss_head_dist(kind, side, 1, r, f, n_global, gsum=g)
        g6 = torch.cat([g, dp.all_reduce_sum(s1.clone())])
        _, loss, dr, df = K.loss_head_dist(kind, side, 2, r, f, n_global, gsum=g6, need_dr=need_r, need_df=need_f)
    else:
        s0, _, _, _ = K.loss_head_dist(kind, side, 0, r, f, n_global)
        g = dp.all_reduce_sum(s0[:1].clone())
        _, loss, dr, df = K.loss_head_dist(kind, side, 2, r, f, n_global, gsum=g, need_dr=need_r, need_df=need_f)
    return loss, dr, df


def _flat(t):
    return None if t is None else t.reshape(-1)


def loss_D_real(kind, y_pred):
    """errD_real for heads 1-4 (GLI:595-604)."""
    assert 1 <= kind <= 4
    return _Head.apply(_flat(y_pred), None, kind, 0)


def loss_D_fake(kind, y_pred_fake):
    """errD_fake for heads 1-4 (GLI:614-623)."""
    assert 1 <= kind <= 4
    return _Head.apply(None, _flat(y_pred_fake), kind, 1)


class _HeadPair(torch.autograd.Function):
    """errD_real + errD_fake of heads 1-4 (GLI:595-624) as one kernel launch; returns
    (errD, errD_real, errD_fake) with errD carrying the graph."""

    @staticmethod
    def forward(ctx, r, f, kind):
        ctx.set_materialize_grads(False)
        loss3, dr, df = K.loss_head_pair(kind, r, f, need_dr=ctx.needs_input_grad[0],
                                         need_df=ctx.needs_input_grad[1])
        ctx.save_for_backward(dr, df)
        ctx.mark_non_differentiable(loss3)
        return loss3[2], loss3

    @staticmethod
    def backward(ctx, g, _g3):
        dr, df = ctx.saved_tensors
        return _times(dr, g), _times(df, g), None


def loss_D_pair(kind, y_pred, y_pred_fake):
    """(errD, errD_real, errD_fake) for heads 1-4: errD.backward() is the reference's
    errD_real.backward(); errD_fake.backward() (GLI:605, 624) accumulated."""
    assert 1 <= kind <= 4
    if dp.active():
        er, ef = loss_D_real(kind, y_pred), loss_D_fake(kind, y_pred_fake)
        return er + ef, er.detach(), ef.detach()
    err, loss3 = _HeadPair.apply(_flat(y_pred), _flat(y_pred_fake), kind)
    return err, loss3[0], loss3[1]


class _HeadCat(torch.autograd.Function):
    """The D-step loss on the batched pass's joint output y = [D(x); D(x_fake)] (one
    autograd input: the gradient is written into one [2B] buffer, no concatenation).
    Heads 1-4: errD_real + errD_fake (GLI:595-624); heads 5-8: errD (GLI:634-641)."""

    @staticmethod
    def forward(ctx, y, kind):
        ctx.set_materialize_grads(False)
        B = y.numel() // 2
        dy = torch.empty_like(y)
        if kind <= 4:
            loss3, _, _ = K.loss_head_pair(kind, y[:B], y[B:], dr=dy[:B], df=dy[B:])
            loss = loss3[2]
        else:
            loss, _, _ = K.loss_head(kind, 0, y[:B], y[B:], dr=dy[:B], df=dy[B:])
        ctx.save_for_backward(dy)
        return loss

    @staticmethod
    def backward(ctx, g):
        dy, = ctx.saved_tensors
        return _times(dy, g), None


def loss_D_cat(kind, y):
    """errD of the D step from the joint [D(x); D(x_fake)] output (single process)."""
    if dp.active():
        B = y.numel() // 2
        return (loss_D_pair(kind, y[:B], y[B:])[0] if kind <= 4 else loss_D(kind, y[:B], y[B:]))
    return _HeadCat.apply(y, kind)


class _HeadCatG(torch.autograd.Function):
    """errG of heads 5-8 (GLI:695-707) on the G step's batched output y = [D(G(z)); D(x)]:
    the gradient of the fake half, and zeros for the real half (D(x) is a no-grad constant
    there, GLI:681) -- written by the head's own launch; the batched pass's backward reads the
    fake rows only (ConvLayerFn ``gsegs``)."""

    @staticmethod
    def forward(ctx, y, kind):
        B = y.numel() // 2
        if dp.active():
            loss, _, df = _head_dist(kind, 2, y[B:], y[:B], False, True)
        else:
            loss, df = K.loss_head_joint(kind, y)  # [d errG / d D(G(z)); 0]
        ctx.save_for_backward(df)
        ctx.B = B
        return loss

    @staticmethod
    def backward(ctx, g):
        df, = ctx.saved_tensors
        B = ctx.B
        if df.numel() == 2 * B and _is_unit(g):
            return df, None
        out = torch.zeros(2 * B, dtype=df.dtype, device=df.device)
        K.scale(df[:B], g.contiguous(), out=out[:B])
        return out, None


def loss_G_cat(kind, y):
    """errG (heads 5-8) from the G step's joint [D(G(z)); D(x)] output."""
    assert 5 <= kind <= 8
    return _HeadCatG.apply(y, kind)


def loss_D(kind, y_pred, y_pred_fake):
    """errD for heads 5-8 (GLI:634-641)."""
    assert 5 <= kind <= 8
    return _Head.apply(_flat(y_pred), _flat(y_pred_fake), kind, 0)


def loss_G(kind, y_pred_fake, y_pred=None):
    """errG (GLI:686-709); y_pred (a no-grad D(x) of a fresh real batch) for heads 5-8."""
    if kind <= 4:
        return _Head.apply(None, _flat(y_pred_fake), kind, 2)
    return _Head.apply(_flat(y_pred), _flat(y_pred_fake), kind, 2)


# ---------------------------------------------------------------- gradient penalty
class _GPPenalty(torch.autograd.Function):
    @staticmethod
    def forward(ctx, g, lam, n_global):
        loss, norms, gc = K.gp_penalty(g, lam, n_global)
        ctx.lam, ctx.n_global = lam, n_global
        ctx.save_for_backward(gc, norms)
        return loss

    @staticmethod
    def backward(ctx, gl):
        gc, norms = ctx.saved_tensors
        return K.gp_penalty_backward(gc, norms, ctx.lam, ctx.n_global, gl.contiguous()), None, None


def gradient_penalty(D, x, x_fake, u, penalty):
    """penalty * mean((||dD(x_hat)/dx_hat||_2 - 1)^2), x_hat = x*u + x_fake*(1-u) (GLI:648-657).

    Native engine (gp.py): forward, create-graph backward and double backward as explicit
    kernel sweeps, with per-shard BatchNorm or SyncBN (cross-rank BN sums all-reduced).  The
    autograd composite below is the engine's test reference (tests/test_gp_gpu.py)."""
    from . import gp as _gp
    if _gp.supported(D):
        return _gp.gradient_penalty(D, x, x_fake, u, penalty)
    return gradient_penalty_composite(D, x, x_fake, u, penalty)


def gradient_penalty_composite(D, x, x_fake, u, penalty):
    """The autograd form of the penalty (create_graph through ConvLayerFn)."""
    x_both = K.gp_interp(x.detach(), x_fake.detach(), u.detach()).requires_grad_(True)
    out = D(x_both)
    grad = torch.autograd.grad(outputs=out, inputs=x_both, grad_outputs=torch.ones_like(out),
                               retain_graph=True, create_graph=True, only_inputs=True)[0]
    return _GPPenalty.apply(grad, float(penalty), x.shape[0] * dp.world())
