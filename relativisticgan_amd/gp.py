"""WGAN-GP on the HIP kernels: the penalty and its double backward (GLI:646-658).

The reference builds the penalty with autograd:

    x_both = x*u + x_fake*(1-u);  g = autograd.grad(D(x_both), x_both, ones, create_graph=True)
    gp = penalty * mean((||g||_2 - 1)^2);  gp.backward()

i.e. a forward pass of D, its backward as a differentiable graph, and a backward through
that graph.  Here the three sweeps are explicit, with every tensor they need saved once
(no re-run of any forward, no autograd re-tracing, no ATen arithmetic):

forward   h_l = act(BN(conv(h_{l-1}, W_l)))  (train-mode BN: running stats move, one more
          spectral power iteration -- exactly as the reference's D(x_both) call)
backward  dy_l = BNback(dh_l act'),  dh_{l-1} = dgrad(dy_l, W_l),  g = dh_0 (image)
penalty   gp, norms = rgan_gp_penalty(g)

and, when gp.backward() runs (GLI:658), with v = dgp/dg:

sweep 1 (up, through the backward chain; ubar_l = dP/d(dh_l), ubar_0 = v):
          a_l = conv(ubar_{l-1}, W_l)                 adjoint of dgrad's dy input
          ubar_l, ydir_l, dgamma2, dbeta2 = rgan_bn_dd_apply(a_l, ...)   (BN layers) or
          rgan_act_dd (no BN): the adjoint through BN-backward/act', plus the DIRECT
          dP/dy_l of the forward activations (bn_act.hip documents the algebra)
sweep 2 (down, through the forward chain; gbar_l = dP/dh_l):
          ybar_l = BNback(gbar_l act') + ydir_l        (rgan_bn_backward_apply_ex add=)
          dW_l  += wgrad([ubar_{l-1}; h_{l-1}], [dy_l; ybar_l])   ONE K-doubled GEMM: the
                   dgrad op's weight adjoint and the forward's weight gradient share it
          gbar_{l-1} = dgrad(ybar_l, W_l)

Every weight/affine gradient is ADDED into the existing .grad in the kernels' epilogues
(the errD backward has already filled them), so the step needs no add pass either.
The [adjoint; forward] operand pairs live in one [2B, ...] buffer per layer, written in
place by the producing kernels (no concatenation copies).  Cost: 6 D-forward-equivalents
of MFMA work, the minimum the algebra allows.

SyncBN (--rgan_sync_bn True): every BatchNorm sum of the three sweeps (the first
backward's, the double backward's stage-1 / stage-2 sums, sweep 2's) is all-reduced before
it normalises anything and the kernels get the global pixel count, while the affine
gradients come from the rank's own (pre-all-reduce) sums -- the bucketed gradient
all-reduce then sums them like every other gradient (include/rgan.h rgan_bn_dd_apply's
*_local sums, rgan_bn_affine_grads).  No ATen arithmetic under either BatchNorm mode.
"""
import torch

from . import autograd as AG
from . import dp
from . import kernels as K
from .kernels import ACT_HAS_GRAD2, empty_nhwc

_ONES = {}


def _ones(shape, device):
    """A cached all-ones upstream gradient (grad_outputs=ones, GLI:654)."""
    key = (tuple(shape), str(device))
    t = _ONES.get(key)
    if t is None:
        t = _ONES[key] = torch.ones(shape, dtype=torch.float32, device=device)
    return t


def _grad_buf(p):
    """p.grad to accumulate into (created when the first-order backward left none)."""
    if p.grad is None:
        p.grad = torch.zeros_like(p)
    return p.grad


class _Rec:
    __slots__ = ("layer", "spec", "w", "wparam", "bias", "gamma", "beta", "wscale", "sn", "xc", "h_in", "y",
                 "a", "stats", "dh", "dy", "yc", "fs")


def supported(D):
    """The native engine covers every D of the reference (arch 0/1, spectral, BN, any
    activation), with per-shard BatchNorm or SyncBN."""
    return True


def _global(sums):
    """(global sums, local sums): the SyncBN all-reduce of a rank's BatchNorm sums (a copy;
    the local ones give the affine gradients), or the sums themselves."""
    if not dp.sync_bn():
        return sums, sums
    return dp.all_reduce_sum(sums.clone()), sums


class GPEngine:
    def __init__(self, D, x, x_fake, u, penalty):
        self.D, self.lam = D, float(penalty)
        self.B = x.shape[0]
        self.n_global = self.B * dp.world()
        self.dev = x.device
        B = self.B
        # [adjoint; forward] image pair: v (the penalty's gradient) | x_hat
        self.img = torch.empty((2 * B,) + tuple(x.shape[1:]), dtype=torch.float32, device=self.dev)
        self.x_hat = K.gp_interp(x.detach(), x_fake.detach(), u.detach(), out=self.img[B:])
        self._forward()
        self._first_backward()
        self.gp, self.norms, _ = K.gp_penalty(self.g, self.lam, self.n_global)

    # ------------------------------------------------------------ forward
    def _forward(self):
        D, B = self.D, self.B
        self.recs = []
        h, xc = self.x_hat, self.img
        AG.TRACE_NET = "D"
        plan = D._plan
        sns = D._spectral()  # one power iteration per spectral layer, as the reference's D(x_both)
        for li, layer in enumerate(plan):
            AG.TRACE_LAYER = li
            r = _Rec()
            conv, bn, spec = layer.conv, layer.bn, layer.spec
            r.layer, r.spec = layer, spec
            r.wparam = conv.w if hasattr(conv, "w") else conv.weight
            r.w = r.wparam.view(*layer.w_view) if layer.w_view is not None else r.wparam
            r.bias = conv.bias
            r.gamma = bn.weight if bn is not None else None
            r.beta = bn.bias if bn is not None else None
            if layer.in_view is not None:
                raise NotImplementedError("GP engine: reshaping D layers")
            r.sn = sns.get(li)
            r.wscale = r.sn[2] if r.sn is not None else None
            r.xc, r.h_in = xc, h
            last = li == len(plan) - 1
            cout = r.w.shape[1] if spec.geom.transposed else r.w.shape[0]
            Ho, Wo = spec.geom.out_hw(h.shape[2], h.shape[3])
            if last:
                xc_next, out = None, empty_nhwc(B, cout, Ho, Wo, self.dev)
            else:
                xc_next = empty_nhwc(2 * B, cout, Ho, Wo, self.dev)
                out = xc_next[B:]
            w = r.w  # the parameter (or its view) itself: the pack cache is keyed by the weight's base
            if spec.bn:
                y, part, S = K.conv_fwd_bn(h, w, spec.geom, bias=r.bias, wscale=r.wscale, cache=True)
                r.y = y
                if part is not None and not dp.sync_bn() and y.shape[1] % 4 == 0 and out.data_ptr() % 16 == 0:
                    # statistics + normalisation in one call (one launch for small layers)
                    r.stats = torch.empty(2 * y.shape[1], dtype=torch.float32, device=self.dev)
                    r.a = K.bn_segment_apply(part, S, y, spec.eps, spec.momentum, bn.running_mean, bn.running_var,
                                             bn.num_batches_tracked, r.gamma, r.beta, spec.act, spec.alpha,
                                             r.stats.view(1, -1), out)
                else:
                    r.stats = AG._train_stats(y, spec, bn.running_mean, bn.running_var, bn.num_batches_tracked,
                                              (part, 0, S) if part is not None else None)
                    r.a = K.bn_apply(y, r.stats, r.gamma, r.beta, spec.act, spec.alpha, out=out)
            else:
                r.y, r.stats = None, None
                r.a = K.conv_fwd(h, w, spec.geom, bias=r.bias, act=spec.act, alpha=spec.alpha, wscale=r.wscale,
                                 out=out, cache=True)
            if AG.ACT_TRACE is not None and spec.act in AG._KINKED:
                AG.ACT_TRACE.append((r.a > 0).cpu())
                AG.ACT_TAGS.append("D")
                AG.ACT_LAYERS.append(li)
            self.recs.append(r)
            h, xc = r.a, xc_next
        self.out = h

    # ------------------------------------------------------------ create-graph backward (values)
    def _first_backward(self):
        B, recs = self.B, self.recs
        dh = _ones(self.out.shape, self.dev)
        for li in range(len(recs) - 1, -1, -1):
            r = recs[li]
            spec = r.spec
            r.dh = dh
            r.yc = None
            if spec.bn or spec.act != "none":
                C, Ho, Wo = r.a.shape[1], r.a.shape[2], r.a.shape[3]
                r.yc = empty_nhwc(2 * B, C, Ho, Wo, self.dev)
            if spec.bn and not dp.sync_bn():
                # sums (kept for the double backward) + apply in one call
                r.fs, r.dy = K.bn_backward_sums_apply(dh, r.y, r.stats, r.gamma, r.beta, spec.act, spec.alpha,
                                                      out=r.yc[:B])
            elif spec.bn:
                fs, dh_c = K.bn_backward_sums(dh, r.y, r.stats, r.gamma, r.beta, spec.act, spec.alpha)
                r.fs, _ = _global(fs)
                r.dy, _, _ = K.bn_backward_apply(dh_c, r.y, r.stats, r.gamma, r.beta, spec.act, spec.alpha, r.fs,
                                                 self._P(r), need_affine=False, out=r.yc[:B])
            elif spec.act != "none":
                r.fs = None
                r.dy = K.act_backward_ex(dh, r.a, spec.act, spec.alpha, out=r.yc[:B])
            else:
                r.fs, r.dy = None, dh
            dh = K.conv_dgrad(r.dy, r.w, spec.geom, tuple(r.h_in.shape), wscale=r.wscale, like=r.h_in,
                              cache=True, out=(r.xc[:B] if li == 0 else None))
        self.g = dh  # dD(x_hat)/dx_hat, in the image pair's first half (backward() overwrites it with v)

    # ------------------------------------------------------------ gp.backward()
    def backward(self, dgp):
        B, recs = self.B, self.recs
        # v = dP/dg, in place over g in the image pair's first half (the penalty kept its norms)
        ubar = K.gp_penalty_backward(self.g, self.norms, self.lam, self.n_global, dgp.contiguous(), out=self.img[:B])
        ydirs = [None] * len(recs)
        # sweep 1: up through the backward chain
        for li, r in enumerate(recs):
            spec = r.spec
            last = li == len(recs) - 1
            has2 = ACT_HAS_GRAD2[spec.act]
            if last and not spec.bn and not has2:
                break  # dy_L = dh_L act' with dh_L = ones and act'' = 0: no adjoint flows on
            nxt = None if last else recs[li + 1].xc[:B]
            w = r.w
            if spec.bn:
                a_adj = K.conv_fwd(ubar, w, spec.geom, wscale=r.wscale, cache=True)
                P = self._P(r)
                s1, s1_loc = _global(K.bn_dd_sums(a_adj, r.y, r.dh, r.stats, r.gamma, r.beta, spec.act, spec.alpha, 1))
                s2, s2_loc = (_global(K.bn_dd_sums(a_adj, r.y, r.dh, r.stats, r.gamma, r.beta, spec.act, spec.alpha,
                                                   2, s1, P)) if has2 else (None, None))
                sync = dp.sync_bn()
                adj, ydir = K.bn_dd_apply(a_adj, r.y, r.dh, r.stats, r.gamma, r.beta, spec.act, spec.alpha, r.fs,
                                          s1, s2, P, s1_local=s1_loc if sync else None,
                                          s2_local=s2_loc if sync else None, adj_dh=nxt, ydir=r.yc[B:],
                                          need_adj=not last,
                                          dgamma2=_grad_buf(r.gamma) if r.gamma is not None else None,
                                          dbeta2=_grad_buf(r.beta) if r.beta is not None else None,
                                          accumulate_affine=True)
            elif spec.act != "none":
                a_adj = K.conv_fwd(ubar, w, spec.geom, wscale=r.wscale, cache=True)
                adj, ydir = K.act_dd(a_adj, r.a, r.dh, spec.act, spec.alpha, need_adj=not last, need_ydir=has2,
                                     adj_dh=nxt, ydir=r.yc[B:] if has2 else None)
            else:  # linear layer without BN: the adjoint passes straight through
                adj = K.conv_fwd(ubar, w, spec.geom, wscale=r.wscale, cache=True, out=nxt)
                ydir = None
            ydirs[li] = ydir
            ubar = adj
        # sweep 2: down through the forward chain
        gbar = None
        for li in range(len(recs) - 1, -1, -1):
            r = recs[li]
            spec = r.spec
            ydir = ydirs[li]
            ybar = None
            if gbar is not None:
                if spec.bn and not dp.sync_bn():
                    # BN backward of gbar + the double backward's direct term, one call
                    _, ybar = K.bn_backward_sums_apply(gbar, r.y, r.stats, r.gamma, r.beta, spec.act, spec.alpha,
                                                       add=ydir, out=r.yc[B:],
                                                       dgamma=_grad_buf(r.gamma) if r.gamma is not None else None,
                                                       dbeta=_grad_buf(r.beta) if r.beta is not None else None,
                                                       accumulate_affine=True)
                elif spec.bn:
                    sums, g_c = K.bn_backward_sums(gbar, r.y, r.stats, r.gamma, r.beta, spec.act, spec.alpha)
                    sums, sums_loc = _global(sums)
                    dgb = _grad_buf(r.gamma) if r.gamma is not None else None
                    dbb = _grad_buf(r.beta) if r.beta is not None else None
                    sync = dp.sync_bn()
                    ybar = K.bn_backward_apply_ex(g_c, r.y, r.stats, r.gamma, r.beta, spec.act, spec.alpha, sums,
                                                  self._P(r), add=ydir, out=r.yc[B:],
                                                  dgamma=None if sync else dgb, dbeta=None if sync else dbb,
                                                  accumulate_affine=True)
                    if sync:  # the affine gradients from this rank's own sums
                        K.bn_affine_grads(sums_loc, r.stats, r.y.shape[1], dgb, dbb, accumulate=True)
                elif spec.act != "none":
                    ybar = K.act_backward_ex(gbar, r.a, spec.act, spec.alpha, add=ydir, out=r.yc[B:])
                else:
                    raise NotImplementedError("GP engine: a linear layer below another layer")
            elif ydir is not None:
                ybar = ydir  # already in the pair buffer's second half
            self._weight_grad(li, r, ybar)
            gbar = (K.conv_dgrad(ybar, r.w, spec.geom, tuple(r.h_in.shape), wscale=r.wscale,
                                 like=r.h_in, cache=True) if (ybar is not None and li > 0) else None)

    @staticmethod
    def _P(r):
        """Pixels per channel the layer's BatchNorm normalises over: the rank's shard, or the
        global batch under SyncBN."""
        P = r.y.shape[0] * r.y.shape[2] * r.y.shape[3]
        return P * dp.world() if dp.sync_bn() else P

    def _weight_grad(self, li, r, ybar):
        """dW_l += wgrad(ubar_{l-1}, dy_l) [+ wgrad(h_{l-1}, ybar_l)] as one GEMM over the pair
        buffers; bias += sum(ybar_l) (the dgrad op does not see the bias)."""
        B, spec = self.B, r.spec
        if ybar is not None:
            X, Y = r.xc, r.yc
        else:
            X, Y = r.xc[:B], (r.yc[:B] if r.yc is not None else r.dy)
        gw = _grad_buf(r.wparam)
        gw = gw.view(*r.layer.w_view) if r.layer.w_view is not None else gw
        sn = r.sn
        bias_on = r.bias is not None and ybar is not None
        if sn is None and bias_on and not AG.ConvLayerFn._patch_conv(spec, r.h_in):
            # bias += sum(ybar): the forward half's rows of the pair -- summed by the weight
            # gradient GEMM itself from the staged rows >= B * Ho * Wo (rgan_conv_wgrad_rows)
            K.conv_wgrad(X, Y, spec.geom, tuple(r.w.shape), out=gw, with_bias=True, out_bias=_grad_buf(r.bias),
                         bias_row0=B * Y.shape[2] * Y.shape[3])
            return
        if AG.ConvLayerFn._patch_conv(spec, r.h_in):
            g1, _ = K.conv_wgrad(K.patches_k4s2(X), Y, K.G1X1, (r.w.shape[0], 64, 1, 1))
            if sn is None:
                K.unpatch_grad(g1, r.w.shape[0], r.w.shape[1], 64, 1, out=gw)
            else:
                K.spectral_backward(r.w.detach(), K.unpatch_grad(g1, r.w.shape[0], r.w.shape[1], 64, 1), sn[0],
                                    sn[1], sn[2], spec.geom.transposed, out=gw)
        elif sn is None:
            K.conv_wgrad(X, Y, spec.geom, tuple(r.w.shape), out=gw)
        else:
            dw_eff, _ = K.conv_wgrad(X, Y, spec.geom, tuple(r.w.shape))
            K.spectral_backward(r.w.detach(), dw_eff, sn[0], sn[1], sn[2], spec.geom.transposed, out=gw)
        if r.bias is not None and ybar is not None:
            K.channel_sum(ybar, _grad_buf(r.bias), accumulate=True)


class _GPFn(torch.autograd.Function):
    """gp with a backward node: gp.backward() (GLI:658) runs the engine's double backward,
    which adds straight into D's .grad tensors (nothing is returned through autograd)."""

    @staticmethod
    def forward(ctx, engine, anchor):
        ctx.engine = engine
        return engine.gp

    @staticmethod
    def backward(ctx, dgp):
        ctx.engine.backward(dgp)
        ctx.engine = None
        return None, None


def gradient_penalty(D, x, x_fake, u, penalty):
    """penalty * mean((||dD(x_hat)/dx_hat||_2 - 1)^2), x_hat = x*u + x_fake*(1-u) (GLI:648-657)."""
    eng = GPEngine(D, x, x_fake, u, penalty)
    anchor = next(p for p in D.parameters() if p.requires_grad)
    return _GPFn.apply(eng, anchor)
