"""Autograd Functions over the HIP kernels.

``ConvLayerFn`` is one fused layer of the reference's Sequentials: Conv2d /
ConvTranspose2d (+bias) (+BatchNorm2d in train mode) (+activation), optionally with
spectral norm on the weight (GLI:326-452 arch 0, GLI:190-307 arch 1).  Forward:
implicit-GEMM conv with the activation fused in the epilogue (no BN) or conv -> BN
moments -> fused normalise+activation (BN).  Backward: fused act'+BN backward, conv
dgrad and wgrad GEMMs, spectral sigma correction.

Double backward (WGAN-GP, ``torch.autograd.grad(..., create_graph=True)`` at GLI:655):
when the backward itself runs with grad mode on, the layer is re-expressed with
differentiable pieces -- ``ConvPrim``/``ConvDgradPrim``/``ConvWgradPrim`` (HIP GEMMs
whose backwards are each other, so any order of derivative stays on the MFMA kernels)
plus torch tensor algebra for the per-channel BN normalisation and the activation --
and differentiated with ``torch.autograd.grad``; ``gp.backward()`` then runs through
those pieces.
"""

import torch
import torch.nn.functional as F

from . import dp
from . import kernels as K


# Test/diagnostic hook: when a list, every fused layer whose activation has a derivative
# discontinuous at 0 (ReLU, LeakyReLU, SELU) appends the sign mask of its output, in call
# order, so parity tests can count sign flips against an exact (fp64) forward.
# Image-layer gradients (k4 s2 p1, <= 4 image channels) run as 1x1 GEMMs over a patch matrix
# (kernels.patches_k4s2); the forwards keep the direct narrow kernels (as fast: both are
# bound by writing the 128-channel side).


class owning_grads:
    """Context of a ``loss.backward()`` whose weight gradients the layers may write into
    ``.grad`` themselves (train.Trainer wraps its backwards in it).  Outside it -- e.g. a
    ``torch.autograd.grad`` call, which must not touch ``.grad`` -- autograd's own
    accumulation is used."""
    active = False
    # (Round 4 also ran these weight gradients on a second stream overlapping the data-gradient
    # chain: bitwise equal and slower everywhere -- C1 -5 %, C3 -1.7 %, DESIGN §3 -- and removed
    # in round 5.)

    def __enter__(self):
        self.prev, owning_grads.active = owning_grads.active, True

    def __exit__(self, *exc):
        owning_grads.active = self.prev

ACT_TRACE = None
ACT_TAGS = []      # per ACT_TRACE entry: the net that produced it ("G" / "D", set by nets._Net)
ACT_LAYERS = []    # per ACT_TRACE entry: the layer's index in the net's plan
TRACE_NET = None
TRACE_LAYER = -1
_KINKED = ("relu", "lrelu", "selu")
_POST_ACTS = ("relu", "lrelu", "tanh", "selu")  # act' from the output (act_grad_from_out)
LINKS = True  # LayerLink hand-offs on (tools/ab_links.py measures them off in the same process)


class LayerLink:
    """Hand-off between two consecutive fused layers of one net call (nets._Net): the lower
    layer's forward records how its backward starts -- its activation (``mode`` 1), or its
    train-mode BatchNorm + activation (``mode`` 2) -- and the upper layer's backward applies
    that in the epilogue of the GEMM that produces the lower layer's output gradient
    (kernels.Post), leaving ``done`` = (gradient data_ptr, Post); the lower layer's backward
    then starts from that gradient instead of running its own pass (act_bwd_kernel /
    bn_bwd_partial).  Only within one chain: each layer output has this one consumer."""

    __slots__ = ("mode", "act", "alpha", "x", "stats", "gamma", "beta", "segs", "done")

    def __init__(self):
        self.mode = 0
        self.done = None

    def post(self, rows, gsegs):
        """The kernels.Post for the lower layer's leading ``rows`` (its ``gsegs`` of ``segs``
        batch segments), or None."""
        if self.mode == 1:
            return K.Post(1, self.act, self.alpha, self.x[:rows])
        if self.mode == 2:
            st = self.stats if self.stats.dim() == 2 else self.stats.view(1, -1)
            return K.Post(2, self.act, self.alpha, self.x[:rows], stats=st[:gsegs].contiguous(), gamma=self.gamma,
                          beta=self.beta, nseg=gsegs)
        return None


class LayerSpec:
    """Static description of one fused layer."""

    __slots__ = ("geom", "act", "alpha", "bn", "eps", "momentum", "spectral", "nchw_out")

    def __init__(self, geom, act="none", alpha=0.0, bn=False, eps=1e-5, momentum=0.1, spectral=False,
                 nchw_out=False):
        self.geom, self.act, self.alpha, self.bn = geom, act, alpha, bn
        self.eps, self.momentum, self.spectral, self.nchw_out = eps, momentum, spectral, nchw_out


# ---------------------------------------------------------------- differentiable conv primitives
class ConvPrim(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, geom):
        ctx.geom = geom
        ctx.save_for_backward(x, w)
        return K.conv_fwd(x, w, geom)

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        dx = ConvDgradPrim.apply(dy, w, ctx.geom, tuple(x.shape)) if ctx.needs_input_grad[0] else None
        dw = ConvWgradPrim.apply(x, dy, ctx.geom, tuple(w.shape)) if ctx.needs_input_grad[1] else None
        return dx, dw, None


class ConvDgradPrim(torch.autograd.Function):
    @staticmethod
    def forward(ctx, dy, w, geom, x_shape):
        ctx.geom = geom
        ctx.save_for_backward(dy, w)
        return K.conv_dgrad(dy, w, geom, x_shape)

    @staticmethod
    def backward(ctx, ddx):
        dy, w = ctx.saved_tensors
        d_dy = ConvPrim.apply(ddx, w, ctx.geom) if ctx.needs_input_grad[0] else None
        d_w = ConvWgradPrim.apply(ddx, dy, ctx.geom, tuple(w.shape)) if ctx.needs_input_grad[1] else None
        return d_dy, d_w, None, None


class ConvWgradPrim(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, dy, geom, w_shape):
        ctx.geom = geom
        ctx.save_for_backward(x, dy)
        return K.conv_wgrad(x, dy, geom, w_shape)[0]

    @staticmethod
    def backward(ctx, ddw):
        x, dy = ctx.saved_tensors
        d_x = ConvDgradPrim.apply(dy, ddw, ctx.geom, tuple(x.shape)) if ctx.needs_input_grad[0] else None
        d_dy = ConvPrim.apply(x, ddw, ctx.geom) if ctx.needs_input_grad[1] else None
        return d_x, d_dy, None, None


def _torch_act(t, act, alpha):
    if act == "relu":
        return F.relu(t)
    if act == "lrelu":
        return F.leaky_relu(t, alpha)
    if act == "tanh":
        return torch.tanh(t)
    if act == "sigmoid":
        return torch.sigmoid(t)
    if act == "selu":
        return F.selu(t)
    return t


def _sn_sigma(w, u, v, transposed):
    wm = w.permute(1, 0, 2, 3) if (transposed and w.dim() == 4) else w
    wm = wm.reshape(wm.shape[0], -1)
    return torch.dot(u, torch.mv(wm, v))


def composite_layer(x, w, bias, gamma, beta, spec, stats_mode, sn):
    """The layer as differentiable pieces (used for create_graph backward)."""
    if spec.spectral:
        u, v, _ = sn
        w = w / _sn_sigma(w, u, v, spec.geom.transposed)
    y = ConvPrim.apply(x, w, spec.geom)
    if bias is not None:
        y = y + bias.view(1, -1, 1, 1)
    if spec.bn:
        if stats_mode is None:  # train mode: batch statistics (global batch under SyncBN)
            if dp.sync_bn():
                n_loc = torch.tensor([y.shape[0] * y.shape[2] * y.shape[3]], dtype=y.dtype, device=y.device)
                s = torch.cat([y.sum((0, 2, 3)), n_loc])
                s = _AllReduceSum.apply(s)
                mean = (s[:-1] / s[-1]).view(1, -1, 1, 1)
                c = y - mean
                q = _AllReduceSum.apply(torch.cat([(c * c).sum((0, 2, 3)), n_loc]))
                var = (q[:-1] / q[-1]).view(1, -1, 1, 1)
            else:
                mean = y.mean((0, 2, 3), keepdim=True)
                c = y - mean
                var = (c * c).mean((0, 2, 3), keepdim=True)
            y = c / torch.sqrt(var + spec.eps)
        else:
            mean, invstd = stats_mode
            y = (y - mean.view(1, -1, 1, 1)) * invstd.view(1, -1, 1, 1)
        y = y * gamma.view(1, -1, 1, 1) + beta.view(1, -1, 1, 1)
    return _torch_act(y, spec.act, spec.alpha)


class _AllReduceSum(torch.autograd.Function):
    """Differentiable SUM over ranks (the backward of a sum-all-reduce is a sum-all-reduce)."""

    @staticmethod
    def forward(ctx, t):
        return dp.all_reduce_sum(t.clone())

    @staticmethod
    def backward(ctx, g):
        # itself differentiable: the WGAN-GP second backward runs through this node
        return _AllReduceSum.apply(g)


# ---------------------------------------------------------------- fused layer
def _train_stats(y, spec, rm, rv, nbt, seg=None, out=None):
    """Batch statistics of y; ``seg`` = (part, s0, s1): the conv epilogue's segment moments
    covering y (rgan_conv_fwd_bn) replace the separate moments pass over y."""
    C = y.shape[1]
    if dp.sync_bn():
        mom = K.bn_segment_moments(seg[0], seg[1], seg[2], C) if seg is not None else K.bn_moments(y)
        mom = dp.all_gather_cat(mom)
        return K.bn_finalize(mom, dp.world(), C, spec.eps, spec.momentum, rm, rv, nbt, out=out)
    if seg is not None:
        return K.bn_segment_stats(seg[0], seg[1], seg[2], C, spec.eps, spec.momentum, rm, rv, nbt, out=out)
    return K.bn_stats(y, spec.eps, spec.momentum, rm, rv, nbt, out=out)


class ConvLayerFn(torch.autograd.Function):
    """a = act(BN(conv(x, w_eff) + bias)); see module docstring.

    ``segs`` > 1: the batch holds that many equal segments which the reference runs as
    separate forward calls of the same net (D(x) and D(x_fake), GLI:580-605): one conv
    GEMM over all of them, BatchNorm statistics and running-stat updates per segment in
    segment order, one dgrad and one wgrad in the backward (the weight gradient of both
    calls in a single K-doubled GEMM instead of two GEMMs and a gradient add).
    ``gsegs`` < ``segs``: only the leading ``gsegs`` segments carry an output gradient (the
    G step's batched [D(G(z)); D(x)] pass, whose D(x) half the reference runs without a
    graph, GLI:673-707): the backward runs over those rows only, and the input gradient's
    rows of the later segments are left unwritten (nothing reads them: the layer below is
    restricted the same way, and the net's input hands only the leading rows on)."""

    @staticmethod
    def forward(ctx, x, w, bias, gamma, beta, spec, bufs, sn, segs=1, out=None, gsegs=None, link_in=None,
                link_out=None):
        # bufs = (running_mean, running_var, num_batches_tracked, training)
        # sn   = (u, v, inv_sigma) clones for spectral layers, else None
        wscale = sn[2] if spec.spectral else None
        stats_eval = None
        g1 = False
        if spec.bn:
            rm, rv, nbt, training = bufs
            g1 = (training and segs == 1 and bias is None and wscale is None and not dp.sync_bn()
                  and K.g1_ok(x, w, spec.geom))
            if g1:
                # G's first layer on its 1x1 input: conv + BatchNorm + act in one launch
                y, a, stats = K.g1_fwd_bn(x, w, gamma, beta, spec.eps, spec.momentum, rm, rv, nbt, spec.act,
                                          spec.alpha, out=out)
                part, S = None, 0
            elif training:
                y, part, S = K.conv_fwd_bn(x, w, spec.geom, bias=bias, wscale=wscale, cache=True, segs=segs)
            else:
                y, part, S = K.conv_fwd(x, w, spec.geom, bias=bias, wscale=wscale, cache=True), None, 0
            C = y.shape[1]
            # statistics from the epilogue's segment sums + normalisation in one call (one
            # launch for small layers): one process / per-shard BN, dense aligned NHWC
            seg_fused = (training and part is not None and segs <= 2 and S % segs == 0 and not dp.sync_bn()
                         and K.is_nhwc(y) and y.data_ptr() % 16 == 0 and C % 4 == 0
                         and (out is None or (K.is_nhwc(out) and out.data_ptr() % 16 == 0)))
            if g1:
                pass
            elif seg_fused:
                a = torch.empty_like(y) if out is None else out
                stats = torch.empty((segs, 2 * C) if segs > 1 else (2 * C,), dtype=torch.float32, device=y.device)
                K.bn_segment_apply(part, S, y, spec.eps, spec.momentum, rm, rv, nbt, gamma, beta, spec.act,
                                   spec.alpha, stats.view(segs, 2 * C), a)
            elif training and segs > 1:
                Bs = y.shape[0] // segs
                a = torch.empty_like(y) if out is None else out
                stats = torch.empty((segs, 2 * C), dtype=torch.float32, device=y.device)
                for s_ in range(segs):
                    sl = slice(s_ * Bs, (s_ + 1) * Bs)
                    seg = (part, s_ * S // segs, (s_ + 1) * S // segs) if part is not None else None
                    _train_stats(y[sl], spec, rm, rv, nbt, seg, out=stats[s_])
                    K.bn_apply(y[sl], stats[s_], gamma, beta, spec.act, spec.alpha, out=a[sl])
            else:
                if training:
                    stats = _train_stats(y, spec, rm, rv, nbt, (part, 0, S) if part is not None else None)
                else:
                    stats = torch.cat([rm, torch.rsqrt(rv + spec.eps)])
                    stats_eval = (rm, stats[C:])
                a = K.bn_apply(y, stats, gamma, beta, spec.act, spec.alpha, out=out)
            ctx.save_for_backward(x, w, bias, gamma, beta, y, stats, *(sn if spec.spectral else ()))
        else:
            a = K.conv_fwd(x, w, spec.geom, bias=bias, act=spec.act, alpha=spec.alpha, wscale=wscale,
                           nchw_out=spec.nchw_out, cache=True, out=out)
            ctx.save_for_backward(x, w, bias, gamma, beta, a, None, *(sn if spec.spectral else ()))
        if ACT_TRACE is not None and spec.act in _KINKED:
            ACT_TRACE.append((a.detach() > 0).cpu())
            ACT_TAGS.append(TRACE_NET)
            ACT_LAYERS.append(TRACE_LAYER)
        ctx.spec = spec
        ctx.stats_eval = stats_eval
        ctx.training = bufs[3] if bufs is not None else True
        ctx.segs = segs
        ctx.g1 = g1
        ctx.gsegs = segs if gsegs is None else gsegs
        ctx.link_in, ctx.link_out = link_in, link_out
        if link_out is not None and LINKS:
            # how this layer's backward starts, for the layer above to fuse (LayerLink)
            link_out.done = None
            link_out.mode = 0
            if spec.bn and ctx.stats_eval is None and ctx.training and not dp.sync_bn() and K.is_nhwc(y):
                link_out.mode, link_out.x, link_out.stats = 2, y, stats
                link_out.gamma, link_out.beta, link_out.segs = gamma, beta, segs
            elif not spec.bn and spec.act in _POST_ACTS and not spec.nchw_out and K.is_nhwc(a):
                link_out.mode, link_out.x = 1, a
            link_out.act, link_out.alpha = spec.act, spec.alpha
        return a

    @staticmethod
    def backward(ctx, da):
        spec = ctx.spec
        saved = ctx.saved_tensors
        x, w, bias, gamma, beta, t5, stats = saved[:7]
        sn = saved[7:10] if spec.spectral else None
        nx, nw, nb, ng, nbeta = ctx.needs_input_grad[:5]
        if torch.is_grad_enabled():
            if ctx.segs > 1:
                raise NotImplementedError("double backward through a segmented (batched) layer call")
            # the graph this builds reads the layer's activations: a later backward through the
            # forward nodes sums its gradients with the chain's, so the chain's hand-offs
            # (LayerLink: one consumer per output) are off for this call
            for lk in (ctx.link_in, ctx.link_out):
                if lk is not None:
                    lk.mode, lk.done = 0, None
            return ConvLayerFn._create_graph_backward(ctx, da, x, w, bias, gamma, beta, sn)
        dx_full = dx_out = None
        Bg = x.shape[0]
        if ctx.gsegs < ctx.segs:
            # gradient rows of the leading segments only (NHWC / NCHW: a batch prefix)
            Bg = x.shape[0] * ctx.gsegs // ctx.segs
            da, x, t5 = da[:Bg], x[:Bg], t5[:Bg]
            if stats is not None and stats.dim() == 2:
                stats = stats[0] if ctx.gsegs == 1 else stats[:ctx.gsegs]
            if nx:
                # rows of the trailing (no-grad) segments are never read by the batched pass's
                # consumer and stay unwritten; zeroed only under anomaly detection, which
                # inspects every backward output
                dx_full = torch.empty_like(saved[0])
                dx_out = dx_full[:Bg]
                if torch.is_anomaly_enabled():
                    dx_full[Bg:].zero_()
        # this layer's output gradient may arrive with its first backward pass already applied
        # by the layer above (LayerLink): g = da * act' (+ BN sums), or da * act'
        done = ctx.link_out.done if ctx.link_out is not None else None
        if done is not None:
            ctx.link_out.done = None
            if not done[1].fused:
                done = None  # the GEMM above wrote the plain gradient
            elif done[0] != da.data_ptr():
                # the layer above applied this layer's act' / BatchNorm sums to the gradient it
                # produced, but a different tensor arrived here.  Links exist only between
                # consecutive layers inside one nets._Net call, whose intermediate activations
                # never leave the call (no user hook or second consumer can reach them), so this
                # is an internal assertion: running the first pass again would be silently wrong
                raise RuntimeError("LayerLink: the fused output gradient was replaced before this layer's "
                                   "backward (hook / cast / second consumer of the activation)")
        # ... and this layer's data gradient may carry the layer below's first pass
        # (the two layers ran in one chain call: same batch segments, same gradient rows)
        post = ctx.link_in.post(Bg, ctx.gsegs) if nx and ctx.link_in is not None else None
        wscale = sn[2] if spec.spectral else None
        dgamma = dbeta = None
        if spec.bn:
            y = t5
            P = y.shape[0] * y.shape[2] * y.shape[3]
            if ctx.stats_eval is not None:
                # the reference never calls .eval() (GLI:560-714): no training path reaches this
                raise NotImplementedError("backward through eval-mode BatchNorm is not on the training path")
            if done is not None and done[1].mode == 2:
                # da is g = da * act' and the sums are in done[1].part (the layer above's GEMM)
                dy, dgamma, dbeta = K.bn_backward_parts(da, y, stats, gamma, beta, done[1], ng, nbeta)
            elif stats.dim() == 2:  # segmented call: BN backward per segment, one dy
                dy, dgamma, dbeta = ConvLayerFn._seg_bn_backward(ctx, da, y, stats, gamma, beta, ng, nbeta)
            elif dp.sync_bn():
                sums, da_c = K.bn_backward_sums(da, y, stats, gamma, beta, spec.act, spec.alpha)
                # dgamma/dbeta stay shard-local (from the pre-all-reduce sums): the bucketed
                # gradient all-reduce sums them like every other parameter gradient
                C = y.shape[1]
                dgamma = torch.empty(C, dtype=torch.float32, device=y.device) if ng and gamma is not None else None
                dbeta = torch.empty(C, dtype=torch.float32, device=y.device) if nbeta and beta is not None else None
                K.bn_affine_grads(sums, stats, C, dgamma, dbeta)
                dp.all_reduce_sum(sums)
                dy, _, _ = K.bn_backward_apply(da_c, y, stats, gamma, beta, spec.act, spec.alpha, sums,
                                               P * dp.world(), need_affine=False)
            else:
                dy, dgamma, dbeta = K.bn_backward(da, y, stats, gamma, beta, spec.act, spec.alpha,
                                                  need_affine=ng or nbeta)
        elif spec.act != "none" and not (done is not None and done[1].mode == 1):
            dy = K.act_backward(da, t5, spec.act, spec.alpha)
        else:
            dy = da
        if ConvLayerFn._patch_conv(spec, x):
            # image-side Conv2d (D's first layer; the forward ran the direct narrow kernel):
            # the weight gradient is a 1x1 GEMM over the image's patch matrix
            dx = (K.conv_dgrad(dy, w, spec.geom, tuple(x.shape), wscale=wscale, out=dx_out, like=x, cache=True,
                               post=post) if nx else None)
            dw = db = None
            if nw or nb:
                g1, db = K.conv_wgrad(K.patches_k4s2(x), dy, K.G1X1, (w.shape[0], 64, 1, 1),
                                      with_bias=bias is not None and nb)
                dw = K.unpatch_grad(g1, w.shape[0], w.shape[1], 64, 1,
                                    into=dp.grad_view(w) if nw and not spec.spectral else None)
        elif ConvLayerFn._patch_convt(spec, w, bias):
            # image-side ConvTranspose2d (G's last layer): both gradients are 1x1 GEMMs over
            # the patch matrix of the image gradient, on x's grid
            Xg = K.patches_k4s2(dy)
            dx = (K.conv_fwd(Xg, K.PATCHW.get(w, True), K.G1X1, wscale=wscale, out=dx_out, cache=True, post=post)
                  if nx else None)
            dw = db = None
            if nw:
                g1, _ = K.conv_wgrad(Xg, x, K.G1X1, (w.shape[0], 64, 1, 1))
                dw = K.unpatch_grad(g1, w.shape[0], w.shape[1], 64, 1,
                                    into=dp.grad_view(w) if not spec.spectral else None)
        else:
            dx = (K.conv_dgrad(dy, w, spec.geom, tuple(x.shape), wscale=wscale, out=dx_out, like=x, cache=True,
                               post=post) if nx else None)
            dw = db = None
            if nw and not nb and spec.geom.upsample == 1 and ConvLayerFn._own_grad(w, bias):
                # The weight gradient goes straight into w.grad: set when it is empty (what
                # AccumulateGrad would do), added in the GEMM epilogue / sigma correction when
                # an earlier call of the net left one (spectral D's separate D(x) / D(G(z))
                # calls, heads 1-4's two backwards) -- instead of autograd summing the calls'
                # gradients with an add kernel (same values: grad + dw, one rounding).  No
                # gradient is returned for w.
                acc = w.grad
                if spec.spectral:
                    u, v, inv_sigma = sn
                    dwe, _ = K.conv_wgrad(x, dy, spec.geom, tuple(w.shape))
                    g = K.spectral_backward(w, dwe, u, v, inv_sigma, spec.geom.transposed, out=acc)
                elif ctx.g1:
                    g = K.g1_wgrad(x, dy, tuple(w.shape), out=acc)
                else:
                    g, _ = K.conv_wgrad(x, dy, spec.geom, tuple(w.shape), out=acc)
                if acc is None:
                    w.grad = g
                ConvLayerFn._hand_down(ctx, post, dx)
                return ((dx if dx_full is None else dx_full), None, None, dgamma, dbeta, None, None, None, None, None,
                        None, None, None)
            if nw or nb:
                # data parallel: the weight gradient lands in its gradient bucket's slice
                # (dp.grad_view), which autograd then adopts as .grad (no bucket copy)
                into = (dp.grad_view(w) if nw and not (bias is not None and nb) and not spec.spectral
                        and spec.geom.upsample == 1 else None)
                if ctx.g1 and nw:
                    dw, db = K.g1_wgrad(x, dy, tuple(w.shape), into=into), None
                else:
                    dw, db = K.conv_wgrad(x, dy, spec.geom, tuple(w.shape), with_bias=bias is not None and nb,
                                          into=into)
        if nw or nb:
            if spec.spectral and nw:
                u, v, inv_sigma = sn
                dw = K.spectral_backward(w, dw, u, v, inv_sigma, spec.geom.transposed)
            if not nw:
                dw = None
        ConvLayerFn._hand_down(ctx, post, dx)
        if dx_full is not None:
            dx = dx_full
        return dx, dw, db, dgamma, dbeta, None, None, None, None, None, None, None, None

    @staticmethod
    def _hand_down(ctx, post, dx):
        """The layer below starts its backward from dx as the post-op left it (LayerLink)."""
        if post is not None and post.fused and dx is not None:
            ctx.link_in.done = (dx.data_ptr(), post)

    @staticmethod
    def _own_grad(w, bias):
        """This call may write its weight gradient into w.grad itself: one process (no
        gradient-bucket hooks waiting on AccumulateGrad), w a leaf, no bias gradient to
        accumulate alongside, no tensor / post-accumulate hook on w (they fire from autograd's
        AccumulateGrad, which this path bypasses), and .grad empty or a plain contiguous fp32
        tensor of w's shape."""
        if not (owning_grads.active and not dp.active() and w.is_leaf and bias is None):
            return False
        if getattr(w, "_backward_hooks", None) or getattr(w, "_post_accumulate_grad_hooks", None):
            return False
        g = w.grad
        return g is None or (g.shape == w.shape and g.dtype == torch.float32 and g.is_contiguous()
                             and not g.requires_grad and g.device == w.device)

    @staticmethod
    def _patch_conv(spec, x):
        return (not spec.geom.transposed and not spec.bn and K.patchable(spec.geom, x.shape[1])
                and x.shape[2] % 2 == 0 and x.shape[3] % 2 == 0)

    @staticmethod
    def _patch_convt(spec, w, bias):
        return (spec.geom.transposed and not spec.bn and bias is None
                and K.patchable(spec.geom, w.shape[1]))

    @staticmethod
    def _seg_bn_backward(ctx, da, y, stats, gamma, beta, ng, nbeta):
        spec = ctx.spec
        if not K.is_nhwc(da):
            da = da.contiguous(memory_format=torch.channels_last)
        dy = torch.empty_like(y)
        Bs = y.shape[0] // ctx.segs
        P = Bs * y.shape[2] * y.shape[3]
        C = y.shape[1]
        dgamma = dbeta = None
        if (ctx.segs == 2 and not dp.sync_bn() and K.is_nhwc(y) and C % 4 == 0
                and y.data_ptr() % 16 == 0 and da.data_ptr() % 16 == 0 and dy.data_ptr() % 16 == 0):
            # both calls' BatchNorm backward in one set of launches (affine gradients summed)
            return K.bn_backward_segments(da, y, stats, gamma, beta, spec.act, spec.alpha, ng, nbeta, dy)
        for s_ in range(ctx.segs):
            sl = slice(s_ * Bs, (s_ + 1) * Bs)
            if dp.sync_bn():
                sums, da_c = K.bn_backward_sums(da[sl], y[sl], stats[s_], gamma, beta, spec.act, spec.alpha)
                dg = (sums[C:] * stats[s_, C:2 * C].double()).float() if ng and gamma is not None else None
                db = sums[:C].float() if nbeta and beta is not None else None
                dp.all_reduce_sum(sums)
                K.bn_backward_apply(da_c, y[sl], stats[s_], gamma, beta, spec.act, spec.alpha, sums,
                                    P * dp.world(), need_affine=False, out=dy[sl])
                dgamma = dg if dgamma is None or dg is None else dgamma + dg
                dbeta = db if dbeta is None or db is None else dbeta + db
            else:
                # the segments' affine gradients are summed in the apply kernel (segment 0
                # writes, later segments add): no separate add pass
                if s_ == 0:
                    dgamma = torch.empty(C, dtype=torch.float32, device=y.device) if ng and gamma is not None else None
                    dbeta = torch.empty(C, dtype=torch.float32, device=y.device) if nbeta and beta is not None else None
                sums, da_c = K.bn_backward_sums(da[sl], y[sl], stats[s_], gamma, beta, spec.act, spec.alpha)
                K.bn_backward_apply_ex(da_c, y[sl], stats[s_], gamma, beta, spec.act, spec.alpha, sums, P,
                                       out=dy[sl], dgamma=dgamma, dbeta=dbeta, accumulate_affine=s_ > 0)
        return dy, dgamma, dbeta

    @staticmethod
    def _create_graph_backward(ctx, da, x, w, bias, gamma, beta, sn):
        """Differentiable backward: rebuild the layer from its REAL inputs (x keeps its
        history, w is the Parameter) and let autograd differentiate the composite, so the
        returned gradients are functions of (da, x, w, ...) that gp.backward() can follow."""
        spec = ctx.spec
        slots = [i for i, t in enumerate((x, w, bias, gamma, beta))
                 if t is not None and ctx.needs_input_grad[i]]
        out = [None] * 13
        if not slots:
            return tuple(out)
        src = (x, w, bias, gamma, beta)
        with torch.enable_grad():
            a = composite_layer(x, w, bias, gamma, beta, spec, ctx.stats_eval, sn)
            grads = torch.autograd.grad(a, [src[i] for i in slots], da, create_graph=True, allow_unused=True)
        for i, g in zip(slots, grads):
            out[i] = g
        return tuple(out)
