"""Tensor-level wrappers over the C-ABI (no autograd here; see autograd.py).

Every function takes CUDA (HIP) tensors, allocates outputs with torch's caching
allocator and launches on the current stream.  Internal activations are NHWC
(torch channels_last strides on a [B, C, H, W] tensor); NCHW tensors are accepted
wherever the reference hands them over (images into D, out of G).
"""
import ctypes
import weakref
from dataclasses import dataclass

import torch

from . import _lib as L


@dataclass(frozen=True)
class ConvGeom:
    """One conv layer as the reference declares it (k, stride, pad, transposed)."""
    k: int
    stride: int
    pad: int
    transposed: bool
    upsample: int = 1  # 2: nearest Upsample(x2) in front of the conv (--NN_conv, GLI:351-356)

    def out_hw(self, h, w):
        h, w = h * self.upsample, w * self.upsample
        if self.transposed:
            return ((h - 1) * self.stride - 2 * self.pad + self.k, (w - 1) * self.stride - 2 * self.pad + self.k)
        return ((h + 2 * self.pad - self.k) // self.stride + 1, (w + 2 * self.pad - self.k) // self.stride + 1)

    def in_hw(self, ho, wo):
        if self.transposed:
            h, w = (ho + 2 * self.pad - self.k) // self.stride + 1, (wo + 2 * self.pad - self.k) // self.stride + 1
        else:
            h, w = (ho - 1) * self.stride - 2 * self.pad + self.k, (wo - 1) * self.stride - 2 * self.pad + self.k
        return h // self.upsample, w // self.upsample


# Upsample(x2)+Conv2d(k3,s1,p1) runs as this transposed conv on the folded weight
# (csrc/upsample.hip; include/rgan.h rgan_nn_fold_weight).
NN_T = ConvGeom(4, 2, 1, True)


# activations with a nonzero second derivative (the WGAN-GP double backward needs act'')
ACT_HAS_GRAD2 = {"none": False, "relu": False, "lrelu": False, "tanh": True, "sigmoid": True, "selu": True}


def _nn_check(geom):
    if geom.upsample != 2 or geom.transposed or (geom.k, geom.stride, geom.pad) != (3, 1, 1):
        raise L.RganError(f"unsupported upsampling conv {geom}: only Upsample(x2)+Conv2d(k3,s1,p1) (--NN_conv)")


def empty_nhwc(B, C, H, W, device):
    return torch.empty_strided((B, C, H, W), (H * W * C, 1, W * C, C), dtype=torch.float32, device=device)


def is_nhwc(t):
    B, C, H, W = t.shape
    return t.stride() == (H * W * C, 1, W * C, C) or (H == 1 and W == 1 and t.stride()[1] == 1)


def _desc(x_shape, x_stride, y_shape, y_stride, geom):
    d = L.RganConv()
    B, cin, hin, win = x_shape
    _, cout, hout, wout = y_shape
    d.batch, d.cin, d.hin, d.win = B, cin, hin, win
    d.cout, d.hout, d.wout = cout, hout, wout
    d.kh = d.kw = geom.k
    d.stride, d.pad, d.transposed = geom.stride, geom.pad, int(geom.transposed)
    for i in range(4):
        d.xs[i] = x_stride[i]
        d.ys[i] = y_stride[i]
    return d


def _f32(*ts):
    for t in ts:
        if t is not None and t.dtype != torch.float32:
            raise L.RganError(f"expected float32 tensors, got {t.dtype}")


class _PackCache:
    """GEMM-ready weight layouts, cached per (weight tensor, layout, version).

    Weights change only at optimizer steps (fused Adam bumps the autograd version
    counter), while every net runs 2-4 times per iteration, so most conv launches reuse
    a packed copy.  Entries are keyed by the weight's base tensor object (held weakly:
    a storage address can be reused by a later tensor with the same version count) and
    one buffer per (weight, layout) is refilled in place when the version moves."""

    def __init__(self):
        self.entries = {}

    def get(self, w, which, geom, d):
        base = w._base if w._base is not None else w
        key = (id(base), which, geom, d.cin, d.cout, d.hin, d.win, d.hout, d.wout)
        ver = w._version
        ent = self.entries.get(key)
        if ent is not None and ent[0]() is base and ent[1] == ver and ent[3] == w.data_ptr():
            return ent[2]
        lib = L.lib()
        n = lib.rgan_conv_pack_floats(ctypes.byref(d), which)
        if n == 0:
            return None  # the op reads the torch layout directly (or is unsupported: workspace says)
        reuse = ent is not None and ent[0]() is base and ent[2].numel() == n
        buf = ent[2] if reuse else torch.empty(n, dtype=torch.float32, device=w.device)
        L.check(lib.rgan_conv_pack(ctypes.byref(d), which, L.ptr(w), L.ptr(buf), L.stream()), "rgan_conv_pack")
        # (the descriptor, layout and w's view geometry on its base let refresh() and the
        # optimizer's layout writer find the weight again: a view such as arch 1's dense layers
        # viewed as convolutions is a new tensor object at every call, so a weak reference to it
        # would die with the call and its layout would be repacked at every use)
        geo = None if w is base else (tuple(w.shape), tuple(w.stride()), w.storage_offset())
        self.entries[key] = (weakref.ref(base, self._drop(key)), ver, buf, w.data_ptr(), d, which, geo)
        return buf

    @staticmethod
    def _weight(ent):
        """The packed weight of an entry (its base parameter, or the view of it that was packed),
        or None when the entry is stale: the base is gone, or its storage no longer covers the
        saved view (e.g. ``p.data = smaller``) -- such an entry is never a valid layout source."""
        base = ent[0]()
        if base is None or ent[6] is None:
            return base
        shape, stride, offset = ent[6]
        extent = offset + 1 + sum((n - 1) * st for n, st in zip(shape, stride))  # elements, all n >= 1
        if any(n == 0 for n in shape) or base.untyped_storage().nbytes() < extent * base.element_size():
            return None
        return base.as_strided(shape, stride, offset)

    def _stale(self, key, ent):
        """Drop an entry whose weight view can no longer be rebuilt (see _weight)."""
        if ent[0]() is not None and self.entries.get(key) is ent:
            del self.entries[key]

    def refresh(self, params):
        """Repack, in one batched launch, every cached layout of ``params`` whose weight
        moved (called right after an optimizer step): the next convolutions find them
        current instead of packing one launch at a time."""
        ids = {id(p) for p in params}
        todo = []
        for key, ent in list(self.entries.items()):
            base, w = ent[0](), self._weight(ent)
            if base is not None and w is None:
                self._stale(key, ent)
                continue
            if base is None or id(base) not in ids:
                continue
            if ent[1] == w._version and ent[3] == w.data_ptr():
                continue
            todo.append((key, ent, w))
        if not todo:
            return
        n = len(todo)
        descs = (ctypes.POINTER(L.RganConv) * n)(*[ctypes.pointer(e[4]) for _, e, _ in todo])
        which = (ctypes.c_int * n)(*[e[5] for _, e, _ in todo])
        ws = (ctypes.c_void_p * n)(*[w.data_ptr() for _, _, w in todo])
        outs = (ctypes.c_void_p * n)(*[e[2].data_ptr() for _, e, _ in todo])
        L.check(L.lib().rgan_conv_pack_batch(n, ctypes.cast(descs, ctypes.c_void_p), ctypes.cast(which, ctypes.c_void_p),
                                             ctypes.cast(ws, ctypes.c_void_p), ctypes.cast(outs, ctypes.c_void_p),
                                             L.stream()), "rgan_conv_pack_batch")
        for key, ent, w in todo:
            self.entries[key] = (ent[0], w._version, ent[2], w.data_ptr()) + ent[4:]

    def layouts_of(self, params):
        """[(param index, key, entry)] of every cached layout of ``params`` (for
        rgan_adam_packed, which rewrites them with the new values)."""
        idx = {id(p): i for i, p in enumerate(params)}
        out = []
        for key, ent in list(self.entries.items()):
            base, w = ent[0](), self._weight(ent)
            if base is not None and w is None:
                self._stale(key, ent)
                continue
            if base is None or id(base) not in idx or w.data_ptr() != params[idx[id(base)]].data_ptr():
                continue
            if w.numel() != params[idx[id(base)]].numel():
                continue
            out.append((idx[id(base)], key, ent))
        return out

    def mark_current(self, layouts):
        """The listed layouts were rewritten from their weights' current values."""
        for _, key, ent in layouts:
            w = self._weight(ent)
            if w is not None and self.entries.get(key) is ent:
                self.entries[key] = (ent[0], w._version, ent[2], w.data_ptr()) + ent[4:]

    def _drop(self, key):
        def cb(_ref):
            ent = self.entries.get(key)
            if ent is not None and ent[0] is _ref:
                del self.entries[key]
        return cb

    def clear(self):
        self.entries.clear()


PACKS = _PackCache()


class _FoldCache:
    """Folded --NN_conv weights (Wt = A W A^T), one per (weight, version): like the packs,
    refolded only after an optimizer step.  A new Wt tensor is made per version so the
    pack cache (keyed by the Wt object) never sees a stale layout.  ``fn`` is the fold
    (nn_fold here; the image-layer patch weights use their own instance)."""

    def __init__(self, fn=None):
        self.entries = {}
        self.fn = fn

    def get(self, w, *args):
        base = w._base if w._base is not None else w
        key = (id(base),) + args
        ent = self.entries.get(key)
        if ent is not None and ent[0]() is base and ent[1] == w._version and ent[2] == w.data_ptr():
            return ent[3]
        wt = (self.fn or nn_fold)(w, *args)
        self.entries[key] = (weakref.ref(base, self._drop(key)), w._version, w.data_ptr(), wt)
        return wt

    def _drop(self, key):
        def cb(_ref):
            ent = self.entries.get(key)
            if ent is not None and ent[0] is _ref:
                del self.entries[key]
        return cb

    def clear(self):
        self.entries.clear()


FOLDS = _FoldCache()


# ------------------------------------------------------------------ image layers as 1x1 GEMMs
G1X1 = ConvGeom(1, 1, 0, False)


def patchable(geom, cin_img):
    """k4 s2 p1 layer whose image side has <= 4 channels (D's first conv, G's last convT)."""
    return (geom.k, geom.stride, geom.pad, geom.upsample) == (4, 2, 1, 1) and cin_img <= 4


def patches_k4s2(img):
    """Patch matrix of an image [B][C][H][W] (any strides, C <= 4) on the half-size grid,
    as an NHWC [B, 64, H/2, W/2] tensor (rgan_patches_k4s2)."""
    L.require_cuda(img)
    _f32(img)
    B, C, H, W = img.shape
    X = empty_nhwc(B, 64, H // 2, W // 2, img.device)
    st = (L.c_ll * 4)(*img.stride())
    L.check(L.lib().rgan_patches_k4s2(L.ptr(img), B, C, H, W, st, L.ptr(X), L.stream()), "rgan_patches_k4s2")
    return X


def patch_weight(w, transposed):
    """Image-layer weight -> the 1x1 GEMM weight [O][64][1][1], W1[o][4t+c] = W[o][c][t]:
    Conv2d [co][ci][4][4] (o = co, c = ci) or ConvTranspose2d [ci][co][4][4] (o = ci, c = co)."""
    wc = w.contiguous()
    O, C = wc.shape[0], wc.shape[1]
    w1 = torch.empty((O, 64, 1, 1), dtype=torch.float32, device=w.device)
    L.check(L.lib().rgan_patch_weight(L.ptr(wc), O, C, C * 16, 16, L.ptr(w1), L.stream()), "rgan_patch_weight")
    return w1


PATCHW = _FoldCache(patch_weight)


def unpatch_grad(g1, O, C, row_stride, col_stride, out=None, into=None):
    """1x1-GEMM weight gradient -> torch layout [O][C][4][4] (dw[o][c][t] = g1[o*rs + (4t+c)*cs]);
    ``out`` given: added into it (gradient accumulation); ``into``: written into it."""
    acc = out is not None
    if into is not None and (acc or tuple(into.shape) != (O, C, 4, 4) or not into.is_contiguous()):
        raise L.RganError("unpatch_grad: `into` must be a contiguous [O][C][4][4] tensor (no accumulation)")
    dw = out if acc else (into if into is not None else torch.empty((O, C, 4, 4), dtype=torch.float32,
                                                                    device=g1.device))
    L.check(L.lib().rgan_unpatch_grad(L.ptr(g1), O, C, row_stride, col_stride, L.ptr(dw), int(acc), L.stream()),
            "rgan_unpatch_grad")
    return dw


def nn_fold(w):
    """Conv2d weight [cout][cin][3][3] -> ConvTranspose2d weight [cin][cout][4][4]."""
    L.require_cuda(w)
    _f32(w)
    cout, cin = w.shape[0], w.shape[1]
    if tuple(w.shape[2:]) != (3, 3):
        raise L.RganError(f"nn_fold expects a 3x3 kernel, got {tuple(w.shape)}")
    wt = torch.empty((cin, cout, 4, 4), dtype=torch.float32, device=w.device)
    L.check(L.lib().rgan_nn_fold_weight(L.ptr(w.contiguous()), cout, cin, L.ptr(wt), L.stream()),
            "rgan_nn_fold_weight")
    return wt


def nn_unfold_grad(dwt, w_shape):
    """Adjoint of nn_fold: dWt [cin][cout][4][4] -> dW [cout][cin][3][3]."""
    cout, cin = w_shape[0], w_shape[1]
    dw = torch.empty(w_shape, dtype=torch.float32, device=dwt.device)
    L.check(L.lib().rgan_nn_unfold_grad(L.ptr(dwt.contiguous()), cout, cin, L.ptr(dw), L.stream()),
            "rgan_nn_unfold_grad")
    return dw


def conv_fwd(x, w, geom, bias=None, act="none", alpha=0.0, wscale=None, out=None, nchw_out=False, cache=False,
             post=None):
    """y = act(conv(x, w)*wscale + bias); x [B,Cin,H,W] any strides; w torch layout.

    ``cache=True`` (module parameters only) reuses a packed weight while its version is
    unchanged.  ``post`` (no bias / act): a Post for the producer of ... (see conv_dgrad) --
    used when this conv computes a gradient (G's image-layer data gradient as a 1x1 GEMM)."""
    L.require_cuda(x, w, bias, wscale)
    _f32(x, w, bias)
    if geom.upsample != 1:
        _nn_check(geom)
        wt = FOLDS.get(w) if cache else nn_fold(w)
        return conv_fwd(x, wt, NN_T, bias=bias, act=act, alpha=alpha, wscale=wscale, out=out, nchw_out=nchw_out,
                        cache=cache, post=post)
    B, cin, H, W = x.shape
    cout = w.shape[1] if geom.transposed else w.shape[0]
    Ho, Wo = geom.out_hw(H, W)
    if out is None:
        out = (torch.empty((B, cout, Ho, Wo), dtype=torch.float32, device=x.device) if nchw_out
               else empty_nhwc(B, cout, Ho, Wo, x.device))
    d = _desc(x.shape, x.stride(), out.shape, out.stride(), geom)
    lib = L.lib()
    packed = PACKS.get(w, 0, geom, d) if cache else None
    nbytes = lib.rgan_conv_workspace(ctypes.byref(d), 0, int(packed is not None))
    if nbytes == 0:
        raise L.RganError(f"unsupported conv {geom} for input {tuple(x.shape)}")
    ws = L.workspace(nbytes, x.device)
    if post is not None:
        post.fused = False
        if bias is None and act == "none" and _conv_post(0, d, x, w, packed, wscale, out, ws, post) is not False:
            return out
    L.check(lib.rgan_conv_fwd(ctypes.byref(d), L.ptr(x), L.ptr(w), L.ptr(packed), L.ptr(wscale), L.ptr(bias),
                              L.ptr(out), L.ACT[act], float(alpha), L.ptr(ws), ws.numel(), L.stream()),
            "rgan_conv_fwd")
    return out


def conv_fwd_bn(x, w, geom, bias=None, wscale=None, cache=False, segs=1):
    """y = conv(x, w)*wscale + bias (NHWC) for a layer followed by train-mode BatchNorm.

    Returns (y, part, S): when the GEMM's vector epilogue or its split-K reduce covered the
    layer, ``part`` is
    its per-64-row segment sums (sum y, sum y^2) double[S][2][C] (merge with bn_segment_stats; batch
    segment k = segments [k*S/segs, (k+1)*S/segs)); otherwise (y, None, 0)."""
    if geom.upsample != 1:
        return conv_fwd(x, w, geom, bias=bias, wscale=wscale, cache=cache), None, 0
    L.require_cuda(x, w, bias, wscale)
    _f32(x, w, bias)
    B, cin, H, W = x.shape
    cout = w.shape[1] if geom.transposed else w.shape[0]
    Ho, Wo = geom.out_hw(H, W)
    out = empty_nhwc(B, cout, Ho, Wo, x.device)
    d = _desc(x.shape, x.stride(), out.shape, out.stride(), geom)
    lib = L.lib()
    S = lib.rgan_conv_bn_segments(ctypes.byref(d), int(segs))
    if S <= 0:
        return conv_fwd(x, w, geom, bias=bias, wscale=wscale, out=out, cache=cache), None, 0
    packed = PACKS.get(w, 0, geom, d) if cache else None
    nbytes = lib.rgan_conv_workspace(ctypes.byref(d), 0, int(packed is not None))
    if nbytes == 0:
        raise L.RganError(f"unsupported conv {geom} for input {tuple(x.shape)}")
    ws = L.workspace(nbytes, x.device)
    part = torch.empty((S, 2, cout), dtype=torch.float64, device=x.device)
    fused = L.c_int(0)
    L.check(lib.rgan_conv_fwd_bn(ctypes.byref(d), L.ptr(x), L.ptr(w), L.ptr(packed), L.ptr(wscale), L.ptr(bias),
                                 L.ptr(out), L.ptr(ws), ws.numel(), L.ptr(part), S, int(segs), ctypes.byref(fused),
                                 L.stream()), "rgan_conv_fwd_bn")
    return (out, part, S) if fused.value else (out, None, 0)


def bn_segment_stats(part, s0, s1, C, eps, momentum, running_mean=None, running_var=None,
                     num_batches_tracked=None, out=None):
    """Segment moments [s0, s1) of conv_fwd_bn -> (mean, invstd) float[2C] + running stats."""
    stats = torch.empty(2 * C, dtype=torch.float32, device=part.device) if out is None else out
    L.check(L.lib().rgan_bn_segment_stats(L.ptr(part), int(s0), int(s1), C, 64, float(eps), float(momentum),
                                          L.ptr(running_mean), L.ptr(running_var), L.ptr(num_batches_tracked),
                                          L.ptr(stats), None, L.stream()), "rgan_bn_segment_stats")
    return stats


def bn_segment_moments(part, s0, s1, C):
    """Segment moments [s0, s1) -> this rank's (count, mean, M2) double[3C] (SyncBN stage 1)."""
    mom = torch.empty(3 * C, dtype=torch.float64, device=part.device)
    L.check(L.lib().rgan_bn_segment_stats(L.ptr(part), int(s0), int(s1), C, 64, 0.0, 0.0, None, None, None, None,
                                          L.ptr(mom), L.stream()), "rgan_bn_segment_stats")
    return mom


class Post:
    """Producer post-op of rgan_conv_post (include/rgan.h RganPost): the backward pass of the
    layer that produced this GEMM's output operand, applied in the GEMM's epilogue / split-K
    reduce.  mode 1: out *= act'(x) (x = its activation output); mode 2: out = g = out *
    act'(BN(x)) and the BatchNorm backward sums per 64-row segment (x = its BN input y; finish
    with bn_backward_parts).  After the call ``fused`` says whether the GEMM applied it
    (else the output is the plain gradient) and, for mode 2, ``part`` / ``S`` / ``phases``
    hold the sums."""

    __slots__ = ("mode", "act", "alpha", "x", "stats", "gamma", "beta", "nseg", "fused", "part", "S", "phases")

    def __init__(self, mode, act, alpha, x, stats=None, gamma=None, beta=None, nseg=1):
        self.mode, self.act, self.alpha, self.x = mode, act, float(alpha), x
        self.stats, self.gamma, self.beta, self.nseg = stats, gamma, beta, nseg
        self.fused, self.part, self.S, self.phases = False, None, 0, 1


def _conv_post(which, d, inp, w, packed, wscale, out, ws, post):
    """rgan_conv_post for ``post`` (see Post); returns False when the GEMM cannot apply it."""
    if (tuple(post.x.shape) != tuple(out.shape) or post.x.stride() != out.stride()
            or post.x.data_ptr() % 16 or out.data_ptr() % 16):
        return False
    lib = L.lib()
    part, S = None, 0
    if post.mode == 2:
        ph = L.c_int(1)
        S = lib.rgan_conv_post_segments(ctypes.byref(d), which, 2, int(post.nseg), ctypes.byref(ph))
        post.phases = ph.value
        if S <= 0:
            return False
        part = torch.empty((S, 2, out.shape[1]), dtype=torch.float64, device=out.device)
    rp = L.RganPost(int(post.mode), L.ACT[post.act], float(post.alpha), int(post.nseg), post.x.data_ptr(),
                    L.ptr(post.stats), L.ptr(post.gamma), L.ptr(post.beta), L.ptr(part), int(S))
    fused = L.c_int(0)
    L.check(lib.rgan_conv_post(ctypes.byref(d), which, L.ptr(inp), L.ptr(w), L.ptr(packed), L.ptr(wscale),
                               L.ptr(out), L.ptr(ws), ws.numel(), ctypes.byref(rp), ctypes.byref(fused), L.stream()),
            "rgan_conv_post")
    if not fused.value:
        return None  # the plain result was written
    post.fused, post.part, post.S = True, part, S
    return True


def conv_dgrad(dy, w, geom, x_shape, wscale=None, out=None, like=None, cache=False, post=None):
    """dx of the conv (input grad), NHWC unless `like` (a tensor whose strides to copy) is given.
    ``post``: a Post for the layer that produced x (applied when the GEMM can: post.fused)."""
    L.require_cuda(dy, w, wscale)
    _f32(dy, w)
    if geom.upsample != 1:
        _nn_check(geom)
        wt = FOLDS.get(w) if cache else nn_fold(w)
        return conv_dgrad(dy, wt, NN_T, x_shape, wscale=wscale, out=out, like=like, cache=cache, post=post)
    B, cin, H, W = x_shape
    if out is None:
        if like is not None and not is_nhwc(like):
            out = torch.empty(x_shape, dtype=torch.float32, device=dy.device)
        else:
            out = empty_nhwc(B, cin, H, W, dy.device)
    d = _desc(out.shape, out.stride(), dy.shape, dy.stride(), geom)
    lib = L.lib()
    packed = PACKS.get(w, 1, geom, d) if cache else None
    nbytes = lib.rgan_conv_workspace(ctypes.byref(d), 1, int(packed is not None))
    if nbytes == 0:
        raise L.RganError(f"unsupported conv dgrad {geom} for {tuple(x_shape)}")
    ws = L.workspace(nbytes, dy.device)
    if post is not None:
        post.fused = False
        if _conv_post(1, d, dy, w, packed, wscale, out, ws, post) is not False:
            return out
    L.check(lib.rgan_conv_dgrad(ctypes.byref(d), L.ptr(dy), L.ptr(w), L.ptr(packed), L.ptr(wscale), L.ptr(out),
                                L.ptr(ws), ws.numel(), L.stream()), "rgan_conv_dgrad")
    return out


def g1_ok(x, w, geom):
    """G's first layer on its 1x1 input can run as rgan_g1_fwd_bn / rgan_g1_wgrad."""
    return (geom.transposed and geom.k == 4 and geom.stride == 1 and geom.pad == 0 and geom.upsample == 1
            and x.dim() == 4 and tuple(x.shape[2:]) == (1, 1) and x.shape[0] in (32, 64) and x.shape[1] in (64, 128)
            and w.shape[1] % 16 == 0 and w.is_contiguous() and x.is_contiguous() and x.data_ptr() % 16 == 0)


def g1_fwd_bn(x, w, gamma, beta, eps, momentum, running_mean, running_var, num_batches_tracked, act, alpha,
              out=None):
    """(y, a, stats) of G's first layer + BatchNorm + act in one launch (rgan_g1_fwd_bn)."""
    L.require_cuda(x, w)
    B, cin = x.shape[0], x.shape[1]
    cout = w.shape[1]
    y = empty_nhwc(B, cout, 4, 4, x.device)
    a = empty_nhwc(B, cout, 4, 4, x.device) if out is None else out
    if not is_nhwc(a):
        raise L.RganError("g1_fwd_bn: out must be NHWC")
    stats = torch.empty(2 * cout, dtype=torch.float32, device=x.device)
    L.check(L.lib().rgan_g1_fwd_bn(L.ptr(x), B, cin, L.ptr(w), cout, L.ptr(gamma), L.ptr(beta), float(eps),
                                   float(momentum), L.ptr(running_mean), L.ptr(running_var),
                                   L.ptr(num_batches_tracked), L.ACT[act], float(alpha), L.ptr(y), L.ptr(a),
                                   L.ptr(stats), L.stream()), "rgan_g1_fwd_bn")
    return y, a, stats


def g1_wgrad(x, dy, w_shape, out=None, into=None):
    """dW of G's first layer (rgan_g1_wgrad); ``out``: add into it, ``into``: write into it."""
    L.require_cuda(x, dy)
    if not is_nhwc(dy):
        dy = dy.contiguous(memory_format=torch.channels_last)
    dw = out if out is not None else (into if into is not None else
                                      torch.empty(w_shape, dtype=torch.float32, device=x.device))
    L.check(L.lib().rgan_g1_wgrad(L.ptr(x), x.shape[0], x.shape[1], L.ptr(dy), w_shape[1], L.ptr(dw),
                                  int(out is not None), L.stream()), "rgan_g1_wgrad")
    return dw


def conv_wgrad(x, dy, geom, w_shape, with_bias=False, out=None, out_bias=None, into=None, bias_row0=0):
    """(dw in torch layout, dbias or None).  ``out`` / ``out_bias`` given: the gradients are
    ADDED into them in the GEMM epilogue (autograd accumulation without an add pass);
    ``into``: dw is WRITTEN into that tensor (e.g. its slice of a data-parallel gradient
    bucket, dp.grad_view) instead of a new one.  ``bias_row0``: dbias sums dy's pixel rows
    (b, h, w) from that one on (rgan_conv_wgrad_rows: the GP engine's [adjoint; forward] pairs)."""
    L.require_cuda(x, dy)
    _f32(x, dy)
    if into is not None:
        if out is not None or geom.upsample != 1:
            raise L.RganError("conv_wgrad: `into` excludes accumulation and NN_conv")
        if tuple(into.shape) != tuple(w_shape) or not into.is_contiguous():
            raise L.RganError("conv_wgrad: `into` must be a contiguous tensor of the weight's shape")
    if geom.upsample != 1:
        _nn_check(geom)
        if out is not None:
            raise L.RganError("accumulating NN_conv weight gradients is not supported")
        cout, cin = w_shape[0], w_shape[1]
        dwt, db = conv_wgrad(x, dy, NN_T, (cin, cout, 4, 4), with_bias=with_bias, bias_row0=bias_row0)
        return nn_unfold_grad(dwt, tuple(w_shape)), db
    acc = out is not None
    if acc and (tuple(out.shape) != tuple(w_shape) or not out.is_contiguous()):
        raise L.RganError("conv_wgrad: out must be a contiguous tensor of the weight's shape")
    dw = out if acc else (into if into is not None else torch.empty(w_shape, dtype=torch.float32, device=x.device))
    db = None
    if with_bias:
        if acc != (out_bias is not None):
            raise L.RganError("conv_wgrad: accumulate weight and bias gradients together")
        db = out_bias if acc else torch.empty(dy.shape[1], dtype=torch.float32, device=x.device)
        if not is_nhwc(dy):
            dy = dy.contiguous(memory_format=torch.channels_last)
    d = _desc(x.shape, x.stride(), dy.shape, dy.stride(), geom)
    lib = L.lib()
    nbytes = lib.rgan_conv_workspace(ctypes.byref(d), 2, 0)
    if nbytes == 0:
        raise L.RganError(f"unsupported conv wgrad {geom} for {tuple(x.shape)}")
    ws = L.workspace(nbytes, x.device)
    L.check(lib.rgan_conv_wgrad_rows(ctypes.byref(d), L.ptr(x), L.ptr(dy), L.ptr(dw), L.ptr(db), int(bias_row0),
                                     int(acc), L.ptr(ws), ws.numel(), L.stream()), "rgan_conv_wgrad_rows")
    return dw, db


# ------------------------------------------------------------------ BatchNorm
def _pc(t):
    """[P][C] view parameters of an NHWC tensor."""
    B, C, H, W = t.shape
    if not is_nhwc(t):
        raise L.RganError("BatchNorm kernels expect NHWC (channels_last) activations")
    return B * H * W, C, C, 1


def bn_stats(y, eps, momentum, running_mean=None, running_var=None, num_batches_tracked=None, out=None):
    """Batch (mean, invstd) as float[2C]; updates running buffers when given."""
    P, C, sp, sc = _pc(y)
    lib = L.lib()
    stats = torch.empty(2 * C, dtype=torch.float32, device=y.device) if out is None else out
    part = L.workspace(lib.rgan_bn_partial_bytes(P, C), y.device)
    L.check(lib.rgan_bn_stats(L.ptr(y), P, C, sp, sc, float(eps), float(momentum), L.ptr(running_mean),
                              L.ptr(running_var), L.ptr(num_batches_tracked), L.ptr(stats), L.ptr(part),
                              L.stream()), "rgan_bn_stats")
    return stats


def bn_moments(y):
    """This rank's per-channel (count, mean, M2) as double[3C] (SyncBN stage 1)."""
    P, C, sp, sc = _pc(y)
    lib = L.lib()
    mom = torch.empty(3 * C, dtype=torch.float64, device=y.device)
    part = L.workspace(lib.rgan_bn_partial_bytes(P, C), y.device)
    L.check(lib.rgan_bn_moments(L.ptr(y), P, C, sp, sc, L.ptr(mom), L.ptr(part), L.stream()), "rgan_bn_moments")
    return mom


def bn_finalize(moments, nranks, C, eps, momentum, running_mean=None, running_var=None,
                num_batches_tracked=None, out=None):
    """Merge [nranks][3][C] moments in rank order -> stats float[2C] (SyncBN stage 2)."""
    stats = torch.empty(2 * C, dtype=torch.float32, device=moments.device) if out is None else out
    L.check(L.lib().rgan_bn_finalize(L.ptr(moments), int(nranks), C, float(eps), float(momentum),
                                     L.ptr(running_mean), L.ptr(running_var), L.ptr(num_batches_tracked),
                                     L.ptr(stats), L.stream()), "rgan_bn_finalize")
    return stats


def bn_backward_sums(da, y, stats, gamma, beta, act="none", alpha=0.0):
    if not is_nhwc(da):
        da = da.contiguous(memory_format=torch.channels_last)
    P, C, sp, sc = _pc(y)
    _, _, dsp, dsc = _pc(da)
    sums = torch.empty(2 * C, dtype=torch.float64, device=y.device)
    lib = L.lib()
    part = L.workspace(lib.rgan_bn_partial_bytes(P, C), y.device)
    L.check(lib.rgan_bn_backward_sums(L.ptr(da), dsp, dsc, L.ptr(y), P, C, sp, sc, L.ptr(stats), L.ptr(gamma),
                                      L.ptr(beta), L.ACT[act], float(alpha), L.ptr(sums), L.ptr(part),
                                      L.stream()), "rgan_bn_backward_sums")
    return sums, da


def bn_backward_apply(da, y, stats, gamma, beta, act, alpha, sums, P_global, need_affine=True, out=None):
    P, C, sp, sc = _pc(y)
    _, _, dsp, dsc = _pc(da)
    dy = torch.empty_like(y) if out is None else out
    if dy.stride() != y.stride():
        raise L.RganError("bn_backward_apply: out must have y's strides")
    dgamma = torch.empty(C, dtype=torch.float32, device=y.device) if need_affine and gamma is not None else None
    dbeta = torch.empty(C, dtype=torch.float32, device=y.device) if need_affine and beta is not None else None
    L.check(L.lib().rgan_bn_backward_apply(L.ptr(da), dsp, dsc, L.ptr(y), P, C, sp, sc, L.ptr(stats),
                                           L.ptr(gamma), L.ptr(beta), L.ACT[act], float(alpha), L.ptr(sums),
                                           int(P_global), L.ptr(dy), sp, sc, L.ptr(dgamma), L.ptr(dbeta),
                                           L.stream()), "rgan_bn_backward_apply")
    return dy, dgamma, dbeta


def bn_backward_sums_apply(da, y, stats, gamma, beta, act, alpha, add=None, out=None, dgamma=None, dbeta=None,
                           accumulate_affine=False):
    """(sums double[2C], dy) of act(BN(y))'s backward in one call (rgan_bn_backward_sums_apply:
    one launch for <= 2048 rows): sums as bn_backward_sums returns them, dy = BN-backward(da *
    act') + add; dgamma / dbeta (given buffers) written or, with accumulate_affine, added into.
    Dense NHWC da / y / out / add."""
    if not is_nhwc(da):
        da = da.contiguous(memory_format=torch.channels_last)
    P, C, _, _ = _pc(y)
    dy = torch.empty_like(y) if out is None else out
    if not is_nhwc(dy) or (add is not None and not is_nhwc(add)):
        raise L.RganError("bn_backward_sums_apply: out / add must be NHWC")
    sums = torch.empty(2 * C, dtype=torch.float64, device=y.device)
    lib = L.lib()
    part = L.workspace(lib.rgan_bn_partial_bytes(P, C), y.device)
    L.check(lib.rgan_bn_backward_sums_apply(L.ptr(da), L.ptr(y), P, C, L.ptr(stats), L.ptr(gamma), L.ptr(beta),
                                            L.ACT[act], float(alpha), L.ptr(add), L.ptr(dy), L.ptr(dgamma),
                                            L.ptr(dbeta), int(bool(accumulate_affine)), L.ptr(sums), L.ptr(part),
                                            L.stream()), "rgan_bn_backward_sums_apply")
    return sums, dy


def bn_affine_grads(sums, stats, C, dgamma=None, dbeta=None, accumulate=False):
    """dgamma / dbeta (given buffers) from BatchNorm backward sums [2][C] (rgan_bn_affine_grads):
    written, or added into with ``accumulate``."""
    L.check(L.lib().rgan_bn_affine_grads(L.ptr(sums), L.ptr(stats), int(C), L.ptr(dgamma), L.ptr(dbeta),
                                         int(bool(accumulate)), L.stream()), "rgan_bn_affine_grads")


def bn_segment_stats_n(part, S, nseg, C, eps, momentum, running_mean, running_var, num_batches_tracked, out):
    """bn_segment_stats of the nseg equal batch segments of [0, S) in one launch: out[nseg][2C],
    running statistics updated in segment order."""
    L.check(L.lib().rgan_bn_segment_stats_n(L.ptr(part), 0, int(S), int(nseg), C, 64, float(eps), float(momentum),
                                            L.ptr(running_mean), L.ptr(running_var), L.ptr(num_batches_tracked),
                                            L.ptr(out), L.stream()), "rgan_bn_segment_stats_n")
    return out


def bn_segment_apply(part, S, y, eps, momentum, running_mean, running_var, num_batches_tracked, gamma, beta, act,
                     alpha, stats, out):
    """bn_segment_stats_n + bn_apply_segments in one call (rgan_bn_segment_apply): nseg =
    stats.shape[0] equal batch segments of y (dense NHWC, 16-byte aligned) and of conv_fwd_bn's
    S segment sums; one launch for small layers."""
    P, C, _, _ = _pc(y)
    L.check(L.lib().rgan_bn_segment_apply(L.ptr(part), int(S), int(stats.shape[0]), 64, L.ptr(y), P, C, float(eps),
                                          float(momentum), L.ptr(running_mean), L.ptr(running_var),
                                          L.ptr(num_batches_tracked), L.ptr(gamma), L.ptr(beta), L.ACT[act],
                                          float(alpha), L.ptr(stats), L.ptr(out), L.stream()),
            "rgan_bn_segment_apply")
    return out


def bn_apply_segments(y, stats, gamma, beta, act, alpha, out):
    """bn_apply of y's nseg = stats.shape[0] equal batch segments, each with its stats row,
    in one launch (dense NHWC y and out)."""
    P, C, _, _ = _pc(y)
    L.check(L.lib().rgan_bn_apply_segments(L.ptr(y), P, C, stats.shape[0], L.ptr(stats), L.ptr(gamma), L.ptr(beta),
                                           L.ACT[act], float(alpha), L.ptr(out), L.stream()),
            "rgan_bn_apply_segments")
    return out


def bn_backward_segments(da, y, stats, gamma, beta, act, alpha, need_gamma, need_beta, out):
    """bn_backward of y's nseg = stats.shape[0] equal batch segments in one set of launches
    (dense NHWC da, y, out); dgamma / dbeta summed over the segments."""
    P, C, _, _ = _pc(y)
    nseg = stats.shape[0]
    dgamma = torch.empty(C, dtype=torch.float32, device=y.device) if need_gamma and gamma is not None else None
    dbeta = torch.empty(C, dtype=torch.float32, device=y.device) if need_beta and beta is not None else None
    lib = L.lib()
    ws = L.workspace(nseg * lib.rgan_bn_partial_bytes(P // nseg, C), y.device)
    L.check(lib.rgan_bn_backward_segments(L.ptr(da), L.ptr(y), P, C, nseg, L.ptr(stats), L.ptr(gamma), L.ptr(beta),
                                          L.ACT[act], float(alpha), L.ptr(out), L.ptr(dgamma), L.ptr(dbeta),
                                          L.ptr(ws), L.stream()), "rgan_bn_backward_segments")
    return out, dgamma, dbeta


def bn_backward_parts(g, y, stats, gamma, beta, post, need_gamma, need_beta, out=None):
    """dy (and dgamma / dbeta summed over the batch segments) from g = da * act' and the
    segment sums a GEMM's post-op wrote (Post mode 2, post.fused): merge + apply."""
    P, C, _, _ = _pc(y)
    nseg = post.nseg
    if stats.dim() == 1:
        stats = stats.view(1, -1)
    dy = torch.empty_like(y) if out is None else out
    dgamma = torch.empty(C, dtype=torch.float32, device=y.device) if need_gamma and gamma is not None else None
    dbeta = torch.empty(C, dtype=torch.float32, device=y.device) if need_beta and beta is not None else None
    sums = torch.empty((nseg, 2, C), dtype=torch.float64, device=y.device)
    L.check(L.lib().rgan_bn_backward_parts(L.ptr(g), L.ptr(y), P, C, nseg, L.ptr(stats), L.ptr(gamma), L.ptr(beta),
                                           L.ptr(post.part), int(post.S), int(post.phases), L.ptr(dy),
                                           L.ptr(dgamma), L.ptr(dbeta), L.ptr(sums), L.stream()),
            "rgan_bn_backward_parts")
    return dy, dgamma, dbeta


def bn_apply(y, stats, gamma, beta, act="none", alpha=0.0, out=None):
    P, C, sp, sc = _pc(y)
    if out is None:
        out = torch.empty_like(y)
    Pa, Ca, asp, asc = _pc(out)
    L.check(L.lib().rgan_bn_apply(L.ptr(y), P, C, sp, sc, L.ptr(stats), L.ptr(gamma), L.ptr(beta), L.ACT[act],
                                  float(alpha), L.ptr(out), asp, asc, L.stream()), "rgan_bn_apply")
    return out


def bn_backward(da, y, stats, gamma, beta, act="none", alpha=0.0, need_affine=True, out=None):
    if not is_nhwc(da):
        da = da.contiguous(memory_format=torch.channels_last)
    P, C, sp, sc = _pc(y)
    _, _, dsp, dsc = _pc(da)
    dy = torch.empty_like(y) if out is None else out
    if dy.stride() != y.stride():
        raise L.RganError("bn_backward: out must have y's strides")
    dgamma = torch.empty(C, dtype=torch.float32, device=y.device) if need_affine and gamma is not None else None
    dbeta = torch.empty(C, dtype=torch.float32, device=y.device) if need_affine and beta is not None else None
    lib = L.lib()
    part = L.workspace(lib.rgan_bn_partial_bytes(P, C), y.device)
    L.check(lib.rgan_bn_backward(L.ptr(da), dsp, dsc, L.ptr(y), P, C, sp, sc, L.ptr(stats), L.ptr(gamma),
                                 L.ptr(beta), L.ACT[act], float(alpha), L.ptr(dy), sp, sc, L.ptr(dgamma),
                                 L.ptr(dbeta), L.ptr(part), L.stream()), "rgan_bn_backward")
    return dy, dgamma, dbeta


def bn_backward_apply_ex(da, y, stats, gamma, beta, act, alpha, sums, P_global, add=None, out=None,
                         dgamma=None, dbeta=None, accumulate_affine=False):
    """dy = BN-backward(da * act') + add; dgamma/dbeta (given buffers) written or, with
    accumulate_affine, added into."""
    if not is_nhwc(da):
        da = da.contiguous(memory_format=torch.channels_last)
    P, C, sp, sc = _pc(y)
    _, _, dsp, dsc = _pc(da)
    dy = torch.empty_like(y) if out is None else out
    if dy.stride() != y.stride() or (add is not None and add.stride() != y.stride()):
        raise L.RganError("bn_backward_apply_ex: out / add must have y's strides")
    L.check(L.lib().rgan_bn_backward_apply_ex(L.ptr(da), dsp, dsc, L.ptr(y), P, C, sp, sc, L.ptr(stats),
                                              L.ptr(gamma), L.ptr(beta), L.ACT[act], float(alpha), L.ptr(sums),
                                              int(P_global), L.ptr(add), L.ptr(dy), sp, sc, L.ptr(dgamma),
                                              L.ptr(dbeta), int(bool(accumulate_affine)), L.stream()),
            "rgan_bn_backward_apply_ex")
    return dy


def bn_dd_sums(a, y, dh, stats, gamma, beta, act, alpha, stage, stage1=None, P_global=0):
    """WGAN-GP double backward through BN+act: stage 1 -> double[3C], stage 2 -> double[2C]."""
    P, C, sp, sc = _pc(y)
    for t in (a, dh):
        if t.stride() != y.stride():
            raise L.RganError("bn_dd_sums: a, dh must have y's strides")
    lib = L.lib()
    out = torch.empty((3 if stage == 1 else 2) * C, dtype=torch.float64, device=y.device)
    part = L.workspace(lib.rgan_bn_dd_partial_bytes(P, C), y.device)
    L.check(lib.rgan_bn_dd_sums(L.ptr(a), L.ptr(y), L.ptr(dh), P, C, sp, sc, L.ptr(stats), L.ptr(gamma),
                                L.ptr(beta), L.ACT[act], float(alpha), int(stage), L.ptr(stage1), int(P_global),
                                L.ptr(out), L.ptr(part), L.stream()), "rgan_bn_dd_sums")
    return out


def bn_dd_apply(a, y, dh, stats, gamma, beta, act, alpha, first_sums, s1, s2, P_global, s1_local=None,
                s2_local=None, adj_dh=None, ydir=None, need_adj=True, dgamma2=None, dbeta2=None,
                accumulate_affine=False):
    """-> (adj_dh or None, ydir); dgamma2 / dbeta2 buffers written (or added into)."""
    P, C, sp, sc = _pc(y)
    if adj_dh is None and need_adj:
        adj_dh = torch.empty_like(y)
    if ydir is None:
        ydir = torch.empty_like(y)
    for t in (a, dh, ydir) + ((adj_dh,) if adj_dh is not None else ()):
        if t.stride() != y.stride():
            raise L.RganError("bn_dd_apply: tensors must share y's strides")
    L.check(L.lib().rgan_bn_dd_apply(L.ptr(a), L.ptr(y), L.ptr(dh), P, C, sp, sc, L.ptr(stats), L.ptr(gamma),
                                     L.ptr(beta), L.ACT[act], float(alpha), L.ptr(first_sums), L.ptr(s1),
                                     L.ptr(s2), L.ptr(s1_local), L.ptr(s2_local), int(P_global),
                                     L.ptr(adj_dh if need_adj else None), L.ptr(ydir), L.ptr(dgamma2),
                                     L.ptr(dbeta2), int(bool(accumulate_affine)), L.stream()), "rgan_bn_dd_apply")
    return (adj_dh if need_adj else None), ydir


def act_dd(a, act_out, dh, act, alpha, need_adj=True, need_ydir=False, adj_dh=None, ydir=None):
    """No-BN layer: (adj_dh = a act'(y) or None, ydir = a dh act''(y) or None)."""
    for t in (a, dh, adj_dh, ydir):
        if t is not None and t.stride() != act_out.stride():
            raise L.RganError("act_dd: a, act_out, dh and the outputs must share strides")
    if need_adj and adj_dh is None:
        adj_dh = torch.empty_like(act_out)
    if need_ydir and ydir is None:
        ydir = torch.empty_like(act_out)
    if not need_ydir:
        ydir = None
    L.check(L.lib().rgan_act_dd(L.ptr(a), L.ptr(act_out), L.ptr(dh), act_out.numel(), L.ACT[act], float(alpha),
                                L.ptr(adj_dh if need_adj else None), L.ptr(ydir), L.stream()), "rgan_act_dd")
    return (adj_dh if need_adj else None), ydir


def act_backward_ex(da, a, act, alpha=0.0, add=None, out=None):
    """dx = da * act'(a) + add."""
    if da.stride() != a.stride() or (add is not None and add.stride() != a.stride()):
        raise L.RganError("act_backward_ex: da, a, add must share strides")
    dx = torch.empty_like(a) if out is None else out
    L.check(L.lib().rgan_act_backward_ex(L.ptr(da), L.ptr(a), L.ptr(add), a.numel(), L.ACT[act], float(alpha),
                                         L.ptr(dx), L.stream()), "rgan_act_backward_ex")
    return dx


def act_backward(da, a, act, alpha=0.0):
    """dx = da * act'(x) from the activation output a (same strides required)."""
    if da.stride() != a.stride():
        da = da.contiguous(memory_format=torch.channels_last) if is_nhwc(a) else da.contiguous()
    dx = torch.empty_like(a)
    L.check(L.lib().rgan_act_backward(L.ptr(da), L.ptr(a), a.numel(), L.ACT[act], float(alpha), L.ptr(dx),
                                      L.stream()), "rgan_act_backward")
    return dx


def channel_sum(t, out, accumulate=False):
    """out[c] (+)= sum over (b, h, w) of t[:, c] (bias gradients), NHWC or [B, C, 1, 1]."""
    B, C, H, W = t.shape
    if is_nhwc(t):
        sp, sc = (t.stride()[0] if H * W == 1 else C), 1
    else:
        raise L.RganError("channel_sum expects NHWC (channels_last) input")
    part = L.workspace(L.lib().rgan_bn_partial_bytes(B * H * W, C), t.device)
    L.check(L.lib().rgan_channel_sum(L.ptr(t), B * H * W, C, sp, sc, L.ptr(out), int(bool(accumulate)),
                                     L.ptr(part), L.stream()), "rgan_channel_sum")
    return out


# ------------------------------------------------------------------ loss heads / GP
def loss_head(kind, side, r, f, need_dr=True, need_df=True, dr=None, df=None):
    t = r if r is not None else f
    n = t.numel()
    loss = torch.empty((), dtype=torch.float32, device=t.device)
    if dr is None:
        dr = torch.empty_like(r) if (r is not None and need_dr) else None
    if df is None:
        df = torch.empty_like(f) if (f is not None and need_df) else None
    L.check(L.lib().rgan_loss_head(int(kind), int(side), L.ptr(r), L.ptr(f), n, L.ptr(loss), L.ptr(dr),
                                   L.ptr(df), L.stream()), "rgan_loss_head")
    return loss, dr, df


def loss_head_pair(kind, r, f, need_dr=True, need_df=True, dr=None, df=None):
    """Heads 1-4 D side: (loss3 = [real, fake, sum], dr, df) in one launch."""
    loss3 = torch.empty(3, dtype=torch.float32, device=r.device)
    if dr is None and need_dr:
        dr = torch.empty_like(r)
    if df is None and need_df:
        df = torch.empty_like(f)
    L.check(L.lib().rgan_loss_head_pair(int(kind), L.ptr(r), L.ptr(f), r.numel(), L.ptr(loss3), L.ptr(dr),
                                        L.ptr(df), L.stream()), "rgan_loss_head_pair")
    return loss3, dr, df


def loss_head_joint(kind, y):
    """Heads 5-8, G side, on the joint [D(G(z)); D(x)] output: (loss, dy) with dy's second
    half zero (rgan_loss_head_joint)."""
    n = y.numel() // 2
    loss = torch.empty((), dtype=torch.float32, device=y.device)
    dy = torch.empty_like(y)
    L.check(L.lib().rgan_loss_head_joint(int(kind), L.ptr(y), n, L.ptr(loss), L.ptr(dy), L.stream()),
            "rgan_loss_head_joint")
    return loss, dy


def loss_head_dist(kind, side, phase, r, f, n_global, gsum=None, need_dr=True, need_df=True):
    t = r if r is not None else f
    n = t.numel()
    sums = torch.zeros(4, dtype=torch.float32, device=t.device)
    loss = torch.empty((), dtype=torch.float32, device=t.device)
    dr = torch.empty_like(r) if (phase == 2 and r is not None and need_dr) else None
    df = torch.empty_like(f) if (phase == 2 and f is not None and need_df) else None
    L.check(L.lib().rgan_loss_head_dist(int(kind), int(side), int(phase), L.ptr(r), L.ptr(f), n, int(n_global),
                                        L.ptr(gsum), L.ptr(sums), L.ptr(loss), L.ptr(dr), L.ptr(df), L.stream()),
            "rgan_loss_head_dist")
    return sums, loss, dr, df


def scale(t, s, out=None):
    if out is None:
        out = torch.empty_like(t)
    L.check(L.lib().rgan_scale(L.ptr(t), L.ptr(s), t.numel(), L.ptr(out), L.stream()), "rgan_scale")
    return out


def gp_interp(x, xf, u, out=None):
    B = x.shape[0]
    x = x.contiguous()
    xf = xf.contiguous()
    if out is None:
        out = torch.empty_like(x)
    elif not out.is_contiguous() or out.shape != x.shape:
        raise L.RganError("gp_interp: out must be contiguous and shaped like x")
    L.check(L.lib().rgan_gp_interp(L.ptr(x), L.ptr(xf), L.ptr(u.contiguous()), B, x[0].numel(), L.ptr(out),
                                   L.stream()), "rgan_gp_interp")
    return out


def gp_penalty(g, lam, n_global):
    g = g.contiguous()
    B = g.shape[0]
    norms = torch.empty(B, dtype=torch.float32, device=g.device)
    loss = torch.empty((), dtype=torch.float32, device=g.device)
    L.check(L.lib().rgan_gp_penalty(L.ptr(g), B, g[0].numel(), float(lam), int(n_global), L.ptr(norms),
                                    L.ptr(loss), L.stream()), "rgan_gp_penalty")
    return loss, norms, g


def gp_penalty_backward(g, norms, lam, n_global, gscale, out=None):
    """dGP/dg = gscale * lam * 2 (n_b - 1) / n_global * g / n_b per sample b.  ``out`` may be
    ``g`` itself (in place: each element is read before it is written)."""
    B = g.shape[0]
    if not g.is_contiguous():
        raise L.RganError("gp_penalty_backward: g must be contiguous")
    dg = torch.empty_like(g) if out is None else out
    if not dg.is_contiguous() or dg.shape != g.shape:
        raise L.RganError("gp_penalty_backward: out must be contiguous and shaped like g")
    L.check(L.lib().rgan_gp_penalty_backward(L.ptr(g), L.ptr(norms), B, g[0].numel(), float(lam), int(n_global),
                                             L.ptr(gscale), L.ptr(dg), L.stream()), "rgan_gp_penalty_backward")
    return dg


# ------------------------------------------------------------------ spectral norm
def sn_view(w, transposed):
    """(rows, cols, rs, hs, lo) of torch's reshape_weight_to_matrix (dim 0 conv, dim 1 convT)."""
    if w.dim() == 2:
        w = w.view(w.shape[0], w.shape[1], 1, 1)
    a, b, kh, kw = w.shape
    kk = kh * kw
    if transposed:  # [cin][cout][kh][kw] -> rows = cout
        return b, a * kk, kk, b * kk, kk
    return a, b * kk, b * kk, kk, kk


def spectral_power(w, u, v, transposed, eps=1e-12, do_iter=True):
    rows, cols, rs, hs, lo = sn_view(w, transposed)
    lib = L.lib()
    inv_sigma = torch.empty(1, dtype=torch.float32, device=w.device)
    ws = L.workspace(lib.rgan_spectral_ws_bytes(rows, cols), w.device)
    L.check(lib.rgan_spectral_power(L.ptr(w), rows, cols, rs, hs, lo, float(eps), L.ptr(u), L.ptr(v),
                                     L.ptr(inv_sigma), int(bool(do_iter)), L.ptr(ws), L.stream()),
            "rgan_spectral_power")
    return inv_sigma


def spectral_power_batch(layers, eps=1e-12):
    """One power iteration for every (w, u, v, transposed) of a net call, in four launches
    (rgan_spectral_power_batch): u, v updated in place; returns [(u_copy, v_copy, inv_sigma)]
    per layer (the copies autograd saves, as torch spectral_norm's clones)."""
    n = len(layers)
    if n == 0:
        return []
    if n > 16:
        raise L.RganError("spectral_power_batch: at most 16 layers per call")
    dev = layers[0][0].device
    arr = (L.RganSnLayer * n)()
    outs = []
    for i, (w, u, v, tr) in enumerate(layers):
        rows, cols, rs, hs, lo = sn_view(w, tr)
        uc, vc = torch.empty_like(u), torch.empty_like(v)
        inv = torch.empty(1, dtype=torch.float32, device=dev)
        arr[i] = L.RganSnLayer(w.data_ptr(), rows, cols, lo, rs, hs, u.data_ptr(), v.data_ptr(), uc.data_ptr(),
                               vc.data_ptr(), inv.data_ptr())
        outs.append((uc, vc, inv))
    lib = L.lib()
    ws = L.workspace(lib.rgan_spectral_batch_ws_bytes(n, ctypes.cast(arr, ctypes.c_void_p)), dev)
    L.check(lib.rgan_spectral_power_batch(n, ctypes.cast(arr, ctypes.c_void_p), float(eps), L.ptr(ws), L.stream()),
            "rgan_spectral_power_batch")
    return outs


def spectral_backward(w, dw_eff, u, v, inv_sigma, transposed, out=None):
    """dW_orig of W_eff = W / sigma(W) (u, v constant); ``out`` given: added into it."""
    rows, cols, rs, hs, lo = sn_view(w, transposed)
    acc = out is not None
    dw = out if acc else torch.empty_like(w)
    ws = L.workspace(4096, w.device)
    L.check(L.lib().rgan_spectral_backward(L.ptr(w), L.ptr(dw_eff), rows, cols, rs, hs, lo, L.ptr(u), L.ptr(v),
                                           L.ptr(inv_sigma), L.ptr(dw), int(acc), L.ptr(ws), L.stream()),
            "rgan_spectral_backward")
    return dw


# ------------------------------------------------------------------ device sampling
class DeviceRNG:
    """Counter-based device draws for --rgan_rng device (rgan_rng_fill / rgan_rng_choice):
    the counter is a device int64 the kernels advance, so graph replays draw fresh values."""

    def __init__(self, seed, device):
        self.seed = (int(seed) * 0x9E3779B97F4A7C15 + 0x632BE59BD9B4E019) & ((1 << 64) - 1)
        self.counter = torch.zeros(1, dtype=torch.int64, device=device)

    def normal(self, shape):
        out = torch.empty(shape, dtype=torch.float32, device=self.counter.device)
        L.check(L.lib().rgan_rng_fill(L.ptr(out), out.numel(), 0, self.seed, L.ptr(self.counter), L.stream()),
                "rgan_rng_fill")
        return out

    def uniform(self, shape):
        out = torch.empty(shape, dtype=torch.float32, device=self.counter.device)
        L.check(L.lib().rgan_rng_fill(L.ptr(out), out.numel(), 1, self.seed, L.ptr(self.counter), L.stream()),
                "rgan_rng_fill")
        return out

    def choice(self, N, n):
        """n distinct indices of [0, N) (numpy.random.choice(N, n, replace=False))."""
        out = torch.empty(n, dtype=torch.int64, device=self.counter.device)
        L.check(L.lib().rgan_rng_choice(L.ptr(out), int(N), int(n), self.seed, L.ptr(self.counter), L.stream()),
                "rgan_rng_choice")
        return out


# ------------------------------------------------------------------ Adam / data
def adam(params, grads, exp_avgs, exp_avg_sqs, hyper, step):
    n = len(params)
    arr = ctypes.c_void_p * max(n, 1)
    P = arr(*[p.data_ptr() for p in params])
    G = arr(*[g.data_ptr() for g in grads])
    M = arr(*[m.data_ptr() for m in exp_avgs])
    V = arr(*[v.data_ptr() for v in exp_avg_sqs])
    N = (ctypes.c_longlong * max(n, 1))(*[p.numel() for p in params])
    L.check(L.lib().rgan_adam(n, ctypes.cast(P, ctypes.c_void_p), ctypes.cast(G, ctypes.c_void_p),
                              ctypes.cast(M, ctypes.c_void_p), ctypes.cast(V, ctypes.c_void_p),
                              ctypes.cast(N, ctypes.c_void_p), L.ptr(hyper), L.ptr(step), L.stream()), "rgan_adam")


def adam_packed(params, grads, exp_avgs, exp_avg_sqs, hyper, step, layouts):
    """``adam`` that also writes the cached GEMM layouts ``layouts`` ([(param index, key,
    pack-cache entry)], _PackCache.layouts_of) from the updated values (rgan_adam_packed).
    ``step``: the count, a view whose next float is the group's arrival ticket (optim.Adam)."""
    if step.untyped_storage().nbytes() < 4 * (step.storage_offset() + 2):
        raise L.RganError("adam_packed: step must be followed by its arrival-ticket word (float[2] storage)")
    n = len(params)
    arr = ctypes.c_void_p * max(n, 1)
    P = arr(*[p.data_ptr() for p in params])
    G = arr(*[g.data_ptr() for g in grads])
    M = arr(*[m.data_ptr() for m in exp_avgs])
    V = arr(*[v.data_ptr() for v in exp_avg_sqs])
    N = (ctypes.c_longlong * max(n, 1))(*[p.numel() for p in params])
    k = len(layouts)
    packs = (L.RganAdamPack * max(k, 1))()
    for i, (j, _key, ent) in enumerate(layouts):
        packs[i] = L.RganAdamPack(j, ent[5], ctypes.pointer(ent[4]), ent[2].data_ptr())
    L.check(L.lib().rgan_adam_packed(n, ctypes.cast(P, ctypes.c_void_p), ctypes.cast(G, ctypes.c_void_p),
                                     ctypes.cast(M, ctypes.c_void_p), ctypes.cast(V, ctypes.c_void_p),
                                     ctypes.cast(N, ctypes.c_void_p), L.ptr(hyper), L.ptr(step), k,
                                     ctypes.cast(packs, ctypes.c_void_p), L.stream()), "rgan_adam_packed")


def lr_decay(hyper, gamma):
    L.check(L.lib().rgan_lr_decay(L.ptr(hyper), float(gamma), L.stream()), "rgan_lr_decay")


def gather_images(images, idx, out=None):
    """images[idx] as float32; a uint8 dataset (decoded images, relativisticgan_amd.data) is
    converted on the fly with ToTensor + Normalize(0.5, 0.5) (GLI:160-166)."""
    B = idx.numel()
    per = images[0].numel()
    if out is None:
        out = torch.empty((B,) + tuple(images.shape[1:]), dtype=torch.float32, device=images.device)
    if images.dtype == torch.uint8:
        L.check(L.lib().rgan_gather_images_u8(L.ptr(images), L.ptr(idx), B, per, L.ptr(out), L.stream()),
                "rgan_gather_images_u8")
        return out
    L.check(L.lib().rgan_gather_images(L.ptr(images), L.ptr(idx), B, per, L.ptr(out), L.stream()),
            "rgan_gather_images")
    return out


# ------------------------------------------------------------------ GEMM arithmetic
def set_gemm_emulation(on):
    """Run the FAST 128x128 forward / data-gradient conv GEMMs as fp32 emulated on the bf16 MFMA
    (bf16x6, see include/rgan.h) instead of the fp32 MFMA; returns the previous setting."""
    prev = L.lib().rgan_set_gemm_emulation(1 if on else 0)
    if prev < 0:
        raise L.RganError("rgan_set_gemm_emulation failed")
    return bool(prev)


# ------------------------------------------------------------------ live launch timing
def profile_begin(capacity=100000):
    L.check(L.lib().rgan_profile_begin(int(capacity)), "rgan_profile_begin")


def profile_end():
    """{'ms', 'flops', 'launches', 'kernels': [{name, ms, flops, launches}]} of the GEMM launches."""
    lib = L.lib()
    ms, fl, n = ctypes.c_double(), ctypes.c_double(), ctypes.c_longlong()
    L.check(lib.rgan_profile_end(ctypes.byref(ms), ctypes.byref(fl), ctypes.byref(n)), "rgan_profile_end")
    kern = []
    for i in range(256):
        name = ctypes.create_string_buffer(200)
        kms, kfl, kn = ctypes.c_double(), ctypes.c_double(), ctypes.c_longlong()
        if lib.rgan_profile_kernel(i, name, 200, ctypes.byref(kms), ctypes.byref(kfl), ctypes.byref(kn)) != 0:
            break  # past the last kernel id
        if kn.value:
            kern.append({"name": name.value.decode(), "ms": kms.value, "flops": kfl.value, "launches": kn.value,
                         "tflops": kfl.value / kms.value / 1e9 if kms.value > 0 else 0.0})
    return {"ms": ms.value, "flops": fl.value, "launches": n.value, "kernels": kern}
