"""Kernel-level numerics: every HIP kernel vs a plain PyTorch reference of the same op.

GPU-only (marked ``gpu``).  References are torch fp64 on the CPU for small shapes and
torch fp32 on the device (MIOpen/ATen) for the full-size layer shapes of BASELINE's
configs.  Tolerances are stated per test (fp32 accumulation over K terms).
"""
import math

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _rel(a, b):
    a = a.double().cpu()
    b = b.double().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


def _nhwc(t):
    return t.contiguous(memory_format=torch.channels_last)


@pytest.fixture(scope="module")
def K():
    from relativisticgan_amd import kernels
    return kernels


def _ref_conv(x, w, g, bias=None):
    x64, w64 = x.double().cpu(), w.double().cpu()
    b64 = bias.double().cpu() if bias is not None else None
    if g.transposed:
        return F.conv_transpose2d(x64, w64, b64, stride=g.stride, padding=g.pad)
    return F.conv2d(x64, w64, b64, stride=g.stride, padding=g.pad)


# (B, cin, cout, H, k, s, p, transposed)
SMALL = [
    (2, 8, 16, 16, 4, 2, 1, False),
    (3, 3, 8, 16, 4, 2, 1, False),      # first D layer, Cin=3 (scalar gather)
    (2, 16, 8, 8, 4, 2, 1, True),       # ConvT k4s2p1
    (2, 8, 3, 8, 4, 2, 1, True),        # last G layer, Cout=3
    (5, 16, 32, 1, 4, 1, 0, True),      # G start 1x1 -> 4x4
    (4, 64, 32, 1, 4, 1, 0, True),      # G start, Cin % 32 == 0: FAST loaders on a 1x1 image
    (5, 32, 1, 4, 4, 1, 0, False),      # D end 4x4 -> 1x1
    (2, 12, 20, 8, 3, 1, 1, False),     # arch-1 3x3
    (2, 64, 128, 8, 4, 2, 1, False),
    (2, 128, 64, 4, 4, 2, 1, True),
    (7, 20, 36, 10, 4, 2, 1, False),    # ragged sizes
    (2, 32, 64, 16, 4, 2, 1, False),    # FAST WGRAD, Cin = 32: four taps per 128-wide n tile
    (2, 64, 32, 16, 4, 2, 1, True),     # ConvT WGRAD over a 32-channel dy: four taps per tile
    (3, 64, 128, 16, 4, 2, 1, False),   # two taps per tile
]


@pytest.mark.parametrize("case", SMALL)
@pytest.mark.parametrize("layout", ["nhwc", "nchw"])
def test_conv_fwd_dgrad_wgrad_small(K, case, layout):
    B, cin, cout, H, k, s, p, tr = case
    g = K.ConvGeom(k, s, p, tr)
    torch.manual_seed(0)
    x = torch.randn(B, cin, H, H, device=DEV)
    w = torch.randn((cin, cout, k, k) if tr else (cout, cin, k, k), device=DEV) * 0.1
    if layout == "nhwc":
        x = _nhwc(x)
    y = K.conv_fwd(x, w, g)
    ref = _ref_conv(x, w, g)
    assert y.shape == ref.shape
    assert _rel(y, ref) < 2e-6
    dy = torch.randn_like(ref, dtype=torch.float32).to(DEV)
    if layout == "nhwc":
        dy = _nhwc(dy)
    x64 = x.double().cpu().requires_grad_(True)
    w64 = w.double().cpu().requires_grad_(True)
    out64 = (F.conv_transpose2d if tr else F.conv2d)(x64, w64, stride=s, padding=p)
    out64.backward(dy.double().cpu())
    dx = K.conv_dgrad(dy, w, g, x.shape)
    assert _rel(dx, x64.grad) < 2e-6
    dw, _ = K.conv_wgrad(x, dy, g, w.shape)
    assert _rel(dw, w64.grad) < 2e-6


@pytest.mark.parametrize("case", [(32, 128, 128, 16, 4, 2, 1, False), (32, 256, 128, 8, 4, 2, 1, True),
                                  (32, 128, 256, 8, 3, 1, 1, False), (32, 64, 64, 32, 4, 2, 1, False),
                                  (32, 128, 64, 8, 4, 2, 1, True)])
def test_small_gemm_tiles(K, case):
    """Arch 1's small GEMMs (< 4 GFLOP that would split K 4+ ways on 128x128 tiles, or with
    N <= 64) run on smaller tiles with fewer splits (conv_gemm.hip choose_tiling): the forward
    and data gradient on 64x64 tiles, the weight gradient on 128x64 (64x64 for <= 64 output
    channels) -- vs torch fp64, and those kernels are the ones that ran."""
    B, cin, cout, H, k, s, p, tr = case
    g = K.ConvGeom(k, s, p, tr)
    torch.manual_seed(3)
    x = _nhwc(torch.randn(B, cin, H, H, device=DEV))
    w = torch.randn((cin, cout, k, k) if tr else (cout, cin, k, k), device=DEV) * 0.05
    x64 = x.double().cpu().requires_grad_(True)
    w64 = w.double().cpu().requires_grad_(True)
    out64 = (F.conv_transpose2d if tr else F.conv2d)(x64, w64, stride=s, padding=p)
    dy = _nhwc(torch.randn(out64.shape, device=DEV))
    out64.backward(dy.double().cpu())

    def gemm_names(fn):
        K.profile_begin(64)
        out = fn()
        return out, [kk["name"] for kk in K.profile_end()["kernels"] if "gemm_kernel" in kk["name"]]

    y, fwd = gemm_names(lambda: K.conv_fwd(x, w, g))
    dx = K.conv_dgrad(dy, w, g, x.shape, like=x)  # tiling depends on its own K (not asserted)
    (dw, _), wgr = gemm_names(lambda: K.conv_wgrad(x, dy, g, tuple(w.shape)))
    assert len(fwd) == 1 and "64, 64, 2, 2" in fwd[0], fwd
    # the weight gradient's M: w.shape[0] (Conv2d: output channels, ConvT: input channels)
    wtile = "64, 64, 2, 2" if w.shape[0] <= 64 else "128, 64, 2, 2"
    assert len(wgr) == 1 and wtile in wgr[0], wgr
    assert _rel(y, out64.detach()) < 2e-6
    assert _rel(dx, x64.grad) < 2e-6
    assert _rel(dw, w64.grad) < 2e-6


@pytest.mark.parametrize("case", [(2, 16, 8, 4), (3, 8, 3, 8), (2, 32, 64, 8), (2, 5, 7, 6), (2, 64, 32, 16)])
@pytest.mark.parametrize("cached", [False, True])
def test_nn_conv_upsample_fold(K, case, cached):
    """--NN_conv: Upsample(x2)+Conv2d(k3,s1,p1)+bias (GLI:351-356,377-382) as one folded
    k4 s2 p1 transposed conv; fwd/dgrad/wgrad/dbias vs torch fp64 interpolate+conv2d."""
    B, cin, cout, H = case
    g = K.ConvGeom(3, 1, 1, False, 2)
    torch.manual_seed(1)
    x = _nhwc(torch.randn(B, cin, H, H, device=DEV))
    w = (torch.randn(cout, cin, 3, 3, device=DEV) * 0.1).requires_grad_(False)
    b = torch.randn(cout, device=DEV)
    x64 = x.double().cpu().requires_grad_(True)
    w64 = w.double().cpu().requires_grad_(True)
    b64 = b.double().cpu().requires_grad_(True)
    ref = F.conv2d(F.interpolate(x64, scale_factor=2, mode="nearest"), w64, b64, padding=1)
    y = K.conv_fwd(x, w, g, bias=b, cache=cached)
    assert y.shape == ref.shape
    assert _rel(y, ref.detach()) < 3e-6
    dy = _nhwc(torch.randn(ref.shape, device=DEV))
    ref.backward(dy.double().cpu())
    dx = K.conv_dgrad(dy, w, g, tuple(x.shape), cache=cached)
    assert _rel(dx, x64.grad) < 3e-6
    dw, db = K.conv_wgrad(x, dy, g, tuple(w.shape), with_bias=True)
    assert dw.shape == w.shape
    assert _rel(dw, w64.grad) < 3e-6
    assert _rel(db, b64.grad) < 1e-6
    if cached:  # second call reuses the folded weight; an in-place update must refold
        w.mul_(0.5)
        y2 = K.conv_fwd(x, w, g, bias=b, cache=True)
        ref2 = F.conv2d(F.interpolate(x.double().cpu(), scale_factor=2), w.double().cpu(), b.double().cpu(), padding=1)
        assert _rel(y2, ref2) < 3e-6


def test_conv_bias_act(K):
    g = K.ConvGeom(3, 1, 1, False)
    x = _nhwc(torch.randn(2, 12, 8, 8, device=DEV))
    w = torch.randn(20, 12, 3, 3, device=DEV) * 0.1
    b = torch.randn(20, device=DEV)
    for act, fn in [("lrelu", lambda t: F.leaky_relu(t, 0.1)), ("relu", F.relu), ("tanh", torch.tanh),
                    ("sigmoid", torch.sigmoid), ("selu", F.selu)]:
        y = K.conv_fwd(x, w, g, bias=b, act=act, alpha=0.1)
        assert _rel(y, fn(_ref_conv(x, w, g, b))) < 3e-6, act
    dy = _nhwc(torch.randn(2, 20, 8, 8, device=DEV))
    _, db = K.conv_wgrad(x, dy, g, w.shape, with_bias=True)
    assert _rel(db, dy.double().sum((0, 2, 3))) < 1e-6


# arch 1's Conv2d layers with a bias (GLI:202-223, 260-302) at the C4 bench shapes (2B = 64):
# FAST weight gradients, split-K and unsplit, 128 x 128 and 128 x 64 tiles
WGRAD_BIAS = [(64, 64, 128, 16, 3, 1, 1), (64, 64, 64, 32, 4, 2, 1), (64, 256, 512, 4, 3, 1, 1),
              (64, 128, 256, 8, 3, 1, 1), (2, 64, 128, 4, 3, 1, 1), (8, 128, 128, 32, 4, 2, 1),
              (64, 3, 64, 32, 3, 1, 1)]  # arch 1's image input layer (N = 27: the 64 x 64 tile, round 6)


@pytest.mark.parametrize("case", WGRAD_BIAS)
def test_conv_wgrad_fused_bias(K, case):
    """The bias gradient a FAST Conv2d weight-gradient GEMM forms from its staged dy tiles
    (GemmArgs::dbias: unsplit written directly, split summed by the WGRAD reduce in split
    order), written and accumulated, vs torch fp64 -- and the weight gradient beside it."""
    B, cin, cout, H, k, s, p = case
    g = K.ConvGeom(k, s, p, False)
    torch.manual_seed(cin + cout + H)
    x = _nhwc(torch.randn(B, cin, H, H, device=DEV))
    Ho = (H + 2 * p - k) // s + 1
    dy = _nhwc(torch.randn(B, cout, Ho, Ho, device=DEV))
    w_shape = (cout, cin, k, k)
    x64 = x.double().requires_grad_(True)
    w64 = torch.zeros(w_shape, dtype=torch.float64, device=DEV, requires_grad=True)
    b64 = torch.zeros(cout, dtype=torch.float64, device=DEV, requires_grad=True)
    with torch.backends.cudnn.flags(enabled=False):
        F.conv2d(x64, w64, b64, stride=s, padding=p).backward(dy.double())
    dw, db = K.conv_wgrad(x, dy, g, w_shape, with_bias=True)
    assert _rel(dw, w64.grad) < 1e-5
    assert _rel(db, b64.grad) < 1e-6
    # accumulation into existing gradients (autograd's second backward of heads 1-4 / WGAN-GP)
    dw0, db0 = torch.randn_like(dw), torch.randn_like(db)
    dwa, dba = dw0.clone(), db0.clone()
    K.conv_wgrad(x, dy, g, w_shape, with_bias=True, out=dwa, out_bias=dba)
    assert _rel(dwa, dw0.double() + w64.grad) < 1e-5
    assert _rel(dba, db0.double() + b64.grad) < 1e-6
    # bias over the second half of the batch only (rgan_conv_wgrad_rows: the GP engine's
    # [adjoint; forward] pairs), fused where the row offset is tile-aligned, else the
    # channel-sum fallback; the weight gradient still over every row
    if B >= 2:
        row0 = (B // 2) * Ho * Ho
        dwr, dbr = dw0.clone(), db0.clone()
        K.conv_wgrad(x, dy, g, w_shape, with_bias=True, out=dwr, out_bias=dbr, bias_row0=row0)
        assert _rel(dwr, dw0.double() + w64.grad) < 1e-5
        assert _rel(dbr, db0.double() + dy[B // 2:].double().sum((0, 2, 3))) < 1e-6


@pytest.mark.parametrize("case", [(64, 2048, 4, "nhwc"), (3, 20, 5, "nhwc"), (5, 7, 3, "nchw"), (1, 1, 1, "nchw")])
def test_conv_dense_one_output(K, case):
    """D's closing Conv2d(C, 1, k, 1, 0) over a k x k map (dense1 kernels): fwd with bias,
    wscale and activation, dgrad with wscale, wgrad + dbias, vs torch fp64."""
    B, C, k, layout = case
    g = K.ConvGeom(k, 1, 0, False)
    torch.manual_seed(k)
    x = torch.randn(B, C, k, k, device=DEV)
    if layout == "nhwc":
        x = _nhwc(x)
    w = torch.nn.Parameter(torch.randn(1, C, k, k, device=DEV) * 0.1)
    b = torch.randn(1, device=DEV)
    ws = torch.tensor([0.7], device=DEV)
    ref = F.conv2d(x.double().cpu(), w.detach().double().cpu() * 0.7, b.double().cpu())
    for act, fn in [("none", lambda t: t), ("sigmoid", torch.sigmoid), ("lrelu", lambda t: F.leaky_relu(t, 0.2))]:
        for cache in (False, True):
            y = K.conv_fwd(x, w, g, bias=b, act=act, alpha=0.2, wscale=ws, cache=cache)
            assert y.shape == (B, 1, 1, 1)
            assert _rel(y, fn(ref)) < 3e-6, (act, cache)
    dy = torch.randn(B, 1, 1, 1, device=DEV)
    x64 = x.double().cpu().requires_grad_(True)
    w64 = w.detach().double().cpu().requires_grad_(True)
    F.conv2d(x64, w64).backward(dy.double().cpu())
    dx = K.conv_dgrad(dy, w, g, x.shape, wscale=ws, like=x)
    assert dx.stride() == x.stride()
    assert _rel(dx, x64.grad * 0.7) < 2e-6
    dw, db = K.conv_wgrad(x, dy, g, w.shape, with_bias=True)
    assert _rel(dw, w64.grad) < 2e-6
    assert _rel(db, dy.double().cpu().sum((0, 2, 3))) < 1e-6


@pytest.mark.parametrize("B,C,N", [(32, 128, 8192), (1, 4, 256), (64, 100, 300), (7, 512, 1024), (33, 20, 260)])
def test_conv_dense_wide(K, B, C, N):
    """A wide dense layer as a 1x1 conv over a 1x1 map (arch 1's G input Linear, GLI:205-207: the
    GEMM's 64x64 tiles for the thin-M forward and the K <= 64 weight gradient): fwd with bias,
    wscale and activation, wgrad + dbias (written, accumulated, the bias over a row range),
    through a weight view as arch 1 calls it, vs torch fp64; ragged N and B."""
    g = K.ConvGeom(1, 1, 0, False)
    torch.manual_seed(B + C)
    x = torch.randn(B, C, 1, 1, device=DEV)
    p = torch.nn.Parameter(torch.randn(N, C, device=DEV) * 0.05)
    w = p.view(N, C, 1, 1)
    b = torch.randn(N, device=DEV)
    ws = torch.tensor([0.7], device=DEV)
    ref = F.conv2d(x.double().cpu(), w.detach().double().cpu() * 0.7, b.double().cpu())
    for act, fn in [("none", lambda t: t), ("relu", F.relu), ("lrelu", lambda t: F.leaky_relu(t, 0.2))]:
        y = K.conv_fwd(x, w, g, bias=b, act=act, alpha=0.2, wscale=ws, cache=True)
        assert y.shape == (B, N, 1, 1)
        assert _rel(y, fn(ref)) < 3e-6, act
    dy = torch.randn(B, N, 1, 1, device=DEV)
    w64 = w.detach().double().cpu().requires_grad_(True)
    b64 = torch.zeros(N, dtype=torch.float64, requires_grad=True)
    F.conv2d(x.double().cpu(), w64, b64).backward(dy.double().cpu())
    dw, db = K.conv_wgrad(x, dy, g, w.shape, with_bias=True)
    assert _rel(dw, w64.grad) < 2e-6
    assert _rel(db, b64.grad) < 1e-6
    dw0, db0 = torch.randn(N, C, 1, 1, device=DEV), torch.randn(N, device=DEV)
    dwa, dba = dw0.clone(), db0.clone()
    K.conv_wgrad(x, dy, g, w.shape, with_bias=True, out=dwa, out_bias=dba)
    assert _rel(dwa, dw0.double().cpu() + w64.grad) < 1e-5
    assert _rel(dba, db0.double().cpu() + b64.grad) < 1e-6
    if B >= 2:  # bias over rows [B/2, B) (rgan_conv_wgrad_rows)
        dwr, dbr = dw0.clone(), db0.clone()
        K.conv_wgrad(x, dy, g, w.shape, with_bias=True, out=dwr, out_bias=dbr, bias_row0=B // 2)
        assert _rel(dwr, dw0.double().cpu() + w64.grad) < 1e-5
        assert _rel(dbr, db0.double().cpu() + dy[B // 2:].double().cpu().sum((0, 2, 3))) < 1e-6


@pytest.mark.parametrize("C", [1, 3, 4])
@pytest.mark.parametrize("layout", ["nchw", "nhwc"])
def test_image_layer_patches(K, C, layout):
    """Patch matrix X[(b,i,j)][4t+c] of a k4 s2 p1 window vs torch unfold, and the image
    layers run as 1x1 GEMMs over it (conv fwd / wgrad, convT dgrad / wgrad) vs torch fp64."""
    torch.manual_seed(C)
    img = torch.randn(3, C, 10, 12, device=DEV)
    if layout == "nhwc":
        img = _nhwc(img)
    X = K.patches_k4s2(img)
    assert X.shape == (3, 64, 5, 6) and K.is_nhwc(X)
    cols = F.unfold(img.double().cpu(), 4, padding=1, stride=2)          # [B, C*16, 30], (c, t)
    ref = cols.view(3, C, 16, 30).permute(0, 3, 2, 1)                   # [B, p, t, c]
    got = X.double().cpu().permute(0, 2, 3, 1).reshape(3, 30, 16, 4)    # [B, p, t, 4]
    assert torch.equal(got[..., :C], ref)
    assert not got[..., C:].any()
    # D's first conv as a 1x1 GEMM over X, and its weight gradient
    g = K.ConvGeom(4, 2, 1, False)
    w = torch.nn.Parameter(torch.randn(40, C, 4, 4, device=DEV) * 0.1)
    y = K.conv_fwd(X, K.patch_weight(w, False), K.G1X1)
    assert _rel(y, _ref_conv(img, w, g)) < 2e-6
    dy = _nhwc(torch.randn(3, 40, 5, 6, device=DEV))
    g1, _ = K.conv_wgrad(X, dy, K.G1X1, (40, 64, 1, 1))
    x64 = img.double().cpu()
    w64 = w.detach().double().cpu().requires_grad_(True)
    F.conv2d(x64, w64, stride=2, padding=1).backward(dy.double().cpu())
    assert _rel(K.unpatch_grad(g1, 40, C, 64, 1), w64.grad) < 2e-6
    # G's last convT: x [3, 40, 5, 6] -> image [3, C, 10, 12]; gradients over Xg = patches(dimg)
    gt = K.ConvGeom(4, 2, 1, True)
    wt = torch.randn(40, C, 4, 4, device=DEV) * 0.1
    x = _nhwc(torch.randn(3, 40, 5, 6, device=DEV))
    dimg = torch.randn(3, C, 10, 12, device=DEV)
    Xg = K.patches_k4s2(dimg)
    xr = x.double().cpu().requires_grad_(True)
    wr = wt.double().cpu().requires_grad_(True)
    F.conv_transpose2d(xr, wr, stride=2, padding=1).backward(dimg.double().cpu())
    assert _rel(K.conv_fwd(Xg, K.patch_weight(wt, True), K.G1X1), xr.grad) < 2e-6
    g1, _ = K.conv_wgrad(Xg, x, K.G1X1, (40, 64, 1, 1))
    assert _rel(K.unpatch_grad(g1, 40, C, 64, 1), wr.grad) < 2e-6


@pytest.mark.parametrize("B", [32, 64])
def test_image_layer_wgrad_full_size(K, B):
    """The image layers' weight gradients at the C1 shapes (64x64 RGB, 128 channels): a
    128 x 64 patch-GEMM output split-K hundreds of ways, reduced by the 16-lane split reduce
    (splitk_reduce_wide) -- vs torch fp64."""
    torch.manual_seed(B)
    img = _nhwc(torch.randn(B, 3, 64, 64, device=DEV))
    dy = _nhwc(torch.randn(B, 128, 32, 32, device=DEV))
    X = K.patches_k4s2(img)
    g1, _ = K.conv_wgrad(X, dy, K.G1X1, (128, 64, 1, 1))
    w64 = torch.zeros(128, 3, 4, 4, dtype=torch.float64, requires_grad=True)
    F.conv2d(img.double().cpu(), w64, stride=2, padding=1).backward(dy.double().cpu())
    assert _rel(K.unpatch_grad(g1, 128, 3, 64, 1), w64.grad) < 2e-6
    # G's last ConvTranspose2d (128 -> 3, 32x32 -> 64x64): dW over the image gradient's patches
    x = _nhwc(torch.randn(B, 128, 32, 32, device=DEV))
    dimg = torch.randn(B, 3, 64, 64, device=DEV)
    g1, _ = K.conv_wgrad(K.patches_k4s2(dimg), x, K.G1X1, (128, 64, 1, 1))
    wr = torch.zeros(128, 3, 4, 4, dtype=torch.float64, requires_grad=True)
    F.conv_transpose2d(x.double().cpu(), wr, stride=2, padding=1).backward(dimg.double().cpu())
    assert _rel(K.unpatch_grad(g1, 128, 3, 64, 1), wr.grad) < 2e-6


@pytest.mark.parametrize("nc", [1, 2, 3, 4])
def test_conv_narrow_paths(K, nc):
    """Narrow kernels: ConvT k4s2p1 with nc outputs (and the Conv2d dgrad of that shape),
    Conv2d with nc inputs; bias / activation / wscale epilogue and the cached pack."""
    torch.manual_seed(nc)
    gt, gc = K.ConvGeom(4, 2, 1, True), K.ConvGeom(4, 2, 1, False)
    x = _nhwc(torch.randn(3, 16, 6, 6, device=DEV))
    w = torch.nn.Parameter(torch.randn(16, nc, 4, 4, device=DEV) * 0.1)
    b = torch.randn(nc, device=DEV)
    s = torch.tensor([0.5], device=DEV)
    for cache in (False, True, True):
        y = K.conv_fwd(x, w, gt, bias=b, act="tanh", wscale=s, nchw_out=True, cache=cache)
        assert _rel(y, torch.tanh(_ref_conv(x, w * 0.5, gt, b))) < 3e-6
    # few tiles: the channel sum split over blocks (5 splits, the last one 8 channels) + reduce
    x2 = _nhwc(torch.randn(2, 72, 10, 10, device=DEV))
    w2 = torch.randn(72, nc, 4, 4, device=DEV) * 0.1
    for cache in (False, True):
        y = K.conv_fwd(x2, w2, gt, bias=b, act="tanh", wscale=s, nchw_out=True, cache=cache)
        assert _rel(y, torch.tanh(_ref_conv(x2, w2 * 0.5, gt, b))) < 3e-6
    # the ConvT's dgrad (a Conv2d over the nc-channel image: narrow-in kernel), NCHW image grad
    gy = torch.randn(3, nc, 12, 12, device=DEV)
    x64 = x.double().cpu().requires_grad_(True)
    F.conv_transpose2d(x64, (w * 0.5).detach().double().cpu(), stride=2, padding=1).backward(gy.double().cpu())
    for cache in (False, True):
        assert _rel(K.conv_dgrad(gy, w, gt, x.shape, wscale=s, cache=cache), x64.grad) < 3e-6
    img = torch.randn(3, nc, 12, 12, device=DEV)
    wc = torch.nn.Parameter(torch.randn(40, nc, 4, 4, device=DEV) * 0.1)
    bc = torch.randn(40, device=DEV)
    for cache in (False, True):
        y = K.conv_fwd(img, wc, gc, bias=bc, act="lrelu", alpha=0.2, wscale=s, cache=cache)
        assert _rel(y, F.leaky_relu(_ref_conv(img, wc * 0.5, gc, bc), 0.2)) < 3e-6
        if nc == 3:  # > 128 output channels: several channel tiles, the last one partial
            wc2 = torch.randn(200, nc, 4, 4, device=DEV) * 0.1
            y2 = K.conv_fwd(img, wc2, gc, act="lrelu", alpha=0.2)
            assert _rel(y2, F.leaky_relu(_ref_conv(img, wc2, gc), 0.2)) < 3e-6
        dy = _nhwc(torch.randn(3, 40, 6, 6, device=DEV))
        dx = K.conv_dgrad(dy, wc, gc, img.shape, wscale=s, like=img, cache=cache)
        x64 = img.double().cpu().requires_grad_(True)
        F.conv2d(x64, (wc * 0.5).double().cpu(), stride=2, padding=1).backward(dy.double().cpu())
        assert _rel(dx, x64.grad) < 3e-6


def test_conv_wscale(K):
    g = K.ConvGeom(4, 2, 1, False)
    x = _nhwc(torch.randn(2, 8, 8, 8, device=DEV))
    w = torch.randn(16, 8, 4, 4, device=DEV)
    s = torch.tensor([0.25], device=DEV)
    assert _rel(K.conv_fwd(x, w, g, wscale=s), _ref_conv(x, w * 0.25, g)) < 2e-6
    dy = _nhwc(torch.randn(2, 16, 4, 4, device=DEV))
    dx = K.conv_dgrad(dy, w, g, x.shape, wscale=s)
    dx_ref = K.conv_dgrad(dy, w * 0.25, g, x.shape)
    assert _rel(dx, dx_ref) < 1e-6


# full-size layer shapes of C2 (RaSGAN 128^2, B=64, h=128): a few representative ones
BIG = [
    (64, 128, 256, 64, 4, 2, 1, False),
    (64, 1024, 2048, 8, 4, 2, 1, False),
    (64, 2048, 1024, 4, 4, 2, 1, True),
    (64, 256, 128, 32, 4, 2, 1, True),
    (64, 128, 3, 64, 4, 2, 1, True),
    (64, 3, 128, 128, 4, 2, 1, False),
    (64, 128, 2048, 1, 4, 1, 0, True),
    (64, 2048, 1, 4, 4, 1, 0, False),
]


@pytest.mark.parametrize("case", BIG)
def test_conv_full_size(K, case):
    B, cin, cout, H, k, s, p, tr = case
    g = K.ConvGeom(k, s, p, tr)
    torch.manual_seed(1)
    x = torch.randn(B, cin, H, H, device=DEV)
    if cin != 3:
        x = _nhwc(x)
    w = torch.randn((cin, cout, k, k) if tr else (cout, cin, k, k), device=DEV) * 0.02
    xr = x.detach().clone().requires_grad_(True)
    wr = w.detach().clone().requires_grad_(True)
    with torch.backends.cudnn.flags(enabled=False):
        ref = (F.conv_transpose2d if tr else F.conv2d)(xr, wr, stride=s, padding=p)
        dy = torch.randn_like(ref)
        ref.backward(dy)
    y = K.conv_fwd(x, w, g)
    assert _rel(y, ref.detach()) < 2e-5
    dyk = dy if cout == 3 else _nhwc(dy)
    assert _rel(K.conv_dgrad(dyk, w, g, x.shape, like=x), xr.grad) < 2e-5
    assert _rel(K.conv_wgrad(x, dyk, g, w.shape)[0], wr.grad) < 2e-5


# the per-GPU layer shapes of BASELINE configs[2] (RaLSGAN 256^2, h=128, 32 images per GPU;
# SURVEY Appendix A "C3 per GPU"): the deepest D conv (2048 -> 4096 @ 8 -> 4, fwd K = 32768,
# wgrad N = 32768), G's deepest ConvT (4096 -> 2048 @ 4 -> 8), the M = 524,288-pixel image
# layers (D 3 -> 128 @ 256 -> 128, G 128 -> 3 @ 128 -> 256), a mid layer, and both ends
C3_SHAPES = [
    (32, 2048, 4096, 8, 4, 2, 1, False),
    (32, 4096, 2048, 4, 4, 2, 1, True),
    (32, 3, 128, 256, 4, 2, 1, False),
    (32, 128, 3, 128, 4, 2, 1, True),
    (32, 256, 512, 64, 4, 2, 1, False),
    (32, 128, 4096, 1, 4, 1, 0, True),
    (32, 4096, 1, 4, 4, 1, 0, False),
]


@pytest.mark.parametrize("case", C3_SHAPES)
def test_conv_c3_full_size(K, case):
    """fwd / dgrad / wgrad at the 256^2 shard's full layer shapes vs torch fp64 on the
    device (ATen's GEMM convolution in double, MIOpen off): rel L2 <= 1e-5 (fp32 MFMA
    accumulation over K <= 32768 terms; observed ~1e-6)."""
    B, cin, cout, H, k, s, p, tr = case
    g = K.ConvGeom(k, s, p, tr)
    torch.manual_seed(3)
    x = torch.randn(B, cin, H, H, device=DEV)
    if cin != 3:
        x = _nhwc(x)
    w = torch.randn((cin, cout, k, k) if tr else (cout, cin, k, k), device=DEV) * 0.02
    xr = x.detach().double().contiguous().requires_grad_(True)
    wr = w.detach().double().requires_grad_(True)
    with torch.backends.cudnn.flags(enabled=False):
        ref = (F.conv_transpose2d if tr else F.conv2d)(xr, wr, stride=s, padding=p)
        dy = torch.randn(ref.shape, device=DEV)
        ref.backward(dy.double())
    y = K.conv_fwd(x, w, g)
    assert _rel(y, ref.detach()) < 1e-5
    del ref, y
    dyk = dy if cout == 3 else _nhwc(dy)
    assert _rel(K.conv_dgrad(dyk, w, g, x.shape, like=x), xr.grad) < 1e-5
    assert _rel(K.conv_wgrad(x, dyk, g, w.shape)[0], wr.grad) < 1e-5


EMU_SHAPES = [
    (32, 2048, 4096, 8, 4, 2, 1, False),   # C3 deepest D conv (K = 32768)
    (32, 4096, 2048, 4, 4, 2, 1, True),    # C3 deepest G ConvT
    (32, 256, 512, 64, 4, 2, 1, False),    # C3 mid layer
    (3, 96, 160, 34, 4, 2, 1, False),      # ragged tiles: fwd M = 867, N = 160; dgrad M = 3468, N = 96
    (5, 96, 160, 5, 4, 2, 1, True),        # ragged ConvT: 4 phases of M = 125, N = 160; dgrad N = 96
]


@pytest.mark.parametrize("case", EMU_SHAPES)
def test_conv_bf16x6_emulation(K, case):
    """fp32 GEMM emulated on the bf16 MFMA (rgan_set_gemm_emulation(1)): forward and data
    gradient vs torch fp64 at the fp32 path's tolerance (rel L2 <= 1e-5), within 2x of the
    fp32 MFMA path's own error, and the emulated kernel is the one that ran."""
    B, cin, cout, H, k, s, p, tr = case
    g = K.ConvGeom(k, s, p, tr)
    torch.manual_seed(5)
    x = _nhwc(torch.randn(B, cin, H, H, device=DEV))
    w = torch.randn((cin, cout, k, k) if tr else (cout, cin, k, k), device=DEV) * 0.02
    xr = x.detach().double().contiguous().requires_grad_(True)
    with torch.backends.cudnn.flags(enabled=False):
        ref = (F.conv_transpose2d if tr else F.conv2d)(xr, w.double(), stride=s, padding=p)
        dy = torch.randn(ref.shape, device=DEV)
        ref.backward(dy.double())
    dyk = _nhwc(dy)
    y32, dx32 = K.conv_fwd(x, w, g), K.conv_dgrad(dyk, w, g, x.shape, like=x)
    prev = K.set_gemm_emulation(True)
    try:
        K.profile_begin(64)
        y, dx = K.conv_fwd(x, w, g), K.conv_dgrad(dyk, w, g, x.shape, like=x)
        names = [kk["name"] for kk in K.profile_end()["kernels"]]
    finally:
        K.set_gemm_emulation(prev)
    assert any("bf16x6" in n for n in names), names
    for got, fp32, want in ((y, y32, ref.detach()), (dx, dx32, xr.grad)):
        e = _rel(got, want)
        assert e < 1e-5
        assert e < 2 * _rel(fp32, want) + 1e-7
    assert K.set_gemm_emulation(prev) == prev


def _bn_ref(y, gamma, beta, eps=1e-5):
    y64 = y.double().cpu()
    mean = y64.mean((0, 2, 3))
    var = y64.var((0, 2, 3), unbiased=False)
    xh = (y64 - mean[None, :, None, None]) / torch.sqrt(var + eps)[None, :, None, None]
    return xh * gamma.double().cpu()[None, :, None, None] + beta.double().cpu()[None, :, None, None], mean, var


@pytest.mark.parametrize("shape", [(4, 8, 5, 5), (64, 256, 32, 32), (2, 2048, 4, 4), (3, 3, 1, 1),
                                   (32, 4096, 4, 4), (32, 256, 64, 64)])   # the last two: C3 D layers
@pytest.mark.parametrize("act", ["relu", "lrelu", "none", "tanh"])
def test_batchnorm_train(K, shape, act):
    torch.manual_seed(2)
    B, C, H, W = shape
    y = _nhwc(torch.randn(shape, device=DEV) * 3 + 1.5)
    gamma = 1 + 0.1 * torch.randn(C, device=DEV)
    beta = 0.1 * torch.randn(C, device=DEV)
    rm = torch.zeros(C, device=DEV)
    rv = torch.ones(C, device=DEV)
    nbt = torch.zeros((), dtype=torch.long, device=DEV)
    stats = K.bn_stats(y, 1e-5, 0.1, rm, rv, nbt)
    a = K.bn_apply(y, stats, gamma, beta, act, 0.2)
    z, mean, var = _bn_ref(y, gamma, beta)
    fn = {"relu": F.relu, "lrelu": lambda t: F.leaky_relu(t, 0.2), "none": lambda t: t, "tanh": torch.tanh}[act]
    assert _rel(a, fn(z)) < 1e-5
    n = B * H * W
    assert _rel(rm, 0.1 * mean) < 1e-5
    assert _rel(rv, 0.9 + 0.1 * var * n / max(n - 1, 1)) < 1e-5
    assert int(nbt.item()) == 1
    # backward vs torch autograd in fp64
    da = _nhwc(torch.randn(shape, device=DEV))
    y64 = y.double().cpu().requires_grad_(True)
    g64 = gamma.double().cpu().requires_grad_(True)
    b64 = beta.double().cpu().requires_grad_(True)
    out = fn(F.batch_norm(y64, None, None, g64, b64, training=True, eps=1e-5))
    out.backward(da.double().cpu())
    dy, dg, db = K.bn_backward(da, y, stats, gamma, beta, act, 0.2)
    tol = 1e-4 if n == 1 else 2e-5
    keep = torch.ones_like(y64, dtype=torch.bool)
    if act in ("relu", "lrelu"):
        # act' jumps at 0: elements whose pre-activation is within fp32 rounding of 0 may
        # take the other branch (a flip moves that element by (1-alpha)*da*gamma*invstd)
        zn = (y64.detach() - mean[None, :, None, None]) / torch.sqrt(var + 1e-5)[None, :, None, None]
        zn = zn * gamma.double().cpu()[None, :, None, None] + beta.double().cpu()[None, :, None, None]
        keep = zn.abs() > 1e-5
    assert _rel(dy.cpu()[keep], y64.grad[keep]) < tol
    assert _rel(dg, g64.grad) < 2e-5
    assert _rel(db, b64.grad) < 2e-5


# conv feeding BatchNorm: (B, cin, cout, H, transposed, segs, fused) -- FAST 128x128 layers
# whose vector epilogue emits the BN segment moments (D conv, G k4s2 ConvT = 4 phases,
# batched D halves), split-K layers whose reduce emits them (splitk_reduce_bn: deep D
# layer, narrow N, 4-phase ConvT, batched halves, N = 1024 in 4 column chunks), and a
# ragged M that must fall back to the moments pass
BN_EPI = [
    (16, 32, 128, 128, False, 1, True),    # >= 512 output tiles: no split-K
    (32, 32, 128, 128, False, 2, True),
    (16, 128, 128, 32, True, 1, True),
    (4, 256, 128, 16, False, 1, True),     # M = 256 rows: split-K reduce
    (8, 256, 128, 16, False, 2, True),     # split-K, two batch segments
    (4, 256, 128, 8, True, 1, True),       # split-K ConvT, 4 phases
    (4, 64, 1024, 8, False, 1, True),      # split-K, N = 1024
    (3, 64, 128, 10, False, 1, False),     # M = 75: not a multiple of 64 -> fallback
    (8, 64, 32, 32, False, 1, True),       # N = 32: narrow tile
]


@pytest.mark.parametrize("case", BN_EPI)
def test_conv_bn_epilogue_stats(K, case):
    """rgan_conv_fwd_bn + rgan_bn_segment_stats == rgan_conv_fwd + rgan_bn_stats (fp64 torch)."""
    B, cin, cout, H, tr, segs, expect_fused = case
    _bn_epilogue_case(K, B, cin, cout, H, (4, 2, 1), tr, segs, expect_fused, bias=False)


# the 64 x 64 tiles of arch 1's small GEMMs (C4; round 6: their scalar epilogue emits the
# segment sums too): (B, cin, cout, H, (k, stride, pad), transposed, segs)
BN_EPI_SMALL = [
    (64, 64, 128, 16, (3, 1, 1), False, 2),   # D's 3x3 64 -> 128 at 16x16, batched halves
    (32, 128, 64, 16, (4, 2, 1), True, 1),    # G's ConvT 128 -> 64, 16 -> 32 (4 phases)
    (64, 3, 64, 32, (3, 1, 1), False, 2),     # D's image layer 3 -> 64 (K = 27)
    (32, 64, 128, 16, (3, 1, 1), False, 1),   # the WGAN-GP D(x_hat) call of the first case
]


@pytest.mark.parametrize("case", BN_EPI_SMALL)
def test_conv_bn_epilogue_stats_small_tiles(K, case):
    """The same on the 64 x 64 tiles, with the arch-1 conv bias (GLI:260-302)."""
    B, cin, cout, H, kgeo, tr, segs = case
    _bn_epilogue_case(K, B, cin, cout, H, kgeo, tr, segs, True, bias=True)


def _bn_epilogue_case(K, B, cin, cout, H, kgeo, tr, segs, expect_fused, bias):
    from relativisticgan_amd.kernels import ConvGeom
    torch.manual_seed(11)
    k = kgeo[0]
    g = ConvGeom(k, kgeo[1], kgeo[2], tr)
    x = _nhwc(torch.randn(B, cin, H, H, device=DEV))
    w = torch.randn((cin, cout, k, k) if tr else (cout, cin, k, k), device=DEV) * 0.05 + 0.01
    bvec = torch.randn(cout, device=DEV) * 0.1 if bias else None
    y, part, S = K.conv_fwd_bn(x, w, g, bias=bvec, segs=segs)
    assert (part is not None) == expect_fused
    y_ref = K.conv_fwd(x, w, g, bias=bvec)
    assert torch.equal(y, y_ref)  # the epilogue statistics do not touch the stored output
    Bs = B // segs
    for k in range(segs):
        ys = y[k * Bs:(k + 1) * Bs]
        rm, rv = torch.zeros(cout, device=DEV), torch.ones(cout, device=DEV)
        nbt = torch.zeros((), dtype=torch.long, device=DEV)
        if part is not None:
            stats = K.bn_segment_stats(part, k * S // segs, (k + 1) * S // segs, cout, 1e-5, 0.1, rm, rv, nbt)
            mom = K.bn_segment_moments(part, k * S // segs, (k + 1) * S // segs, cout).cpu()
        else:
            stats = K.bn_stats(ys, 1e-5, 0.1, rm, rv, nbt)
            mom = K.bn_moments(ys).cpu()
        y64 = ys.double().cpu()
        mean, var = y64.mean((0, 2, 3)), y64.var((0, 2, 3), unbiased=False)
        n = ys.shape[0] * ys.shape[2] * ys.shape[3]
        assert _rel(stats[:cout], mean) < 1e-6
        assert _rel(stats[cout:], 1 / torch.sqrt(var + 1e-5)) < 1e-6
        assert _rel(rv, 0.9 + 0.1 * var * n / (n - 1)) < 1e-6
        assert int(nbt.item()) == 1
        assert mom[0].item() == n
        assert _rel(mom[cout:2 * cout], mean) < 1e-6 and _rel(mom[2 * cout:], var * n) < 1e-6


def _torch_head(kind, side, r, f):
    """The reference's expressions (GLI:592-709) in fp64 with torch autograd."""
    ones = torch.ones_like(r if r is not None else f)
    zeros = torch.zeros_like(ones)
    bce, bcel = torch.nn.BCELoss(), torch.nn.BCEWithLogitsLoss()
    relu = torch.nn.ReLU()
    if kind <= 4:
        t = r if side == 0 else f
        if kind == 1:
            return bce(t, zeros if side == 1 else ones)
        if kind == 2:
            return torch.mean(t ** 2) if side == 1 else torch.mean((t - ones) ** 2)
        if kind == 3 or side == 2:
            return torch.mean(t) if side == 1 else -torch.mean(t)
        return torch.mean(relu(1.0 - t)) if side == 0 else torch.mean(relu(1.0 + t))
    if kind == 5:
        return bcel(r - f, ones) if side == 0 else bcel(f - r, ones)
    if kind == 6:
        if side == 0:
            return (bcel(r - torch.mean(f), ones) + bcel(f - torch.mean(r), zeros)) / 2
        return (bcel(r - torch.mean(f), zeros) + bcel(f - torch.mean(r), ones)) / 2
    if kind == 7:
        if side == 0:
            return (torch.mean((r - torch.mean(f) - ones) ** 2) + torch.mean((f - torch.mean(r) + ones) ** 2)) / 2
        return (torch.mean((r - torch.mean(f) + ones) ** 2) + torch.mean((f - torch.mean(r) - ones) ** 2)) / 2
    if side == 0:
        return (torch.mean(relu(1.0 - (r - torch.mean(f)))) + torch.mean(relu(1.0 + (f - torch.mean(r))))) / 2
    return (torch.mean(relu(1.0 + (r - torch.mean(f)))) + torch.mean(relu(1.0 - (f - torch.mean(r))))) / 2


HEAD_CASES = [(k, s) for k in (1, 2, 3, 4) for s in (0, 1, 2)] + [(k, s) for k in (5, 6, 7, 8) for s in (0, 2)]


@pytest.mark.parametrize("kind,side", HEAD_CASES)
@pytest.mark.parametrize("n", [1, 8, 64, 3000])
def test_loss_heads(K, kind, side, n):
    torch.manual_seed(kind * 10 + side)
    if kind == 1:
        r = torch.rand(n, device=DEV) * 0.98 + 0.01
        f = torch.rand(n, device=DEV) * 0.98 + 0.01
    else:
        r = torch.randn(n, device=DEV) * 2
        f = torch.randn(n, device=DEV) * 2
    needs_r = kind > 4 or side == 0
    needs_f = kind > 4 or side != 0
    loss, dr, df = K.loss_head(kind, side, r if needs_r else None, f if needs_f else None)
    r64 = r.double().cpu().requires_grad_(True)
    f64 = f.double().cpu().requires_grad_(True)
    ref = _torch_head(kind, side, r64 if needs_r else None, f64 if needs_f else None)
    ref.backward()
    assert abs(loss.item() - ref.item()) <= 1e-5 * max(1.0, abs(ref.item()))
    if needs_r:
        assert _rel(dr, r64.grad) < 1e-5 or r64.grad.abs().max() < 1e-12
    if needs_f:
        assert _rel(df, f64.grad) < 1e-5 or f64.grad.abs().max() < 1e-12


def test_gp_kernels(K):
    torch.manual_seed(3)
    x = torch.randn(8, 3, 16, 16, device=DEV)
    xf = torch.randn(8, 3, 16, 16, device=DEV)
    u = torch.rand(8, 1, 1, 1, device=DEV)
    xb = K.gp_interp(x, xf, u)
    assert _rel(xb, x * u + xf * (1 - u)) < 1e-6
    g = torch.randn(8, 3, 16, 16, device=DEV)
    loss, norms, gc = K.gp_penalty(g, 10.0, 8)
    g64 = g.double().cpu().requires_grad_(True)
    ref = 10.0 * ((g64.norm(2, 1).norm(2, 1).norm(2, 1) - 1) ** 2).mean()
    ref.backward()
    assert abs(loss.item() - ref.item()) < 1e-5 * ref.item()
    one = torch.ones((), device=DEV)
    dg = K.gp_penalty_backward(gc, norms, 10.0, 8, one)
    assert _rel(dg, g64.grad) < 1e-5


@pytest.mark.parametrize("transposed", [False, True])
def test_spectral_norm(K, transposed):
    torch.manual_seed(4)
    conv = (torch.nn.ConvTranspose2d(24, 16, 4, 2, 1, bias=False) if transposed
            else torch.nn.Conv2d(24, 16, 4, 2, 1, bias=False))
    sn = torch.nn.utils.spectral_norm(conv)
    w = sn.weight_orig.detach().to(DEV)
    u = sn.weight_u.detach().clone().to(DEV)
    v = sn.weight_v.detach().clone().to(DEV)
    inv_sigma = K.spectral_power(w, u, v, transposed)
    # reference: one power iteration in fp64
    dim = 1 if transposed else 0
    W = sn.weight_orig.detach().double()
    if dim == 1:
        W = W.permute(1, 0, 2, 3)
    Wm = W.reshape(W.shape[0], -1)
    u0 = sn.weight_u.double()
    v1 = F.normalize(Wm.t() @ u0, dim=0, eps=1e-12)
    u1 = F.normalize(Wm @ v1, dim=0, eps=1e-12)
    sigma = torch.dot(u1, Wm @ v1)
    assert _rel(u, u1) < 1e-5 and _rel(v, v1) < 1e-5
    assert abs(1 / inv_sigma.item() - sigma.item()) < 1e-5 * sigma.item()
    # backward of W_eff = W / sigma(W) with u, v held constant
    Wt = sn.weight_orig.detach().double().requires_grad_(True)
    W2 = Wt.permute(1, 0, 2, 3) if dim == 1 else Wt
    sig = torch.dot(u1, W2.reshape(W2.shape[0], -1) @ v1)
    G = torch.randn_like(Wt)
    (Wt / sig).backward(G)
    dw = K.spectral_backward(w, G.float().to(DEV), u, v, inv_sigma, transposed)
    assert _rel(dw, Wt.grad) < 1e-5


def test_adam_matches_torch(K):
    torch.manual_seed(5)
    # one block / several blocks with a partial last one (float4 path), scalar path (n % 4 != 0)
    # over two blocks, a 16-B-misaligned view (scalar path), and > 48 tensors (two launches)
    shapes = [(64, 3, 4, 4), (128,), (7, 9), (3000, 7), (4099,), (1001,)] + [(5, 4)] * 46
    params = [torch.randn(s, device=DEV) for s in shapes]
    params[5] = torch.randn(1002, device=DEV)[1:]
    ref = [p.detach().cpu().clone().requires_grad_(True) for p in params]
    opt = torch.optim.Adam(ref, lr=1e-4, betas=(0.5, 0.999), weight_decay=0.01)
    m = [torch.zeros_like(p) for p in params]
    v = [torch.zeros_like(p) for p in params]
    hyper = torch.tensor([1e-4, 0.5, 0.999, 1e-8, 0.01, 0, 0, 0], dtype=torch.float64, device=DEV)
    step = torch.zeros(1, device=DEV)
    for it in range(3):
        grads = [torch.randn(s, device=DEV) for s in shapes]
        for r, g in zip(ref, grads):
            r.grad = g.cpu()
        opt.step()
        K.adam(params, grads, m, v, hyper, step)
    for p, r in zip(params, ref):
        assert torch.allclose(p.cpu(), r.detach(), rtol=1e-6, atol=1e-7)
    assert step.item() == 3


def test_adam_packed_step_counter_many_tensors(K):
    """optim.Adam over more tensors than one packed launch holds (two launches, the step
    counter stored by the second one's last block) == torch.optim.Adam, the device step
    counter at the step count."""
    from relativisticgan_amd.optim import Adam
    torch.manual_seed(6)
    shapes = [(33,), (4096 * 3 + 8,), (5, 7)] * 11
    params = [torch.nn.Parameter(torch.randn(s, device=DEV)) for s in shapes]
    ref = [torch.nn.Parameter(p.detach().cpu().clone()) for p in params]
    opt = Adam(params, lr=1e-3, betas=(0.5, 0.999))
    topt = torch.optim.Adam(ref, lr=1e-3, betas=(0.5, 0.999))
    for it in range(3):
        for p, r in zip(params, ref):
            p.grad = torch.randn_like(p)
            r.grad = p.grad.cpu()
        opt.step()
        topt.step()
        assert opt._dev[0][2].item() == it + 1
    for p, r in zip(params, ref):
        assert torch.allclose(p.detach().cpu(), r.detach(), rtol=1e-6, atol=1e-7)


def test_gather(K):
    imgs = torch.randn(10, 3, 4, 4, device=DEV)
    idx = torch.tensor([3, 0, 9], dtype=torch.long, device=DEV)
    assert torch.equal(K.gather_images(imgs, idx), imgs[idx])


def test_spectral_power_batch(K):
    """All spectral layers of a call in four launches == one power iteration per layer
    (torch spectral_norm, fp64 reference), incl. ConvT (dim 1), the rows = 1 end layer, a
    non-float4 view, multi-chunk layers (cols > 1024, rows > 64) and the largest layer of
    the C5 D (Conv2d(1024, 2048): 2048 rows x 16384 columns); a second call (from the
    updated u) equals a second fp64 iteration."""
    torch.manual_seed(9)
    specs = [(torch.nn.Conv2d(3, 16, 4, 2, 1, bias=False), False), (torch.nn.Conv2d(16, 300, 4, 2, 1, bias=False), False),
             (torch.nn.ConvTranspose2d(64, 24, 4, 2, 1, bias=False), True), (torch.nn.Conv2d(300, 1, 4, 1, 0, bias=False), False),
             # scalar path (3-column rows, 2 row chunks), a 1024-row layer (8 x 17 blocks) and the
             # C5 D's largest layer, Middle-Conv2d [4] at 128x128, h = 128: 1024 -> 2048 (GLI:420-428)
             (torch.nn.Conv2d(3, 70, 1, bias=False), False), (torch.nn.Conv2d(512, 1024, 4, 2, 1, bias=False), False),
             (torch.nn.Conv2d(1024, 2048, 4, 2, 1, bias=False), False)]
    layers, refs = [], []
    for conv, tr in specs:
        sn = torch.nn.utils.spectral_norm(conv)
        w = sn.weight_orig.detach().to(DEV)
        u, v = sn.weight_u.detach().clone().to(DEV), sn.weight_v.detach().clone().to(DEV)
        layers.append((w, u, v, tr))
        W = sn.weight_orig.detach().double()
        if tr:
            W = W.permute(1, 0, 2, 3)
        Wm = W.reshape(W.shape[0], -1)
        v1 = F.normalize(Wm.t() @ sn.weight_u.double(), dim=0, eps=1e-12)
        u1 = F.normalize(Wm @ v1, dim=0, eps=1e-12)
        refs.append((u1, v1, torch.dot(u1, Wm @ v1)))
    for rep in range(2):  # twice: the second call starts from the u the first one wrote
        outs = K.spectral_power_batch(layers)
        torch.cuda.synchronize()
        for (w, u, v, tr), (uc, vc, inv), (u1, v1, sig) in zip(layers, outs, refs):
            assert _rel(u, u1) < 1e-5 and _rel(v, v1) < 1e-5
            assert torch.equal(uc, u) and torch.equal(vc, v)
            assert abs(1 / inv.item() - sig.item()) < 1e-5 * sig.item()
        for k, ((w, u, v, tr), (u1, v1, sig)) in enumerate(zip(layers, refs)):  # next fp64 iteration
            W = w.detach().double().cpu()
            Wm = (W.permute(1, 0, 2, 3) if tr else W).reshape(W.shape[1] if tr else W.shape[0], -1)
            v2 = F.normalize(Wm.t() @ u1, dim=0, eps=1e-12)
            u2 = F.normalize(Wm @ v2, dim=0, eps=1e-12)
            refs[k] = (u2, v2, torch.dot(u2, Wm @ v2))


@pytest.mark.parametrize("ci", [1, 3, 4])
@pytest.mark.parametrize("hw", [(32, 32), (64, 128), (128, 64), (16, 512), (256, 256)])
@pytest.mark.parametrize("cout", [256, 96, 32])
def test_conv_image_window_kernel(K, ci, hw, cout):
    """conv_img_in (windowed image conv: k4 s2 p1, <= 4 input channels, 128-channel tiles,
    or 32-channel tiles for 3-channel images when the width is not a multiple of 128):
    fwd with bias / LeakyReLU / wscale on NCHW and NHWC images, and the ConvTranspose2d
    image-layer dgrad that runs on it, vs torch fp64 (every tile shape: 128-wide row
    segments and 128 / Wo whole rows)."""
    H, W = hw
    B = 2 if H * W <= 128 * 128 else 1
    torch.manual_seed(ci + H + cout)
    gc, gt = K.ConvGeom(4, 2, 1, False), K.ConvGeom(4, 2, 1, True)
    img = torch.randn(B, ci, H, W, device=DEV)
    w = torch.nn.Parameter(torch.randn(cout, ci, 4, 4, device=DEV) * 0.1)
    b = torch.randn(cout, device=DEV)
    s = torch.tensor([0.7], device=DEV)
    ref = F.leaky_relu(F.conv2d(img.double().cpu(), (w * 0.7).detach().double().cpu(), b.double().cpu(), stride=2,
                                padding=1), 0.2)
    for x in (img, _nhwc(img)):
        for cache in (False, True):
            y = K.conv_fwd(x, w, gc, bias=b, act="lrelu", alpha=0.2, wscale=s, cache=cache)
            assert K.is_nhwc(y)
            assert _rel(y, ref) < 3e-6
    if cout != 256:
        return
    # G's image layer ConvT(256 -> ci): its input gradient is a Conv2d over the image gradient
    wt = torch.randn(256, ci, 4, 4, device=DEV) * 0.1
    gy = torch.randn(B, ci, H, W, device=DEV)
    x64 = torch.zeros(B, 256, H // 2, W // 2, dtype=torch.float64, requires_grad=True)
    F.conv_transpose2d(x64, wt.double().cpu(), stride=2, padding=1).backward(gy.double().cpu())
    dx = K.conv_dgrad(gy, wt, gt, (B, 256, H // 2, W // 2))
    assert _rel(dx, x64.grad) < 3e-6


@pytest.mark.parametrize("B,S,C", [(32, 128, 128), (64, 128, 128), (8, 256, 128), (32, 256, 32), (16, 256, 128)])
def test_conv_image_window_full_batch(K, B, S, C):
    """conv_img_in at the BASELINE batch sizes, where every persistent wave runs several
    tiles and two blocks share a CU (C2's batched D pass: 128 x 128^2; C3: 256^2; C3 at
    h = 32: 32-channel tiles): each sample's outputs vs torch fp64.  The bounded per-sample
    max error catches the two faults smaller grids never reached: a wide store's data VGPR
    rewritten behind it (lanes 12-15 of every 16) and a window read before its DMA landed."""
    g = K.ConvGeom(4, 2, 1, False)
    torch.manual_seed(B + S + C)
    img = torch.rand(B, 3, S, S, device=DEV) * 2 - 1
    w = torch.nn.Parameter(torch.randn(C, 3, 4, 4, device=DEV) * 0.05)
    y = K.conv_fwd(img, w, g, act="lrelu", alpha=0.2, cache=True)
    torch.cuda.synchronize()
    ref = F.leaky_relu(F.conv2d(img.double().cpu(), w.detach().double().cpu(), stride=2, padding=1), 0.2)
    err = (y.double().cpu() - ref).abs().flatten(1).amax(1) / ref.abs().amax()
    assert err.max().item() < 1e-6, f"samples off: {(err > 1e-6).nonzero().flatten().tolist()[:16]}"


def test_pack_batch_refresh(K):
    """PACKS.refresh (one rgan_conv_pack_batch launch after an optimizer step) leaves every
    cached layout bitwise equal to a fresh single pack: 4x4 tiled16 (fwd, ConvT phases),
    3x3 tiled, the narrow-ConvT pack and > 16 layouts (two batches)."""
    import ctypes
    from relativisticgan_amd import _lib as L
    torch.manual_seed(13)
    g4, gt, g3 = K.ConvGeom(4, 2, 1, False), K.ConvGeom(4, 2, 1, True), K.ConvGeom(3, 1, 1, False)
    ws, runs = [], []
    for i in range(7):
        w = torch.nn.Parameter(torch.randn(64, 32, 4, 4, device=DEV) * 0.1)
        x = _nhwc(torch.randn(2, 32, 8, 8, device=DEV))
        y = K.conv_fwd(x, w, g4, cache=True)
        K.conv_dgrad(y, w, g4, x.shape, like=x, cache=True)
        ws.append(w)
    wt = torch.nn.Parameter(torch.randn(32, 64, 4, 4, device=DEV) * 0.1)
    K.conv_fwd(_nhwc(torch.randn(2, 32, 8, 8, device=DEV)), wt, gt, cache=True)
    w3 = torch.nn.Parameter(torch.randn(24, 20, 3, 3, device=DEV) * 0.1)
    K.conv_fwd(_nhwc(torch.randn(2, 20, 8, 8, device=DEV)), w3, g3, cache=True)
    wn = torch.nn.Parameter(torch.randn(32, 3, 4, 4, device=DEV) * 0.1)
    K.conv_fwd(_nhwc(torch.randn(2, 32, 8, 8, device=DEV)), wn, gt, cache=True)
    params = ws + [wt, w3, wn]
    with torch.no_grad():
        for p in params:
            p.mul_(1.5).add_(0.25)  # an optimizer step: new values, new version
    K.PACKS.refresh(params)
    ids = {id(p) for p in params}
    checked = 0
    for ent in list(K.PACKS.entries.values()):
        base, w = ent[0](), K.PACKS._weight(ent)
        if base is None or id(base) not in ids:
            continue
        assert ent[1] == w._version
        fresh = torch.empty_like(ent[2])
        L.check(L.lib().rgan_conv_pack(ctypes.byref(ent[4]), ent[5], L.ptr(w), L.ptr(fresh), L.stream()), "pack")
        assert torch.equal(fresh, ent[2])
        checked += 1
    assert checked >= 17


def test_pack_cache_keeps_views_current(K):
    """A weight packed through a view (arch 1's dense layers run as convolutions on
    p.view(...), GLI:186-319): the layout stays listed for the optimizer after the call
    (layouts_of), Adam rewrites it, and the next call reuses it without a repack."""
    from relativisticgan_amd.optim import Adam
    torch.manual_seed(11)
    p = torch.nn.Parameter(torch.randn(1, 512 * 16, device=DEV) * 0.02)
    g = K.ConvGeom(4, 1, 0, False)
    x = _nhwc(torch.randn(8, 512, 4, 4, device=DEV))
    y0 = K.conv_fwd(x, p.view(1, 512, 4, 4), g, cache=True)
    lay = K.PACKS.layouts_of([p])
    assert len(lay) == 1
    p.grad = torch.randn_like(p)
    Adam([p], lr=1e-3, betas=(0.5, 0.999)).step()
    ent = K.PACKS.layouts_of([p])[0][2]
    assert ent[1] == p._version  # rewritten from the stepped values: current
    y1 = K.conv_fwd(x, p.view(1, 512, 4, 4), g, cache=True)
    with torch.backends.cudnn.flags(enabled=False):
        ref = F.conv2d(x.double(), p.detach().double().view(1, 512, 4, 4))
    assert _rel(y1, ref) < 2e-6 and not torch.equal(y0, y1)


def test_adam_writes_packed_layouts(K):
    """optim.Adam (rgan_adam_packed) rewrites every cached GEMM layout of the weights it
    steps from the new values: p / exp_avg / exp_avg_sq bitwise equal to the plain multi-
    tensor Adam (rgan_adam), every layout bitwise equal to a fresh rgan_conv_pack of the
    updated weight -- brick path (4x4 tiled, both directions: Conv2d fwd + its 4-phase dgrad,
    ConvTranspose2d), per-element scatters (a 3x3 tiled layout, the t2d layout of G's 1x1 ->
    4x4 first layer, the narrow ConvT layouts of both image layers), BN vectors without
    layouts -- and the cache then serves them without repacking."""
    import ctypes
    from relativisticgan_amd import _lib as L
    from relativisticgan_amd.optim import Adam
    torch.manual_seed(21)
    g4, gt, g3, g41 = K.ConvGeom(4, 2, 1, False), K.ConvGeom(4, 2, 1, True), K.ConvGeom(3, 1, 1, False), \
        K.ConvGeom(4, 1, 0, True)
    conv = torch.nn.Parameter(torch.randn(256, 128, 4, 4, device=DEV) * 0.05)   # D middle: fwd + dgrad
    convt = torch.nn.Parameter(torch.randn(128, 64, 4, 4, device=DEV) * 0.05)   # G middle: fwd + dgrad
    start = torch.nn.Parameter(torch.randn(32, 512, 4, 4, device=DEV) * 0.05)   # G 1x1 -> 4x4 (t2d)
    g_end = torch.nn.Parameter(torch.randn(64, 3, 4, 4, device=DEV) * 0.05)     # G image ConvT (narrow)
    d_img = torch.nn.Parameter(torch.randn(64, 3, 4, 4, device=DEV) * 0.05)     # D image conv (narrow dgrad)
    c3 = torch.nn.Parameter(torch.randn(24, 20, 3, 3, device=DEV) * 0.05)       # 3x3 (arch 1)
    gamma = torch.nn.Parameter(torch.randn(256, device=DEV))
    beta = torch.nn.Parameter(torch.randn(256, device=DEV))
    x = _nhwc(torch.randn(2, 128, 16, 16, device=DEV))
    y = K.conv_fwd(x, conv, g4, cache=True)
    K.conv_dgrad(y, conv, g4, x.shape, like=x, cache=True)
    xt = _nhwc(torch.randn(2, 128, 8, 8, device=DEV))
    yt = K.conv_fwd(xt, convt, gt, cache=True)
    K.conv_dgrad(yt, convt, gt, xt.shape, like=xt, cache=True)
    K.conv_fwd(_nhwc(torch.randn(4, 32, 1, 1, device=DEV)), start, g41, cache=True)
    K.conv_fwd(_nhwc(torch.randn(2, 64, 16, 16, device=DEV)), g_end, gt, cache=True)
    img = torch.randn(2, 3, 32, 32, device=DEV)
    K.conv_dgrad(_nhwc(torch.randn(2, 64, 16, 16, device=DEV)), d_img, g4, img.shape, like=img, cache=True)
    K.conv_fwd(_nhwc(torch.randn(2, 20, 8, 8, device=DEV)), c3, g3, cache=True)
    params = [conv, convt, start, g_end, d_img, c3, gamma, beta]
    for p in params:
        p.grad = torch.randn_like(p) * 1e-3
    twins = [torch.nn.Parameter(p.detach().clone()) for p in params]
    for p, q in zip(params, twins):
        q.grad = p.grad.clone()
    before = len(K.PACKS.layouts_of(params))
    assert before >= 7, before
    opt, ref = Adam(params, lr=1e-3, betas=(0.5, 0.999)), Adam(twins, lr=1e-3, betas=(0.5, 0.999))
    for step in range(2):
        opt.step()
        # the reference: the plain multi-tensor kernel on the twins
        hyper, _, dstep = ref._group_dev(0, ref.param_groups[0], DEV, ref.state.get(twins[0]) or None)
        for q in twins:
            st = ref.state[q]
            if not st:
                st["step"] = torch.tensor(0.0)
                st["exp_avg"] = torch.zeros_like(q)
                st["exp_avg_sq"] = torch.zeros_like(q)
        K.adam(twins, [q.grad for q in twins], [ref.state[q]["exp_avg"] for q in twins],
               [ref.state[q]["exp_avg_sq"] for q in twins], hyper, dstep)
        for q in twins:
            ref.state[q]["step"] += 1
        torch.cuda.synchronize()
        # the packed kernel's last block stores step + 1 (no separate increment launch)
        assert opt._dev[0][2].item() == dstep.item() == step + 1
        for p, q in zip(params, twins):
            assert torch.equal(p.detach(), q.detach())
            assert torch.equal(opt.state[p]["exp_avg"], ref.state[q]["exp_avg"])
            assert torch.equal(opt.state[p]["exp_avg_sq"], ref.state[q]["exp_avg_sq"])
        lay = K.PACKS.layouts_of(params)
        assert len(lay) == before
        for _, _, ent in lay:
            w = K.PACKS._weight(ent)
            assert ent[1] == w._version  # current: the next conv reuses it
            fresh = torch.empty_like(ent[2])
            L.check(L.lib().rgan_conv_pack(ctypes.byref(ent[4]), ent[5], L.ptr(w), L.ptr(fresh), L.stream()), "pack")
            torch.cuda.synchronize()
            assert torch.equal(fresh, ent[2]), (tuple(w.shape), ent[5])


def test_device_rng(K):
    """--rgan_rng device draws: N(0,1) / U[0,1) moments, distinct in-range batch indices, the
    device counter advancing (fresh draws per call, the same sequence for the same seed --
    every data-parallel rank draws the global batch), and fresh draws per HIP-graph replay."""
    a, b = K.DeviceRNG(7, DEV), K.DeviceRNG(7, DEV)
    z = a.normal((400, 1000))
    assert abs(z.mean().item()) < 0.01 and abs(z.std().item() - 1) < 0.01 and torch.isfinite(z).all()
    u = a.uniform((1000, 1001))
    assert u.min().item() >= 0 and u.max().item() < 1 and abs(u.mean().item() - 0.5) < 0.01
    idx = a.choice(1000, 64)
    assert idx.unique().numel() == 64 and idx.min().item() >= 0 and idx.max().item() < 1000
    full = a.choice(50, 50)
    assert sorted(full.tolist()) == list(range(50))
    big = a.choice(5000, 300)  # > 64: the LDS path
    assert big.unique().numel() == 300 and big.min().item() >= 0 and big.max().item() < 5000
    assert torch.equal(b.normal((400, 1000)), z)  # same seed, same counter: same draws
    assert not torch.equal(b.normal((400, 1000)), z)  # the counter moved
    # z-sized draws run as one block that advances the counter itself: the same numbers as
    # the multi-block fill from the same counter, and the counter moved by the quads consumed
    c, d = K.DeviceRNG(9, DEV), K.DeviceRNG(9, DEV)
    small = c.normal((32, 128))
    assert torch.equal(small.flatten(), d.normal((20000,))[:4096])
    assert int(c.counter.item()) == 1024 and int(d.counter.item()) == 5000
    assert not torch.equal(c.normal((32, 128)), small)
    counts = torch.zeros(20, device=DEV)
    for _ in range(200):
        counts.index_add_(0, a.choice(20, 5), torch.ones(5, device=DEV))
    assert counts.min().item() > 20 and counts.max().item() < 80  # ~50 each
    # positional uniformity (numpy.random.choice's order is exchangeable; callers split the
    # draw by position): every position's index is uniform over [0, N): chi-square per
    # position below N - 1 + 6 sd, for the wave path (n <= 64) and the LDS path
    for N, n, reps in ((12, 8, 3000), (100, 80, 600)):
        pos = torch.zeros(n, N, dtype=torch.float64)
        for _ in range(reps):
            d = a.choice(N, n).cpu()
            assert d.unique().numel() == n
            pos[torch.arange(n), d] += 1
        exp = reps / N
        chi = ((pos - exp) ** 2 / exp).sum(1)
        assert chi.max().item() < N - 1 + 6 * (2 * (N - 1)) ** 0.5, (N, n, chi.max().item())
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            zz = a.normal((16,))
    g.replay()
    first = zz.clone()
    g.replay()
    assert not torch.equal(first, zz)


def test_bn_two_segments_one_launch(K):
    """rgan_bn_segment_stats_n + rgan_bn_apply_segments (the batched D pass's two calls in
    one launch each) == the two calls one at a time, bitwise, incl. the running statistics."""
    from relativisticgan_amd.kernels import ConvGeom
    torch.manual_seed(17)
    g = ConvGeom(4, 2, 1, False)
    x = _nhwc(torch.randn(16, 32, 32, 32, device=DEV))
    w = torch.randn(128, 32, 4, 4, device=DEV) * 0.05
    y, part, S = K.conv_fwd_bn(x, w, g, segs=2)
    assert part is not None
    C = 128
    gamma, beta = torch.rand(C, device=DEV) + 0.5, torch.randn(C, device=DEV)
    rm1, rv1, n1 = torch.randn(C, device=DEV), torch.rand(C, device=DEV) + 0.5, torch.zeros((), dtype=torch.long, device=DEV)
    rm2, rv2, n2 = rm1.clone(), rv1.clone(), n1.clone()
    st1 = torch.empty(2, 2 * C, device=DEV)
    a1 = torch.empty_like(y)
    for k in range(2):
        sl = slice(8 * k, 8 * (k + 1))
        K.bn_segment_stats(part, k * S // 2, (k + 1) * S // 2, C, 1e-5, 0.1, rm1, rv1, n1, out=st1[k])
        K.bn_apply(y[sl], st1[k], gamma, beta, "lrelu", 0.2, out=a1[sl])
    st2 = torch.empty(2, 2 * C, device=DEV)
    K.bn_segment_stats_n(part, S, 2, C, 1e-5, 0.1, rm2, rv2, n2, out=st2)
    a2 = K.bn_apply_segments(y, st2, gamma, beta, "lrelu", 0.2, out=torch.empty_like(y))
    assert torch.equal(st1, st2) and torch.equal(a1, a2)
    assert torch.equal(rm1, rm2) and torch.equal(rv1, rv2) and int(n2.item()) == 2


@pytest.mark.parametrize("B,cin,H,cout,tr,nseg", [
    (16, 32, 8, 128, False, 2),     # 4x4 output, 2 x 2 segments
    (16, 32, 8, 128, False, 1),     # 256 rows x 128: one launch
    (16, 32, 32, 64, False, 2),     # 16x16 output, 2 x 32 segments
    (32, 512, 4, 256, True, 1),     # ConvT (4 phase GEMMs; C4's G layer 1), 8x8 output: 2048 x 256
    (32, 32, 64, 128, False, 2),    # 32x32 output, 2 x 256 segments: merge + apply launches
])
def test_bn_segment_apply_one_call(K, B, cin, H, cout, tr, nseg):
    """rgan_bn_segment_apply (segment statistics + normalisation + LeakyReLU in one call; one
    launch for a single batch segment of <= 2^18 elements, whose blocks each merge their
    channels' sums)
    == rgan_bn_segment_stats_n + rgan_bn_apply_segments: stats / output / running statistics
    within 1e-6 (the one-launch merge adds the segments' double sums in another order: equal
    after rounding to fp32 but for rare ties) and bitwise on the two-launch path;
    num_batches_tracked counted once per batch segment."""
    from relativisticgan_amd.kernels import ConvGeom
    torch.manual_seed(29)
    g = ConvGeom(4, 2, 1, tr)
    x = _nhwc(torch.randn(B, cin, H, H, device=DEV))
    w = torch.randn(cin, cout, 4, 4, device=DEV) * 0.05 if tr else torch.randn(cout, cin, 4, 4, device=DEV) * 0.05
    y, part, S = K.conv_fwd_bn(x, w, g, segs=nseg)
    assert part is not None
    C = cout
    gamma, beta = torch.rand(C, device=DEV) + 0.5, torch.randn(C, device=DEV)
    rm1, rv1, n1 = torch.randn(C, device=DEV), torch.rand(C, device=DEV) + 0.5, torch.zeros((), dtype=torch.long, device=DEV)
    rm2, rv2, n2 = rm1.clone(), rv1.clone(), n1.clone()
    st1 = torch.empty(nseg, 2 * C, device=DEV)
    K.bn_segment_stats_n(part, S, nseg, C, 1e-5, 0.1, rm1, rv1, n1, out=st1)
    a1 = K.bn_apply_segments(y, st1, gamma, beta, "lrelu", 0.2, out=torch.empty_like(y))
    st2 = torch.full((nseg, 2 * C), float("nan"), device=DEV)
    a2 = K.bn_segment_apply(part, S, y, 1e-5, 0.1, rm2, rv2, n2, gamma, beta, "lrelu", 0.2, st2, torch.empty_like(y))
    P = y.shape[0] * y.shape[2] * y.shape[3]
    one_launch = S // nseg <= 64 and nseg == 1 and P * C <= (1 << 18)  # rgan_bn_segment_apply's rule
    same = (lambda a, b: torch.allclose(a, b, rtol=1e-6, atol=1e-6)) if one_launch else torch.equal
    assert same(st1, st2) and same(a1, a2)
    assert same(rm1, rm2) and same(rv1, rv2) and int(n2.item()) == nseg


@pytest.mark.parametrize("C,B,H", [(256, 32, 4), (128, 32, 8), (64, 32, 16), (64, 32, 32), (36, 8, 8)])
def test_bn_backward_sums_apply_one_call(K, C, B, H):
    """rgan_bn_backward_sums_apply (the WGAN-GP engine's BatchNorm backward: sums kept, + add,
    affine gradients accumulated) == rgan_bn_backward_sums + rgan_bn_backward_apply_ex: within
    1e-6 on the one-launch small-layer kernel (<= 2048 rows, C % 16 == 0: its double sums
    associate differently), bitwise on the two-call path."""
    torch.manual_seed(31)
    P = B * H * H
    small = P <= 2048 and C % 16 == 0
    same = (lambda a, b: torch.allclose(a, b, rtol=1e-6, atol=1e-6)) if small else torch.equal
    for act, with_add in (("lrelu", True), ("relu", False), ("tanh", True)):
        y = _nhwc(torch.randn(B, C, H, H, device=DEV))
        da = _nhwc(torch.randn(B, C, H, H, device=DEV))
        add = _nhwc(torch.randn(B, C, H, H, device=DEV)) if with_add else None
        stats = torch.cat([torch.randn(C, device=DEV), torch.rand(C, device=DEV) + 0.5])
        gamma, beta = torch.rand(C, device=DEV) + 0.5, torch.randn(C, device=DEV)
        g0, b0 = torch.randn(C, device=DEV), torch.randn(C, device=DEV)
        dg1, db1 = g0.clone(), b0.clone()
        sums1, da_c = K.bn_backward_sums(da, y, stats, gamma, beta, act, 0.2)
        dy1 = K.bn_backward_apply_ex(da_c, y, stats, gamma, beta, act, 0.2, sums1, P,
                                     add=add.clone() if add is not None else None, dgamma=dg1, dbeta=db1,
                                     accumulate_affine=True)
        dg2, db2 = g0.clone(), b0.clone()
        out = add.clone() if add is not None else None  # in place over the addend, as the GP engine runs it
        sums2, dy2 = K.bn_backward_sums_apply(da, y, stats, gamma, beta, act, 0.2, add=out, out=out, dgamma=dg2,
                                              dbeta=db2, accumulate_affine=True)
        assert same(sums1, sums2) and same(dy1, dy2) and same(dg1, dg2) and same(db1, db2), (act, with_add)


@pytest.mark.parametrize("C,B,H", [(64, 8, 32), (64, 8, 16), (1024, 64, 4), (4096, 64, 4), (64, 16, 16), (36, 8, 8)])
def test_bn_backward_two_segments(K, C, B, H):
    """rgan_bn_backward_segments (both calls of the batched pass at once) == the per-call
    backward sums + apply: dy and the summed affine gradients -- bitwise for the three-launch
    path (4096 rows per call), within 1e-6 for the one-launch small-layer kernel
    (bn_bwd_small: <= 2048 rows per call, e.g. the 4x4 layer under D's dense layer), whose
    double sums associate differently; and rgan_bn_backward (one call) likewise."""
    torch.manual_seed(19)
    small = (B // 2) * H * H <= 2048
    same = (lambda a, b: torch.allclose(a, b, rtol=1e-6, atol=1e-6)) if small else torch.equal
    for act in ("lrelu", "relu", "none"):
        y = _nhwc(torch.randn(B, C, H, H, device=DEV))
        da = _nhwc(torch.randn(B, C, H, H, device=DEV))
        stats = torch.cat([torch.randn(2, C, device=DEV), torch.rand(2, C, device=DEV) + 0.5], 1)  # [2][2C]
        gamma, beta = torch.rand(C, device=DEV) + 0.5, torch.randn(C, device=DEV)
        dy1 = torch.empty_like(y)
        dg1, db1 = torch.empty(C, device=DEV), torch.empty(C, device=DEV)
        P = (B // 2) * H * H
        for k in range(2):
            sl = slice(k * B // 2, (k + 1) * B // 2)
            sums, da_c = K.bn_backward_sums(da[sl], y[sl], stats[k], gamma, beta, act, 0.2)
            K.bn_backward_apply_ex(da_c, y[sl], stats[k], gamma, beta, act, 0.2, sums, P, out=dy1[sl], dgamma=dg1,
                                   dbeta=db1, accumulate_affine=k > 0)
        dy2, dg2, db2 = K.bn_backward_segments(da, y, stats, gamma, beta, act, 0.2, True, True, torch.empty_like(y))
        assert same(dy1, dy2) and same(dg1, dg2) and same(db1, db2), act
        # one call (rgan_bn_backward) vs its sums + apply
        h = slice(0, B // 2)
        sums, da_c = K.bn_backward_sums(da[h], y[h], stats[0], gamma, beta, act, 0.2)
        dy3 = torch.empty_like(y[h])
        dg3, db3 = torch.empty(C, device=DEV), torch.empty(C, device=DEV)
        K.bn_backward_apply_ex(da_c, y[h], stats[0], gamma, beta, act, 0.2, sums, P, out=dy3, dgamma=dg3, dbeta=db3)
        dy4, dg4, db4 = K.bn_backward(da[h], y[h], stats[0], gamma, beta, act, 0.2)
        assert same(dy3, dy4) and same(dg3, dg4) and same(db3, db4), act


# (B, cin, cout, H, transposed): the data gradient of a k4 s2 p1 conv of this shape, whose
# output x (cin channels) a lower layer produced.  Conv: CONVT2 (4 phases); ConvT: CONV.
# Large M -> unsplit vector epilogue; small M -> split-K reduce.
POST_CASES = [
    (64, 128, 256, 32, False),   # CONVT2, M = 64*16*16 per phase: 512 unsplit 128x128 tiles
    (4, 128, 256, 16, False),    # CONVT2, split-K
    (8, 256, 128, 16, True),     # CONV (ConvT dgrad), M = 8*16*16 = 2048: split-K
    (64, 128, 64, 32, True),     # CONV, M = 65536: unsplit
]


@pytest.mark.parametrize("case", POST_CASES)
@pytest.mark.parametrize("mode", [1, 2])
def test_dgrad_post_op(K, case, mode):
    """rgan_conv_post (the layer below's first backward pass in the data-gradient GEMM's
    epilogue / split-K reduce) == conv_dgrad followed by that pass: mode 1 = act_backward
    (LeakyReLU, Tanh), mode 2 = bn_backward (g = da * act', the BatchNorm sums, then
    bn_backward_parts) with 1 and 2 batch segments."""
    from relativisticgan_amd.kernels import ConvGeom, Post
    B, cin, cout, H, tr = case
    torch.manual_seed(23)
    g = ConvGeom(4, 2, 1, tr)
    Ho = H // 2 if not tr else H * 2
    w = (torch.randn(cin, cout, 4, 4, device=DEV) if tr else torch.randn(cout, cin, 4, 4, device=DEV)) * 0.05
    dy = _nhwc(torch.randn(B, cout, Ho, Ho, device=DEV))
    xs = (B, cin, H, H)
    ref_da = K.conv_dgrad(dy, w, g, xs)
    for act in ("lrelu", "tanh"):
        if mode == 1:
            a = _nhwc(torch.tanh(torch.randn(xs, device=DEV))) if act == "tanh" else \
                _nhwc(F.leaky_relu(torch.randn(xs, device=DEV), 0.2))
            post = Post(1, act, 0.2, a)
            got = K.conv_dgrad(dy, w, g, xs, post=post)
            assert post.fused, (case, act)
            want = K.act_backward(ref_da, a, act, 0.2)
            assert _rel(got, want) < 1e-6, (case, act, _rel(got, want))
            continue
        y = _nhwc(torch.randn(xs, device=DEV) * 2 + 0.3)
        gamma, beta = torch.rand(cin, device=DEV) + 0.5, torch.randn(cin, device=DEV)
        for nseg in (1, 2):
            stats = torch.cat([torch.randn(nseg, cin, device=DEV) * 0.1 + 0.3,
                               torch.rand(nseg, cin, device=DEV) + 0.5], 1)
            post = Post(2, act, 0.2, y, stats=stats, gamma=gamma, beta=beta, nseg=nseg)
            gz = K.conv_dgrad(dy, w, g, xs, post=post)
            assert post.fused, (case, act, nseg)
            dyb, dgb, dbb = K.bn_backward_parts(gz, y, stats, gamma, beta, post, True, True)
            if nseg == 1:
                dyw, dgw, dbw = K.bn_backward(ref_da, y, stats[0], gamma, beta, act, 0.2)
            else:
                dyw, dgw, dbw = K.bn_backward_segments(ref_da, y, stats, gamma, beta, act, 0.2, True, True,
                                                       torch.empty_like(y))
            for k, (u, v) in {"dy": (dyb, dyw), "dgamma": (dgb, dgw), "dbeta": (dbb, dbw)}.items():
                assert _rel(u, v) < 1e-5, (case, act, nseg, k, _rel(u, v))


@pytest.mark.parametrize("B,cin,cout,act", [(32, 128, 1024, "relu"), (64, 128, 512, "tanh"), (64, 64, 256, "relu"),
                                         (32, 100, 256, "relu")])
def test_first_layer_fused(K, B, cin, cout, act):
    """rgan_g1_fwd_bn (G's 1x1 -> 4x4 ConvTranspose2d + train-mode BatchNorm2d + act in one
    launch) and rgan_g1_wgrad vs torch fp64: y, a, batch statistics, running statistics and
    num_batches_tracked, and the weight gradient (written and accumulated).  Cin = 100 (no
    instantiation) must be refused by g1_ok (the GEMM + BatchNorm path runs)."""
    from relativisticgan_amd.kernels import ConvGeom
    torch.manual_seed(29)
    g = ConvGeom(4, 1, 0, True)
    z = torch.randn(B, cin, 1, 1, device=DEV)
    w = torch.randn(cin, cout, 4, 4, device=DEV) * 0.05
    if cin not in (64, 128):
        assert not K.g1_ok(z, w, g)
        return
    assert K.g1_ok(z, w, g)
    gamma, beta = torch.rand(cout, device=DEV) + 0.5, torch.randn(cout, device=DEV) * 0.1
    rm, rv = torch.randn(cout, device=DEV) * 0.1, torch.rand(cout, device=DEV) + 0.5
    nbt = torch.zeros((), dtype=torch.long, device=DEV)
    rm0, rv0 = rm.clone(), rv.clone()
    y, a, stats = K.g1_fwd_bn(z, w, gamma, beta, 1e-5, 0.1, rm, rv, nbt, act, 0.0)
    y64 = F.conv_transpose2d(z.double().cpu(), w.double().cpu())
    mean = y64.mean((0, 2, 3))
    var = y64.var((0, 2, 3), unbiased=False)
    a64 = F.batch_norm(y64, None, None, gamma.double().cpu(), beta.double().cpu(), training=True, eps=1e-5)
    a64 = torch.relu(a64) if act == "relu" else torch.tanh(a64)
    assert K.is_nhwc(y) and K.is_nhwc(a)
    assert _rel(y, y64) < 1e-6 and _rel(a, a64) < 1e-5
    assert _rel(stats[:cout], mean) < 1e-6 and _rel(stats[cout:], 1 / torch.sqrt(var + 1e-5)) < 1e-6
    n = B * 16
    assert _rel(rm, 0.9 * rm0.double().cpu() + 0.1 * mean) < 1e-6
    assert _rel(rv, 0.9 * rv0.double().cpu() + 0.1 * var * n / (n - 1)) < 1e-6
    assert int(nbt.item()) == 1
    dy = _nhwc(torch.randn(B, cout, 4, 4, device=DEV))
    dw = K.g1_wgrad(z, dy, tuple(w.shape))
    dw64 = torch.einsum("bi,bohw->iohw", z.double().cpu().flatten(1), dy.double().cpu())
    assert _rel(dw, dw64) < 1e-6
    base = torch.randn_like(dw)
    acc = base.clone()
    K.g1_wgrad(z, dy, tuple(w.shape), out=acc)
    assert _rel(acc - base, dw64) < 1e-5


@pytest.mark.parametrize("mode", [1, 2])
def test_dgrad_post_op_emulated(K, mode):
    """The post-op GEMM on the opt-in fp32-on-bf16x6 products (gemm_post_bf16x6) == the fp32
    post-op GEMM within the emulation's accuracy (unsplit CONVT2 data gradient)."""
    from relativisticgan_amd.kernels import ConvGeom, Post
    torch.manual_seed(31)
    g = ConvGeom(4, 2, 1, False)
    B, cin, cout, H = 64, 128, 256, 32
    w = torch.randn(cout, cin, 4, 4, device=DEV) * 0.05
    dy = _nhwc(torch.randn(B, cout, H // 2, H // 2, device=DEV))
    xs = (B, cin, H, H)
    x = _nhwc(torch.randn(xs, device=DEV))
    if mode == 1:
        mk = lambda: Post(1, "lrelu", 0.2, _nhwc(F.leaky_relu(x, 0.2)))  # noqa: E731
    else:
        st = torch.cat([torch.full((1, cin), 0.1, device=DEV), torch.full((1, cin), 1.3, device=DEV)], 1)
        mk = lambda: Post(2, "relu", 0.0, x, stats=st, nseg=1)  # noqa: E731
    p32 = mk()
    want = K.conv_dgrad(dy, w, g, xs, post=p32)
    prev = K.set_gemm_emulation(True)
    try:
        pe = mk()
        got = K.conv_dgrad(dy, w, g, xs, post=pe)
    finally:
        K.set_gemm_emulation(prev)
    assert p32.fused and pe.fused
    assert _rel(got, want) < 2e-6, _rel(got, want)
    if mode == 2:
        assert _rel(pe.part, p32.part) < 2e-6


@pytest.mark.parametrize("B,cin,cout,H,tr", [(2, 8, 16, 16, False), (64, 128, 256, 16, False), (1, 256, 512, 8, False),
                                             (2, 16, 8, 8, True), (16, 256, 128, 8, True), (4, 24, 40, 12, False)])
def test_wgrad_write_accumulate_into(K, B, cin, cout, H, tr):
    """4x4 weight gradients (FAST tap-major tiles + taps_transpose, split-K for small batches,
    the generic path for Cin = 24), written, accumulated (``out``) and into a given tensor
    (``into``) -- vs torch fp64."""
    g = K.ConvGeom(4, 2, 1, tr)
    torch.manual_seed(B + cin)
    x = _nhwc(torch.randn(B, cin, H, H, device=DEV))
    Ho = 2 * H if tr else H // 2
    dy = _nhwc(torch.randn(B, cout, Ho, Ho, device=DEV))
    wshape = (cin, cout, 4, 4) if tr else (cout, cin, 4, 4)
    w64 = torch.zeros(wshape, dtype=torch.float64, requires_grad=True)
    (F.conv_transpose2d if tr else F.conv2d)(x.double().cpu(), w64, stride=2, padding=1).backward(dy.double().cpu())
    dw, _ = K.conv_wgrad(x, dy, g, wshape)
    assert _rel(dw, w64.grad) < 2e-6
    base = torch.randn(wshape, device=DEV)
    acc = base.clone()
    K.conv_wgrad(x, dy, g, wshape, out=acc)
    assert _rel(acc - base, w64.grad) < 2e-5
    into = torch.full(wshape, float("nan"), device=DEV)
    K.conv_wgrad(x, dy, g, wshape, into=into)
    assert torch.equal(into, dw)


# arch 1's 3x3 stride-1 image layers (GLI:202 / 222-223, 260 / 300-301): the narrow-out
# per-pixel kernel (conv3_narrow_out: the output layer's forward, the input layer's data
# gradient), the narrow weight gradient (wgrad3_narrow + the WGRAD split reduce), and the
# generic GEMM for the rest.  (B, H): pixel counts below one chunk, a few chunks (generic
# reduce) and the C4 shape (wide reduce).
@pytest.mark.parametrize("nc", [1, 3, 4])
@pytest.mark.parametrize("B,H", [(2, 5), (3, 16), (32, 32)])
def test_conv3x3_narrow_layers(K, nc, B, H):
    g = K.ConvGeom(3, 1, 1, False)
    torch.manual_seed(nc * 100 + B)
    s = torch.tensor([0.5], device=DEV)
    # D's input layer: nc -> 64 over the NCHW image
    img = torch.randn(B, nc, H, H, device=DEV)
    w_in = torch.randn(64, nc, 3, 3, device=DEV) * 0.2
    b_in = torch.randn(64, device=DEV)
    y = K.conv_fwd(img, w_in, g, bias=b_in, act="lrelu", alpha=0.1, wscale=s)
    assert _rel(y, F.leaky_relu(_ref_conv(img, w_in * 0.5, g, b_in), 0.1)) < 3e-6
    dy = _nhwc(torch.randn(B, 64, H, H, device=DEV))
    x64 = img.double().cpu().requires_grad_(True)
    w64 = (w_in * 0.5).double().cpu().requires_grad_(True)
    F.conv2d(x64, w64, padding=1).backward(dy.double().cpu())
    dx = K.conv_dgrad(dy, w_in, g, img.shape, wscale=s, like=img)
    assert _rel(dx, x64.grad) < 3e-6
    dw, db = K.conv_wgrad(img, dy, g, w_in.shape, with_bias=True)
    assert _rel(dw, w64.grad) < 3e-6
    assert _rel(db, dy.double().cpu().sum((0, 2, 3))) < 3e-6
    acc = torch.randn_like(w_in)
    base = acc.clone()
    K.conv_wgrad(img, dy, g, w_in.shape, out=acc)
    assert _rel(acc - base, w64.grad) < 2e-5
    # G's output layer: 64 -> nc, NCHW image out with tanh
    x = _nhwc(torch.randn(B, 64, H, H, device=DEV))
    w_out = torch.randn(nc, 64, 3, 3, device=DEV) * 0.1
    b_out = torch.randn(nc, device=DEV)
    y = K.conv_fwd(x, w_out, g, bias=b_out, act="tanh", wscale=s, nchw_out=True)
    assert _rel(y, torch.tanh(_ref_conv(x, w_out * 0.5, g, b_out))) < 3e-6
    gy = torch.randn(B, nc, H, H, device=DEV)
    x64 = x.double().cpu().requires_grad_(True)
    w64 = (w_out * 0.5).double().cpu().requires_grad_(True)
    F.conv2d(x64, w64, padding=1).backward(gy.double().cpu())
    dx = K.conv_dgrad(gy, w_out, g, x.shape, wscale=s)
    assert _rel(dx, x64.grad) < 3e-6
    dw, _ = K.conv_wgrad(x, gy, g, w_out.shape)
    assert _rel(dw, w64.grad) < 3e-6


# conv3_narrow_out's channel-lane layout (C / 4 lanes per pixel, 64 / (C / 4) pixels per wave
# step, `steps` groups per wave): C = 4 / 8 (fewer lanes than outputs), 16, 128 (C4) and 256 (one
# pixel per step), ragged pixel counts, pad 0; C = 48 is not a power of two and takes the GEMM.
@pytest.mark.parametrize("C", [4, 8, 16, 48, 128, 256])
@pytest.mark.parametrize("B,H,pad", [(3, 17, 1), (32, 32, 1), (2, 9, 0)])
def test_conv3x3_narrow_channel_widths(K, C, B, H, pad):
    g = K.ConvGeom(3, 1, pad, False)
    Ho = H + 2 * pad - 2
    s = torch.tensor([0.5], device=DEV)
    for nc in (1, 3, 4):
        torch.manual_seed(C * 10 + nc + B)
        x = _nhwc(torch.randn(B, C, H, H, device=DEV))
        w = torch.randn(nc, C, 3, 3, device=DEV) * 0.1
        b = torch.randn(nc, device=DEV)
        y = K.conv_fwd(x, w, g, bias=b, act="tanh", wscale=s, nchw_out=True)
        assert _rel(y, torch.tanh(_ref_conv(x, w * 0.5, g, b))) < 3e-6, (nc, "fwd")
        # the mirror: D's nc-channel input layer's data gradient (C-channel dy, flipped taps)
        w_in = torch.randn(C, nc, 3, 3, device=DEV) * 0.1
        dy = _nhwc(torch.randn(B, C, Ho, Ho, device=DEV))
        x64 = torch.zeros(B, nc, H, H, dtype=torch.float64, requires_grad=True)
        F.conv2d(x64, (w_in * 0.5).double().cpu(), padding=pad).backward(dy.double().cpu())
        dx = K.conv_dgrad(dy, w_in, g, (B, nc, H, H), wscale=s)
        assert _rel(dx, x64.grad) < 3e-6, (nc, "dgrad")


@pytest.mark.parametrize("B,C,H", [(1, 16, 1), (3, 64, 5), (64, 512, 4), (32, 256, 8), (2, 64, 33), (64, 64, 8),
                                   (8, 20, 4), (64, 128, 16)])
def test_channel_sum(K, B, C, H):
    """Bias-gradient channel sums: the one-launch kernel (<= 2048 rows, C % 16 == 0) and the
    two-level one (more rows / other C), written and accumulated, vs torch fp64."""
    torch.manual_seed(B * C + H)
    t = _nhwc(torch.randn(B, C, H, H, device=DEV))
    ref = t.double().cpu().sum((0, 2, 3))
    out = torch.full((C,), float("nan"), device=DEV)
    K.channel_sum(t, out)
    assert _rel(out, ref) < 1e-6
    base = torch.randn(C, device=DEV)
    acc = base.clone()
    K.channel_sum(t, acc, accumulate=True)
    assert _rel(acc.double().cpu() - base.double().cpu(), ref) < 1e-5
