/*
 * rgan.h — C-ABI of the MI355X (gfx950) RelativisticGAN training core.
 *
 * The reference has no FFI of its own: its hot path is the module-level PyTorch
 * training loop of code/GAN_losses_iter.py (GLI).  Each entry point below replaces
 * the PyTorch op(s) that loop reaches, cited per function.
 *
 * Conventions:
 *   - plain device pointers (fp32 unless stated) and sizes; no torch types;
 *   - the caller allocates every output and every workspace; kernels never allocate;
 *   - return 0 on success, a hipError_t-compatible code otherwise
 *     (RGAN_EINVAL = invalid descriptor / sizes, checked on the host before launch);
 *   - every launch goes on `stream` (hipStream_t passed as void*); no host syncs, so
 *     every entry point is hipGraph-capturable.
 */
#ifndef RGAN_H
#define RGAN_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RGAN_EINVAL 1001

/* ABI revision.  2: rgan_adam_packed takes step = device float[2] (step[1] is the
 * call's uint32 arrival ticket, zero before the first call); revision 1 took float[1].
 * 3: adds rgan_conv_wgrad_rows.  4: adds rgan_bn_segment_apply and rgan_bn_backward_sums_apply. */
#define RGAN_ABI_VERSION 4

/* Activation codes fused into epilogues (GLI:345,370,388,417,437,450; SELU GLI:338). */
enum {
  RGAN_ACT_NONE = 0, RGAN_ACT_RELU = 1, RGAN_ACT_LRELU = 2, RGAN_ACT_TANH = 3,
  RGAN_ACT_SIGMOID = 4, RGAN_ACT_SELU = 5
};

/* One 2-D convolution as the reference's torch.nn.Conv2d / ConvTranspose2d sees it.
 * "x" is the op's input image, "y" its output.  Element strides are given for
 * (batch, channel, h, w) so NCHW (reference layout) and NHWC (internal layout,
 * torch channels_last) tensors are both accepted.  Weights are in torch layout:
 * Conv2d [cout][cin][kh][kw], ConvTranspose2d [cin][cout][kh][kw], contiguous. */
typedef struct RganConv {
  int batch;
  int cin, hin, win;
  int cout, hout, wout;
  int kh, kw, stride, pad;
  int transposed;          /* 0: Conv2d, 1: ConvTranspose2d */
  long long xs[4];         /* x strides (b, c, h, w) in elements */
  long long ys[4];         /* y strides (b, c, h, w) in elements */
} RganConv;

/* Workspace bytes needed by rgan_conv_{fwd,dgrad,wgrad}; `which` = 0 fwd, 1 dgrad, 2 wgrad
 * (wgrad's includes the bias-gradient reduction scratch);
 * `prepacked` != 0: the caller passes packed weights (no packing scratch).  0 = unsupported. */
size_t rgan_conv_workspace(const RganConv* d, int which, int prepacked);

/* Kernel-ready weight layout for which = 0 (fwd) or 1 (dgrad): [phases][N][K] floats for
 * the implicit GEMMs (k contiguous: the B operand's LDS rows), [4][Cin][16] for the narrow
 * (<= 4 output channel) transposed conv.  Packing is separated so callers can cache it per weight version (weights change
 * only at the optimizer step, but each net is run 2-4 times per iteration).
 * rgan_conv_pack_floats returns 0 when the op reads the torch layout directly (narrow
 * 4x4 convs with <= 4 input channels) -- or when the descriptor is unsupported, which
 * rgan_conv_workspace reports separately (0). */
size_t rgan_conv_pack_floats(const RganConv* d, int which);
int rgan_conv_pack(const RganConv* d, int which, const float* w, float* packed, void* stream);
/* n packs at once (the stale layouts of a net after its optimizer step, torch.optim's
 * step at GLI:659/712 being what moved them): entry i = rgan_conv_pack(d[i], which[i], w[i],
 * packed[i]); the tiled layouts share one launch per 16, others get their own. */
int rgan_conv_pack_batch(int n, const RganConv* const* d, const int* which, const float* const* w,
                         float* const* packed, void* stream);

/* y = act(conv(x, w) * (*wscale) + bias).  Replaces Conv2d/ConvTranspose2d.forward
 * (GLI:336,361,387,410,428,448; arch 1 GLI:202-223,260-302) fused with the
 * following activation when no BatchNorm sits between them.  wpacked: nullable
 * rgan_conv_pack(which=0) output (then w may be NULL).  wscale: nullable device scalar
 * (spectral norm's 1/sigma, torch/nn/utils/spectral_norm.py:115-116), applied to the
 * accumulator in the epilogue. */
int rgan_conv_fwd(const RganConv* d, const float* x, const float* w, const float* wpacked,
                  const float* wscale, const float* bias, float* y, int act, float act_alpha,
                  void* ws, size_t ws_bytes, void* stream);

/* Conv2d/ConvTranspose2d.forward feeding a train-mode BatchNorm2d (GLI:361-366,387-391,
 * 428-433): y = conv(x, w) * (*wscale) + bias, and -- when the GEMM's vector epilogue
 * or its split-K reduce covers the layer -- the BatchNorm batch statistics of y as per-64-row
 * segment moments bn_part[S][2][C] = (sum y, sum y^2) in double, computed from the finished
 * tile in LDS or from the reduced rows in registers (no re-read of y).
 * S = rgan_conv_bn_segments(d, segs) (0: the epilogue cannot, use rgan_bn_stats); `segs`
 * equal batch segments are kept apart (the batched D(x)/D(G(z)) call: segment k's rows are
 * segments [k*S/segs, (k+1)*S/segs)).  *fused (host int) = 1 when bn_part was written.
 * Merge with rgan_bn_segment_stats. */
long long rgan_conv_bn_segments(const RganConv* d, int segs);
int rgan_conv_fwd_bn(const RganConv* d, const float* x, const float* w, const float* wpacked,
                     const float* wscale, const float* bias, float* y, void* ws, size_t ws_bytes,
                     double* bn_part, long long part_segments, int segs, int* fused, void* stream);

/* dx = d conv / d x applied to dy  (aten convolution_backward, grad_input). */
int rgan_conv_dgrad(const RganConv* d, const float* dy, const float* w, const float* wpacked,
                    const float* wscale, float* dx, void* ws, size_t ws_bytes, void* stream);

/* Post-op for the layer that PRODUCED a GEMM's output operand, applied where the output
 * value is final (the GEMM epilogue or its split-K reduce) instead of a separate pass over
 * it.  `x` has the output's element strides (same shape).
 *   mode 1 (activation backward, aten's threshold/leaky_relu/tanh backward of GLI:345,370,
 *          417 behind the conv's data gradient): out = v * act'(x), x = the producer's
 *          activation output;
 *   mode 2 (BatchNorm2d backward sums, the first half of aten native_batch_norm_backward,
 *          GLI:341-345/366-370/433-437): out = g = v * act'(x * al + be), x = the producer's
 *          BatchNorm input y, al = gamma * invstd, be = beta - mean * al from stats[k] of the
 *          output row's batch segment k (nseg equal segments of every phase's rows), and
 *          part[S][2][C] = (sum g, sum g (y - mean)) per 64-row segment in double, S =
 *          rgan_conv_post_segments(...); finish with rgan_bn_backward_parts. */
typedef struct RganPost {
  int mode;                /* 1 or 2 */
  int act;                 /* RGAN_ACT_* of the producer */
  float alpha;
  int nseg;                /* mode 2: batch segments with their own statistics (1 or 2) */
  const float* x;          /* activation output (mode 1) / BatchNorm input y (mode 2) */
  const float* stats;      /* mode 2: [nseg][2C] (mean, invstd) */
  const float* gamma;      /* mode 2: nullable */
  const float* beta;       /* mode 2: nullable */
  double* part;            /* mode 2: [part_segments][2][C] */
  long long part_segments;
} RganPost;

/* rgan_conv_fwd (which = 0, act none, no bias) or rgan_conv_dgrad (which = 1) with a
 * producer post-op.  *fused (host int) = 1 when the post-op was applied (else `out` holds
 * the plain result and the caller runs the separate pass).  rgan_conv_post_segments: S for
 * mode 2 (0: this GEMM cannot emit the sums) and (nullable *phases) the phase-major blocks
 * the S segments come in (4 for a k4 s2 p1 Conv2d data gradient, else 1). */
long long rgan_conv_post_segments(const RganConv* d, int which, int mode, int nseg, int* phases);
int rgan_conv_post(const RganConv* d, int which, const float* in, const float* w, const float* wpacked,
                   const float* wscale, float* out, void* ws, size_t ws_bytes, const RganPost* post,
                   int* fused, void* stream);

/* G's first layer on its 1x1 input (GLI:334-345: ConvTranspose2d(z, Cout, 4, 1, 0) + train-
 * mode BatchNorm2d + activation) in one launch: y[b][t][c] = sum_ci z[b][ci] W[ci][c][t]
 * (t = 4 kh + kw; y, a NHWC [B][4][4][Cout]), the BatchNorm batch statistics of each channel
 * over its B x 16 values (exact two-pass, double), running statistics + num_batches_tracked
 * updated as torch does, stats = (mean, invstd) [2][Cout], a = act(BN(y)).  z [B][Cin]
 * contiguous, 16-B aligned; B in {32, 64} (the batch sizes of BASELINE's configs); Cin (z size)
 * in {64, 128}; Cout % 16 == 0 (other shapes run the GEMM + BatchNorm entry points).
 * rgan_g1_wgrad: its weight gradient dW[ci][c][t] (+)= sum_b z[b][ci] dy[b][t][c] (dy NHWC). */
int rgan_g1_fwd_bn(const float* z, int B, int Cin, const float* w, int Cout, const float* gamma,
                   const float* beta, float eps, float momentum, float* running_mean, float* running_var,
                   long long* num_batches_tracked, int act, float act_alpha, float* y, float* a, float* stats,
                   void* stream);
int rgan_g1_wgrad(const float* z, int B, int Cin, const float* dy, int Cout, float* dw, int accumulate,
                  void* stream);

/* dw = d conv / d w applied to dy (aten convolution_backward, grad_weight), written
 * in torch weight layout; dbias (nullable) = per-output-channel sum of dy.
 * accumulate != 0: dw += ..., dbias += ... (autograd's gradient accumulation into an
 * existing .grad, GLI:605/624/658's repeated backward calls, done in the GEMM's epilogue
 * instead of a separate add pass). */
int rgan_conv_wgrad(const RganConv* d, const float* x, const float* dy, float* dw, float* dbias,
                    int accumulate, void* ws, size_t ws_bytes, void* stream);
/* The same with dbias summed over the pixel rows p >= dbias_row0 only (p = (b, h, w) in
 * order; 0 <= dbias_row0 < batch*hout*wout): the WGAN-GP double backward's weight gradient
 * runs one GEMM over [adjoint; forward] row pairs while the bias gradient is the forward
 * half's alone.  rgan_conv_wgrad(...) == rgan_conv_wgrad_rows(..., 0, ...). */
int rgan_conv_wgrad_rows(const RganConv* d, const float* x, const float* dy, float* dw, float* dbias,
                         long long dbias_row0, int accumulate, void* ws, size_t ws_bytes, void* stream);

/* ---- --NN_conv blocks: Upsample(scale_factor=2, nearest) + Conv2d(k3, s1, p1) ----
 * (GLI:351-356 middle, GLI:377-382 end).  conv3x3(up2(x), W) equals a k4 s2 p1
 * ConvTranspose2d of x with the folded weight Wt = A W A^T per 3x3 slice
 * (A = [[0,0,1],[0,1,1],[1,1,0],[1,0,0]]), so the layer runs as rgan_conv_* with
 * transposed = 1, k = 4, stride 2, pad 1 on Wt.
 * rgan_nn_fold_weight: W [cout][cin][3][3] -> Wt [cin][cout][4][4] (16-byte aligned).
 * rgan_nn_unfold_grad: the adjoint, dWt [cin][cout][4][4] -> dW [cout][cin][3][3]
 * (the Conv2d weight gradient, aten convolution_backward grad_weight). */
int rgan_nn_fold_weight(const float* w, int cout, int cin, float* wt, void* stream);
int rgan_nn_unfold_grad(const float* dwt, int cout, int cin, float* dw, void* stream);

/* ---- image layers (k4 s2 p1 with <= 4 image channels: GLI:404 D start, GLI:386 G end) ----
 * rgan_patches_k4s2: patch matrix of an image [B][C][H][W] (element strides b,c,h,w; C <= 4,
 * H, W even) on the half-size grid: X[(b, i, j)][4 t + c] = img[b][c][2i-1+kh][2j-1+kw],
 * t = 4 kh + kw, zero outside the image and for c >= C; X is [B*(H/2)*(W/2)][64] floats,
 * 16-byte aligned.  Every image-layer GEMM then runs as a 1x1 rgan_conv_* over X.
 * rgan_patch_weight: W1[o][4 t + c] = w[o*row_stride + c*channel_stride + t] (rows x 64).
 * rgan_unpatch_grad: dw[o][c][t] = g1[o*row_stride + (4 t + c)*col_stride] (rows x C x 16). */
int rgan_patches_k4s2(const float* img, int batch, int channels, int height, int width,
                      const long long* strides, float* patches, void* stream);
int rgan_patch_weight(const float* w, int rows, int channels, long long row_stride, long long channel_stride,
                      float* w1, void* stream);
int rgan_unpatch_grad(const float* g1, int rows, int channels, long long row_stride, long long col_stride,
                      float* dw, int accumulate, void* stream);

/* ---- image export (GLI:563-565 sample grid, GLI:759-768 extra FID images) ----
 * torchvision.utils.save_image's float -> uint8 step on the device: t = x*scale + shift;
 * optional normalize with range = device float[2] {min, max} of the batch
 * (make_grid(normalize=True): t = (clamp(t, lo, hi) - lo) / max(hi - lo, 1e-5)); then
 * u8 = trunc(clamp(t*255 + 0.5, 0, 255)).  x: [B][C][H][W] with element strides
 * strides[4]; grid = 0: out [B][H][W][C] (one image per file, padding 0);
 * grid = 1: make_grid layout [Hg][Wg][C], nrow tiles per row, `padding` pixels of 0.
 * rgan_minmax: out2 = {min, max} of x[0..n) (ws: rgan_minmax_ws_bytes). */
/* Real-image batch (GLI:173-177 + ToTensor/Normalize GLI:160-166): out[b] = (u8 / 255 - 0.5)
 * / 0.5 of images[idx[b]], images = decoded uint8 [N][per] resident on the device
 * (per = C*S*S, a multiple of 4; out 16-byte aligned). */
int rgan_gather_images_u8(const unsigned char* images, const long long* idx, int batch, long long per,
                          float* out, void* stream);
size_t rgan_minmax_ws_bytes(long long n);
int rgan_minmax(const float* x, long long n, float* out2, void* ws, void* stream);
int rgan_images_to_u8(const float* x, int B, int C, int H, int W, const long long* strides,
                      float scale, float shift, const float* range, int grid, int nrow, int padding,
                      unsigned char* out, void* stream);

/* ---- BatchNorm2d, train mode (GLI:341,366,433; arch 1 GLI:204-218,262-297) ----
 * Tensors are [batch*h*w][C] with element strides (sp = pixel stride, sc = channel
 * stride); P = batch*h*w.  stats = float[2*C] workspace slot receiving (mean, invstd).
 * Running stats follow torch: r = (1-m) r + m * stat, unbiased var for running_var;
 * num_batches_tracked (int64, nullable) += 1.  `partial` workspace: rgan_bn_partial_bytes. */
size_t rgan_bn_partial_bytes(long long P, int C);
int rgan_bn_stats(const float* y, long long P, int C, long long sp, long long sc,
                  float eps, float momentum, float* running_mean, float* running_var,
                  long long* num_batches_tracked, float* stats, void* partial, void* stream);
/* rgan_conv_fwd_bn's segment moments [s0, s1) -> stats + running stats (moments == NULL),
 * or this rank's (count, mean, M2) double[3*C] for SyncBN (moments != NULL, as
 * rgan_bn_moments).  Chan merges in a fixed order (deterministic). */
int rgan_bn_segment_stats(const double* part, long long s0, long long s1, int C, int seg_rows,
                          float eps, float momentum, float* running_mean, float* running_var,
                          long long* num_batches_tracked, float* stats, double* moments, void* stream);
/* The batched D pass's two calls (GLI:580-605 run D(x) then D(x_fake)) in one launch each:
 * segment stats of the nseg (1 or 2) equal halves of segments [s0, s1) -> stats[nseg][2C],
 * running statistics updated in call order; and the normalisation + activation of y's nseg
 * equal row ranges with their stats rows (dense NHWC y and a, P % nseg == 0). */
int rgan_bn_segment_stats_n(const double* part, long long s0, long long s1, int nseg, int C, int seg_rows,
                            float eps, float momentum, float* running_mean, float* running_var,
                            long long* num_batches_tracked, float* stats, void* stream);
int rgan_bn_apply_segments(const float* y, long long P, int C, int nseg, const float* stats, const float* gamma,
                           const float* beta, int act, float act_alpha, float* a, void* stream);
/* Both of the above in one call (ABI 4): stats[nseg][2C] of y's nseg equal row ranges from
 * rgan_conv_fwd_bn's segment sums part[S][2][C] (P == S * seg_rows), running statistics in call
 * order, and a = act(BN(y)).  A small layer (S / nseg <= 64 segments) runs as ONE launch whose
 * blocks each merge their channels' segment sums in the same fixed order; a larger one as
 * rgan_bn_segment_stats_n + rgan_bn_apply_segments.  Dense NHWC y and a, 16-byte aligned. */
int rgan_bn_segment_apply(const double* part, long long S, int nseg, int seg_rows, const float* y, long long P,
                          int C, float eps, float momentum, float* running_mean, float* running_var,
                          long long* num_batches_tracked, const float* gamma, const float* beta, int act,
                          float act_alpha, float* stats, float* a, void* stream);
/* a = act(gamma * (y - mean) * invstd + beta)  (torch's alpha/beta form) */
int rgan_bn_apply(const float* y, long long P, int C, long long sp, long long sc,
                  const float* stats, const float* gamma, const float* beta,
                  int act, float act_alpha, float* a, long long asp, long long asc, void* stream);
/* Staged form for data parallelism (SyncBN): local moments (count, mean, M2) as
 * double[3][C]; the caller gathers them from all ranks into [nranks][3][C] and merges
 * in rank order with rgan_bn_finalize (Chan's parallel variance; deterministic). */
int rgan_bn_moments(const float* y, long long P, int C, long long sp, long long sc,
                    double* moments, void* partial, void* stream);
int rgan_bn_finalize(const double* moments, int nranks, int C, float eps, float momentum,
                     float* running_mean, float* running_var, long long* num_batches_tracked,
                     float* stats, void* stream);
/* The batched D pass's two calls' BatchNorm backward (GLI:605/624/644 through each call's
 * BatchNorm) in three launches instead of six: dy of y's nseg (1 or 2) equal row ranges, each
 * with its stats row [nseg][2C] and its own sums; dgamma / dbeta = the segments' sum.  Dense
 * NHWC da, y, dy; partial >= nseg * rgan_bn_partial_bytes(P / nseg, C). */
int rgan_bn_backward_segments(const float* da, const float* y, long long P, int C, int nseg, const float* stats,
                              const float* gamma, const float* beta, int act, float act_alpha, float* dy,
                              float* dgamma, float* dbeta, void* partial, void* stream);
/* The rest of the BatchNorm backward after a GEMM's post-op wrote g = da * act' and the
 * segment sums (rgan_conv_post mode 2): merge part[S][2][C] (phases phase-major blocks of
 * S / phases segments, each split into nseg batch segments) into sums[nseg][2][C] (caller's
 * scratch), then dy = al (g - sum_g / Pk - (y - mean) invstd^2 sum_gx / Pk) per batch segment,
 * dgamma / dbeta = the segments' sum (nullable).  Dense NHWC g, y, dy. */
int rgan_bn_backward_parts(const float* g, const float* y, long long P, int C, int nseg, const float* stats,
                           const float* gamma, const float* beta, const double* part, long long S, int phases,
                           float* dy, float* dgamma, float* dbeta, double* sums, void* stream);
/* The staged backward's sums and apply in one call (ABI 4; one process or per-shard BN): writes
 * sums[2][C] = (sum g, sum g (y - mean)), g = da * act' (the WGAN-GP engine keeps them for the
 * double backward), dy = BN-backward(g) + add (add nullable), dgamma / dbeta written or, with
 * accumulate_affine, added into (nullable).  Dense NHWC da, y, dy, add.  P <= 2048 rows (C % 16
 * == 0): one launch; otherwise rgan_bn_backward_sums + rgan_bn_backward_apply_ex.  partial:
 * rgan_bn_partial_bytes(P, C). */
int rgan_bn_backward_sums_apply(const float* da, const float* y, long long P, int C, const float* stats,
                                const float* gamma, const float* beta, int act, float act_alpha, const float* add,
                                float* dy, float* dgamma, float* dbeta, int accumulate_affine, double* sums,
                                void* partial, void* stream);
/* Backward through act(BN(y)): given da, produce dy, dgamma, dbeta. */
int rgan_bn_backward(const float* da, long long dsp, long long dsc,
                     const float* y, long long P, int C, long long sp, long long sc,
                     const float* stats, const float* gamma, const float* beta,
                     int act, float act_alpha, float* dy, long long ysp, long long ysc,
                     float* dgamma, float* dbeta, void* partial, void* stream);
/* Staged backward: local sums double[2][C] = (sum g, sum g*(y-mean)), g = da*act'; the
 * caller all-reduces them over ranks, then apply with the global pixel count P_global.
 * All BN sums accumulate in double (torch's CPU kernel does too): the backward sums can
 * cancel almost completely and a float accumulator leaves a coherent error in dy. */
int rgan_bn_backward_sums(const float* da, long long dsp, long long dsc, const float* y,
                          long long P, int C, long long sp, long long sc, const float* stats,
                          const float* gamma, const float* beta, int act, float act_alpha,
                          double* sums, void* partial, void* stream);
int rgan_bn_backward_apply(const float* da, long long dsp, long long dsc, const float* y,
                           long long P, int C, long long sp, long long sc, const float* stats,
                           const float* gamma, const float* beta, int act, float act_alpha,
                           const double* sums, long long P_global, float* dy, long long ysp,
                           long long ysc, float* dgamma, float* dbeta, void* stream);

/* rgan_bn_backward_apply plus: add (nullable, y's strides) is added to dy, and
 * accumulate_affine != 0 adds dgamma/dbeta into the given buffers (the batched D
 * step's two BN calls, the WGAN-GP double backward's second-order terms). */
int rgan_bn_backward_apply_ex(const float* da, long long dsp, long long dsc, const float* y,
                              long long P, int C, long long sp, long long sc, const float* stats,
                              const float* gamma, const float* beta, int act, float act_alpha,
                              const double* sums, long long P_global, const float* add, float* dy,
                              long long ysp, long long ysc, float* dgamma, float* dbeta,
                              int accumulate_affine, void* stream);

/* ---- WGAN-GP double backward (GLI:655 create_graph=True, differentiated by GLI:658) ----
 * Layer act(BN(y)) with batch statistics `stats`, whose create-graph backward took dh
 * (the upstream gradient) to dy = BNback(dh act'(z)) with first-order sums
 * first_sums = (sum e, sum e (y - mean)) [2C] (rgan_bn_backward_sums, global).  Given
 * a = dP/d(dy) (all [P][C] with strides sp, sc):
 *   rgan_bn_dd_sums stage 1: sums[3][C] = (sum a, sum a xhat, sum a e);
 *                   stage 2 (only for act'' != 0: tanh, sigmoid, SELU; needs the global
 *                   stage-1 sums): sums[2][C] = (sum t, sum t xhat);
 *   rgan_bn_dd_apply: adj_dh = dP/d(dh) (nullable), ydir = the direct dP/dy of the
 *                   double backward, dgamma2/dbeta2 (nullable, accumulate_affine: +=)
 *                   its gamma/beta terms (from the *_local sums when given: under
 *                   SyncBN the gradient all-reduce sums them over ranks).
 * Cross-rank: the caller all-reduces first_sums and each stage's sums (SyncBN) and
 * passes the global pixel count P_global.  partial: rgan_bn_dd_partial_bytes. */
size_t rgan_bn_dd_partial_bytes(long long P, int C);
int rgan_bn_dd_sums(const float* a, const float* y, const float* dh, long long P, int C,
                    long long sp, long long sc, const float* stats, const float* gamma,
                    const float* beta, int act, float act_alpha, int stage, const double* stage1,
                    long long P_global, double* sums, void* partial, void* stream);
int rgan_bn_dd_apply(const float* a, const float* y, const float* dh, long long P, int C,
                     long long sp, long long sc, const float* stats, const float* gamma,
                     const float* beta, int act, float act_alpha, const double* first_sums,
                     const double* stage1, const double* stage2, const double* stage1_local,
                     const double* stage2_local, long long P_global, float* adj_dh, float* ydir,
                     float* dgamma2, float* dbeta2, int accumulate_affine, void* stream);
/* Without BatchNorm (dy = dh act'(y), act_out = act(y)): adj_dh = a act'(y),
 * ydir = a dh act''(y); either output nullable. */
int rgan_act_dd(const float* a, const float* act_out, const float* dh, long long n, int act,
                float act_alpha, float* adj_dh, float* ydir, void* stream);

/* ---- elementwise ---- */
/* dx = da * act'(a) where a = act(x) is the saved activation output. */
int rgan_act_backward(const float* da, const float* a, long long n, int act, float act_alpha,
                      float* dx, void* stream);
/* dx = da * act'(a) + add (add nullable, same layout) */
int rgan_act_backward_ex(const float* da, const float* a, const float* add, long long n, int act,
                         float act_alpha, float* dx, void* stream);
/* out[n] (+)= sum over pixels of t (per channel; bias gradient), strided like bn;
 * accumulate != 0 adds into out (gradient accumulation, no separate add pass).
 * partial: rgan_bn_partial_bytes(P, C) of scratch (fixed-order two-level sum). */
int rgan_channel_sum(const float* t, long long P, int C, long long sp, long long sc,
                     float* out, int accumulate, void* partial, void* stream);

/* dgamma (+)= (float)(sums[1][c] * invstd[c]), dbeta (+)= (float)sums[0][c] (accumulate != 0:
 * added) from [2][C] BatchNorm backward sums (rgan_bn_backward_sums) and stats [mean; invstd]:
 * the affine gradients from a rank's LOCAL sums under SyncBN, where the normalisation uses the
 * all-reduced ones (either output nullable). */
int rgan_bn_affine_grads(const double* sums, const float* stats, int C, float* dgamma, float* dbeta,
                         int accumulate, void* stream);

/* ---- loss heads (GLI:481-484, 592-644, 686-709) ----
 * kind = --loss_D (1..8); side 0 = D-real (heads 1-4) / D (heads 5-8), 1 = D-fake
 * (heads 1-4), 2 = G.  r, f: [n] (either nullable per head).  loss: device float[1];
 * dr, df: [n] gradients of loss w.r.t. r and f (nullable).  n <= 65536. */
int rgan_loss_head(int kind, int side, const float* r, const float* f, int n,
                   float* loss, float* dr, float* df, void* stream);
/* Heads 1-4, D side as ONE launch: loss3 = {errD_real, errD_fake, errD_real + errD_fake}
 * and both gradients (nullable) -- the batched D step's pair of losses. */
int rgan_loss_head_pair(int kind, const float* r, const float* f, int n, float* loss3, float* dr,
                        float* df, void* stream);
/* Heads 5-8, G side, on the G step's batched output y = [D(G(z)); D(x)] (2n values): loss
 * and dy[0..n) = d loss / d D(G(z)), dy[n..2n) = 0 (D(x) is a no-grad forward, GLI:681),
 * in one launch. */
int rgan_loss_head_joint(int kind, const float* y, int n, float* loss, float* dy, void* stream);
/* Distributed form: the three phases of the same head with the cross-rank sums done by
 * the caller between them.  phase 0: sums[0..1] = (sum r, sum f) local;
 * phase 1: given global means in gsum[0..1] (sum r, sum f over n_global), sums[0..3] =
 * local (sum a, sum b, sum a', sum b'); phase 2: loss and grads from global gsum[0..5]. */
int rgan_loss_head_dist(int kind, int side, int phase, const float* r, const float* f, int n,
                        int n_global, const float* gsum, float* sums, float* loss,
                        float* dr, float* df, void* stream);
/* out = in * (*scale) (device scalar), used to apply an upstream gradient. */
int rgan_scale(const float* in, const float* scale, long long n, float* out, void* stream);

/* ---- WGAN-GP (GLI:646-658) ---- */
/* xb[b] = x[b]*u[b] + xf[b]*(1-u[b]) over per-sample blocks of `per` elements. */
int rgan_gp_interp(const float* x, const float* xf, const float* u, int batch, long long per,
                   float* xb, void* stream);
/* norms[b] = ||g_b||_2 ; loss = lam * mean_b (norms-1)^2 over n_global samples. */
int rgan_gp_penalty(const float* g, int batch, long long per, float lam, int n_global,
                    float* norms, float* loss, void* stream);
/* dg = (*gscale) * lam * 2 (norm_b - 1)/n_global * g_b / norm_b (0 where norm_b == 0). */
int rgan_gp_penalty_backward(const float* g, const float* norms, int batch, long long per,
                             float lam, int n_global, const float* gscale, float* dg,
                             void* stream);

/* ---- spectral norm (torch/nn/utils/spectral_norm.py:62-139; GLI call sites 334-446) ----
 * W viewed as [rows][cols]; element (r, c) sits at r*rs + (c / lo)*hs + (c % lo).
 * Conv2d weight (dim 0): rs = cin*kk, hs = kk, lo = kk.  ConvTranspose2d (dim 1, the
 * permute(1,0,2,3) view): rs = kk, hs = cout*kk, lo = kk.
 * One power iteration: v = normalize(W^T u), u = normalize(W v), sigma = u.(W v);
 * writes u, v in place and inv_sigma[0] = 1/sigma.  do_iter = 0 only recomputes sigma.
 * ws: rgan_spectral_ws_bytes(rows, cols). */
size_t rgan_spectral_ws_bytes(int rows, int cols);
int rgan_spectral_power(const float* W, int rows, int cols, long long rs, long long hs, int lo,
                        float eps, float* u, float* v, float* inv_sigma, int do_iter,
                        void* ws, void* stream);
/* All spectral layers of one net call in FOUR launches (instead of four per layer):
 * each layer gets one power iteration exactly as rgan_spectral_power(do_iter=1).
 * n <= 16 layers; every sum in a fixed order (no cross-block hand-off, no counters); ws:
 * rgan_spectral_batch_ws_bytes(n, layers). */
typedef struct RganSnLayer {
  const float* W;
  int rows, cols, lo;
  long long rs, hs;
  float* u;                /* updated in place (the module's weight_u / weight_v buffers) */
  float* v;
  float* u_copy;           /* nullable: the new u, v also written here (the call's own copy,
                              torch spectral_norm's u.clone() / v.clone(), spectral_norm.py:112-114) */
  float* v_copy;
  float* inv_sigma;
} RganSnLayer;
size_t rgan_spectral_batch_ws_bytes(int n, const RganSnLayer* layers);
int rgan_spectral_power_batch(int n, const RganSnLayer* layers, float eps, void* ws, void* stream);
/* dW_orig = dW_eff/sigma - (<dW_eff, W_orig>/sigma^2) u v^T (u, v constants); ws >= 2 KiB. */
int rgan_spectral_backward(const float* W, const float* dWeff, int rows, int cols,
                           long long rs, long long hs, int lo, const float* u, const float* v,
                           const float* inv_sigma, float* dW, int accumulate, void* ws, void* stream);

/* ---- Adam (torch/optim/adam.py:347-547, _single_tensor_adam semantics) ----
 * Updates `ntensors` tensors (any count; launched in chunks).  hyper = device double[8]:
 * {lr, beta1, beta2, eps, weight_decay, 0, 0, 0} (doubles, as torch keeps them in
 * Python floats); step = device float[1], incremented once per call before use, like
 * state['step'].  Pointer arrays are host arrays of device pointers. */
int rgan_adam(int ntensors, float* const* params, const float* const* grads,
              float* const* exp_avg, float* const* exp_avg_sq, const long long* numel,
              const double* hyper, float* step, void* stream);
/* step[0] += 1 (the bump rgan_adam / rgan_adam_packed issue before the update). */
int rgan_adam_step_inc(float* step, void* stream);
/* rgan_adam that also writes the cached GEMM layouts of the weights it updates (what
 * rgan_conv_pack(d, which, w, packed) would produce from the new values), instead of a
 * repack pass reading every weight again after the step.  packs[i].tensor indexes the
 * params arrays; layouts the Adam kernel cannot write (non-contiguous weights, generic
 * packs) are repacked by their own launch after it, so every listed layout is current
 * when the call's work completes.  step = device float[2]: step[0] the count (as rgan_adam),
 * step[1] the call's arrival ticket (a uint32, 0 before the first call; left 0). */
typedef struct RganAdamPack {
  int tensor;
  int which;               /* 0 forward layout, 1 data-gradient layout (rgan_conv_pack) */
  const RganConv* d;       /* the descriptor the layout was packed for */
  float* packed;           /* rgan_conv_pack_floats(d, which) floats */
} RganAdamPack;
int rgan_adam_packed(int ntensors, float* const* params, const float* const* grads,
                     float* const* exp_avg, float* const* exp_avg_sq, const long long* numel,
                     const double* hyper, float* step, int npacks, const RganAdamPack* packs,
                     void* stream);
/* hyper[0] *= gamma (ExponentialLR.step, GLI:533-534,713-714). */
int rgan_lr_decay(double* hyper, double gamma, void* stream);

/* ---- data movement ---- */
/* out[b] = images[idx[b]] for per-image blocks of `per` floats (the real-batch draw,
 * GLI:176-178, 581-583, on a dataset resident in HBM). */
int rgan_gather_images(const float* images, const long long* idx, int batch, long long per,
                       float* out, void* stream);

/* ---- live launch timing (bench.py roofline) ----
 * rgan_profile_begin(capacity): bracket each subsequent conv GEMM launch with HIP events
 * on its stream (up to `capacity` launches).  rgan_profile_end: wait, stop, return
 * summed GEMM time, summed algorithmic FLOPs (2*B*Cin*Cout*k*k*pixels per conv op) and
 * the launch count.  rgan_profile_kernel(i = 0, 1, ... until it returns RGAN_EINVAL): the same per kernel symbol. */
int rgan_profile_begin(int capacity);
int rgan_profile_end(double* total_ms, double* total_flops, long long* launches);
int rgan_profile_kernel(int idx, char* name, int name_len, double* ms, double* flops, long long* n);

/* GEMM arithmetic of the FAST 128x128 forward and data-gradient GEMMs (Conv and ConvT; the
 * weight gradients stay on the fp32 MFMA): 0 = fp32 MFMA (default),
 * 1 = fp32 emulated on the bf16 MFMA (each operand split exactly into three bf16 pieces,
 * the six products down to 2^-16 relative accumulated in fp32: per-product error <= 2^-23
 * relative, the fp32 rounding scale).  Also settable at load by RGAN_EMU_BF16X6=1.  Read
 * at launch time (a captured graph keeps the kernels it captured).  Returns the previous
 * setting, or -1 for a value other than 0 / 1.  No reference counterpart (an MI355X
 * arithmetic option; the reference computes fp32 on the CPU). */
int rgan_set_gemm_emulation(int on);

/* Library self-description: number of exported compute entry points, version string
 * (ends in "abi<RGAN_ABI_VERSION>"; rgan_abi_version() returns the number). */
int rgan_abi_version(void);
const char* rgan_version(void);

/* Device sampling (--rgan_rng device; replaces the draws of GLI:176,608,630,648-649,674):
 * Philox-4x32-10 keyed by `seed` at the device counter *counter, which the call advances
 * on the stream by the numbers it used (graph-replay safe).
 * rgan_rng_fill: out[0..n) ~ N(0, 1) (kind 0, Box-Muller) or U[0, 1) (kind 1).
 * rgan_rng_choice: n <= 4096 distinct indices of [0, N) (numpy.random.choice(N, n,
 * replace=False)'s distribution; Floyd's algorithm on one wave), int64. */
int rgan_rng_fill(float* out, long long n, int kind, unsigned long long seed, unsigned long long* counter,
                  void* stream);
int rgan_rng_choice(long long* out, int N, int n, unsigned long long seed, unsigned long long* counter,
                    void* stream);

#ifdef __cplusplus
}
#endif
#endif
