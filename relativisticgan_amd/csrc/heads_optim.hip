// Loss heads, gradient penalty, spectral norm, Adam and data movement for gfx950.
//
//  * loss heads: the eight --loss_D variants (GLI:481-484, 592-644, 686-709; algebra in
//    SURVEY Appendix D) as ONE single-workgroup kernel computing loss and dL/dr, dL/df;
//  * WGAN-GP: interpolation + per-sample norm/penalty and its backward (GLI:646-658);
//  * spectral norm power iteration and the sigma-gradient correction
//    (torch/nn/utils/spectral_norm.py:62-139 as reached from GLI:126,334-446);
//  * fused multi-tensor Adam (torch/optim/adam.py _single_tensor_adam, GLI:529-530,659,712);
//  * real-batch gather from a dataset resident in HBM (GLI:176-178, 581-583).
#include "common.h"

namespace rgan {

// ------------------------------------------------------------------ loss heads
__device__ __forceinline__ float softplus(float x) { return fmaxf(x, 0.f) + log1pf(expf(-fabsf(x))); }
__device__ __forceinline__ float sigm(float x) { return 1.f / (1.f + expf(-x)); }

// relativistic-average pair (a on r - m_f, b on f - m_r); returns value, writes derivative
__device__ __forceinline__ float ra_a(int kind, bool gside, float d, float& der) {
  if (kind == 6) {
    if (!gside) { der = sigm(d) - 1.f; return softplus(-d); }
    der = sigm(d); return softplus(d);
  }
  if (kind == 7) {
    const float s = gside ? d + 1.f : d - 1.f;
    der = 2.f * s; return s * s;
  }
  // 8: hinge
  if (!gside) { const float h = 1.f - d; der = h > 0.f ? -1.f : 0.f; return h > 0.f ? h : 0.f; }
  const float h = 1.f + d; der = h > 0.f ? 1.f : 0.f; return h > 0.f ? h : 0.f;
}
__device__ __forceinline__ float ra_b(int kind, bool gside, float d, float& der) {
  if (kind == 6) {
    if (!gside) { der = sigm(d); return softplus(d); }
    der = sigm(d) - 1.f; return softplus(-d);
  }
  if (kind == 7) {
    const float s = gside ? d - 1.f : d + 1.f;
    der = 2.f * s; return s * s;
  }
  if (!gside) { const float h = 1.f + d; der = h > 0.f ? 1.f : 0.f; return h > 0.f ? h : 0.f; }
  const float h = 1.f - d; der = h > 0.f ? -1.f : 0.f; return h > 0.f ? h : 0.f;
}

// heads 1-4 on one tensor t; side 0 D-real, 1 D-fake, 2 G
__device__ __forceinline__ float single_term(int kind, int side, float t, float& der) {
  if (kind == 1) {
    const float y = side == 1 ? 0.f : 1.f;
    const float lv = y > 0.5f ? fmaxf(logf(t), -100.f) : fmaxf(logf(1.f - t), -100.f);
    der = (t - y) / fmaxf((1.f - t) * t, 1e-12f);
    return -lv;
  }
  if (kind == 2) {
    const float s = side == 1 ? t : t - 1.f;
    der = 2.f * s; return s * s;
  }
  if (kind == 3 || (kind == 4 && side == 2)) {
    const float sg = side == 1 ? 1.f : -1.f;
    der = sg; return sg * t;
  }
  // hinge D
  if (side == 0) { const float h = 1.f - t; der = h > 0.f ? -1.f : 0.f; return h > 0.f ? h : 0.f; }
  const float h = 1.f + t; der = h > 0.f ? 1.f : 0.f; return h > 0.f ? h : 0.f;
}

// phase < 0: everything in one launch (single process).  Otherwise the distributed phases
// of rgan_loss_head_dist.  One workgroup of 1024 threads.
__global__ __launch_bounds__(1024) void loss_head_kernel(int kind, int side, int phase, const float* r,
                                                         const float* f, int n, int n_global,
                                                         const float* gsum, float* sums, float* loss,
                                                         float* dr, float* df, float* zr = nullptr) {
  __shared__ float red[16];
  const int tid = threadIdx.x;
  const float ng = (float)n_global;
  if (zr)  // rgan_loss_head_joint: the joint gradient's no-grad half is zero
    for (int i = tid; i < n; i += blockDim.x) zr[i] = 0.f;
  if (kind <= 4) {
    const float* t = side == 0 ? r : f;
    float* dt = side == 0 ? dr : df;
    float s = 0.f;
    for (int i = tid; i < n; i += blockDim.x) {
      float der;
      s += single_term(kind, side, t[i], der);
      if (dt && phase != 0) dt[i] = der / ng;
    }
    s = block_sum(s, red);
    if (tid == 0) {
      if (phase < 0) loss[0] = s / ng;
      else if (phase == 0) sums[0] = s;
      else if (loss) loss[0] = gsum[0] / ng;
    }
    return;
  }
  if (kind == 5) {
    // RSGAN: BCEwL(r - f, 1) for D, BCEwL(f - r, 1) for G (elementwise pairs)
    float s = 0.f;
    for (int i = tid; i < n; i += blockDim.x) {
      const float d = side == 2 ? f[i] - r[i] : r[i] - f[i];
      s += softplus(-d);
      const float g = (sigm(d) - 1.f) / ng;
      if (phase != 0) {
        if (side == 2) { if (df) df[i] = g; if (dr) dr[i] = -g; }
        else { if (dr) dr[i] = g; if (df) df[i] = -g; }
      }
    }
    s = block_sum(s, red);
    if (tid == 0) {
      if (phase < 0) loss[0] = s / ng;
      else if (phase == 0) sums[0] = s;
      else if (loss) loss[0] = gsum[0] / ng;
    }
    return;
  }
  // relativistic average heads 6-8
  const bool gside = side == 2;
  float mr, mf;
  if (phase < 0 || phase == 0) {
    float sr = 0.f, sf = 0.f;
    for (int i = tid; i < n; i += blockDim.x) { sr += r[i]; sf += f[i]; }
    sr = block_sum(sr, red);
    sf = block_sum(sf, red);
    if (phase == 0) {
      if (tid == 0) { sums[0] = sr; sums[1] = sf; }
      return;
    }
    mr = sr / ng; mf = sf / ng;
  } else {
    mr = gsum[0] / ng; mf = gsum[1] / ng;
  }
  if (phase < 0 || phase == 1) {
    float sa = 0.f, sb = 0.f, sda = 0.f, sdb = 0.f;
    for (int i = tid; i < n; i += blockDim.x) {
      float da, db;
      sa += ra_a(kind, gside, r[i] - mf, da);
      sb += ra_b(kind, gside, f[i] - mr, db);
      sda += da; sdb += db;
    }
    sa = block_sum(sa, red); sb = block_sum(sb, red);
    sda = block_sum(sda, red); sdb = block_sum(sdb, red);
    if (phase == 1) {
      if (tid == 0) { sums[0] = sa; sums[1] = sb; sums[2] = sda; sums[3] = sdb; }
      return;
    }
    // single-process: fall through with local == global sums
    if (tid == 0) loss[0] = (sa / ng + sb / ng) / 2.f;
    const float inv2 = 0.5f / ng;
    for (int i = tid; i < n; i += blockDim.x) {
      float da, db;
      ra_a(kind, gside, r[i] - mf, da);
      ra_b(kind, gside, f[i] - mr, db);
      if (dr) dr[i] = inv2 * (da - sdb / ng);
      if (df) df[i] = inv2 * (db - sda / ng);
    }
    return;
  }
  // phase 2: gsum = (sum r, sum f, sum a, sum b, sum a', sum b') global
  if (tid == 0 && loss) loss[0] = (gsum[2] / ng + gsum[3] / ng) / 2.f;
  const float inv2 = 0.5f / ng;
  for (int i = tid; i < n; i += blockDim.x) {
    float da, db;
    ra_a(kind, gside, r[i] - mf, da);
    ra_b(kind, gside, f[i] - mr, db);
    if (dr) dr[i] = inv2 * (da - gsum[5] / ng);
    if (df) df[i] = inv2 * (db - gsum[4] / ng);
  }
}

// heads 1-4, D side: errD_real (on r) and errD_fake (on f) and their sum in one launch --
// the reference's two losses and two backward calls (GLI:595-624); loss3 = {real, fake, sum}
__global__ __launch_bounds__(1024) void loss_head_pair_kernel(int kind, const float* __restrict__ r,
                                                              const float* __restrict__ f, int n,
                                                              float* __restrict__ loss3, float* __restrict__ dr,
                                                              float* __restrict__ df) {
  __shared__ float red[16];
  const int tid = threadIdx.x;
  const float ng = (float)n;
  float sr = 0.f, sf = 0.f;
  for (int i = tid; i < n; i += blockDim.x) {
    float der;
    sr += single_term(kind, 0, r[i], der);
    if (dr) dr[i] = der / ng;
    sf += single_term(kind, 1, f[i], der);
    if (df) df[i] = der / ng;
  }
  sr = block_sum(sr, red);
  sf = block_sum(sf, red);
  if (tid == 0) {
    const float lr = sr / ng, lf = sf / ng;
    loss3[0] = lr;
    loss3[1] = lf;
    loss3[2] = lr + lf;
  }
}

extern "C" int rgan_loss_head_pair(int kind, const float* r, const float* f, int n, float* loss3, float* dr,
                                   float* df, void* stream) {
  RGAN_REQUIRE(kind >= 1 && kind <= 4 && r && f && loss3 && n > 0 && n <= 65536);
  loss_head_pair_kernel<<<1, 1024, 0, (hipStream_t)stream>>>(kind, r, f, n, loss3, dr, df);
  RGAN_CHECK_LAUNCH();
  return 0;
}

static bool head_args_ok(int kind, int side, const float* r, const float* f, int n) {
  if (kind < 1 || kind > 8 || n <= 0 || n > 65536) return false;
  if (kind <= 4) return side >= 0 && side <= 2 && (side == 0 ? r != nullptr : f != nullptr);
  return (side == 0 || side == 2) && r && f;
}

extern "C" int rgan_loss_head(int kind, int side, const float* r, const float* f, int n, float* loss,
                              float* dr, float* df, void* stream) {
  RGAN_REQUIRE(head_args_ok(kind, side, r, f, n) && loss);
  loss_head_kernel<<<1, 1024, 0, (hipStream_t)stream>>>(kind, side, -1, r, f, n, n, nullptr, nullptr, loss,
                                                       dr, df);
  RGAN_CHECK_LAUNCH();
  return 0;
}

// Heads 5-8, G side, on the G step's joint output y = [D(G(z)); D(x)] (2n values, the batched
// pass of GLI:673-707): loss and dy = [d loss / d D(G(z)); 0] -- D(x) is a no-grad forward in
// the reference (GLI:681), so the second half of the joint gradient is zero, in the same launch.
extern "C" int rgan_loss_head_joint(int kind, const float* y, int n, float* loss, float* dy, void* stream) {
  RGAN_REQUIRE(kind >= 5 && kind <= 8 && y && dy && head_args_ok(kind, 2, y + n, y, n) && loss);
  loss_head_kernel<<<1, 1024, 0, (hipStream_t)stream>>>(kind, 2, -1, y + n, y, n, n, nullptr, nullptr, loss,
                                                       nullptr, dy, dy + n);
  RGAN_CHECK_LAUNCH();
  return 0;
}

extern "C" int rgan_loss_head_dist(int kind, int side, int phase, const float* r, const float* f, int n,
                                   int n_global, const float* gsum, float* sums, float* loss, float* dr,
                                   float* df, void* stream) {
  RGAN_REQUIRE(head_args_ok(kind, side, r, f, n) && n_global >= n && phase >= 0 && phase <= 2);
  if (kind <= 5) RGAN_REQUIRE(phase != 1);
  if (phase == 0 || phase == 1) RGAN_REQUIRE(sums != nullptr);
  if (phase >= 1) RGAN_REQUIRE(gsum != nullptr);
  loss_head_kernel<<<1, 1024, 0, (hipStream_t)stream>>>(kind, side, phase, r, f, n, n_global, gsum, sums,
                                                       loss, dr, df);
  RGAN_CHECK_LAUNCH();
  return 0;
}

__global__ void scale_kernel(const float* __restrict__ in, const float* __restrict__ sc, long long n,
                             float* __restrict__ out) {
  const float s = sc[0];
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n;
       i += (long long)gridDim.x * blockDim.x)
    out[i] = in[i] * s;
}

static int grid1(long long n) {
  return (int)std::max<long long>(1, std::min<long long>((n + 255) / 256, 8192));
}

extern "C" int rgan_scale(const float* in, const float* scale, long long n, float* out, void* stream) {
  RGAN_REQUIRE(in && scale && out && n >= 0);
  if (n == 0) return 0;
  scale_kernel<<<grid1(n), 256, 0, (hipStream_t)stream>>>(in, scale, n, out);
  RGAN_CHECK_LAUNCH();
  return 0;
}

// ------------------------------------------------------------------ gradient penalty
__global__ void gp_interp_kernel(const float* __restrict__ x, const float* __restrict__ xf,
                                 const float* __restrict__ u, int batch, long long per, float* __restrict__ xb) {
  const long long total = (long long)batch * per;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const float uu = u[i / per];
    xb[i] = x[i] * uu + xf[i] * (1.f - uu);
  }
}

extern "C" int rgan_gp_interp(const float* x, const float* xf, const float* u, int batch, long long per,
                              float* xb, void* stream) {
  RGAN_REQUIRE(x && xf && u && xb && batch > 0 && per > 0);
  gp_interp_kernel<<<grid1(batch * per), 256, 0, (hipStream_t)stream>>>(x, xf, u, batch, per, xb);
  RGAN_CHECK_LAUNCH();
  return 0;
}

__global__ __launch_bounds__(1024) void gp_norm_kernel(const float* __restrict__ g, long long per,
                                                       float* __restrict__ norms) {
  __shared__ float red[16];
  const float* gb = g + blockIdx.x * per;
  float s = 0.f;
  for (long long i = threadIdx.x; i < per; i += blockDim.x) s += gb[i] * gb[i];
  s = block_sum(s, red);
  if (threadIdx.x == 0) norms[blockIdx.x] = sqrtf(s);
}

__global__ __launch_bounds__(1024) void gp_loss_kernel(const float* __restrict__ norms, int batch, float lam,
                                                       int n_global, float* loss) {
  __shared__ float red[16];
  float s = 0.f;
  for (int i = threadIdx.x; i < batch; i += blockDim.x) {
    const float d = norms[i] - 1.f;
    s += d * d;
  }
  s = block_sum(s, red);
  if (threadIdx.x == 0) loss[0] = lam * (s / (float)n_global);
}

extern "C" int rgan_gp_penalty(const float* g, int batch, long long per, float lam, int n_global, float* norms,
                               float* loss, void* stream) {
  RGAN_REQUIRE(g && norms && loss && batch > 0 && per > 0 && n_global >= batch);
  hipStream_t s = (hipStream_t)stream;
  gp_norm_kernel<<<batch, 1024, 0, s>>>(g, per, norms);
  RGAN_CHECK_LAUNCH();
  gp_loss_kernel<<<1, 1024, 0, s>>>(norms, batch, lam, n_global, loss);
  RGAN_CHECK_LAUNCH();
  return 0;
}

// dg may alias g (the GP engine rewrites the gradient image in place): each thread reads
// g[i] and then writes dg[i], so neither pointer is __restrict__
__global__ void gp_bwd_kernel(const float* g, const float* __restrict__ norms, int batch,
                              long long per, float lam, int n_global, const float* gscale,
                              float* dg) {
  const long long total = (long long)batch * per;
  const float gs = gscale ? gscale[0] : 1.f;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const float nb = norms[i / per];
    const float coef = nb > 0.f ? gs * lam * 2.f * (nb - 1.f) / (float)n_global / nb : 0.f;
    dg[i] = coef * g[i];
  }
}

extern "C" int rgan_gp_penalty_backward(const float* g, const float* norms, int batch, long long per, float lam,
                                        int n_global, const float* gscale, float* dg, void* stream) {
  RGAN_REQUIRE(g && norms && dg && batch > 0 && per > 0 && n_global >= batch);
  gp_bwd_kernel<<<grid1(batch * per), 256, 0, (hipStream_t)stream>>>(g, norms, batch, per, lam, n_global,
                                                                     gscale, dg);
  RGAN_CHECK_LAUNCH();
  return 0;
}

// ------------------------------------------------------------------ spectral norm
// W viewed [rows][cols]; element (r, c) at r*rs + (c / lo)*hs + (c % lo)
struct SnView {
  const float* W;
  int rows, cols, lo;
  long long rs, hs;
  __device__ __forceinline__ long long off(int r, int c) const {
    const int ch = c / lo;
    return (long long)r * rs + (long long)ch * hs + (c - ch * lo);
  }
};

constexpr int SN_RCHUNK = 64;

// partial[k][c] = sum_{r in chunk k} W(r,c) u[r]
__global__ __launch_bounds__(256) void sn_wtu_kernel(SnView w, const float* __restrict__ u,
                                                     float* __restrict__ part) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  const int k = blockIdx.y;
  if (c >= w.cols) return;
  const int r0 = k * SN_RCHUNK, r1 = min(w.rows, r0 + SN_RCHUNK);
  float s = 0.f;
  for (int r = r0; r < r1; ++r) s += w.W[w.off(r, c)] * u[r];
  part[(size_t)k * w.cols + c] = s;
}

// v = t / max(||t||, eps), t[c] = sum_k part[k][c]
__global__ __launch_bounds__(1024) void sn_norm_v_kernel(const float* __restrict__ part, int nchunks, int cols,
                                                         float eps, float* __restrict__ v, float* __restrict__ t) {
  __shared__ float red[16];
  float s = 0.f;
  for (int c = threadIdx.x; c < cols; c += blockDim.x) {
    float a = 0.f;
    for (int k = 0; k < nchunks; ++k) a += part[(size_t)k * cols + c];
    t[c] = a;
    s += a * a;
  }
  s = block_sum(s, red);
  const float den = fmaxf(sqrtf(s), eps);
  __syncthreads();
  for (int c = threadIdx.x; c < cols; c += blockDim.x) v[c] = t[c] / den;
}

// w[r] = sum_c W(r,c) v[c]; one wave per row
__global__ __launch_bounds__(256) void sn_wv_kernel(SnView w, const float* __restrict__ v, float* __restrict__ out) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= w.rows) return;
  float s = 0.f;
  for (int c = lane; c < w.cols; c += 64) s += w.W[w.off(row, c)] * v[c];
  s = wave_sum(s);
  if (lane == 0) out[row] = s;
}

// u = w/max(||w||,eps) (if do_iter); sigma = u . w; inv_sigma = 1/sigma
__global__ __launch_bounds__(1024) void sn_norm_u_kernel(const float* __restrict__ wv, int rows, float eps,
                                                         int do_iter, float* __restrict__ u,
                                                         float* __restrict__ inv_sigma) {
  __shared__ float red[16];
  float den = 1.f;
  if (do_iter) {
    float s = 0.f;
    for (int r = threadIdx.x; r < rows; r += blockDim.x) s += wv[r] * wv[r];
    s = block_sum(s, red);
    den = fmaxf(sqrtf(s), eps);
    for (int r = threadIdx.x; r < rows; r += blockDim.x) u[r] = wv[r] / den;
    __syncthreads();
  }
  float d = 0.f;
  for (int r = threadIdx.x; r < rows; r += blockDim.x) d += u[r] * wv[r];
  d = block_sum(d, red);
  if (threadIdx.x == 0) inv_sigma[0] = 1.f / d;
}

static int sn_nchunks(int rows) { return ceil_div(rows, SN_RCHUNK); }

extern "C" size_t rgan_spectral_ws_bytes(int rows, int cols) {
  return ((size_t)sn_nchunks(rows) * cols + cols + rows + 64) * sizeof(float);
}

extern "C" int rgan_spectral_power(const float* W, int rows, int cols, long long rs, long long hs, int lo,
                                   float eps, float* u, float* v, float* inv_sigma, int do_iter, void* ws,
                                   void* stream) {
  RGAN_REQUIRE(W && u && v && inv_sigma && ws && rows > 0 && cols > 0 && lo > 0);
  hipStream_t s = (hipStream_t)stream;
  SnView w{W, rows, cols, lo, rs, hs};
  const int nch = sn_nchunks(rows);
  float* part = (float*)ws;
  float* t = part + (size_t)nch * cols;
  float* wv = t + cols;
  if (do_iter) {
    sn_wtu_kernel<<<dim3(ceil_div(cols, 256), nch), 256, 0, s>>>(w, u, part);
    RGAN_CHECK_LAUNCH();
    sn_norm_v_kernel<<<1, 1024, 0, s>>>(part, nch, cols, eps, v, t);
    RGAN_CHECK_LAUNCH();
  }
  sn_wv_kernel<<<ceil_div(rows, 4), 256, 0, s>>>(w, v, wv);
  RGAN_CHECK_LAUNCH();
  sn_norm_u_kernel<<<1, 1024, 0, s>>>(wv, rows, eps, do_iter, u, inv_sigma);
  RGAN_CHECK_LAUNCH();
  return 0;
}

// ---- all of a net's spectral layers in four launches (one power iteration each) ----
// W is read once for t = W^T u and once for w = W v: 2 x sizeof(W) of HBM traffic.  When W
// is not cache-resident (a training step), HBM latency bounds any dependent sequence of row
// loads, so every phase issues all of a thread's row loads at once over many blocks:
//   V1: blocks over (layer, 1024-column chunk, 16-row chunk): a thread's 4 columns summed
//       over the chunk's 16 rows (16 float4 loads in flight) -> row-chunk partials;
//   V2: blocks over (layer, 256 columns): t = sum of the partials (row-chunk order), and
//       per-block sums of t^2;
//   U:  blocks over (layer, row), the block's threads splitting the row: w = (W t) / ||t||
//       (8 float4 loads in flight per thread); every block forms ||t|| from the V2 partials
//       (same fixed order) and writes its slice of v = t / max(||t||, eps);
//   fin: a block per layer writes u = w / max(||w||, eps) and 1/sigma, sigma = u . w.
// All sums are in a fixed order (deterministic); no atomics, no cross-block hand-off.
constexpr int SNB_MAX = 16;
constexpr int SNB_CC = 1024;           // columns per V1 block
constexpr int SNB_RC = 16;             // rows per V1 block
struct SnBatch {
  SnView w[SNB_MAX];
  float* u[SNB_MAX];
  float* v[SNB_MAX];
  float* u2[SNB_MAX];       // nullable second copies (the autograd-saved u, v of this call)
  float* v2[SNB_MAX];
  float* inv_sigma[SNB_MAX];
  float* t[SNB_MAX];        // workspace: [cols] t, then [rows] w
  float* part[SNB_MAX];     // workspace: V1 [nrc][cols] row-chunk partials
  float* sq[SNB_MAX];       // workspace: V2 per-block sums of t^2 [nt]
  float* wv[SNB_MAX];       // workspace: [rows] w
  int vec[SNB_MAX];         // 16-B contiguous 4-column runs
  int ncc[SNB_MAX], nrc[SNB_MAX], nt[SNB_MAX];
  int first[SNB_MAX + 1];   // block prefix per layer (of the launch this struct is for)
  int n;
  float eps;
};

__device__ __forceinline__ int snb_layer(const SnBatch& b, int blk) {
  int l = 0;
  while (l + 1 < b.n && blk >= b.first[l + 1]) ++l;
  return l;
}

// fixed-order sum of n per-block partials by wave 0 with lane-indexed (vector) loads; the
// result is valid in thread 0
__device__ __forceinline__ float snb_sum_parts(const float* part, int n) {
  float a = 0.f;
  if (threadIdx.x < 64) {
    for (int i = threadIdx.x; i < n; i += 64) a += part[i];
    a = wave_sum(a);
  }
  return a;
}

__global__ __launch_bounds__(256) void sn_batch_v(SnBatch b) {
  const int l = snb_layer(b, blockIdx.x), blk = blockIdx.x - b.first[l];
  const SnView& w = b.w[l];
  const int ncc = b.ncc[l];
  const int cc = blk % ncc, rc = blk / ncc;
  const int tid = threadIdx.x;
  const int r0 = rc * SNB_RC, r1 = min(w.rows, r0 + SNB_RC);
  const float* u = b.u[l];
  float* part = b.part[l] + (size_t)rc * w.cols;
  const int c0 = cc * SNB_CC;
  float ur[SNB_RC];
#pragma unroll
  for (int q = 0; q < SNB_RC; ++q) ur[q] = r0 + q < r1 ? u[r0 + q] : 0.f;
  if (b.vec[l]) {
    const int c = c0 + 4 * tid;
    if (c >= w.cols) return;
    const float* wc = w.W + w.off(0, c) + (long long)r0 * w.rs;
    float4 x[SNB_RC];
#pragma unroll
    for (int q = 0; q < SNB_RC; ++q)
      x[q] = r0 + q < r1 ? *reinterpret_cast<const float4*>(wc + (long long)q * w.rs) : make_float4(0.f, 0.f, 0.f, 0.f);
    float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
#pragma unroll
    for (int q = 0; q < SNB_RC; ++q) {
      a0 += x[q].x * ur[q]; a1 += x[q].y * ur[q]; a2 += x[q].z * ur[q]; a3 += x[q].w * ur[q];
    }
    *reinterpret_cast<float4*>(part + c) = make_float4(a0, a1, a2, a3);
  } else {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int c = c0 + tid + 256 * k;
      if (c >= w.cols) continue;
      float x[SNB_RC];
#pragma unroll
      for (int q = 0; q < SNB_RC; ++q) x[q] = r0 + q < r1 ? w.W[w.off(r0 + q, c)] : 0.f;
      float a = 0.f;
#pragma unroll
      for (int q = 0; q < SNB_RC; ++q) a += x[q] * ur[q];
      part[c] = a;
    }
  }
}

__global__ __launch_bounds__(256) void sn_batch_t(SnBatch b) {
  __shared__ float red[16];
  const int l = snb_layer(b, blockIdx.x), blk = blockIdx.x - b.first[l];
  const SnView& w = b.w[l];
  const int c = blk * 256 + threadIdx.x, nrc = b.nrc[l];
  float t = 0.f;
  if (c < w.cols) {
    const float* part = b.part[l] + c;
    int q = 0;
    for (; q + 16 <= nrc; q += 16) {  // 16 loads in flight, summed in row-chunk order
      float x[16];
#pragma unroll
      for (int k = 0; k < 16; ++k) x[k] = part[(size_t)(q + k) * w.cols];
#pragma unroll
      for (int k = 0; k < 16; ++k) t += x[k];
    }
    for (; q < nrc; ++q) t += part[(size_t)q * w.cols];
    b.t[l][c] = t;
  }
  const float s2 = block_sum(c < w.cols ? t * t : 0.f, red);
  if (threadIdx.x == 0) b.sq[l][blk] = s2;
}

__global__ __launch_bounds__(256) void sn_batch_u(SnBatch b) {
  __shared__ float red[16];
  __shared__ float den_s;
  const int l = snb_layer(b, blockIdx.x), row = blockIdx.x - b.first[l];
  const int nblk = b.first[l + 1] - b.first[l];  // = rows: a block per row
  const SnView& w = b.w[l];
  const int tid = threadIdx.x;
  const float* t = b.t[l];
  // w[row] = (W t)[row] / ||t||: the block's 256 threads split the row, 8 float4 in flight
  // each.  The row loads go out first: ||t|| (a sum of V2's partials) and the v slice only
  // scale the result, so their round trips overlap the row's instead of preceding it.
  float s = 0.f;
  if (b.vec[l] && w.lo < w.cols && w.lo == 16) {
    // dim-1 (ConvTranspose) view: runs of 16 contiguous columns at row * rs + ch * hs
    const float* wr = w.W + (long long)row * w.rs;
    const int nq = w.cols / 4;  // float4 quarters of runs
    for (int e0 = 0; e0 < nq; e0 += 2048) {
      float4 x[8], y[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const int e = e0 + tid + 256 * k;
        const bool ok = e < nq;
        x[k] = ok ? *reinterpret_cast<const float4*>(wr + (long long)(e >> 2) * w.hs + 4 * (e & 3)) : make_float4(0.f, 0.f, 0.f, 0.f);
        y[k] = ok ? *reinterpret_cast<const float4*>(t + 4 * e) : make_float4(0.f, 0.f, 0.f, 0.f);
      }
#pragma unroll
      for (int k = 0; k < 8; ++k) s += x[k].x * y[k].x + x[k].y * y[k].y + x[k].z * y[k].z + x[k].w * y[k].w;
    }
  } else if (b.vec[l] && w.lo >= w.cols) {
    // dim-0 view: the row is one contiguous run
    const float* wr = w.W + (long long)row * w.rs;
    for (int c0 = 0; c0 < w.cols; c0 += 8 * 1024) {
      float4 x[8], y[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const int c = c0 + 4 * tid + 1024 * k;
        const bool ok = c < w.cols;
        x[k] = ok ? *reinterpret_cast<const float4*>(wr + c) : make_float4(0.f, 0.f, 0.f, 0.f);
        y[k] = ok ? *reinterpret_cast<const float4*>(t + c) : make_float4(0.f, 0.f, 0.f, 0.f);
      }
#pragma unroll
      for (int k = 0; k < 8; ++k) s += x[k].x * y[k].x + x[k].y * y[k].y + x[k].z * y[k].z + x[k].w * y[k].w;
    }
  } else {
    for (int c = tid; c < w.cols; c += 256) s += w.W[w.off(row, c)] * t[c];
  }
  // ||t|| from V2's per-block sums (the same fixed order in every block)
  const float tsq = snb_sum_parts(b.sq[l], b.nt[l]);
  if (tid == 0) den_s = fmaxf(sqrtf(tsq), b.eps);
  s = block_sum(s, red);  // (its barriers also publish den_s)
  const float den = den_s;
  // this block's slice of v = t / max(||t||, eps)
  {
    const int per = (w.cols + nblk - 1) / nblk, c0 = row * per, c1 = min(w.cols, c0 + per);
    float* v2 = b.v2[l];
    for (int c = c0 + tid; c < c1; c += blockDim.x) {
      const float x = t[c] / den;
      b.v[l][c] = x;
      if (v2) v2[c] = x;
    }
  }
  if (tid == 0) b.wv[l][row] = s / den;  // (W t) / ||t|| = W v
}

// one block per layer: u = w / max(||w||, eps), sigma = u . w (fixed-order sums).  A launch
// of its own: a completion counter in sn_batch_u would cost every one of its (row) blocks
// an agent-scope release, which measured slower than the whole phase.
__global__ __launch_bounds__(256) void sn_batch_fin(SnBatch b) {
  __shared__ float red[16];
  __shared__ float wden;
  const int l = blockIdx.x, tid = threadIdx.x;
  const SnView& w = b.w[l];
  float q = 0.f;
  for (int r = tid; r < w.rows; r += blockDim.x) q += b.wv[l][r] * b.wv[l][r];
  q = block_sum(q, red);
  if (tid == 0) wden = fmaxf(sqrtf(q), b.eps);
  __syncthreads();
  float d = 0.f;
  float* u2 = b.u2[l];
  for (int r = tid; r < w.rows; r += blockDim.x) {
    const float wr = b.wv[l][r], ur = wr / wden;
    b.u[l][r] = ur;
    if (u2) u2[r] = ur;
    d += ur * wr;
  }
  d = block_sum(d, red);
  if (tid == 0) b.inv_sigma[l][0] = 1.f / d;
}

struct SnGeom {
  int ncc, nrc, nt, nu;
  size_t floats;
};
static SnGeom snb_geom(const RganSnLayer& L) {
  SnGeom g;
  g.ncc = ceil_div(L.cols, SNB_CC);
  g.nrc = ceil_div(L.rows, SNB_RC);
  g.nt = ceil_div(L.cols, 256);
  g.nu = L.rows;  // U: a block per row
  auto al = [](size_t f) { return (f + 63) / 64 * 64; };  // 256-B aligned pieces (float4 partials)
  g.floats = al(L.cols) + al((size_t)g.nrc * L.cols) + al(g.nt) + al(L.rows);
  return g;
}

extern "C" size_t rgan_spectral_batch_ws_bytes(int n, const RganSnLayer* layers) {
  if (n <= 0 || n > SNB_MAX || !layers) return 0;
  size_t f = 0;
  for (int i = 0; i < n; ++i) f += snb_geom(layers[i]).floats;
  return f * sizeof(float) + 256;
}

extern "C" int rgan_spectral_power_batch(int n, const RganSnLayer* layers, float eps, void* ws, void* stream) {
  RGAN_REQUIRE(n > 0 && n <= SNB_MAX && layers && ws);
  SnBatch bv{}, bt{}, bu{};
  float* p = (float*)(((uintptr_t)ws + 255) & ~(uintptr_t)255);
  int nv = 0, nt = 0, nu = 0;
  for (int i = 0; i < n; ++i) {
    const RganSnLayer& L = layers[i];
    RGAN_REQUIRE(L.W && L.u && L.v && L.inv_sigma && L.rows > 0 && L.cols > 0 && L.lo > 0);
    const SnGeom g = snb_geom(L);
    const SnView w{L.W, L.rows, L.cols, L.lo, L.rs, L.hs};
    auto al = [](size_t f) { return (f + 63) / 64 * 64; };
    float* t = p;
    float* part = t + al(L.cols);
    float* sq = part + al((size_t)g.nrc * L.cols);
    float* wv = sq + al(g.nt);
    p += g.floats;
    const int vec = L.lo % 4 == 0 && L.rs % 4 == 0 && L.hs % 4 == 0 && L.cols % 4 == 0 && ((uintptr_t)L.W & 15) == 0;
    for (SnBatch* b : {&bv, &bt, &bu}) {
      b->w[i] = w; b->u[i] = L.u; b->v[i] = L.v; b->inv_sigma[i] = L.inv_sigma; b->t[i] = t; b->part[i] = part;
      b->sq[i] = sq; b->wv[i] = wv; b->u2[i] = L.u_copy; b->v2[i] = L.v_copy; b->vec[i] = vec;
      b->ncc[i] = g.ncc; b->nrc[i] = g.nrc; b->nt[i] = g.nt;
    }
    bv.first[i] = nv; nv += g.ncc * g.nrc;
    bt.first[i] = nt; nt += g.nt;
    bu.first[i] = nu; nu += g.nu;
  }
  bv.first[n] = nv; bt.first[n] = nt; bu.first[n] = nu;
  for (SnBatch* b : {&bv, &bt, &bu}) { b->n = n; b->eps = eps; }
  hipStream_t s = (hipStream_t)stream;
  sn_batch_v<<<nv, 256, 0, s>>>(bv);
  RGAN_CHECK_LAUNCH();
  sn_batch_t<<<nt, 256, 0, s>>>(bt);
  RGAN_CHECK_LAUNCH();
  sn_batch_u<<<nu, 256, 0, s>>>(bu);
  RGAN_CHECK_LAUNCH();
  sn_batch_fin<<<n, 256, 0, s>>>(bu);
  RGAN_CHECK_LAUNCH();
  return 0;
}

// <dWeff, W>: the view enumerates every element once, so this is the flat dot product of the
// two (same-layout) tensors: float4 grid-stride per-block partials, summed in block order
// by the backward kernel.
constexpr int SN_DOT_PARTS = 512;
__global__ __launch_bounds__(256) void sn_dot_kernel(const float* __restrict__ a, const float* __restrict__ w,
                                                     long long n, float* __restrict__ part) {
  __shared__ float red[16];
  float s = 0.f;
  const long long n4 = ((((uintptr_t)a | (uintptr_t)w) & 15) == 0) ? n / 4 : 0;
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < n4; i += (long long)gridDim.x * 256) {
    const float4 x = reinterpret_cast<const float4*>(a)[i], y = reinterpret_cast<const float4*>(w)[i];
    s += x.x * y.x + x.y * y.y + x.z * y.z + x.w * y.w;
  }
  for (long long i = 4 * n4 + blockIdx.x * 256LL + threadIdx.x; i < n; i += (long long)gridDim.x * 256) s += a[i] * w[i];
  s = block_sum(s, red);
  if (threadIdx.x == 0) part[blockIdx.x] = s;
}

// dW (+)= dWe / sigma - (<dWe, W> / sigma^2) u[r] v[c]: a block per view row r (u[r]
// uniform), its columns in 4-column runs (float4 when the runs are 16-B contiguous)
__global__ __launch_bounds__(256) void sn_bwd_kernel(SnView w, const float* __restrict__ dWe,
                                                     const float* __restrict__ part, int nparts,
                                                     const float* __restrict__ u, const float* __restrict__ v,
                                                     const float* __restrict__ inv_sigma, float* __restrict__ dW,
                                                     int accum, int vec) {
  __shared__ float red[16];
  __shared__ float kk;
  float d = 0.f;
  if (threadIdx.x < 64)
    for (int i = threadIdx.x; i < nparts; i += 64) d += part[i];
  d = threadIdx.x < 64 ? wave_sum(d) : 0.f;
  (void)red;
  const float is = inv_sigma[0];
  if (threadIdx.x == 0) kk = d * is * is;
  __syncthreads();
  const float k = kk;
  const int r = blockIdx.x;
  const float ku = k * u[r];
  const bool flat = w.lo >= w.cols;
  auto at = [&](int c) { return flat ? (long long)r * w.rs + c : w.off(r, c); };
  if (vec && !flat && w.lo == 16) {
    // dim-1 (ConvTranspose) view: a thread takes 4-column quarters of 16-column runs
    const float* wd = dWe + (long long)r * w.rs;
    float* od = dW + (long long)r * w.rs;
    for (int e = threadIdx.x; e < w.cols / 4; e += 256) {
      const int ch = e >> 2, c = 4 * e;
      const long long o = (long long)ch * w.hs + 4 * (e & 3);
      const float4 g = *reinterpret_cast<const float4*>(wd + o);
      const float4 vv = *reinterpret_cast<const float4*>(v + c);
      float4 y = make_float4(g.x * is - ku * vv.x, g.y * is - ku * vv.y, g.z * is - ku * vv.z, g.w * is - ku * vv.w);
      if (accum) {
        const float4 o4 = *reinterpret_cast<const float4*>(od + o);
        y.x += o4.x; y.y += o4.y; y.z += o4.z; y.w += o4.w;
      }
      *reinterpret_cast<float4*>(od + o) = y;
    }
  } else if (vec) {
    for (int c = 4 * threadIdx.x; c < w.cols; c += 1024) {
      const long long o = at(c);
      const float4 g = *reinterpret_cast<const float4*>(dWe + o);
      const float4 vv = *reinterpret_cast<const float4*>(v + c);
      float4 y = make_float4(g.x * is - ku * vv.x, g.y * is - ku * vv.y, g.z * is - ku * vv.z, g.w * is - ku * vv.w);
      if (accum) {
        const float4 o4 = *reinterpret_cast<const float4*>(dW + o);
        y.x += o4.x; y.y += o4.y; y.z += o4.z; y.w += o4.w;
      }
      *reinterpret_cast<float4*>(dW + o) = y;
    }
  } else {
    for (int c = threadIdx.x; c < w.cols; c += 256) {
      const long long o = at(c);
      const float g = dWe[o] * is - ku * v[c];
      dW[o] = accum ? dW[o] + g : g;
    }
  }
}

extern "C" int rgan_spectral_backward(const float* W, const float* dWeff, int rows, int cols, long long rs,
                                      long long hs, int lo, const float* u, const float* v,
                                      const float* inv_sigma, float* dW, int accumulate, void* ws, void* stream) {
  RGAN_REQUIRE(W && dWeff && u && v && inv_sigma && dW && ws && rows > 0 && cols > 0 && lo > 0);
  hipStream_t s = (hipStream_t)stream;
  SnView w{W, rows, cols, lo, rs, hs};
  const long long total = (long long)rows * cols;
  const int nparts = (int)std::min<long long>(SN_DOT_PARTS, (total + 1023) / 1024);
  float* part = (float*)ws;
  sn_dot_kernel<<<nparts, 256, 0, s>>>(dWeff, W, total, part);
  RGAN_CHECK_LAUNCH();
  const int vec = lo % 4 == 0 && rs % 4 == 0 && hs % 4 == 0 && cols % 4 == 0 &&
                  (((uintptr_t)dWeff | (uintptr_t)dW | (uintptr_t)v) & 15) == 0;
  sn_bwd_kernel<<<rows, 256, 0, s>>>(w, dWeff, part, nparts, u, v, inv_sigma, dW, accumulate, vec);
  RGAN_CHECK_LAUNCH();
  return 0;
}

// ------------------------------------------------------------------ Adam
struct AdamTensor {
  float* p;
  const float* g;
  float* m;
  float* v;
  long long n;
};
constexpr int ADAM_CHUNK = 48;
// Work split in proportion to size: tensor j owns blocks [first[j], first[j+1]) of a 1-D
// grid, ADAM_BLOCK_ELEMS elements per block (16 per thread: 4 float4 of each of p, g, m, v
// in flight).  A block-per-(chunk, tensor) 2-D grid sized by the largest tensor left most
// blocks of the small tensors idle and gave the big ones 1 scalar element per load.
constexpr int ADAM_BLOCK_ELEMS = 4096;
struct AdamBatch {
  AdamTensor t[ADAM_CHUNK];
  int first[ADAM_CHUNK + 1];
  int cnt;
};

__global__ void adam_step_inc(float* step) { step[0] += 1.f; }
extern "C" int rgan_adam_step_inc(float* step, void* stream) {  // (rgan_adam_packed, conv_gemm.hip)
  RGAN_REQUIRE(step);
  adam_step_inc<<<1, 1, 0, (hipStream_t)stream>>>(step);
  RGAN_CHECK_LAUNCH();
  return 0;
}

__global__ __launch_bounds__(256) void adam_kernel(AdamBatch b, const double* __restrict__ hyper,
                                                   const float* __restrict__ step) {
  int j = 0;
  while (j + 1 < b.cnt && (int)blockIdx.x >= b.first[j + 1]) ++j;
  const AdamTensor T = b.t[j];
  const AdamConst k = adam_const(hyper, step);
  const long long e0 = (long long)((int)blockIdx.x - b.first[j]) * ADAM_BLOCK_ELEMS;
  const long long e1 = min(T.n, e0 + ADAM_BLOCK_ELEMS);
  const bool vec = (T.n & 3) == 0 && ((((uintptr_t)T.p | (uintptr_t)T.g | (uintptr_t)T.m | (uintptr_t)T.v) & 15) == 0);
  if (vec) {
    constexpr int U = ADAM_BLOCK_ELEMS / 1024;  // float4 per thread
    float4 P[U], G[U], M[U], V[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long long i = e0 + 4 * (threadIdx.x + 256 * u);
      if (i < e1) {
        P[u] = *reinterpret_cast<const float4*>(T.p + i);
        G[u] = *reinterpret_cast<const float4*>(T.g + i);
        M[u] = *reinterpret_cast<const float4*>(T.m + i);
        V[u] = *reinterpret_cast<const float4*>(T.v + i);
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long long i = e0 + 4 * (threadIdx.x + 256 * u);
      if (i < e1) {
        adam_elem(k, G[u].x, P[u].x, M[u].x, V[u].x);
        adam_elem(k, G[u].y, P[u].y, M[u].y, V[u].y);
        adam_elem(k, G[u].z, P[u].z, M[u].z, V[u].z);
        adam_elem(k, G[u].w, P[u].w, M[u].w, V[u].w);
        *reinterpret_cast<float4*>(T.m + i) = M[u];
        *reinterpret_cast<float4*>(T.v + i) = V[u];
        *reinterpret_cast<float4*>(T.p + i) = P[u];
      }
    }
  } else {
    for (long long i = e0 + threadIdx.x; i < e1; i += 256) {
      float p = T.p[i], m = T.m[i], v = T.v[i];
      adam_elem(k, T.g[i], p, m, v);
      T.m[i] = m;
      T.v[i] = v;
      T.p[i] = p;
    }
  }
}

extern "C" int rgan_adam(int ntensors, float* const* params, const float* const* grads, float* const* exp_avg,
                         float* const* exp_avg_sq, const long long* numel, const double* hyper, float* step,
                         void* stream) {
  RGAN_REQUIRE(ntensors >= 0 && hyper && step);
  RGAN_REQUIRE(ntensors == 0 || (params && grads && exp_avg && exp_avg_sq && numel));
  // every tensor checked before the first launch: a refused call changes nothing
  for (int j = 0; j < ntensors; ++j)
    RGAN_REQUIRE(params[j] && grads[j] && exp_avg[j] && exp_avg_sq[j] && numel[j] >= 0 && numel[j] < (1LL << 31));
  hipStream_t s = (hipStream_t)stream;
  adam_step_inc<<<1, 1, 0, s>>>(step);
  RGAN_CHECK_LAUNCH();
  for (int base = 0; base < ntensors; base += ADAM_CHUNK) {
    const int cnt = std::min(ADAM_CHUNK, ntensors - base);
    AdamBatch b{};
    b.cnt = cnt;
    long long blocks = 0;
    for (int i = 0; i < cnt; ++i) {
      const int j = base + i;
      b.t[i] = AdamTensor{params[j], grads[j], exp_avg[j], exp_avg_sq[j], numel[j]};
      b.first[i] = (int)blocks;
      blocks += (numel[j] + ADAM_BLOCK_ELEMS - 1) / ADAM_BLOCK_ELEMS;
      RGAN_REQUIRE(blocks < (1LL << 30));
    }
    b.first[cnt] = (int)blocks;
    if (blocks == 0) continue;
    adam_kernel<<<(unsigned)blocks, 256, 0, s>>>(b, hyper, step);
    RGAN_CHECK_LAUNCH();
  }
  return 0;
}

__global__ void lr_decay_kernel(double* hyper, double gamma) { hyper[0] *= gamma; }

extern "C" int rgan_lr_decay(double* hyper, double gamma, void* stream) {
  RGAN_REQUIRE(hyper);
  lr_decay_kernel<<<1, 1, 0, (hipStream_t)stream>>>(hyper, gamma);
  RGAN_CHECK_LAUNCH();
  return 0;
}

// ------------------------------------------------------------------ data movement
__global__ void gather_kernel(const float* __restrict__ images, const long long* __restrict__ idx, int batch,
                              long long per, float* __restrict__ out) {
  const long long total = (long long)batch * per;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const long long b = i / per, e = i - b * per;
    out[i] = images[idx[b] * per + e];
  }
}

extern "C" int rgan_gather_images(const float* images, const long long* idx, int batch, long long per,
                                  float* out, void* stream) {
  RGAN_REQUIRE(images && idx && out && batch > 0 && per > 0);
  gather_kernel<<<grid1(batch * per), 256, 0, (hipStream_t)stream>>>(images, idx, batch, per, out);
  RGAN_CHECK_LAUNCH();
  return 0;
}

extern "C" const char* rgan_version(void) { return "rgan-mi355x 0.2 gfx950 fp32-mfma abi4"; }
extern "C" int rgan_abi_version(void) { return RGAN_ABI_VERSION; }

}  // namespace rgan
