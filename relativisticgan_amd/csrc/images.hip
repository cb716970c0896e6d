// Image export for the sample / FID image path (GLI:563-565 sample grid, GLI:759-768 extra
// images; code/inference_art.py): the float -> uint8 quantisation that
// torchvision.utils.save_image performs before handing pixels to PIL, fused with make_grid's
// tiling and the optional min/max normalisation, on the device.  The host only encodes PNG.
//
// Per output byte: t = x * scale + shift (the reference's `fake*.5+.5` for extra images);
// normalize: t = (clamp(t, lo, hi) - lo) / max(hi - lo, 1e-5) with (lo, hi) = min / max of the
// whole batch (make_grid(normalize=True)); then u8 = trunc(clamp(t * 255 + 0.5, 0, 255))
// (grid.mul(255).add_(0.5).clamp_(0, 255).to(uint8)).  Every step is a separately rounded fp32
// operation, as in torch (no FMA contraction).  Grid padding pixels are pad value 0 -> 0.
#include "common.h"

namespace rgan {

__global__ __launch_bounds__(256) void minmax_partial(const float* __restrict__ x, long long n,
                                                      float* __restrict__ part) {
  __shared__ float lo_s[256], hi_s[256];
  float lo = INFINITY, hi = -INFINITY;
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
    const float v = x[i];
    lo = fminf(lo, v);
    hi = fmaxf(hi, v);
  }
  lo_s[threadIdx.x] = lo;
  hi_s[threadIdx.x] = hi;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if (threadIdx.x < s) {
      lo_s[threadIdx.x] = fminf(lo_s[threadIdx.x], lo_s[threadIdx.x + s]);
      hi_s[threadIdx.x] = fmaxf(hi_s[threadIdx.x], hi_s[threadIdx.x + s]);
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    part[2 * blockIdx.x] = lo_s[0];
    part[2 * blockIdx.x + 1] = hi_s[0];
  }
}

__global__ void minmax_final(const float* __restrict__ part, int nparts, float* __restrict__ out) {
  if (threadIdx.x != 0) return;
  float lo = INFINITY, hi = -INFINITY;
  for (int i = 0; i < nparts; ++i) {
    lo = fminf(lo, part[2 * i]);
    hi = fmaxf(hi, part[2 * i + 1]);
  }
  out[0] = lo;
  out[1] = hi;
}

struct ImgArgs {
  const float* x;
  int B, C, H, W;
  long long sb, sc, sh, sw;
  float scale, shift;
  const float* range;  // nullable [lo, hi]
  int grid;            // 0: per-image [B][H][W][C]; 1: make_grid [Hg][Wg][C]
  int nrow, pad, xmaps, Hg, Wg;
  unsigned char* out;
};

__global__ __launch_bounds__(256) void to_u8_kernel(ImgArgs a) {
  const long long total = a.grid ? (long long)a.Hg * a.Wg * a.C : (long long)a.B * a.H * a.W * a.C;
  float lo = 0.f, den = 1.f;
  if (a.range) {
    lo = a.range[0];
    den = fmaxf(__fsub_rn(a.range[1], lo), 1e-5f);
  }
  for (long long e = blockIdx.x * 256LL + threadIdx.x; e < total; e += (long long)gridDim.x * 256) {
    const int c = (int)(e % a.C);
    const long long pix = e / a.C;
    int b, i, j;
    bool inside = true;
    if (a.grid) {
      const int gy = (int)(pix / a.Wg), gx = (int)(pix % a.Wg);
      const int th = a.H + a.pad, tw = a.W + a.pad;
      const int ty = (gy - a.pad) / th, tx = (gx - a.pad) / tw;
      i = gy - a.pad - ty * th;
      j = gx - a.pad - tx * tw;
      b = ty * a.xmaps + tx;
      inside = gy >= a.pad && gx >= a.pad && i < a.H && j < a.W && tx < a.xmaps && b < a.B;
    } else {
      b = (int)(pix / ((long long)a.H * a.W));
      const int r = (int)(pix % ((long long)a.H * a.W));
      i = r / a.W;
      j = r % a.W;
    }
    float t = 0.f;  // make_grid's pad value
    if (inside) {
      t = __fadd_rn(__fmul_rn(a.x[b * a.sb + c * a.sc + i * a.sh + j * a.sw], a.scale), a.shift);
      if (a.range) t = __fdiv_rn(__fsub_rn(fminf(fmaxf(t, lo), a.range[1]), lo), den);
    }
    const float q = fminf(fmaxf(__fadd_rn(__fmul_rn(t, 255.f), 0.5f), 0.f), 255.f);
    a.out[e] = (unsigned char)(int)q;
  }
}

// Real-image batches (GLI:159-179): the dataset lives in HBM as decoded uint8 [N][C][S][S]
// (ImageFolder + Resize done once at load); a batch is a gather of sampled images fused with
// ToTensor + Normalize(0.5, 0.5): x = (u8 / 255 - 0.5) / 0.5, each op rounded in fp32 like
// torchvision's div(255).sub_(0.5).div_(0.5).  4 bytes -> float4 per thread (per % 4 == 0).
__global__ __launch_bounds__(256) void gather_u8_kernel(const unsigned char* __restrict__ images,
                                                        const long long* __restrict__ idx, int batch, long long per,
                                                        float* __restrict__ out) {
  const long long q = per / 4, total = (long long)batch * q;
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < total; i += (long long)gridDim.x * 256) {
    const long long b = i / q, e = i - b * q;
    const uchar4 v = reinterpret_cast<const uchar4*>(images + idx[b] * per)[e];
    auto f = [](unsigned char u) { return __fdiv_rn(__fsub_rn(__fdiv_rn((float)u, 255.f), 0.5f), 0.5f); };
    reinterpret_cast<float4*>(out)[i] = make_float4(f(v.x), f(v.y), f(v.z), f(v.w));
  }
}

}  // namespace rgan

using namespace rgan;

extern "C" int rgan_gather_images_u8(const unsigned char* images, const long long* idx, int batch, long long per,
                                     float* out, void* stream) {
  RGAN_REQUIRE(images && idx && out && batch > 0 && per > 0 && per % 4 == 0 && ((uintptr_t)out & 15) == 0);
  const long long total = (long long)batch * per / 4;
  const int blocks = (int)std::min<long long>((total + 255) / 256, 8192);
  gather_u8_kernel<<<blocks, 256, 0, (hipStream_t)stream>>>(images, idx, batch, per, out);
  RGAN_CHECK_LAUNCH();
  return 0;
}

extern "C" size_t rgan_minmax_ws_bytes(long long n) {
  (void)n;
  return 2 * 256 * sizeof(float);
}

extern "C" int rgan_minmax(const float* x, long long n, float* out2, void* ws, void* stream) {
  RGAN_REQUIRE(x && out2 && ws && n > 0);
  hipStream_t s = (hipStream_t)stream;
  const int parts = (int)std::min<long long>(256, (n + 255) / 256);
  minmax_partial<<<parts, 256, 0, s>>>(x, n, (float*)ws);
  RGAN_CHECK_LAUNCH();
  minmax_final<<<1, 64, 0, s>>>((const float*)ws, parts, out2);
  RGAN_CHECK_LAUNCH();
  return 0;
}

extern "C" int rgan_images_to_u8(const float* x, int B, int C, int H, int W, const long long* strides,
                                 float scale, float shift, const float* range, int grid, int nrow, int padding,
                                 unsigned char* out, void* stream) {
  RGAN_REQUIRE(x && strides && out && B > 0 && C > 0 && H > 0 && W > 0 && nrow > 0 && padding >= 0);
  ImgArgs a;
  a.x = x; a.B = B; a.C = C; a.H = H; a.W = W;
  a.sb = strides[0]; a.sc = strides[1]; a.sh = strides[2]; a.sw = strides[3];
  a.scale = scale; a.shift = shift; a.range = range;
  a.grid = grid; a.nrow = nrow; a.pad = padding;
  a.xmaps = std::min(nrow, B);
  const int ymaps = (B + a.xmaps - 1) / a.xmaps;
  a.Hg = (H + padding) * ymaps + padding;
  a.Wg = (W + padding) * a.xmaps + padding;
  a.out = out;
  const long long total = grid ? (long long)a.Hg * a.Wg * C : (long long)B * H * W * C;
  const int blocks = (int)std::min<long long>((total + 255) / 256, 4096);
  to_u8_kernel<<<blocks, 256, 0, (hipStream_t)stream>>>(a);
  RGAN_CHECK_LAUNCH();
  return 0;
}
