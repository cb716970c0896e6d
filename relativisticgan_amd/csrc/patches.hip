// Image layers as plain GEMMs over a materialised patch matrix.
//
// The DCGAN image layers are k4 s2 p1 convolutions with <= 4 image channels: D's first
// Conv2d (GLI:404) and G's closing ConvTranspose2d (GLI:386).  Their weight gradients (and
// the ConvT's data gradient) reduce over a 16-tap x <= 4-channel window of the image; as an
// implicit GEMM that window is a scalar gather with index math per element, which the fp32
// MFMA cannot hide (it shares the VALU).  Here the window is materialised once per pass as
// X[(b, i, j)][t * 4 + c] = img[b][c][2i - 1 + kh][2j - 1 + kw]   (t = 4 kh + kw, c < 4,
// zero outside the image and for c >= C), a dense 64-float row per grid pixel (256 B), so
// every use becomes a 1x1 GEMM on the FAST path (K or N = 64):
//   D conv forward       y[p][co]   = sum_n X[p][n] W1[co][n]          (conv_fwd 1x1)
//   D conv weight grad   dW1[co][n] = sum_p dy[p][co] X[p][n]          (conv_wgrad 1x1)
//   G convT data grad    dx[p][ci]  = sum_n Xg[p][n] W1[ci][n]         (Xg = patches of dy)
//   G convT weight grad  dW1[n][ci] = sum_p Xg[p][n] x[p][ci]          (conv_wgrad 1x1)
// with W1[o][t * 4 + c] = W[o][c][t] (Conv2d [co][ci][t] or ConvTranspose2d [ci][co][t] read
// as [o][c]); the grid is the small side of the layer (the conv output / the convT input).
#include "common.h"

#include <algorithm>

namespace rgan {

// one thread per (grid pixel, tap): 4 channels -> one float4; 16 lanes write a pixel's row
__global__ __launch_bounds__(256) void patches_k4s2_kernel(const float* __restrict__ img, int B, int C, int H,
                                                           int W, long long sb, long long sc, long long sh,
                                                           long long sw, float* __restrict__ X) {
  const int Hg = H / 2, Wg = W / 2;
  const long long total = (long long)B * Hg * Wg * 16;
  for (long long idx = (long long)blockIdx.x * 256 + threadIdx.x; idx < total; idx += (long long)gridDim.x * 256) {
    const int t = (int)(idx & 15);
    const long long p = idx >> 4;
    const int j = (int)(p % Wg);
    const long long r = p / Wg;
    const int i = (int)(r % Hg), b = (int)(r / Hg);
    const int ih = 2 * i - 1 + (t >> 2), iw = 2 * j - 1 + (t & 3);
    float v[4] = {0.f, 0.f, 0.f, 0.f};
    if ((unsigned)ih < (unsigned)H && (unsigned)iw < (unsigned)W) {
      const float* s = img + (long long)b * sb + (long long)ih * sh + (long long)iw * sw;
#pragma unroll
      for (int c = 0; c < 4; ++c)
        if (c < C) v[c] = s[(long long)c * sc];
    }
    *reinterpret_cast<float4*>(X + p * 64 + 4 * t) = make_float4(v[0], v[1], v[2], v[3]);
  }
}

// W1[o][t * 4 + c] = W[o * so + c * sc + t]  (c < C, else 0)
__global__ void patch_weight_kernel(const float* __restrict__ Wt, int O, int C, long long so, long long sc,
                                    float* __restrict__ W1) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= O * 64) return;
  const int o = e >> 6, n = e & 63, t = n >> 2, c = n & 3;
  W1[e] = c < C ? Wt[(long long)o * so + (long long)c * sc + t] : 0.f;
}

// dW[o][c][t] = G1[o * so + (t * 4 + c) * sn]  (c < C): back to torch weight layout
__global__ void unpatch_grad_kernel(const float* __restrict__ G1, int O, int C, long long so, long long sn,
                                    float* __restrict__ dW, int accum) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= O * C * 16) return;
  const int t = e & 15, oc = e >> 4, c = oc % C, o = oc / C;
  const float v = G1[(long long)o * so + (long long)(t * 4 + c) * sn];
  dW[e] = accum ? dW[e] + v : v;
}

}  // namespace rgan

using namespace rgan;

extern "C" int rgan_patches_k4s2(const float* img, int batch, int channels, int height, int width,
                                 const long long* strides, float* patches, void* stream) {
  RGAN_REQUIRE(img && patches && strides && batch > 0 && channels > 0 && channels <= 4 && height >= 2 &&
               width >= 2 && height % 2 == 0 && width % 2 == 0 && ((uintptr_t)patches & 15) == 0);
  const long long total = (long long)batch * (height / 2) * (width / 2) * 16;
  const int blocks = (int)std::min<long long>((total + 255) / 256, 65536);
  patches_k4s2_kernel<<<blocks, 256, 0, (hipStream_t)stream>>>(img, batch, channels, height, width, strides[0],
                                                               strides[1], strides[2], strides[3], patches);
  RGAN_CHECK_LAUNCH();
  return 0;
}

extern "C" int rgan_patch_weight(const float* w, int rows, int channels, long long row_stride,
                                 long long channel_stride, float* w1, void* stream) {
  RGAN_REQUIRE(w && w1 && rows > 0 && channels > 0 && channels <= 4);
  patch_weight_kernel<<<ceil_div((long long)rows * 64, 256), 256, 0, (hipStream_t)stream>>>(
      w, rows, channels, row_stride, channel_stride, w1);
  RGAN_CHECK_LAUNCH();
  return 0;
}

extern "C" int rgan_unpatch_grad(const float* g1, int rows, int channels, long long row_stride,
                                 long long col_stride, float* dw, int accumulate, void* stream) {
  RGAN_REQUIRE(g1 && dw && rows > 0 && channels > 0 && channels <= 4);
  unpatch_grad_kernel<<<ceil_div((long long)rows * channels * 16, 256), 256, 0, (hipStream_t)stream>>>(
      g1, rows, channels, row_stride, col_stride, dw, accumulate);
  RGAN_CHECK_LAUNCH();
  return 0;
}
