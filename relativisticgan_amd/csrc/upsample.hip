// --NN_conv generator blocks: nearest-neighbour Upsample(x2) followed by Conv2d(k3, s1, p1)
// (GLI:351-356, 377-382) executed as ONE stride-2 transposed convolution.
//
// Output pixel (2m+a) of conv3x3(up2(x)) reads up-sampled rows 2m+a-1 .. 2m+a+1, i.e. input
// rows {m-1, m} (a = 0) or {m, m+1} (a = 1) -- the same two rows, per phase, that a k4 s2 p1
// ConvTranspose2d reads.  Folding the 3 taps onto the 4 transposed-conv taps per dimension,
//     Wt[kh] = sum_d A[kh][d] W[d],   A = [[0,0,1], [0,1,1], [1,1,0], [1,0,0]],
// gives conv3x3(up2(x), W) == conv_transpose2d(x, Wt, stride 2, pad 1) exactly in real
// arithmetic, with 4*Cin instead of 9*Cin MACs per output pixel and no up-sampled tensor in
// HBM.  The MFMA sub-pixel-phase GEMMs (MODE_CONVT2) then run the layer unchanged; the weight
// gradient is the adjoint fold of the transposed conv's weight gradient (A^T per dimension).
#include "common.h"

namespace rgan {

// one dimension of the fold: w4 = A w3
__device__ __forceinline__ void fold_row(const float* w3, float* w4) {
  w4[0] = w3[2];
  w4[1] = w3[1] + w3[2];
  w4[2] = w3[0] + w3[1];
  w4[3] = w3[0];
}

// one thread per (co, ci): reads the contiguous 9 taps of W[co][ci] (lanes read adjacent
// 36-byte runs), writes the 16 contiguous taps of Wt[ci][co] as four float4 stores.
__global__ __launch_bounds__(256) void nn_fold_kernel(const float* __restrict__ W, int cout, int cin,
                                                      float* __restrict__ Wt) {
  const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (long long)cout * cin) return;
  const int co = (int)(t / cin), ci = (int)(t % cin);
  const float* w = W + t * 9;
  float r[3][4];
  for (int dh = 0; dh < 3; ++dh) fold_row(w + dh * 3, r[dh]);
  float o[16];
  for (int kw = 0; kw < 4; ++kw) {
    float c3[3] = {r[0][kw], r[1][kw], r[2][kw]}, c4[4];
    fold_row(c3, c4);
    for (int kh = 0; kh < 4; ++kh) o[kh * 4 + kw] = c4[kh];
  }
  float4* dst = reinterpret_cast<float4*>(Wt + ((long long)ci * cout + co) * 16);
  for (int q = 0; q < 4; ++q) dst[q] = make_float4(o[4 * q], o[4 * q + 1], o[4 * q + 2], o[4 * q + 3]);
}

// adjoint: dW[co][ci][dh][dw] = sum_{kh,kw} A[kh][dh] A[kw][dw] dWt[ci][co][kh][kw]
__device__ __forceinline__ void unfold_row(const float* g4, float* g3) {
  g3[0] = g4[2] + g4[3];
  g3[1] = g4[1] + g4[2];
  g3[2] = g4[0] + g4[1];
}

__global__ __launch_bounds__(256) void nn_unfold_kernel(const float* __restrict__ dWt, int cout, int cin,
                                                        float* __restrict__ dW) {
  const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (long long)cout * cin) return;
  const int co = (int)(t / cin), ci = (int)(t % cin);
  const float4* src = reinterpret_cast<const float4*>(dWt + ((long long)ci * cout + co) * 16);
  float g[16];
  for (int q = 0; q < 4; ++q) {
    const float4 v = src[q];
    g[4 * q] = v.x; g[4 * q + 1] = v.y; g[4 * q + 2] = v.z; g[4 * q + 3] = v.w;
  }
  float rows[4][3];  // per kh: the 3 folded-back columns
  for (int kh = 0; kh < 4; ++kh) unfold_row(g + kh * 4, rows[kh]);
  float* out = dW + t * 9;
  for (int dw = 0; dw < 3; ++dw) {
    float c4[4] = {rows[0][dw], rows[1][dw], rows[2][dw], rows[3][dw]}, c3[3];
    unfold_row(c4, c3);
    for (int dh = 0; dh < 3; ++dh) out[dh * 3 + dw] = c3[dh];
  }
}

}  // namespace rgan

using namespace rgan;

extern "C" int rgan_nn_fold_weight(const float* w, int cout, int cin, float* wt, void* stream) {
  RGAN_REQUIRE(w && wt && cout > 0 && cin > 0 && ((uintptr_t)wt & 15) == 0);
  const long long n = (long long)cout * cin;
  hipLaunchKernelGGL(nn_fold_kernel, dim3(ceil_div(n, 256)), dim3(256), 0, (hipStream_t)stream, w, cout, cin, wt);
  RGAN_CHECK_LAUNCH();
  return 0;
}

extern "C" int rgan_nn_unfold_grad(const float* dwt, int cout, int cin, float* dw, void* stream) {
  RGAN_REQUIRE(dwt && dw && cout > 0 && cin > 0 && ((uintptr_t)dwt & 15) == 0);
  const long long n = (long long)cout * cin;
  hipLaunchKernelGGL(nn_unfold_kernel, dim3(ceil_div(n, 256)), dim3(256), 0, (hipStream_t)stream, dwt, cout, cin,
                     dw);
  RGAN_CHECK_LAUNCH();
  return 0;
}
