// G's first layer: ConvTranspose2d(z, Cout, 4, 1, 0) on a 1x1 input + train-mode BatchNorm2d
// + activation (GLI:334-345 "Start-ConvTranspose2d" / "Start-BatchNorm2d" / "Start-ReLU"), and
// its weight gradient.
//
// On a 1x1 input the transposed conv is a plain product y[b][t][co] = sum_ci z[b][ci] *
// W[ci][co][t] (t = 4 kh + kw) with M = B rows only: as an implicit GEMM it is one 128-row m
// tile (B = 32 uses a quarter) over 4 k tiles, latency-bound (17 us at C1, 7 TF/s) and
// followed by three BatchNorm launches.  Here ONE launch does all of it: a block owns 16
// output channels x 16 taps = 256 columns (thread = column) and the whole batch, so each
// channel's B x 16 BatchNorm population is inside the block:
//   1. y columns by fp32 FMA over ci (z staged in LDS, read as broadcasts; W rows of the
//      block's 256 columns are contiguous in torch layout [ci][co][t]);
//   2. per channel: exact two-pass mean / variance in double over the block-resident values
//      (the 16 tap lanes of a channel are 16 consecutive lanes: fixed xor-butterfly), running
//      statistics updated as torch does (unbiased variance), (mean, invstd) written;
//   3. a = act(y * al + be) with al = gamma * invstd, be = beta - mean * al (bn_apply's form);
//      y (for the backward) and a written NHWC through an LDS transpose (64-B channel runs).
// The block's columns stay in registers for the whole batch (B <= 64): W is read once.
// rgan_g1_wgrad: dW[ci][co][t] (+)= sum_b z[b][ci] * dy[b][t][co], thread = column, the
// column's B gradient values in registers, z broadcast from LDS.
#include "common.h"

namespace rgan {

constexpr int G1_CB = 16;   // channels per block (x 16 taps = 256 threads)
// batch sizes with an instantiation (the column's B values live in registers): 32, 64

template <int B>
__global__ __launch_bounds__(256) void g1_fwd_bn_kernel(const float* __restrict__ z, int Cin,
                                                        const float* __restrict__ w, int Cout,
                                                        const float* __restrict__ gamma,
                                                        const float* __restrict__ beta, float eps, float momentum,
                                                        float* running_mean, float* running_var, long long* nbt,
                                                        int act, float alpha, float* __restrict__ y,
                                                        float* __restrict__ a, float* __restrict__ stats) {
  extern __shared__ float lds[];
  float* zs = lds;                        // [B][Cin]
  float* ys = lds + (size_t)B * Cin;      // [32][16 taps][16 channels]: output staging
  __shared__ float alv[G1_CB], bev[G1_CB];
  const int tid = threadIdx.x;
  const int co0 = blockIdx.x * G1_CB;
  for (int i = tid; i < B * Cin; i += 256) zs[i] = z[i];
  __syncthreads();
  // thread t computes column (channel co0 + (t >> 4), tap t & 15) for the whole batch: its W
  // entries W[ci][co][tap] are contiguous in t
  const int c_l = tid >> 4, t_l = tid & 15;
  const float* wp = w + (size_t)(co0 + c_l) * 16 + t_l;
  const size_t wstride = (size_t)Cout * 16;
  float acc[B];
#pragma unroll
  for (int b = 0; b < B; ++b) acc[b] = 0.f;
  // ci in order; z rows read as float4 broadcasts (4 ci per LDS read)
  for (int ci = 0; ci < Cin; ci += 4) {
    const float w0 = wp[(size_t)ci * wstride], w1 = wp[(size_t)(ci + 1) * wstride];
    const float w2 = wp[(size_t)(ci + 2) * wstride], w3 = wp[(size_t)(ci + 3) * wstride];
#pragma unroll
    for (int b = 0; b < B; ++b) {
      const float4 zz = *reinterpret_cast<const float4*>(zs + b * Cin + ci);
      acc[b] = fmaf(zz.w, w3, fmaf(zz.z, w2, fmaf(zz.y, w1, fmaf(zz.x, w0, acc[b]))));
    }
  }
  // channel statistics, exact two-pass in double: the channel's 16 taps are lanes
  // 16 c_l .. 16 c_l + 15 of one wave (fixed xor-butterfly)
  double s1 = 0.0;
#pragma unroll
  for (int b = 0; b < B; ++b) s1 += (double)acc[b];
#pragma unroll
  for (int o = 1; o < 16; o <<= 1) s1 += __shfl_xor(s1, o);
  const double n = (double)B * 16.0, mean = s1 / n;
  double s2 = 0.0;
#pragma unroll
  for (int b = 0; b < B; ++b) {
    const double d = (double)acc[b] - mean;
    s2 += d * d;
  }
#pragma unroll
  for (int o = 1; o < 16; o <<= 1) s2 += __shfl_xor(s2, o);
  const int co = co0 + c_l;
  const double var = s2 / n;
  const float st_mean = (float)mean, st_inv = (float)(1.0 / sqrt(var + (double)eps));
  if (t_l == 0) {
    stats[co] = st_mean;
    stats[Cout + co] = st_inv;
    if (running_mean) running_mean[co] = (1.f - momentum) * running_mean[co] + momentum * st_mean;
    if (running_var) {
      const float unb = n > 1.0 ? (float)(s2 / (n - 1.0)) : (float)var;
      running_var[co] = (1.f - momentum) * running_var[co] + momentum * unb;
    }
    const float al = (gamma ? gamma[co] : 1.f) * st_inv;  // bn_apply's affine form
    alv[c_l] = al;
    bev[c_l] = (beta ? beta[co] : 0.f) - st_mean * al;
  }
  if (blockIdx.x == 0 && tid == 0 && nbt) nbt[0] += 1;
  // y and a NHWC, 32 rows at a time through LDS: thread = (tap, channel) with the channel
  // fastest (64-B runs of the 16 channels)
  const int wc = tid & 15, wt = tid >> 4;
#pragma unroll
  for (int h = 0; h < B / 32; ++h) {  // unrolled: acc indices stay compile-time (registers)
    const int b0 = 32 * h;
    __syncthreads();  // alv / bev written; the previous chunk's reads done
#pragma unroll
    for (int b = 0; b < 32; ++b) ys[(b * 16 + t_l) * 16 + c_l] = acc[b0 + b];
    __syncthreads();
    const float al = alv[wc], be = bev[wc];
    for (int b = 0; b < 32; ++b) {
      const float v = ys[(b * 16 + wt) * 16 + wc];
      const size_t o = ((size_t)(b0 + b) * 16 + wt) * Cout + co0 + wc;
      y[o] = v;
      a[o] = act_fwd(v * al + be, act, alpha);
    }
  }
}

template <int B>
__global__ __launch_bounds__(256) void g1_wgrad_kernel(const float* __restrict__ z, int Cin,
                                                       const float* __restrict__ dy, int Cout, float* dw,
                                                       int accumulate) {
  extern __shared__ float zs[];  // [B][Cin]
  const int tid = threadIdx.x, c_l = tid >> 4, t_l = tid & 15;
  const int co0 = blockIdx.x * G1_CB, co = co0 + c_l;
  for (int i = tid; i < B * Cin; i += 256) zs[i] = z[i];
  float g[B];
#pragma unroll
  for (int b = 0; b < B; ++b) g[b] = dy[((size_t)b * 16 + t_l) * Cout + co];
  __syncthreads();
  float* wp = dw + (size_t)co * 16 + t_l;
  const size_t wstride = (size_t)Cout * 16;
  for (int ci = 0; ci < Cin; ci += 4) {  // b in order per output, as the GEMM's K loop
    float s[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int b = 0; b < B; ++b) {
      const float4 zz = *reinterpret_cast<const float4*>(zs + b * Cin + ci);
      s[0] = fmaf(zz.x, g[b], s[0]);
      s[1] = fmaf(zz.y, g[b], s[1]);
      s[2] = fmaf(zz.z, g[b], s[2]);
      s[3] = fmaf(zz.w, g[b], s[3]);
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      float* d = wp + (size_t)(ci + k) * wstride;
      *d = accumulate ? *d + s[k] : s[k];
    }
  }
}

}  // namespace rgan

using namespace rgan;

extern "C" int rgan_g1_fwd_bn(const float* z, int B, int Cin, const float* w, int Cout, const float* gamma,
                              const float* beta, float eps, float momentum, float* running_mean, float* running_var,
                              long long* num_batches_tracked, int act, float act_alpha, float* y, float* a,
                              float* stats, void* stream) {
  RGAN_REQUIRE(z && w && y && a && stats && (B == 32 || B == 64) && Cin >= 4 && Cin % 4 == 0 &&
               Cout >= G1_CB && Cout % G1_CB == 0 && ((uintptr_t)z & 15) == 0);
  const size_t lds = ((size_t)B * Cin + 32 * 256) * sizeof(float);
  RGAN_REQUIRE(lds <= 64 * 1024);
  const hipStream_t s = (hipStream_t)stream;
  if (B == 32)
    g1_fwd_bn_kernel<32><<<Cout / G1_CB, 256, lds, s>>>(z, Cin, w, Cout, gamma, beta, eps, momentum, running_mean,
                                                        running_var, num_batches_tracked, act, act_alpha, y, a, stats);
  else
    g1_fwd_bn_kernel<64><<<Cout / G1_CB, 256, lds, s>>>(z, Cin, w, Cout, gamma, beta, eps, momentum, running_mean,
                                                        running_var, num_batches_tracked, act, act_alpha, y, a, stats);
  RGAN_CHECK_LAUNCH();
  return 0;
}

extern "C" int rgan_g1_wgrad(const float* z, int B, int Cin, const float* dy, int Cout, float* dw, int accumulate,
                             void* stream) {
  RGAN_REQUIRE(z && dy && dw && (B == 32 || B == 64) && Cin >= 4 && Cin % 4 == 0 && Cout >= G1_CB &&
               Cout % G1_CB == 0 && ((uintptr_t)z & 15) == 0);
  const size_t lds = (size_t)B * Cin * sizeof(float);
  RGAN_REQUIRE(lds <= 64 * 1024);
  const hipStream_t s = (hipStream_t)stream;
  if (B == 32) g1_wgrad_kernel<32><<<Cout / G1_CB, 256, lds, s>>>(z, Cin, dy, Cout, dw, accumulate);
  else g1_wgrad_kernel<64><<<Cout / G1_CB, 256, lds, s>>>(z, Cin, dy, Cout, dw, accumulate);
  RGAN_CHECK_LAUNCH();
  return 0;
}
