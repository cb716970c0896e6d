// G's first layer: ConvTranspose2d(z, Cout, 4, 1, 0) on a 1x1 input + train-mode BatchNorm2d
// + activation (GLI:334-345 "Start-ConvTranspose2d" / "Start-BatchNorm2d" / "Start-ReLU"), and
// its weight gradient.
//
// On a 1x1 input the transposed conv is a plain product y[b][t][co] = sum_ci z[b][ci] *
// W[ci][co][t] (t = 4 kh + kw) with M = B rows only: as an implicit GEMM it is one 128-row m
// tile (B = 32 uses a quarter) over 4 k tiles, latency-bound (17 us at C1, 7 TF/s) and
// followed by three BatchNorm launches.  Here ONE launch does all of it: a block owns 4
// output channels x 16 taps and the whole batch (256 threads: a thread = one column x a
// quarter of the batch rows), so each channel's B x 16 BatchNorm population is one wave's:
//   1. y by fp32 FMA over ci in order (z staged in LDS, read as float4 broadcasts; a thread's
//      W column read 64 entries at a time into registers -- one load latency per chunk);
//   2. per channel: exact two-pass mean / variance in double over the wave's registers
//      (fixed xor-butterfly), running statistics updated as torch does (unbiased
//      variance), (mean, invstd) written;
//   3. a = act(y * al + be) with al = gamma * invstd, be = beta - mean * al (bn_apply's form);
//      y (for the backward) and a written NHWC through an LDS transpose (64-B channel runs).
// The block's columns stay in registers for the whole batch (B <= 64): W is read once.
// rgan_g1_wgrad: dW[ci][co][t] (+)= sum_b z[b][ci] * dy[b][t][co], thread = column x a quarter
// of the ci range, the column's B gradient values in registers, z broadcast from LDS.
#include "common.h"

namespace rgan {

constexpr int G1_CB = 4;    // channels per block (x 16 taps x 4 batch / ci groups = 256 threads):
                            // Cout / 4 blocks, so even C1's 1024 channels spread over all CUs
constexpr int G1_T = G1_CB * 64;
constexpr int G1_WCH = 32;  // W entries of a thread's column held in registers at a time
// instantiated for B (batch: a thread's rows live in registers) in {32, 64} and CIN (z size)
// in {64, 128}

// thread = (channel c_l, group q, tap t): tid = 64 c_l + 16 q + t -- a channel's 64 threads are
// one wave (its BatchNorm population B x 16 sits in that wave's registers)
template <int B, int Cin>
__global__ __launch_bounds__(G1_T) void g1_fwd_bn_kernel(const float* __restrict__ z,
                                                         const float* __restrict__ w, int Cout,
                                                         const float* __restrict__ gamma,
                                                         const float* __restrict__ beta, float eps, float momentum,
                                                         float* running_mean, float* running_var, long long* nbt,
                                                         int act, float alpha, float* __restrict__ y,
                                                         float* __restrict__ a, float* __restrict__ stats) {
  constexpr int R = B / 4;                // batch rows per thread: 4 j + q, j < R
  constexpr int ZS = Cin + 4;             // z row stride in LDS: the 4 groups' rows (consecutive
                                          // b) sit 16 B apart mod 256 -- conflict-free b128 reads
  extern __shared__ float lds[];
  float* zs = lds;                        // [B][ZS]
  float* ys = lds + (size_t)B * ZS;       // [32][16 taps][G1_CB channels]: output staging
  __shared__ float alv[G1_CB], bev[G1_CB];
  const int tid = threadIdx.x, c_l = tid >> 6, q = (tid >> 4) & 3, t_l = tid & 15;
  const int co0 = blockIdx.x * G1_CB, co = co0 + c_l;
  for (int i = tid; i < B * Cin; i += G1_T) zs[(i / Cin) * ZS + i % Cin] = z[i];
  __syncthreads();
  const float* wp = w + (size_t)co * 16 + t_l;  // W[ci][co][t]: the 16 taps contiguous
  const size_t wstride = (size_t)Cout * 16;
  float acc[R];
#pragma unroll
  for (int j = 0; j < R; ++j) acc[j] = 0.f;
#pragma unroll
  for (int c0 = 0; c0 < Cin; c0 += G1_WCH) {
    // the next G1_WCH entries of the column in flight together (one latency per chunk)
    float wv[G1_WCH];
#pragma unroll
    for (int k = 0; k < G1_WCH; ++k) wv[k] = wp[(size_t)(c0 + k) * wstride];
#pragma unroll
    for (int k = 0; k < G1_WCH; k += 4) {
#pragma unroll
      for (int j = 0; j < R; ++j) {  // ci in order per output
        const float4 zz = *reinterpret_cast<const float4*>(zs + (4 * j + q) * ZS + c0 + k);
        acc[j] = fmaf(zz.w, wv[k + 3], fmaf(zz.z, wv[k + 2], fmaf(zz.y, wv[k + 1], fmaf(zz.x, wv[k], acc[j]))));
      }
    }
  }
  // channel statistics, exact two-pass in double over the wave (fixed xor-butterfly)
  double s1 = 0.0;
#pragma unroll
  for (int j = 0; j < R; ++j) s1 += (double)acc[j];
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) s1 += __shfl_xor(s1, o);
  const double n = (double)B * 16.0, mean = s1 / n;
  double s2 = 0.0;
#pragma unroll
  for (int j = 0; j < R; ++j) {
    const double d = (double)acc[j] - mean;
    s2 += d * d;
  }
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) s2 += __shfl_xor(s2, o);
  const double var = s2 / n;
  const float st_mean = (float)mean, st_inv = (float)(1.0 / sqrt(var + (double)eps));
  if ((tid & 63) == 0) {
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
  // y and a NHWC, 32 rows at a time through LDS: out thread = (row, tap, channel) with the
  // channel fastest (G1_CB-channel runs)
  const int wc = tid % G1_CB, wt = (tid / G1_CB) & 15, wr = tid / (16 * G1_CB);
  constexpr int WROWS = G1_T / (16 * G1_CB);  // rows per pass
#pragma unroll
  for (int h = 0; h < B / 32; ++h) {  // rows 32 h .. 32 h + 31: those of groups 4 h / (B / 32) ...
    __syncthreads();  // alv / bev written; the previous chunk's reads done
#pragma unroll
    for (int j = 0; j < R; ++j) {
      const int b = 4 * j + q;
      if (b >= 32 * h && b < 32 * h + 32) ys[((b - 32 * h) * 16 + t_l) * G1_CB + c_l] = acc[j];
    }
    __syncthreads();
    const float al = alv[wc], be = bev[wc];
#pragma unroll
    for (int i = 0; i < 32 / WROWS; ++i) {
      const int b = wr + WROWS * i;
      const float v = ys[(b * 16 + wt) * G1_CB + wc];
      const size_t o = ((size_t)(32 * h + b) * 16 + wt) * Cout + co0 + wc;
      y[o] = v;
      a[o] = act_fwd(v * al + be, act, alpha);
    }
  }
}

// thread = (channel c_l, ci group q, tap t): the group's Cin/4 outputs dW[ci][co][t] in
// registers (ci quads q, q + 4, q + 8, ...: the 4 groups read adjacent float4 of a z row, no
// bank conflict), b in order (each output's sum as the GEMM's K loop)
template <int B, int Cin>
__global__ __launch_bounds__(G1_T) void g1_wgrad_kernel(const float* __restrict__ z, const float* __restrict__ dy,
                                                        int Cout, float* dw, int accumulate) {
  constexpr int NQ = Cin / 16;  // ci quads per group
  __shared__ __attribute__((aligned(16))) float zs[B * Cin];
  const int tid = threadIdx.x, c_l = tid >> 6, q = (tid >> 4) & 3, t_l = tid & 15;
  const int co = blockIdx.x * G1_CB + c_l;
  for (int i = tid; i < B * Cin; i += G1_T) zs[i] = z[i];
  __syncthreads();
  const float* gp = dy + (size_t)t_l * Cout + co;  // dy[b][t][co], b stride 16 Cout
  float s[NQ][4];
#pragma unroll
  for (int k = 0; k < NQ; ++k)
#pragma unroll
    for (int i = 0; i < 4; ++i) s[k][i] = 0.f;
#pragma unroll 2
  for (int b = 0; b < B; ++b) {
    const float gb = gp[(size_t)b * 16 * Cout];
    const float* zr = zs + b * Cin + 4 * q;
#pragma unroll
    for (int k = 0; k < NQ; ++k) {
      const float4 zz = *reinterpret_cast<const float4*>(zr + 16 * k);
      s[k][0] = fmaf(zz.x, gb, s[k][0]);
      s[k][1] = fmaf(zz.y, gb, s[k][1]);
      s[k][2] = fmaf(zz.z, gb, s[k][2]);
      s[k][3] = fmaf(zz.w, gb, s[k][3]);
    }
  }
  float* wp = dw + (size_t)co * 16 + t_l;
  const size_t wstride = (size_t)Cout * 16;
#pragma unroll
  for (int k = 0; k < NQ; ++k)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      float* d = wp + (size_t)(16 * k + 4 * q + i) * wstride;
      *d = accumulate ? *d + s[k][i] : s[k][i];
    }
}

}  // namespace rgan

using namespace rgan;

template <int B, int Cin>
static void g1_fwd_launch(int Cout, const float* z, const float* w, const float* gamma, const float* beta, float eps,
                          float momentum, float* rm, float* rv, long long* nbt, int act, float alpha, float* y,
                          float* a, float* stats, hipStream_t s) {
  const size_t lds = ((size_t)B * (Cin + 4) + 32 * 16 * G1_CB) * sizeof(float);
  g1_fwd_bn_kernel<B, Cin><<<Cout / G1_CB, G1_T, lds, s>>>(z, w, Cout, gamma, beta, eps, momentum, rm, rv, nbt, act,
                                                           alpha, y, a, stats);
}

extern "C" int rgan_g1_fwd_bn(const float* z, int B, int Cin, const float* w, int Cout, const float* gamma,
                              const float* beta, float eps, float momentum, float* running_mean, float* running_var,
                              long long* num_batches_tracked, int act, float act_alpha, float* y, float* a,
                              float* stats, void* stream) {
  RGAN_REQUIRE(act_ok(act));
  RGAN_REQUIRE(z && w && y && a && stats && (B == 32 || B == 64) && (Cin == 64 || Cin == 128) &&
               Cout >= G1_CB && Cout % G1_CB == 0 && ((uintptr_t)z & 15) == 0);
  const hipStream_t s = (hipStream_t)stream;
#define RGAN_G1F(BB, CC)                                                                                     \
  g1_fwd_launch<BB, CC>(Cout, z, w, gamma, beta, eps, momentum, running_mean, running_var, num_batches_tracked, \
                        act, act_alpha, y, a, stats, s)
  if (B == 32) { if (Cin == 64) RGAN_G1F(32, 64); else RGAN_G1F(32, 128); }
  else { if (Cin == 64) RGAN_G1F(64, 64); else RGAN_G1F(64, 128); }
#undef RGAN_G1F
  RGAN_CHECK_LAUNCH();
  return 0;
}

extern "C" int rgan_g1_wgrad(const float* z, int B, int Cin, const float* dy, int Cout, float* dw, int accumulate,
                             void* stream) {
  RGAN_REQUIRE(z && dy && dw && (B == 32 || B == 64) && (Cin == 64 || Cin == 128) && Cout >= G1_CB &&
               Cout % G1_CB == 0 && ((uintptr_t)z & 15) == 0);
  const hipStream_t s = (hipStream_t)stream;
  const dim3 grid(Cout / G1_CB);
  if (B == 32 && Cin == 64) g1_wgrad_kernel<32, 64><<<grid, G1_T, 0, s>>>(z, dy, Cout, dw, accumulate);
  else if (B == 32) g1_wgrad_kernel<32, 128><<<grid, G1_T, 0, s>>>(z, dy, Cout, dw, accumulate);
  else if (Cin == 64) g1_wgrad_kernel<64, 64><<<grid, G1_T, 0, s>>>(z, dy, Cout, dw, accumulate);
  else g1_wgrad_kernel<64, 128><<<grid, G1_T, 0, s>>>(z, dy, Cout, dw, accumulate);
  RGAN_CHECK_LAUNCH();
  return 0;
}
