// Shared device helpers for the gfx950 kernels (wave64, CDNA4).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "../../include/rgan.h"

#define RGAN_CHECK_LAUNCH()                         \
  do {                                              \
    hipError_t _e = hipGetLastError();              \
    if (_e != hipSuccess) return (int)_e;           \
  } while (0)

// host-side check of an RGAN_ACT_* code passed through the C-ABI
static inline bool act_ok(int act) { return act >= RGAN_ACT_NONE && act <= RGAN_ACT_SELU; }

#define RGAN_REQUIRE(cond)                          \
  do {                                              \
    if (!(cond)) return RGAN_EINVAL;                \
  } while (0)

namespace rgan {

constexpr int WAVE = 64;

// The transcendental activations (tanh, sigmoid, SELU) behind a call: the piecewise-linear
// ones the hot epilogues run (none, ReLU, LeakyReLU) are one select, and a per-element
// inlined six-way switch with expf/tanhf bodies no longer bloats every unrolled epilogue
// (it cost the image-layer conv ~10k issue cycles per tile).
__device__ __noinline__ float act_fwd_curved(float v, int act, float alpha);

// Bare v_max_f32 / v_min_f32: fmaxf's IEEE semantics make the compiler canonicalize both
// inputs first (two extra VALU per call); the epilogue values here are never sNaN.
__device__ __forceinline__ float vmaxf(float a, float b) {
  float r;
  asm("v_max_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
__device__ __forceinline__ float vminf(float a, float b) {
  float r;
  asm("v_min_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}

__device__ __forceinline__ float act_fwd(float v, int act, float alpha) {
  if (act <= RGAN_ACT_LRELU) {
    const float neg = act == RGAN_ACT_NONE ? 1.f : (act == RGAN_ACT_RELU ? 0.f : alpha);
    return v > 0.f ? v : v * neg;
  }
  return act_fwd_curved(v, act, alpha);
}

__device__ __noinline__ float act_fwd_curved(float v, int act, float alpha) {
  switch (act) {
    case RGAN_ACT_RELU: return v > 0.f ? v : 0.f;
    case RGAN_ACT_LRELU: return v > 0.f ? v : v * alpha;
    case RGAN_ACT_TANH: return tanhf(v);
    case RGAN_ACT_SIGMOID: return 1.f / (1.f + expf(-v));
    case RGAN_ACT_SELU: {
      const float scale = 1.0507009873554804934193349852946f;
      const float a = 1.6732632423543772848170429916717f;
      return v > 0.f ? scale * v : scale * (a * expm1f(v));
    }
    default: return v;
  }
}

// derivative of act expressed through the activation OUTPUT a = act(x)
__device__ __forceinline__ float act_grad_from_out(float a, int act, float alpha) {
  switch (act) {
    case RGAN_ACT_RELU: return a > 0.f ? 1.f : 0.f;
    case RGAN_ACT_LRELU: return a > 0.f ? 1.f : alpha;
    case RGAN_ACT_TANH: return 1.f - a * a;
    case RGAN_ACT_SIGMOID: return a * (1.f - a);
    case RGAN_ACT_SELU: {
      const float scale = 1.0507009873554804934193349852946f;
      const float sa = 1.7580993408473768599402175208123f;  // scale * alpha
      return a > 0.f ? scale : a + sa;
    }
    default: return 1.f;
  }
}

// derivative of act expressed through the activation INPUT x
__device__ __forceinline__ float act_grad_from_in(float x, int act, float alpha) {
  switch (act) {
    case RGAN_ACT_RELU: return x > 0.f ? 1.f : 0.f;
    case RGAN_ACT_LRELU: return x > 0.f ? 1.f : alpha;
    case RGAN_ACT_TANH: { float t = tanhf(x); return 1.f - t * t; }
    case RGAN_ACT_SIGMOID: { float s = 1.f / (1.f + expf(-x)); return s * (1.f - s); }
    case RGAN_ACT_SELU: {
      const float scale = 1.0507009873554804934193349852946f;
      const float sa = 1.7580993408473768599402175208123f;
      return x > 0.f ? scale : sa * expf(x);
    }
    default: return 1.f;
  }
}

// second derivative of act through its INPUT x (0 for the piecewise-linear ReLU/LeakyReLU):
// the WGAN-GP double backward differentiates act' itself
__device__ __forceinline__ float act_grad2_from_in(float x, int act, float alpha) {
  (void)alpha;
  switch (act) {
    case RGAN_ACT_TANH: { float t = tanhf(x); return -2.f * t * (1.f - t * t); }
    case RGAN_ACT_SIGMOID: { float s = 1.f / (1.f + expf(-x)); return s * (1.f - s) * (1.f - 2.f * s); }
    case RGAN_ACT_SELU: {
      const float sa = 1.7580993408473768599402175208123f;
      return x > 0.f ? 0.f : sa * expf(x);
    }
    default: return 0.f;
  }
}

// the same through the OUTPUT a = act(x)
__device__ __forceinline__ float act_grad2_from_out(float a, int act, float alpha) {
  (void)alpha;
  switch (act) {
    case RGAN_ACT_TANH: return -2.f * a * (1.f - a * a);
    case RGAN_ACT_SIGMOID: return a * (1.f - a) * (1.f - 2.f * a);
    case RGAN_ACT_SELU: {
      const float sa = 1.7580993408473768599402175208123f;
      return a > 0.f ? 0.f : a + sa;
    }
    default: return 0.f;
  }
}

__host__ __device__ inline bool act_has_grad2(int act) {
  return act == RGAN_ACT_TANH || act == RGAN_ACT_SIGMOID || act == RGAN_ACT_SELU;
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// Block-wide sum (blockDim.x multiple of 64, <= 1024).  `red` >= 16 floats of LDS.
// Result valid in every thread.  Fixed order: deterministic.
__device__ __forceinline__ float block_sum(float v, float* red) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  v = wave_sum(v);
  __syncthreads();
  if (lane == 0) red[wid] = v;
  __syncthreads();
  float t = 0.f;
  for (int i = 0; i < nw; ++i) t += red[i];
  return t;
}

__device__ __forceinline__ double block_sum_d(double v, double* red) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  v = wave_sum_d(v);
  __syncthreads();
  if (lane == 0) red[wid] = v;
  __syncthreads();
  double t = 0.0;
  for (int i = 0; i < nw; ++i) t += red[i];
  return t;
}

inline int ceil_div(long long a, long long b) { return (int)((a + b - 1) / b); }

// ---- Adam (torch/optim/adam.py _single_tensor_adam, the reference's optimizer GLI:529-530):
// the per-step constants in double (torch computes them in Python floats), the update in fp32
// with torch's operation order (lerp for m; v * b2 + (1 - b2) g^2; sqrt(v) / sqrt(bc2) + eps)
struct AdamConst {
  float neg_step, bc2s, w, fb2, f1mb2, feps, fwd;
  bool has_wd;
};

// hyper = {lr, beta1, beta2, eps, weight_decay}; step = the step being taken (>= 1)
__device__ __forceinline__ AdamConst adam_const(const double* hyper, const float* step) {
  const double lr = hyper[0], b1 = hyper[1], b2 = hyper[2], eps = hyper[3], wd = hyper[4];
  const double st = (double)step[0];
  const double bc1 = 1.0 - pow(b1, st), bc2 = 1.0 - pow(b2, st);
  AdamConst k;
  k.neg_step = (float)(-(lr / bc1));
  k.bc2s = (float)sqrt(bc2);
  k.w = (float)(1.0 - b1);
  k.fb2 = (float)b2;
  k.f1mb2 = (float)(1.0 - b2);
  k.feps = (float)eps;
  k.fwd = (float)wd;
  k.has_wd = wd != 0.0;
  return k;
}

// Every rounding spelled out (explicit fmaf / _rn intrinsics: no contraction left to the
// compiler, so every kernel inlining this rounds alike), as torch's CPU kernels round:
// lerp = fma(w, end - m, m) or fma(w - 1, end - m, end) (ATen lerp_vec), addcmul =
// fma(value * g, g, v), addcdiv = p + (value * m) / denom (checked elementwise against
// torch.optim.Adam on the CPU).
__device__ __forceinline__ void adam_elem(const AdamConst& k, float g, float& p, float& m, float& v) {
  if (k.has_wd) g = fmaf(k.fwd, p, g);
  const float diff = __fsub_rn(g, m);
  m = k.w < 0.5f ? fmaf(k.w, diff, m) : fmaf(k.w - 1.f, diff, g);
  v = fmaf(__fmul_rn(k.f1mb2, g), g, __fmul_rn(v, k.fb2));
  const float denom = __fadd_rn(__fdiv_rn(__fsqrt_rn(v), k.bc2s), k.feps);
  p = __fadd_rn(p, __fdiv_rn(__fmul_rn(k.neg_step, m), denom));
}

}  // namespace rgan
