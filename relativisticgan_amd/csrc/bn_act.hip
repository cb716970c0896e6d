// BatchNorm2d (train mode) + activation kernels, NHWC ([P][C] with strides).
//
// Replaces torch.nn.BatchNorm2d forward/backward in training mode and the activation
// modules that follow it (GLI:341-345,366-370,433-437; arch 1 GLI:204-218,262-297).
// Statistics: per (pixel-chunk, channel) Welford partials merged by Chan's formula in a
// fixed order -> deterministic and free of the E[x^2]-E[x]^2 cancellation.
// HBM-bound: algorithmic bytes per element are 4 (stats read) + 8 (apply read+write)
// forward and 8 (reduce: da, y) + 12 (apply: da, y read, dy write) backward.
#include "common.h"

namespace rgan {

constexpr int BN_CG = 64;     // channels per block (one lane per channel)
constexpr int BN_ROWS = 4;    // waves per block, each walks its own pixel rows

static int bn_chunks(long long P, int C) {
  // aim for ~1024 blocks total, at least 64 pixels per chunk
  const int cgroups = ceil_div(C, BN_CG);
  long long want = std::max<long long>(1, 1024 / cgroups);
  long long per = std::max<long long>(64, (P + want - 1) / want);
  return ceil_div(P, per);
}

extern "C" size_t rgan_bn_partial_bytes(long long P, int C) {
  return ((size_t)bn_chunks(P, C) * 3 + 3) * C * sizeof(float) + 256;
}

// partial layout: [chunk][3][C] = (count, mean, M2)
__global__ __launch_bounds__(256) void bn_stats_partial(const float* __restrict__ y, long long P, int C,
                                                        long long sp, long long sc, int chunks,
                                                        float* __restrict__ part) {
  __shared__ float sh[3][BN_ROWS][BN_CG];
  const int lane = threadIdx.x & 63, row = threadIdx.x >> 6;
  const int c = blockIdx.y * BN_CG + lane;
  const int chunk = blockIdx.x;
  const long long per = (P + chunks - 1) / chunks;
  const long long p0 = chunk * per, p1 = min(P, p0 + per);
  float n = 0.f, mean = 0.f, m2 = 0.f;
  if (c < C) {
    for (long long p = p0 + row; p < p1; p += BN_ROWS) {
      const float v = y[p * sp + c * sc];
      n += 1.f;
      const float d = v - mean;
      mean += d / n;
      m2 += d * (v - mean);
    }
  }
  sh[0][row][lane] = n; sh[1][row][lane] = mean; sh[2][row][lane] = m2;
  __syncthreads();
  if (row == 0 && c < C) {
    float N = sh[0][0][lane], M = sh[1][0][lane], S = sh[2][0][lane];
    for (int r = 1; r < BN_ROWS; ++r) {
      const float nb = sh[0][r][lane];
      if (nb == 0.f) continue;
      const float mb = sh[1][r][lane], sb = sh[2][r][lane];
      const float nt = N + nb, d = mb - M;
      M += d * (nb / nt);
      S += sb + d * d * (N * nb / nt);
      N = nt;
    }
    part[((size_t)chunk * 3 + 0) * C + c] = N;
    part[((size_t)chunk * 3 + 1) * C + c] = M;
    part[((size_t)chunk * 3 + 2) * C + c] = S;
  }
}

// chunk partials -> per-channel moments (count, mean, M2) of this rank's batch
__global__ void bn_moments_reduce(const float* __restrict__ part, int chunks, int C, float* __restrict__ mom) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  double N = 0.0, M = 0.0, S = 0.0;
  for (int k = 0; k < chunks; ++k) {
    const double nb = part[((size_t)k * 3 + 0) * C + c];
    if (nb == 0.0) continue;
    const double mb = part[((size_t)k * 3 + 1) * C + c], sb = part[((size_t)k * 3 + 2) * C + c];
    const double nt = N + nb, d = mb - M;
    M += d * (nb / nt);
    S += sb + d * d * (N * nb / nt);
    N = nt;
  }
  mom[c] = (float)N;
  mom[C + c] = (float)M;
  mom[2 * C + c] = (float)S;
}

// merge `nranks` moment blocks [r][3][C] in rank order -> (mean, invstd), running stats
__global__ void bn_finalize_kernel(const float* __restrict__ mom, int nranks, int C, float eps, float momentum,
                                   float* running_mean, float* running_var, long long* nbt, float* stats) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c == 0 && nbt) nbt[0] += 1;
  if (c >= C) return;
  double N = 0.0, M = 0.0, S = 0.0;
  for (int k = 0; k < nranks; ++k) {
    const double nb = mom[((size_t)k * 3 + 0) * C + c];
    if (nb == 0.0) continue;
    const double mb = mom[((size_t)k * 3 + 1) * C + c], sb = mom[((size_t)k * 3 + 2) * C + c];
    const double nt = N + nb, d = mb - M;
    M += d * (nb / nt);
    S += sb + d * d * (N * nb / nt);
    N = nt;
  }
  const float mean = (float)M;
  const float var = (float)(S / N);
  stats[c] = mean;
  stats[C + c] = 1.f / sqrtf(var + eps);
  if (running_mean) running_mean[c] = (1.f - momentum) * running_mean[c] + momentum * mean;
  if (running_var) {
    const float unb = N > 1.0 ? (float)(S / (N - 1.0)) : var;
    running_var[c] = (1.f - momentum) * running_var[c] + momentum * unb;
  }
}

extern "C" int rgan_bn_moments(const float* y, long long P, int C, long long sp, long long sc, float* moments,
                               void* partial, void* stream) {
  RGAN_REQUIRE(y && moments && partial && P > 0 && C > 0);
  hipStream_t s = (hipStream_t)stream;
  const int chunks = bn_chunks(P, C);
  float* part = (float*)partial;
  bn_stats_partial<<<dim3(chunks, ceil_div(C, BN_CG)), 256, 0, s>>>(y, P, C, sp, sc, chunks, part);
  RGAN_CHECK_LAUNCH();
  bn_moments_reduce<<<ceil_div(C, 256), 256, 0, s>>>(part, chunks, C, moments);
  RGAN_CHECK_LAUNCH();
  return 0;
}

extern "C" int rgan_bn_finalize(const float* moments, int nranks, int C, float eps, float momentum,
                                float* running_mean, float* running_var, long long* num_batches_tracked,
                                float* stats, void* stream) {
  RGAN_REQUIRE(moments && stats && nranks > 0 && C > 0);
  bn_finalize_kernel<<<ceil_div(C, 256), 256, 0, (hipStream_t)stream>>>(moments, nranks, C, eps, momentum,
                                                                        running_mean, running_var,
                                                                        num_batches_tracked, stats);
  RGAN_CHECK_LAUNCH();
  return 0;
}

extern "C" int rgan_bn_stats(const float* y, long long P, int C, long long sp, long long sc, float eps,
                             float momentum, float* running_mean, float* running_var,
                             long long* num_batches_tracked, float* stats, void* partial, void* stream) {
  RGAN_REQUIRE(y && stats && partial && P > 0 && C > 0);
  const int chunks = bn_chunks(P, C);
  float* mom = (float*)partial + (size_t)chunks * 3 * C;
  int rc = rgan_bn_moments(y, P, C, sp, sc, mom, partial, stream);
  if (rc) return rc;
  return rgan_bn_finalize(mom, 1, C, eps, momentum, running_mean, running_var, num_batches_tracked, stats,
                          stream);
}

// a = act(y*alpha_c + beta_c), alpha_c = gamma*invstd, beta_c = beta - mean*alpha_c
__global__ __launch_bounds__(256) void bn_apply_kernel(const float* __restrict__ y, long long P, int C,
                                                       long long sp, long long sc,
                                                       const float* __restrict__ stats,
                                                       const float* __restrict__ gamma,
                                                       const float* __restrict__ beta, int act,
                                                       float alpha, float* __restrict__ a, long long asp,
                                                       long long asc) {
  const long long total = P * C;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const long long p = i / C;
    const int c = (int)(i - p * C);
    const float al = (gamma ? gamma[c] : 1.f) * stats[C + c];
    const float be = (beta ? beta[c] : 0.f) - stats[c] * al;
    a[p * asp + c * asc] = act_fwd(y[p * sp + c * sc] * al + be, act, alpha);
  }
}

// vectorised NHWC form (sc == asc == 1, sp == asp == C, C % 4 == 0)
__global__ __launch_bounds__(256) void bn_apply_vec(const float4* __restrict__ y, long long n4, int C,
                                                    const float* __restrict__ stats,
                                                    const float* __restrict__ gamma,
                                                    const float* __restrict__ beta, int act, float alpha,
                                                    float4* __restrict__ a) {
  const int C4 = C >> 2;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n4;
       i += (long long)gridDim.x * blockDim.x) {
    const int c = (int)(i % C4) * 4;
    float4 v = y[i];
    float r[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float al = (gamma ? gamma[c + j] : 1.f) * stats[C + c + j];
      const float be = (beta ? beta[c + j] : 0.f) - stats[c + j] * al;
      r[j] = act_fwd(r[j] * al + be, act, alpha);
    }
    a[i] = make_float4(r[0], r[1], r[2], r[3]);
  }
}

static int grid_for(long long n, int per_thread = 1) {
  long long b = (n / per_thread + 255) / 256;
  return (int)std::max<long long>(1, std::min<long long>(b, 8192));
}

extern "C" int rgan_bn_apply(const float* y, long long P, int C, long long sp, long long sc,
                             const float* stats, const float* gamma, const float* beta, int act,
                             float act_alpha, float* a, long long asp, long long asc, void* stream) {
  RGAN_REQUIRE(y && stats && a && P > 0 && C > 0);
  hipStream_t s = (hipStream_t)stream;
  const bool vec = sc == 1 && asc == 1 && sp == C && asp == C && C % 4 == 0 &&
                   ((uintptr_t)y & 15) == 0 && ((uintptr_t)a & 15) == 0;
  if (vec) {
    const long long n4 = P * C / 4;
    bn_apply_vec<<<grid_for(n4), 256, 0, s>>>((const float4*)y, n4, C, stats, gamma, beta, act, act_alpha,
                                             (float4*)a);
  } else {
    bn_apply_kernel<<<grid_for(P * C), 256, 0, s>>>(y, P, C, sp, sc, stats, gamma, beta, act, act_alpha, a,
                                                   asp, asc);
  }
  RGAN_CHECK_LAUNCH();
  return 0;
}

// backward reduce: per (chunk, channel) sum g and sum g*(y-mean), g = da * act'(z)
__global__ __launch_bounds__(256) void bn_bwd_partial(const float* __restrict__ da, long long dsp,
                                                      long long dsc, const float* __restrict__ y,
                                                      long long P, int C, long long sp, long long sc,
                                                      const float* __restrict__ stats,
                                                      const float* __restrict__ gamma,
                                                      const float* __restrict__ beta, int act, float alpha,
                                                      int chunks, float* __restrict__ part) {
  __shared__ float sh[2][BN_ROWS][BN_CG];
  const int lane = threadIdx.x & 63, row = threadIdx.x >> 6;
  const int c = blockIdx.y * BN_CG + lane;
  const int chunk = blockIdx.x;
  const long long per = (P + chunks - 1) / chunks;
  const long long p0 = chunk * per, p1 = min(P, p0 + per);
  float s1 = 0.f, s2 = 0.f;
  if (c < C) {
    const float mean = stats[c], inv = stats[C + c];
    const float al = (gamma ? gamma[c] : 1.f) * inv;
    const float be = (beta ? beta[c] : 0.f) - mean * al;
    for (long long p = p0 + row; p < p1; p += BN_ROWS) {
      const float v = y[p * sp + c * sc];
      const float gz = da[p * dsp + c * dsc] * act_grad_from_in(v * al + be, act, alpha);
      s1 += gz;
      s2 += gz * (v - mean);
    }
  }
  sh[0][row][lane] = s1; sh[1][row][lane] = s2;
  __syncthreads();
  if (row == 0 && c < C) {
    float a1 = 0.f, a2 = 0.f;
    for (int r = 0; r < BN_ROWS; ++r) { a1 += sh[0][r][lane]; a2 += sh[1][r][lane]; }
    part[((size_t)chunk * 2 + 0) * C + c] = a1;
    part[((size_t)chunk * 2 + 1) * C + c] = a2;
  }
}

// chunk partials -> this rank's per-channel (sum g, sum g*(y-mean)) = sums[2][C]
__global__ void bn_bwd_sums_reduce(const float* __restrict__ part, int chunks, int C, float* __restrict__ sums) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  double a1 = 0.0, a2 = 0.0;
  for (int k = 0; k < chunks; ++k) {
    a1 += part[((size_t)k * 2 + 0) * C + c];
    a2 += part[((size_t)k * 2 + 1) * C + c];
  }
  sums[c] = (float)a1;
  sums[C + c] = (float)a2;
}

// dy = al*(g - sum_g/Pg - (y-mean)*invstd^2*sum_gx/Pg); dgamma = invstd*sum_gx, dbeta = sum_g
__global__ __launch_bounds__(256) void bn_bwd_apply(const float* __restrict__ da, long long dsp,
                                                    long long dsc, const float* __restrict__ y, long long P,
                                                    int C, long long sp, long long sc,
                                                    const float* __restrict__ stats,
                                                    const float* __restrict__ gamma,
                                                    const float* __restrict__ beta, int act, float alpha,
                                                    const float* __restrict__ sums, float inv_pg,
                                                    float* __restrict__ dy, long long ysp, long long ysc,
                                                    float* dgamma, float* dbeta) {
  const long long total = P * C;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const long long p = i / C;
    const int c = (int)(i - p * C);
    const float mean = stats[c], inv = stats[C + c];
    const float al = (gamma ? gamma[c] : 1.f) * inv;
    const float be = (beta ? beta[c] : 0.f) - mean * al;
    const float k1 = sums[c] * inv_pg, k2 = sums[C + c] * inv * inv * inv_pg;
    const float v = y[p * sp + c * sc];
    const float gz = da[p * dsp + c * dsc] * act_grad_from_in(v * al + be, act, alpha);
    dy[p * ysp + c * ysc] = al * (gz - k1 - (v - mean) * k2);
    if (p == 0) {
      if (dbeta) dbeta[c] = sums[c];
      if (dgamma) dgamma[c] = sums[C + c] * inv;
    }
  }
}

extern "C" int rgan_bn_backward_sums(const float* da, long long dsp, long long dsc, const float* y, long long P,
                                     int C, long long sp, long long sc, const float* stats, const float* gamma,
                                     const float* beta, int act, float act_alpha, float* sums, void* partial,
                                     void* stream) {
  RGAN_REQUIRE(da && y && stats && sums && partial && P > 0 && C > 0);
  hipStream_t s = (hipStream_t)stream;
  const int chunks = bn_chunks(P, C);
  float* part = (float*)partial;
  bn_bwd_partial<<<dim3(chunks, ceil_div(C, BN_CG)), 256, 0, s>>>(da, dsp, dsc, y, P, C, sp, sc, stats,
                                                                   gamma, beta, act, act_alpha, chunks, part);
  RGAN_CHECK_LAUNCH();
  bn_bwd_sums_reduce<<<ceil_div(C, 256), 256, 0, s>>>(part, chunks, C, sums);
  RGAN_CHECK_LAUNCH();
  return 0;
}

extern "C" int rgan_bn_backward_apply(const float* da, long long dsp, long long dsc, const float* y, long long P,
                                      int C, long long sp, long long sc, const float* stats, const float* gamma,
                                      const float* beta, int act, float act_alpha, const float* sums,
                                      long long P_global, float* dy, long long ysp, long long ysc, float* dgamma,
                                      float* dbeta, void* stream) {
  RGAN_REQUIRE(da && y && stats && sums && dy && P > 0 && C > 0 && P_global >= P);
  bn_bwd_apply<<<grid_for(P * C), 256, 0, (hipStream_t)stream>>>(da, dsp, dsc, y, P, C, sp, sc, stats, gamma,
                                                                 beta, act, act_alpha, sums,
                                                                 1.f / (float)P_global, dy, ysp, ysc, dgamma,
                                                                 dbeta);
  RGAN_CHECK_LAUNCH();
  return 0;
}

extern "C" int rgan_bn_backward(const float* da, long long dsp, long long dsc, const float* y, long long P,
                                int C, long long sp, long long sc, const float* stats, const float* gamma,
                                const float* beta, int act, float act_alpha, float* dy, long long ysp,
                                long long ysc, float* dgamma, float* dbeta, void* partial, void* stream) {
  RGAN_REQUIRE(partial);
  const int chunks = bn_chunks(P, C);
  float* sums = (float*)partial + (size_t)chunks * 2 * C;
  int rc = rgan_bn_backward_sums(da, dsp, dsc, y, P, C, sp, sc, stats, gamma, beta, act, act_alpha, sums,
                                 partial, stream);
  if (rc) return rc;
  return rgan_bn_backward_apply(da, dsp, dsc, y, P, C, sp, sc, stats, gamma, beta, act, act_alpha, sums, P,
                                dy, ysp, ysc, dgamma, dbeta, stream);
}

// ------------------------------------------------------------------ activations
__global__ void act_bwd_kernel(const float* __restrict__ da, const float* __restrict__ a, long long n, int act,
                               float alpha, float* __restrict__ dx) {
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n;
       i += (long long)gridDim.x * blockDim.x)
    dx[i] = da[i] * act_grad_from_out(a[i], act, alpha);
}

extern "C" int rgan_act_backward(const float* da, const float* a, long long n, int act, float act_alpha,
                                 float* dx, void* stream) {
  RGAN_REQUIRE(da && a && dx && n >= 0);
  if (n == 0) return 0;
  act_bwd_kernel<<<grid_for(n), 256, 0, (hipStream_t)stream>>>(da, a, n, act, act_alpha, dx);
  RGAN_CHECK_LAUNCH();
  return 0;
}

// per-channel sum over pixels (bias gradients); one block per 64 channels, fixed order
__global__ __launch_bounds__(256) void channel_sum_kernel(const float* __restrict__ t, long long P, int C,
                                                          long long sp, long long sc, float* __restrict__ out) {
  __shared__ float sh[BN_ROWS][BN_CG];
  const int lane = threadIdx.x & 63, row = threadIdx.x >> 6;
  const int c = blockIdx.x * BN_CG + lane;
  float s = 0.f;
  if (c < C)
    for (long long p = row; p < P; p += BN_ROWS) s += t[p * sp + c * sc];
  sh[row][lane] = s;
  __syncthreads();
  if (row == 0 && c < C) out[c] = sh[0][lane] + sh[1][lane] + sh[2][lane] + sh[3][lane];
}

extern "C" int rgan_channel_sum(const float* t, long long P, int C, long long sp, long long sc, float* out,
                                void* partial, void* stream) {
  (void)partial;
  RGAN_REQUIRE(t && out && P > 0 && C > 0);
  channel_sum_kernel<<<ceil_div(C, BN_CG), 256, 0, (hipStream_t)stream>>>(t, P, C, sp, sc, out);
  RGAN_CHECK_LAUNCH();
  return 0;
}

}  // namespace rgan
