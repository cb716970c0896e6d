// BatchNorm2d (train mode) + activation kernels on NHWC activations ([P][C], P = B*H*W).
//
// Replaces torch.nn.BatchNorm2d forward/backward in training mode and the activation
// that follows it (GLI:341-345,366-370,433-437; arch 1 GLI:204-218,262-297).
//
// Numerics: per-thread sums are accumulated in double (torch's CPU kernel uses a double
// accumulator too): the backward sums sum(g) and sum(g*(y-mean)) can cancel almost
// completely when the upstream gradient lies near BN's null space, and a float sum
// there leaves a coherent per-channel offset in dy.  Forward moments use shifted sums
// (shift = the thread's first sample) in double; partials are merged with Chan's
// parallel formula in a fixed order (deterministic, no E[x^2]-E[x]^2 cancellation).
//
// Layout/perf: the vector path gives every thread a fixed quad of 4 channels (float4
// loads, no per-element index division) and walks pixels; HBM-bound with algorithmic
// bytes per element 4 (moments) + 8 (apply) forward, 8 (sums: da, y) + 12 (apply: da,
// y -> dy) backward.  Chunk partials are reduced by a parallel merge kernel.
#include "common.h"

#include <cstdlib>

namespace rgan {

// ------------------------------------------------------------------ geometry
struct BnGeo {
  bool vec;        // NHWC dense, C % 4 == 0
  int Q;           // channels per thread (4 or 1)
  int tpr;         // threads per pixel row (power of two)
  int rp;          // pixel rows in flight per block (256 / tpr)
  int cgroups;     // channel groups
  int chunks;      // pixel chunks
  long long rows;  // pixels per chunk
};

static int pow2_floor(int v) {
  int p = 1;
  while (p * 2 <= v) p *= 2;
  return p;
}

static BnGeo bn_geo(long long P, int C, long long sp, long long sc) {
  BnGeo g;
  g.vec = sc == 1 && sp == C && C % 4 == 0;
  g.Q = g.vec ? 4 : 1;
  const int cq = C / g.Q;
  int t = 1;
  if (g.vec) {
    while (t < 64 && cq % (t * 2) == 0) t *= 2;
  } else {
    t = std::min(64, pow2_floor(C));
  }
  g.tpr = t;
  g.rp = 256 / t;
  g.cgroups = ceil_div(cq, t);
  constexpr long long want_blocks = 512;  // round-1 sweep (tools/bn_micro.py)
  long long chunks = std::max<long long>(1, want_blocks / g.cgroups);
  long long rows = (P + chunks - 1) / chunks;
  rows = std::max<long long>(rows, (long long)g.rp * 4);
  g.rows = rows;
  g.chunks = ceil_div(P, rows);
  return g;
}

static int max_chunks(long long P, int C) {
  return std::max(bn_geo(P, C, C, 1).chunks, bn_geo(P, C, 1, 2).chunks);
}

extern "C" size_t rgan_bn_dd_partial_bytes(long long P, int C) {
  if (P <= 0 || C <= 0) return 0;  // no such layer
  return (size_t)max_chunks(P, C) * 3 * C * sizeof(double) + 256;
}

extern "C" size_t rgan_bn_partial_bytes(long long P, int C) {
  // [chunks][2][C] partial sums + [2][C] merged sums + [3][C] moments, doubles
  if (P <= 0 || C <= 0) return 0;  // no such layer
  return ((size_t)max_chunks(P, C) * 2 + 5) * C * sizeof(double) + 256;
}

// pixel rows whose loads each thread issues before consuming the first (bytes in flight)
constexpr int BN_UNR = 4;

template <int Q>
__device__ __forceinline__ void load_q(const float* __restrict__ y, long long off, float (&v)[Q]) {
  if constexpr (Q == 4) {
    const float4 t = *reinterpret_cast<const float4*>(y + off);
    v[0] = t.x; v[1] = t.y; v[2] = t.z; v[3] = t.w;
  } else {
    v[0] = y[off];
  }
}

__device__ __forceinline__ void chan_merge(double& N, double& M, double& S, double nb, double mb, double sb) {
  if (nb == 0.0) return;
  const double nt = N + nb, d = mb - M;
  M += d * (nb / nt);
  S += sb + d * d * (N * nb / nt);
  N = nt;
}

// ------------------------------------------------------------------ forward moments
// Shifted sums with ONE shift per channel (its first pixel, y[0][c]) shared by every
// block: partials are plain (sum d, sum d^2), d = y - shift, accumulated in double, so
// the merge is a division-free parallel sum.  partial layout: [chunk][2][C] doubles.
template <int Q>
__global__ __launch_bounds__(256) void bn_moments_partial(const float* __restrict__ y, long long P, int C,
                                                          long long sp, long long sc, int tpr, long long rows,
                                                          double* __restrict__ part) {
  __shared__ double sh[2][256][Q];
  const int tid = threadIdx.x, lc = tid % tpr, rl = tid / tpr, rp = blockDim.x / tpr;
  const int c0 = (blockIdx.y * tpr + lc) * Q;
  const long long p0 = blockIdx.x * rows, p1 = min(P, p0 + rows);
  double s1[Q], s2[Q];
  float sft[Q];
#pragma unroll
  for (int q = 0; q < Q; ++q) { s1[q] = 0.0; s2[q] = 0.0; sft[q] = 0.f; }
  if (c0 < C) {
    load_q<Q>(y, (long long)c0 * sc, sft);
    auto acc = [&](const float (&v)[Q]) {
#pragma unroll
      for (int q = 0; q < Q; ++q) {
        const double d = (double)(v[q] - sft[q]);
        s1[q] += d;
        s2[q] += d * d;
      }
    };
    long long p = p0 + rl;
    for (; p + (BN_UNR - 1) * rp < p1; p += BN_UNR * rp) {  // loads issued ahead, summed in p order
      float v[BN_UNR][Q];
#pragma unroll
      for (int u = 0; u < BN_UNR; ++u) load_q<Q>(y, (p + u * rp) * sp + (long long)c0 * sc, v[u]);
#pragma unroll
      for (int u = 0; u < BN_UNR; ++u) acc(v[u]);
    }
    for (; p < p1; p += rp) {
      float v[Q];
      load_q<Q>(y, p * sp + (long long)c0 * sc, v);
      acc(v);
    }
  }
#pragma unroll
  for (int q = 0; q < Q; ++q) { sh[0][tid][q] = s1[q]; sh[1][tid][q] = s2[q]; }
  __syncthreads();
  if (rl == 0 && c0 < C) {
#pragma unroll
    for (int q = 0; q < Q; ++q) {
      if (c0 + q < C) {
        double a1 = 0.0, a2 = 0.0;
        for (int r = 0; r < rp; ++r) { a1 += sh[0][r * tpr + lc][q]; a2 += sh[1][r * tpr + lc][q]; }
        part[((size_t)blockIdx.x * 2 + 0) * C + c0 + q] = a1;
        part[((size_t)blockIdx.x * 2 + 1) * C + c0 + q] = a2;
      }
    }
  }
}

// [k][2][C] partial sums -> per-channel totals in a fixed order (deterministic).  Block =
// 16 channels x 64 chunk lanes (1024 threads): each lane sums chunks r, r+64, ... and the
// 64 lane totals are added in lane order -- 8x the channel-parallelism of a 64-channel
// block, so the merge of C = 128 channels x 1024 chunks runs on 8 CUs, not 2.
//   FIN 0: sums[2][C] (backward: sum g, sum g*(y-mean))
//   FIN 1: moments [3][C] (count, mean, M2) of this rank (SyncBN stage 1)
//   FIN 2: one rank: (mean, invstd) stats + running-stat update, as bn_finalize_kernel
constexpr int MERGE_CPB = 16, MERGE_ROWS = 64;

template <int FIN>
__global__ __launch_bounds__(1024) void bn_merge(const double* __restrict__ part, int chunks, int C,
                                                 double* __restrict__ out, const float* __restrict__ y, long long P,
                                                 long long sc, float eps, float momentum, float* running_mean,
                                                 float* running_var, long long* nbt, float* stats) {
  __shared__ double sh[2][MERGE_ROWS][MERGE_CPB];
  if constexpr (FIN == 0) {  // gridDim.y segments: [seg][chunks][2][C] -> [seg][2][C]
    part += (size_t)blockIdx.y * chunks * 2 * C;
    out += (size_t)blockIdx.y * 2 * C;
  }
  const int cl = threadIdx.x % MERGE_CPB, r = threadIdx.x / MERGE_CPB;
  const int c = blockIdx.x * MERGE_CPB + cl;
  double a1 = 0.0, a2 = 0.0;
  if (c < C)
    for (int k = r; k < chunks; k += MERGE_ROWS) {
      a1 += part[((size_t)k * 2 + 0) * C + c];
      a2 += part[((size_t)k * 2 + 1) * C + c];
    }
  sh[0][r][cl] = a1;
  sh[1][r][cl] = a2;
  __syncthreads();
  if constexpr (FIN == 2) {
    if (blockIdx.x == 0 && threadIdx.x == 0 && nbt) nbt[0] += 1;
  }
  if (r != 0 || c >= C) return;
  double s1 = 0.0, s2 = 0.0;
  for (int q = 0; q < MERGE_ROWS; ++q) { s1 += sh[0][q][cl]; s2 += sh[1][q][cl]; }
  if constexpr (FIN == 0) {
    out[c] = s1;
    out[C + c] = s2;
  } else {
    // shifted sums (shift = y[0][c]) -> moments
    const double n = (double)P, mean = (double)y[(long long)c * sc] + s1 / n, m2 = fmax(s2 - s1 * s1 / n, 0.0);
    if constexpr (FIN == 1) {
      out[c] = n;
      out[C + c] = mean;
      out[2 * C + c] = m2;
    } else {
      const double var = m2 / n;
      stats[c] = (float)mean;
      stats[C + c] = (float)(1.0 / sqrt(var + (double)eps));
      if (running_mean) running_mean[c] = (1.f - momentum) * running_mean[c] + momentum * (float)mean;
      if (running_var) {
        const float unb = n > 1.0 ? (float)(m2 / (n - 1.0)) : (float)var;
        running_var[c] = (1.f - momentum) * running_var[c] + momentum * unb;
      }
    }
  }
}

// Segment sums written by the conv GEMM's epilogue (rgan_conv_fwd_bn): [S][2][C] = (sum y,
// sum y^2) of 64-row segments, in double -> moments of segments [s0, s1).  Block = 4
// channels x 256 lanes: lane r sums segments s0 + r, s0 + r + 256, ... (loads issued 4
// ahead), then a fixed-order LDS tree adds the 256 lane sums (deterministic).  Unshifted
// double sums: var = (S2 - S1^2/n)/n loses ~1e-16 * mean^2/var relative -- far inside fp32
// (the moments pass over y keeps its shifted sums; it has no segment structure to exploit).
//   FIN 1: moments [3][C] (count, mean, M2) (SyncBN stage 1)
//   FIN 2: (mean, invstd) stats + running-stat update, as bn_merge<2>
constexpr int SEG_CPB = 4, SEG_LANES = 256;

// NSEG > 1 (FIN 2): the batch segments [s0 + k L, s0 + (k+1) L), L = (s1 - s0) / NSEG, of
// the batched D pass, one after the other in one launch: stats[k][2C], running statistics
// updated in segment order (as NSEG separate calls would).
template <int FIN, int NSEG = 1>
__global__ __launch_bounds__(1024) void bn_seg_merge(const double* __restrict__ part, long long s0_all,
                                                     long long s1_all, int C, double seg_n, double* __restrict__ out,
                                                     float eps, float momentum, float* running_mean,
                                                     float* running_var, long long* nbt, float* stats) {
  __shared__ double sh[2][SEG_LANES][SEG_CPB];
  const int cl = threadIdx.x % SEG_CPB, r = threadIdx.x / SEG_CPB;
  const int c = blockIdx.x * SEG_CPB + cl;
  const long long seg_len = (s1_all - s0_all) / NSEG;
  for (int sg = 0; sg < NSEG; ++sg) {
  const long long s0 = s0_all + sg * seg_len, s1 = s0 + seg_len;
  if (sg > 0) __syncthreads();  // the previous segment's tree reads are done
  double a1 = 0.0, a2 = 0.0;
  if (c < C) {
    long long k = s0 + r;
    for (; k + 3 * SEG_LANES < s1; k += 4 * SEG_LANES) {
      double v[4][2];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        v[u][0] = part[((size_t)(k + u * SEG_LANES) * 2 + 0) * C + c];
        v[u][1] = part[((size_t)(k + u * SEG_LANES) * 2 + 1) * C + c];
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) { a1 += v[u][0]; a2 += v[u][1]; }
    }
    for (; k < s1; k += SEG_LANES) {
      a1 += part[((size_t)k * 2 + 0) * C + c];
      a2 += part[((size_t)k * 2 + 1) * C + c];
    }
  }
  sh[0][r][cl] = a1;
  sh[1][r][cl] = a2;
  __syncthreads();
  for (int h = SEG_LANES / 2; h > 0; h >>= 1) {
    if (r < h) {
      sh[0][r][cl] += sh[0][r + h][cl];
      sh[1][r][cl] += sh[1][r + h][cl];
    }
    __syncthreads();
  }
  if constexpr (FIN == 2) {
    if (blockIdx.x == 0 && threadIdx.x == 0 && nbt) nbt[0] += 1;
  }
  if (r == 0 && c < C) {
    const double n = seg_n * (double)(s1 - s0), S1 = sh[0][0][cl], S2 = sh[1][0][cl];
    const double mean = S1 / n, m2 = fmax(S2 - S1 * mean, 0.0);
    if constexpr (FIN == 1) {
      out[c] = n;
      out[C + c] = mean;
      out[2 * C + c] = m2;
    } else {
      const double var = m2 / n;
      float* st = stats + (size_t)sg * 2 * C;
      st[c] = (float)mean;
      st[C + c] = (float)(1.0 / sqrt(var + (double)eps));
      if (running_mean) running_mean[c] = (1.f - momentum) * running_mean[c] + momentum * (float)mean;
      if (running_var) {
        const float unb = n > 1.0 ? (float)(m2 / (n - 1.0)) : (float)var;
        running_var[c] = (1.f - momentum) * running_var[c] + momentum * unb;
      }
    }
  }
  }  // segments
}

extern "C" int rgan_bn_segment_stats_n(const double* part, long long s0, long long s1, int nseg, int C, int seg_rows,
                                       float eps, float momentum, float* running_mean, float* running_var,
                                       long long* num_batches_tracked, float* stats, void* stream) {
  RGAN_REQUIRE(part && s1 > s0 && s0 >= 0 && C > 0 && seg_rows > 0 && stats && (nseg == 1 || nseg == 2) &&
               (s1 - s0) % nseg == 0);
  const hipStream_t s = (hipStream_t)stream;
  const int blocks = ceil_div(C, SEG_CPB);
  if (nseg == 1)
    bn_seg_merge<2, 1><<<blocks, 1024, 0, s>>>(part, s0, s1, C, (double)seg_rows, nullptr, eps, momentum,
                                               running_mean, running_var, num_batches_tracked, stats);
  else
    bn_seg_merge<2, 2><<<blocks, 1024, 0, s>>>(part, s0, s1, C, (double)seg_rows, nullptr, eps, momentum,
                                               running_mean, running_var, num_batches_tracked, stats);
  RGAN_CHECK_LAUNCH();
  return 0;
}

extern "C" int rgan_bn_segment_stats(const double* part, long long s0, long long s1, int C, int seg_rows,
                                     float eps, float momentum, float* running_mean, float* running_var,
                                     long long* num_batches_tracked, float* stats, double* moments, void* stream) {
  RGAN_REQUIRE(part && s1 > s0 && s0 >= 0 && C > 0 && seg_rows > 0 && (stats || moments));
  const hipStream_t s = (hipStream_t)stream;
  const int blocks = ceil_div(C, SEG_CPB);
  if (moments)
    bn_seg_merge<1><<<blocks, 1024, 0, s>>>(part, s0, s1, C, (double)seg_rows, moments, 0.f, 0.f, nullptr,
                                            nullptr, nullptr, nullptr);
  else
    bn_seg_merge<2><<<blocks, 1024, 0, s>>>(part, s0, s1, C, (double)seg_rows, nullptr, eps, momentum,
                                            running_mean, running_var, num_batches_tracked, stats);
  RGAN_CHECK_LAUNCH();
  return 0;
}

// merge `nranks` moment blocks [r][3][C] in rank order -> (mean, invstd) float, running stats
__global__ void bn_finalize_kernel(const double* __restrict__ mom, int nranks, int C, float eps, float momentum,
                                   float* running_mean, float* running_var, long long* nbt, float* stats) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c == 0 && nbt) nbt[0] += 1;
  if (c >= C) return;
  double N = 0.0, M = 0.0, S = 0.0;
  for (int k = 0; k < nranks; ++k)
    chan_merge(N, M, S, mom[((size_t)k * 3 + 0) * C + c], mom[((size_t)k * 3 + 1) * C + c],
               mom[((size_t)k * 3 + 2) * C + c]);
  const double var = S / N;
  stats[c] = (float)M;
  stats[C + c] = (float)(1.0 / sqrt(var + (double)eps));
  if (running_mean) running_mean[c] = (1.f - momentum) * running_mean[c] + momentum * (float)M;
  if (running_var) {
    const float unb = N > 1.0 ? (float)(S / (N - 1.0)) : (float)var;
    running_var[c] = (1.f - momentum) * running_var[c] + momentum * unb;
  }
}

// partial pass + fused merge (FIN 1: moments into `moments`; FIN 2: stats + running stats)
static int bn_forward_stats(const float* y, long long P, int C, long long sp, long long sc, int fin,
                            double* moments, float eps, float momentum, float* running_mean, float* running_var,
                            long long* nbt, float* stats, void* partial, hipStream_t s) {
  BnGeo g = bn_geo(P, C, sp, sc);
  if (g.vec && ((uintptr_t)y & 15)) g = bn_geo(P, C, 1, 2);
  double* part = (double*)partial;
  dim3 grid(g.chunks, g.cgroups);
  if (g.vec) bn_moments_partial<4><<<grid, 256, 0, s>>>(y, P, C, sp, sc, g.tpr, g.rows, part);
  else bn_moments_partial<1><<<grid, 256, 0, s>>>(y, P, C, sp, sc, g.tpr, g.rows, part);
  RGAN_CHECK_LAUNCH();
  const int blocks = ceil_div(C, MERGE_CPB);
  if (fin == 1)
    bn_merge<1><<<blocks, 1024, 0, s>>>(part, g.chunks, C, moments, y, P, sc, 0.f, 0.f, nullptr, nullptr, nullptr,
                                        nullptr);
  else
    bn_merge<2><<<blocks, 1024, 0, s>>>(part, g.chunks, C, nullptr, y, P, sc, eps, momentum, running_mean,
                                        running_var, nbt, stats);
  RGAN_CHECK_LAUNCH();
  return 0;
}

extern "C" int rgan_bn_moments(const float* y, long long P, int C, long long sp, long long sc, double* moments,
                               void* partial, void* stream) {
  RGAN_REQUIRE(y && moments && partial && P > 0 && C > 0);
  return bn_forward_stats(y, P, C, sp, sc, 1, moments, 0.f, 0.f, nullptr, nullptr, nullptr, nullptr, partial,
                          (hipStream_t)stream);
}

extern "C" int rgan_bn_finalize(const double* moments, int nranks, int C, float eps, float momentum,
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
  return bn_forward_stats(y, P, C, sp, sc, 2, nullptr, eps, momentum, running_mean, running_var,
                          num_batches_tracked, stats, partial, (hipStream_t)stream);
}

// ------------------------------------------------------------------ apply
// per-thread fixed channel quad (blockIdx.x = channel group); pixels strided over blockIdx.y
// NSEG 2: rows [0, seg_rows) normalised with stats[0], the rest with stats[1] ([2][2C]: the
// batched D pass's two calls in one launch)
template <int Q, int NSEG = 1>
__global__ __launch_bounds__(256) void bn_apply_kernel(const float* __restrict__ y, long long P, int C,
                                                       long long sp, long long sc, const float* __restrict__ stats,
                                                       const float* __restrict__ gamma,
                                                       const float* __restrict__ beta, int act, float alpha,
                                                       float* __restrict__ a, long long asp, long long asc,
                                                       int tpr, long long seg_rows = 0) {
  const int tid = threadIdx.x, lc = tid % tpr, rl = tid / tpr, rp = blockDim.x / tpr;
  const int c0 = (blockIdx.x * tpr + lc) * Q;
  if (c0 >= C) return;
  float al_s[NSEG][Q], be_s[NSEG][Q];
#pragma unroll
  for (int sg = 0; sg < NSEG; ++sg)
#pragma unroll
    for (int q = 0; q < Q; ++q) {
      const int c = min(c0 + q, C - 1);
      const float* st = stats + (size_t)sg * 2 * C;
      al_s[sg][q] = (gamma ? gamma[c] : 1.f) * st[C + c];
      be_s[sg][q] = (beta ? beta[c] : 0.f) - st[c] * al_s[sg][q];
    }
  const long long step = (long long)gridDim.y * rp;
  auto out = [&](long long p, float (&v)[Q]) {
    const int sg = NSEG > 1 && p >= seg_rows ? 1 : 0;
#pragma unroll
    for (int q = 0; q < Q; ++q) v[q] = act_fwd(v[q] * al_s[sg][q] + be_s[sg][q], act, alpha);
    if constexpr (Q == 4) {
      *reinterpret_cast<float4*>(a + p * asp + c0) = make_float4(v[0], v[1], v[2], v[3]);
    } else {
      a[p * asp + (long long)c0 * asc] = v[0];
    }
  };
  long long p = (long long)blockIdx.y * rp + rl;
  for (; p + (BN_UNR - 1) * step < P; p += BN_UNR * step) {
    float v[BN_UNR][Q];
#pragma unroll
    for (int u = 0; u < BN_UNR; ++u) load_q<Q>(y, (p + u * step) * sp + (long long)c0 * sc, v[u]);
#pragma unroll
    for (int u = 0; u < BN_UNR; ++u) out(p + u * step, v[u]);
  }
  for (; p < P; p += step) {
    float v[Q];
    load_q<Q>(y, p * sp + (long long)c0 * sc, v);
    out(p, v);
  }
}

// apply-pass grid: pixel blocks per channel group, each thread at least `min_iter` pixel
// rows (round-1 sweep with tools/bn_micro.py: 4096 blocks, 4 rows)
static dim3 apply_grid(const BnGeo& g, long long P, long long blocks = 4096) {
  constexpr long long min_iter = 4;
  const long long rb = std::max<long long>(
      1, std::min<long long>((P + g.rp * min_iter - 1) / (g.rp * min_iter), std::max<long long>(1, blocks / g.cgroups)));
  return dim3(g.cgroups, (unsigned)rb);
}

// the forward normalise + activation pass (2 streams: y in, a out) on twice the blocks: at
// C3's largest layer (537 MB moved) 4.36-4.39 -> 4.68-4.72 TB/s (run r6m); the backward
// passes (3-4 streams) measured slower there, and stay on 4096
static dim3 fwd_apply_grid(const BnGeo& g, long long P) { return apply_grid(g, P, 8192); }

extern "C" int rgan_bn_apply_segments(const float* y, long long P, int C, int nseg, const float* stats,
                                      const float* gamma, const float* beta, int act, float act_alpha, float* a,
                                      void* stream) {
  RGAN_REQUIRE(act_ok(act));
  // dense NHWC y and a, P % nseg == 0; stats [nseg][2C]
  RGAN_REQUIRE(y && stats && a && P > 0 && C > 0 && (nseg == 1 || nseg == 2) && P % nseg == 0);
  hipStream_t s = (hipStream_t)stream;
  BnGeo g = bn_geo(P, C, C, 1);
  RGAN_REQUIRE(g.vec && ((uintptr_t)y & 15) == 0 && ((uintptr_t)a & 15) == 0);
  if (nseg == 1)
    bn_apply_kernel<4, 1><<<fwd_apply_grid(g, P), 256, 0, s>>>(y, P, C, C, 1, stats, gamma, beta, act, act_alpha, a, C,
                                                          1, g.tpr, 0);
  else
    bn_apply_kernel<4, 2><<<fwd_apply_grid(g, P), 256, 0, s>>>(y, P, C, C, 1, stats, gamma, beta, act, act_alpha, a, C,
                                                          1, g.tpr, P / 2);
  RGAN_CHECK_LAUNCH();
  return 0;
}

extern "C" int rgan_bn_apply(const float* y, long long P, int C, long long sp, long long sc,
                             const float* stats, const float* gamma, const float* beta, int act,
                             float act_alpha, float* a, long long asp, long long asc, void* stream) {
  RGAN_REQUIRE(act_ok(act));
  RGAN_REQUIRE(y && stats && a && P > 0 && C > 0);
  hipStream_t s = (hipStream_t)stream;
  BnGeo g = bn_geo(P, C, sp, sc);
  const bool vec = g.vec && asc == 1 && asp == C && ((uintptr_t)y & 15) == 0 && ((uintptr_t)a & 15) == 0;
  if (!vec && g.vec) g = bn_geo(P, C, 1, 2);
  if (vec)
    bn_apply_kernel<4><<<fwd_apply_grid(g, P), 256, 0, s>>>(y, P, C, sp, sc, stats, gamma, beta, act, act_alpha, a,
                                                       asp, asc, g.tpr);
  else
    bn_apply_kernel<1><<<fwd_apply_grid(g, P), 256, 0, s>>>(y, P, C, sp, sc, stats, gamma, beta, act, act_alpha, a,
                                                       asp, asc, g.tpr);
  RGAN_CHECK_LAUNCH();
  return 0;
}

// ------------------------------------------------------------------ stats + apply, one launch
// Small layers (<= SA_MAX_SEGS 64-row segments per batch segment): the conv epilogue's
// segment sums part[S][2][C] (batch segment k = segments [k S/NSEG, (k+1) S/NSEG)) are merged
// by EVERY block for its own channels -- lane (lc, rl) sums segments rl, rl + rp, ... of its
// channel quad, then the rp lane sums are added in lane order through LDS: a fixed order, so
// every block derives bitwise the same (mean, invstd) -- and the block normalises + activates
// its rows as bn_apply_kernel does.  Blocks with blockIdx.y == 0 publish the stats (the
// backward's) and update the running statistics in segment order; block (0, 0) counts
// num_batches_tracked.  Replaces bn_seg_merge + bn_apply_kernel (two launches) where the
// redundant merge reads (each block: S/4 bytes per channel, from L2) stay well under the
// apply's own 8 B/element.
constexpr long long SA_MAX_SEGS = 64;
constexpr int SA_MAX_ROW_BLOCKS = 256;

// One lane's share of a per-block merge: entries e = rl, rl + rp, ... < n, entry e = segment
// seg_of(e) of part[S][2][C]; s1 / s2 += that segment's two sums of the channel quad at c0, in
// entry order, with QM_UNR entries' 16-B loads in flight at once (the merge is a latency chain
// of L2 round trips otherwise).
constexpr int QM_UNR = 8;
template <typename SegOf>
__device__ __forceinline__ void quad_merge(const double* __restrict__ part, int C, int c0, int rl, int rp, int n,
                                           SegOf seg_of, double (&s1)[4], double (&s2)[4]) {
  auto load = [&](int e, double2 (&v)[4]) {
    const double* r = part + (size_t)seg_of(e) * 2 * C + c0;
    v[0] = reinterpret_cast<const double2*>(r)[0];
    v[1] = reinterpret_cast<const double2*>(r)[1];
    v[2] = reinterpret_cast<const double2*>(r + C)[0];
    v[3] = reinterpret_cast<const double2*>(r + C)[1];
  };
  auto add = [&](const double2 (&v)[4]) {
    s1[0] += v[0].x; s1[1] += v[0].y; s1[2] += v[1].x; s1[3] += v[1].y;
    s2[0] += v[2].x; s2[1] += v[2].y; s2[2] += v[3].x; s2[3] += v[3].y;
  };
  int e = rl;
  for (; e + (QM_UNR - 1) * rp < n; e += QM_UNR * rp) {
    double2 v[QM_UNR][4];
#pragma unroll
    for (int u = 0; u < QM_UNR; ++u) load(e + u * rp, v[u]);
#pragma unroll
    for (int u = 0; u < QM_UNR; ++u) add(v[u]);
  }
  for (; e < n; e += rp) {
    double2 v[4];
    load(e, v);
    add(v);
  }
}

template <int NSEG>
__global__ __launch_bounds__(256) void bn_seg_apply_kernel(const double* __restrict__ part, long long S, double seg_n,
                                                           float eps, float momentum, float* running_mean,
                                                           float* running_var, long long* nbt, float* stats_out,
                                                           const float* __restrict__ y, long long P, int C,
                                                           const float* __restrict__ gamma,
                                                           const float* __restrict__ beta, int act, float alpha,
                                                           float* __restrict__ a, int tpr) {
  __shared__ double sh[2][256][4];
  const int tid = threadIdx.x, lc = tid % tpr, rl = tid / tpr, rp = blockDim.x / tpr;
  const int c0 = (blockIdx.x * tpr + lc) * 4;
  const bool live = c0 < C;
  const long long Sk = S / NSEG;
  float al_s[NSEG][4], be_s[NSEG][4];
#pragma unroll
  for (int sg = 0; sg < NSEG; ++sg) {
    double s1[4] = {0.0, 0.0, 0.0, 0.0}, s2[4] = {0.0, 0.0, 0.0, 0.0};
    if (live) {
      const long long k0 = sg * Sk;
      quad_merge(part, C, c0, rl, rp, (int)Sk, [&](int e) { return k0 + e; }, s1, s2);
    }
    if (sg > 0) __syncthreads();  // the previous segment's lane sums are read
#pragma unroll
    for (int q = 0; q < 4; ++q) { sh[0][tid][q] = s1[q]; sh[1][tid][q] = s2[q]; }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      double S1 = 0.0, S2 = 0.0;
      for (int r = 0; r < rp; ++r) { S1 += sh[0][r * tpr + lc][q]; S2 += sh[1][r * tpr + lc][q]; }
      // bn_seg_merge's formulas: unshifted double sums of the 64-row segments
      const double n = seg_n * (double)Sk, mean = S1 / n, m2 = fmax(S2 - S1 * mean, 0.0), var = m2 / n;
      const float fmean = (float)mean, finv = (float)(1.0 / sqrt(var + (double)eps));
      const int c = min(c0 + q, C - 1);
      al_s[sg][q] = (gamma ? gamma[c] : 1.f) * finv;
      be_s[sg][q] = (beta ? beta[c] : 0.f) - fmean * al_s[sg][q];
      if (blockIdx.y == 0 && rl == 0 && live && c0 + q < C) {
        float* st = stats_out + (size_t)sg * 2 * C;
        st[c] = fmean;
        st[C + c] = finv;
        if (running_mean) running_mean[c] = (1.f - momentum) * running_mean[c] + momentum * fmean;
        if (running_var) {
          const float unb = n > 1.0 ? (float)(m2 / (n - 1.0)) : (float)var;
          running_var[c] = (1.f - momentum) * running_var[c] + momentum * unb;
        }
      }
    }
    if (blockIdx.x == 0 && blockIdx.y == 0 && tid == 0 && nbt) nbt[0] += 1;
  }
  if (!live) return;
  const long long seg_rows = P / NSEG;
  const long long step = (long long)gridDim.y * rp;
  auto out = [&](long long p, float (&v)[4]) {
    const int sg = NSEG > 1 && p >= seg_rows ? 1 : 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) v[q] = act_fwd(v[q] * al_s[sg][q] + be_s[sg][q], act, alpha);
    *reinterpret_cast<float4*>(a + p * C + c0) = make_float4(v[0], v[1], v[2], v[3]);
  };
  long long p = (long long)blockIdx.y * rp + rl;
  for (; p + (BN_UNR - 1) * step < P; p += BN_UNR * step) {
    float v[BN_UNR][4];
#pragma unroll
    for (int u = 0; u < BN_UNR; ++u) load_q<4>(y, (p + u * step) * C + c0, v[u]);
#pragma unroll
    for (int u = 0; u < BN_UNR; ++u) out(p + u * step, v[u]);
  }
  for (; p < P; p += step) {
    float v[4];
    load_q<4>(y, p * C + c0, v);
    out(p, v);
  }
}

extern "C" int rgan_bn_segment_apply(const double* part, long long S, int nseg, int seg_rows, const float* y,
                                     long long P, int C, float eps, float momentum, float* running_mean,
                                     float* running_var, long long* num_batches_tracked, const float* gamma,
                                     const float* beta, int act, float act_alpha, float* stats, float* a,
                                     void* stream) {
  RGAN_REQUIRE(act_ok(act));
  RGAN_REQUIRE(part && y && a && stats && S > 0 && P > 0 && C > 0 && seg_rows > 0 && (nseg == 1 || nseg == 2) &&
               S % nseg == 0 && P % nseg == 0 && P == S * (long long)seg_rows);
  const BnGeo g = bn_geo(P, C, C, 1);
  RGAN_REQUIRE(g.vec && ((uintptr_t)y & 15) == 0 && ((uintptr_t)a & 15) == 0);
  // one launch only where it measured faster than the two (tools/bn_small_micro.py, run r6g, graph
  // replays): a single batch segment of <= 2^18 elements (512 x 256: 6.1 vs 6.7 us; 2048 x 128:
  // 6.4 vs 6.8); at 2048 x 256 (7.3 vs 6.8) and every two-segment call (1024-4096 rows: 9.8-12.5
  // vs 9.3-9.6) the serial in-block merge costs more than the launch it saves
  if (S / nseg > SA_MAX_SEGS || nseg != 1 || P * C > (1LL << 18)) {  // merge once, then apply
    int rc = rgan_bn_segment_stats_n(part, 0, S, nseg, C, seg_rows, eps, momentum, running_mean, running_var,
                                     num_batches_tracked, stats, stream);
    if (rc) return rc;
    return rgan_bn_apply_segments(y, P, C, nseg, stats, gamma, beta, act, act_alpha, a, stream);
  }
  const hipStream_t s = (hipStream_t)stream;
  dim3 grid = apply_grid(g, P);
  grid.y = std::min<unsigned>(grid.y, SA_MAX_ROW_BLOCKS);
  if (nseg == 1)
    bn_seg_apply_kernel<1><<<grid, 256, 0, s>>>(part, S, (double)seg_rows, eps, momentum, running_mean, running_var,
                                                num_batches_tracked, stats, y, P, C, gamma, beta, act, act_alpha, a,
                                                g.tpr);
  else
    bn_seg_apply_kernel<2><<<grid, 256, 0, s>>>(part, S, (double)seg_rows, eps, momentum, running_mean, running_var,
                                                num_batches_tracked, stats, y, P, C, gamma, beta, act, act_alpha, a,
                                                g.tpr);
  RGAN_CHECK_LAUNCH();
  return 0;
}

// ------------------------------------------------------------------ backward
// partial [chunk][2][C] doubles: sum g, sum g*(y-mean);  g = da * act'(y*al + be)
// NSEG 2: the batched D pass's two calls in one launch -- chunk x of segment x / chunks_seg
// covers rows of that segment only, with its stats row (partials [seg][chunk][2][C])
template <int Q, int NSEG = 1>
__global__ __launch_bounds__(256) void bn_bwd_partial(const float* __restrict__ da, long long dsp, long long dsc,
                                                      const float* __restrict__ y, long long P, int C, long long sp,
                                                      long long sc, const float* __restrict__ stats_all,
                                                      const float* __restrict__ gamma,
                                                      const float* __restrict__ beta, int act, float alpha, int tpr,
                                                      long long rows, double* __restrict__ part, int chunks_seg = 1) {
  __shared__ double sh[2][256][Q];
  const int tid = threadIdx.x, lc = tid % tpr, rl = tid / tpr, rp = blockDim.x / tpr;
  const int c0 = (blockIdx.y * tpr + lc) * Q;
  const int seg = NSEG > 1 ? (int)blockIdx.x / chunks_seg : 0;
  const int chunk = NSEG > 1 ? (int)blockIdx.x - seg * chunks_seg : (int)blockIdx.x;
  const float* stats = stats_all + (size_t)seg * 2 * C;
  const long long pb = (long long)seg * P;  // NSEG > 1: P = rows per segment
  const long long p0 = pb + chunk * rows, p1 = min(pb + P, p0 + rows);
  double s1[Q], s2[Q];
  float mean[Q], al[Q], be[Q];
#pragma unroll
  for (int q = 0; q < Q; ++q) {
    s1[q] = 0.0; s2[q] = 0.0;
    const int c = min(c0 + q, C - 1);
    mean[q] = stats[c];
    al[q] = (gamma ? gamma[c] : 1.f) * stats[C + c];
    be[q] = (beta ? beta[c] : 0.f) - mean[q] * al[q];
  }
  if (c0 < C) {
    auto acc = [&](const float (&v)[Q], const float (&g)[Q]) {
#pragma unroll
      for (int q = 0; q < Q; ++q) {
        const double gz = (double)(g[q] * act_grad_from_in(v[q] * al[q] + be[q], act, alpha));
        s1[q] += gz;
        s2[q] += gz * (double)(v[q] - mean[q]);
      }
    };
    long long p = p0 + rl;
    for (; p + (BN_UNR - 1) * rp < p1; p += BN_UNR * rp) {
      float v[BN_UNR][Q], g[BN_UNR][Q];
#pragma unroll
      for (int u = 0; u < BN_UNR; ++u) {
        load_q<Q>(y, (p + u * rp) * sp + (long long)c0 * sc, v[u]);
        load_q<Q>(da, (p + u * rp) * dsp + (long long)c0 * dsc, g[u]);
      }
#pragma unroll
      for (int u = 0; u < BN_UNR; ++u) acc(v[u], g[u]);
    }
    for (; p < p1; p += rp) {
      float v[Q], g[Q];
      load_q<Q>(y, p * sp + (long long)c0 * sc, v);
      load_q<Q>(da, p * dsp + (long long)c0 * dsc, g);
      acc(v, g);
    }
  }
#pragma unroll
  for (int q = 0; q < Q; ++q) { sh[0][tid][q] = s1[q]; sh[1][tid][q] = s2[q]; }
  __syncthreads();
  if (rl == 0 && c0 < C) {
#pragma unroll
    for (int q = 0; q < Q; ++q) {
      if (c0 + q < C) {
        double a1 = 0.0, a2 = 0.0;
        for (int r = 0; r < rp; ++r) { a1 += sh[0][r * tpr + lc][q]; a2 += sh[1][r * tpr + lc][q]; }
        part[((size_t)blockIdx.x * 2 + 0) * C + c0 + q] = a1;
        part[((size_t)blockIdx.x * 2 + 1) * C + c0 + q] = a2;
      }
    }
  }
}

// dy = al*(g - sum_g/Pg - (y-mean)*invstd^2*sum_gx/Pg); dgamma = invstd*sum_gx, dbeta = sum_g
// NSEG 2: rows [0, seg_rows) with stats / sums row 0, the rest with row 1 (the batched
// pass's two calls); the affine gradients are the segments' sum (segment order)
template <int Q, int NSEG = 1>
__global__ __launch_bounds__(256) void bn_bwd_apply(const float* __restrict__ da, long long dsp, long long dsc,
                                                    const float* __restrict__ y, long long P, int C, long long sp,
                                                    long long sc, const float* __restrict__ stats,
                                                    const float* __restrict__ gamma,
                                                    const float* __restrict__ beta, int act, float alpha,
                                                    const double* __restrict__ sums, double inv_pg,
                                                    float* __restrict__ dy, long long ysp, long long ysc,
                                                    float* dgamma, float* dbeta, int tpr,
                                                    const float* __restrict__ add, int accum_affine,
                                                    long long seg_rows = 0) {
  const int tid = threadIdx.x, lc = tid % tpr, rl = tid / tpr, rp = blockDim.x / tpr;
  const int c0 = (blockIdx.x * tpr + lc) * Q;
  if (c0 >= C) return;
  float mean_s[NSEG][Q], al_s[NSEG][Q], be_s[NSEG][Q], k1_s[NSEG][Q], k2_s[NSEG][Q];
#pragma unroll
  for (int q = 0; q < Q; ++q) {
    const int c = min(c0 + q, C - 1);
    float db = 0.f, dg = 0.f;
#pragma unroll
    for (int sg = 0; sg < NSEG; ++sg) {
      const float* st = stats + (size_t)sg * 2 * C;
      const double* su = sums + (size_t)sg * 2 * C;
      const float inv = st[C + c];
      mean_s[sg][q] = st[c];
      al_s[sg][q] = (gamma ? gamma[c] : 1.f) * inv;
      be_s[sg][q] = (beta ? beta[c] : 0.f) - mean_s[sg][q] * al_s[sg][q];
      k1_s[sg][q] = (float)(su[c] * inv_pg);
      k2_s[sg][q] = (float)(su[C + c] * (double)inv * (double)inv * inv_pg);
      const float dbs = (float)su[c], dgs = (float)(su[C + c] * (double)inv);
      db = sg == 0 ? dbs : db + dbs;
      dg = sg == 0 ? dgs : dg + dgs;
    }
    if (blockIdx.y == 0 && rl == 0 && c0 + q < C) {
      if (dbeta) dbeta[c] = accum_affine ? dbeta[c] + db : db;
      if (dgamma) dgamma[c] = accum_affine ? dgamma[c] + dg : dg;
    }
  }
  const long long step = (long long)gridDim.y * rp;
  auto out = [&](long long p, float (&v)[Q], const float (&g)[Q]) {
    const int sg = NSEG > 1 && p >= seg_rows ? 1 : 0;
    const float(&mean)[Q] = mean_s[sg];
    const float(&al)[Q] = al_s[sg];
    const float(&be)[Q] = be_s[sg];
    const float(&k1)[Q] = k1_s[sg];
    const float(&k2)[Q] = k2_s[sg];
#pragma unroll
    for (int q = 0; q < Q; ++q) {
      const float gz = g[q] * act_grad_from_in(v[q] * al[q] + be[q], act, alpha);
      v[q] = al[q] * (gz - k1[q] - (v[q] - mean[q]) * k2[q]);
    }
    if (add) {
      float w[Q];
      load_q<Q>(add, p * ysp + (long long)c0 * ysc, w);
#pragma unroll
      for (int q = 0; q < Q; ++q) v[q] += w[q];
    }
    if constexpr (Q == 4) {
      *reinterpret_cast<float4*>(dy + p * ysp + c0) = make_float4(v[0], v[1], v[2], v[3]);
    } else {
      dy[p * ysp + (long long)c0 * ysc] = v[0];
    }
  };
  long long p = (long long)blockIdx.y * rp + rl;
  for (; p + (BN_UNR - 1) * step < P; p += BN_UNR * step) {
    float v[BN_UNR][Q], g[BN_UNR][Q];
#pragma unroll
    for (int u = 0; u < BN_UNR; ++u) {
      load_q<Q>(y, (p + u * step) * sp + (long long)c0 * sc, v[u]);
      load_q<Q>(da, (p + u * step) * dsp + (long long)c0 * dsc, g[u]);
    }
#pragma unroll
    for (int u = 0; u < BN_UNR; ++u) out(p + u * step, v[u], g[u]);
  }
  for (; p < P; p += step) {
    float v[Q], g[Q];
    load_q<Q>(y, p * sp + (long long)c0 * sc, v);
    load_q<Q>(da, p * dsp + (long long)c0 * dsc, g);
    out(p, v, g);
  }
}

// Small-P BatchNorm backward (the 4x4 layer under D's closing dense layer: 512 rows per
// call at B = 32): the sums, their merge and the apply in one launch instead of three.
// Block = 16 channels (one 64-B piece of every NHWC row: four lanes x float4) x 128 row
// lanes (512 threads); the block holding the other half of those 128-B lines runs on the same
// XCD (a 4-channel block shared every line with three other blocks, usually on other XCDs).
// Lane (r, q) reads rows r, r + 128, ... of each segment -- the first BNS_RC rows per
// segment kept in registers for the apply pass (no second read; rows past them are read
// again) -- and sums bn_bwd_partial's terms in double; the 16 row lanes of a wave are added
// by a fixed xor butterfly, the 8 waves by a fixed LDS sum, then every lane applies its rows
// with bn_bwd_apply's constants and formula.  NSEG 2: rows [0, Ps) use stats / sums row 0,
// [Ps, 2 Ps) row 1; the affine gradients are the segments' sum.
// (round 6: 16 / NSEG cached rows per lane, was 8 / NSEG -- a 2048-row call re-read its last 8
// rows per lane one dependent round trip at a time, 24-28 us per call at C = 128-256 in the
// WGAN-GP engine; every row of a <= 2048-row single call now stays in registers, 128 VGPRs of
// the 256 two waves per SIMD allow)
constexpr int BNS_LANES = 128, BNS_CH = 16, BNS_THREADS = 512;
constexpr long long BNS_MAX_ROWS = 2048;  // rows per segment
template <int NSEG>
__global__ __launch_bounds__(BNS_THREADS) void bn_bwd_small(const float* __restrict__ da, const float* __restrict__ y,
                                                            long long Ps, int C, const float* __restrict__ stats,
                                                            const float* __restrict__ gamma,
                                                            const float* __restrict__ beta, int act, float alpha,
                                                            float* __restrict__ dy, float* dgamma, float* dbeta,
                                                            const float* __restrict__ add = nullptr,
                                                            int accum_affine = 0, double* sums_out = nullptr) {
  constexpr int RC = 16 / NSEG;  // rows per segment cached in registers
  constexpr int NW = BNS_THREADS / 64;
  __shared__ double sh[2][NSEG][NW][BNS_CH];
  const int tid = threadIdx.x, q = tid & 3, r = tid >> 2, lane = tid & 63, wv = tid >> 6;
  // XCD-aware channel groups: blocks are dispatched round-robin over the 8 XCDs, so group
  // (b % 8) * (nb / 8) + b / 8 puts consecutive 16-channel groups -- the two 64-B halves of
  // every 128-B line -- on one XCD (one L2 fetch per line)
  const int nb = gridDim.x;
  const int grp = (nb % 8 == 0) ? (int)(blockIdx.x % 8) * (nb / 8) + (int)(blockIdx.x / 8) : (int)blockIdx.x;
  const int c0 = grp * BNS_CH + 4 * q;
  float mean[NSEG][4], al[NSEG][4], be[NSEG][4], inv[NSEG][4];
#pragma unroll
  for (int sg = 0; sg < NSEG; ++sg)
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float* st = stats + (size_t)sg * 2 * C;
      const int c = c0 + k;
      inv[sg][k] = st[C + c];
      mean[sg][k] = st[c];
      al[sg][k] = (gamma ? gamma[c] : 1.f) * inv[sg][k];
      be[sg][k] = (beta ? beta[c] : 0.f) - mean[sg][k] * al[sg][k];
    }
  float4 cv[NSEG][RC], cg[NSEG][RC];
#pragma unroll
  for (int sg = 0; sg < NSEG; ++sg) {
    const long long rb = (long long)sg * Ps;
#pragma unroll
    for (int j = 0; j < RC; ++j) {  // every cached row's loads in flight together
      const long long p = r + (long long)j * BNS_LANES;
      if (p < Ps) {
        cv[sg][j] = *reinterpret_cast<const float4*>(y + (rb + p) * C + c0);
        cg[sg][j] = *reinterpret_cast<const float4*>(da + (rb + p) * C + c0);
      }
    }
  }
  auto terms = [&](int sg, const float4& v4, const float4& g4, double (&s1)[4], double (&s2)[4]) {
    const float vv[4] = {v4.x, v4.y, v4.z, v4.w}, gg[4] = {g4.x, g4.y, g4.z, g4.w};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const double gz = (double)(gg[k] * act_grad_from_in(vv[k] * al[sg][k] + be[sg][k], act, alpha));
      s1[k] += gz;
      s2[k] += gz * (double)(vv[k] - mean[sg][k]);
    }
  };
#pragma unroll
  for (int sg = 0; sg < NSEG; ++sg) {
    double s1[4] = {0.0, 0.0, 0.0, 0.0}, s2[4] = {0.0, 0.0, 0.0, 0.0};
    const long long rb = (long long)sg * Ps;
#pragma unroll
    for (int j = 0; j < RC; ++j)
      if (r + (long long)j * BNS_LANES < Ps) terms(sg, cv[sg][j], cg[sg][j], s1, s2);
    for (long long p = r + (long long)RC * BNS_LANES; p < Ps; p += BNS_LANES) {
      const float4 v4 = *reinterpret_cast<const float4*>(y + (rb + p) * C + c0);
      const float4 g4 = *reinterpret_cast<const float4*>(da + (rb + p) * C + c0);
      terms(sg, v4, g4, s1, s2);
    }
    // the wave's 16 row lanes of each channel: fixed xor butterfly over lane bits 2..5
#pragma unroll
    for (int o = 4; o < 64; o <<= 1)
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        s1[k] += __shfl_xor(s1[k], o);
        s2[k] += __shfl_xor(s2[k], o);
      }
    if (lane < 4)
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        sh[0][sg][wv][4 * q + k] = s1[k];
        sh[1][sg][wv][4 * q + k] = s2[k];
      }
  }
  __syncthreads();
  const double inv_pg = 1.0 / (double)Ps;
  float k1[NSEG][4], k2[NSEG][4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    float db = 0.f, dg = 0.f;
#pragma unroll
    for (int sg = 0; sg < NSEG; ++sg) {
      double S1 = sh[0][sg][0][4 * q + k], S2 = sh[1][sg][0][4 * q + k];
#pragma unroll
      for (int w = 1; w < NW; ++w) {  // waves in order
        S1 += sh[0][sg][w][4 * q + k];
        S2 += sh[1][sg][w][4 * q + k];
      }
      const double iv = (double)inv[sg][k];
      k1[sg][k] = (float)(S1 * inv_pg);
      k2[sg][k] = (float)(S2 * iv * iv * inv_pg);
      const float dbs = (float)S1, dgs = (float)(S2 * iv);
      db = sg == 0 ? dbs : db + dbs;
      dg = sg == 0 ? dgs : dg + dgs;
      if (sums_out && r == 0) {  // the sums themselves (the WGAN-GP engine keeps them)
        sums_out[((size_t)sg * 2 + 0) * C + c0 + k] = S1;
        sums_out[((size_t)sg * 2 + 1) * C + c0 + k] = S2;
      }
    }
    if (r == 0) {
      if (dbeta) dbeta[c0 + k] = accum_affine ? dbeta[c0 + k] + db : db;
      if (dgamma) dgamma[c0 + k] = accum_affine ? dgamma[c0 + k] + dg : dg;
    }
  }
  auto apply = [&](int sg, const float4& v4, const float4& g4, long long row) {
    float vv[4] = {v4.x, v4.y, v4.z, v4.w};
    const float gg[4] = {g4.x, g4.y, g4.z, g4.w};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float gz = gg[k] * act_grad_from_in(vv[k] * al[sg][k] + be[sg][k], act, alpha);
      vv[k] = al[sg][k] * (gz - k1[sg][k] - (vv[k] - mean[sg][k]) * k2[sg][k]);
    }
    if (add) {
      const float4 w4 = *reinterpret_cast<const float4*>(add + row * C + c0);
      vv[0] += w4.x; vv[1] += w4.y; vv[2] += w4.z; vv[3] += w4.w;
    }
    *reinterpret_cast<float4*>(dy + row * C + c0) = make_float4(vv[0], vv[1], vv[2], vv[3]);
  };
#pragma unroll
  for (int sg = 0; sg < NSEG; ++sg) {
    const long long rb = (long long)sg * Ps;
#pragma unroll
    for (int j = 0; j < RC; ++j)
      if (r + (long long)j * BNS_LANES < Ps) apply(sg, cv[sg][j], cg[sg][j], rb + r + (long long)j * BNS_LANES);
    for (long long p = r + (long long)RC * BNS_LANES; p < Ps; p += BNS_LANES) {
      const float4 v4 = *reinterpret_cast<const float4*>(y + (rb + p) * C + c0);
      const float4 g4 = *reinterpret_cast<const float4*>(da + (rb + p) * C + c0);
      apply(sg, v4, g4, rb + p);
    }
  }
}

static bool dense_nhwc(long long sp, long long sc, int C, const void* p) {
  return sc == 1 && sp == C && ((uintptr_t)p & 15) == 0;
}

extern "C" int rgan_bn_backward_sums(const float* da, long long dsp, long long dsc, const float* y, long long P,
                                     int C, long long sp, long long sc, const float* stats, const float* gamma,
                                     const float* beta, int act, float act_alpha, double* sums, void* partial,
                                     void* stream) {
  RGAN_REQUIRE(act_ok(act));
  RGAN_REQUIRE(da && y && stats && sums && partial && P > 0 && C > 0);
  hipStream_t s = (hipStream_t)stream;
  BnGeo g = bn_geo(P, C, sp, sc);
  const bool vec = g.vec && dense_nhwc(sp, sc, C, y) && dense_nhwc(dsp, dsc, C, da);
  if (!vec && g.vec) g = bn_geo(P, C, 1, 2);
  double* part = (double*)partial;
  dim3 grid(g.chunks, g.cgroups);
  if (vec)
    bn_bwd_partial<4><<<grid, 256, 0, s>>>(da, dsp, dsc, y, P, C, sp, sc, stats, gamma, beta, act, act_alpha,
                                           g.tpr, g.rows, part);
  else
    bn_bwd_partial<1><<<grid, 256, 0, s>>>(da, dsp, dsc, y, P, C, sp, sc, stats, gamma, beta, act, act_alpha,
                                           g.tpr, g.rows, part);
  RGAN_CHECK_LAUNCH();
  bn_merge<0><<<ceil_div(C, MERGE_CPB), 1024, 0, s>>>(part, g.chunks, C, sums, nullptr, 0, 0, 0.f, 0.f, nullptr,
                                                       nullptr, nullptr, nullptr);
  RGAN_CHECK_LAUNCH();
  return 0;
}

extern "C" int rgan_bn_backward_apply_ex(const float* da, long long dsp, long long dsc, const float* y,
                                         long long P, int C, long long sp, long long sc, const float* stats,
                                         const float* gamma, const float* beta, int act, float act_alpha,
                                         const double* sums, long long P_global, const float* add, float* dy,
                                         long long ysp, long long ysc, float* dgamma, float* dbeta,
                                         int accumulate_affine, void* stream) {
  RGAN_REQUIRE(act_ok(act));
  RGAN_REQUIRE(da && y && stats && sums && dy && P > 0 && C > 0 && P_global >= P);
  hipStream_t s = (hipStream_t)stream;
  BnGeo g = bn_geo(P, C, sp, sc);
  const bool vec = g.vec && dense_nhwc(sp, sc, C, y) && dense_nhwc(dsp, dsc, C, da) &&
                   dense_nhwc(ysp, ysc, C, dy) && (!add || ((uintptr_t)add & 15) == 0);
  if (!vec && g.vec) g = bn_geo(P, C, 1, 2);
  const double inv_pg = 1.0 / (double)P_global;
  if (vec)
    bn_bwd_apply<4><<<apply_grid(g, P), 256, 0, s>>>(da, dsp, dsc, y, P, C, sp, sc, stats, gamma, beta, act,
                                                    act_alpha, sums, inv_pg, dy, ysp, ysc, dgamma, dbeta, g.tpr,
                                                    add, accumulate_affine);
  else
    bn_bwd_apply<1><<<apply_grid(g, P), 256, 0, s>>>(da, dsp, dsc, y, P, C, sp, sc, stats, gamma, beta, act,
                                                    act_alpha, sums, inv_pg, dy, ysp, ysc, dgamma, dbeta, g.tpr,
                                                    add, accumulate_affine);
  RGAN_CHECK_LAUNCH();
  return 0;
}

extern "C" int rgan_bn_backward_sums_apply(const float* da, const float* y, long long P, int C, const float* stats,
                                           const float* gamma, const float* beta, int act, float act_alpha,
                                           const float* add, float* dy, float* dgamma, float* dbeta,
                                           int accumulate_affine, double* sums, void* partial, void* stream) {
  RGAN_REQUIRE(act_ok(act));
  RGAN_REQUIRE(da && y && stats && dy && sums && partial && P > 0 && C > 0);
  // one launch only with >= 64 channel-group blocks: at C = 128-256 (8-16 blocks, the WGAN-GP
  // engine's arch-1 layers) bn_bwd_small measured 25-28 us per call against ~18 us for the
  // three launches below (run r6d)
  if (P <= BNS_MAX_ROWS && C % BNS_CH == 0 && C / BNS_CH >= 64 && dense_nhwc(C, 1, C, y) && dense_nhwc(C, 1, C, da) &&
      dense_nhwc(C, 1, C, dy) && (!add || dense_nhwc(C, 1, C, add))) {  // small layers: one launch
    bn_bwd_small<1><<<C / BNS_CH, BNS_THREADS, 0, (hipStream_t)stream>>>(da, y, P, C, stats, gamma, beta, act,
                                                                         act_alpha, dy, dgamma, dbeta, add,
                                                                         accumulate_affine, sums);
    RGAN_CHECK_LAUNCH();
    return 0;
  }
  int rc = rgan_bn_backward_sums(da, C, 1, y, P, C, C, 1, stats, gamma, beta, act, act_alpha, sums, partial, stream);
  if (rc) return rc;
  return rgan_bn_backward_apply_ex(da, C, 1, y, P, C, C, 1, stats, gamma, beta, act, act_alpha, sums, P, add, dy, C,
                                   1, dgamma, dbeta, accumulate_affine, stream);
}

// dgamma (+)= (float)(sum g (y - mean) * invstd), dbeta (+)= (float)sum g from [2][C] sums --
// the affine gradients bn_bwd_apply writes, from a rank's LOCAL sums under SyncBN (the
// normalisation uses the all-reduced sums; the bucketed gradient all-reduce sums these)
__global__ void bn_affine_from_sums(const double* __restrict__ sums, const float* __restrict__ stats, int C,
                                    float* dgamma, float* dbeta, int accumulate) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  const float db = (float)sums[c], dg = (float)(sums[C + c] * (double)stats[C + c]);
  if (dbeta) dbeta[c] = accumulate ? dbeta[c] + db : db;
  if (dgamma) dgamma[c] = accumulate ? dgamma[c] + dg : dg;
}

extern "C" int rgan_bn_affine_grads(const double* sums, const float* stats, int C, float* dgamma, float* dbeta,
                                    int accumulate, void* stream) {
  RGAN_REQUIRE(sums && stats && C > 0);
  if (!dgamma && !dbeta) return 0;
  bn_affine_from_sums<<<ceil_div(C, 256), 256, 0, (hipStream_t)stream>>>(sums, stats, C, dgamma, dbeta, accumulate);
  RGAN_CHECK_LAUNCH();
  return 0;
}

extern "C" int rgan_bn_backward_apply(const float* da, long long dsp, long long dsc, const float* y, long long P,
                                      int C, long long sp, long long sc, const float* stats, const float* gamma,
                                      const float* beta, int act, float act_alpha, const double* sums,
                                      long long P_global, float* dy, long long ysp, long long ysc, float* dgamma,
                                      float* dbeta, void* stream) {
  RGAN_REQUIRE(act_ok(act));
  return rgan_bn_backward_apply_ex(da, dsp, dsc, y, P, C, sp, sc, stats, gamma, beta, act, act_alpha, sums,
                                   P_global, nullptr, dy, ysp, ysc, dgamma, dbeta, 0, stream);
}

extern "C" int rgan_bn_backward_segments(const float* da, const float* y, long long P, int C, int nseg,
                                         const float* stats, const float* gamma, const float* beta, int act,
                                         float act_alpha, float* dy, float* dgamma, float* dbeta, void* partial,
                                         void* stream) {
  RGAN_REQUIRE(act_ok(act));
  // dense NHWC da, y, dy; P % nseg == 0; stats [nseg][2C]; partial: nseg * rgan_bn_partial_bytes(P / nseg, C)
  RGAN_REQUIRE(da && y && stats && dy && partial && P > 0 && C > 0 && (nseg == 1 || nseg == 2) && P % nseg == 0);
  hipStream_t s = (hipStream_t)stream;
  const long long Ps = P / nseg;
  if (Ps <= BNS_MAX_ROWS && C % BNS_CH == 0 && dense_nhwc(C, 1, C, y) && dense_nhwc(C, 1, C, da) &&
      dense_nhwc(C, 1, C, dy)) {  // small layers: one launch
    if (nseg == 1)
      bn_bwd_small<1><<<C / BNS_CH, BNS_THREADS, 0, s>>>(da, y, Ps, C, stats, gamma, beta, act, act_alpha, dy, dgamma,
                                                         dbeta);
    else
      bn_bwd_small<2><<<C / BNS_CH, BNS_THREADS, 0, s>>>(da, y, Ps, C, stats, gamma, beta, act, act_alpha, dy, dgamma,
                                                         dbeta);
    RGAN_CHECK_LAUNCH();
    return 0;
  }
  BnGeo g = bn_geo(Ps, C, C, 1);
  RGAN_REQUIRE(g.vec && dense_nhwc(C, 1, C, y) && dense_nhwc(C, 1, C, da) && dense_nhwc(C, 1, C, dy));
  double* part = (double*)partial;
  double* sums = part + (size_t)nseg * g.chunks * 2 * C;
  const dim3 pgrid(nseg * g.chunks, g.cgroups);
  if (nseg == 1)
    bn_bwd_partial<4, 1><<<pgrid, 256, 0, s>>>(da, C, 1, y, Ps, C, C, 1, stats, gamma, beta, act, act_alpha, g.tpr,
                                               g.rows, part, g.chunks);
  else
    bn_bwd_partial<4, 2><<<pgrid, 256, 0, s>>>(da, C, 1, y, Ps, C, C, 1, stats, gamma, beta, act, act_alpha, g.tpr,
                                               g.rows, part, g.chunks);
  RGAN_CHECK_LAUNCH();
  bn_merge<0><<<dim3(ceil_div(C, MERGE_CPB), nseg), 1024, 0, s>>>(part, g.chunks, C, sums, nullptr, 0, 0, 0.f, 0.f,
                                                                  nullptr, nullptr, nullptr, nullptr);
  RGAN_CHECK_LAUNCH();
  const BnGeo ga = bn_geo(P, C, C, 1);
  const double inv_pg = 1.0 / (double)Ps;
  if (nseg == 1)
    bn_bwd_apply<4, 1><<<apply_grid(ga, P), 256, 0, s>>>(da, C, 1, y, P, C, C, 1, stats, gamma, beta, act, act_alpha,
                                                        sums, inv_pg, dy, C, 1, dgamma, dbeta, ga.tpr, nullptr, 0, 0);
  else
    bn_bwd_apply<4, 2><<<apply_grid(ga, P), 256, 0, s>>>(da, C, 1, y, P, C, C, 1, stats, gamma, beta, act, act_alpha,
                                                        sums, inv_pg, dy, C, 1, dgamma, dbeta, ga.tpr, nullptr, 0, Ps);
  RGAN_CHECK_LAUNCH();
  return 0;
}

// Backward sums written by a GEMM's post-op (rgan_conv_post mode 2): part[S][2][C], segment
// s = phase * Sp + j (Sp = S / phases 64-row segments per phase); batch segment k owns
// j in [k Sp/nseg, (k+1) Sp/nseg) of every phase.  -> sums[k][2][C]: lane r of a 16-channel x
// 64-lane block sums its segments in order, then a fixed LDS tree (deterministic).
__global__ __launch_bounds__(1024) void bn_part_merge(const double* __restrict__ part, int S, int phases, int C,
                                                      double* __restrict__ sums) {
  __shared__ double sh[2][MERGE_ROWS][MERGE_CPB];
  const int k = blockIdx.y, nseg = gridDim.y;
  const int cl = threadIdx.x % MERGE_CPB, r = threadIdx.x / MERGE_CPB;
  const int c = blockIdx.x * MERGE_CPB + cl;
  const int Sp = S / phases, J = Sp / nseg, cnt = phases * J;
  double a1 = 0.0, a2 = 0.0;
  if (c < C)
    for (int i = r; i < cnt; i += MERGE_ROWS) {
      const int ph = i / J, s = ph * Sp + k * J + (i - ph * J);
      a1 += part[((size_t)s * 2 + 0) * C + c];
      a2 += part[((size_t)s * 2 + 1) * C + c];
    }
  sh[0][r][cl] = a1;
  sh[1][r][cl] = a2;
  __syncthreads();
  for (int h = MERGE_ROWS / 2; h > 0; h >>= 1) {
    if (r < h) {
      sh[0][r][cl] += sh[0][r + h][cl];
      sh[1][r][cl] += sh[1][r + h][cl];
    }
    __syncthreads();
  }
  if (r == 0 && c < C) {
    sums[((size_t)k * 2 + 0) * C + c] = sh[0][0][cl];
    sums[((size_t)k * 2 + 1) * C + c] = sh[1][0][cl];
  }
}

// bn_part_merge + bn_bwd_apply (act = none: g already carries act') in one launch for small
// layers (<= SA_MAX_SEGS post-op segments per batch segment): every block merges its channels'
// segment sums in bn_part_merge's segment order with the fixed lane layout of
// bn_seg_apply_kernel (bitwise the same sums in every block), blocks with blockIdx.y == 0
// write the affine gradients, then the block applies its rows.
template <int NSEG>
__global__ __launch_bounds__(256) void bn_parts_apply_kernel(const float* __restrict__ g, const float* __restrict__ y,
                                                             long long P, int C, const float* __restrict__ stats,
                                                             const float* __restrict__ gamma,
                                                             const float* __restrict__ beta,
                                                             const double* __restrict__ part, int S, int phases,
                                                             float* __restrict__ dy, float* dgamma, float* dbeta,
                                                             int tpr) {
  __shared__ double sh[2][256][4];
  const int tid = threadIdx.x, lc = tid % tpr, rl = tid / tpr, rp = blockDim.x / tpr;
  const int c0 = (blockIdx.x * tpr + lc) * 4;
  const bool live = c0 < C;
  const int Sp = S / phases, J = Sp / NSEG, cnt = phases * J;
  const long long seg_rows = P / NSEG;
  const double inv_pg = 1.0 / (double)seg_rows;
  float mean_s[NSEG][4], al_s[NSEG][4], be_s[NSEG][4], k1_s[NSEG][4], k2_s[NSEG][4];
  float db[4] = {0.f, 0.f, 0.f, 0.f}, dg[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int sg = 0; sg < NSEG; ++sg) {
    double s1[4] = {0.0, 0.0, 0.0, 0.0}, s2[4] = {0.0, 0.0, 0.0, 0.0};
    if (live)
      quad_merge(part, C, c0, rl, rp, cnt, [&](int i) { const int ph = i / J; return ph * Sp + sg * J + (i - ph * J); },
                 s1, s2);
    if (sg > 0) __syncthreads();
#pragma unroll
    for (int q = 0; q < 4; ++q) { sh[0][tid][q] = s1[q]; sh[1][tid][q] = s2[q]; }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      double S1 = 0.0, S2 = 0.0;
      for (int r = 0; r < rp; ++r) { S1 += sh[0][r * tpr + lc][q]; S2 += sh[1][r * tpr + lc][q]; }
      const int c = min(c0 + q, C - 1);
      const float* st = stats + (size_t)sg * 2 * C;
      const float inv = st[C + c];
      mean_s[sg][q] = st[c];
      al_s[sg][q] = (gamma ? gamma[c] : 1.f) * inv;
      be_s[sg][q] = (beta ? beta[c] : 0.f) - mean_s[sg][q] * al_s[sg][q];
      k1_s[sg][q] = (float)(S1 * inv_pg);
      k2_s[sg][q] = (float)(S2 * (double)inv * (double)inv * inv_pg);
      const float dbs = (float)S1, dgs = (float)(S2 * (double)inv);
      db[q] = sg == 0 ? dbs : db[q] + dbs;
      dg[q] = sg == 0 ? dgs : dg[q] + dgs;
    }
  }
  if (!live) return;
  if (blockIdx.y == 0 && rl == 0)
#pragma unroll
    for (int q = 0; q < 4; ++q)
      if (c0 + q < C) {
        if (dbeta) dbeta[c0 + q] = db[q];
        if (dgamma) dgamma[c0 + q] = dg[q];
      }
  const long long step = (long long)gridDim.y * rp;
  auto out = [&](long long p, float (&v)[4], const float (&gz)[4]) {
    const int sg = NSEG > 1 && p >= seg_rows ? 1 : 0;
#pragma unroll
    for (int q = 0; q < 4; ++q)
      v[q] = al_s[sg][q] * (gz[q] - k1_s[sg][q] - (v[q] - mean_s[sg][q]) * k2_s[sg][q]);
    *reinterpret_cast<float4*>(dy + p * C + c0) = make_float4(v[0], v[1], v[2], v[3]);
  };
  long long p = (long long)blockIdx.y * rp + rl;
  for (; p + (BN_UNR - 1) * step < P; p += BN_UNR * step) {
    float v[BN_UNR][4], gz[BN_UNR][4];
#pragma unroll
    for (int u = 0; u < BN_UNR; ++u) {
      load_q<4>(y, (p + u * step) * C + c0, v[u]);
      load_q<4>(g, (p + u * step) * C + c0, gz[u]);
    }
#pragma unroll
    for (int u = 0; u < BN_UNR; ++u) out(p + u * step, v[u], gz[u]);
  }
  for (; p < P; p += step) {
    float v[4], gz[4];
    load_q<4>(y, p * C + c0, v);
    load_q<4>(g, p * C + c0, gz);
    out(p, v, gz);
  }
}

extern "C" int rgan_bn_backward_parts(const float* g, const float* y, long long P, int C, int nseg,
                                      const float* stats, const float* gamma, const float* beta, const double* part,
                                      long long S, int phases, float* dy, float* dgamma, float* dbeta, double* sums,
                                      void* stream) {
  // g = da * act' (rgan_conv_post mode 2 output), dense NHWC g, y, dy; stats [nseg][2C];
  // sums: [nseg][2][C] doubles of scratch
  RGAN_REQUIRE(g && y && stats && part && dy && sums && P > 0 && C > 0 && (nseg == 1 || nseg == 2) &&
               P % nseg == 0 && phases >= 1 && S > 0 && S % phases == 0 && (S / phases) % nseg == 0);
  hipStream_t s = (hipStream_t)stream;
  const BnGeo ga = bn_geo(P, C, C, 1);
  RGAN_REQUIRE(ga.vec && dense_nhwc(C, 1, C, y) && dense_nhwc(C, 1, C, g) && dense_nhwc(C, 1, C, dy));
  if (S / nseg <= SA_MAX_SEGS) {  // small layer: merge + apply in one launch
    dim3 grid = apply_grid(ga, P);
    grid.y = std::min<unsigned>(grid.y, SA_MAX_ROW_BLOCKS);
    if (nseg == 1)
      bn_parts_apply_kernel<1><<<grid, 256, 0, s>>>(g, y, P, C, stats, gamma, beta, part, (int)S, phases, dy, dgamma,
                                                    dbeta, ga.tpr);
    else
      bn_parts_apply_kernel<2><<<grid, 256, 0, s>>>(g, y, P, C, stats, gamma, beta, part, (int)S, phases, dy, dgamma,
                                                    dbeta, ga.tpr);
    RGAN_CHECK_LAUNCH();
    return 0;
  }
  bn_part_merge<<<dim3(ceil_div(C, MERGE_CPB), nseg), 1024, 0, s>>>(part, (int)S, phases, C, sums);
  RGAN_CHECK_LAUNCH();
  const long long Ps = P / nseg;
  const double inv_pg = 1.0 / (double)Ps;
  if (nseg == 1)
    bn_bwd_apply<4, 1><<<apply_grid(ga, P), 256, 0, s>>>(g, C, 1, y, P, C, C, 1, stats, gamma, beta, RGAN_ACT_NONE,
                                                        0.f, sums, inv_pg, dy, C, 1, dgamma, dbeta, ga.tpr, nullptr, 0,
                                                        0);
  else
    bn_bwd_apply<4, 2><<<apply_grid(ga, P), 256, 0, s>>>(g, C, 1, y, P, C, C, 1, stats, gamma, beta, RGAN_ACT_NONE,
                                                        0.f, sums, inv_pg, dy, C, 1, dgamma, dbeta, ga.tpr, nullptr, 0,
                                                        Ps);
  RGAN_CHECK_LAUNCH();
  return 0;
}

extern "C" int rgan_bn_backward(const float* da, long long dsp, long long dsc, const float* y, long long P,
                                int C, long long sp, long long sc, const float* stats, const float* gamma,
                                const float* beta, int act, float act_alpha, float* dy, long long ysp,
                                long long ysc, float* dgamma, float* dbeta, void* partial, void* stream) {
  RGAN_REQUIRE(act_ok(act));
  RGAN_REQUIRE(partial && P > 0 && C > 0);
  if (P <= BNS_MAX_ROWS && C % BNS_CH == 0 && dense_nhwc(sp, sc, C, y) && dense_nhwc(dsp, dsc, C, da) &&
      dense_nhwc(ysp, ysc, C, dy) && stats && dy) {  // small layers: one launch
    bn_bwd_small<1><<<C / BNS_CH, BNS_THREADS, 0, (hipStream_t)stream>>>(da, y, P, C, stats, gamma, beta, act,
                                                                         act_alpha, dy, dgamma, dbeta);
    RGAN_CHECK_LAUNCH();
    return 0;
  }
  double* sums = (double*)partial + (size_t)max_chunks(P, C) * 2 * C;
  int rc = rgan_bn_backward_sums(da, dsp, dsc, y, P, C, sp, sc, stats, gamma, beta, act, act_alpha, sums,
                                 partial, stream);
  if (rc) return rc;
  return rgan_bn_backward_apply(da, dsp, dsc, y, P, C, sp, sc, stats, gamma, beta, act, act_alpha, sums, P,
                                dy, ysp, ysc, dgamma, dbeta, stream);
}

// ------------------------------------------------------------------ WGAN-GP double backward
// The penalty (GLI:646-658) differentiates the create-graph backward of every D layer.
// Through train-mode BatchNorm2d + activation that backward is (per channel, N pixels):
//   xhat = (y - mean) invstd,  z = gamma xhat + beta,  e = dh act'(z),
//   dy = s (e - mean(e) - xhat mean(e xhat)),  s = gamma invstd.
// Given a = dP/d(dy) (the adjoint conv of the layer's dgrad), the adjoints are
//   dP/de   = pe = s (a - A - xhat Ax),         A = mean(a), Ax = mean(a xhat)
//   dP/d(dh) = pe act'(z)                        (feeds the next layer's adjoint conv)
//   t       = pe dh act''(z)                     (0 for ReLU / LeakyReLU)
//   gx      = -s (a c + e Ax) + gamma t          (dP/dxhat, c = mean(e xhat))
//   dP/dy   = invstd (gx - mean(gx) - xhat mean(gx xhat)) - dPds gamma invstd^2 xhat / N
//   dPds    = sum a e - mean(e) sum a - c sum a xhat     (s = gamma invstd depends on y)
//   dgamma += dPds invstd + sum t xhat,  dbeta += sum t.
// mean(gx) and mean(gx xhat) follow from the stage sums, so one elementwise pass writes
// both outputs: stage 1 sums (a, a xhat, a e); stage 2 (only when act'' != 0) sums (t, t xhat).
template <int Q, int STAGE>
__global__ __launch_bounds__(256) void bn_dd_partial(const float* __restrict__ a, const float* __restrict__ y,
                                                     const float* __restrict__ dh, long long P, int C, long long sp,
                                                     long long sc, const float* __restrict__ stats,
                                                     const float* __restrict__ gamma, const float* __restrict__ beta,
                                                     int act, float alpha, const double* __restrict__ s1,
                                                     double inv_pg, int tpr, long long rows,
                                                     double* __restrict__ part) {
  constexpr int NS = STAGE == 1 ? 3 : 2;
  __shared__ double sh[NS][256][Q];
  const int tid = threadIdx.x, lc = tid % tpr, rl = tid / tpr, rp = blockDim.x / tpr;
  const int c0 = (blockIdx.y * tpr + lc) * Q;
  const long long p0 = blockIdx.x * rows, p1 = min(P, p0 + rows);
  double acc[NS][Q];
  float mean[Q], inv[Q], gam[Q], bet[Q], sg[Q], A[Q], Ax[Q];
#pragma unroll
  for (int q = 0; q < Q; ++q) {
#pragma unroll
    for (int k = 0; k < NS; ++k) acc[k][q] = 0.0;
    const int c = min(c0 + q, C - 1);
    mean[q] = stats[c];
    inv[q] = stats[C + c];
    gam[q] = gamma ? gamma[c] : 1.f;
    bet[q] = beta ? beta[c] : 0.f;
    sg[q] = gam[q] * inv[q];
    A[q] = STAGE == 2 ? (float)(s1[c] * inv_pg) : 0.f;
    Ax[q] = STAGE == 2 ? (float)(s1[C + c] * inv_pg) : 0.f;
  }
  if (c0 < C) {
    for (long long p = p0 + rl; p < p1; p += rp) {
      float va[Q], vy[Q], vd[Q];
      const long long off = p * sp + (long long)c0 * sc;
      load_q<Q>(a, off, va);
      load_q<Q>(y, off, vy);
      load_q<Q>(dh, off, vd);
#pragma unroll
      for (int q = 0; q < Q; ++q) {
        const float xh = (vy[q] - mean[q]) * inv[q], z = gam[q] * xh + bet[q];
        if constexpr (STAGE == 1) {
          const float e = vd[q] * act_grad_from_in(z, act, alpha);
          acc[0][q] += (double)va[q];
          acc[1][q] += (double)(va[q] * xh);
          acc[2][q] += (double)(va[q] * e);
        } else {
          const float pe = sg[q] * (va[q] - A[q] - xh * Ax[q]);
          const float t = pe * vd[q] * act_grad2_from_in(z, act, alpha);
          acc[0][q] += (double)t;
          acc[1][q] += (double)(t * xh);
        }
      }
    }
  }
#pragma unroll
  for (int k = 0; k < NS; ++k)
#pragma unroll
    for (int q = 0; q < Q; ++q) sh[k][tid][q] = acc[k][q];
  __syncthreads();
  if (rl == 0 && c0 < C) {
#pragma unroll
    for (int q = 0; q < Q; ++q) {
      if (c0 + q >= C) continue;
#pragma unroll
      for (int k = 0; k < NS; ++k) {
        double t = 0.0;
        for (int r = 0; r < rp; ++r) t += sh[k][r * tpr + lc][q];
        part[((size_t)blockIdx.x * NS + k) * C + c0 + q] = t;
      }
    }
  }
}

// [chunks][NS][C] partials -> [NS][C] totals, fixed order (bn_merge's layout, NS rows)
template <int NS>
__global__ __launch_bounds__(1024) void bn_merge_n(const double* __restrict__ part, int chunks, int C,
                                                   double* __restrict__ out) {
  __shared__ double sh[NS][MERGE_ROWS][MERGE_CPB];
  const int cl = threadIdx.x % MERGE_CPB, r = threadIdx.x / MERGE_CPB;
  const int c = blockIdx.x * MERGE_CPB + cl;
  double acc[NS];
#pragma unroll
  for (int k = 0; k < NS; ++k) acc[k] = 0.0;
  if (c < C)
    for (int j = r; j < chunks; j += MERGE_ROWS)
#pragma unroll
      for (int k = 0; k < NS; ++k) acc[k] += part[((size_t)j * NS + k) * C + c];
#pragma unroll
  for (int k = 0; k < NS; ++k) sh[k][r][cl] = acc[k];
  __syncthreads();
  if (r != 0 || c >= C) return;
#pragma unroll
  for (int k = 0; k < NS; ++k) {
    double t = 0.0;
    for (int q = 0; q < MERGE_ROWS; ++q) t += sh[k][q][cl];
    out[(size_t)k * C + c] = t;
  }
}

template <int Q>
__global__ __launch_bounds__(256) void bn_dd_apply(const float* __restrict__ a, const float* __restrict__ y,
                                                   const float* __restrict__ dh, long long P, int C, long long sp,
                                                   long long sc, const float* __restrict__ stats,
                                                   const float* __restrict__ gamma, const float* __restrict__ beta,
                                                   int act, float alpha, const double* __restrict__ fs,
                                                   const double* __restrict__ s1, const double* __restrict__ s2,
                                                   const double* __restrict__ s1l, const double* __restrict__ s2l,
                                                   double inv_pg, float* __restrict__ adj_dh,
                                                   float* __restrict__ ydir, float* dgamma2, float* dbeta2,
                                                   int accum_affine, int tpr) {
  const int tid = threadIdx.x, lc = tid % tpr, rl = tid / tpr, rp = blockDim.x / tpr;
  const int c0 = (blockIdx.x * tpr + lc) * Q;
  if (c0 >= C) return;
  const bool two = act_has_grad2(act);
  float mean[Q], inv[Q], gam[Q], bet[Q], sg[Q], A[Q], Ax[Q], c1[Q], mgx[Q], mgxx[Q], kk[Q];
#pragma unroll
  for (int q = 0; q < Q; ++q) {
    const int c = min(c0 + q, C - 1);
    const double dinv = stats[C + c], dgam = gamma ? gamma[c] : 1.0, ds = dgam * dinv;
    mean[q] = stats[c];
    inv[q] = (float)dinv;
    gam[q] = (float)dgam;
    bet[q] = beta ? beta[c] : 0.f;
    sg[q] = (float)ds;
    const double em = fs[c] * inv_pg, dc1 = dinv * fs[C + c] * inv_pg;
    const double dA = s1[c] * inv_pg, dAx = s1[C + c] * inv_pg;
    const double dPds = s1[2 * C + c] - em * s1[c] - dc1 * s1[C + c];
    const double T0 = s2 ? s2[c] : 0.0, T1 = s2 ? s2[C + c] : 0.0;
    A[q] = (float)dA;
    Ax[q] = (float)dAx;
    c1[q] = (float)dc1;
    mgx[q] = (float)(-ds * (dc1 * dA + dAx * em) + dgam * T0 * inv_pg);
    mgxx[q] = (float)(-2.0 * ds * dc1 * dAx + dgam * T1 * inv_pg);
    kk[q] = (float)(dPds * dgam * dinv * dinv * inv_pg);
    if (blockIdx.y == 0 && rl == 0 && c0 + q < C) {
      const double dPl = s1l[2 * C + c] - em * s1l[c] - dc1 * s1l[C + c];
      const float dg = (float)(dPl * dinv + (s2l ? s2l[C + c] : 0.0));
      const float db = (float)(s2l ? s2l[c] : 0.0);
      if (dgamma2) dgamma2[c] = accum_affine ? dgamma2[c] + dg : dg;
      if (dbeta2) dbeta2[c] = accum_affine ? dbeta2[c] + db : db;
    }
  }
  const long long step = (long long)gridDim.y * rp;
  for (long long p = (long long)blockIdx.y * rp + rl; p < P; p += step) {
    float va[Q], vy[Q], vd[Q], oh[Q], oy[Q];
    const long long off = p * sp + (long long)c0 * sc;
    load_q<Q>(a, off, va);
    load_q<Q>(y, off, vy);
    load_q<Q>(dh, off, vd);
#pragma unroll
    for (int q = 0; q < Q; ++q) {
      const float xh = (vy[q] - mean[q]) * inv[q], z = gam[q] * xh + bet[q];
      const float d1 = act_grad_from_in(z, act, alpha), e = vd[q] * d1;
      const float pe = sg[q] * (va[q] - A[q] - xh * Ax[q]);
      oh[q] = pe * d1;
      const float t = two ? pe * vd[q] * act_grad2_from_in(z, act, alpha) : 0.f;
      const float gx = -sg[q] * (va[q] * c1[q] + e * Ax[q]) + gam[q] * t;
      oy[q] = inv[q] * (gx - mgx[q] - xh * mgxx[q]) - kk[q] * xh;
    }
    if constexpr (Q == 4) {
      if (adj_dh) *reinterpret_cast<float4*>(adj_dh + off) = make_float4(oh[0], oh[1], oh[2], oh[3]);
      *reinterpret_cast<float4*>(ydir + off) = make_float4(oy[0], oy[1], oy[2], oy[3]);
    } else {
      if (adj_dh) adj_dh[off] = oh[0];
      ydir[off] = oy[0];
    }
  }
}

extern "C" int rgan_bn_dd_sums(const float* a, const float* y, const float* dh, long long P, int C, long long sp,
                               long long sc, const float* stats, const float* gamma, const float* beta, int act,
                               float act_alpha, int stage, const double* stage1, long long P_global, double* sums,
                               void* partial, void* stream) {
  RGAN_REQUIRE(act_ok(act));
  RGAN_REQUIRE(a && y && dh && stats && sums && partial && P > 0 && C > 0 && (stage == 1 || stage == 2));
  RGAN_REQUIRE(stage == 1 || (stage1 && P_global >= P));
  hipStream_t s = (hipStream_t)stream;
  BnGeo g = bn_geo(P, C, sp, sc);
  const bool vec = g.vec && dense_nhwc(sp, sc, C, a) && dense_nhwc(sp, sc, C, y) && dense_nhwc(sp, sc, C, dh);
  if (!vec && g.vec) g = bn_geo(P, C, 1, 2);
  double* part = (double*)partial;
  const dim3 grid(g.chunks, g.cgroups);
  const double inv_pg = stage == 2 ? 1.0 / (double)P_global : 0.0;
#define RGAN_DD(QQ, ST) \
  bn_dd_partial<QQ, ST><<<grid, 256, 0, s>>>(a, y, dh, P, C, sp, sc, stats, gamma, beta, act, act_alpha, stage1, \
                                             inv_pg, g.tpr, g.rows, part)
  if (stage == 1) {
    if (vec) RGAN_DD(4, 1); else RGAN_DD(1, 1);
  } else {
    if (vec) RGAN_DD(4, 2); else RGAN_DD(1, 2);
  }
#undef RGAN_DD
  RGAN_CHECK_LAUNCH();
  if (stage == 1)
    bn_merge_n<3><<<ceil_div(C, MERGE_CPB), 1024, 0, s>>>(part, g.chunks, C, sums);
  else
    bn_merge_n<2><<<ceil_div(C, MERGE_CPB), 1024, 0, s>>>(part, g.chunks, C, sums);
  RGAN_CHECK_LAUNCH();
  return 0;
}

extern "C" int rgan_bn_dd_apply(const float* a, const float* y, const float* dh, long long P, int C, long long sp,
                                long long sc, const float* stats, const float* gamma, const float* beta, int act,
                                float act_alpha, const double* first_sums, const double* stage1,
                                const double* stage2, const double* stage1_local, const double* stage2_local,
                                long long P_global, float* adj_dh, float* ydir, float* dgamma2, float* dbeta2,
                                int accumulate_affine, void* stream) {
  RGAN_REQUIRE(act_ok(act));
  RGAN_REQUIRE(a && y && dh && stats && first_sums && stage1 && ydir && P > 0 && C > 0 && P_global >= P);
  RGAN_REQUIRE(!act_has_grad2(act) || stage2);
  hipStream_t s = (hipStream_t)stream;
  BnGeo g = bn_geo(P, C, sp, sc);
  const bool vec = g.vec && dense_nhwc(sp, sc, C, a) && dense_nhwc(sp, sc, C, y) && dense_nhwc(sp, sc, C, dh) &&
                   dense_nhwc(sp, sc, C, ydir) && (!adj_dh || dense_nhwc(sp, sc, C, adj_dh));
  if (!vec && g.vec) g = bn_geo(P, C, 1, 2);
  const double inv_pg = 1.0 / (double)P_global;
  const double* s1l = stage1_local ? stage1_local : stage1;
  const double* s2l = stage2_local ? stage2_local : stage2;
  if (vec)
    bn_dd_apply<4><<<apply_grid(g, P), 256, 0, s>>>(a, y, dh, P, C, sp, sc, stats, gamma, beta, act, act_alpha,
                                                   first_sums, stage1, stage2, s1l, s2l, inv_pg, adj_dh, ydir,
                                                   dgamma2, dbeta2, accumulate_affine, g.tpr);
  else
    bn_dd_apply<1><<<apply_grid(g, P), 256, 0, s>>>(a, y, dh, P, C, sp, sc, stats, gamma, beta, act, act_alpha,
                                                   first_sums, stage1, stage2, s1l, s2l, inv_pg, adj_dh, ydir,
                                                   dgamma2, dbeta2, accumulate_affine, g.tpr);
  RGAN_CHECK_LAUNCH();
  return 0;
}

// The same without BatchNorm: dy = dh act'(y) (act from its output o = act(y)):
//   dP/d(dh) = a act'(y),  dP/dy = a dh act''(y)  (ydir nullable: only when act'' != 0)
__global__ void act_dd_kernel(const float* __restrict__ a, const float* __restrict__ o,
                              const float* __restrict__ dh, long long n, int act, float alpha,
                              float* __restrict__ adj_dh, float* __restrict__ ydir) {
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += stride) {
    const float v = a[i], out = o[i];
    if (adj_dh) adj_dh[i] = v * act_grad_from_out(out, act, alpha);
    if (ydir) ydir[i] = v * dh[i] * act_grad2_from_out(out, act, alpha);
  }
}

extern "C" int rgan_act_dd(const float* a, const float* act_out, const float* dh, long long n, int act,
                           float act_alpha, float* adj_dh, float* ydir, void* stream) {
  RGAN_REQUIRE(act_ok(act));
  RGAN_REQUIRE(a && act_out && n >= 0 && (adj_dh || ydir) && (!ydir || dh));
  if (n == 0) return 0;
  const int blocks = (int)std::max<long long>(1, std::min<long long>((n + 255) / 256, 8192));
  act_dd_kernel<<<blocks, 256, 0, (hipStream_t)stream>>>(a, act_out, dh, n, act, act_alpha, adj_dh, ydir);
  RGAN_CHECK_LAUNCH();
  return 0;
}

// ------------------------------------------------------------------ activations
__global__ void act_bwd_kernel(const float* __restrict__ da, const float* __restrict__ a, long long n, int act,
                               float alpha, float* __restrict__ dx, int vec, const float* __restrict__ add) {
  const long long n4 = vec ? n >> 2 : 0;
  const float4* da4 = reinterpret_cast<const float4*>(da);
  const float4* a4 = reinterpret_cast<const float4*>(a);
  const float4* add4 = reinterpret_cast<const float4*>(add);
  float4* dx4 = reinterpret_cast<float4*>(dx);
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n4; i += stride) {
    const float4 g = da4[i], v = a4[i];
    float4 o = make_float4(g.x * act_grad_from_out(v.x, act, alpha), g.y * act_grad_from_out(v.y, act, alpha),
                           g.z * act_grad_from_out(v.z, act, alpha), g.w * act_grad_from_out(v.w, act, alpha));
    if (add) {
      const float4 w = add4[i];
      o.x += w.x; o.y += w.y; o.z += w.z; o.w += w.w;
    }
    dx4[i] = o;
  }
  for (long long i = (n4 << 2) + blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += stride)
    dx[i] = da[i] * act_grad_from_out(a[i], act, alpha) + (add ? add[i] : 0.f);
}

extern "C" int rgan_act_backward(const float* da, const float* a, long long n, int act, float act_alpha,
                                 float* dx, void* stream) {
  RGAN_REQUIRE(act_ok(act));
  RGAN_REQUIRE(da && a && dx && n >= 0);
  if (n == 0) return 0;
  return rgan_act_backward_ex(da, a, nullptr, n, act, act_alpha, dx, stream);
}

extern "C" int rgan_act_backward_ex(const float* da, const float* a, const float* add, long long n, int act,
                                    float act_alpha, float* dx, void* stream) {
  RGAN_REQUIRE(act_ok(act));
  RGAN_REQUIRE(da && a && dx && n >= 0);
  if (n == 0) return 0;
  const int vec = ((((uintptr_t)da | (uintptr_t)a | (uintptr_t)dx | (uintptr_t)add) & 15) == 0) ? 1 : 0;
  const int blocks = (int)std::max<long long>(1, std::min<long long>((n / 4 + 255) / 256, 4096));
  act_bwd_kernel<<<blocks, 256, 0, (hipStream_t)stream>>>(da, a, n, act, act_alpha, dx, vec, add);
  RGAN_CHECK_LAUNCH();
  return 0;
}

// per-channel sum over pixels (bias gradients, GLI:202-223 / 260-302 arch-1 convs with bias):
// the BN grid (pixel chunks x channel groups, double partials [chunk][C]) and a fixed-order
// merge that writes (or adds into) the float result -- deterministic, and parallel over
// pixels (one block per 64 channels walking every pixel took 0.75 ms at 32x64x32x32).
template <int Q>
__global__ __launch_bounds__(256) void chsum_partial(const float* __restrict__ t, long long P, int C, long long sp,
                                                     long long sc, int tpr, long long rows,
                                                     double* __restrict__ part) {
  __shared__ double sh[256][Q];
  const int tid = threadIdx.x, lc = tid % tpr, rl = tid / tpr, rp = blockDim.x / tpr;
  const int c0 = (blockIdx.y * tpr + lc) * Q;
  const long long p0 = blockIdx.x * rows, p1 = min(P, p0 + rows);
  double s[Q];
#pragma unroll
  for (int q = 0; q < Q; ++q) s[q] = 0.0;
  if (c0 < C) {
    long long p = p0 + rl;
    for (; p + (BN_UNR - 1) * rp < p1; p += BN_UNR * rp) {
      float v[BN_UNR][Q];
#pragma unroll
      for (int u = 0; u < BN_UNR; ++u) load_q<Q>(t, (p + u * rp) * sp + (long long)c0 * sc, v[u]);
#pragma unroll
      for (int u = 0; u < BN_UNR; ++u)
#pragma unroll
        for (int q = 0; q < Q; ++q) s[q] += (double)v[u][q];
    }
    for (; p < p1; p += rp) {
      float v[Q];
      load_q<Q>(t, p * sp + (long long)c0 * sc, v);
#pragma unroll
      for (int q = 0; q < Q; ++q) s[q] += (double)v[q];
    }
  }
#pragma unroll
  for (int q = 0; q < Q; ++q) sh[tid][q] = s[q];
  __syncthreads();
  if (rl == 0 && c0 < C) {
#pragma unroll
    for (int q = 0; q < Q; ++q) {
      if (c0 + q >= C) continue;
      double a = 0.0;
      for (int r = 0; r < rp; ++r) a += sh[r * tpr + lc][q];
      part[(size_t)blockIdx.x * C + c0 + q] = a;
    }
  }
}

__global__ __launch_bounds__(1024) void chsum_merge(const double* __restrict__ part, int chunks, int C,
                                                    float* __restrict__ out, int accum) {
  __shared__ double sh[MERGE_ROWS][MERGE_CPB];
  const int cl = threadIdx.x % MERGE_CPB, r = threadIdx.x / MERGE_CPB;
  const int c = blockIdx.x * MERGE_CPB + cl;
  double a = 0.0;
  if (c < C)
    for (int j = r; j < chunks; j += MERGE_ROWS) a += part[(size_t)j * C + c];
  sh[r][cl] = a;
  __syncthreads();
  if (r != 0 || c >= C) return;
  double t = 0.0;
  for (int q = 0; q < MERGE_ROWS; ++q) t += sh[q][cl];
  out[c] = accum ? out[c] + (float)t : (float)t;
}

// One-launch channel sum for few pixel rows (the bias gradients of arch 1's deep 8x8 / 4x4 layers
// and their GP sweeps: P <= CS_MAX_ROWS): block = 16 channels (4 lanes x float4) x 64 row lanes,
// each lane sums rows r, r + 64, ... in double (4 loads in flight), the 64 lanes are added by a
// fixed LDS tree, and the result is written (or added) directly -- no partials, no merge launch.
constexpr int CS_LANES = 64;
constexpr long long CS_MAX_ROWS = 2048;
__global__ __launch_bounds__(256) void chsum_small(const float* __restrict__ t, long long P, int C,
                                                   float* __restrict__ out, int accum) {
  __shared__ double sh[CS_LANES][16];
  const int q = threadIdx.x & 3, r = threadIdx.x >> 2, c0 = blockIdx.x * 16 + 4 * q;
  double s[4] = {0.0, 0.0, 0.0, 0.0};
  long long p = r;
  for (; p + 3 * CS_LANES < P; p += 4 * CS_LANES) {
    float4 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = *reinterpret_cast<const float4*>(t + (p + u * CS_LANES) * C + c0);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      s[0] += (double)v[u].x; s[1] += (double)v[u].y; s[2] += (double)v[u].z; s[3] += (double)v[u].w;
    }
  }
  for (; p < P; p += CS_LANES) {
    const float4 v = *reinterpret_cast<const float4*>(t + p * C + c0);
    s[0] += (double)v.x; s[1] += (double)v.y; s[2] += (double)v.z; s[3] += (double)v.w;
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) sh[r][4 * q + i] = s[i];
  __syncthreads();
  for (int h = CS_LANES / 2; h > 0; h >>= 1) {
    if (r < h)
#pragma unroll
      for (int i = 0; i < 4; ++i) sh[r][4 * q + i] += sh[r + h][4 * q + i];
    __syncthreads();
  }
  if (r == 0)
#pragma unroll
    for (int i = 0; i < 4; ++i) out[c0 + i] = accum ? out[c0 + i] + (float)sh[0][4 * q + i] : (float)sh[0][4 * q + i];
}

extern "C" int rgan_channel_sum(const float* t, long long P, int C, long long sp, long long sc, float* out,
                                int accumulate, void* partial, void* stream) {
  RGAN_REQUIRE(t && out && partial && P > 0 && C > 0);
  hipStream_t s = (hipStream_t)stream;
  if (P <= CS_MAX_ROWS && C % 16 == 0 && sc == 1 && sp == C && ((uintptr_t)t & 15) == 0) {
    chsum_small<<<C / 16, 256, 0, s>>>(t, P, C, out, accumulate);
    RGAN_CHECK_LAUNCH();
    return 0;
  }
  BnGeo g = bn_geo(P, C, sp, sc);
  if (g.vec && ((uintptr_t)t & 15)) g = bn_geo(P, C, 1, 2);
  double* part = (double*)partial;
  const dim3 grid(g.chunks, g.cgroups);
  if (g.vec) chsum_partial<4><<<grid, 256, 0, s>>>(t, P, C, sp, sc, g.tpr, g.rows, part);
  else chsum_partial<1><<<grid, 256, 0, s>>>(t, P, C, sp, sc, g.tpr, g.rows, part);
  RGAN_CHECK_LAUNCH();
  chsum_merge<<<ceil_div(C, MERGE_CPB), 1024, 0, s>>>(part, g.chunks, C, out, accumulate);
  RGAN_CHECK_LAUNCH();
  return 0;
}

}  // namespace rgan
