// Device sampling for --rgan_rng device: the z / u draws (GLI:608,630,648-649,674 draw them
// with normal_ / uniform_ on the host generator) and the real batch's indices (GLI:176:
// numpy.random.choice(N, B, replace=False)), as counter-based draws on the GPU.
//
// Philox-4x32-10 keyed by the run's seed; the 64-bit counter lives on the device and every
// call advances it by the numbers it consumed (the one-block fill of a z / u draw or the
// sampling wave itself; a trailing one-thread launch after a large fill), so a call
// captured in a HIP graph draws fresh numbers at every replay with no host involvement.
// Every rank of a data-parallel run holds the same seed and counter and draws the global
// batch (each keeps its shard), like torch's device generator did here before.
#include "common.h"

namespace rgan {

struct u32x4s {
  uint32_t x, y, z, w;
};

__device__ __forceinline__ u32x4s philox(unsigned long long ctr, unsigned long long seed) {
  uint32_t c0 = (uint32_t)ctr, c1 = (uint32_t)(ctr >> 32), c2 = 0u, c3 = 0u;
  uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint32_t lo0 = 0xD2511F53u * c0, hi0 = __umulhi(0xD2511F53u, c0);
    const uint32_t lo1 = 0xCD9E8D57u * c2, hi1 = __umulhi(0xCD9E8D57u, c2);
    const uint32_t n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
    c0 = n0; c1 = lo1; c2 = n2; c3 = lo0;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return {c0, c1, c2, c3};
}

// uniform in (0, 1]: 24 random bits
__device__ __forceinline__ float u01(uint32_t v) { return ((float)(v >> 8) + 1.f) * (1.f / 16777216.f); }

// kind 0: N(0, 1) (Box-Muller on the four words: two normals per pair); kind 1: U[0, 1)
// advance != 0 (one-block launches): the block also moves the counter on by `advance`
// after every thread has read it (the barrier orders the reads before thread 0's store)
__global__ __launch_bounds__(256) void rng_fill(float* out, long long n, int kind, unsigned long long seed,
                                                unsigned long long* counter, unsigned long long advance) {
  const unsigned long long base = counter[0];
  for (long long q = blockIdx.x * 256LL + threadIdx.x; 4 * q < n; q += (long long)gridDim.x * 256) {
    const u32x4s r = philox(base + (unsigned long long)q, seed);
    float v[4];
    if (kind == 0) {
      const float r0 = sqrtf(-2.f * logf(u01(r.x))), r1 = sqrtf(-2.f * logf(u01(r.z)));
      float s0, c0, s1, c1;
      sincospif(2.f * u01(r.y), &s0, &c0);
      sincospif(2.f * u01(r.w), &s1, &c1);
      v[0] = r0 * c0; v[1] = r0 * s0; v[2] = r1 * c1; v[3] = r1 * s1;
    } else {
      v[0] = u01(r.x) - 1.f / 16777216.f; v[1] = u01(r.y) - 1.f / 16777216.f;
      v[2] = u01(r.z) - 1.f / 16777216.f; v[3] = u01(r.w) - 1.f / 16777216.f;
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
      if (4 * q + i < n) out[4 * q + i] = v[i];
  }
  if (advance) {
    __syncthreads();
    if (threadIdx.x == 0) counter[0] = base + advance;
  }
}

__global__ void rng_advance(unsigned long long* counter, unsigned long long by) { counter[0] += by; }

// n distinct indices of [0, N) in uniformly random order, like numpy.random.choice(N, n,
// replace=False) (every ordered n-tuple equally likely; callers split the draw by position:
// data-parallel shards, PacGAN slots).  Floyd's algorithm (for j = N-n .. N-1 take t
// uniform in [0, j], or j itself when t is already taken) picks a uniform SET, but step s
// yields j = N-n+s on a collision, so late positions lean to high indices; a Fisher-Yates
// pass over the n picks then makes the order uniform.  Uniform integers in [0, m) are
// 64 random bits x m >> 64 (bias <= m / 2^64).  One wave; counters base .. base+n-1 feed
// Floyd, base+n .. base+2n-1 the shuffle; the wave advances the counter by 2n itself
// (every lane read it before lane 0 writes).
//   n <= 64: lane s draws step s and keeps its pick in a register; each step broadcasts its
//            t, the lanes holding earlier picks compare, a ballot decides (no LDS, no
//            barrier); the shuffle swaps registers through wave shuffles;
//   else:    the taken set in LDS, the membership test a ballot over it; the shuffle's
//            swap positions drawn lane-parallel, the swaps by one lane.
constexpr int CHOICE_MAX = 4096;

__device__ __forceinline__ int uniform_below(const u32x4s& r, unsigned long long m) {
  return (int)__umul64hi(((unsigned long long)r.y << 32) | r.x, m);
}

__global__ __launch_bounds__(64) void rng_choice_small(long long* out, int N, int n, unsigned long long seed,
                                                       unsigned long long* counter) {
  const unsigned long long base = counter[0];
  const int lane = threadIdx.x;
  int t_own = 0, pick = -1;  // -1: no pick yet (never equal to a draw)
  int j_own = 0;  // Fisher-Yates: position `lane` swaps with j_own, uniform in [0, lane]
  if (lane < n) {
    const u32x4s r = philox(base + (unsigned long long)lane, seed);
    t_own = uniform_below(r, (unsigned long long)(N - n + lane + 1));
    j_own = uniform_below(philox(base + (unsigned long long)(n + lane), seed), (unsigned long long)(lane + 1));
  }
  for (int s = 0; s < n; ++s) {
    const int t = __shfl(t_own, s);
    const bool any = __ballot(pick == t) != 0;
    if (lane == s) pick = any ? N - n + s : t;
  }
  for (int s = n - 1; s >= 1; --s) {
    const int j = __shfl(j_own, s);
    const int ps = __shfl(pick, s), pj = __shfl(pick, j);
    if (lane == s) pick = pj;
    else if (lane == j) pick = ps;
  }
  if (lane < n) out[lane] = pick;
  if (lane == 0) counter[0] = base + 2ULL * (unsigned long long)n;
}

__global__ __launch_bounds__(64) void rng_choice(long long* out, int N, int n, unsigned long long seed,
                                                 unsigned long long* counter) {
  __shared__ int taken[CHOICE_MAX];
  __shared__ int swap_with[CHOICE_MAX];
  const unsigned long long base = counter[0];
  const int lane = threadIdx.x;
  for (int s = lane; s < n; s += 64)
    swap_with[s] = uniform_below(philox(base + (unsigned long long)(n + s), seed), (unsigned long long)(s + 1));
  for (int s = 0; s < n; ++s) {
    const int j = N - n + s;
    const u32x4s r = philox(base + (unsigned long long)s, seed);
    const int t = uniform_below(r, (unsigned long long)(j + 1));
    bool hit = false;
    for (int i = lane; i < s; i += 64) hit |= taken[i] == t;
    const bool any = __ballot(hit) != 0;
    if (lane == 0) taken[s] = any ? j : t;
    __syncthreads();
  }
  if (lane == 0) {
    for (int s = n - 1; s >= 1; --s) {
      const int j = swap_with[s], v = taken[s];
      taken[s] = taken[j];
      taken[j] = v;
    }
  }
  __syncthreads();
  for (int s = lane; s < n; s += 64) out[s] = taken[s];
  if (lane == 0) counter[0] = base + 2ULL * (unsigned long long)n;
}

}  // namespace rgan

using namespace rgan;

extern "C" int rgan_rng_fill(float* out, long long n, int kind, unsigned long long seed, unsigned long long* counter,
                             void* stream) {
  RGAN_REQUIRE(out && counter && n >= 0 && (kind == 0 || kind == 1));
  if (n == 0) return 0;
  hipStream_t s = (hipStream_t)stream;
  const long long quads = (n + 3) / 4;
  if (quads <= 16 * 256) {  // z / u draws: one block that also advances the counter (one launch)
    rng_fill<<<1, 256, 0, s>>>(out, n, kind, seed, counter, (unsigned long long)quads);
    RGAN_CHECK_LAUNCH();
    return 0;
  }
  rng_fill<<<(unsigned)std::min<long long>((quads + 255) / 256, 2048), 256, 0, s>>>(out, n, kind, seed, counter, 0ull);
  RGAN_CHECK_LAUNCH();
  rng_advance<<<1, 1, 0, s>>>(counter, (unsigned long long)quads);
  RGAN_CHECK_LAUNCH();
  return 0;
}

extern "C" int rgan_rng_choice(long long* out, int N, int n, unsigned long long seed, unsigned long long* counter,
                               void* stream) {
  RGAN_REQUIRE(out && counter && N > 0 && n >= 0 && n <= N && n <= CHOICE_MAX);
  if (n == 0) return 0;
  hipStream_t s = (hipStream_t)stream;
  if (n <= 64) rng_choice_small<<<1, 64, 0, s>>>(out, N, n, seed, counter);
  else rng_choice<<<1, 64, 0, s>>>(out, N, n, seed, counter);
  RGAN_CHECK_LAUNCH();
  return 0;
}
