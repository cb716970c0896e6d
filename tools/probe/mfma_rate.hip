// Probe: achievable v_mfma_f32_32x32x2_f32 rate for a few chain structures (diagnostic).
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f32x16 __attribute__((ext_vector_type(16)));
template <int CH, int MODE>  // CH independent accumulators; MODE 0 interleaved, 1 chain-sequential,
                             // 2 interleaved + per-96 restart (acc re-init, result read: a tile)
__global__ __launch_bounds__(256, 2) void k(float* out, int iters, float x) {
  f32x16 acc[CH];
  for (int c = 0; c < CH; ++c)
    for (int r = 0; r < 16; ++r) acc[c][r] = 0.f;
  float a = x * threadIdx.x, b = x + threadIdx.x;
  float keep = 0.f;
  for (int it = 0; it < iters; ++it) {
    if (MODE == 2) {
      const f32x16 z = {};
#pragma unroll
      for (int c = 0; c < CH; ++c) acc[c] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b + c, z, 0, 0, 0);
#pragma unroll
      for (int s = 1; s < 96 / CH; ++s)
#pragma unroll
        for (int c = 0; c < CH; ++c) acc[c] = __builtin_amdgcn_mfma_f32_32x32x2f32(a + c, b, acc[c], 0, 0, 0);
#pragma unroll
      for (int c = 0; c < CH; ++c)
#pragma unroll
        for (int r = 0; r < 16; ++r) keep += acc[c][r];
    } else if (MODE == 0) {
#pragma unroll
      for (int s = 0; s < 96 / CH; ++s)
#pragma unroll
        for (int c = 0; c < CH; ++c) acc[c] = __builtin_amdgcn_mfma_f32_32x32x2f32(a + c, b, acc[c], 0, 0, 0);
    } else {
#pragma unroll
      for (int c = 0; c < CH; ++c)
#pragma unroll
        for (int s = 0; s < 96 / CH; ++s) acc[c] = __builtin_amdgcn_mfma_f32_32x32x2f32(a + c, b, acc[c], 0, 0, 0);
    }
  }
  float t = keep;
  for (int c = 0; c < CH; ++c) t += acc[c][0];
  if (t == 1234.5f) out[threadIdx.x] = t;
}
typedef float f32x4 __attribute__((ext_vector_type(4)));
template <int CH>  // 4x4x1 (16 blocks) MFMAs over CH independent accumulators, 8 per 32x32x2 in FLOPs
__global__ __launch_bounds__(256, 2) void k4(float* out, int iters, float x) {
  f32x4 acc[CH];
  for (int c = 0; c < CH; ++c) acc[c] = f32x4{0.f, 0.f, 0.f, 0.f};
  float a = x * threadIdx.x, b = x + threadIdx.x;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int s = 0; s < 768 / CH; ++s)
#pragma unroll
      for (int c = 0; c < CH; ++c) acc[c] = __builtin_amdgcn_mfma_f32_4x4x1f32(a + c, b, acc[c], 0, 0, 0);
  }
  float t = 0.f;
  for (int c = 0; c < CH; ++c) t += acc[c][0];
  if (t == 1234.5f) out[threadIdx.x] = t;
}
template <int CH>
void run4(const char* name, int blocks, int iters = 200) {
  float* o;
  (void)hipMalloc(&o, 4096);
  k4<CH><<<blocks, 256>>>(o, iters, 1e-3f);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
  (void)hipEventRecord(e0);
  k4<CH><<<blocks, 256>>>(o, iters, 1e-3f);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms;
  (void)hipEventElapsedTime(&ms, e0, e1);
  const double flops = 2.0 * 16 * 4 * 4 * 768.0 * iters * blocks * 4;
  printf("%-28s blocks %4d  %8.1f us  %6.1f TF/s\n", name, blocks, ms * 1e3, flops / ms / 1e9);
  (void)hipFree(o);
}
template <int CH, int MODE>
void run(const char* name, int blocks, int iters = 200) {
  float* o;
  (void)hipMalloc(&o, 4096);
  k<CH, MODE><<<blocks, 256>>>(o, iters, 1e-3f);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
  (void)hipEventRecord(e0);
  k<CH, MODE><<<blocks, 256>>>(o, iters, 1e-3f);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms;
  (void)hipEventElapsedTime(&ms, e0, e1);
  const double flops = 2.0 * 32 * 32 * 2 * 96.0 * iters * blocks * 4;
  printf("%-28s blocks %4d  %8.1f us  %6.1f TF/s\n", name, blocks, ms * 1e3, flops / ms / 1e9);
  (void)hipFree(o);
}
int main() {
  run<4, 0>("4 chains interleaved", 512);
  run<4, 1>("4 chains sequential", 512);
  run<2, 0>("2 chains interleaved", 512);
  run<8, 0>("8 chains interleaved", 512);
  run<4, 2>("4 chains, tiles of 96", 512);
  run<4, 2>("4 chains, tiles of 96", 1024);
  run<4, 2>("tiles of 96, 8 per wave", 512, 8);
  run<4, 2>("tiles of 96, 16 per wave", 512, 16);
  run<4, 2>("tiles of 96, 4 per wave", 1024, 4);
  run4<8>("4x4x1, 8 chains", 512);
  run4<2>("4x4x1, 2 chains", 512);
  run4<16>("4x4x1, 16 chains", 512);
  return 0;
}
