// Probe: v_mfma_f32_32x32x16_bf16 rate, and whether independent VALU work co-executes with
// it (fp32 MFMA does not on gfx950: SQ_VALU_MFMA_COEXEC_CYCLES = 0).  Diagnostic.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
template <int VALU>
__global__ __launch_bounds__(256, 2) void k(float* out, int iters, float x) {
  f32x16 acc[4];
  for (int c = 0; c < 4; ++c)
    for (int r = 0; r < 16; ++r) acc[c][r] = 0.f;
  bf16x8 a, b;
  for (int i = 0; i < 8; ++i) { a[i] = (__bf16)(x * (threadIdx.x + i)); b[i] = (__bf16)(x + i); }
  float v0 = x * threadIdx.x, v1 = v0 + 1.f, v2 = v0 + 2.f, v3 = v0 + 3.f;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int s = 0; s < 24; ++s) {
#pragma unroll
      for (int c = 0; c < 4; ++c) acc[c] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc[c], 0, 0, 0);
#pragma unroll
      for (int q = 0; q < VALU; ++q) {  // independent VALU chains
        v0 = __builtin_fmaf(v0, 1.0001f, 0.5f); v1 = __builtin_fmaf(v1, 1.0001f, 0.5f);
        v2 = __builtin_fmaf(v2, 1.0001f, 0.5f); v3 = __builtin_fmaf(v3, 1.0001f, 0.5f);
      }
    }
  }
  float t = v0 + v1 + v2 + v3;
  for (int c = 0; c < 4; ++c) t += acc[c][0];
  if (t == 1234.5f) out[threadIdx.x] = t;
}
template <int VALU>
void run(int blocks, int iters) {
  float* o;
  (void)hipMalloc(&o, 4096);
  k<VALU><<<blocks, 256>>>(o, iters, 1e-3f);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
  (void)hipEventRecord(e0);
  k<VALU><<<blocks, 256>>>(o, iters, 1e-3f);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms;
  (void)hipEventElapsedTime(&ms, e0, e1);
  const double flops = 2.0 * 32 * 32 * 16 * 96.0 * iters * blocks * 4;
  printf("bf16 32x32x16, %2d x4 VALU per 4 MFMA: %8.1f us  %7.1f TF/s (bf16)\n", VALU, ms * 1e3, flops / ms / 1e9);
  (void)hipFree(o);
}
int main() {
  run<0>(512, 400);
  run<2>(512, 400);
  run<4>(512, 400);
  run<8>(512, 400);
  return 0;
}
