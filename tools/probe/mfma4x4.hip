// Probe of v_mfma_f32_4x4x1_16b_f32 operand/result lanes (diagnostic, GPU).
// A[l] = l + 1, B[l] = 100 * (l + 1); prints which (a, b) products land in each result slot.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f32x4 __attribute__((ext_vector_type(4)));
__global__ void k(float* out) {
  const int l = threadIdx.x;
  f32x4 c = {0.f, 0.f, 0.f, 0.f};
  c = __builtin_amdgcn_mfma_f32_4x4x1f32((float)(l + 1), 1000.f * (float)(l + 1), c, 0, 0, 0);
  for (int r = 0; r < 4; ++r) out[l * 4 + r] = c[r];
}
int main() {
  float* d;
  hipMalloc(&d, 64 * 4 * 4);
  k<<<1, 64>>>(d);
  float h[256];
  hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  for (int l = 0; l < 16; ++l) {
    printf("lane %2d:", l);
    for (int r = 0; r < 4; ++r) {
      const float v = h[l * 4 + r];
      const int b = (int)(v / 1000.f + 0.5f);
      // v = a * 1000 * bl  -> report (a, bl) with a*bl = v/1000
      printf("  r%d=%8.0f", r, v / 1000.f);
    }
    printf("\n");
  }
  hipFree(d);
  return 0;
}
