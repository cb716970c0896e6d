// Probe: operand / result layout of v_mfma_f32_32x32x16_bf16 (diagnostic).
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
__global__ void k(float* out) {
  const int l = threadIdx.x;
  bf16x8 a, b;
  // assumed: lane l holds A[row = l % 32][k = 8 (l / 32) + e], B[k = 8 (l / 32) + e][col = l % 32]
  for (int e = 0; e < 8; ++e) {
    const int kk = 8 * (l / 32) + e, r = l % 32;
    a[e] = (__bf16)(r == kk ? 1.f : 0.f);          // A = [I16 ; 0]
    b[e] = (__bf16)(float)(r * 16 + kk);           // B[k][j] = 16 j + k
  }
  f32x16 c = {};
  c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
  for (int r = 0; r < 16; ++r) out[l * 16 + r] = c[r];
}
int main() {
  float* d; float h[1024];
  (void)hipMalloc(&d, 4096);
  k<<<1, 64>>>(d);
  (void)hipMemcpy(h, d, 4096, hipMemcpyDeviceToHost);
  // expected with D[i][j] = B[i][j] = 16 j + i (i < 16), 0 for i >= 16, and the 32x32 result
  // layout lane l: col j = l % 32, reg r: row i = 8 (r / 4) + 4 (l / 32) + r % 4
  int ok = 0, bad = 0;
  for (int l = 0; l < 64; ++l)
    for (int r = 0; r < 16; ++r) {
      const int j = l % 32, i = 8 * (r / 4) + 4 * (l / 32) + r % 4;
      const float want = i < 16 ? 16 * j + i : 0;
      if (h[l * 16 + r] == want) ++ok; else { if (bad < 8) printf("lane %d reg %d: got %g want %g\n", l, r, h[l * 16 + r], want); ++bad; }
    }
  printf("ok %d bad %d\n", ok, bad);
  for (int r = 0; r < 16; ++r) printf("%g ", h[r]);
  printf("\n");
  for (int r = 0; r < 16; ++r) printf("%g ", h[32 * 16 + r]);
  printf("\n");
  return 0;
}
