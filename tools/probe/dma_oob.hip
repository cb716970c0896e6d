// Probe: does an out-of-range raw buffer LDS-DMA lane write 0 into LDS or leave it untouched?
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(const float* x, float* y, int n) {
  __shared__ float s[64];
  s[threadIdx.x] = 7.f;
  __syncthreads();
  __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)x, (short)0, n * 4, 0x00020000);
  const int off = (threadIdx.x & 1) ? 0x7ffffff0 : threadIdx.x * 4;  // odd lanes out of range
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)s, 4, off, 0, 0, 0);
  __builtin_amdgcn_s_waitcnt(0x0f70);
  __syncthreads();
  y[threadIdx.x] = s[threadIdx.x];
}
int main() {
  float *x, *y, h[64];
  hipMalloc(&x, 64 * 4); hipMalloc(&y, 64 * 4);
  for (int i = 0; i < 64; ++i) h[i] = 100.f + i;
  hipMemcpy(x, h, 256, hipMemcpyHostToDevice);
  k<<<1, 64>>>(x, y, 64);
  hipMemcpy(h, y, 256, hipMemcpyDeviceToHost);
  printf("lane0 %g lane1 %g lane2 %g lane3 %g\n", h[0], h[1], h[2], h[3]);
  return 0;
}
