// FETCH_SIZE calibration for the access patterns of the narrow kernels (MI355X_MICROARCH.md:
// "other access widths are uncalibrated: calibrate on a known byte count").  A 2 GiB buffer
// (past the 256 MiB Infinity Cache) is read with each pattern once; rocprofv3 --pmc
// FETCH_SIZE per dispatch / the bytes the pattern requests = the counter's tally factor.
//   stream16      every float4 of the buffer, lanes contiguous (the guide's reference case)
//   piece64_s512  the first 64 B of every 512-B row (16 of 128 channels: convt2_narrow's halo)
//   pair64_s512   both 64-B halves of the first 128 B of every 512-B row, by different blocks
//                 8 dispatch slots apart (same XCD)
//   piece64_s16k  the first 64 B of every 16-KB row (bn_bwd_small's new 16-channel blocks)
//   quad16_s16k   the same 64 B read as 4 x 16 B by 4 consecutive blocks (the old 4-channel
//                 bn_bwd_small: neighbouring blocks on different XCDs)
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void stream16(const float4* __restrict__ x, long long n4, float* out) {
  float s = 0.f;
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < n4; i += (long long)gridDim.x * 256) {
    const float4 v = x[i];
    s += v.x + v.y + v.z + v.w;
  }
  if (s == 12345.f) out[0] = s;
}

// rows of `row` floats; block reads floats [c0, c0 + 4 * lanes) of rows; grid = rows / rpb
template <int LANES>
__global__ void pieces(const float* __restrict__ x, long long rows, int row, int cgroups, float* out) {
  // cgroups channel groups of 4*LANES floats; block b -> (row chunk, group) with the group
  // fastest over consecutive blocks (old bn_bwd_small) or 8 apart (same XCD) when cgroups < 0
  const int ng = cgroups < 0 ? -cgroups : cgroups;
  int grp, chunk;
  if (cgroups < 0) { grp = (blockIdx.x / 8) % ng; chunk = (blockIdx.x / (8 * ng)) * 8 + blockIdx.x % 8; }
  else { grp = blockIdx.x % ng; chunk = blockIdx.x / ng; }
  const int q = threadIdx.x % LANES, rl = threadIdx.x / LANES, rpb = 256 / LANES;
  float s = 0.f;
  for (long long r = (long long)chunk * rpb * 16 + rl; r < rows && r < (long long)(chunk + 1) * rpb * 16; r += rpb) {
    const float4 v = *reinterpret_cast<const float4*>(x + r * row + grp * 4 * LANES + 4 * q);
    s += v.x + v.y + v.z + v.w;
  }
  if (s == 12345.f) out[0] = s;
}

int main() {
  const long long bytes = 2LL << 30, n = bytes / 4;
  float *x, *out;
  hipMalloc(&x, bytes);
  hipMalloc(&out, 64);
  hipMemset(x, 0, bytes);
  hipDeviceSynchronize();
  for (int rep = 0; rep < 2; ++rep) {
    stream16<<<4096, 256>>>((const float4*)x, n / 4, out);
    // 512-B rows: n / 128 rows, 16 rows per lane-row chunk
    const long long r512 = n / 128, r16k = n / 4096;
    pieces<4><<<(unsigned)(r512 / (64 * 16)), 256>>>(x, r512, 128, 1, out);        // piece64_s512
    pieces<4><<<(unsigned)(r512 / (64 * 16)) * 2, 256>>>(x, r512, 128, -2, out);   // pair64_s512
    pieces<4><<<(unsigned)(r16k / (64 * 16)), 256>>>(x, r16k, 4096, 1, out);       // piece64_s16k
    pieces<1><<<(unsigned)(r16k / (256 * 16)) * 4, 256>>>(x, r16k, 4096, 4, out);  // quad16_s16k
    hipDeviceSynchronize();
  }
  printf("requested bytes: stream16 %lld, piece64_s512 %lld, pair64_s512 %lld, piece64_s16k %lld, quad16_s16k %lld\n",
         bytes, (n / 128) * 64, (n / 128) * 128, (n / 4096) * 64, (n / 4096) * 64);
  hipFree(x);
  hipFree(out);
  return 0;
}
