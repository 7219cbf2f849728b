// Bit-identity of pp3_device.h sincos_f32 with the device library's sincosf (|x| < 2^17): N
// arguments spread over [-2^17, 2^17] plus a dense sweep of [-8, 8] and the specials.
//   hipcc --offload-arch=gfx950 -O3 -I include -fno-hip-fp32-correctly-rounded-divide-sqrt \
//     -fgpu-flush-denormals-to-zero -o tools/bin/sincos_check tools/sincos_check.hip
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>
#include <string.h>
#include "../pupperv3-mjx_amd/csrc/pp3_device.h"

__global__ void check(long n, unsigned long long* bad, float* first) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float x;
  if (i < n / 2) {
    x = -8.0f + 16.0f * (float)i / (float)(n / 2);                  // dense small angles
  } else {
    const uint32_t h = (uint32_t)(i * 2654435761u) ^ (uint32_t)(i >> 7);
    x = __uint_as_float((h & 0x807fffffu) | ((100u + (h >> 24) % 44u) << 23));  // |x| up to ~2^16
  }
  if (i == 0) x = 0.0f;
  if (i == 1) x = -0.0f;
  if (i == 2) x = INFINITY;
  if (i == 3) x = NAN;
  if (i == 4) x = 131071.9f;
  float s0, c0, s1, c1;
  sincosf(x, &s0, &c0);
  pp3::sincos_f32(x, &s1, &c1);
  const bool same = (__float_as_uint(s0) == __float_as_uint(s1) || (isnan(s0) && isnan(s1))) &&
                    (__float_as_uint(c0) == __float_as_uint(c1) || (isnan(c0) && isnan(c1)));
  if (!same) {
    const unsigned long long k = atomicAdd(bad, 1ull);
    if (k == 0) { first[0] = x; first[1] = s0; first[2] = s1; first[3] = c0; first[4] = c1; }
  }
}

int main() {
  const long n = 1L << 26;
  unsigned long long* bad;
  float* first;
  hipMalloc(&bad, 8);
  hipMalloc(&first, 5 * 4);
  hipMemset(bad, 0, 8);
  hipLaunchKernelGGL(check, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, 0, n, bad, first);
  unsigned long long hb = 0;
  float hf[5] = {0};
  hipMemcpy(&hb, bad, 8, hipMemcpyDeviceToHost);
  hipMemcpy(hf, first, 20, hipMemcpyDeviceToHost);
  printf("sincos_f32 vs sincosf: %llu mismatches of %ld arguments\n", hb, n);
  if (hb) printf("first: x=%a sin %a / %a cos %a / %a\n", hf[0], hf[1], hf[2], hf[3], hf[4]);
  return hb != 0;
}
