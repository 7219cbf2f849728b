// D2H paths for the host API's per-step output (obs | reward | done, ~1.2 MB at 4096 envs):
// copy-engine hipMemcpyAsync into page-locked memory (default / non-coherent), a kernel storing
// straight into the mapped page-locked block, and hipMemcpy into pageable memory.  Median of
// 30 reps each, including the stream synchronisation.
//   hipcc --offload-arch=gfx950 -O2 -o /tmp/d2h tools/d2h_microbench.hip && /tmp/d2h
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <algorithm>
#include <chrono>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

__global__ void store_kernel(const float4* __restrict__ src, float4* dst, size_t n4) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (size_t)gridDim.x * blockDim.x) dst[i] = src[i];
}

template <class F>
double med_us(F f) {
  std::vector<double> t;
  for (int r = 0; r < 33; r++) {
    auto a = std::chrono::steady_clock::now();
    f();
    auto b = std::chrono::steady_clock::now();
    if (r >= 3) t.push_back(std::chrono::duration<double, std::micro>(b - a).count());
  }
  std::sort(t.begin(), t.end());
  return t[t.size() / 2];
}

int main() {
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  const size_t sizes[] = {4096 * 74 * 4, 8192 * 74 * 4, 4096 * 2 * 4};
  for (size_t bytes : sizes) {
    float* d;
    CK(hipMalloc(&d, bytes));
    CK(hipMemset(d, 1, bytes));
    float *h_def, *h_nc, *h_map;
    CK(hipHostMalloc((void**)&h_def, bytes, hipHostMallocDefault));
    CK(hipHostMalloc((void**)&h_nc, bytes, hipHostMallocNonCoherent));
    CK(hipHostMalloc((void**)&h_map, bytes, hipHostMallocMapped));
    float* h_map_dev;
    CK(hipHostGetDevicePointer((void**)&h_map_dev, h_map, 0));
    float* h_page = (float*)malloc(bytes);
    const double t_def = med_us([&] { CK(hipMemcpyAsync(h_def, d, bytes, hipMemcpyDeviceToHost, s)); CK(hipStreamSynchronize(s)); });
    const double t_nc = med_us([&] { CK(hipMemcpyAsync(h_nc, d, bytes, hipMemcpyDeviceToHost, s)); CK(hipStreamSynchronize(s)); });
    const double t_page = med_us([&] { CK(hipMemcpy(h_page, d, bytes, hipMemcpyDeviceToHost)); });
    const size_t n4 = bytes / 16;
    double t_k[4];
    const int grids[4] = {64, 256, 1024, 4096};
    for (int g = 0; g < 4; g++)
      t_k[g] = med_us([&] {
        hipLaunchKernelGGL(store_kernel, dim3(grids[g]), dim3(256), 0, s, (const float4*)d, (float4*)h_map_dev, n4);
        CK(hipStreamSynchronize(s));
      });
    const double t_k_def = med_us([&] {  // the default (non-mapped flag) block through its host pointer
      hipLaunchKernelGGL(store_kernel, dim3(256), dim3(256), 0, s, (const float4*)d, (float4*)h_def, n4);
      CK(hipStreamSynchronize(s));
    });
    const double t_sync = med_us([&] { CK(hipStreamSynchronize(s)); });
    const double t_empty = med_us([&] {
      hipLaunchKernelGGL(store_kernel, dim3(1), dim3(64), 0, s, (const float4*)d, (float4*)d, (size_t)0);
      CK(hipStreamSynchronize(s));
    });
    printf("%8zu B: memcpyAsync->pinned %.1f us (%.1f GB/s) | ->nonCoherent %.1f | hipMemcpy->pageable %.1f | "
           "kernel->mapped grid64 %.1f grid256 %.1f grid1024 %.1f grid4096 %.1f | kernel->default-pinned %.1f | "
           "empty launch+sync %.1f | sync %.1f\n",
           bytes, t_def, bytes / t_def / 1e3, t_nc, t_page, t_k[0], t_k[1], t_k[2], t_k[3], t_k_def, t_empty, t_sync);
    CK(hipFree(d));
    CK(hipHostFree(h_def));
    CK(hipHostFree(h_nc));
    CK(hipHostFree(h_map));
    free(h_page);
  }
  return 0;
}
