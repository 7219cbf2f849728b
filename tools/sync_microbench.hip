// Host wait latency after a short kernel (the host-policy loop's per-step round trip): launch a
// ~100 us spin kernel, then wait by hipStreamSynchronize / hipEventSynchronize / a hipEventQuery
// spin; reports the mean round trip per method.   hipcc --offload-arch=gfx950 -O2 -o /tmp/syncmb tools/sync_microbench.hip
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>

__global__ void spin_kernel(unsigned long long cycles, int* out) {
  const unsigned long long t0 = __builtin_readcyclecounter();
  while (__builtin_readcyclecounter() - t0 < cycles) {
  }
  if (threadIdx.x == 0 && blockIdx.x == 0) out[0] = 1;
}

int main() {
  hipStream_t s;
  hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  hipEvent_t ev;
  hipEventCreateWithFlags(&ev, hipEventDisableTiming);
  int* d;
  hipMalloc(&d, 4);
  const unsigned long long cyc = 100000;  // s_memtime-rate cycles
  const int N = 300;
  for (int method = 0; method < 3; method++) {
    for (int w = 0; w < 20; w++) {
      hipLaunchKernelGGL(spin_kernel, dim3(1024), dim3(64), 0, s, cyc, d);
      hipStreamSynchronize(s);
    }
    auto t0 = std::chrono::high_resolution_clock::now();
    for (int i = 0; i < N; i++) {
      hipLaunchKernelGGL(spin_kernel, dim3(1024), dim3(64), 0, s, cyc, d);
      if (method == 0) {
        hipStreamSynchronize(s);
      } else {
        hipEventRecord(ev, s);
        if (method == 1) hipEventSynchronize(ev);
        else
          while (hipEventQuery(ev) == hipErrorNotReady) {
          }
      }
    }
    auto t1 = std::chrono::high_resolution_clock::now();
    const double us = std::chrono::duration<double, std::micro>(t1 - t0).count() / N;
    printf("%s: %.1f us per launch + wait\n", method == 0 ? "hipStreamSynchronize" : (method == 1 ? "hipEventSynchronize" : "hipEventQuery spin"), us);
  }
  // the kernel alone, back to back
  auto t0 = std::chrono::high_resolution_clock::now();
  for (int i = 0; i < N; i++) hipLaunchKernelGGL(spin_kernel, dim3(1024), dim3(64), 0, s, cyc, d);
  hipStreamSynchronize(s);
  auto t1 = std::chrono::high_resolution_clock::now();
  printf("back to back: %.1f us per launch\n", std::chrono::duration<double, std::micro>(t1 - t0).count() / N);
  return 0;
}
