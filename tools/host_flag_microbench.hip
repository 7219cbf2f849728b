// Host wait latency after a launch that stores its outputs into page-locked host memory (the host
// policy loop's step): the HIP waits (hipStreamSynchronize / hipEventSynchronize) against a spin on
// a page-locked flag that the launch's last workgroup stores after every workgroup's output stores
// are released at system scope.  Also checks, every launch, that all outputs are visible when the
// flag is.   hipcc --offload-arch=gfx950 -O2 -o tools/bin/host_flag_mb tools/host_flag_microbench.hip
#include <hip/hip_runtime.h>
#include <immintrin.h>
#include <chrono>
#include <cstdio>

constexpr int NBLK = 2048, PAYLOAD = 150;  // 2048 two-env waves x 600 B ~ the 4096-env obs rows

constexpr int STATE = 512;  // floats of device-memory state each workgroup rewrites (dirty L2 lines)

template <int MODE>
__global__ void step_like(unsigned long long cycles, float* out, float* state, unsigned epoch, unsigned* counter,
                          unsigned* flag) {
  const unsigned long long t0 = __builtin_readcyclecounter();
  while (__builtin_readcyclecounter() - t0 < cycles) {
  }
  for (int i = threadIdx.x; i < STATE; i += 64) state[blockIdx.x * STATE + i] += 1.0f;
  for (int i = threadIdx.x; i < PAYLOAD; i += 64) out[blockIdx.x * PAYLOAD + i] = (float)epoch;
  if (MODE == 1) {
    // every wave's stores released at system scope (an L2 write-back per wave), then the last
    // workgroup in publishes
    __atomic_thread_fence(__ATOMIC_RELEASE);
    if (threadIdx.x == 0) {
      const unsigned old = __hip_atomic_fetch_add(counter, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_SYSTEM);
      if (old == epoch * NBLK - 1) __hip_atomic_store(flag, epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  } else if (MODE == 2) {
    // the page-locked stores bypass L2: each wave only waits for its own stores' completion
    // (workgroup-scope release), counts in at agent scope; the last wave publishes at system scope
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    if (threadIdx.x == 0) {
      const unsigned old = __hip_atomic_fetch_add(counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (old == epoch * NBLK - 1) __hip_atomic_store(flag, epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
}

int main() {
  hipStream_t s;
  hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  hipEvent_t ev;
  hipEventCreateWithFlags(&ev, hipEventDisableTiming);
  float* out;
  unsigned *flag, *counter;
  hipHostMalloc((void**)&out, sizeof(float) * NBLK * PAYLOAD, 0);
  hipHostMalloc((void**)&flag, 64, 0);
  hipMalloc((void**)&counter, 4);
  float* state;
  hipMalloc((void**)&state, sizeof(float) * NBLK * STATE);
  hipMemset(state, 0, sizeof(float) * NBLK * STATE);
  const int N = 300;
  for (const unsigned long long cyc : {1000ull, 100000ull}) {
    for (int method = 0; method < 4; method++) {
      hipMemset(counter, 0, 4);
      *(volatile unsigned*)flag = 0;
      hipDeviceSynchronize();
      unsigned epoch = 0;
      long bad = 0;
      double us = 0;
      for (int rep = 0; rep < 2; rep++) {  // rep 0: warm-up
        auto t0 = std::chrono::high_resolution_clock::now();
        for (int i = 0; i < N; i++) {
          ++epoch;
          if (method < 2) hipLaunchKernelGGL(step_like<0>, dim3(NBLK), dim3(64), 0, s, cyc, out, state, epoch, counter, flag);
          else if (method == 2) hipLaunchKernelGGL(step_like<1>, dim3(NBLK), dim3(64), 0, s, cyc, out, state, epoch, counter, flag);
          else hipLaunchKernelGGL(step_like<2>, dim3(NBLK), dim3(64), 0, s, cyc, out, state, epoch, counter, flag);
          if (method == 0) {
            hipStreamSynchronize(s);
          } else if (method == 1) {
            hipEventRecord(ev, s);
            hipEventSynchronize(ev);
          } else {
            const auto ts = std::chrono::steady_clock::now();
            while (__atomic_load_n((volatile unsigned*)flag, __ATOMIC_ACQUIRE) != epoch) {
              _mm_pause();
              if (std::chrono::steady_clock::now() - ts > std::chrono::seconds(1)) {
                printf("flag wait timed out at epoch %u (flag %u)\n", epoch, *(volatile unsigned*)flag);
                hipStreamSynchronize(s);
                return 1;
              }
            }
          }
          // the outputs are all visible now
          for (int b = 0; b < NBLK; b += 7)
            if (((volatile float*)out)[b * PAYLOAD + PAYLOAD - 1] != (float)epoch) bad++;
        }
        auto t1 = std::chrono::high_resolution_clock::now();
        us = std::chrono::duration<double, std::micro>(t1 - t0).count() / N;
      }
      hipStreamSynchronize(s);
      printf("spin %6llu cycles  %-22s %7.1f us per launch + wait   (stale outputs seen: %ld)\n", cyc,
             method == 0 ? "hipStreamSynchronize" : method == 1 ? "hipEventSynchronize" : method == 2 ? "flag, system fences" : "flag, wave fences", us, bad);
    }
    hipDeviceSynchronize();
    auto t0 = std::chrono::high_resolution_clock::now();
    for (int i = 0; i < N; i++) hipLaunchKernelGGL(step_like<0>, dim3(NBLK), dim3(64), 0, s, cyc, out, state, 0u, counter, flag);
    hipStreamSynchronize(s);
    auto t1 = std::chrono::high_resolution_clock::now();
    printf("spin %6llu cycles  back to back           %7.1f us per launch\n", cyc,
           std::chrono::duration<double, std::micro>(t1 - t0).count() / N);
  }
  return 0;
}
