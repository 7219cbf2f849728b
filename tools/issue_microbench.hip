// Issue-cost microbenchmark for gfx950 (one wave per SIMD or two): cycles per loop iteration of
// hand-written instruction streams, timed with s_memtime inside the kernel.  Answers which
// instructions cost a wave's issue slots in env_step_kernel's regime: VALU alone, VALU with
// interleaved SALU, VALU with s_nop, and the exec-mask scaffolding of a divergent `if`.
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/issue_mb tools/issue_microbench.hip && /tmp/issue_mb
#include <hip/hip_runtime.h>
#include <cstdio>

#define ITERS 2000

__global__ void k_valu(unsigned long long* out, float x0) {
  float a = x0, b = x0 + 1, c = x0 + 2, d = x0 + 3;
  __syncthreads();
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < ITERS; i++) {
    asm volatile(
        "v_add_f32 %0, %0, 1.0\n v_add_f32 %1, %1, 1.0\n v_add_f32 %2, %2, 1.0\n v_add_f32 %3, %3, 1.0\n"
        "v_add_f32 %0, %0, 1.0\n v_add_f32 %1, %1, 1.0\n v_add_f32 %2, %2, 1.0\n v_add_f32 %3, %3, 1.0\n"
        : "+v"(a), "+v"(b), "+v"(c), "+v"(d));
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) out[blockIdx.x] = t1 - t0;
  if (a + b + c + d == 12345.0f) out[0] = 0;
}

__global__ void k_valu_salu(unsigned long long* out, float x0) {
  float a = x0, b = x0 + 1, c = x0 + 2, d = x0 + 3;
  int s0 = 0, s1 = 1, s2 = 2, s3 = 3;
  __syncthreads();
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < ITERS; i++) {
    asm volatile(
        "v_add_f32 %0, %0, 1.0\n s_movk_i32 %4, 0x11\n v_add_f32 %1, %1, 1.0\n s_movk_i32 %5, 0x12\n"
        "v_add_f32 %2, %2, 1.0\n s_movk_i32 %6, 0x13\n v_add_f32 %3, %3, 1.0\n s_movk_i32 %7, 0x14\n"
        "v_add_f32 %0, %0, 1.0\n s_movk_i32 %4, 0x21\n v_add_f32 %1, %1, 1.0\n s_movk_i32 %5, 0x22\n"
        "v_add_f32 %2, %2, 1.0\n s_movk_i32 %6, 0x23\n v_add_f32 %3, %3, 1.0\n s_movk_i32 %7, 0x24\n"
        : "+v"(a), "+v"(b), "+v"(c), "+v"(d), "+s"(s0), "+s"(s1), "+s"(s2), "+s"(s3));
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) out[blockIdx.x] = t1 - t0;
  if (a + b + c + d + s0 + s1 + s2 + s3 == 12345.0f) out[0] = 0;
}

__global__ void k_valu_nop(unsigned long long* out, float x0) {
  float a = x0, b = x0 + 1, c = x0 + 2, d = x0 + 3;
  __syncthreads();
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < ITERS; i++) {
    asm volatile(
        "v_add_f32 %0, %0, 1.0\n s_nop 0\n v_add_f32 %1, %1, 1.0\n s_nop 0\n"
        "v_add_f32 %2, %2, 1.0\n s_nop 0\n v_add_f32 %3, %3, 1.0\n s_nop 0\n"
        "v_add_f32 %0, %0, 1.0\n s_nop 0\n v_add_f32 %1, %1, 1.0\n s_nop 0\n"
        "v_add_f32 %2, %2, 1.0\n s_nop 0\n v_add_f32 %3, %3, 1.0\n s_nop 0\n"
        : "+v"(a), "+v"(b), "+v"(c), "+v"(d));
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) out[blockIdx.x] = t1 - t0;
  if (a + b + c + d == 12345.0f) out[0] = 0;
}

// the scaffolding of `if (lane < k) { v += 1 }`: compare, save exec, skip-branch, body, restore
__global__ void k_valu_ifs(unsigned long long* out, float x0) {
  float a = x0, b = x0 + 1, c = x0 + 2, d = x0 + 3;
  const int lane = threadIdx.x;
  __syncthreads();
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < ITERS; i++) {
    asm volatile(
        "v_cmp_gt_u32 vcc, 18, %4\n s_and_saveexec_b64 s[20:21], vcc\n s_cbranch_execz 1f\n"
        "v_add_f32 %0, %0, 1.0\n v_add_f32 %1, %1, 1.0\n"
        "1:\n s_or_b64 exec, exec, s[20:21]\n"
        "v_cmp_gt_u32 vcc, 18, %4\n s_and_saveexec_b64 s[20:21], vcc\n s_cbranch_execz 2f\n"
        "v_add_f32 %2, %2, 1.0\n v_add_f32 %3, %3, 1.0\n"
        "2:\n s_or_b64 exec, exec, s[20:21]\n"
        "v_add_f32 %0, %0, 1.0\n v_add_f32 %1, %1, 1.0\n v_add_f32 %2, %2, 1.0\n v_add_f32 %3, %3, 1.0\n"
        : "+v"(a), "+v"(b), "+v"(c), "+v"(d)
        : "v"(lane)
        : "vcc", "s20", "s21", "scc");
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) out[blockIdx.x] = t1 - t0;
  if (a + b + c + d == 12345.0f) out[0] = 0;
}


// the same without the skip branch: compare, save exec, body, restore
__global__ void k_ifs_nobranch(unsigned long long* out, float x0) {
  float a = x0, b = x0 + 1, c = x0 + 2, d = x0 + 3;
  const int lane = threadIdx.x;
  __syncthreads();
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < ITERS; i++) {
    asm volatile(
        "v_cmp_gt_u32 vcc, 18, %4\n s_and_saveexec_b64 s[20:21], vcc\n"
        "v_add_f32 %0, %0, 1.0\n v_add_f32 %1, %1, 1.0\n"
        "s_or_b64 exec, exec, s[20:21]\n"
        "v_cmp_gt_u32 vcc, 18, %4\n s_and_saveexec_b64 s[20:21], vcc\n"
        "v_add_f32 %2, %2, 1.0\n v_add_f32 %3, %3, 1.0\n"
        "s_or_b64 exec, exec, s[20:21]\n"
        "v_add_f32 %0, %0, 1.0\n v_add_f32 %1, %1, 1.0\n v_add_f32 %2, %2, 1.0\n v_add_f32 %3, %3, 1.0\n"
        : "+v"(a), "+v"(b), "+v"(c), "+v"(d)
        : "v"(lane)
        : "vcc", "s20", "s21", "scc");
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) out[blockIdx.x] = t1 - t0;
  if (a + b + c + d == 12345.0f) out[0] = 0;
}

// only the (never taken) skip branches
__global__ void k_branch_only(unsigned long long* out, float x0) {
  float a = x0, b = x0 + 1, c = x0 + 2, d = x0 + 3;
  __syncthreads();
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < ITERS; i++) {
    asm volatile(
        "s_cbranch_execz 1f\n v_add_f32 %0, %0, 1.0\n v_add_f32 %1, %1, 1.0\n 1:\n"
        "s_cbranch_execz 2f\n v_add_f32 %2, %2, 1.0\n v_add_f32 %3, %3, 1.0\n 2:\n"
        "v_add_f32 %0, %0, 1.0\n v_add_f32 %1, %1, 1.0\n v_add_f32 %2, %2, 1.0\n v_add_f32 %3, %3, 1.0\n"
        : "+v"(a), "+v"(b), "+v"(c), "+v"(d));
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) out[blockIdx.x] = t1 - t0;
  if (a + b + c + d == 12345.0f) out[0] = 0;
}

// the select form of the same two guarded updates: compare, then v_cndmask per output
__global__ void k_select(unsigned long long* out, float x0) {
  float a = x0, b = x0 + 1, c = x0 + 2, d = x0 + 3;
  const int lane = threadIdx.x;
  __syncthreads();
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < ITERS; i++) {
    asm volatile(
        "v_cmp_gt_u32 s[20:21], 18, %4\n v_add_f32 v250, %0, 1.0\n v_add_f32 v251, %1, 1.0\n"
        "v_add_f32 v252, %2, 1.0\n v_add_f32 v253, %3, 1.0\n"
        "v_cndmask_b32 %0, %0, v250, s[20:21]\n v_cndmask_b32 %1, %1, v251, s[20:21]\n"
        "v_cndmask_b32 %2, %2, v252, s[20:21]\n v_cndmask_b32 %3, %3, v253, s[20:21]\n"
        "v_add_f32 %0, %0, 1.0\n v_add_f32 %1, %1, 1.0\n v_add_f32 %2, %2, 1.0\n v_add_f32 %3, %3, 1.0\n"
        : "+v"(a), "+v"(b), "+v"(c), "+v"(d)
        : "v"(lane)
        : "s20", "s21", "v250", "v251", "v252", "v253");
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) out[blockIdx.x] = t1 - t0;
  if (a + b + c + d == 12345.0f) out[0] = 0;
}

// dependent LDS round trips: ds_write then ds_read of another lane's word, waited each time
__global__ void k_lds_chain(unsigned long long* out, float x0) {
  __shared__ float buf[64];
  float a = x0;
  const int lane = threadIdx.x;
  __syncthreads();
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < ITERS / 8; i++) {
    buf[lane] = a;
    asm volatile("" ::: "memory");
    a = buf[(lane + 1) & 63] + 1.0f;
    asm volatile("" ::: "memory");
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) out[blockIdx.x] = t1 - t0;
  if (a == 12345.0f) out[0] = 0;
}

static void run(const char* name, void (*k)(unsigned long long*, float), int waves_per_simd, double instrs_per_iter,
                int iters) {
  // one workgroup of 64 threads per SIMD slot: 1024 SIMDs x waves_per_simd (the chip is 256 CUs x 4 SIMDs)
  const int nblk = 1024 * waves_per_simd;
  unsigned long long* d;
  (void)hipMalloc(&d, sizeof(unsigned long long) * nblk);
  hipLaunchKernelGGL(k, dim3(nblk), dim3(64), 0, 0, d, 0.5f);  // warm-up
  hipLaunchKernelGGL(k, dim3(nblk), dim3(64), 0, 0, d, 0.5f);
  (void)hipDeviceSynchronize();
  unsigned long long h[8192];
  (void)hipMemcpy(h, d, sizeof(unsigned long long) * nblk, hipMemcpyDeviceToHost);
  double m = 0;
  for (int i = 0; i < nblk; i++) m += (double)h[i];
  m /= nblk;
  fflush(stdout);
  printf("%-14s waves/SIMD %d: %8.1f cycles/iter, %5.2f cycles/instr (%g instrs/iter)\n", name, waves_per_simd, m / iters,
         m / iters / instrs_per_iter, instrs_per_iter);
  fflush(stdout);
  (void)hipFree(d);
}

int main() {
  for (int w = 1; w <= 2; w++) {
    run("valu", k_valu, w, 8, ITERS);
    run("valu+salu", k_valu_salu, w, 16, ITERS);
    run("valu+nop", k_valu_nop, w, 16, ITERS);
    run("valu+ifs", k_valu_ifs, w, 16, ITERS);
    run("ifs_nobranch", k_ifs_nobranch, w, 14, ITERS);
    run("branch_only", k_branch_only, w, 10, ITERS);
    run("select", k_select, w, 13, ITERS);
    run("lds_chain", k_lds_chain, w, 1, ITERS / 8);
  }
  return 0;
}
