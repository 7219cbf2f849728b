// pp3_diag.h -- diagnostic-build hooks of env_step_kernel (never part of the product library).
//
// The product target (`make`, libpupper_hip.so) defines none of the macros below, so every hook
// compiles to nothing.  `make prof` (-DPP3_PHASE_PROF -> libpupper_hip_prof.so) and `make debug`
// (-DPP3_DEBUG -> libpupper_hip_dbg.so) build separate libraries for tests/diag_*.py and the
// tools/ scripts, and `make loopback` (-DPP3_TEST_RCCL_SONAME -> tests/loopback/) the multi-rank
// test build whose collectives go through the loopback test transport; pp3_create refuses to run
// from any of them unless the caller opts in with PP3_ALLOW_DIAG_BUILD=1 (pp3_env.hip), so a
// stray -D can never pass for the product.
#pragma once

#include "pupper_hip_diag.h"  // the C declarations of the diagnostic entry points

#if defined(PP3_PHASE_PROF) || defined(PP3_DEBUG) || defined(PP3_TEST_RCCL_SONAME)
#define PP3_DIAG_BUILD 1
#else
#define PP3_DIAG_BUILD 0
#endif

namespace pp3 {

// Diagnostic build only (-DPP3_PHASE_PROF): per-phase shader-cycle deltas summed over all
// waves.  A stamp is one s_memtime (its lgkmcnt wait drains the LDS reads in flight) and two VALU:
// lane k of a per-wave register accumulates phase k's cycles, one global atomic per lane at the
// end of the launch (gfx950 has no SHADER_CYCLES hwreg).
#ifdef PP3_PHASE_PROF
constexpr int NPROF = 25;  // 0..18 phase cycles, 19 line-search evaluations per wave (max of its two envs), 20 per env,
                           // 21..23 sub-phase cycles (line-search setup, Newton row update, warm-start row costs)
struct Prof {
  uint32_t t, acc;
  uint32_t t0, dense, ncmax, evals;  // per wave: start stamp, dense-Hessian substeps, max contacts, line-search evaluations
  uint32_t csum, slot2;               // contacts summed over substeps (max of the two envs), substeps using row slot 1
  uint32_t n, tr0, tr1, k0, k1;       // stamp trace: stamp i held by lane i % 64 in tr{i / 64}, its phase in k{i / 64}
};
constexpr int MAXWAVE = 16384;
constexpr int NTRACE = 128;
constexpr int WREC = 32 + 2 * NTRACE;  // + the stamp trace (stamps, then phase ids; 0xffffffff = unused)
__device__ uint32_t g_wave[MAXWAVE][WREC];  // last launch: lifetime cycles, dense substeps, max ncon, evaluations,
                                            // start stamp, end stamp, HW_ID, XCC_ID, 8..26 the wave's cycles
                                            // per phase, 27 csum, 28 slot2, 29/30 s_memrealtime at start/end
// per-wave slots summed on the host: no contended device-scope atomics at wave exit (45 k atomics
// on 22 addresses clogged the memory path that the remaining waves' scalar loads share, and
// stalled them by 20-80 k cycles: tools/wave_trace.py)
__device__ unsigned long long g_prof[MAXWAVE][NPROF];
__device__ __forceinline__ uint32_t shader_cycles() { return (uint32_t)__builtin_amdgcn_s_memtime(); }
#define PROF_PARAM , Prof* pf
#define PROF_ARG , pf
#define PROF_NULL , (Prof*)nullptr
#define PROF_ADD(k, v) do { if (pf) pf->acc += ((int)(threadIdx.x) == (k)) ? (uint32_t)(v) : 0u; } while (0)
#define PHASE(k)                                                            \
  do {                                                                      \
    if (pf) {                                                               \
      asm volatile("; PP3PHASE " #k);                                       \
      const uint32_t t_ = shader_cycles();                                  \
      pf->acc += ((int)(threadIdx.x) == (k)) ? (t_ - pf->t) : 0u;         \
      pf->t = t_;                                                           \
      const uint32_t i_ = pf->n++;                                          \
      if ((i_ & 63u) == (threadIdx.x & 63u)) {                              \
        if (i_ < 64u) { pf->tr0 = t_; pf->k0 = (k); }                        \
        else if (i_ < 128u) { pf->tr1 = t_; pf->k1 = (k); }                  \
      }                                                                     \
    }                                                                       \
  } while (0)
#else
#define PROF_PARAM
#define PROF_ARG
#define PROF_NULL
#define PROF_ADD(k, v) do { } while (0)
#define PHASE(k) do { } while (0)
#endif

#ifdef PP3_DEBUG
__device__ float g_dbg[512];  // last Newton iteration of env 0 (debug build only)
#endif

}  // namespace pp3
