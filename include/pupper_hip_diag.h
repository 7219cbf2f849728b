/*
 * pupper_hip_diag.h -- diagnostic entry points of libpupper_hip.so (not part of the drop-in
 * boundary in pupper_hip.h; nothing on the env path calls them).  They read the per-phase and
 * per-wave shader-clock records of a library built with -DPP3_PHASE_PROF (`make prof`, used by
 * tests/diag_phases.py and tests/diag_waves_fused.py); the production library exports them only
 * to return PP3_ERR_ARG, and a diagnostic library refuses pp3_create unless PP3_ALLOW_DIAG_BUILD
 * is set.
 */
#ifndef PUPPER_HIP_DIAG_H_
#define PUPPER_HIP_DIAG_H_

#include <stdint.h>

#include "pupper_hip.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Diagnostic build only (-DPP3_PHASE_PROF): per-phase shader-clock totals of env_step_kernel
 * summed over envs (n <= 16 slots); returns PP3_ERR_ARG in the production build. */
int pp3_phase_profile(uint64_t* host_out, int32_t n, int32_t reset);

/* Diagnostic builds only: per-wave record of the last env-step launch, 288 words per wave (lifetime
 * cycles, dense-Hessian substeps, max contacts, line-search evaluations, start and end stamps,
 * HW_ID, XCC_ID, then 19 per-phase cycle counts, contacts summed over substeps, substeps that
 * used the second constraint-row slot, s_memrealtime (100 MHz) at start and end, 1 unused; then 128 phase stamps and their 128 phase ids). */
int pp3_wave_profile(uint32_t* host_out, int32_t n);

/* Which path pp3_rollout_policy takes on env `e`: 1 = ONE fused launch for the K steps
 * (env_step_kernel<8, true, 8>), 0 = per-step policy + step launches (max_contacts = 16,
 * action_repeat > 1, PP3_POLICY_UNFUSED=1, or a diagnostic build), -1 = null handle.  bench.py
 * labels its policy roofline with it. */
int32_t pp3_rollout_policy_fused(const pp3_env_t* e);

/* Whether env `e`'s step kernels cull the narrow phase's sphere-box pairs by box (1: the model has
 * 1..32 obstacle boxes and at most 160 candidate pairs -- 16 boxes for the Pupper's 8 spheres --, the launches
 * are env_step_kernel<..., CULL = true>; 0: every pair is evaluated, e.g. a flat model or
 * PP3_NO_CULL=1 at creation), -1 = null handle.  The cull is exact (tests/test_gpu_cull.py). */
int32_t pp3_narrow_cull(const pp3_env_t* e);

#ifdef __cplusplus
}
#endif
#endif /* PUPPER_HIP_DIAG_H_ */
