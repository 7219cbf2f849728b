// pp3_env.hip -- MI355X (gfx950) kernels for the Pupper-v3 environment hot path.
//
// TWO environments per 64-lane wavefront: lanes 0..31 own env 2b, lanes 32..63 own env
// 2b+1 (workgroup b = one wave).  The whole env step of PupperV3Env.step
// (environment.py:348-483) runs in ONE launch: RNG/kick/latency prologue, n_frames (=5)
// MuJoCo-semantics physics substeps (kinematics, CRB mass matrix, collision, pyramidal
// contact + frictionloss + limit constraints, RNE, Newton solve with exact line search,
// Euler), then the observation/reward/termination epilogue.
//
// Why two per wave: the kernel is VALU-issue bound (rocprofv3: SQ_WAVE_CYCLES ~= 4 waves x
// SQ_INSTS_VALU x 4 cycles) and almost every phase needs <= 32 lanes per env (13 bodies,
// 18 dofs, 32 candidate pairs, <= 3 constraint rows per lane), so packing two envs into one
// wave halves the VALU instructions per env.  Per-env state lives in LDS for the whole
// launch (~10 KB per env, 8 waves = 16 envs per CU); HBM sees one read and one write of
// each env's state record per env step.  18x18 LDL^T runs one matrix row per lane with the
// pivot column broadcast through LDS; half-wave reductions run on the DPP network.
#include <hip/hip_runtime.h>

#include <float.h>
#include <math.h>
#include <stddef.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <string>
#include <algorithm>
#include <vector>

#include "pp3_device.h"
#include "pp3_diag.h"
#include "pp3_mlp.h"

namespace pp3 {

constexpr int HW = 32;      // lanes per environment (half wave)
typedef __attribute__((address_space(4))) const DevModel GModel;  // DevModel: read-only (constant AS)
typedef __attribute__((address_space(4))) const float GFloat;
constexpr int HMAX = 16;    // observation_history limit
constexpr int OBS_MOVE = (PP3_OBS_DIM * (HMAX - 1) + HW - 1) / HW;
constexpr int NROBOT_GEOM = 8;  // collidable spheres on moving bodies (LDS table)
constexpr int NHIT = 64;        // contact-overflow ranking window (hits kept for ranking)
constexpr float CULL_SLACK = 0.05f;  // collision's cached near-box mask: re-tested after body 1 moves this far (m)
constexpr float LS_NOISE = 64.0f;  // line-search convergence floor, in roundoffs of alpha (oracle LS_NOISE)

// Phase-local scratch that never lives across a phase boundary it does not own.
template <int NC>
union alignas(16) Scratch {
  float xipos[NB][3];      // phase 1 (kinematics) -> phase 2 (com_pos)
  struct {                 // phases 3-4
    float F[NV][6];        // crb*cdof -> M entries
    float cacc[NB][6];     // rne chain -> body forces (overwritten in place by cfrc)
    float hit_dist[NHIT];  // collision overflow ranking
    int hit_pair[NHIT];
    float con_pos[NC][3];  // collision -> contact Jacobians
    float con_frame[NC][9];
  } a;
  float L[NV][NV + 1];     // LDL pivot column (row 0) / transposed factor, phases 5-7
  struct {                 // env prologue / epilogue
    float u[40];
    float o[PP3_OBS_DIM];
    float rw[PP3_NREWARD];
    float xdv[NB][3], xda[NB][3];
    int contact[4], filt_mm[4], filt_cm[4];
    float first[4];
    int done;
    float knee, bodyc;
  } e;
};

template <int NC>
struct alignas(16) Shared {
  static constexpr int NEFC = NFR + NLMAX + 4 * NC;
  float qpos[20], qvel[20], qws[20], qacc[20], ctrl[12];
  float st[PP3_S_ACT_BUF];  // head of the state record (latency buffers stay in HBM)
  // per-env dynamic parameters (domain randomisation)
  float mass[NB], inertia[NB][3], ipos[NB][3];
  float fric, kp, kd;
  int dr_on;
  float ep[PP3_EP_STRIDE], ep_prev_done;  // auto-reset mode: episode record, previous done
  float ep_racc;                          // action repeat: the reward summed over this step's earlier repeats
  // kinematics / dynamics of the current substep (the last one feeds the epilogue)
  float xpos[NB][3], xquat[NB][4], xaxis[NJ][3];
  float com[4];
  float cinert[NB][10];
  float crb_base[10], cfrc_base[6];  // root-subtree sums (half-wave reductions)
  float cdof[NV][6];
  float cvel[NB][6];
  float M[NV][NV + 1];
  float gxpos[NROBOT_GEOM][3];
  float foot_xpos[4][3];
  alignas(16) float search[20];  // (read as b128 words by mrow_dot_reg)
  float qfrc_smooth[NV], qfrc_act[NV], qacc_smooth[NV], grad[NV], dofD[NV];
  // contacts
  int ncon, nhit, nl;
  int con_pair[NC], con_sup[NC];
  uint32_t con_dm[NC][2];  // dof masks of the contact's two bodies
  float con_dist[NC], con_mu[NC];
  float con_G[NC][5];
  float Jc[NC][3][NV];
  // constraint rows
  int lim_dof[NLMAX];
  float lim_sgn[NLMAX];
  float efc_D[NEFC], efc_R[NEFC], efc_aref[NEFC], efc_force[NEFC];
  Scratch<NC> x;
};

// A workgroup is ONE wave and LDS executes a wave's instructions in issue order, so a lane's
// LDS store is visible to every later LDS load of the same wave: phase boundaries only need to
// stop the compiler from reordering LDS accesses across them.  (__syncthreads would also
// drain outstanding global loads, s_waitcnt vmcnt(0), and serialise the LDS queue.)
#define SYNC() asm volatile("" ::: "memory")
typedef float v4f __attribute__((ext_vector_type(4)));
// Forces every listed value into a VGPR at this point: the loads feeding them are issued
// together ahead of it and retired by one vmcnt wait, instead of each load being placed (and
// waited for) right before its first use.
#define PIN(...) asm volatile("" : __VA_ARGS__)
// a record of N 16-byte word groups, group k at p + k * STRIDE floats: N loads issued back to
// back, pinned together
template <int N, int STRIDE>
__device__ __forceinline__ LaneRec<N> fetch_groups(const float* p) {
  v4f v[N];
#pragma unroll
  for (int k = 0; k < N; k++) v[k] = *reinterpret_cast<const v4f*>(p + k * STRIDE);
  if constexpr (N == 1) PIN("+v"(v[0]));
  else if constexpr (N == 2) PIN("+v"(v[0]), "+v"(v[1]));
  else if constexpr (N == 3) PIN("+v"(v[0]), "+v"(v[1]), "+v"(v[2]));
  else if constexpr (N == 4) PIN("+v"(v[0]), "+v"(v[1]), "+v"(v[2]), "+v"(v[3]));
  else if constexpr (N == 7) PIN("+v"(v[0]), "+v"(v[1]), "+v"(v[2]), "+v"(v[3]), "+v"(v[4]), "+v"(v[5]), "+v"(v[6]));
  else static_assert(N == 1, "fetch_rec: add a PIN arity");
  LaneRec<N> r;
#pragma unroll
  for (int k = 0; k < N; k++)
#pragma unroll
    for (int c = 0; c < 4; c++) r.f[4 * k + c] = v[k][c];
  return r;
}
// a contiguous record (indexed by pair: PairCon)
template <int N>
__device__ __forceinline__ LaneRec<N> fetch_rec(const LaneRec<N>& src) {
  return fetch_groups<N, 4>(src.f);
}
// lane l's phase record from a word-group-major table
template <int N>
__device__ __forceinline__ LaneRec<N> fetch_rec(const LaneTab<N>& t, int l) {
  return fetch_groups<N, 4 * 32>(t.g[0][l]);
}
__device__ __forceinline__ int as_i(float f) { return __float_as_int(f); }

__device__ __forceinline__ float frcp(float x) { return __builtin_amdgcn_rcpf(x); }
// lane i <- i-4 (row); lanes 0..3 of a row read 0 (bound_ctrl): every caller selects its own value
// there, and with no old value to keep the shift is one v_mov_dpp instead of a copy plus the DPP
__device__ __forceinline__ float dpp_shr4(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x114, 0xF, 0xF, true));
}

// wave priority by load (env_step_kernel): the contact weight (contacts of the busier env of the
// wave, +2 on the leg-leg Newton path) from which a wave takes the upper priority pair
constexpr int HEAVY_WEIGHT = 5;

// ---------------------------- half-wave primitives ----------------------------
// value of lane k of this lane's half (k compile-time or wave-uniform)
__device__ __forceinline__ float hb(float v, int k, int h) {
  const float a = rlane(v, k), b = rlane(v, k + HW);
  return h ? b : a;
}
__device__ __forceinline__ uint32_t hbu(uint32_t v, int k, int h) {
  const uint32_t a = (uint32_t)__builtin_amdgcn_readlane((int)v, k);
  const uint32_t b = (uint32_t)__builtin_amdgcn_readlane((int)v, k + HW);
  return h ? b : a;
}
__device__ __forceinline__ Key hkey(Key k, int l, int h) { return Key{hbu(k.a, l, h), hbu(k.b, l, h)}; }
// sum over the 32 lanes of this lane's half, left in every lane: DPP butterflies give each
// 16-lane row its sum, then v_permlane16_swap (gfx950) pairs row 0 with row 1 and row 2 with
// row 3.  No SGPR round trip, so no readlane hazard stalls.
__device__ __forceinline__ float hsum(float v, int) {
  v += dpp_f<0xB1, 0xF>(v, 0.0f);   // quad_perm [1,0,3,2]
  v += dpp_f<0x4E, 0xF>(v, 0.0f);   // quad_perm [2,3,0,1]
  v += dpp_f<0x141, 0xF>(v, 0.0f);  // row_half_mirror
  v += dpp_f<0x140, 0xF>(v, 0.0f);  // row_mirror
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
// the same sum, wanted in ONE lane per half (a value the half then stores): after the row
// butterflies, row_bcast:15 adds row 0's sum into row 1 and row 2's into row 3, so lane 16 of each
// half (rows 1 and 3) holds R0 + R1 -- the sum hsum leaves there too (fp add commutes) -- without
// the copy, the wait states and the swap of the full broadcast
__device__ __forceinline__ float hsum_lane16(float v) {
  v += dpp_f<0xB1, 0xF>(v, 0.0f);   // quad_perm [1,0,3,2]
  v += dpp_f<0x4E, 0xF>(v, 0.0f);   // quad_perm [2,3,0,1]
  v += dpp_f<0x141, 0xF>(v, 0.0f);  // row_half_mirror
  v += dpp_f<0x140, 0xF>(v, 0.0f);  // row_mirror
  // row_bcast:15 -> rows 1, 3; rows 0, 2 are not written (their value is never read)
  v += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x142, 0xA, 0xF, false));
  return v;
}
// this half's bits of a ballot
__device__ __forceinline__ uint32_t hballot(bool p, int h) {
  const uint64_t m = __ballot(p);
  return h ? (uint32_t)(m >> 32) : (uint32_t)m;
}
// max over both halves of a half-uniform int (wave-uniform loop bound)
__device__ __forceinline__ int wmax2(int v) {
  const int a = __builtin_amdgcn_readlane(v, 0), b = __builtin_amdgcn_readlane(v, HW);
  return a > b ? a : b;
}

// ------------------------------------------------------------------------------------
// Phase 1: forward kinematics (mj_kinematics).  12 lanes build the local link rotations
// (body_quat * joint rotation) in parallel, then lanes 0..3 compose base -> leg chain.
// Hinge anchors coincide with body origins (jnt_pos = 0, checked at pp3_create).
// ------------------------------------------------------------------------------------
// The kinematics phase's per-lane model constants (lane l < 12 owns leg body bl = 2 + 3 gl + kl:
// level kl = l / 4, leg gl = l % 4), loaded once per launch and kept in registers across the
// substeps: otherwise every substep opens with an L2 round trip for them.
struct KinConst {
  float jax[3], bq[4], q0, bpos[3], cpos[3];
};
__device__ __forceinline__ KinConst kin_const(const DevModel& m, int l) {
  const int lc = l < 12 ? l : 11, gl = lc & 3, kl = lc >> 2;
  const int bl = 2 + 3 * gl + kl, jl = 1 + 3 * gl + kl, ql = 7 + 3 * gl + kl;
  KinConst k;
  for (int c = 0; c < 3; c++) k.jax[c] = m.jnt_axis[jl][c];
  for (int c = 0; c < 4; c++) k.bq[c] = m.body_quat[bl][c];
  k.q0 = m.qpos0[ql];
#pragma unroll
  for (int c = 0; c < 3; c++) {
    k.bpos[c] = m.body_pos[bl][c];                    // this body's offset in its parent
    k.cpos[c] = m.body_pos[kl < 2 ? bl + 1 : bl][c];  // its child's offset in it (levels 0, 1)
  }
  return k;
}

template <int NC, bool LIBSC = true>
__device__ __forceinline__ void kinematics(Shared<NC>& s, const DevModel& m, int l, bool euler, const KinConst& kc) {
  // lane l < 12 owns leg body (level kl = l / 4, leg gl = l % 4): body bl, joint jl, qpos ql
  const int lc = l < 12 ? l : 11, gl = lc & 3, kl = lc >> 2;
  const int bl = 2 + 3 * gl + kl, jl = 1 + 3 * gl + kl, ql = 7 + 3 * gl + kl;
  float jax[3] = {kc.jax[0], kc.jax[1], kc.jax[2]}, bq[4] = {kc.bq[0], kc.bq[1], kc.bq[2], kc.bq[3]}, q0 = kc.q0;
  const float bpos[3] = {kc.bpos[0], kc.bpos[1], kc.bpos[2]}, cpos[3] = {kc.cpos[0], kc.cpos[1], kc.cpos[2]};
  // The previous substep's Euler step (eulerdamp disabled), deferred to here when `euler`: the
  // joint lanes integrate their own dof (so the new angle stays in a register), lanes 12..17 the
  // base dofs, and lane 15 integrates the base quaternion -- its axis-angle rotation shares the
  // joints' sincos instructions instead of a serial sequence of its own (same arithmetic as
  // euler_step, which integrates the last substep).
  float qj = s.qpos[ql], aax[3] = {jax[0], jax[1], jax[2]}, ang = 0.0f, qb[4];
  if (euler) {
    const float hstep = m.h;
    const int d = l < 12 ? ql - 1 : l - 12;  // the dof this lane integrates (l < 18)
    float vn = 0.0f, w[3] = {0, 0, 0};
    if (l < 18) vn = s.qvel[d] + hstep * s.qacc[d];
    if (l == 15)
      for (int k = 0; k < 3; k++) w[k] = s.qvel[3 + k] + hstep * s.qacc[3 + k];
    for (int k = 0; k < 4; k++) qb[k] = s.qpos[3 + k];
    SYNC();
    if (l < 18) s.qvel[d] = vn;
    if (l < 12) { qj += hstep * vn; s.qpos[ql] = qj; }
    if (l >= 12 && l < 15) s.qpos[l - 12] += hstep * vn;
    if (l == 15) {
      const float n = sqrtf(dot3(w, w));
      if (n < MINVAL) { w[0] = 1; w[1] = 0; w[2] = 0; } else { const float in = 1.0f / n; w[0] *= in; w[1] *= in; w[2] *= in; }
      aax[0] = w[0]; aax[1] = w[1]; aax[2] = w[2];
      ang = hstep * n;
    }
  }
  if (l < 12) ang = qj - q0;
#ifdef PP3_PAD_VALU  // timing diagnostic only: N extra VALU instructions per substep (4 independent chains)
  {
    float p0 = 0.0f, p1 = 0.0f, p2 = 0.0f, p3 = 0.0f;
#pragma unroll
    for (int i = 0; i < PP3_PAD_VALU / 4; i++)
      asm volatile("v_add_f32 %0, %0, %0\n v_add_f32 %1, %1, %1\n v_add_f32 %2, %2, %2\n v_add_f32 %3, %3, %3"
                   : "+v"(p0), "+v"(p1), "+v"(p2), "+v"(p3));
  }
#endif
#ifdef PP3_PAD_NOP  // timing diagnostic only: N x s_nop 7 (8 issue-stall cycles each) per substep
#pragma unroll
  for (int i = 0; i < PP3_PAD_NOP; i++) asm volatile("s_nop 7");
#endif
  float lq[4] = {1, 0, 0, 0};
  {
    float qloc[4];
    axisangle2quat<LIBSC>(qloc, aax, ang);
    if (l < 12) mulquat(lq, bq, qloc);
    if (euler && l == 15) {
      normalize4(qb);
      mulquat(qb, qb, qloc);
      for (int k = 0; k < 4; k++) s.qpos[3 + k] = qb[k];
    }
  }
  SYNC();  // the base position / quaternion stores above precede the reads below
  float pq[4] = {s.qpos[3], s.qpos[4], s.qpos[5], s.qpos[6]};
  normalize4(pq);
  const float pp[3] = {s.qpos[0], s.qpos[1], s.qpos[2]};
  float pR[9];
  quat2mat(pq, pR);
  if (l == 0) {
    float off[3];
    matvec(off, pR, s.ipos[1]);
    for (int c = 0; c < 3; c++) {
      s.xpos[1][c] = pp[c];
      s.x.xipos[1][c] = pp[c] + off[c];
      s.xaxis[0][c] = m.jnt_axis[0][c];
    }
    for (int c = 0; c < 4; c++) s.xquat[1][c] = pq[c];
  }
  // The 12 leg bodies on their own lanes: lane l = 4 level + leg, so a body's parent (level - 1,
  // same leg) is lane l - 4 of the same 16-lane DPP row and each level's frame reaches the next
  // by one row_shr:4.  Same arithmetic as walking each chain on one lane (mj_kinematics:
  // xquat_k = normalize(xquat_{k-1} lq_k), xpos_k = xpos_{k-1} + R_{k-1} bpos_k), but only the
  // quaternion composition and the position sums are serial across levels: every rotation matrix,
  // child offset, axis and COM is computed by its body's lane at once.
  // (every DPP source is pinned on all lanes first: otherwise the compiler may compute it, and
  // run the DPP, only on the lanes that consume the result -- which are not the source lanes)
  float xq[4];
  mulquat(xq, pq, lq);
  normalize4(xq);  // level 0 final
#pragma unroll
  for (int lev = 1; lev < 3; lev++) {
    float par[4], t[4];
    PIN("+v"(xq[0]), "+v"(xq[1]), "+v"(xq[2]), "+v"(xq[3]));
#pragma unroll
    for (int c = 0; c < 4; c++) par[c] = dpp_shr4(xq[c]);
    PIN("+v"(par[0]), "+v"(par[1]), "+v"(par[2]), "+v"(par[3]));
    mulquat(t, par, lq);
    normalize4(t);
#pragma unroll
    for (int c = 0; c < 4; c++) xq[c] = kl >= lev ? t[c] : xq[c];  // level lev final
  }
  float R[9], ob[3], co[3], o[3], xp[3];
  quat2mat(xq, R);
  matvec(ob, pR, bpos);  // level 0: R_base bpos
  matvec(co, R, cpos);   // this body's child offset R_k bpos_{k+1}
  PIN("+v"(co[0]), "+v"(co[1]), "+v"(co[2]));
  float sh[3];
#pragma unroll
  for (int c = 0; c < 3; c++) sh[c] = dpp_shr4(co[c]);
  PIN("+v"(sh[0]), "+v"(sh[1]), "+v"(sh[2]));
#pragma unroll
  for (int c = 0; c < 3; c++) {
    o[c] = kl == 0 ? ob[c] : sh[c];  // R_{k-1} bpos_k
    xp[c] = pp[c] + o[c];            // level 0 final
  }
#pragma unroll
  for (int lev = 1; lev < 3; lev++) {
    PIN("+v"(xp[0]), "+v"(xp[1]), "+v"(xp[2]));
#pragma unroll
    for (int c = 0; c < 3; c++) sh[c] = dpp_shr4(xp[c]);
    PIN("+v"(sh[0]), "+v"(sh[1]), "+v"(sh[2]));
#pragma unroll
    for (int c = 0; c < 3; c++) xp[c] = kl >= lev ? sh[c] + o[c] : xp[c];  // level lev final
  }
  if (l < 12) {
    float ax[3], off[3];
    matvec(ax, R, jax);
    matvec(off, R, s.ipos[bl]);
    for (int c = 0; c < 3; c++) {
      s.xpos[bl][c] = xp[c];
      s.x.xipos[bl][c] = xp[c] + off[c];
      s.xaxis[jl][c] = ax[c];
    }
    for (int c = 0; c < 4; c++) s.xquat[bl][c] = xq[c];
  }
}

// ------------------------------------------------------------------------------------
// Phase 2: subtree com, cinert (mju_inertCom), cdof, robot geom and foot-site positions.
// lanes 1..13 bodies, 14..31 dofs; then lanes 0..7 geoms, 16..19 feet.
// ------------------------------------------------------------------------------------
// Straight-line form: every lane runs every part (clamped indices; results selected, stores in
// lane branches at the end), with all LDS operands in one pinned round.  What does not need the
// subtree com -- the bodies' rotated inertias, the geom / site positions, the base rotation's
// columns -- then issues while the com's four half-wave sums run, instead of behind them (+1.2 %
// against the round-4 branchy form, whose results it matches except for the FMA contraction of the
// rotated inertia R I R', which differs in the last bit on some lanes: profiles/AB_LOG.md round 5).
template <int NC>
__device__ __forceinline__ void com_pos(Shared<NC>& s, const DevModel& m, int l, int h, const LaneRec<2>& rc) {
  const bool body = l >= 1 && l < NB;
  const int b = body ? l : 1;
  const bool geom = l < m.nrobot_geom, foot = l >= 16 && l < 20;
  const int gb = as_i(rc.f[LC_PT_BODY]);  // (0 on lanes without a point: the world body's words)
  const int d = l >= 14 ? l - 14 : 0;      // cdof lanes 14..31: dof d
  const int jx = d >= 6 ? d - 5 : 1, bd = d < 6 ? 1 : 2 + (d - 6);
  float mb0 = s.mass[b], xi[3], bq[4], I[3], gq[4], gx[3], q1[4], x1[3], ax6[3], xb[3];
#pragma unroll
  for (int k = 0; k < 3; k++) {
    xi[k] = s.x.xipos[b][k]; I[k] = s.inertia[b][k]; gx[k] = s.xpos[gb][k];
    x1[k] = s.x.xipos[1][k]; ax6[k] = s.xaxis[jx][k]; xb[k] = s.xpos[bd][k];
  }
#pragma unroll
  for (int k = 0; k < 4; k++) { bq[k] = s.xquat[b][k]; gq[k] = s.xquat[gb][k]; q1[k] = s.xquat[1][k]; }
  PIN("+v"(mb0), "+v"(xi[0]), "+v"(xi[1]), "+v"(xi[2]), "+v"(I[0]), "+v"(I[1]), "+v"(I[2]), "+v"(gx[0]), "+v"(gx[1]),
      "+v"(gx[2]), "+v"(x1[0]), "+v"(x1[1]), "+v"(x1[2]), "+v"(ax6[0]), "+v"(ax6[1]), "+v"(ax6[2]), "+v"(xb[0]),
      "+v"(xb[1]), "+v"(xb[2]));
  PIN("+v"(bq[0]), "+v"(bq[1]), "+v"(bq[2]), "+v"(bq[3]), "+v"(gq[0]), "+v"(gq[1]), "+v"(gq[2]), "+v"(gq[3]),
      "+v"(q1[0]), "+v"(q1[1]), "+v"(q1[2]), "+v"(q1[3]));
  float mb = body ? mb0 : 0.0f, mx = body ? mb0 * xi[0] : 0.0f, my = body ? mb0 * xi[1] : 0.0f,
        mz = body ? mb0 * xi[2] : 0.0f;
  mb = hsum(mb, h);
  mx = hsum(mx, h);
  my = hsum(my, h);
  mz = hsum(mz, h);
  // com-independent parts
  float A[3][3];
  {
    float iq[4], R[9];
    const float biq[4] = {rc.f[LC_IQUAT], rc.f[LC_IQUAT + 1], rc.f[LC_IQUAT + 2], rc.f[LC_IQUAT + 3]};
    mulquat(iq, bq, biq);
    quat2mat(iq, R);
#pragma unroll
    for (int i = 0; i < 3; i++)
#pragma unroll
      for (int j = 0; j < 3; j++)
        A[i][j] = R[3 * i] * I[0] * R[3 * j] + R[3 * i + 1] * I[1] * R[3 * j + 1] + R[3 * i + 2] * I[2] * R[3 * j + 2];
  }
  float gpos[3];
  {
    const float lp[3] = {rc.f[LC_PT_POS], rc.f[LC_PT_POS + 1], rc.f[LC_PT_POS + 2]};
    float R[9], off[3];
    quat2mat(gq, R);
    matvec(off, R, lp);
#pragma unroll
    for (int k = 0; k < 3; k++) gpos[k] = gx[k] + off[k];
  }
  float ax[3];
  {
    float R[9];
    quat2mat(q1, R);
    const int cc = d - 3;
    ax[0] = cc == 0 ? R[0] : (cc == 1 ? R[1] : R[2]);
    ax[1] = cc == 0 ? R[3] : (cc == 1 ? R[4] : R[5]);
    ax[2] = cc == 0 ? R[6] : (cc == 1 ? R[7] : R[8]);
#pragma unroll
    for (int k = 0; k < 3; k++) ax[k] = d < 6 ? ax[k] : ax6[k];
  }
  float com[3];
  const bool mok = mb > MINVAL;
  {
    const float im = 1.0f / mb;
    com[0] = mok ? mx * im : x1[0];
    com[1] = mok ? my * im : x1[1];
    com[2] = mok ? mz * im : x1[2];
  }
  if (l == 0) { s.com[0] = com[0]; s.com[1] = com[1]; s.com[2] = com[2]; }
  float ci[10];
  {
    const float mm = mb0;
    const float dx = xi[0] - com[0], dy = xi[1] - com[1], dz = xi[2] - com[2];
    ci[0] = A[0][0] + mm * (dy * dy + dz * dz);
    ci[1] = A[1][1] + mm * (dx * dx + dz * dz);
    ci[2] = A[2][2] + mm * (dx * dx + dy * dy);
    ci[3] = A[0][1] - mm * dx * dy;
    ci[4] = A[0][2] - mm * dx * dz;
    ci[5] = A[1][2] - mm * dy * dz;
    ci[6] = mm * dx; ci[7] = mm * dy; ci[8] = mm * dz;
    ci[9] = mm;
#pragma unroll
    for (int k = 0; k < 10; k++) ci[k] = body ? ci[k] : 0.0f;
  }
  float cd[6];
  {
    float off[3], c[3];
#pragma unroll
    for (int k = 0; k < 3; k++) off[k] = com[k] - xb[k];
    cross3(c, ax, off);
#pragma unroll
    for (int k = 0; k < 3; k++) {
      cd[k] = d < 3 ? 0.0f : ax[k];
      cd[3 + k] = d < 3 ? (k == d ? 1.0f : 0.0f) : c[k];
    }
  }
  if (body)
#pragma unroll
    for (int k = 0; k < 10; k++) s.cinert[b][k] = ci[k];
  if (l >= 14)
#pragma unroll
    for (int k = 0; k < 6; k++) s.cdof[d][k] = cd[k];
  {  // composite inertia of the whole tree (body 1's subtree) for the 6 base dofs
    float t[10];
#pragma unroll
    for (int k = 0; k < 10; k++) t[k] = hsum_lane16(ci[k]);
    if (l == 16)
#pragma unroll
      for (int k = 0; k < 10; k++) s.crb_base[k] = t[k];
  }
  if (geom || foot) {
    float* dst = geom ? s.gxpos[l] : s.foot_xpos[l - 16];
    for (int k = 0; k < 3; k++) dst[k] = gpos[k];
  }
}

__device__ __forceinline__ void make_frame(float f[9], const float nin[3]) {
  float a[3] = {nin[0], nin[1], nin[2]};
  float n = sqrtf(dot3(a, a));
  if (n < MINVAL) { a[0] = 1; a[1] = 0; a[2] = 0; } else { const float in = 1.0f / n; a[0] *= in; a[1] *= in; a[2] *= in; }
  float y[3] = {0, 0, 0};
  if (a[1] < 0.5f && a[1] > -0.5f) y[1] = 1; else y[2] = 1;
  float ad = dot3(a, y);
  for (int k = 0; k < 3; k++) y[k] -= a[k] * ad;
  float yn = sqrtf(dot3(y, y));
  if (yn < MINVAL) { y[0] = 1; y[1] = 0; y[2] = 0; } else { const float in = 1.0f / yn; y[0] *= in; y[1] *= in; y[2] *= in; }
  float z[3];
  cross3(z, a, y);
  for (int k = 0; k < 3; k++) { f[k] = a[k]; f[3 + k] = y[k]; f[6 + k] = z[k]; }
}

// narrow phase for pair p; returns hit and fills dist/pos/normal.  One dependent global level:
// the pair's flattened record (PairRec), then robot-geom world positions from LDS.
// the pair record (6 x 16 B) and the first word group of its PairCon (for store_contact): one
// batch of loads
struct PairLoad {
  v4f v[7];
};
__device__ __forceinline__ PairLoad load_pair(const DevModel& m, int p) {
  PairLoad r;
#pragma unroll
  for (int k = 0; k < 6; k++) r.v[k] = *reinterpret_cast<const v4f*>(m.pair_rec.g[k][p]);
  r.v[6] = *reinterpret_cast<const v4f*>(&m.pair_con[p]);
  return r;
}
// the per-env terrain table and its row length, read once per collision pass (above the
// lane-divergent pair-kind branches, which would otherwise each re-issue both scalar loads, one
// round trip after the other)
struct TerrainRef {
  uint64_t terrain;
  int nbox;
};
template <int NC, int NWV = 1>
__device__ __forceinline__ bool narrow(const Shared<NC>& s, const TerrainRef& tr, PairLoad pl, float& dist, float pos[3],
                                       float nrm[3], v4f& pc0) {
  PairRec rec;
  {
    PIN("+v"(pl.v[0]), "+v"(pl.v[1]), "+v"(pl.v[2]), "+v"(pl.v[3]), "+v"(pl.v[4]), "+v"(pl.v[5]), "+v"(pl.v[6]));
    __builtin_memcpy(&rec, pl.v, sizeof(rec));
    pc0 = pl.v[6];
  }
  const float margin = rec.margin;
  float p1[3], p2[3];
  {  // robot geoms: world position from LDS; static geoms: from the record (value select)
    const int i1 = rec.s1 >= 0 ? rec.s1 : 0, i2 = rec.s2 >= 0 ? rec.s2 : 0;
    float l1[3], l2[3];
#pragma unroll
    for (int k = 0; k < 3; k++) { l1[k] = s.gxpos[i1][k]; l2[k] = s.gxpos[i2][k]; }
    // keep both loads (a pointer select would be a flat load), all six in one LDS round trip
    asm volatile("" : "+v"(l1[0]), "+v"(l1[1]), "+v"(l1[2]), "+v"(l2[0]), "+v"(l2[1]), "+v"(l2[2]));
#pragma unroll
    for (int k = 0; k < 3; k++) {
      p1[k] = rec.s1 >= 0 ? l1[k] : rec.p1[k];
      p2[k] = rec.s2 >= 0 ? l2[k] : rec.p2[k];
    }
  }
  if (rec.kind == PK_PLANE_SPHERE) {
    const float nz[3] = {rec.R[2], rec.R[5], rec.R[8]};
    const float v[3] = {p2[0] - p1[0], p2[1] - p1[1], p2[2] - p1[2]};
    const float r = rec.r2;
    dist = dot3(nz, v) - r;
    if (dist > margin) return false;
    for (int k = 0; k < 3; k++) { nrm[k] = nz[k]; pos[k] = p2[k] - nz[k] * (r + 0.5f * dist); }
    return true;
  }
  if (rec.kind == PK_SPHERE_SPHERE) {
    const float v[3] = {p2[0] - p1[0], p2[1] - p1[1], p2[2] - p1[2]};
    const float r1 = rec.r1, r2 = rec.r2;
    const float len = sqrtf(dot3(v, v));
    dist = len - r1 - r2;
    if (dist > margin) return false;
    if (len < MINVAL) { nrm[0] = 1; nrm[1] = 0; nrm[2] = 0; }
    else { const float il = 1.0f / len; nrm[0] = v[0] * il; nrm[1] = v[1] * il; nrm[2] = v[2] * il; }
    for (int k = 0; k < 3; k++) pos[k] = p1[k] + nrm[k] * (r1 + 0.5f * dist);
    return true;
  }
  if (rec.kind == PK_SPHERE_BOX) {
    float R2[9], hh[3];
    for (int k = 0; k < 9; k++) R2[k] = rec.R[k];
    for (int k = 0; k < 3; k++) hh[k] = rec.half[k];
    if (tr.terrain) {  // per-env terrain: this env's box in slot -1 - s2 (rows padded to an even env count)
      typedef float v4f __attribute__((ext_vector_type(4)));
      typedef __attribute__((address_space(1))) const v4f GF4;
      const int env_raw = 2 * NWV * blockIdx.x + (threadIdx.x >> 5);  // (NWV waves = 2 NWV envs per workgroup)
      const GF4* t = (const GF4*)(uintptr_t)tr.terrain + ((size_t)env_raw * tr.nbox + (-1 - rec.s2)) * 4;
      const v4f t0 = t[0], t1 = t[1], t2 = t[2], t3 = t[3];
      p2[0] = t0.x; p2[1] = t0.y; p2[2] = t0.z;
      R2[0] = t0.w; R2[1] = t1.x; R2[2] = t1.y; R2[3] = t1.z; R2[4] = t1.w;
      R2[5] = t2.x; R2[6] = t2.y; R2[7] = t2.z; R2[8] = t2.w;
      hh[0] = t3.x; hh[1] = t3.y; hh[2] = t3.z;
    }
    const float r = rec.r1;
    float rel[3] = {p1[0] - p2[0], p1[1] - p2[1], p1[2] - p2[2]}, dl[3], cl[3];
    for (int k = 0; k < 3; k++) dl[k] = R2[k] * rel[0] + R2[3 + k] * rel[1] + R2[6 + k] * rel[2];
    bool inside = true;
    for (int k = 0; k < 3; k++) {
      cl[k] = dl[k];
      if (cl[k] > hh[k]) { cl[k] = hh[k]; inside = false; }
      if (cl[k] < -hh[k]) { cl[k] = -hh[k]; inside = false; }
    }
    float nl[3], dd;
    if (!inside) {
      float v[3] = {cl[0] - dl[0], cl[1] - dl[1], cl[2] - dl[2]};
      float len = sqrtf(dot3(v, v));
      dd = len - r;
      if (dd > margin) return false;
      if (len < MINVAL) { nl[0] = 0; nl[1] = 0; nl[2] = -1; }
      else { const float il = 1.0f / len; for (int k = 0; k < 3; k++) nl[k] = v[k] * il; }
    } else {
      const float t0 = hh[0] - fabsf(dl[0]), t1b = hh[1] - fabsf(dl[1]), t2b = hh[2] - fabsf(dl[2]);
      const int ax = (t1b < t0 && t1b <= t2b) ? 1 : (t2b < t0 && t2b < t1b) ? 2 : 0;
      const float best = ax == 0 ? t0 : (ax == 1 ? t1b : t2b);
      const float sg = (ax == 0 ? dl[0] : (ax == 1 ? dl[1] : dl[2])) >= 0 ? -1.0f : 1.0f;
      nl[0] = ax == 0 ? sg : 0.0f;
      nl[1] = ax == 1 ? sg : 0.0f;
      nl[2] = ax == 2 ? sg : 0.0f;
      dd = -best - r;
    }
    matvec(nrm, R2, nl);
    dist = dd;
    for (int k = 0; k < 3; k++) pos[k] = p1[k] + nrm[k] * (r + 0.5f * dd);
    return true;
  }
  return false;
}

template <int NC>
__device__ __forceinline__ void store_contact(Shared<NC>& s, const v4f& pc0, int slot, int p, float dist,
                                              const float pos[3], const float nrm[3]) {
  // pc0 = the pair's first PairCon word group (sup, dm[2], mu), fetched with the pair record
  s.con_pair[slot] = p;
  s.con_sup[slot] = as_i(pc0[0]);
  s.con_dm[slot][0] = (uint32_t)as_i(pc0[1]);
  s.con_dm[slot][1] = (uint32_t)as_i(pc0[2]);
  s.con_dist[slot] = dist;
  for (int k = 0; k < 3; k++) s.x.a.con_pos[slot][k] = pos[k];
  make_frame(s.x.a.con_frame[slot], nrm);
  const float mu_dr = s.fric, mu_model = pc0[3];
  s.con_mu[slot] = s.dr_on ? mu_dr : mu_model;
}

// Phase 3a: collision (mj_collision), contacts compacted in pair order; when more than
// NC pairs penetrate, the NC deepest are kept (same rule as the oracle).  Returns lane c's
// contact support (pair_sup of contact c; 4 = no contact): the Newton phases read contact
// supports with v_readlane from this register instead of LDS round trips per contact.
// position of the r-th (0-based) set bit of m; r < popc(m)
__device__ __forceinline__ int nth_bit(uint32_t m, int r) {
  int pos = 0, c = __popc(m & 0xFFFFu);
  if (r >= c) { r -= c; m >>= 16; pos += 16; }
  c = __popc(m & 0xFFu);
  if (r >= c) { r -= c; m >>= 8; pos += 8; }
  c = __popc(m & 0xFu);
  if (r >= c) { r -= c; m >>= 4; pos += 4; }
  c = __popc(m & 0x3u);
  if (r >= c) { r -= c; m >>= 2; pos += 2; }
  return pos + (r >= (int)(m & 1u) ? 1 : 0);
}

template <int NC, int NWV = 1, bool CULL = false>
__device__ __forceinline__ int collision(Shared<NC>& s, const DevModel& m, int l, int h, const PairLoad& pre,
                                         float* ccache = nullptr) {
  int nhit = 0;
  const TerrainRef tr{m.terrain, m.nbox};
  // (cull path) narrow phase of pair p on this lane (p < 0: none), hits compacted in lane order
  auto run = [&](int p, const PairLoad& pl) {
    float dist = 0, pos[3], nrm[3];
    v4f pc0;
    const bool hit = narrow<NC, NWV>(s, tr, pl, dist, pos, nrm, pc0) && p >= 0;
    const uint32_t mask = hballot(hit, h);
    const int slot = nhit + __popc(mask & ((1u << l) - 1u));
    if (hit) {
      if (slot < NC) store_contact(s, pc0, slot, p, dist, pos, nrm);
      if (slot < NHIT) { s.x.a.hit_dist[slot] = dist; s.x.a.hit_pair[slot] = p; }
    }
    nhit += __popc(mask);
  };
  if (!CULL || !m.cull_on) {
    for (int base = 0; base < m.npair; base += HW) {
      const int p = base + l;
      float dist = 0, pos[3], nrm[3];
      v4f pc0;
      // the first 32 pairs' records were fetched at the substep start (they arrive during kinematics)
      const PairLoad pl = base == 0 ? pre : load_pair(m, p < m.npair ? p : 0);
      const bool hit = narrow<NC, NWV>(s, tr, pl, dist, pos, nrm, pc0) && (p < m.npair);
      const uint32_t mask = hballot(hit, h);
      const int slot = nhit + __popc(mask & ((1u << l) - 1u));
      if (hit) {
        if (slot < NC) store_contact(s, pc0, slot, p, dist, pos, nrm);
        if (slot < NHIT) { s.x.a.hit_dist[slot] = dist; s.x.a.hit_pair[slot] = p; }
      }
      nhit += __popc(mask);
    }
  } else {
    // boxes (DevModel::cull_on).  The near-box mask is cached (ccache: body 1's origin at the
    // test, then the mask's bits; one per env, in LDS) and re-tested
    // only when body 1's origin has moved more than CULL_SLACK from where it was tested (the
    // test widens the reach by the slack), i.e. about once per env step
    const uint32_t pbox = m.pair_box4[l];
    const float b0 = s.xpos[1][0], b1 = s.xpos[1][1], b2 = s.xpos[1][2];
    {
      const float c0 = b0 - ccache[0], c1 = b1 - ccache[1], c2 = b2 - ccache[2];
      const bool stale = !(c0 * c0 + c1 * c1 + c2 * c2 <= CULL_SLACK * CULL_SLACK);
      if (__ballot(stale)) {  // lane b: box b out of reach when body 1's origin lies farther than
        // the reach outside one of its slabs (box frame: local = R^T (x - c), as in narrow())
        const int b = l < tr.nbox ? l : 0;
        v4f bx[4];
        if (tr.terrain) {
          typedef __attribute__((address_space(1))) const v4f GF4;
          const int env_raw = 2 * NWV * blockIdx.x + (threadIdx.x >> 5);
          const GF4* t = (const GF4*)(uintptr_t)tr.terrain + ((size_t)env_raw * tr.nbox + b) * 4;
#pragma unroll
          for (int k = 0; k < 4; k++) bx[k] = t[k];
        } else {
#pragma unroll
          for (int k = 0; k < 4; k++) bx[k] = reinterpret_cast<const v4f*>(&m.box_tab[b])[k];
        }
        const float reach = m.cull_reach + CULL_SLACK;
        const float d0 = b0 - bx[0][0], d1 = b1 - bx[0][1], d2 = b2 - bx[0][2];
        const float R[9] = {bx[0][3], bx[1][0], bx[1][1], bx[1][2], bx[1][3], bx[2][0], bx[2][1], bx[2][2], bx[2][3]};
        bool far = false;
#pragma unroll
        for (int k = 0; k < 3; k++) far |= fabsf(R[k] * d0 + R[3 + k] * d1 + R[6 + k] * d2) > bx[3][k] + reach;
        const uint32_t nm = hballot(l < tr.nbox && !far, h);
        if (l == 0) {  // (both halves refresh: a fresh test is valid whether or not it was due)
          ccache[0] = b0;
          ccache[1] = b1;
          ccache[2] = b2;
          ccache[3] = __uint_as_float(nm);
        }
        SYNC();
      }
    }
    const uint32_t near = __float_as_uint(ccache[3]);
    // this half's candidates among pairs 32 .. npair - 1 (every non-box pair, the box pairs of
    // near boxes), in pair order
    uint32_t cm[4];
    int total = 0;
#pragma unroll
    for (int k = 0; k < 4; k++) {
      const int p = 32 * (k + 1) + l;
      const uint32_t bs = (pbox >> (8 * k)) & 0xFFu;
      const bool c = p < m.npair && (bs >= 32u || ((near >> (bs & 31u)) & 1u));
      cm[k] = hballot(c, h);
      total += __popc(cm[k]);
    }
    const int rounds = wmax2(total);
    // this lane's candidate of round `base`: the (base + l)-th set bit over cm[0..3]
    auto cand = [&](int base) {
      int p = -1, r = base + l;
#pragma unroll
      for (int k = 0; k < 4; k++) {
        const int c = __popc(cm[k]);
        if (p < 0 && r < c) p = 32 * (k + 1) + nth_bit(cm[k], r);
        if (p < 0) r -= c;
      }
      return p;
    };
    // the first round's records issued before the first 32 pairs run (they arrive meanwhile)
    const int p1 = cand(0);
    const PairLoad pl1 = load_pair(m, p1 >= 0 ? p1 : 0);
    run(l < m.npair ? l : -1, pre);
    if (rounds > 0) run(p1, pl1);
    for (int base = HW; base < rounds; base += HW) {
      const int p = cand(base);
      run(p, load_pair(m, p >= 0 ? p : 0));
    }
  }
  if (l == 0) { s.nhit = nhit; s.ncon = nhit < NC ? nhit : NC; }
  const bool ovf = nhit > NC;
  if (__ballot(ovf)) {  // rare: keep the NC deepest among the first NHIT hits, in pair order
    SYNC();
    const int nh = nhit < NHIT ? nhit : NHIT;
    int keep_p[NHIT / HW];
    bool keep[NHIT / HW];
    int rank[NHIT / HW];
#pragma unroll
    for (int t = 0; t < NHIT / HW; t++) {
      const int i = l + HW * t;
      const float myd = i < nh ? s.x.a.hit_dist[i] : 0.0f;
      int r = 0;
      for (int c = 0; c < nh; c++) {
        const float dc = s.x.a.hit_dist[c];
        r += (dc < myd || (dc == myd && c < i)) ? 1 : 0;
      }
      rank[t] = r;
      keep[t] = ovf && i < nh && r < NC;
      keep_p[t] = i < nh ? s.x.a.hit_pair[i] : 0;
    }
    // slot = number of kept hits with a smaller hit index
    int before = 0;
    int slot[NHIT / HW];
#pragma unroll
    for (int t = 0; t < NHIT / HW; t++) {
      const uint32_t km = hballot(keep[t], h);
      slot[t] = before + __popc(km & ((1u << l) - 1u));
      before += __popc(km);
    }
    (void)rank;
    SYNC();
#pragma unroll
    for (int t = 0; t < NHIT / HW; t++) {
      if (keep[t]) {
        float dist, pos[3], nrm[3];
        v4f pc0;
        narrow<NC, NWV>(s, tr, load_pair(m, keep_p[t]), dist, pos, nrm, pc0);
        store_contact(s, pc0, slot[t], keep_p[t], dist, pos, nrm);
      }
    }
  }
  SYNC();
  const int ncon_h = nhit < NC ? nhit : NC;
  const int sup = s.con_sup[l < NC ? l : 0];
  return l < ncon_h ? sup : 4;
}

// RNE velocity/acceleration chain (mj_comVel + forward half of mj_rne): lanes 0..3 each
// walk base -> leg l writing cvel and cacc of its links (lane 0 also the base).  The leg's three
// cdof rows and joint velocities are loaded (pinned) before the first store: a level's loads
// would otherwise be placed after the previous level's stores and each waited for.
template <int NC>
__device__ __forceinline__ void rne_chain(Shared<NC>& s, const DevModel& m, int l) {
  if (l >= 4) return;
  float lcd[3][6], lqd[3];
#pragma unroll
  for (int k = 0; k < 3; k++) {
    const int d = 6 + 3 * l + k;
#pragma unroll
    for (int c = 0; c < 6; c++) lcd[k][c] = s.cdof[d][c];
    lqd[k] = s.qvel[d];
  }
  PIN("+v"(lcd[0][0]), "+v"(lcd[0][1]), "+v"(lcd[0][2]), "+v"(lcd[0][3]), "+v"(lcd[0][4]), "+v"(lcd[0][5]),
      "+v"(lcd[1][0]), "+v"(lcd[1][1]), "+v"(lcd[1][2]), "+v"(lcd[1][3]), "+v"(lcd[1][4]), "+v"(lcd[1][5]),
      "+v"(lcd[2][0]), "+v"(lcd[2][1]), "+v"(lcd[2][2]), "+v"(lcd[2][3]), "+v"(lcd[2][4]), "+v"(lcd[2][5]),
      "+v"(lqd[0]), "+v"(lqd[1]), "+v"(lqd[2]));
  // free joint in closed form: its translational cdof are the unit vectors (com_pos), so the
  // velocity after them is (0, v); each rotational dof's cdof_dot = (0, v) x cdof = (0, v x a_d),
  // hence cacc = (0, -g + v x w) with w = sum_d a_d qvel[3+d], and cvel = (w, v + sum_d b_d qvel[3+d])
  // (the base's three rotational cdof rows and six velocities in one pinned LDS round)
  float bcd[3][6], bq[6];
#pragma unroll
  for (int d = 0; d < 3; d++)
#pragma unroll
    for (int k = 0; k < 6; k++) bcd[d][k] = s.cdof[3 + d][k];
#pragma unroll
  for (int k = 0; k < 6; k++) bq[k] = s.qvel[k];
  PIN("+v"(bcd[0][0]), "+v"(bcd[0][1]), "+v"(bcd[0][2]), "+v"(bcd[0][3]), "+v"(bcd[0][4]), "+v"(bcd[0][5]),
      "+v"(bcd[1][0]), "+v"(bcd[1][1]), "+v"(bcd[1][2]), "+v"(bcd[1][3]), "+v"(bcd[1][4]), "+v"(bcd[1][5]),
      "+v"(bcd[2][0]), "+v"(bcd[2][1]), "+v"(bcd[2][2]), "+v"(bcd[2][3]), "+v"(bcd[2][4]), "+v"(bcd[2][5]),
      "+v"(bq[0]), "+v"(bq[1]), "+v"(bq[2]), "+v"(bq[3]), "+v"(bq[4]), "+v"(bq[5]));
  float w[3] = {0, 0, 0}, bsum[3] = {0, 0, 0};
#pragma unroll
  for (int d = 0; d < 3; d++) {
    const float q = bq[3 + d];
#pragma unroll
    for (int k = 0; k < 3; k++) { w[k] += bcd[d][k] * q; bsum[k] += bcd[d][3 + k] * q; }
  }
  const float v0 = bq[0], v1 = bq[1], v2 = bq[2];
  float cv[6] = {w[0], w[1], w[2], v0 + bsum[0], v1 + bsum[1], v2 + bsum[2]};
  float ca[6] = {0, 0, 0, -m.gravity[0] + (v1 * w[2] - v2 * w[1]), -m.gravity[1] + (v2 * w[0] - v0 * w[2]),
                 -m.gravity[2] + (v0 * w[1] - v1 * w[0])};
  float cdd[6];
  if (l == 0)
    for (int k = 0; k < 6; k++) { s.cvel[1][k] = cv[k]; s.x.a.cacc[1][k] = ca[k]; }
#pragma unroll
  for (int k = 0; k < 3; k++) {
    const int b = 2 + 3 * l + k;
    cross_motion(cdd, cv, lcd[k]);
    const float qd = lqd[k];
    for (int c = 0; c < 6; c++) { cv[c] += lcd[k][c] * qd; ca[c] += cdd[c] * qd; }
    for (int c = 0; c < 6; c++) { s.cvel[b][c] = cv[c]; s.x.a.cacc[b][c] = ca[c]; }
  }
}

// body forces cinert*cacc + cvel x* (cinert*cvel), lanes 1..13 (one body each), plus the
// whole-tree sum of cfrc for the base dofs' bias forces
template <int NC>
__device__ __forceinline__ void rne_body_forces(Shared<NC>& s, int l, int h) {
  float cf[6] = {0, 0, 0, 0, 0, 0};
  if (l >= 1 && l < NB) {
    float f1[6], f2[6], f3[6];
    mul_inert_vec(f1, s.cinert[l], s.x.a.cacc[l]);
    mul_inert_vec(f2, s.cinert[l], s.cvel[l]);
    cross_force(f3, s.cvel[l], f2);
    for (int k = 0; k < 6; k++) { cf[k] = f1[k] + f3[k]; s.x.a.cacc[l][k] = cf[k]; }  // cfrc, in place
  }
  // all six sums first (independent DPP chains interleave), then the stores
  float t[6];
#pragma unroll
  for (int k = 0; k < 6; k++) t[k] = hsum_lane16(cf[k]);
  if (l == 16)
#pragma unroll
    for (int k = 0; k < 6; k++) s.cfrc_base[k] = t[k];
}

// composite inertia of body b's subtree times cdof d (for M), lanes < NV.  Branch-free: the
// base dofs read crb_base, a leg link its own cinert plus the (<= 2) links below it with weight 1
// (weight 0 past the leg's end: adding exact zeros), so the loads form one block.
template <int NC>
__device__ __forceinline__ void crb_times_cdof(Shared<NC>& s, const DevModel& m, int l) {
  if (l >= NV) return;
  const bool base = l < 6;
  const int b = base ? 2 : l - 4, last = 2 + 3 * ((b - 2) / 3) + 2;  // dof 6+3g+k <-> body 2+3g+k
  const float* r0 = base ? s.crb_base : s.cinert[b];
  // every operand (36 words) in one pinned LDS round: unpinned, the compiler reused one register
  // pair for the links' rows and waited after each pair of words
  const int b1 = b + 1 <= last ? b + 1 : b, b2 = b + 2 <= last ? b + 2 : b;
  float crb[10], c1[10], c2[10], cdv[6];
#pragma unroll
  for (int k = 0; k < 10; k++) { crb[k] = r0[k]; c1[k] = s.cinert[b1][k]; c2[k] = s.cinert[b2][k]; }
#pragma unroll
  for (int k = 0; k < 6; k++) cdv[k] = s.cdof[l][k];
  PIN("+v"(crb[0]), "+v"(crb[1]), "+v"(crb[2]), "+v"(crb[3]), "+v"(crb[4]), "+v"(crb[5]), "+v"(crb[6]), "+v"(crb[7]),
      "+v"(crb[8]), "+v"(crb[9]), "+v"(cdv[0]), "+v"(cdv[1]), "+v"(cdv[2]), "+v"(cdv[3]), "+v"(cdv[4]), "+v"(cdv[5]));
  PIN("+v"(c1[0]), "+v"(c1[1]), "+v"(c1[2]), "+v"(c1[3]), "+v"(c1[4]), "+v"(c1[5]), "+v"(c1[6]), "+v"(c1[7]),
      "+v"(c1[8]), "+v"(c1[9]), "+v"(c2[0]), "+v"(c2[1]), "+v"(c2[2]), "+v"(c2[3]), "+v"(c2[4]), "+v"(c2[5]),
      "+v"(c2[6]), "+v"(c2[7]), "+v"(c2[8]), "+v"(c2[9]));
  const float w1 = (!base && b + 1 <= last) ? 1.0f : 0.0f, w2 = (!base && b + 2 <= last) ? 1.0f : 0.0f;
#pragma unroll
  for (int k = 0; k < 10; k++) crb[k] += w1 * c1[k];
#pragma unroll
  for (int k = 0; k < 10; k++) crb[k] += w2 * c2[k];
  mul_inert_vec(s.x.a.F[l], crb, cdv);
}


// ------------------------------------------------------------------------------------
// LDL^T in registers: lane i (< NV) of each half holds row i; returns L_ik (k<i) in a[k],
// 1/D_i in dinv.  The pivot column is broadcast through LDS: every lane stores its a[k]
// (= A'[lane][k] = A'[k][lane]) in col[], then reads col[k..17] back with 16-byte broadcast
// loads, so each trailing update is one v_fma with VGPR operands.  col = 20 floats, 16-byte
// aligned, owned by this half.
// ------------------------------------------------------------------------------------
// The lane index made opaque at the top of a routine: its lane-index masks (l == k, l > k, ...)
// are then recomputed per call (one v_cmp each) instead of being hoisted out of the substep
// loop as ~100 live 64-bit SGPR masks that spill to VGPR lanes (two v_readlane per use).
__device__ __forceinline__ int opaque_lane(int l) {
  asm volatile("" : "+v"(l));
  __builtin_assume(l >= 0 && l < HW);
  return l;
}

__device__ __forceinline__ void ldl_rows(float (&a)[NV], float& dinv, int l, float* col) {
  l = opaque_lane(l);
  const int slot = l < NV ? l : NV;  // lanes >= NV carry copies of row NV-1: dummy slot
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    col[slot] = a[k];
    SYNC();
    float r[20];
#pragma unroll
    for (int q = (k & ~3); q < 20; q += 4) {
      const float4 v = *reinterpret_cast<const float4*>(col + q);
      r[q] = v.x; r[q + 1] = v.y; r[q + 2] = v.z; r[q + 3] = v.w;
    }
    const float ik = frcp(fmaxf(r[k], MINVAL));
    dinv = (l == k) ? ik : dinv;
    const float lik = a[k] * ik;
#pragma unroll
    for (int j = k + 1; j < NV; ++j) a[j] -= lik * r[j];
    a[k] = (l > k) ? lik : a[k];
    SYNC();  // col is rewritten by the next pivot
  }
}
// solve L D L^T x = b; x = b_i on entry (lane i).  Uses s.x.L for the transposed factor.
template <int NC>
__device__ __forceinline__ float ldl_solve(Shared<NC>& s, const float (&a)[NV], float dinv, float x, int l, int h) {
  l = opaque_lane(l);
  const int li = l < NV ? l : NV - 1;
#pragma unroll
  for (int k = 0; k < NV; ++k)
    if (k < l && l < NV) s.x.L[l][k] = a[k];
#pragma unroll
  for (int k = 0; k < NV - 1; ++k) {
    const float yk = hb(x, k, h);
    x = (l > k) ? x - a[k] * yk : x;
  }
  x = x * dinv;
  SYNC();
  float col[NV];
#pragma unroll
  for (int k = 1; k < NV; ++k) col[k] = s.x.L[k][li];
#pragma unroll
  for (int k = NV - 1; k > 0; --k) {
    const float xk = hb(x, k, h);
    x = (l < k) ? x - col[k] * xk : x;
  }
  return x;  // callers SYNC before s.x is rewritten
}

// ------------------------------------------------------------------------------------
// Tree-sparse (arrowhead) LDL^T.  In the permuted dof order P = [legs 6..17, base 0..5] the
// mass matrix and every Hessian whose contacts touch one leg (plus the base) have no
// leg-leg coupling, so eliminating the legs first creates no fill outside each leg's rows
// and the base block.  The four legs are independent: pivot level s (0..2) of all four
// legs is eliminated in ONE round, then the 6 base pivots -- 9 sequential LDS rounds
// instead of 18, and 99 instead of 153 multiply-adds.  Lane p (< NV) holds permuted row p.
// ------------------------------------------------------------------------------------
__host__ __device__ constexpr int pnat(int p) { return p < 12 ? p + 6 : p - 12; }  // permuted -> dof
__host__ __device__ constexpr int npos(int d) { return d < 6 ? d + 12 : d - 6; }   // dof -> permuted

__device__ __forceinline__ float dpp_shl1(float v) { return dpp_f<0x101, 0xF>(v, 0.0f); }  // lane i <- i+1 (row)
__device__ __forceinline__ float dpp_shl2(float v) { return dpp_f<0x102, 0xF>(v, 0.0f); }  // lane i <- i+2 (row)

// Factor AND solve A x = b in one pass (Gaussian elimination of the augmented rows [A | b]; A
// symmetric positive definite, arrowhead).  Lane p holds permuted row p in a[] and b_p; returns
// x_p.  Elimination only updates rows below the pivot, so every lane keeps its row of U (= the
// row at the time it became pivot) and U x = y is back-substituted from registers:
//  * 3 leg rounds (4 legs at once): each lane publishes its pivot-column entry, the pivot lane
//    also its rhs; rows below update their entries and rhs (forward substitution fused in);
//  * ONE exchange of the base Schur complement S and its rhs, then every lane factors and solves
//    the 6x6 base block in registers (x_base on every lane);
//  * leg rows back-substitute against x_base from registers and against the rows below them in
//    the same leg through two DPP lane shifts (a leg's rows are adjacent lanes of one DPP row).
// No transposed factor in LDS and no per-pivot lane broadcasts (cf. mj_factorM / mj_solveM).
__device__ __forceinline__ float ldl_arrow_solve(float (&a)[NV], float b, int l, float* col /* >= 80 floats */) {
  l = opaque_lane(l);
  const int slot = l < NV ? l : NV;
  const int lp = l < NV ? l : NV - 1;
  // lane p < 12 is the pivot of leg p / 3 in round p % 3; its 1/D is the reciprocal of the value
  // it publishes then (its own diagonal), read back with that round's pivot columns: one select
  // per round instead of a compare and select per pivot (12 per call)
  const int pg = lp < 12 ? lp / 3 : 0, pst = lp < 12 ? lp - 3 * pg : 3;
  float mydiag = 1.0f;
#pragma unroll
  for (int st = 0; st < 3; st++) {
#pragma unroll
    for (int g = 0; g < 4; g++) col[20 * g + slot] = a[3 * g + st];
    // the four pivots' rhs (lane 3 g + st of leg g) in one masked store, not one branch per leg
    if (l < 12 && l - 3 * (l / 3) == st) col[20 * (l / 3) + 19] = b;
    SYNC();
    {
      const float pv = col[20 * pg + slot];
      mydiag = (pst == st) ? pv : mydiag;
    }
#pragma unroll
    for (int g = 0; g < 4; g++) {
      const int k = 3 * g + st;
      const float* c = col + 20 * g;
      float r[20];
      // inner loops have constant trip counts (guards fold once g and st are unrolled): a bound
      // that depends on an outer induction variable is not unrolled first and ends up as a
      // runtime loop over s_set_gpr_idx register indexing
#pragma unroll
      for (int qq = 0; qq < 2; qq++) {
        const int q = ((3 * g) & ~3) + 4 * qq;  // the float4 words holding this leg's 3 entries
        if (q < 12 && q <= 3 * g + 2) {
          const float4 v = *reinterpret_cast<const float4*>(c + q);
          r[q] = v.x; r[q + 1] = v.y; r[q + 2] = v.z; r[q + 3] = v.w;
        }
      }
#pragma unroll
      for (int q = 12; q < 20; q += 4) {
        const float4 v = *reinterpret_cast<const float4*>(c + q);
        r[q] = v.x; r[q + 1] = v.y; r[q + 2] = v.z; r[q + 3] = v.w;
      }
      float ik = frcp(fmaxf(r[k], MINVAL));
      PIN("+v"(ik));  // (on every lane: otherwise the pivot read and rcp sink into a branch on l > k)
      const float lik = (l > k) ? a[k] * ik : 0.0f;  // zero on rows above the pivot and other legs
#pragma unroll
      for (int jj = 0; jj < 3; ++jj)
        if (jj > st) a[3 * g + jj] -= lik * r[3 * g + jj];
#pragma unroll
      for (int j = 12; j < NV; ++j) a[j] -= lik * r[j];
      b -= lik * r[19];
    }
    SYNC();
  }
  // base Schur complement and its rhs: ONE exchange; every lane then factors and solves it
  if (l >= 12 && l < NV) {
#pragma unroll
    for (int c = 0; c < 6; c++) col[6 * (l - 12) + c] = a[12 + c];
    col[36 + (l - 12)] = b;
  }
  SYNC();
  float S[6][6], y[6];
#pragma unroll
  for (int q = 0; q < 36; q += 4) {
    const float4 v = *reinterpret_cast<const float4*>(col + q);
    S[q / 6][q % 6] = v.x; S[(q + 1) / 6][(q + 1) % 6] = v.y;
    S[(q + 2) / 6][(q + 2) % 6] = v.z; S[(q + 3) / 6][(q + 3) % 6] = v.w;
  }
  {
    const float4 v0 = *reinterpret_cast<const float4*>(col + 36);
    const float2 v1 = *reinterpret_cast<const float2*>(col + 40);
    y[0] = v0.x; y[1] = v0.y; y[2] = v0.z; y[3] = v0.w; y[4] = v1.x; y[5] = v1.y;
  }
  SYNC();  // col is rewritten by the next use
  float db[6];
#pragma unroll
  for (int k = 0; k < 6; ++k) {
    const float ik = frcp(fmaxf(S[k][k], MINVAL));
    db[k] = ik;
#pragma unroll
    for (int i = 5; i > k; --i) {  // descending: rows below still hold their unscaled column k
      const float lik = S[i][k] * ik;
#pragma unroll
      for (int j = k + 1; j <= i; ++j) S[i][j] -= lik * S[j][k];
      S[i][k] = lik;
    }
  }
#pragma unroll
  for (int c = 1; c < 6; c++)
#pragma unroll
    for (int k = 0; k < c; k++) y[c] = y[c] - S[c][k] * y[k];
#pragma unroll
  for (int c = 0; c < 6; c++) y[c] = y[c] * db[c];
#pragma unroll
  for (int c = 4; c >= 0; --c)
#pragma unroll
    for (int i = 5; i > c; --i) y[c] = y[c] - S[i][c] * y[i];
  // leg rows: U x = y from registers (base part) and the rows below in the same leg (DPP)
  const float dinv = frcp(fmaxf(mydiag, MINVAL));  // the pivot's ik (base and dummy lanes: rcp(1) = 1)
  const int li = pst;  // level in the leg (3 = base row)
  float t = b;
#pragma unroll
  for (int c = 0; c < 6; c++) t -= a[12 + c] * y[c];
  // U entries to the next rows of this lane's leg: other legs' columns are exactly zero
  const float u1 = a[1] + a[4] + a[7] + a[10], u2 = a[2] + a[5] + a[8] + a[11];
  float x = t * dinv;                             // level 2 final
  float v1 = dpp_shl1(x);
  x = (li == 1) ? (t - u2 * v1) * dinv : x;       // level 1
  v1 = dpp_shl1(x);
  const float v2 = dpp_shl2(x);
  x = (li == 0) ? (t - u1 * v1 - u2 * v2) * dinv : x;  // level 0
#pragma unroll
  for (int c = 0; c < 6; c++) x = (lp == 12 + c) ? y[c] : x;
  return x;
}

// ldl_arrow_solve with leg `lb` (per half) moved into the base block.  A Hessian whose leg-leg
// couplings (contacts between two legs) all involve leg lb is arrowhead once lb's three rows are
// counted with the base: eliminating the other three legs (the same three rounds) creates fill
// only in their own rows, lb's rows and the base, and the 9 x 9 Schur complement of [leg lb |
// base] is factored and solved in registers on every lane, instead of the dense path's 18
// sequential pivots and 34 broadcast substitution steps.  Lane p holds permuted row p in a[];
// lb's columns are carried in e[] (the array's lb entries are zeroed, so the per-lane sums over
// the other legs' columns stay exact).
__device__ __forceinline__ float ldl_arrow_solve_b(float (&a)[NV], float rhs, int l, float* col /* >= 93 floats */,
                                                   int lb) {
  l = opaque_lane(l);
  const int slot = l < NV ? l : NV;
  const int lp = l < NV ? l : NV - 1;
  const bool brow = lp >= 3 * lb && lp < 3 * lb + 3;  // one of leg lb's rows
  float e[3];
#pragma unroll
  for (int jj = 0; jj < 3; jj++) e[jj] = lb == 0 ? a[jj] : lb == 1 ? a[3 + jj] : lb == 2 ? a[6 + jj] : a[9 + jj];
#pragma unroll
  for (int g = 0; g < 4; g++)
#pragma unroll
    for (int jj = 0; jj < 3; jj++) a[3 * g + jj] = (lb == g) ? 0.0f : a[3 * g + jj];
  float dinv = 1.0f;
#pragma unroll
  for (int st = 0; st < 3; st++) {
#pragma unroll
    for (int g = 0; g < 4; g++) {
      col[20 * g + slot] = a[3 * g + st];
      if (l == 3 * g + st) col[20 * g + 19] = rhs;  // pivot rhs
    }
    SYNC();
#pragma unroll
    for (int g = 0; g < 4; g++) {
      const int k = 3 * g + st;
      const float* c = col + 20 * g;
      float r[20], rb[3];
#pragma unroll
      for (int qq = 0; qq < 2; qq++) {
        const int q = ((3 * g) & ~3) + 4 * qq;
        if (q < 12 && q <= 3 * g + 2) {
          const float4 v = *reinterpret_cast<const float4*>(c + q);
          r[q] = v.x; r[q + 1] = v.y; r[q + 2] = v.z; r[q + 3] = v.w;
        }
      }
#pragma unroll
      for (int q = 12; q < 20; q += 4) {
        const float4 v = *reinterpret_cast<const float4*>(c + q);
        r[q] = v.x; r[q + 1] = v.y; r[q + 2] = v.z; r[q + 3] = v.w;
      }
#pragma unroll
      for (int jj = 0; jj < 3; jj++) rb[jj] = c[3 * lb + jj];  // pivot row's entries in lb's columns (symmetry)
      const bool act = lb != g;  // lb's rows are not pivots here
      const float ik = frcp(fmaxf(r[k], MINVAL));
      dinv = (l == k && act) ? ik : dinv;
      // rows after the pivot, and lb's rows (eliminated with the base); other legs' entries are 0
      const float lik = (act && (l > k || brow)) ? a[k] * ik : 0.0f;
#pragma unroll
      for (int jj = 0; jj < 3; ++jj)
        if (jj > st) a[3 * g + jj] -= lik * r[3 * g + jj];
#pragma unroll
      for (int j = 12; j < NV; ++j) a[j] -= lik * r[j];
#pragma unroll
      for (int jj = 0; jj < 3; ++jj) e[jj] -= lik * rb[jj];
      rhs -= lik * r[19];
    }
    SYNC();
  }
  // Schur complement of [lb | base] (rows lb0..2, base0..5) and its rhs: ONE exchange
  const int bi = brow ? lp - 3 * lb : (lp >= 12 ? 3 + lp - 12 : -1);
  if (l < NV && bi >= 0) {
#pragma unroll
    for (int c = 0; c < 3; c++) col[9 * bi + c] = e[c];
#pragma unroll
    for (int c = 0; c < 6; c++) col[9 * bi + 3 + c] = a[12 + c];
    col[84 + bi] = rhs;
  }
  SYNC();
  float S[9][9], y[9];
#pragma unroll
  for (int q = 0; q < 84; q += 4) {
    const float4 v = *reinterpret_cast<const float4*>(col + q);
    const float w4[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int u = 0; u < 4; u++)
      if (q + u < 81) S[(q + u) / 9][(q + u) % 9] = w4[u];
  }
  {
    const float4 v0 = *reinterpret_cast<const float4*>(col + 84);
    const float4 v1 = *reinterpret_cast<const float4*>(col + 88);
    y[0] = v0.x; y[1] = v0.y; y[2] = v0.z; y[3] = v0.w;
    y[4] = v1.x; y[5] = v1.y; y[6] = v1.z; y[7] = v1.w;
    y[8] = col[92];
  }
  SYNC();  // col is rewritten by the next use
  float db[9];
#pragma unroll
  for (int k = 0; k < 9; ++k) {
    const float ik = frcp(fmaxf(S[k][k], MINVAL));
    db[k] = ik;
#pragma unroll
    for (int i = 8; i > k; --i) {  // descending: rows below still hold their unscaled column k
      const float lik = S[i][k] * ik;
#pragma unroll
      for (int j = k + 1; j <= i; ++j) S[i][j] -= lik * S[j][k];
      S[i][k] = lik;
    }
  }
#pragma unroll
  for (int c = 1; c < 9; c++)
#pragma unroll
    for (int k = 0; k < c; k++) y[c] = y[c] - S[c][k] * y[k];
#pragma unroll
  for (int c = 0; c < 9; c++) y[c] = y[c] * db[c];
#pragma unroll
  for (int c = 7; c >= 0; --c)
#pragma unroll
    for (int i = 8; i > c; --i) y[c] = y[c] - S[i][c] * y[i];
  // the other legs' rows: U x = y from registers (lb and base parts) and the rows below in the
  // same leg (DPP), as in ldl_arrow_solve
  const int li = lp < 12 ? lp - 3 * (lp / 3) : 3;
  float t = rhs;
#pragma unroll
  for (int c = 0; c < 3; c++) t -= e[c] * y[c];
#pragma unroll
  for (int c = 0; c < 6; c++) t -= a[12 + c] * y[3 + c];
  const float u1 = a[1] + a[4] + a[7] + a[10], u2 = a[2] + a[5] + a[8] + a[11];
  float x = t * dinv;
  float v1 = dpp_shl1(x);
  x = (li == 1) ? (t - u2 * v1) * dinv : x;
  v1 = dpp_shl1(x);
  const float v2 = dpp_shl2(x);
  x = (li == 0) ? (t - u1 * v1 - u2 * v2) * dinv : x;
#pragma unroll
  for (int c = 0; c < 9; c++) x = (bi == c) ? y[c] : x;
  return x;
}

// a[npos(j)] += w . J[.][j] over natural columns [J0, J1) (arrowhead Hessian rows)
template <int J0, int J1, int W>
__device__ __forceinline__ void hess_acc_p(float (&a)[NV], const float (&J)[3][W], float w0, float w1, float w2) {
  static_assert(J1 <= W, "hess_acc_p: columns beyond the operand rows");
#pragma unroll
  for (int j = J0; j < J1; j++) {  // three FMAs into the entry (not mul + 2 fma + add)
    float v = a[npos(j)];
    v = fmaf(w0, J[0][j], v);
    v = fmaf(w1, J[1][j], v);
    a[npos(j)] = fmaf(w2, J[2][j], v);
  }
}

// (M x)[pnat(l)] from this lane's permuted M row held in registers (mrow[j] = M[pnat(l)][pnat(j)])
// and the LDS vector x (16-byte aligned, read as broadcast b128 words): no per-element LDS round
// trip.  The sum runs in permuted column order.
__device__ __forceinline__ float mrow_dot_reg(const float (&mrow)[NV], const float* x) {
  float xv[20];
#pragma unroll
  for (int q = 0; q < 20; q += 4) {
    const float4 v = *reinterpret_cast<const float4*>(x + q);
    xv[q] = v.x; xv[q + 1] = v.y; xv[q + 2] = v.z; xv[q + 3] = v.w;
  }
  float acc = 0;
#pragma unroll
  for (int j = 0; j < NV; j++) acc += mrow[j] * xv[pnat(j)];
  return acc;
}

// J row r dotted with K LDS vectors in one pass (the row's J entries loaded once).  Branch-light:
// frictionloss rows (one dof), limit rows (one dof, signed) and pyramidal contact rows are all
// evaluated with clamped indices and the row's value selected, instead of three divergent
// branches per call.  Contact rows: support = base + one leg (base-only contacts: that leg's
// columns are zero), in ascending column order, so skipping exact zeros leaves the sums
// bit-identical; a leg-leg contact anywhere in the wave (rare) takes full rows.  nl / ncon come
// from the caller's registers, so the row's metadata (limit dof and sign, contact support and
// friction) is one round of independent LDS loads, and the sparse path's J entries and vector
// entries are a second round, pinned so they issue back to back and retire with one wait.
typedef float v2f __attribute__((ext_vector_type(2)));
template <int NC, int K>
__device__ __forceinline__ void row_dotk(const Shared<NC>& s, int r, int nl, int ncon, const float* const (&xs)[K],
                                         float (&out)[K]) {
  const bool isf = r < NFR, isl = !isf && r < NFR + nl;
  const int li = isl ? r - NFR : 0;
  const int e0 = r - NFR - nl, e = e0 < 0 ? 0 : e0;
  const int c = (e >> 2) < NC ? (e >> 2) : NC - 1, ed = e & 3, t = 1 + (ed >> 1);
  const bool isc = !isf && !isl && (e0 >> 2) < ncon;
  const float sg = (ed & 1) ? -1.0f : 1.0f;
  const int ld = s.lim_dof[li];
  const float ls = s.lim_sgn[li];
  const int sup = s.con_sup[c];
  const float mu = s.con_mu[c];
  const int col1 = isf ? 6 + r : (isl ? ld : 0);  // (never an uninitialised index)
  const float sg1 = isf ? 1.0f : ls;
  float a[K], b[K];
#pragma unroll
  for (int k = 0; k < K; k++) { a[k] = 0.0f; b[k] = 0.0f; }
  if (__ballot(isc && (sup & 7) == 5)) {
#pragma unroll
    for (int i = 0; i < NV; i++) {
      const float j0 = s.Jc[c][0][i], jt = s.Jc[c][t][i];
#pragma unroll
      for (int k = 0; k < K; k++) { a[k] += j0 * xs[k][i]; b[k] += jt * xs[k][i]; }
    }
  } else {
    const int o = 6 + 3 * (sup & 3);
    v2f jj[9];      // (J normal, J tangent) of the row's 9 support columns
    float xv[K][9];
    float x1[K];    // the single-dof rows' entry
#pragma unroll
    for (int i = 0; i < 9; i++) {
      const int col = i < 6 ? i : o + i - 6;
      jj[i] = v2f{s.Jc[c][0][col], s.Jc[c][t][col]};
#pragma unroll
      for (int k = 0; k < K; k++) xv[k][i] = xs[k][col];
    }
#pragma unroll
    for (int k = 0; k < K; k++) x1[k] = xs[k][col1];
    if constexpr (K == 1) {
      PIN("+v"(jj[0]), "+v"(jj[1]), "+v"(jj[2]), "+v"(jj[3]), "+v"(jj[4]), "+v"(jj[5]), "+v"(jj[6]), "+v"(jj[7]),
          "+v"(jj[8]), "+v"(xv[0][0]), "+v"(xv[0][1]), "+v"(xv[0][2]), "+v"(xv[0][3]), "+v"(xv[0][4]),
          "+v"(xv[0][5]), "+v"(xv[0][6]), "+v"(xv[0][7]), "+v"(xv[0][8]), "+v"(x1[0]));
    } else {
      static_assert(K == 2, "row_dotk: K = 1 or 2");
      PIN("+v"(jj[0]), "+v"(jj[1]), "+v"(jj[2]), "+v"(jj[3]), "+v"(jj[4]), "+v"(jj[5]), "+v"(jj[6]), "+v"(jj[7]),
          "+v"(jj[8]), "+v"(xv[0][0]), "+v"(xv[0][1]), "+v"(xv[0][2]), "+v"(xv[0][3]), "+v"(xv[0][4]),
          "+v"(xv[0][5]), "+v"(xv[0][6]), "+v"(xv[0][7]), "+v"(xv[0][8]), "+v"(xv[1][0]), "+v"(xv[1][1]),
          "+v"(xv[1][2]), "+v"(xv[1][3]), "+v"(xv[1][4]), "+v"(xv[1][5]), "+v"(xv[1][6]), "+v"(xv[1][7]),
          "+v"(xv[1][8]), "+v"(x1[0]), "+v"(x1[1]));
    }
#pragma unroll
    for (int i = 0; i < 9; i++)
#pragma unroll
      for (int k = 0; k < K; k++) { a[k] += jj[i].x * xv[k][i]; b[k] += jj[i].y * xv[k][i]; }
#pragma unroll
    for (int k = 0; k < K; k++) out[k] = (isf || isl) ? sg1 * x1[k] : a[k] + sg * mu * b[k];
    return;
  }
#pragma unroll
  for (int k = 0; k < K; k++) out[k] = (isf || isl) ? sg1 * xs[k][col1] : a[k] + sg * mu * b[k];
}
// J row r dotted with x (LDS vector)
template <int NC>
__device__ __forceinline__ float row_dot(const Shared<NC>& s, int r, int nl, int ncon, const float* x) {
  const float* const xs[1] = {x};
  float o[1];
  row_dotk<NC, 1>(s, r, nl, ncon, xs, o);
  return o[0];
}
// J row r dotted with two LDS vectors in one pass
template <int NC>
__device__ __forceinline__ void row_dot2(const Shared<NC>& s, int r, int nl, int ncon, const float* x, const float* y,
                                         float& rx, float& ry) {
  const float* const xs[2] = {x, y};
  float o[2];
  row_dotk<NC, 2>(s, r, nl, ncon, xs, o);
  rx = o[0];
  ry = o[1];
}

// a[j] += w . J[.][j] over the columns [J0, J1) (base: 0..6, leg g: 6+3g..9+3g, dense: 0..18)
template <int J0, int J1>
__device__ __forceinline__ void hess_acc(float (&a)[NV], const float (&J)[3][NV], float w0, float w1, float w2) {
#pragma unroll
  for (int j = J0; j < J1; j++) a[j] = fmaf(w2, J[2][j], fmaf(w1, J[1][j], fmaf(w0, J[0][j], a[j])));
}

// index drawn by jax.random.choice(p) from u = uniform(key): searchsorted_left(cumsum(p), cumsum[-1]*(1-u))
// (n <= PP3_MAX_LAG; unrolled over the cap so the wave-uniform dist reads are one scalar load)
__device__ __forceinline__ int choice_from_uniform(const GFloat* dist, int n, float u) {
  // the whole (fixed-size) table first: one batch of scalar loads and one wait, not a load and a
  // wait behind every `i < n` branch (16 serial round trips per call)
  float d[PP3_MAX_LAG];
#pragma unroll
  for (int i = 0; i < PP3_MAX_LAG; i++) d[i] = dist[i];
  float total = 0.0f;
#pragma unroll
  for (int i = 0; i < PP3_MAX_LAG; i++)
    if (i < n) total += d[i];
  const float r = total * (1.0f - u);
  float acc = 0.0f;
  int li = 0;
#pragma unroll
  for (int i = 0; i < PP3_MAX_LAG; i++)
    if (i < n) {
      acc += d[i];
      li += (acc < r) ? 1 : 0;
    }
  return li < n ? li : n - 1;
}

// Newton direction with a leg-leg contact (rare): out of line, so its registers and code do not
// shape the allocation and scheduling of the arrowhead path.  When every leg-leg contact of an
// env involves one leg lb (the usual case: one pair of legs touching), the Hessian is arrowhead
// with lb counted in the base block (ldl_arrow_solve_b); otherwise the dense LDL^T below.
template <int NC>
using LdsShared = __attribute__((address_space(3))) Shared<NC>;
template <int NC>
__device__ __attribute__((noinline)) void dense_search(LdsShared<NC>* sp, int l, int h, int cmax, int ncon, int lsup) {
  Shared<NC>& s = *(Shared<NC>*)sp;
  {
    // per half: the leg common to all of its leg-leg contacts (sup = 5 | 8 | lo << 4 | hi << 6)
    const bool ll = (lsup & 7) == 5;
    const bool known = (lsup & 8) != 0;
    const int p = (lsup >> 4) & 3, q = (lsup >> 6) & 3;
    const uint64_t bll = __ballot(ll), bunk = __ballot(ll && !known);
    uint64_t bl[4];
#pragma unroll
    for (int g = 0; g < 4; g++) bl[g] = __ballot(ll && known && (p == g || q == g));
    int lbh[2];
    bool okh[2];
#pragma unroll
    for (int hh = 0; hh < 2; hh++) {
      const uint64_t hm = hh ? 0xFFFFFFFF00000000ull : 0xFFFFFFFFull;
      const int n = __popcll(bll & hm);
      int b = 0;
      bool found = false;
#pragma unroll
      for (int g = 3; g >= 0; g--)
        if (__popcll(bl[g] & hm) == n) { b = g; found = true; }
      okh[hh] = found && (bunk & hm) == 0;
      lbh[hh] = b;
    }
    if (okh[0] && okh[1]) {
      const int lb = h ? lbh[1] : lbh[0];
      const int lp = l < NV ? l : NV - 1, dn = pnat(lp);  // permuted row held by this lane
      float a[NV];
#pragma unroll
      for (int j = 0; j < NV; j++) a[j] = s.M[dn][pnat(j)];
      const float dD = s.dofD[dn];
#pragma unroll
      for (int j = 0; j < NV; j++) a[j] += (j == lp) ? dD : 0.0f;
      for (int c = 0; c < cmax; c++) {
        const int sa = __builtin_amdgcn_readlane(lsup, c), sb = __builtin_amdgcn_readlane(lsup, HW + c);
        if (c < ncon) {
          const float* G = s.con_G[c];
          const float jn = s.Jc[c][0][dn], j1 = s.Jc[c][1][dn], j2 = s.Jc[c][2][dn];
          const float w0 = jn * G[0] + j1 * G[1] + j2 * G[2];
          const float w1 = jn * G[1] + j1 * G[3];
          const float w2 = jn * G[2] + j2 * G[4];
          // a leg-leg contact: every leg block (the legs it does not touch have zero columns)
          const bool any = (sa & 7) == 5 || (sb & 7) == 5;
          hess_acc_p<0, 6>(a, s.Jc[c], w0, w1, w2);
          if (any || sa == 0 || sb == 0) hess_acc_p<6, 9>(a, s.Jc[c], w0, w1, w2);
          if (any || sa == 1 || sb == 1) hess_acc_p<9, 12>(a, s.Jc[c], w0, w1, w2);
          if (any || sa == 2 || sb == 2) hess_acc_p<12, 15>(a, s.Jc[c], w0, w1, w2);
          if (any || sa == 3 || sb == 3) hess_acc_p<15, 18>(a, s.Jc[c], w0, w1, w2);
        }
      }
      const float x = ldl_arrow_solve_b(a, s.grad[dn], l, &s.x.L[0][0], lb);
      if (l < NV) s.search[dn] = -x;
      return;
    }
  }
  const int li = l < NV ? l : NV - 1;
  float a[NV], dinv = 1.0f;
#pragma unroll
  for (int j = 0; j < NV; j++) a[j] = s.M[li][j];
  const float dD = s.dofD[li];
#pragma unroll
  for (int j = 0; j < NV; j++) a[j] += (j == li) ? dD : 0.0f;
  for (int c = 0; c < cmax; c++) {
    if (c < ncon) {
      const float* G = s.con_G[c];
      const float jn = s.Jc[c][0][li], j1 = s.Jc[c][1][li], j2 = s.Jc[c][2][li];
      const float w0 = jn * G[0] + j1 * G[1] + j2 * G[2];
      const float w1 = jn * G[1] + j1 * G[3];
      const float w2 = jn * G[2] + j2 * G[4];
      hess_acc<0, NV>(a, s.Jc[c], w0, w1, w2);
    }
  }
  ldl_rows(a, dinv, l, &s.x.L[0][0]);
  const float x = ldl_solve(s, a, dinv, s.grad[li], l, h);
  if (l < NV) s.search[l] = -x;
}

// ------------------------------------------------------------------------------------
// one physics substep (mj_step): forward + Newton + Euler.  `integrate` = false for reset
// (mj_forward only).  Must be called by all 64 lanes (both halves).
// ------------------------------------------------------------------------------------
template <int NC, int NWV = 1, bool LIBSC = true, bool CULL = false>
__device__ __forceinline__ int substep(Shared<NC>& s, const DevModel& m, int l, int h, bool integrate_prev,
                                       const KinConst& kc PROF_PARAM, float* ccache = nullptr) {
  constexpr int NR = (Shared<NC>::NEFC + HW - 1) / HW;  // constraint rows per lane
  l = opaque_lane(l);
  // the com and M-entry phases' lane records, loaded here without a wait: they arrive while
  // kinematics runs (a pinned fetch at the phase itself costs a round trip there)
  LaneRec<2> rc_pf;
  LaneRec<3> rm_pf;
  {
    v4f v[5];
#pragma unroll
    for (int k = 0; k < 2; k++) v[k] = *reinterpret_cast<const v4f*>(m.lane_com.g[k][l]);
#pragma unroll
    for (int k = 0; k < 2; k++)
      for (int c = 0; c < 4; c++) rc_pf.f[4 * k + c] = v[k][c];
#pragma unroll
    for (int k = 0; k < 3; k++) v[2 + k] = *reinterpret_cast<const v4f*>(m.lane_m.g[k][l]);
#pragma unroll
    for (int k = 0; k < 3; k++)
      for (int c = 0; c < 4; c++) rm_pf.f[4 * k + c] = v[2 + k][c];
  }
  kinematics<NC, LIBSC>(s, m, l, integrate_prev, kc); SYNC();
  PHASE(0); l = opaque_lane(l);
  { com_pos(s, m, l, h, rc_pf); SYNC(); }
  PHASE(1); l = opaque_lane(l);
  // the narrow phase's pair records for this lane's first pair, loaded without a wait: they arrive
  // during CRB x cdof and the RNE chain (issued at the substep start they measured 0.3 % slower in
  // v22: 28 more registers live through kinematics and com)
  const PairLoad pair_pf = load_pair(m, l < m.npair ? l : 0);
  // ---- phase 3: CRB*cdof, RNE chain, collision, actuation/passive, limit + friction rows ----
  { crb_times_cdof(s, m, l); rne_chain(s, m, l); SYNC(); }
  PHASE(15); l = opaque_lane(l);
  int lsup = 4;  // lane c: support of contact c (4 = none)
  { lsup = collision<NC, NWV, CULL>(s, m, l, h, pair_pf, ccache); SYNC(); }
  PHASE(16); l = opaque_lane(l);
  // the PairCon of contact c = l / 4 for the first batch of phase 13's edge rows (lane e = 4c + k),
  // loaded here unpinned: it arrives during the limit/actuation and M-entry phases
  v4f pcv[4];
  {
    const int c = l >> 2;
    const int p = c < s.ncon ? s.con_pair[c < NC ? c : 0] : 0;
    const v4f* src = reinterpret_cast<const v4f*>(&m.pair_con[p]);
#pragma unroll
    for (int k = 0; k < 4; k++) pcv[k] = src[k];
  }
  {
    const LaneRec<7> rl = fetch_rec(m.lane_lim, l);
    // every LDS operand of the phase in one pinned round, indices clamped on the lanes that do
    // not use them (read inside the lane branches below, each was a round trip of its own)
    const int jlim = l < 2 * (NJ - 1) ? 1 + (l >> 1) : 1;
    const bool actl = l < NU;
    const int adof = actl ? as_i(rl.f[LL_ACT_DOF]) : 0, aqadr = actl ? as_i(rl.f[LL_ACT_QADR]) : 0;
    float lq = s.qpos[7 + jlim - 1], lqv = s.qvel[6 + jlim - 1], fqv = s.qvel[6 + (l < NFR ? l : 0)];
    float actrl = s.ctrl[actl ? l : 0], aq = s.qpos[aqadr], aqv = s.qvel[adof];
    float skp = s.kp, skd = s.kd;
    int sdr = s.dr_on;
    PIN("+v"(lq), "+v"(lqv), "+v"(fqv), "+v"(actrl), "+v"(aq), "+v"(aqv), "+v"(skp), "+v"(skd), "+v"(sdr));
    // joint limits: lane = 2*(j-1) + side_hi, rows ordered like the oracle (mj_instantiateLimit)
    bool act = false;
    float value = 0;
    int j = 0;
    if (l < 2 * (NJ - 1)) {
      j = 1 + (l >> 1);
      const float side = (l & 1) ? 1.0f : -1.0f;
      if (as_i(rl.f[LL_LIM_ON])) {
        value = side * (rl.f[LL_RANGE] - lq);
        act = value < rl.f[LL_MARGIN];
      }
    }
    const uint32_t mask = hballot(act, h);
    const int slot = __popc(mask & ((1u << l) - 1u));
    if (act && slot < NLMAX) {  // (<= one side per hinge: never more than NLMAX rows)
      const int dof = 6 + j - 1;
      const float sg = (l & 1) ? -1.0f : 1.0f;  // J = -side
      s.lim_dof[slot] = dof;
      s.lim_sgn[slot] = sg;
      const float imp = getimp(&rl.f[LL_SOLIMP], value, rl.f[LL_MARGIN]);
      const float R = fmaxf(MINVAL, (1.0f - imp) / imp * rl.f[LL_INVW]);
      const int r = NFR + slot;
      s.efc_R[r] = R;
      s.efc_D[r] = 1.0f / R;
      s.efc_aref[r] = -rl.f[LL_B] * (sg * lqv) - rl.f[LL_K] * imp * (value - rl.f[LL_MARGIN]);
      (void)dof;
    }
    if (l == 0) s.nl = __popc(mask) < NLMAX ? __popc(mask) : NLMAX;
    if (l < NFR) {  // dof frictionloss rows (R, b precomputed: pos = 0)
      const int dof = 6 + l;
      s.efc_R[l] = rl.f[LL_FR_R];
      s.efc_D[l] = 1.0f / rl.f[LL_FR_R];
      s.efc_aref[l] = -rl.f[LL_FR_B] * fqv;
      (void)dof;
    }
    if (l < NU) {  // actuation (affine PD + force clamp)
      const int d = adof, flags = as_i(rl.f[LL_ACT_FLAGS]);
      float ctrl = actrl;
      if (flags & ACTF_CTRLLIMITED) ctrl = fminf(fmaxf(ctrl, rl.f[LL_CRANGE]), rl.f[LL_CRANGE + 1]);
      const float gear = rl.f[LL_GEAR];
      const float len = gear * aq, vel = gear * aqv;
      float gain = rl.f[LL_GAIN], b0 = rl.f[LL_BIAS], b1 = rl.f[LL_BIAS + 1], b2 = rl.f[LL_BIAS + 2];
      if (sdr) { gain = skp; b1 = -skp; b2 = -skd; }
      float force = gain * ctrl;
      if (flags & ACTF_AFFINE) force += b0 + b1 * len + b2 * vel;
      if (flags & ACTF_FORCELIMITED) force = fminf(fmaxf(force, rl.f[LL_FRANGE]), rl.f[LL_FRANGE + 1]);
      s.qfrc_act[d] = gear * force;
    }
    if (l < 6) s.qfrc_act[l] = 0.0f;
  }
  SYNC();
  PHASE(2); l = opaque_lane(l);
  // ---- phase 4: M entries, RNE body forces, contact Jacobians ----
  const LaneRec<3> rm = rm_pf;  // (prefetched at the substep start; also read by phases 13 and 7)
  
  // every M pair's twelve operands in one LDS round (pinned; lanes without a pair read row 0):
  // otherwise each pair waits for its own loads, behind the previous pair's stores
  constexpr int NT = (NMPAIR + HW - 1) / HW;  // compile-time trip count
  float cd[NT][6], fi[NT][6];
#pragma unroll
  for (int t = 0; t < NT; t++) {
    const int ij = as_i(rm.f[LM_IJ + t]);
    const int i = ij < 0 ? 0 : (ij & 0xff), j = ij < 0 ? 0 : (ij >> 8);
#pragma unroll
    for (int k = 0; k < 6; k++) { cd[t][k] = s.cdof[j][k]; fi[t][k] = s.x.a.F[i][k]; }
  }
#pragma unroll
  for (int t = 0; t < NT; t++)
    PIN("+v"(cd[t][0]), "+v"(cd[t][1]), "+v"(cd[t][2]), "+v"(cd[t][3]), "+v"(cd[t][4]), "+v"(cd[t][5]),
        "+v"(fi[t][0]), "+v"(fi[t][1]), "+v"(fi[t][2]), "+v"(fi[t][3]), "+v"(fi[t][4]), "+v"(fi[t][5]));
#pragma unroll
  for (int t = 0; t < NT; t++) {
    const int ij = as_i(rm.f[LM_IJ + t]);
    if (ij < 0) continue;
    const int i = ij & 0xff, j = ij >> 8;
    float v = 0;
#pragma unroll
    for (int k = 0; k < 6; k++) v += cd[t][k] * fi[t][k];
    v += rm.f[LM_ARM + t];  // armature on the diagonal, 0 elsewhere
    s.M[i][j] = v;
    s.M[j][i] = v;
  }
  rne_body_forces(s, l, h);
  const int ncon = s.ncon;
  __builtin_assume(ncon >= 0 && ncon <= NC);  // (collision caps it): NC = 8 -> one edge-row pass
  for (int it = l; it < ncon * NV; it += HW) {
    const int c = it / NV, i = it - c * NV;
    const uint32_t bit = 1u << i;
    // every operand loaded up front and pinned (one LDS round), then the three stores: otherwise
    // each load is placed after the previous store (possible alias) and waited for on its own
    float cp[3], cm[3], cd[6], fr[9];
    uint32_t dm0 = s.con_dm[c][0], dm1 = s.con_dm[c][1];
#pragma unroll
    for (int k = 0; k < 3; k++) { cp[k] = s.x.a.con_pos[c][k]; cm[k] = s.com[k]; }
#pragma unroll
    for (int k = 0; k < 6; k++) cd[k] = s.cdof[i][k];
#pragma unroll
    for (int k = 0; k < 9; k++) fr[k] = s.x.a.con_frame[c][k];
    PIN("+v"(cp[0]), "+v"(cp[1]), "+v"(cp[2]), "+v"(cm[0]), "+v"(cm[1]), "+v"(cm[2]), "+v"(cd[0]), "+v"(cd[1]),
        "+v"(cd[2]), "+v"(cd[3]), "+v"(cd[4]), "+v"(cd[5]), "+v"(fr[0]), "+v"(fr[1]), "+v"(fr[2]), "+v"(fr[3]),
        "+v"(fr[4]), "+v"(fr[5]), "+v"(fr[6]), "+v"(fr[7]), "+v"(fr[8]), "+v"(dm0), "+v"(dm1));
    const float off[3] = {cp[0] - cm[0], cp[1] - cm[1], cp[2] - cm[2]};
    float cr[3], jp[3];
    cross3(cr, cd, off);
    const float w = ((dm1 & bit) ? 1.0f : 0.0f) - ((dm0 & bit) ? 1.0f : 0.0f);
    for (int k = 0; k < 3; k++) jp[k] = w * (cd[3 + k] + cr[k]);
    s.Jc[c][0][i] = fr[0] * jp[0] + fr[1] * jp[1] + fr[2] * jp[2];
    s.Jc[c][1][i] = fr[3] * jp[0] + fr[4] * jp[1] + fr[5] * jp[2];
    s.Jc[c][2][i] = fr[6] * jp[0] + fr[7] * jp[1] + fr[8] * jp[2];
  }
  SYNC();
  PHASE(3); l = opaque_lane(l);
  // ---- phase 5: qfrc_bias/smooth (subtree sums of body forces), contact edge rows ----
  {
  if (l < NV) {
    // base dofs: the whole tree's cfrc; a leg link: itself + the (<= 2) links below (cacc holds
    // cfrc now; dof 6+3g+k <-> body 2+3g+k, checked at create).  Every operand (32 words) in one
    // pinned LDS round, the base/leg choice a select: unpinned, the links' rows and the cdof row
    // were loaded a register pair at a time, each waited for
    const bool base = l < 6;
    const int b = base ? 2 : l - 4, last = 2 + 3 * ((b - 2) / 3) + 2;
    const int b1 = b + 1 <= last ? b + 1 : b, b2 = b + 2 <= last ? b + 2 : b;
    float r0[6], c0[6], c1[6], c2[6], cdv[6];
#pragma unroll
    for (int k = 0; k < 6; k++) {
      r0[k] = s.cfrc_base[k];
      c0[k] = s.x.a.cacc[b][k];
      c1[k] = s.x.a.cacc[b1][k];
      c2[k] = s.x.a.cacc[b2][k];
      cdv[k] = s.cdof[l][k];
    }
    float qv = s.qvel[l], qa = s.qfrc_act[l];
    PIN("+v"(r0[0]), "+v"(r0[1]), "+v"(r0[2]), "+v"(r0[3]), "+v"(r0[4]), "+v"(r0[5]), "+v"(c0[0]), "+v"(c0[1]),
        "+v"(c0[2]), "+v"(c0[3]), "+v"(c0[4]), "+v"(c0[5]), "+v"(cdv[0]), "+v"(cdv[1]), "+v"(cdv[2]), "+v"(cdv[3]),
        "+v"(cdv[4]), "+v"(cdv[5]), "+v"(qv), "+v"(qa));
    PIN("+v"(c1[0]), "+v"(c1[1]), "+v"(c1[2]), "+v"(c1[3]), "+v"(c1[4]), "+v"(c1[5]), "+v"(c2[0]), "+v"(c2[1]),
        "+v"(c2[2]), "+v"(c2[3]), "+v"(c2[4]), "+v"(c2[5]));
    const float w1 = b + 1 <= last ? 1.0f : 0.0f, w2 = b + 2 <= last ? 1.0f : 0.0f;
    float cf[6];
#pragma unroll
    for (int k = 0; k < 6; k++) {
      float t = c0[k];
      t += w1 * c1[k];
      t += w2 * c2[k];
      cf[k] = base ? r0[k] : t;
    }
    float bias = 0;
    for (int k = 0; k < 6; k++) bias += cdv[k] * cf[k];
    s.qfrc_smooth[l] = -rm.f[LM_DAMP] * qv - bias + qa;
  }
  }
  const int nl = s.nl;
  __builtin_assume(nl >= 0 && nl <= NLMAX);
  const int nefc = NFR + nl + 4 * ncon;
  for (int e = l; e < 4 * ncon; e += HW) {
    const int c = e >> 2, p = s.con_pair[c], r = NFR + nl + e;
    LaneRec<4> pc;
    if (e < HW) {  // first batch (every row when 4 * ncon <= 32): prefetched after the collision
#pragma unroll
      for (int k = 0; k < 4; k++)
#pragma unroll
        for (int cc = 0; cc < 4; cc++) pc.f[4 * k + cc] = pcv[k][cc];
    } else {
      pc = fetch_rec(*reinterpret_cast<const LaneRec<4>*>(&m.pair_con[p]));
    }
    const PairCon& q = *reinterpret_cast<const PairCon*>(&pc);
    const float mu = s.con_mu[c];
    const float dist = s.con_dist[c];
    const float vel = row_dot(s, r, nl, ncon, s.qvel);
    const float tran = q.tran;
    const float invw = (tran + mu * mu * tran) * 2.0f * mu * mu / m.impratio;
    const float imp = getimp(q.solimp, dist, q.margin);
    const float R = fmaxf(MINVAL, (1.0f - imp) / imp * invw);
    s.efc_R[r] = R;
    s.efc_D[r] = 1.0f / R;
    s.efc_aref[r] = -q.b * vel - q.k * imp * (dist - q.margin);
  }
  SYNC();
  PHASE(13); l = opaque_lane(l);
  // ---- phase 6: qacc_smooth = M^-1 qfrc_smooth (register LDL) ----
  float mrow[NV];  // this lane's permuted row of M, kept for the Newton Hessian (no second load)
  {
    const int lp = l < NV ? l : NV - 1, dn = pnat(lp);  // permuted row held by this lane
    float a[NV];
#pragma unroll
    for (int j = 0; j < NV; j++) { a[j] = s.M[dn][pnat(j)]; mrow[j] = a[j]; }
    const float x = ldl_arrow_solve(a, s.qfrc_smooth[dn], l, &s.x.L[0][0]);
    if (l < NV) s.qacc_smooth[dn] = x;
  }
  SYNC();
  PHASE(4); l = opaque_lane(l);

  // ---- phase 7: Newton solver (mj_solNewton), warm-started ----
  // per-lane rows r = l + HW * t
  float Dr[NR], Rr[NR], ar[NR], fl[NR];
  bool valid[NR], isfr[NR];
#pragma unroll
  for (int t = 0; t < NR; t++) {
    const int r = l + HW * t;
    valid[t] = r < nefc;
    isfr[t] = r < NFR;
    Dr[t] = valid[t] ? s.efc_D[r] : 0.0f;
    Rr[t] = valid[t] ? s.efc_R[r] : 0.0f;
    ar[t] = valid[t] ? s.efc_aref[r] : 0.0f;
    fl[t] = (valid[t] && isfr[t]) ? rm.f[LM_FLOSS] : 0.0f;  // row r = l (t = 0) for frictionloss rows
  }
  // warm start: total cost at qacc_warmstart vs at qacc_smooth.  J qacc and M qacc of the first
  // Newton iteration are one of the two candidates' products (qacc is a copy of one of them), so
  // they are kept instead of recomputed.
  float cws = 0, csm = 0;
  float xws[NR], xsm[NR], ma_ws = 0.0f;
  bool use_smooth;
  {
#pragma unroll
    for (int t = 0; t < NR; t++) {
      xws[t] = 0.0f;
      xsm[t] = 0.0f;
      if (!valid[t]) continue;
      const int r = l + HW * t;
      float d1, d2;
      row_dot2(s, r, nl, ncon, s.qws, s.qacc_smooth, d1, d2);
      const float x1 = d1 - ar[t];
      const float x2 = d2 - ar[t];
      xws[t] = x1;
      xsm[t] = x2;
      // both row kinds' costs as selects (a wave holds both kinds, so both were executed anyway,
      // behind exec-mask branches)
      const float rf = Rr[t] * fl[t];
      const float q1 = 0.5f * Dr[t] * x1 * x1, q2 = 0.5f * Dr[t] * x2 * x2;
      const float f1 = (x1 <= -rf) ? (-fl[t] * x1 - 0.5f * rf * fl[t]) : (x1 >= rf) ? (fl[t] * x1 - 0.5f * rf * fl[t]) : q1;
      const float f2 = (x2 <= -rf) ? (-fl[t] * x2 - 0.5f * rf * fl[t]) : (x2 >= rf) ? (fl[t] * x2 - 0.5f * rf * fl[t]) : q2;
      cws += isfr[t] ? f1 : ((x1 < 0) ? q1 : 0.0f);
      csm += isfr[t] ? f2 : ((x2 < 0) ? q2 : 0.0f);
    }
    PHASE(23);  // (prof build: warm-start row costs; phase 5 is then M qws, the sums and the choice)
    if (l < NV) {  // lane l: dof dn = pnat(l), the row it holds in mrow
      const int dn = pnat(l);
      ma_ws = mrow_dot_reg(mrow, s.qws);
      cws += 0.5f * (ma_ws - s.qfrc_smooth[dn]) * (s.qws[dn] - s.qacc_smooth[dn]);
    }
    cws = hsum(cws, h);
    csm = hsum(csm, h);
    use_smooth = cws > csm;
    if (l < NV) s.qacc[l] = use_smooth ? s.qacc_smooth[l] : s.qws[l];
  }
  SYNC();
  PHASE(5); l = opaque_lane(l);
  const int cmax = wmax2(ncon);
  __builtin_assume(cmax >= 0 && cmax <= NC);
  int weight = cmax;  // returned: the wave's load this substep (contacts, +2 on the leg-leg path)
  bool live = true;  // this env still iterating (per half)
  for (int iter = 0; iter < m.iterations; iter++) {
    // Ma, Jaref, constraint state/force
    float ma = 0;  // (M qacc)[pnat(l)], kept in this lane's register through the line search
    if (l < NV) {
      if (iter > 0 || use_smooth) ma = mrow_dot_reg(mrow, s.qacc);
      else ma = ma_ws;
    }
    float jar[NR];
#pragma unroll
    for (int t = 0; t < NR; t++) {
      jar[t] = 0;
      if (!valid[t]) continue;
      const int r = l + HW * t;
      const float x = iter > 0 ? row_dot(s, r, nl, ncon, s.qacc) - ar[t] : (use_smooth ? xsm[t] : xws[t]);
      jar[t] = x;
      // constraint state and force, as selects (the nested branches cost more exec-mask scalar
      // instructions than the few selects): frictionloss rows linear below -R f / above +R f,
      // quadratic between; contact and limit rows zero when x >= 0, quadratic below
      const float rf = Rr[t] * fl[t];
      const float fq = -Dr[t] * x;
      const bool lo = isfr[t] && x <= -rf;
      const bool hi = !lo && (isfr[t] ? x >= rf : x >= 0);
      const float f = lo ? fl[t] : (hi ? (isfr[t] ? -fl[t] : 0.0f) : fq);
      const float Dq = (lo || hi) ? 0.0f : Dr[t];
      s.efc_force[r] = f;
      s.efc_D[r] = Dq;  // active D (0 when not quadratic) for the Hessian
    }
    SYNC();
    PHASE(22);  // (prof build: constraint state update; phase 6 is then the gradient and G blocks)
    // gradient, diagonal D per dof, contact Hessian blocks
    float gauss = 0;
    if (l < NV) {  // lane l: dof dn = pnat(l) (its (M qacc) entry is ma)
      const int dn = pnat(l);
      float qc = 0;
      if (dn >= 6) qc += s.efc_force[dn - 6];
      float dD = (dn >= 6) ? s.efc_D[dn - 6] : 0.0f;
      for (int i = 0; i < nl; i++)
        if (s.lim_dof[i] == dn) { qc += s.lim_sgn[i] * s.efc_force[NFR + i]; dD += s.efc_D[NFR + i]; }
      for (int c = 0; c < ncon; c++) {
        const int r = NFR + nl + 4 * c;
        const float f0 = s.efc_force[r], f1 = s.efc_force[r + 1], f2 = s.efc_force[r + 2], f3 = s.efc_force[r + 3];
        const float mu = s.con_mu[c];
        qc += s.Jc[c][0][dn] * (f0 + f1 + f2 + f3) + mu * s.Jc[c][1][dn] * (f0 - f1) + mu * s.Jc[c][2][dn] * (f2 - f3);
      }
      s.grad[dn] = ma - s.qfrc_smooth[dn] - qc;
      s.dofD[dn] = dD;
      gauss = 0.5f * (ma - s.qfrc_smooth[dn]) * (s.qacc[dn] - s.qacc_smooth[dn]);
    }
    for (int c = l; c < ncon; c += HW) {
      const int r = NFR + nl + 4 * c;
      const float mu = s.con_mu[c];
      const float d0 = s.efc_D[r], d1 = s.efc_D[r + 1], d2 = s.efc_D[r + 2], d3 = s.efc_D[r + 3];
      s.con_G[c][0] = d0 + d1 + d2 + d3;
      s.con_G[c][1] = mu * (d0 - d1);
      s.con_G[c][2] = mu * (d2 - d3);
      s.con_G[c][3] = mu * mu * (d0 + d1);
      s.con_G[c][4] = mu * mu * (d2 + d3);
    }
    gauss = hsum(gauss, h);
    SYNC();
    PHASE(6); l = opaque_lane(l);
    // Hessian rows H = M + J' D J (registers), LDL^T, search = -H^-1 grad.  Contacts that
    // touch one leg (+ base) keep H arrowhead -> tree-sparse LDL in permuted order; a contact
    // coupling two legs (either env of the wave) switches the wave to the dense factorisation.
    {
      const bool dense = __ballot((lsup & 7) == 5) != 0;  // a leg-leg contact in either env
      weight = cmax + (dense ? 2 : 0);
#ifdef PP3_PHASE_PROF
      if (pf) {
        pf->dense += dense ? 1u : 0u;
        pf->ncmax = pf->ncmax > (uint32_t)cmax ? pf->ncmax : (uint32_t)cmax;
        pf->csum += (uint32_t)cmax;
      }
#endif
      if (!dense) {
        const int lp = l < NV ? l : NV - 1, dn = pnat(lp);
        float a[NV];
#pragma unroll
        for (int j = 0; j < NV; j++) a[j] = mrow[j];
        const float dD = s.dofD[dn];
        // the diagonal D on this lane's own column: a[j] + dD * [j == lp] as one fma per column
        // (dD >= 0, so the other columns add +0 exactly as a + 0.0f did), the 0/1 factor from a
        // bit field -- no per-column VCC compare and the wait states a v_cndmask needs after it
        const uint32_t onehot = 1u << lp;
#pragma unroll
        for (int j = 0; j < NV; j++) a[j] = fmaf(dD, (float)((onehot >> j) & 1u), a[j]);
        for (int c = 0; c < cmax; c++) {
          const bool cv = c < ncon;
          const int sa = __builtin_amdgcn_readlane(lsup, c), sb = __builtin_amdgcn_readlane(lsup, HW + c);
          // the legs either env's contact c touches, as one scalar bit set (arrowhead path: supports
          // 0..3 = a leg, 4 = base only): one bit test per leg instead of two compares and an or
          const uint32_t legs = (1u << (sa & 7)) | (1u << (sb & 7));
          if (cv) {
            // the contact's G, this lane's three J entries and the 18 base-column entries in ONE
            // pinned LDS round: unpinned, the base columns streamed three loads deep behind the
            // weights (the last serial LDS chain on the substep's path, tools/lds_chains.py)
            float G[5], jb[3][6];
#pragma unroll
            for (int k = 0; k < 5; k++) G[k] = s.con_G[c][k];
            float jn = s.Jc[c][0][dn], j1 = s.Jc[c][1][dn], j2 = s.Jc[c][2][dn];
#pragma unroll
            for (int r = 0; r < 3; r++)
#pragma unroll
              for (int j = 0; j < 6; j++) jb[r][j] = s.Jc[c][r][j];
            PIN("+v"(G[0]), "+v"(G[1]), "+v"(G[2]), "+v"(G[3]), "+v"(G[4]), "+v"(jn), "+v"(j1), "+v"(j2),
                "+v"(jb[0][0]), "+v"(jb[0][1]), "+v"(jb[0][2]), "+v"(jb[0][3]), "+v"(jb[0][4]), "+v"(jb[0][5]),
                "+v"(jb[1][0]), "+v"(jb[1][1]), "+v"(jb[1][2]), "+v"(jb[1][3]), "+v"(jb[1][4]), "+v"(jb[1][5]),
                "+v"(jb[2][0]), "+v"(jb[2][1]), "+v"(jb[2][2]), "+v"(jb[2][3]), "+v"(jb[2][4]), "+v"(jb[2][5]));
            const float w0 = jn * G[0] + j1 * G[1] + j2 * G[2];
            const float w1 = jn * G[1] + j1 * G[3];
            const float w2 = jn * G[2] + j2 * G[4];
            hess_acc_p<0, 6>(a, jb, w0, w1, w2);
            if (legs & 1u) hess_acc_p<6, 9>(a, s.Jc[c], w0, w1, w2);
            if (legs & 2u) hess_acc_p<9, 12>(a, s.Jc[c], w0, w1, w2);
            if (legs & 4u) hess_acc_p<12, 15>(a, s.Jc[c], w0, w1, w2);
            if (legs & 8u) hess_acc_p<15, 18>(a, s.Jc[c], w0, w1, w2);
          }
        }
        PHASE(14); l = opaque_lane(l);
        const float x = ldl_arrow_solve(a, s.grad[dn], l, &s.x.L[0][0]);
        if (l < NV) s.search[dn] = -x;
      } else {
        dense_search<NC>((LdsShared<NC>*)&s, l, h, cmax, ncon, lsup);
      }
    }
    SYNC();
    PHASE(7); l = opaque_lane(l);
    // line-search quadratics (Gauss part) and search-direction norm
    float q1 = 0, q2 = 0, sn = 0;
    if (l < NV) {  // lane l: dof pnat(l)
      const int dn = pnat(l);
      const float sv = s.search[dn];
      const float mv = mrow_dot_reg(mrow, s.search);
      q1 = sv * (ma - s.qfrc_smooth[dn]);
      q2 = 0.5f * sv * mv;
      sn = sv * sv;
    }
    float jv[NR];
#pragma unroll
    for (int t = 0; t < NR; t++) jv[t] = valid[t] ? row_dot(s, l + HW * t, nl, ncon, s.search) : 0.0f;
    // Each row's cost on the line qacc + alpha*search is piecewise quadratic in alpha: the three
    // pieces' coefficients (below the lower switch point, above the upper one, in between) are
    // alpha-independent and computed once here; an evaluation only picks the piece per row.
    // Contact / limit rows: quadratic below 0, zero above; frictionloss rows: linear below -R f,
    // linear above +R f, quadratic in between (engine_solver.c PrimalSearch cost).
    float thr_lo[NR], thr_hi[NR], cq[NR][3], clo[NR][2], chi[NR][2];
    bool rowany[NR];
#pragma unroll
    for (int t = 0; t < NR; t++) {
      const float D = Dr[t], jr = jar[t], jw = jv[t];
      cq[t][0] = valid[t] ? 0.5f * D * jr * jr : 0.0f;
      cq[t][1] = valid[t] ? D * jr * jw : 0.0f;
      cq[t][2] = valid[t] ? 0.5f * D * jw * jw : 0.0f;
      const float rf = Rr[t] * fl[t];
      const bool fr = valid[t] && isfr[t];
      thr_lo[t] = fr ? -rf : -INFINITY;
      thr_hi[t] = fr ? rf : (valid[t] ? 0.0f : INFINITY);
      clo[t][0] = fr ? -fl[t] * jr - 0.5f * rf * fl[t] : 0.0f;
      clo[t][1] = fr ? -fl[t] * jw : 0.0f;
      chi[t][0] = fr ? fl[t] * jr - 0.5f * rf * fl[t] : 0.0f;
      chi[t][1] = fr ? fl[t] * jw : 0.0f;
      rowany[t] = __ballot(valid[t]) != 0;  // wave-uniform: skip row slots no lane uses
    }
#ifdef PP3_PHASE_PROF
    if (pf && NR > 1 && rowany[NR - 1]) pf->slot2++;
#endif
    // this half's row pieces of the 1-D piecewise quadratic at alpha (alpha is per half)
    auto pieces = [&](float alpha, float& t0, float& t1, float& t2) {
      // row slot 0 always holds rows (the NFR frictionloss rows come first): its pieces start the
      // sums instead of being added to zeros
      static_assert(NFR > 0, "row slot 0 is never empty");
#pragma unroll
      for (int t = 0; t < NR; t++) {
        if (t > 0 && !rowany[t]) continue;
        const float x = jar[t] + alpha * jv[t];
        const bool lo = x <= thr_lo[t], hi = !lo && x >= thr_hi[t], qd = !lo && !hi;
        const float p0 = lo ? clo[t][0] : (hi ? chi[t][0] : cq[t][0]);
        const float p1 = lo ? clo[t][1] : (hi ? chi[t][1] : cq[t][1]);
        const float p2 = qd ? cq[t][2] : 0.0f;
        if (t == 0) { t0 = p0; t1 = p1; t2 = p2; }
        else { t0 += p0; t1 += p1; t2 += p2; }
      }
    };
    // cost and derivatives at alpha from the half-summed pieces
    auto finish = [&](float alpha, float t0, float t1, float t2, float& cost, float& d0, float& d1) {
      t0 = t0 + gauss;
      t1 = t1 + q1;
      t2 = t2 + q2;
      cost = t0 + alpha * t1 + alpha * alpha * t2;
      d0 = t1 + 2.0f * alpha * t2;
      d1 = fmaxf(2.0f * t2, MINVAL);
    };
    // the first evaluation (alpha = 0) needs nothing the direction's sums produce: its three sums
    // run beside them (six independent DPP chains) instead of after them
    float e0s0, e0s1, e0s2;
    pieces(0.0f, e0s0, e0s1, e0s2);
    e0s0 = hsum(e0s0, h);
    e0s1 = hsum(e0s1, h);
    e0s2 = hsum(e0s2, h);
    q1 = hsum(q1, h);
    q2 = hsum(q2, h);
    sn = sqrtf(hsum(sn, h));
    live = live && !(sn < MINVAL);
    const float gtol = m.gtol_scale * sn;
    PHASE(21);  // (prof build: the line search's setup ends here; phase 8 is then its evaluations)
    auto eval = [&](float alpha, float& cost, float& d0, float& d1) {
      float t0, t1, t2;
      pieces(alpha, t0, t1, t2);
      finish(alpha, hsum(t0, h), hsum(t1, h), hsum(t2, h), cost, d0, d1);
    };
    // converged at (alpha, d0, d1): MuJoCo's |d0| < gtol, or the remaining Newton correction
    // |d0 / d1| within LS_NOISE roundoffs of alpha -- the fp32 floor below which the search would
    // only move alpha by rounding noise (the oracle's ls_converged, FLT_EPSILON in its float build)
    auto conv = [&](float a, float d0, float d1) {
      return fabsf(d0) < gtol || fabsf(d0) <= LS_NOISE * FLT_EPSILON * d1 * fabsf(a);
    };
    // PrimalSearch-style exact line search (same control flow as the oracle); every branch
    // below is per env (per half), the wave runs the union of both envs' evaluations
    float alpha = 0.0f;
    int evals = 0;
    if (live) {
      const int maxit = m.ls_iterations;
      float c0, g0, h0;
      finish(0.0f, e0s0, e0s1, e0s2, c0, g0, h0);
      evals++;
      float a1 = -g0 / h0, c1, g1, h1;
      eval(a1, c1, g1, h1);
      evals++;
      if (c0 < c1) { a1 = 0.0f; c1 = c0; g1 = g0; h1 = h0; }
      if (conv(a1, g1, h1)) {
        alpha = a1;
      } else {
        const float dir = g1 < 0 ? 1.0f : -1.0f;
        float a2 = a1, c2 = c1, g2 = g1, h2 = h1;
        bool done = false;
        while (g1 * dir <= -gtol && evals < maxit) {
          a2 = a1; c2 = c1; g2 = g1; h2 = h1;
          a1 = a1 - g1 / h1;
          eval(a1, c1, g1, h1);
          evals++;
          if (conv(a1, g1, h1)) { done = true; break; }
        }
        if (done || evals >= maxit) {
          alpha = a1;
        } else {
          // bracket [p2, p1]; candidates p1next, p2next (= p1 initially), midpoint
          float a2n = a1, c2n = c1, g2n = g1, h2n = h1;
          float a1n = a1 - g1 / h1, c1n, g1n, h1n;
          eval(a1n, c1n, g1n, h1n);
          evals++;
          bool finished = false;
          alpha = c1 < c2 ? a1 : a2;
          while (evals < maxit) {
            const float am = 0.5f * (a1 + a2);
            float cm, gm, hm;
            eval(am, cm, gm, hm);
            evals++;
            // converged candidate with the lowest cost (order: p1next, p2next, mid)
            bool ok0 = conv(a1n, g1n, h1n), ok1 = conv(a2n, g2n, h2n), ok2 = conv(am, gm, hm);
            if (ok0 || ok1 || ok2) {
              float ba = ok0 ? a1n : (ok1 ? a2n : am), bc = ok0 ? c1n : (ok1 ? c2n : cm);
              if (ok1 && c2n < bc) { ba = a2n; bc = c2n; }
              if (ok2 && cm < bc) { ba = am; bc = cm; }
              alpha = ba;
              finished = true;
              break;
            }
            bool up1 = false, up2 = false;
#define PP3_TIGHTEN(CA, CC, CG, CH)                                                          \
  if (g1 * (CG) > 0 && fabsf(CG) < fabsf(g1)) { a1 = CA; c1 = CC; g1 = CG; h1 = CH; up1 = true; } \
  if (g2 * (CG) > 0 && fabsf(CG) < fabsf(g2)) { a2 = CA; c2 = CC; g2 = CG; h2 = CH; up2 = true; }
            PP3_TIGHTEN(a1n, c1n, g1n, h1n)
            PP3_TIGHTEN(a2n, c2n, g2n, h2n)
            PP3_TIGHTEN(am, cm, gm, hm)
#undef PP3_TIGHTEN
            if (!up1 && !up2) break;
            if (up1) { a1n = a1 - g1 / h1; eval(a1n, c1n, g1n, h1n); evals++; }
            if (up2) { a2n = a2 - g2 / h2; eval(a2n, c2n, g2n, h2n); evals++; }
          }
          if (!finished) alpha = c1 < c2 ? a1 : a2;
        }
      }
    }
#ifdef PP3_PHASE_PROF
    {
      const int ew = wmax2(evals);
      if (pf) pf->evals += ew;
      PROF_ADD(19, ew);
      PROF_ADD(20, evals);       // env 2b's evaluations (lane 20 is in the first half)
      PROF_ADD(HW + 20, evals);  // env 2b+1's
    }
#endif
    PHASE(8); l = opaque_lane(l);
#ifdef PP3_DEBUG
    if (blockIdx.x == 0 && h == 0) {
      if (l < NV) { g_dbg[l] = s.qacc[l]; g_dbg[18 + l] = s.grad[l]; g_dbg[36 + l] = s.search[l]; }
      if (l == 0) {
        g_dbg[54] = gauss; g_dbg[55] = q1; g_dbg[56] = q2; g_dbg[57] = sn; g_dbg[58] = gtol;
        g_dbg[59] = alpha; g_dbg[60] = (float)evals; g_dbg[61] = cws; g_dbg[62] = csm; g_dbg[63] = (float)nefc;
      }
    }
#endif
    live = live && alpha != 0.0f;
    if (live && l < NV) s.qacc[l] += alpha * s.search[l];
    SYNC();
  }
  if (l < NV) s.qws[l] = s.qacc[l];
  // the forward's velocity, kept for the sensors of the pipeline record (efc_aref is dead until
  // the next substep rebuilds its rows)
  if (l < NV) s.efc_aref[l] = s.qvel[l];
  SYNC();
  return weight;  // the Euler step follows in the next substep's kinematics or in euler_step
}

// ---- phase 8: Euler (eulerdamp disabled) of the last substep of a step (the earlier ones run
// fused into the next substep's kinematics) ----
template <int NC, bool LIBSC = true>
__device__ __forceinline__ void euler_step(Shared<NC>& s, const DevModel& m, int l) {
  const float hstep = m.h;
  float vn = 0;
  float w[3] = {0, 0, 0};
  if (l < NV) vn = s.qvel[l] + hstep * s.qacc[l];
  if (l == 3)
    for (int k = 0; k < 3; k++) w[k] = s.qvel[3 + k] + hstep * s.qacc[3 + k];
  SYNC();
  if (l < NV) s.qvel[l] = vn;
  if (l < 3) s.qpos[l] += hstep * vn;
  if (l >= 6 && l < NV) s.qpos[l + 1] += hstep * vn;
  if (l == 3) {
    const float n = sqrtf(dot3(w, w));
    if (n < MINVAL) { w[0] = 1; w[1] = 0; w[2] = 0; } else { const float in = 1.0f / n; w[0] *= in; w[1] *= in; w[2] *= in; }
    float qr[4], q[4] = {s.qpos[3], s.qpos[4], s.qpos[5], s.qpos[6]};
    axisangle2quat<LIBSC>(qr, w, hstep * n);
    normalize4(q);
    mulquat(q, q, qr);
    for (int k = 0; k < 4; k++) s.qpos[3 + k] = q[k];
  }
  SYNC();
}

// ------------------------------------------------------------------------------------
// environment helpers
// ------------------------------------------------------------------------------------
template <int NC>
__device__ __forceinline__ void load_params(Shared<NC>& s, const DevModel& m, const float* dr, int l) {
  if (l < NB) {
    s.mass[l] = dr ? dr[PP3_DR_MASS + l] : m.body_mass[l];
    for (int k = 0; k < 3; k++) {
      s.inertia[l][k] = dr ? dr[PP3_DR_INERTIA + 3 * l + k] : m.body_inertia[l][k];
      s.ipos[l][k] = (dr && l == 1) ? dr[PP3_DR_BASE_IPOS + k] : m.body_ipos[l][k];
    }
  }
  if (l == 0) {
    s.dr_on = dr != nullptr;
    s.fric = dr ? dr[PP3_DR_FRICTION] : 0.0f;
    s.kp = dr ? dr[PP3_DR_KP] : 0.0f;
    s.kd = dr ? dr[PP3_DR_KD] : 0.0f;
  }
  // zero M once per launch (its sparsity pattern is fixed)
  for (int i = l; i < NV * (NV + 1); i += HW) (&s.M[0][0])[i] = 0.0f;
}

// sample_lagged_value on one buffer row in HBM (utils.py:34-69): push `v` to the front of
// row[0..n), return the value now at column li.  Register-staged (read all, then write).
__device__ __forceinline__ float push_lagged(float* row, int n, float v, int li, bool store) {
  float old[PP3_MAX_LAG];
#pragma unroll
  for (int q = 0; q < PP3_MAX_LAG; q++) old[q] = q < n ? row[q] : 0.0f;
  float out = v;
#pragma unroll
  for (int q = 0; q < PP3_MAX_LAG; q++) {
    const float nv = q == 0 ? v : old[q - 1];
    if (store && q < n) row[q] = nv;
    out = (q == li) ? nv : out;
  }
  return out;
}

// push_lagged with the row's old values already loaded (prefetched at kernel start)
__device__ __forceinline__ float push_lagged_pre(float* row, int n, float v, int li, bool store, const float* old) {
  float out = v;
#pragma unroll
  for (int q = 0; q < PP3_MAX_LAG; q++) {
    const float nv = q == 0 ? v : old[q - 1];
    if (store && q < n) row[q] = nv;
    out = (q == li) ? nv : out;
  }
  return out;
}

// sample_command (environment.py:246-272): lanes 0..6 draw, lane 0 writes out[3]
__device__ __forceinline__ void sample_command(const DevModel& m, Key rng, float* out, int l, int h) {
  const int part = m.partitionable;
  float u = 0;
  if (l < 3) {
    const Key k = split_i(rng, 6, 1 + l, part);
    const float lo = l == 0 ? m.cmd_x[0] : l == 1 ? m.cmd_y[0] : m.cmd_w[0];
    const float hi = l == 0 ? m.cmd_x[1] : l == 1 ? m.cmd_y[1] : m.cmd_w[1];
    u = uniform_i(k, 1, 0, lo, hi, part);
  } else if (l == 3) {
    u = uniform_i(split_i(rng, 6, 4, part), 1, 0, 0.0f, 1.0f, part);
  } else if (l < 7) {
    u = uniform_i(split_i(rng, 6, 5, part), 3, l - 4, -m.stand_thr, m.stand_thr, part);
  }
  const bool zero = hb(u, 3, h) < m.zero_cmd_p;
  const float c0 = hb(u, 0, h), c1 = hb(u, 1, h), c2 = hb(u, 2, h);
  const float z0 = hb(u, 4, h), z1 = hb(u, 5, h), z2 = hb(u, 6, h);
  if (l == 0) {
    out[0] = zero ? z0 : c0;
    out[1] = zero ? z1 : c1;
    out[2] = zero ? z2 : c2;
  }
}

// sample_body_orientation (environment.py:274-298), brax math.euler_to_quat (degrees)
__device__ __forceinline__ void sample_orientation(const DevModel& m, Key rng, float* out, int l, int h) {
  const int part = m.partitionable;
  float u = 0;
  if (l < 2) u = uniform_i(split_i(rng, 3, 1 + l, part), 1, 0, -1.0f, 1.0f, part);
  const float pitch = hb(u, 0, h) * m.max_pitch;
  const float roll = hb(u, 1, h) * m.max_roll;
  if (l == 0) {
    const float pi = m.pi_f;
    const float c1 = cosf(roll * pi / 360.0f), c2 = cosf(pitch * pi / 360.0f), c3 = 1.0f;
    const float s1 = sinf(roll * pi / 360.0f), s2 = sinf(pitch * pi / 360.0f), s3 = 0.0f;
    const float q[4] = {c1 * c2 * c3 - s1 * s2 * s3, s1 * c2 * c3 + c1 * s2 * s3, c1 * s2 * c3 - s1 * c2 * s3,
                        c1 * c2 * s3 + s1 * s2 * c3};
    float r[3];
    b_rotate(r, m.des_z, q);
    out[0] = r[0]; out[1] = r[1]; out[2] = r[2];
  }
}

// _get_obs (environment.py:485-543): consumes the st rng, pushes the IMU buffer (HBM row
// gimu = [6][Li]), writes s.x.e.o[36]
template <int NC>
__device__ __forceinline__ void get_obs(Shared<NC>& s, const DevModel& m, float* gimu, int l, int h, float pose16, bool store,
                                        const float* imu_stash PROF_PARAM) {
  const int part = m.partitionable;
  const Key rng{__float_as_uint(s.st[PP3_S_RNG]), __float_as_uint(s.st[PP3_S_RNG + 1])};
  const Key kl = split_i(rng, 6, l < 6 ? l : 0, part);  // lane i holds split(rng, 6)[i]
  const Key k0 = hkey(kl, 0, h), ka = hkey(kl, 1, h), kg = hkey(kl, 2, h);
  const Key km = hkey(kl, 3, h), kla = hkey(kl, 4, h), ki = hkey(kl, 5, h);
  // noise draws: 0-2 ang, 3-5 grav, 6-17 motor, 18-29 last act, 30 imu choice
  if (l < 31) {
    const Key kk = l < 3 ? ka : l < 6 ? kg : l < 18 ? km : l < 30 ? kla : ki;
    const int cnt = l < 6 ? 3 : l < 30 ? 12 : 1;
    const int idx = l < 3 ? l : l < 6 ? l - 3 : l < 18 ? l - 6 : l < 30 ? l - 18 : 0;
    const float scale = l < 3 ? m.n_ang : l < 6 ? m.n_grav : l < 18 ? m.n_motor : l < 30 ? m.n_act : 1.0f;
    const float lo = l < 30 ? -1.0f : 0.0f;
    const float v = uniform_i(kk, cnt, idx, lo, 1.0f, part);
    s.x.e.u[l] = l < 30 ? v * scale : v;
  }
  SYNC();
  PHASE(17);
  if (l < 6) {  // one IMU channel per lane
    float inv[4] = {1, 0, 0, 0}, angl[3] = {0, 0, 0};
    if (m.use_imu) {
      inv[0] = s.xquat[1][0]; inv[1] = -s.xquat[1][1]; inv[2] = -s.xquat[1][2]; inv[3] = -s.xquat[1][3];
      b_rotate(angl, s.cvel[1], inv);
    }
    const float g0[3] = {0, 0, -1};
    float g[3];
    b_rotate(g, g0, inv);
    for (int k = 0; k < 3; k++) g[k] += s.x.e.u[3 + k];
    const float gn = sqrtf(dot3(g, g));
    const float v = l < 3 ? angl[l] + s.x.e.u[l] : g[l - 3] / gn;
    const int li = choice_from_uniform((const GFloat*)m.imu_lat_dist, m.Li, s.x.e.u[30]);
    float lagged;
    if (imu_stash) {  // the row's old values were fetched at kernel start (one memory round trip)
      float old[PP3_MAX_LAG];
#pragma unroll
      for (int q = 0; q < PP3_MAX_LAG; q++) old[q] = imu_stash[PP3_MAX_LAG * l + q];
      lagged = push_lagged_pre(gimu + l * m.Li, m.Li, v, li, store, old);
    } else {
      lagged = push_lagged(gimu + l * m.Li, m.Li, v, li, store);
    }
    s.x.e.o[l] = fminf(fmaxf(lagged, -100.0f), 100.0f);
  }
  if (l == 6) {
    s.st[PP3_S_RNG] = __uint_as_float(k0.a);
    s.st[PP3_S_RNG + 1] = __uint_as_float(k0.b);
  }
  if (l >= 8 && l < 11) {
    const int k = l - 8;
    s.x.e.o[6 + k] = fminf(fmaxf(s.st[PP3_S_COMMAND + k], -100.0f), 100.0f);
    s.x.e.o[9 + k] = fminf(fmaxf(s.st[PP3_S_DESIRED_Z + k], -100.0f), 100.0f);
  }
  if (l >= 16 && l < 28) {
    const int j = l - 16;
    const float a = s.qpos[7 + j] - pose16 + s.x.e.u[6 + j];
    const float b = s.st[PP3_S_LAST_ACT + j] + s.x.e.u[18 + j];
    s.x.e.o[12 + j] = fminf(fmaxf(a, -100.0f), 100.0f);
    s.x.e.o[24 + j] = fminf(fmaxf(b, -100.0f), 100.0f);
  }
  SYNC();
  PHASE(18);
}

template <int NC>
__device__ __forceinline__ void write_obs(Shared<NC>& s, const DevModel& m, const float* obs_in, float* obs_out,
                                          int l, bool store) {
  const int nmove = PP3_OBS_DIM * (m.H - 1);
  float tmp[OBS_MOVE];
#pragma unroll
  for (int t = 0; t < OBS_MOVE; t++) {
    const int k = l + HW * t;
    tmp[t] = (k < nmove && obs_in) ? obs_in[k] : 0.0f;
  }
  if (!store) return;
#pragma unroll
  for (int t = 0; t < OBS_MOVE; t++) {
    const int k = l + HW * t;
    if (k < nmove) obs_out[PP3_OBS_DIM + k] = tmp[t];
  }
  for (int k = l; k < PP3_OBS_DIM; k += HW) obs_out[k] = s.x.e.o[k];
}

// mjData.sensordata from the last forward: mj_sensorPos/Vel/Acc with mj_objectVelocity /
// mj_objectAcceleration, cacc by mj_rnePostConstraint's recursion along the site body's path
// (oracle/pp3_oracle.c sensors() is the same restatement).  s.efc_aref holds the forward's qvel
// (stashed before integration).
// Sensor lane l (< nsensor) from its host-flattened record (LS_*): every model word fetched in one
// round instead of dependent lane-indexed loads (sensor -> site -> body -> chain), and the frame's
// LDS operands pinned.
template <int NC>
__device__ __forceinline__ void sensor_eval_rec(const Shared<NC>& s, const DevModel& m, const LaneRec<(LS_WORDS + 3) / 4>& r,
                                                float* out) {
  const int typ = as_i(r.f[LS_TYPE]), b = as_i(r.f[LS_BODY]);
  const float* qv = s.efc_aref;
  float xq[4], xb[3], cm[3], cvb[6];
#pragma unroll
  for (int k = 0; k < 4; k++) xq[k] = s.xquat[b][k];
#pragma unroll
  for (int k = 0; k < 3; k++) { xb[k] = s.xpos[b][k]; cm[k] = s.com[k]; }
#pragma unroll
  for (int k = 0; k < 6; k++) cvb[k] = s.cvel[b][k];
  PIN("+v"(xq[0]), "+v"(xq[1]), "+v"(xq[2]), "+v"(xq[3]), "+v"(xb[0]), "+v"(xb[1]), "+v"(xb[2]), "+v"(cm[0]),
      "+v"(cm[1]), "+v"(cm[2]), "+v"(cvb[0]), "+v"(cvb[1]), "+v"(cvb[2]), "+v"(cvb[3]), "+v"(cvb[4]), "+v"(cvb[5]));
  const float spos[3] = {r.f[LS_SPOS], r.f[LS_SPOS + 1], r.f[LS_SPOS + 2]};
  const float squat[4] = {r.f[LS_SQUAT], r.f[LS_SQUAT + 1], r.f[LS_SQUAT + 2], r.f[LS_SQUAT + 3]};
  float Rb[9], sq[4], R[9], sx[3], off[3], dif[3], cr[3], vang[3], vlin[3], v[4] = {0, 0, 0, 0};
  quat2mat(xq, Rb);
  matvec(off, Rb, spos);
  for (int k = 0; k < 3; k++) sx[k] = xb[k] + off[k];
  mulquat(sq, xq, squat);
  quat2mat(sq, R);
  for (int k = 0; k < 3; k++) { dif[k] = sx[k] - cm[k]; vang[k] = cvb[k]; }
  cross3(cr, dif, vang);
  for (int k = 0; k < 3; k++) vlin[k] = cvb[3 + k] - cr[k];
  int dim = 3;
  if (typ == PP3_SENS_FRAMEPOS) { for (int k = 0; k < 3; k++) v[k] = sx[k]; }
  else if (typ == PP3_SENS_FRAMEQUAT) { for (int k = 0; k < 4; k++) v[k] = sq[k]; dim = 4; }
  else if (typ == PP3_SENS_FRAMELINVEL) { for (int k = 0; k < 3; k++) v[k] = vlin[k]; }
  else if (typ == PP3_SENS_FRAMEANGVEL) { for (int k = 0; k < 3; k++) v[k] = vang[k]; }
  else if (typ == PP3_SENS_GYRO || typ == PP3_SENS_VELOCIMETER) {
    const float* w = typ == PP3_SENS_GYRO ? vang : vlin;
    for (int k = 0; k < 3; k++) v[k] = R[k] * w[0] + R[3 + k] * w[1] + R[6 + k] * w[2];
  } else if (typ == PP3_SENS_ACCELEROMETER) {
    const int n = as_i(r.f[LS_NCH]);
    float ca[6] = {0, 0, 0, -m.gravity[0], -m.gravity[1], -m.gravity[2]};
    for (int c = 0; c < n; c++) {  // root first
      const int d0 = as_i(r.f[LS_CH + 4 * c + 1]), nd = as_i(r.f[LS_CH + 4 * c + 2]);
      const int pb = as_i(r.f[LS_CH + 4 * c + 3]);
      float pv[6] = {0, 0, 0, 0, 0, 0};  // velocity the body's dof_dot terms see (parent, + free translation)
      if (pb > 0)
        for (int k = 0; k < 6; k++) pv[k] = s.cvel[pb][k];
      if (nd == 6)
        for (int d = d0; d < d0 + 3; d++)
          for (int k = 0; k < 6; k++) pv[k] += s.cdof[d][k] * qv[d];
      float t1[6] = {0, 0, 0, 0, 0, 0}, t2[6] = {0, 0, 0, 0, 0, 0};
      for (int d = d0; d < d0 + nd; d++) {
        float cdd[6] = {0, 0, 0, 0, 0, 0};
        if (!(nd == 6 && d < d0 + 3)) cross_motion(cdd, pv, s.cdof[d]);
        for (int k = 0; k < 6; k++) { t1[k] += cdd[k] * qv[d]; t2[k] += s.cdof[d][k] * s.qacc[d]; }
      }
      for (int k = 0; k < 6; k++) ca[k] = ca[k] + t1[k] + t2[k];
    }
    float aang[3] = {ca[0], ca[1], ca[2]}, alin[3], wl[3], vl[3], c2[3];
    cross3(cr, dif, aang);
    for (int k = 0; k < 3; k++) alin[k] = ca[3 + k] - cr[k];
    for (int k = 0; k < 3; k++) {
      v[k] = R[k] * alin[0] + R[3 + k] * alin[1] + R[6 + k] * alin[2];
      wl[k] = R[k] * vang[0] + R[3 + k] * vang[1] + R[6 + k] * vang[2];
      vl[k] = R[k] * vlin[0] + R[3 + k] * vlin[1] + R[6 + k] * vlin[2];
    }
    cross3(c2, wl, vl);
    for (int k = 0; k < 3; k++) v[k] += c2[k];
  }
  const float co = r.f[LS_CUT];
  if (co > 0 && typ != PP3_SENS_FRAMEQUAT)
    for (int k = 0; k < 3; k++) v[k] = fminf(fmaxf(v[k], -co), co);
  const int adr = as_i(r.f[LS_ADR]);
  for (int k = 0; k < dim; k++) out[adr + k] = v[k];
}

// The Brax pipeline record of this env (PP3_P_* layout).  Every element below the sensors is one
// LDS word (x, its velocities as the epilogue's s.x.e.xdv / xda, site positions, qfrc_actuator,
// qacc, the contact fields, subtree com): the lane selects its element's word per 32-element block
// (the block bounds are compile-time), all blocks' loads issue as one pinned round, then one
// coalesced store per block; the contact geoms take one more round (pair -> geom ids).
template <int NC>
__device__ __forceinline__ void write_pipeline(Shared<NC>& s, const DevModel& m, float* p, int l, bool have_xd = true) {
  const LaneRec<(LS_WORDS + 3) / 4> rsens = fetch_rec(m.lane_sens, l);  // (arrives during the element loads)
  if (!have_xd) {  // (reset / bare physics launches: Brax xd as the step's epilogue computes it)
    if (l >= 1 && l < NB) {
      float off[3], cv[6], cr[3];
      for (int k = 0; k < 6; k++) cv[k] = s.cvel[l][k];
      for (int k = 0; k < 3; k++) off[k] = s.xpos[l][k] - s.com[k];
      cross3(cr, cv, off);
      for (int k = 0; k < 3; k++) { s.x.e.xdv[l][k] = cv[3 + k] + cr[k]; s.x.e.xda[l][k] = cv[k]; }
    }
    SYNC();
  }
  const float* w = reinterpret_cast<const float*>(&s);
  const int o_xpos = (int)(&s.xpos[1][0] - w), o_xq = (int)(&s.xquat[1][0] - w), o_xdv = (int)(&s.x.e.xdv[1][0] - w),
            o_xda = (int)(&s.x.e.xda[1][0] - w), o_foot = (int)(&s.foot_xpos[0][0] - w), o_fa = (int)(&s.qfrc_act[0] - w),
            o_qacc = (int)(&s.qacc[0] - w), o_cd = (int)(&s.con_dist[0] - w),
            o_cp = (int)(reinterpret_cast<const float*>(&s.con_pair[0]) - w), o_com = (int)(&s.com[0] - w),
            o_ncon = (int)(reinterpret_cast<const float*>(&s.ncon) - w),
            o_nhit = (int)(reinterpret_cast<const float*>(&s.nhit) - w);
  constexpr int NBLK = (PP3_P_SENSOR + HW - 1) / HW;
  float v[NBLK];
  int kind[NBLK];  // 0 float word, 1 int word, 2 zero, 3 contact distance, 4 contact geom
  int ncon = s.ncon;
#pragma unroll
  for (int t = 0; t < NBLK; t++) {
    const int i = l + HW * t;
    const int cdi = i - PP3_P_CON_DIST, cgi = (i - PP3_P_CON_GEOM) >> 1;
    const int cdc = cdi < NC ? cdi : NC - 1, cgc = cgi < NC ? cgi : NC - 1;
    int src = o_com, k = 2;
    if (i < PP3_P_XQUAT) { src = o_xpos + i; k = 0; }
    else if (i < PP3_P_XD_VEL) { src = o_xq + (i - PP3_P_XQUAT); k = 0; }
    else if (i < PP3_P_XD_ANG) { src = o_xdv + (i - PP3_P_XD_VEL); k = 0; }
    else if (i < PP3_P_SITE_XPOS) { src = o_xda + (i - PP3_P_XD_ANG); k = 0; }
    else if (i < PP3_P_QFRC_ACT) { src = o_foot + (i - PP3_P_SITE_XPOS); k = 0; }
    else if (i < PP3_P_QACC) { src = o_fa + (i - PP3_P_QFRC_ACT); k = 0; }
    else if (i < PP3_P_NCON) { src = o_qacc + (i - PP3_P_QACC); k = 0; }
    else if (i == PP3_P_NCON) { src = o_ncon; k = 1; }
    else if (i < PP3_P_CON_GEOM) { src = o_cd + cdc; k = 3; }
    else if (i < PP3_P_SUBTREE_COM) { src = o_cp + cgc; k = 4; }
    else if (i < PP3_P_SUBTREE_COM + 3) { src = o_com + (i - PP3_P_SUBTREE_COM); k = 0; }
    else if (i == PP3_P_NHIT) { src = o_nhit; k = 1; }
    kind[t] = k;
    v[t] = w[src];
  }
  static_assert(NBLK == 9, "write_pipeline: PIN arity");
  PIN("+v"(v[0]), "+v"(v[1]), "+v"(v[2]), "+v"(v[3]), "+v"(v[4]), "+v"(v[5]), "+v"(v[6]), "+v"(v[7]), "+v"(v[8]),
      "+v"(ncon));
  float out[NBLK];
#pragma unroll
  for (int t = 0; t < NBLK; t++) {
    const int i = l + HW * t;
    const int k = kind[t];
    const int cdi = i - PP3_P_CON_DIST, cgi = (i - PP3_P_CON_GEOM) >> 1;
    float o = v[t];
    if (k == 1) o = (float)as_i(v[t]);
    if (k == 2) o = 0.0f;
    if (k == 3) o = cdi < ncon ? v[t] : 0.0f;
    if (k == 4) {  // the pair's geom id (contacts c < ncon; 0 past them)
      const int pp = cgi < ncon ? as_i(v[t]) : 0;
      const float g = m.pair_gid[pp][(i - PP3_P_CON_GEOM) & 1];
      o = cgi < ncon ? g : 0.0f;
    }
    out[t] = o;
  }
#pragma unroll
  for (int t = 0; t < NBLK; t++)
    if (l + HW * t < PP3_P_SENSOR) p[l + HW * t] = out[t];
  if (l < m.nsensor) sensor_eval_rec(s, m, rsens, p + PP3_P_SENSOR);
  for (int i = PP3_P_SENSOR + m.nsensordata + l; i < PP3_PIPE_STRIDE; i += HW) p[i] = 0.0f;
}

// ------------------------------------------------------------------------------------
// kernels: workgroup b = one wave = envs 2b (lanes 0..31) and 2b+1 (lanes 32..63).  With an
// odd N the last wave's second half recomputes env N-1 and stores nothing.
// ------------------------------------------------------------------------------------
struct StepArgs;
typedef __attribute__((address_space(4))) const StepArgs GArgs;
struct StepArgs {
  const DevModel* m;
  float* state;          // [N][stride]
  const float* obs_in;   // [N][36H]
  float* obs_out;        // [N][36H]
  const float* actions;  // [N][12]
  float* reward;
  float* done;
  float* metrics;        // [N][19]
  const float* dr;       // [N][62] or null
  float* pipe;           // [N][PIPE] or null
  float* episode;        // [N][PP3_EP_STRIDE] (auto-reset mode) or null
  const float* first_state;  // [N][PP3_FIRST_STRIDE]
  const float* first_obs;    // [N][36H]
  int episode_length;
  int repeat, phase;  // auto-reset mode: action_repeat and this launch's repeat index
  int N;
  int nsteps;            // env steps per launch (a fused rollout: step t reads actions + t * act_stride)
  int64_t act_stride;
  float* traj_reward;    // fused rollout outputs, each optional: [nsteps][N]
  float* traj_done;      // [nsteps][N]
  float* traj_obs;       // [nsteps][N][36H]
};

// The fused policy rollout (pp3_rollout_policy): the env step kernel with eight waves = 16 envs
// per workgroup, whose waves run the exported MLP on their 16 envs' observations (pp3_mlp.h
// mlp_tile, the code of pp3_policy_act) before every step, into the step's action row.
struct PolicyStepArgs {
  StepArgs s;       // s.actions = act: step t reads the actions the MLP wrote at t * s.act_stride
  float* act;       // [nsteps][N][12] action trajectory (written by the MLP)
  pp3pol::Net net;  // the policy (device weight pointers)
};

// The policy's MLP on this workgroup's tile, out of line: its registers are allocated on their own
// instead of shaping the env step's allocation around it (inlined, the fused kernel spilled 17
// VGPRs).  Weight chunks of MLP_CG k-groups, no prefetch (chunks of 2 / 8 and a one-chunk-ahead
// prefetch measured neutral to slower: profiles/AB_LOG.md rounds 4-5).
constexpr int MLP_CG = 4;
__device__ __noinline__ void policy_mlp(pp3pol::KNet* net, const float* obs, int obs_stride, float* act, int n,
                                        int row0, pp3pol::LdsTileBuf* buf) {
  pp3pol::mlp_tile<pp3pol::KNet, pp3pol::LdsTileBuf, pp3pol::TileRows, MLP_CG>(
      *net, obs, obs_stride, act, NU, n, row0, *buf, threadIdx.x);
}
// The same with the observation rows already in the workgroup's LDS tile (observation_history
// <= 2: 36H <= OBS_TILE_W - 4 floats per row), written by the env steps themselves
constexpr int OBS_TILE_W = 2 * PP3_OBS_DIM + 4;
typedef __attribute__((address_space(3))) float LdsObsTile[pp3pol::TILE][OBS_TILE_W];
__device__ __noinline__ void policy_mlp_tile(pp3pol::KNet* net, float* act, int n, int row0, pp3pol::LdsTileBuf* buf,
                                             LdsObsTile* in) {
  pp3pol::mlp_tile<pp3pol::KNet, pp3pol::LdsTileBuf, LdsObsTile, MLP_CG>(
      *net, nullptr, 0, act, NU, n, row0, *buf, threadIdx.x, in);
}
// Between the fused steps every global value a wave reads back was stored by a wave of the same
// workgroup (the env step: by the same lane), so on the same CU: the acquire is at workgroup scope,
// which the gfx942/950 memory model (non-tgsplit) serves from the CU's own L1 without an invalidate
// (agent scope -- buffer_inv sc1, the whole vector L1 dropped every step -- measured 0.4 % slower on
// the env rollout and 35 us per step slower on the policy rollout: profiles/AB_LOG.md round 4).
#define PP3_STEP_ACQUIRE() __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup")

// Fused rollout, steps after the first: the wave keeps what the previous step left in the env's LDS
// block instead of reading it back from global memory (bitwise equal, +0.6 % over 200 fused steps,
// +0.7 % at the driver's window: profiles/AB_LOG.md round 5) -- the state record head (s.st is what
// was stored), the per-env parameters (load_params) and, with observation_history 2, the history
// frame (the previous step's newest observation, s.x.e.o).

// PP3_AB_ALIAS (timing probe only, tools/occ_probe.py): both halves of a wave share ONE env block
// in LDS -- correct only when the wave's two envs are identical (same reset key, actions, no DR), as
// the probe sets them up -- so a wave needs half the LDS and the occupancy a register budget of
// PP3_AB_WPE waves per SIMD allows can be timed on the real step code
#ifndef PP3_AB_ALIAS
#define PP3_AB_ALIAS 0
#endif
#if PP3_AB_ALIAS
#define PP3_STEP_WPE PP3_AB_WPE
#else
#define PP3_STEP_WPE 2
#endif
// CULL: models with obstacle boxes (DevModel::cull_on) launch the instantiation with the
// sphere-box cull of collision() compiled in; the flat model's code is the same without it
template <int NC, bool FUSED, int NWV = 1, bool CULL = false>
__global__ __launch_bounds__(WAVE * NWV, PP3_STEP_WPE) void env_step_kernel(
    typename std::conditional<(NWV > 1), PolicyStepArgs, StepArgs>::type a_arg) {
  static_assert(NWV == 1 || (FUSED && NWV == pp3pol::NWAVE), "the policy rollout is fused, one MLP tile per workgroup");
  constexpr bool alias = PP3_AB_ALIAS && NWV == 1;
  __shared__ Shared<NC> sh[alias ? 1 : 2 * NWV];
  static_assert(NWV == 1 || sizeof(sh) >= pp3pol::TILE_BUF_BYTES, "the MLP's LDS scratch aliases the envs' blocks");
  // the policy rollout's observation tile (its own LDS, next to the env blocks): each env step
  // writes its env's new observation row into it, the next step's MLP reads it in place
  __shared__ float obs_tile[NWV > 1 ? pp3pol::TILE : 1][OBS_TILE_W];
  int nsteps;
  if constexpr (NWV > 1) nsteps = a_arg.s.nsteps;
  else nsteps = FUSED ? a_arg.nsteps : 1;
  constexpr bool TG = true;  // trajectory rows (optional pointers) written by both kernels: free in the single-step one
#ifdef PP3_PHASE_PROF
  const uint32_t t_start_ = shader_cycles();
  const uint32_t rt_start_ = (uint32_t)__builtin_amdgcn_s_memrealtime();  // 100 MHz, chip-wide
  Prof pf_local{t_start_, 0u, t_start_, 0u, 0u, 0u, 0u, 0u, 0u, 0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu};
  Prof* pf = &pf_local;
#endif
  // FUSED (pp3_rollout): the wave runs its two envs' nsteps steps back to back, each step reading
  // back the previous one's global stores (state record, lag rows, obs history; the fence at the
  // bottom).  The arguments are re-read every step through an opaque kernarg pointer and the lane
  // id is opaque too: otherwise the argument / model loads and the lane masks are hoisted out of
  // the loop and kept live across it (SGPR and VGPR spills).  With FUSED false the loop runs once
  // and the kernel compiles to the single-step code it always was.
  int heavy_prev = 0;  // fused: the load flag carries over into the next step's first substep
  // obstacle models (CULL): per env, collision's cached near-box mask and body 1's origin when it
  // was tested (its own array: the env blocks' layout stays the flat model's); invalid at launch start
  __shared__ float cull_cache[CULL ? 2 * NWV : 1][4];
  if constexpr (CULL) {
    const int t = (int)threadIdx.x;
    if ((t & (HW - 1)) == 0) cull_cache[t >> 5][0] = 1.0e30f;
  }
  for (int it = 0;;) {
#ifdef PP3_PHASE_PROF
  if (it == 1) pf->n = 0;  // fused launch: the stamp trace holds the second step (a warm one)
#endif
  const GArgs* ap = (const GArgs*)__builtin_amdgcn_kernarg_segment_ptr();
  if (FUSED) asm volatile("" : "+s"(ap));
  const StepArgs* ap_step;
  if constexpr (NWV > 1) ap_step = (const StepArgs*)ap;
  else ap_step = FUSED ? (const StepArgs*)ap : &a_arg;
  const StepArgs& a = *ap_step;
  if constexpr (NWV > 1) {
    // policy-in-the-loop: the workgroup's MLP on its 16 envs' current observations (the previous
    // step's, or the reset's), into this step's action row; its LDS scratch is the envs' blocks
    // (nothing in them lives across steps).  The barrier makes every wave's previous-step stores
    // (obs rows) visible; mlp_tile ends with one, after which the actions are visible.
    typedef __attribute__((address_space(4))) const PolicyStepArgs GPArgs;
    const GPArgs& pa = *(const GPArgs*)ap;
    const int Hm = ((const DevModel*)(const GModel*)a.m)->H;
    const bool tile_in = PP3_OBS_DIM * Hm + 4 <= OBS_TILE_W;
    if (tile_in && it == 0) {  // first step of the launch: the observations come from global memory
      for (int i = threadIdx.x; i < pp3pol::TILE * PP3_OBS_DIM * Hm; i += WAVE * NWV) {
        const int r = i / (PP3_OBS_DIM * Hm), k = i - r * (PP3_OBS_DIM * Hm);
        const int row = blockIdx.x * pp3pol::TILE + r;
        obs_tile[r][k] = row < a.N ? a.obs_out[(size_t)row * (PP3_OBS_DIM * Hm) + k] : 0.0f;
      }
    }
    __syncthreads();
    PP3_STEP_ACQUIRE();
    {
      if (tile_in)
        policy_mlp_tile(&pa.net, pa.act + (size_t)it * a.act_stride, a.N, blockIdx.x * pp3pol::TILE,
                        (pp3pol::LdsTileBuf*)(reinterpret_cast<pp3pol::TileBuf*>(sh)), (LdsObsTile*)obs_tile);
      else
        policy_mlp(&pa.net, a.obs_out, PP3_OBS_DIM * Hm, pa.act + (size_t)it * a.act_stride, a.N,
                   blockIdx.x * pp3pol::TILE, (pp3pol::LdsTileBuf*)(reinterpret_cast<pp3pol::TileBuf*>(sh)));
      PP3_STEP_ACQUIRE();
    }
  }
  int lane = NWV > 1 ? (int)(threadIdx.x & (WAVE - 1)) : (int)threadIdx.x;  // (opaque too: lane masks and LDS addresses are rebuilt where used)
  if (FUSED) asm volatile("" : "+v"(lane));
  const int wv = NWV > 1 ? __builtin_amdgcn_readfirstlane(threadIdx.x >> 6) : 0;  // this wave in the workgroup
  const int h = lane >> 5, l = lane & (HW - 1);
  Shared<NC>& s = sh[alias ? 0 : 2 * wv + h];
  const int env_raw = 2 * (blockIdx.x * NWV + wv) + h;
  const bool own = env_raw < a.N;
  const int env = own ? env_raw : a.N - 1;
  // constant AS: uniform reads -> s_load.  Through a fresh opaque pointer, as in the epilogue: in
  // the fused loop the kernel-level reference's reads were vector loads, five of them each waited
  // for on its own (H, n_frames, La / Li, stride, imu_off: ~5 k cycles per step)
  const GModel* mp_pro = (const GModel*)(a.m);
  if (FUSED) asm volatile("" : "+s"(mp_pro));
  const DevModel& m = *(const DevModel*)mp_pro;
  const int stride = m.stride;
  const int part = m.partitionable;
  float* gst = a.state + (size_t)env * stride;
  // fused rollout: this step's observation row of the trajectory (optional)
  float* const to = TG && a.traj_obs ? a.traj_obs + ((size_t)it * a.N + env) * (PP3_OBS_DIM * m.H) : nullptr;
  // ---- every global load of this env step issued together (one memory round trip): state
  // record head, this lane's action-latency row and IMU row, the action, the obs history, the
  // lane's env constants and body parameters; the global stores only after all of them ----
  int n_frames = __builtin_amdgcn_readfirstlane(m.n_frames);
  const float* act_env = a.actions + (size_t)it * a.act_stride + (size_t)env * NU;
  const size_t obs_base = (size_t)env * (PP3_OBS_DIM * m.H);
  const float* oi = a.obs_in + obs_base;
  float* oo = a.obs_out + obs_base;
  // fused steps after the first: the env's LDS block still holds what this wave left in it
  const bool carry = FUSED && NWV == 1 && it > 0;
  float arow[PP3_MAX_LAG], irow[PP3_MAX_LAG], act_in = 0.0f;
  {
    const float* ar = gst + PP3_S_ACT_BUF + (l < NU ? l : 0) * m.La;
    const float* ir = gst + m.imu_off + (l < 6 ? l : 0) * m.Li;
#pragma unroll
    for (int q = 0; q < PP3_MAX_LAG; q++) {
      arow[q] = (l < NU && q < m.La) ? ar[q] : 0.0f;
      irow[q] = (l < 6 && q < m.Li) ? ir[q] : 0.0f;
    }
    if (l < NU) act_in = act_env[l];
  }
  LaneRec<2> re;  // plain loads (no pin): retired with the batch's first wait
  for (int k = 0; k < 2; k++)
    for (int c = 0; c < 4; c++) re.f[4 * k + c] = m.lane_env.g[k][l][c];
  const KinConst kc = kin_const(m, l);  // (kept in registers for all substeps)
  // observation history: obs_out[36:] = obs_in[:36(H-1)] (environment.py:540-543)
  const int nmove = PP3_OBS_DIM * (m.H - 1);
  // carry with H = 2: the history frame is the previous step's newest observation, still in LDS
  const bool hist_lds = carry && nmove == PP3_OBS_DIM;
  float tmp[OBS_MOVE];
#pragma unroll
  for (int t = 0; t < OBS_MOVE; t++) {
    const int k = l + HW * t;
    if (hist_lds) tmp[t] = (k < PP3_OBS_DIM) ? s.x.e.o[k < PP3_OBS_DIM ? k : 0] : 0.0f;
    else tmp[t] = (k < nmove) ? oi[k] : 0.0f;
  }
  float v[(PP3_S_ACT_BUF + HW - 1) / HW];  // state record head
  if (!carry)
#pragma unroll
    for (int t = 0; t < (PP3_S_ACT_BUF + HW - 1) / HW; t++) v[t] = l + HW * t < PP3_S_ACT_BUF ? gst[l + HW * t] : 0.0f;
  // auto-reset mode: the previous step's done and this env's episode record (kept in LDS)
  if (a.episode) {
    if (l == 0) {
      s.ep_prev_done = a.done[env];  // the previous wrapper step's (earlier repeats leave it alone)
      s.ep_racc = a.phase > 0 ? a.reward[env] : 0.0f;
    }
    if (l < PP3_EP_STRIDE) s.ep[l] = a.episode[(size_t)env * PP3_EP_STRIDE + l];
  }
  if (!carry) load_params(s, m, a.dr ? a.dr + (size_t)env * PP3_NDR : nullptr, l);
  // obs is updated in place (obs_in == obs_out): every history load of this half has returned
  // before the first history store (for H >= 3 the shifted window overlaps the one it is read from)
  if (!hist_lds) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (own)
#pragma unroll
    for (int t = 0; t < OBS_MOVE; t++)
      if (l + HW * t < nmove) {
        oo[PP3_OBS_DIM + l + HW * t] = tmp[t];
        if constexpr (NWV > 1)
          if (PP3_OBS_DIM * m.H + 4 <= OBS_TILE_W) obs_tile[2 * wv + h][PP3_OBS_DIM + l + HW * t] = tmp[t];
        if (TG && to) to[PP3_OBS_DIM + l + HW * t] = tmp[t];
      }
  if (!carry)
#pragma unroll
    for (int t = 0; t < (PP3_S_ACT_BUF + HW - 1) / HW; t++)
      if (l + HW * t < PP3_S_ACT_BUF) s.st[l + HW * t] = v[t];
  SYNC();
  if (l < NQ) s.qpos[l] = s.st[PP3_S_QPOS + l];
  if (l < NV) { s.qvel[l] = s.st[PP3_S_QVEL + l]; s.qws[l] = s.st[PP3_S_QACC_WS + l]; }
  // ---- prologue: rng split (environment.py:349), kick (:352-356), action latency (:359-365) ----
  const Key rng{__float_as_uint(s.st[PP3_S_RNG]), __float_as_uint(s.st[PP3_S_RNG + 1])};
  const Key kl = split_i(rng, 5, l < 5 ? l : 0, part);  // lane i holds split(rng, 5)[i]
  const Key k_new = hkey(kl, 0, h), cmd_key = hkey(kl, 1, h);
  const Key kkick = hkey(kl, 2, h), kbern = hkey(kl, 3, h), klat = hkey(kl, 4, h);
  float u = 0;
  if (l < 4) {
    const Key kk = l < 2 ? kkick : (l == 2 ? kbern : klat);
    u = uniform_i(kk, l < 2 ? 2 : 1, l < 2 ? l : 0, l < 2 ? -1.0f : 0.0f, 1.0f, part);
  }
  const float bern = hb(u, 2, h) < m.kick_p ? 1.0f : 0.0f;
  const float kick0 = hb(u, 0, h) * m.kick_vel * bern, kick1 = hb(u, 1, h) * m.kick_vel * bern;
  const int li = choice_from_uniform((const GFloat*)m.lat_dist, m.La, hb(u, 3, h));
  if (l == 0) {
    s.qvel[0] += kick0;
    s.qvel[1] += kick1;
    s.st[PP3_S_KICK] = kick0;
    s.st[PP3_S_KICK + 1] = kick1;
    s.st[PP3_S_RNG] = __uint_as_float(k_new.a);
    s.st[PP3_S_RNG + 1] = __uint_as_float(k_new.b);
  }
  if (l < NU) {
    const float lagged = push_lagged_pre(gst + PP3_S_ACT_BUF + l * m.La, m.La, act_in, li, own, arow);
    const float t = re.f[LE_POSE] + lagged * m.action_scale;
    s.ctrl[l] = fminf(fmaxf(t, re.f[LE_JLO]), re.f[LE_JHI]);
  }
  SYNC();
  // the state head's qpos|qvel|qacc_ws words are copied out (above) and only rewritten after the
  // observation, so they hold the IMU rows' old values meanwhile (6 x MAX_LAG <= 55 floats)
  float* imu_stash = s.st + PP3_S_QPOS;
  if (l < 6)
#pragma unroll
    for (int q = 0; q < PP3_MAX_LAG; q++) imu_stash[PP3_MAX_LAG * l + q] = irow[q];
  SYNC();
  PHASE(10);
  // ---- physics: n_frames x mj_step (environment.py:366) ----
  asm volatile("" : "+s"(n_frames));  // one scalar load (an invariant load is otherwise re-issued per substep)
  // VALU issue between the two waves of a SIMD goes by priority, then age: at equal priority the
  // younger wave (wave slot 1 in 97 % of pairs) only gets the older one's leftover issue cycles
  // and finished ~19 % later (per-wave lifetimes, diag_phases.py), and the launch ends with the
  // slowest wave.  The two slots take turns at the higher priority, one substep each.
  uint32_t hwid;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hwid));
  const int wslot = (int)(hwid & 1u);
  int heavy = heavy_prev;  // the previous substep's load was high: this wave sets the launch's tail
  for (int f = 0; f < n_frames; f++) {
    // the heavy waves (many contacts, leg-leg Newton path) ahead of their partners, which have
    // slack; between equals the two slots alternate
    const int prio = 2 * heavy + ((f + wslot) & 1);
    if (prio == 3) __builtin_amdgcn_s_setprio(3);
    else if (prio == 2) __builtin_amdgcn_s_setprio(2);
    else if (prio == 1) __builtin_amdgcn_s_setprio(1);
    else __builtin_amdgcn_s_setprio(0);
    // opaque per iteration: keep model loads inside the substep (hoisting them costs more
    // registers than reloading them); the constant address space is restated after the asm so
    // uniform loads become s_load and the rest global_load (a generic pointer would turn them into flat loads)
    const GModel* mp = (const GModel*)(a.m);
    asm volatile("" : "+s"(mp));
    // (the single-step kernel takes sincos_f32, the fused one the library's sincosf: same values)
    const int wgt = substep<NC, NWV, FUSED, CULL>(s, *(const DevModel*)mp, l, h, f > 0, kc PROF_ARG,
                                                  CULL ? cull_cache[alias ? 0 : 2 * wv + h] : nullptr);
    heavy = wgt >= HEAVY_WEIGHT ? 1 : 0;
  }
  if (n_frames > 0) {  // the last substep's Euler step (the others ran inside the next kinematics)
    const GModel* mp = (const GModel*)(a.m);
    asm volatile("" : "+s"(mp));
    euler_step<NC, FUSED>(s, *(const DevModel*)mp, l);
    PHASE(9);
  }
  if (heavy) __builtin_amdgcn_s_setprio(3);  // the epilogue: heavy waves, then the younger slot, ahead
  else if (wslot) __builtin_amdgcn_s_setprio(1);
  else __builtin_amdgcn_s_setprio(0);
  SYNC();
  // The epilogue reads the model through a fresh opaque constant-AS pointer: after the loop's
  // asm'd pointer, reads through the kernel-level reference are no longer proven uniform and
  // turn into per-use vector loads (one vmcnt round trip each) instead of s_load.
  const GModel* mq = (const GModel*)(a.m);
  asm volatile("" : "+s"(mq));
  {
  const DevModel& m = *(const DevModel*)mq;
  const LaneRec<2> re = fetch_rec(m.lane_env, l);  // this lane's env constants (one round trip)
  // ---- observation (history already shifted in the prologue) ----
  get_obs(s, m, gst + m.imu_off, l, h, re.f[LE_POSE16], own, imu_stash PROF_ARG);
  {
    if (own)
      for (int k = l; k < PP3_OBS_DIM; k += HW) {
        oo[k] = s.x.e.o[k];
        if constexpr (NWV > 1)
          if (PP3_OBS_DIM * m.H + 4 <= OBS_TILE_W) obs_tile[2 * wv + h][k] = s.x.e.o[k];
        if (TG && to) to[k] = s.x.e.o[k];
      }
  }
  SYNC();
  if (l < NQ) s.st[PP3_S_QPOS + l] = s.qpos[l];
  if (l < NV) { s.st[PP3_S_QVEL + l] = s.qvel[l]; s.st[PP3_S_QACC_WS + l] = s.qws[l]; }
  SYNC();
  PHASE(11);
  // ---- brax x/xd (lanes 1..13), feet (16..19) ----
  // every LDS operand of x/xd, the feet, done and the command in one pinned round (indices
  // clamped on the lanes that do not use them; none of them is written before its use below)
  const int tb = m.torso_body;
  const int bx = (l >= 1 && l < NB) ? l : 1, fx = (l >= 16 && l < 20) ? l - 16 : 0;
  float xbb[3], cm[3], cv[6], qt[4];
#pragma unroll
  for (int k = 0; k < 3; k++) { xbb[k] = s.xpos[bx][k]; cm[k] = s.com[k]; }
#pragma unroll
  for (int k = 0; k < 6; k++) cv[k] = s.cvel[bx][k];
#pragma unroll
  for (int k = 0; k < 4; k++) qt[k] = s.xquat[tb][k];
  float fz = s.foot_xpos[fx][2], lcst = s.st[PP3_S_LAST_CONTACT + fx], airt0 = s.st[PP3_S_AIR_TIME + fx];
  float xtz = s.xpos[tb][2], qpl = s.qpos[7 + (l < 12 ? l : 0)];
  float cmd0 = s.st[PP3_S_COMMAND], cmd1 = s.st[PP3_S_COMMAND + 1], cmd2 = s.st[PP3_S_COMMAND + 2];
  PIN("+v"(xbb[0]), "+v"(xbb[1]), "+v"(xbb[2]), "+v"(cm[0]), "+v"(cm[1]), "+v"(cm[2]), "+v"(cv[0]), "+v"(cv[1]),
      "+v"(cv[2]), "+v"(cv[3]), "+v"(cv[4]), "+v"(cv[5]), "+v"(qt[0]), "+v"(qt[1]), "+v"(qt[2]), "+v"(qt[3]));
  PIN("+v"(fz), "+v"(lcst), "+v"(airt0), "+v"(xtz), "+v"(qpl), "+v"(cmd0), "+v"(cmd1), "+v"(cmd2));
  if (l >= 1 && l < NB) {
    const int b = l;
    const float off[3] = {xbb[0] - cm[0], xbb[1] - cm[1], xbb[2] - cm[2]};
    float cr[3];
    cross3(cr, cv, off);
    for (int k = 0; k < 3; k++) { s.x.e.xdv[b][k] = cv[3 + k] + cr[k]; s.x.e.xda[b][k] = cv[k]; }
  }
  if (l >= 16 && l < 20) {
    const int f = l - 16;
    const float cz = fz - m.foot_radius;
    const int last = lcst != 0.0f;
    const int c = cz < 1e-3f;
    s.x.e.contact[f] = c;
    s.x.e.filt_mm[f] = c | last;
    s.x.e.filt_cm[f] = (cz < 3e-2f) | last;
    s.x.e.first[f] = (airt0 > 0.0f && (c | last)) ? 1.0f : 0.0f;
    s.st[PP3_S_AIR_TIME + f] = airt0 + m.dt;
  }
  SYNC();
  // ---- done (environment.py:383-388): tilt and height on every lane, joint limits on 0..11 ----
  const float z0[3] = {0, 0, 1};
  float ru_t[3];
  b_rotate(ru_t, z0, qt);
  const bool jviol = l < 12 && (qpl < re.f[LE_JLO] || qpl > re.f[LE_JHI]);
  const bool isdone = hballot(jviol, h) != 0 || ru_t[2] < m.cos_term_angle || xtz < m.term_z;
  // ---- rewards (rewards.py) ----
  // sums over joints / dofs / feet / contacts: one element per lane, then a half-wave sum
  const float cn = sqrtf(cmd0 * cmd0 + cmd1 * cmd1 + cmd2 * cmd2);
  float r_torq = 0, r_jacc = 0, r_mech = 0, r_arate = 0, r_stand = 0, r_standv = 0, r_abd = 0;
  float r_air = 0, r_slip = 0, r_knee = 0, r_body = 0;
  // every per-lane LDS operand of the terms below in one pinned round (indices clamped on the
  // lanes that do not use them); read inside the lane branches they were round trips of their own
  const int l18 = l < NV ? l : 0, l12 = l < 12 ? l : 0, l4 = l < 4 ? l : 0, lc = l < NC ? l : 0;
  const int bleg = l < 4 ? as_i(re.f[LE_LEG]) : 1;
  float fa = s.qfrc_act[l18], fa6 = s.qfrc_act[6 + l12], qv = s.qvel[6 + l12], qp = s.qpos[7 + l12];
  float lvel = s.st[PP3_S_LAST_VEL + l12], lact = s.st[PP3_S_LAST_ACT + l12];
  float airt = s.st[PP3_S_AIR_TIME + l4], fst = s.x.e.first[l4];
  float sp[3], xb[3], xdab[3], xdvb[2];
#pragma unroll
  for (int k = 0; k < 3; k++) { sp[k] = s.foot_xpos[l4][k]; xb[k] = s.xpos[bleg][k]; xdab[k] = s.x.e.xda[bleg][k]; }
  xdvb[0] = s.x.e.xdv[bleg][0];
  xdvb[1] = s.x.e.xdv[bleg][1];
  int fcm = s.x.e.filt_cm[l4], ncon_r = s.ncon, cpair = s.con_pair[lc];
  float cdist = s.con_dist[lc];
  PIN("+v"(fa), "+v"(fa6), "+v"(qv), "+v"(qp), "+v"(lvel), "+v"(lact), "+v"(airt), "+v"(fst), "+v"(sp[0]), "+v"(sp[1]),
      "+v"(sp[2]), "+v"(xb[0]), "+v"(xb[1]), "+v"(xb[2]), "+v"(xdab[0]), "+v"(xdab[1]), "+v"(xdab[2]), "+v"(xdvb[0]),
      "+v"(xdvb[1]), "+v"(fcm), "+v"(ncon_r), "+v"(cpair), "+v"(cdist));
  if (l < NV) r_torq = fa * fa;
  if (l < 12) {
    const float acc = (qv - lvel) / m.env_dt;
    r_jacc = acc * acc;
    r_mech = fabsf(fa6 * qv);
    const float da = act_in - lact;  // act_in = action[l] (prologue load)
    r_arate = da * da;
    r_stand = fabsf(qp - re.f[LE_POSE]);
    r_standv = fabsf(qv);
    if (l % 3 == 1) { const float t = qp - re.f[LE_ABD]; r_abd = t * t; }
  }
  if (l < 4) {
    r_air = (airt - 0.1f) * fst;
    const float off[3] = {sp[0] - xb[0], sp[1] - xb[1], sp[2] - xb[2]};
    float cr[3];
    cross3(cr, xdab, off);
    const float vx = xdvb[0] + cr[0], vy = xdvb[1] + cr[1];
    r_slip = (vx * vx + vy * vy) * (fcm ? 1.0f : 0.0f);
  }
  if (l < ncon_r && cdist < 0.0f) {  // geom_collision: (contact, id) matches with dist < 0
    const v4f kb = reinterpret_cast<const v4f*>(&m.pair_con[cpair])[3];  // knee, body counts (host)
    r_knee = kb[1];
    r_body = kb[2];
  }
  r_torq = hsum(r_torq, h);
  r_jacc = hsum(r_jacc, h);
  r_mech = hsum(r_mech, h);
  r_arate = hsum(r_arate, h);
  r_stand = hsum(r_stand, h) * ((cn < 0.1f) ? 1.0f : 0.0f);
  r_standv = hsum(r_standv, h) * ((cn < m.stand_thr) ? 1.0f : 0.0f);
  r_abd = hsum(r_abd, h);
  r_air = hsum(r_air, h) * ((cn > 0.05f) ? 1.0f : 0.0f);
  r_slip = hsum(r_slip, h);
  r_knee = hsum(r_knee, h);
  r_body = hsum(r_body, h);
  // single-valued terms: straight-line code on every lane (no divergent switch)
  float rw[PP3_NREWARD];
  {
    const float inv[4] = {s.xquat[1][0], -s.xquat[1][1], -s.xquat[1][2], -s.xquat[1][3]};
    const float sig = m.sigma;
    const float* xdv1 = s.x.e.xdv[1];
    const float* xda1 = s.x.e.xda[1];
    float lv[3], av[3], wz[3], ru[3];
    b_rotate(lv, xdv1, inv);
    b_rotate(av, xda1, inv);
    b_rotate(wz, z0, inv);
    b_rotate(ru, z0, s.xquat[1]);
    const float e_lin = (cmd0 - lv[0]) * (cmd0 - lv[0]) + (cmd1 - lv[1]) * (cmd1 - lv[1]);
    float e_ori = 0;
    for (int k = 0; k < 3; k++) e_ori += (wz[k] - s.st[PP3_S_DESIRED_Z + k]) * (wz[k] - s.st[PP3_S_DESIRED_Z + k]);
    rw[PP3_REWARD_TRACKING_LIN_VEL] = expf(-e_lin / sig);
    rw[PP3_REWARD_TRACKING_ANG_VEL] = expf(-(cmd2 - av[2]) * (cmd2 - av[2]) / sig);
    rw[PP3_REWARD_TRACKING_ORIENTATION] = expf(-e_ori / sig);
    rw[PP3_REWARD_LIN_VEL_Z] = xdv1[2] * xdv1[2];
    rw[PP3_REWARD_ANG_VEL_XY] = xda1[0] * xda1[0] + xda1[1] * xda1[1];
    rw[PP3_REWARD_ORIENTATION] = ru[0] * ru[0] + ru[1] * ru[1];
  }
  rw[PP3_REWARD_TORQUES] = r_torq;
  rw[PP3_REWARD_JOINT_ACCELERATION] = r_jacc;
  rw[PP3_REWARD_MECHANICAL_WORK] = r_mech;
  rw[PP3_REWARD_ACTION_RATE] = r_arate;
  rw[PP3_REWARD_STAND_STILL] = r_stand;
  rw[PP3_REWARD_STAND_STILL_JOINT_VELOCITY] = r_standv;
  rw[PP3_REWARD_ABDUCTION_ANGLE] = r_abd;
  rw[PP3_REWARD_FEET_AIR_TIME] = r_air;
  rw[PP3_REWARD_FOOT_SLIP] = r_slip;
  rw[PP3_REWARD_TERMINATION] = (isdone && (int)s.st[PP3_S_STEP] < m.term_step) ? 1.0f : 0.0f;
  rw[PP3_REWARD_KNEE_COLLISION] = r_knee;
  rw[PP3_REWARD_BODY_COLLISION] = r_body;
  float rsum = 0.0f, rmine = 0.0f;  // reward = clip(sum_k scale_k * term_k * dt) in dict order (:446)
#pragma unroll
  for (int k = 0; k < PP3_NREWARD; k++) {
    const float v = rw[k] * m.scales[k];
    rsum += v;
    rmine = (l == k) ? v : rmine;
  }
  // ---- state management (environment.py:448-482) ----
  int stepc = (int)s.st[PP3_S_STEP] + 1;
  const bool resample = stepc > m.resample_step;
  const float reward = fminf(fmaxf(rsum * m.dt, 0.0f), 10000.0f);
  bool done_out = isdone;
  // brax EpisodeWrapper.step / AutoResetWrapper.step ([ext] brax 0.12.1): with action_repeat k a
  // wrapper step is k launches with the same action; the reward is summed over them, and the
  // episode bookkeeping, done and the auto-reset happen at the last one
  const bool last = a.phase == a.repeat - 1;
  // the output pointers read here, above the one-lane branches: read inside them, each is a
  // scalar load and a wait of its own, one after the other
  float* const o_reward = a.reward;
  float* const o_done = a.done;
  float* const o_metrics = a.metrics;
  float* const o_treward = a.traj_reward;
  float* const o_tdone = a.traj_done;
  float rout = reward;
  if (a.episode) {
    rout = reward + s.ep_racc;
    if (last) {
      const float keep = 1.0f - s.ep_prev_done;  // previous step done -> counters restart
      const float ep_rec = l < PP3_EP_STRIDE ? s.ep[l] : 0.0f;
      const float steps = s.ep[PP3_EP_STEPS] * keep + (float)a.repeat;
      const bool trunc_hit = steps >= (float)a.episode_length;
      done_out = isdone || trunc_hit;
      float v = steps;
      if (l == PP3_EP_TRUNCATION) v = (trunc_hit && !isdone) ? 1.0f : 0.0f;
      if (l == PP3_EP_SUM_REWARD) v = (ep_rec + rout) * keep;
      if (l == PP3_EP_LENGTH) v = (ep_rec + (float)a.repeat) * keep;
      if (own && l < PP3_EP_STRIDE) a.episode[(size_t)env * PP3_EP_STRIDE + l] = v;
    }
  }
  if (own && l == 0) {
    o_reward[env] = rout;
    if (!a.episode || last) o_done[env] = done_out ? 1.0f : 0.0f;
    if (TG && (!a.episode || last)) {
      if (o_treward) o_treward[(size_t)it * a.N + env] = rout;
      if (o_tdone) o_tdone[(size_t)it * a.N + env] = done_out ? 1.0f : 0.0f;
    }
    o_metrics[(size_t)env * PP3_NMETRIC] =
        sqrtf(s.xpos[tb][0] * s.xpos[tb][0] + s.xpos[tb][1] * s.xpos[tb][1] + s.xpos[tb][2] * s.xpos[tb][2]);
  }
  if (own && l < PP3_NREWARD) o_metrics[(size_t)env * PP3_NMETRIC + 1 + l] = rmine;
  if (l < NU) {
    s.st[PP3_S_LAST_ACT + l] = act_in;
    s.st[PP3_S_LAST_VEL + l] = s.qvel[6 + l];
  }
  if (l < 4) {
    if (s.x.e.filt_mm[l]) s.st[PP3_S_AIR_TIME + l] = 0.0f;
    s.st[PP3_S_LAST_CONTACT + l] = s.x.e.contact[l] ? 1.0f : 0.0f;
  }
  if (resample) {
    sample_command(m, cmd_key, s.st + PP3_S_COMMAND, l, h);
    sample_orientation(m, cmd_key, s.st + PP3_S_DESIRED_Z, l, h);
  }
  if (isdone || resample) stepc = 0;
  if (l == 0) s.st[PP3_S_STEP] = (float)stepc;
  // the Brax pipeline record is the returned state's: a fused rollout writes it at its last step only
  if (own && a.pipe && (!FUSED || it == nsteps - 1)) write_pipeline(s, m, a.pipe + (size_t)env * PP3_PIPE_STRIDE, l);
  if (a.episode && last && done_out) {  // AutoResetWrapper: pipeline state and obs <- the reset's
    const float* fs = a.first_state + (size_t)env * PP3_FIRST_STRIDE;
    for (int i = l; i < PP3_FIRST_STRIDE; i += HW) s.st[PP3_S_QPOS + i] = fs[i];
    const float* fo = a.first_obs + (size_t)env * PP3_OBS_DIM * m.H;
    __threadfence_block();  // the prologue's history stores (other lanes, same addresses) land first
    if (FUSED && NWV == 1)  // the next step's carried history frame (H = 2)
      for (int i = l; i < PP3_OBS_DIM; i += HW) s.x.e.o[i] = fo[i];
    if (own)
      for (int i = l; i < PP3_OBS_DIM * m.H; i += HW) {
        oo[i] = fo[i];
        if constexpr (NWV > 1)
          if (PP3_OBS_DIM * m.H + 4 <= OBS_TILE_W) obs_tile[2 * wv + h][i] = fo[i];
        if (TG && to) to[i] = fo[i];
      }
  }
  SYNC();
  if (own)
#pragma unroll
    for (int t = 0; t < (PP3_S_ACT_BUF + HW - 1) / HW; t++)
      if (l + HW * t < PP3_S_ACT_BUF) gst[l + HW * t] = s.st[l + HW * t];
  PHASE(12);
  }
  heavy_prev = heavy;
  if (!FUSED || ++it >= nsteps) break;
  // the next step reads back this step's global stores (state record, lag rows, obs history)
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  PP3_STEP_ACQUIRE();
  }
#ifdef PP3_PHASE_PROF
  static_assert(NWV == 1, "the per-wave profile records index waves by workgroup");
  const int lane = threadIdx.x;
  if (lane < NPROF - 1 && blockIdx.x < MAXWAVE) g_prof[blockIdx.x][lane] += pf->acc;
  if (lane == 0 && blockIdx.x < MAXWAVE) {
    uint32_t hwid, xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hwid));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    const uint32_t t_end = shader_cycles();
    const uint32_t rec[8] = {t_end - pf->t0, pf->dense, pf->ncmax, pf->evals, pf->t0, t_end, hwid, xcc};
    for (int k = 0; k < 8; k++) g_wave[blockIdx.x][k] = rec[k];
    g_wave[blockIdx.x][27] = pf->csum;
    g_wave[blockIdx.x][28] = pf->slot2;
    g_wave[blockIdx.x][29] = rt_start_;
    g_wave[blockIdx.x][30] = (uint32_t)__builtin_amdgcn_s_memrealtime();
  }
  if (lane < 19 && blockIdx.x < MAXWAVE) g_wave[blockIdx.x][8 + lane] = pf->acc;
  if (blockIdx.x < MAXWAVE) {
    g_wave[blockIdx.x][32 + lane] = pf->tr0;
    g_wave[blockIdx.x][32 + 64 + lane] = pf->tr1;
    g_wave[blockIdx.x][32 + NTRACE + lane] = pf->k0;
    g_wave[blockIdx.x][32 + NTRACE + 64 + lane] = pf->k1;
  }
  if (lane == HW + 20 && blockIdx.x < MAXWAVE) g_prof[blockIdx.x][NPROF - 1] += pf->acc;
#endif
}


struct ResetArgs {
  const DevModel* m;
  float* state;
  float* obs;
  float* reward;
  float* done;
  float* metrics;
  const uint32_t* keys;  // [N][2]
  const uint8_t* mask;   // [N] or null
  const float* dr;
  float* pipe;
  float* episode;      // auto-reset mode: zeroed
  float* first_state;  // auto-reset mode: [N][PP3_FIRST_STRIDE] <- this reset
  float* first_obs;    // auto-reset mode: [N][36H] <- this reset's obs
  int N;
};

template <int NC>
__global__ __launch_bounds__(WAVE, 2) void env_reset_kernel(ResetArgs a) {
  __shared__ Shared<NC> sh[2];
  const int lane = threadIdx.x;
  const int h = lane >> 5, l = lane & (HW - 1);
  const int env_raw = 2 * blockIdx.x + h;
  const int env = env_raw < a.N ? env_raw : a.N - 1;
  // envs outside N or masked out compute alongside their wave partner but store nothing
  const bool own = env_raw < a.N && (!a.mask || a.mask[env]);
  Shared<NC>& s = sh[h];
  const DevModel& m = *(const DevModel*)(const GModel*)a.m;  // constant AS: uniform reads -> s_load
  const int part = m.partitionable;
  float* gst = a.state + (size_t)env * m.stride;
  load_params(s, m, a.dr ? a.dr + (size_t)env * PP3_NDR : nullptr, l);
  for (int i = l; i < PP3_S_ACT_BUF; i += HW) s.st[i] = 0.0f;
  if (own)
    for (int i = PP3_S_ACT_BUF + l; i < m.stride; i += HW) gst[i] = 0.0f;  // latency buffers
  SYNC();
  const Key rng{a.keys[2 * env], a.keys[2 * env + 1]};
  const Key kl = split_i(rng, 4, l < 4 ? l : 0, part);
  const Key k0 = hkey(kl, 0, h), kcmd = hkey(kl, 1, h), kori = hkey(kl, 2, h), kpos = hkey(kl, 3, h);
  // randomize_qpos (domain_randomization.py:188-210) on the home keyframe with default_pose
  float u = 0;
  if (l < 4) {
    const Key kk = split_i(kpos, 3, l < 3 ? 1 : 2, part);
    u = l < 3 ? uniform_i(kk, 3, l, m.start_lo[l], m.start_hi[l], part)
              : uniform_i(kk, 1, 0, -m.pi_f, m.pi_f, part);
  }
  const float yaw = hb(u, 3, h);
  if (l < NQ) {
    float q = l >= 7 ? m.default_pose[l - 7] : m.key_qpos[l];
    if (l < 3) q = u;
    if (l == 3) q = cosf(yaw / 2.0f);
    if (l == 4 || l == 5) q = 0.0f;
    if (l == 6) q = sinf(yaw / 2.0f);
    s.qpos[l] = q;
  }
  if (l < NV) { s.qvel[l] = 0.0f; s.qws[l] = 0.0f; }
  if (l < NU) s.ctrl[l] = 0.0f;
  SYNC();
  substep(s, m, l, h, false, kin_const(m, l) PROF_NULL);  // pipeline_init: mjx.forward at (q, qd=0, ctrl=0)
  if (l < NQ) s.st[PP3_S_QPOS + l] = s.qpos[l];
  if (l < NV) { s.st[PP3_S_QVEL + l] = 0.0f; s.st[PP3_S_QACC_WS + l] = s.qws[l]; }
  if (l == 0) {
    s.st[PP3_S_RNG] = __uint_as_float(k0.a);
    s.st[PP3_S_RNG + 1] = __uint_as_float(k0.b);
  }
  sample_command(m, kcmd, s.st + PP3_S_COMMAND, l, h);
  sample_orientation(m, kori, s.st + PP3_S_DESIRED_Z, l, h);
  if (own && l < m.Li) gst[m.imu_off + 5 * m.Li + l] = -1.0f;  // initial_imu_buffer gravity row
  __threadfence_block();
  __syncthreads();  // the gravity row above is global memory written by other lanes
  get_obs(s, m, gst + m.imu_off, l, h, m.lane_env.g[LE_POSE16 / 4][l][LE_POSE16 % 4], own, nullptr PROF_NULL);
  write_obs(s, m, nullptr, a.obs + (size_t)env * PP3_OBS_DIM * m.H, l, own);
  if (own && a.episode) {
    if (l < PP3_EP_STRIDE) a.episode[(size_t)env * PP3_EP_STRIDE + l] = 0.0f;
    float* fs = a.first_state + (size_t)env * PP3_FIRST_STRIDE;
    for (int i = l; i < PP3_FIRST_STRIDE; i += HW) fs[i] = s.st[PP3_S_QPOS + i];
    write_obs(s, m, nullptr, a.first_obs + (size_t)env * PP3_OBS_DIM * m.H, l, true);
  }
  if (own && l == 0) { a.reward[env] = 0.0f; a.done[env] = 0.0f; }
  if (own && l < PP3_NMETRIC) a.metrics[(size_t)env * PP3_NMETRIC + l] = 0.0f;
  if (own && a.pipe) write_pipeline(s, m, a.pipe + (size_t)env * PP3_PIPE_STRIDE, l, false);
  SYNC();
  if (own)
#pragma unroll
    for (int t = 0; t < (PP3_S_ACT_BUF + HW - 1) / HW; t++)
      if (l + HW * t < PP3_S_ACT_BUF) gst[l + HW * t] = s.st[l + HW * t];
}

struct PhysArgs {
  const DevModel* m;
  float* state;
  const float* ctrl;  // [N][12]
  const float* dr;
  float* pipe;
  int nsteps;
  int N;
};

template <int NC>
__global__ __launch_bounds__(WAVE, 2) void physics_kernel(PhysArgs a) {
  __shared__ Shared<NC> sh[2];
  const int lane = threadIdx.x;
  const int h = lane >> 5, l = lane & (HW - 1);
  const int env_raw = 2 * blockIdx.x + h;
  const bool own = env_raw < a.N;
  const int env = own ? env_raw : a.N - 1;
  Shared<NC>& s = sh[h];
  const DevModel& m = *(const DevModel*)(const GModel*)a.m;  // constant AS: uniform reads -> s_load
  float* gst = a.state + (size_t)env * m.stride;
  load_params(s, m, a.dr ? a.dr + (size_t)env * PP3_NDR : nullptr, l);
  if (l < NQ) s.qpos[l] = gst[PP3_S_QPOS + l];
  if (l < NV) { s.qvel[l] = gst[PP3_S_QVEL + l]; s.qws[l] = gst[PP3_S_QACC_WS + l]; }
  if (l < NU) s.ctrl[l] = a.ctrl[(size_t)env * NU + l];
  const KinConst kc = kin_const(m, l);
  SYNC();
  for (int i = 0; i < a.nsteps; i++) {
    const GModel* mp = (const GModel*)(a.m);
    asm volatile("" : "+s"(mp));
    substep(s, *(const DevModel*)mp, l, h, i > 0, kc PROF_NULL);
  }
  if (a.nsteps > 0) euler_step(s, m, l);
  if (!own) return;
  if (a.pipe) write_pipeline(s, m, a.pipe + (size_t)env * PP3_PIPE_STRIDE, l, false);
  if (l < NQ) gst[PP3_S_QPOS + l] = s.qpos[l];
  if (l < NV) { gst[PP3_S_QVEL + l] = s.qvel[l]; gst[PP3_S_QACC_WS + l] = s.qws[l]; }
}

__global__ void fill_uniform_kernel(float* p, int64_t n, uint32_t seed, uint32_t ctr, float lo, float hi) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t y0, y1;
  threefry(seed, ctr, (uint32_t)(i >> 32), (uint32_t)i, y0, y1);
  const float u = __uint_as_float(((y0 ^ y1) >> 9) | 0x3F800000u) - 1.0f;
  p[i] = lo + u * (hi - lo);
}

}  // namespace pp3

// ======================================================================================
// host side: C-ABI
// ======================================================================================
using namespace pp3;

struct pp3_env {
  int device;
  int N;
  int stride;
  int H;
  hipStream_t stream;
  DevModel* dmodel;
  float* state;
  float* obs;  // [N][36H], updated in place by every step (stable pointer: pp3_field(PP3_F_OBS))
  float* reward;
  float* done;
  float* metrics;
  float* dr;
  int dr_on;
  float* pipe;
  int pipe_on;
  int nc;  // contact cap (kernel template): 8 on flat terrain, 16 with obstacle geoms
  float* action;
  float* episode;      // auto-reset mode buffers (null when off)
  float* first_state;
  float* first_obs;
  int episode_length;
  int action_repeat;  // auto-reset mode: launches per wrapper step (1 otherwise)
  float* terrain;  // TerrainRec rows (pp3_set_terrain), null until first set
  int nbox;        // world box-geom slots in the model
  int cull;        // DevModel::cull_on: steps launch env_step_kernel<..., CULL = true>
  hipEvent_t ev0, ev1;
};

static thread_local std::string g_err;
static int set_err(int code, const std::string& msg) {
  g_err = msg;
  return code;
}
#define HIPCHK(x)                                                                              \
  do {                                                                                         \
    hipError_t e_ = (x);                                                                       \
    if (e_ != hipSuccess) return set_err(PP3_ERR_HIP, std::string(#x) + ": " + hipGetErrorString(e_)); \
  } while (0)

static void clamp_solimp(const double in[5], float out[5]) {
  double dmin = in[0], dmax = in[1], width = in[2], mid = in[3], power = in[4];
  dmin = dmin < 0.0001 ? 0.0001 : dmin > 0.9999 ? 0.9999 : dmin;
  dmax = dmax < 0.0001 ? 0.0001 : dmax > 0.9999 ? 0.9999 : dmax;
  width = width < 1e-15 ? 1e-15 : width;
  mid = mid < 0.0001 ? 0.0001 : mid > 0.9999 ? 0.9999 : mid;
  power = power < 1 ? 1 : power;
  out[0] = (float)dmin; out[1] = (float)dmax; out[2] = (float)width; out[3] = (float)mid; out[4] = (float)power;
}
static void kb_of(const double solref[2], const double solimp[5], double h, float* k, float* b) {
  float si[5];
  clamp_solimp(solimp, si);
  double dmax = si[1];
  if (solref[0] > 0) {
    double tc = solref[0] < 2 * h ? 2 * h : solref[0], dr = solref[1];
    *k = (float)(1.0 / (dmax * dmax * tc * tc * dr * dr));
    *b = (float)(2.0 / (dmax * tc));
  } else {
    *k = (float)(-solref[0] / (dmax * dmax));
    *b = (float)(-solref[1] / dmax);
  }
}
static double imp_host(const float si[5], double pos, double margin) {
  double x = fabs((pos - margin) / si[2]);
  if (x >= 1) return si[1];
  if (x <= 0) return si[0];
  double y;
  if (si[4] == 1) y = x;
  else if (x <= si[3]) y = pow(x, si[4]) / pow(si[3], si[4] - 1);
  else y = 1 - pow(1 - x, si[4]) / pow(1 - si[3], si[4] - 1);
  return si[0] + y * (si[1] - si[0]);
}

static void quat2mat_d(const double q[4], double R[9]) {
  double w = q[0], x = q[1], y = q[2], z = q[3];
  R[0] = 1 - 2 * (y * y + z * z); R[1] = 2 * (x * y - w * z); R[2] = 2 * (x * z + w * y);
  R[3] = 2 * (x * y + w * z); R[4] = 1 - 2 * (x * x + z * z); R[5] = 2 * (y * z - w * x);
  R[6] = 2 * (x * z - w * y); R[7] = 2 * (y * z + w * x); R[8] = 1 - 2 * (x * x + y * y);
}

// the per-lane phase records (pp3_device.h LaneRec) from the already filled model fields
static void set_i(float& f, int32_t v) { memcpy(&f, &v, 4); }
template <int N>
static void put_rec(LaneTab<N>& t, int l, const LaneRec<N>& r) {
  for (int k = 0; k < N; k++)
    for (int c = 0; c < 4; c++) t.g[k][l][c] = r.f[4 * k + c];
}
static void fill_lane_records(DevModel* d) {
  for (int l = 0; l < 32; l++) {
    LaneRec<(LL_WORDS + 3) / 4> rl = {};
    float* f = rl.f;
    if (l < 2 * (NJ - 1)) {
      const int j = 1 + l / 2, hi = l & 1;
      set_i(f[LL_LIM_ON], d->jnt_limited[j] ? 1 : 0);
      f[LL_RANGE] = d->jnt_range[j][hi];
      f[LL_MARGIN] = d->lim_margin[j];
      f[LL_INVW] = d->lim_invw[j];
      f[LL_B] = d->lim_b[j];
      f[LL_K] = d->lim_k[j];
      for (int k = 0; k < 5; k++) f[LL_SOLIMP + k] = d->lim_solimp[j][k];
    }
    if (l < NFR) {
      f[LL_FR_R] = d->fr_R[6 + l];
      f[LL_FR_B] = d->fr_b[6 + l];
    }
    if (l < NU) {
      set_i(f[LL_ACT_DOF], d->act_dof[l]);
      set_i(f[LL_ACT_QADR], d->act_qadr[l]);
      set_i(f[LL_ACT_FLAGS], (d->act_ctrllimited[l] ? ACTF_CTRLLIMITED : 0) | (d->act_forcelimited[l] ? ACTF_FORCELIMITED : 0) |
                                 (d->act_biastype[l] == PP3_BIAS_AFFINE ? ACTF_AFFINE : 0));
      f[LL_CRANGE] = d->act_crange[l][0];
      f[LL_CRANGE + 1] = d->act_crange[l][1];
      f[LL_GEAR] = d->act_gear[l];
      f[LL_GAIN] = d->act_gain[l];
      for (int k = 0; k < 3; k++) f[LL_BIAS + k] = d->act_bias[l][k];
      f[LL_FRANGE] = d->act_frange[l][0];
      f[LL_FRANGE + 1] = d->act_frange[l][1];
    }
    LaneRec<(LC_WORDS + 3) / 4> rc = {};
    float* c = rc.f;
    if (l >= 1 && l < NB)
      for (int k = 0; k < 4; k++) c[LC_IQUAT + k] = d->body_iquat[l][k];
    if (l < d->nrobot_geom) {
      const int g = d->robot_geom[l];
      set_i(c[LC_PT_BODY], d->cg_body[g]);
      for (int k = 0; k < 3; k++) c[LC_PT_POS + k] = d->cg_pos[g][k];
    } else if (l >= 16 && l < 20) {
      const int si = d->feet_site[l - 16];
      set_i(c[LC_PT_BODY], d->site_body[si]);
      for (int k = 0; k < 3; k++) c[LC_PT_POS + k] = d->site_pos[si][k];
    }
    LaneRec<(LM_WORDS + 3) / 4> rm = {};
    float* mr = rm.f;
    for (int t = 0; t < 4; t++) {
      const int p = l + 32 * t;
      if (p < d->nmpair) {
        const int i = d->mp_i[p], j = d->mp_j[p];
        set_i(mr[LM_IJ + t], i | (j << 8));
        mr[LM_ARM + t] = i == j ? d->dof_armature[i] : 0.0f;
      } else {
        set_i(mr[LM_IJ + t], -1);
      }
    }
    if (l < NV) mr[LM_DAMP] = d->dof_damping[l];
    if (l < NFR) mr[LM_FLOSS] = d->fr_floss[6 + l];
    LaneRec<(LE_WORDS + 3) / 4> re = {};
    float* e = re.f;
    if (l < NU) {
      e[LE_POSE] = d->default_pose[l];
      e[LE_JLO] = d->jlo[l];
      e[LE_JHI] = d->jhi[l];
      if (l % 3 == 1) e[LE_ABD] = d->des_abd[l / 3];
    }
    if (l < 4) set_i(e[LE_LEG], d->lower_leg_body[l]);
    if (l >= 16 && l < 16 + NU) e[LE_POSE16] = d->default_pose[l - 16];
    put_rec(d->lane_lim, l, rl);
    put_rec(d->lane_com, l, rc);
    put_rec(d->lane_m, l, rm);
    put_rec(d->lane_env, l, re);
    LaneRec<(LS_WORDS + 3) / 4> rs = {};
    float* sr = rs.f;
    if (l < d->nsensor) {
      const int sid = d->sensor_objid[l], b = d->site_body[sid];
      set_i(sr[LS_TYPE], d->sensor_type[l]);
      set_i(sr[LS_ADR], d->sensor_adr[l]);
      sr[LS_CUT] = d->sensor_cutoff[l];
      set_i(sr[LS_BODY], b);
      for (int k = 0; k < 3; k++) sr[LS_SPOS + k] = d->site_pos[sid][k];
      for (int k = 0; k < 4; k++) sr[LS_SQUAT + k] = d->site_quat[sid][k];
      int chain[NB], n = 0;  // (depth checked at create)
      for (int bb = b; bb > 0 && n < LS_MAXCH; bb = d->body_parent[bb]) chain[n++] = bb;
      set_i(sr[LS_NCH], n);
      for (int c = 0; c < n; c++) {  // root first
        const int bb = chain[n - 1 - c];
        set_i(sr[LS_CH + 4 * c], bb);
        set_i(sr[LS_CH + 4 * c + 1], d->body_dofadr[bb]);
        set_i(sr[LS_CH + 4 * c + 2], d->body_dofnum[bb]);
        set_i(sr[LS_CH + 4 * c + 3], d->body_parent[bb]);
      }
    }
    put_rec(d->lane_sens, l, rs);
  }
  for (int p = 0; p < d->npair; p++) {
    d->pair_gid[p][0] = (float)d->cg_id[d->pair_g1[p]];
    d->pair_gid[p][1] = (float)d->cg_id[d->pair_g2[p]];
  }
  for (int p = 0; p < d->npair; p++) {
    const int ga = d->cg_id[d->pair_g1[p]], gb = d->cg_id[d->pair_g2[p]];
    int kn = 0, bo = 0;
    for (int i = 0; i < d->n_knee_geoms; i++) kn += (ga == d->knee_geoms[i] || gb == d->knee_geoms[i]) ? 1 : 0;
    for (int i = 0; i < d->n_torso_geoms; i++) bo += (ga == d->torso_geoms[i] || gb == d->torso_geoms[i]) ? 1 : 0;
    d->pair_con[p].knee = (float)kn;
    d->pair_con[p].body = (float)bo;
  }
}

static int build_devmodel(const pp3_model_t* mm, const pp3_env_config_t* c, DevModel* d) {
  memset(d, 0, sizeof(*d));
  // topology checks (fixed-structure kernel)
  if (mm->jnt_type[0] != PP3_JNT_FREE || mm->body_parentid[1] != 0) return set_err(PP3_ERR_MODEL, "base must be a free body");
  for (int l = 0; l < 4; l++)
    for (int k = 0; k < 3; k++) {
      int b = 2 + 3 * l + k, j = 1 + 3 * l + k;
      if (mm->body_parentid[b] != (k == 0 ? 1 : b - 1) || mm->body_jntadr[b] != j || mm->jnt_type[j] != PP3_JNT_HINGE ||
          mm->jnt_dofadr[j] != 6 + 3 * l + k || mm->jnt_qposadr[j] != 7 + 3 * l + k)
        return set_err(PP3_ERR_MODEL, "legs must be 4 serial chains of 3 hinge bodies");
    }
  if (mm->cone != PP3_CONE_PYRAMIDAL) return set_err(PP3_ERR_MODEL, "only pyramidal cones");
  for (int j = 1; j < NJ; j++)
    if (mm->jnt_pos[j][0] != 0 || mm->jnt_pos[j][1] != 0 || mm->jnt_pos[j][2] != 0)
      return set_err(PP3_ERR_MODEL, "hinge anchors must coincide with body origins (jnt_pos = 0)");
  if (mm->eulerdamp) {
    for (int i = 0; i < NV; i++)
      if (mm->dof_damping[i] > 0) return set_err(PP3_ERR_MODEL, "eulerdamp with joint damping is not supported (xml:58 disables it)");
  }
  if (c->obs_history < 1 || c->obs_history > HMAX) return set_err(PP3_ERR_ARG, "observation_history must be in [1, 16]");
  if (c->latency_len < 1 || c->latency_len > PP3_MAX_LAG || c->imu_latency_len < 1 || c->imu_latency_len > PP3_MAX_LAG)
    return set_err(PP3_ERR_ARG, "latency distributions must have 1..8 entries");
  if (c->n_frames < 1) return set_err(PP3_ERR_ARG, "n_frames < 1");
  const double h = mm->timestep;
  d->h = (float)h;
  for (int k = 0; k < 3; k++) d->gravity[k] = (float)mm->gravity[k];
  d->impratio = (float)mm->impratio;
  d->gtol_scale = (float)(mm->tolerance * mm->ls_tolerance * mm->meaninertia * NV);
  d->ls_iterations = mm->ls_iterations;
  d->iterations = mm->iterations;
  for (int b = 0; b < NB; b++) {
    for (int k = 0; k < 3; k++) {
      d->body_pos[b][k] = (float)mm->body_pos[b][k];
      d->body_ipos[b][k] = (float)mm->body_ipos[b][k];
      d->body_inertia[b][k] = (float)mm->body_inertia[b][k];
    }
    for (int k = 0; k < 4; k++) {
      d->body_quat[b][k] = (float)mm->body_quat[b][k];
      d->body_iquat[b][k] = (float)mm->body_iquat[b][k];
    }
    d->body_mass[b] = (float)mm->body_mass[b];
    uint32_t mask = 0;
    for (int bb = b; bb > 0; bb = mm->body_parentid[bb])
      for (int i = 0; i < mm->body_dofnum[bb]; i++) mask |= 1u << (mm->body_dofadr[bb] + i);
    d->body_dofmask[b] = mask;
  }
  for (int i = 0; i < NV; i++) d->dof_body[i] = mm->dof_bodyid[i];
  for (int j = 0; j < NJ; j++) {
    for (int k = 0; k < 3; k++) {
      d->jnt_pos[j][k] = (float)mm->jnt_pos[j][k];
      d->jnt_axis[j][k] = (float)mm->jnt_axis[j][k];
    }
    d->jnt_range[j][0] = (float)mm->jnt_range[j][0];
    d->jnt_range[j][1] = (float)mm->jnt_range[j][1];
    d->jnt_limited[j] = mm->jnt_limited[j];
    kb_of(mm->jnt_solref[j], mm->jnt_solimp[j], h, &d->lim_k[j], &d->lim_b[j]);
    clamp_solimp(mm->jnt_solimp[j], d->lim_solimp[j]);
    d->lim_margin[j] = (float)mm->jnt_margin[j];
    d->lim_invw[j] = (float)mm->dof_invweight0[mm->jnt_dofadr[j]];
    // both sides of one hinge can only be violated together when the range is narrower than
    // twice the margin; excluding that bounds the limit rows at one per hinge (NLMAX)
    if (j > 0 && mm->jnt_limited[j] && !(mm->jnt_range[j][1] - mm->jnt_range[j][0] > 2.0 * mm->jnt_margin[j]))
      return set_err(PP3_ERR_MODEL, "joint " + std::to_string(j) +
                                        ": range narrower than twice the margin (both limit sides could be active)");
  }
  for (int i = 0; i < NQ; i++) { d->qpos0[i] = (float)mm->qpos0[i]; d->key_qpos[i] = (float)mm->key_qpos[i]; }
  for (int i = 0; i < NV; i++) {
    d->dof_armature[i] = (float)mm->dof_armature[i];
    d->dof_damping[i] = (float)mm->dof_damping[i];
    d->fr_floss[i] = (float)mm->dof_frictionloss[i];
    float si[5], k, b;
    clamp_solimp(mm->dof_solimp[i], si);
    kb_of(mm->dof_solref[i], mm->dof_solimp[i], h, &k, &b);
    double imp = imp_host(si, 0.0, 0.0);
    double R = (1 - imp) / imp * mm->dof_invweight0[i];
    d->fr_R[i] = (float)(R < 1e-15 ? 1e-15 : R);
    d->fr_b[i] = b;
    if (i >= 6 && mm->dof_frictionloss[i] <= 0) return set_err(PP3_ERR_MODEL, "every hinge needs frictionloss > 0 (xml:55)");
    if (i < 6 && mm->dof_frictionloss[i] > 0) return set_err(PP3_ERR_MODEL, "free-joint frictionloss unsupported");
  }
  // M sparsity pairs
  int np = 0;
  for (int i = 0; i < NV; i++)
    for (int j = i; j >= 0; j = mm->dof_parentid[j]) {
      if (np >= NMPAIR_MAX) return set_err(PP3_ERR_MODEL, "M too dense");
      d->mp_i[np] = (uint8_t)i;
      d->mp_j[np] = (uint8_t)j;
      np++;
    }
  d->nmpair = np;
  if (np != NMPAIR) return set_err(PP3_ERR_MODEL, "mass-matrix sparsity differs from the 13-body quadruped tree");
  // collision geoms
  d->ncgeom = mm->ncgeom;
  int nslot = 0;
  int box_slot[PP3_MAX_CGEOM];
  d->nbox = 0;
  d->terrain = 0;
  for (int g = 0; g < mm->ncgeom; g++) {
    box_slot[g] = (mm->cgeom_bodyid[g] == 0 && mm->cgeom_type[g] == PP3_GEOM_BOX) ? d->nbox++ : -1;
    d->cg_type[g] = mm->cgeom_type[g];
    d->cg_body[g] = mm->cgeom_bodyid[g];
    d->cg_id[g] = mm->cgeom_id[g];
    for (int k = 0; k < 3; k++) d->cg_size[g][k] = (float)mm->cgeom_size[g][k];
    if (mm->cgeom_bodyid[g] == 0) {
      d->cg_slot[g] = -1;
      double R[9];
      quat2mat_d(mm->cgeom_quat[g], R);
      for (int k = 0; k < 9; k++) d->cg_wmat[g][k] = (float)R[k];
      for (int k = 0; k < 3; k++) d->cg_pos[g][k] = (float)mm->cgeom_pos[g][k];
    } else {
      if (mm->cgeom_type[g] != PP3_GEOM_SPHERE) return set_err(PP3_ERR_MODEL, "moving collision geoms must be spheres");
      if (nslot >= NROBOT_GEOM) return set_err(PP3_ERR_MODEL, "too many robot collision geoms (max 8)");
      d->cg_slot[g] = nslot;
      d->robot_geom[nslot++] = g;
      for (int k = 0; k < 3; k++) d->cg_pos[g][k] = (float)mm->cgeom_pos[g][k];
    }
  }
  d->nrobot_geom = nslot;
  d->npair = mm->npair;
  for (int p = 0; p < mm->npair; p++) {
    int g1 = mm->pair_g1[p], g2 = mm->pair_g2[p];
    d->pair_g1[p] = g1;
    d->pair_g2[p] = g2;
    // mj_contactParam
    double solref[2], solimp[5], mu;
    int p1 = mm->cgeom_priority[g1], p2 = mm->cgeom_priority[g2];
    if (p1 != p2) {
      int g = p1 > p2 ? g1 : g2;
      mu = mm->cgeom_friction[g][0];
      for (int k = 0; k < 2; k++) solref[k] = mm->cgeom_solref[g][k];
      for (int k = 0; k < 5; k++) solimp[k] = mm->cgeom_solimp[g][k];
    } else {
      double s1 = mm->cgeom_solmix[g1], s2 = mm->cgeom_solmix[g2], mix;
      if (s1 >= 1e-15 && s2 >= 1e-15) mix = s1 / (s1 + s2);
      else if (s1 < 1e-15 && s2 < 1e-15) mix = 0.5;
      else if (s1 < 1e-15) mix = 0;
      else mix = 1;
      if (mm->cgeom_solref[g1][0] > 0 && mm->cgeom_solref[g2][0] > 0)
        for (int k = 0; k < 2; k++) solref[k] = mix * mm->cgeom_solref[g1][k] + (1 - mix) * mm->cgeom_solref[g2][k];
      else
        for (int k = 0; k < 2; k++) solref[k] = fmin(mm->cgeom_solref[g1][k], mm->cgeom_solref[g2][k]);
      for (int k = 0; k < 5; k++) solimp[k] = mix * mm->cgeom_solimp[g1][k] + (1 - mix) * mm->cgeom_solimp[g2][k];
      mu = fmax(mm->cgeom_friction[g1][0], mm->cgeom_friction[g2][0]);
    }
    d->pair_mu[p] = (float)mu;
    kb_of(solref, solimp, h, &d->pair_k[p], &d->pair_b[p]);
    clamp_solimp(solimp, d->pair_solimp[p]);
    d->pair_margin[p] = (float)(fmax(mm->cgeom_margin[g1], mm->cgeom_margin[g2]) - fmax(mm->cgeom_gap[g1], mm->cgeom_gap[g2]));
    d->pair_tran[p] = (float)(mm->body_invweight0[mm->cgeom_bodyid[g1]][0] + mm->body_invweight0[mm->cgeom_bodyid[g2]][0]);
    {  // column support of this pair's contact Jacobian (bodies 2..13 = legs of 3 links, 1 = base)
      auto cls = [](int b) { return b == 0 ? -1 : (b == 1 ? 4 : (b - 2) / 3); };
      const int c1 = cls(mm->cgeom_bodyid[g1]), c2 = cls(mm->cgeom_bodyid[g2]);
      int sup;
      if (c1 < 0) sup = c2;
      else if (c2 < 0) sup = c1;
      else if (c1 == c2) sup = c1;
      else if (c1 == 4) sup = c2;
      else if (c2 == 4) sup = c1;
      else sup = 5 | 8 | ((c1 < c2 ? c1 : c2) << 4) | ((c1 < c2 ? c2 : c1) << 6);  // leg-leg: the pair
      d->pair_sup[p] = sup < 0 ? 5 : sup;  // (5 without bit 3: legs unknown -> dense LDL^T)
    }
    d->pair_dm[p][0] = d->body_dofmask[mm->cgeom_bodyid[g1]];
    d->pair_dm[p][1] = d->body_dofmask[mm->cgeom_bodyid[g2]];
    {  // flattened narrow-phase record
      PairRec r;
      memset(&r, 0, sizeof(r));
      const int t1 = mm->cgeom_type[g1], t2 = mm->cgeom_type[g2];
      r.kind = (t1 == PP3_GEOM_PLANE && t2 == PP3_GEOM_SPHERE) ? PK_PLANE_SPHERE
               : (t1 == PP3_GEOM_SPHERE && t2 == PP3_GEOM_SPHERE) ? PK_SPHERE_SPHERE
               : (t1 == PP3_GEOM_SPHERE && t2 == PP3_GEOM_BOX) ? PK_SPHERE_BOX : -1;
      r.s1 = d->cg_slot[g1];
      r.s2 = r.kind == PK_SPHERE_BOX ? -1 - box_slot[g2] : d->cg_slot[g2];
      r.r1 = d->cg_size[g1][0];
      r.r2 = d->cg_size[g2][0];
      r.margin = d->pair_margin[p];
      for (int k = 0; k < 3; k++) { r.p1[k] = d->cg_pos[g1][k]; r.p2[k] = d->cg_pos[g2][k]; }
      const int gf = r.kind == PK_SPHERE_BOX ? g2 : g1;  // plane frame / box frame
      for (int k = 0; k < 9; k++) r.R[k] = d->cg_wmat[gf][k];
      if (r.kind == PK_SPHERE_BOX)
        for (int k = 0; k < 3; k++) r.half[k] = d->cg_size[g2][k];
      const float* rf = reinterpret_cast<const float*>(&r);
      for (int k = 0; k < PAIR_REC / 4; k++)
        for (int c = 0; c < 4; c++) d->pair_rec.g[k][p][c] = rf[4 * k + c];
    }
    {  // contact-side record
      PairCon& q = d->pair_con[p];
      memset(&q, 0, sizeof(q));
      q.sup = d->pair_sup[p];
      q.dm[0] = d->pair_dm[p][0];
      q.dm[1] = d->pair_dm[p][1];
      q.mu = d->pair_mu[p];
      q.tran = d->pair_tran[p];
      q.margin = d->pair_margin[p];
      q.b = d->pair_b[p];
      q.k = d->pair_k[p];
      for (int k = 0; k < 5; k++) q.solimp[k] = d->pair_solimp[p][k];
    }
    if (mm->cgeom_margin[g1] != 0 || mm->cgeom_margin[g2] != 0) return set_err(PP3_ERR_MODEL, "nonzero geom margins unsupported");
  }
  {  // sphere-box cull tables (DevModel::cull_on)
    d->cull_on = 0;
    d->cull_reach = 0.0f;
    memset(d->pair_box4, 0xFF, sizeof(d->pair_box4));
    memset(d->box_tab, 0, sizeof(d->box_tab));
    bool ok = d->nbox >= 1 && d->nbox <= 32 && d->npair > 32 && d->npair <= 32 * 5 && mm->body_parentid[1] == 0;
    const char* off = getenv("PP3_NO_CULL");  // tests only: every pair through the narrow phase
    if (off && off[0] == '1') ok = false;
    double reach = 0.0, margin = 0.0;
    for (int sl = 0; ok && sl < d->nrobot_geom; sl++) {  // chain of link offsets from body 1's origin
      const int g = d->robot_geom[sl];
      const double* gp = mm->cgeom_pos[g];
      double dist = sqrt(gp[0] * gp[0] + gp[1] * gp[1] + gp[2] * gp[2]);
      int b = mm->cgeom_bodyid[g];
      for (; b > 1; b = mm->body_parentid[b]) {
        const double* bp = mm->body_pos[b];
        dist += sqrt(bp[0] * bp[0] + bp[1] * bp[1] + bp[2] * bp[2]);
      }
      if (b != 1) ok = false;
      reach = fmax(reach, dist + mm->cgeom_size[g][0]);
    }
    for (int p = 0; ok && p < d->npair; p++) {
      const int g1 = mm->pair_g1[p], g2 = mm->pair_g2[p];
      const bool sb = mm->cgeom_type[g1] == PP3_GEOM_SPHERE && mm->cgeom_type[g2] == PP3_GEOM_BOX && box_slot[g2] >= 0;
      if (sb) margin = fmax(margin, (double)d->pair_margin[p]);
      if (p >= 32 && sb) {
        const int k = p / 32 - 1, ln = p % 32;
        d->pair_box4[ln] = (d->pair_box4[ln] & ~(0xFFu << (8 * k))) | ((uint32_t)box_slot[g2] << (8 * k));
      }
    }
    for (int g = 0; ok && g < mm->ncgeom; g++) {
      if (box_slot[g] < 0) continue;
      TerrainRec& t = d->box_tab[box_slot[g]];
      for (int k = 0; k < 3; k++) { t.p[k] = d->cg_pos[g][k]; t.half[k] = d->cg_size[g][k]; }
      for (int k = 0; k < 9; k++) t.R[k] = d->cg_wmat[g][k];
    }
    if (ok) {
      d->cull_reach = (float)(reach + margin + 0.01);
      d->cull_on = 1;
    }
  }
  d->nsite = mm->nsite;
  for (int s = 0; s < mm->nsite; s++) {
    d->site_body[s] = mm->site_bodyid[s];
    for (int k = 0; k < 3; k++) d->site_pos[s][k] = (float)mm->site_pos[s][k];
    for (int k = 0; k < 4; k++) d->site_quat[s][k] = (float)mm->site_quat[s][k];
  }
  if (mm->nsensor < 0 || mm->nsensor > PP3_MAX_SENSOR || mm->nsensordata > PP3_MAX_SENSORDATA)
    return set_err(PP3_ERR_MODEL, "too many sensors");
  d->nsensor = mm->nsensor;
  d->nsensordata = mm->nsensordata;
  for (int i = 0; i < mm->nsensor; i++) {
    d->sensor_type[i] = mm->sensor_type[i];
    d->sensor_objid[i] = mm->sensor_objid[i];
    d->sensor_adr[i] = mm->sensor_adr[i];
    d->sensor_cutoff[i] = (float)mm->sensor_cutoff[i];
    if (mm->sensor_objid[i] < 0 || mm->sensor_objid[i] >= mm->nsite) return set_err(PP3_ERR_MODEL, "sensor site id");
  }
  for (int b = 0; b < NB; b++) {
    d->body_parent[b] = mm->body_parentid[b];
    d->body_dofadr[b] = mm->body_dofadr[b];
    d->body_dofnum[b] = mm->body_dofnum[b];
  }
  for (int i = 0; i < mm->nsensor; i++) {  // the pipeline record's sensor lane records (fill_lane_records)
    int depth = 0;
    for (int bb = mm->site_bodyid[mm->sensor_objid[i]]; bb > 0; bb = mm->body_parentid[bb]) depth++;
    if (depth > LS_MAXCH) return set_err(PP3_ERR_MODEL, "sensor site body deeper than 4 levels");
  }
  for (int a = 0; a < NU; a++) {
    int j = mm->actuator_trnid[a];
    d->act_dof[a] = mm->jnt_dofadr[j];
    d->act_qadr[a] = mm->jnt_qposadr[j];
    if (mm->jnt_dofadr[j] != 6 + a) return set_err(PP3_ERR_MODEL, "actuator i must drive hinge dof 6+i");
    d->act_biastype[a] = mm->actuator_biastype[a];
    d->act_forcelimited[a] = mm->actuator_forcelimited[a];
    d->act_ctrllimited[a] = mm->actuator_ctrllimited[a];
    d->act_gear[a] = (float)mm->actuator_gear[a];
    d->act_gain[a] = (float)mm->actuator_gainprm[a][0];
    for (int k = 0; k < 3; k++) d->act_bias[a][k] = (float)mm->actuator_biasprm[a][k];
    for (int k = 0; k < 2; k++) {
      d->act_frange[a][k] = (float)mm->actuator_forcerange[a][k];
      d->act_crange[a][k] = (float)mm->actuator_ctrlrange[a][k];
    }
  }
  // environment
  d->n_frames = c->n_frames;
  d->H = c->obs_history;
  d->La = c->latency_len;
  d->Li = c->imu_latency_len;
  d->use_imu = c->use_imu;
  d->resample_step = c->resample_velocity_step;
  d->term_step = c->early_termination_step_threshold;
  d->torso_body = c->torso_body;
  if (c->torso_body < 1 || c->torso_body >= NB) return set_err(PP3_ERR_ARG, "torso body id out of range");
  for (int f = 0; f < 4; f++) {
    d->feet_site[f] = c->feet_site[f];
    d->lower_leg_body[f] = c->lower_leg_body[f];
    if (c->feet_site[f] < 0 || c->feet_site[f] >= mm->nsite) return set_err(PP3_ERR_ARG, "foot site not found");
    if (c->lower_leg_body[f] < 1 || c->lower_leg_body[f] >= NB) return set_err(PP3_ERR_ARG, "lower-leg body id out of range");
  }
  if (c->n_upper_leg_geoms < 0 || c->n_upper_leg_geoms > 16) return set_err(PP3_ERR_ARG, "n_upper_leg_geoms must be 0..16");
  if (c->n_torso_geoms < 0 || c->n_torso_geoms > 8) return set_err(PP3_ERR_ARG, "n_torso_geoms must be 0..8");
  d->n_knee_geoms = c->n_upper_leg_geoms;
  for (int i = 0; i < c->n_upper_leg_geoms && i < 16; i++) d->knee_geoms[i] = c->upper_leg_geoms[i];
  d->n_torso_geoms = c->n_torso_geoms;
  for (int i = 0; i < c->n_torso_geoms && i < 8; i++) d->torso_geoms[i] = c->torso_geoms[i];
  d->partitionable = c->rng_partitionable;
  d->imu_off = PP3_S_ACT_BUF + 12 * c->latency_len;
  d->stride = d->imu_off + 6 * c->imu_latency_len;
  for (int i = 0; i < PP3_MAX_LAG; i++) {
    d->lat_dist[i] = (float)c->latency_dist[i];
    d->imu_lat_dist[i] = (float)c->imu_latency_dist[i];
  }
  d->action_scale = (float)c->action_scale;
  for (int j = 0; j < NU; j++) {
    d->default_pose[j] = (float)c->default_pose[j];
    d->jlo[j] = (float)c->joint_lower[j];
    d->jhi[j] = (float)c->joint_upper[j];
  }
  for (int k = 0; k < 4; k++) d->des_abd[k] = (float)c->desired_abduction[k];
  for (int k = 0; k < 3; k++) {
    d->start_lo[k] = (float)c->start_pos_min[k];
    d->start_hi[k] = (float)c->start_pos_max[k];
    d->des_z[k] = (float)c->desired_world_z[k];
  }
  for (int k = 0; k < 2; k++) {
    d->cmd_x[k] = (float)c->lin_vel_x_range[k];
    d->cmd_y[k] = (float)c->lin_vel_y_range[k];
    d->cmd_w[k] = (float)c->ang_vel_range[k];
  }
  d->zero_cmd_p = (float)c->zero_command_probability;
  d->stand_thr = (float)c->stand_still_command_threshold;
  d->max_pitch = (float)c->max_pitch_command;
  d->max_roll = (float)c->max_roll_command;
  d->n_ang = (float)c->ang_vel_noise;
  d->n_grav = (float)c->gravity_noise;
  d->n_motor = (float)c->motor_angle_noise;
  d->n_act = (float)c->last_action_noise;
  d->kick_vel = (float)c->kick_vel;
  d->kick_p = (float)c->kick_probability;
  d->term_z = (float)c->terminal_body_z;
  d->cos_term_angle = (float)cos(c->terminal_body_angle);
  d->foot_radius = (float)c->foot_radius;
  d->env_dt = (float)c->env_dt;
  d->dt = (float)c->dt;
  for (int k = 0; k < PP3_NREWARD; k++) d->scales[k] = (float)c->reward_scales[k];
  d->sigma = (float)c->tracking_sigma;
  d->pi_f = 3.14159265358979323846f;
  fill_lane_records(d);
  return PP3_OK;
}

extern "C" {

int pp3_abi_version(void) { return PP3_ABI_VERSION; }

size_t pp3_struct_size(int which) {
  if (which == 0) return sizeof(pp3_model_t);
  if (which == 1) return sizeof(pp3_env_config_t);
  if (which == 2) return sizeof(DevModel);
  if (which == 3) return sizeof(Shared<8>);
  if (which == 4) return sizeof(Shared<16>);
  return 0;
}

const char* pp3_last_error(void) { return g_err.c_str(); }

int pp3_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

static int alloc_env_buffers(pp3_env* e, const DevModel& hm);

int pp3_create(const pp3_model_t* model, const pp3_env_config_t* cfg, int32_t num_envs, int32_t device, pp3_env_t** out) {
  if (!model || !cfg || !out || num_envs < 1) return set_err(PP3_ERR_ARG, "bad arguments to pp3_create");
  if (PP3_DIAG_BUILD) {  // pp3_diag.h: a diagnostic library is never the product
    const char* ok = getenv("PP3_ALLOW_DIAG_BUILD");
    if (!ok || strcmp(ok, "1") != 0)
      return set_err(PP3_ERR_ARG, "pp3_create: this library is a diagnostic build (PP3_PHASE_PROF / PP3_DEBUG); "
                                  "set PP3_ALLOW_DIAG_BUILD=1 to use it for diagnostics");
  }
  DevModel hm;
  int rc = build_devmodel(model, cfg, &hm);
  if (rc) return rc;
  HIPCHK(hipSetDevice(device));
  pp3_env* e = new pp3_env();
  memset(e, 0, sizeof(*e));
  e->action_repeat = 1;
  e->device = device;
  e->N = num_envs;
  e->stride = hm.stride;
  e->H = hm.H;
  e->nbox = hm.nbox;
  e->cull = hm.cull_on;
  {
    // contact cap: 8 deepest per env by default, flat or with obstacle boxes (the reference's
    // MJX keeps max_contact_points = 5, test_pupper_model.xml:227-230); 16 on request
    e->nc = cfg->ncon_max > 0 ? cfg->ncon_max : 8;
    if (e->nc != 8 && e->nc != 16) {
      delete e;
      return set_err(PP3_ERR_ARG, "ncon_max must be 0 (auto), 8 or 16");
    }
  }
  rc = alloc_env_buffers(e, hm);
  if (rc) {
    pp3_destroy(e);  // frees what was allocated (hipFree(nullptr) is a no-op)
    return rc;
  }
  *out = e;
  return PP3_OK;
}

// device buffers of a new handle (pp3_create); on failure the caller destroys the handle
static int alloc_env_buffers(pp3_env* e, const DevModel& hm) {
  const size_t N = (size_t)e->N;
  HIPCHK(hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking));
  HIPCHK(hipMalloc(&e->dmodel, sizeof(DevModel)));
  HIPCHK(hipMemcpy(e->dmodel, &hm, sizeof(DevModel), hipMemcpyHostToDevice));
  HIPCHK(hipMalloc(&e->state, N * e->stride * sizeof(float)));
  HIPCHK(hipMalloc(&e->obs, N * PP3_OBS_DIM * e->H * sizeof(float)));
  HIPCHK(hipMalloc(&e->reward, N * sizeof(float)));
  HIPCHK(hipMalloc(&e->done, N * sizeof(float)));
  HIPCHK(hipMalloc(&e->metrics, N * PP3_NMETRIC * sizeof(float)));
  HIPCHK(hipMalloc(&e->dr, N * PP3_NDR * sizeof(float)));
  HIPCHK(hipMalloc(&e->pipe, N * PP3_PIPE_STRIDE * sizeof(float)));
  HIPCHK(hipMalloc(&e->action, N * PP3_NU * sizeof(float)));
  HIPCHK(hipMemset(e->state, 0, N * e->stride * sizeof(float)));
  HIPCHK(hipMemset(e->obs, 0, N * PP3_OBS_DIM * e->H * sizeof(float)));
  HIPCHK(hipMemset(e->pipe, 0, N * PP3_PIPE_STRIDE * sizeof(float)));
  HIPCHK(hipMemset(e->action, 0, N * PP3_NU * sizeof(float)));
  HIPCHK(hipEventCreate(&e->ev0));
  HIPCHK(hipEventCreate(&e->ev1));
  return PP3_OK;
}

int pp3_destroy(pp3_env_t* e) {
  if (!e) return PP3_OK;
  (void)hipSetDevice(e->device);
  if (e->stream) (void)hipStreamSynchronize(e->stream);
  void* bufs[] = {e->dmodel, e->state, e->obs, e->reward, e->done, e->metrics, e->dr, e->pipe, e->action,
                  e->episode, e->first_state, e->first_obs, e->terrain};
  for (void* b : bufs) (void)hipFree(b);
  if (e->ev0) (void)hipEventDestroy(e->ev0);
  if (e->ev1) (void)hipEventDestroy(e->ev1);
  if (e->stream) (void)hipStreamDestroy(e->stream);
  delete e;
  return PP3_OK;
}

int32_t pp3_num_envs(const pp3_env_t* e) { return e ? e->N : 0; }
int32_t pp3_state_stride(const pp3_env_t* e) { return e ? e->stride : 0; }
int32_t pp3_env_device(const pp3_env_t* e) { return e ? e->device : -1; }

static hipStream_t stream_of(pp3_env_t* e, void* s) { return s ? (hipStream_t)s : e->stream; }

int pp3_reset(pp3_env_t* e, const uint32_t* keys_dev, const uint8_t* mask_dev, void* stream) {
  if (!e || !keys_dev) return set_err(PP3_ERR_ARG, "pp3_reset: null argument");
  HIPCHK(hipSetDevice(e->device));
  ResetArgs a;
  a.m = e->dmodel;
  a.state = e->state;
  a.obs = e->obs;
  a.reward = e->reward;
  a.done = e->done;
  a.metrics = e->metrics;
  a.keys = keys_dev;
  a.mask = mask_dev;
  a.dr = e->dr_on ? e->dr : nullptr;
  a.pipe = e->pipe_on ? e->pipe : nullptr;
  a.episode = e->episode_length > 0 ? e->episode : nullptr;
  a.first_state = e->first_state;
  a.first_obs = e->first_obs;
  a.N = e->N;
  if (e->nc == 8) hipLaunchKernelGGL(env_reset_kernel<8>, dim3((e->N + 1) / 2), dim3(WAVE), 0, stream_of(e, stream), a);
  else hipLaunchKernelGGL(env_reset_kernel<16>, dim3((e->N + 1) / 2), dim3(WAVE), 0, stream_of(e, stream), a);
  HIPCHK(hipGetLastError());
  return PP3_OK;
}

// One env step per launch (pp3_step), or nsteps fused into each launch (pp3_rollout: every wave
// runs its envs' steps back to back, so a slow wave of step t no longer holds up the whole batch
// at step t + 1).  With action_repeat > 1 (auto-reset mode) each wrapper step stays `repeat`
// single-step launches.
// tests / A-B only (PP3_POLICY_UNFUSED=1 in the environment): the policy rollout as per-step
// policy + step launches even where the fused kernel applies
static const bool g_policy_unfused = [] {
  const char* v = getenv("PP3_POLICY_UNFUSED");
  return v && v[0] == '1';
}();

static int launch_steps(pp3_env_t* e, const float* actions_dev, int64_t action_stride, int32_t nsteps,
                        float* traj_reward, float* traj_done, float* traj_obs, bool fused, void* stream) {
  HIPCHK(hipSetDevice(e->device));
  StepArgs a;
  a.m = e->dmodel;
  a.state = e->state;
  a.obs_in = e->obs;  // in place: each half-wave loads its env's history before storing it
  a.obs_out = e->obs;
  a.actions = actions_dev;
  a.reward = e->reward;
  a.done = e->done;
  a.metrics = e->metrics;
  a.dr = e->dr_on ? e->dr : nullptr;
  a.pipe = e->pipe_on ? e->pipe : nullptr;
  a.episode = e->episode_length > 0 ? e->episode : nullptr;
  a.first_state = e->first_state;
  a.first_obs = e->first_obs;
  a.episode_length = e->episode_length;
  a.N = e->N;
  a.repeat = e->episode_length > 0 && e->action_repeat > 1 ? e->action_repeat : 1;
  a.act_stride = action_stride;
  // a one-step rollout takes the single-step kernel: a fused launch of one step measured 7 % slower
  // than it (the fused kernel only pays off across steps)
  if (nsteps == 1) fused = false;
  const bool one_launch = fused && a.repeat == 1;
  a.nsteps = one_launch ? nsteps : 1;
  const dim3 grid((e->N + 1) / 2), block(WAVE);
  const hipStream_t st = stream_of(e, stream);
  const size_t on = (size_t)e->N * PP3_OBS_DIM * e->H;
  for (int t = 0; t < (one_launch ? 1 : nsteps); t++) {
    a.actions = actions_dev + (one_launch ? 0 : (size_t)t * (size_t)action_stride);
    a.traj_reward = traj_reward ? traj_reward + (one_launch ? 0 : (size_t)t * e->N) : nullptr;
    a.traj_done = traj_done ? traj_done + (one_launch ? 0 : (size_t)t * e->N) : nullptr;
    a.traj_obs = traj_obs ? traj_obs + (one_launch ? 0 : (size_t)t * on) : nullptr;
    for (a.phase = 0; a.phase < a.repeat; a.phase++) {  // action_repeat: the same action, k launches
      if (e->cull) {
        if (fused) {
          if (e->nc == 8) hipLaunchKernelGGL((env_step_kernel<8, true, 1, true>), grid, block, 0, st, a);
          else hipLaunchKernelGGL((env_step_kernel<16, true, 1, true>), grid, block, 0, st, a);
        } else {
          if (e->nc == 8) hipLaunchKernelGGL((env_step_kernel<8, false, 1, true>), grid, block, 0, st, a);
          else hipLaunchKernelGGL((env_step_kernel<16, false, 1, true>), grid, block, 0, st, a);
        }
      } else if (fused) {
        if (e->nc == 8) hipLaunchKernelGGL((env_step_kernel<8, true>), grid, block, 0, st, a);
        else hipLaunchKernelGGL((env_step_kernel<16, true>), grid, block, 0, st, a);
      } else {
        if (e->nc == 8) hipLaunchKernelGGL((env_step_kernel<8, false>), grid, block, 0, st, a);
        else hipLaunchKernelGGL((env_step_kernel<16, false>), grid, block, 0, st, a);
      }
      HIPCHK(hipGetLastError());
    }
  }
  return PP3_OK;
}

int pp3_step(pp3_env_t* e, const float* actions_dev, void* stream) {
  if (!e || !actions_dev) return set_err(PP3_ERR_ARG, "pp3_step: null argument");
  return launch_steps(e, actions_dev, 0, 1, nullptr, nullptr, nullptr, false, stream);
}

int pp3_rollout(pp3_env_t* e, const float* actions_dev, int64_t action_stride, int32_t nsteps, float* reward_dev,
                float* done_dev, float* obs_dev, void* stream) {
  if (!e || !actions_dev) return set_err(PP3_ERR_ARG, "pp3_rollout: null argument");
  if (nsteps < 1) return set_err(PP3_ERR_ARG, "pp3_rollout: nsteps must be >= 1");
  if (action_stride < 0) return set_err(PP3_ERR_ARG, "pp3_rollout: negative action_stride");
  return launch_steps(e, actions_dev, action_stride, nsteps, reward_dev, done_dev, obs_dev, true, stream);
}

// Which path pp3_rollout_policy takes on this env: ONE fused launch (env_step_kernel<8, true, 8>)
// unless the contact cap is 16 (its blocks do not fit 16 envs per workgroup), action_repeat > 1
// (a wrapper step is `repeat` launches), PP3_POLICY_UNFUSED=1 (A/B) or a diagnostic build (no fused
// policy kernel): then per-step policy + step launches.
static bool policy_rollout_fused(const pp3_env_t* e) {
#ifdef PP3_PHASE_PROF
  (void)e;
  return false;
#else
  const int repeat = e->episode_length > 0 && e->action_repeat > 1 ? e->action_repeat : 1;
  return e->nc == 8 && repeat == 1 && !g_policy_unfused;
#endif
}

int32_t pp3_rollout_policy_fused(const pp3_env_t* e) { return e ? (policy_rollout_fused(e) ? 1 : 0) : -1; }
int32_t pp3_narrow_cull(const pp3_env_t* e) { return e ? (e->cull ? 1 : 0) : -1; }

int pp3_rollout_policy(pp3_env_t* e, pp3_policy_t* policy, int32_t nsteps, float* actions_dev, float* reward_dev,
                       float* done_dev, float* obs_dev, void* stream) {
  if (!e || !policy || !actions_dev) return set_err(PP3_ERR_ARG, "pp3_rollout_policy: null argument");
  if (nsteps < 1) return set_err(PP3_ERR_ARG, "pp3_rollout_policy: nsteps must be >= 1");
  if (pp3_policy_out_dim(policy) != NU) return set_err(PP3_ERR_ARG, "pp3_rollout_policy: the policy must have 12 outputs");
  if (pp3_policy_device(policy) != e->device) return set_err(PP3_ERR_ARG, "pp3_rollout_policy: policy and env on different devices");
  if (pp3_policy_net(policy)->in_dim != PP3_OBS_DIM * e->H)
    return set_err(PP3_ERR_ARG, "pp3_rollout_policy: the policy's input width must equal the observation size 36 * observation_history");
  const size_t on = (size_t)e->N * PP3_OBS_DIM * e->H;
  const hipStream_t st = stream_of(e, stream);
#ifndef PP3_PHASE_PROF
  if (policy_rollout_fused(e)) {
    // ONE launch for the K steps: 8-wave workgroups of 16 envs run the MLP (mlp_tile, the code of
    // pp3_policy_act) on their envs' observations before each step, then each wave steps its two
    // envs (env_step_kernel<8, true, 8>)
    HIPCHK(hipSetDevice(e->device));
    PolicyStepArgs pa;
    StepArgs& a = pa.s;
    a.m = e->dmodel;
    a.state = e->state;
    a.obs_in = e->obs;
    a.obs_out = e->obs;
    a.actions = actions_dev;
    a.reward = e->reward;
    a.done = e->done;
    a.metrics = e->metrics;
    a.dr = e->dr_on ? e->dr : nullptr;
    a.pipe = e->pipe_on ? e->pipe : nullptr;
    a.episode = e->episode_length > 0 ? e->episode : nullptr;
    a.first_state = e->first_state;
    a.first_obs = e->first_obs;
    a.episode_length = e->episode_length;
    a.N = e->N;
    a.repeat = 1;
    a.phase = 0;
    a.nsteps = nsteps;
    a.act_stride = (int64_t)e->N * NU;
    a.traj_reward = reward_dev;
    a.traj_done = done_dev;
    a.traj_obs = obs_dev;
    pa.act = actions_dev;
    pa.net = *pp3_policy_net(policy);
    const dim3 grid((e->N + pp3pol::TILE - 1) / pp3pol::TILE), block(WAVE * pp3pol::NWAVE);
    if (e->cull) hipLaunchKernelGGL((env_step_kernel<8, true, pp3pol::NWAVE, true>), grid, block, 0, st, pa);
    else hipLaunchKernelGGL((env_step_kernel<8, true, pp3pol::NWAVE>), grid, block, 0, st, pa);
    HIPCHK(hipGetLastError());
    return PP3_OK;
  }
#endif
  // per step: the policy launch on the env's obs buffer, then one single-step launch that writes
  // this step's trajectory rows (max_contacts = 16, whose blocks do not fit 16 envs per
  // workgroup; action_repeat > 1, whose wrapper step is `repeat` launches)
  for (int t = 0; t < nsteps; t++) {
    float* act = actions_dev + (size_t)t * e->N * NU;
    if (pp3_policy_act(policy, e->obs, PP3_OBS_DIM * e->H, e->N, act, NU, (void*)st) != PP3_OK)
      return set_err(PP3_ERR_ARG, std::string("pp3_rollout_policy: ") + pp3_policy_last_error());
    const int rc = launch_steps(e, act, 0, 1, reward_dev ? reward_dev + (size_t)t * e->N : nullptr,
                                done_dev ? done_dev + (size_t)t * e->N : nullptr, obs_dev ? obs_dev + (size_t)t * on : nullptr,
                                false, (void*)st);
    if (rc) return rc;
  }
  return PP3_OK;
}

void* pp3_stream(pp3_env_t* e) { return e ? (void*)e->stream : nullptr; }

// completion markers of the host API's asynchronous step (timing disabled: a record is one packet)
int pp3_event_create(pp3_env_t* e, void** out) {
  if (!e || !out) return set_err(PP3_ERR_ARG, "pp3_event_create: null argument");
  HIPCHK(hipSetDevice(e->device));
  hipEvent_t ev;
  HIPCHK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
  *out = (void*)ev;
  return PP3_OK;
}
int pp3_event_record(pp3_env_t* e, void* ev) {
  if (!e || !ev) return set_err(PP3_ERR_ARG, "pp3_event_record: null argument");
  HIPCHK(hipEventRecord((hipEvent_t)ev, e->stream));
  return PP3_OK;
}
int pp3_event_synchronize(void* ev) {
  if (!ev) return set_err(PP3_ERR_ARG, "pp3_event_synchronize: null event");
  HIPCHK(hipEventSynchronize((hipEvent_t)ev));
  return PP3_OK;
}
int pp3_event_destroy(void* ev) {
  if (ev) HIPCHK(hipEventDestroy((hipEvent_t)ev));
  return PP3_OK;
}

int pp3_set_auto_reset(pp3_env_t* e, int32_t episode_length) {
  if (!e) return set_err(PP3_ERR_ARG, "null env");
  HIPCHK(hipSetDevice(e->device));
  if (episode_length > 0 && !e->episode) {
    HIPCHK(hipMalloc(&e->episode, sizeof(float) * (size_t)e->N * PP3_EP_STRIDE));
    HIPCHK(hipMalloc(&e->first_state, sizeof(float) * (size_t)e->N * PP3_FIRST_STRIDE));
    HIPCHK(hipMalloc(&e->first_obs, sizeof(float) * (size_t)e->N * PP3_OBS_DIM * e->H));
    HIPCHK(hipMemsetAsync(e->episode, 0, sizeof(float) * (size_t)e->N * PP3_EP_STRIDE, e->stream));
    // until the next pp3_reset the current state is the "first" state
    HIPCHK(hipMemcpy2DAsync(e->first_state, sizeof(float) * PP3_FIRST_STRIDE, e->state, sizeof(float) * e->stride,
                            sizeof(float) * PP3_FIRST_STRIDE, e->N, hipMemcpyDeviceToDevice, e->stream));
    HIPCHK(hipMemcpyAsync(e->first_obs, e->obs, sizeof(float) * (size_t)e->N * PP3_OBS_DIM * e->H,
                          hipMemcpyDeviceToDevice, e->stream));
  }
  e->episode_length = episode_length > 0 ? episode_length : 0;
  if (e->episode_length == 0) e->action_repeat = 1;
  return PP3_OK;
}

int pp3_set_action_repeat(pp3_env_t* e, int32_t action_repeat) {
  if (!e) return set_err(PP3_ERR_ARG, "null env");
  if (action_repeat < 1) return set_err(PP3_ERR_ARG, "action_repeat must be >= 1");
  if (action_repeat > 1 && e->episode_length <= 0)
    return set_err(PP3_ERR_ARG, "action_repeat > 1 needs auto-reset mode (pp3_set_auto_reset first)");
  e->action_repeat = action_repeat;
  return PP3_OK;
}

int pp3_set_dr(pp3_env_t* e, const float* dr_dev) {
  if (!e) return set_err(PP3_ERR_ARG, "null env");
  HIPCHK(hipSetDevice(e->device));
  if (!dr_dev) { e->dr_on = 0; return PP3_OK; }
  HIPCHK(hipMemcpyAsync(e->dr, dr_dev, (size_t)e->N * PP3_NDR * sizeof(float), hipMemcpyDeviceToDevice, e->stream));
  e->dr_on = 1;
  return PP3_OK;
}

int32_t pp3_terrain_slots(const pp3_env_t* e) { return e ? e->nbox : 0; }

int pp3_set_terrain(pp3_env_t* e, const float* boxes, int32_t n_boxes) {
  if (!e) return set_err(PP3_ERR_ARG, "null env");
  HIPCHK(hipSetDevice(e->device));
  uint64_t ptr = 0;
  if (boxes) {
    if (n_boxes != e->nbox)
      return set_err(PP3_ERR_ARG, "pp3_set_terrain: n_boxes must equal the model's world box-geom count (" +
                                      std::to_string(e->nbox) + ")");
    if (n_boxes == 0) return set_err(PP3_ERR_ARG, "pp3_set_terrain: the model has no box geoms to use as slots");
    const size_t rows = (size_t)(e->N + 1) / 2 * 2;  // even: the kernel indexes by 2 * block + half
    std::vector<TerrainRec> rec(rows * n_boxes);
    memset(rec.data(), 0, rec.size() * sizeof(TerrainRec));
    for (size_t i = 0; i < rows; i++)
      for (int b = 0; b < n_boxes; b++) {
        TerrainRec& r = rec[i * n_boxes + b];
        if (i >= (size_t)e->N) {  // padding row: absent boxes
          r.p[2] = -1e4f;
          continue;
        }
        const float* x = boxes + (i * n_boxes + b) * PP3_TERRAIN_BOX;
        if (!(x[7] > 0 || x[8] > 0 || x[9] > 0)) {  // absent: far below the floor, zero size
          r.p[2] = -1e4f;
          r.R[0] = r.R[4] = r.R[8] = 1.0f;
          continue;
        }
        double q[4] = {x[3], x[4], x[5], x[6]};
        const double qn = sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
        if (!(qn > 0)) return set_err(PP3_ERR_ARG, "pp3_set_terrain: zero quaternion");
        for (int k = 0; k < 4; k++) q[k] /= qn;
        double R[9];
        quat2mat_d(q, R);
        for (int k = 0; k < 3; k++) { r.p[k] = x[k]; r.half[k] = x[7 + k]; }
        for (int k = 0; k < 9; k++) r.R[k] = (float)R[k];
      }
    HIPCHK(hipStreamSynchronize(e->stream));
    if (!e->terrain) HIPCHK(hipMalloc(&e->terrain, rows * n_boxes * sizeof(TerrainRec)));
    HIPCHK(hipMemcpy(e->terrain, rec.data(), rec.size() * sizeof(TerrainRec), hipMemcpyHostToDevice));
    ptr = (uint64_t)(uintptr_t)e->terrain;
  } else {
    HIPCHK(hipStreamSynchronize(e->stream));
  }
  HIPCHK(hipMemcpy((char*)e->dmodel + offsetof(DevModel, terrain), &ptr, sizeof(ptr), hipMemcpyHostToDevice));
  return PP3_OK;
}

int pp3_set_pipeline_output(pp3_env_t* e, int32_t enable) {
  if (!e) return set_err(PP3_ERR_ARG, "null env");
  e->pipe_on = enable ? 1 : 0;
  return PP3_OK;
}

int pp3_physics_step(pp3_env_t* e, const float* ctrl_dev, int32_t nsteps, void* stream) {
  if (!e || !ctrl_dev || nsteps < 0) return set_err(PP3_ERR_ARG, "pp3_physics_step: bad argument");
  HIPCHK(hipSetDevice(e->device));
  PhysArgs a;
  a.m = e->dmodel;
  a.state = e->state;
  a.ctrl = ctrl_dev;
  a.dr = e->dr_on ? e->dr : nullptr;
  a.pipe = e->pipe;
  a.nsteps = nsteps;
  a.N = e->N;
  if (e->nc == 8) hipLaunchKernelGGL(physics_kernel<8>, dim3((e->N + 1) / 2), dim3(WAVE), 0, stream_of(e, stream), a);
  else hipLaunchKernelGGL(physics_kernel<16>, dim3((e->N + 1) / 2), dim3(WAVE), 0, stream_of(e, stream), a);
  HIPCHK(hipGetLastError());
  return PP3_OK;
}

int pp3_field(pp3_env_t* e, int32_t field, void** ptr, int64_t* elems) {
  if (!e || !ptr) return set_err(PP3_ERR_ARG, "null argument");
  int64_t n = 0;
  void* p = nullptr;
  switch (field) {
    case PP3_F_STATE: p = e->state; n = e->stride; break;
    case PP3_F_OBS: p = e->obs; n = (int64_t)PP3_OBS_DIM * e->H; break;
    case PP3_F_REWARD: p = e->reward; n = 1; break;
    case PP3_F_DONE: p = e->done; n = 1; break;
    case PP3_F_METRICS: p = e->metrics; n = PP3_NMETRIC; break;
    case PP3_F_DR: p = e->dr; n = PP3_NDR; break;
    case PP3_F_PIPELINE: p = e->pipe; n = PP3_PIPE_STRIDE; break;
    case PP3_F_ACTION: p = e->action; n = PP3_NU; break;
    case PP3_F_EPISODE: p = e->episode; n = PP3_EP_STRIDE; break;
    case PP3_F_FIRST_STATE: p = e->first_state; n = PP3_FIRST_STRIDE; break;
    case PP3_F_FIRST_OBS: p = e->first_obs; n = (int64_t)PP3_OBS_DIM * e->H; break;
    default: return set_err(PP3_ERR_ARG, "unknown field");
  }
  *ptr = p;
  if (elems) *elems = n;
  return PP3_OK;
}

int pp3_copy_field_to_host(pp3_env_t* e, int32_t field, void* host, size_t bytes) {
  void* p;
  int64_t n;
  int rc = pp3_field(e, field, &p, &n);
  if (rc) return rc;
  if (bytes != (size_t)n * e->N * 4) return set_err(PP3_ERR_ARG, "pp3_copy_field_to_host: size mismatch");
  if (!p) return set_err(PP3_ERR_ARG, "pp3_copy_field_to_host: field not allocated (auto-reset fields need pp3_set_auto_reset)");
  HIPCHK(hipSetDevice(e->device));
  HIPCHK(hipStreamSynchronize(e->stream));
  HIPCHK(hipMemcpy(host, p, bytes, hipMemcpyDeviceToHost));
  return PP3_OK;
}

int pp3_copy_field_from_host(pp3_env_t* e, int32_t field, const void* host, size_t bytes) {
  void* p;
  int64_t n;
  int rc = pp3_field(e, field, &p, &n);
  if (rc) return rc;
  if (bytes != (size_t)n * e->N * 4) return set_err(PP3_ERR_ARG, "pp3_copy_field_from_host: size mismatch");
  if (!p) return set_err(PP3_ERR_ARG, "pp3_copy_field_from_host: field not allocated (auto-reset fields need pp3_set_auto_reset)");
  HIPCHK(hipSetDevice(e->device));
  HIPCHK(hipStreamSynchronize(e->stream));
  HIPCHK(hipMemcpy(p, host, bytes, hipMemcpyHostToDevice));
  if (field == PP3_F_DR) e->dr_on = 1;
  return PP3_OK;
}

int pp3_synchronize(pp3_env_t* e) {
  if (!e) return set_err(PP3_ERR_ARG, "null env");
  HIPCHK(hipSetDevice(e->device));
  HIPCHK(hipStreamSynchronize(e->stream));
  HIPCHK(hipDeviceSynchronize());
  return PP3_OK;
}

int pp3_copy_field_to_host_async(pp3_env_t* e, int32_t field, void* host, size_t bytes) {
  void* p;
  int64_t n;
  int rc = pp3_field(e, field, &p, &n);
  if (rc) return rc;
  if (bytes != (size_t)n * e->N * 4) return set_err(PP3_ERR_ARG, "pp3_copy_field_to_host_async: size mismatch");
  if (!p) return set_err(PP3_ERR_ARG, "pp3_copy_field_to_host_async: field not allocated");
  HIPCHK(hipSetDevice(e->device));
  HIPCHK(hipMemcpyAsync(host, p, bytes, hipMemcpyDeviceToHost, e->stream));
  return PP3_OK;
}

// obs | reward | done -> one page-locked host block, stored by the CUs through its device mapping
// (PCIe writes from the kernel; a copy-engine transfer of the same 1.2 MB measured slower)
__global__ void outputs_to_host_kernel(const float* __restrict__ obs, const float* __restrict__ rew,
                                       const float* __restrict__ done, int64_t nobs, int n, float* host) {
  const int64_t total = nobs + 2 * (int64_t)n;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x)
    host[i] = i < nobs ? obs[i] : (i < nobs + n ? rew[i - nobs] : done[i - nobs - n]);
}

int pp3_outputs_to_host(pp3_env_t* e, float* host) {
  if (!e || !host) return set_err(PP3_ERR_ARG, "pp3_outputs_to_host: null argument");
  HIPCHK(hipSetDevice(e->device));
  float* hdev = nullptr;
  if (hipHostGetDevicePointer((void**)&hdev, host, 0) != hipSuccess || !hdev)
    return set_err(PP3_ERR_ARG, "pp3_outputs_to_host: host block is not page-locked memory from pp3_host_malloc");
  const int64_t nobs = (int64_t)e->N * PP3_OBS_DIM * e->H;
  const int64_t total = nobs + 2 * (int64_t)e->N;
  const int blocks = (int)std::min<int64_t>((total + 255) / 256, 1024);
  hipLaunchKernelGGL(outputs_to_host_kernel, dim3(blocks), dim3(256), 0, e->stream, e->obs, e->reward, e->done, nobs,
                     e->N, hdev);
  HIPCHK(hipGetLastError());
  return PP3_OK;
}

int pp3_host_device_ptr(void* host, void** dev) {
  if (!host || !dev) return set_err(PP3_ERR_ARG, "pp3_host_device_ptr: null argument");
  *dev = nullptr;
  if (hipHostGetDevicePointer(dev, host, 0) != hipSuccess || !*dev)
    return set_err(PP3_ERR_ARG, "pp3_host_device_ptr: not page-locked memory from pp3_host_malloc");
  return PP3_OK;
}

int pp3_memcpy_h2d_async(void* dst, const void* src, size_t bytes, void* stream) {
  HIPCHK(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, (hipStream_t)stream));
  return PP3_OK;
}

int pp3_host_malloc(size_t bytes, void** out) {
  if (!out) return set_err(PP3_ERR_ARG, "pp3_host_malloc: null output");
  HIPCHK(hipHostMalloc(out, bytes, hipHostMallocDefault));
  return PP3_OK;
}
int pp3_host_free(void* p) {
  HIPCHK(hipHostFree(p));
  return PP3_OK;
}

int pp3_device_malloc(int32_t device, size_t bytes, void** out) {
  HIPCHK(hipSetDevice(device));
  HIPCHK(hipMalloc(out, bytes));
  return PP3_OK;
}
int pp3_device_free(void* p) {
  HIPCHK(hipFree(p));
  return PP3_OK;
}
int pp3_memcpy_h2d(void* dst, const void* src, size_t bytes) {
  HIPCHK(hipMemcpy(dst, src, bytes, hipMemcpyHostToDevice));
  return PP3_OK;
}
int pp3_memcpy_d2h(void* dst, const void* src, size_t bytes) {
  HIPCHK(hipMemcpy(dst, src, bytes, hipMemcpyDeviceToHost));
  return PP3_OK;
}
int pp3_memcpy_d2d(void* dst, const void* src, size_t bytes, void* stream) {
  HIPCHK(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, (hipStream_t)stream));
  return PP3_OK;
}

int pp3_fill_uniform(pp3_env_t* e, float* dev, int64_t count, uint32_t seed, uint32_t ctr, float lo, float hi, void* stream) {
  if (!e || !dev) return set_err(PP3_ERR_ARG, "null argument");
  HIPCHK(hipSetDevice(e->device));
  const int64_t blocks = (count + 255) / 256;
  hipLaunchKernelGGL(fill_uniform_kernel, dim3((unsigned)blocks), dim3(256), 0, stream_of(e, stream), dev, count, seed, ctr, lo, hi);
  HIPCHK(hipGetLastError());
  return PP3_OK;
}

#ifdef PP3_DEBUG
extern "C" int pp3_debug_read(float* out) {
  HIPCHK(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_dbg), sizeof(float) * 512));
  return PP3_OK;
}
#endif
// prof build: per-wave record of the last env-step launch (WREC words per wave: lifetime cycles,
// dense substeps, max contacts, line-search evaluations, ..., cycles per phase, stamp trace), n waves
int pp3_wave_profile(uint32_t* host_out, int32_t n) {
#ifdef PP3_PHASE_PROF
  if (n > MAXWAVE) n = MAXWAVE;
  HIPCHK(hipDeviceSynchronize());
  HIPCHK(hipMemcpyFromSymbol(host_out, HIP_SYMBOL(g_wave), sizeof(uint32_t) * WREC * n));
  return PP3_OK;
#else
  (void)host_out; (void)n;
  return set_err(PP3_ERR_ARG, "pp3_wave_profile: library built without -DPP3_PHASE_PROF");
#endif
}

int pp3_phase_profile(uint64_t* host_out, int32_t n, int32_t reset) {
#ifdef PP3_PHASE_PROF
  if (n > NPROF) n = NPROF;
  HIPCHK(hipDeviceSynchronize());
  std::vector<unsigned long long> all((size_t)MAXWAVE * NPROF);
  HIPCHK(hipMemcpyFromSymbol(all.data(), HIP_SYMBOL(g_prof), sizeof(unsigned long long) * all.size()));
  unsigned long long sum[NPROF] = {0};
  for (int w = 0; w < MAXWAVE; w++)
    for (int k = 0; k < NPROF; k++) sum[k] += all[(size_t)w * NPROF + k];
  sum[20] += sum[NPROF - 1];  // the second env's evaluations (lane HW + 20)
  sum[NPROF - 1] = 0;
  for (int k = 0; k < n; k++) host_out[k] = sum[k];
  if (reset) {
    std::fill(all.begin(), all.end(), 0ull);
    HIPCHK(hipMemcpyToSymbol(HIP_SYMBOL(g_prof), all.data(), sizeof(unsigned long long) * all.size()));
  }
  return PP3_OK;
#else
  (void)host_out; (void)n; (void)reset;
  return set_err(PP3_ERR_ARG, "pp3_phase_profile: library built without -DPP3_PHASE_PROF");
#endif
}

int pp3_step_timed(pp3_env_t* e, const float* actions_dev, int64_t action_stride, int32_t nsteps,
                   float* kernel_ms_total) {
  if (!e || !actions_dev || !kernel_ms_total) return set_err(PP3_ERR_ARG, "null argument");
  HIPCHK(hipSetDevice(e->device));
  HIPCHK(hipEventRecord(e->ev0, e->stream));
  for (int i = 0; i < nsteps; i++) {
    int rc = pp3_step(e, actions_dev + (size_t)i * (size_t)action_stride, e->stream);
    if (rc) return rc;
  }
  HIPCHK(hipEventRecord(e->ev1, e->stream));
  HIPCHK(hipEventSynchronize(e->ev1));
  HIPCHK(hipEventElapsedTime(kernel_ms_total, e->ev0, e->ev1));
  return PP3_OK;
}

int pp3_rollout_timed(pp3_env_t* e, const float* actions_dev, int64_t action_stride, int32_t nsteps,
                      float* reward_dev, float* done_dev, float* obs_dev, float* kernel_ms_total) {
  if (!e || !actions_dev || !kernel_ms_total) return set_err(PP3_ERR_ARG, "null argument");
  HIPCHK(hipSetDevice(e->device));
  HIPCHK(hipEventRecord(e->ev0, e->stream));
  const int rc = pp3_rollout(e, actions_dev, action_stride, nsteps, reward_dev, done_dev, obs_dev, e->stream);
  if (rc) return rc;
  HIPCHK(hipEventRecord(e->ev1, e->stream));
  HIPCHK(hipEventSynchronize(e->ev1));
  HIPCHK(hipEventElapsedTime(kernel_ms_total, e->ev0, e->ev1));
  return PP3_OK;
}

int pp3_rollout_policy_timed(pp3_env_t* e, pp3_policy_t* policy, int32_t nsteps, float* actions_dev,
                             float* reward_dev, float* done_dev, float* obs_dev, float* kernel_ms_total) {
  if (!e || !policy || !actions_dev || !kernel_ms_total) return set_err(PP3_ERR_ARG, "null argument");
  HIPCHK(hipSetDevice(e->device));
  HIPCHK(hipEventRecord(e->ev0, e->stream));
  const int rc = pp3_rollout_policy(e, policy, nsteps, actions_dev, reward_dev, done_dev, obs_dev, e->stream);
  if (rc) return rc;
  HIPCHK(hipEventRecord(e->ev1, e->stream));
  HIPCHK(hipEventSynchronize(e->ev1));
  HIPCHK(hipEventElapsedTime(kernel_ms_total, e->ev0, e->ev1));
  return PP3_OK;
}

}  // extern "C"
