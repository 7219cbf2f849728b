// pp3_env.hip -- MI355X (gfx950) kernels for the Pupper-v3 environment hot path.
//
// One wavefront (64 lanes) per environment, one environment per workgroup.  The whole
// env step of PupperV3Env.step (environment.py:348-483) runs in ONE launch: RNG/kick/
// latency prologue, n_frames (=5) MuJoCo-semantics physics substeps (kinematics, CRB mass
// matrix, collision, pyramidal contact + frictionloss + limit constraints, RNE, Newton
// solve with exact line search, Euler), then the observation/reward/termination epilogue.
// Per-env state lives in LDS for the whole launch; HBM sees one read and one write of the
// env's state record per env step.  Small dense linear algebra (18x18 LDL^T) runs in
// registers, one matrix row per lane, with v_readlane broadcasts.
#include <hip/hip_runtime.h>

#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <mutex>
#include <string>
#include <vector>

#include "pp3_device.h"

namespace pp3 {

constexpr int STRIDE_MAX = PP3_S_ACT_BUF + 12 * PP3_MAX_LAG + 6 * PP3_MAX_LAG;
constexpr int HMAX = 16;  // observation_history limit
constexpr int OBS_MOVE = (PP3_OBS_DIM * (HMAX - 1) + WAVE - 1) / WAVE;

struct alignas(16) Shared {
  float qpos[20], qvel[20], qws[20], qacc[20], ctrl[12];
  float xpos[NB][3], xquat[NB][4], xmat[NB][9], xipos[NB][3];
  float xanchor[NJ][3], xaxis[NJ][3];
  float com[4];
  float cinert[NB][10];
  float cdof[NV][6];
  float F[NV][6];
  float cvel[NB][6];
  float cfrc[NB][6];  // subtree-accumulated (legs) / own (base) RNE body forces
  float M[NV][NV + 1];
  float L[NV][NV + 1];
  float gxpos[MAX_ROBOT_GEOM][3];
  float site_xpos[PP3_MAX_SITE][3];
  // per-env dynamic parameters (domain randomisation)
  float mass[NB], inertia[NB][3], ipos[NB][3];
  float fric, kp, kd;
  int dr_on;
  // forces / accelerations
  float qfrc_bias[NV], qfrc_smooth[NV], qfrc_act[NV], qacc_smooth[NV], Ma[NV], grad[NV], search[NV], dofD[NV];
  // contacts
  int ncon, nhit;
  int con_pair[NCMAX];
  float con_pos[NCMAX][3], con_frame[NCMAX][9], con_dist[NCMAX], con_mu[NCMAX];
  float con_G[NCMAX][5];
  float Jc[NCMAX][3][NV + 2];
  float hit_dist[WAVE];
  int hit_pair[WAVE];
  // constraint rows
  int nl;
  int lim_dof[NLMAX];
  float lim_sgn[NLMAX];
  float efc_D[NEFC_MAX], efc_R[NEFC_MAX], efc_aref[NEFC_MAX], efc_force[NEFC_MAX];
  // env scratch
  float st[STRIDE_MAX];
  uint32_t keys[8][2];
  float u[40];
  float o[PP3_OBS_DIM];
  float rw[PP3_NREWARD];
  float xdv[NB][3], xda[NB][3];
  int contact[4], filt_mm[4], filt_cm[4];
  float first[4];
  int done;
  float knee, bodyc;
  int li;
};

#define SYNC() __syncthreads()

__device__ __forceinline__ Key key_of(const Shared& s, int i) { return Key{s.keys[i][0], s.keys[i][1]}; }

// ------------------------------------------------------------------------------------
// Phase 1: forward kinematics (mj_kinematics).  Lanes 0..3 each walk base -> leg chain.
// ------------------------------------------------------------------------------------
__device__ void kinematics(Shared& s, const DevModel& m, int lane) {
  if (lane < 4) {
    float bq[4] = {s.qpos[3], s.qpos[4], s.qpos[5], s.qpos[6]};
    normalize4(bq);
    float pp[3] = {s.qpos[0], s.qpos[1], s.qpos[2]};
    float pq[4] = {bq[0], bq[1], bq[2], bq[3]};
    float pR[9];
    quat2mat(pq, pR);
    if (lane == 0) {
      float off[3];
      matvec(off, pR, s.ipos[1]);
      for (int k = 0; k < 3; k++) {
        s.xpos[1][k] = pp[k];
        s.xipos[1][k] = pp[k] + off[k];
        s.xanchor[0][k] = pp[k];
        s.xaxis[0][k] = m.jnt_axis[0][k];
      }
      for (int k = 0; k < 4; k++) s.xquat[1][k] = pq[k];
      for (int k = 0; k < 9; k++) s.xmat[1][k] = pR[k];
    }
#pragma unroll
    for (int k = 0; k < 3; k++) {
      const int b = 2 + 3 * lane + k, j = 1 + 3 * lane + k, qa = 7 + 3 * lane + k;
      float xp[3], xq[4], off[3], R[9], ax[3], an[3], qloc[4], v[3];
      matvec(off, pR, m.body_pos[b]);
      for (int c = 0; c < 3; c++) xp[c] = pp[c] + off[c];
      mulquat(xq, pq, m.body_quat[b]);
      quat2mat(xq, R);
      matvec(ax, R, m.jnt_axis[j]);
      matvec(an, R, m.jnt_pos[j]);
      for (int c = 0; c < 3; c++) an[c] += xp[c];
      axisangle2quat(qloc, m.jnt_axis[j], s.qpos[qa] - m.qpos0[qa]);
      mulquat(xq, xq, qloc);
      quat2mat(xq, R);
      matvec(v, R, m.jnt_pos[j]);
      for (int c = 0; c < 3; c++) xp[c] = an[c] - v[c];
      normalize4(xq);
      quat2mat(xq, R);
      matvec(off, R, s.ipos[b]);
      for (int c = 0; c < 3; c++) {
        s.xpos[b][c] = xp[c];
        s.xipos[b][c] = xp[c] + off[c];
        s.xaxis[j][c] = ax[c];
        s.xanchor[j][c] = an[c];
        pp[c] = xp[c];
      }
      for (int c = 0; c < 4; c++) { s.xquat[b][c] = xq[c]; pq[c] = xq[c]; }
      for (int c = 0; c < 9; c++) { s.xmat[b][c] = R[c]; pR[c] = R[c]; }
    }
  }
}

// ------------------------------------------------------------------------------------
// Phase 2: subtree com, cinert (mju_inertCom), cdof, robot geom and site positions.
// ------------------------------------------------------------------------------------
__device__ void com_pos(Shared& s, const DevModel& m, int lane) {
  float mb = 0, mx = 0, my = 0, mz = 0;
  if (lane >= 1 && lane < NB) {
    mb = s.mass[lane];
    mx = mb * s.xipos[lane][0];
    my = mb * s.xipos[lane][1];
    mz = mb * s.xipos[lane][2];
  }
  mb = wave_sum(mb);
  mx = wave_sum(mx);
  my = wave_sum(my);
  mz = wave_sum(mz);
  float com[3];
  if (mb > MINVAL) { com[0] = mx / mb; com[1] = my / mb; com[2] = mz / mb; }
  else { com[0] = s.xipos[1][0]; com[1] = s.xipos[1][1]; com[2] = s.xipos[1][2]; }
  if (lane == 0) { s.com[0] = com[0]; s.com[1] = com[1]; s.com[2] = com[2]; }
  if (lane >= 1 && lane < NB) {
    const int b = lane;
    float iq[4], R[9];
    mulquat(iq, s.xquat[b], m.body_iquat[b]);
    quat2mat(iq, R);
    const float* I = s.inertia[b];
    float A[3][3];
#pragma unroll
    for (int i = 0; i < 3; i++)
#pragma unroll
      for (int j = 0; j < 3; j++)
        A[i][j] = R[3 * i] * I[0] * R[3 * j] + R[3 * i + 1] * I[1] * R[3 * j + 1] + R[3 * i + 2] * I[2] * R[3 * j + 2];
    float mm = s.mass[b];
    float dx = s.xipos[b][0] - com[0], dy = s.xipos[b][1] - com[1], dz = s.xipos[b][2] - com[2];
    float* r = s.cinert[b];
    r[0] = A[0][0] + mm * (dy * dy + dz * dz);
    r[1] = A[1][1] + mm * (dx * dx + dz * dz);
    r[2] = A[2][2] + mm * (dx * dx + dy * dy);
    r[3] = A[0][1] - mm * dx * dy;
    r[4] = A[0][2] - mm * dx * dz;
    r[5] = A[1][2] - mm * dy * dz;
    r[6] = mm * dx; r[7] = mm * dy; r[8] = mm * dz;
    r[9] = mm;
  } else if (lane >= 14 && lane < 14 + NV) {
    const int d = lane - 14;
    float* cd = s.cdof[d];
    if (d < 3) {
      for (int k = 0; k < 6; k++) cd[k] = 0;
      cd[3 + d] = 1;
    } else {
      float ax[3], off[3], c[3];
      int j;
      if (d < 6) {
        ax[0] = s.xmat[1][d - 3]; ax[1] = s.xmat[1][3 + d - 3]; ax[2] = s.xmat[1][6 + d - 3];
        j = 0;
      } else {
        j = d - 5;
        ax[0] = s.xaxis[j][0]; ax[1] = s.xaxis[j][1]; ax[2] = s.xaxis[j][2];
      }
      for (int k = 0; k < 3; k++) off[k] = com[k] - s.xanchor[j][k];
      cross3(c, ax, off);
      for (int k = 0; k < 3; k++) { cd[k] = ax[k]; cd[3 + k] = c[k]; }
    }
  } else if (lane >= 32 && lane < 32 + m.nrobot_geom) {
    const int g = m.robot_geom[lane - 32], b = m.cg_body[g];
    float off[3];
    matvec(off, s.xmat[b], m.cg_pos[g]);
    for (int k = 0; k < 3; k++) s.gxpos[lane - 32][k] = s.xpos[b][k] + off[k];
  } else if (lane >= 48 && lane < 48 + m.nsite) {
    const int si = lane - 48, b = m.site_body[si];
    float off[3];
    matvec(off, s.xmat[b], m.site_pos[si]);
    for (int k = 0; k < 3; k++) s.site_xpos[si][k] = s.xpos[b][k] + off[k];
  }
}

// geometry of collidable geom g in this env
__device__ __forceinline__ void geom_pose(const Shared& s, const DevModel& m, int g, float p[3], const float** R) {
  const int slot = m.cg_slot[g];
  if (slot >= 0) {
    p[0] = s.gxpos[slot][0]; p[1] = s.gxpos[slot][1]; p[2] = s.gxpos[slot][2];
    *R = s.xmat[m.cg_body[g]];  // sphere orientation is irrelevant; body frame is fine
  } else {
    p[0] = m.cg_pos[g][0]; p[1] = m.cg_pos[g][1]; p[2] = m.cg_pos[g][2];
    *R = m.cg_wmat[g];
  }
}

__device__ __forceinline__ void make_frame(float f[9], const float nin[3]) {
  float a[3] = {nin[0], nin[1], nin[2]};
  float n = sqrtf(dot3(a, a));
  if (n < MINVAL) { a[0] = 1; a[1] = 0; a[2] = 0; } else { a[0] /= n; a[1] /= n; a[2] /= n; }
  float y[3] = {0, 0, 0};
  if (a[1] < 0.5f && a[1] > -0.5f) y[1] = 1; else y[2] = 1;
  float ad = dot3(a, y);
  for (int k = 0; k < 3; k++) y[k] -= a[k] * ad;
  float yn = sqrtf(dot3(y, y));
  if (yn < MINVAL) { y[0] = 1; y[1] = 0; y[2] = 0; } else { y[0] /= yn; y[1] /= yn; y[2] /= yn; }
  float z[3];
  cross3(z, a, y);
  for (int k = 0; k < 3; k++) { f[k] = a[k]; f[3 + k] = y[k]; f[6 + k] = z[k]; }
}

// narrow phase for pair p; returns hit and fills dist/pos/normal
__device__ bool narrow(const Shared& s, const DevModel& m, int p, float& dist, float pos[3], float nrm[3]) {
  const int g1 = m.pair_g1[p], g2 = m.pair_g2[p];
  const int t1 = m.cg_type[g1], t2 = m.cg_type[g2];
  const float margin = m.pair_margin[p];
  float p1[3], p2[3];
  const float *R1, *R2;
  geom_pose(s, m, g1, p1, &R1);
  geom_pose(s, m, g2, p2, &R2);
  if (t1 == PP3_GEOM_PLANE && t2 == PP3_GEOM_SPHERE) {
    float nz[3] = {R1[2], R1[5], R1[8]};
    float v[3] = {p2[0] - p1[0], p2[1] - p1[1], p2[2] - p1[2]};
    float r = m.cg_size[g2][0];
    dist = dot3(nz, v) - r;
    if (dist > margin) return false;
    for (int k = 0; k < 3; k++) { nrm[k] = nz[k]; pos[k] = p2[k] - nz[k] * (r + 0.5f * dist); }
    return true;
  }
  if (t1 == PP3_GEOM_SPHERE && t2 == PP3_GEOM_SPHERE) {
    float v[3] = {p2[0] - p1[0], p2[1] - p1[1], p2[2] - p1[2]};
    float r1 = m.cg_size[g1][0], r2 = m.cg_size[g2][0];
    float len = sqrtf(dot3(v, v));
    dist = len - r1 - r2;
    if (dist > margin) return false;
    if (len < MINVAL) { nrm[0] = 1; nrm[1] = 0; nrm[2] = 0; }
    else { float il = 1.0f / len; nrm[0] = v[0] * il; nrm[1] = v[1] * il; nrm[2] = v[2] * il; }
    for (int k = 0; k < 3; k++) pos[k] = p1[k] + nrm[k] * (r1 + 0.5f * dist);
    return true;
  }
  if (t1 == PP3_GEOM_SPHERE && t2 == PP3_GEOM_BOX) {
    const float* h = m.cg_size[g2];
    float r = m.cg_size[g1][0];
    float rel[3] = {p1[0] - p2[0], p1[1] - p2[1], p1[2] - p2[2]}, dl[3], cl[3];
    for (int k = 0; k < 3; k++) dl[k] = R2[k] * rel[0] + R2[3 + k] * rel[1] + R2[6 + k] * rel[2];
    bool inside = true;
    for (int k = 0; k < 3; k++) {
      cl[k] = dl[k];
      if (cl[k] > h[k]) { cl[k] = h[k]; inside = false; }
      if (cl[k] < -h[k]) { cl[k] = -h[k]; inside = false; }
    }
    float nl[3], dd;
    if (!inside) {
      float v[3] = {cl[0] - dl[0], cl[1] - dl[1], cl[2] - dl[2]};
      float len = sqrtf(dot3(v, v));
      dd = len - r;
      if (dd > margin) return false;
      if (len < MINVAL) { nl[0] = 0; nl[1] = 0; nl[2] = -1; }
      else { for (int k = 0; k < 3; k++) nl[k] = v[k] / len; }
    } else {
      int ax = 0;
      float best = h[0] - fabsf(dl[0]);
      for (int k = 1; k < 3; k++) {
        float t = h[k] - fabsf(dl[k]);
        if (t < best) { best = t; ax = k; }
      }
      nl[0] = nl[1] = nl[2] = 0;
      nl[ax] = dl[ax] >= 0 ? -1.0f : 1.0f;
      dd = -best - r;
    }
    matvec(nrm, R2, nl);
    dist = dd;
    for (int k = 0; k < 3; k++) pos[k] = p1[k] + nrm[k] * (r + 0.5f * dd);
    return true;
  }
  return false;
}

__device__ __forceinline__ void store_contact(Shared& s, const DevModel& m, int slot, int p, float dist,
                                              const float pos[3], const float nrm[3]) {
  s.con_pair[slot] = p;
  s.con_dist[slot] = dist;
  for (int k = 0; k < 3; k++) s.con_pos[slot][k] = pos[k];
  make_frame(s.con_frame[slot], nrm);
  s.con_mu[slot] = s.dr_on ? s.fric : m.pair_mu[p];
}

// Phase 3a: collision (mj_collision), contacts compacted in pair order; when more than
// NCMAX pairs penetrate, the NCMAX deepest are kept (same rule as the oracle).
__device__ void collision(Shared& s, const DevModel& m, int lane) {
  int nhit = 0;
  for (int base = 0; base < m.npair; base += WAVE) {
    const int p = base + lane;
    float dist = 0, pos[3], nrm[3];
    bool hit = (p < m.npair) && narrow(s, m, p, dist, pos, nrm);
    const uint64_t mask = __ballot(hit);
    const int before = __popcll(mask & ((1ull << lane) - 1ull));
    const int slot = nhit + before;
    if (hit) {
      if (slot < NCMAX) store_contact(s, m, slot, p, dist, pos, nrm);
      if (slot < WAVE) { s.hit_dist[slot] = dist; s.hit_pair[slot] = p; }
    }
    nhit += __popcll(mask);
  }
  if (lane == 0) { s.nhit = nhit; s.ncon = nhit < NCMAX ? nhit : NCMAX; }
  if (nhit > NCMAX) {  // rare: keep the NCMAX deepest among the first WAVE hits, in pair order
    SYNC();
    const int nh = nhit < WAVE ? nhit : WAVE;
    float myd = lane < nh ? s.hit_dist[lane] : 0.0f;
    int rank = 0;
    for (int c = 0; c < nh; c++) {
      float dc = s.hit_dist[c];
      rank += (dc < myd || (dc == myd && c < lane)) ? 1 : 0;
    }
    const bool keep = lane < nh && rank < NCMAX;
    const uint64_t km = __ballot(keep);
    const int slot = __popcll(km & ((1ull << lane) - 1ull));
    int p = lane < nh ? s.hit_pair[lane] : 0;
    SYNC();
    if (keep) {
      float dist, pos[3], nrm[3];
      narrow(s, m, p, dist, pos, nrm);
      store_contact(s, m, slot, p, dist, pos, nrm);
    }
  }
}

// RNE leg pass (mj_comVel + mj_rne): lane l in 0..3 walks base then leg l; writes cvel,
// subtree-accumulated leg cfrc and (lane 0) the base's own cfrc.
__device__ void rne_pass(Shared& s, const DevModel& m, int lane) {
  if (lane >= 4) return;
  float cv[6] = {0, 0, 0, 0, 0, 0}, ca[6] = {0, 0, 0, -m.gravity[0], -m.gravity[1], -m.gravity[2]};
  float cdd[6];
  for (int d = 0; d < 3; d++)
    for (int k = 0; k < 6; k++) cv[k] += s.cdof[d][k] * s.qvel[d];
  float cddr[3][6];
  for (int d = 0; d < 3; d++) cross_motion(cddr[d], cv, s.cdof[3 + d]);
  for (int d = 0; d < 3; d++)
    for (int k = 0; k < 6; k++) cv[k] += s.cdof[3 + d][k] * s.qvel[3 + d];
  for (int d = 0; d < 3; d++)
    for (int k = 0; k < 6; k++) ca[k] += cddr[d][k] * s.qvel[3 + d];
  float f1[6], f2[6], f3[6];
  if (lane == 0) {
    mul_inert_vec(f1, s.cinert[1], ca);
    mul_inert_vec(f2, s.cinert[1], cv);
    cross_force(f3, cv, f2);
    for (int k = 0; k < 6; k++) { s.cvel[1][k] = cv[k]; s.cfrc[1][k] = f1[k] + f3[k]; }
  }
  float fb[3][6];
#pragma unroll
  for (int k = 0; k < 3; k++) {
    const int b = 2 + 3 * lane + k, d = 6 + 3 * lane + k;
    cross_motion(cdd, cv, s.cdof[d]);
    const float qd = s.qvel[d];
    for (int c = 0; c < 6; c++) { cv[c] += s.cdof[d][c] * qd; ca[c] += cdd[c] * qd; }
    mul_inert_vec(f1, s.cinert[b], ca);
    mul_inert_vec(f2, s.cinert[b], cv);
    cross_force(f3, cv, f2);
    for (int c = 0; c < 6; c++) { fb[k][c] = f1[c] + f3[c]; s.cvel[b][c] = cv[c]; }
  }
  for (int c = 0; c < 6; c++) {
    fb[1][c] += fb[2][c];
    fb[0][c] += fb[1][c];
  }
#pragma unroll
  for (int k = 0; k < 3; k++)
    for (int c = 0; c < 6; c++) s.cfrc[2 + 3 * lane + k][c] = fb[k][c];
}

// composite inertia of body b's subtree times cdof d (for M), lanes < NV
__device__ void crb_times_cdof(Shared& s, const DevModel& m, int lane) {
  if (lane >= NV) return;
  const int b = m.dof_body[lane];
  float crb[10];
  for (int k = 0; k < 10; k++) crb[k] = 0;
  if (b == 1) {
    for (int bb = 1; bb < NB; bb++)
      for (int k = 0; k < 10; k++) crb[k] += s.cinert[bb][k];
  } else {
    const int last = 2 + 3 * ((b - 2) / 3) + 2;
    for (int bb = b; bb <= last; bb++)
      for (int k = 0; k < 10; k++) crb[k] += s.cinert[bb][k];
  }
  mul_inert_vec(s.F[lane], crb, s.cdof[lane]);
}

// ------------------------------------------------------------------------------------
// register LDL^T: lane i (< NV) holds row i; returns L_ik (k<i) in a[k], D_i in dd
// ------------------------------------------------------------------------------------
__device__ __forceinline__ void ldl_rows(float (&a)[NV], float& dd, int lane) {
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    float dk = fmaxf(rlane(a[k], k), MINVAL);
    dd = (lane == k) ? dk : dd;
    const float lik = a[k] / dk;
#pragma unroll
    for (int j = k + 1; j < NV; ++j) a[j] -= lik * rlane(a[k], j);
    a[k] = (lane > k) ? lik : a[k];
  }
}
// solve L D L^T x = b; x = b_i on entry (lane i).  Uses s.L for the transposed factor.
__device__ __forceinline__ float ldl_solve(Shared& s, const float (&a)[NV], float dd, float x, int lane) {
  const int li = lane < NV ? lane : NV - 1;
#pragma unroll
  for (int k = 0; k < NV; ++k)
    if (k < lane && lane < NV) s.L[lane][k] = a[k];
#pragma unroll
  for (int k = 0; k < NV - 1; ++k) {
    const float yk = rlane(x, k);
    x = (lane > k) ? x - a[k] * yk : x;
  }
  x = x / dd;
  SYNC();
  float col[NV];
#pragma unroll
  for (int k = 0; k < NV; ++k) col[k] = s.L[k][li];
#pragma unroll
  for (int k = NV - 1; k > 0; --k) {
    const float xk = rlane(x, k);
    x = (lane < k) ? x - col[k] * xk : x;
  }
  return x;
}

// J row r dotted with x (LDS vector)
__device__ __forceinline__ float row_dot(const Shared& s, int r, const float* x) {
  if (r < NFR) return x[6 + r];
  if (r < NFR + s.nl) {
    const int i = r - NFR;
    return s.lim_sgn[i] * x[s.lim_dof[i]];
  }
  const int e = r - NFR - s.nl, c = e >> 2, ed = e & 3, t = 1 + (ed >> 1);
  const float sg = (ed & 1) ? -1.0f : 1.0f;
  float a = 0, b = 0;
#pragma unroll
  for (int i = 0; i < NV; i++) { a += s.Jc[c][0][i] * x[i]; b += s.Jc[c][t][i] * x[i]; }
  return a + sg * s.con_mu[c] * b;
}

// ------------------------------------------------------------------------------------
// one physics substep (mj_step): forward + Newton + Euler.  `integrate` = 0 for reset
// (mj_forward only).  Must be called by all 64 lanes.
// ------------------------------------------------------------------------------------
__device__ void substep(Shared& s, const DevModel& m, int lane, bool integrate) {
  kinematics(s, m, lane);
  SYNC();
  com_pos(s, m, lane);
  SYNC();
  // ---- phase 3: CRB*cdof, RNE, collision, actuation/passive, limit rows ----
  crb_times_cdof(s, m, lane);
  rne_pass(s, m, lane);
  collision(s, m, lane);
  {
    // joint limits: lane = 2*(j-1) + side_hi, rows ordered like the oracle
    bool act = false;
    float value = 0;
    int j = 0;
    if (lane < 2 * (NJ - 1)) {
      j = 1 + (lane >> 1);
      const int side = (lane & 1) ? 1 : -1;
      if (m.jnt_limited[j]) {
        value = side * (m.jnt_range[j][(side + 1) / 2] - s.qpos[7 + j - 1]);
        act = value < m.lim_margin[j];
      }
    }
    const uint64_t mask = __ballot(act);
    const int slot = __popcll(mask & ((1ull << lane) - 1ull));
    if (act) {
      const int dof = 6 + j - 1;
      const float sg = (lane & 1) ? -1.0f : 1.0f;  // J = -side
      s.lim_dof[slot] = dof;
      s.lim_sgn[slot] = sg;
      const float imp = getimp(m.lim_solimp[j], value, m.lim_margin[j]);
      const float R = fmaxf(MINVAL, (1.0f - imp) / imp * m.lim_invw[j]);
      const int r = NFR + slot;
      s.efc_R[r] = R;
      s.efc_D[r] = 1.0f / R;
      s.efc_aref[r] = -m.lim_b[j] * (sg * s.qvel[dof]) - m.lim_k[j] * imp * (value - m.lim_margin[j]);
    }
    if (lane == 0) s.nl = __popcll(mask);
    // frictionloss rows
    if (lane < NFR) {
      const int dof = 6 + lane;
      s.efc_R[lane] = m.fr_R[dof];
      s.efc_D[lane] = 1.0f / m.fr_R[dof];
      s.efc_aref[lane] = -m.fr_b[dof] * s.qvel[dof];
    }
    // actuation + passive
    if (lane < NU) {
      const int d = m.act_dof[lane];
      float ctrl = s.ctrl[lane];
      if (m.act_ctrllimited[lane]) ctrl = fminf(fmaxf(ctrl, m.act_crange[lane][0]), m.act_crange[lane][1]);
      const float gear = m.act_gear[lane];
      const float len = gear * s.qpos[m.act_qadr[lane]], vel = gear * s.qvel[d];
      float gain = m.act_gain[lane], b0 = m.act_bias[lane][0], b1 = m.act_bias[lane][1], b2 = m.act_bias[lane][2];
      if (s.dr_on) { gain = s.kp; b1 = -s.kp; b2 = -s.kd; }
      float force = gain * ctrl;
      if (m.act_biastype[lane] == PP3_BIAS_AFFINE) force += b0 + b1 * len + b2 * vel;
      if (m.act_forcelimited[lane]) force = fminf(fmaxf(force, m.act_frange[lane][0]), m.act_frange[lane][1]);
      s.qfrc_act[d] = gear * force;
    }
    if (lane < 6) s.qfrc_act[lane] = 0.0f;
  }
  SYNC();
  // ---- phase 4: M entries, qfrc_bias/smooth, contact Jacobians ----
  for (int p = lane; p < m.nmpair; p += WAVE) {
    const int i = m.mp_i[p], j = m.mp_j[p];
    float v = 0;
    for (int k = 0; k < 6; k++) v += s.cdof[j][k] * s.F[i][k];
    if (i == j) v += m.dof_armature[i];
    s.M[i][j] = v;
    s.M[j][i] = v;
  }
  if (lane < NV) {
    const int b = m.dof_body[lane];
    float cf[6];
    for (int k = 0; k < 6; k++) cf[k] = s.cfrc[b][k];
    if (b == 1)
      for (int l = 0; l < 4; l++)
        for (int k = 0; k < 6; k++) cf[k] += s.cfrc[2 + 3 * l][k];
    float bias = 0;
    for (int k = 0; k < 6; k++) bias += s.cdof[lane][k] * cf[k];
    s.qfrc_bias[lane] = bias;
    s.qfrc_smooth[lane] = -m.dof_damping[lane] * s.qvel[lane] - bias + s.qfrc_act[lane];
  }
  const int ncon = s.ncon;
  for (int it = lane; it < ncon * NV; it += WAVE) {
    const int c = it / NV, i = it - c * NV;
    const int p = s.con_pair[c];
    const int b1 = m.cg_body[m.pair_g1[p]], b2 = m.cg_body[m.pair_g2[p]];
    const uint32_t bit = 1u << i;
    float off[3] = {s.con_pos[c][0] - s.com[0], s.con_pos[c][1] - s.com[1], s.con_pos[c][2] - s.com[2]};
    float jp[3] = {0, 0, 0};
    const float* cd = s.cdof[i];
    float cr[3];
    cross3(cr, cd, off);
    const float w = ((m.body_dofmask[b2] & bit) ? 1.0f : 0.0f) - ((m.body_dofmask[b1] & bit) ? 1.0f : 0.0f);
    for (int k = 0; k < 3; k++) jp[k] = w * (cd[3 + k] + cr[k]);
    const float* fr = s.con_frame[c];
    s.Jc[c][0][i] = fr[0] * jp[0] + fr[1] * jp[1] + fr[2] * jp[2];
    s.Jc[c][1][i] = fr[3] * jp[0] + fr[4] * jp[1] + fr[5] * jp[2];
    s.Jc[c][2][i] = fr[6] * jp[0] + fr[7] * jp[1] + fr[8] * jp[2];
  }
  SYNC();
  // ---- phase 5: contact edge rows (R, D, aref) ----
  const int nl = s.nl;
  const int nefc = NFR + nl + 4 * ncon;
  for (int e = lane; e < 4 * ncon; e += WAVE) {
    const int c = e >> 2, p = s.con_pair[c], r = NFR + nl + e;
    const float mu = s.con_mu[c];
    const float dist = s.con_dist[c];
    const float vel = row_dot(s, r, s.qvel);
    const float tran = m.pair_tran[p];
    const float invw = (tran + mu * mu * tran) * 2.0f * mu * mu / m.impratio;
    const float imp = getimp(m.pair_solimp[p], dist, m.pair_margin[p]);
    const float R = fmaxf(MINVAL, (1.0f - imp) / imp * invw);
    s.efc_R[r] = R;
    s.efc_D[r] = 1.0f / R;
    s.efc_aref[r] = -m.pair_b[p] * vel - m.pair_k[p] * imp * (dist - m.pair_margin[p]);
  }
  // ---- phase 6: qacc_smooth = M^-1 qfrc_smooth (register LDL) ----
  {
    const int li = lane < NV ? lane : NV - 1;
    float a[NV], dd = 1.0f;
#pragma unroll
    for (int j = 0; j < NV; j++) a[j] = s.M[li][j];
    ldl_rows(a, dd, lane);
    const float x = ldl_solve(s, a, dd, s.qfrc_smooth[li], lane);
    if (lane < NV) s.qacc_smooth[lane] = x;
  }
  SYNC();

  // ---- phase 7: Newton solver, 1..iterations, warm-started ----
  // per-lane rows r0 = lane, r1 = lane + 64
  float Dr[2], Rr[2], ar[2], fl[2];
  bool valid[2], isfr[2];
#pragma unroll
  for (int t = 0; t < 2; t++) {
    const int r = lane + WAVE * t;
    valid[t] = r < nefc;
    isfr[t] = r < NFR;
    Dr[t] = valid[t] ? s.efc_D[r] : 0.0f;
    Rr[t] = valid[t] ? s.efc_R[r] : 0.0f;
    ar[t] = valid[t] ? s.efc_aref[r] : 0.0f;
    fl[t] = (valid[t] && isfr[t]) ? m.fr_floss[6 + r] : 0.0f;
  }
  // warm start: cost at qacc_warmstart vs qacc_smooth
  {
    float cws = 0, csm = 0;
#pragma unroll
    for (int t = 0; t < 2; t++) {
      if (!valid[t]) continue;
      const int r = lane + WAVE * t;
      const float x1 = row_dot(s, r, s.qws) - ar[t];
      const float x2 = row_dot(s, r, s.qacc_smooth) - ar[t];
      if (isfr[t]) {
        const float rf = Rr[t] * fl[t];
        cws += (x1 <= -rf) ? (-fl[t] * x1 - 0.5f * rf * fl[t]) : (x1 >= rf) ? (fl[t] * x1 - 0.5f * rf * fl[t]) : 0.5f * Dr[t] * x1 * x1;
        csm += (x2 <= -rf) ? (-fl[t] * x2 - 0.5f * rf * fl[t]) : (x2 >= rf) ? (fl[t] * x2 - 0.5f * rf * fl[t]) : 0.5f * Dr[t] * x2 * x2;
      } else {
        cws += (x1 < 0) ? 0.5f * Dr[t] * x1 * x1 : 0.0f;
        csm += (x2 < 0) ? 0.5f * Dr[t] * x2 * x2 : 0.0f;
      }
    }
    if (lane < NV) {
      float ma = 0;
      for (int j = 0; j < NV; j++) ma += s.M[lane][j] * s.qws[j];
      cws += 0.5f * (ma - s.qfrc_smooth[lane]) * (s.qws[lane] - s.qacc_smooth[lane]);
    }
    cws = wave_sum(cws);
    csm = wave_sum(csm);
    const bool use_smooth = cws > csm;
    if (lane < NV) s.qacc[lane] = use_smooth ? s.qacc_smooth[lane] : s.qws[lane];
  }
  SYNC();
  for (int iter = 0; iter < m.iterations; iter++) {
    // Ma, Jaref, constraint state/force
    float ma = 0;
    if (lane < NV) {
      for (int j = 0; j < NV; j++) ma += s.M[lane][j] * s.qacc[j];
      s.Ma[lane] = ma;
    }
    float jar[2], Dq[2];
#pragma unroll
    for (int t = 0; t < 2; t++) {
      jar[t] = 0;
      Dq[t] = 0;
      if (!valid[t]) continue;
      const int r = lane + WAVE * t;
      const float x = row_dot(s, r, s.qacc) - ar[t];
      jar[t] = x;
      float f;
      if (isfr[t]) {
        const float rf = Rr[t] * fl[t];
        if (x <= -rf) f = fl[t];
        else if (x >= rf) f = -fl[t];
        else { f = -Dr[t] * x; Dq[t] = Dr[t]; }
      } else {
        if (x >= 0) f = 0;
        else { f = -Dr[t] * x; Dq[t] = Dr[t]; }
      }
      s.efc_force[r] = f;
      s.efc_D[r] = Dq[t];  // active D (0 when not quadratic) for the Hessian
    }
    SYNC();
    // gradient, diagonal D per dof, contact Hessian blocks
    float gauss = 0;
    if (lane < NV) {
      float qc = 0;
      if (lane >= 6) qc += s.efc_force[lane - 6];
      float dD = (lane >= 6) ? s.efc_D[lane - 6] : 0.0f;
      for (int i = 0; i < nl; i++)
        if (s.lim_dof[i] == lane) { qc += s.lim_sgn[i] * s.efc_force[NFR + i]; dD += s.efc_D[NFR + i]; }
      for (int c = 0; c < ncon; c++) {
        const int r = NFR + nl + 4 * c;
        const float f0 = s.efc_force[r], f1 = s.efc_force[r + 1], f2 = s.efc_force[r + 2], f3 = s.efc_force[r + 3];
        const float mu = s.con_mu[c];
        qc += s.Jc[c][0][lane] * (f0 + f1 + f2 + f3) + mu * s.Jc[c][1][lane] * (f0 - f1) + mu * s.Jc[c][2][lane] * (f2 - f3);
      }
      s.grad[lane] = ma - s.qfrc_smooth[lane] - qc;
      s.dofD[lane] = dD;
      gauss = 0.5f * (ma - s.qfrc_smooth[lane]) * (s.qacc[lane] - s.qacc_smooth[lane]);
    }
    if (lane >= 32 && lane < 32 + ncon) {
      const int c = lane - 32, r = NFR + nl + 4 * c;
      const float mu = s.con_mu[c];
      const float d0 = s.efc_D[r], d1 = s.efc_D[r + 1], d2 = s.efc_D[r + 2], d3 = s.efc_D[r + 3];
      s.con_G[c][0] = d0 + d1 + d2 + d3;
      s.con_G[c][1] = mu * (d0 - d1);
      s.con_G[c][2] = mu * (d2 - d3);
      s.con_G[c][3] = mu * mu * (d0 + d1);
      s.con_G[c][4] = mu * mu * (d2 + d3);
    }
    gauss = wave_sum(gauss);
    SYNC();
    // Hessian rows H = M + J' D J (registers), LDL^T, search = -H^-1 grad
    {
      const int li = lane < NV ? lane : NV - 1;
      float a[NV], dd = 1.0f;
#pragma unroll
      for (int j = 0; j < NV; j++) a[j] = s.M[li][j];
#pragma unroll
      for (int j = 0; j < NV; j++) a[j] += (j == li) ? s.dofD[li] : 0.0f;
      for (int c = 0; c < ncon; c++) {
        const float* G = s.con_G[c];
        const float jn = s.Jc[c][0][li], j1 = s.Jc[c][1][li], j2 = s.Jc[c][2][li];
        const float w0 = jn * G[0] + j1 * G[1] + j2 * G[2];
        const float w1 = jn * G[1] + j1 * G[3];
        const float w2 = jn * G[2] + j2 * G[4];
#pragma unroll
        for (int j = 0; j < NV; j++) a[j] += w0 * s.Jc[c][0][j] + w1 * s.Jc[c][1][j] + w2 * s.Jc[c][2][j];
      }
      ldl_rows(a, dd, lane);
      const float x = ldl_solve(s, a, dd, s.grad[li], lane);
      if (lane < NV) s.search[lane] = -x;
    }
    SYNC();
    // line-search quadratics
    float q1 = 0, q2 = 0, sn = 0;
    if (lane < NV) {
      const float sv = s.search[lane];
      float mv = 0;
      for (int j = 0; j < NV; j++) mv += s.M[lane][j] * s.search[j];
      q1 = sv * (s.Ma[lane] - s.qfrc_smooth[lane]);
      q2 = 0.5f * sv * mv;
      sn = sv * sv;
    }
    q1 = wave_sum(q1);
    q2 = wave_sum(q2);
    sn = sqrtf(wave_sum(sn));
    if (sn < MINVAL) break;
    float jv[2];
#pragma unroll
    for (int t = 0; t < 2; t++) jv[t] = valid[t] ? row_dot(s, lane + WAVE * t, s.search) : 0.0f;
    const float gtol = m.gtol_scale * sn;
    // evaluate cost/derivatives at alpha
    auto eval = [&](float alpha, float& cost, float& d0, float& d1) {
      float t0 = 0, t1 = 0, t2 = 0;
#pragma unroll
      for (int t = 0; t < 2; t++) {
        if (!valid[t]) continue;
        const float x = jar[t] + alpha * jv[t];
        const float D = Dr[t];
        if (isfr[t]) {
          const float rf = Rr[t] * fl[t];
          if (x <= -rf) { t0 += -fl[t] * jar[t] - 0.5f * rf * fl[t]; t1 += -fl[t] * jv[t]; continue; }
          if (x >= rf) { t0 += fl[t] * jar[t] - 0.5f * rf * fl[t]; t1 += fl[t] * jv[t]; continue; }
        } else if (x >= 0) {
          continue;
        }
        t0 += 0.5f * D * jar[t] * jar[t];
        t1 += D * jar[t] * jv[t];
        t2 += 0.5f * D * jv[t] * jv[t];
      }
      t0 = wave_sum(t0) + gauss;
      t1 = wave_sum(t1) + q1;
      t2 = wave_sum(t2) + q2;
      cost = t0 + alpha * t1 + alpha * alpha * t2;
      d0 = t1 + 2.0f * alpha * t2;
      d1 = fmaxf(2.0f * t2, MINVAL);
    };
    int evals = 0;
    const int maxit = m.ls_iterations;
    float alpha;
    {
      float a0 = 0, c0, g0, h0;
      eval(a0, c0, g0, h0);
      evals++;
      float a1 = a0 - g0 / h0, c1, g1, h1;
      eval(a1, c1, g1, h1);
      evals++;
      if (c0 < c1) { a1 = a0; c1 = c0; g1 = g0; h1 = h0; }
      if (fabsf(g1) < gtol) {
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
          if (fabsf(g1) < gtol) { done = true; break; }
        }
        if (done || evals >= maxit) {
          alpha = a1;
        } else {
          // bracket [p2, p1]
          float a2n = a1, c2n = c1, g2n = g1;
          float a1n = a1 - g1 / h1, c1n, g1n, h1n;
          eval(a1n, c1n, g1n, h1n);
          evals++;
          float h2n = h1;
          (void)h2n;
          alpha = c1 < c2 ? a1 : a2;
          bool finished = false;
          while (evals < maxit) {
            const float am = 0.5f * (a1 + a2);
            float cm, gm, hm;
            eval(am, cm, gm, hm);
            evals++;
            float ca[3] = {a1n, a2n, am}, cc[3] = {c1n, c2n, cm}, cg[3] = {g1n, g2n, gm};
            float ch[3] = {h1n, h1, hm};
            int best = -1;
            for (int i = 0; i < 3; i++)
              if (fabsf(cg[i]) < gtol && (best < 0 || cc[i] < cc[best])) best = i;
            if (best >= 0) { alpha = ca[best]; finished = true; break; }
            bool up1 = false, up2 = false;
            for (int i = 0; i < 3; i++) {
              if (g1 * cg[i] > 0 && fabsf(cg[i]) < fabsf(g1)) { a1 = ca[i]; c1 = cc[i]; g1 = cg[i]; h1 = ch[i]; up1 = true; }
              if (g2 * cg[i] > 0 && fabsf(cg[i]) < fabsf(g2)) { a2 = ca[i]; c2 = cc[i]; g2 = cg[i]; h2 = ch[i]; up2 = true; }
            }
            if (!up1 && !up2) break;
            if (up1) { a1n = a1 - g1 / h1; eval(a1n, c1n, g1n, h1n); evals++; }
            if (up2) { float hh; a2n = a2 - g2 / h2; eval(a2n, c2n, g2n, hh); evals++; }
          }
          if (!finished) alpha = c1 < c2 ? a1 : a2;
        }
      }
    }
    if (alpha == 0.0f) break;
    if (lane < NV) s.qacc[lane] += alpha * s.search[lane];
    SYNC();
  }
  if (lane < NV) s.qws[lane] = s.qacc[lane];
  SYNC();
  if (!integrate) return;
  // ---- phase 8: Euler (eulerdamp disabled) ----
  const float h = m.h;
  float vn = 0;
  float w[3] = {0, 0, 0};
  if (lane < NV) vn = s.qvel[lane] + h * s.qacc[lane];
  if (lane == 3)
    for (int k = 0; k < 3; k++) w[k] = s.qvel[3 + k] + h * s.qacc[3 + k];
  SYNC();
  if (lane < NV) s.qvel[lane] = vn;
  if (lane < 3) s.qpos[lane] += h * vn;
  if (lane >= 6 && lane < NV) s.qpos[lane + 1] += h * vn;
  if (lane == 3) {
    float n = sqrtf(dot3(w, w));
    if (n < MINVAL) { w[0] = 1; w[1] = 0; w[2] = 0; } else { w[0] /= n; w[1] /= n; w[2] /= n; }
    float qr[4], q[4] = {s.qpos[3], s.qpos[4], s.qpos[5], s.qpos[6]};
    axisangle2quat(qr, w, h * n);
    normalize4(q);
    mulquat(q, q, qr);
    for (int k = 0; k < 4; k++) s.qpos[3 + k] = q[k];
  }
  SYNC();
}

// ------------------------------------------------------------------------------------
// environment helpers
// ------------------------------------------------------------------------------------
__device__ void load_params(Shared& s, const DevModel& m, const float* dr, int lane) {
  if (lane < NB) {
    const float* src = dr;
    s.mass[lane] = src ? src[PP3_DR_MASS + lane] : m.body_mass[lane];
    for (int k = 0; k < 3; k++) {
      s.inertia[lane][k] = src ? src[PP3_DR_INERTIA + 3 * lane + k] : m.body_inertia[lane][k];
      s.ipos[lane][k] = (src && lane == 1) ? src[PP3_DR_BASE_IPOS + k] : m.body_ipos[lane][k];
    }
  }
  if (lane == 0) {
    s.dr_on = dr != nullptr;
    s.fric = dr ? dr[PP3_DR_FRICTION] : 0.0f;
    s.kp = dr ? dr[PP3_DR_KP] : 0.0f;
    s.kd = dr ? dr[PP3_DR_KD] : 0.0f;
  }
  // zero M once (its sparsity pattern is fixed)
  for (int i = lane; i < NV * (NV + 1); i += WAVE) (&s.M[0][0])[i] = 0.0f;
}

// sample_command (environment.py:246-272): uses lanes 0..7, writes out[3] in LDS
__device__ void sample_command(Shared& s, const DevModel& m, Key rng, float* out, int lane) {
  const int part = m.partitionable;
  float u = 0;
  if (lane < 3) {
    Key k = split_i(rng, 6, 1 + lane, part);
    const float lo = lane == 0 ? m.cmd_x[0] : lane == 1 ? m.cmd_y[0] : m.cmd_w[0];
    const float hi = lane == 0 ? m.cmd_x[1] : lane == 1 ? m.cmd_y[1] : m.cmd_w[1];
    u = uniform_i(k, 1, 0, lo, hi, part);
  } else if (lane == 3) {
    Key k = split_i(rng, 6, 4, part);
    u = uniform_i(k, 1, 0, 0.0f, 1.0f, part);
  } else if (lane < 7) {
    Key k = split_i(rng, 6, 5, part);
    u = uniform_i(k, 3, lane - 4, -m.stand_thr, m.stand_thr, part);
  }
  const bool zero = rlane(u, 3) < m.zero_cmd_p;
  const float c0 = rlane(u, 0), c1 = rlane(u, 1), c2 = rlane(u, 2);
  const float z0 = rlane(u, 4), z1 = rlane(u, 5), z2 = rlane(u, 6);
  if (lane == 0) {
    out[0] = zero ? z0 : c0;
    out[1] = zero ? z1 : c1;
    out[2] = zero ? z2 : c2;
  }
}

// sample_body_orientation (environment.py:274-298)
__device__ void sample_orientation(Shared& s, const DevModel& m, Key rng, float* out, int lane) {
  const int part = m.partitionable;
  float u = 0;
  if (lane < 2) {
    Key k = split_i(rng, 3, 1 + lane, part);
    u = uniform_i(k, 1, 0, -1.0f, 1.0f, part);
  }
  const float pitch = rlane(u, 0) * m.max_pitch;
  const float roll = rlane(u, 1) * m.max_roll;
  if (lane == 0) {
    const float pi = m.pi_f;
    float v[3] = {roll, pitch, 0.0f};
    float c1 = cosf(v[0] * pi / 360.0f), c2 = cosf(v[1] * pi / 360.0f), c3 = cosf(v[2] * pi / 360.0f);
    float s1 = sinf(v[0] * pi / 360.0f), s2 = sinf(v[1] * pi / 360.0f), s3 = sinf(v[2] * pi / 360.0f);
    float q[4] = {c1 * c2 * c3 - s1 * s2 * s3, s1 * c2 * c3 + c1 * s2 * s3, c1 * s2 * c3 - s1 * c2 * s3,
                  c1 * c2 * s3 + s1 * s2 * c3};
    float r[3];
    b_rotate(r, m.des_z, q);
    out[0] = r[0]; out[1] = r[1]; out[2] = r[2];
  }
}

// _get_obs (environment.py:485-543): consumes st rng, pushes IMU buffer, writes s.o[36]
__device__ void get_obs(Shared& s, const DevModel& m, int lane) {
  const int part = m.partitionable;
  Key rng{__float_as_uint(s.st[PP3_S_RNG]), __float_as_uint(s.st[PP3_S_RNG + 1])};
  if (lane < 6) {
    Key k = split_i(rng, 6, lane, part);
    s.keys[lane][0] = k.a;
    s.keys[lane][1] = k.b;
  }
  SYNC();
  // noise draws: 0-2 ang(k1), 3-5 grav(k2), 6-17 motor(k3), 18-29 last act(k4), 30 imu choice(k5)
  if (lane < 3) s.u[lane] = uniform_i(key_of(s, 1), 3, lane, -1.0f, 1.0f, part) * m.n_ang;
  else if (lane < 6) s.u[lane] = uniform_i(key_of(s, 2), 3, lane - 3, -1.0f, 1.0f, part) * m.n_grav;
  else if (lane < 18) s.u[lane] = uniform_i(key_of(s, 3), 12, lane - 6, -1.0f, 1.0f, part) * m.n_motor;
  else if (lane < 30) s.u[lane] = uniform_i(key_of(s, 4), 12, lane - 18, -1.0f, 1.0f, part) * m.n_act;
  else if (lane == 30) s.u[30] = uniform_i(key_of(s, 5), 1, 0, 0.0f, 1.0f, part);
  SYNC();
  if (lane == 0) {
    float inv[4] = {1, 0, 0, 0}, angl[3] = {0, 0, 0};
    if (m.use_imu) {
      inv[0] = s.xquat[1][0]; inv[1] = -s.xquat[1][1]; inv[2] = -s.xquat[1][2]; inv[3] = -s.xquat[1][3];
      b_rotate(angl, s.cvel[1], inv);
    }
    float g0[3] = {0, 0, -1}, g[3];
    b_rotate(g, g0, inv);
    for (int k = 0; k < 3; k++) g[k] += s.u[3 + k];
    const float gn = sqrtf(dot3(g, g));
    float imu[6];
    for (int k = 0; k < 3; k++) { imu[k] = angl[k] + s.u[k]; imu[3 + k] = g[k] / gn; }
    const int Li = m.Li;
    float* ib = s.st + m.imu_off;
    for (int r = 0; r < 6; r++) {
      for (int l = Li - 1; l > 0; l--) ib[r * Li + l] = ib[r * Li + l - 1];
      ib[r * Li] = imu[r];
    }
    // jax.random.choice with p (searchsorted left on the f32 cumsum)
    float cum[PP3_MAX_LAG], acc = 0.0f;
    for (int i = 0; i < Li; i++) { acc += m.imu_lat_dist[i]; cum[i] = acc; }
    const float r = cum[Li - 1] * (1.0f - s.u[30]);
    int li = 0;
    while (li < Li && cum[li] < r) li++;
    for (int k = 0; k < 6; k++) s.o[k] = fminf(fmaxf(ib[k * Li + li], -100.0f), 100.0f);
    s.st[PP3_S_RNG] = __uint_as_float(s.keys[0][0]);
    s.st[PP3_S_RNG + 1] = __uint_as_float(s.keys[0][1]);
  }
  if (lane < 3) {
    s.o[6 + lane] = fminf(fmaxf(s.st[PP3_S_COMMAND + lane], -100.0f), 100.0f);
    s.o[9 + lane] = fminf(fmaxf(s.st[PP3_S_DESIRED_Z + lane], -100.0f), 100.0f);
  }
  if (lane < 12) {
    const float a = s.qpos[7 + lane] - m.default_pose[lane] + s.u[6 + lane];
    const float b = s.st[PP3_S_LAST_ACT + lane] + s.u[18 + lane];
    s.o[12 + lane] = fminf(fmaxf(a, -100.0f), 100.0f);
    s.o[24 + lane] = fminf(fmaxf(b, -100.0f), 100.0f);
  }
  SYNC();
}

__device__ void write_obs(Shared& s, const DevModel& m, const float* obs_in, float* obs_out, int lane) {
  const int H = m.H;
  const int nmove = PP3_OBS_DIM * (H - 1);
  float tmp[OBS_MOVE];
#pragma unroll
  for (int t = 0; t < OBS_MOVE; t++) {
    const int k = lane + WAVE * t;
    tmp[t] = (k < nmove && obs_in) ? obs_in[k] : 0.0f;
  }
  SYNC();
#pragma unroll
  for (int t = 0; t < OBS_MOVE; t++) {
    const int k = lane + WAVE * t;
    if (k < nmove) obs_out[PP3_OBS_DIM + k] = tmp[t];
  }
  if (lane < PP3_OBS_DIM) obs_out[lane] = s.o[lane];
}

__device__ void write_pipeline(Shared& s, const DevModel& m, float* p, int lane) {
  for (int i = lane; i < PP3_PIPE_STRIDE; i += WAVE) {
    float v = 0.0f;
    if (i < PP3_P_XQUAT) { int b = 1 + i / 3, k = i % 3; v = s.xpos[b][k]; }
    else if (i < PP3_P_XD_VEL) { int q = i - PP3_P_XQUAT, b = 1 + q / 4, k = q % 4; v = s.xquat[b][k]; }
    else if (i < PP3_P_XD_ANG) {
      int q = i - PP3_P_XD_VEL, b = 1 + q / 3, k = q % 3;
      float off[3] = {s.xpos[b][0] - s.com[0], s.xpos[b][1] - s.com[1], s.xpos[b][2] - s.com[2]}, cr[3];
      cross3(cr, s.cvel[b], off);
      v = s.cvel[b][3 + k] + cr[k];
    } else if (i < PP3_P_SITE_XPOS) { int q = i - PP3_P_XD_ANG, b = 1 + q / 3, k = q % 3; v = s.cvel[b][k]; }
    else if (i < PP3_P_QFRC_ACT) { int q = i - PP3_P_SITE_XPOS, f = q / 3, k = q % 3; v = s.site_xpos[m.feet_site[f]][k]; }
    else if (i < PP3_P_QACC) v = s.qfrc_act[i - PP3_P_QFRC_ACT];
    else if (i < PP3_P_NCON) v = s.qacc[i - PP3_P_QACC];
    else if (i == PP3_P_NCON) v = (float)s.ncon;
    else if (i < PP3_P_CON_GEOM) { int c = i - PP3_P_CON_DIST; v = c < s.ncon ? s.con_dist[c] : 0.0f; }
    else if (i < PP3_P_SUBTREE_COM) {
      int q = i - PP3_P_CON_GEOM, c = q / 2;
      if (c < s.ncon) { int pp = s.con_pair[c]; v = (float)m.cg_id[(q & 1) ? m.pair_g2[pp] : m.pair_g1[pp]]; }
    } else if (i < PP3_P_SUBTREE_COM + 3) v = s.com[i - PP3_P_SUBTREE_COM];
    p[i] = v;
  }
}

// ------------------------------------------------------------------------------------
// kernels
// ------------------------------------------------------------------------------------
struct StepArgs {
  const DevModel* m;
  float* state;      // [N][stride]
  const float* obs_in;
  float* obs_out;    // [N][36H]
  const float* actions;  // [N][12]
  float* reward;
  float* done;
  float* metrics;    // [N][19]
  const float* dr;   // [N][62] or null
  float* pipe;       // [N][PIPE] or null
  int N;
};

__global__ __launch_bounds__(WAVE) void env_step_kernel(StepArgs a) {
  __shared__ Shared s;
  const int env = blockIdx.x;
  const int lane = threadIdx.x;
  if (env >= a.N) return;
  const DevModel& m = *a.m;
  const int stride = m.stride;
  const int part = m.partitionable;
  float* gst = a.state + (size_t)env * stride;
  for (int i = lane; i < stride; i += WAVE) s.st[i] = gst[i];
  load_params(s, m, a.dr ? a.dr + (size_t)env * PP3_NDR : nullptr, lane);
  SYNC();
  if (lane < NQ) s.qpos[lane] = s.st[PP3_S_QPOS + lane];
  if (lane < NV) { s.qvel[lane] = s.st[PP3_S_QVEL + lane]; s.qws[lane] = s.st[PP3_S_QACC_WS + lane]; }
  // ---- prologue: rng split, kick, action latency ----
  Key rng{__float_as_uint(s.st[PP3_S_RNG]), __float_as_uint(s.st[PP3_S_RNG + 1])};
  if (lane < 5) {
    Key k = split_i(rng, 5, lane, part);
    s.keys[lane][0] = k.a;
    s.keys[lane][1] = k.b;
  }
  SYNC();
  float u = 0;
  if (lane < 2) u = uniform_i(key_of(s, 2), 2, lane, -1.0f, 1.0f, part);
  else if (lane < 4) u = uniform_i(key_of(s, lane == 2 ? 3 : 4), 1, 0, 0.0f, 1.0f, part);
  const float bern = rlane(u, 2) < m.kick_p ? 1.0f : 0.0f;
  const float kick0 = rlane(u, 0) * m.kick_vel * bern, kick1 = rlane(u, 1) * m.kick_vel * bern;
  const Key cmd_key = key_of(s, 1);
  if (lane == 0) {
    s.qvel[0] += kick0;
    s.qvel[1] += kick1;
    s.st[PP3_S_KICK] = kick0;
    s.st[PP3_S_KICK + 1] = kick1;
    s.st[PP3_S_RNG] = __uint_as_float(s.keys[0][0]);
    s.st[PP3_S_RNG + 1] = __uint_as_float(s.keys[0][1]);
  }
  {
    float cum[PP3_MAX_LAG], acc = 0.0f;
    const int La = m.La;
    for (int i = 0; i < La; i++) { acc += m.lat_dist[i]; cum[i] = acc; }
    const float r = cum[La - 1] * (1.0f - rlane(u, 3));
    int li = 0;
    while (li < La && cum[li] < r) li++;
    if (lane < NU) {
      const float act = a.actions[(size_t)env * NU + lane];
      float* ab = s.st + PP3_S_ACT_BUF + lane * La;
      for (int l = La - 1; l > 0; l--) ab[l] = ab[l - 1];
      ab[0] = act;
      const float t = m.default_pose[lane] + ab[li] * m.action_scale;
      s.ctrl[lane] = fminf(fmaxf(t, m.jlo[lane]), m.jhi[lane]);
    }
  }
  SYNC();
  // ---- physics ----
  for (int f = 0; f < m.n_frames; f++) substep(s, m, lane, true);
  if (lane < NQ) s.st[PP3_S_QPOS + lane] = s.qpos[lane];
  if (lane < NV) { s.st[PP3_S_QVEL + lane] = s.qvel[lane]; s.st[PP3_S_QACC_WS + lane] = s.qws[lane]; }
  SYNC();
  // ---- observation ----
  get_obs(s, m, lane);
  write_obs(s, m, a.obs_in + (size_t)env * PP3_OBS_DIM * m.H, a.obs_out + (size_t)env * PP3_OBS_DIM * m.H, lane);
  // ---- brax x/xd, feet, done, collisions ----
  if (lane >= 1 && lane < NB) {
    const int b = lane;
    float off[3] = {s.xpos[b][0] - s.com[0], s.xpos[b][1] - s.com[1], s.xpos[b][2] - s.com[2]}, cr[3];
    cross3(cr, s.cvel[b], off);
    for (int k = 0; k < 3; k++) { s.xdv[b][k] = s.cvel[b][3 + k] + cr[k]; s.xda[b][k] = s.cvel[b][k]; }
  }
  if (lane >= 16 && lane < 20) {
    const int f = lane - 16;
    const float cz = s.site_xpos[m.feet_site[f]][2] - m.foot_radius;
    const int last = s.st[PP3_S_LAST_CONTACT + f] != 0.0f;
    const int c = cz < 1e-3f;
    s.contact[f] = c;
    s.filt_mm[f] = c | last;
    s.filt_cm[f] = (cz < 3e-2f) | last;
    s.first[f] = (s.st[PP3_S_AIR_TIME + f] > 0.0f && (c | last)) ? 1.0f : 0.0f;
    s.st[PP3_S_AIR_TIME + f] += m.dt;
  }
  if (lane == 20) {
    const int tb = m.torso_body;
    float up[3] = {0, 0, 1}, ru[3];
    b_rotate(ru, up, s.xquat[tb]);
    int d = dot3(ru, up) < m.cos_term_angle;
    for (int j = 0; j < 12; j++) {
      if (s.qpos[7 + j] < m.jlo[j]) d = 1;
      if (s.qpos[7 + j] > m.jhi[j]) d = 1;
    }
    if (s.xpos[tb][2] < m.term_z) d = 1;
    s.done = d;
  }
  if (lane == 21) {
    float knee = 0, bodyc = 0;
    for (int k = 0; k < s.ncon; k++) {
      if (!(s.con_dist[k] < 0.0f)) continue;
      const int pp = s.con_pair[k];
      const int ga = m.cg_id[m.pair_g1[pp]], gb = m.cg_id[m.pair_g2[pp]];
      for (int i = 0; i < m.n_knee_geoms; i++) knee += (ga == m.knee_geoms[i] || gb == m.knee_geoms[i]) ? 1.0f : 0.0f;
      for (int i = 0; i < m.n_torso_geoms; i++) bodyc += (ga == m.torso_geoms[i] || gb == m.torso_geoms[i]) ? 1.0f : 0.0f;
    }
    s.knee = knee;
    s.bodyc = bodyc;
  }
  SYNC();
  // ---- rewards (rewards.py), one term per lane ----
  if (lane < PP3_NREWARD) {
    float inv[4] = {s.xquat[1][0], -s.xquat[1][1], -s.xquat[1][2], -s.xquat[1][3]};
    const float cmd0 = s.st[PP3_S_COMMAND], cmd1 = s.st[PP3_S_COMMAND + 1], cmd2 = s.st[PP3_S_COMMAND + 2];
    const float cn = sqrtf(cmd0 * cmd0 + cmd1 * cmd1 + cmd2 * cmd2);
    const float sig = m.sigma;
    float v = 0;
    switch (lane) {
      case PP3_REWARD_TRACKING_LIN_VEL: {
        float lv[3];
        b_rotate(lv, s.xdv[1], inv);
        const float e = (cmd0 - lv[0]) * (cmd0 - lv[0]) + (cmd1 - lv[1]) * (cmd1 - lv[1]);
        v = expf(-e / sig);
      } break;
      case PP3_REWARD_TRACKING_ANG_VEL: {
        float av[3];
        b_rotate(av, s.xda[1], inv);
        v = expf(-(cmd2 - av[2]) * (cmd2 - av[2]) / sig);
      } break;
      case PP3_REWARD_TRACKING_ORIENTATION: {
        float z0[3] = {0, 0, 1}, wz[3];
        b_rotate(wz, z0, inv);
        float e = 0;
        for (int k = 0; k < 3; k++) e += (wz[k] - s.st[PP3_S_DESIRED_Z + k]) * (wz[k] - s.st[PP3_S_DESIRED_Z + k]);
        v = expf(-e / sig);
      } break;
      case PP3_REWARD_LIN_VEL_Z: v = s.xdv[1][2] * s.xdv[1][2]; break;
      case PP3_REWARD_ANG_VEL_XY: v = s.xda[1][0] * s.xda[1][0] + s.xda[1][1] * s.xda[1][1]; break;
      case PP3_REWARD_ORIENTATION: {
        float z0[3] = {0, 0, 1}, ru[3];
        b_rotate(ru, z0, s.xquat[1]);
        v = ru[0] * ru[0] + ru[1] * ru[1];
      } break;
      case PP3_REWARD_TORQUES:
        for (int i = 0; i < NV; i++) v += s.qfrc_act[i] * s.qfrc_act[i];
        break;
      case PP3_REWARD_JOINT_ACCELERATION:
        for (int j = 0; j < 12; j++) {
          const float acc = (s.qvel[6 + j] - s.st[PP3_S_LAST_VEL + j]) / m.env_dt;
          v += acc * acc;
        }
        break;
      case PP3_REWARD_MECHANICAL_WORK:
        for (int j = 0; j < 12; j++) v += fabsf(s.qfrc_act[6 + j] * s.qvel[6 + j]);
        break;
      case PP3_REWARD_ACTION_RATE:
        for (int j = 0; j < 12; j++) {
          const float d = a.actions[(size_t)env * NU + j] - s.st[PP3_S_LAST_ACT + j];
          v += d * d;
        }
        break;
      case PP3_REWARD_STAND_STILL:
        for (int j = 0; j < 12; j++) v += fabsf(s.qpos[7 + j] - m.default_pose[j]);
        v *= (cn < 0.1f) ? 1.0f : 0.0f;
        break;
      case PP3_REWARD_STAND_STILL_JOINT_VELOCITY:
        for (int j = 0; j < 12; j++) v += fabsf(s.qvel[6 + j]);
        v *= (cn < m.stand_thr) ? 1.0f : 0.0f;
        break;
      case PP3_REWARD_ABDUCTION_ANGLE:
        for (int l = 0; l < 4; l++) {
          const float t = s.qpos[7 + 3 * l + 1] - m.des_abd[l];
          v += t * t;
        }
        break;
      case PP3_REWARD_FEET_AIR_TIME:
        for (int f = 0; f < 4; f++) v += (s.st[PP3_S_AIR_TIME + f] - 0.1f) * s.first[f];
        v *= (cn > 0.05f) ? 1.0f : 0.0f;
        break;
      case PP3_REWARD_FOOT_SLIP:
        for (int f = 0; f < 4; f++) {
          const int b = m.lower_leg_body[f];
          const float* sp = s.site_xpos[m.feet_site[f]];
          float off[3] = {sp[0] - s.xpos[b][0], sp[1] - s.xpos[b][1], sp[2] - s.xpos[b][2]}, cr[3];
          cross3(cr, s.xda[b], off);
          const float vx = s.xdv[b][0] + cr[0], vy = s.xdv[b][1] + cr[1];
          v += (vx * vx + vy * vy) * (s.filt_cm[f] ? 1.0f : 0.0f);
        }
        break;
      case PP3_REWARD_TERMINATION:
        v = (s.done && (int)s.st[PP3_S_STEP] < m.term_step) ? 1.0f : 0.0f;
        break;
      case PP3_REWARD_KNEE_COLLISION: v = s.knee; break;
      case PP3_REWARD_BODY_COLLISION: v = s.bodyc; break;
    }
    s.rw[lane] = v * m.scales[lane];
  }
  SYNC();
  // ---- state management (environment.py:448-482) ----
  int stepc = (int)s.st[PP3_S_STEP] + 1;
  const bool resample = stepc > m.resample_step;
  const bool isdone = s.done != 0;
  if (lane == 0) {
    float sum = 0.0f;
    for (int k = 0; k < PP3_NREWARD; k++) sum += s.rw[k];
    const float rew = fminf(fmaxf(sum * m.dt, 0.0f), 10000.0f);
    a.reward[env] = rew;
    a.done[env] = isdone ? 1.0f : 0.0f;
    const int tb = m.torso_body;
    float* met = a.metrics + (size_t)env * PP3_NMETRIC;
    met[0] = sqrtf(s.xpos[tb][0] * s.xpos[tb][0] + s.xpos[tb][1] * s.xpos[tb][1] + s.xpos[tb][2] * s.xpos[tb][2]);
  }
  if (lane < PP3_NREWARD) a.metrics[(size_t)env * PP3_NMETRIC + 1 + lane] = s.rw[lane];
  if (lane < NU) {
    s.st[PP3_S_LAST_ACT + lane] = a.actions[(size_t)env * NU + lane];
    s.st[PP3_S_LAST_VEL + lane] = s.qvel[6 + lane];
  }
  if (lane < 4) {
    if (s.filt_mm[lane]) s.st[PP3_S_AIR_TIME + lane] = 0.0f;
    s.st[PP3_S_LAST_CONTACT + lane] = s.contact[lane] ? 1.0f : 0.0f;
  }
  if (resample) {
    sample_command(s, m, cmd_key, s.st + PP3_S_COMMAND, lane);
    sample_orientation(s, m, cmd_key, s.st + PP3_S_DESIRED_Z, lane);
  }
  if (isdone || resample) stepc = 0;
  if (lane == 0) s.st[PP3_S_STEP] = (float)stepc;
  if (a.pipe) write_pipeline(s, m, a.pipe + (size_t)env * PP3_PIPE_STRIDE, lane);
  SYNC();
  for (int i = lane; i < stride; i += WAVE) gst[i] = s.st[i];
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
  int N;
};

__global__ __launch_bounds__(WAVE) void env_reset_kernel(ResetArgs a) {
  __shared__ Shared s;
  const int env = blockIdx.x;
  const int lane = threadIdx.x;
  if (env >= a.N) return;
  if (a.mask && !a.mask[env]) return;
  const DevModel& m = *a.m;
  const int part = m.partitionable;
  load_params(s, m, a.dr ? a.dr + (size_t)env * PP3_NDR : nullptr, lane);
  for (int i = lane; i < m.stride; i += WAVE) s.st[i] = 0.0f;
  SYNC();
  const Key rng{a.keys[2 * env], a.keys[2 * env + 1]};
  if (lane < 4) {
    Key k = split_i(rng, 4, lane, part);
    s.keys[lane][0] = k.a;
    s.keys[lane][1] = k.b;
  }
  SYNC();
  const Key k0 = key_of(s, 0), kcmd = key_of(s, 1), kori = key_of(s, 2), kpos = key_of(s, 3);
  // randomize_qpos (domain_randomization.py:188-210)
  float u = 0;
  if (lane < 3) {
    Key kp = split_i(kpos, 3, 1, part);
    u = uniform_i(kp, 3, lane, m.start_lo[lane], m.start_hi[lane], part);
  } else if (lane == 3) {
    Key ky = split_i(kpos, 3, 2, part);
    u = uniform_i(ky, 1, 0, -m.pi_f, m.pi_f, part);
  }
  const float yaw = rlane(u, 3);
  if (lane < NQ) {
    float q = m.key_qpos[lane];
    if (lane >= 7) q = m.default_pose[lane - 7];
    if (lane < 3) q = u;
    if (lane == 3) q = cosf(yaw / 2.0f);
    if (lane == 4 || lane == 5) q = 0.0f;
    if (lane == 6) q = sinf(yaw / 2.0f);
    s.qpos[lane] = q;
  }
  if (lane < NV) { s.qvel[lane] = 0.0f; s.qws[lane] = 0.0f; }
  if (lane < NU) s.ctrl[lane] = 0.0f;
  SYNC();
  substep(s, m, lane, false);  // pipeline_init: mjx.forward
  if (lane < NQ) s.st[PP3_S_QPOS + lane] = s.qpos[lane];
  if (lane < NV) { s.st[PP3_S_QVEL + lane] = 0.0f; s.st[PP3_S_QACC_WS + lane] = s.qws[lane]; }
  if (lane == 0) {
    s.st[PP3_S_RNG] = __uint_as_float(k0.a);
    s.st[PP3_S_RNG + 1] = __uint_as_float(k0.b);
  }
  SYNC();
  sample_command(s, m, kcmd, s.st + PP3_S_COMMAND, lane);
  sample_orientation(s, m, kori, s.st + PP3_S_DESIRED_Z, lane);
  if (lane < m.Li) s.st[m.imu_off + 5 * m.Li + lane] = -1.0f;
  SYNC();
  get_obs(s, m, lane);
  write_obs(s, m, nullptr, a.obs + (size_t)env * PP3_OBS_DIM * m.H, lane);
  if (lane == 0) { a.reward[env] = 0.0f; a.done[env] = 0.0f; }
  if (lane < PP3_NMETRIC) a.metrics[(size_t)env * PP3_NMETRIC + lane] = 0.0f;
  if (a.pipe) write_pipeline(s, m, a.pipe + (size_t)env * PP3_PIPE_STRIDE, lane);
  SYNC();
  float* gst = a.state + (size_t)env * m.stride;
  for (int i = lane; i < m.stride; i += WAVE) gst[i] = s.st[i];
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

__global__ __launch_bounds__(WAVE) void physics_kernel(PhysArgs a) {
  __shared__ Shared s;
  const int env = blockIdx.x;
  const int lane = threadIdx.x;
  if (env >= a.N) return;
  const DevModel& m = *a.m;
  float* gst = a.state + (size_t)env * m.stride;
  load_params(s, m, a.dr ? a.dr + (size_t)env * PP3_NDR : nullptr, lane);
  if (lane < NQ) s.qpos[lane] = gst[PP3_S_QPOS + lane];
  if (lane < NV) { s.qvel[lane] = gst[PP3_S_QVEL + lane]; s.qws[lane] = gst[PP3_S_QACC_WS + lane]; }
  if (lane < NU) s.ctrl[lane] = a.ctrl[(size_t)env * NU + lane];
  SYNC();
  for (int i = 0; i < a.nsteps; i++) substep(s, m, lane, true);
  if (a.pipe) write_pipeline(s, m, a.pipe + (size_t)env * PP3_PIPE_STRIDE, lane);
  if (lane < NQ) gst[PP3_S_QPOS + lane] = s.qpos[lane];
  if (lane < NV) { gst[PP3_S_QVEL + lane] = s.qvel[lane]; gst[PP3_S_QACC_WS + lane] = s.qws[lane]; }
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
  float* obs[2];
  int obs_cur;
  float* reward;
  float* done;
  float* metrics;
  float* dr;
  int dr_on;
  float* pipe;
  int pipe_on;
  float* action;
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
  // collision geoms
  d->ncgeom = mm->ncgeom;
  int nslot = 0;
  for (int g = 0; g < mm->ncgeom; g++) {
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
      if (nslot >= MAX_ROBOT_GEOM) return set_err(PP3_ERR_MODEL, "too many robot collision geoms");
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
    if (mm->cgeom_margin[g1] != 0 || mm->cgeom_margin[g2] != 0) return set_err(PP3_ERR_MODEL, "nonzero geom margins unsupported");
  }
  d->nsite = mm->nsite;
  for (int s = 0; s < mm->nsite; s++) {
    d->site_body[s] = mm->site_bodyid[s];
    for (int k = 0; k < 3; k++) d->site_pos[s][k] = (float)mm->site_pos[s][k];
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
  for (int f = 0; f < 4; f++) {
    d->feet_site[f] = c->feet_site[f];
    d->lower_leg_body[f] = c->lower_leg_body[f];
    if (c->feet_site[f] < 0 || c->feet_site[f] >= mm->nsite) return set_err(PP3_ERR_ARG, "foot site not found");
  }
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
  return PP3_OK;
}

extern "C" {

int pp3_abi_version(void) { return PP3_ABI_VERSION; }

size_t pp3_struct_size(int which) {
  if (which == 0) return sizeof(pp3_model_t);
  if (which == 1) return sizeof(pp3_env_config_t);
  if (which == 2) return sizeof(DevModel);
  if (which == 3) return sizeof(Shared);
  return 0;
}

const char* pp3_last_error(void) { return g_err.c_str(); }

int pp3_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

int pp3_create(const pp3_model_t* model, const pp3_env_config_t* cfg, int32_t num_envs, int32_t device, pp3_env_t** out) {
  if (!model || !cfg || !out || num_envs < 1) return set_err(PP3_ERR_ARG, "bad arguments to pp3_create");
  DevModel hm;
  int rc = build_devmodel(model, cfg, &hm);
  if (rc) return rc;
  HIPCHK(hipSetDevice(device));
  pp3_env* e = new pp3_env();
  memset(e, 0, sizeof(*e));
  e->device = device;
  e->N = num_envs;
  e->stride = hm.stride;
  e->H = hm.H;
  const size_t N = (size_t)num_envs;
  HIPCHK(hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking));
  HIPCHK(hipMalloc(&e->dmodel, sizeof(DevModel)));
  HIPCHK(hipMemcpy(e->dmodel, &hm, sizeof(DevModel), hipMemcpyHostToDevice));
  HIPCHK(hipMalloc(&e->state, N * e->stride * sizeof(float)));
  HIPCHK(hipMalloc(&e->obs[0], N * PP3_OBS_DIM * e->H * sizeof(float)));
  HIPCHK(hipMalloc(&e->obs[1], N * PP3_OBS_DIM * e->H * sizeof(float)));
  HIPCHK(hipMalloc(&e->reward, N * sizeof(float)));
  HIPCHK(hipMalloc(&e->done, N * sizeof(float)));
  HIPCHK(hipMalloc(&e->metrics, N * PP3_NMETRIC * sizeof(float)));
  HIPCHK(hipMalloc(&e->dr, N * PP3_NDR * sizeof(float)));
  HIPCHK(hipMalloc(&e->pipe, N * PP3_PIPE_STRIDE * sizeof(float)));
  HIPCHK(hipMalloc(&e->action, N * PP3_NU * sizeof(float)));
  HIPCHK(hipMemset(e->state, 0, N * e->stride * sizeof(float)));
  HIPCHK(hipMemset(e->obs[0], 0, N * PP3_OBS_DIM * e->H * sizeof(float)));
  HIPCHK(hipMemset(e->obs[1], 0, N * PP3_OBS_DIM * e->H * sizeof(float)));
  HIPCHK(hipMemset(e->pipe, 0, N * PP3_PIPE_STRIDE * sizeof(float)));
  HIPCHK(hipMemset(e->action, 0, N * PP3_NU * sizeof(float)));
  HIPCHK(hipEventCreate(&e->ev0));
  HIPCHK(hipEventCreate(&e->ev1));
  *out = e;
  return PP3_OK;
}

int pp3_destroy(pp3_env_t* e) {
  if (!e) return PP3_OK;
  (void)hipSetDevice(e->device);
  (void)hipStreamSynchronize(e->stream);
  void* bufs[] = {e->dmodel, e->state, e->obs[0], e->obs[1], e->reward, e->done, e->metrics, e->dr, e->pipe, e->action};
  for (void* b : bufs) (void)hipFree(b);
  (void)hipEventDestroy(e->ev0);
  (void)hipEventDestroy(e->ev1);
  (void)hipStreamDestroy(e->stream);
  delete e;
  return PP3_OK;
}

int32_t pp3_num_envs(const pp3_env_t* e) { return e ? e->N : 0; }
int32_t pp3_state_stride(const pp3_env_t* e) { return e ? e->stride : 0; }

static hipStream_t stream_of(pp3_env_t* e, void* s) { return s ? (hipStream_t)s : e->stream; }

int pp3_reset(pp3_env_t* e, const uint32_t* keys_dev, const uint8_t* mask_dev, void* stream) {
  if (!e || !keys_dev) return set_err(PP3_ERR_ARG, "pp3_reset: null argument");
  HIPCHK(hipSetDevice(e->device));
  ResetArgs a;
  a.m = e->dmodel;
  a.state = e->state;
  a.obs = e->obs[e->obs_cur];
  a.reward = e->reward;
  a.done = e->done;
  a.metrics = e->metrics;
  a.keys = keys_dev;
  a.mask = mask_dev;
  a.dr = e->dr_on ? e->dr : nullptr;
  a.pipe = e->pipe_on ? e->pipe : nullptr;
  a.N = e->N;
  hipLaunchKernelGGL(env_reset_kernel, dim3(e->N), dim3(WAVE), 0, stream_of(e, stream), a);
  HIPCHK(hipGetLastError());
  return PP3_OK;
}

int pp3_step(pp3_env_t* e, const float* actions_dev, void* stream) {
  if (!e || !actions_dev) return set_err(PP3_ERR_ARG, "pp3_step: null argument");
  HIPCHK(hipSetDevice(e->device));
  StepArgs a;
  a.m = e->dmodel;
  a.state = e->state;
  a.obs_in = e->obs[e->obs_cur];
  a.obs_out = e->obs[e->obs_cur ^ 1];
  a.actions = actions_dev;
  a.reward = e->reward;
  a.done = e->done;
  a.metrics = e->metrics;
  a.dr = e->dr_on ? e->dr : nullptr;
  a.pipe = e->pipe_on ? e->pipe : nullptr;
  a.N = e->N;
  hipLaunchKernelGGL(env_step_kernel, dim3(e->N), dim3(WAVE), 0, stream_of(e, stream), a);
  HIPCHK(hipGetLastError());
  e->obs_cur ^= 1;
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
  hipLaunchKernelGGL(physics_kernel, dim3(e->N), dim3(WAVE), 0, stream_of(e, stream), a);
  HIPCHK(hipGetLastError());
  return PP3_OK;
}

int pp3_field(pp3_env_t* e, int32_t field, void** ptr, int64_t* elems) {
  if (!e || !ptr) return set_err(PP3_ERR_ARG, "null argument");
  int64_t n = 0;
  void* p = nullptr;
  switch (field) {
    case PP3_F_STATE: p = e->state; n = e->stride; break;
    case PP3_F_OBS: p = e->obs[e->obs_cur]; n = (int64_t)PP3_OBS_DIM * e->H; break;
    case PP3_F_REWARD: p = e->reward; n = 1; break;
    case PP3_F_DONE: p = e->done; n = 1; break;
    case PP3_F_METRICS: p = e->metrics; n = PP3_NMETRIC; break;
    case PP3_F_DR: p = e->dr; n = PP3_NDR; break;
    case PP3_F_PIPELINE: p = e->pipe; n = PP3_PIPE_STRIDE; break;
    case PP3_F_ACTION: p = e->action; n = PP3_NU; break;
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

}  // extern "C"
