/*
 * pp3_oracle.c -- CPU ORACLE (test infrastructure only; never linked into the product).
 *
 * Plain-C restatement, compiled twice (REAL=double -> liboracle64.so, REAL=float ->
 * liboracle32.so), of the hot path behind PupperV3Env.reset/step:
 *
 *   environment.py:314-346 reset, :348-483 step, :485-543 _get_obs      (reference code)
 *   rewards.py:9-138 reward terms; utils.py:34-69 latency buffers       (reference code)
 *   domain_randomization.py:8-112 per-env parameters                    (reference code)
 *   mj_step for the MJCF features of test_pupper_model.xml              ([ext] mujoco 3.2.7,
 *       not vendored; restated from MuJoCo's documented algorithm:
 *       mj_kinematics, mj_comPos, mj_crb, mj_collision (plane/sphere/box),
 *       mj_makeConstraint (frictionloss, joint limits, pyramidal contacts),
 *       mj_makeImpedance, mj_comVel, mj_passive, mj_rne, mj_fwdActuation,
 *       mj_fwdAcceleration, Newton solver (engine_solver.c PrimalSearch-style line
 *       search), mj_Euler without eulerdamp)
 *   jax.random threefry2x32 / split / uniform / bernoulli / choice      ([ext] jax 0.5.0)
 *
 * PARITY STATUS: the physics restatement is "parity unpinned" against MuJoCo itself
 * (mujoco/mujoco_mjx are absent from this container and from the GPU box, and the
 * reference's tests pin no physics values).  The RNG is pinned by the
 * Random123 threefry known-answer vectors, the latency buffers by test_utils.py:54-105,
 * the IMU lag by test_environment.py:136-156 (see tests/).  The physics shared with the
 * kernel is pinned by known answers derived from MuJoCo's documented model without either
 * restatement: M, invweight0, frictionloss, joint limits, resting contacts
 * (tests/test_physics_kat.py), pyramidal friction with impratio (tests/test_friction_kat.py) and
 * the narrow phase's distances, contact sets and sphere-box normals (tests/test_collision_kat.py).
 *
 * This file is algorithm-for-algorithm "textbook" MuJoCo over general tree arrays
 * (dense nv x nv matrices, loops over bodies/dofs/rows); the HIP kernel is an
 * independent, specialised implementation checked against it.
 */
#include <math.h>
#include <stdio.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../include/pupper_hip.h"
#if defined(_OPENMP)
#include <omp.h>
#endif

#ifndef REAL
#define REAL double
#endif
typedef REAL real;

#if defined(ORC_FLOAT)
#define REPS ((real)1.1920929e-7)  /* FLT_EPSILON */
#define RSQRT sqrtf
#define RCOS cosf
#define RSIN sinf
#define REXP expf
#define RFABS fabsf
#define RPOW powf
#else
#define REPS ((real)2.220446049250313e-16)  /* DBL_EPSILON */
#define RSQRT sqrt
#define RCOS cos
#define RSIN sin
#define REXP exp
#define RFABS fabs
#define RPOW pow
#endif

#define NB PP3_NBODY
#define NJ PP3_NJNT
#define NV PP3_NV
#define NQ PP3_NQ
#define NU PP3_NU
#define MINVAL ((real)1e-15)
#define MINIMP ((real)0.0001)
#define MAXIMP ((real)0.9999)
#define ORC_MAXCON 64
#define ORC_MAXEFC (2 * NV + 4 * ORC_MAXCON)

enum { CN_FRICTION = 0, CN_LIMIT = 1, CN_CONTACT = 2 };
enum { ST_SATISFIED = 0, ST_QUADRATIC = 1, ST_LINNEG = 2, ST_LINPOS = 3 };

/* ================================ RNG (jax) ================================ */
static uint32_t rotl32(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }

void orc_threefry2x32(uint32_t k0, uint32_t k1, uint32_t x0, uint32_t x1, uint32_t out[2]) {
  static const int rot[2][4] = {{13, 15, 26, 6}, {17, 29, 16, 24}};
  uint32_t ks[3] = {k0, k1, k0 ^ k1 ^ 0x1BD11BDAu};
  x0 += ks[0];
  x1 += ks[1];
  for (int i = 0; i < 5; i++) {
    for (int j = 0; j < 4; j++) {
      x0 += x1;
      x1 = rotl32(x1, rot[i % 2][j]);
      x1 ^= x0;
    }
    x0 += ks[(i + 1) % 3];
    x1 += ks[(i + 2) % 3] + (uint32_t)(i + 1);
  }
  out[0] = x0;
  out[1] = x1;
}

typedef struct { uint32_t k[2]; } key_t2;

static int g_partitionable = 1;
static _Thread_local double g_dbg[512];
static _Thread_local int g_boundary = 0;  /* near-switch constraint rows seen since the last orc_boundary_take() */
#define BOUNDARY_REL ((real)1e-4)  /* last Newton iteration's intermediates (debugging aid) */
static int g_ncon_max = 0; /* contact cap shared with the HIP kernel: 0 = default 8 */

/* jax.random.split(key, n)[i] */
static key_t2 split_i(key_t2 key, int n, int i) {
  key_t2 r;
  uint32_t o[2];
  if (g_partitionable) {
    orc_threefry2x32(key.k[0], key.k[1], 0u, (uint32_t)i, o);
    r.k[0] = o[0];
    r.k[1] = o[1];
  } else {
    /* original: counts = iota(2n); x0 = counts[:n], x1 = counts[n:]; out = [y0 | y1];
     * key_i = (out[2i], out[2i+1]) */
    for (int w = 0; w < 2; w++) {
      int flat = 2 * i + w;
      int lane = flat % n, half = flat / n;
      orc_threefry2x32(key.k[0], key.k[1], (uint32_t)lane, (uint32_t)(lane + n), o);
      r.k[w] = o[half];
    }
  }
  return r;
}

/* 32-bit random_bits element i of a draw of `count` elements */
static uint32_t bits_i(key_t2 key, int count, int i) {
  uint32_t o[2];
  if (g_partitionable) {
    orc_threefry2x32(key.k[0], key.k[1], 0u, (uint32_t)i, o);
    return o[0] ^ o[1];
  }
  int n = count + (count & 1), h = n / 2;
  int lane = i % h, half = i / h;
  uint32_t c0 = (uint32_t)lane, c1 = (uint32_t)(lane + h);
  if (lane + h >= count) c1 = 0u; /* padded zero */
  orc_threefry2x32(key.k[0], key.k[1], c0, c1, o);
  return o[half];
}

static float unit_f32(uint32_t bits) {
  uint32_t fb = (bits >> 9) | 0x3F800000u;
  float f;
  memcpy(&f, &fb, 4);
  return f - 1.0f;
}

/* jax.random.uniform(key, (count,), minval, maxval)[i] in float32 */
static float uniform_i(key_t2 key, int count, int i, float lo, float hi) {
  float u = unit_f32(bits_i(key, count, i));
  float v = u * (hi - lo) + lo;
  return v > lo ? v : lo;
}

/* jax.random.choice(key, n, p=dist) index (replace=True, shape=()) */
static int choice_idx(key_t2 key, const double* dist, int n) {
  float cum[PP3_MAX_LAG];
  float acc = 0.0f;
  for (int i = 0; i < n; i++) {
    acc += (float)dist[i];
    cum[i] = acc;
  }
  float u = uniform_i(key, 1, 0, 0.0f, 1.0f);
  float r = cum[n - 1] * (1.0f - u);
  int idx = 0;
  while (idx < n && cum[idx] < r) idx++; /* searchsorted side='left' */
  return idx;
}

/* ============================== small math ============================== */
static void quat2mat(const real q[4], real R[9]) {
  real w = q[0], x = q[1], y = q[2], z = q[3];
  R[0] = 1 - 2 * (y * y + z * z); R[1] = 2 * (x * y - w * z); R[2] = 2 * (x * z + w * y);
  R[3] = 2 * (x * y + w * z); R[4] = 1 - 2 * (x * x + z * z); R[5] = 2 * (y * z - w * x);
  R[6] = 2 * (x * z - w * y); R[7] = 2 * (y * z + w * x); R[8] = 1 - 2 * (x * x + y * y);
}
static void mulquat(real r[4], const real a[4], const real b[4]) {
  real t[4];
  t[0] = a[0] * b[0] - a[1] * b[1] - a[2] * b[2] - a[3] * b[3];
  t[1] = a[0] * b[1] + a[1] * b[0] + a[2] * b[3] - a[3] * b[2];
  t[2] = a[0] * b[2] - a[1] * b[3] + a[2] * b[0] + a[3] * b[1];
  t[3] = a[0] * b[3] + a[1] * b[2] - a[2] * b[1] + a[3] * b[0];
  memcpy(r, t, sizeof(t));
}
static void matvec(real r[3], const real R[9], const real v[3]) {
  real t0 = R[0] * v[0] + R[1] * v[1] + R[2] * v[2];
  real t1 = R[3] * v[0] + R[4] * v[1] + R[5] * v[2];
  real t2 = R[6] * v[0] + R[7] * v[1] + R[8] * v[2];
  r[0] = t0; r[1] = t1; r[2] = t2;
}
static void rotvecquat(real r[3], const real v[3], const real q[4]) {
  real R[9];
  quat2mat(q, R);
  matvec(r, R, v);
}
static void cross3(real r[3], const real a[3], const real b[3]) {
  real t0 = a[1] * b[2] - a[2] * b[1];
  real t1 = a[2] * b[0] - a[0] * b[2];
  real t2 = a[0] * b[1] - a[1] * b[0];
  r[0] = t0; r[1] = t1; r[2] = t2;
}
static real dot3(const real a[3], const real b[3]) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }
static real normalize3(real v[3]) {
  real n = RSQRT(dot3(v, v));
  if (n < MINVAL) { v[0] = 1; v[1] = 0; v[2] = 0; }
  else { v[0] /= n; v[1] /= n; v[2] /= n; }
  return n;
}
static void normalize4(real q[4]) {
  real n = RSQRT(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
  if (n < MINVAL) { q[0] = 1; q[1] = q[2] = q[3] = 0; }
  else { for (int i = 0; i < 4; i++) q[i] /= n; }
}
static void axisangle2quat(real r[4], const real axis[3], real angle) {
  if (angle == 0) { r[0] = 1; r[1] = r[2] = r[3] = 0; return; }
  real s = RSIN(angle / 2);
  r[0] = RCOS(angle / 2); r[1] = axis[0] * s; r[2] = axis[1] * s; r[3] = axis[2] * s;
}
/* mju_crossMotion: [w x v_ang ; w x v_lin + vlin x v_ang] */
static void cross_motion(real r[6], const real vel[6], const real v[6]) {
  real t[6];
  t[0] = -vel[2] * v[1] + vel[1] * v[2];
  t[1] = vel[2] * v[0] - vel[0] * v[2];
  t[2] = -vel[1] * v[0] + vel[0] * v[1];
  t[3] = -vel[2] * v[4] + vel[1] * v[5] - vel[5] * v[1] + vel[4] * v[2];
  t[4] = vel[2] * v[3] - vel[0] * v[5] + vel[5] * v[0] - vel[3] * v[2];
  t[5] = -vel[1] * v[3] + vel[0] * v[4] - vel[4] * v[0] + vel[3] * v[1];
  memcpy(r, t, sizeof(t));
}
/* mju_crossForce: [w x f_rot + vlin x f_lin ; w x f_lin] */
static void cross_force(real r[6], const real vel[6], const real f[6]) {
  real t[6];
  t[0] = -vel[2] * f[1] + vel[1] * f[2] - vel[5] * f[4] + vel[4] * f[5];
  t[1] = vel[2] * f[0] - vel[0] * f[2] + vel[5] * f[3] - vel[3] * f[5];
  t[2] = -vel[1] * f[0] + vel[0] * f[1] - vel[4] * f[3] + vel[3] * f[4];
  t[3] = -vel[2] * f[4] + vel[1] * f[5];
  t[4] = vel[2] * f[3] - vel[0] * f[5];
  t[5] = -vel[1] * f[3] + vel[0] * f[4];
  memcpy(r, t, sizeof(t));
}
/* spatial inertia (10-vector, com-frame) times motion vector */
static void mul_inert_vec(real r[6], const real i[10], const real v[6]) {
  r[0] = i[0] * v[0] + i[3] * v[1] + i[4] * v[2] - i[8] * v[4] + i[7] * v[5];
  r[1] = i[3] * v[0] + i[1] * v[1] + i[5] * v[2] + i[8] * v[3] - i[6] * v[5];
  r[2] = i[4] * v[0] + i[5] * v[1] + i[2] * v[2] - i[7] * v[3] + i[6] * v[4];
  r[3] = i[8] * v[1] - i[7] * v[2] + i[9] * v[3];
  r[4] = i[6] * v[2] - i[8] * v[0] + i[9] * v[4];
  r[5] = i[7] * v[0] - i[6] * v[1] + i[9] * v[5];
}
static real dot6(const real a[6], const real b[6]) {
  real s = 0;
  for (int k = 0; k < 6; k++) s += a[k] * b[k];
  return s;
}

/* ============================== model / data ============================== */
typedef struct {
  real timestep, gravity[3], impratio, tolerance, ls_tolerance, meaninertia;
  int iterations, ls_iterations;
  int parent[NB], dofadr[NB], dofnum[NB], jntadr[NB];
  real body_pos[NB][3], body_quat[NB][4], body_ipos[NB][3], body_iquat[NB][4];
  real body_mass[NB], body_inertia[NB][3], body_invweight0[NB][2];
  int jnt_type[NJ], jnt_qposadr[NJ], jnt_dofadr[NJ], jnt_limited[NJ], jnt_bodyid[NJ];
  real jnt_pos[NJ][3], jnt_axis[NJ][3], jnt_range[NJ][2], jnt_margin[NJ], jnt_solref[NJ][2], jnt_solimp[NJ][5];
  int dof_bodyid[NV], dof_parentid[NV];
  real dof_armature[NV], dof_damping[NV], dof_frictionloss[NV], dof_invweight0[NV];
  real dof_solref[NV][2], dof_solimp[NV][5];
  real qpos0[NQ];
  int ncgeom, npair;
  int cg_type[PP3_MAX_CGEOM], cg_body[PP3_MAX_CGEOM], cg_priority[PP3_MAX_CGEOM], cg_id[PP3_MAX_CGEOM];
  real cg_size[PP3_MAX_CGEOM][3], cg_pos[PP3_MAX_CGEOM][3], cg_quat[PP3_MAX_CGEOM][4];
  real cg_friction[PP3_MAX_CGEOM][3], cg_solref[PP3_MAX_CGEOM][2], cg_solimp[PP3_MAX_CGEOM][5];
  real cg_solmix[PP3_MAX_CGEOM], cg_margin[PP3_MAX_CGEOM], cg_gap[PP3_MAX_CGEOM];
  int pair_g1[PP3_MAX_PAIR], pair_g2[PP3_MAX_PAIR];
  int nsite, site_body[PP3_MAX_SITE];
  real site_pos[PP3_MAX_SITE][3], site_quat[PP3_MAX_SITE][4];
  int nsensor, sensor_type[PP3_MAX_SENSOR], sensor_objid[PP3_MAX_SENSOR], sensor_adr[PP3_MAX_SENSOR];
  real sensor_cutoff[PP3_MAX_SENSOR];
  int act_jnt[NU], act_biastype[NU], act_forcelimited[NU], act_ctrllimited[NU];
  real act_gear[NU], act_gain[NU][3], act_bias[NU][3], act_forcerange[NU][2], act_ctrlrange[NU][2];
  int ncon_max;
} Model;

typedef struct {
  int g1, g2;      /* cgeom indices */
  real dist, pos[3], frame[9], mu, solref[2], solimp[5], margin;
} Contact;

typedef struct {
  real qpos[NQ], qvel[NV], qacc_warmstart[NV], ctrl[NU];
  real xpos[NB][3], xquat[NB][4], xmat[NB][9], xipos[NB][3], ximat[NB][9];
  real xanchor[NJ][3], xaxis[NJ][3];
  real gxpos[PP3_MAX_CGEOM][3], gxmat[PP3_MAX_CGEOM][9];
  real site_xpos[PP3_MAX_SITE][3];
  real com[3]; /* subtree_com of the root body */
  real cinert[NB][10], crb[NB][10], cdof[NV][6], cvel[NB][6], cdof_dot[NV][6];
  real M[NV][NV];
  int ncon, ncon_all;
  Contact con[ORC_MAXCON];
  int nefc, nf, nl;
  int efc_type[ORC_MAXEFC], efc_id[ORC_MAXEFC];
  real efc_J[ORC_MAXEFC][NV];
  real efc_pos[ORC_MAXEFC], efc_margin[ORC_MAXEFC], efc_floss[ORC_MAXEFC];
  real efc_R[ORC_MAXEFC], efc_D[ORC_MAXEFC], efc_aref[ORC_MAXEFC];
  real efc_force[ORC_MAXEFC];
  int efc_state[ORC_MAXEFC];
  real qfrc_passive[NV], qfrc_bias[NV], qfrc_actuator[NV], qfrc_smooth[NV];
  real qacc_smooth[NV], qacc[NV], qfrc_constraint[NV];
  int ls_evals; /* diagnostics */
  real sensordata[PP3_MAX_SENSORDATA];
} Data;

static void model_from_abi(Model* M, const pp3_model_t* m, const real* dr) {
  memset(M, 0, sizeof(*M));
  M->timestep = (real)m->timestep;
  for (int k = 0; k < 3; k++) M->gravity[k] = (real)m->gravity[k];
  M->impratio = (real)m->impratio;
  M->tolerance = (real)m->tolerance;
  M->ls_tolerance = (real)m->ls_tolerance;
  M->meaninertia = (real)m->meaninertia;
  M->iterations = m->iterations;
  M->ls_iterations = m->ls_iterations;
  for (int b = 0; b < NB; b++) {
    M->parent[b] = m->body_parentid[b];
    M->dofadr[b] = m->body_dofadr[b];
    M->dofnum[b] = m->body_dofnum[b];
    M->jntadr[b] = m->body_jntadr[b];
    for (int k = 0; k < 3; k++) {
      M->body_pos[b][k] = (real)m->body_pos[b][k];
      M->body_ipos[b][k] = (real)m->body_ipos[b][k];
      M->body_inertia[b][k] = (real)m->body_inertia[b][k];
    }
    for (int k = 0; k < 4; k++) {
      M->body_quat[b][k] = (real)m->body_quat[b][k];
      M->body_iquat[b][k] = (real)m->body_iquat[b][k];
    }
    M->body_mass[b] = (real)m->body_mass[b];
    M->body_invweight0[b][0] = (real)m->body_invweight0[b][0];
    M->body_invweight0[b][1] = (real)m->body_invweight0[b][1];
  }
  for (int j = 0; j < NJ; j++) {
    M->jnt_type[j] = m->jnt_type[j];
    M->jnt_qposadr[j] = m->jnt_qposadr[j];
    M->jnt_dofadr[j] = m->jnt_dofadr[j];
    M->jnt_limited[j] = m->jnt_limited[j];
    M->jnt_bodyid[j] = m->jnt_bodyid[j];
    for (int k = 0; k < 3; k++) {
      M->jnt_pos[j][k] = (real)m->jnt_pos[j][k];
      M->jnt_axis[j][k] = (real)m->jnt_axis[j][k];
    }
    M->jnt_range[j][0] = (real)m->jnt_range[j][0];
    M->jnt_range[j][1] = (real)m->jnt_range[j][1];
    M->jnt_margin[j] = (real)m->jnt_margin[j];
    for (int k = 0; k < 2; k++) M->jnt_solref[j][k] = (real)m->jnt_solref[j][k];
    for (int k = 0; k < 5; k++) M->jnt_solimp[j][k] = (real)m->jnt_solimp[j][k];
  }
  for (int i = 0; i < NV; i++) {
    M->dof_bodyid[i] = m->dof_bodyid[i];
    M->dof_parentid[i] = m->dof_parentid[i];
    M->dof_armature[i] = (real)m->dof_armature[i];
    M->dof_damping[i] = (real)m->dof_damping[i];
    M->dof_frictionloss[i] = (real)m->dof_frictionloss[i];
    M->dof_invweight0[i] = (real)m->dof_invweight0[i];
    for (int k = 0; k < 2; k++) M->dof_solref[i][k] = (real)m->dof_solref[i][k];
    for (int k = 0; k < 5; k++) M->dof_solimp[i][k] = (real)m->dof_solimp[i][k];
  }
  for (int i = 0; i < NQ; i++) M->qpos0[i] = (real)m->qpos0[i];
  M->ncgeom = m->ncgeom;
  for (int g = 0; g < m->ncgeom; g++) {
    M->cg_type[g] = m->cgeom_type[g];
    M->cg_body[g] = m->cgeom_bodyid[g];
    M->cg_priority[g] = m->cgeom_priority[g];
    M->cg_id[g] = m->cgeom_id[g];
    for (int k = 0; k < 3; k++) {
      M->cg_size[g][k] = (real)m->cgeom_size[g][k];
      M->cg_pos[g][k] = (real)m->cgeom_pos[g][k];
      M->cg_friction[g][k] = (real)m->cgeom_friction[g][k];
    }
    for (int k = 0; k < 4; k++) M->cg_quat[g][k] = (real)m->cgeom_quat[g][k];
    for (int k = 0; k < 2; k++) M->cg_solref[g][k] = (real)m->cgeom_solref[g][k];
    for (int k = 0; k < 5; k++) M->cg_solimp[g][k] = (real)m->cgeom_solimp[g][k];
    M->cg_solmix[g] = (real)m->cgeom_solmix[g];
    M->cg_margin[g] = (real)m->cgeom_margin[g];
    M->cg_gap[g] = (real)m->cgeom_gap[g];
  }
  M->npair = m->npair;
  for (int p = 0; p < m->npair; p++) {
    M->pair_g1[p] = m->pair_g1[p];
    M->pair_g2[p] = m->pair_g2[p];
  }
  M->nsite = m->nsite;
  M->nsensor = m->nsensor;
  for (int i = 0; i < m->nsensor; i++) {
    M->sensor_type[i] = m->sensor_type[i];
    M->sensor_objid[i] = m->sensor_objid[i];
    M->sensor_adr[i] = m->sensor_adr[i];
    M->sensor_cutoff[i] = (real)m->sensor_cutoff[i];
  }
  for (int s = 0; s < m->nsite; s++) {
    M->site_body[s] = m->site_bodyid[s];
    for (int k = 0; k < 3; k++) M->site_pos[s][k] = (real)m->site_pos[s][k];
    for (int k = 0; k < 4; k++) M->site_quat[s][k] = (real)m->site_quat[s][k];
  }
  for (int a = 0; a < NU; a++) {
    M->act_jnt[a] = m->actuator_trnid[a];
    M->act_biastype[a] = m->actuator_biastype[a];
    M->act_forcelimited[a] = m->actuator_forcelimited[a];
    M->act_ctrllimited[a] = m->actuator_ctrllimited[a];
    M->act_gear[a] = (real)m->actuator_gear[a];
    for (int k = 0; k < 3; k++) {
      M->act_gain[a][k] = (real)m->actuator_gainprm[a][k];
      M->act_bias[a][k] = (real)m->actuator_biasprm[a][k];
    }
    for (int k = 0; k < 2; k++) {
      M->act_forcerange[a][k] = (real)m->actuator_forcerange[a][k];
      M->act_ctrlrange[a][k] = (real)m->actuator_ctrlrange[a][k];
    }
  }
  M->ncon_max = g_ncon_max > 0 ? g_ncon_max : 8; /* same default cap as the kernel (8 deepest) */
  if (dr) {
    /* domain_randomization.py:21-66: one friction scalar for all geoms, Kp/Kd for all
     * actuators, torso COM shift, elementwise inertia / mass scales (values absolute). */
    for (int g = 0; g < M->ncgeom; g++) M->cg_friction[g][0] = dr[PP3_DR_FRICTION];
    for (int a = 0; a < NU; a++) {
      M->act_gain[a][0] = dr[PP3_DR_KP];
      M->act_bias[a][1] = -dr[PP3_DR_KP];
      M->act_bias[a][2] = -dr[PP3_DR_KD];
    }
    for (int k = 0; k < 3; k++) M->body_ipos[1][k] = dr[PP3_DR_BASE_IPOS + k];
    for (int b = 0; b < NB; b++) {
      for (int k = 0; k < 3; k++) M->body_inertia[b][k] = dr[PP3_DR_INERTIA + 3 * b + k];
      M->body_mass[b] = dr[PP3_DR_MASS + b];
    }
  }
}

/* ============================ mj_kinematics ============================ */
static void kinematics(const Model* m, Data* d) {
  for (int k = 0; k < 3; k++) d->xpos[0][k] = 0;
  d->xquat[0][0] = 1; d->xquat[0][1] = d->xquat[0][2] = d->xquat[0][3] = 0;
  quat2mat(d->xquat[0], d->xmat[0]);
  for (int k = 0; k < 3; k++) d->xipos[0][k] = 0;
  memcpy(d->ximat[0], d->xmat[0], sizeof(d->xmat[0]));
  for (int b = 1; b < NB; b++) {
    int p = m->parent[b];
    int j = m->jntadr[b];
    real xp[3], xq[4];
    if (j >= 0 && m->jnt_type[j] == PP3_JNT_FREE) {
      int a = m->jnt_qposadr[j];
      for (int k = 0; k < 3; k++) xp[k] = d->qpos[a + k];
      for (int k = 0; k < 4; k++) xq[k] = d->qpos[a + 3 + k];
      normalize4(xq);
      for (int k = 0; k < 3; k++) { d->xanchor[j][k] = xp[k]; d->xaxis[j][k] = m->jnt_axis[j][k]; }
    } else {
      real off[3];
      matvec(off, d->xmat[p], m->body_pos[b]);
      for (int k = 0; k < 3; k++) xp[k] = d->xpos[p][k] + off[k];
      mulquat(xq, d->xquat[p], m->body_quat[b]);
      if (j >= 0) { /* single hinge */
        real v[3], qloc[4];
        rotvecquat(d->xaxis[j], m->jnt_axis[j], xq);
        rotvecquat(v, m->jnt_pos[j], xq);
        for (int k = 0; k < 3; k++) d->xanchor[j][k] = v[k] + xp[k];
        int a = m->jnt_qposadr[j];
        axisangle2quat(qloc, m->jnt_axis[j], d->qpos[a] - m->qpos0[a]);
        mulquat(xq, xq, qloc);
        rotvecquat(v, m->jnt_pos[j], xq);
        for (int k = 0; k < 3; k++) xp[k] = d->xanchor[j][k] - v[k];
      }
      normalize4(xq);
    }
    memcpy(d->xpos[b], xp, sizeof(xp));
    memcpy(d->xquat[b], xq, sizeof(xq));
    quat2mat(xq, d->xmat[b]);
    real off[3], iq[4];
    matvec(off, d->xmat[b], m->body_ipos[b]);
    for (int k = 0; k < 3; k++) d->xipos[b][k] = xp[k] + off[k];
    mulquat(iq, xq, m->body_iquat[b]);
    quat2mat(iq, d->ximat[b]);
  }
  for (int g = 0; g < m->ncgeom; g++) {
    int b = m->cg_body[g];
    real off[3], gq[4];
    matvec(off, d->xmat[b], m->cg_pos[g]);
    for (int k = 0; k < 3; k++) d->gxpos[g][k] = d->xpos[b][k] + off[k];
    mulquat(gq, d->xquat[b], m->cg_quat[g]);
    quat2mat(gq, d->gxmat[g]);
  }
  for (int s = 0; s < m->nsite; s++) {
    int b = m->site_body[s];
    real off[3];
    matvec(off, d->xmat[b], m->site_pos[s]);
    for (int k = 0; k < 3; k++) d->site_xpos[s][k] = d->xpos[b][k] + off[k];
  }
}

/* ============================== mj_comPos ============================== */
static void com_pos(const Model* m, Data* d) {
  real mass = 0, c[3] = {0, 0, 0};
  for (int b = 1; b < NB; b++) {
    mass += m->body_mass[b];
    for (int k = 0; k < 3; k++) c[k] += m->body_mass[b] * d->xipos[b][k];
  }
  for (int k = 0; k < 3; k++) d->com[k] = mass > MINVAL ? c[k] / mass : d->xipos[1][k];
  for (int b = 1; b < NB; b++) {
    /* mju_inertCom: rotational inertia about the root subtree com, offset mass*dif */
    const real* R = d->ximat[b];
    const real* I = m->body_inertia[b];
    real mm = m->body_mass[b], dif[3];
    for (int k = 0; k < 3; k++) dif[k] = d->xipos[b][k] - d->com[k];
    real* r = d->cinert[b];
    /* R diag(I) R^T */
    real A[3][3];
    for (int i = 0; i < 3; i++)
      for (int j = 0; j < 3; j++)
        A[i][j] = R[3 * i + 0] * I[0] * R[3 * j + 0] + R[3 * i + 1] * I[1] * R[3 * j + 1] + R[3 * i + 2] * I[2] * R[3 * j + 2];
    r[0] = A[0][0] + mm * (dif[1] * dif[1] + dif[2] * dif[2]);
    r[1] = A[1][1] + mm * (dif[0] * dif[0] + dif[2] * dif[2]);
    r[2] = A[2][2] + mm * (dif[0] * dif[0] + dif[1] * dif[1]);
    r[3] = A[0][1] - mm * dif[0] * dif[1];
    r[4] = A[0][2] - mm * dif[0] * dif[2];
    r[5] = A[1][2] - mm * dif[1] * dif[2];
    r[6] = mm * dif[0]; r[7] = mm * dif[1]; r[8] = mm * dif[2];
    r[9] = mm;
  }
  /* cdof */
  for (int j = 0; j < NJ; j++) {
    int b = m->jnt_bodyid[j], da = m->jnt_dofadr[j];
    real off[3];
    for (int k = 0; k < 3; k++) off[k] = d->com[k] - d->xanchor[j][k];
    if (m->jnt_type[j] == PP3_JNT_FREE) {
      for (int i = 0; i < 3; i++) {
        for (int k = 0; k < 6; k++) d->cdof[da + i][k] = 0;
        d->cdof[da + i][3 + i] = 1;
      }
      for (int i = 0; i < 3; i++) {
        real ax[3] = {d->xmat[b][i], d->xmat[b][3 + i], d->xmat[b][6 + i]};
        real c[3];
        cross3(c, ax, off);
        for (int k = 0; k < 3; k++) { d->cdof[da + 3 + i][k] = ax[k]; d->cdof[da + 3 + i][3 + k] = c[k]; }
      }
    } else {
      real c[3];
      cross3(c, d->xaxis[j], off);
      for (int k = 0; k < 3; k++) { d->cdof[da][k] = d->xaxis[j][k]; d->cdof[da][3 + k] = c[k]; }
    }
  }
}

/* ================================ mj_crb ================================ */
static void crb(const Model* m, Data* d) {
  memcpy(d->crb, d->cinert, sizeof(d->crb));
  for (int b = NB - 1; b > 0; b--)
    if (m->parent[b] > 0)
      for (int k = 0; k < 10; k++) d->crb[m->parent[b]][k] += d->crb[b][k];
  memset(d->M, 0, sizeof(d->M));
  for (int i = 0; i < NV; i++) {
    real buf[6];
    mul_inert_vec(buf, d->crb[m->dof_bodyid[i]], d->cdof[i]);
    for (int j = i; j >= 0; j = m->dof_parentid[j]) {
      d->M[i][j] = dot6(d->cdof[j], buf);
      d->M[j][i] = d->M[i][j];
    }
    d->M[i][i] += m->dof_armature[i];
  }
}

/* ============================== collision ============================== */
static void make_frame(real f[9], const real n[3]) {
  real a[3] = {n[0], n[1], n[2]};
  normalize3(a);
  real y[3] = {0, 0, 0};
  if (a[1] < (real)0.5 && a[1] > (real)-0.5) y[1] = 1; else y[2] = 1;
  real ad = dot3(a, y);
  for (int k = 0; k < 3; k++) y[k] -= a[k] * ad;
  normalize3(y);
  real z[3];
  cross3(z, a, y);
  for (int k = 0; k < 3; k++) { f[k] = a[k]; f[3 + k] = y[k]; f[6 + k] = z[k]; }
}

/* sphere (center c, radius r) vs box (center p, rotation R, half sizes h).
 * Normal points from the sphere into the box (geom1 = sphere, geom2 = box). */
static int sphere_box(const real c[3], real r, const real p[3], const real R[9], const real h[3], real margin,
                      real* dist, real pos[3], real n[3]) {
  real dl[3], rel[3];
  for (int k = 0; k < 3; k++) rel[k] = c[k] - p[k];
  for (int k = 0; k < 3; k++) dl[k] = R[k] * rel[0] + R[3 + k] * rel[1] + R[6 + k] * rel[2]; /* R^T rel */
  real cl[3];
  int inside = 1;
  for (int k = 0; k < 3; k++) {
    cl[k] = dl[k];
    if (cl[k] > h[k]) { cl[k] = h[k]; inside = 0; }
    if (cl[k] < -h[k]) { cl[k] = -h[k]; inside = 0; }
  }
  real nl[3], dd;
  if (!inside) {
    real v[3] = {cl[0] - dl[0], cl[1] - dl[1], cl[2] - dl[2]};
    real len = RSQRT(dot3(v, v));
    dd = len - r;
    if (dd > margin) return 0;
    if (len < MINVAL) { nl[0] = 0; nl[1] = 0; nl[2] = -1; } else { for (int k = 0; k < 3; k++) nl[k] = v[k] / len; }
  } else {
    /* deepest-face: smallest distance to a face */
    int ax = 0;
    real best = h[0] - RFABS(dl[0]);
    for (int k = 1; k < 3; k++) {
      real t = h[k] - RFABS(dl[k]);
      if (t < best) { best = t; ax = k; }
    }
    for (int k = 0; k < 3; k++) nl[k] = 0;
    nl[ax] = dl[ax] >= 0 ? -1 : 1; /* from sphere center toward (and through) the nearest face */
    dd = -best - r;
  }
  matvec(n, R, nl);
  *dist = dd;
  for (int k = 0; k < 3; k++) pos[k] = c[k] + n[k] * (r + dd / 2);
  return 1;
}

static void contact_param(const Model* m, int g1, int g2, Contact* c) {
  int p1 = m->cg_priority[g1], p2 = m->cg_priority[g2];
  if (p1 != p2) {
    int g = p1 > p2 ? g1 : g2;
    c->mu = m->cg_friction[g][0];
    for (int k = 0; k < 2; k++) c->solref[k] = m->cg_solref[g][k];
    for (int k = 0; k < 5; k++) c->solimp[k] = m->cg_solimp[g][k];
  } else {
    real s1 = m->cg_solmix[g1], s2 = m->cg_solmix[g2], mix;
    if (s1 >= MINVAL && s2 >= MINVAL) mix = s1 / (s1 + s2);
    else if (s1 < MINVAL && s2 < MINVAL) mix = (real)0.5;
    else if (s1 < MINVAL) mix = 0;
    else mix = 1;
    if (m->cg_solref[g1][0] > 0 && m->cg_solref[g2][0] > 0)
      for (int k = 0; k < 2; k++) c->solref[k] = mix * m->cg_solref[g1][k] + (1 - mix) * m->cg_solref[g2][k];
    else
      for (int k = 0; k < 2; k++) c->solref[k] = m->cg_solref[g1][k] < m->cg_solref[g2][k] ? m->cg_solref[g1][k] : m->cg_solref[g2][k];
    for (int k = 0; k < 5; k++) c->solimp[k] = mix * m->cg_solimp[g1][k] + (1 - mix) * m->cg_solimp[g2][k];
    c->mu = m->cg_friction[g1][0] > m->cg_friction[g2][0] ? m->cg_friction[g1][0] : m->cg_friction[g2][0];
  }
  real mg1 = m->cg_margin[g1], mg2 = m->cg_margin[g2];
  real gp1 = m->cg_gap[g1], gp2 = m->cg_gap[g2];
  c->margin = (mg1 > mg2 ? mg1 : mg2) - (gp1 > gp2 ? gp1 : gp2);
}

static void collision(const Model* m, Data* d) {
  Contact all[PP3_MAX_PAIR > 256 ? 256 : PP3_MAX_PAIR];
  int n = 0;
  d->ncon_all = 0;
  for (int p = 0; p < m->npair; p++) {
    int g1 = m->pair_g1[p], g2 = m->pair_g2[p];
    int t1 = m->cg_type[g1], t2 = m->cg_type[g2];
    real margin = m->cg_margin[g1] > m->cg_margin[g2] ? m->cg_margin[g1] : m->cg_margin[g2];
    real dist, pos[3], nrm[3];
    int hit = 0;
    if (t1 == PP3_GEOM_PLANE && t2 == PP3_GEOM_SPHERE) {
      real nz[3] = {d->gxmat[g1][2], d->gxmat[g1][5], d->gxmat[g1][8]};
      real v[3] = {d->gxpos[g2][0] - d->gxpos[g1][0], d->gxpos[g2][1] - d->gxpos[g1][1], d->gxpos[g2][2] - d->gxpos[g1][2]};
      real r = m->cg_size[g2][0];
      dist = dot3(nz, v) - r;
      if (dist <= margin) {
        hit = 1;
        for (int k = 0; k < 3; k++) { nrm[k] = nz[k]; pos[k] = d->gxpos[g2][k] - nz[k] * (r + dist / 2); }
      }
    } else if (t1 == PP3_GEOM_SPHERE && t2 == PP3_GEOM_SPHERE) {
      real v[3] = {d->gxpos[g2][0] - d->gxpos[g1][0], d->gxpos[g2][1] - d->gxpos[g1][1], d->gxpos[g2][2] - d->gxpos[g1][2]};
      real r1 = m->cg_size[g1][0], r2 = m->cg_size[g2][0];
      real len = RSQRT(dot3(v, v));
      dist = len - r1 - r2;
      if (dist <= margin) {
        hit = 1;
        if (len < MINVAL) { nrm[0] = 1; nrm[1] = 0; nrm[2] = 0; }
        else for (int k = 0; k < 3; k++) nrm[k] = v[k] / len;
        for (int k = 0; k < 3; k++) pos[k] = d->gxpos[g1][k] + nrm[k] * (r1 + dist / 2);
      }
    } else if (t1 == PP3_GEOM_SPHERE && t2 == PP3_GEOM_BOX) {
      hit = sphere_box(d->gxpos[g1], m->cg_size[g1][0], d->gxpos[g2], d->gxmat[g2], m->cg_size[g2], margin, &dist, pos, nrm);
    }
    if (!hit) continue;
    d->ncon_all++;
    if (n >= (int)(sizeof(all) / sizeof(all[0]))) continue;
    Contact* c = &all[n++];
    c->g1 = g1; c->g2 = g2; c->dist = dist;
    memcpy(c->pos, pos, sizeof(pos));
    make_frame(c->frame, nrm);
    contact_param(m, g1, g2, c);
  }
  /* contact cap: keep the ncon_max deepest (stable by pair order) */
  int cap = m->ncon_max < ORC_MAXCON ? m->ncon_max : ORC_MAXCON;
  if (n <= cap) {
    memcpy(d->con, all, sizeof(Contact) * n);
    d->ncon = n;
  } else {
    int used[256] = {0};
    int k = 0;
    /* select the cap deepest, then emit in pair order */
    for (int s = 0; s < cap; s++) {
      int best = -1;
      for (int i = 0; i < n; i++)
        if (!used[i] && (best < 0 || all[i].dist < all[best].dist)) best = i;
      used[best] = 1;
    }
    for (int i = 0; i < n; i++) if (used[i]) d->con[k++] = all[i];
    d->ncon = k;
  }
}

/* ===================== constraints: J, R, D, aref ===================== */
/* translational Jacobian of a point attached to body b (zero for the world body) */
static void jac_point(const Model* m, const Data* d, int b, const real pt[3], real J[3][NV]) {
  memset(J, 0, sizeof(real) * 3 * NV);
  if (b == 0) return;
  real off[3] = {pt[0] - d->com[0], pt[1] - d->com[1], pt[2] - d->com[2]};
  int i = m->dofadr[b] + m->dofnum[b] - 1;
  for (; i >= 0; i = m->dof_parentid[i]) {
    real c[3];
    cross3(c, d->cdof[i], off);
    for (int k = 0; k < 3; k++) J[k][i] = d->cdof[i][3 + k] + c[k];
  }
}

static real getimp(const real solimp[5], real pos, real margin) {
  real dmin = solimp[0], dmax = solimp[1], width = solimp[2], mid = solimp[3], power = solimp[4];
  if (dmin < MINIMP) dmin = MINIMP;
  if (dmin > MAXIMP) dmin = MAXIMP;
  if (dmax < MINIMP) dmax = MINIMP;
  if (dmax > MAXIMP) dmax = MAXIMP;
  if (width < MINVAL) width = MINVAL;
  if (mid < MINIMP) mid = MINIMP;
  if (mid > MAXIMP) mid = MAXIMP;
  if (power < 1) power = 1;
  real x = (pos - margin) / width;
  if (x < 0) x = -x;
  if (x >= 1) return dmax;
  if (x <= 0) return dmin;
  real y;
  if (power == 1) y = x;
  else if (x <= mid) y = RPOW(x, power) / RPOW(mid, power - 1);
  else y = 1 - RPOW(1 - x, power) / RPOW(1 - mid, power - 1);
  return dmin + y * (dmax - dmin);
}

static void add_row(const Model* m, Data* d, int type, int id, const real* J, real pos, real margin, real floss,
                    real invweight, const real solref[2], const real solimp[5]) {
  int r = d->nefc++;
  d->efc_type[r] = type;
  d->efc_id[r] = id;
  memcpy(d->efc_J[r], J, sizeof(real) * NV);
  d->efc_pos[r] = pos;
  d->efc_margin[r] = margin;
  d->efc_floss[r] = floss;
  real imp = getimp(solimp, pos, margin);
  real R = (1 - imp) / imp * invweight;
  if (R < MINVAL) R = MINVAL;
  d->efc_R[r] = R;
  d->efc_D[r] = 1 / R;
  /* KBIP: standard (timeconst, dampratio) or direct (-stiffness, -damping) */
  real dmax = solimp[1];
  if (dmax < MINIMP) dmax = MINIMP;
  if (dmax > MAXIMP) dmax = MAXIMP;
  real k, b;
  if (solref[0] > 0) {
    real tc = solref[0], dr = solref[1];
    if (tc < 2 * m->timestep) tc = 2 * m->timestep; /* REFSAFE */
    k = 1 / (dmax * dmax * tc * tc * dr * dr);
    b = 2 / (dmax * tc);
  } else {
    k = -solref[0] / (dmax * dmax);
    b = -solref[1] / dmax;
  }
  real vel = 0;
  for (int i = 0; i < NV; i++) vel += J[i] * d->qvel[i];
  d->efc_aref[r] = -b * vel - k * imp * (pos - margin);
}

static void make_constraint(const Model* m, Data* d) {
  d->nefc = 0;
  real J[NV];
  /* dof frictionloss rows (mj_instantiateFriction) */
  for (int i = 0; i < NV; i++) {
    if (m->dof_frictionloss[i] > 0) {
      memset(J, 0, sizeof(J));
      J[i] = 1;
      add_row(m, d, CN_FRICTION, i, J, 0, 0, m->dof_frictionloss[i], m->dof_invweight0[i], m->dof_solref[i], m->dof_solimp[i]);
    }
  }
  d->nf = d->nefc;
  /* joint limits (mj_instantiateLimit): hinge, both sides */
  for (int j = 0; j < NJ; j++) {
    if (!m->jnt_limited[j] || m->jnt_type[j] != PP3_JNT_HINGE) continue;
    int a = m->jnt_qposadr[j], da = m->jnt_dofadr[j];
    for (int side = -1; side <= 1; side += 2) {
      real value = side * (m->jnt_range[j][(side + 1) / 2] - d->qpos[a]);
      if (value < m->jnt_margin[j]) {
        memset(J, 0, sizeof(J));
        J[da] = (real)(-side);
        add_row(m, d, CN_LIMIT, j, J, value, m->jnt_margin[j], 0, m->dof_invweight0[da], m->jnt_solref[j], m->jnt_solimp[j]);
      }
    }
  }
  d->nl = d->nefc - d->nf;
  /* pyramidal contacts (mj_instantiateContact), condim 3 -> 4 edges */
  for (int c = 0; c < d->ncon; c++) {
    Contact* con = &d->con[c];
    int b1 = m->cg_body[con->g1], b2 = m->cg_body[con->g2];
    real J1[3][NV], J2[3][NV], Jd[3][NV], Jc[3][NV];
    jac_point(m, d, b1, con->pos, J1);
    jac_point(m, d, b2, con->pos, J2);
    for (int k = 0; k < 3; k++)
      for (int i = 0; i < NV; i++) Jd[k][i] = J2[k][i] - J1[k][i];
    for (int r = 0; r < 3; r++)
      for (int i = 0; i < NV; i++)
        Jc[r][i] = con->frame[3 * r] * Jd[0][i] + con->frame[3 * r + 1] * Jd[1][i] + con->frame[3 * r + 2] * Jd[2][i];
    real tran = m->body_invweight0[b1][0] + m->body_invweight0[b2][0];
    real mu = con->mu;
    /* pyramidal: common invweight for all edges, scaled by 2 mu^2 / impratio */
    real invw = (tran + mu * mu * tran) * 2 * mu * mu / m->impratio;
    for (int e = 0; e < 4; e++) {
      int t = 1 + e / 2;
      real sgn = (e % 2 == 0) ? 1 : -1;
      for (int i = 0; i < NV; i++) J[i] = Jc[0][i] + sgn * mu * Jc[t][i];
      add_row(m, d, CN_CONTACT, c, J, con->dist, con->margin, 0, invw, con->solref, con->solimp);
    }
  }
}

/* ============================ velocity stage ============================ */
static void com_vel(const Model* m, Data* d) {
  for (int k = 0; k < 6; k++) d->cvel[0][k] = 0;
  for (int b = 1; b < NB; b++) {
    real cv[6];
    memcpy(cv, d->cvel[m->parent[b]], sizeof(cv));
    int j = m->jntadr[b];
    if (j >= 0) {
      int da = m->jnt_dofadr[j];
      if (m->jnt_type[j] == PP3_JNT_FREE) {
        for (int i = 0; i < 3; i++) {
          for (int k = 0; k < 6; k++) d->cdof_dot[da + i][k] = 0;
          for (int k = 0; k < 6; k++) cv[k] += d->cdof[da + i][k] * d->qvel[da + i];
        }
        for (int i = 0; i < 3; i++) cross_motion(d->cdof_dot[da + 3 + i], cv, d->cdof[da + 3 + i]);
        for (int i = 0; i < 3; i++)
          for (int k = 0; k < 6; k++) cv[k] += d->cdof[da + 3 + i][k] * d->qvel[da + 3 + i];
      } else {
        cross_motion(d->cdof_dot[da], cv, d->cdof[da]);
        for (int k = 0; k < 6; k++) cv[k] += d->cdof[da][k] * d->qvel[da];
      }
    }
    memcpy(d->cvel[b], cv, sizeof(cv));
  }
}

static void rne(const Model* m, Data* d) {
  real cacc[NB][6], cfrc[NB][6];
  for (int k = 0; k < 3; k++) { cacc[0][k] = 0; cacc[0][3 + k] = -m->gravity[k]; }
  for (int b = 1; b < NB; b++) {
    memcpy(cacc[b], cacc[m->parent[b]], sizeof(cacc[b]));
    for (int i = m->dofadr[b]; i >= 0 && i < m->dofadr[b] + m->dofnum[b]; i++)
      for (int k = 0; k < 6; k++) cacc[b][k] += d->cdof_dot[i][k] * d->qvel[i];
    real f1[6], f2[6], f3[6];
    mul_inert_vec(f1, d->cinert[b], cacc[b]);
    mul_inert_vec(f2, d->cinert[b], d->cvel[b]);
    cross_force(f3, d->cvel[b], f2);
    for (int k = 0; k < 6; k++) cfrc[b][k] = f1[k] + f3[k];
  }
  for (int b = NB - 1; b > 0; b--)
    if (m->parent[b] > 0)
      for (int k = 0; k < 6; k++) cfrc[m->parent[b]][k] += cfrc[b][k];
  for (int i = 0; i < NV; i++) d->qfrc_bias[i] = dot6(d->cdof[i], cfrc[m->dof_bodyid[i]]);
}

static void actuation(const Model* m, Data* d) {
  memset(d->qfrc_actuator, 0, sizeof(d->qfrc_actuator));
  for (int a = 0; a < NU; a++) {
    int j = m->act_jnt[a];
    int qa = m->jnt_qposadr[j], da = m->jnt_dofadr[j];
    real ctrl = d->ctrl[a];
    if (m->act_ctrllimited[a]) {
      if (ctrl < m->act_ctrlrange[a][0]) ctrl = m->act_ctrlrange[a][0];
      if (ctrl > m->act_ctrlrange[a][1]) ctrl = m->act_ctrlrange[a][1];
    }
    real len = m->act_gear[a] * d->qpos[qa], vel = m->act_gear[a] * d->qvel[da];
    real force = m->act_gain[a][0] * ctrl;
    if (m->act_biastype[a] == PP3_BIAS_AFFINE) force += m->act_bias[a][0] + m->act_bias[a][1] * len + m->act_bias[a][2] * vel;
    if (m->act_forcelimited[a]) {
      if (force < m->act_forcerange[a][0]) force = m->act_forcerange[a][0];
      if (force > m->act_forcerange[a][1]) force = m->act_forcerange[a][1];
    }
    d->qfrc_actuator[da] += m->act_gear[a] * force;
  }
}

/* =============================== linear algebra =============================== */
/* dense Cholesky in place (lower), pivots floored at MINVAL (mju_cholFactor) */
static void chol_factor(real A[NV][NV]) {
  for (int j = 0; j < NV; j++) {
    real s = A[j][j];
    for (int k = 0; k < j; k++) s -= A[j][k] * A[j][k];
    if (s < MINVAL) s = MINVAL;
    A[j][j] = RSQRT(s);
    for (int i = j + 1; i < NV; i++) {
      real t = A[i][j];
      for (int k = 0; k < j; k++) t -= A[i][k] * A[j][k];
      A[i][j] = t / A[j][j];
    }
  }
}
static void chol_solve(real L[NV][NV], real x[NV], const real b[NV]) {
  real y[NV];
  for (int i = 0; i < NV; i++) {
    real t = b[i];
    for (int k = 0; k < i; k++) t -= L[i][k] * y[k];
    y[i] = t / L[i][i];
  }
  for (int i = NV - 1; i >= 0; i--) {
    real t = y[i];
    for (int k = i + 1; k < NV; k++) t -= L[k][i] * x[k];
    x[i] = t / L[i][i];
  }
}
static void mulM(const Data* d, real r[NV], const real v[NV]) {
  for (int i = 0; i < NV; i++) {
    real s = 0;
    for (int j = 0; j < NV; j++) s += d->M[i][j] * v[j];
    r[i] = s;
  }
}

/* ================================ Newton solver ================================ */
/* constraint cost/state/force at jar = J qacc - aref (mj_constraintUpdate) */
static real constraint_update(Data* d, const real* jar, int store) {
  real cost = 0;
  for (int r = 0; r < d->nefc; r++) {
    real f, st;
    real D = d->efc_D[r], x = jar[r];
    if (d->efc_type[r] == CN_FRICTION) {
      real fl = d->efc_floss[r], rf = d->efc_R[r] * fl;
      if (x <= -rf) { st = ST_LINNEG; f = fl; cost += -fl * x - (real)0.5 * rf * fl; }
      else if (x >= rf) { st = ST_LINPOS; f = -fl; cost += fl * x - (real)0.5 * rf * fl; }
      else { st = ST_QUADRATIC; f = -D * x; cost += (real)0.5 * D * x * x; }
    } else {
      if (x >= 0) { st = ST_SATISFIED; f = 0; }
      else { st = ST_QUADRATIC; f = -D * x; cost += (real)0.5 * D * x * x; }
    }
    if (store) { d->efc_state[r] = (int)st; d->efc_force[r] = f; }
  }
  return cost;
}

typedef struct { real alpha, cost, d0, d1; } LSPoint;

typedef struct {
  const Data* d;
  const real* Jaref;
  const real* Jv;
  real quadG[3];
  int evals;
} LSCtx;

static int g_ls_trace = 0;
static void ls_eval(LSCtx* c, LSPoint* p) {
  const Data* d = c->d;
  real a = p->alpha;
  if (g_ls_trace) {
    static char prev[ORC_MAXEFC];
    int nch = 0;
    for (int r = 0; r < d->nefc; r++) {
      real x = c->Jaref[r] + a * c->Jv[r];
      char st;
      if (d->efc_type[r] == CN_FRICTION) { real rf = d->efc_R[r] * d->efc_floss[r]; st = x <= -rf ? 1 : (x >= rf ? 2 : 0); }
      else st = x >= 0 ? 3 : 0;
      if (c->evals > 0 && st != prev[r]) nch++;
      prev[r] = st;
    }
    printf("  eval %d alpha %.9g changed %d\n", c->evals, (double)a, nch);
  }
  real t0 = c->quadG[0], t1 = c->quadG[1], t2 = c->quadG[2];
  for (int r = 0; r < d->nefc; r++) {
    real jar = c->Jaref[r], jv = c->Jv[r], D = d->efc_D[r];
    real x = jar + a * jv;
    if (d->efc_type[r] == CN_FRICTION) {
      real fl = d->efc_floss[r], rf = d->efc_R[r] * fl;
      if (x <= -rf) { t0 += -fl * jar - (real)0.5 * rf * fl; t1 += -fl * jv; continue; }
      if (x >= rf) { t0 += fl * jar - (real)0.5 * rf * fl; t1 += fl * jv; continue; }
    } else if (x >= 0) {
      continue;
    }
    t0 += (real)0.5 * D * jar * jar;
    t1 += D * jar * jv;
    t2 += (real)0.5 * D * jv * jv;
  }
  p->cost = t0 + a * t1 + a * a * t2;
  p->d0 = t1 + 2 * a * t2;
  p->d1 = 2 * t2;
  if (p->d1 < MINVAL) p->d1 = MINVAL;
  c->evals++;
}

/* Line-search convergence: MuJoCo's |derivative| < gtol, or -- the arithmetic's floor -- the
 * remaining Newton correction |d0 / d1| at or below LS_NOISE roundoffs of alpha in the precision
 * of `real` (a derivative that small is rounding noise: below it the search only moves alpha by
 * noise).  In double this floor sits ~1e-14 relative, far below any gtol MuJoCo's tolerances give,
 * so the fp64 oracle is PrimalSearch unchanged; in float it stops the search where MuJoCo in
 * double stops (a Newton step that landed on the 1-D minimum) instead of spending the remaining
 * ls_iterations on noise.  The HIP kernel applies the same rule with FLT_EPSILON. */
#define LS_NOISE ((real)64)
static int g_ls_noise = 1;
static _Thread_local long g_ls_total = 0, g_ls_calls = 0, g_ls_smooth = 0, g_ls_starts = 0;  /* line-search evaluations / searches (diagnostics) */
/* how each search ended (orc_ls_take): LS_CONVERGED = a point passed ls_converged; LS_CAPPED = the
 * evaluation budget ls_iterations ran out first, so the returned alpha is set by the exit rule below
 * (PrimalSearch's, restated from memory of engine_solver.c: MuJoCo's documentation does not specify
 * it); LS_STALLED = the bracket stopped shrinking (no candidate closer to the root on either side) */
enum { LS_CONVERGED = 0, LS_CAPPED = 1, LS_STALLED = 2 };
static _Thread_local long g_ls_exit[3] = {0, 0, 0};
/* of the searches: those that reached the bracketing phase, and those capped there (the rest of
 * LS_CAPPED ended in the one-sided phase, whose exit returns the last Newton point unexamined) */
static _Thread_local long g_ls_bracket = 0, g_ls_cap_bracket = 0;
static int ls_converged(const LSPoint* p, real gtol) {
  if (RFABS(p->d0) < gtol) return 1;
  return g_ls_noise && RFABS(p->d0) <= LS_NOISE * REPS * p->d1 * RFABS(p->alpha);
}

/* engine_solver.c PrimalSearch-style exact line search: Newton step from 0, one-sided Newton
 * until the derivative changes sign, then bracketed Newton/midpoint refinement. */
static real line_search(LSCtx* c, real gtol, int maxit) {
  /* labels P0 ... B7: DESIGN.md 5 (the branch-by-branch statement, for checking against
   * engine_solver.c PrimalSearch / updateBracket) */
  LSPoint p0, p1, p2, pmid, p1n, p2n;
  p0.alpha = 0;
  ls_eval(c, &p0);                                          /* P0 */
  p1.alpha = p0.alpha - p0.d0 / p0.d1;
  ls_eval(c, &p1);                                          /* P1 */
  if (p0.cost < p1.cost) p1 = p0;                           /* P2 */
  if (ls_converged(&p1, gtol)) { g_ls_exit[LS_CONVERGED]++; return p1.alpha; }  /* P3 */
  real dir = p1.d0 < 0 ? 1 : -1;                            /* O1 */
  p2 = p1;
  while (p1.d0 * dir <= -gtol && c->evals < maxit) {        /* O2 */
    p2 = p1;
    p1.alpha -= p1.d0 / p1.d1;
    ls_eval(c, &p1);
    if (ls_converged(&p1, gtol)) { g_ls_exit[LS_CONVERGED]++; return p1.alpha; }
  }
  if (c->evals >= maxit) { g_ls_exit[LS_CAPPED]++; return p1.alpha; }  /* O3 */
  /* bracket [p2, p1]: p2.d0*dir < 0 < p1.d0*dir */
  g_ls_bracket++;
  p2n = p1;                                                 /* B0 */
  p1n.alpha = p1.alpha - p1.d0 / p1.d1;
  ls_eval(c, &p1n);
  while (c->evals < maxit) {                                /* B1 */
    pmid.alpha = (real)0.5 * (p1.alpha + p2.alpha);
    ls_eval(c, &pmid);                                      /* B2 */
    LSPoint cand[3] = {p1n, p2n, pmid};
    int best = -1;
    for (int i = 0; i < 3; i++)                             /* B3 */
      if (ls_converged(&cand[i], gtol) && (best < 0 || cand[i].cost < cand[best].cost)) best = i;
    if (best >= 0) { g_ls_exit[LS_CONVERGED]++; return cand[best].alpha; }
    int up1 = 0, up2 = 0;
    for (int i = 0; i < 3; i++) {                           /* B4 */
      /* tighten each bracket end with any candidate on its side that is closer to the root */
      if (p1.d0 * cand[i].d0 > 0 && RFABS(cand[i].d0) < RFABS(p1.d0)) { p1 = cand[i]; up1 = 1; }
      if (p2.d0 * cand[i].d0 > 0 && RFABS(cand[i].d0) < RFABS(p2.d0)) { p2 = cand[i]; up2 = 1; }
    }
    if (!up1 && !up2) break;                                /* B5 */
    if (up1) { p1n.alpha = p1.alpha - p1.d0 / p1.d1; ls_eval(c, &p1n); }  /* B6 */
    if (up2) { p2n.alpha = p2.alpha - p2.d0 / p2.d1; ls_eval(c, &p2n); }
  }
  g_ls_exit[c->evals >= maxit ? LS_CAPPED : LS_STALLED]++;
  g_ls_cap_bracket += c->evals >= maxit;
  return p1.cost < p2.cost ? p1.alpha : p2.alpha;           /* B7 */
}

static void solve_newton(const Model* m, Data* d) {
  int nefc = d->nefc;
  real jar[ORC_MAXEFC], jar_s[ORC_MAXEFC];
  real Ma[NV], qacc[NV];
  /* warm start: best of qacc_warmstart and qacc_smooth (mj_fwdConstraint warmstart) */
  for (int r = 0; r < nefc; r++) {
    real s1 = 0, s2 = 0;
    for (int i = 0; i < NV; i++) { s1 += d->efc_J[r][i] * d->qacc_warmstart[i]; s2 += d->efc_J[r][i] * d->qacc_smooth[i]; }
    jar[r] = s1 - d->efc_aref[r];
    jar_s[r] = s2 - d->efc_aref[r];
  }
  real cost_ws = constraint_update(d, jar, 0);
  mulM(d, Ma, d->qacc_warmstart);
  for (int i = 0; i < NV; i++) cost_ws += (real)0.5 * (Ma[i] - d->qfrc_smooth[i]) * (d->qacc_warmstart[i] - d->qacc_smooth[i]);
  real cost_sm = constraint_update(d, jar_s, 0);
  if (RFABS(cost_ws - cost_sm) < BOUNDARY_REL * (RFABS(cost_ws) + RFABS(cost_sm))) g_boundary++;
  g_ls_smooth += cost_ws > cost_sm;
  g_ls_starts++;
  if (cost_ws > cost_sm) memcpy(qacc, d->qacc_smooth, sizeof(qacc));
  else memcpy(qacc, d->qacc_warmstart, sizeof(qacc));

  real scale = 1 / (m->meaninertia * (NV > 1 ? NV : 1));
  d->ls_evals = 0;
  for (int it = 0; it < m->iterations; it++) {
    /* Ma, Jaref, constraint state at qacc */
    mulM(d, Ma, qacc);
    for (int r = 0; r < nefc; r++) {
      real s = 0;
      for (int i = 0; i < NV; i++) s += d->efc_J[r][i] * qacc[i];
      jar[r] = s - d->efc_aref[r];
    }
    real cost = constraint_update(d, jar, 1);
    /* fp32 sensitivity flag: a row whose constraint state (satisfied / quadratic / linear) is
     * decided within rounding of its switch point makes the Newton Hessian, and so this
     * one-iteration solve, discontinuous in the input; count such rows for the parity tests */
    for (int r = 0; r < nefc; r++) {
      const real x = jar[r], sc = BOUNDARY_REL * (1 + RFABS(d->efc_aref[r]));
      if (d->efc_type[r] == CN_FRICTION) {
        const real rf = d->efc_R[r] * d->efc_floss[r];
        if (RFABS(x - rf) < sc || RFABS(x + rf) < sc) g_boundary++;
      } else if (RFABS(x) < sc) {
        g_boundary++;
      }
    }
    real gauss = 0;
    for (int i = 0; i < NV; i++) gauss += (real)0.5 * (Ma[i] - d->qfrc_smooth[i]) * (qacc[i] - d->qacc_smooth[i]);
    cost += gauss;
    /* gradient and Hessian */
    real grad[NV], H[NV][NV], search[NV];
    for (int i = 0; i < NV; i++) {
      real qc = 0;
      for (int r = 0; r < nefc; r++) qc += d->efc_J[r][i] * d->efc_force[r];
      grad[i] = Ma[i] - d->qfrc_smooth[i] - qc;
    }
    memcpy(H, d->M, sizeof(H));
    for (int r = 0; r < nefc; r++) {
      if (d->efc_state[r] != ST_QUADRATIC) continue;
      real D = d->efc_D[r];
      for (int i = 0; i < NV; i++) {
        real ji = d->efc_J[r][i] * D;
        if (ji == 0) continue;
        for (int j = 0; j < NV; j++) H[i][j] += ji * d->efc_J[r][j];
      }
    }
    for (int i = 0; i < NV; i++)
      for (int j = 0; j < NV; j++) g_dbg[64 + NV * i + j] = (double)H[i][j];
    for (int r = 12; r < nefc && r < 20; r++) {
      g_dbg[400 + r - 12] = d->efc_state[r] == ST_QUADRATIC ? (double)d->efc_D[r] : 0.0;
      g_dbg[430 + r - 12] = (double)jar[r];
      g_dbg[440 + r - 12] = (double)d->efc_force[r];
    }
    chol_factor(H);
    chol_solve(H, search, grad);
    for (int i = 0; i < NV; i++) search[i] = -search[i];
    /* line search */
    real snorm = 0;
    for (int i = 0; i < NV; i++) snorm += search[i] * search[i];
    snorm = RSQRT(snorm);
    if (snorm < MINVAL) break;
    real Mv[NV], Jv[ORC_MAXEFC];
    mulM(d, Mv, search);
    for (int r = 0; r < nefc; r++) {
      real s = 0;
      for (int i = 0; i < NV; i++) s += d->efc_J[r][i] * search[i];
      Jv[r] = s;
    }
    LSCtx c;
    c.d = d; c.Jaref = jar; c.Jv = Jv; c.evals = 0;
    c.quadG[0] = gauss;
    c.quadG[1] = 0;
    c.quadG[2] = 0;
    for (int i = 0; i < NV; i++) {
      c.quadG[1] += search[i] * (Ma[i] - d->qfrc_smooth[i]);
      c.quadG[2] += (real)0.5 * search[i] * Mv[i];
    }
    real gtol = m->tolerance * m->ls_tolerance * snorm / scale;
    real alpha = line_search(&c, gtol, m->ls_iterations);
    if (g_ls_trace) printf(" -> alpha %.9g evals %d nefc %d gtol %.3g\n", (double)alpha, c.evals, nefc, (double)gtol);
    /* debug record of the last Newton iteration (orc_debug_read) */
    for (int i = 0; i < NV; i++) { g_dbg[i] = (double)qacc[i]; g_dbg[18 + i] = (double)grad[i]; g_dbg[36 + i] = (double)search[i]; }
    g_dbg[54] = (double)c.quadG[0]; g_dbg[55] = (double)c.quadG[1]; g_dbg[56] = (double)c.quadG[2];
    g_dbg[57] = (double)snorm; g_dbg[58] = (double)gtol; g_dbg[59] = (double)alpha; g_dbg[60] = (double)c.evals;
    g_dbg[61] = (double)cost_ws; g_dbg[62] = (double)cost_sm; g_dbg[63] = (double)nefc;
    d->ls_evals += c.evals;
    g_ls_total += c.evals;
    g_ls_calls++;
    if (alpha == 0) break;
    for (int i = 0; i < NV; i++) qacc[i] += alpha * search[i];
    (void)cost;
  }
  /* final constraint forces */
  memcpy(d->qacc, qacc, sizeof(qacc));
  for (int r = 0; r < nefc; r++) {
    real s = 0;
    for (int i = 0; i < NV; i++) s += d->efc_J[r][i] * qacc[i];
    jar[r] = s - d->efc_aref[r];
  }
  constraint_update(d, jar, 1);
  for (int i = 0; i < NV; i++) {
    real qc = 0;
    for (int r = 0; r < nefc; r++) qc += d->efc_J[r][i] * d->efc_force[r];
    d->qfrc_constraint[i] = qc;
  }
  memcpy(d->qacc_warmstart, qacc, sizeof(qacc));
}

/* ================================ mj_forward / mj_step ================================ */
/* mjData.sensordata of the last forward (mj_sensorPos/Vel/Acc for site sensors, SURVEY 8f rank
 * 4).  Accelerations follow mj_rnePostConstraint (cacc = cacc_parent + cdof_dot.qvel + cdof.qacc,
 * cacc_world = -gravity) and mj_objectAcceleration (transport to the site, rotate into the site
 * frame, add the rotating-frame term omega x v); velocities follow mj_objectVelocity.  The site
 * frame is xquat(body) * site_quat. */
static void sensors(const Model* m, const Data* d, real* out) {
  real cacc[NB][6];
  for (int k = 0; k < 3; k++) { cacc[0][k] = 0; cacc[0][3 + k] = -m->gravity[k]; }
  for (int b = 1; b < NB; b++) {
    real t1[6] = {0, 0, 0, 0, 0, 0}, t2[6] = {0, 0, 0, 0, 0, 0};
    for (int i = m->dofadr[b]; i >= 0 && i < m->dofadr[b] + m->dofnum[b]; i++)
      for (int k = 0; k < 6; k++) { t1[k] += d->cdof_dot[i][k] * d->qvel[i]; t2[k] += d->cdof[i][k] * d->qacc[i]; }
    for (int k = 0; k < 6; k++) cacc[b][k] = cacc[m->parent[b]][k] + t1[k] + t2[k];
  }
  for (int i = 0; i < m->nsensor; i++) {
    const int sid = m->sensor_objid[i], b = m->site_body[sid], typ = m->sensor_type[i];
    real sq[4], R[9], dif[3], cr[3], vang[3], vlin[3], v[4] = {0, 0, 0, 0};
    mulquat(sq, d->xquat[b], m->site_quat[sid]);
    quat2mat(sq, R);
    for (int k = 0; k < 3; k++) dif[k] = d->site_xpos[sid][k] - d->com[k];
    for (int k = 0; k < 3; k++) vang[k] = d->cvel[b][k];
    cross3(cr, dif, vang);
    for (int k = 0; k < 3; k++) vlin[k] = d->cvel[b][3 + k] - cr[k];
    int dim = 3;
    if (typ == PP3_SENS_FRAMEPOS) for (int k = 0; k < 3; k++) v[k] = d->site_xpos[sid][k];
    else if (typ == PP3_SENS_FRAMEQUAT) { for (int k = 0; k < 4; k++) v[k] = sq[k]; dim = 4; }
    else if (typ == PP3_SENS_FRAMELINVEL) for (int k = 0; k < 3; k++) v[k] = vlin[k];
    else if (typ == PP3_SENS_FRAMEANGVEL) for (int k = 0; k < 3; k++) v[k] = vang[k];
    else if (typ == PP3_SENS_GYRO || typ == PP3_SENS_VELOCIMETER) {
      const real* w = typ == PP3_SENS_GYRO ? vang : vlin;
      for (int k = 0; k < 3; k++) v[k] = R[k] * w[0] + R[3 + k] * w[1] + R[6 + k] * w[2];  /* R^T w */
    } else if (typ == PP3_SENS_ACCELEROMETER) {
      real aang[3], alin[3], wl[3], vl[3], c2[3];
      for (int k = 0; k < 3; k++) aang[k] = cacc[b][k];
      cross3(cr, dif, aang);
      for (int k = 0; k < 3; k++) alin[k] = cacc[b][3 + k] - cr[k];
      for (int k = 0; k < 3; k++) {
        v[k] = R[k] * alin[0] + R[3 + k] * alin[1] + R[6 + k] * alin[2];
        wl[k] = R[k] * vang[0] + R[3 + k] * vang[1] + R[6 + k] * vang[2];
        vl[k] = R[k] * vlin[0] + R[3 + k] * vlin[1] + R[6 + k] * vlin[2];
      }
      cross3(c2, wl, vl);
      for (int k = 0; k < 3; k++) v[k] += c2[k];
    }
    const real co = m->sensor_cutoff[i];
    if (co > 0 && typ != PP3_SENS_FRAMEQUAT)
      for (int k = 0; k < 3; k++) v[k] = v[k] > co ? co : (v[k] < -co ? -co : v[k]);
    for (int k = 0; k < dim; k++) out[m->sensor_adr[i] + k] = v[k];
  }
}

static void forward(const Model* m, Data* d) {
  kinematics(m, d);
  com_pos(m, d);
  crb(m, d);
  collision(m, d);
  make_constraint(m, d);
  com_vel(m, d);
  for (int i = 0; i < NV; i++) d->qfrc_passive[i] = -m->dof_damping[i] * d->qvel[i];
  rne(m, d);
  actuation(m, d);
  for (int i = 0; i < NV; i++) d->qfrc_smooth[i] = d->qfrc_passive[i] - d->qfrc_bias[i] + d->qfrc_actuator[i];
  real L[NV][NV];
  memcpy(L, d->M, sizeof(L));
  chol_factor(L);
  chol_solve(L, d->qacc_smooth, d->qfrc_smooth);
  solve_newton(m, d);
  sensors(m, d, d->sensordata);  /* mj_sensorPos/Vel/Acc: before integration */
}

static void integrate(const Model* m, Data* d) {
  real h = m->timestep;
  for (int i = 0; i < NV; i++) d->qvel[i] += h * d->qacc[i];
  for (int j = 0; j < NJ; j++) {
    int a = m->jnt_qposadr[j], da = m->jnt_dofadr[j];
    if (m->jnt_type[j] == PP3_JNT_FREE) {
      for (int k = 0; k < 3; k++) d->qpos[a + k] += h * d->qvel[da + k];
      real w[3] = {d->qvel[da + 3], d->qvel[da + 4], d->qvel[da + 5]};
      real ang = h * normalize3(w);
      real qr[4], *q = &d->qpos[a + 3];
      axisangle2quat(qr, w, ang);
      normalize4(q);
      mulquat(q, q, qr);
    } else {
      d->qpos[a] += h * d->qvel[da];
    }
  }
}

static void step(const Model* m, Data* d) {
  forward(m, d);
  integrate(m, d);
}

/* pipeline record (brax State.x/xd of the last forward; PP3_P_* layout) */
static void write_pipeline(const Model* m, const Data* d, real* p) {
  if (!p) return;
  memset(p, 0, sizeof(real) * PP3_PIPE_STRIDE);
  for (int b = 1; b < NB; b++) {
    real off[3], w[3], v[3];
    for (int k = 0; k < 3; k++) {
      p[PP3_P_XPOS + 3 * (b - 1) + k] = d->xpos[b][k];
      off[k] = d->xpos[b][k] - d->com[k];
      w[k] = d->cvel[b][k];
    }
    for (int k = 0; k < 4; k++) p[PP3_P_XQUAT + 4 * (b - 1) + k] = d->xquat[b][k];
    cross3(v, w, off);
    for (int k = 0; k < 3; k++) {
      p[PP3_P_XD_VEL + 3 * (b - 1) + k] = d->cvel[b][3 + k] + v[k];
      p[PP3_P_XD_ANG + 3 * (b - 1) + k] = w[k];
    }
  }
  for (int i = 0; i < NV; i++) { p[PP3_P_QFRC_ACT + i] = d->qfrc_actuator[i]; p[PP3_P_QACC + i] = d->qacc[i]; }
  p[PP3_P_NCON] = (real)d->ncon;
  p[PP3_P_NHIT] = (real)d->ncon_all;
  for (int c = 0; c < d->ncon && c < 16; c++) {
    p[PP3_P_CON_DIST + c] = d->con[c].dist;
    p[PP3_P_CON_GEOM + 2 * c] = (real)m->cg_id[d->con[c].g1];
    p[PP3_P_CON_GEOM + 2 * c + 1] = (real)m->cg_id[d->con[c].g2];
  }
  for (int k = 0; k < 3; k++) p[PP3_P_SUBTREE_COM + k] = d->com[k];
  for (int k = 0; k < PP3_MAX_SENSORDATA; k++) p[PP3_P_SENSOR + k] = d->sensordata[k];
}

/* ============================ exported physics API ============================ */
size_t orc_data_size(void) { return sizeof(Data); }

/* nsteps x mj_step with fixed ctrl; qpos/qvel/qacc_ws updated in place (double I/O). */
void orc_mj_step(const pp3_model_t* mm, const double* dr, int ncon_max, double* qpos, double* qvel, double* qws,
                 const double* ctrl, int nsteps, double* pipe, double* site_xpos_out) {
  Model* m = (Model*)malloc(sizeof(Model));
  Data* d = (Data*)calloc(1, sizeof(Data));
  real drr[PP3_NDR];
  if (dr) for (int k = 0; k < PP3_NDR; k++) drr[k] = (real)dr[k];
  model_from_abi(m, mm, dr ? drr : NULL);
  if (ncon_max > 0) m->ncon_max = ncon_max;
  for (int i = 0; i < NQ; i++) d->qpos[i] = (real)qpos[i];
  for (int i = 0; i < NV; i++) { d->qvel[i] = (real)qvel[i]; d->qacc_warmstart[i] = (real)qws[i]; }
  for (int i = 0; i < NU; i++) d->ctrl[i] = (real)ctrl[i];
  for (int s = 0; s < nsteps; s++) step(m, d);
  for (int i = 0; i < NQ; i++) qpos[i] = (double)d->qpos[i];
  for (int i = 0; i < NV; i++) { qvel[i] = (double)d->qvel[i]; qws[i] = (double)d->qacc_warmstart[i]; }
  if (pipe) {
    real p[PP3_PIPE_STRIDE];
    write_pipeline(m, d, p);
    for (int k = 0; k < PP3_PIPE_STRIDE; k++) pipe[k] = (double)p[k];
  }
  if (site_xpos_out)
    for (int s = 0; s < m->nsite; s++)
      for (int k = 0; k < 3; k++) site_xpos_out[3 * s + k] = (double)d->site_xpos[s][k];
  free(m);
  free(d);
}

/* mj_forward only (no integration); returns M, qacc_smooth, qacc, nefc for diagnostics. */
void orc_mj_forward(const pp3_model_t* mm, const double* qpos, const double* qvel, const double* qws, const double* ctrl,
                    double* M_out, double* qacc_smooth_out, double* qacc_out, double* qfrc_bias_out, int* nefc_out,
                    double* pipe) {
  Model* m = (Model*)malloc(sizeof(Model));
  Data* d = (Data*)calloc(1, sizeof(Data));
  model_from_abi(m, mm, NULL);
  for (int i = 0; i < NQ; i++) d->qpos[i] = (real)qpos[i];
  for (int i = 0; i < NV; i++) { d->qvel[i] = (real)qvel[i]; d->qacc_warmstart[i] = (real)qws[i]; }
  for (int i = 0; i < NU; i++) d->ctrl[i] = (real)ctrl[i];
  forward(m, d);
  if (M_out) for (int i = 0; i < NV; i++) for (int j = 0; j < NV; j++) M_out[i * NV + j] = (double)d->M[i][j];
  if (qacc_smooth_out) for (int i = 0; i < NV; i++) qacc_smooth_out[i] = (double)d->qacc_smooth[i];
  if (qacc_out) for (int i = 0; i < NV; i++) qacc_out[i] = (double)d->qacc[i];
  if (qfrc_bias_out) for (int i = 0; i < NV; i++) qfrc_bias_out[i] = (double)d->qfrc_bias[i];
  if (nefc_out) *nefc_out = d->nefc;
  if (pipe) {
    real p[PP3_PIPE_STRIDE];
    write_pipeline(m, d, p);
    for (int k = 0; k < PP3_PIPE_STRIDE; k++) pipe[k] = (double)p[k];
  }
  free(m);
  free(d);
}

/* ================================ environment ================================ */
/* brax.math restated (float32 in the reference; REAL here) */
static void b_rotate(real r[3], const real v[3], const real q[4]) {
  /* r = 2 (u.v) u + (s^2 - u.u) v + 2 s (u x v) */
  real s = q[0], u[3] = {q[1], q[2], q[3]}, c[3];
  real uv = dot3(u, v), uu = dot3(u, u);
  cross3(c, u, v);
  for (int k = 0; k < 3; k++) r[k] = 2 * uv * u[k] + (s * s - uu) * v[k] + 2 * s * c[k];
}
static void b_quat_inv(real r[4], const real q[4]) { r[0] = q[0]; r[1] = -q[1]; r[2] = -q[2]; r[3] = -q[3]; }

typedef struct {
  Model m;
  pp3_env_config_t c;
  int stride, imu_off, La, Li, H;
} Env;

/* sample_command (environment.py:246-272) */
static void sample_command(const Env* e, key_t2 rng, real cmd[3]) {
  key_t2 k1 = split_i(rng, 6, 1), k2 = split_i(rng, 6, 2), k3 = split_i(rng, 6, 3);
  key_t2 k4 = split_i(rng, 6, 4), k5 = split_i(rng, 6, 5);
  const pp3_env_config_t* c = &e->c;
  float vx = uniform_i(k1, 1, 0, (float)c->lin_vel_x_range[0], (float)c->lin_vel_x_range[1]);
  float vy = uniform_i(k2, 1, 0, (float)c->lin_vel_y_range[0], (float)c->lin_vel_y_range[1]);
  float wz = uniform_i(k3, 1, 0, (float)c->ang_vel_range[0], (float)c->ang_vel_range[1]);
  float pz = uniform_i(k4, 1, 0, 0.0f, 1.0f);
  float thr = (float)c->stand_still_command_threshold;
  if (pz < (float)c->zero_command_probability) {
    for (int i = 0; i < 3; i++) cmd[i] = uniform_i(k5, 3, i, -thr, thr);
  } else {
    cmd[0] = vx; cmd[1] = vy; cmd[2] = wz;
  }
}

/* sample_body_orientation (environment.py:274-298), brax math.euler_to_quat in degrees */
static void sample_orientation(const Env* e, key_t2 rng, real out[3]) {
  key_t2 kp = split_i(rng, 3, 1), kr = split_i(rng, 3, 2);
  float pitch = uniform_i(kp, 1, 0, -1.0f, 1.0f) * (float)e->c.max_pitch_command;
  float roll = uniform_i(kr, 1, 0, -1.0f, 1.0f) * (float)e->c.max_roll_command;
  real v[3] = {roll, pitch, 0};
  real pi = (real)3.14159265358979323846;
  real c1 = RCOS(v[0] * pi / 360), c2 = RCOS(v[1] * pi / 360), c3 = RCOS(v[2] * pi / 360);
  real s1 = RSIN(v[0] * pi / 360), s2 = RSIN(v[1] * pi / 360), s3 = RSIN(v[2] * pi / 360);
  real q[4] = {c1 * c2 * c3 - s1 * s2 * s3, s1 * c2 * c3 + c1 * s2 * s3, c1 * s2 * c3 - s1 * c2 * s3,
               c1 * c2 * s3 + s1 * s2 * c3};
  real dz[3] = {(real)e->c.desired_world_z[0], (real)e->c.desired_world_z[1], (real)e->c.desired_world_z[2]};
  b_rotate(out, dz, q);
}

/* _get_obs (environment.py:485-543): consumes state rng, pushes the IMU buffer, rolls history */
static void get_obs(const Env* e, const Data* d, real* st, uint32_t* rngw, real* obs) {
  const pp3_env_config_t* c = &e->c;
  real inv[4] = {1, 0, 0, 0}, angl[3] = {0, 0, 0};
  if (c->use_imu) {
    b_quat_inv(inv, d->xquat[1]);
    b_rotate(angl, d->cvel[1], inv);
  }
  key_t2 rng = {{rngw[0], rngw[1]}};
  key_t2 nr = split_i(rng, 6, 0), ka = split_i(rng, 6, 1), kg = split_i(rng, 6, 2);
  key_t2 km = split_i(rng, 6, 3), kl = split_i(rng, 6, 4), ki = split_i(rng, 6, 5);
  rngw[0] = nr.k[0];
  rngw[1] = nr.k[1];
  real imu[6];
  real g0[3] = {0, 0, -1}, g[3];
  b_rotate(g, g0, inv);
  for (int k = 0; k < 3; k++) g[k] += uniform_i(kg, 3, k, -1.0f, 1.0f) * (float)c->gravity_noise;
  real gn = RSQRT(dot3(g, g));
  for (int k = 0; k < 3; k++) {
    imu[k] = angl[k] + uniform_i(ka, 3, k, -1.0f, 1.0f) * (float)c->ang_vel_noise;
    imu[3 + k] = g[k] / gn;
  }
  /* sample_lagged_value on the [6][Li] buffer (push front, choose column) */
  real* ib = st + e->imu_off;
  int Li = e->Li;
  for (int r = 0; r < 6; r++) {
    for (int l = Li - 1; l > 0; l--) ib[r * Li + l] = ib[r * Li + l - 1];
    ib[r * Li] = imu[r];
  }
  int li = choice_idx(ki, c->imu_latency_dist, Li);
  real o[PP3_OBS_DIM];
  for (int r = 0; r < 6; r++) o[r] = ib[r * Li + li];
  for (int k = 0; k < 3; k++) { o[6 + k] = st[PP3_S_COMMAND + k]; o[9 + k] = st[PP3_S_DESIRED_Z + k]; }
  for (int j = 0; j < 12; j++) {
    o[12 + j] = d->qpos[7 + j] - (real)c->default_pose[j] + uniform_i(km, 12, j, -1.0f, 1.0f) * (float)c->motor_angle_noise;
    o[24 + j] = st[PP3_S_LAST_ACT + j] + uniform_i(kl, 12, j, -1.0f, 1.0f) * (float)c->last_action_noise;
  }
  for (int k = 0; k < PP3_OBS_DIM; k++) { if (o[k] < -100) o[k] = -100; if (o[k] > 100) o[k] = 100; }
  int H = e->H;
  for (int k = PP3_OBS_DIM * H - 1; k >= PP3_OBS_DIM; k--) obs[k] = obs[k - PP3_OBS_DIM];
  for (int k = 0; k < PP3_OBS_DIM; k++) obs[k] = o[k];
}

static void env_setup(Env* e, const pp3_model_t* mm, const pp3_env_config_t* cfg, const double* dr) {
  real drr[PP3_NDR];
  if (dr) for (int k = 0; k < PP3_NDR; k++) drr[k] = (real)dr[k];
  model_from_abi(&e->m, mm, dr ? drr : NULL);
  e->c = *cfg;
  e->La = cfg->latency_len;
  e->Li = cfg->imu_latency_len;
  e->H = cfg->obs_history;
  e->imu_off = PP3_S_ACT_BUF + 12 * e->La;
  e->stride = e->imu_off + 6 * e->Li;
  e->m.timestep = (real)mm->timestep;
  if (cfg->ncon_max > 0) e->m.ncon_max = cfg->ncon_max;
  g_partitionable = cfg->rng_partitionable;
}

/* reset(rng) (environment.py:314-346).  state: double[stride]; obs: double[36H]; outputs
 * reward/done/metrics zeroed like the reference. */
void orc_env_reset(const pp3_model_t* mm, const pp3_env_config_t* cfg, const double* dr, const uint32_t key[2],
                   double* state, double* obs, double* reward, double* done, double* metrics, double* pipe) {
  Env* e = (Env*)malloc(sizeof(Env));
  Data* d = (Data*)calloc(1, sizeof(Data));
  env_setup(e, mm, cfg, dr);
  real* st = (real*)calloc(e->stride, sizeof(real));
  real* ob = (real*)calloc(PP3_OBS_DIM * e->H, sizeof(real));
  key_t2 rng = {{key[0], key[1]}};
  key_t2 rng0 = split_i(rng, 4, 0), kcmd = split_i(rng, 4, 1), kori = split_i(rng, 4, 2), kpos = split_i(rng, 4, 3);
  /* randomize_qpos (domain_randomization.py:188-210) on the home keyframe with default_pose */
  for (int i = 0; i < NQ; i++) d->qpos[i] = (real)mm->key_qpos[i];
  for (int j = 0; j < 12; j++) d->qpos[7 + j] = (real)cfg->default_pose[j];
  key_t2 kp = split_i(kpos, 3, 1), ky = split_i(kpos, 3, 2);
  for (int k = 0; k < 3; k++) d->qpos[k] = uniform_i(kp, 3, k, (float)cfg->start_pos_min[k], (float)cfg->start_pos_max[k]);
  float yaw = uniform_i(ky, 1, 0, -3.14159265358979323846f, 3.14159265358979323846f);
  d->qpos[3] = RCOS((real)yaw / 2); d->qpos[4] = 0; d->qpos[5] = 0; d->qpos[6] = RSIN((real)yaw / 2);
  /* pipeline_init: mjx.forward at (q, qd=0, ctrl=0) from make_data (qacc_warmstart=0) */
  forward(&e->m, d);
  for (int i = 0; i < NQ; i++) st[PP3_S_QPOS + i] = d->qpos[i];
  for (int i = 0; i < NV; i++) { st[PP3_S_QVEL + i] = d->qvel[i]; st[PP3_S_QACC_WS + i] = d->qacc_warmstart[i]; }
  uint32_t rngw[2] = {rng0.k[0], rng0.k[1]};
  real cmd[3], dz[3];
  sample_command(e, kcmd, cmd);
  sample_orientation(e, kori, dz);
  for (int k = 0; k < 3; k++) { st[PP3_S_COMMAND + k] = cmd[k]; st[PP3_S_DESIRED_Z + k] = dz[k]; }
  for (int l = 0; l < e->Li; l++) st[e->imu_off + 5 * e->Li + l] = -1; /* gravity z row */
  get_obs(e, d, st, rngw, ob);
  for (int k = 0; k < e->stride; k++) state[k] = (double)st[k];
  state[PP3_S_RNG] = (double)rngw[0];
  state[PP3_S_RNG + 1] = (double)rngw[1];
  for (int k = 0; k < PP3_OBS_DIM * e->H; k++) obs[k] = (double)ob[k];
  *reward = 0;
  *done = 0;
  for (int k = 0; k < PP3_NMETRIC; k++) metrics[k] = 0;
  if (pipe) {
    real p[PP3_PIPE_STRIDE];
    write_pipeline(&e->m, d, p);
    for (int k = 0; k < PP3_PIPE_STRIDE; k++) pipe[k] = (double)p[k];
  }
  free(st); free(ob); free(e); free(d);
}

static void env_step_impl(const Env* e, Data* d, real* st, uint32_t* rngw, real* ob, const double* action, double* reward,
                          double* done, double* metrics, double* pipe) {
  const pp3_env_config_t* c = &e->c;
  const Model* m = &e->m;
  real dt = (real)c->dt;
  for (int i = 0; i < NQ; i++) d->qpos[i] = st[PP3_S_QPOS + i];
  for (int i = 0; i < NV; i++) { d->qvel[i] = st[PP3_S_QVEL + i]; d->qacc_warmstart[i] = st[PP3_S_QACC_WS + i]; }
  key_t2 rng = {{rngw[0], rngw[1]}};
  key_t2 r0 = split_i(rng, 5, 0), kcmd = split_i(rng, 5, 1), kkick = split_i(rng, 5, 2);
  key_t2 kbern = split_i(rng, 5, 3), klat = split_i(rng, 5, 4);
  rngw[0] = r0.k[0];
  rngw[1] = r0.k[1];
  /* kick (environment.py:352-356) */
  float bern = uniform_i(kbern, 1, 0, 0.0f, 1.0f) < (float)c->kick_probability ? 1.0f : 0.0f;
  float kick[2];
  for (int k = 0; k < 2; k++) {
    kick[k] = uniform_i(kkick, 2, k, -1.0f, 1.0f) * (float)c->kick_vel * bern;
    d->qvel[k] += kick[k];
  }
  /* action latency (utils.py:49-69) */
  int La = e->La;
  real* ab = st + PP3_S_ACT_BUF;
  for (int r = 0; r < 12; r++) {
    for (int l = La - 1; l > 0; l--) ab[r * La + l] = ab[r * La + l - 1];
    ab[r * La] = (real)action[r];
  }
  int li = choice_idx(klat, c->latency_dist, La);
  for (int j = 0; j < 12; j++) {
    real t = (real)c->default_pose[j] + ab[j * La + li] * (real)c->action_scale;
    if (t < (real)c->joint_lower[j]) t = (real)c->joint_lower[j];
    if (t > (real)c->joint_upper[j]) t = (real)c->joint_upper[j];
    d->ctrl[j] = t;
  }
  /* physics: n_frames x mj_step; x/xd/site/contacts are those of the last forward */
  for (int f = 0; f < c->n_frames; f++) step(m, d);
  for (int i = 0; i < NQ; i++) st[PP3_S_QPOS + i] = d->qpos[i];
  for (int i = 0; i < NV; i++) { st[PP3_S_QVEL + i] = d->qvel[i]; st[PP3_S_QACC_WS + i] = d->qacc_warmstart[i]; }
  /* observation (uses pre-update last_act / command) */
  get_obs(e, d, st, rngw, ob);
  /* brax x/xd of bodies (index b-1) */
  real xdv[NB][3], xda[NB][3];
  for (int b = 1; b < NB; b++) {
    real off[3], v[3];
    for (int k = 0; k < 3; k++) off[k] = d->xpos[b][k] - d->com[k];
    cross3(v, d->cvel[b], off);
    for (int k = 0; k < 3; k++) { xdv[b][k] = d->cvel[b][3 + k] + v[k]; xda[b][k] = d->cvel[b][k]; }
  }
  /* foot contacts (environment.py:374-381) */
  int contact[4], filt_mm[4], filt_cm[4];
  real first[4];
  for (int f = 0; f < 4; f++) {
    real cz = d->site_xpos[c->feet_site[f]][2] - (real)c->foot_radius;
    int last = st[PP3_S_LAST_CONTACT + f] != 0;
    contact[f] = cz < (real)1e-3;
    filt_mm[f] = contact[f] | last;
    filt_cm[f] = (cz < (real)3e-2) | last;
    first[f] = (st[PP3_S_AIR_TIME + f] > 0) && filt_mm[f] ? 1 : 0;
    st[PP3_S_AIR_TIME + f] += dt;
  }
  /* done (environment.py:383-388) */
  int tb = c->torso_body;
  real up[3] = {0, 0, 1}, ru[3];
  b_rotate(ru, up, d->xquat[tb]);
  int isdone = dot3(ru, up) < (real)cos(c->terminal_body_angle);
  for (int j = 0; j < 12; j++) {
    if (d->qpos[7 + j] < (real)c->joint_lower[j]) isdone = 1;
    if (d->qpos[7 + j] > (real)c->joint_upper[j]) isdone = 1;
  }
  if (d->xpos[tb][2] < (real)c->terminal_body_z) isdone = 1;
  /* rewards (rewards.py) */
  real rw[PP3_NREWARD];
  real inv[4], cmd[3], sig = (real)c->tracking_sigma;
  b_quat_inv(inv, d->xquat[1]);
  for (int k = 0; k < 3; k++) cmd[k] = st[PP3_S_COMMAND + k];
  real lv[3], av[3], wz[3], z0[3] = {0, 0, 1};
  b_rotate(lv, xdv[1], inv);
  b_rotate(av, xda[1], inv);
  b_rotate(wz, z0, inv);
  real e0 = (cmd[0] - lv[0]) * (cmd[0] - lv[0]) + (cmd[1] - lv[1]) * (cmd[1] - lv[1]);
  rw[PP3_REWARD_TRACKING_LIN_VEL] = REXP(-e0 / sig);
  rw[PP3_REWARD_TRACKING_ANG_VEL] = REXP(-(cmd[2] - av[2]) * (cmd[2] - av[2]) / sig);
  real eo = 0;
  for (int k = 0; k < 3; k++) eo += (wz[k] - st[PP3_S_DESIRED_Z + k]) * (wz[k] - st[PP3_S_DESIRED_Z + k]);
  rw[PP3_REWARD_TRACKING_ORIENTATION] = REXP(-eo / sig);
  rw[PP3_REWARD_LIN_VEL_Z] = xdv[1][2] * xdv[1][2];
  rw[PP3_REWARD_ANG_VEL_XY] = xda[1][0] * xda[1][0] + xda[1][1] * xda[1][1];
  real rup[3];
  b_rotate(rup, z0, d->xquat[1]);
  rw[PP3_REWARD_ORIENTATION] = rup[0] * rup[0] + rup[1] * rup[1];
  real tq = 0;
  for (int i = 0; i < NV; i++) tq += d->qfrc_actuator[i] * d->qfrc_actuator[i];
  rw[PP3_REWARD_TORQUES] = tq;
  real ja = 0, mw = 0, ar = 0, ssa = 0, ssv = 0, abd = 0;
  for (int j = 0; j < 12; j++) {
    real jv = d->qvel[6 + j];
    real acc = (jv - st[PP3_S_LAST_VEL + j]) / (real)c->env_dt;
    ja += acc * acc;
    mw += RFABS(d->qfrc_actuator[6 + j] * jv);
    real da = (real)action[j] - st[PP3_S_LAST_ACT + j];
    ar += da * da;
    ssa += RFABS(d->qpos[7 + j] - (real)c->default_pose[j]);
    ssv += RFABS(jv);
  }
  for (int l = 0; l < 4; l++) {
    real t = d->qpos[7 + 3 * l + 1] - (real)c->desired_abduction[l];
    abd += t * t;
  }
  real cn = RSQRT(cmd[0] * cmd[0] + cmd[1] * cmd[1] + cmd[2] * cmd[2]);
  rw[PP3_REWARD_JOINT_ACCELERATION] = ja;
  rw[PP3_REWARD_MECHANICAL_WORK] = mw;
  rw[PP3_REWARD_ACTION_RATE] = ar;
  rw[PP3_REWARD_STAND_STILL] = ssa * (cn < (real)0.1 ? 1 : 0);
  rw[PP3_REWARD_STAND_STILL_JOINT_VELOCITY] = ssv * (cn < (real)c->stand_still_command_threshold ? 1 : 0);
  rw[PP3_REWARD_ABDUCTION_ANGLE] = abd;
  real fat = 0;
  for (int f = 0; f < 4; f++) fat += (st[PP3_S_AIR_TIME + f] - (real)0.1) * first[f];
  rw[PP3_REWARD_FEET_AIR_TIME] = fat * (cn > (real)0.05 ? 1 : 0);
  real slip = 0;
  for (int f = 0; f < 4; f++) {
    int b = c->lower_leg_body[f];
    real off[3], v[3];
    for (int k = 0; k < 3; k++) off[k] = d->site_xpos[c->feet_site[f]][k] - d->xpos[b][k];
    cross3(v, xda[b], off);
    real vx = xdv[b][0] + v[0], vy = xdv[b][1] + v[1];
    slip += (vx * vx + vy * vy) * (filt_cm[f] ? 1 : 0);
  }
  rw[PP3_REWARD_FOOT_SLIP] = slip;
  int stepc = (int)st[PP3_S_STEP];
  rw[PP3_REWARD_TERMINATION] = (isdone && stepc < c->early_termination_step_threshold) ? 1 : 0;
  real knee = 0, bodyc = 0;
  for (int k = 0; k < d->ncon; k++) {
    if (!(d->con[k].dist < 0)) continue;
    int ga = m->cg_id[d->con[k].g1], gb = m->cg_id[d->con[k].g2];
    for (int i = 0; i < c->n_upper_leg_geoms; i++) {
      int id = c->upper_leg_geoms[i];
      if (ga == id || gb == id) knee += 1;
    }
    for (int i = 0; i < c->n_torso_geoms; i++) {
      int id = c->torso_geoms[i];
      if (ga == id || gb == id) bodyc += 1;
    }
  }
  rw[PP3_REWARD_KNEE_COLLISION] = knee;
  rw[PP3_REWARD_BODY_COLLISION] = bodyc;
  real sum = 0;
  for (int k = 0; k < PP3_NREWARD; k++) {
    rw[k] *= (real)c->reward_scales[k];
    sum += rw[k];
  }
  real rew = sum * dt;
  if (rew < 0) rew = 0;
  if (rew > 10000) rew = 10000;
  /* state management (environment.py:448-482) */
  for (int k = 0; k < 2; k++) st[PP3_S_KICK + k] = kick[k];
  for (int j = 0; j < 12; j++) { st[PP3_S_LAST_ACT + j] = (real)action[j]; st[PP3_S_LAST_VEL + j] = d->qvel[6 + j]; }
  for (int f = 0; f < 4; f++) {
    if (filt_mm[f]) st[PP3_S_AIR_TIME + f] = 0;
    st[PP3_S_LAST_CONTACT + f] = contact[f] ? 1 : 0;
  }
  stepc += 1;
  if (stepc > c->resample_velocity_step) {
    real nc[3], nz[3];
    sample_command(e, kcmd, nc);
    sample_orientation(e, kcmd, nz);
    for (int k = 0; k < 3; k++) { st[PP3_S_COMMAND + k] = nc[k]; st[PP3_S_DESIRED_Z + k] = nz[k]; }
  }
  if (isdone || stepc > c->resample_velocity_step) stepc = 0;
  st[PP3_S_STEP] = (real)stepc;
  *reward = (double)rew;
  *done = isdone ? 1.0 : 0.0;
  metrics[0] = (double)RSQRT(d->xpos[tb][0] * d->xpos[tb][0] + d->xpos[tb][1] * d->xpos[tb][1] + d->xpos[tb][2] * d->xpos[tb][2]);
  for (int k = 0; k < PP3_NREWARD; k++) metrics[1 + k] = (double)rw[k];
  if (pipe) {
    real p[PP3_PIPE_STRIDE];
    write_pipeline(m, d, p);
    for (int f = 0; f < 4; f++)
      for (int k = 0; k < 3; k++) p[PP3_P_SITE_XPOS + 3 * f + k] = d->site_xpos[c->feet_site[f]][k];
    for (int k = 0; k < PP3_PIPE_STRIDE; k++) pipe[k] = (double)p[k];
  }
}

/* step(state, action) for one env (double I/O). */
void orc_env_step(const pp3_model_t* mm, const pp3_env_config_t* cfg, const double* dr, double* state, double* obs,
                  const double* action, double* reward, double* done, double* metrics, double* pipe) {
  Env* e = (Env*)malloc(sizeof(Env));
  Data* d = (Data*)calloc(1, sizeof(Data));
  env_setup(e, mm, cfg, dr);
  real* st = (real*)malloc(sizeof(real) * e->stride);
  real* ob = (real*)malloc(sizeof(real) * PP3_OBS_DIM * e->H);
  for (int k = 0; k < e->stride; k++) st[k] = (real)state[k];
  for (int k = 0; k < PP3_OBS_DIM * e->H; k++) ob[k] = (real)obs[k];
  uint32_t rngw[2] = {(uint32_t)state[PP3_S_RNG], (uint32_t)state[PP3_S_RNG + 1]};
  env_step_impl(e, d, st, rngw, ob, action, reward, done, metrics, pipe);
  for (int k = 0; k < e->stride; k++) state[k] = (double)st[k];
  state[PP3_S_RNG] = (double)rngw[0];
  state[PP3_S_RNG + 1] = (double)rngw[1];
  for (int k = 0; k < PP3_OBS_DIM * e->H; k++) obs[k] = (double)ob[k];
  free(st); free(ob); free(e); free(d);
}

/* Batched rollout for the CPU baseline: n envs x nsteps, actions[nsteps][n][12] (or NULL =
 * zeros), OpenMP over envs.  Returns the number of threads used. */
int orc_env_rollout(const pp3_model_t* mm, const pp3_env_config_t* cfg, int n, int nsteps, double* states,
                    double* obs, const double* actions, double* rewards, int nthreads) {
  Env* e = (Env*)malloc(sizeof(Env));
  env_setup(e, mm, cfg, NULL);
  int used = 1;
#if defined(_OPENMP)
  if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel
  {
#pragma omp single
    used = omp_get_num_threads();
  }
#pragma omp parallel for schedule(dynamic, 1)
#endif
  for (int i = 0; i < n; i++) {
    Data* d = (Data*)calloc(1, sizeof(Data));
    real* st = (real*)malloc(sizeof(real) * e->stride);
    real* ob = (real*)malloc(sizeof(real) * PP3_OBS_DIM * e->H);
    for (int k = 0; k < e->stride; k++) st[k] = (real)states[(size_t)i * e->stride + k];
    for (int k = 0; k < PP3_OBS_DIM * e->H; k++) ob[k] = (real)obs[(size_t)i * PP3_OBS_DIM * e->H + k];
    uint32_t rngw[2] = {(uint32_t)states[(size_t)i * e->stride + PP3_S_RNG], (uint32_t)states[(size_t)i * e->stride + PP3_S_RNG + 1]};
    double zero[12] = {0};
    for (int s = 0; s < nsteps; s++) {
      double rew, dn, met[PP3_NMETRIC];
      const double* a = actions ? actions + ((size_t)s * n + i) * 12 : zero;
      env_step_impl(e, d, st, rngw, ob, a, &rew, &dn, met, NULL);
      if (rewards) rewards[(size_t)s * n + i] = rew;
    }
    for (int k = 0; k < e->stride; k++) states[(size_t)i * e->stride + k] = (double)st[k];
    states[(size_t)i * e->stride + PP3_S_RNG] = (double)rngw[0];
    states[(size_t)i * e->stride + PP3_S_RNG + 1] = (double)rngw[1];
    for (int k = 0; k < PP3_OBS_DIM * e->H; k++) obs[(size_t)i * PP3_OBS_DIM * e->H + k] = (double)ob[k];
    free(st); free(ob); free(d);
  }
  free(e);
  return used;
}

void orc_set_ncon_max(int n) { g_ncon_max = n; }
void orc_set_ls_noise(int on) { g_ls_noise = on; }
void orc_set_ls_trace(int on) { g_ls_trace = on; }
/* line-search evaluations and searches of this thread since the last call */
void orc_ls_take(long* out) {
  out[0] = g_ls_total; out[1] = g_ls_calls; out[2] = g_ls_smooth; out[3] = g_ls_starts;
  out[4] = g_ls_exit[LS_CONVERGED]; out[5] = g_ls_exit[LS_CAPPED]; out[6] = g_ls_exit[LS_STALLED];
  out[7] = g_ls_bracket; out[8] = g_ls_cap_bracket;
  g_ls_total = 0; g_ls_calls = 0; g_ls_smooth = 0; g_ls_starts = 0;
  g_ls_exit[0] = g_ls_exit[1] = g_ls_exit[2] = 0;
  g_ls_bracket = 0; g_ls_cap_bracket = 0;
}
void orc_debug_read(double* out) { memcpy(out, g_dbg, sizeof(g_dbg)); }
int orc_boundary_take(void) { const int n = g_boundary; g_boundary = 0; return n; }

/* RNG test hooks */
void orc_set_partitionable(int p) { g_partitionable = p; }
void orc_split(const uint32_t key[2], int n, uint32_t* out) {
  key_t2 k = {{key[0], key[1]}};
  for (int i = 0; i < n; i++) { key_t2 r = split_i(k, n, i); out[2 * i] = r.k[0]; out[2 * i + 1] = r.k[1]; }
}
void orc_uniform(const uint32_t key[2], int n, float lo, float hi, float* out) {
  key_t2 k = {{key[0], key[1]}};
  for (int i = 0; i < n; i++) out[i] = uniform_i(k, n, i, lo, hi);
}
int orc_choice(const uint32_t key[2], const double* p, int n) {
  key_t2 k = {{key[0], key[1]}};
  return choice_idx(k, p, n);
}
