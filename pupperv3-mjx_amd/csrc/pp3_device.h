// pp3_device.h -- device-side model layout and small math/RNG helpers for the
// MI355X (gfx950) Pupper-v3 environment kernels.  fp32 throughout.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "pupper_hip.h"

namespace pp3 {

constexpr int NB = PP3_NBODY;
constexpr int NJ = PP3_NJNT;
constexpr int NV = PP3_NV;
constexpr int NQ = PP3_NQ;
constexpr int NU = PP3_NU;
constexpr int WAVE = 64;
constexpr int NLMAX = 12;                 // joint-limit rows: one side per hinge at a time (checked at pp3_create)
constexpr int NFR = 12;                   // frictionloss rows (hinge dofs)
constexpr int MAX_ROBOT_GEOM = 16;        // DevModel table size for collidable geoms on moving bodies
constexpr int NMPAIR_MAX = 128;           // nonzero (i, j<=i) entries of M
constexpr int NMPAIR = 117;               // ... for the 13-body quadruped tree (21 base + 4 x 24 leg)
constexpr int PAIR_REC = 24;              // floats per flattened collision-pair record

// Flattened narrow-phase record of one candidate pair (host precomputed, one 96-byte row per
// pair so a lane fetches everything with six 16-byte loads): kind, robot-geom slots (-1 =
// static), radii, margin, static positions, static frame (plane / box), box half sizes.
enum { PK_PLANE_SPHERE = 0, PK_SPHERE_SPHERE = 1, PK_SPHERE_BOX = 2 };
struct alignas(16) PairRec {
  int32_t kind, s1, s2;
  float r1, r2, margin;
  float p1[3], p2[3];
  float R[9];
  float half[3];
};
static_assert(sizeof(PairRec) == PAIR_REC * 4, "PairRec layout");
// One per-env terrain box (host packed from pos/quat/half): world centre, world rotation
// (row-major), half sizes; 64 bytes = four 16-byte loads.
struct alignas(16) TerrainRec {
  float p[3];
  float R[9];
  float half[3];
  float pad;
};
static_assert(sizeof(TerrainRec) == 64, "TerrainRec layout");
// Contact-side constants of a candidate pair (host precomputed, 64 bytes): what store_contact
// and the contact constraint rows read by pair index, fetched with four 16-byte loads.
struct alignas(16) PairCon {
  int32_t sup;       // Jacobian column support (pair_sup)
  uint32_t dm[2];    // dof masks of the two bodies
  float mu;          // friction (mj_contactParam)
  float tran;        // body_invweight0 translational sum
  float margin, b, k;
  float solimp[5];   // clamped
  float knee, body;  // rewards.py geom_collision counts: knee / torso geoms among the pair's two
  float pad;
};
static_assert(sizeof(PairCon) == 64, "PairCon layout");
static_assert(offsetof(PairCon, knee) == 52, "PairCon: knee/body in the 4th 16-byte word group");

// Per-lane constant records: everything lane l of one phase reads from the model, flattened on
// the host so the lane fetches it with N back-to-back 16-byte loads at the top of the phase and
// one vmcnt wait (lane-indexed model reads issued one by one each cost an L1/L2 round trip).
template <int N>
struct alignas(16) LaneRec {
  float f[4 * N];
};
// The model stores a phase's 32 lane records word-group major (group k of lane l at g[k][l]):
// the wave's k-th 16-byte load then covers 512 contiguous bytes (4 cache lines) instead of
// 16-byte pieces of 32 records strided across up to 32 lines.
template <int N>
struct alignas(16) LaneTab {
  float g[N][32][4];
};
// the narrow phase's pair records, laid out the same way (lane = pair within a 32-pair batch)
struct alignas(16) PairTab {
  float g[PAIR_REC / 4][PP3_MAX_PAIR][4];
};
// phase "limits/friction/actuation": lane l < 24 = joint-limit side (j = 1 + l/2, hi side when
// l is odd), lane l < 12 = frictionloss row of dof 6+l and actuator l
enum {
  LL_LIM_ON = 0, LL_RANGE, LL_MARGIN, LL_INVW, LL_B, LL_K, LL_SOLIMP,   // solimp: 5 words
  LL_FR_R = 11, LL_FR_B, LL_ACT_DOF, LL_ACT_QADR, LL_ACT_FLAGS, LL_CRANGE,  // crange: 2 words
  LL_GEAR = 18, LL_GAIN, LL_BIAS,  // bias: 3 words
  LL_FRANGE = 23,                  // 2 words
  LL_WORDS = 25
};
enum { ACTF_CTRLLIMITED = 1, ACTF_FORCELIMITED = 2, ACTF_AFFINE = 4 };
// phase "com/cinert/cdof": body lanes 1..12 -> body_iquat; geom lanes (< nrobot_geom) and foot
// lanes (16..19) -> the point's body and body-frame position
enum { LC_IQUAT = 0, LC_PT_BODY = 4, LC_PT_POS = 5, LC_WORDS = 8 };
// phases "M entries" / "bias" / Newton: lane l holds M pairs p = l + 32 t (t < 4) packed i | j << 8
// (-1 = none) and their armature (i == j), dof l's damping, frictionloss of dof 6 + l
enum { LM_IJ = 0, LM_ARM = 4, LM_DAMP = 8, LM_FLOSS = 9, LM_WORDS = 10 };
// prologue / epilogue (env logic): lane l < 12 -> joint l's default pose, ctrl range, desired
// abduction (l % 3 == 1); lane f < 4 -> lower-leg body of foot f; lanes 16..27 -> default pose
// of joint l - 16 (the observation's lanes)
enum { LE_POSE = 0, LE_JLO, LE_JHI, LE_ABD, LE_LEG, LE_POSE16, LE_WORDS = 6 };
// pipeline record (write_pipeline), lane i < nsensor: sensor i's type, sensordata address, cutoff,
// site body, site frame in the body, and for an accelerometer the body chain root .. site body
// (per level: body, dofadr, dofnum, parent; at most LS_MAXCH levels, checked at pp3_create)
enum { LS_TYPE = 0, LS_ADR, LS_CUT, LS_BODY, LS_SPOS, LS_SQUAT = 7, LS_NCH = 11, LS_CH = 12, LS_MAXCH = 4,
       LS_WORDS = LS_CH + 4 * LS_MAXCH };

constexpr float MINVAL = 1e-15f;
constexpr float MINIMP = 0.0001f;
constexpr float MAXIMP = 0.9999f;

// fp32 model + env constants, built on the host from pp3_model_t / pp3_env_config_t.
struct DevModel {
  // ---- per-lane phase records (first: small offsets) ----
  LaneTab<(LL_WORDS + 3) / 4> lane_lim;
  LaneTab<(LC_WORDS + 3) / 4> lane_com;
  LaneTab<(LM_WORDS + 3) / 4> lane_m;
  // ---- options ----
  float h;
  float gravity[3];
  float impratio;
  float gtol_scale;  // tolerance * ls_tolerance * meaninertia * nv  (gtol = gtol_scale * |search|)
  int32_t ls_iterations;
  int32_t iterations;
  // ---- bodies ----
  float body_pos[NB][3];
  float body_quat[NB][4];
  float body_iquat[NB][4];
  float body_ipos[NB][3];
  float body_mass[NB];
  float body_inertia[NB][3];
  uint32_t body_dofmask[NB];  // dofs on the path root..body (ancestor-or-self)
  int32_t dof_body[NV];
  // ---- joints (0 = free, 1..12 hinges) ----
  float jnt_pos[NJ][3];
  float jnt_axis[NJ][3];
  float jnt_range[NJ][2];
  int32_t jnt_limited[NJ];
  float lim_k[NJ], lim_b[NJ], lim_margin[NJ], lim_invw[NJ];
  float lim_solimp[NJ][5];  // clamped
  float qpos0[NQ];
  // ---- dofs ----
  float dof_armature[NV];
  float dof_damping[NV];
  float fr_floss[NV];  // frictionloss
  float fr_R[NV];      // R of the frictionloss row (pos = 0 -> imp = dmin)
  float fr_b[NV];      // damping coefficient of its reference acceleration
  // ---- mass-matrix sparsity (j ancestor-or-self of i) ----
  int32_t nmpair;
  uint8_t mp_i[NMPAIR_MAX], mp_j[NMPAIR_MAX];
  // ---- collision geoms ----
  int32_t ncgeom;
  int32_t cg_type[PP3_MAX_CGEOM];
  int32_t cg_body[PP3_MAX_CGEOM];
  int32_t cg_id[PP3_MAX_CGEOM];
  int32_t cg_slot[PP3_MAX_CGEOM];  // slot in the per-env robot-geom table (-1 = static)
  float cg_size[PP3_MAX_CGEOM][3];
  float cg_pos[PP3_MAX_CGEOM][3];      // body frame (robot) or world frame (static)
  float cg_wmat[PP3_MAX_CGEOM][9];     // world rotation of static geoms
  int32_t nrobot_geom;
  int32_t robot_geom[MAX_ROBOT_GEOM];  // cgeom index of each slot
  int32_t npair;
  int32_t pair_g1[PP3_MAX_PAIR], pair_g2[PP3_MAX_PAIR];
  float pair_mu[PP3_MAX_PAIR];
  float pair_k[PP3_MAX_PAIR], pair_b[PP3_MAX_PAIR];
  float pair_margin[PP3_MAX_PAIR];
  float pair_tran[PP3_MAX_PAIR];       // body_invweight0 translational sum
  int32_t pair_sup[PP3_MAX_PAIR];      // Jacobian column support: leg 0..3 (+base), 4 base only, 5 dense
                                       // (leg-leg: | 8 | lower leg << 4 | higher leg << 6)
  uint32_t pair_dm[PP3_MAX_PAIR][2];   // dof masks (ancestor-or-self) of the pair's two bodies
  PairTab pair_rec;                    // PairRec of pair p, word-group major; sphere-box: s2 = -1 - (box slot)
  PairCon pair_con[PP3_MAX_PAIR];
  float pair_solimp[PP3_MAX_PAIR][5];  // clamped
  // per-env terrain (pp3_set_terrain): TerrainRec[N (padded even)][nbox], or 0 = static boxes
  uint64_t terrain;
  int32_t nbox;
  // ---- sites ----
  int32_t nsite;
  int32_t site_body[PP3_MAX_SITE];
  float site_pos[PP3_MAX_SITE][3];
  float site_quat[PP3_MAX_SITE][4];
  // ---- sensors (pipeline record only) ----
  int32_t nsensor, nsensordata;
  int32_t sensor_type[PP3_MAX_SENSOR], sensor_objid[PP3_MAX_SENSOR], sensor_adr[PP3_MAX_SENSOR];
  float sensor_cutoff[PP3_MAX_SENSOR];
  int32_t body_parent[NB], body_dofadr[NB], body_dofnum[NB];
  // ---- actuators ----
  int32_t act_dof[NU], act_qadr[NU], act_biastype[NU], act_forcelimited[NU], act_ctrllimited[NU];
  float act_gear[NU], act_gain[NU], act_bias[NU][3], act_frange[NU][2], act_crange[NU][2];
  // ---- environment (PupperV3Env kwargs) ----
  int32_t n_frames, H, La, Li, use_imu, resample_step, term_step;
  int32_t torso_body;
  int32_t feet_site[4], lower_leg_body[4];
  int32_t n_knee_geoms, knee_geoms[16], n_torso_geoms, torso_geoms[8];
  int32_t partitionable;
  int32_t stride, imu_off;
  float lat_dist[PP3_MAX_LAG], imu_lat_dist[PP3_MAX_LAG];
  float action_scale;
  float default_pose[NU], jlo[NU], jhi[NU];
  float des_abd[4];
  float start_lo[3], start_hi[3];
  float cmd_x[2], cmd_y[2], cmd_w[2];
  float zero_cmd_p, stand_thr, max_pitch, max_roll;
  float n_ang, n_grav, n_motor, n_act;
  float kick_vel, kick_p;
  float term_z, cos_term_angle, foot_radius, env_dt, dt;
  float des_z[3];
  float scales[PP3_NREWARD];
  float sigma;
  float key_qpos[NQ];
  float pi_f;
  // last: the same 1 KB inserted after lane_m (shifting every later field) measured 1.3 % slower
  LaneTab<(LE_WORDS + 3) / 4> lane_env;
  // pipeline record only (after everything the step reads)
  LaneTab<(LS_WORDS + 3) / 4> lane_sens;
  float pair_gid[PP3_MAX_PAIR][2];  // MuJoCo geom ids of the pair's two geoms (contact geom fields)
  // sphere-box cull of the narrow phase (collision): the pairs after the first 32 whose box lies
  // out of the robot's reach are not evaluated.  Exact: such a pair cannot come within its
  // margin, so the narrow phase would return no contact for it (the contact set is unchanged)
  int32_t cull_on;            // 1 <= nbox <= 32, 32 < npair <= 160, every robot geom below body 1
  float cull_reach;           // >= |sphere centre - body-1 origin| + radius + margin, + 1 cm slack
  uint32_t pair_box4[32];     // lane l, byte k: box slot of pair 32 (k + 1) + l (0xFF: not sphere-box)
  TerrainRec box_tab[32];     // static boxes by slot, in the per-env terrain row layout
};

// ------------------------------- float helpers -------------------------------
__device__ __forceinline__ float rlane(float v, int l) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
}
// Wave-wide reductions on the DPP network (no LDS round trips): butterfly
// within each 16-lane row (quad_perm, row_half_mirror, row_mirror), then
// row_bcast:15 / row_bcast:31 fold the four rows into lane 63, which is
// read back as a wave-uniform scalar.
template <int CTRL, int ROWMASK>
__device__ __forceinline__ float dpp_f(float v, float old) {
  return __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(old), __float_as_int(v), CTRL,
                                                    ROWMASK, 0xF, false));
}
__device__ __forceinline__ float lane63(float v) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 63));
}
__device__ __forceinline__ float wave_sum(float v) {
  v += dpp_f<0xB1, 0xF>(v, 0.0f);   // quad_perm [1,0,3,2]
  v += dpp_f<0x4E, 0xF>(v, 0.0f);   // quad_perm [2,3,0,1]
  v += dpp_f<0x141, 0xF>(v, 0.0f);  // row_half_mirror
  v += dpp_f<0x140, 0xF>(v, 0.0f);  // row_mirror
  v += dpp_f<0x142, 0xA>(v, 0.0f);  // row_bcast:15 -> rows 1,3
  v += dpp_f<0x143, 0xC>(v, 0.0f);  // row_bcast:31 -> rows 2,3
  return lane63(v);
}
__device__ __forceinline__ float wave_min(float v) {
  v = fminf(v, dpp_f<0xB1, 0xF>(v, v));
  v = fminf(v, dpp_f<0x4E, 0xF>(v, v));
  v = fminf(v, dpp_f<0x141, 0xF>(v, v));
  v = fminf(v, dpp_f<0x140, 0xF>(v, v));
  v = fminf(v, dpp_f<0x142, 0xA>(v, v));
  v = fminf(v, dpp_f<0x143, 0xC>(v, v));
  return lane63(v);
}
__device__ __forceinline__ void quat2mat(const float q[4], float R[9]) {
  float w = q[0], x = q[1], y = q[2], z = q[3];
  R[0] = 1 - 2 * (y * y + z * z); R[1] = 2 * (x * y - w * z); R[2] = 2 * (x * z + w * y);
  R[3] = 2 * (x * y + w * z); R[4] = 1 - 2 * (x * x + z * z); R[5] = 2 * (y * z - w * x);
  R[6] = 2 * (x * z - w * y); R[7] = 2 * (y * z + w * x); R[8] = 1 - 2 * (x * x + y * y);
}
__device__ __forceinline__ void mulquat(float r[4], const float a[4], const float b[4]) {
  float t0 = a[0] * b[0] - a[1] * b[1] - a[2] * b[2] - a[3] * b[3];
  float t1 = a[0] * b[1] + a[1] * b[0] + a[2] * b[3] - a[3] * b[2];
  float t2 = a[0] * b[2] - a[1] * b[3] + a[2] * b[0] + a[3] * b[1];
  float t3 = a[0] * b[3] + a[1] * b[2] - a[2] * b[1] + a[3] * b[0];
  r[0] = t0; r[1] = t1; r[2] = t2; r[3] = t3;
}
__device__ __forceinline__ void matvec(float r[3], const float R[9], const float v[3]) {
  float t0 = R[0] * v[0] + R[1] * v[1] + R[2] * v[2];
  float t1 = R[3] * v[0] + R[4] * v[1] + R[5] * v[2];
  float t2 = R[6] * v[0] + R[7] * v[1] + R[8] * v[2];
  r[0] = t0; r[1] = t1; r[2] = t2;
}
__device__ __forceinline__ void cross3(float r[3], const float a[3], const float b[3]) {
  float t0 = a[1] * b[2] - a[2] * b[1];
  float t1 = a[2] * b[0] - a[0] * b[2];
  float t2 = a[0] * b[1] - a[1] * b[0];
  r[0] = t0; r[1] = t1; r[2] = t2;
}
__device__ __forceinline__ float dot3(const float a[3], const float b[3]) {
  return a[0] * b[0] + a[1] * b[1] + a[2] * b[2];
}
__device__ __forceinline__ void normalize4(float q[4]) {
  float n = sqrtf(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
  if (n < MINVAL) { q[0] = 1; q[1] = q[2] = q[3] = 0; }
  else { float i = 1.0f / n; q[0] *= i; q[1] *= i; q[2] *= i; q[3] *= i; }
}
// sincosf restricted to |x| < 2^17: the device library's own small-argument path, operation for
// operation (Cody-Waite reduction by pi/2 in three parts, its sin / cos polynomials, the quadrant
// signs), so the results are bit-identical there (tools/sincos_check.hip) -- without the
// Payne-Hanek branch for larger arguments, whose dead code and hoisted constants the library call
// leaves in every caller.  Joint half-angles never come near 2^17 (beyond it the reduction loses
// accuracy instead); non-finite arguments give NaN as sincosf does.
__device__ __forceinline__ void sincos_f32(float x, float* sp, float* cp) {
  const float ax = __builtin_fabsf(x);
  const float n = __builtin_rintf(ax * 0x1.45f306p-1f);  // x 2/pi
  const int q = (int)n;
  float r = __builtin_fmaf(n, -0x1.921fb4p+0f, ax);
  r = __builtin_fmaf(n, -0x1.4442d0p-24f, r);
  r = __builtin_fmaf(n, -0x1.846988p-48f, r);
  const float x2 = r * r;
  float ps = __builtin_fmaf(-0x1.983304p-13f, x2, 0x1.110388p-7f);
  ps = __builtin_fmaf(x2, ps, -0x1.55553ap-3f);
  ps = x2 * ps;
  const float sr = __builtin_fmaf(r, ps, r);
  float pc = __builtin_fmaf(0x1.aea668p-16f, x2, -0x1.6c9e76p-10f);
  pc = __builtin_fmaf(x2, pc, 0x1.5557eep-5f);
  pc = __builtin_fmaf(x2, pc, -0x1.000008p-1f);
  const float cr = __builtin_fmaf(x2, pc, 1.0f);
  const bool odd = (q & 1) != 0;
  const uint32_t qs = ((uint32_t)q << 30) & 0x80000000u;  // quadrants 2, 3: both signs flip
  const float sv = odd ? cr : sr, cv = odd ? -sr : cr;
  const float s = __uint_as_float(__float_as_uint(sv) ^ (__float_as_uint(x) & 0x80000000u) ^ qs);
  const float c = __uint_as_float(__float_as_uint(cv) ^ qs);
  const bool fin = __builtin_isfinite(x);
  *sp = fin ? s : __builtin_nanf("");
  *cp = fin ? c : __builtin_nanf("");
}
// branch-free (sincos(0) = (0, 1) exactly gives mju_axisAngle2Quat's angle == 0 case); an early
// return here made the result array a dynamically indexed private array (scratch memory).  LIB:
// the library's sincosf; else sincos_f32 (the same values; the single-step kernel, where it removes
// the VGPR spills and is 0.8 % faster, while the fused kernel measured 0.3 % slower with it:
// profiles/AB_LOG.md round 6)
template <bool LIB = true>
__device__ __forceinline__ void axisangle2quat(float r[4], const float a[3], float ang) {
  float s, c;
  if constexpr (LIB) sincosf(0.5f * ang, &s, &c);
  else sincos_f32(0.5f * ang, &s, &c);
  r[0] = c; r[1] = a[0] * s; r[2] = a[1] * s; r[3] = a[2] * s;
}
// spatial inertia (10-vector about the root subtree com) times a motion vector
__device__ __forceinline__ void mul_inert_vec(float r[6], const float* i, const float* v) {
  r[0] = i[0] * v[0] + i[3] * v[1] + i[4] * v[2] - i[8] * v[4] + i[7] * v[5];
  r[1] = i[3] * v[0] + i[1] * v[1] + i[5] * v[2] + i[8] * v[3] - i[6] * v[5];
  r[2] = i[4] * v[0] + i[5] * v[1] + i[2] * v[2] - i[7] * v[3] + i[6] * v[4];
  r[3] = i[8] * v[1] - i[7] * v[2] + i[9] * v[3];
  r[4] = i[6] * v[2] - i[8] * v[0] + i[9] * v[4];
  r[5] = i[7] * v[0] - i[6] * v[1] + i[9] * v[5];
}
// [w x v_ang ; w x v_lin + vlin x v_ang]
__device__ __forceinline__ void cross_motion(float r[6], const float* vel, const float* v) {
  float t0 = -vel[2] * v[1] + vel[1] * v[2];
  float t1 = vel[2] * v[0] - vel[0] * v[2];
  float t2 = -vel[1] * v[0] + vel[0] * v[1];
  float t3 = -vel[2] * v[4] + vel[1] * v[5] - vel[5] * v[1] + vel[4] * v[2];
  float t4 = vel[2] * v[3] - vel[0] * v[5] + vel[5] * v[0] - vel[3] * v[2];
  float t5 = -vel[1] * v[3] + vel[0] * v[4] - vel[4] * v[0] + vel[3] * v[1];
  r[0] = t0; r[1] = t1; r[2] = t2; r[3] = t3; r[4] = t4; r[5] = t5;
}
// [w x f_rot + vlin x f_lin ; w x f_lin]
__device__ __forceinline__ void cross_force(float r[6], const float* vel, const float* f) {
  float t0 = -vel[2] * f[1] + vel[1] * f[2] - vel[5] * f[4] + vel[4] * f[5];
  float t1 = vel[2] * f[0] - vel[0] * f[2] + vel[5] * f[3] - vel[3] * f[5];
  float t2 = -vel[1] * f[0] + vel[0] * f[1] - vel[4] * f[3] + vel[3] * f[4];
  float t3 = -vel[2] * f[4] + vel[1] * f[5];
  float t4 = vel[2] * f[3] - vel[0] * f[5];
  float t5 = -vel[1] * f[3] + vel[0] * f[4];
  r[0] = t0; r[1] = t1; r[2] = t2; r[3] = t3; r[4] = t4; r[5] = t5;
}
// brax.math.rotate(v, q) = 2 (u.v) u + (s^2 - u.u) v + 2 s (u x v)
__device__ __forceinline__ void b_rotate(float r[3], const float v[3], const float q[4]) {
  float u[3] = {q[1], q[2], q[3]}, c[3];
  float s = q[0], uv = dot3(u, v), uu = dot3(u, u);
  cross3(c, u, v);
  for (int k = 0; k < 3; k++) r[k] = 2 * uv * u[k] + (s * s - uu) * v[k] + 2 * s * c[k];
}

// MuJoCo impedance (getimpedance), solimp pre-clamped on the host
// solimp with a power other than 1 or 2: out of line -- its four powf calls are ~750 instructions
// per call site that the common powers never run, inside a substep loop whose code is about the
// size of the CU pair's instruction cache
__device__ __attribute__((noinline)) float getimp_pow(float x, float mid, float p) {
  return (x <= mid) ? powf(x, p) / powf(mid, p - 1.0f) : 1.0f - powf(1.0f - x, p) / powf(1.0f - mid, p - 1.0f);
}
__device__ __forceinline__ float getimp(const float* si, float pos, float margin) {
  float x = fabsf((pos - margin) / si[2]);
  if (x >= 1.0f) return si[1];
  if (x <= 0.0f) return si[0];
  float y;
  float p = si[4], mid = si[3];
  if (p == 1.0f) {
    y = x;
  } else if (p == 2.0f) {  // MuJoCo's default power: no powf (4 divergent powf calls cost ~200 VALU)
    y = (x <= mid) ? x * x / mid : 1.0f - (1.0f - x) * (1.0f - x) / (1.0f - mid);
  } else {
    y = getimp_pow(x, mid, p);
  }
  return si[0] + y * (si[1] - si[0]);
}

// ------------------------------- jax threefry RNG -------------------------------
__device__ __forceinline__ uint32_t rotl32(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }
__device__ __forceinline__ void threefry(uint32_t k0, uint32_t k1, uint32_t x0, uint32_t x1, uint32_t& y0, uint32_t& y1) {
  const uint32_t k2 = k0 ^ k1 ^ 0x1BD11BDAu;
  const uint32_t ks[3] = {k0, k1, k2};
  x0 += k0;
  x1 += k1;
#pragma unroll
  for (int i = 0; i < 5; i++) {
    const int r0 = (i & 1) ? 17 : 13, r1 = (i & 1) ? 29 : 15, r2 = (i & 1) ? 16 : 26, r3 = (i & 1) ? 24 : 6;
    x0 += x1; x1 = rotl32(x1, r0); x1 ^= x0;
    x0 += x1; x1 = rotl32(x1, r1); x1 ^= x0;
    x0 += x1; x1 = rotl32(x1, r2); x1 ^= x0;
    x0 += x1; x1 = rotl32(x1, r3); x1 ^= x0;
    x0 += ks[(i + 1) % 3];
    x1 += ks[(i + 2) % 3] + (uint32_t)(i + 1);
  }
  y0 = x0;
  y1 = x1;
}
struct Key { uint32_t a, b; };
// jax.random.split(key, n)[i]
__device__ __forceinline__ Key split_i(Key k, int n, int i, int part) {
  Key r;
  uint32_t y0, y1;
  if (part) {
    threefry(k.a, k.b, 0u, (uint32_t)i, y0, y1);
    r.a = y0; r.b = y1;
  } else {
    int f0 = 2 * i, f1 = 2 * i + 1;
    threefry(k.a, k.b, (uint32_t)(f0 % n), (uint32_t)(f0 % n + n), y0, y1);
    r.a = (f0 / n) ? y1 : y0;
    threefry(k.a, k.b, (uint32_t)(f1 % n), (uint32_t)(f1 % n + n), y0, y1);
    r.b = (f1 / n) ? y1 : y0;
  }
  return r;
}
__device__ __forceinline__ uint32_t bits_i(Key k, int count, int i, int part) {
  uint32_t y0, y1;
  if (part) {
    threefry(k.a, k.b, 0u, (uint32_t)i, y0, y1);
    return y0 ^ y1;
  }
  int n = count + (count & 1), h = n / 2;
  int lane = i % h, half = i / h;
  uint32_t c1 = (lane + h >= count) ? 0u : (uint32_t)(lane + h);
  threefry(k.a, k.b, (uint32_t)lane, c1, y0, y1);
  return half ? y1 : y0;
}
// jax.random.uniform element i of `count`, float32, no FMA contraction (bit-exact with JAX)
__device__ __forceinline__ float uniform_i(Key k, int count, int i, float lo, float hi, int part) {
#pragma clang fp contract(off)
  uint32_t b = (bits_i(k, count, i, part) >> 9) | 0x3F800000u;
  float u = __uint_as_float(b) - 1.0f;
  float v = u * (hi - lo) + lo;
  return v > lo ? v : lo;
}

}  // namespace pp3
