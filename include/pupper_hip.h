/*
 * pupper_hip.h -- C-ABI of the MI355X-native Pupper-v3 environment.
 *
 * This is the drop-in boundary for the hot path named by BASELINE.json
 * `north_star`: the batched replacement for
 *
 *   pupperv3_mjx.environment.PupperV3Env.reset(rng)  (environment.py:314-346)
 *   pupperv3_mjx.environment.PupperV3Env.step(state, action)  (environment.py:348-483)
 *
 * including the MJX physics they call (`pipeline_init` environment.py:319,
 * `pipeline_step` environment.py:366 -> 5 x mjx.step), the reward stack
 * (rewards.py:9-138), the observation pipeline (environment.py:485-543) and the
 * per-env domain randomisation (domain_randomization.py:8-112).
 *
 * Plain C types only: pointers + sizes, int status codes, no exceptions and no
 * torch types across the boundary.  All `*_dev` arguments are device pointers
 * on the handle's device; `stream` is a hipStream_t passed as void* (NULL =
 * the handle's own stream).
 *
 * The reference's FFI for this path is Python (Brax `Env.reset/step`,
 * [ext] brax 0.12.1 brax/envs/base.py); the ctypes binding a maintainer adds is
 * shown in INTEGRATION.md and implemented in pupperv3-mjx_amd/pupperv3_mjx/_lib.py.
 */
#ifndef PUPPER_HIP_H_
#define PUPPER_HIP_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PP3_ABI_VERSION 2

/* ---- fixed topology of test_pupper_model.xml (checked at pp3_create) ---- */
#define PP3_NBODY 14      /* world + base_link + 4 legs x 3 links          */
#define PP3_NJNT 13       /* 1 free joint + 12 hinges                      */
#define PP3_NQ 19
#define PP3_NV 18
#define PP3_NU 12
#define PP3_NLEG 4
#define PP3_NFOOT 4
#define PP3_MAX_CGEOM 96  /* collidable geoms (8 spheres + floor + boxes)  */
#define PP3_MAX_PAIR 640  /* candidate collision pairs after filtering     */
#define PP3_MAX_SITE 8
#define PP3_MAX_SENSOR 16     /* <sensor> entries (site-based types below)   */
#define PP3_MAX_SENSORDATA 32 /* total sensordata floats                      */
#define PP3_MAX_LAG 8     /* latency-buffer length limit                   */
#define PP3_NREWARD 18    /* reward terms, order = PP3_REWARD_* below      */
#define PP3_NMETRIC 19    /* total_dist + 18 scaled reward terms           */
#define PP3_NDR 62        /* per-env domain-randomisation scalars          */
#define PP3_OBS_DIM 36    /* environment.py:226                            */

/* MuJoCo enums restated (mjtGeom / mjtJoint / mjtCone / mjtBias) */
enum { PP3_GEOM_PLANE = 0, PP3_GEOM_SPHERE = 2, PP3_GEOM_BOX = 6 };
enum { PP3_JNT_FREE = 0, PP3_JNT_HINGE = 3 };
enum { PP3_CONE_PYRAMIDAL = 0 };
enum { PP3_BIAS_NONE = 0, PP3_BIAS_AFFINE = 1 };
/* sensor types (own numbering; each is attached to a site, objtype="site") */
enum {
  PP3_SENS_ACCELEROMETER = 1,
  PP3_SENS_VELOCIMETER = 2,
  PP3_SENS_GYRO = 3,
  PP3_SENS_FRAMEPOS = 26,
  PP3_SENS_FRAMEQUAT = 27,
  PP3_SENS_FRAMELINVEL = 32,
  PP3_SENS_FRAMEANGVEL = 33
};

/* Reward-term order = the rewards_dict literal in environment.py:391-444
 * (this order is also the fp32 summation order of environment.py:446). */
enum {
  PP3_REWARD_TRACKING_LIN_VEL = 0,
  PP3_REWARD_TRACKING_ANG_VEL,
  PP3_REWARD_TRACKING_ORIENTATION,
  PP3_REWARD_LIN_VEL_Z,
  PP3_REWARD_ANG_VEL_XY,
  PP3_REWARD_ORIENTATION,
  PP3_REWARD_TORQUES,
  PP3_REWARD_JOINT_ACCELERATION,
  PP3_REWARD_MECHANICAL_WORK,
  PP3_REWARD_ACTION_RATE,
  PP3_REWARD_STAND_STILL,
  PP3_REWARD_STAND_STILL_JOINT_VELOCITY,
  PP3_REWARD_ABDUCTION_ANGLE,
  PP3_REWARD_FEET_AIR_TIME,
  PP3_REWARD_FOOT_SLIP,
  PP3_REWARD_TERMINATION,
  PP3_REWARD_KNEE_COLLISION,
  PP3_REWARD_BODY_COLLISION
};

/* Compiled model (host, fp64).  Produced by the MJCF-subset compiler
 * pupperv3_mjx/mjcf.py from test_pupper_model.xml (+ obstacles.py boxes).
 * Field names follow mjModel. */
typedef struct pp3_model_t {
  /* <option> */
  double timestep;
  double gravity[3];
  double impratio;
  double tolerance;
  double ls_tolerance;
  int32_t iterations;
  int32_t ls_iterations;
  int32_t cone;
  int32_t eulerdamp;   /* 1 = enabled; the model disables it (xml:58) */
  double meaninertia;  /* mjStatistic.meaninertia: mean diag(M) at qpos0 */
  /* bodies (0 = world) */
  int32_t body_parentid[PP3_NBODY];
  int32_t body_jntadr[PP3_NBODY];
  int32_t body_dofadr[PP3_NBODY];
  int32_t body_dofnum[PP3_NBODY];
  double body_pos[PP3_NBODY][3];
  double body_quat[PP3_NBODY][4];
  double body_ipos[PP3_NBODY][3];
  double body_iquat[PP3_NBODY][4];
  double body_mass[PP3_NBODY];
  double body_inertia[PP3_NBODY][3];
  double body_invweight0[PP3_NBODY][2];
  /* joints */
  int32_t jnt_type[PP3_NJNT];
  int32_t jnt_bodyid[PP3_NJNT];
  int32_t jnt_qposadr[PP3_NJNT];
  int32_t jnt_dofadr[PP3_NJNT];
  int32_t jnt_limited[PP3_NJNT];
  double jnt_pos[PP3_NJNT][3];
  double jnt_axis[PP3_NJNT][3];
  double jnt_range[PP3_NJNT][2];
  double jnt_margin[PP3_NJNT];
  double jnt_solref[PP3_NJNT][2];
  double jnt_solimp[PP3_NJNT][5];
  /* dofs */
  int32_t dof_bodyid[PP3_NV];
  int32_t dof_jntid[PP3_NV];
  int32_t dof_parentid[PP3_NV];
  double dof_armature[PP3_NV];
  double dof_damping[PP3_NV];
  double dof_frictionloss[PP3_NV];
  double dof_invweight0[PP3_NV];
  double dof_solref[PP3_NV][2];
  double dof_solimp[PP3_NV][5];
  double qpos0[PP3_NQ];
  double key_qpos[PP3_NQ]; /* keyframe "home" */
  /* collidable geoms (contype|conaffinity != 0); cgeom_id = MuJoCo geom id */
  int32_t ngeom;  /* total MuJoCo geoms (ids) */
  int32_t ncgeom;
  int32_t cgeom_id[PP3_MAX_CGEOM];
  int32_t cgeom_type[PP3_MAX_CGEOM];
  int32_t cgeom_bodyid[PP3_MAX_CGEOM];
  int32_t cgeom_condim[PP3_MAX_CGEOM];
  int32_t cgeom_priority[PP3_MAX_CGEOM];
  double cgeom_size[PP3_MAX_CGEOM][3];
  double cgeom_pos[PP3_MAX_CGEOM][3];   /* in body frame */
  double cgeom_quat[PP3_MAX_CGEOM][4];  /* in body frame */
  double cgeom_friction[PP3_MAX_CGEOM][3];
  double cgeom_solref[PP3_MAX_CGEOM][2];
  double cgeom_solimp[PP3_MAX_CGEOM][5];
  double cgeom_solmix[PP3_MAX_CGEOM];
  double cgeom_margin[PP3_MAX_CGEOM];
  double cgeom_gap[PP3_MAX_CGEOM];
  /* candidate pairs (indices into cgeom_*), type(g1) <= type(g2) */
  int32_t npair;
  int32_t pair_g1[PP3_MAX_PAIR];
  int32_t pair_g2[PP3_MAX_PAIR];
  /* sites */
  int32_t nsite;
  int32_t site_bodyid[PP3_MAX_SITE];
  double site_pos[PP3_MAX_SITE][3];
  double site_quat[PP3_MAX_SITE][4];
  /* actuators (general, joint transmission) */
  int32_t actuator_trnid[PP3_NU];  /* joint id */
  int32_t actuator_biastype[PP3_NU];
  int32_t actuator_forcelimited[PP3_NU];
  int32_t actuator_ctrllimited[PP3_NU];
  double actuator_gear[PP3_NU];
  double actuator_gainprm[PP3_NU][3];
  double actuator_biasprm[PP3_NU][3];
  double actuator_forcerange[PP3_NU][2];
  double actuator_ctrlrange[PP3_NU][2];
  /* <custom> numerics (MJX collision caps; -1 = absent) */
  int32_t max_contact_points;
  int32_t max_geom_pairs;
  /* <sensor> (xml:14-23): site sensors, sensordata = mjData.sensordata layout */
  int32_t nsensor;
  int32_t nsensordata;
  int32_t sensor_type[PP3_MAX_SENSOR];   /* PP3_SENS_* */
  int32_t sensor_objid[PP3_MAX_SENSOR];  /* site id */
  int32_t sensor_adr[PP3_MAX_SENSOR];
  int32_t sensor_dim[PP3_MAX_SENSOR];
  double sensor_cutoff[PP3_MAX_SENSOR];  /* 0 = none */
} pp3_model_t;

/* Environment configuration: PupperV3Env.__init__ kwargs
 * (environment.py:35-121) + config.py reward scales. */
typedef struct pp3_env_config_t {
  int32_t n_frames;            /* physics substeps per env step (5)        */
  int32_t obs_history;         /* H                                         */
  int32_t use_imu;
  int32_t latency_len;         /* La = len(latency_distribution)           */
  int32_t imu_latency_len;     /* Li                                        */
  int32_t resample_velocity_step;
  int32_t early_termination_step_threshold;
  int32_t torso_body;
  int32_t feet_site[PP3_NFOOT];
  int32_t lower_leg_body[PP3_NFOOT];
  int32_t n_upper_leg_geoms;
  int32_t upper_leg_geoms[16];
  int32_t n_torso_geoms;
  int32_t torso_geoms[8];
  int32_t rng_partitionable;   /* jax_threefry_partitionable (jax 0.5.0: 1) */
  int32_t ncon_max;            /* contact cap per env (deepest kept): 0 = default 8, 8, 16 */
  double latency_dist[PP3_MAX_LAG];
  double imu_latency_dist[PP3_MAX_LAG];
  double action_scale;
  double default_pose[PP3_NU];
  double joint_lower[PP3_NU];
  double joint_upper[PP3_NU];
  double desired_abduction[4];
  double start_pos_min[3];
  double start_pos_max[3];
  double lin_vel_x_range[2];
  double lin_vel_y_range[2];
  double ang_vel_range[2];
  double zero_command_probability;
  double stand_still_command_threshold;
  double max_pitch_command;    /* degrees */
  double max_roll_command;     /* degrees */
  double ang_vel_noise;
  double gravity_noise;
  double motor_angle_noise;
  double last_action_noise;
  double kick_vel;
  double kick_probability;
  double terminal_body_z;
  double terminal_body_angle;
  double foot_radius;
  double env_dt;               /* self._dt = environment_timestep          */
  double dt;                   /* self.dt = opt.timestep * n_frames        */
  double desired_world_z[3];
  double reward_scales[PP3_NREWARD];
  double tracking_sigma;
} pp3_env_config_t;

typedef struct pp3_env pp3_env_t;

/* ---- per-env state record (float32 words, env-major: state[N][stride]) ---- */
enum {
  PP3_S_QPOS = 0,          /* 19 */
  PP3_S_QVEL = 19,         /* 18 */
  PP3_S_QACC_WS = 37,      /* 18  qacc_warmstart                         */
  PP3_S_RNG = 55,          /*  2  uint32 key words, bit-cast into f32    */
  PP3_S_LAST_ACT = 57,     /* 12 */
  PP3_S_LAST_VEL = 69,     /* 12 */
  PP3_S_COMMAND = 81,      /*  3 */
  PP3_S_DESIRED_Z = 84,    /*  3 */
  PP3_S_AIR_TIME = 87,     /*  4 */
  PP3_S_LAST_CONTACT = 91, /*  4  0.0 / 1.0                             */
  PP3_S_KICK = 95,         /*  2 */
  PP3_S_STEP = 97,         /*  1  step counter (integral value as float) */
  PP3_S_ACT_BUF = 98       /* 12*La action buffer [12][La], then 6*Li imu buffer [6][Li] */
};

/* Field ids for pp3_field / pp3_copy_field.  Every field is ONE device buffer owned by the
 * handle, allocated at pp3_create and updated in place: the pointer pp3_field returns stays
 * valid (and constant) until pp3_destroy, so a training loop may wrap it once; its contents are
 * overwritten by every pp3_step / pp3_reset launched on the handle's stream (copy a field out
 * first, on that stream, to keep a previous step's values). */
enum {
  PP3_F_STATE = 0,    /* [N][state_stride] f32 */
  PP3_F_OBS = 1,      /* [N][36H] f32 */
  PP3_F_REWARD = 2,   /* [N] f32 */
  PP3_F_DONE = 3,     /* [N] f32 */
  PP3_F_METRICS = 4,  /* [N][19] f32: total_dist, scaled rewards */
  PP3_F_DR = 5,       /* [N][62] f32 */
  PP3_F_PIPELINE = 6, /* [N][PP3_PIPE_STRIDE] f32 (when enabled) */
  PP3_F_ACTION = 7,   /* [N][12] f32 scratch action buffer owned by the handle */
  PP3_F_EPISODE = 8,  /* [N][PP3_EP_STRIDE] f32 episode bookkeeping (auto-reset mode) */
  PP3_F_FIRST_STATE = 9, /* [N][PP3_FIRST_STRIDE] f32 qpos|qvel|qacc_warmstart of the reset */
  PP3_F_FIRST_OBS = 10   /* [N][36H] f32 observation of the reset */
};

/* Optional pipeline-state output (brax State.x / xd of the last substep,
 * environment.py:367): written only when pp3_set_pipeline_output(h, 1). */
enum {
  PP3_P_XPOS = 0,           /* 13 x 3  body origins (bodies 1..13)       */
  PP3_P_XQUAT = 39,         /* 13 x 4 */
  PP3_P_XD_VEL = 91,        /* 13 x 3 */
  PP3_P_XD_ANG = 130,       /* 13 x 3 */
  PP3_P_SITE_XPOS = 169,    /*  4 x 3  foot sites                         */
  PP3_P_QFRC_ACT = 181,     /* 18 */
  PP3_P_QACC = 199,         /* 18 */
  PP3_P_NCON = 217,         /*  1  penetrating contacts (float)           */
  PP3_P_CON_DIST = 218,     /* 16  dist of contacts 0..15                  */
  PP3_P_CON_GEOM = 234,     /* 32  geom1, geom2 of contacts 0..15 (float)  */
  PP3_P_SUBTREE_COM = 266,  /*  3 */
  PP3_P_NHIT = 269,         /*  1  penetrating pairs before the contact cap (> ncon: the cap bound) */
  PP3_P_SENSOR = 272,       /* 32  mjData.sensordata (model's <sensor>) */
  PP3_PIPE_STRIDE = 304
};

/* DR record layout (domain_randomization.py:21-66, absolute values). */
enum {
  PP3_DR_FRICTION = 0,  /* geom_friction[:,0] for every geom            */
  PP3_DR_KP = 1,        /* actuator_gainprm[:,0] = -biasprm[:,1]         */
  PP3_DR_KD = 2,        /* -actuator_biasprm[:,2]                        */
  PP3_DR_BASE_IPOS = 3, /* body_ipos[1] (3)                               */
  PP3_DR_INERTIA = 6,   /* body_inertia[14][3]                            */
  PP3_DR_MASS = 48      /* body_mass[14]                                  */
};

/* Status codes */
enum {
  PP3_OK = 0,
  PP3_ERR_ARG = 1,
  PP3_ERR_MODEL = 2,   /* model topology / options unsupported          */
  PP3_ERR_HIP = 3,
  PP3_ERR_NOMEM = 4,
  PP3_ERR_COMM = 5     /* RCCL unavailable or a collective failed        */
};

int pp3_abi_version(void);
/* sizeof the ABI structs: which = 0 model, 1 env config (ctypes layout check). */
size_t pp3_struct_size(int which);
const char* pp3_last_error(void);
/* HIP device count (0 when no runtime / no GPU). */
int pp3_device_count(void);

/* Create a batch of `num_envs` environments on `device`.  Validates the model
 * (replaces the trace-time assert of environment.py:534 and the name lookups of
 * environment.py:183-203). */
int pp3_create(const pp3_model_t* model, const pp3_env_config_t* cfg,
               int32_t num_envs, int32_t device, pp3_env_t** out);
int pp3_destroy(pp3_env_t* env);
int32_t pp3_num_envs(const pp3_env_t* env);
int32_t pp3_state_stride(const pp3_env_t* env);
/* The HIP device the handle was created on (-1 for NULL). */
int32_t pp3_env_device(const pp3_env_t* env);

/* reset(rng): keys_dev = uint32[N][2] (one jax PRNG key per env); mask_dev =
 * optional uint8[N] (NULL = all envs).  environment.py:314-346. */
int pp3_reset(pp3_env_t* env, const uint32_t* keys_dev, const uint8_t* mask_dev, void* stream);
/* step(state, action): actions_dev = f32[N][12].  environment.py:348-483. */
int pp3_step(pp3_env_t* env, const float* actions_dev, void* stream);
/* nsteps env steps fused into one launch: the unroll of brax's PPO generate_unroll (a lax.scan of
 * env.step, [ext] brax 0.12.1 training/acting.py) with the actions given up front.  Step t reads
 * actions_dev + t * action_stride (elements; 0 = the same action every step) and is the same
 * computation as the t-th of nsteps pp3_step calls (bit for bit); the handle ends in the same
 * state.  Optional trajectory outputs (device, NULL = not written): reward_dev f32[nsteps][N],
 * done_dev f32[nsteps][N], obs_dev f32[nsteps][N][36H] -- step t's reward, done and observation
 * as pp3_step leaves them in the handle (auto-reset: the reset's obs for done envs).  Each wave
 * runs its two envs' steps back to back, so the launch ends with the slowest wave's SUM of step
 * times instead of every step waiting for that step's slowest wave.  With auto-reset and
 * action_repeat > 1 every wrapper step stays `repeat` launches. */
int pp3_rollout(pp3_env_t* env, const float* actions_dev, int64_t action_stride, int32_t nsteps, float* reward_dev,
                float* done_dev, float* obs_dev, void* stream);
/* Per-env DR parameters f32[N][62] (device), or NULL to disable DR. */
int pp3_set_dr(pp3_env_t* env, const float* dr_dev);
int pp3_set_pipeline_output(pp3_env_t* env, int32_t enable);

/* Per-env terrain (the reference's obstacles.py:16-57 boxes are static and
 * shared by all envs).  The model's world-body box geoms become per-env slots: boxes_host =
 * f32[N][n_boxes][PP3_TERRAIN_BOX] host array, per box pos[3] (world), quat[4] (w,x,y,z, any
 * norm) and half sizes[3]; a box whose half sizes are all <= 0 is absent in that env, so envs
 * may hold different numbers of boxes.  n_boxes must equal the model's world box-geom count
 * (pp3_terrain_slots).  Contact parameters (friction, solref, solimp) stay the model's.
 * boxes_host = NULL returns to the model's static boxes.  Synchronises the handle's stream. */
#define PP3_TERRAIN_BOX 10
int pp3_set_terrain(pp3_env_t* env, const float* boxes_host, int32_t n_boxes);
int32_t pp3_terrain_slots(const pp3_env_t* env);

/* Raw physics: `nsteps` x mj_step on the qpos/qvel/qacc_warmstart stored in the
 * state records, with ctrl_dev = f32[N][12] held fixed (no env logic).  Used by
 * the substep parity tests; writes the pipeline record of the last substep. */
int pp3_physics_step(pp3_env_t* env, const float* ctrl_dev, int32_t nsteps, void* stream);

/* Auto-reset mode = brax.envs.training.wrap(env, episode_length, action_repeat) on device
 * ([ext] brax 0.12.1 EpisodeWrapper + AutoResetWrapper, the wrappers Brax PPO puts around
 * PupperV3Env).  Per env: episode step counter, truncation flag and the
 * episode sum_reward / length; pp3_reset stores the reset's qpos/qvel/qacc_warmstart and obs
 * as the env's "first" state; every pp3_step then
 *   - zeroes the episode counter if the previous step was done (AutoResetWrapper.step),
 *   - runs the env step, increments the counter, sets done |= counter >= episode_length and
 *     truncation = (counter >= episode_length) & !env_done (EpisodeWrapper.step),
 *   - replaces qpos/qvel/qacc_warmstart and obs by the first state where done (the env's
 *     info -- rng, command, last action, ... -- carries over, as in Brax).
 * episode_length <= 0 turns the mode off (plain PupperV3Env.step semantics). */
#define PP3_EP_STEPS 0
#define PP3_EP_TRUNCATION 1
#define PP3_EP_SUM_REWARD 2
#define PP3_EP_LENGTH 3
#define PP3_EP_STRIDE 4
#define PP3_FIRST_STRIDE 55
int pp3_set_auto_reset(pp3_env_t* env, int32_t episode_length);
/* brax.envs.training.wrap(..., action_repeat=k) (EpisodeWrapper.step scans env.step k times with
 * the same action): in auto-reset mode every pp3_step launches the env step k times; reward =
 * the sum over the k repeats, the episode counter and length advance by k, and done, truncation
 * and the auto-reset are decided after the last repeat (the env's own done of that repeat, as in
 * Brax).  k = 1 is the plain mode; k > 1 needs auto-reset mode (PP3_ERR_ARG otherwise); turning
 * auto-reset off resets k to 1. */
int pp3_set_action_repeat(pp3_env_t* env, int32_t action_repeat);

/* Device pointer + element count per env of a field (PP3_F_*). */
int pp3_field(pp3_env_t* env, int32_t field, void** dev_ptr, int64_t* elems_per_env);
/* Synchronous host <-> device copies of a whole field (tests / host API). */
int pp3_copy_field_to_host(pp3_env_t* env, int32_t field, void* host, size_t bytes);
int pp3_copy_field_from_host(pp3_env_t* env, int32_t field, const void* host, size_t bytes);
int pp3_synchronize(pp3_env_t* env);
/* Asynchronous device -> host copy of a whole field on the handle's stream (no synchronisation:
 * pair it with pp3_synchronize).  Meant for page-locked host memory (pp3_host_malloc), which is
 * what lets it run at PCIe speed without a staging copy (the host API's per-step outputs). */
int pp3_copy_field_to_host_async(pp3_env_t* env, int32_t field, void* host, size_t bytes);
/* The host API's per-step outputs in one go (environment.py:348 `step` returns State.obs /
 * .reward / .done): a kernel on the handle's stream stores [obs N x 36H | reward N | done N] straight
 * into `host`, page-locked memory from pp3_host_malloc of at least N * (36H + 2) floats, through its
 * device mapping (no copy-engine transfer).  No synchronisation: pair it with pp3_synchronize. */
int pp3_outputs_to_host(pp3_env_t* env, float* host);
/* The device address of page-locked host memory from pp3_host_malloc, e.g. to pass a host block as
 * pp3_rollout's trajectory outputs so the step kernel stores its rows straight into host memory
 * (the host API's step). */
int pp3_host_device_ptr(void* host, void** dev_ptr);
/* The handle's own HIP stream (hipStream_t), for ordering other work (e.g. pp3_policy_act) with it. */
void* pp3_stream(pp3_env_t* env);
/* Completion markers for the host API's asynchronous step (environment.py:348 `step`: the State
 * returns at once and its obs / reward / done wait for their own step only): a HIP event (timing
 * disabled) on the handle's device, recorded on the handle's stream; synchronize waits until every
 * operation queued before its last record has completed (at once if never recorded). */
int pp3_event_create(pp3_env_t* env, void** ev_out);
int pp3_event_record(pp3_env_t* env, void* ev);
int pp3_event_synchronize(void* ev);
int pp3_event_destroy(void* ev);

/* Small device-memory helpers so a host can run without any other GPU runtime. */
int pp3_device_malloc(int32_t device, size_t bytes, void** out);
int pp3_device_free(void* ptr);
int pp3_memcpy_h2d(void* dst_dev, const void* src_host, size_t bytes);
int pp3_memcpy_d2h(void* dst_host, const void* src_dev, size_t bytes);
int pp3_memcpy_d2d(void* dst_dev, const void* src_dev, size_t bytes, void* stream);
/* Asynchronous host -> device copy on `stream` (from page-locked memory: the host API's actions). */
int pp3_memcpy_h2d_async(void* dst_dev, const void* src_host, size_t bytes, void* stream);
/* Page-locked host memory (hipHostMalloc) for the host API's output arrays. */
int pp3_host_malloc(size_t bytes, void** out);
int pp3_host_free(void* ptr);

/* Benchmark helpers: fill actions f32[N][12] with U(lo,hi) from a counter hash
 * keyed by (seed, step) on device; record HIP events around the step kernel
 * launches on the handle's stream so the average kernel duration can be read. */
int pp3_fill_uniform(pp3_env_t* env, float* dev, int64_t count, uint32_t seed, uint32_t ctr, float lo, float hi, void* stream);
/* nsteps back-to-back pp3_step launches on the handle's stream, step i reading actions
 * actions_dev + i * action_stride (elements; 0 = reuse); HIP events bracket the launches and
 * kernel_ms_total receives their elapsed time. */
int pp3_step_timed(pp3_env_t* env, const float* actions_dev, int64_t action_stride, int32_t nsteps,
                   float* kernel_ms_total);
/* The same for one pp3_rollout over nsteps (trajectory outputs as pp3_rollout). */
int pp3_rollout_timed(pp3_env_t* env, const float* actions_dev, int64_t action_stride, int32_t nsteps,
                      float* reward_dev, float* done_dev, float* obs_dev, float* kernel_ms_total);

/* Rendering (environment.py:545-547 PupperV3Env.render -> Brax PipelineEnv.render, the policy
 * videos of utils.py:214-293; not on the training path).  A z-buffer rasteriser over a triangle
 * soup built on the host by pupperv3_mjx/render.py from the model's visual geoms:
 *   tris [ntri][9]        vertices in the geom's local frame (device)
 *   tri_geom [ntri]       geom index of each triangle (device)
 *   geom_rgb [ngeom][3]   colour in 0..1 (device)
 *   geom_xf [F][ngeom][12] per frame: world rotation (row-major 3x3) then translation (device)
 *   cams [F][16]          per frame: position, right, up, forward (unit), focal length in pixels
 *                         (= height / 2 / tan(fovy / 2)), 3 pad (device)
 *   scene [17]            floor checker colours rgb1[3], rgb2[3], square size, floor height, sky
 *                         top[3], sky bottom[3], ambient, diffuse, floor on (HOST pointer)
 *   out [F][H][W][3]      u8 RGB (device)
 * Nearest fragment per pixel by a 64-bit atomicMin of (depth bits, rgb): deterministic.
 * Synchronous on `stream` (NULL = default stream); its own errors via pp3_render_last_error(). */
int pp3_render(int32_t device, const float* tris, const int32_t* tri_geom, int32_t ntri, const float* geom_rgb,
               int32_t ngeom, const float* geom_xf, const float* cams, int32_t nframes, int32_t height,
               int32_t width, const float* scene, uint8_t* out, void* stream);
const char* pp3_render_last_error(void);


/* ---------------------------------------------------------------------------------------
 * On-device MLP policy in the reference's deployment format (export.py:13-81 convert_params:
 * "layers": dense, "weights": [kernel [in][out], bias [out]], normalisation folded into the
 * first layer, final layer = Gaussian-head mean, "activation" per layer, final tanh).
 * pupperv3_mjx/export.py loads such a dict into this API.  Batch forward on the f32 matrix
 * cores (csrc/pp3_policy.hip).
 * ------------------------------------------------------------------------------------- */
typedef struct pp3_policy pp3_policy_t;
#define PP3_POLICY_MAX_LAYERS 8
#define PP3_POLICY_MAX_WIDTH 576 /* >= 36 * 15 (observation_history 15) */
enum { PP3_ACT_LINEAR = 0, PP3_ACT_RELU = 1, PP3_ACT_ELU = 2, PP3_ACT_TANH = 3, PP3_ACT_SIGMOID = 4 };
/* weights = for each layer: kernel [in][out] row-major, then bias [out] (host memory). */
int pp3_policy_create(int32_t device, int32_t in_dim, int32_t n_layers, const int32_t* out_dims,
                      const int32_t* activations, const float* weights, pp3_policy_t** out);
/* actions[i][0:out_dim] = policy(obs[i][0:in_dim]) for i < n (device pointers, strides in floats). */
int pp3_policy_act(pp3_policy_t* policy, const float* obs_dev, int64_t obs_stride, int32_t n,
                   float* actions_dev, int64_t action_stride, void* stream);
int pp3_policy_out_dim(const pp3_policy_t* policy);
int pp3_policy_destroy(pp3_policy_t* policy);
/* The unroll of brax's generate_unroll with the policy in the loop ([ext] brax 0.12.1
 * training/acting.py: actions = policy(obs), state = env.step(state, actions), nsteps times), on the
 * env's stream with no host round trip: before step t the policy acts on the env's observation
 * buffer, writing actions_dev + t * N * 12 (f32[nsteps][N][12], required: the trajectory's
 * actions), then the env steps on them; reward / done / obs trajectories as pp3_rollout
 * (optional).  ONE launch for the nsteps steps (workgroups of 16 envs run the policy's MLP, the
 * code of pp3_policy_act, before each step: the actions equal pp3_policy_act's bit for bit); with
 * max_contacts = 16 or action_repeat > 1, per step a pp3_policy_act launch then a step launch.
 * The policy must have 12 outputs and 36H inputs and live on the env's device. */
int pp3_rollout_policy(pp3_env_t* env, pp3_policy_t* policy, int32_t nsteps, float* actions_dev,
                       float* reward_dev, float* done_dev, float* obs_dev, void* stream);
/* The same bracketed by HIP events on the handle's stream (kernel_ms_total = their elapsed time). */
int pp3_rollout_policy_timed(pp3_env_t* env, pp3_policy_t* policy, int32_t nsteps, float* actions_dev,
                             float* reward_dev, float* done_dev, float* obs_dev, float* kernel_ms_total);
const char* pp3_policy_last_error(void);

/* ---------------------------------------------------------------------------------------
 * Multi-GPU (no reference code: the reference runs one process per device under
 * Brax PPO's pmap, [ext] brax 0.12.1 brax/training/agents/ppo/train.py, where the env batch is
 * sharded across devices and XLA gathers it).  One process per GPU, each owning a contiguous
 * shard of the global env batch (pupperv3_mjx/sharding.py); envs never exchange data inside a
 * step.  The only data-path collective is the optional per-step hand-over of the learner batch
 * obs | reward | done over RCCL (xGMI), launched on the env's stream behind the step kernel with
 * no host synchronisation.  RCCL is dlopen'ed on first use (the single-GPU path never loads it).
 * ------------------------------------------------------------------------------------- */
typedef struct pp3_comm pp3_comm_t;
#define PP3_COMM_ID_BYTES 128 /* ncclUniqueId */
enum { PP3_REDUCE_SUM = 0, PP3_REDUCE_MAX = 1 };
/* Rank 0 creates the communicator id and hands its 128 bytes to the other ranks out of band. */
int pp3_comm_unique_id(uint8_t* id_out);
int pp3_comm_init(const uint8_t* id, int32_t rank, int32_t world, int32_t device, pp3_comm_t** out);
int pp3_comm_destroy(pp3_comm_t* comm);
int32_t pp3_comm_rank(const pp3_comm_t* comm);
int32_t pp3_comm_world(const pp3_comm_t* comm);
const char* pp3_comm_last_error(void);
/* Learner batch of every rank's env shard: each rank contributes nmax rows (nmax >= its env
 * count; rows past the count are zero) of width 36H + 2 = [obs | reward | done], rank r's rows
 * at dst_dev + r * nmax * (36H + 2).  root >= 0: gather to rank `root` (grouped send/recv,
 * dst_dev needed on the root only); root < 0: all-gather (dst_dev on every rank).  Enqueued on
 * `stream` (NULL = the env's stream): ordered after the env's last step, no host sync.  The env
 * must live on the communicator's device (PP3_ERR_ARG otherwise); the caller's current HIP device
 * is restored on return. */
int pp3_gather(pp3_comm_t* comm, pp3_env_t* env, int32_t nmax, int32_t root, float* dst_dev, void* stream);
/* The same hand-over for a K-step unroll (replaces the per-device trajectory of Brax's
 * generate_unroll, [ext] brax 0.12.1 brax/training/acting.py, that PPO's pmap hands to the learner
 * once per unroll): the trajectory outputs of one fused pp3_rollout of this env (traj_obs
 * [nsteps][N][36H], traj_reward / traj_done [nsteps][N], device pointers) -> rank r's block
 * [nsteps][nmax][36H + 2] at dst_dev + r * nsteps * nmax * (36H + 2); rows past the rank's env
 * count are zero.  ONE collective per unroll instead of one per step; root, stream and device
 * rules as pp3_gather. */
int pp3_gather_rollout(pp3_comm_t* comm, pp3_env_t* env, const float* traj_obs, const float* traj_reward,
                       const float* traj_done, int32_t nsteps, int32_t nmax, int32_t root, float* dst_dev,
                       void* stream);
/* Host-blocking helpers for timing: element-wise sum / max of n <= 64 doubles over ranks, and
 * a barrier. */
int pp3_comm_allreduce(pp3_comm_t* comm, const double* in, double* out, int32_t n, int32_t op);
int pp3_comm_barrier(pp3_comm_t* comm);

#ifdef __cplusplus
}
#endif
#endif /* PUPPER_HIP_H_ */
