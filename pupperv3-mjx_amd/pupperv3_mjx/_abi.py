"""ctypes mirror of include/pupper_hip.h (struct layouts + constants).

Layouts are checked against the compiled library with ``pp3_struct_size`` in
tests/test_abi.py, so a drift between this file and the header fails loudly.
"""
import ctypes as C

ABI_VERSION = 2
NBODY, NJNT, NQ, NV, NU = 14, 13, 19, 18, 12
NLEG, NFOOT = 4, 4
MAX_CGEOM, MAX_PAIR, MAX_SITE, MAX_LAG = 96, 640, 8, 8
MAX_SENSOR, MAX_SENSORDATA = 16, 32
SENS_ACCELEROMETER, SENS_VELOCIMETER, SENS_GYRO = 1, 2, 3
SENS_FRAMEPOS, SENS_FRAMEQUAT, SENS_FRAMELINVEL, SENS_FRAMEANGVEL = 26, 27, 32, 33
NREWARD, NMETRIC, NDR, OBS_DIM = 18, 19, 62, 36

# state record offsets (float32 words)
S_QPOS, S_QVEL, S_QACC_WS, S_RNG = 0, 19, 37, 55
S_LAST_ACT, S_LAST_VEL, S_COMMAND, S_DESIRED_Z = 57, 69, 81, 84
S_AIR_TIME, S_LAST_CONTACT, S_KICK, S_STEP, S_ACT_BUF = 87, 91, 95, 97, 98

GEOM_PLANE, GEOM_SPHERE, GEOM_BOX = 0, 2, 6

F_STATE, F_OBS, F_REWARD, F_DONE, F_METRICS, F_DR, F_PIPELINE, F_ACTION = range(8)
TERRAIN_BOX = 10  # PP3_TERRAIN_BOX: pos[3], quat[4] (w,x,y,z), half sizes[3]
F_EPISODE, F_FIRST_STATE, F_FIRST_OBS = 8, 9, 10
EP_STEPS, EP_TRUNCATION, EP_SUM_REWARD, EP_LENGTH, EP_STRIDE = 0, 1, 2, 3, 4
FIRST_STRIDE = 55

P_XPOS, P_XQUAT, P_XD_VEL, P_XD_ANG = 0, 39, 91, 130
P_SITE_XPOS, P_QFRC_ACT, P_QACC, P_NCON = 169, 181, 199, 217
P_CON_DIST, P_CON_GEOM, P_SUBTREE_COM, P_SENSOR, PIPE_STRIDE = 218, 234, 266, 272, 304
P_NHIT = 269  # penetrating pairs before the contact cap

ERR_ARG, ERR_MODEL, ERR_HIP, ERR_NOMEM, ERR_COMM = 1, 2, 3, 4, 5
COMM_ID_BYTES = 128  # PP3_COMM_ID_BYTES (ncclUniqueId)
REDUCE_SUM, REDUCE_MAX = 0, 1

DR_FRICTION, DR_KP, DR_KD, DR_BASE_IPOS, DR_INERTIA, DR_MASS = 0, 1, 2, 3, 6, 48

# reward order = environment.py:391-444 literal order (also summation order, :446)
REWARD_NAMES = (
    "tracking_lin_vel", "tracking_ang_vel", "tracking_orientation", "lin_vel_z", "ang_vel_xy",
    "orientation", "torques", "joint_acceleration", "mechanical_work", "action_rate",
    "stand_still", "stand_still_joint_velocity", "abduction_angle", "feet_air_time",
    "foot_slip", "termination", "knee_collision", "body_collision",
)

d, i32 = C.c_double, C.c_int32


def _a(t, *dims):
    for n in reversed(dims):
        t = t * n
    return t


class Model(C.Structure):
    _fields_ = [
        ("timestep", d), ("gravity", _a(d, 3)), ("impratio", d), ("tolerance", d),
        ("ls_tolerance", d), ("iterations", i32), ("ls_iterations", i32), ("cone", i32),
        ("eulerdamp", i32), ("meaninertia", d),
        ("body_parentid", _a(i32, NBODY)), ("body_jntadr", _a(i32, NBODY)),
        ("body_dofadr", _a(i32, NBODY)), ("body_dofnum", _a(i32, NBODY)),
        ("body_pos", _a(d, NBODY, 3)), ("body_quat", _a(d, NBODY, 4)),
        ("body_ipos", _a(d, NBODY, 3)), ("body_iquat", _a(d, NBODY, 4)),
        ("body_mass", _a(d, NBODY)), ("body_inertia", _a(d, NBODY, 3)),
        ("body_invweight0", _a(d, NBODY, 2)),
        ("jnt_type", _a(i32, NJNT)), ("jnt_bodyid", _a(i32, NJNT)), ("jnt_qposadr", _a(i32, NJNT)),
        ("jnt_dofadr", _a(i32, NJNT)), ("jnt_limited", _a(i32, NJNT)),
        ("jnt_pos", _a(d, NJNT, 3)), ("jnt_axis", _a(d, NJNT, 3)), ("jnt_range", _a(d, NJNT, 2)),
        ("jnt_margin", _a(d, NJNT)), ("jnt_solref", _a(d, NJNT, 2)), ("jnt_solimp", _a(d, NJNT, 5)),
        ("dof_bodyid", _a(i32, NV)), ("dof_jntid", _a(i32, NV)), ("dof_parentid", _a(i32, NV)),
        ("dof_armature", _a(d, NV)), ("dof_damping", _a(d, NV)), ("dof_frictionloss", _a(d, NV)),
        ("dof_invweight0", _a(d, NV)), ("dof_solref", _a(d, NV, 2)), ("dof_solimp", _a(d, NV, 5)),
        ("qpos0", _a(d, NQ)), ("key_qpos", _a(d, NQ)),
        ("ngeom", i32), ("ncgeom", i32),
        ("cgeom_id", _a(i32, MAX_CGEOM)), ("cgeom_type", _a(i32, MAX_CGEOM)),
        ("cgeom_bodyid", _a(i32, MAX_CGEOM)), ("cgeom_condim", _a(i32, MAX_CGEOM)),
        ("cgeom_priority", _a(i32, MAX_CGEOM)),
        ("cgeom_size", _a(d, MAX_CGEOM, 3)), ("cgeom_pos", _a(d, MAX_CGEOM, 3)),
        ("cgeom_quat", _a(d, MAX_CGEOM, 4)), ("cgeom_friction", _a(d, MAX_CGEOM, 3)),
        ("cgeom_solref", _a(d, MAX_CGEOM, 2)), ("cgeom_solimp", _a(d, MAX_CGEOM, 5)),
        ("cgeom_solmix", _a(d, MAX_CGEOM)), ("cgeom_margin", _a(d, MAX_CGEOM)),
        ("cgeom_gap", _a(d, MAX_CGEOM)),
        ("npair", i32), ("pair_g1", _a(i32, MAX_PAIR)), ("pair_g2", _a(i32, MAX_PAIR)),
        ("nsite", i32), ("site_bodyid", _a(i32, MAX_SITE)), ("site_pos", _a(d, MAX_SITE, 3)),
        ("site_quat", _a(d, MAX_SITE, 4)),
        ("actuator_trnid", _a(i32, NU)), ("actuator_biastype", _a(i32, NU)),
        ("actuator_forcelimited", _a(i32, NU)), ("actuator_ctrllimited", _a(i32, NU)),
        ("actuator_gear", _a(d, NU)), ("actuator_gainprm", _a(d, NU, 3)),
        ("actuator_biasprm", _a(d, NU, 3)), ("actuator_forcerange", _a(d, NU, 2)),
        ("actuator_ctrlrange", _a(d, NU, 2)),
        ("max_contact_points", i32), ("max_geom_pairs", i32),
        ("nsensor", i32), ("nsensordata", i32), ("sensor_type", _a(i32, MAX_SENSOR)),
        ("sensor_objid", _a(i32, MAX_SENSOR)), ("sensor_adr", _a(i32, MAX_SENSOR)), ("sensor_dim", _a(i32, MAX_SENSOR)),
        ("sensor_cutoff", _a(d, MAX_SENSOR)),
    ]


class EnvConfig(C.Structure):
    _fields_ = [
        ("n_frames", i32), ("obs_history", i32), ("use_imu", i32), ("latency_len", i32),
        ("imu_latency_len", i32), ("resample_velocity_step", i32),
        ("early_termination_step_threshold", i32), ("torso_body", i32),
        ("feet_site", _a(i32, NFOOT)), ("lower_leg_body", _a(i32, NFOOT)),
        ("n_upper_leg_geoms", i32), ("upper_leg_geoms", _a(i32, 16)),
        ("n_torso_geoms", i32), ("torso_geoms", _a(i32, 8)),
        ("rng_partitionable", i32), ("ncon_max", i32),
        ("latency_dist", _a(d, MAX_LAG)), ("imu_latency_dist", _a(d, MAX_LAG)),
        ("action_scale", d), ("default_pose", _a(d, NU)), ("joint_lower", _a(d, NU)),
        ("joint_upper", _a(d, NU)), ("desired_abduction", _a(d, 4)),
        ("start_pos_min", _a(d, 3)), ("start_pos_max", _a(d, 3)),
        ("lin_vel_x_range", _a(d, 2)), ("lin_vel_y_range", _a(d, 2)), ("ang_vel_range", _a(d, 2)),
        ("zero_command_probability", d), ("stand_still_command_threshold", d),
        ("max_pitch_command", d), ("max_roll_command", d),
        ("ang_vel_noise", d), ("gravity_noise", d), ("motor_angle_noise", d),
        ("last_action_noise", d), ("kick_vel", d), ("kick_probability", d),
        ("terminal_body_z", d), ("terminal_body_angle", d), ("foot_radius", d),
        ("env_dt", d), ("dt", d), ("desired_world_z", _a(d, 3)),
        ("reward_scales", _a(d, NREWARD)), ("tracking_sigma", d),
    ]


def state_stride(latency_len: int, imu_latency_len: int) -> int:
    return S_ACT_BUF + 12 * latency_len + 6 * imu_latency_len


def imu_buf_offset(latency_len: int) -> int:
    return S_ACT_BUF + 12 * latency_len
