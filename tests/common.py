"""Shared builders: the reference test fixture's env kwargs (test_environment.py:64-113)."""
import copy
import os
import xml.etree.ElementTree as ET

import numpy as np

from pupperv3_mjx import MODEL_XML, _abi, config, domain_randomization, mjcf, obstacles

DEFAULT_POSE = [0.26, 0.0, -0.52, -0.26, 0.0, 0.52, 0.26, 0.0, -0.52, -0.26, 0.0, 0.52]
GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def model_with_obstacles_xml(n=10):
    tree = ET.ElementTree(ET.fromstring(open(MODEL_XML).read()))
    obstacles.add_boxes_to_model(tree, n_boxes=n, x_range=(-5, 5), y_range=(-5, 5), height=0.02, length=6.0)
    return ET.tostring(tree.getroot(), encoding="unicode")


def write_model(tmp_path, obstacles_n=0):
    if obstacles_n:
        xml = model_with_obstacles_xml(obstacles_n)
    else:
        xml = open(MODEL_XML).read()
    os.makedirs(str(tmp_path), exist_ok=True)
    p = os.path.join(str(tmp_path), f"model_{obstacles_n}.xml")
    with open(p, "w") as f:
        f.write(xml)
    return p


def fixture_kwargs(path, **over):
    """test_environment.py:64-113 env kwargs (joint limits taken from the model's jnt_range)."""
    cm = mjcf.load(path)
    kw = dict(
        path=path, action_scale=0.75, observation_history=2,
        joint_lower_limits=list(cm.jnt_range[1:, 0]), joint_upper_limits=list(cm.jnt_range[1:, 1]),
        dof_damping=0.25, position_control_kp=5.0,
        foot_site_names=["leg_front_r_3_foot_site", "leg_front_l_3_foot_site", "leg_back_r_3_foot_site",
                         "leg_back_l_3_foot_site"],
        torso_name="base_link",
        upper_leg_body_names=["leg_front_r_2", "leg_front_l_2", "leg_back_r_2", "leg_back_l_2"],
        lower_leg_body_names=["leg_front_r_3", "leg_front_l_3", "leg_back_r_3", "leg_back_l_3"],
        resample_velocity_step=100, linear_velocity_x_range=[-0.75, 0.75], linear_velocity_y_range=[-0.5, 0.5],
        angular_velocity_range=[-2.0, 2.0], maximum_pitch_command=30, maximum_roll_command=30,
        default_pose=DEFAULT_POSE,
        start_position_config=domain_randomization.StartPositionRandomization(
            x_min=-1.0, x_max=1.0, y_min=-1.0, y_max=1.0, z_min=0.18, z_max=0.24),
        reward_config=config.get_config(), kick_vel=1.0, kick_probability=0.04, terminal_body_z=0.1,
        early_termination_step_threshold=500,
    )
    kw.update(over)
    return kw


def env_model_and_config(path, **over):
    """(model struct, env config struct, host-only env) built exactly as PupperV3Env.__init__ does."""
    from pupperv3_mjx.environment import PupperV3Env
    env = PupperV3Env(**fixture_kwargs(path, **over), create_device=False)
    return env.sys_model.struct, env.config_struct, env


def pd_model(path=None):
    """Model with the env's PD overrides (Kp=5, Kd=0.25) and dt=0.004."""
    cm = mjcf.load(path or MODEL_XML)
    m = cm.struct
    m.timestep = 0.004
    for i in range(12):
        m.actuator_gainprm[i][0] = 5.0
        m.actuator_biasprm[i][1] = -5.0
        m.actuator_biasprm[i][2] = -0.25
    return cm


def random_physics_states(n, seed=0, mode="mixed"):
    """Seeded initial (qpos, qvel, qacc_ws, ctrl) covering air, standing and contact-rich cases."""
    rs = np.random.RandomState(seed)
    qpos = np.zeros((n, 19))
    qvel = np.zeros((n, 18))
    ctrl = np.zeros((n, 12))
    for i in range(n):
        kind = mode if mode != "mixed" else ("air", "stand", "low", "tilt")[i % 4]
        yaw = rs.uniform(-np.pi, np.pi)
        q = np.array([np.cos(yaw / 2), 0, 0, np.sin(yaw / 2)])
        z = {"air": 0.5, "stand": 0.155, "low": 0.12, "tilt": 0.16}[kind]
        if kind == "tilt":
            ax = rs.normal(size=3)
            ax /= np.linalg.norm(ax)
            ang = rs.uniform(0.2, 0.8)
            dq = np.concatenate([[np.cos(ang / 2)], ax * np.sin(ang / 2)])
            q = mjcf.quat_mul(q, dq)
        qpos[i, :3] = [rs.uniform(-1, 1), rs.uniform(-1, 1), z]
        qpos[i, 3:7] = q
        qpos[i, 7:] = np.array(DEFAULT_POSE) + rs.uniform(-0.3, 0.3, 12)
        qvel[i] = rs.normal(scale=0.3, size=18)
        ctrl[i] = np.array(DEFAULT_POSE) + rs.uniform(-0.5, 0.5, 12)
    return qpos, qvel, np.zeros((n, 18)), ctrl


def states_on_boxes(model, n, seed=0, z_range=(0.15, 0.175)):
    """Seeded (qpos, qvel, qacc_ws, ctrl) with the robot straddling the obstacle walls
    (obstacles.py boxes: 2 cm wide, 6 m long, top at z=0.02) so sphere-box contacts occur."""
    rs = np.random.RandomState(seed)
    boxes = [g for g in range(model.ncgeom) if model.cgeom_type[g] == _abi.GEOM_BOX]
    assert boxes, "model has no box geoms"
    qpos, qvel, qws, ctrl = random_physics_states(n, seed=seed, mode="stand")
    for i in range(n):
        g = boxes[rs.randint(len(boxes))]
        c = np.array(model.cgeom_pos[g][:])
        w, x, y, z = model.cgeom_quat[g][:]
        # box local y axis (the 6 m length) in world
        ay = np.array([2 * (x * y - w * z), 1 - 2 * (x * x + z * z), 2 * (y * z + w * x)])
        t = rs.uniform(-2.5, 2.5)
        p = c + t * ay + np.array([rs.uniform(-0.12, 0.12), rs.uniform(-0.12, 0.12), 0.0])
        qpos[i, 0:2] = p[:2]
        qpos[i, 2] = rs.uniform(*z_range)
        qvel[i] *= 0.3
    return qpos, qvel, qws, ctrl


def _leg_of_body(b):
    return -1 if b == 0 else (4 if b == 1 else (b - 2) // 3)


def states_with_self_contact(model, jnt_range, n, seed=0, z=0.5, kind="any"):
    """Seeded states (joint angles uniform in their ranges, base at height z) in which at least
    one contact is between two robot geoms (a sphere-sphere pair of two different legs), found
    by rejection sampling against the oracle.  These contacts couple two legs in the Jacobian,
    which takes the kernel's leg-leg Newton path (dense_search).  kind="disjoint": the contacts
    couple two disjoint pairs of legs (no leg common to all), which the kernel can only factor
    densely; "any": at least one leg-leg contact (one pair: the arrowhead solve with that pair's
    leg in the base block)."""
    from oracle import oracle as O
    static = {int(model.cgeom_id[g]) for g in range(model.ncgeom) if model.cgeom_bodyid[g] == 0}
    body = {int(model.cgeom_id[g]): int(model.cgeom_bodyid[g]) for g in range(model.ncgeom)}
    rs = np.random.RandomState(seed)
    lo, hi = jnt_range[1:, 0], jnt_range[1:, 1]
    qs = []
    while len(qs) < n:
        q = np.zeros(19)
        q[2], q[3] = z, 1
        q[7:] = rs.uniform(lo, hi)
        p = O.mj_step(model, q, np.zeros(18), np.zeros(18), q[7:].copy(), nsteps=1)[3]
        k = int(p[_abi.P_NCON])
        g = p[_abi.P_CON_GEOM:_abi.P_CON_GEOM + 2 * k].reshape(k, 2).astype(int)
        if kind == "any":
            if any(a not in static and b not in static for a, b in g):
                qs.append(q)
            continue
        pairs = set()
        for a, b in g:
            la, lb = _leg_of_body(body[a]), _leg_of_body(body[b])
            if 0 <= la < 4 and 0 <= lb < 4 and la != lb:
                pairs.add((min(la, lb), max(la, lb)))
        if len(pairs) > 1 and not any(all(x in pr for pr in pairs) for x in range(4)):
            qs.append(q)
    qpos = np.array(qs)
    qvel = rs.normal(scale=0.3, size=(n, 18))
    return qpos, qvel, np.zeros((n, 18)), qpos[:, 7:].copy()


from oracle.oracle import model_with_terrain, terrain_slots  # noqa: E402  (the oracle's terrain view)

assert _abi.GEOM_BOX == 6


def model_terrain_rows(model):
    """The model's own static boxes as one terrain row f32[n_boxes, 10]."""
    return np.array([[*model.cgeom_pos[g][:], *model.cgeom_quat[g][:], *model.cgeom_size[g][:]]
                     for g in terrain_slots(model)], dtype=np.float32)


def terrain_under(xy, n_boxes, seed=0, absent_p=0.3):
    """Per-env terrain f32[n, n_boxes, 10]: slot 0 is a rail (obstacles.py sizes) straddled by
    the robot at xy[i], slot 1 a second rail crossing nearby, the other slots random boxes of
    the reference's distribution or (probability absent_p) absent."""
    rs = np.random.RandomState(seed)
    n = xy.shape[0]
    t = obstacles.sample_terrain(n, n_boxes, (-5, 5), (-5, 5), seed=seed)
    for i in range(n):
        for slot in (0, 1):
            yaw = rs.uniform(-np.pi, np.pi)
            ax = np.array([-np.sin(yaw), np.cos(yaw)])  # rail's long (local y) axis in world
            nrm = np.array([np.cos(yaw), np.sin(yaw)])
            c = xy[i] + nrm * rs.uniform(-0.12, 0.12) + ax * rs.uniform(-1.0, 1.0)
            t[i, slot, 0:3] = (c[0], c[1], 0.0)
            t[i, slot, 3:7] = (np.cos(yaw / 2), 0.0, 0.0, np.sin(yaw / 2))
            t[i, slot, 7:10] = (0.01, 1.5, 0.02)
        for slot in range(2, n_boxes):
            if rs.uniform() < absent_p:
                t[i, slot, 7:10] = 0.0
    return t
