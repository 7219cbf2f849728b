"""pupperv3_mjx.rewards (host restatement of rewards.py:9-138, the reference's public module).

* known answers for every term on hand-built states;
* every term, evaluated from the oracle's step outputs (Brax x / xd, site_xpos, qfrc_actuator,
  contacts of the pipeline record) and the pre-step info exactly as environment.py:371-444
  calls them, equals the oracle's own reward stack term by term (all scales 1: nothing hidden);
* the same against the HIP kernel's per-term metrics, from the kernel's own pipeline record
  (``-m gpu``): the kernel's fused reward epilogue agrees with the reference formulas applied to
  the kernel's physics outputs.
"""
import numpy as np
import pytest

import common
from oracle import oracle as O
from pupperv3_mjx import _abi, config, rewards as R
from pupperv3_mjx.environment import Contact, Motion, PipelineState, Transform, make_keys

DISCRETE = ("termination", "knee_collision", "body_collision")


def _q(axis, ang):
    a = np.asarray(axis, float) / np.linalg.norm(axis)
    return np.concatenate([[np.cos(ang / 2)], np.sin(ang / 2) * a])


# ------------------------------------------------------------------ known answers
def test_known_answers():
    nb = 13
    rot = np.tile([1.0, 0, 0, 0], (nb, 1))
    x = Transform(pos=np.zeros((nb, 3)), rot=rot.copy())
    xd = Motion(vel=np.zeros((nb, 3)), ang=np.zeros((nb, 3)))
    xd.vel[0] = [0.3, -0.2, 0.5]
    xd.ang[0] = [0.1, 0.2, 0.7]
    assert R.reward_lin_vel_z(xd) == pytest.approx(0.25)
    assert R.reward_ang_vel_xy(xd) == pytest.approx(0.05)
    assert R.reward_orientation(x) == pytest.approx(0.0)
    assert R.reward_tracking_lin_vel(np.array([0.3, -0.2, 0.0]), x, xd, 0.25) == pytest.approx(1.0)
    assert R.reward_tracking_ang_vel(np.array([0, 0, 0.2]), x, xd, 0.25) == pytest.approx(np.exp(-0.25 / 0.25))
    # body yawed by 90 deg: world x velocity is body -y
    x.rot[0] = _q([0, 0, 1], np.pi / 2)
    assert R.reward_tracking_lin_vel(np.array([0.0, -0.3, 0.0]), x, xd, 0.25) == pytest.approx(np.exp(-0.04 / 0.25))
    # body pitched by 30 deg: up axis tilts by sin(30) in x, world z in body frame tilts the other way
    x.rot[0] = _q([0, 1, 0], np.pi / 6)
    assert R.reward_orientation(x) == pytest.approx(0.25)
    dz = np.array([-0.5, 0.0, np.sqrt(3) / 2])
    assert R.reward_tracking_orientation(dz, x, 0.25) == pytest.approx(1.0)
    assert R.reward_tracking_orientation(np.array([0, 0, 1.0]), x, 0.25) < 1.0
    t = np.arange(12.0)
    assert R.reward_torques(t) == pytest.approx(np.sum(t * t))
    assert R.reward_mechanical_work(t, -np.ones(12)) == pytest.approx(np.sum(t))
    assert R.reward_joint_acceleration(np.ones(12), np.zeros(12), 0.02) == pytest.approx(12 * 2500)
    assert R.reward_action_rate(np.ones(12), np.zeros(12)) == pytest.approx(12)
    ang = np.zeros(12)
    ang[1::3] = [0.1, -0.1, 0.2, 0.0]
    assert R.reward_abduction_angle(ang) == pytest.approx(0.06)
    assert R.reward_abduction_angle(ang, np.array([0.1, -0.1, 0.2, 0.0])) == pytest.approx(0.0)
    assert R.reward_stand_still(np.array([0.01, 0, 0]), ang, np.zeros(12), 0.1) == pytest.approx(0.4)
    assert R.reward_stand_still(np.array([0.5, 0, 0]), ang, np.zeros(12), 0.1) == 0.0
    air = np.array([0.3, 0.05, 0.0, 0.2])
    first = np.array([1, 1, 0, 0])
    assert R.reward_feet_air_time(air, first, np.array([0.5, 0, 0])) == pytest.approx(0.2 - 0.05)
    assert R.reward_feet_air_time(air, first, np.array([0.01, 0.01, 0])) == 0.0
    assert bool(R.reward_termination(True, 10, 500)) and not bool(R.reward_termination(True, 500, 500))
    assert not bool(R.reward_termination(False, 10, 500))
    con = Contact(dist=np.array([-0.01, 0.02, -0.003, -0.2]), geom1=np.array([0, 0, 5, 7]),
                  geom2=np.array([5, 6, 9, 5]))
    ps = PipelineState(q=None, qd=None, qacc_warmstart=None, contact=con)
    assert R.reward_geom_collision(ps, [5]) == 3          # slots 0, 2, 3 (slot 1 separated)
    con.ncon = 2                                          # slots past the contact count are empty
    assert R.reward_geom_collision(ps, [5]) == 1
    assert R.reward_geom_collision(ps, [6, 9]) == 0
    # foot slip: a lower leg spinning about z at the foot's offset moves the foot sideways
    ps = PipelineState(q=None, qd=None, qacc_warmstart=None, x=Transform(pos=np.zeros((nb, 3)), rot=rot),
                       xd=Motion(vel=np.zeros((nb, 3)), ang=np.zeros((nb, 3))), site_xpos=np.zeros((4, 3)))
    legs = np.array([4, 7, 10, 13])
    ps.xd.ang[legs - 1] = [0, 0, 2.0]
    ps.site_xpos[:] = [0.1, 0, 0]                         # foot 0.1 m along x from each lower leg
    assert R.reward_foot_slip(ps, np.array([1, 0, 0, 1]), np.arange(4), legs) == pytest.approx(2 * 0.04)


# ------------------------------------------------------------------ the env's reward stack
def _ps_from_pipe(p):
    """PipelineState (Brax view, as PupperV3Env builds it) from pipeline records [..., PIPE_STRIDE]."""
    nb = _abi.NBODY - 1
    lead = p.shape[:-1]
    ps = PipelineState(q=None, qd=None, qacc_warmstart=None)
    ps.x = Transform(pos=p[..., _abi.P_XPOS:_abi.P_XPOS + 3 * nb].reshape(lead + (nb, 3)),
                     rot=p[..., _abi.P_XQUAT:_abi.P_XQUAT + 4 * nb].reshape(lead + (nb, 4)))
    ps.xd = Motion(vel=p[..., _abi.P_XD_VEL:_abi.P_XD_VEL + 3 * nb].reshape(lead + (nb, 3)),
                   ang=p[..., _abi.P_XD_ANG:_abi.P_XD_ANG + 3 * nb].reshape(lead + (nb, 3)))
    ps.site_xpos = p[..., _abi.P_SITE_XPOS:_abi.P_SITE_XPOS + 12].reshape(lead + (4, 3))
    ps.qfrc_actuator = p[..., _abi.P_QFRC_ACT:_abi.P_QFRC_ACT + 18]
    g = p[..., _abi.P_CON_GEOM:_abi.P_CON_GEOM + 32].reshape(lead + (16, 2)).astype(np.int64)
    ps.contact = Contact(dist=p[..., _abi.P_CON_DIST:_abi.P_CON_DIST + 16], geom1=g[..., 0], geom2=g[..., 1])
    ps.contact.ncon = p[..., _abi.P_NCON].astype(np.int64)
    return ps


def env_terms(env, rec0, action, rec1, pipe1, done1):
    """environment.py:371-444 through pupperv3_mjx.rewards: the unscaled terms of the step
    rec0 -> rec1 (state records), with the step's pipeline record and done."""
    c = env.config_struct
    sigma = env._reward_config.rewards.tracking_sigma
    ps = _ps_from_pipe(pipe1)
    q, qd = rec1[..., _abi.S_QPOS:_abi.S_QPOS + 19], rec1[..., _abi.S_QVEL:_abi.S_QVEL + 18]
    joint_angles, joint_vel = q[..., 7:], qd[..., 6:]
    last_contact = rec0[..., _abi.S_LAST_CONTACT:_abi.S_LAST_CONTACT + 4] != 0
    air0 = rec0[..., _abi.S_AIR_TIME:_abi.S_AIR_TIME + 4]
    cmd = rec0[..., _abi.S_COMMAND:_abi.S_COMMAND + 3]
    dz = rec0[..., _abi.S_DESIRED_Z:_abi.S_DESIRED_Z + 3]
    foot_z = ps.site_xpos[..., 2] - c.foot_radius
    contact = foot_z < 1e-3
    filt_mm = contact | last_contact
    filt_cm = (foot_z < 3e-2) | last_contact
    first = (air0 > 0) * filt_mm
    return {
        "tracking_lin_vel": R.reward_tracking_lin_vel(cmd, ps.x, ps.xd, sigma),
        "tracking_ang_vel": R.reward_tracking_ang_vel(cmd, ps.x, ps.xd, sigma),
        "tracking_orientation": R.reward_tracking_orientation(dz, ps.x, sigma),
        "lin_vel_z": R.reward_lin_vel_z(ps.xd),
        "ang_vel_xy": R.reward_ang_vel_xy(ps.xd),
        "orientation": R.reward_orientation(ps.x),
        "torques": R.reward_torques(ps.qfrc_actuator),
        "joint_acceleration": R.reward_joint_acceleration(joint_vel, rec0[..., _abi.S_LAST_VEL:_abi.S_LAST_VEL + 12],
                                                          env._dt),
        "mechanical_work": R.reward_mechanical_work(ps.qfrc_actuator[..., 6:], qd[..., 6:]),
        "action_rate": R.reward_action_rate(action, rec0[..., _abi.S_LAST_ACT:_abi.S_LAST_ACT + 12]),
        "stand_still": R.reward_stand_still(cmd, joint_angles, env._default_pose, 0.1),
        "stand_still_joint_velocity": R.reward_stand_still(cmd, joint_vel, np.zeros(12),
                                                           c.stand_still_command_threshold),
        "abduction_angle": R.reward_abduction_angle(joint_angles, np.array(c.desired_abduction[:])),
        "feet_air_time": R.reward_feet_air_time(air0 + env.dt, first, cmd),
        "foot_slip": R.reward_foot_slip(ps, filt_cm, env._feet_site_id, env._lower_leg_body_id),
        "termination": R.reward_termination(done1, rec0[..., _abi.S_STEP], c.early_termination_step_threshold),
        "knee_collision": R.reward_geom_collision(ps, env._upper_leg_geom_ids),
        "body_collision": R.reward_geom_collision(ps, env._torso_geom_ids),
    }, foot_z


def all_ones_config():
    cfg = config.get_config()
    for k in list(cfg.rewards.scales.keys()):
        cfg.rewards.scales[k] = 1.0
    return cfg


def compare_terms(terms, metrics, rtol, atol, where):
    """metrics: [19] (total_dist, then REWARD_NAMES order) with every scale 1."""
    for i, k in enumerate(_abi.REWARD_NAMES):
        h, m = float(terms[k]), float(metrics[1 + i])
        if k in DISCRETE:
            assert h == m, f"{where}: {k} host {h} vs {m}"
        else:
            assert abs(h - m) <= atol + rtol * abs(m), f"{where}: {k} host {h:.9g} vs {m:.9g}"


def test_reward_module_reproduces_oracle_reward_stack(tmp_path):
    path = common.write_model(tmp_path)
    m, cfg, env = common.env_model_and_config(path, reward_config=all_ones_config(), resample_velocity_step=4,
                                              zero_command_probability=0.3)
    oe = O.OracleEnv(m, cfg)
    rs = np.random.RandomState(5)
    keys = make_keys(2, 6)
    nonzero = set()
    for e, k in enumerate(keys):
        s = oe.reset(k)
        for t in range(40):
            a = rs.uniform(-1, 1, 12)
            o = oe.step(s, a)
            terms, _ = env_terms(env, s["state"], a, o["state"], o["pipe"], o["done"])
            compare_terms(terms, o["metrics"], 1e-7, 1e-9, f"env {e} step {t}")
            nonzero.update(kk for kk in _abi.REWARD_NAMES if terms[kk] != 0)
            s = o
    # the rollout exercised (nearly) every term
    assert len(nonzero) >= 14, sorted(set(_abi.REWARD_NAMES) - nonzero)


@pytest.mark.gpu
def test_reward_module_reproduces_kernel_metrics(require_gpu, tmp_path):
    from pupperv3_mjx.environment import PupperV3Env
    path = common.write_model(tmp_path)
    n, steps = 64, 30
    env = PupperV3Env(**common.fixture_kwargs(path, reward_config=all_ones_config(), resample_velocity_step=4,
                                              zero_command_probability=0.3), num_envs=n)
    try:
        st = env.reset(make_keys(4, n))
        rs = np.random.RandomState(9)
        worst = {}
        flips = 0
        for t in range(steps):
            a = rs.uniform(-1, 1, (n, 12)).astype(np.float32)
            nx = env.step(st, a)
            p = env._get(_abi.F_PIPELINE)
            terms, foot_z = env_terms(env, st._record, a, nx._record, p, nx.done)
            for i in range(n):
                # a foot height within rounding of a contact threshold may decide differently
                near = np.abs(foot_z[i] - 1e-3).min() < 1e-6 or np.abs(foot_z[i] - 3e-2).min() < 1e-6
                try:
                    compare_terms({k: v[i] for k, v in terms.items()}, nx._metrics_raw[i], 2e-3, 2e-4,
                                  f"env {i} step {t}")
                except AssertionError:
                    if not near:
                        raise
                    flips += 1
            for j, k in enumerate(_abi.REWARD_NAMES):
                worst[k] = max(worst.get(k, 0.0), float(np.abs(terms[k] - nx._metrics_raw[:, 1 + j]).max()))
            st = nx
        assert flips <= 0.01 * n * steps
        print("REPORT rewards-module vs kernel worst abs error per term:", worst, "threshold flips:", flips)
    finally:
        env.close()
