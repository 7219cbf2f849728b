"""obstacles.py golden fixture (generated from the reference module), MJCF compiler, XML editors."""
import json
import os
import xml.etree.ElementTree as ET

import numpy as np
import pytest

import common
from pupperv3_mjx import MODEL_XML, _abi, mjcf, obstacles, utils


@pytest.mark.parametrize("case", ["seed0_n10_len6.0", "seed3_n25_len3.0"])
def test_obstacles_match_reference_golden(case):
    gold = json.load(open(os.path.join(common.GOLDEN, "obstacles_golden.json")))[case]
    seed = int(case.split("_")[0][4:])
    n = int(case.split("_")[1][1:])
    length = float(case.split("len")[1])
    tree = ET.ElementTree(ET.fromstring(open(MODEL_XML).read()))
    obstacles.add_boxes_to_model(tree, n_boxes=n, x_range=(-5, 5), y_range=(-5, 5), height=0.02, length=length,
                                 seed=seed)
    boxes = [dict(g.attrib) for g in tree.getroot().find("worldbody").findall("geom")
             if g.get("name", "").startswith("box_geom_")]
    assert boxes == gold


def test_model_counts():
    cm = mjcf.load(MODEL_XML)
    m = cm.struct
    assert cm.ngeom == 23 and m.ncgeom == 9 and m.npair == 32 and m.nsite == 5
    assert abs(sum(m.body_mass[:]) - 3.17) < 1e-12
    assert list(cm.body_geom_ids("base_link")) == [2]
    assert [list(cm.body_geom_ids(n)) for n in ("leg_front_r_2", "leg_front_l_2", "leg_back_r_2", "leg_back_l_2")] \
        == [[4, 5], [9, 10], [14, 15], [19, 20]]
    assert cm.site_id("leg_back_l_3_foot_site") == 4
    assert list(m.dof_armature[:6]) == [0] * 6 and list(m.dof_armature[6:]) == [0.0016] * 12
    assert list(m.dof_frictionloss[6:]) == [0.125] * 12 and list(m.dof_damping[6:]) == [0.01] * 12
    assert list(m.jnt_limited[:]) == [0] + [1] * 12
    assert list(m.actuator_forcelimited[:]) == [1] * 12 and list(m.actuator_ctrllimited[:]) == [0] * 12
    assert m.iterations == 1 and m.ls_iterations == 5 and m.impratio == 10 and m.eulerdamp == 0
    assert m.max_contact_points == 5 and m.max_geom_pairs == 4
    # the 8 sphere-plane + 24 sphere-sphere candidates (parent-child legs filtered)
    types = [(m.cgeom_type[m.pair_g1[p]], m.cgeom_type[m.pair_g2[p]]) for p in range(m.npair)]
    assert types.count((0, 2)) == 8 and types.count((2, 2)) == 24


def test_obstacle_model_pairs():
    xml = common.model_with_obstacles_xml(10)
    cm = mjcf.load(xml, is_string=True)
    m = cm.struct
    assert cm.ngeom == 33 and m.npair == 32 + 80
    # grouped by geom-type pair: the robot's 32 candidates first (the kernel's prefetched batch),
    # then the sphere-box pairs that pp3_env.hip's collision() culls box by box
    types = [(m.cgeom_type[m.pair_g1[p]], m.cgeom_type[m.pair_g2[p]]) for p in range(m.npair)]
    assert types == [(0, 2)] * 8 + [(2, 2)] * 24 + [(2, 6)] * 80


def test_invweight_and_mass_matrix_cross_check():
    """mjcf's numpy M (sum of J'MJ) equals the oracle's CRB M; invweight0 is diag-based and positive."""
    from oracle import oracle as O
    cm = common.pd_model()
    m = cm.struct
    rs = np.random.RandomState(0)
    for _ in range(5):
        q = np.zeros(19)
        q[:3] = rs.normal(size=3)
        qq = rs.normal(size=4)
        q[3:7] = qq / np.linalg.norm(qq)
        q[7:] = rs.uniform(-1, 1, 12)
        M_np, _, _, _ = mjcf.mass_matrix_and_jacobians(m, q)
        M_or = O.mj_forward(m, q, np.zeros(18), np.zeros(18), np.zeros(12))["M"]
        np.testing.assert_allclose(M_or, M_np, rtol=1e-10, atol=1e-12)
        assert np.all(np.linalg.eigvalsh(M_or) > 0)
    assert np.all(np.array(m.dof_invweight0[:]) > 0)
    assert np.all(np.array(m.body_invweight0[1:]) > 0)
    assert abs(m.meaninertia - np.trace(mjcf.mass_matrix_and_jacobians(m, np.array(m.qpos0[:]))[0]) / 18) < 1e-12


def test_set_starting_position():
    tree = ET.ElementTree(ET.fromstring(open(MODEL_XML).read()))
    utils.set_robot_starting_position(tree, starting_pos=[0.1, 0.2, 0.5], starting_quat=[0.1, 0.2, 0.3, 0.4])
    body = tree.find(".//worldbody/body[@name='base_link']")
    assert body.get("pos").split(" ") == ["0.1", "0.2", "0.5"]
    assert body.get("quat").split(" ") == ["0.1", "0.2", "0.3", "0.4"]
    home = tree.find(".//keyframe/key[@name='home']")
    assert list(map(float, home.get("qpos").split(" ")))[:7] == [0.1, 0.2, 0.5, 0.1, 0.2, 0.3, 0.4]


def test_set_mjx_custom_options():
    tree = ET.ElementTree(ET.fromstring(open(MODEL_XML).read()))
    utils.set_mjx_custom_options(tree, max_contact_points=9, max_geom_pairs=7)
    cm = mjcf.load(tree)
    assert cm.struct.max_contact_points == 9 and cm.struct.max_geom_pairs == 7


def test_unsupported_features_fail_loudly():
    xml = open(MODEL_XML).read().replace('cone="pyramidal"', 'cone="elliptic"')
    with pytest.raises(NotImplementedError):
        mjcf.load(xml, is_string=True)


def test_sample_terrain_distribution_and_absent_slots():
    """Per-env terrain rows follow one obstacles.py:16-57 box draw per slot."""
    t = obstacles.sample_terrain(256, 10, (-5, 5), (-4, 4), height=0.02, depth=0.02, length=6.0, seed=3, min_boxes=2)
    assert t.shape == (256, 10, 10) and t.dtype == np.float32
    present = np.any(t[..., 7:10] > 0, axis=2)
    assert present[:, :2].all() and not present.all()  # at least min_boxes, some absent
    p = t[present]
    assert np.all(np.abs(p[:, 0]) <= 5) and np.all(np.abs(p[:, 1]) <= 4) and np.all(p[:, 2] == 0)
    np.testing.assert_allclose(np.linalg.norm(p[:, 3:7], axis=1), 1, atol=1e-6)
    assert np.all(p[:, 4:6] == 0)
    np.testing.assert_allclose(p[:, 7:10], np.broadcast_to([0.01, 3.0, 0.02], p[:, 7:10].shape), rtol=1e-6)
    a = obstacles.sample_terrain(4, 10, (-5, 5), (-5, 5), seed=0)
    b = obstacles.sample_terrain(4, 10, (-5, 5), (-5, 5), seed=0)
    np.testing.assert_array_equal(a, b)


def test_terrain_from_specs_equals_model_boxes(tmp_path):
    """The static reference layout as terrain rows == the compiled model's box geoms, and the
    oracle's per-env-terrain model view of those rows reproduces the model's physics."""
    from oracle import oracle as O
    path = common.write_model(tmp_path, 10)
    m = mjcf.load(path).struct
    specs = obstacles.sample_boxes(10, (-5, 5), (-5, 5), height=0.02, length=6.0, seed=0)
    rows = obstacles.terrain_from_specs(specs, 3)
    np.testing.assert_allclose(rows[1], common.model_terrain_rows(m), rtol=0, atol=1e-6)
    mt = common.model_with_terrain(m, common.model_terrain_rows(m))
    qpos, qvel, qws, ctrl = common.states_on_boxes(m, 4, seed=1)
    for i in range(4):
        a = O.mj_step(m, qpos[i], qvel[i], qws[i], ctrl[i], nsteps=2)
        b = O.mj_step(mt, qpos[i], qvel[i], qws[i], ctrl[i], nsteps=2)
        np.testing.assert_allclose(a[0], b[0], rtol=0, atol=1e-6)


def test_rail_start_xy_on_the_boxes():
    """configs[4] starts (bench.py --obstacles, test_gpu_headline): each position lies over its box,
    within the lateral offset of the centre line and the middle `along` fraction of its length."""
    import math
    import numpy as np
    specs = obstacles.sample_boxes(10, (-5, 5), (-5, 5), 0.02, length=6.0)
    xy = obstacles.rail_start_xy(specs, 500, seed=1, offset=0.06, along=0.8)
    for i, (x, y) in enumerate(xy):
        b = specs[i % 10]
        yaw = 2.0 * math.atan2(b.quat[3], b.quat[0])
        dx, dy = x - b.x, y - b.y
        lx = dx * math.cos(yaw) + dy * math.sin(yaw)   # across the rail
        ly = -dx * math.sin(yaw) + dy * math.cos(yaw)  # along the rail
        assert abs(lx) <= 0.06 + 1e-12 and abs(ly) <= 0.8 * 3.0 + 1e-12
    assert np.ptp(xy[:, 0]) > 1.0  # spread over the field, not one spot
