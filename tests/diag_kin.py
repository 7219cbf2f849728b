"""Diagnostic: body positions / orientations of one forward (pipeline record) vs the oracle."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "pupperv3-mjx_amd"), os.path.join(ROOT, "tests")]
import numpy as np  # noqa: E402

import common  # noqa: E402
import gpu_harness as G  # noqa: E402
from pupperv3_mjx import _abi  # noqa: E402

m = common.pd_model().struct
e = G.env_with_model(common.MODEL_XML, m, 4)
qpos, qvel, qws, ctrl = common.random_physics_states(4, seed=1)
gq, gv, gw, gp = G.gpu_physics(e, qpos, qvel, qws, ctrl, 1)
oq, ov, ow, op = G.oracle_physics(m, qpos, qvel, qws, ctrl, 1)
np.set_printoptions(precision=5, suppress=True, linewidth=160)
for k, n in ((_abi.P_XPOS, 3), (_abi.P_XQUAT, 4)):
    g = gp[0, k:k + 13 * n].reshape(13, n)
    o = op[0, k:k + 13 * n].reshape(13, n)
    print("field", k, "max err per body", np.abs(g - o).max(axis=1))
print("qpos err", np.abs(gq - oq).max())
