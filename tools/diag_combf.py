"""Diagnostic (debug build ab/combf_dbg.so: -DPP3_DEBUG -DPP3_COM_BF=1 -DPP3_COM_CHECK): count, over
a few env steps at 4096 envs, the lanes where the straight-line com phase differs bit-wise from the
branchy form (g_dbg[100 + slot]: com 0..2, cinert 3..12, rotated inertia 30..38)."""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "pupperv3-mjx_amd")]
os.environ["PP3_LIB_PATH"] = os.path.join(ROOT, "ab_dbg", "combf_dbg.so")
os.environ["PP3_ALLOW_DIAG_BUILD"] = "1"
import numpy as np  # noqa: E402

import bench  # noqa: E402
from pupperv3_mjx import MODEL_XML, _lib, sharding  # noqa: E402
from pupperv3_mjx.environment import PupperV3Env  # noqa: E402

E = 4096
env = PupperV3Env(**bench.bench_kwargs(MODEL_XML), num_envs=E)
st = env.reset(sharding.shard_keys(0, E, 1, 0))
rs = np.random.RandomState(1)
for t in range(3):
    st = env.step(st, rs.uniform(-1, 1, (E, 12)).astype(np.float32))
_ = st.obs
L = _lib.load()
L.pp3_debug_read.argtypes = [C.c_void_p]
gd = np.zeros(512, dtype=np.float32)
L.pp3_debug_read(gd.ctypes.data_as(C.c_void_p))
print("com", gd[100:103], "cinert", gd[103:113], "A", gd[130:139], flush=True)
env.close()
