"""Diagnostic: Newton intermediates (debug builds) GPU vs oracle for the diag_env11 state."""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "pupperv3-mjx_amd"), os.path.join(ROOT, "tests")]
os.environ["PP3_LIB_PATH"] = os.path.join(ROOT, "pupperv3-mjx_amd", "pupperv3_mjx", "libpupper_hip_dbg.so")
os.environ["PP3_ALLOW_DIAG_BUILD"] = "1"  # pp3_diag.h: the debug library refuses to run otherwise
import tempfile  # noqa: E402

import numpy as np  # noqa: E402

import common  # noqa: E402
import gpu_harness as G  # noqa: E402
from oracle import oracle as O  # noqa: E402
from pupperv3_mjx import _abi, _lib  # noqa: E402
from pupperv3_mjx import rng as R  # noqa: E402
from pupperv3_mjx.environment import PupperV3Env, make_keys  # noqa: E402

np.set_printoptions(precision=5, suppress=True, linewidth=220)
d = tempfile.mkdtemp()
path = common.write_model(d, 10)
kw = common.fixture_kwargs(path, latency_distribution=[0.1, 0.2, 0.3, 0.4], imu_latency_distribution=[0.2, 0.3, 0.5])
n = 16
e = PupperV3Env(**kw, num_envs=n)
st = e.reset(make_keys(9, n))
rs = np.random.RandomState(4)
for t in range(7):
    a = rs.uniform(-1, 1, size=(n, 12)).astype(np.float32)
    prev = st
    st = e.step(prev, a)
i = 11
rec0, rec1 = prev._record[i], st._record[i]
La = e.config_struct.latency_len
ks = R.split(rec0[_abi.S_RNG:_abi.S_RNG + 2].copy().view(np.uint32), 5)
li = int(R.choice_index(ks[4], np.array(kw["latency_distribution"], dtype=np.float32)))
buf = rec1[_abi.S_ACT_BUF:_abi.S_ACT_BUF + 12 * La].reshape(12, La)
ctrl = np.clip(np.array(kw["default_pose"]) + buf[:, li] * 0.75, e.lowers, e.uppers)
q0 = rec0[0:19].astype(np.float64)
v0 = rec0[19:37].astype(np.float64)
v0[0:2] += rec1[_abi.S_KICK:_abi.S_KICK + 2]
w0 = rec0[37:55].astype(np.float64)
e1 = PupperV3Env(**kw, num_envs=1)
m = e1.sys_model.struct
oq1, ov1, ow1, _ = G.oracle_physics(m, q0[None], v0[None], w0[None], ctrl[None], 1)
L = _lib.load()
L.pp3_debug_read.argtypes = [C.c_void_p]
gq, gv, gw, gp = G.gpu_physics(e1, oq1, ov1, ow1, ctrl[None], 1)
gd = np.zeros(512, dtype=np.float32)
L.pp3_debug_read(gd.ctypes.data_as(C.c_void_p))
OL = O.lib("f64")
OL.orc_debug_read.argtypes = [C.POINTER(C.c_double)]
oq, ov, ow, op = G.oracle_physics(m, oq1, ov1, ow1, ctrl[None], 1)
od = np.zeros(512)
OL.orc_debug_read(od.ctypes.data_as(C.POINTER(C.c_double)))
for name, sl in (("qacc0", slice(0, 18)), ("grad", slice(18, 36)), ("search", slice(36, 54))):
    print(name, "gpu", gd[sl], "\n      orc", od[sl])
print("gauss q1 q2 sn gtol alpha evals cws csm nefc")
print("gpu", gd[54:64])
print("orc", od[54:64])

Hg = gd[64:64 + 324].reshape(18, 18)
Ho = od[64:64 + 324].reshape(18, 18)
print("H max abs diff", np.abs(Hg - Ho).max(), "at", np.unravel_index(np.argmax(np.abs(Hg - Ho)), (18, 18)))
print("H diag gpu", np.diag(Hg), "\n       orc", np.diag(Ho))
dd = np.abs(Hg - Ho) > 1e-3 * (np.abs(Ho) + 1)
print("mismatch pattern\n", dd.astype(int))
print("search from gpu H (f64 solve)", -np.linalg.solve(Hg.astype(np.float64), od[18:36]))

print("activeD gpu", gd[400:408], "\n        orc", od[400:408])
print("jar gpu", gd[430:438], "\n    orc", od[430:438])
print("force gpu", gd[440:448], "\n      orc", od[440:448])
print("conG gpu", gd[410:420])
