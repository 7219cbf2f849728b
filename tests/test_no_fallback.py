"""The product path has no CPU fallback: without the HIP library, or without a visible GPU, creating
an env raises (CPU tests, fresh interpreters so the library path is read at import)."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

_SNIPPET = """
import sys
sys.path[:0] = [{root!r}, {pkg!r}]
from bench import bench_kwargs
from pupperv3_mjx import MODEL_XML
from pupperv3_mjx.environment import PupperV3Env
try:
    PupperV3Env(**bench_kwargs(MODEL_XML), num_envs=4)
except Exception as exc:
    print(type(exc).__name__ + ": " + str(exc))
    sys.exit(3)
print("created")
"""


def _run(env_extra):
    env = dict(os.environ, **env_extra)
    code = _SNIPPET.format(root=ROOT, pkg=os.path.join(ROOT, "pupperv3-mjx_amd"))
    return subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=300)


def test_missing_library_raises():
    r = _run({"PP3_LIB_PATH": "/nonexistent/libpupper_hip.so"})
    assert r.returncode == 3, (r.stdout, r.stderr)
    assert "PupperHipError" in r.stdout and "no CPU fallback" in r.stdout, r.stdout


def test_no_gpu_raises_instead_of_falling_back():
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is visible here")
    lib = os.path.join(ROOT, "pupperv3-mjx_amd", "pupperv3_mjx", "libpupper_hip.so")
    if not os.path.exists(lib):
        pytest.skip("library not built")
    r = _run({})
    assert r.returncode == 3, (r.stdout, r.stderr)
    assert r.stdout.startswith("PupperHipError"), r.stdout  # the library's own error, not a CPU path
