"""bench.py's multi-GPU launch on CPU (no HIP call is made): `--gpus N` starts N rank processes by
itself (BASELINE configs[3]/[4]), so the driver's `python bench.py --gpus 8` is an
8-rank job even without torch.distributed.run; under a launcher --gpus must match WORLD_SIZE."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _clean_env(**extra):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT", "PP3_LAUNCH_ID")}
    env.update(extra)
    return env


@pytest.mark.parametrize("n", [2, 3, 8])  # 8: the driver's SCALE run on a full node
def test_gpus_n_starts_n_distinct_ranks(n):
    out = subprocess.run([sys.executable, BENCH, "--gpus", str(n), "--dry-launch"], env=_clean_env(),
                         capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr
    lines = [json.loads(x) for x in out.stdout.splitlines() if x.startswith("{")]
    assert sorted(r["rank"] for r in lines) == list(range(n))
    assert sorted(r["local_rank"] for r in lines) == list(range(n))
    assert {r["world"] for r in lines} == {n}
    assert len({r["pid"] for r in lines}) == n
    # one launch id shared by the ranks (the rendezvous key), new for every launch
    assert len({r["launch"] for r in lines}) == 1 and lines[0]["launch"]
    again = subprocess.run([sys.executable, BENCH, "--gpus", str(n), "--dry-launch"], env=_clean_env(),
                           capture_output=True, text=True, timeout=120)
    assert json.loads(again.stdout.splitlines()[0])["launch"] != lines[0]["launch"]


def test_single_gpu_default_is_one_rank_without_spawning():
    out = subprocess.run([sys.executable, BENCH, "--dry-launch"], env=_clean_env(), capture_output=True, text=True,
                         timeout=120)
    assert out.returncode == 0, out.stderr
    lines = [json.loads(x) for x in out.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1 and lines[0]["rank"] == 0 and lines[0]["world"] == 1
    assert lines[0]["pid"] == lines[0]["pid"] and lines[0]["launch"] is None  # no launcher nonce: no child


def test_launcher_world_size_must_match_gpus():
    env = _clean_env(WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    out = subprocess.run([sys.executable, BENCH, "--gpus", "3", "--dry-launch"], env=env, capture_output=True,
                         text=True, timeout=120)
    assert out.returncode != 0 and "WORLD_SIZE=2" in out.stderr
    ok = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--dry-launch"], env=env, capture_output=True,
                        text=True, timeout=120)
    assert ok.returncode == 0 and json.loads(ok.stdout)["world"] == 2


def test_failing_rank_fails_the_job():
    """Without a GPU every rank fails when it creates its env: the launcher must return non-zero
    (and not hang on a rank waiting in a barrier)."""
    out = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--steps", "1", "--warmup", "0"],
                         env=_clean_env(HIP_VISIBLE_DEVICES="", PP3_RDZV_DIR=os.environ.get("TMPDIR", "/tmp")),
                         capture_output=True, text=True, timeout=300)
    assert out.returncode != 0
    assert not [x for x in out.stdout.splitlines() if x.startswith('{"metric"')]
    assert "exited with" in out.stderr
