"""export.py restatement (export.py:7-81): normalisation folding, final-layer split, JSON layout,
and the numpy meaning of the exported policy.  The reference module imports jax (absent), so
parity is pinned by the folding identity and a hand-built Brax-style forward, not by a
reference run."""
import json
from collections import OrderedDict
from types import SimpleNamespace

import numpy as np
import pytest

from pupperv3_mjx import export


def _brax_like_params(rs, sizes):
    params = OrderedDict()
    for i in range(len(sizes) - 1):
        params[f"hidden_{i}"] = {"kernel": rs.normal(scale=1.0 / np.sqrt(sizes[i]), size=(sizes[i], sizes[i + 1])),
                                 "bias": rs.normal(scale=0.1, size=sizes[i + 1])}
    norm = SimpleNamespace(mean=rs.normal(size=sizes[0]), std=rs.uniform(0.5, 2.0, size=sizes[0]))
    return (norm, {"params": params})


def test_fold_in_normalization_identity():
    rs = np.random.RandomState(0)
    A, b = rs.normal(size=(9, 5)), rs.normal(size=5)
    mean, std = rs.normal(size=9), rs.uniform(0.5, 2, size=9)
    x = rs.normal(size=(7, 9))
    A2, b2 = export.fold_in_normalization(A, b, mean, std)
    np.testing.assert_allclose(x @ A2 + b2, ((x - mean) / std) @ A + b, rtol=1e-12, atol=1e-12)


@pytest.mark.parametrize("act", ["elu", "relu", "tanh", "sigmoid"])
def test_convert_params_matches_brax_style_forward(act):
    rs = np.random.RandomState(1)
    sizes = [72, 32, 16, 24]  # final layer 2*12: loc | scale of the tanh-Gaussian head
    params = _brax_like_params(rs, sizes)
    pol = export.convert_params(params, act, 0.75, 5.0, 0.25, np.zeros(12), np.ones(12), -np.ones(12), True, 2,
                                30.0, 30.0)
    assert pol["in_shape"] == [None, 72]
    assert [l["shape"] for l in pol["layers"]] == [[None, 32], [None, 16], [None, 12]]
    assert [l["activation"] for l in pol["layers"]] == [act, act, "tanh"]
    assert set(pol) == {"use_imu", "control_orientation", "observation_history", "action_scale", "kp", "kd",
                        "default_joint_pos", "joint_upper_limits", "joint_lower_limits", "maximum_pitch_command",
                        "maximum_roll_command", "in_shape", "layers"}
    json.loads(json.dumps(pol))  # plain JSON types only
    x = rs.normal(size=(5, 72))
    h = (x - params[0].mean) / params[0].std
    layers = list(params[1]["params"].values())
    for i, lp in enumerate(layers):
        h = h @ lp["kernel"] + lp["bias"]
        if i < len(layers) - 1:
            h = export._act_np(h, act)
    want = np.tanh(h[:, :12])  # deterministic action = tanh(loc)
    np.testing.assert_allclose(export.policy_forward(pol, x), want, rtol=1e-10, atol=1e-10)


def test_unsupported_activation_rejected():
    with pytest.raises(ValueError):
        export._act_np(np.zeros(3), "softplus")
