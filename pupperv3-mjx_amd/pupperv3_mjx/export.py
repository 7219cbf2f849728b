"""Policy export in the reference's deployment format (export.py:7-81) and its device runner.

`convert_params` restates export.py:13-81 in numpy (the reference imports jax only for
`jp.split`): observation normalisation folded into the first dense layer
(`fold_in_normalization`, export.py:7-10), the final layer cut to its first half (the mean of
Brax PPO's tanh-Gaussian head), per-layer activation names from utils.activation_fn_map
(relu, sigmoid, elu, tanh), metadata keys as in export.py:63-79.  `policy_forward` is the numpy
meaning of that JSON (what the robot runs); `DevicePolicy` runs it batched on the GPU
(csrc/pp3_policy.hip, f32 matrix cores) straight from the env's observation buffer, so a
policy + env rollout never leaves the device.
"""
from __future__ import annotations

import ctypes as C
from typing import Any, Dict, Mapping

import numpy as np

ACTIVATIONS = {"linear": 0, "relu": 1, "elu": 2, "tanh": 3, "sigmoid": 4}


def fold_in_normalization(A, b, mean, std):
    """export.py:7-10: dense(x_norm) with x_norm = (x - mean) / std  ==  dense'(x)."""
    A = np.asarray(A)
    b = np.asarray(b)
    mean = np.asarray(mean)
    std = np.asarray(std)
    A_prime = A / std[:, np.newaxis]
    b_prime = (b - (A.T @ (mean / std)[:, np.newaxis]).T)[0]
    return A_prime, b_prime


def _field(obj, name):
    return obj[name] if isinstance(obj, Mapping) else getattr(obj, name)


def convert_params(params, activation: str, action_scale: float, kp: float, kd: float, default_pose,
                   joint_upper_limits, joint_lower_limits, use_imu: bool, observation_history: int,
                   maximum_pitch_command: float, maximum_roll_command: float,
                   final_activation: str = "tanh") -> Dict[str, Any]:
    """export.py:13-81.  params = (normalizer with .mean/.std, {"params": {layer: {"kernel", "bias"}}})."""
    mean, std = _field(params[0], "mean"), _field(params[0], "std")
    params_dict = params[1]["params"]
    layers = []
    input_size = None
    for i, (layer_name, layer_params) in enumerate(params_dict.items()):
        is_first_layer = i == 0
        is_final_layer = i == len(params_dict) - 1
        bias = np.asarray(layer_params["bias"])
        kernel = np.asarray(layer_params["kernel"])
        if is_first_layer:
            kernel, bias = fold_in_normalization(A=kernel, b=bias, mean=mean, std=std)
            input_size = kernel.shape[0]
        if is_final_layer:
            bias, _ = np.split(bias, 2, axis=-1)
            kernel, _ = np.split(kernel, 2, axis=-1)
        layers.append({
            "type": "dense",
            "activation": activation if not is_final_layer else final_activation,
            "shape": [None, len(bias)],
            "weights": [kernel.tolist(), bias.tolist()],
        })
    return {
        "use_imu": use_imu,
        "control_orientation": True,
        "observation_history": observation_history,
        "action_scale": action_scale,
        "kp": kp,
        "kd": kd,
        "default_joint_pos": np.array(default_pose).tolist(),
        "joint_upper_limits": np.array(joint_upper_limits).tolist(),
        "joint_lower_limits": np.array(joint_lower_limits).tolist(),
        "maximum_pitch_command": maximum_pitch_command,
        "maximum_roll_command": maximum_roll_command,
        "in_shape": [None, input_size],
        "layers": layers,
    }


def _act_np(x, name):
    name = name.lower()
    if name == "relu":
        return np.maximum(x, 0)
    if name == "elu":
        return np.where(x > 0, x, np.expm1(np.minimum(x, 0)))
    if name == "tanh":
        return np.tanh(x)
    if name == "sigmoid":
        return 1 / (1 + np.exp(-x))
    if name == "linear":
        return x
    raise ValueError(f"unsupported activation {name!r}")


def policy_forward(policy: Dict[str, Any], obs) -> np.ndarray:
    """Reference meaning of a converted policy: h = act(h @ kernel + bias) per layer."""
    h = np.asarray(obs, dtype=np.float64)
    for layer in policy["layers"]:
        k, b = layer["weights"]
        h = _act_np(h @ np.asarray(k, dtype=np.float64) + np.asarray(b, dtype=np.float64), layer["activation"])
    return h


class DevicePolicy:
    """Batched on-device forward of a converted policy dict (pp3_policy_* C ABI)."""

    def __init__(self, policy: Dict[str, Any], device: int = 0):
        from . import _lib
        self._lib = _lib
        L = _lib.load()
        self._L = L
        layers = policy["layers"]
        in_dim = int(policy["in_shape"][1])
        outs, acts, blob = [], [], []
        k_in = in_dim
        for layer in layers:
            k, b = np.asarray(layer["weights"][0], dtype=np.float32), np.asarray(layer["weights"][1], dtype=np.float32)
            if k.shape != (k_in, b.shape[0]):
                raise ValueError(f"layer kernel {k.shape} does not follow input width {k_in}")
            name = layer["activation"].lower()
            if name not in ACTIVATIONS:
                raise ValueError(f"unsupported activation {name!r} (device: {sorted(ACTIVATIONS)})")
            outs.append(b.shape[0])
            acts.append(ACTIVATIONS[name])
            blob += [k.ravel(), b]
            k_in = b.shape[0]
        w = np.ascontiguousarray(np.concatenate(blob), dtype=np.float32)
        o = np.array(outs, dtype=np.int32)
        a = np.array(acts, dtype=np.int32)
        h = C.c_void_p()
        rc = L.pp3_policy_create(int(device), in_dim, len(layers), o.ctypes.data_as(C.c_void_p),
                                 a.ctypes.data_as(C.c_void_p), w.ctypes.data_as(C.c_void_p), C.byref(h))
        if rc != 0:
            raise _lib.PupperHipError(L.pp3_policy_last_error().decode())
        self._h = h
        self.in_dim = in_dim
        self.out_dim = int(outs[-1])
        self.device = int(device)

    def act(self, obs_dev: int, obs_stride: int, n: int, actions_dev: int, action_stride: int, stream=None) -> None:
        rc = self._L.pp3_policy_act(self._h, C.c_void_p(obs_dev), int(obs_stride), int(n), C.c_void_p(actions_dev),
                                    int(action_stride), C.c_void_p(stream) if stream else None)
        if rc != 0:
            raise self._lib.PupperHipError(self._L.pp3_policy_last_error().decode())

    def act_env(self, env, actions_dev: int, stream=None) -> None:
        """actions[N][12] = policy(env's current observation buffer)."""
        from . import _abi
        if self.out_dim != _abi.NU:
            raise ValueError(f"act_env needs a policy with {_abi.NU} outputs (the action), this one has {self.out_dim}")
        obs_ptr, obs_n = env.device_field(_abi.F_OBS)
        if stream is None:  # order with the env's kernels
            stream = env._L.pp3_stream(env._h)
        self.act(obs_ptr, obs_n, env.num_envs, actions_dev, _abi.NU, stream)

    def close(self) -> None:
        if getattr(self, "_h", None):
            self._L.pp3_policy_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
