"""Known-answer tests of test_utils.py:54-105 re-expressed on the host restatement."""
import numpy as np
import pytest

from pupperv3_mjx import rng
from pupperv3_mjx.utils import (activation_fn_map, circular_buffer_push_back, circular_buffer_push_front,
                                sample_lagged_value)


def test_circular_buffer_push_back():
    out = circular_buffer_push_back(np.array([[1, 2, 3], [4, 5, 6]]), np.array([7, 8]))
    np.testing.assert_array_equal(out, [[2, 3, 7], [5, 6, 8]])


def test_circular_buffer_push_front():
    out = circular_buffer_push_front(np.array([[1, 2, 3], [4, 5, 6]]), np.array([7, 8]))
    np.testing.assert_array_equal(out, [[7, 1, 2], [8, 4, 5]])


def test_sample_lagged_value():
    buf = np.zeros((12, 4))
    expected = np.arange(12)
    buf[:, -2] = expected
    val, buf2 = sample_lagged_value(rng.PRNGKey(1), buf, np.zeros(12), np.array([0, 0, 0, 1]))
    np.testing.assert_allclose(val, expected, atol=1e-5)
    exp_buf = np.zeros((12, 4))
    exp_buf[:, -1] = expected
    np.testing.assert_allclose(buf2, exp_buf, atol=1e-5)


def test_sample_lagged_value_buffer_size_one():
    val, _ = sample_lagged_value(rng.PRNGKey(1), np.zeros((12, 1)), np.ones(12), np.array([0]))
    np.testing.assert_allclose(val, np.ones(12), atol=1e-5)


def test_activations():
    x = np.array([-1.0, 0.0, 1.0])
    np.testing.assert_array_equal(activation_fn_map("relu")(x), [0, 0, 1])
    np.testing.assert_allclose(activation_fn_map("sigmoid")(x), 1 / (1 + np.exp(-x)))
    np.testing.assert_allclose(activation_fn_map("tanh")(x), np.tanh(x))
    np.testing.assert_allclose(activation_fn_map("elu")(x), [np.expm1(-1), 0, 1])
    s = activation_fn_map("softmax")(np.array([1.0, 2.0, 3.0]))
    np.testing.assert_allclose(s, np.exp([1, 2, 3]) / np.exp([1, 2, 3]).sum())
    with pytest.raises(KeyError):
        activation_fn_map("invalid")
