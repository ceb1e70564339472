"""Accuracy of the kernel's float32 math sequences (csrc/quad_physics.h), host-instantiated."""
import numpy as np

import native_host as NH


def test_sincos_accuracy_over_hinge_range():
    rng = np.random.default_rng(0)
    x = np.concatenate([rng.uniform(-1e3, 1e3, 200000), rng.uniform(-4, 4, 100000),
                        np.array([0.0, -0.0, np.pi / 4, np.pi / 2, np.pi, -np.pi, 1e4, -3e4])]).astype(np.float32)
    s, c = NH.fsincos(x)
    xd = x.astype(np.float64)
    assert np.abs(s - np.sin(xd)).max() < 3e-7
    assert np.abs(c - np.cos(xd)).max() < 3e-7


def test_atan2_accuracy_and_conventions():
    rng = np.random.default_rng(1)
    y = rng.normal(size=300000).astype(np.float32)
    x = rng.normal(size=300000).astype(np.float32)
    r = NH.fatan2(y, x)
    assert np.abs(r - np.arctan2(y.astype(np.float64), x.astype(np.float64))).max() < 4e-7  # ~1.3 ulp near pi
    ys = np.array([0.0, -0.0, 0.0, -0.0, 1.0, -1.0, 0.0, 0.0, 2.0, 1e-30], np.float32)
    xs = np.array([0.0, 0.0, -0.0, -0.0, 0.0, -0.0, 1.0, -1.0, 2.0, 1.0], np.float32)
    got = NH.fatan2(ys, xs)
    ref = np.arctan2(ys, xs).astype(np.float32)
    assert np.all(np.abs(got - ref) < 3e-7) and np.array_equal(np.signbit(got), np.signbit(ref))


def test_div_const_is_correctly_rounded_for_obs_spans():
    pi = np.float32(np.pi)
    spans = [np.float32(8), np.float32(4), np.float32(pi - (-pi)), np.float32(20),
             np.float32(np.float32(6 * np.pi) - np.float32(-6 * np.pi))]
    rng = np.random.default_rng(2)
    # the normalize numerators 2 (x - lo): zero or normal floats; sample every binade
    a = (rng.uniform(1, 2, 400000) * 2.0 ** rng.integers(-40, 40, 400000)).astype(np.float32)
    a = np.concatenate([a, -a, np.float32([0.0, 1.0, 2.0, 3.0, 40.0])])
    for b in spans:
        assert np.array_equal(NH.div_const(a, b), (a / b).astype(np.float32)), b
