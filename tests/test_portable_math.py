"""include/fks_portable_math.h (the libm both the HIP kernel and the oracle use)
against glibc: <= 1 ulp on the ranges the path uses."""
import math

import numpy as np
import pytest


def ulps(a, b):
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    spacing = np.abs(np.spacing(b))
    spacing[spacing == 0] = np.finfo(float).tiny
    return np.abs(a - b) / spacing


@pytest.fixture(scope="module")
def inputs():
    rng = np.random.default_rng(0)
    x = rng.uniform(-60, 60, 200000)
    x[::7] *= 1e-4
    x[::11] *= 1e-9
    return x


@pytest.mark.parametrize("fn,ref", [(0, np.sin), (1, np.cos), (3, np.arctan)])
def test_trig_within_one_ulp(oracle_lib, inputs, fn, ref):
    import oracle

    got = oracle.portable_math(fn, inputs)
    assert np.max(ulps(got, ref(inputs))) <= 1.0


def test_log_within_one_ulp(oracle_lib):
    import oracle

    rng = np.random.default_rng(1)
    x = rng.uniform(0, 1, 200000) * 10.0 ** rng.integers(-300, 300, 200000)
    x = x[x > 0]
    got = oracle.portable_math(2, x)
    assert np.max(ulps(got, np.log(x))) <= 1.0
    assert oracle.portable_math(2, np.array([1.0]))[0] == 0.0
    assert np.isneginf(oracle.portable_math(2, np.array([0.0]))[0])


def test_atan2_within_one_ulp(oracle_lib):
    import oracle

    rng = np.random.default_rng(2)
    y = rng.uniform(-5, 5, 100000)
    x = rng.uniform(-5, 5, 100000)
    got = oracle.portable_math(4, y, x)
    assert np.max(ulps(got, np.arctan2(y, x))) <= 1.0
    assert oracle.portable_math(4, np.array([0.0]), np.array([-1.0]))[0] == math.pi


def test_continuous_wrap(oracle_lib):
    """EigenHelpers::EnforceContinuousRevoluteBounds: result in (-pi, pi]."""
    import oracle

    x = np.array([0.0, math.pi, -math.pi, 3 * math.pi, -3.5, 7.0, 100.0])
    w = oracle.portable_math(5, x)
    assert np.all(w <= math.pi) and np.all(w > -math.pi)
    assert w[1] == math.pi and w[2] == math.pi
    assert np.allclose(np.cos(w), np.cos(x)) and np.allclose(np.sin(w), np.sin(x))


def test_fmod_two_pi_matches_glibc_bit_for_bit(oracle_lib):
    """fks_math::fmod_two_pi (the kernel's continuous-joint wrap, no libm call) returns glibc's
    fmod(x, 2*pi) bit for bit, over every binade and at the multiples of 2*pi; wrap_revolute
    equals enforce_continuous_revolute_bounds."""
    import oracle

    rng = np.random.default_rng(6)
    two_pi = 2.0 * math.pi
    x = rng.uniform(-1, 1, 400000) * 10.0 ** rng.uniform(-3, 20, 400000)
    k = rng.integers(-10**6, 10**6, 20000).astype(np.float64)
    near = np.concatenate([k * two_pi, np.nextafter(k * two_pi, np.inf), np.nextafter(k * two_pi, -np.inf)])
    edge = np.array([0.0, -0.0, two_pi, -two_pi, math.pi, -math.pi, 1e308, -1e308, 5e-324,
                     np.finfo(float).max, -np.finfo(float).max, 2.0**53, 3 * two_pi])
    x = np.concatenate([x, near, edge, rng.uniform(-1e300, 1e300, 2000)])
    got = oracle.portable_math(6, x)
    want = np.fmod(x, two_pi)
    assert np.array_equal(got.view(np.uint64), want.view(np.uint64))
    assert np.array_equal(oracle.portable_math(7, x).view(np.uint64), oracle.portable_math(5, x).view(np.uint64))
    assert np.isnan(oracle.portable_math(6, np.array([np.inf, -np.inf, np.nan]))).all()
