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
