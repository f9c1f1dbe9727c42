"""SampledUncertainVelocityActuator (UNC:123-281).

CPU: LoadModel's binning (UNC:156-221: equal steps over [-limit, limit], outer bins
open, first matching closed interval wins, UNC:140-154) in
make_sampled_actuator_model; the oracle's sampled actuator against the
truncated-normal one where both must add exactly zero noise (all samples 0 vs noise
bounds 0); commands outside every bin flag FKS_PARTICLE_ERR_NO_NOISE_BIN (the
reference asserts, UNC:152-153).
GPU: the HIP kernels with sampled actuators against the oracle, bit-exact, for the
linked, SE(2) and SE(3) robot families."""
import dataclasses

import numpy as np
import pytest

from fast_kinematic_simulator_amd import make_sampled_actuator_model
from fast_kinematic_simulator_amd import workloads as W
from fast_kinematic_simulator_amd.robots import SampledActuatorModel

ERR_NO_NOISE_BIN = 0x100


def _model(vmax, seed, scale=0.05, bins=8, elems=32):
    rng = np.random.default_rng(seed)
    cmd = rng.uniform(-vmax, vmax, size=4000)
    err = rng.normal(0.0, scale * vmax, size=4000)
    return make_sampled_actuator_model(np.stack([cmd, err], axis=1), vmax, bins, elems, seed=seed)


def _with_sampled(wl, zero=False, seed=7):
    models = []
    for k, c in enumerate(wl.robot.controllers):
        m = _model(abs(c.velocity_limit), seed + k)
        if zero:
            m = SampledActuatorModel(m.bounds, np.zeros_like(m.samples))
        models.append(m)
    return dataclasses.replace(wl.robot, sampled_actuators=models)


def test_model_binning_follows_load_model():
    data = np.array([[-2.0, 0.1], [-0.5, 0.2], [0.0, 0.3], [0.5, 0.4], [2.0, 0.5], [-1.0, 0.6]])
    m = make_sampled_actuator_model(data, 1.0, 4, 6, seed=1)
    assert m.bounds[0, 0] == -np.inf and m.bounds[-1, 1] == np.inf
    assert np.array_equal(m.bounds[1:, 0], m.bounds[:-1, 1])
    assert np.allclose(m.bounds[:-1, 1], [-0.5, 0.0, 0.5])
    # closed intervals, first match wins: -0.5 -> bin 0, 0.0 -> bin 1, 0.5 -> bin 2
    assert set(m.samples[0]) <= {0.1, 0.2, 0.6}
    assert set(m.samples[1]) <= {0.3} and set(m.samples[2]) <= {0.4} and set(m.samples[3]) <= {0.5}
    with pytest.raises(ValueError):
        make_sampled_actuator_model(np.array([[0.9, 0.0]]), 1.0, 4, 2)  # bins 0-2 empty


@pytest.mark.parametrize("name,scale", [("cfg1", 0.25), ("cfg2", 16 / 4096), ("cfg4", 8 / 1048576)])
def test_oracle_zero_samples_equal_zero_noise(name, scale):
    import oracle

    wl = W.WORKLOADS[name](scale)
    env = wl.environment()
    quiet = dataclasses.replace(wl.robot, controllers=[dataclasses.replace(c, max_actuator_proportional_noise=0.0,
                                                                           max_actuator_minimum_noise=0.0)
                                                       for c in wl.robot.controllers])
    a = oracle.forward_simulate(env, quiet, wl.solver, wl.controller_frequency, wl.seed, wl.starts, wl.targets, True)
    b = oracle.forward_simulate(env, _with_sampled(wl, zero=True), wl.solver, wl.controller_frequency, wl.seed, wl.starts,
                                wl.targets, True)
    for k in ("positions", "collided", "microsteps", "resolver_iterations", "error_flags"):
        assert np.array_equal(a[k], b[k]), k
    # with real samples the particles spread
    c = oracle.forward_simulate(env, _with_sampled(wl), wl.solver, wl.controller_frequency, wl.seed, wl.starts, wl.targets, True)
    assert not np.array_equal(a["positions"], c["positions"]) and not c["error_flags"].any()


def test_oracle_uncovered_command_flags_error():
    import oracle

    wl = W.cfg1(0.125)
    narrow = [SampledActuatorModel(np.array([[10.0, 20.0]]), np.zeros((1, 4))) for _ in wl.robot.controllers]
    robot = dataclasses.replace(wl.robot, sampled_actuators=narrow)
    r = oracle.forward_simulate(wl.environment(), robot, wl.solver, wl.controller_frequency, wl.seed, wl.starts, wl.targets, True)
    assert np.all(r["error_flags"] & ERR_NO_NOISE_BIN)


@pytest.mark.gpu
@pytest.mark.parametrize("segment_steps", [0, 4])
@pytest.mark.parametrize("name,scale,narrow", [("cfg1", 0.25, False), ("cfg2", 32 / 4096, False), ("cfg3", 16 / 65536, False),
                                               ("cfg4", 16 / 1048576, False), ("cfg1", 0.125, True)])
def test_gpu_sampled_actuator_matches_oracle(fks_lib, name, scale, narrow, segment_steps):
    import oracle
    from fast_kinematic_simulator_amd import make_linked_simulator

    wl = W.WORKLOADS[name](scale)
    if narrow:
        robot = dataclasses.replace(wl.robot, sampled_actuators=[SampledActuatorModel(np.array([[10.0, 20.0]]), np.zeros((1, 4)))
                                                                 for _ in wl.robot.controllers])
    else:
        robot = _with_sampled(wl)
    env = wl.environment()
    sim = make_linked_simulator(env, wl.solver, wl.controller_frequency, wl.seed)
    try:
        sim.set_segment_steps(segment_steps)  # 4: particles handed between waves every 4 steps
        sim.set_call_index(0)
        g = sim.forward_simulate_arrays(robot, wl.starts, wl.targets, True)
    finally:
        sim.close()
    o = oracle.forward_simulate(env, robot, wl.solver, wl.controller_frequency, wl.seed, wl.starts, wl.targets, True)
    for k in ("positions", "collided", "microsteps", "resolver_iterations", "error_flags"):
        assert np.array_equal(g[k], o[k]), k
    if narrow:
        assert np.all(g["error_flags"] & ERR_NO_NOISE_BIN)
