"""The TnuvaRobot control interface (TNUVA:15-23) through the host C-ABI
(fks_robot_control_action / fks_robot_apply_control_input) from Python, no GPU: a robot
stepped by hand with GenerateControlAction + clean ApplyControlInput equals the oracle's robot
stepped the same way, bit for bit, for SE(2), SE(3) and linked robots (incl. a continuous
joint); the noisy form adds the actuator's bounded noise; bad arguments are refused."""
import numpy as np
import pytest

from fast_kinematic_simulator_amd import workloads as W
from fast_kinematic_simulator_amd.robots import RobotController

CASES = {
    "se2": lambda: W.cfg1(1.0),
    "se3": lambda: W.cfg4(16 / 1048576),
    "linked_cfg3": lambda: W.cfg3(16 / 65536),
    "linked_continuous": lambda: W.folding_arm(0.5, continuous=True),
    "dual_arm": lambda: W.cfg5(16 / 1048576),
}


@pytest.mark.parametrize("name", sorted(CASES))
def test_clean_steps_match_oracle(oracle_lib, name):
    import oracle

    wl = CASES[name]()
    dt = 1.0 / wl.controller_frequency
    u_o, q_o, pid_o = oracle.robot_steps(wl.robot, wl.starts[0], wl.targets[0], dt, 40, 1)
    r = RobotController(wl.robot, wl.starts[0])
    r.reset_position(wl.starts[0])
    for k in range(40):
        u = r.generate_control_action(wl.targets[0], dt)
        assert np.array_equal(u, u_o[k]), k
        q = r.apply_control_input(u)
        assert np.array_equal(q, q_o[k]), k
    assert np.array_equal(r.controller_state, pid_o)
    assert np.any(q_o[-1] != wl.starts[0])


def test_noisy_step_stays_within_the_actuator_bound():
    wl = W.cfg3(16 / 65536)
    r = RobotController(wl.robot, wl.starts[0])
    u = r.generate_control_action(wl.targets[0], 1.0 / wl.controller_frequency)
    clean = RobotController(wl.robot, wl.starts[0]).apply_control_input(u)
    for noise in (np.ones(wl.robot.num_dofs), -np.ones(wl.robot.num_dofs)):
        q = RobotController(wl.robot, wl.starts[0]).apply_control_input(u, unit_noise=noise)
        for d, c in enumerate(wl.robot.controllers):
            vmax = abs(c.velocity_limit)
            bound = max(abs(c.max_actuator_proportional_noise) * min(abs(u[d]), vmax), abs(c.max_actuator_minimum_noise) * vmax)
            assert abs(q[d] - clean[d]) <= bound * (1 + 1e-12) + 1e-15
    assert not np.array_equal(RobotController(wl.robot, wl.starts[0]).apply_control_input(u, unit_noise=np.full(7, 0.5)), clean)


def test_bad_arguments_are_refused():
    from fast_kinematic_simulator_amd._capi import FksError

    wl = W.cfg3(16 / 65536)
    r = RobotController(wl.robot, wl.starts[0])
    with pytest.raises((FksError, ValueError)):
        r.apply_control_input(np.zeros(wl.robot.num_dofs + 1))


def test_simple_pid_controller_header_matches_reference_golden():
    """simple_pid_controller::SimplePIDController of the drop-in header
    (<fast_kinematic_simulator/simple_pid_controller.hpp>, PID:17-136, over fks_control.h's
    shared arithmetic) reproduces the reference header's own outputs bit for bit
    (tests/golden/pid_golden.json: the reference compiled by oracle/ref/pid_golden_driver.cpp),
    including Zero() mid-sequence and negative gains made positive by Initialize()."""
    import json
    import os
    import subprocess

    from fast_kinematic_simulator_amd.build import build_planner_test

    with open(os.path.join(os.path.dirname(__file__), "golden", "pid_golden.json")) as f:
        golden = json.load(f)
    lines, expected = [], []
    for case in golden["cases"]:
        steps = case["steps"]
        lines.append(" ".join(float(case[k]).hex() for k in ("kp", "ki", "kd", "iclamp")) + f" {len(steps)}")
        for e, dt, out, zero in steps:
            lines.append(f"{float(e).hex()} {float(dt).hex()} {int(zero)}")
            expected.append(float(out))
    exe = build_planner_test()
    p = subprocess.run([exe, "--pid-replay"], input="\n".join(lines) + "\n", stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True,
                       timeout=120)
    assert p.returncode == 0, p.stderr
    got = [float.fromhex(v) for v in p.stdout.split()]
    assert len(got) == len(expected) == 4 * 64
    assert got == expected


@pytest.mark.gpu
@pytest.mark.parametrize("name,scale", [("cfg1", 0.25), ("cfg3", 8 / 65536), ("cfg4", 8 / 1048576)])
def test_host_control_twin_equals_the_gpu(fks_lib, name, scale):
    """The host robot-control entry points (fks_robot_control.cpp) against the GPU's own
    arithmetic, bit for bit (TNUVA:538-614):
      - ApplyControlInput(u): fks_robot_apply_control_input vs the kernels' apply_input through
        fks_kinematics(FKS_KIN_APPLY_CONTROL_INPUT), on configurations and inputs spread over
        (and past) the joint and velocity limits;
      - GenerateControlAction: a robot stepped by hand from each particle's traced step-start
        configurations vs the traced kernel's real_control_input (u * dt, SPCS:1549) of every
        controller step, the PID state carried across steps on both sides."""
    from fast_kinematic_simulator_amd import make_linked_simulator

    wl = W.WORKLOADS[name](scale)
    r = wl.robot
    rng = np.random.default_rng(17)
    sim = make_linked_simulator(wl.environment(), wl.solver, wl.controller_frequency, wl.seed)
    try:
        n, D, Wd = 48, r.num_dofs, r.config_width
        configs = np.repeat(wl.starts[:1], n, axis=0) if len(wl.starts) == 1 else wl.starts[rng.integers(0, len(wl.starts), n)]
        if r.robot_type != 2:  # SE(3) configurations are poses; linked / SE(2): perturb the values
            configs = configs + rng.normal(0.0, 2.0, size=configs.shape)
        # a robot's position is a SetPosition result (joint limits, angle wrap): the kernels apply
        # SetPosition to the configurations they are given, so start both sides from such ones
        configs = sim.apply_control_input(r, configs, np.zeros((n, D)))
        vmax = np.array([abs(c.velocity_limit) for c in r.controllers])
        inputs = rng.uniform(-2.0, 2.0, size=(n, D)) * vmax
        gpu = sim.apply_control_input(r, configs, inputs)
        for i in range(n):
            rc = RobotController(r, configs[i])
            host = rc.apply_control_input(inputs[i])
            assert np.array_equal(host, gpu[i]), (i, host, gpu[i])
        # GenerateControlAction along traced trajectories
        sim.set_call_index(0)
        res, buf = sim.forward_simulate_traced(r, wl.starts, wl.targets, wl.allow_contacts, config_capacity=1 << 15)
        dt = 1.0 / wl.controller_frequency
        checked = 0
        for p in range(len(wl.starts)):
            steps, ncfg = int(buf.num_steps[p]), int(buf.num_configs[p])
            assert ncfg <= buf.config_capacity
            tags = buf.config_tags[p, :ncfg]
            rc = RobotController(r, wl.starts[p])
            rc.position = np.array(wl.starts[p], dtype=np.float64)
            # ResetPosition's SetPosition (joint limits / angle wrap) is the kernel's first step start
            rc.position = sim.apply_control_input(r, wl.starts[p:p + 1], np.zeros((1, D)))[0] if r.robot_type != 2 else rc.position
            for k in range(steps):
                target = wl.targets[p] if len(wl.targets) == len(wl.starts) else wl.targets[0]
                u = rc.generate_control_action(target, dt)
                assert np.array_equal(u * dt, buf.step_inputs[p, k, 0]), (p, k)
                checked += 1
                last = np.nonzero(tags[:, 0] == k)[0]
                assert len(last) > 0
                rc.position = buf.configs[p, last[-1]].copy()  # the configuration the step ended at
        assert checked > len(wl.starts)
    finally:
        sim.close()
