"""Every branch of the resolver reaches parity, each asserted to have run.

SURVEY.md §8(a) rows a5, a10, a14-a16, a18 and the VERDICT r01 gaps: the self-collision
impulse solve (ExtractSelfCollidingPoints SPCS:983-1171) applied as corrections
(SPCS:1846-1853, 1909-1916), `failed_resolves_end_motion = false` with recovered resolves
(SPCS:884-896), the shortcut distance (SPCS:897-902, ComputeConfigurationDistanceTo),
non-default decay / initial-step / min-scaling / iteration limits (SPCS:1624, 1705-1761),
continuous joints (angle wrap), the individual-Jacobian solve (SPCS:1966-1988, the
simulate_with_individual_jacobians flag of SPCS:420, 1629), a self-collision cell shared by
ten links (no capacity limit, as the reference's maps), a 32-DOF chain, and the largest
robot the descriptor admits (64 links, 63 dofs, 4096 points; run with fewer waves per
workgroup since its LDS block does not fit four times in a CU).

The CPU tests show on the oracle that each scene reaches its branch (counter > 0); the
GPU tests compare the HIP path with the oracle on the same scenes, every output, statistic
and counter bit for bit, and assert the branch counter on the GPU side as well.

The PID tests pin the controller of a whole simulated trajectory to the reference itself:
tests/golden/pid_trace_golden.json holds the per-step errors of a free-space run and the
outputs of the reference's simple_pid_controller.hpp on them (make_pid_trace_golden.py);
the control inputs a traced run records must equal clamp(term, +-vmax) * dt."""
import dataclasses
import json
import os

import numpy as np
import pytest

from fast_kinematic_simulator_amd import workloads as W

from parity_util import assert_counters_identical, assert_identical, mismatch_report, run_both

HERE = os.path.dirname(os.path.abspath(__file__))


def _solver(wl, **kw):
    wl.solver = dataclasses.replace(wl.solver, **kw)
    return wl


def _scene(name):
    """(workload, run_both keyword arguments, check(counters, statistics, result)) per branch."""
    if name == "self_collision":
        return W.folding_arm(), {}, lambda c, s, r: c["self_collision_checks"] > 0 and c["self_corrected_points"] > 0 and \
            s["unsuccessful_self_collision_resolves"] > 0
    if name == "no_end_on_failure":
        return _solver(W.folding_arm(), failed_resolves_end_motion=False), {}, \
            lambda c, s, r: s["recovered_unsuccessful_resolves"] > 0 and s["unsuccessful_resolves"] > 0
    if name == "shortcut":
        wl = _solver(W.folding_arm(), simulation_shortcut_distance=0.6)
        return wl, {}, lambda c, s, r: c["controller_steps"] < wl.num_particles * wl.steps
    if name == "resolver_params":
        return _solver(W.folding_arm(), resolve_correction_step_scaling_decay_rate=0.7, resolve_correction_initial_step_size=0.8,
                       resolve_correction_min_step_scaling=0.1, resolve_correction_step_scaling_decay_iterations=3,
                       max_resolver_iterations=15), {}, lambda c, s, r: s["unsuccessful_resolves"] > 0 and c["resolver_iterations"] > 0
    if name == "continuous":
        return W.folding_arm(continuous=True), {}, lambda c, s, r: bool(np.any(r["positions"][:, 0] < 0.0))  # starts at +2.8: crossed +-pi
    if name == "individual_jacobians":
        return W.folding_arm(), {"individual_jacobians": True}, lambda c, s, r: c["resolver_iterations"] > 0
    if name == "individual_jacobians_cfg3":
        return W.cfg3(32 / 65536), {"individual_jacobians": True}, lambda c, s, r: c["resolver_iterations"] > 0
    if name == "crowded_cell":
        # more than 8 links corrected in one iteration: all 10 links x 8 points share one cell
        return W.crowded_cell(), {}, lambda c, s, r: c["self_corrected_points"] >= 80 * c["resolver_iterations"] > 0
    if name == "giant_chain":
        # 64 links / 63 dofs / 4096 points: fewer waves per workgroup (its LDS block does not fit four times)
        return W.giant_chain(), {}, lambda c, s, r: c["microsteps"] > 0 and r["positions"].shape[1] == 63
    if name == "chain_32dof":
        return W.long_chain(), {}, lambda c, s, r: c["resolver_iterations"] > 0 and c["self_collision_checks"] > 0
    raise KeyError(name)


SCENES = ["self_collision", "no_end_on_failure", "shortcut", "resolver_params", "continuous", "individual_jacobians",
          "individual_jacobians_cfg3", "crowded_cell", "chain_32dof", "giant_chain"]


@pytest.mark.parametrize("name", SCENES)
def test_oracle_scene_reaches_branch(oracle_lib, name):
    import oracle

    wl, kw, check = _scene(name)
    o = oracle.forward_simulate(wl.environment(), wl.robot, wl.solver, wl.controller_frequency, wl.seed, wl.starts, wl.targets,
                                True, **kw)
    assert not np.any(o["error_flags"]), np.unique(o["error_flags"])
    assert check(o["counters"], o["statistics"], o), (o["counters"], o["statistics"])


def test_individual_jacobians_change_the_step(oracle_lib):
    """The flag selects a different solver (SPCS:1629): results must differ from the stacked solve."""
    import oracle

    wl = W.folding_arm()
    a = oracle.forward_simulate(wl.environment(), wl.robot, wl.solver, wl.controller_frequency, wl.seed, wl.starts, wl.targets, True)
    b = oracle.forward_simulate(wl.environment(), wl.robot, wl.solver, wl.controller_frequency, wl.seed, wl.starts, wl.targets, True,
                                individual_jacobians=True)
    assert not np.array_equal(a["positions"], b["positions"])


@pytest.mark.gpu
@pytest.mark.parametrize("segment_steps", [None, 3])
@pytest.mark.parametrize("name", SCENES)
def test_gpu_scene_parity(fks_lib, oracle_lib, name, segment_steps):
    wl, kw, check = _scene(name)
    g, o = run_both(wl, segment_steps=segment_steps, call_index=4, **kw)
    print(name, segment_steps, mismatch_report(g, o), g["counters"])
    assert_identical(g, o)
    assert_counters_identical(g, o)
    assert check(g["counters"], g["statistics"], g), (g["counters"], g["statistics"])


# ---------------------------------------------------------------- PID pinned on a trajectory
def _pid_golden():
    with open(os.path.join(HERE, "golden", "pid_trace_golden.json")) as f:
        gold = json.load(f)
    hexa = np.vectorize(float.fromhex, otypes=[np.float64])
    return (float.fromhex(gold["dt"]), hexa(np.array(gold["velocity_limits"])), hexa(np.array(gold["errors"])),
            hexa(np.array(gold["pid_terms"])))


def _check_pid_trace(result, buf, wl):
    from golden.make_pid_trace_golden import step_errors

    dt, vmax, errors, terms = _pid_golden()
    assert dt == 1.0 / wl.controller_frequency
    err = step_errors(wl.starts, wl.targets, buf, wl.steps)
    assert np.array_equal(err, errors), "the trajectory's PID inputs differ from the fixture's"
    expected = np.clip(terms, -vmax, vmax) * dt  # GenerateControlAction: PID, actuator clamp (UNC:70-75); u * dt (SPCS:1549)
    got = buf.step_inputs[:, :wl.steps, 0, :]
    assert np.array_equal(got, expected), np.max(np.abs(got - expected))


def test_oracle_pid_trace_matches_reference(oracle_lib):
    import oracle

    wl = W.pid_free_space()
    r, buf = oracle.forward_simulate_traced(wl.environment(), wl.robot, wl.solver, wl.controller_frequency, wl.seed, wl.starts,
                                            wl.targets, True)
    _check_pid_trace(r, buf, wl)


@pytest.mark.gpu
def test_gpu_pid_trace_matches_reference(fks_lib):
    """The GPU's controller on a whole trajectory == the reference's PID header."""
    from fast_kinematic_simulator_amd import make_linked_simulator

    wl = W.pid_free_space()
    sim = make_linked_simulator(wl.environment(), wl.solver, wl.controller_frequency, wl.seed)
    try:
        sim.set_call_index(0)
        r, buf = sim.forward_simulate_traced(wl.robot, wl.starts, wl.targets, True)
    finally:
        sim.close()
    _check_pid_trace(r, buf, wl)
