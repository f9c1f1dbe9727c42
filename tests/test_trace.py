"""Traced forward simulation (ForwardSimulationStepTrace).

The reference records, when enable_tracing is set, one resolver step per
controller step (SPCS:1583-1588) holding real_control_input and
control_input_step, one contact-resolver step per microstep (SPCS:1593), and
pushes the post-action configuration (SPCS:1617), every resolver iterate
(SPCS:1703), the restored configuration of a failed resolve (SPCS:1714) and of a
contact with allow_contacts == false (SPCS:1778).

CPU: the oracle's trace against the structure those lines imply (record counts
equal the microstep / resolver counters, the last configuration of a microstep is
where the particle went on from, tracing does not change results).
GPU: the traced HIP kernels against the oracle's trace, bit-exact, and against
the untraced HIP kernels' results."""
import numpy as np
import pytest

from fast_kinematic_simulator_amd import workloads as W
from fast_kinematic_simulator_amd.trace import (TRACE_CONTACT_STOP, TRACE_POST_ACTION, TRACE_RESOLVE_FAILED,
                                                TRACE_RESOLVER_STEP)

CASES = [("cfg1", 0.25, True), ("cfg1", 0.25, False), ("cfg2", 24 / 4096, True), ("cfg3", 12 / 65536, True),
         ("cfg3", 12 / 65536, False), ("cfg4", 16 / 1048576, True), ("cfg5", 6 / 1048576, True)]


def _oracle_traced(wl, allow, call_index=0, config_capacity=4096):
    import oracle

    return oracle.forward_simulate_traced(wl.environment(), wl.robot, wl.solver, wl.controller_frequency, wl.seed, wl.starts,
                                          wl.targets, allow, call_index=call_index, config_capacity=config_capacity)


def _check_structure(wl, r, buf):
    """Invariants of SPCS:1583-1779 on every particle's trace."""
    n = len(wl.starts)
    for i in range(n):
        nc = int(buf.num_configs[i])
        assert nc <= buf.config_capacity
        tags = buf.config_tags[i, :nc]
        kinds = tags[:, 2]
        assert int(np.sum(kinds == TRACE_POST_ACTION)) == int(r["microsteps"][i])
        assert int(np.sum(kinds == TRACE_RESOLVER_STEP)) == int(r["resolver_iterations"][i])
        ns = int(buf.num_steps[i])
        assert ns >= 1 and int(np.max(tags[:, 0])) == ns - 1
        # control_input_step == real_control_input / M (SPCS:1568)
        u, ustep, m = buf.step_inputs[i, :ns, 0], buf.step_inputs[i, :ns, 1], buf.step_microsteps[i, :ns]
        assert np.array_equal(ustep, u / m[:, None].astype(np.float64))
        tr = buf.particle(i)
        assert not tr.truncated and len(tr.resolver_steps) == ns
        for s, rs in enumerate(tr.resolver_steps):
            assert 1 <= len(rs.contact_resolver_steps) <= rs.number_microsteps
            for c in rs.contact_resolver_steps:
                assert c.kinds[0] == TRACE_POST_ACTION and TRACE_POST_ACTION not in c.kinds[1:]
                assert all(k != TRACE_CONTACT_STOP for k in c.kinds[:-1])
                assert all(k != TRACE_RESOLVE_FAILED for k in c.kinds[:-1])
        # allow_contacts: every step runs to the end unless a resolve failed (failed_resolves_end_motion)
        last = tr.resolver_steps[-1].contact_resolver_steps[-1]
        if wl.allow_contacts and last.kinds[-1] not in (TRACE_RESOLVE_FAILED, TRACE_CONTACT_STOP) and not r["error_flags"][i]:
            # the particle ends where its last microstep ended (SPCS:875, 1815)
            assert np.array_equal(last.contact_resolution_steps[-1], r["positions"][i])


@pytest.mark.parametrize("name,scale,allow", [c for c in CASES if c[0] in ("cfg1", "cfg2", "cfg3")])
def test_oracle_trace_structure_and_results(name, scale, allow):
    import oracle

    wl = W.WORKLOADS[name](scale)
    wl.allow_contacts = allow
    r, buf = _oracle_traced(wl, allow)
    plain = oracle.forward_simulate(wl.environment(), wl.robot, wl.solver, wl.controller_frequency, wl.seed, wl.starts,
                                    wl.targets, allow)
    for k in ("positions", "collided", "microsteps", "resolver_iterations", "error_flags"):
        assert np.array_equal(r[k], plain[k]), k
    _check_structure(wl, r, buf)
    if name == "cfg1" and not allow:
        # SPCS:1776-1779 + 904-909: a contact ends the simulation without updating the
        # configuration or the collided flag, so the particle stays at the start of that step
        stopped = 0
        for i in range(len(wl.starts)):
            tr = buf.particle(i)
            if tr.resolver_steps[-1].contact_resolver_steps[-1].kinds[-1] != TRACE_CONTACT_STOP:
                continue
            stopped += 1
            assert not r["collided"][i]
            step_start = (tr.resolver_steps[-2].contact_resolver_steps[-1].contact_resolution_steps[-1]
                          if len(tr.resolver_steps) > 1 else wl.starts[i])
            assert np.array_equal(r["positions"][i], step_start)
        assert stopped > 0


def test_oracle_trace_capacity_truncates():
    wl = W.cfg1(0.125)
    full_r, full = _oracle_traced(wl, True)
    small_r, small = _oracle_traced(wl, True, config_capacity=8)
    assert np.array_equal(full.num_configs, small.num_configs)
    assert np.array_equal(full.configs[:, :8], small.configs)
    assert any(small.particle(i).truncated for i in range(len(wl.starts)))


@pytest.mark.gpu
@pytest.mark.parametrize("name,scale,allow", CASES)
def test_gpu_trace_matches_oracle(name, scale, allow):
    from fast_kinematic_simulator_amd import make_linked_simulator

    wl = W.WORKLOADS[name](scale)
    wl.allow_contacts = allow
    sim = make_linked_simulator(wl.environment(), wl.solver, wl.controller_frequency, wl.seed)
    try:
        sim.set_call_index(0)
        g, gb = sim.forward_simulate_traced(wl.robot, wl.starts, wl.targets, allow)
        sim.set_call_index(0)
        plain = sim.forward_simulate_arrays(wl.robot, wl.starts, wl.targets, allow)
    finally:
        sim.close()
    o, ob = _oracle_traced(wl, allow)
    for k in ("positions", "collided", "microsteps", "resolver_iterations", "error_flags"):
        assert np.array_equal(g[k], plain[k]), k
        assert np.array_equal(g[k], o[k]), k
    for k in ("num_steps", "num_configs", "step_microsteps", "step_inputs", "config_tags", "configs"):
        assert np.array_equal(getattr(gb, k), getattr(ob, k)), k
    _check_structure(wl, g, gb)
