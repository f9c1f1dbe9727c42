"""Cooperative point rounds (fks_set_cooperative): waves left without a particle evaluate a
share of the environment-check and correction rounds of the particles their workgroup's
other waves still run.  It is a scheduling choice only: every output and counter must be
bit-identical with it on and off, and equal to the oracle (the parity suite runs with it on,
the default).  Small batches are spread one particle per wave (helpers from the start);
segmented batches get helpers once the ticket queue drains (the contact-heavy tail)."""
import numpy as np
import pytest

from fast_kinematic_simulator_amd import workloads as W

from parity_util import COUNTER_KEYS, assert_counters_identical, assert_identical, run_both

SCENES = {
    "cfg1": lambda: W.cfg1(),
    "cfg2": lambda: W.cfg2(256 / 4096),
    "cfg3": lambda: W.cfg3(192 / 65536),
    "cfg4": lambda: W.cfg4(192 / 1048576),
    "cfg5": lambda: W.cfg5(48 / 1048576),
    "folding_arm": lambda: W.folding_arm(),
    "crowded_cell": lambda: W.crowded_cell(),
}
# scenes with enough 64-point rounds in contact that helpers must have been used
ENGAGED = {"cfg3", "cfg4", "cfg5", "folding_arm", "crowded_cell"}


def _run(wl, cooperative, segment_steps):
    from fast_kinematic_simulator_amd import make_linked_simulator

    sim = make_linked_simulator(wl.environment(), wl.solver, wl.controller_frequency, wl.seed)
    try:
        sim.set_cooperative(cooperative)
        if segment_steps is not None:
            sim.set_segment_steps(segment_steps)
        sim.set_call_index(0)
        r = sim.forward_simulate_arrays(wl.robot, wl.starts, wl.targets, wl.allow_contacts)
        r["statistics"] = sim.get_statistics()
        r["counters"] = sim.last_call_counters()
        return r
    finally:
        sim.close()


@pytest.mark.gpu
@pytest.mark.parametrize("segment_steps", [None, 7])
@pytest.mark.parametrize("name", sorted(SCENES))
def test_cooperative_on_off_identical(fks_lib, name, segment_steps):
    wl = SCENES[name]()
    on = _run(wl, True, segment_steps)
    off = _run(wl, False, segment_steps)
    for k in ("positions", "collided", "microsteps", "resolver_iterations", "error_flags"):
        assert np.array_equal(np.asarray(on[k]), np.asarray(off[k])), (name, k)
    assert on["statistics"] == off["statistics"]
    for k in COUNTER_KEYS:
        assert on["counters"][k] == off["counters"][k], (name, k, on["counters"][k], off["counters"][k])
    assert off["counters"]["cooperative_tasks"] == 0
    if name in ENGAGED and segment_steps is None:
        assert on["counters"]["cooperative_tasks"] > 0, name


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["cfg3", "folding_arm"])
def test_cooperative_matches_oracle(fks_lib, oracle_lib, name):
    """helpers on (spread batch): the GPU equals the oracle bit for bit"""
    wl = SCENES[name]()
    g, o = run_both(wl)
    assert g["counters"]["cooperative_tasks"] > 0
    assert_identical(g, o)
    assert_counters_identical(g, o)
