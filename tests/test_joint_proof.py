"""The joint-space proof of free microsteps (fks_set_joint_proof) changes
the work, never the results: the same batch with the proof on and off returns the same
reached configurations, collided flags, microstep / resolver counts, error bits,
statistics and call counters, bit for bit, while the proof settles a share of the
microsteps (proven_free_microsteps > 0).  A batch checked this way with the proof on is
also checked against the CPU oracle, which knows nothing of the proof."""
import numpy as np
import pytest

from fast_kinematic_simulator_amd import make_linked_simulator
from fast_kinematic_simulator_amd import workloads as W

from parity_util import COUNTER_KEYS, assert_identical, mismatch_report, run_both

CASES = [("cfg2", 1024 / 4096, True), ("cfg3", 2048 / 65536, True), ("cfg5", 256 / 1048576, False)]


def _run(wl, env, proof, segment_steps=None):
    sim = make_linked_simulator(env, wl.solver, wl.controller_frequency, wl.seed)
    try:
        sim.set_joint_proof(proof)
        if segment_steps is not None:
            sim.set_segment_steps(segment_steps)
        out = sim.forward_simulate_arrays(wl.robot, wl.starts, wl.targets, wl.allow_contacts)
        out["statistics"] = sim.get_statistics()
        out["counters"] = sim.last_call_counters()
    finally:
        sim.close()
    return out


def _assert_same(a, b):
    for k in ("positions", "collided", "microsteps", "resolver_iterations", "error_flags"):
        assert np.array_equal(np.asarray(a[k]), np.asarray(b[k])), k
    assert a["statistics"] == b["statistics"]
    for k in COUNTER_KEYS:
        assert a["counters"][k] == b["counters"][k], (k, a["counters"][k], b["counters"][k])


@pytest.mark.gpu
@pytest.mark.parametrize("name,scale,expect_proven", CASES)
def test_joint_proof_bit_identical(fks_lib, name, scale, expect_proven):
    wl = W.WORKLOADS[name](scale)
    env = wl.environment()
    off = _run(wl, env, False)
    on = _run(wl, env, True)
    _assert_same(off, on)
    assert off["counters"]["proven_free_microsteps"] == 0
    proven = on["counters"]["proven_free_microsteps"]
    print(name, "proven", proven, "of", on["counters"]["microsteps"])
    if expect_proven:
        assert proven > 0
    assert proven <= on["counters"]["microsteps"]


@pytest.mark.gpu
def test_joint_proof_segmented_bit_identical(fks_lib):
    """Segments rest between waves: the anchor does not travel, the results still agree."""
    wl = W.cfg3(512 / 65536)
    env = wl.environment()
    _assert_same(_run(wl, env, False, segment_steps=3), _run(wl, env, True, segment_steps=3))


@pytest.mark.gpu
def test_joint_proof_matches_oracle(fks_lib, oracle_lib):
    wl = W.cfg3(96 / 65536)
    sim = make_linked_simulator(wl.environment(), wl.solver, wl.controller_frequency, wl.seed)
    try:
        sim.set_joint_proof(True)
        g, o = run_both(wl, sim=sim)
    finally:
        sim.close()
    print(mismatch_report(g, o))
    assert_identical(g, o)
    assert g["counters"]["proven_free_microsteps"] > 0


@pytest.mark.gpu
def test_joint_proof_self_collision_branch(fks_lib):
    """The folding arm self-collides: the pair slack must never hide a self contact."""
    wl = W.folding_arm()
    env = wl.environment()
    off = _run(wl, env, False)
    on = _run(wl, env, True)
    _assert_same(off, on)
    assert on["counters"]["self_collision_checks"] > 0


@pytest.mark.gpu
def test_joint_proof_full_cfg3_bit_identical(fks_lib):
    """The whole cfg3 headline batch (65,536 particles x 200 steps, segmented): an unsound
    proof would skip a contact and change that particle's trajectory."""
    wl = W.cfg3()
    env = wl.environment()
    off = _run(wl, env, False)
    on = _run(wl, env, True)
    _assert_same(off, on)
    print("cfg3 full: proven", on["counters"]["proven_free_microsteps"], "of", on["counters"]["microsteps"])
    assert on["counters"]["proven_free_microsteps"] > on["counters"]["microsteps"] // 10


@pytest.mark.gpu
@pytest.mark.parametrize("name,scale", [("cfg2", 1.0), ("cfg3", 4096 / 65536)])
def test_exact_edt_skip_route_bit_identical(fks_lib, name, scale):
    """A simulator made from the GPU-built, device-resident environment also skips rounds by
    the exact-EDT (Euclidean) proof (SimArgs.skip_euclid); the host copy of the same bytes
    does not.  Results and counters must agree, with the joint-space proof off and on."""
    wl = W.WORKLOADS[name](scale)
    host_env = W.SCENES[name](device=0)
    dev_env = W.SCENES[name](device=0, resident=True)
    for proof in (False, True):
        outs = []
        for env in (host_env, dev_env):
            sim = make_linked_simulator(env, wl.solver, wl.controller_frequency, wl.seed)
            try:
                sim.set_joint_proof(proof)
                out = sim.forward_simulate_arrays(wl.robot, wl.starts, wl.targets, wl.allow_contacts)
                out["statistics"] = sim.get_statistics()
                out["counters"] = sim.last_call_counters()
            finally:
                sim.close()
            outs.append(out)
        _assert_same(outs[0], outs[1])
        print(name, "proof", proof, "proven host/device", outs[0]["counters"]["proven_free_microsteps"],
              outs[1]["counters"]["proven_free_microsteps"])
        if proof:
            assert outs[1]["counters"]["proven_free_microsteps"] >= outs[0]["counters"]["proven_free_microsteps"]
