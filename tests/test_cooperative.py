"""Cooperative small batches (fks_set_cooperative_waves, opt-in): one particle per workgroup,
its environment checks and correction passes shared out over the workgroup's waves (DESIGN.md
§4.11).  The cooperative kernel must give every output, every call counter (algorithmic SDF
bytes included) and every statistic of the one-wave kernels and of the oracle: the first
colliding point of an environment check and its byte count are resolved in round order, and
correction rows land in the sequential order."""
import numpy as np
import pytest

from fast_kinematic_simulator_amd import workloads as W

from parity_util import COUNTER_KEYS, assert_counters_identical, assert_identical, mismatch_report, run_both

KEYS = ("positions", "collided", "microsteps", "resolver_iterations", "error_flags")


def _run_device(sim, wl, starts, first_id, call_index=0):
    """one call through fks_forward_simulate_device with an explicit first particle id (the
    particles keep their noise streams when run apart from their batch)"""
    import torch

    dev = torch.device("cuda", 0)
    n = starts.shape[0]
    W_ = wl.robot.config_width
    d_starts = torch.from_numpy(np.ascontiguousarray(starts)).to(dev)
    d_targets = torch.from_numpy(np.ascontiguousarray(wl.targets)).to(dev)
    q = torch.empty((n, W_), dtype=torch.float64, device=dev)
    col = torch.empty(n, dtype=torch.uint8, device=dev)
    micro = torch.empty(n, dtype=torch.int32, device=dev)
    res = torch.empty(n, dtype=torch.int32, device=dev)
    err = torch.empty(n, dtype=torch.int32, device=dev)
    sim.set_call_index(call_index)
    sim.reset_statistics()
    sim.forward_simulate_device(wl.robot, d_starts.data_ptr(), n, d_targets.data_ptr(), wl.targets.shape[0], first_id,
                                wl.allow_contacts, q.data_ptr(), d_out_collided=col.data_ptr(), d_out_microsteps=micro.data_ptr(),
                                d_out_resolver_iterations=res.data_ptr(), d_out_error_flags=err.data_ptr(), synchronize=True)
    return {"positions": q.cpu().numpy(), "collided": col.cpu().numpy(), "microsteps": micro.cpu().numpy().astype(np.uint32),
            "resolver_iterations": res.cpu().numpy().astype(np.uint32), "error_flags": err.cpu().numpy().astype(np.uint32),
            "counters": sim.last_call_counters(), "statistics": sim.get_statistics(),
            "kernel": sim.launch_info()["last_kernel"]}


def _same(a, b, what):
    for k in KEYS:
        assert np.array_equal(a[k], b[k]), (what, k)
    for k in COUNTER_KEYS:
        assert a["counters"][k] == b["counters"][k], (what, k, a["counters"][k], b["counters"][k])
    assert a["statistics"] == b["statistics"], what


@pytest.mark.gpu
@pytest.mark.parametrize("name,scale", [("cfg2", 256 / 4096), ("cfg3", 96 / 65536), ("cfg4", 256 / 1048576),
                                        ("folding_arm", 1.0)])
def test_cooperative_matches_oracle(fks_lib, oracle_lib, name, scale):
    """up to a full cooperative grid (256 particles) against the oracle, exactly"""
    wl = getattr(W, name)(scale)
    g, o = run_both(wl, small_batch_kernel=True, cooperative=True, call_index=1)
    print(name, mismatch_report(g, o), g["launch"])
    assert g["launch"]["cooperative_resident_particles"] >= min(256, len(wl.starts)), g["launch"]
    assert g["launch"]["last_kernel"] == "cooperative", g["launch"]
    assert_identical(g, o)
    assert_counters_identical(g, o)


@pytest.mark.gpu
def test_heaviest_particles_alone_equal_their_batch(fks_lib):
    """cfg3's most contact-heavy particles (thousands of resolver iterations each), each run
    alone on the cooperative kernel and on the one-wave kernels: identical outputs and counters,
    and the outputs equal the particle's row of the full 65,536-particle batch"""
    from fast_kinematic_simulator_amd import make_linked_simulator

    wl = W.cfg3()
    sim = make_linked_simulator(wl.environment(), wl.solver, wl.controller_frequency, wl.seed)
    try:
        sim.set_robot(wl.robot)
        full = _run_device(sim, wl, wl.starts, 0)
        assert full["kernel"] == "shaped", full["kernel"]
        heavy = [int(i) for i in np.argsort(-full["resolver_iterations"].astype(np.int64))[:6]]
        for i in heavy:
            sim.set_small_batch_kernel(True)
            sim.set_cooperative_waves(True)
            c = _run_device(sim, wl, wl.starts[i:i + 1], i)
            assert c["kernel"] == "cooperative", c["kernel"]
            sim.set_cooperative_waves(False)
            s1 = _run_device(sim, wl, wl.starts[i:i + 1], i)
            assert s1["kernel"] == "shaped_small_batch", s1["kernel"]  # the module is built by now
            sim.set_small_batch_kernel(False)
            t1 = _run_device(sim, wl, wl.starts[i:i + 1], i)
            assert t1["kernel"] == "shaped", t1["kernel"]
            _same(c, s1, f"particle {i}: cooperative vs small-batch")
            _same(c, t1, f"particle {i}: cooperative vs shaped")
            for k in KEYS:
                assert np.array_equal(c[k][0], full[k][i]), (i, k)
            assert c["resolver_iterations"][0] > 1000
    finally:
        sim.close()


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["cfg3", "cfg2"])
def test_cooperative_grid_equals_throughput(fks_lib, name):
    """a full cooperative grid of contiguous particles around the heaviest one, against the
    shape-specialised throughput kernel on the same ids"""
    from fast_kinematic_simulator_amd import make_linked_simulator

    wl = getattr(W, name)()
    sim = make_linked_simulator(wl.environment(), wl.solver, wl.controller_frequency, wl.seed)
    try:
        sim.set_robot(wl.robot)
        n = sim.launch_info()["cooperative_resident_particles"]
        assert n >= 64
        full = _run_device(sim, wl, wl.starts, 0)
        top = int(np.argmax(full["resolver_iterations"]))
        i0 = max(0, min(top - n // 2, len(wl.starts) - n))
        sim.set_cooperative_waves(True)
        c = _run_device(sim, wl, wl.starts[i0:i0 + n], i0, call_index=0)
        assert c["kernel"] == "cooperative", c["kernel"]
        sim.set_small_batch_kernel(False)
        t = _run_device(sim, wl, wl.starts[i0:i0 + n], i0, call_index=0)
        assert t["kernel"] == "shaped", t["kernel"]
        _same(c, t, f"{name} particles {i0}..{i0 + n}")
        for k in KEYS:
            assert np.array_equal(c[k], full[k][i0:i0 + n]), k
    finally:
        sim.close()
