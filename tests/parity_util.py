"""Helpers shared by the parity tests: run the HIP path and the CPU oracle on the
same inputs and compare every output field exactly."""
import numpy as np


COUNTER_KEYS = ("microsteps", "resolver_iterations", "controller_steps", "sdf_bytes", "error_particles", "least_squares_rows",
                "self_collision_checks", "self_corrected_points")


def run_both(wl, starts=None, targets=None, allow_contacts=None, call_index=0, first_particle_id=0, sim=None,
             individual_jacobians=False, segment_steps=None, small_batch_kernel=None, specialize=False, cooperative=None):
    import oracle
    from fast_kinematic_simulator_amd import make_linked_simulator

    env = wl.environment()
    starts = wl.starts if starts is None else starts
    targets = wl.targets if targets is None else targets
    allow = wl.allow_contacts if allow_contacts is None else allow_contacts
    own = sim is None
    if own:
        sim = make_linked_simulator(env, wl.solver, wl.controller_frequency, wl.seed)
    if individual_jacobians:
        sim.set_individual_jacobians(True)
    if segment_steps is not None:
        sim.set_segment_steps(segment_steps)
    if small_batch_kernel is not None:
        sim.set_small_batch_kernel(small_batch_kernel)
    if cooperative is not None:
        sim.set_cooperative_waves(cooperative)
    if specialize:
        # the robot-shape-specialised throughput kernel (fks_set_specialization); small batches
        # would otherwise run the small-batch kernel
        sim.set_robot(wl.robot)
        sim.set_specialization(True)
        sim.set_small_batch_kernel(False)
        before = sim.specialization()["launches"]
    elif own:
        # the generic kernels (the library's default is the specialised one: test_specialize.py
        # and the planner / full-size tests run that)
        sim.set_specialization(False)
    sim.set_call_index(call_index)
    g = sim.forward_simulate_arrays(wl.robot, starts, targets, allow)
    g["statistics"] = sim.get_statistics()
    g["counters"] = sim.last_call_counters()
    g["launch"] = sim.launch_info()
    if specialize:
        info = sim.specialization()
        assert info["active"] and info["launches"] == before + 1, info
        assert g["launch"]["last_kernel"] == "shaped", g["launch"]
        g["specialization"] = info
    if own:
        sim.close()
    o = oracle.forward_simulate(env, wl.robot, wl.solver, wl.controller_frequency, wl.seed, starts, targets, allow,
                                call_index=call_index, first_particle_id=first_particle_id,
                                individual_jacobians=individual_jacobians)
    return g, o


def assert_counters_identical(g, o):
    assert g["statistics"] == o["statistics"]
    for k in COUNTER_KEYS:
        assert g["counters"][k] == o["counters"][k], (k, g["counters"][k], o["counters"][k])


def mismatch_report(g, o, limit=5):
    lines = []
    n = len(o["microsteps"])
    bad = np.zeros(n, dtype=bool)
    for k in ("collided", "microsteps", "resolver_iterations", "error_flags"):
        bad |= np.asarray(g[k]) != np.asarray(o[k])
    bad |= np.any(g["positions"] != o["positions"], axis=1)
    idx = np.nonzero(bad)[0]
    lines.append(f"{len(idx)} / {n} particles differ")
    for i in idx[:limit]:
        lines.append(f"  particle {i}: micro {g['microsteps'][i]} vs {o['microsteps'][i]}, resolver "
                     f"{g['resolver_iterations'][i]} vs {o['resolver_iterations'][i]}, collided {g['collided'][i]} vs "
                     f"{o['collided'][i]}, err {g['error_flags'][i]} vs {o['error_flags'][i]}, max|dq| "
                     f"{np.max(np.abs(g['positions'][i] - o['positions'][i])):.3e}")
    return "\n".join(lines)


def assert_identical(g, o):
    report = mismatch_report(g, o)
    assert np.array_equal(g["collided"], o["collided"]), report
    assert np.array_equal(g["microsteps"], o["microsteps"]), report
    assert np.array_equal(g["resolver_iterations"], o["resolver_iterations"]), report
    assert np.array_equal(g["error_flags"], o["error_flags"]), report
    # joint states: bit-exact in practice; the contract (BASELINE.json) is 1e-6
    assert np.array_equal(g["positions"], o["positions"]), report + f"\nmax |dq| {np.max(np.abs(g['positions'] - o['positions']))}"
