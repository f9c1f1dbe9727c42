"""Regenerate the simulation golden fixtures tests/golden/sim_<case>.npz.

Each fixture holds the inputs of a small seeded batch (starts, targets, call index,
allow_contacts, the workload scale) and the CPU oracle's outputs for it (reached
configurations, collided flags, microsteps, resolver iterations, error bits,
statistics, work counters), plus the SHA-256 of the scene's SDF so a drift in the
environment builder is caught before the simulation is compared.  The scenes
themselves are rebuilt from fast_kinematic_simulator_amd.workloads (seeded).

These are regression vectors of the restatement (the reference itself cannot be
built here): tests/test_golden.py checks that the oracle still
reproduces them on the CPU and that the HIP path reproduces them on the GPU.

    python tests/golden/make_sim_golden.py
"""
import hashlib
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

# (fixture, workload, particles, allow_contacts, call_index, per-particle targets)
CASES = [
    ("cfg1_contacts", "cfg1", 32, True, 0, False),
    ("cfg1_no_contacts_targets", "cfg1", 32, False, 5, True),
    ("cfg2", "cfg2", 32, True, 0, False),
    ("cfg3", "cfg3", 16, True, 0, False),
    ("cfg4", "cfg4", 32, True, 2, False),
    ("cfg5", "cfg5", 8, True, 0, False),
]
FULL = {"cfg1": 32, "cfg2": 4096, "cfg3": 65536, "cfg4": 1048576, "cfg5": 1048576}
STAT_KEYS = ["successful_resolves", "unsuccessful_resolves", "free_resolves", "collision_resolves", "fallback_resolves",
             "unsuccessful_env_collision_resolves", "unsuccessful_self_collision_resolves", "recovered_unsuccessful_resolves"]
COUNTER_KEYS = ["particles", "controller_steps", "microsteps", "resolver_iterations", "sdf_bytes", "error_particles",
                "least_squares_rows"]


def case_inputs(workload, n, per_particle_targets):
    from fast_kinematic_simulator_amd import workloads as W

    wl = W.WORKLOADS[workload](n / FULL[workload])
    starts = wl.starts[:n]
    targets = wl.targets
    if per_particle_targets:
        rng = np.random.default_rng(11)
        targets = starts + rng.uniform(-0.6, 0.6, size=starts.shape)
    return wl, starts, targets


def sdf_digest(env):
    return hashlib.sha256(np.ascontiguousarray(env.sdf).tobytes()).hexdigest()


def main():
    import oracle

    for name, workload, n, allow, call_index, ppt in CASES:
        wl, starts, targets = case_inputs(workload, n, ppt)
        env = wl.environment()
        r = oracle.forward_simulate(env, wl.robot, wl.solver, wl.controller_frequency, wl.seed, starts, targets, allow,
                                    call_index=call_index)
        path = os.path.join(HERE, f"sim_{name}.npz")
        np.savez_compressed(
            path, workload=workload, particles=n, allow_contacts=allow, call_index=call_index,
            per_particle_targets=ppt, sdf_sha256=sdf_digest(env), starts=starts, targets=targets,
            positions=r["positions"], collided=r["collided"], microsteps=r["microsteps"],
            resolver_iterations=r["resolver_iterations"], error_flags=r["error_flags"],
            statistics=np.array([r["statistics"][k] for k in STAT_KEYS]),
            counters=np.array([r["counters"][k] for k in COUNTER_KEYS], dtype=np.uint64))
        print(f"{path}: {int(r['collided'].sum())}/{n} collided, {int(r['resolver_iterations'].sum())} resolver iterations")


if __name__ == "__main__":
    main()
