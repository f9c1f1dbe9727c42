"""Committed golden fixtures (tests/golden/sim_*.npz, written by
tests/golden/make_sim_golden.py): the CPU oracle must keep reproducing them, and the
HIP path must reproduce them bit for bit on the GPU (positions, collided flags,
microsteps, resolver iterations, error bits, statistics, work counters)."""
import functools
import glob
import hashlib
import os
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "golden"))

from make_sim_golden import COUNTER_KEYS, FULL, STAT_KEYS  # noqa: E402

FIXTURES = sorted(glob.glob(os.path.join(HERE, "golden", "sim_*.npz")))


def _load(path):
    return dict(np.load(path, allow_pickle=False))


@functools.lru_cache(maxsize=None)
def _scene(workload, n):
    from fast_kinematic_simulator_amd import workloads as W

    wl = W.WORKLOADS[workload](n / FULL[workload])
    return wl, wl.environment()


def _check(f, r, stats, counters):
    assert np.array_equal(r["positions"], f["positions"])
    assert np.array_equal(np.asarray(r["collided"], dtype=bool), f["collided"])
    assert np.array_equal(r["microsteps"], f["microsteps"])
    assert np.array_equal(r["resolver_iterations"], f["resolver_iterations"])
    assert np.array_equal(r["error_flags"], f["error_flags"])
    assert [stats[k] for k in STAT_KEYS] == list(f["statistics"])
    assert [int(counters[k]) for k in COUNTER_KEYS] == [int(v) for v in f["counters"]]


def _prepare(path):
    f = _load(path)
    wl, env = _scene(str(f["workload"]), int(f["particles"]))
    assert hashlib.sha256(np.ascontiguousarray(env.sdf).tobytes()).hexdigest() == str(f["sdf_sha256"]), \
        "the seeded scene no longer matches the fixture (environment builder drift)"
    return f, wl, env


def test_fixtures_present():
    assert len(FIXTURES) >= 6


@pytest.mark.parametrize("path", FIXTURES, ids=[os.path.basename(p) for p in FIXTURES])
def test_oracle_reproduces_golden(oracle_lib, path):
    import oracle

    f, wl, env = _prepare(path)
    r = oracle.forward_simulate(env, wl.robot, wl.solver, wl.controller_frequency, wl.seed, f["starts"], f["targets"],
                                bool(f["allow_contacts"]), call_index=int(f["call_index"]))
    _check(f, r, r["statistics"], r["counters"])


@pytest.mark.gpu
@pytest.mark.parametrize("path", FIXTURES, ids=[os.path.basename(p) for p in FIXTURES])
def test_hip_reproduces_golden(fks_lib, path):
    from fast_kinematic_simulator_amd import make_linked_simulator

    f, wl, env = _prepare(path)
    sim = make_linked_simulator(env, wl.solver, wl.controller_frequency, wl.seed)
    sim.set_call_index(int(f["call_index"]))
    r = sim.forward_simulate_arrays(wl.robot, f["starts"], f["targets"], bool(f["allow_contacts"]))
    _check(f, r, sim.get_statistics(), sim.last_call_counters())
    sim.close()
