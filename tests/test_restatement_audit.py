"""The restatement audit's oracle variants (oracle/Makefile `audit`)
build, load, and keep the batch-level quantities DESIGN.md reports as robust: no
collided flag moves and total microsteps stay within a few percent, while per-particle
microstep counts may change (contact resolution is chaotic under one-ulp changes)."""
import numpy as np
import pytest

import oracle
from fast_kinematic_simulator_amd import workloads


@pytest.mark.parametrize("variant", oracle.AUDIT_VARIANTS)
def test_audit_variant_batch_statistics(variant):
    wl = workloads.cfg2()
    n = 64
    def run():
        return oracle.forward_simulate(wl.environment(), wl.robot, wl.solver, wl.controller_frequency, wl.seed, wl.starts[:n],
                                       wl.targets, True, threads=4)
    base = run()
    with oracle.audit_variant(variant):
        alt = run()
    assert np.array_equal(base["collided"], alt["collided"])
    tb, ta = int(np.sum(base["microsteps"])), int(np.sum(alt["microsteps"]))
    assert abs(ta - tb) <= 0.05 * tb
    assert oracle.lib() is not None  # the parity oracle is restored after the block
