"""The skip proofs at full size: the product kernel against the same kernel with every proof
compiled out.

The product's speed rests on shortcuts that decide "this work cannot change the result" from
a cached state and a floating-point margin: the environment / correction
round proofs, the motion estimate's round pruning, the self-collision gap proof and the two
lever-arm shortcuts of the resolver (SPCS:1563-1575, 1663-1682).  The oracle has none of
them, but it re-simulates only sampled blocks of a full batch (test_full_size.py).  Here the
whole batch (every particle of cfg3's 65,536 and of the 131,072-particle cfg4 / cfg5 shards)
runs twice on the GPU: through the product's shape-specialised kernel and through the same
source built with FKS_NO_SKIP_PROOFS (fks_set_specialization(ctx, FKS_SPECIALIZE_NO_PROOFS)),
which evaluates every check in full as the reference does.  Every output byte, every call
counter (algorithmic SDF bytes included) and every statistic must be equal."""
import os
import subprocess

import numpy as np
import pytest

from fast_kinematic_simulator_amd import _capi
from fast_kinematic_simulator_amd import make_linked_simulator
from fast_kinematic_simulator_amd import workloads as W

from parity_util import COUNTER_KEYS, assert_counters_identical, assert_identical, run_both

KEYS = ("positions", "collided", "microsteps", "resolver_iterations", "error_flags")


def test_proof_free_shape_compiles(tmp_path):
    """The validation build (what fks_shapec compiles for FKS_SPECIALIZE_NO_PROOFS) compiles for
    gfx950 here, within the throughput kernel's register budget."""
    from fast_kinematic_simulator_amd import build

    shapec = build.build_shapec()
    src = tmp_path / "src"
    src.mkdir()
    for name, rel in build.EMBEDDED:
        (src / name).write_bytes(open(os.path.join(build.PKG, rel), "rb").read())
    out = tmp_path / "k.hsaco"
    shape = dict(TYPE=0, L=8, J=7, D=7, W=7, G=8, P=512, PAIR=1, LEAN=0)
    cmd = [shapec, str(out), str(src), "--offload-arch=gfx950", "-O3", "-ffp-contract=off", "-std=c++17",
           "-DFKS_NO_SKIP_PROOFS=1"] + [f"-DFKS_SHAPE_{k}={v}" for k, v in shape.items()]
    p = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, timeout=600)
    assert p.returncode == 0, p.stdout[-3000:]
    notes = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-readelf", "--notes", str(out)], stdout=subprocess.PIPE, text=True).stdout
    vgprs = [int(l.split(":")[1]) for l in notes.splitlines() if l.strip().startswith(".vgpr_count:")]
    assert vgprs and vgprs[0] <= 96, vgprs


def _run(sim, wl, mode, call_index):
    sim.set_specialization(mode)
    info = sim.specialization()
    assert info["active"] and not info["failed"], info
    assert info["shape"].endswith("-np") == (mode == _capi.SPECIALIZE_NO_PROOFS), info
    sim.set_call_index(call_index)
    sim.reset_statistics()
    r = sim.forward_simulate_arrays(wl.robot, wl.starts, wl.targets, wl.allow_contacts)
    assert sim.launch_info()["last_kernel"] == "shaped", sim.launch_info()
    r["counters"] = sim.last_call_counters()
    r["statistics"] = sim.get_statistics()
    return r


@pytest.mark.gpu
@pytest.mark.parametrize("name,scale", [("cfg3", 1.0), ("cfg4", 131072 / 1048576), ("cfg5", 131072 / 1048576),
                                        ("folding_arm", 4096 / 32)])
def test_full_batch_equals_the_proof_free_kernel(fks_lib, name, scale):
    wl = {**W.WORKLOADS, **W.COVERAGE}[name](scale)
    if name in W.SCENES:
        wl._env = W.SCENES[name](device=0)  # the GPU build: the host build's bytes, seconds faster at 512^3
    sim = make_linked_simulator(wl.environment(), wl.solver, wl.controller_frequency, wl.seed)
    try:
        sim.set_robot(wl.robot)
        sim.set_small_batch_kernel(False)
        p = _run(sim, wl, _capi.SPECIALIZE_ON, 7)
        q = _run(sim, wl, _capi.SPECIALIZE_NO_PROOFS, 7)
    finally:
        sim.close()
    print(name, "product", p["counters"]["kernel_ms"], "ms; proof-free", q["counters"]["kernel_ms"], "ms;",
          len(wl.starts), "particles,", p["counters"]["microsteps"], "microsteps,", p["counters"]["resolver_iterations"],
          "resolver iterations,", p["counters"]["self_collision_checks"], "self-collision checks")
    for k in KEYS:
        assert np.array_equal(p[k], q[k]), (k, int(np.sum(np.any(np.atleast_2d(p[k] != q[k]).reshape(len(wl.starts), -1), axis=1))))
    for k in COUNTER_KEYS:
        assert p["counters"][k] == q["counters"][k], (k, p["counters"][k], q["counters"][k])
    assert p["statistics"] == q["statistics"]
    assert p["counters"]["microsteps"] > 0 and p["collided"].any()


@pytest.mark.gpu
@pytest.mark.parametrize("name,scale", [("cfg3", 96 / 65536), ("cfg4", 64 / 1048576), ("folding_arm", 1.0)])
def test_proof_free_kernel_matches_the_oracle(fks_lib, oracle_lib, name, scale):
    """The validation kernel is itself exact against the oracle (so the full-batch equality
    above compares the product with the reference's own evaluation order)."""
    wl = {**W.WORKLOADS, **W.COVERAGE}[name](scale)
    sim = make_linked_simulator(wl.environment(), wl.solver, wl.controller_frequency, wl.seed)
    try:
        sim.set_robot(wl.robot)
        sim.set_small_batch_kernel(False)
        sim.set_specialization(_capi.SPECIALIZE_NO_PROOFS)
        g, o = run_both(wl, sim=sim)
        assert g["launch"]["last_kernel"] == "shaped" and sim.specialization()["shape"].endswith("-np")
    finally:
        sim.close()
    assert_identical(g, o)
    assert_counters_identical(g, o)
