"""Robot-shape-specialised throughput kernels (fks_set_specialization, fks_specialize.cpp):
the library's own kernel source compiled at run time (hiprtc) with the robot's dimensions
and LDS / scratch carve-outs as constants.  The arithmetic is the generic kernel's, so every
output must still equal the CPU oracle bit for bit, on every robot family and layout:
SE(2), SE(3), linked arms with the paired FK (cfg2, cfg3), the lean LDS block (cfg5), a
self-colliding arm and a chain too long for the paired FK."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

from fast_kinematic_simulator_amd import workloads as W

from parity_util import assert_counters_identical, assert_identical, mismatch_report, run_both

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SPEC_CASES = [("cfg1", 1.0), ("cfg2", 48 / 4096), ("cfg3", 96 / 65536), ("cfg4", 64 / 1048576), ("cfg5", 32 / 1048576),
              ("folding_arm", 1.0), ("long_chain", 1.0)]


def test_shape_build_compiles_for_every_family():
    """The shape-specialised build (what hiprtc compiles on the GPU box) compiles for gfx950
    here: a linked arm with the paired FK, a lean linked block, SE(2) and SE(3)."""
    shapes = [dict(TYPE=0, L=8, J=7, D=7, W=7, G=8, P=512, PAIR=1, LEAN=0), dict(TYPE=0, L=17, J=16, D=14, W=14, G=17, P=1088, PAIR=0, LEAN=1),
              dict(TYPE=1, L=1, J=0, D=3, W=3, G=1, P=64, PAIR=0, LEAN=0), dict(TYPE=2, L=1, J=0, D=6, W=12, G=1, P=256, PAIR=0, LEAN=0)]
    for sh in shapes[:2] if os.environ.get("FKS_QUICK") else shapes:
        cmd = ["hipcc", "--offload-arch=gfx950", "-O1", "-std=c++17", "-ffp-contract=off", f"-I{ROOT}/include",
               f"-I{ROOT}/fast_kinematic_simulator_amd/csrc", "--cuda-device-only", "-c", "-x", "hip",
               f"{ROOT}/fast_kinematic_simulator_amd/csrc/fks_kernels.hip", "-o", os.devnull] + [f"-DFKS_SHAPE_{k}={v}" for k, v in sh.items()]
        p = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, timeout=600)
        assert p.returncode == 0, p.stdout[-3000:]


def test_shapec_compiles_the_sources_it_is_handed(tmp_path):
    """fks_shapec (the compiler process the library starts) compiles the kernel sources the
    library writes out for it, with hiprtc, into a gfx950 code object; a robot whose LDS block
    holds 4 waves per SIMD (cfg5's lean block) gets their registers (FKS_WAVES_PER_EU=4)."""
    from fast_kinematic_simulator_amd import build

    shapec = build.build_shapec()
    src = tmp_path / "src"
    src.mkdir()
    for name, rel in build.EMBEDDED:
        (src / name).write_bytes(open(os.path.join(build.PKG, rel), "rb").read())
    out = tmp_path / "k.hsaco"
    shape = dict(TYPE=0, L=17, J=16, D=14, W=14, G=17, P=1088, PAIR=0, LEAN=1)
    cmd = [shapec, str(out), str(src), "--offload-arch=gfx950", "-O3", "-ffp-contract=off", "-std=c++17",
           "-DFKS_WAVES_PER_EU=4"] + [f"-DFKS_SHAPE_{k}={v}" for k, v in shape.items()]
    p = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, timeout=600)
    assert p.returncode == 0, p.stdout[-3000:]
    notes = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-readelf", "--notes", str(out)], stdout=subprocess.PIPE, text=True).stdout
    vgprs = [int(l.split(":")[1]) for l in notes.splitlines() if l.strip().startswith(".vgpr_count:")]
    assert vgprs and 96 < vgprs[0] <= 128, vgprs
    assert ".name:           fks_simulate_shaped" in notes
    bad = subprocess.run([shapec, str(out), str(tmp_path / "missing")], stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    assert bad.returncode != 0 and "fks_kernels.hip" in bad.stdout


@pytest.mark.gpu
@pytest.mark.parametrize("name,scale", SPEC_CASES)
def test_specialized_kernel_parity(fks_lib, oracle_lib, name, scale):
    wl = {**W.WORKLOADS, **W.COVERAGE}[name](scale)
    g, o = run_both(wl, specialize=True)
    print(name, g["specialization"], mismatch_report(g, o))
    if name == "cfg5":  # the lean block holds 4 waves per SIMD: the kernel gets their registers
        assert g["specialization"]["shape"].endswith("-w4"), g["specialization"]
    assert_identical(g, o)
    assert_counters_identical(g, o)


@pytest.mark.gpu
@pytest.mark.parametrize("name,scale", [c for c in SPEC_CASES if c[0] not in ("cfg5", "long_chain")])  # lean blocks: no small kernel
def test_shaped_small_batch_kernel_parity(fks_lib, oracle_lib, name, scale):
    """Once a robot's module is built, a batch that fits the small-batch grid runs the module's
    small-batch kernel (fks_simulate_shaped_small; lean shapes have none): oracle-exact"""
    from fast_kinematic_simulator_amd import make_linked_simulator

    wl = getattr(W, name)(scale)
    sim = make_linked_simulator(wl.environment(), wl.solver, wl.controller_frequency, wl.seed)
    try:
        sim.set_robot(wl.robot)
        sim.set_specialization(True)  # builds the module now
        assert sim.specialization()["active"], sim.specialization()
        g, o = run_both(wl, sim=sim, call_index=4)
        print(name, mismatch_report(g, o), g["launch"])
        assert g["launch"]["last_kernel"] == "shaped_small_batch", g["launch"]
        assert_identical(g, o)
        assert_counters_identical(g, o)
    finally:
        sim.close()


@pytest.mark.gpu
def test_specialized_segmented_cfg3(fks_lib, oracle_lib):
    """Segment hand-over through the specialised kernel (segments of 3 controller steps)."""
    wl = W.cfg3(64 / 65536)
    g, o = run_both(wl, specialize=True, segment_steps=3)
    assert_identical(g, o)
    assert_counters_identical(g, o)


@pytest.mark.gpu
def test_specialization_follows_the_robot_and_is_cached(fks_lib, tmp_path, monkeypatch):
    """Specialisation is on by default and lazy: setting a robot leaves its kernel pending, a
    small batch (small-batch kernel) does not build it, the first throughput call does.
    Setting another robot releases the old kernel; a second context finds the code object in
    the process cache; switching it off returns to the generic kernel; results never change."""
    from fast_kinematic_simulator_amd import make_linked_simulator

    a, b = W.cfg3(32 / 65536), W.folding_arm(1.0)
    sim = make_linked_simulator(a.environment(), a.solver, a.controller_frequency, a.seed)
    sim.set_robot(a.robot)
    i0 = sim.specialization()
    assert i0["enabled"] and i0["pending"] and not i0["active"], i0
    sim.forward_simulate_arrays(a.robot, a.starts, a.targets, True)  # 32 particles: the small-batch kernel
    assert sim.launch_info()["last_kernel"] == "small_batch" and sim.specialization()["pending"]
    sim.set_small_batch_kernel(False)
    sim.set_call_index(0)
    ra = sim.forward_simulate_arrays(a.robot, a.starts, a.targets, True)  # builds the kernel, then runs it
    ia = sim.specialization()
    assert ia["active"] and not ia["pending"] and ia["launches"] == 1 and ia["shape"].startswith("t0-L8-J7-D7"), ia
    assert sim.launch_info()["last_kernel"] == "shaped"
    sim.set_robot(b.robot)
    ib = sim.specialization()
    assert ib["pending"] and not ib["active"] and ib["launches"] == 0
    sim.forward_simulate_arrays(b.robot, b.starts, b.targets, True)
    ib = sim.specialization()
    assert ib["active"] and ib["shape"] != ia["shape"] and ib["launches"] == 1
    sim.set_robot(a.robot)
    sim.set_specialization(True)  # builds now (from the process cache)
    assert sim.specialization()["active"] and sim.specialization()["from_cache"]
    sim.set_specialization(False)
    assert not sim.specialization()["active"] and not sim.specialization()["pending"]
    sim.set_call_index(0)
    rg = sim.forward_simulate_arrays(a.robot, a.starts, a.targets, True)
    assert sim.launch_info()["last_kernel"] == "throughput"
    for k in ("positions", "collided", "microsteps", "resolver_iterations", "error_flags"):
        assert np.array_equal(ra[k], rg[k]), k
    sim.close()
    sim2 = make_linked_simulator(a.environment(), a.solver, a.controller_frequency, a.seed)
    sim2.set_robot(a.robot)
    sim2.set_specialization(True)
    assert sim2.specialization()["from_cache"] and sim2.specialization()["compile_seconds"] == 0.0
    sim2.close()


@pytest.mark.gpu
def test_failed_build_falls_back_and_is_reported(fks_lib, monkeypatch, tmp_path):
    """A shape build that cannot run (no compiler helper) leaves the generic kernel in place:
    the same results, reported through fks_get_specialization (failed, message), and an
    explicit fks_set_specialization(ctx, 1) raises with the log.  The C++ classes report the
    same record through SpecializationStatus() (tests/cpp/planner_interface_test.cpp)."""
    from fast_kinematic_simulator_amd import FksError, make_linked_simulator

    wl = W.cfg2(48 / 4096)
    sim = make_linked_simulator(wl.environment(), wl.solver, wl.controller_frequency, wl.seed)
    try:
        sim.set_robot(wl.robot)
        sim.set_small_batch_kernel(False)
        monkeypatch.setenv("FKS_SHAPEC", str(tmp_path / "no-such-fks_shapec"))
        monkeypatch.setenv("FKS_KERNEL_CACHE", "off")
        sim.set_call_index(0)
        r_fallback = sim.forward_simulate_arrays(wl.robot, wl.starts, wl.targets, True)  # the lazy build fails here
        info = sim.specialization()
        assert info["failed"] and not info["active"] and not info["pending"], info
        assert "cannot run" in info["message"] and info["shape"].startswith("t0-"), info
        assert sim.launch_info()["last_kernel"] == "throughput"
        with pytest.raises(FksError):
            sim.set_specialization(True)
        assert sim.specialization()["failed"]
        monkeypatch.delenv("FKS_SHAPEC")
        sim.set_specialization(True)
        info = sim.specialization()
        assert info["active"] and not info["failed"] and info["message"] == "", info
        sim.set_call_index(0)
        r_shaped = sim.forward_simulate_arrays(wl.robot, wl.starts, wl.targets, True)
        assert sim.launch_info()["last_kernel"] == "shaped"
    finally:
        sim.close()
    for k in ("positions", "collided", "microsteps", "resolver_iterations", "error_flags"):
        assert np.array_equal(r_fallback[k], r_shaped[k]), k


_CACHE_CHILD = r"""
import json, sys
sys.path.insert(0, sys.argv[1])
from fast_kinematic_simulator_amd import make_linked_simulator
from fast_kinematic_simulator_amd import workloads as W
wl = W.cfg2(48 / 4096)
sim = make_linked_simulator(wl.environment(), wl.solver, wl.controller_frequency, wl.seed)
sim.set_robot(wl.robot)
sim.set_small_batch_kernel(False)
sim.set_call_index(0)
r = sim.forward_simulate_arrays(wl.robot, wl.starts, wl.targets, True)
print(json.dumps({"spec": sim.specialization(), "kernel": sim.launch_info()["last_kernel"],
                  "q": r["positions"].tobytes().hex(), "micro": r["microsteps"].tolist()}))
sim.close()
"""


@pytest.mark.gpu
def test_unusable_cached_code_object_is_rebuilt(fks_lib, tmp_path):
    """The disk cache is validated: an entry that is not a code object, or one the runtime
    refuses to load, is dropped and compiled afresh (each run is a fresh process, so the
    process cache cannot hide the disk file), and the results do not change."""
    cache = tmp_path / "cache"
    env = dict(os.environ, FKS_KERNEL_CACHE=str(cache))
    env.pop("FKS_SHAPEC", None)

    def child():
        p = subprocess.run([sys.executable, "-c", _CACHE_CHILD, ROOT], stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True,
                           timeout=300, env=env)
        assert p.returncode == 0, p.stderr[-3000:]
        return json.loads(p.stdout.strip().splitlines()[-1])

    first = child()
    assert first["kernel"] == "shaped" and not first["spec"]["from_cache"], first["spec"]
    files = sorted(cache.glob("*.hsaco"))
    assert len(files) == 1 and oct(cache.stat().st_mode & 0o777) == "0o700"
    again = child()
    assert again["spec"]["from_cache"] and again["q"] == first["q"]
    for bad in (b"not a code object" * 64, b"\x7fELF" + b"\0" * 4096):
        files[0].write_bytes(bad)
        r = child()
        assert r["kernel"] == "shaped" and r["spec"]["active"] and not r["spec"]["from_cache"], r["spec"]
        assert r["q"] == first["q"] and r["micro"] == first["micro"]
        assert files[0].read_bytes()[:4] == b"\x7fELF" and len(files[0].read_bytes()) > 4096 + 4
