"""The C-ABI library: loads without a GPU, exports every symbol include/*.h
declares, validates arguments; the CPU environment builder (SEB.cpp restated)
against an independent exact EDT (scipy)."""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    syms = set()
    for name in os.listdir(os.path.join(ROOT, "include")):
        if not name.endswith(".h"):
            continue
        text = open(os.path.join(ROOT, "include", name)).read()
        text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
        for m in re.finditer(r"^[A-Za-z_][\w\s\*]*?\b(fks_\w+)\s*\(", text, flags=re.M):
            syms.add(m.group(1))
    return syms


def test_library_exports_every_declared_symbol(fks_lib):
    from fast_kinematic_simulator_amd import _capi

    syms = declared_symbols()
    assert len(syms) >= 25
    out = subprocess.run(["nm", "-D", "--defined-only", _capi.LIB_PATH], capture_output=True, text=True, check=True).stdout
    exported = {line.split()[-1] for line in out.splitlines() if line.strip()}
    missing = sorted(syms - exported)
    assert not missing, missing
    bound = {p[0] for p in _capi.PROTOTYPES}
    assert syms == bound, (syms ^ bound)


def test_abi_basics(fks_lib):
    from fast_kinematic_simulator_amd import _capi, get_default_solver_parameters

    assert fks_lib.fks_abi_version() == 10
    assert fks_lib.fks_status_string(0) == b"ok"
    p = _capi.SolverParams()
    assert fks_lib.fks_default_solver_params(ctypes.byref(p)) == 0
    d = get_default_solver_parameters()
    for name, _ in _capi.SolverParams._fields_:
        if name != "reserved":
            assert getattr(p, name) == getattr(d, name), name
    # SPCS:357-368 literal defaults
    assert (p.forward_simulation_time, p.simulation_shortcut_distance, p.environment_collision_check_tolerance) == (1.0, 0.0, 0.001)
    assert (p.max_resolver_iterations, p.resolve_correction_step_scaling_decay_iterations) == (25, 5)
    assert p.failed_resolves_end_motion == 1 and p.resolve_correction_min_step_scaling == 0.03125


def test_argument_validation(fks_lib):
    from fast_kinematic_simulator_amd import _capi

    ctx = ctypes.c_void_p()
    assert fks_lib.fks_create(None, None, 100.0, 1, 0, 0, ctypes.byref(ctx)) == 1
    assert fks_lib.fks_forward_simulate(None, None, 0, None, 0, 1, None, None, None, None, None) == 1
    assert fks_lib.fks_set_robot(None, None) == 1
    assert fks_lib.fks_default_solver_params(None) == 1
    h = ctypes.c_void_p()
    assert fks_lib.fks_env_build(None, 0, -1.0, None, None, ctypes.byref(h)) == 1
    # scheduling knob and grid diagnostics (no reference counterpart)
    assert fks_lib.fks_set_segment_steps(None, 10) == 1
    assert fks_lib.fks_set_segment_policy(None, 2, 1) == 1
    assert fks_lib.fks_set_small_batch_kernel(None, 1) == 1
    assert fks_lib.fks_set_segment_heavy_relative(None, 3) == 1
    assert fks_lib.fks_set_cooperative_waves(None, 1) == 1
    assert fks_lib.fks_set_individual_jacobians(None, 1) == 1
    waves, lds = ctypes.c_uint32(0), ctypes.c_uint64(0)
    assert fks_lib.fks_get_launch_geometry(None, ctypes.byref(waves), ctypes.byref(lds)) == 1
    assert _capi.PHASE_NAMES[15] == "wave_residency" and len(_capi.PHASE_NAMES) == _capi.NUM_PHASES


def test_create_without_gpu_reports_no_device(fks_lib):
    """On a host without a HIP device the product refuses loudly (no CPU fallback)."""
    from fast_kinematic_simulator_amd import SimulatorSolverParameters, _capi

    n = ctypes.c_int(0)
    import fast_kinematic_simulator_amd._capi as C

    hip = ctypes.CDLL("libamdhip64.so")
    if hip.hipGetDeviceCount(ctypes.byref(n)) == 0 and n.value > 0:
        pytest.skip("a HIP device is present")
    from fast_kinematic_simulator_amd import ObstacleConfig, build_complete_environment, transform34

    env = build_complete_environment([ObstacleConfig(1, transform34([0.5, 0.5, 0.5]), [0.1, 0.1, 0.1])], 0.1,
                                     origin=transform34([0, 0, 0]), num_cells=(10, 10, 10))
    env_c, keep = env.to_c()
    params = SimulatorSolverParameters().to_c()
    ctx = ctypes.c_void_p()
    assert fks_lib.fks_create(ctypes.byref(env_c), ctypes.byref(params), 100.0, 1, 0, 0, ctypes.byref(ctx)) == 6  # NO_DEVICE
    assert not ctx.value


def test_environment_builder_matches_exact_edt(fks_lib):
    """SDF = +distance to the nearest filled cell (free) / -distance to the nearest
    free cell (filled), in cell units x resolution (sdf_tools convention), against
    scipy.ndimage.distance_transform_edt."""
    from scipy import ndimage

    from fast_kinematic_simulator_amd import ObstacleConfig, build_complete_environment, transform34
    from fast_kinematic_simulator_amd.robots import rotation_from_axis_angle

    res = 0.04
    obs = [ObstacleConfig(1, transform34([0.6, 0.6, 0.5], rotation_from_axis_angle([0, 0, 1], 0.3)), [0.2, 0.1, 0.15]),
           ObstacleConfig(2, transform34([1.1, 0.4, 0.9]), [0.08, 0.3, 0.1])]
    n = (40, 36, 44)
    env = build_complete_environment(obs, res, origin=transform34([0.0, 0.0, 0.0]), num_cells=n)
    sdf = env.sdf.reshape(n)
    filled = sdf < 0
    assert 0.01 < filled.mean() < 0.2
    to_filled = ndimage.distance_transform_edt(~filled)
    to_free = ndimage.distance_transform_edt(filled)
    ref = (to_filled * res - to_free * res).astype(np.float32)
    assert np.array_equal(sdf, ref)


def test_environment_builder_auto_bounds_and_normals(fks_lib):
    """Auto-sized grid (SEB.cpp:128-149: 3-cell border) and the surface-normal CSR:
    every filled cell holds >= 1 unit normal; cube faces carry the exact face normal."""
    from fast_kinematic_simulator_amd import ObstacleConfig, build_complete_environment, transform34

    res = 0.05
    env = build_complete_environment([ObstacleConfig(1, transform34([0.0, 0.0, 0.0]), [0.2, 0.2, 0.2])], res)
    o = np.asarray(env.geometry.origin).reshape(3, 4)
    assert np.allclose(o[:, :3], np.eye(3))
    # samples start at -(extent - res/2) (SEB.cpp:37); origin = min - res/2 - 3 res (SEB.cpp:130-136)
    assert np.allclose(o[:, 3], -(0.2 - 0.5 * res) - 0.5 * res - 3 * res)
    off = env.normal_offsets
    counts = np.diff(off)
    filled = env.sdf < 0
    assert np.all(counts[filled] >= 1)
    ent = env.normal_entries.reshape(-1, 6)
    norms = np.linalg.norm(ent[:, 3:], axis=1)
    # SafeNormal leaves a zero SDF gradient (the centre of a symmetric solid) as zero
    assert np.all(np.isclose(norms, 1.0) | (norms == 0.0))
    assert np.mean(norms == 0.0) < 0.05
    # the +x face samples sit at x = 0.2 (SEB.cpp:296, xidx = x_cells-1); their cell holds
    # the +x normal with entry direction -x
    p = np.array([[0.2 + 0.25 * res, 0.0, 0.0]])
    g = (p - o[:, 3]) / res
    i, j, k = np.trunc(g[0]).astype(int)
    nc = env.geometry.num_cells
    c = (i * nc[1] + j) * nc[2] + k
    cell = ent[off[c]:off[c + 1]]
    assert any(np.allclose(e[3:], [1, 0, 0]) and np.allclose(e[:3], [-1, 0, 0]) for e in cell)
