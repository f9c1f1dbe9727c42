"""GPU environment build: fks_env_build_gpu against the host
builder fks_env_build (which restates SEB.cpp:21-476 with an exact EDT).

CPU: the C-ABI contract without a device (status codes) and the host builder's
own invariants (the SDF sign is the collision grid, the CSR covers every interior
cell).
GPU: every output byte -- grid geometry, collision grid, SDF (float32 bits), CSR
offsets and entries (float64 bits) -- equal to the host build, for the five bench
scenes, an auto-sized grid around rotated obstacles, a non-cubic grid, a grid
without obstacles and one that is entirely filled."""
import ctypes

import numpy as np
import pytest

from fast_kinematic_simulator_amd import _capi
from fast_kinematic_simulator_amd import workloads as W
from fast_kinematic_simulator_amd.environment import ObstacleConfig, build_complete_environment
from fast_kinematic_simulator_amd.robots import transform34


def _rot(axis, angle):
    axis = np.asarray(axis, dtype=np.float64) / np.linalg.norm(axis)
    K = np.array([[0, -axis[2], axis[1]], [axis[2], 0, -axis[0]], [-axis[1], axis[0], 0]])
    return np.eye(3) + np.sin(angle) * K + (1 - np.cos(angle)) * (K @ K)


def _pose(R, t):
    return np.hstack([R, np.asarray(t, dtype=np.float64).reshape(3, 1)]).reshape(12)


def _rotated_scene():
    rng = np.random.default_rng(11)
    obs = []
    for i in range(9):
        R = _rot(rng.normal(size=3), rng.uniform(0, np.pi))
        obs.append(ObstacleConfig(i + 1, _pose(R, rng.uniform(-0.5, 0.5, size=3)), list(rng.uniform(0.04, 0.2, size=3))))
    return obs


EXTRA = {
    "auto_rotated": lambda dev: build_complete_environment(_rotated_scene(), 0.02, device=dev),
    "non_cubic": lambda dev: build_complete_environment(_rotated_scene(), 0.025, origin=transform34((-0.6, -0.9, -0.4)),
                                                        num_cells=(40, 71, 33), device=dev),
    "empty": lambda dev: build_complete_environment([], 0.05, origin=transform34((0.0, 0.0, 0.0)), num_cells=(8, 9, 10),
                                                    device=dev),
    "all_filled": lambda dev: build_complete_environment([ObstacleConfig(1, transform34((0.2, 0.2, 0.2)), [1.0, 1.0, 1.0])], 0.05,
                                                         origin=transform34((0.0, 0.0, 0.0)), num_cells=(8, 8, 8), device=dev),
}


def assert_same_environment(a, b):
    assert np.array_equal(np.asarray(a.geometry.origin), np.asarray(b.geometry.origin))
    assert a.geometry.resolution == b.geometry.resolution
    assert tuple(a.geometry.num_cells) == tuple(b.geometry.num_cells)
    assert np.array_equal(a.occupancy, b.occupancy)
    assert np.array_equal(a.sdf.view(np.uint32), b.sdf.view(np.uint32)), \
        f"{np.count_nonzero(a.sdf.view(np.uint32) != b.sdf.view(np.uint32))} SDF cells differ"
    assert np.array_equal(a.normal_offsets, b.normal_offsets)
    assert np.array_equal(a.normal_entries.view(np.uint64), b.normal_entries.view(np.uint64))


def test_env_build_gpu_without_device_reports_it():
    L = _capi.lib()
    h = ctypes.c_void_p()
    # invalid arguments are rejected before the device is looked up
    assert L.fks_env_build_gpu(None, 0, -1.0, None, None, 0, ctypes.byref(h), None) == _capi.ERR_INVALID_ARGUMENT
    st = L.fks_env_build_gpu(None, 0, 0.05, None, None, 0, ctypes.byref(h), None)
    try:
        import torch

        has_gpu = torch.cuda.is_available()
    except ImportError:
        has_gpu = False
    if not has_gpu:
        assert st == _capi.ERR_NO_DEVICE
    elif st == 0:
        L.fks_env_free(h)


@pytest.mark.parametrize("name", ["auto_rotated", "non_cubic", "empty", "all_filled"])
def test_host_build_invariants(name):
    env = EXTRA[name](None)
    n = int(np.prod(env.geometry.num_cells))
    assert env.occupancy.shape == (n,) and env.sdf.shape == (n,)
    # SDF sign is the collision grid (filled: -distance to free; free: +distance to filled)
    assert np.array_equal(env.sdf < 0, env.occupancy == 1)
    # every interior cell has at least one normal entry (gradient or surface)
    counts = np.diff(env.normal_offsets.astype(np.int64))
    assert np.all(counts[env.occupancy == 1] >= 1) and np.all(counts <= 3)
    assert env.normal_entries.size == 6 * int(env.normal_offsets[-1])


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["cfg1", "cfg2", "cfg3", "cfg4", "cfg5", "auto_rotated", "non_cubic", "empty", "all_filled"])
def test_gpu_env_build_matches_host(fks_lib, name):
    build = W.SCENES[name] if name in W.SCENES else EXTRA[name]
    stats = {}
    if name in W.SCENES:
        host, gpu = build(), build(device=0, stats=stats)
    else:
        host, gpu = build(None), build(0)
    assert_same_environment(gpu, host)
    if stats:
        assert stats["cells"] == int(np.prod(host.geometry.num_cells))
        assert stats["normal_entries"] == int(host.normal_offsets[-1])
        print(f"{name}: {stats['cells']} cells, GPU build {stats['gpu_ms']:.2f} ms (call {stats['total_ms']:.1f} ms)")


def test_device_env_entry_points_without_device():
    L = _capi.lib()
    h = ctypes.c_void_p()
    assert L.fks_env_build_device(None, 0, -1.0, None, None, 0, ctypes.byref(h), None) == _capi.ERR_INVALID_ARGUMENT
    assert L.fks_create_from_device_env(None, None, 100.0, 0, 0, ctypes.byref(h)) == _capi.ERR_INVALID_ARGUMENT
    assert L.fks_device_env_download(None, ctypes.byref(h)) == _capi.ERR_INVALID_ARGUMENT
    L.fks_device_env_free(None)


@pytest.mark.gpu
@pytest.mark.parametrize("name,scale", [("cfg3", 32 / 65536), ("cfg5", 6 / 1048576)])
def test_device_resident_environment_feeds_the_simulator(fks_lib, name, scale):
    """fks_env_build_device + fks_create_from_device_env: the downloaded bytes equal the
    host build and a simulator made from the device copy gives identical results."""
    import time

    from fast_kinematic_simulator_amd import make_linked_simulator

    wl = W.WORKLOADS[name](scale)
    host = wl.environment()
    t0 = time.perf_counter()
    denv = W.SCENES[name](device=0, resident=True)
    a = make_linked_simulator(denv, wl.solver, wl.controller_frequency, wl.seed)
    setup_device = time.perf_counter() - t0
    t0 = time.perf_counter()
    b = make_linked_simulator(host, wl.solver, wl.controller_frequency, wl.seed)
    setup_host_env = time.perf_counter() - t0
    try:
        assert_same_environment(denv.download(), host)
        a.set_call_index(2)
        b.set_call_index(2)
        ra = a.forward_simulate_arrays(wl.robot, wl.starts, wl.targets, True)
        rb = b.forward_simulate_arrays(wl.robot, wl.starts, wl.targets, True)
        for k in ("positions", "collided", "microsteps", "resolver_iterations", "error_flags"):
            assert np.array_equal(ra[k], rb[k]), k
        assert a.last_call_counters()["sdf_bytes"] == b.last_call_counters()["sdf_bytes"]
    finally:
        a.close()
        b.close()
        denv.close()
    print(f"{name}: device build + create {setup_device:.3f}s, create from host arrays {setup_host_env:.3f}s")
