"""Simulator environment: collision map geometry, signed distance field and the
surface-normal grid, the three inputs ``SimpleParticleContactSimulator`` copies
at construction (SPCS:379-381, 420).

:func:`build_complete_environment` mirrors
``simulator_environment_builder::BuildCompleteEnvironment`` (SEB.cpp:470-476);
the work happens in C++ (``fks_env_build`` in fks_env_builder.cpp).
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass
from typing import Optional, Sequence

import numpy as np

from . import _capi


@dataclass
class ObstacleConfig:
    """simulator_environment_builder::OBSTACLE_CONFIG: pose (3x4), half extents, id > 0."""

    object_id: int
    pose: np.ndarray
    extents: Sequence[float]


@dataclass
class GridGeometry:
    origin: np.ndarray  # 3x4 row-major (12)
    resolution: float
    num_cells: tuple

    def to_c(self) -> _capi.GridGeometry:
        g = _capi.GridGeometry()
        g.origin[:] = [float(v) for v in np.asarray(self.origin).reshape(12)]
        g.resolution = float(self.resolution)
        g.num_cells[:] = [int(v) for v in self.num_cells]
        return g


class SimulatorEnvironment:
    """Host copy of (collision map geometry, SDF, surface normals CSR)."""

    def __init__(self, geometry: GridGeometry, sdf: np.ndarray, normal_offsets: np.ndarray, normal_entries: np.ndarray,
                 oob_value: float = np.inf, occupancy: Optional[np.ndarray] = None):
        self.geometry = geometry
        self.sdf = np.ascontiguousarray(sdf, dtype=np.float32)
        self.normal_offsets = np.ascontiguousarray(normal_offsets, dtype=np.uint32)
        self.normal_entries = np.ascontiguousarray(normal_entries, dtype=np.float64)
        self.oob_value = float(oob_value)
        self.occupancy = occupancy
        self.frame = "uncertainty_planning_simulator"  # TaggedObjectCollisionMapGrid::GetFrame (SPCS:519; SEB.cpp:148 names it)

    @property
    def resolution(self) -> float:
        return self.geometry.resolution

    def to_c(self):
        env = _capi.Environment()
        g = self.geometry.to_c()
        env.collision_map = g
        env.sdf = g
        env.normals = g
        env.sdf_values = _capi.as_ptr(self.sdf, ctypes.c_float)
        env.sdf_oob_value = self.oob_value
        env.normal_offsets = _capi.as_ptr(self.normal_offsets, ctypes.c_uint32)
        env.normal_entries = _capi.as_ptr(self.normal_entries, ctypes.c_double) if self.normal_entries.size else None
        return env, [self.sdf, self.normal_offsets, self.normal_entries]

    def nearest(self, points: np.ndarray) -> np.ndarray:
        """SignedDistanceField::GetImmutable (nearest cell, truncating index) for (n,3)
        world points with an identity-rotation origin; out of bounds -> oob value."""
        o = np.asarray(self.geometry.origin).reshape(3, 4)
        g = (np.asarray(points, dtype=np.float64)[:, :3] - o[:, 3]) @ o[:, :3]
        idx = np.trunc(g * (1.0 / self.geometry.resolution)).astype(np.int64)
        n = np.array(self.geometry.num_cells)
        ok = np.all((idx >= 0) & (idx < n), axis=1)
        out = np.full(len(points), self.oob_value, dtype=np.float64)
        lin = (idx[ok, 0] * n[1] + idx[ok, 1]) * n[2] + idx[ok, 2]
        out[ok] = self.sdf[lin]
        return out


def _obstacle_array(obstacles):
    arr = (_capi.Obstacle * max(1, len(obstacles)))()
    for i, ob in enumerate(obstacles):
        arr[i].pose[:] = [float(v) for v in np.asarray(ob.pose).reshape(12)]
        arr[i].extents[:] = [float(v) for v in ob.extents]
        arr[i].object_id = int(ob.object_id)
    return arr


class DeviceEnvironment:
    """An environment built on a HIP device and kept there (fks_env_build_device):
    a simulator made from it copies the SDF and normal CSR device to device.
    ``download()`` gives the host copy (the same bytes as build_complete_environment)."""

    def __init__(self, handle, device: int, stats: dict):
        self._lib = _capi.lib()
        self._handle = handle
        self.device = int(device)
        self.stats = stats
        g = _capi.GridGeometry()
        _capi.check(self._lib.fks_device_env_geometry(handle, ctypes.byref(g)), None, "fks_device_env_geometry")
        self.geometry = GridGeometry(np.array(g.origin[:]), g.resolution, tuple(g.num_cells[:]))
        self.frame = "uncertainty_planning_simulator"
        self._host = None

    @property
    def handle(self):
        return self._handle

    @property
    def resolution(self) -> float:
        return self.geometry.resolution

    def download(self) -> SimulatorEnvironment:
        if self._host is None:
            L = self._lib
            h = ctypes.c_void_p()
            _capi.check(L.fks_device_env_download(self._handle, ctypes.byref(h)), None, "fks_device_env_download")
            self._host = _host_environment(h)
        return self._host

    def close(self):
        if getattr(self, "_handle", None):
            self._lib.fks_device_env_free(self._handle)
            self._handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def build_device_environment(obstacles: Sequence[ObstacleConfig], resolution: float, origin=None, num_cells=None,
                             device: int = 0) -> DeviceEnvironment:
    """BuildCompleteEnvironment on HIP device `device`, result kept in device memory."""
    L = _capi.lib()
    arr = _obstacle_array(obstacles)
    o_ptr = n_ptr = None
    if origin is not None and num_cells is not None:
        o_arr = np.ascontiguousarray(np.asarray(origin, dtype=np.float64).reshape(12))
        n_arr = np.ascontiguousarray(np.asarray(num_cells, dtype=np.int64))
        o_ptr = _capi.as_ptr(o_arr, ctypes.c_double)
        n_ptr = _capi.as_ptr(n_arr, ctypes.c_int64)
    handle = ctypes.c_void_p()
    bs = _capi.EnvBuildStats()
    st = L.fks_env_build_device(arr, len(obstacles), float(resolution), o_ptr, n_ptr, int(device), ctypes.byref(handle),
                                ctypes.byref(bs))
    _capi.check(st, None, "fks_env_build_device")
    return DeviceEnvironment(handle, device, bs.as_dict())


def _host_environment(handle) -> SimulatorEnvironment:
    """Copy a host fks_env_handle into a SimulatorEnvironment and free the handle."""
    L = _capi.lib()
    try:
        view = _capi.Environment()
        _capi.check(L.fks_env_view(handle, ctypes.byref(view)), None, "fks_env_view")
        geom = GridGeometry(np.array(view.sdf.origin[:]), view.sdf.resolution, tuple(view.sdf.num_cells[:]))
        ncells = int(np.prod(geom.num_cells))
        sdf = np.ctypeslib.as_array(view.sdf_values, shape=(ncells,)).copy()
        offsets = np.ctypeslib.as_array(view.normal_offsets, shape=(ncells + 1,)).copy()
        nent = int(offsets[-1])
        entries = np.ctypeslib.as_array(view.normal_entries, shape=(6 * nent,)).copy() if nent else np.zeros(0)
        oob = float(view.sdf_oob_value)
        occupancy = _env_occupancy(handle, ncells)
    finally:
        L.fks_env_free(handle)
    return SimulatorEnvironment(geom, sdf, offsets, entries, oob, occupancy)


def build_complete_environment(obstacles: Sequence[ObstacleConfig], resolution: float, origin=None,
                               num_cells=None, device: Optional[int] = None, stats: Optional[dict] = None,
                               resident: bool = False):
    """BuildCompleteEnvironment(obstacles, resolution) (SEB.cpp:470-476).  With
    `origin` (3x4) and `num_cells` the grid is that fixed box (e.g. 256^3).
    device=None builds on the host (fks_env_build); device=g builds on HIP device g
    (fks_env_build_gpu, the same bytes).  `stats`, if given, receives the GPU
    build's sizes and timings.  resident=True (with a device) keeps the result on the
    device and returns a DeviceEnvironment."""
    if resident:
        denv = build_device_environment(obstacles, resolution, origin, num_cells, 0 if device is None else device)
        if stats is not None:
            stats.update(denv.stats)
        return denv
    L = _capi.lib()
    arr = _obstacle_array(obstacles)
    handle = ctypes.c_void_p()
    o_ptr = None
    n_ptr = None
    if origin is not None and num_cells is not None:
        o_arr = np.ascontiguousarray(np.asarray(origin, dtype=np.float64).reshape(12))
        n_arr = np.ascontiguousarray(np.asarray(num_cells, dtype=np.int64))
        o_ptr = _capi.as_ptr(o_arr, ctypes.c_double)
        n_ptr = _capi.as_ptr(n_arr, ctypes.c_int64)
    if device is None:
        st = L.fks_env_build(arr, len(obstacles), float(resolution), o_ptr, n_ptr, ctypes.byref(handle))
        _capi.check(st, None, "fks_env_build")
    else:
        bs = _capi.EnvBuildStats()
        st = L.fks_env_build_gpu(arr, len(obstacles), float(resolution), o_ptr, n_ptr, int(device), ctypes.byref(handle),
                                 ctypes.byref(bs))
        _capi.check(st, None, "fks_env_build_gpu")
        if stats is not None:
            stats.update(bs.as_dict())
    return _host_environment(handle)


def _env_occupancy(handle, ncells):
    """The collision grid of a built environment (fks_env_occupancy)."""
    L = _capi.lib()
    out = np.zeros(ncells, dtype=np.uint8)
    _capi.check(L.fks_env_occupancy(handle, _capi.as_ptr(out, ctypes.c_uint8), ncells), None, "fks_env_occupancy")
    return out
