"""Host-side mirror of the reference simulator interface over the C-ABI.

Mirrors ``simple_particle_contact_simulator::SimpleParticleContactSimulator``
(SPCS:371-1999) as seen through ``uncertainty_planning_core``'s
``SimulatorInterface`` and the ``fast_kinematic_simulator`` factories
(FKS.hpp:11-22, FKS.cpp:4-71).  Batch calls run on the GPU through
``libfks_hip.so``; there is no CPU fallback.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass, fields
from typing import Callable, List, Optional, Sequence

import numpy as np

from . import _capi
from .environment import DeviceEnvironment, SimulatorEnvironment
from .robots import RobotDescription
from .trace import ForwardSimulationStepTrace, TraceBuffers


@dataclass
class SimulatorSolverParameters:
    """SimulatorSolverParameters with the defaults of SPCS:357-368."""

    forward_simulation_time: float = 1.0
    simulation_shortcut_distance: float = 0.0
    environment_collision_check_tolerance: float = 0.001
    resolve_correction_step_scaling_decay_rate: float = 0.5
    resolve_correction_initial_step_size: float = 1.0
    resolve_correction_min_step_scaling: float = 0.03125
    max_resolver_iterations: int = 25
    resolve_correction_step_scaling_decay_iterations: int = 5
    failed_resolves_end_motion: bool = True

    def to_c(self) -> _capi.SolverParams:
        p = _capi.SolverParams()
        for f in fields(self):
            v = getattr(self, f.name)
            setattr(p, f.name, int(v) if isinstance(v, (bool, int)) and not isinstance(v, float) else v)
        return p


def get_default_solver_parameters() -> SimulatorSolverParameters:
    """fast_kinematic_simulator::GetDefaultSolverParameters (FKS.hpp:13-16)."""
    return SimulatorSolverParameters()


@dataclass
class SimulationResult:
    """simple_simulator_interface::SimulationResult(reached, target, collided, true) (SPCS:918)."""

    result_config: np.ndarray
    target_config: np.ndarray
    did_contact: bool
    outcome_is_valid: bool = True
    microsteps: int = 0
    resolver_iterations: int = 0
    error_flags: int = 0


class HipParticleContactSimulator:
    """SimpleParticleContactSimulator on one MI355X.  The stacked-Jacobian resolver
    is always used, as the factories hard-wire (FKS.cpp:22,45,68)."""

    def __init__(self, environment: SimulatorEnvironment, solver_config: SimulatorSolverParameters,
                 simulation_controller_frequency: float, prng_seed: int, debug_level: int = 0, device: int = 0):
        self._lib = _capi.lib()
        self.environment = environment
        self.solver_config = solver_config
        self.simulation_controller_frequency = float(simulation_controller_frequency)
        self.prng_seed = int(prng_seed)
        params = solver_config.to_c()
        ctx = ctypes.c_void_p()
        if isinstance(environment, DeviceEnvironment):
            # device-resident GPU build: SDF + normal CSR copied device to device (fks_create_from_device_env)
            self._env_keep = None
            st = self._lib.fks_create_from_device_env(environment.handle, ctypes.byref(params),
                                                      self.simulation_controller_frequency,
                                                      ctypes.c_uint64(self.prng_seed & 0xFFFFFFFFFFFFFFFF), int(debug_level),
                                                      ctypes.byref(ctx))
            _capi.check(st, None, "fks_create_from_device_env")
        else:
            env_c, self._env_keep = environment.to_c()
            st = self._lib.fks_create(ctypes.byref(env_c), ctypes.byref(params), self.simulation_controller_frequency,
                                      ctypes.c_uint64(self.prng_seed & 0xFFFFFFFFFFFFFFFF), int(debug_level), int(device),
                                      ctypes.byref(ctx))
            _capi.check(st, None, "fks_create")
        self._ctx = ctx
        self._robot_key = None
        self._robot = None

    # ---- lifetime ----
    def close(self):
        if getattr(self, "_ctx", None):
            self._lib.fks_destroy(self._ctx)
            self._ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---- reference interface ----
    def get_debug_level(self) -> int:
        return int(self._lib.fks_get_debug_level(self._ctx))

    def set_debug_level(self, debug_level: int) -> int:
        return int(self._lib.fks_set_debug_level(self._ctx, int(debug_level)))

    def get_statistics(self) -> dict:
        s = _capi.Statistics()
        _capi.check(self._lib.fks_get_statistics(self._ctx, ctypes.byref(s)), self._ctx, "fks_get_statistics")
        return s.as_dict()

    def reset_statistics(self):
        _capi.check(self._lib.fks_reset_statistics(self._ctx), self._ctx, "fks_reset_statistics")

    def reset_generators(self, prng_seed: int):
        _capi.check(self._lib.fks_reset_generators(self._ctx, ctypes.c_uint64(int(prng_seed))), self._ctx, "reset")

    def set_call_index(self, call_index: int):
        _capi.check(self._lib.fks_set_call_index(self._ctx, ctypes.c_uint64(int(call_index))), self._ctx, "call index")

    def get_call_index(self) -> int:
        return int(self._lib.fks_get_call_index(self._ctx))

    def last_call_counters(self) -> dict:
        c = _capi.CallCounters()
        _capi.check(self._lib.fks_get_last_call_counters(self._ctx, ctypes.byref(c)), self._ctx, "counters")
        return c.as_dict()

    def total_counters(self) -> dict:
        c = _capi.CallCounters()
        _capi.check(self._lib.fks_get_total_counters(self._ctx, ctypes.byref(c)), self._ctx, "counters")
        return c.as_dict()

    def reset_total_counters(self):
        _capi.check(self._lib.fks_reset_total_counters(self._ctx), self._ctx, "counters")

    def phase_cycles(self, total: bool = True) -> dict:
        """Shader-clock cycles per kernel phase (fks_get_phase_cycles), summed over waves."""
        arr = (ctypes.c_uint64 * _capi.NUM_PHASES)()
        _capi.check(self._lib.fks_get_phase_cycles(self._ctx, 1 if total else 0, arr), self._ctx, "phase cycles")
        return {name: int(arr[i]) for i, name in enumerate(_capi.PHASE_NAMES)}

    def set_segment_steps(self, controller_steps: int = 0):
        """Controller steps per scheduling segment of a batch (fks_set_segment_steps;
        0 = automatic).  Results do not depend on it."""
        _capi.check(self._lib.fks_set_segment_steps(self._ctx, int(controller_steps)), self._ctx, "segment steps")

    def set_segment_policy(self, heavy_resolver_per_step: int = 2, heavy_priority: int = 2):
        """Scheduling policy of segmented batches (fks_set_segment_policy): contact-heavy
        segments keep their wave and raise its issue priority.  Results do not depend on it."""
        _capi.check(self._lib.fks_set_segment_policy(self._ctx, int(heavy_resolver_per_step), int(heavy_priority)), self._ctx,
                    "segment policy")

    def set_segment_heavy_relative(self, times_mean: int = 3):
        """A heavy segment must also exceed times_mean x the batch's running mean resolver
        iterations per segment (fks_set_segment_heavy_relative; 0 = off).  Results do not depend on it."""
        _capi.check(self._lib.fks_set_segment_heavy_relative(self._ctx, int(times_mean)), self._ctx, "segment heavy relative")

    def set_small_batch_kernel(self, enabled: bool = True):
        """Batches that fit the low-occupancy instantiation's resident waves run it
        (fks_set_small_batch_kernel; default on).  Results do not depend on it."""
        _capi.check(self._lib.fks_set_small_batch_kernel(self._ctx, 1 if enabled else 0), self._ctx, "small batch kernel")

    def set_cooperative_waves(self, enabled: bool = True):
        """Batches of at most launch_info()["cooperative_resident_particles"] particles run one
        particle per workgroup, its environment checks and correction passes shared over the
        workgroup's waves (fks_set_cooperative_waves; default off: slower on the measured
        workloads).  Results do not depend on it."""
        _capi.check(self._lib.fks_set_cooperative_waves(self._ctx, 1 if enabled else 0), self._ctx, "cooperative waves")

    def set_specialization(self, enabled=True):
        """Run the plain throughput simulation of this robot (and of every robot set later) on a
        kernel compiled at run time for its shape (fks_set_specialization: hiprtc, cached per
        process and on disk).  On by default, built at the first call that runs it; enabling
        it builds the current robot's kernel now.  Results do not depend on it; raises FksError
        with the compiler log when the current robot's kernel cannot be built (the calls then
        keep the generic kernel, and specialization()["failed"] says so).  enabled may also be
        an fks_specialization_mode: _capi.SPECIALIZE_NO_PROOFS builds the validation kernel with
        every skip proof compiled out (same results, slower)."""
        mode = int(enabled) if not isinstance(enabled, bool) else (_capi.SPECIALIZE_ON if enabled else _capi.SPECIALIZE_OFF)
        _capi.check(self._lib.fks_set_specialization(self._ctx, mode), self._ctx, "specialization")

    def launch_info(self) -> dict:
        """fks_get_launch_info: the layout fks_set_robot chose and the kernel of the last call."""
        info = _capi.LaunchInfo()
        _capi.check(self._lib.fks_get_launch_info(self._ctx, ctypes.byref(info)), self._ctx, "launch info")
        return info.as_dict()

    def specialization(self) -> dict:
        """fks_get_specialization: enabled (mode), active, pending, from_cache, compile_seconds, launches,
        shape, failed, message"""
        info = _capi.SpecializationInfo()
        _capi.check(self._lib.fks_get_specialization(self._ctx, ctypes.byref(info)), self._ctx, "specialization")
        return info.as_dict()

    def set_individual_jacobians(self, simulate_with_individual_jacobians: bool):
        """The simulate_with_individual_jacobians constructor flag of the reference class
        (SPCS:420-423, 1629): True selects ComputeResolverCorrectionStepIndividualJacobians
        (SPCS:1966-1988) instead of the stacked solve the factories hard-wire (FKS.cpp:22)."""
        _capi.check(self._lib.fks_set_individual_jacobians(self._ctx, 1 if simulate_with_individual_jacobians else 0), self._ctx,
                    "individual jacobians")

    def launch_geometry(self) -> dict:
        """Resident waves of the persistent simulation grid and LDS bytes per workgroup
        (fks_get_launch_geometry) for the robot set last."""
        waves, lds = ctypes.c_uint32(0), ctypes.c_uint64(0)
        _capi.check(self._lib.fks_get_launch_geometry(self._ctx, ctypes.byref(waves), ctypes.byref(lds)), self._ctx,
                    "launch geometry")
        return {"resident_waves": int(waves.value), "lds_bytes_per_group": int(lds.value)}

    def set_robot(self, robot: RobotDescription):
        key = id(robot)
        if self._robot_key == key and self._robot is robot:
            return
        desc, keep = robot.to_c()
        _capi.check(self._lib.fks_set_robot(self._ctx, ctypes.byref(desc)), self._ctx, "fks_set_robot")
        del keep
        self._robot_key = key
        self._robot = robot

    def forward_simulate_arrays(self, robot: RobotDescription, start_positions, target_positions, allow_contacts: bool,
                                reverse: bool = False) -> dict:
        """Batch call with numpy arrays: starts (n, W), targets (1 or n, W)."""
        self.set_robot(robot)
        W = robot.config_width
        starts = np.ascontiguousarray(np.asarray(start_positions, dtype=np.float64).reshape(-1, W))
        targets = np.ascontiguousarray(np.asarray(target_positions, dtype=np.float64).reshape(-1, W))
        n = starts.shape[0]
        if n > 0 and targets.shape[0] not in (1, n):
            raise ValueError("target_positions must hold 1 or len(start_positions) configurations (SPCS:792)")
        out = np.zeros((n, W), dtype=np.float64)
        collided = np.zeros(n, dtype=np.uint8)
        micro = np.zeros(n, dtype=np.uint32)
        resolver = np.zeros(n, dtype=np.uint32)
        errors = np.zeros(n, dtype=np.uint32)
        fn = self._lib.fks_reverse_simulate if reverse else self._lib.fks_forward_simulate
        st = fn(self._ctx, _capi.as_ptr(starts, ctypes.c_double), n, _capi.as_ptr(targets, ctypes.c_double),
                targets.shape[0], 1 if allow_contacts else 0, _capi.as_ptr(out, ctypes.c_double),
                _capi.as_ptr(collided, ctypes.c_uint8), _capi.as_ptr(micro, ctypes.c_uint32),
                _capi.as_ptr(resolver, ctypes.c_uint32), _capi.as_ptr(errors, ctypes.c_uint32))
        _capi.check(st, self._ctx, "fks_forward_simulate")
        return {"positions": out, "collided": collided.astype(bool), "microsteps": micro, "resolver_iterations": resolver,
                "error_flags": errors}

    def forward_simulate_mutable_arrays(self, robot: RobotDescription, start_positions, target_positions, allow_contacts: bool,
                                        controller_state) -> dict:
        """ForwardSimulateMutableRobot (SPCS:843-919) for a batch (fks_forward_simulate_mutable):
        each particle starts with its own PID state; controller_state is an (n, 2D) float64
        array (per dof the error integral, then per dof the last error), updated in place."""
        self.set_robot(robot)
        W, D = robot.config_width, robot.num_dofs
        starts = np.ascontiguousarray(np.asarray(start_positions, dtype=np.float64).reshape(-1, W))
        targets = np.ascontiguousarray(np.asarray(target_positions, dtype=np.float64).reshape(-1, W))
        n = starts.shape[0]
        if not (isinstance(controller_state, np.ndarray) and controller_state.dtype == np.float64 and
                controller_state.flags["C_CONTIGUOUS"] and controller_state.shape == (n, 2 * D)):
            raise ValueError("controller_state must be a C-contiguous float64 array of shape (n, 2 * num_dofs)")
        out = np.zeros((n, W), dtype=np.float64)
        collided = np.zeros(n, dtype=np.uint8)
        micro = np.zeros(n, dtype=np.uint32)
        resolver = np.zeros(n, dtype=np.uint32)
        errors = np.zeros(n, dtype=np.uint32)
        st = self._lib.fks_forward_simulate_mutable(
            self._ctx, _capi.as_ptr(starts, ctypes.c_double), n, _capi.as_ptr(targets, ctypes.c_double), targets.shape[0],
            1 if allow_contacts else 0, _capi.as_ptr(controller_state, ctypes.c_double), _capi.as_ptr(out, ctypes.c_double),
            _capi.as_ptr(collided, ctypes.c_uint8), _capi.as_ptr(micro, ctypes.c_uint32), _capi.as_ptr(resolver, ctypes.c_uint32),
            _capi.as_ptr(errors, ctypes.c_uint32))
        _capi.check(st, self._ctx, "fks_forward_simulate_mutable")
        return {"positions": out, "collided": collided.astype(bool), "microsteps": micro, "resolver_iterations": resolver,
                "error_flags": errors}

    def forward_simulate_robots(self, immutable_robot: RobotDescription, start_positions: Sequence, target_positions: Sequence,
                                allow_contacts: bool, display_fn: Optional[Callable] = None) -> List[SimulationResult]:
        """ForwardSimulateRobots (SPCS:788-804).  display_fn is accepted for interface
        parity; the batch path never draws (SPCS:801 passes enable_tracing=false)."""
        return self._results(immutable_robot, start_positions, target_positions, allow_contacts, reverse=False)

    def reverse_simulate_robots(self, immutable_robot: RobotDescription, start_positions: Sequence, target_positions: Sequence,
                                allow_contacts: bool, display_fn: Optional[Callable] = None) -> List[SimulationResult]:
        """ReverseSimulateRobots (SPCS:806-822) == forward simulation (SPCS:838-841)."""
        return self._results(immutable_robot, start_positions, target_positions, allow_contacts, reverse=True)

    def forward_simulate_robot(self, immutable_robot: RobotDescription, start_position, target_position,
                               allow_contacts: bool) -> SimulationResult:
        """ForwardSimulateRobot (SPCS:824-829) as a batch of one."""
        return self._results(immutable_robot, [start_position], [target_position], allow_contacts, reverse=False)[0]

    def forward_simulate_traced(self, robot: RobotDescription, start_positions, target_positions, allow_contacts: bool,
                                step_capacity: Optional[int] = None, config_capacity: int = 4096):
        """ForwardSimulateRobot with ``enable_tracing = true`` (SPCS:824-829) for a batch:
        returns (result dict as forward_simulate_arrays, TraceBuffers).  Capacities are
        per particle; records past them are counted, not stored (``truncated``)."""
        self.set_robot(robot)
        W, D = robot.config_width, robot.num_dofs
        starts = np.ascontiguousarray(np.asarray(start_positions, dtype=np.float64).reshape(-1, W))
        targets = np.ascontiguousarray(np.asarray(target_positions, dtype=np.float64).reshape(-1, W))
        n = starts.shape[0]
        if n > 0 and targets.shape[0] not in (1, n):
            raise ValueError("target_positions must hold 1 or len(start_positions) configurations (SPCS:792)")
        if step_capacity is None:
            step_capacity = max(1, int(self.solver_config.forward_simulation_time * self.simulation_controller_frequency))
        buf = TraceBuffers(n, D, W, step_capacity, config_capacity)
        tr = buf.to_c()
        out = np.zeros((n, W), dtype=np.float64)
        collided = np.zeros(n, dtype=np.uint8)
        micro = np.zeros(n, dtype=np.uint32)
        resolver = np.zeros(n, dtype=np.uint32)
        errors = np.zeros(n, dtype=np.uint32)
        st = self._lib.fks_forward_simulate_traced(
            self._ctx, _capi.as_ptr(starts, ctypes.c_double), n, _capi.as_ptr(targets, ctypes.c_double), targets.shape[0],
            1 if allow_contacts else 0, _capi.as_ptr(out, ctypes.c_double), _capi.as_ptr(collided, ctypes.c_uint8),
            _capi.as_ptr(micro, ctypes.c_uint32), _capi.as_ptr(resolver, ctypes.c_uint32), _capi.as_ptr(errors, ctypes.c_uint32),
            ctypes.byref(tr))
        _capi.check(st, self._ctx, "fks_forward_simulate_traced")
        return ({"positions": out, "collided": collided.astype(bool), "microsteps": micro, "resolver_iterations": resolver,
                 "error_flags": errors}, buf)

    def forward_simulate_robot_traced(self, immutable_robot: RobotDescription, start_position, target_position,
                                      allow_contacts: bool):
        """ForwardSimulateRobot(..., trace, enable_tracing=true, ...) (SPCS:824-829):
        (SimulationResult, ForwardSimulationStepTrace)."""
        W = immutable_robot.config_width
        r, buf = self.forward_simulate_traced(immutable_robot, [start_position], [target_position], allow_contacts)
        tgt = np.asarray(target_position, dtype=np.float64).reshape(W)
        res = SimulationResult(r["positions"][0].copy(), tgt.copy(), bool(r["collided"][0]), True, int(r["microsteps"][0]),
                               int(r["resolver_iterations"][0]), int(r["error_flags"][0]))
        return res, buf.particle(0)

    def _results(self, robot, starts, targets, allow_contacts, reverse):
        W = robot.config_width
        tarr = np.asarray(targets, dtype=np.float64).reshape(-1, W)
        r = self.forward_simulate_arrays(robot, starts, tarr, allow_contacts, reverse=reverse)
        n = r["positions"].shape[0]
        out = []
        for i in range(n):
            tgt = tarr[i] if tarr.shape[0] == n else tarr[0]
            out.append(SimulationResult(r["positions"][i].copy(), tgt.copy(), bool(r["collided"][i]), True,
                                        int(r["microsteps"][i]), int(r["resolver_iterations"][i]), int(r["error_flags"][i])))
        return out

    def check_config_collisions(self, robot: RobotDescription, configs, inflation_ratio: float = 0.0) -> dict:
        """Batched CheckConfigCollision (SPCS:1398-1416): configs (n, W) -> collided[n]
        (bool) and error_flags[n]."""
        self.set_robot(robot)
        W = robot.config_width
        arr = np.ascontiguousarray(np.asarray(configs, dtype=np.float64).reshape(-1, W))
        n = arr.shape[0]
        collided = np.zeros(n, dtype=np.uint8)
        errors = np.zeros(n, dtype=np.uint32)
        st = self._lib.fks_check_config_collision(self._ctx, _capi.as_ptr(arr, ctypes.c_double), n, float(inflation_ratio),
                                                  _capi.as_ptr(collided, ctypes.c_uint8), _capi.as_ptr(errors, ctypes.c_uint32))
        _capi.check(st, self._ctx, "fks_check_config_collision")
        return {"collided": collided.astype(bool), "error_flags": errors}

    def check_config_collision(self, immutable_robot: RobotDescription, config, inflation_ratio: float) -> bool:
        """CheckConfigCollision (SPCS:1398-1416) for one configuration."""
        return bool(self.check_config_collisions(immutable_robot, [config], inflation_ratio)["collided"][0])

    def check_config_collisions_device(self, robot: RobotDescription, d_configs, n: int, inflation_ratio: float,
                                       d_out_collided, d_out_error_flags=0, stream=0, synchronize=False):
        """fks_check_config_collision_device: device pointers (int) on `stream`."""
        self.set_robot(robot)
        st = self._lib.fks_check_config_collision_device(
            self._ctx, ctypes.c_void_p(d_configs), n, float(inflation_ratio), ctypes.c_void_p(d_out_collided),
            ctypes.c_void_p(d_out_error_flags or None), ctypes.c_void_p(stream or None), 1 if synchronize else 0)
        _capi.check(st, self._ctx, "fks_check_config_collision_device")

    def last_check_counters(self) -> dict:
        c = _capi.CallCounters()
        _capi.check(self._lib.fks_get_last_check_counters(self._ctx, ctypes.byref(c)), self._ctx, "counters")
        return c.as_dict()

    # ---- kinematics helpers of the interface (fks_kinematics) ----
    def _kinematics(self, robot: RobotDescription, mode: int, configs, inputs=None) -> np.ndarray:
        self.set_robot(robot)
        W = robot.config_width
        cfg = np.ascontiguousarray(np.asarray(configs, dtype=np.float64).reshape(-1, W))
        n = cfg.shape[0]
        links, points, dofs = ctypes.c_int32(), ctypes.c_int32(), ctypes.c_int32()
        _capi.check(self._lib.fks_robot_sizes(self._ctx, ctypes.byref(links), ctypes.byref(points), ctypes.byref(dofs), None),
                    self._ctx, "fks_robot_sizes")
        shape = {_capi.KIN_LINK_TRANSFORMS: (n, links.value, 3, 4), _capi.KIN_POINTS: (n, points.value, 3),
                 _capi.KIN_APPLY_CONTROL_INPUT: (n, W)}[mode]
        out = np.zeros(shape, dtype=np.float64)
        u = None
        if mode == _capi.KIN_APPLY_CONTROL_INPUT:
            u = np.ascontiguousarray(np.asarray(inputs, dtype=np.float64).reshape(n, dofs.value))
        st = self._lib.fks_kinematics(self._ctx, mode, _capi.as_ptr(cfg, ctypes.c_double), n,
                                      _capi.as_ptr(u, ctypes.c_double) if u is not None else None,
                                      _capi.as_ptr(out, ctypes.c_double))
        _capi.check(st, self._ctx, "fks_kinematics")
        return out

    def link_transforms(self, robot: RobotDescription, configs) -> np.ndarray:
        """GetLinkTransform of every link after SetPosition: (n, links, 3, 4)."""
        return self._kinematics(robot, _capi.KIN_LINK_TRANSFORMS, configs)

    def world_points(self, robot: RobotDescription, configs) -> np.ndarray:
        """Every link point in the world frame, geometry order: (n, points, 3)."""
        return self._kinematics(robot, _capi.KIN_POINTS, configs)

    def apply_control_input(self, robot: RobotDescription, configs, control_inputs) -> np.ndarray:
        """SetPosition + clean ApplyControlInput (TNUVA:538-566): (n, W)."""
        return self._kinematics(robot, _capi.KIN_APPLY_CONTROL_INPUT, configs, control_inputs)

    def get_frame(self) -> str:
        """GetFrame (SPCS:517-520)."""
        return self.environment.frame

    def get_resolution(self) -> float:
        return float(self.environment.resolution)

    def get_random_generator(self) -> np.random.Generator:
        """GetRandomGenerator (SPCS:473-481) for the caller's own sampling.  The
        simulation's actuation noise does not come from it: that is the counter RNG keyed
        by (seed, call index, particle, step, microstep, dof), DESIGN.md §2.1."""
        if getattr(self, "_host_rng", None) is None:
            self._host_rng = np.random.default_rng(self.prng_seed)
        return self._host_rng

    def get_3d_point_for_config(self, immutable_robot: RobotDescription, config) -> np.ndarray:
        """Get3dPointForConfig (SPCS:776-786): the origin of the last geometry's link."""
        T = self.link_transforms(immutable_robot, [config])[0, immutable_robot.geometry_link[-1]]
        return np.array([T[0, 3], T[1, 3], T[2, 3], 1.0])

    def make_configuration_display_rep(self, immutable_robot: RobotDescription, configuration, color,
                                       starting_index: int, config_marker_ns: str) -> List[dict]:
        """MakeConfigurationDisplayRep for POINTS geometries (SPCS:634-688): one SPHERE_LIST
        marker of every link point, black where the link-frame point is the zero vector."""
        pts = self.world_points(immutable_robot, [configuration])[0]
        res = self.get_resolution()
        m = _marker(config_marker_ns, starting_index, "SPHERE_LIST", self.get_frame(), (res, res, res), color)
        m["points"] = pts.tolist()
        link_pts = immutable_robot.points
        black = [0.0, 0.0, 0.0, 1.0]
        m["colors"] = [black if float(np.linalg.norm(p)) == 0.0 else list(color) for p in link_pts]
        return [m]

    def make_control_input_display_rep(self, immutable_robot: RobotDescription, configuration, control_input, color,
                                       starting_index: int, control_input_marker_ns: str) -> List[dict]:
        """MakeControlInputDisplayRep (SPCS:719-774): a LINE_LIST from every point at
        `configuration` to the same point after the clean control input."""
        after = self.apply_control_input(immutable_robot, [configuration], [control_input])
        pts = self.world_points(immutable_robot, np.concatenate([np.asarray(configuration, dtype=np.float64).reshape(1, -1),
                                                                 after], axis=0))
        res = self.get_resolution() * 0.5
        m = _marker(control_input_marker_ns, starting_index, "LINE_LIST", self.get_frame(), (res, res, res), color)
        m["points"] = np.stack([pts[0], pts[1]], axis=1).reshape(-1, 3).tolist()
        m["colors"] = [list(color)] * (2 * pts.shape[1])
        return [m]

    def make_environment_display_rep(self) -> List[dict]:
        """MakeEnvironmentDisplayRep (SPCS:559-586), reduced to what this repository holds:
        the filled cells of the collision grid ("sim_environment") and the SDF cells
        colored by sign ("sim_environment_sdf").  sdf_tools' connected-component and
        convex-segment exports have no counterpart here."""
        env = self.environment.download() if isinstance(self.environment, DeviceEnvironment) else self.environment
        g = env.geometry
        n = tuple(int(v) for v in g.num_cells)
        o = np.asarray(g.origin, dtype=np.float64).reshape(3, 4)
        idx = np.stack(np.unravel_index(np.arange(int(np.prod(n))), n), axis=1).astype(np.float64)
        centers = (idx + 0.5) * g.resolution @ o[:, :3].T + o[:, 3]
        res = float(g.resolution)
        markers = []
        occ = env.occupancy if env.occupancy is not None else (env.sdf < 0).astype(np.uint8)
        m = _marker("sim_environment", 1, "CUBE_LIST", self.get_frame(), (res, res, res), [1.0, 0.0, 0.0, 1.0])
        m["points"] = centers[occ.astype(bool)].tolist()
        markers.append(m)
        s = _marker("sim_environment_sdf", 1, "CUBE_LIST", self.get_frame(), (res, res, res), [1.0, 1.0, 1.0, 1.0])
        s["points"] = centers.tolist()
        s["colors"] = [[1.0, 0.0, 0.0, 1.0] if v < 0 else [0.0, 0.0, 1.0, 1.0] for v in env.sdf]
        markers.append(s)
        return markers

    def forward_simulate_device(self, robot: RobotDescription, d_starts, n: int, d_targets, num_targets: int,
                                first_particle_id: int, allow_contacts: bool, d_out_positions, d_out_collided=0,
                                d_out_microsteps=0, d_out_resolver_iterations=0, d_out_error_flags=0, stream=0,
                                synchronize=False):
        """fks_forward_simulate_device: every buffer is a device pointer (int), e.g.
        torch_tensor.data_ptr(); `stream` a hipStream_t handle (int)."""
        self.set_robot(robot)
        st = self._lib.fks_forward_simulate_device(
            self._ctx, ctypes.c_void_p(d_starts), n, ctypes.c_void_p(d_targets), num_targets, first_particle_id,
            1 if allow_contacts else 0, ctypes.c_void_p(d_out_positions), ctypes.c_void_p(d_out_collided or None),
            ctypes.c_void_p(d_out_microsteps or None), ctypes.c_void_p(d_out_resolver_iterations or None),
            ctypes.c_void_p(d_out_error_flags or None), ctypes.c_void_p(stream or None), 1 if synchronize else 0)
        _capi.check(st, self._ctx, "fks_forward_simulate_device")


class MultiDeviceSimulator:
    """One process, several MI355X devices (fks_create_multi): every batch is split into
    contiguous particle shards, one per listed device, simulated concurrently with each
    shard's first_particle_id, and gathered into one result (bit-identical to one device).
    Statistics are summed over the devices.  Replaces the reference's OpenMP particle loop
    (SPCS:795) at device granularity; one process per GPU under torch.distributed is the
    other route (sharding.py, bench.py)."""

    def __init__(self, environment: SimulatorEnvironment, solver_config: SimulatorSolverParameters,
                 simulation_controller_frequency: float, prng_seed: int, devices: Sequence[int], debug_level: int = 0):
        self._lib = _capi.lib()
        env_c, self._env_keep = environment.to_c()
        params = solver_config.to_c()
        devs = (ctypes.c_int32 * len(devices))(*[int(d) for d in devices])
        ctx = ctypes.c_void_p()
        st = self._lib.fks_create_multi(ctypes.byref(env_c), ctypes.byref(params), float(simulation_controller_frequency),
                                        ctypes.c_uint64(int(prng_seed) & 0xFFFFFFFFFFFFFFFF), int(debug_level), devs, len(devices),
                                        ctypes.byref(ctx))
        _capi.check(st, None, "fks_create_multi")
        self._ctx = ctx
        self._robot = None

    def close(self):
        if getattr(self, "_ctx", None):
            self._lib.fks_destroy_multi(self._ctx)
            self._ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, st, what):
        if st != _capi.FKS_OK:
            raise _capi.FksError(st, f"{what}: {self._lib.fks_multi_get_last_error(self._ctx).decode()}")

    def num_devices(self) -> int:
        return int(self._lib.fks_multi_num_devices(self._ctx))

    def set_active_devices(self, count: int = 0):
        """Shard the batches that follow over the first `count` listed devices (0 = all;
        fks_multi_set_active_devices).  Results do not depend on it."""
        self._check(self._lib.fks_multi_set_active_devices(self._ctx, int(count)), "fks_multi_set_active_devices")

    def active_devices(self) -> int:
        return int(self._lib.fks_multi_active_devices(self._ctx))

    def device_simulator_specialization(self, shard: int = 0) -> dict:
        """fks_get_specialization of one device's context."""
        info = _capi.SpecializationInfo()
        ctx = self._lib.fks_multi_device_context(self._ctx, int(shard))
        _capi.check(self._lib.fks_get_specialization(ctx, ctypes.byref(info)), ctx, "specialization")
        return info.as_dict()

    def set_robot(self, robot: RobotDescription):
        if self._robot is robot:
            return
        desc, keep = robot.to_c()
        self._check(self._lib.fks_multi_set_robot(self._ctx, ctypes.byref(desc)), "fks_multi_set_robot")
        self._robot = robot

    def set_call_index(self, call_index: int):
        self._check(self._lib.fks_multi_set_call_index(self._ctx, ctypes.c_uint64(int(call_index))), "call index")

    def forward_simulate_arrays(self, robot: RobotDescription, start_positions, target_positions, allow_contacts: bool) -> dict:
        self.set_robot(robot)
        W = robot.config_width
        starts = np.ascontiguousarray(np.asarray(start_positions, dtype=np.float64).reshape(-1, W))
        targets = np.ascontiguousarray(np.asarray(target_positions, dtype=np.float64).reshape(-1, W))
        n = starts.shape[0]
        out = np.zeros((n, W), dtype=np.float64)
        collided = np.zeros(n, dtype=np.uint8)
        micro = np.zeros(n, dtype=np.uint32)
        resolver = np.zeros(n, dtype=np.uint32)
        errors = np.zeros(n, dtype=np.uint32)
        st = self._lib.fks_multi_forward_simulate(
            self._ctx, _capi.as_ptr(starts, ctypes.c_double), n, _capi.as_ptr(targets, ctypes.c_double), targets.shape[0],
            1 if allow_contacts else 0, _capi.as_ptr(out, ctypes.c_double), _capi.as_ptr(collided, ctypes.c_uint8),
            _capi.as_ptr(micro, ctypes.c_uint32), _capi.as_ptr(resolver, ctypes.c_uint32), _capi.as_ptr(errors, ctypes.c_uint32))
        self._check(st, "fks_multi_forward_simulate")
        return {"positions": out, "collided": collided.astype(bool), "microsteps": micro, "resolver_iterations": resolver,
                "error_flags": errors}

    def check_config_collisions(self, robot: RobotDescription, configs, inflation_ratio: float):
        """Batched CheckConfigCollision (SPCS:1398-1416) sharded over the devices:
        (collided bool[n], error bits uint32[n])."""
        self.set_robot(robot)
        W = robot.config_width
        c = np.ascontiguousarray(np.asarray(configs, dtype=np.float64).reshape(-1, W))
        n = c.shape[0]
        collided = np.zeros(n, dtype=np.uint8)
        errors = np.zeros(n, dtype=np.uint32)
        st = self._lib.fks_multi_check_config_collision(self._ctx, _capi.as_ptr(c, ctypes.c_double), n, float(inflation_ratio),
                                                        _capi.as_ptr(collided, ctypes.c_uint8), _capi.as_ptr(errors, ctypes.c_uint32))
        self._check(st, "fks_multi_check_config_collision")
        return collided.astype(bool), errors

    def get_statistics(self) -> dict:
        s = _capi.Statistics()
        self._check(self._lib.fks_multi_get_statistics(self._ctx, ctypes.byref(s)), "statistics")
        return s.as_dict()

    def last_call_counters(self) -> dict:
        c = _capi.CallCounters()
        self._check(self._lib.fks_multi_get_last_call_counters(self._ctx, ctypes.byref(c)), "counters")
        return c.as_dict()


def _marker(ns, marker_id, marker_type, frame, scale, color):
    """A visualization_msgs::Marker as a plain dict (ROS is not part of this repository)."""
    return {"ns": ns, "id": int(marker_id), "type": marker_type, "action": "ADD", "frame_id": frame,
            "frame_locked": False, "scale": [float(v) for v in scale], "color": list(color),
            "pose": {"position": [0.0, 0.0, 0.0], "orientation": [0.0, 0.0, 0.0, 1.0]}, "points": None, "colors": None}


def _make(environment, solver_config, simulation_controller_frequency, prng_seed, debug_level, device=0):
    return HipParticleContactSimulator(environment, solver_config, simulation_controller_frequency, prng_seed, debug_level, device)


def make_se2_simulator(environment, solver_config, simulation_controller_frequency, prng_seed, debug_level=0, device=0):
    """fast_kinematic_simulator::MakeSE2Simulator (FKS.cpp:4-25)."""
    return _make(environment, solver_config, simulation_controller_frequency, prng_seed, debug_level, device)


def make_se3_simulator(environment, solver_config, simulation_controller_frequency, prng_seed, debug_level=0, device=0):
    """fast_kinematic_simulator::MakeSE3Simulator (FKS.cpp:27-48)."""
    return _make(environment, solver_config, simulation_controller_frequency, prng_seed, debug_level, device)


def make_linked_simulator(environment, solver_config, simulation_controller_frequency, prng_seed, debug_level=0, device=0):
    """fast_kinematic_simulator::MakeLinkedSimulator (FKS.cpp:50-71)."""
    return _make(environment, solver_config, simulation_controller_frequency, prng_seed, debug_level, device)
