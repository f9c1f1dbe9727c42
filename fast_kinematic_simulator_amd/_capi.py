"""ctypes binding of the C-ABI declared in include/fks_capi.h.

The shared library ``libfks_hip.so`` (HIP kernels for gfx950 + host C-ABI) is
built in-tree by :func:`fast_kinematic_simulator_amd.build.build_library`.  There
is no CPU fallback: if the library is missing, :func:`lib` raises.
"""
from __future__ import annotations

import ctypes
import os
from ctypes import POINTER, c_char_p, c_double, c_float, c_int32, c_int64, c_uint8, c_uint32, c_uint64, c_void_p

LIB_NAME = "libfks_hip.so"
LIB_PATH = os.environ.get("FKS_LIB_PATH") or os.path.join(os.path.dirname(os.path.abspath(__file__)), LIB_NAME)

FKS_OK = 0
STATUS_NAMES = {
    0: "FKS_OK",
    1: "FKS_ERR_INVALID_ARGUMENT",
    2: "FKS_ERR_HIP",
    3: "FKS_ERR_NO_ROBOT",
    4: "FKS_ERR_OUT_OF_MEMORY",
    5: "FKS_ERR_UNSUPPORTED",
    6: "FKS_ERR_NO_DEVICE",
}

ROBOT_LINKED, ROBOT_SE2, ROBOT_SE3 = 0, 1, 2
JOINT_FIXED, JOINT_REVOLUTE, JOINT_CONTINUOUS, JOINT_PRISMATIC = 0, 1, 2, 4
KIN_LINK_TRANSFORMS, KIN_POINTS, KIN_APPLY_CONTROL_INPUT = 0, 1, 2
OK, ERR_INVALID_ARGUMENT, ERR_HIP, ERR_NO_ROBOT, ERR_OUT_OF_MEMORY, ERR_UNSUPPORTED, ERR_NO_DEVICE = 0, 1, 2, 3, 4, 5, 6

NUM_PHASES = 16
PHASE_NAMES = ["particle", "control", "step_setup", "micro_input", "micro_fk", "env_check", "self_check", "corrections",
               "solve", "resolve_apply", "output", "env_rounds_skipped", "env_rounds_evaluated", "corr_rounds_skipped",
               "corr_rounds_evaluated", "wave_residency"]
PHASE_COUNTS = {"env_rounds_skipped", "env_rounds_evaluated", "corr_rounds_skipped", "corr_rounds_evaluated", "wave_residency"}

PARTICLE_ERR_MICROSTEP_MOTION = 0x1
PARTICLE_ERR_NORMAL_OOB = 0x2
PARTICLE_ERR_ZERO_DIRECTION = 0x4
PARTICLE_ERR_RNG_EXHAUSTED = 0x8
PARTICLE_ERR_SELF_CAPACITY = 0x10
PARTICLE_ERR_KEY_RANGE = 0x20
PARTICLE_ERR_MICROSTEP_CAP = 0x40
PARTICLE_ERR_SELF_SINGULAR = 0x80
PARTICLE_ERR_NO_NOISE_BIN = 0x100


class SolverParams(ctypes.Structure):
    _fields_ = [
        ("forward_simulation_time", c_double),
        ("simulation_shortcut_distance", c_double),
        ("environment_collision_check_tolerance", c_double),
        ("resolve_correction_step_scaling_decay_rate", c_double),
        ("resolve_correction_initial_step_size", c_double),
        ("resolve_correction_min_step_scaling", c_double),
        ("max_resolver_iterations", c_uint32),
        ("resolve_correction_step_scaling_decay_iterations", c_uint32),
        ("failed_resolves_end_motion", c_uint32),
        ("reserved", c_uint32),
    ]


class GridGeometry(ctypes.Structure):
    _fields_ = [("origin", c_double * 12), ("resolution", c_double), ("num_cells", c_int64 * 3)]


class Environment(ctypes.Structure):
    _fields_ = [
        ("collision_map", GridGeometry),
        ("sdf", GridGeometry),
        ("sdf_values", POINTER(c_float)),
        ("sdf_oob_value", c_float),
        ("reserved", c_uint32),
        ("normals", GridGeometry),
        ("normal_offsets", POINTER(c_uint32)),
        ("normal_entries", POINTER(c_double)),
    ]


class DofController(ctypes.Structure):
    _fields_ = [
        ("kp", c_double),
        ("ki", c_double),
        ("kd", c_double),
        ("integral_clamp", c_double),
        ("velocity_limit", c_double),
        ("acceleration_limit", c_double),
        ("max_sensor_noise", c_double),
        ("max_actuator_proportional_noise", c_double),
        ("max_actuator_minimum_noise", c_double),
    ]


class JointDesc(ctypes.Structure):
    _fields_ = [
        ("parent_link", c_int32),
        ("child_link", c_int32),
        ("type", c_int32),
        ("reserved", c_int32),
        ("origin", c_double * 12),
        ("axis", c_double * 3),
        ("limit_lower", c_double),
        ("limit_upper", c_double),
    ]


class SampledActuator(ctypes.Structure):
    """fks_sampled_actuator: SampledUncertainVelocityActuator bins (UNC:123-281)."""
    _fields_ = [
        ("num_bins", c_uint32),
        ("bin_elements", c_uint32),
        ("bin_bounds", POINTER(c_double)),
        ("bin_samples", POINTER(c_double)),
    ]


class RobotDesc(ctypes.Structure):
    _fields_ = [
        ("robot_type", c_int32),
        ("num_links", c_int32),
        ("num_joints", c_int32),
        ("num_geometries", c_int32),
        ("num_dofs", c_int32),
        ("num_allowed_pairs", c_int32),
        ("base_transform", c_double * 12),
        ("joints", POINTER(JointDesc)),
        ("geometry_link", POINTER(c_int32)),
        ("geometry_point_offset", POINTER(c_uint32)),
        ("points", POINTER(c_double)),
        ("allowed_pairs", POINTER(c_int32)),
        ("controllers", POINTER(DofController)),
        ("distance_weights", POINTER(c_double)),
        ("sampled_actuators", POINTER(SampledActuator)),
    ]


class Statistics(ctypes.Structure):
    _fields_ = [
        ("successful_resolves", c_uint64),
        ("unsuccessful_resolves", c_uint64),
        ("free_resolves", c_uint64),
        ("collision_resolves", c_uint64),
        ("fallback_resolves", c_uint64),
        ("unsuccessful_env_collision_resolves", c_uint64),
        ("unsuccessful_self_collision_resolves", c_uint64),
        ("recovered_unsuccessful_resolves", c_uint64),
    ]

    def as_dict(self):
        return {name: float(getattr(self, name)) for name, _ in self._fields_}


class CallCounters(ctypes.Structure):
    _fields_ = [
        ("particles", c_uint64),
        ("controller_steps", c_uint64),
        ("microsteps", c_uint64),
        ("resolver_iterations", c_uint64),
        ("sdf_bytes", c_uint64),
        ("error_particles", c_uint64),
        ("kernel_ms", c_double),
        ("call_ms", c_double),
        ("calls", c_uint64),
        ("least_squares_rows", c_uint64),
        ("self_collision_checks", c_uint64),
        ("self_corrected_points", c_uint64),
        ("reserved0", c_uint64),  # ABI 4: proven_free_microsteps
    ]

    def as_dict(self):
        return {name: getattr(self, name) for name, _ in self._fields_}


SPECIALIZE_OFF, SPECIALIZE_ON, SPECIALIZE_NO_PROOFS = 0, 1, 2  # fks_specialization_mode (ABI 9)


class SpecializationInfo(ctypes.Structure):
    """fks_specialization_info (ABI 9)"""
    _fields_ = [
        ("enabled", c_int32),
        ("active", c_int32),
        ("from_cache", c_int32),
        ("pending", c_int32),
        ("compile_seconds", c_double),
        ("launches", c_uint64),
        ("shape", ctypes.c_char * 64),
        ("failed", c_int32),
        ("reserved", c_int32),
        ("message", ctypes.c_char * 512),
    ]

    def as_dict(self):
        d = {name: getattr(self, name) for name, _ in self._fields_ if name not in ("reserved", "shape", "message")}
        d["shape"] = self.shape.decode()
        d["message"] = self.message.decode(errors="replace")
        return d


class LaunchInfo(ctypes.Structure):
    """fks_launch_info (ABI 10)"""
    _fields_ = [
        ("resident_waves", c_uint32),
        ("waves_per_group", c_uint32),
        ("lds_bytes_per_group", c_uint64),
        ("small_batch_resident_waves", c_uint32),
        ("standard_layout_resident_waves", c_uint32),
        ("fk_pair", c_int32),
        ("lean", c_int32),
        ("last_kernel", c_int32),
        ("last_check_kernel", c_int32),
        ("cooperative_resident_particles", c_uint32),
        ("cooperative_waves_per_particle", c_uint32),
    ]

    def as_dict(self):
        d = {name: getattr(self, name) for name, _ in self._fields_ if name != "reserved"}
        d["last_kernel"] = KERNEL_KINDS.get(d["last_kernel"], d["last_kernel"])
        d["last_check_kernel"] = KERNEL_KINDS.get(d["last_check_kernel"], d["last_check_kernel"])
        return d


KERNEL_KINDS = {0: "none", 1: "throughput", 2: "small_batch", 3: "shaped", 4: "traced", 5: "individual", 6: "cooperative",
                7: "shaped_small_batch"}


class Trace(ctypes.Structure):
    """fks_trace: ForwardSimulationStepTrace flattened per particle (include/fks_capi.h)."""
    _fields_ = [
        ("step_capacity", c_uint32),
        ("config_capacity", c_uint32),
        ("step_inputs", POINTER(c_double)),
        ("step_microsteps", POINTER(c_uint32)),
        ("configs", POINTER(c_double)),
        ("config_tags", POINTER(c_uint32)),
        ("num_steps", POINTER(c_uint32)),
        ("num_configs", POINTER(c_uint32)),
    ]


class Obstacle(ctypes.Structure):
    _fields_ = [("pose", c_double * 12), ("extents", c_double * 3), ("object_id", c_uint32), ("reserved", c_uint32)]


class EnvBuildStats(ctypes.Structure):
    _fields_ = [("cells", c_uint64), ("obstacle_samples", c_uint64), ("normal_entries", c_uint64), ("gpu_ms", c_double),
                ("total_ms", c_double)]

    def as_dict(self):
        return {name: getattr(self, name) for name, _ in self._fields_}


# (name, restype, argtypes) of every symbol include/fks_capi.h declares
PROTOTYPES = [
    ("fks_abi_version", c_int32, []),
    ("fks_status_string", c_char_p, [c_int32]),
    ("fks_default_solver_params", c_int32, [POINTER(SolverParams)]),
    ("fks_create", c_int32, [POINTER(Environment), POINTER(SolverParams), c_double, c_uint64, c_int32, c_int32, POINTER(c_void_p)]),
    ("fks_destroy", None, [c_void_p]),
    ("fks_get_last_error", c_char_p, [c_void_p]),
    ("fks_set_robot", c_int32, [c_void_p, POINTER(RobotDesc)]),
    ("fks_config_width", c_int32, [c_void_p]),
    (
        "fks_forward_simulate",
        c_int32,
        [c_void_p, POINTER(c_double), c_uint64, POINTER(c_double), c_uint64, c_int32, POINTER(c_double), POINTER(c_uint8),
         POINTER(c_uint32), POINTER(c_uint32), POINTER(c_uint32)],
    ),
    (
        "fks_reverse_simulate",
        c_int32,
        [c_void_p, POINTER(c_double), c_uint64, POINTER(c_double), c_uint64, c_int32, POINTER(c_double), POINTER(c_uint8),
         POINTER(c_uint32), POINTER(c_uint32), POINTER(c_uint32)],
    ),
    (
        "fks_forward_simulate_mutable",
        c_int32,
        [c_void_p, POINTER(c_double), c_uint64, POINTER(c_double), c_uint64, c_int32, POINTER(c_double), POINTER(c_double),
         POINTER(c_uint8), POINTER(c_uint32), POINTER(c_uint32), POINTER(c_uint32)],
    ),
    (
        "fks_forward_simulate_device",
        c_int32,
        [c_void_p, c_void_p, c_uint64, c_void_p, c_uint64, c_uint64, c_int32, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
         c_void_p, c_int32],
    ),
    (
        "fks_forward_simulate_traced",
        c_int32,
        [c_void_p, POINTER(c_double), c_uint64, POINTER(c_double), c_uint64, c_int32, POINTER(c_double), POINTER(c_uint8),
         POINTER(c_uint32), POINTER(c_uint32), POINTER(c_uint32), POINTER(Trace)],
    ),
    (
        "fks_forward_simulate_traced_mutable",
        c_int32,
        [c_void_p, POINTER(c_double), c_uint64, POINTER(c_double), c_uint64, c_int32, POINTER(c_double), POINTER(c_double),
         POINTER(c_uint8), POINTER(c_uint32), POINTER(c_uint32), POINTER(c_uint32), POINTER(Trace)],
    ),
    ("fks_check_config_collision", c_int32,
     [c_void_p, POINTER(c_double), c_uint64, c_double, POINTER(c_uint8), POINTER(c_uint32)]),
    ("fks_check_config_collision_device", c_int32,
     [c_void_p, c_void_p, c_uint64, c_double, c_void_p, c_void_p, c_void_p, c_int32]),
    ("fks_get_last_check_counters", c_int32, [c_void_p, POINTER(CallCounters)]),
    ("fks_kinematics", c_int32, [c_void_p, c_int32, POINTER(c_double), c_uint64, POINTER(c_double), POINTER(c_double)]),
    ("fks_robot_sizes", c_int32, [c_void_p, POINTER(c_int32), POINTER(c_int32), POINTER(c_int32), POINTER(c_int32)]),
    ("fks_set_call_index", c_int32, [c_void_p, c_uint64]),
    ("fks_get_call_index", c_uint64, [c_void_p]),
    ("fks_get_statistics", c_int32, [c_void_p, POINTER(Statistics)]),
    ("fks_reset_statistics", c_int32, [c_void_p]),
    ("fks_set_statistics", c_int32, [c_void_p, POINTER(Statistics)]),
    ("fks_reset_generators", c_int32, [c_void_p, c_uint64]),
    ("fks_get_debug_level", c_int32, [c_void_p]),
    ("fks_set_debug_level", c_int32, [c_void_p, c_int32]),
    ("fks_get_last_call_counters", c_int32, [c_void_p, POINTER(CallCounters)]),
    ("fks_get_total_counters", c_int32, [c_void_p, POINTER(CallCounters)]),
    ("fks_reset_total_counters", c_int32, [c_void_p]),
    ("fks_set_total_counters", c_int32, [c_void_p, POINTER(CallCounters)]),
    ("fks_robot_control_action", c_int32, [POINTER(RobotDesc), POINTER(c_double), POINTER(c_double), c_double, POINTER(c_double),
                                           POINTER(c_double)]),
    ("fks_robot_apply_control_input", c_int32, [POINTER(RobotDesc), POINTER(c_double), POINTER(c_double), POINTER(c_double),
                                                POINTER(c_double)]),
    ("fks_get_phase_cycles", c_int32, [c_void_p, c_int32, POINTER(c_uint64)]),
    ("fks_get_launch_geometry", c_int32, [c_void_p, POINTER(c_uint32), POINTER(c_uint64)]),
    ("fks_set_segment_steps", c_int32, [c_void_p, c_uint32]),
    ("fks_set_segment_policy", c_int32, [c_void_p, c_uint32, c_uint32]),
    ("fks_set_segment_heavy_relative", c_int32, [c_void_p, c_uint32]),
    ("fks_set_small_batch_kernel", c_int32, [c_void_p, c_int32]),
    ("fks_set_cooperative_waves", c_int32, [c_void_p, c_int32]),
    ("fks_set_specialization", c_int32, [c_void_p, c_int32]),
    ("fks_get_launch_info", c_int32, [c_void_p, POINTER(LaunchInfo)]),
    ("fks_get_specialization", c_int32, [c_void_p, POINTER(SpecializationInfo)]),
    ("fks_set_individual_jacobians", c_int32, [c_void_p, c_int32]),
    ("fks_env_build", c_int32, [POINTER(Obstacle), c_int32, c_double, POINTER(c_double), POINTER(c_int64), POINTER(c_void_p)]),
    ("fks_env_build_gpu", c_int32, [POINTER(Obstacle), c_int32, c_double, POINTER(c_double), POINTER(c_int64), c_int32,
                                    POINTER(c_void_p), POINTER(EnvBuildStats)]),
    ("fks_env_build_device", c_int32, [POINTER(Obstacle), c_int32, c_double, POINTER(c_double), POINTER(c_int64), c_int32,
                                       POINTER(c_void_p), POINTER(EnvBuildStats)]),
    ("fks_device_env_download", c_int32, [c_void_p, POINTER(c_void_p)]),
    ("fks_device_env_geometry", c_int32, [c_void_p, POINTER(GridGeometry)]),
    ("fks_device_env_free", None, [c_void_p]),
    ("fks_create_from_device_env", c_int32, [c_void_p, POINTER(SolverParams), c_double, c_uint64, c_int32, POINTER(c_void_p)]),
    ("fks_env_view", c_int32, [c_void_p, POINTER(Environment)]),
    ("fks_env_occupancy", c_int32, [c_void_p, POINTER(c_uint8), c_uint64]),
    ("fks_env_discretize_obstacle", c_int32, [POINTER(Obstacle), c_double, POINTER(c_double), c_uint64, POINTER(c_uint64)]),
    ("fks_env_build_normals", c_int32, [POINTER(Obstacle), c_int32, POINTER(GridGeometry), POINTER(c_float), POINTER(c_void_p)]),
    ("fks_env_cell_objects", c_int32, [c_void_p, POINTER(c_uint32), c_uint64]),
    ("fks_env_free", None, [c_void_p]),
    ("fks_selftest_math", c_int32, [c_int32, c_uint64, POINTER(c_uint64)]),
    ("fks_shard_bounds", c_int32, [c_uint64, c_int32, c_int32, POINTER(c_uint64), POINTER(c_uint64)]),
    ("fks_create_multi", c_int32, [POINTER(Environment), POINTER(SolverParams), c_double, c_uint64, c_int32, POINTER(c_int32), c_int32,
                                   POINTER(c_void_p)]),
    ("fks_destroy_multi", None, [c_void_p]),
    ("fks_multi_get_last_error", c_char_p, [c_void_p]),
    ("fks_multi_num_devices", c_int32, [c_void_p]),
    ("fks_multi_device_context", c_void_p, [c_void_p, c_int32]),
    ("fks_multi_set_robot", c_int32, [c_void_p, POINTER(RobotDesc)]),
    (
        "fks_multi_forward_simulate",
        c_int32,
        [c_void_p, POINTER(c_double), c_uint64, POINTER(c_double), c_uint64, c_int32, POINTER(c_double), POINTER(c_uint8),
         POINTER(c_uint32), POINTER(c_uint32), POINTER(c_uint32)],
    ),
    ("fks_multi_get_statistics", c_int32, [c_void_p, POINTER(Statistics)]),
    ("fks_multi_reset_statistics", c_int32, [c_void_p]),
    ("fks_multi_get_last_call_counters", c_int32, [c_void_p, POINTER(CallCounters)]),
    ("fks_multi_set_call_index", c_int32, [c_void_p, c_uint64]),
    ("fks_multi_set_active_devices", c_int32, [c_void_p, c_int32]),
    ("fks_multi_active_devices", c_int32, [c_void_p]),
    ("fks_multi_check_config_collision", c_int32, [c_void_p, POINTER(c_double), c_uint64, c_double, POINTER(c_uint8), POINTER(c_uint32)]),
    ("fks_device_count", c_int32, []),
]

_LIB = None


class FksError(RuntimeError):
    def __init__(self, status, message=""):
        self.status = status
        super().__init__(f"{STATUS_NAMES.get(status, status)}: {message}")


def lib():
    """Load libfks_hip.so (in-tree).  Raises if it has not been built."""
    global _LIB
    if _LIB is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(
                f"{LIB_PATH} is missing: build it with fast_kinematic_simulator_amd.build.build_library() "
                "(there is no CPU fallback for the HIP path)"
            )
        handle = ctypes.CDLL(LIB_PATH)
        # tools/variant_bench.py compares older builds, which may lack newer entries: only
        # there (FKS_VARIANT_LIB=1) are missing symbols skipped; otherwise they fail the load
        variant = os.environ.get("FKS_VARIANT_LIB") == "1"
        missing = [name for name, _, _ in PROTOTYPES if not hasattr(handle, name)]
        if missing and not variant:
            raise RuntimeError(f"{LIB_PATH} lacks {len(missing)} symbol(s) of include/fks_capi.h: {', '.join(missing)} "
                               "(a stale build? rebuild with fast_kinematic_simulator_amd/build.py)")
        for name, restype, argtypes in PROTOTYPES:
            if not hasattr(handle, name):
                continue
            fn = getattr(handle, name)
            fn.restype = restype
            fn.argtypes = argtypes
        _LIB = handle
    return _LIB


def check(status, ctx=None, what=""):
    if status != FKS_OK:
        msg = what
        if ctx:
            err = lib().fks_get_last_error(ctx)
            if err:
                msg = f"{what}: {err.decode()}"
        raise FksError(status, msg)


def as_ptr(array, ctype):
    return array.ctypes.data_as(POINTER(ctype))
