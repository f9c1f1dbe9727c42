"""Robot descriptions for the particle simulator.

Host-side mirror of the reference's robot models (the ``immutable_robot`` that
``ForwardSimulateRobots`` clones per particle, SPCS:788/826):

* :func:`make_linked_robot`  -> ``tnuva_robot_models::TnuvaLinkedRobot`` (TNUVA:415-615)
* :func:`make_se2_robot`     -> ``tnuva_robot_models::TnuvaSE2Robot``    (TNUVA:26-199)
* :func:`make_se3_robot`     -> ``tnuva_robot_models::TnuvaSE3Robot``    (TNUVA:201-413)

Each returns a :class:`RobotDescription` that flattens into the C struct
``fks_robot_desc`` (include/fks_capi.h).
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass, field
from typing import List, Optional, Sequence, Tuple

import numpy as np

from . import _capi

IDENTITY34 = np.array([1.0, 0, 0, 0, 0, 1.0, 0, 0, 0, 0, 1.0, 0])


@dataclass
class ControllerConfig:
    """TnuvaLinkedRobot::LINKED_ROBOT_CONFIG (TNUVA:420-457)."""

    kp: float = 0.0
    ki: float = 0.0
    kd: float = 0.0
    integral_clamp: float = 0.0
    velocity_limit: float = 0.0
    acceleration_limit: float = 0.0
    max_sensor_noise: float = 0.0
    max_actuator_proportional_noise: float = 0.0
    max_actuator_minimum_noise: float = 0.0

    def to_c(self) -> _capi.DofController:
        return _capi.DofController(
            self.kp, self.ki, self.kd, self.integral_clamp, self.velocity_limit, self.acceleration_limit,
            self.max_sensor_noise, self.max_actuator_proportional_noise, self.max_actuator_minimum_noise,
        )


@dataclass
class SampledActuatorModel:
    """JointUncertaintySampleModel (UNC:123) for a SampledUncertainVelocityActuator:
    bins[k] = (lower, upper) of commanded velocity with `samples[k]` velocity errors
    (every bin the same number of samples, as DownsampleBin makes them, UNC:125-138)."""

    bounds: np.ndarray   # (num_bins, 2)
    samples: np.ndarray  # (num_bins, bin_elements)

    def to_c(self):
        b = np.ascontiguousarray(self.bounds, dtype=np.float64).reshape(-1, 2)
        smp = np.ascontiguousarray(self.samples, dtype=np.float64).reshape(b.shape[0], -1)
        return _capi.SampledActuator(b.shape[0], smp.shape[1], _capi.as_ptr(b, ctypes.c_double),
                                     _capi.as_ptr(smp, ctypes.c_double)), [b, smp]


def make_sampled_actuator_model(data, actuator_limit: float, num_bins: int, bin_elements: int,
                                seed: int = 0) -> SampledActuatorModel:
    """LoadModel (UNC:156-221) on (commanded velocity, velocity error) pairs -- a CSV
    path or an (n, 2) array.  Bins split [-limit, limit] into num_bins equal steps, the
    outer two open to -inf / +inf; each pair goes to the first bin holding its command
    (GetMatchingBin, UNC:140-154); each bin is resampled with replacement to
    bin_elements entries (DownsampleBin, UNC:125-138: the reference seeds from
    std::random_device, here from `seed`)."""
    if isinstance(data, str):
        data = np.loadtxt(data, delimiter=",", dtype=np.float64, ndmin=2)
    data = np.asarray(data, dtype=np.float64).reshape(-1, 2)
    bin_size = (actuator_limit * 2.0) / float(num_bins)
    bounds = []
    previous_bin_upper = -actuator_limit
    for idx in range(num_bins):
        lower = -np.inf if idx == 0 else previous_bin_upper
        upper = np.inf if idx >= num_bins - 1 else previous_bin_upper + bin_size
        previous_bin_upper = upper
        bounds.append((lower, upper))
    contents = [[] for _ in range(num_bins)]
    for commanded, error in data:
        for k, (lo, hi) in enumerate(bounds):
            if lo <= commanded <= hi:
                contents[k].append(error)
                break
        else:
            raise ValueError(f"Value {commanded} is not in any bin")
    rng = np.random.default_rng(seed)
    samples = np.zeros((num_bins, bin_elements))
    for k, items in enumerate(contents):
        if not items:
            raise ValueError(f"bin {k} has no data to downsample")
        samples[k] = np.asarray(items)[rng.integers(0, len(items), size=bin_elements)]
    return SampledActuatorModel(np.array(bounds, dtype=np.float64), samples)


@dataclass
class Joint:
    """simple_linked_robot_model::RobotJoint: parent/child link, fixed origin
    (parent link frame -> joint frame, 3x4 row-major), axis, type, limits."""

    parent: int
    child: int
    type: int
    origin: np.ndarray = field(default_factory=lambda: IDENTITY34.copy())
    axis: Tuple[float, float, float] = (0.0, 0.0, 1.0)
    lower: float = -np.pi
    upper: float = np.pi


def transform34(translation=(0.0, 0.0, 0.0), rotation=None) -> np.ndarray:
    """3x4 row-major [R | t]."""
    R = np.eye(3) if rotation is None else np.asarray(rotation, dtype=np.float64).reshape(3, 3)
    T = np.zeros((3, 4))
    T[:, :3] = R
    T[:, 3] = translation
    return T.reshape(12)


def rotation_from_axis_angle(axis, angle) -> np.ndarray:
    axis = np.asarray(axis, dtype=np.float64)
    axis = axis / np.linalg.norm(axis)
    K = np.array([[0, -axis[2], axis[1]], [axis[2], 0, -axis[0]], [-axis[1], axis[0], 0]])
    return np.eye(3) + np.sin(angle) * K + (1 - np.cos(angle)) * (K @ K)


@dataclass
class RobotDescription:
    robot_type: int
    num_links: int
    joints: List[Joint]
    geometry_link: List[int]
    geometry_points: List[np.ndarray]  # (n, 4) x, y, z, w per geometry
    allowed_pairs: List[Tuple[int, int]]
    controllers: List[ControllerConfig]
    distance_weights: List[float]
    base_transform: np.ndarray = field(default_factory=lambda: IDENTITY34.copy())
    name: str = "robot"
    # per dof: None (truncated-normal actuator) or a SampledUncertainVelocityActuator model
    sampled_actuators: Optional[List[Optional[SampledActuatorModel]]] = None

    @property
    def num_dofs(self) -> int:
        if self.robot_type == _capi.ROBOT_SE2:
            return 3
        if self.robot_type == _capi.ROBOT_SE3:
            return 6
        return sum(1 for j in self.joints if j.type != _capi.JOINT_FIXED)

    @property
    def config_width(self) -> int:
        if self.robot_type == _capi.ROBOT_SE2:
            return 3
        if self.robot_type == _capi.ROBOT_SE3:
            return 12
        return self.num_dofs

    @property
    def num_points(self) -> int:
        return int(sum(len(p) for p in self.geometry_points))

    @property
    def points(self) -> np.ndarray:
        return np.ascontiguousarray(np.concatenate(self.geometry_points, axis=0), dtype=np.float64)

    def dof_limits(self) -> Tuple[np.ndarray, np.ndarray]:
        lo = [j.lower for j in self.joints if j.type != _capi.JOINT_FIXED]
        hi = [j.upper for j in self.joints if j.type != _capi.JOINT_FIXED]
        return np.array(lo), np.array(hi)

    def to_c(self):
        """Return (fks_robot_desc, keepalive).  Keep `keepalive` referenced while the
        struct is in use."""
        keep = []
        desc = _capi.RobotDesc()
        desc.robot_type = self.robot_type
        desc.num_links = self.num_links
        desc.num_joints = len(self.joints)
        desc.num_geometries = len(self.geometry_points)
        desc.num_dofs = self.num_dofs
        desc.num_allowed_pairs = len(self.allowed_pairs)
        desc.base_transform[:] = [float(v) for v in np.asarray(self.base_transform).reshape(12)]
        if self.joints:
            jarr = (_capi.JointDesc * len(self.joints))()
            for i, j in enumerate(self.joints):
                jarr[i].parent_link = j.parent
                jarr[i].child_link = j.child
                jarr[i].type = j.type
                jarr[i].origin[:] = [float(v) for v in np.asarray(j.origin).reshape(12)]
                jarr[i].axis[:] = [float(v) for v in j.axis]
                jarr[i].limit_lower = float(j.lower)
                jarr[i].limit_upper = float(j.upper)
            keep.append(jarr)
            desc.joints = ctypes.cast(jarr, ctypes.POINTER(_capi.JointDesc))
        glink = np.ascontiguousarray(self.geometry_link, dtype=np.int32)
        offsets = np.zeros(len(self.geometry_points) + 1, dtype=np.uint32)
        offsets[1:] = np.cumsum([len(p) for p in self.geometry_points])
        pts = self.points
        pairs = np.ascontiguousarray(np.array(self.allowed_pairs, dtype=np.int32).reshape(-1))
        ctrl = (_capi.DofController * len(self.controllers))(*[c.to_c() for c in self.controllers])
        weights = np.ascontiguousarray(self.distance_weights, dtype=np.float64)
        keep += [glink, offsets, pts, pairs, ctrl, weights]
        desc.geometry_link = _capi.as_ptr(glink, ctypes.c_int32)
        desc.geometry_point_offset = _capi.as_ptr(offsets, ctypes.c_uint32)
        desc.points = _capi.as_ptr(pts, ctypes.c_double)
        desc.allowed_pairs = _capi.as_ptr(pairs, ctypes.c_int32) if len(pairs) else None
        desc.controllers = ctypes.cast(ctrl, ctypes.POINTER(_capi.DofController))
        desc.distance_weights = _capi.as_ptr(weights, ctypes.c_double)
        if self.sampled_actuators is not None:
            if len(self.sampled_actuators) != self.num_dofs:
                raise ValueError("sampled_actuators needs one entry (model or None) per dof")
            sarr = (_capi.SampledActuator * self.num_dofs)()
            for k, m in enumerate(self.sampled_actuators):
                if m is not None:
                    sarr[k], k_keep = m.to_c()
                    keep += k_keep
            keep.append(sarr)
            desc.sampled_actuators = ctypes.cast(sarr, ctypes.POINTER(_capi.SampledActuator))
        return desc, keep


def _points4(points) -> np.ndarray:
    p = np.asarray(points, dtype=np.float64)
    if p.shape[1] == 3:
        p = np.concatenate([p, np.ones((len(p), 1))], axis=1)
    return np.ascontiguousarray(p)


def make_se2_robot(points, translation: ControllerConfig, rotation: ControllerConfig,
                   position_distance_weight=1.0, rotation_distance_weight=1.0, name="se2") -> RobotDescription:
    """TnuvaSE2Robot(initial, weights, link_name, geometry, SE2_ROBOT_CONFIG) (TNUVA:109-132):
    x and y use the translational gains, theta the r_* gains."""
    return RobotDescription(
        robot_type=_capi.ROBOT_SE2, num_links=1, joints=[], geometry_link=[0], geometry_points=[_points4(points)],
        allowed_pairs=[], controllers=[translation, translation, rotation],
        distance_weights=[position_distance_weight, rotation_distance_weight], name=name,
    )


def make_se3_robot(points, translation: ControllerConfig, rotation: ControllerConfig,
                   position_distance_weight=1.0, rotation_distance_weight=1.0, name="se3") -> RobotDescription:
    """TnuvaSE3Robot (TNUVA:293-325): x, y, z translational gains; rx, ry, rz rotational."""
    return RobotDescription(
        robot_type=_capi.ROBOT_SE3, num_links=1, joints=[], geometry_link=[0], geometry_points=[_points4(points)],
        allowed_pairs=[], controllers=[translation] * 3 + [rotation] * 3,
        distance_weights=[position_distance_weight, rotation_distance_weight], name=name,
    )


def make_linked_robot(base_transform, num_links: int, joints: Sequence[Joint],
                      link_geometries: Sequence[Tuple[int, np.ndarray]], allowed_self_collisions: Sequence[Tuple[int, int]],
                      joint_configs: Sequence[ControllerConfig], joint_distance_weights: Optional[Sequence[float]] = None,
                      name="linked") -> RobotDescription:
    """TnuvaLinkedRobot(base, links, joints, initial, weights, link_geometries,
    allowed_self_collisions, joint_configs) (TNUVA:486-517).  Throws ValueError when
    the joint-config count differs from the active-joint count (TNUVA:515)."""
    active = sum(1 for j in joints if j.type != _capi.JOINT_FIXED)
    if len(joint_configs) != active:
        raise ValueError("Number of joint configs must match number of active joints")
    weights = list(joint_distance_weights) if joint_distance_weights is not None else [1.0] * active
    return RobotDescription(
        robot_type=_capi.ROBOT_LINKED, num_links=num_links, joints=list(joints),
        geometry_link=[g[0] for g in link_geometries], geometry_points=[_points4(g[1]) for g in link_geometries],
        allowed_pairs=list(allowed_self_collisions), controllers=list(joint_configs), distance_weights=weights,
        base_transform=np.asarray(base_transform, dtype=np.float64).reshape(12), name=name,
    )


def se3_pose(translation=(0.0, 0.0, 0.0), rotation=None) -> np.ndarray:
    """SE(3) configuration (12 doubles, 3x4 row-major)."""
    return transform34(translation, rotation)


class RobotController:
    """One robot stepped by hand through the TnuvaRobot control interface (TNUVA:15-23), on
    the host with the simulation kernels' arithmetic (fks_robot_control_action /
    fks_robot_apply_control_input): the robot's configuration and its controllers' state
    (per dof the error integral, then per dof the last error; ResetPosition zeroes them,
    TNUVA:139-150, 332-336, 524-536)."""

    def __init__(self, robot: RobotDescription, position):
        self.robot = robot
        self.position = np.ascontiguousarray(position, dtype=np.float64).reshape(robot.config_width).copy()
        self.controller_state = np.zeros(2 * robot.num_dofs)

    def reset_position(self, position):
        self.reset_controllers()
        self.position = np.ascontiguousarray(position, dtype=np.float64).reshape(self.robot.config_width).copy()
        return self.position

    def reset_controllers(self):
        self.controller_state[:] = 0.0

    def generate_control_action(self, target, controller_interval: float) -> np.ndarray:
        """GenerateControlAction(target, controller_interval) (TNUVA:179-198, 384-412, 598-614)."""
        desc, keep = self.robot.to_c()
        t = np.ascontiguousarray(target, dtype=np.float64).reshape(self.robot.config_width)
        u = np.zeros(self.robot.num_dofs)
        _capi.check(_capi.lib().fks_robot_control_action(ctypes.byref(desc), _capi.as_ptr(self.position, ctypes.c_double),
                                                         _capi.as_ptr(t, ctypes.c_double), float(controller_interval),
                                                         _capi.as_ptr(self.controller_state, ctypes.c_double),
                                                         _capi.as_ptr(u, ctypes.c_double)))
        del keep
        return u

    def apply_control_input(self, control_input, unit_noise=None) -> np.ndarray:
        """ApplyControlInput(u) (TNUVA:152-163, 348-364, 538-566); with unit_noise (one
        TN(0, 0.5) sample on [-1, 1] per dof) ApplyControlInput(u, rng) (UNC:77-90)."""
        desc, keep = self.robot.to_c()
        u = np.ascontiguousarray(control_input, dtype=np.float64).reshape(self.robot.num_dofs)
        n = None if unit_noise is None else np.ascontiguousarray(unit_noise, dtype=np.float64).reshape(self.robot.num_dofs)
        out = np.zeros(self.robot.config_width)
        _capi.check(_capi.lib().fks_robot_apply_control_input(ctypes.byref(desc), _capi.as_ptr(self.position, ctypes.c_double),
                                                              _capi.as_ptr(u, ctypes.c_double),
                                                              _capi.as_ptr(n, ctypes.c_double) if n is not None else None,
                                                              _capi.as_ptr(out, ctypes.c_double)))
        del keep
        self.position = out
        return out
