"""Synthetic workloads for the five configurations of BASELINE.json / SURVEY.md §8(d).

Each workload is a robot + environment + particle batch + solver parameters.
Sizes are the BASELINE ones; ``scale`` shrinks the particle count (and nothing
else) for parity tests.  All random choices are seeded.

cfg1  SE(2) 3-DOF planar robot, 64 points, 64^3 grid @ 0.0625 m, 32 particles x 50 steps
cfg2  UR5-style 6-DOF arm, 7 links x 64 points, 128^3 @ 0.02 m, 4096 x 100
cfg3  7-DOF arm (iiwa-like), 8 links x 64 points, 256^3 @ 0.01 m, 65536 x 200   <- headline
cfg4  SE(3) free flyer, 256 points, 256^3 @ 0.01 m, 1M x 100 (8 GPUs)
cfg5  dual-arm 14-DOF (Baxter-like), 17 links x 64 points, 512^3 @ 0.005 m, 1M x 200 (8 GPUs)
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Callable, Dict, List, Optional

import numpy as np

from . import _capi
from .environment import ObstacleConfig, SimulatorEnvironment, build_complete_environment
from .robots import (ControllerConfig, Joint, RobotDescription, make_linked_robot, make_se2_robot, make_se3_robot,
                     rotation_from_axis_angle, se3_pose, transform34)
from .simulator import SimulatorSolverParameters


@dataclass
class Workload:
    name: str
    description: str
    robot: RobotDescription
    env_builder: Callable[[], SimulatorEnvironment]
    starts: np.ndarray
    targets: np.ndarray
    solver: SimulatorSolverParameters
    controller_frequency: float
    seed: int
    allow_contacts: bool = True
    grid_cells: int = 0
    resolution: float = 0.0
    _env: Optional[SimulatorEnvironment] = field(default=None, repr=False)

    @property
    def num_particles(self) -> int:
        return int(self.starts.shape[0])

    @property
    def steps(self) -> int:
        return max(int(self.solver.forward_simulation_time * self.controller_frequency), 1)

    def environment(self) -> SimulatorEnvironment:
        if self._env is None:
            self._env = self.env_builder()
        return self._env


def cylinder_points(length: float, radius: float, n: int = 64, rings: int = 16, z0: float = 0.0) -> np.ndarray:
    """n points on rings around the local z axis from z0 to z0+length."""
    per = n // rings
    pts = []
    for r in range(rings):
        z = z0 + length * (r + 0.5) / rings
        for k in range(per):
            a = 2.0 * np.pi * (k + 0.5 * (r % 2)) / per
            pts.append([radius * np.cos(a), radius * np.sin(a), z, 1.0])
    return np.array(pts, dtype=np.float64)


def box(object_id, center, half, rotation=None) -> ObstacleConfig:
    return ObstacleConfig(object_id, transform34(center, rotation), list(half))


def grid_origin(lo) -> np.ndarray:
    return transform34(lo)


# ---------------------------------------------------------------- cfg1: SE(2)
def cfg1_obstacles() -> List[ObstacleConfig]:
    rng = np.random.default_rng(1)
    obstacles = []
    for i in range(12):
        c = [rng.uniform(0.5, 3.5), rng.uniform(0.5, 3.5), 0.0]
        h = [rng.uniform(0.08, 0.25), rng.uniform(0.08, 0.25), 1.0]
        obstacles.append(box(i + 1, c, h, rotation_from_axis_angle([0, 0, 1], rng.uniform(0, np.pi))))
    return obstacles


def _cfg1_env(device=None, stats=None, resident=False):
    return build_complete_environment(cfg1_obstacles(), 0.0625, origin=grid_origin([0.0, 0.0, -2.0]), num_cells=(64, 64, 64),
                                      device=device, stats=stats, resident=resident)


def _se2_points(x, y, th, pts):
    c, s = np.cos(th), np.sin(th)
    return np.stack([c * pts[:, 0] - s * pts[:, 1] + x, s * pts[:, 0] + c * pts[:, 1] + y, pts[:, 2]], axis=1)


def cfg1(scale: float = 1.0) -> Workload:
    res = 0.0625
    g = np.arange(8) * (res * 0.5) - 3.5 * res * 0.5
    pts = np.array([[x, y, 0.0, 1.0] for x in g for y in g])
    tr = ControllerConfig(kp=1.0, ki=0.1, kd=0.01, integral_clamp=1.0, velocity_limit=0.5,
                          max_actuator_proportional_noise=0.2, max_actuator_minimum_noise=0.05)
    robot = make_se2_robot(pts, tr, tr, name="se2_planar_box")
    env = _cfg1_env()
    rng = np.random.default_rng(2)
    n = max(1, int(round(32 * scale)))
    starts = []
    while len(starts) < n:
        q = np.array([rng.uniform(0.4, 3.6), rng.uniform(0.4, 3.6), rng.uniform(-np.pi, np.pi)])
        if np.all(env.nearest(_se2_points(q[0], q[1], q[2], pts)) > 2 * res):
            starts.append(q)
    target = np.array([[2.0, 2.0, 0.5]])
    solver = SimulatorSolverParameters(forward_simulation_time=1.0)
    wl = Workload("cfg1", "SE(2) 3-DOF planar robot, 64^3 grid, 32 particles x 50 steps", robot, lambda: env,
                  np.array(starts), target, solver, 50.0, 11, True, 64, res)
    wl._env = env
    return wl


# ---------------------------------------------------------------- arms
def _arm_controllers(d, vmax=1.0):
    # the actuator noise floor is min_noise * vmax per applied input (UNC:80-86), i.e. per
    # microstep: keep it at ~10% of a typical microstep joint delta (vmax*dt/M ~ 1e-3 rad)
    return [ControllerConfig(kp=10.0, ki=1.0, kd=0.1, integral_clamp=0.5, velocity_limit=vmax, acceleration_limit=vmax * 10,
                             max_actuator_proportional_noise=0.2, max_actuator_minimum_noise=0.0002) for _ in range(d)]


def serial_arm(segments, axes, radii, base_height, base_radius, limits=np.pi, name="arm",
               base_transform=None) -> RobotDescription:
    """Serial revolute chain: joint i sits at the end of segment i-1 (segment 0 = base),
    link i spans segment i along its local +z."""
    n = len(axes)
    joints = []
    geoms = [(0, cylinder_points(base_height, base_radius, 64, 16))]
    for i in range(n):
        offset = base_height if i == 0 else segments[i - 1]
        joints.append(Joint(parent=i, child=i + 1, type=_capi.JOINT_REVOLUTE, origin=transform34([0, 0, offset]),
                            axis=tuple(axes[i]), lower=-limits, upper=limits))
        geoms.append((i + 1, cylinder_points(segments[i], radii[i], 64, 16, z0=0.0)))
    allowed = [(i, i + 1) for i in range(n)] + [(i, i + 2) for i in range(n - 1)]
    return make_linked_robot(base_transform if base_transform is not None else transform34([0, 0, 0.03]), n + 1, joints, geoms,
                             allowed, _arm_controllers(n), [1.0] * n, name=name)


def _cfg2_env(device=None, stats=None, resident=False):
    obstacles = [box(1, [0.0, 0.0, -0.05], [0.9, 0.9, 0.05]),           # table, top at z = 0
                 box(2, [0.45, 0.25, 0.25], [0.06, 0.06, 0.25]),        # post
                 box(3, [0.35, -0.35, 0.12], [0.10, 0.08, 0.12]),       # block
                 box(4, [-0.3, 0.4, 0.35], [0.05, 0.05, 0.35])]         # pillar
    return build_complete_environment(obstacles, 0.02, origin=grid_origin([-1.28, -1.28, -0.4]), num_cells=(128, 128, 128),
                                      device=device, stats=stats, resident=resident)


def cfg2(scale: float = 1.0) -> Workload:
    segs = [0.43, 0.39, 0.11, 0.09, 0.08, 0.06]
    axes = [[0, 0, 1], [0, 1, 0], [0, 1, 0], [0, 1, 0], [0, 0, 1], [0, 1, 0]]
    robot = serial_arm(segs, axes, [0.055, 0.05, 0.045, 0.04, 0.04, 0.035], 0.09, 0.07, name="ur5_style")
    nominal = np.array([0.0, 0.9, 1.2, 0.4, 0.0, 0.3])
    rng = np.random.default_rng(3)
    n = max(1, int(round(4096 * scale)))
    starts = nominal + rng.uniform(-0.05, 0.05, size=(n, 6))
    target = np.array([[0.9, 1.1, 0.8, 0.6, 0.5, -0.3]])
    solver = SimulatorSolverParameters(forward_simulation_time=1.0)
    return Workload("cfg2", "UR5-style 6-DOF arm, 128^3 SDF, 4096 particles x 100 steps", robot, _cfg2_env, starts, target,
                    solver, 100.0, 12, True, 128, 0.02)


def _cfg3_env(device=None, stats=None, resident=False):
    rng = np.random.default_rng(4)
    obstacles = [box(1, [0.0, 0.0, -0.05], [1.1, 1.1, 0.05])]            # table, top at z = 0
    pillars = [[0.55, 0.35], [0.25, 0.62], [-0.45, 0.45], [0.6, -0.3], [-0.2, -0.6]]
    for i, (x, y) in enumerate(pillars):
        h = rng.uniform(0.3, 0.5)
        obstacles.append(box(2 + i, [x, y, h / 2], [0.05, 0.05, h / 2]))
    return build_complete_environment(obstacles, 0.01, origin=grid_origin([-1.28, -1.28, -0.3]), num_cells=(256, 256, 256),
                                      device=device, stats=stats, resident=resident)


def iiwa_style_arm() -> RobotDescription:
    segs = [0.14, 0.2, 0.2, 0.2, 0.2, 0.08, 0.126]
    axes = [[0, 0, 1], [0, 1, 0], [0, 0, 1], [0, -1, 0], [0, 0, 1], [0, 1, 0], [0, 0, 1]]
    radii = [0.06, 0.06, 0.055, 0.055, 0.05, 0.045, 0.04]
    return serial_arm(segs, axes, radii, 0.2, 0.08, limits=2.9, name="iiwa_style_7dof")


CFG3_NOMINAL = np.array([0.0, 0.6, 0.0, -1.2, 0.0, 0.6, 0.0])
CFG3_TARGET = np.array([1.1, 0.9, 0.3, -0.7, 0.4, 1.0, 0.5])


def cfg3(scale: float = 1.0) -> Workload:
    robot = iiwa_style_arm()
    rng = np.random.default_rng(4)
    n = max(1, int(round(65536 * scale)))
    starts = CFG3_NOMINAL + rng.uniform(-0.05, 0.05, size=(n, 7))
    solver = SimulatorSolverParameters(forward_simulation_time=2.0)
    return Workload("cfg3", "7-DOF linked arm, 256^3 SDF, 65536 particles x 200 steps", robot, _cfg3_env, starts,
                    CFG3_TARGET[None, :].copy(), solver, 100.0, 13, True, 256, 0.01)


# ---------------------------------------------------------------- cfg4: SE(3)
def cfg4_obstacles() -> List[ObstacleConfig]:
    rng = np.random.default_rng(5)
    obstacles = []
    for i in range(24):
        c = [rng.uniform(-0.9, 0.9), rng.uniform(-0.9, 0.9), rng.uniform(-0.9, 0.9)]
        if np.linalg.norm(c) < 0.35:
            continue
        h = [rng.uniform(0.04, 0.15) for _ in range(3)]
        obstacles.append(box(i + 1, c, h, rotation_from_axis_angle(rng.normal(size=3), rng.uniform(0, np.pi))))
    # a block across the straight-line path to the target, so particles slide along it
    obstacles.append(box(100, [0.2, 0.14, -0.09], [0.04, 0.04, 0.04], rotation_from_axis_angle([0.0, 0.0, 1.0], 0.3)))
    return obstacles


def _cfg4_env(device=None, stats=None, resident=False):
    return build_complete_environment(cfg4_obstacles(), 0.01, origin=grid_origin([-1.28, -1.28, -1.28]), num_cells=(256, 256, 256),
                                      device=device, stats=stats, resident=resident)


def cfg4(scale: float = 1.0) -> Workload:
    g = (np.arange(8) - 3.5) * 0.02
    gz = (np.arange(4) - 1.5) * 0.02
    pts = np.array([[x, y, z, 1.0] for x in g for y in g for z in gz])
    tr = ControllerConfig(kp=4.0, ki=0.4, kd=0.04, integral_clamp=0.5, velocity_limit=0.5,
                          max_actuator_proportional_noise=0.2, max_actuator_minimum_noise=0.0005)
    rot = ControllerConfig(kp=4.0, ki=0.4, kd=0.04, integral_clamp=0.5, velocity_limit=1.0,
                           max_actuator_proportional_noise=0.2, max_actuator_minimum_noise=0.0005)
    robot = make_se3_robot(pts, tr, rot, name="se3_free_flyer")
    rng = np.random.default_rng(5)
    n = max(1, int(round(1048576 * scale)))
    starts = np.zeros((n, 12))
    for i in range(n):
        R = rotation_from_axis_angle(rng.normal(size=3), rng.uniform(0, 0.1))
        starts[i] = se3_pose(rng.uniform(-0.03, 0.03, size=3), R)
    target = se3_pose([0.45, 0.3, -0.2], rotation_from_axis_angle([0.3, 1.0, 0.2], 0.8))[None, :]
    solver = SimulatorSolverParameters(forward_simulation_time=1.0)
    return Workload("cfg4", "SE(3) free-flying rigid body, 256^3 SDF, 1M particles x 100 steps", robot, _cfg4_env, starts,
                    target, solver, 100.0, 14, True, 256, 0.01)


# ---------------------------------------------------------------- cfg5: dual arm
def dual_arm_robot() -> RobotDescription:
    """Baxter-like: torso (link 0) carrying two 7-DOF arms on fixed shoulder mounts;
    17 links (torso, 2 mounts, 2 x 7 arm links), 14 dofs."""
    joints = []
    geoms = [(0, cylinder_points(0.5, 0.12, 64, 16))]
    segs = [0.12, 0.25, 0.12, 0.25, 0.12, 0.15, 0.1]
    axes = [[0, 0, 1], [0, 1, 0], [1, 0, 0], [0, 1, 0], [1, 0, 0], [0, 1, 0], [1, 0, 0]]
    radii = [0.06, 0.055, 0.05, 0.05, 0.045, 0.04, 0.035]
    link = 1
    allowed = []
    for side, y in ((0, 0.26), (1, -0.26)):
        mount = link
        rot = rotation_from_axis_angle([1, 0, 0], -np.pi / 2 if side == 0 else np.pi / 2)
        joints.append(Joint(parent=0, child=mount, type=_capi.JOINT_FIXED, origin=transform34([0.06, y, 0.5], rot)))
        geoms.append((mount, cylinder_points(0.08, 0.07, 64, 16)))
        allowed.append((0, mount))
        prev = mount
        link += 1
        for i in range(7):
            off = 0.08 if i == 0 else segs[i - 1]
            joints.append(Joint(parent=prev, child=link, type=_capi.JOINT_REVOLUTE, origin=transform34([0, 0, off]),
                                axis=tuple(axes[i]), lower=-2.9, upper=2.9))
            geoms.append((link, cylinder_points(segs[i], radii[i], 64, 16)))
            allowed.append((prev, link))
            if i == 0:
                allowed.append((0, link))
            else:
                allowed.append((prev - 1 if prev - 1 >= mount else 0, link))
            prev = link
            link += 1
    # geometry indices equal link indices here (one geometry per link, in link order)
    return make_linked_robot(transform34([0, 0, 0]), link, joints, geoms, allowed, _arm_controllers(14), [1.0] * 14,
                             name="dual_arm_14dof")


def _cfg5_env(device=None, stats=None, resident=False):
    obstacles = [box(1, [0.6, 0.0, 0.35], [0.35, 0.7, 0.05]),
                 box(2, [0.7, 0.35, 0.48], [0.1, 0.1, 0.08]),
                 box(3, [0.7, -0.35, 0.48], [0.1, 0.1, 0.08])]
    return build_complete_environment(obstacles, 0.005, origin=grid_origin([-0.48, -1.28, -0.2]), num_cells=(512, 512, 512),
                                      device=device, stats=stats, resident=resident)


def cfg5(scale: float = 1.0) -> Workload:
    robot = dual_arm_robot()
    nominal = np.array([0.3, 0.5, 0.0, 0.8, 0.0, 0.4, 0.0] * 2)
    target = nominal + np.array([0.5, 0.3, 0.2, -0.3, 0.3, 0.2, 0.1, -0.5, 0.3, -0.2, -0.3, -0.3, 0.2, -0.1])
    rng = np.random.default_rng(6)
    n = max(1, int(round(1048576 * scale)))
    starts = nominal + rng.uniform(-0.05, 0.05, size=(n, 14))
    solver = SimulatorSolverParameters(forward_simulation_time=2.0)
    return Workload("cfg5", "dual-arm 14-DOF linked model, 512^3 SDF, 1M particles x 200 steps", robot, _cfg5_env, starts,
                    target[None, :], solver, 100.0, 15, True, 512, 0.005)


# the scene of each workload, buildable on the host (device=None) or on a HIP device
SCENES: Dict[str, Callable[..., SimulatorEnvironment]] = {"cfg1": _cfg1_env, "cfg2": _cfg2_env, "cfg3": _cfg3_env,
                                                          "cfg4": _cfg4_env, "cfg5": _cfg5_env}

WORKLOADS: Dict[str, Callable[..., Workload]] = {"cfg1": cfg1, "cfg2": cfg2, "cfg3": cfg3, "cfg4": cfg4, "cfg5": cfg5}


# ---------------------------------------------------------------- branch-coverage scenes (tests)
# Small scenes that drive resolver branches the BASELINE configs rarely or never reach:
# self-collision corrections (ExtractSelfCollidingPoints SPCS:983-1171), a cell shared by
# many links (no capacity limit, as the reference's maps), a 32-DOF chain, continuous joints.
def _open_space_env(device=None, stats=None, resident=False):
    """128^3 @ 1 cm around the origin with a floor well below the robots."""
    obstacles = [box(1, [0.0, 0.0, -0.15], [0.6, 0.6, 0.03])]
    return build_complete_environment(obstacles, 0.01, origin=grid_origin([-0.64, -0.64, -0.2]), num_cells=(128, 128, 128),
                                      device=device, stats=stats, resident=resident)


def folding_arm(scale: float = 1.0, continuous: bool = False) -> Workload:
    """3-link arm whose parallel y axes fold link 3 back onto link 1 and the base: only
    adjacent links may touch, so the fold is a self-collision the resolver must push
    apart (SPCS:1183-1275 -> 983-1171 -> corrections SPCS:1846-1853).  continuous=True
    makes the joints continuous (angle wrap, TNUVA:556 / SetPosition)."""
    segs = [0.25, 0.25, 0.25]
    joints, geoms = [], [(0, cylinder_points(0.1, 0.05, 64, 16))]
    for i in range(3):
        # continuous: the first joint spins the arm about the vertical through +-pi
        jt = _capi.JOINT_CONTINUOUS if (continuous and i == 0) else _capi.JOINT_REVOLUTE
        joints.append(Joint(parent=i, child=i + 1, type=jt, origin=transform34([0, 0, 0.1 if i == 0 else segs[i - 1]]),
                            axis=(0.0, 0.0, 1.0) if (continuous and i == 0) else (0.0, 1.0, 0.0), lower=-3.0, upper=3.0))
        geoms.append((i + 1, cylinder_points(segs[i], 0.02, 64, 16)))
    allowed = [(0, 1), (1, 2), (2, 3)]
    robot = make_linked_robot(transform34([0, 0, 0]), 4, joints, geoms, allowed, _arm_controllers(3, vmax=1.5), [1.0] * 3,
                              name="folding_arm_continuous" if continuous else "folding_arm")
    rng = np.random.default_rng(8)
    n = max(1, int(round(32 * scale)))
    starts = np.array([2.8 if continuous else 0.0, 0.4, 0.4]) + rng.uniform(-0.05, 0.05, size=(n, 3))
    target = np.array([[-2.8 if continuous else 0.0, 2.5, 2.6]])
    solver = SimulatorSolverParameters(forward_simulation_time=2.0)
    return Workload("folding_arm", "3-link arm folding onto itself (self-collision resolver)", robot, _open_space_env, starts,
                    target, solver, 50.0, 21, True, 128, 0.01)


def crowded_cell_robot(links: int = 10) -> RobotDescription:
    """`links` links on revolute z joints at one point: link k carries a ring of 8 points of
    radius 1.5 mm + 0.3 mm k, so every link has points in the same 1 cm self-collision cell
    and no pair is allowed except along the chain.  A cell then holds `links` links (the
    impulse solve of SPCS:1054-1150 runs with n = links - 1 others)."""
    joints, geoms = [], []
    geoms.append((0, np.array([[0.0015 * np.cos(a), 0.0015 * np.sin(a), 0.0, 1.0] for a in np.arange(8) * np.pi / 4])))
    for k in range(1, links):
        joints.append(Joint(parent=k - 1, child=k, type=_capi.JOINT_REVOLUTE, origin=transform34([0, 0, 0]),
                            axis=(0.0, 0.0, 1.0), lower=-3.0, upper=3.0))
        r = 0.0015 + 0.0003 * k
        geoms.append((k, np.array([[r * np.cos(a + 0.1 * k), r * np.sin(a + 0.1 * k), 0.0005 * k, 1.0]
                                   for a in np.arange(8) * np.pi / 4])))
    allowed = [(k - 1, k) for k in range(1, links)]
    return make_linked_robot(transform34([0.105, 0.105, 0.105]), links, joints, geoms, allowed,
                             _arm_controllers(links - 1, vmax=1.0), [1.0] * (links - 1), name=f"crowded_cell_{links}")


def crowded_cell(scale: float = 1.0, links: int = 10) -> Workload:
    robot = crowded_cell_robot(links)
    rng = np.random.default_rng(9)
    n = max(1, int(round(8 * scale)))
    starts = rng.uniform(-0.2, 0.2, size=(n, links - 1))
    target = np.full((1, links - 1), 0.8)
    solver = SimulatorSolverParameters(forward_simulation_time=0.1)
    return Workload("crowded_cell", f"{links} links sharing one self-collision cell", robot, _open_space_env, starts, target,
                    solver, 100.0, 22, True, 128, 0.01)


def long_chain_robot(dofs: int = 32, points_per_link: int = 16) -> RobotDescription:
    """A `dofs`-DOF serial chain of short links (alternating y / x axes), `points_per_link`
    points per link."""
    k = points_per_link
    joints, geoms = [], [(0, cylinder_points(0.05, 0.03, k, k // 4))]
    for i in range(dofs):
        joints.append(Joint(parent=i, child=i + 1, type=_capi.JOINT_REVOLUTE, origin=transform34([0, 0, 0.05 if i == 0 else 0.03]),
                            axis=(0.0, 1.0, 0.0) if i % 2 == 0 else (1.0, 0.0, 0.0), lower=-2.5, upper=2.5))
        geoms.append((i + 1, cylinder_points(0.03, 0.012, k, k // 4)))
    allowed = [(i, i + 1) for i in range(dofs)] + [(i, i + 2) for i in range(dofs - 1)]
    return make_linked_robot(transform34([0, 0, 0]), dofs + 1, joints, geoms, allowed, _arm_controllers(dofs, vmax=1.0),
                             [1.0] * dofs, name=f"chain_{dofs}dof")


def long_chain(scale: float = 1.0, dofs: int = 32) -> Workload:
    robot = long_chain_robot(dofs)
    rng = np.random.default_rng(10)
    n = max(1, int(round(16 * scale)))
    starts = np.tile(np.linspace(0.05, 0.15, dofs), (n, 1)) + rng.uniform(-0.02, 0.02, size=(n, dofs))
    target = np.tile(np.array([0.5, -0.4]), dofs // 2 + 1)[None, :dofs]
    solver = SimulatorSolverParameters(forward_simulation_time=0.5)
    return Workload("long_chain", f"{dofs}-DOF serial chain", robot, _open_space_env, starts, target, solver, 100.0, 23, True,
                    128, 0.01)


def pid_free_space(scale: float = 1.0) -> Workload:
    """The folding arm's geometry moved by small targets through free space with the
    actuator noise bounds at zero and gains that keep the PID term inside the velocity
    clamp: every controller step's control input is the reference PID's output (PID:122-135)
    times dt, so a trace of it can be replayed through the reference header itself
    (tests/golden/make_pid_trace_golden.py)."""
    wl = folding_arm(scale)
    for c in wl.robot.controllers:
        c.kp, c.ki, c.kd, c.integral_clamp = 2.0, 0.5, 0.01, 0.2
        c.velocity_limit = 2.5
        c.max_actuator_proportional_noise = 0.0
        c.max_actuator_minimum_noise = 0.0
    rng = np.random.default_rng(12)
    n = max(1, int(round(4 * scale)))
    wl.starts = np.array([0.0, 0.4, 0.4]) + rng.uniform(-0.05, 0.05, size=(n, 3))
    wl.targets = np.array([[0.5, 0.8, 0.3]])
    wl.solver = SimulatorSolverParameters(forward_simulation_time=1.0)
    wl.name, wl.description = "pid_free_space", "folding-arm geometry in free space, noise bounds 0"
    return wl


def giant_chain(scale: float = 1.0) -> Workload:
    """The largest robot the descriptor admits: 64 links, 63 dofs, 64 geometries of 64
    points (4096 points, 64 rounds).  Its per-wave LDS block does not fit four times in
    a CU, so it runs with fewer waves per workgroup (fks_set_robot); the reference has no
    size limit (TNUVA:486-517)."""
    robot = long_chain_robot(63, 64)
    rng = np.random.default_rng(13)
    n = max(1, int(round(4 * scale)))
    starts = np.tile(np.linspace(0.02, 0.08, 63), (n, 1)) + rng.uniform(-0.01, 0.01, size=(n, 63))
    target = np.tile(np.array([0.3, -0.2]), 32)[None, :63]
    solver = SimulatorSolverParameters(forward_simulation_time=0.05)
    return Workload("giant_chain", "64-link, 63-DOF chain, 4096 points", robot, _open_space_env, starts, target, solver, 100.0,
                    24, True, 128, 0.01)


COVERAGE: Dict[str, Callable[..., Workload]] = {"giant_chain": giant_chain, "folding_arm": folding_arm, "crowded_cell": crowded_cell,
                                                "long_chain": long_chain, "pid_free_space": pid_free_space}
