"""Batched CheckConfigCollision (SPCS:1398-1416).

CPU: the oracle's CheckConfigCollision against an independent numpy restatement
of the reference's control flow (environment check at inflation_ratio * res with
the tolerance of SPCS:923, self-check on extended cells of (inflation_ratio + 1) *
res, SPCS:1277-1396) on configurations that cover free, environment-colliding and
self-colliding cases.
GPU: the HIP kernel against the oracle, collided flags and error bits bit-exact,
for every robot family and several inflation ratios, through the host-buffer and
the device-buffer entry points."""
import numpy as np
import pytest

from fast_kinematic_simulator_amd import workloads as W


def _configs(wl, n, seed):
    """n configurations: uniform in the joint limits (linked), or perturbed starts."""
    rng = np.random.default_rng(seed)
    robot = wl.robot
    if robot.robot_type == 0:
        lo, hi = robot.dof_limits()
        return rng.uniform(lo, hi, size=(n, robot.config_width))
    base = wl.starts[rng.integers(0, len(wl.starts), size=n)]
    if robot.robot_type == 1:
        return base + rng.uniform(-0.4, 0.4, size=base.shape)
    out = base.copy()
    out[:, [3, 7, 11]] += rng.uniform(-0.3, 0.3, size=(n, 3))
    return out


def _xform(T, p):
    """3x4 transform of 4-vectors in the canonical order (r0*p0 + r1*p1) + r2*p2 + t*w."""
    out = np.empty((len(p), 3))
    for r in range(3):
        out[:, r] = ((T[4 * r] * p[:, 0] + T[4 * r + 1] * p[:, 1]) + T[4 * r + 2] * p[:, 2]) + T[4 * r + 3] * p[:, 3]
    return out


def _restated_check(env, robot, solver, cfg, inflation):
    """Numpy restatement of CheckConfigCollision; returns (env_collision, self_collision)."""
    import oracle

    res = env.resolution
    T = oracle.link_transforms(robot, cfg)
    pts = [_xform(T[g], np.asarray(robot.geometry_points[g], dtype=np.float64)) for g in range(len(robot.geometry_points))]
    thr = inflation * res - solver.environment_collision_check_tolerance * res
    env_hit = False
    for x in pts:
        near = env.nearest(x)
        for i in np.nonzero(near < thr)[0]:
            if near[i] < thr - res:
                env_hit = True
                break
            est, _, _ = oracle.estimate_distance(env, np.append(x[i], 1.0)[None, :])
            if est[0] < thr:
                env_hit = True
                break
        if env_hit:
            break
    G = len(pts)
    allowed = {(a, b) for a, b in robot.allowed_pairs} | {(b, a) for a, b in robot.allowed_pairs}
    if G == 1 or (G == 2 and (0, 1) in allowed):
        return env_hit, False
    o = np.asarray(env.geometry.origin).reshape(3, 4)
    check_res = (inflation + 1.0) * res
    cells = {}
    for g, x in enumerate(pts):
        keys = np.trunc((x - o[:, 3]) / check_res).astype(np.int64)  # identity-rotation grid origin
        for k in map(tuple, keys):
            cells.setdefault(k, set()).add(g)
    self_hit = any(a != b and (a, b) not in allowed for s in cells.values() if len(s) > 1 for a in s for b in s)
    return env_hit, self_hit


@pytest.mark.parametrize("name,scale,n", [("cfg2", 8 / 4096, 96), ("cfg3", 8 / 65536, 96), ("cfg1", 1.0, 64)])
def test_oracle_matches_restatement(oracle_lib, name, scale, n):
    import oracle

    wl = W.WORKLOADS[name](scale)
    env = wl.environment()
    cfgs = _configs(wl, n, seed=11)
    kinds = {"env": 0, "self": 0}
    for inflation in (0.0, 1.5):
        o = oracle.check_config_collision(env, wl.robot, wl.solver, cfgs, inflation)
        assert not o["error_flags"].any()
        for i in range(n):
            e, s = _restated_check(env, wl.robot, wl.solver, cfgs[i], inflation)
            assert bool(o["collided"][i]) == (e or s), (i, inflation, e, s)
            kinds["env"] += e
            kinds["self"] += s
    assert kinds["env"] > 0
    if wl.robot.robot_type == 0:
        assert kinds["self"] > 0, "no self-colliding configuration in the sample"


def test_oracle_inflation_is_monotone(oracle_lib):
    """A configuration colliding at ratio r also collides at every larger ratio's
    environment threshold (the self-check cells grow too, but are not nested, so
    only the environment leg is monotone)."""
    import oracle

    wl = W.cfg3(8 / 65536)
    env = wl.environment()
    cfgs = _configs(wl, 64, seed=5)
    prev = None
    for inflation in (0.0, 0.5, 1.0, 3.0):
        env_only = [_restated_check(env, wl.robot, wl.solver, c, inflation)[0] for c in cfgs]
        if prev is not None:
            assert all(b or not a for a, b in zip(prev, env_only))
        prev = env_only


CASES = [("cfg1", 1.0, 512), ("cfg2", 8 / 4096, 2048), ("cfg3", 8 / 65536, 4096), ("cfg4", 64 / 1048576, 2048),
         ("cfg5", 8 / 1048576, 1024)]


@pytest.mark.gpu
@pytest.mark.parametrize("name,scale,n", CASES)
def test_config_check_parity(fks_lib, oracle_lib, name, scale, n):
    import oracle
    from fast_kinematic_simulator_amd import make_linked_simulator

    wl = W.WORKLOADS[name](scale)
    env = wl.environment()
    cfgs = _configs(wl, n, seed=3)
    cfgs[0] = np.nan  # non-finite configuration: error bits must agree too
    sim = make_linked_simulator(env, wl.solver, wl.controller_frequency, wl.seed)
    try:
        for inflation in (0.0, 0.5, 2.0):
            g = sim.check_config_collisions(wl.robot, cfgs, inflation)
            o = oracle.check_config_collision(env, wl.robot, wl.solver, cfgs, inflation)
            bad = np.nonzero((g["collided"] != o["collided"]) | (g["error_flags"] != o["error_flags"]))[0]
            assert len(bad) == 0, f"{name} inflation {inflation}: {len(bad)} of {n} differ, first {bad[:8]}"
            assert sim.last_check_counters()["sdf_bytes"] == int(o["sdf_bytes"].sum())
            print(name, inflation, "collided", int(g["collided"].sum()), "of", n)
            if inflation == 0.0:
                assert 0 < int(g["collided"].sum()) < n
    finally:
        sim.close()


@pytest.mark.gpu
def test_config_check_device_entry(fks_lib, oracle_lib):
    import torch

    import oracle
    from fast_kinematic_simulator_amd import make_linked_simulator

    wl = W.cfg3(8 / 65536)
    env = wl.environment()
    cfgs = _configs(wl, 3000, seed=9)
    sim = make_linked_simulator(env, wl.solver, wl.controller_frequency, wl.seed)
    try:
        d_cfg = torch.from_numpy(cfgs).to("cuda:0")
        d_out = torch.zeros(len(cfgs), dtype=torch.uint8, device="cuda:0")
        d_err = torch.zeros(len(cfgs), dtype=torch.int32, device="cuda:0")
        stream = torch.cuda.current_stream()
        sim.check_config_collisions_device(wl.robot, d_cfg.data_ptr(), len(cfgs), 0.25, d_out.data_ptr(), d_err.data_ptr(),
                                           stream=stream.cuda_stream, synchronize=True)
        o = oracle.check_config_collision(env, wl.robot, wl.solver, cfgs, 0.25)
        assert np.array_equal(d_out.cpu().numpy().astype(bool), o["collided"])
        assert not d_err.cpu().numpy().any()
        # a forward call after a device check still settles its own statistics
        sim.forward_simulate_arrays(wl.robot, wl.starts[:2], wl.targets, True)
        assert sim.last_call_counters()["particles"] == 2
    finally:
        sim.close()


@pytest.mark.gpu
@pytest.mark.parametrize("name,scale,n", [("cfg2", 8 / 4096, 12288), ("cfg3", 8 / 65536, 12288), ("cfg4", 64 / 1048576, 12288),
                                          ("cfg5", 8 / 1048576, 6144)])
def test_shaped_config_check_parity(fks_lib, oracle_lib, name, scale, n):
    """A batch larger than the resident grid runs the robot's shape-specialised check
    (fks_check_configs_shaped, built with the simulation kernel's module): bit-exact against
    the oracle, collided flags, error bits and algorithmic bytes."""
    import oracle
    from fast_kinematic_simulator_amd import make_linked_simulator

    wl = W.WORKLOADS[name](scale)
    wl._env = W.SCENES[name](device=0)  # the GPU build: the host build's bytes, seconds faster at 512^3
    env = wl.environment()
    cfgs = _configs(wl, n, seed=13)
    cfgs[1] = np.nan
    sim = make_linked_simulator(env, wl.solver, wl.controller_frequency, wl.seed)
    try:
        sim.set_robot(wl.robot)
        assert n > sim.launch_info()["resident_waves"]
        for inflation in (0.0, 0.5):
            g = sim.check_config_collisions(wl.robot, cfgs, inflation)
            assert sim.launch_info()["last_check_kernel"] == "shaped", (sim.launch_info(), sim.specialization())
            o = oracle.check_config_collision(env, wl.robot, wl.solver, cfgs, inflation)
            bad = np.nonzero((g["collided"] != o["collided"]) | (g["error_flags"] != o["error_flags"]))[0]
            assert len(bad) == 0, f"{name} inflation {inflation}: {len(bad)} of {n} differ, first {bad[:8]}"
            assert sim.last_check_counters()["sdf_bytes"] == int(o["sdf_bytes"].sum())
            assert 0 < int(g["collided"].sum()) < n
    finally:
        sim.close()
