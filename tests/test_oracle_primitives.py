"""Known-answer tests of the oracle's restated primitives (one KAT
per restated external primitive).  Pinned: Philox (Random123 KATs), PID (golden
vectors produced by the reference's own simple_pid_controller.hpp).  Property-
checked (parity unpinned): QR least squares, SDF estimate, FK,
Jacobian, SE(3) exp/log, truncated-normal noise."""
import json
import math
import os

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))


def test_philox_known_answers(oracle_lib):
    import oracle

    # Random123 kat_vectors, philox4x32_10
    assert oracle.philox([0, 0, 0, 0], [0, 0]) == [0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8]
    assert oracle.philox([0xFFFFFFFF] * 4, [0xFFFFFFFF, 0xFFFFFFFF]) == [0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD]
    assert oracle.philox([0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344], [0xA4093822, 0x299F31D0]) == [
        0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1]


def test_pid_matches_reference_golden(oracle_lib):
    """SimplePIDController::ComputeFeedbackTerm (PID:122-135) bit-exact against
    the reference header's own output (tests/golden/pid_golden.json)."""
    import oracle

    with open(os.path.join(HERE, "golden", "pid_golden.json")) as f:
        golden = json.load(f)
    for case in golden["cases"]:
        steps = np.array(case["steps"])
        reset = int(np.nonzero(steps[:, 3])[0][0])
        for lo, hi in ((0, reset), (reset, len(steps))):  # Zero() == a fresh controller
            out = oracle.pid_sequence(case["kp"], case["ki"], case["kd"], case["iclamp"], steps[lo:hi, 0], steps[lo:hi, 1])
            assert np.array_equal(out, steps[lo:hi, 2])


def test_truncated_normal_noise(oracle_lib):
    """TN(0, 0.5) truncated to [-1, 1] (UNC:61, TNUVA:128): bounds, moments."""
    import oracle

    vals = np.array([oracle.truncated_normal(7, 0, p, s, m, d)[0] for p in range(40) for s in range(10) for m in range(5)
                     for d in range(4)])
    assert np.all(vals >= -1.0) and np.all(vals <= 1.0)
    assert abs(vals.mean()) < 0.03
    # variance of N(0, 0.5^2) truncated at +-2 sigma: 0.25 * (1 - 4 phi(2) / (2 Phi(2) - 1))
    phi2 = math.exp(-2.0) / math.sqrt(2 * math.pi)
    Phi2 = 0.5 * (1 + math.erf(2 / math.sqrt(2)))
    std = math.sqrt(0.25 * (1 - 4 * phi2 / (2 * Phi2 - 1)))
    assert abs(vals.std() - std) < 0.02
    # deterministic and keyed by every counter field
    a = oracle.truncated_normal(7, 0, 3, 4, 5, 6)
    assert a == oracle.truncated_normal(7, 0, 3, 4, 5, 6)
    assert a != oracle.truncated_normal(7, 1, 3, 4, 5, 6)
    assert a != oracle.truncated_normal(7, 0, 3, 4, 5, 5)


def test_qr_full_rank_least_squares(oracle_lib):
    import oracle

    rng = np.random.default_rng(3)
    for rows, cols in ((30, 7), (9, 7), (300, 14), (7, 7)):
        J = rng.normal(size=(rows, cols))
        b = rng.normal(size=rows)
        x = oracle.qr_solve(J, b)
        ref = np.linalg.lstsq(J, b, rcond=None)[0]
        assert np.allclose(x, ref, atol=1e-10)


def test_qr_rank_deficient_basic_solution(oracle_lib):
    """Eigen ColPivHouseholderQR::solve returns a basic solution: one point gives a
    3x7 system, so 4 unknowns are exactly zero and J x = b."""
    import oracle

    rng = np.random.default_rng(4)
    J = rng.normal(size=(3, 7))
    b = rng.normal(size=3)
    x = oracle.qr_solve(J, b)
    assert np.sum(x == 0.0) == 4
    assert np.allclose(J @ x, b, atol=1e-12)
    # a zero column (a joint that cannot move the corrected points): rank 2 of 3
    J2 = np.array([[1.0, 0.0, 0.0], [0.0, 0.0, 1.0], [2.0, 0.0, 0.0], [0.0, 0.0, 3.0]])
    b2 = np.array([1.0, 2.0, 2.0, 6.0])
    x2 = oracle.qr_solve(J2, b2)
    assert x2[1] == 0.0
    assert np.allclose(J2 @ x2, b2)
    # empty system -> zero step (SPCS:1994 on a 0 x D matrix)
    assert np.array_equal(oracle.qr_solve(np.zeros((0, 5)), np.zeros(0)), np.zeros(5))


@pytest.fixture(scope="module")
def box_env(fks_lib):
    from fast_kinematic_simulator_amd import ObstacleConfig, build_complete_environment, transform34

    obs = [ObstacleConfig(1, transform34([0.5, 0.5, 0.5]), [0.2, 0.2, 0.2])]
    return build_complete_environment(obs, 0.05, origin=transform34([0, 0, 0]), num_cells=(20, 20, 20))


def test_estimate_distance(oracle_lib, box_env):
    """sdf_tools EstimateDistance4d: nominal value moved half a cell toward zero plus
    gradient projection; sign never flips against the nominal value; OOB -> +inf."""
    import oracle

    res = 0.05
    pts = np.array([[0.5, 0.5, 0.5, 1.0], [0.5, 0.5, 0.9, 1.0], [0.5, 0.5, 0.72, 1.0], [-1.0, 0.5, 0.5, 1.0],
                    [0.5, 0.5, 0.025, 1.0]])
    d, inb, near = oracle.estimate_distance(box_env, pts)
    assert inb.tolist() == [True, True, True, False, True]
    assert np.isinf(d[3]) and d[3] > 0
    assert d[0] < 0 and near[0] < 0
    assert d[1] > 0 and abs(d[1] - (near[1] - res / 2)) < res
    for i in (0, 1, 2, 4):
        assert np.sign(d[i]) == np.sign(near[i])


def _two_link_arm():
    from fast_kinematic_simulator_amd import ControllerConfig, Joint, make_linked_robot, transform34
    from fast_kinematic_simulator_amd import _capi

    joints = [Joint(0, 1, _capi.JOINT_REVOLUTE, transform34([0, 0, 0.1]), (0, 0, 1), -3, 3),
              Joint(1, 2, _capi.JOINT_REVOLUTE, transform34([0.5, 0, 0]), (0, 0, 1), -3, 3),
              Joint(2, 3, _capi.JOINT_FIXED, transform34([0.3, 0, 0]))]
    geoms = [(1, np.array([[0.25, 0, 0, 1.0]])), (2, np.array([[0.1, 0.0, 0.0, 1.0]])), (3, np.array([[0.05, 0.02, 0.0, 1.0]]))]
    c = ControllerConfig(kp=1, velocity_limit=1)
    return make_linked_robot(transform34([0, 0, 0]), 4, joints, geoms, [], [c, c])


def test_forward_kinematics_closed_form(oracle_lib):
    import oracle

    robot = _two_link_arm()
    q = np.array([0.4, -1.1])
    T = oracle.link_transforms(robot, q)
    # link 3 origin: planar 2R arm with lengths 0.5, 0.3 at height 0.1
    x = 0.5 * math.cos(q[0]) + 0.3 * math.cos(q[0] + q[1])
    y = 0.5 * math.sin(q[0]) + 0.3 * math.sin(q[0] + q[1])
    assert np.allclose(T[2][[3, 7, 11]], [x, y, 0.1], atol=1e-15)
    R = T[2].reshape(3, 4)[:, :3]
    assert np.allclose(R @ R.T, np.eye(3), atol=1e-15)


def test_jacobian_matches_finite_differences(oracle_lib):
    import oracle

    robot = _two_link_arm()
    q = np.array([0.3, 0.7])
    p = np.array([0.05, 0.02, 0.0, 1.0])
    J = oracle.point_jacobian(robot, q, 2, p)

    def pos(qq):
        T = oracle.link_transforms(robot, qq)[2].reshape(3, 4)
        return T[:, :3] @ p[:3] + T[:, 3]

    h = 1e-6
    num = np.stack([(pos(q + h * e) - pos(q - h * e)) / (2 * h) for e in np.eye(2)], axis=1)
    assert np.allclose(J, num, atol=1e-8)
    # a point on link 1 does not move with joint 2
    J1 = oracle.point_jacobian(robot, q, 0, np.array([0.25, 0, 0, 1.0]))
    assert np.all(J1[:, 1] == 0.0)


def test_se3_exp_log_roundtrip(oracle_lib):
    import oracle

    rng = np.random.default_rng(5)
    for scale in (1e-9, 1e-4, 0.3, 2.0, 3.1):
        tw = rng.normal(size=6)
        tw[3:] *= scale / np.linalg.norm(tw[3:])
        T = oracle.se3_exp(tw)
        R = T.reshape(3, 4)[:, :3]
        assert np.allclose(R @ R.T, np.eye(3), atol=1e-12)
        assert np.allclose(oracle.se3_log(T), tw, atol=1e-9)
