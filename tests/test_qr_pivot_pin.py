"""Pin of the least-squares solve (SPCS:1990-1998, Eigen ColPivHouseholderQR) to a published
implementation: LAPACK dgeqp3 (scipy.linalg.qr(..., pivoting=True)), on >= 1,000 stacked
systems recorded from real resolver iterations of cfg3 / cfg4 / cfg5
(tests/golden/qr_systems.npz, tests/golden/make_qr_golden.py).

Both are greedy column pivoting by the largest remaining column norm.  At every step where
the two pick different columns the competing residual norms are compared: a difference
above 1e-12 relative is a genuine disagreement (fails), otherwise it is a tie that rounding
may break either way (counted and reported; the comparison of that system stops there).
Where the pivot sequences agree, the zero set of the basic solution (Eigen's nonzero-pivot
threshold maxColSqNorm * eps^2 / R * (R - k) applied to LAPACK's |R_kk|) and the basic
solution itself (from LAPACK's factors) must agree too, except where a pivot's residual is
rounding noise within 10^4 of that threshold (its side of the threshold is the noise of each
implementation; counted and reported).  The GPU solvers equal the oracle
bit for bit (test_gpu_parity.py), so this pins them as well."""
import os

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
FIXTURE = os.path.join(HERE, "golden", "qr_systems.npz")
EPS = 2.220446049250313e-16


def _systems():
    z = np.load(FIXTURE)
    J, b, shape, perm, rdiag, scene = z["J"], z["b"], z["shape"], z["lapack_perm"], z["lapack_rdiag"], z["scene"]
    oj = ob = op = odg = 0
    for k, (r, c) in enumerate(shape):
        r, c = int(r), int(c)
        kk = min(r, c)
        yield (str(z["scenes"][scene[k]]), J[oj:oj + r * c].reshape(r, c), b[ob:ob + r], perm[op:op + c], rdiag[odg:odg + kk])
        oj += r * c
        ob += r
        op += c
        odg += kk


def test_fixture_is_lapacks_factorisation():
    """The stored pivots are what scipy's LAPACK returns here (the fixture is the published
    implementation's output, not a copy of the oracle's)."""
    import scipy.linalg

    n = 0
    for _, J, _, perm, rdiag in _systems():
        _, R, P = scipy.linalg.qr(J, pivoting=True, mode="economic")
        assert np.array_equal(P, perm)
        assert np.allclose(np.abs(np.diag(R)), rdiag, rtol=1e-12, atol=0)
        n += 1
    assert n >= 1000


def _residual_norms(J, order, k):
    """Norms of every column's component orthogonal to the first k pivot columns `order[:k]`
    (the quantity both algorithms maximise at step k), from an orthonormal basis."""
    if k == 0:
        return np.linalg.norm(J, axis=0)
    Q, _ = np.linalg.qr(J[:, order[:k]], mode="reduced")
    resid = J - Q @ (Q.T @ J)
    return np.linalg.norm(resid, axis=0)


def test_oracle_pivots_zero_set_and_solution_match_lapack():
    import scipy.linalg

    import oracle

    systems = list(_systems())
    assert len(systems) >= 1000
    rank_deficient = ties = compared_steps = solved = noise_rank = 0
    worst_x = 0.0
    by_rows = {}
    for scene, J, b, perm, rdiag in systems:
        R, D = J.shape
        by_rows[R] = by_rows.get(R, 0) + 1
        x_o, perm_o, nz_o = oracle.qr_info(J, b)
        size = min(R, D)
        # zero set: Eigen's threshold on LAPACK's pivots (|R_kk| is the pivot's residual norm)
        maxsq = float(np.max(np.sum(J * J, axis=0)))
        thr = maxsq * (EPS * EPS) / R
        nz_l = size
        for k in range(size):
            if rdiag[k] ** 2 < thr * (R - k):
                nz_l = k
                break
        if nz_l < D:
            rank_deficient += 1
        # a pivot whose residual is rounding noise (within 10^4 of Eigen's threshold, which is
        # maxColSqNorm * eps^2 scaled): which side of the threshold it falls on is decided by
        # the noise of each implementation, so the rank is not compared there
        near = thr > 0 and any(1e-4 < rdiag[k] ** 2 / (thr * (R - k)) < 1e4 for k in range(size))
        noise_rank += 1 if near else 0
        # pivot steps above the rank threshold (beyond it both pick among rounding noise)
        agree = True
        for k in range(min(nz_o, nz_l)):
            compared_steps += 1
            if perm_o[k] == perm[k]:
                continue
            norms = _residual_norms(J, perm, k)
            a, o = norms[perm[k]], norms[perm_o[k]]
            assert abs(a - o) <= 1e-12 * max(a, o), (scene, J.shape, k, a, o)
            ties += 1
            agree = False
            break
        if not agree:
            continue  # a tie decided the pivots: the factorisations differ from here on
        if not near:
            assert nz_o == nz_l, (scene, J.shape, nz_o, nz_l)
            assert set(perm_o[nz_o:].tolist()) == set(perm[nz_l:].tolist()), (scene, J.shape)
        if nz_o != nz_l or nz_o == 0:
            continue
        # basic solution from LAPACK's factors: R11 z = (Q^T b)_1, zeros in the non-pivot unknowns
        Q, Rl, P = scipy.linalg.qr(J, pivoting=True, mode="economic")
        R11 = Rl[:nz_o, :nz_o]
        z = scipy.linalg.solve_triangular(R11, (Q.T @ b)[:nz_o])
        x_l = np.zeros(D)
        x_l[P[:nz_o]] = z
        cond = np.linalg.cond(R11)
        err = np.max(np.abs(x_o - x_l)) / max(1e-300, np.max(np.abs(x_l)))
        assert err <= 1e-10 * max(1.0, cond), (scene, J.shape, err, cond)
        worst_x = max(worst_x, err / max(1.0, cond))
        solved += 1
    print(f"\n{len(systems)} systems (rows: {dict(sorted(by_rows.items()))}), {rank_deficient} rank-deficient, "
          f"{compared_steps} pivot steps compared, {ties} ties within 1e-12, {noise_rank} ranks decided by a noise-level "
          f"pivot (not compared), {solved} basic solutions compared, "
          f"worst relative difference / cond {worst_x:.2e}")
    assert rank_deficient > 0 and solved >= 900
