"""The configuration check's extended-cell keys (LocationToExtendedGridIndex, SPCS:1173-1181:
trunc(coordinate / resolution)) are computed as a product with 1/resolution unless an integer
lies within 8 ulp of the product, then by the division (fks_kernels.hip, config_self_collision).
This restates that rule in IEEE double arithmetic and checks it against the division's
truncation on random coordinates and on adversarial ones next to cell faces (CPU)."""
import numpy as np


def _key_fast(v, res):
    inv = 1.0 / res
    r = v * inv
    q = r if (abs(r) < 4.0e15 and abs(r - np.rint(r)) > abs(r) * 2.0 ** -49) else v / res
    return int(np.trunc(q))


def test_product_rule_truncates_like_the_division():
    rng = np.random.default_rng(5)
    bad = 0
    cases = 0
    for res in (0.015, 0.01 * 1.5, 0.02 * 1.5, 0.005 * 2.0, 0.0625 * 1.5, 0.03, 1.0 / 3.0, 0.1):
        vals = list(rng.uniform(-3.0, 3.0, 20000))
        # coordinates next to cell faces: k * res and its floating-point neighbours
        for k in rng.integers(-300, 300, 2000):
            c = float(k) * res
            vals += [c, np.nextafter(c, np.inf), np.nextafter(c, -np.inf), np.nextafter(np.nextafter(c, np.inf), np.inf)]
        for v in vals:
            cases += 1
            if _key_fast(float(v), res) != int(np.trunc(float(v) / res)):
                bad += 1
    assert cases > 100000 and bad == 0
