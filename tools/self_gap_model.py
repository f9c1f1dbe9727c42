"""CPU model of a self-check skip proof (measured and not adopted): over the
traced oracle's configurations of a few particles (every post-action and resolver
configuration, i.e. every self check the kernel makes), the kernel's box test in
truncated environment-grid cells, the smallest per-axis gap over the checked geometry
pairs, and how many checks a proof "gap >= 4 + 2 x (box-face motion since the last full
evaluation)" would skip.  `unsound` counts skipped checks whose boxes did overlap (must be 0).

    python tools/self_gap_model.py cfg3 20000 32      # workload, first particle, particles
"""
from __future__ import annotations

import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import oracle  # noqa: E402
from fast_kinematic_simulator_amd import workloads as W  # noqa: E402


def main():
    name, first, n = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
    wl = W.WORKLOADS[name]()
    env, robot = wl.environment(), wl.robot
    G = len(robot.geometry_points)
    boxes = []
    for g in range(G):
        p = np.asarray(robot.geometry_points[g])[:, :3]
        boxes.append(((p.min(0) + p.max(0)) / 2, (p.max(0) - p.min(0)) / 2))
    allowed = {(min(a, b), max(a, b)) for a, b in robot.allowed_pairs}
    pairs = [(a, b) for a in range(G) for b in range(a + 1, G) if (a, b) not in allowed]
    org = np.asarray(env.geometry.origin).reshape(3, 4)
    res = env.geometry.resolution
    rinv = org[:, :3].T
    tinv = -rinv @ org[:, 3]
    k1 = max(np.abs(rinv).sum(1)) / res * (1 + 1e-6)
    radius = [np.linalg.norm(c) + np.linalg.norm(h) for c, h in boxes]

    def cells(tg):
        lo, hi = np.zeros((G, 3)), np.zeros((G, 3))
        for g in range(G):
            t = tg[g].reshape(3, 4)
            c, h = boxes[g]
            gc = rinv @ (t[:, :3] @ c + t[:, 3]) + tinv
            gh = np.abs(rinv) @ (np.abs(t[:, :3]) @ h)
            margin = 1e-6 + 1e-9 * (np.abs(gc) + gh)
            lo[g], hi[g] = np.trunc((gc - gh - margin) / res), np.trunc((gc + gh + margin) / res)
        return lo, hi

    def motion(t, tr, rad):
        t, tr = t.reshape(3, 4), tr.reshape(3, 4)
        return (np.linalg.norm(t[:, 3] - tr[:, 3]) + np.linalg.norm(t[:, :3] - tr[:, :3]) * rad) * (1 + 1e-9) + 1e-12

    sel = np.arange(first, first + n)
    _, buf = oracle.forward_simulate_traced(env, robot, wl.solver, wl.controller_frequency, wl.seed, wl.starts[sel], wl.targets, True,
                                            config_capacity=16000, threads=os.cpu_count(), first_particle_id=first)
    total = skipped = unsound = 0
    for j in range(n):
        ref, smin = None, -np.inf
        for q in buf.configs[j, :min(int(buf.num_configs[j]), 16000)]:
            tg = oracle.link_transforms(robot, q)
            lo, hi = cells(tg)
            gap = min(max(np.max(lo[a] - hi[b]), np.max(lo[b] - hi[a])) for a, b in pairs)
            total += 1
            if ref is not None and smin >= 4:
                d = max(motion(tg[g], ref[g], radius[g]) * k1 for g in range(G))
                if smin >= 4 + 2 * d + 1e-6:
                    skipped += 1
                    unsound += int(gap < 1)
                    continue
            ref, smin = tg.copy(), gap
    print({"workload": name, "geometries": G, "pairs": len(pairs), "checks": total, "skipped": round(skipped / total, 4), "unsound": unsound})


if __name__ == "__main__":
    main()
