"""Restatement audit: how many results move when the
oracle is rebuilt under each alternative the reference's own build could plausibly
have used.  The reference (Eigen, arc_utilities, sdf_tools) cannot be built here, so
these counts are the honest error bar of a parity oracle that is pinned only where
noted in DESIGN.md §3.

Variants (oracle/Makefile `audit`; the parity oracle is the default build):
  v4seq   Vector4d dot / squaredNorm summed sequentially ((x+y)+z)+w instead of
          Eigen's SSE2 Packet2d order (x+z)+(y+w)  (round 1's choice)
  seqsum  least-squares long sums (column norms, Householder dot products) as plain
          ascending sums instead of the 64-lane strided butterfly
  libm    the system libm's sin/cos/log/atan/atan2 instead of the portable kernels
  fma     FMA contraction everywhere (-mfma -ffp-contract=fast), i.e. a
          -march=native build of the reference on an FMA host

For every scene: the fraction of particles whose microstep count, resolver-iteration
count, collided flag or final configuration (bitwise) differs from the parity oracle,
the largest final-configuration difference, and the relative change of the call's
total microsteps.  Counter RNG mode throughout, so noise is identical across variants.

    python tools/restatement_audit.py [--particles N] [--json profiles/r02_restatement_audit.json]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import oracle  # noqa: E402  (test infrastructure; this tool is part of the audit, not the product)
from fast_kinematic_simulator_amd import workloads  # noqa: E402


def run(wl, n, threads):
    return oracle.forward_simulate(wl.environment(), wl.robot, wl.solver, wl.controller_frequency, wl.seed, wl.starts[:n],
                                   wl.targets, wl.allow_contacts, threads=threads)


def compare(base, alt):
    pb, pa = np.asarray(base["positions"]), np.asarray(alt["positions"])
    n = pb.shape[0]
    pos_diff = np.any(pb.view(np.uint64) != pa.view(np.uint64), axis=1)
    mb, ma = np.asarray(base["microsteps"], np.int64), np.asarray(alt["microsteps"], np.int64)
    rb, ra = np.asarray(base["resolver_iterations"], np.int64), np.asarray(alt["resolver_iterations"], np.int64)
    cb, ca = np.asarray(base["collided"]), np.asarray(alt["collided"])
    tot_b, tot_a = int(mb.sum()), int(ma.sum())
    return {
        "particles": n,
        "microsteps_changed": int(np.count_nonzero(mb != ma)),
        "resolver_iterations_changed": int(np.count_nonzero(rb != ra)),
        "collided_changed": int(np.count_nonzero(cb != ca)),
        "configuration_changed": int(np.count_nonzero(pos_diff)),
        "max_abs_configuration_diff": float(np.max(np.abs(pb - pa))) if n else 0.0,
        "total_microsteps_rel_change": (tot_a - tot_b) / max(tot_b, 1),
    }


SCENES = {
    "cfg1": (workloads.cfg1, 4096),
    "cfg2": (workloads.cfg2, 1024),
    "cfg3": (workloads.cfg3, 1024),
    "cfg4": (workloads.cfg4, 512),
    "cfg5": (workloads.cfg5, 256),
    "self_collision": (workloads.folding_arm, 256),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--particles", type=int, default=0, help="override every scene's prefix size")
    ap.add_argument("--scenes", default=",".join(SCENES))
    ap.add_argument("--threads", type=int, default=0)
    ap.add_argument("--json", default="")
    a = ap.parse_args()
    out = {"variants": list(oracle.AUDIT_VARIANTS), "scenes": {}}
    for name in a.scenes.split(","):
        make, n = SCENES[name]
        wl = make()
        n = min(a.particles or n, wl.num_particles)
        t0 = time.perf_counter()
        base = run(wl, n, a.threads)
        row = {"particles": n, "controller_steps": wl.steps, "total_microsteps": int(np.sum(base["microsteps"]))}
        for v in oracle.AUDIT_VARIANTS:
            with oracle.audit_variant(v):
                row[v] = compare(base, run(wl, n, a.threads))
        out["scenes"][name] = row
        print(f"{name}: {n} particles, {time.perf_counter() - t0:.1f} s", file=sys.stderr)
        for v in oracle.AUDIT_VARIANTS:
            r = row[v]
            print(f"  {v:7s} microsteps changed {r['microsteps_changed']:5d}/{n}  config changed "
                  f"{r['configuration_changed']:5d}/{n}  collided changed {r['collided_changed']:4d}  max|dq| "
                  f"{r['max_abs_configuration_diff']:.3g}  total microsteps {100 * r['total_microsteps_rel_change']:+.4f} %",
                  file=sys.stderr)
    if a.json:
        with open(a.json, "w") as f:
            json.dump(out, f, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
