"""Build robot-shape-specialised kernels into the disk cache before a planner needs them.

    FKS_KERNEL_CACHE=<dir> python tools/precompile_kernels.py --workload cfg3 [--workload cfg5 ...] [--device 0]

For each named BASELINE workload (or, from Python, any RobotDescription passed to
precompile()), a context is made on the device, the robot set and its shaped kernel built
(fks_set_specialization: the same module also carries the shaped configuration check).  The
code object lands in the disk cache (FKS_KERNEL_CACHE, default ~/.cache/fast_kinematic_simulator_amd),
where every later process on this machine finds it.  The launch layout that fixes a shape
depends on the device, so this runs on the GPU host the planner runs on.  Prints one JSON line
per robot: shape key, whether it was compiled now or found cached, and the failure log if any.
"""
from __future__ import annotations

import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def precompile(robot, environment, solver, controller_frequency, seed=0, device=0) -> dict:
    """Build `robot`'s shaped kernel on `device` into the caches; returns fks_get_specialization."""
    from fast_kinematic_simulator_amd import FksError, make_linked_simulator

    sim = make_linked_simulator(environment, solver, controller_frequency, seed, device=device)
    try:
        sim.set_robot(robot)
        try:
            sim.set_specialization(True)
        except FksError:
            pass  # reported through specialization()["failed"] / ["message"]
        return sim.specialization()
    finally:
        sim.close()


def main() -> int:
    from fast_kinematic_simulator_amd import workloads as W

    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", action="append", default=[], choices=sorted({**W.WORKLOADS, **W.COVERAGE}))
    ap.add_argument("--device", type=int, default=0)
    a = ap.parse_args()
    rc = 0
    for name in a.workload or ["cfg3"]:
        wl = {**W.WORKLOADS, **W.COVERAGE}[name](8 / 65536 if name in W.WORKLOADS else 1.0)
        env = W.SCENES[name](device=a.device) if name in W.SCENES else wl.environment()
        info = precompile(wl.robot, env, wl.solver, wl.controller_frequency, wl.seed, a.device)
        print(json.dumps({"workload": name, "shape": info["shape"], "active": bool(info["active"]),
                          "from_cache": bool(info["from_cache"]), "compile_seconds": info["compile_seconds"],
                          "failed": bool(info["failed"]), "message": info["message"]}), flush=True)
        rc = rc or (1 if info["failed"] else 0)
    return rc


if __name__ == "__main__":
    sys.exit(main())
