"""Per-particle work distribution of a bench workload on the GPU (what sets the tail):
microsteps and resolver iterations per particle, the heaviest particles against the mean
per resident wave slot, and the kernel time of the call.

    python tools/particle_work.py [--workload cfg3] [--json out.json]
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

from fast_kinematic_simulator_amd import workloads as W  # noqa: E402
from fast_kinematic_simulator_amd.simulator import make_linked_simulator  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="cfg3")
    ap.add_argument("--json", default="")
    a = ap.parse_args()
    wl = W.WORKLOADS[a.workload]()
    sim = make_linked_simulator(wl.environment(), wl.solver, wl.controller_frequency, wl.seed)
    sim.set_robot(wl.robot)
    sim.forward_simulate_arrays(wl.robot, wl.starts[:256], wl.targets, True)  # warm-up
    t0 = time.perf_counter()
    r = sim.forward_simulate_arrays(wl.robot, wl.starts, wl.targets, True)
    dt = time.perf_counter() - t0
    c = sim.last_call_counters()
    m = np.asarray(r["microsteps"], dtype=np.float64)
    it = np.asarray(r["resolver_iterations"], dtype=np.float64)
    geo = sim.launch_geometry()
    resident = geo["resident_waves"]
    order = np.argsort(-(m + 4.0 * it))
    out = {"workload": a.workload, "particles": int(m.size), "call_s": dt, "kernel_ms": c.get("kernel_ms"),
           "microsteps_mean": float(m.mean()), "microsteps_max": float(m.max()),
           "resolver_mean": float(it.mean()), "resolver_max": float(it.max()),
           "microsteps_per_slot": float(m.sum() / resident), "resident_waves": int(resident), "lds_bytes_per_group": geo["lds_bytes_per_group"],
           "percentiles_microsteps": {str(p): float(np.percentile(m, p)) for p in (50, 90, 99, 99.9, 100)},
           "percentiles_resolver": {str(p): float(np.percentile(it, p)) for p in (50, 90, 99, 99.9, 100)},
           "heaviest": [{"particle": int(i), "microsteps": int(m[i]), "resolver_iterations": int(it[i])} for i in order[:10]]}
    print(json.dumps(out, indent=1))
    if a.json:
        with open(a.json, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
