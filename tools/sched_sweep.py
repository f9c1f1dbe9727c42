"""Kernel time of the cfg3 batch over the scheduling knobs (segment length, heavy-segment
threshold, heavy issue priority).  Results never depend on them (tests/test_gpu_parity.py
checks segmented against whole runs); this picks the defaults.

    python tools/sched_sweep.py [--json out.json]
"""
from __future__ import annotations

import argparse
import itertools
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from fast_kinematic_simulator_amd import workloads as W  # noqa: E402
from fast_kinematic_simulator_amd.simulator import make_linked_simulator  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="cfg3")
    ap.add_argument("--segments", default="5,10,20")
    ap.add_argument("--heavy", default="1,2,4,65536")
    ap.add_argument("--prio", default="0,1,2")
    ap.add_argument("--rel", default="3", help="fks_set_segment_heavy_relative values (0 = off)")
    ap.add_argument("--json", default="")
    ap.add_argument("--particles", type=int, default=0, help="batch size (default: the workload's base count)")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    wl = W.WORKLOADS[a.workload]()
    if a.particles:
        wl = W.WORKLOADS[a.workload](scale=a.particles / float(wl.num_particles))
    wl._env = W.SCENES[a.workload](device=0)  # the GPU build (same bytes as the host's)
    sim = make_linked_simulator(wl.environment(), wl.solver, wl.controller_frequency, wl.seed)
    sim.set_robot(wl.robot)
    n = wl.num_particles
    d_starts = torch.from_numpy(np.ascontiguousarray(wl.starts)).to(dev)
    d_targets = torch.from_numpy(np.ascontiguousarray(wl.targets)).to(dev)
    q = torch.empty((n, wl.robot.config_width), dtype=torch.float64, device=dev)
    micro = torch.empty(n, dtype=torch.int32, device=dev)

    def run():
        sim.set_call_index(0)
        sim.forward_simulate_device(wl.robot, d_starts.data_ptr(), n, d_targets.data_ptr(), 1, 0, True, q.data_ptr(),
                                    d_out_microsteps=micro.data_ptr(), synchronize=True)
        return sim.last_call_counters()["kernel_ms"]

    run()
    rows = []
    for seg, heavy, prio, rel in itertools.product(*[[int(v) for v in x.split(",")] for x in (a.segments, a.heavy, a.prio, a.rel)]):
        sim.set_segment_steps(seg)
        sim.set_segment_policy(heavy, prio)
        sim.set_segment_heavy_relative(rel)
        ms = min(run(), run())
        rows.append({"segment_steps": seg, "heavy_resolver_per_step": heavy, "heavy_priority": prio, "heavy_relative": rel,
                     "kernel_ms": ms})
        print(json.dumps(rows[-1]), flush=True)
    best = min(rows, key=lambda r: r["kernel_ms"])
    print("best", json.dumps(best))
    if a.json:
        with open(a.json, "w") as f:
            json.dump({"workload": a.workload, "rows": rows, "best": best}, f, indent=1)


if __name__ == "__main__":
    main()
