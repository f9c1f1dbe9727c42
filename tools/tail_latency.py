"""Latency floor of the heaviest particles (what bounds a launch from below): the full
batch once, then each of the heaviest particles alone in a batch of one (same global
particle id, so the same noise and the same trajectory), with its kernel time.

    python tools/tail_latency.py [--workload cfg3] [--top 3] [--json out.json]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from fast_kinematic_simulator_amd import workloads as W  # noqa: E402
from fast_kinematic_simulator_amd.simulator import make_linked_simulator  # noqa: E402


COUNTS = ("env_rounds_skipped", "env_rounds_evaluated", "corr_rounds_skipped", "corr_rounds_evaluated")


def run(sim, wl, starts, first_id, dev):
    n = starts.shape[0]
    d_starts = torch.from_numpy(np.ascontiguousarray(starts)).to(dev)
    d_targets = torch.from_numpy(np.ascontiguousarray(wl.targets)).to(dev)
    q = torch.empty((n, wl.robot.config_width), dtype=torch.float64, device=dev)
    micro = torch.empty(n, dtype=torch.int32, device=dev)
    res = torch.empty(n, dtype=torch.int32, device=dev)
    sim.set_call_index(0)
    sim.forward_simulate_device(wl.robot, d_starts.data_ptr(), n, d_targets.data_ptr(), 1, first_id, True, q.data_ptr(),
                                d_out_microsteps=micro.data_ptr(), d_out_resolver_iterations=res.data_ptr(), synchronize=True)
    c = sim.last_call_counters()
    ph = sim.phase_cycles(total=False)
    return micro.cpu().numpy(), res.cpu().numpy(), c["kernel_ms"], ph


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="cfg3")
    ap.add_argument("--top", type=int, default=3)
    ap.add_argument("--json", default="")
    ap.add_argument("--specialize", choices=("on", "off"), default="on",
                    help="the robot-shape-specialised kernel for the batch (and for lone particles with --lone throughput)")
    ap.add_argument("--lone", choices=("throughput", "small", "cooperative"), default="throughput",
                    help="the kernel of the lone particles: the batch's, the one-wave small-batch kernel, or the "
                         "cooperative kernel (a workgroup per particle)")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    wl = W.WORKLOADS[a.workload]()
    sim = make_linked_simulator(wl.environment(), wl.solver, wl.controller_frequency, wl.seed)
    sim.set_robot(wl.robot)
    # the library specialises by default: "off" must switch it off explicitly
    sim.set_specialization(a.specialize == "on")
    sim.set_small_batch_kernel(False)
    run(sim, wl, wl.starts[:256], 0, dev)
    m, it, kms, ph = run(sim, wl, wl.starts, 0, dev)
    sim.set_small_batch_kernel(a.lone != "throughput")
    sim.set_cooperative_waves(a.lone == "cooperative")
    out = {"workload": a.workload, "specialization": sim.specialization(), "batch_kernel": sim.launch_info()["last_kernel"],
           "batch_kernel_ms": kms, "particles": int(m.size), "alone": [],
           "batch_phase_share": ({k: round(v / max(1, ph.get("particle", 0)), 4) for k, v in ph.items() if k not in COUNTS}
                                 if ph.get("control", 0) > 0 else None),
           "batch_phase_counts": {k: ph[k] for k in COUNTS if k in ph}}
    for i in np.argsort(-it)[:a.top]:
        i = int(i)
        m1, it1, k1, ph1 = run(sim, wl, wl.starts[i:i + 1], i, dev)
        tot = max(1, ph1.get("particle", 0))
        out["alone"].append({"particle": i, "kernel": sim.launch_info()["last_kernel"], "microsteps": int(m1[0]),
                             "resolver_iterations": int(it1[0]), "kernel_ms": k1,
                             "same_as_in_batch": bool(m1[0] == m[i] and it1[0] == it[i]),
                             "us_per_resolver_iteration_upper": 1e3 * k1 / max(int(it1[0]), 1),
                             "phase_share": ({k: round(v / tot, 4) for k, v in ph1.items() if k not in COUNTS}
                                             if ph1.get("control", 0) > 0 else None),
                             "phase_counts": {k: ph1[k] for k in COUNTS if k in ph1}})
    print(json.dumps(out, indent=1))
    if a.json:
        with open(a.json, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
