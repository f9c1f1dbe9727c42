"""When does each cfg3 particle finish, and when did it turn contact-heavy?  (GPU diagnostic)

    python tools/finish_probe.py <probe.so> [--json out.json]

<probe.so> is a build with -DFKS_FINISH_PROBE=1 (fast_kinematic_simulator_amd.build.build_variant):
it writes each particle's end time and first heavy carry time (100 MHz s_memrealtime ticks)
instead of its microstep / resolver counts.  The tool runs the normal library for the work
counts and the probe build for the times (one subprocess each, same batch and call index),
then reports the particles that end the launch: when they ended, when their heavy phase
began, and how much work they did.
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(out_path: str):
    import torch

    sys.path.insert(0, ROOT)
    from fast_kinematic_simulator_amd import workloads as W
    from fast_kinematic_simulator_amd.simulator import make_linked_simulator

    dev = torch.device("cuda", 0)
    wl = W.cfg3()
    sim = make_linked_simulator(wl.environment(), wl.solver, wl.controller_frequency, wl.seed)
    sim.set_robot(wl.robot)
    n = wl.starts.shape[0]
    d_starts = torch.from_numpy(np.ascontiguousarray(wl.starts)).to(dev)
    d_targets = torch.from_numpy(np.ascontiguousarray(wl.targets)).to(dev)
    for rep in range(2):  # the first call warms up
        q = torch.empty((n, wl.robot.config_width), dtype=torch.float64, device=dev)
        micro = torch.zeros(n, dtype=torch.int32, device=dev)
        res = torch.zeros(n, dtype=torch.int32, device=dev)
        sim.set_call_index(0)
        sim.forward_simulate_device(wl.robot, d_starts.data_ptr(), n, d_targets.data_ptr(), 1, 0, True, q.data_ptr(),
                                    d_out_microsteps=micro.data_ptr(), d_out_resolver_iterations=res.data_ptr(), synchronize=True)
    c = sim.last_call_counters()
    np.savez(out_path, a=micro.cpu().numpy().view(np.uint32), b=res.cpu().numpy().view(np.uint32),
             kernel_ms=np.array([c["kernel_ms"]]))


def main():
    if len(sys.argv) > 2 and sys.argv[1] == "--child":
        child(sys.argv[2])
        return
    ap = argparse.ArgumentParser()
    ap.add_argument("probe")
    ap.add_argument("--json", default="")
    ap.add_argument("--top", type=int, default=40)
    a = ap.parse_args()
    tmp = "/tmp/finish_probe_%d" % os.getpid()
    env = dict(os.environ)
    env.pop("FKS_LIB_PATH", None)
    subprocess.run([sys.executable, __file__, "--child", tmp + "_work.npz"], env=env, check=True, timeout=600)
    env.update(FKS_LIB_PATH=os.path.abspath(a.probe), FKS_VARIANT_LIB="1")
    subprocess.run([sys.executable, __file__, "--child", tmp + "_time.npz"], env=env, check=True, timeout=600)
    w = np.load(tmp + "_work.npz")
    t = np.load(tmp + "_time.npz")
    micro, res = w["a"].astype(np.int64), w["b"].astype(np.int64)
    end = t["a"].astype(np.int64)
    heavy = t["b"].astype(np.int64)
    t0 = int(end.min())
    end_ms = (end - t0) / 1e5
    heavy_ms = np.where(heavy > 0, (heavy - t0) / 1e5, np.nan)
    order = np.argsort(-end_ms)
    rows = []
    for i in order[:a.top]:
        rows.append({"particle": int(i), "end_ms": round(float(end_ms[i]), 2),
                     "heavy_from_ms": None if np.isnan(heavy_ms[i]) else round(float(heavy_ms[i]), 2),
                     "microsteps": int(micro[i]), "resolver_iterations": int(res[i])})
    q = np.percentile(end_ms, [50, 90, 99, 99.9, 100])
    out = {"kernel_ms_work_run": float(w["kernel_ms"][0]), "kernel_ms_probe_run": float(t["kernel_ms"][0]),
           "end_ms_percentiles": {"50": q[0], "90": q[1], "99": q[2], "99.9": q[3], "100": q[4]},
           "particles_ending_after_90pct": int(np.sum(end_ms > 0.9 * end_ms.max())),
           "heavy_particles": int(np.sum(heavy > 0)), "last": rows}
    print(json.dumps(out, indent=1))
    if a.json:
        with open(a.json, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
