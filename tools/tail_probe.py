"""How well the persistent grid stays busy on cfg3 (GPU diagnostic, not a test).

    python tools/tail_probe.py [--particles N]

Runs the cfg3 batch, reads the waves' 100 MHz s_memrealtime residency
(FKS_PHASE_WAVE_RESIDENCY: start to queue drained) and compares it with (resident
waves x kernel time).  Prints one JSON line:
slot utilisation (1.0 = no idle wave slots, i.e. no tail), and the spread of
per-particle work (microsteps, resolver iterations).
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from fast_kinematic_simulator_amd import make_linked_simulator  # noqa: E402
from fast_kinematic_simulator_amd import workloads as W  # noqa: E402


def run(sim, wl, n, dev):
    starts = torch.from_numpy(np.ascontiguousarray(wl.starts[:n])).to(dev)
    targets = torch.from_numpy(np.ascontiguousarray(wl.targets)).to(dev)
    Wd = wl.robot.config_width
    out_q = torch.empty((n, Wd), dtype=torch.float64, device=dev)
    out_c = torch.empty(n, dtype=torch.uint8, device=dev)
    out_m = torch.empty(n, dtype=torch.int32, device=dev)
    out_r = torch.empty(n, dtype=torch.int32, device=dev)
    out_e = torch.empty(n, dtype=torch.int32, device=dev)
    sim.reset_total_counters()
    stream = torch.cuda.current_stream(dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    sim.set_call_index(0)
    e0.record(stream)
    sim.forward_simulate_device(wl.robot, starts.data_ptr(), n, targets.data_ptr(), 1, 0, True, out_q.data_ptr(),
                                out_c.data_ptr(), out_m.data_ptr(), out_r.data_ptr(), out_e.data_ptr(),
                                stream=stream.cuda_stream, synchronize=False)
    e1.record(stream)
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1)
    ph = sim.phase_cycles(total=True)
    return ms, ph, out_m.cpu().numpy(), out_r.cpu().numpy()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--particles", type=int, default=65536)
    ap.add_argument("--segment-steps", type=int, nargs="*", default=[0])
    ap.add_argument("--heavy-per-step", type=int, nargs="*", default=[-1],
                    help="FKS_SEGMENT_HEAVY_PER_STEP values to try (-1: library default, 0: off)")
    ap.add_argument("--prio", type=int, nargs="*", default=[-1], help="FKS_SEGMENT_HEAVY_PRIO values (-1: default)")
    ap.add_argument("--save", default="", help="write per-particle microsteps / resolver iterations (.npz)")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    wl = W.WORKLOADS["cfg3"](scale=args.particles / 65536.0)
    denv = W.SCENES["cfg3"](device=0, stats={}, resident=True)
    sim = make_linked_simulator(denv, wl.solver, wl.controller_frequency, wl.seed, device=0)
    sim.set_robot(wl.robot)
    run(sim, wl, 256, dev)  # warm-up
    ms1, ph1, m1, _ = run(sim, wl, 1, dev)
    for seg in args.segment_steps:
        for heavy in args.heavy_per_step:
          for prio in args.prio:
            for var, val in (("FKS_SEGMENT_HEAVY_PER_STEP", heavy), ("FKS_SEGMENT_HEAVY_PRIO", prio)):
                if val >= 0:
                    os.environ[var] = str(val)
                else:
                    os.environ.pop(var, None)
            sim.set_segment_steps(seg)
            ms, ph, m, r = run(sim, wl, args.particles, dev)
            ms, ph, m, r = run(sim, wl, args.particles, dev)
            report(args, sim, f"{seg}/{heavy}/{prio}", ms, ph, m, r, ms1, ph1, m1)


def report(args, sim, seg, ms, ph, m, r, ms1, ph1, m1):
    waves = sim.launch_geometry()["resident_waves"]
    work = m.astype(np.float64)
    out = {
        "segment_steps": seg, "particles": args.particles, "kernel_ms": ms, "single_particle_ms": ms1, "single_particle_microsteps": int(m1[0]),
        "single_particle_residency_ms": ph1["wave_residency"] / 1e5, "resident_waves": waves,
        "memtime_cycles_per_realtime_ms": ph["particle"] / max(1, ph["wave_residency"] / 1e5),
        "wave_slot_busy_fraction": ph["wave_residency"] / 1e5 / (waves * ms),
        "microsteps": {"mean": float(work.mean()), "p50": float(np.median(work)), "p99": float(np.percentile(work, 99)),
                        "max": float(work.max())},
        "resolver": {"mean": float(r.mean()), "p99": float(np.percentile(r, 99)), "max": float(r.max())},
        "last_5120_microsteps_mean": float(work[-5120:].mean()),
    }
    print(json.dumps(out), flush=True)
    if args.save:
        np.savez_compressed(args.save, microsteps=m, resolver=r)


if __name__ == "__main__":
    main()
