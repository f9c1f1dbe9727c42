"""Per-phase cost of the cfg3 hot kernel by repetition (no PC sampling on this pool).

A build with bit b of FKS_PROF_DUP set runs phase b of the microstep / resolver loop
twice with identical inputs and outputs (fks_kernels.hip `prof_reps`), so trajectories
and work are unchanged and the difference of the SQ instruction counters and of the
kernel time against the plain build is the phase's own cost.  `kDupEnvFull` adds one
evaluation of every point with the skip proof off: the cost the skip proof avoids.

    python tools/phase_cost.py build                 # here: build/prof/p_*.so
    bash tools/phase_cost.sh <tag> build/prof/p_*.so # GPU box
    python tools/phase_cost.py report <tag> [--json profiles/<tag>_phase_cost.json]
"""
from __future__ import annotations

import argparse
import csv
import glob
import json
import os
import sys
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

PHASES = ["fk", "input", "env", "self", "corrections", "solve", "resolver_apply", "refill", "env_full"]
COUNTERS = ["SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_SMEM", "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR",
            "SQ_WAVE_CYCLES"]


def build(jobs):
    from fast_kinematic_simulator_amd import build as b

    out = os.path.join(ROOT, "build", "prof")
    os.makedirs(out, exist_ok=True)
    todo = [("p_base", 0)] + [(f"p_{p}", 1 << i) for i, p in enumerate(PHASES)]
    with ThreadPoolExecutor(jobs) as ex:
        for name in ex.map(lambda t: (b.build_variant(os.path.join(out, t[0] + ".so"), [f"FKS_PROF_DUP={t[1]}"]), t[0])[1], todo):
            print(name, flush=True)


def load(tag, name):
    d = os.path.join(ROOT, "gpurun_out", tag, name)
    vals = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Kernel_Name"].startswith("fks_simulate_linked"):
                vals.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    line = json.loads(open(os.path.join(ROOT, "gpurun_out", tag, name + ".json")).read().strip().splitlines()[-1])
    out = {k: sum(v) / len(v) for k, v in vals.items()}
    out["kernel_ms"] = line["roofline"]["avg_kernel_ms"]
    out["microsteps"] = line["config"]["microsteps_per_step"]
    out["resolver_iterations"] = line["config"]["resolver_iterations_per_step"]
    return out


def report(tag, path):
    base = load(tag, "p_base")
    micro = base["microsteps"]
    res = {"tag": tag, "kernel": "fks_simulate_linked", "workload": "cfg3 (bench.py --steps 1 --warmup 1)",
           "base": {k: base[k] for k in base}, "per_microstep_base": {k: base[k] / micro for k in COUNTERS if k in base},
           "phases": {}}
    print(f"base: {base['kernel_ms']:.1f} ms, VALU/microstep {base['SQ_INSTS_VALU'] / micro:.0f}, "
          f"SALU/microstep {base['SQ_INSTS_SALU'] / micro:.0f}")
    for p in PHASES:
        try:
            v = load(tag, "p_" + p)
        except (OSError, KeyError, ValueError, IndexError):
            continue
        row = {"kernel_ms_delta": v["kernel_ms"] - base["kernel_ms"],
               "time_fraction": (v["kernel_ms"] - base["kernel_ms"]) / base["kernel_ms"],
               "work_unchanged": v["microsteps"] == micro and v["resolver_iterations"] == base["resolver_iterations"]}
        for k in COUNTERS:
            if k in v and k in base:
                row[k + "_per_microstep"] = (v[k] - base[k]) / micro
        res["phases"][p] = row
        print(f"{p:15s} time {100 * row['time_fraction']:6.1f} %  VALU/microstep {row.get('SQ_INSTS_VALU_per_microstep', 0):7.0f}"
              f"  SALU {row.get('SQ_INSTS_SALU_per_microstep', 0):6.0f}  LDS {row.get('SQ_INSTS_LDS_per_microstep', 0):5.0f}"
              f"  VMEM_RD {row.get('SQ_INSTS_VMEM_RD_per_microstep', 0):5.1f}  same work {row['work_unchanged']}")
    if path:
        with open(path, "w") as f:
            json.dump(res, f, indent=1)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("mode", choices=["build", "report"])
    ap.add_argument("tag", nargs="?")
    ap.add_argument("--json", default="")
    ap.add_argument("--jobs", type=int, default=3)
    a = ap.parse_args()
    if a.mode == "build":
        build(a.jobs)
    else:
        report(a.tag, a.json)


if __name__ == "__main__":
    main()
