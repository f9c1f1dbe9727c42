"""Summarise the `tailpmc` passes of tools/gpu.sh: per simulate dispatch (the full batch and
the heaviest particle alone, in launch order), the instruction mix, VALU activity and wait
cycles, with the per-resolver-iteration figures of the lone particle.

SQ_WAVE_CYCLES, SQ_BUSY_CYCLES, SQ_ACTIVE_INST_VALU and SQ_WAIT_* count quad-cycles on gfx9
(x4 below).  Instruction counts are per wave instruction (64 lanes).

    python tools/tail_pmc.py gpurun_out/<tag>_tailpmc_cfg3_<lib> [--iterations 4299] [--json out.json]
"""
from __future__ import annotations

import argparse
import collections
import csv
import glob
import json
import os


def dispatches(d):
    out = collections.OrderedDict()
    for path in sorted(glob.glob(os.path.join(d, "*", "*counter_collection.csv"))):
        per = collections.OrderedDict()
        for r in csv.DictReader(open(path)):
            if "simulate" not in r["Kernel_Name"]:
                continue
            c = per.setdefault(int(r["Dispatch_Id"]), {})
            c[r["Counter_Name"]] = c.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        # the passes are separate runs: match dispatches by their order within the run
        for k, (_, c) in enumerate(per.items()):
            out.setdefault(k, {}).update(c)
    return list(out.values())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--iterations", type=int, default=0, help="resolver iterations of the lone particle")
    ap.add_argument("--json", default="")
    a = ap.parse_args()
    rows = []
    for c in dispatches(a.dir):
        valu = c.get("SQ_INSTS_VALU", 0.0)
        f64 = sum(c.get(k, 0.0) for k in ("SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_TRANS_F64"))
        ints = c.get("SQ_INSTS_VALU_INT32", 0.0) + c.get("SQ_INSTS_VALU_INT64", 0.0)
        f32 = sum(c.get(k, 0.0) for k in ("SQ_INSTS_VALU_ADD_F32", "SQ_INSTS_VALU_MUL_F32", "SQ_INSTS_VALU_FMA_F32", "SQ_INSTS_VALU_TRANS_F32"))
        row = {"waves": c.get("SQ_WAVES"), "counters": {k: int(v) for k, v in sorted(c.items())}}
        if valu:
            row["valu_mix"] = {"f64": round(f64 / valu, 4), "int": round(ints / valu, 4), "cvt": round(c.get("SQ_INSTS_VALU_CVT", 0.0) / valu, 4),
                               "f32": round(f32 / valu, 4), "other (moves, selects, compares, lane ops)":
                               round(1.0 - (f64 + ints + f32 + c.get("SQ_INSTS_VALU_CVT", 0.0)) / valu, 4)}
        wave_cycles = 4.0 * c.get("SQ_WAVE_CYCLES", 0.0)
        if wave_cycles:
            row["share_of_wave_cycles"] = {"valu_active": round(4.0 * c.get("SQ_ACTIVE_INST_VALU", 0.0) / wave_cycles, 4),
                                           "waiting_on_memory_lds_smem (s_waitcnt)": round(4.0 * c.get("SQ_WAIT_ANY", 0.0) / wave_cycles, 4),
                                           "waiting_for_issue": round(4.0 * c.get("SQ_WAIT_INST_ANY", 0.0) / wave_cycles, 4)}
            insts = sum(c.get(k, 0.0) for k in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_SMEM", "SQ_INSTS_VMEM", "SQ_INSTS_BRANCH"))
            row["cycles_per_instruction"] = round(wave_cycles / max(1.0, insts), 2)
        rows.append(row)
    out = {"dir": a.dir, "dispatches": rows}
    if a.iterations and rows:
        lone = rows[-1]["counters"]
        out["lone_per_resolver_iteration"] = {k.replace("SQ_INSTS_", ""): round(lone.get(k, 0) / a.iterations, 1)
                                             for k in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_SMEM", "SQ_INSTS_VMEM",
                                                       "SQ_INSTS_BRANCH")}
    s = json.dumps(out, indent=1)
    print(s)
    if a.json:
        open(a.json, "w").write(s + "\n")


if __name__ == "__main__":
    main()
