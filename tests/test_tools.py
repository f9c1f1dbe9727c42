"""The measurement tools DESIGN.md §5.1 cites: the segment-scheduler model and the SQ-counter
summariser (CPU, synthetic inputs)."""
import csv
import importlib.util
import json
import os

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _tool(name):
    spec = importlib.util.spec_from_file_location(name, os.path.join(ROOT, "tools", name + ".py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_sched_model_bounds():
    m = _tool("sched_model")
    # equal particles, as many as slots: every slot runs one particle start to end
    cost = np.full((8, 20), 1.0)
    cost /= cost.sum() / 8
    mk, med, p99 = m.makespan(cost, np.zeros((8, 20), np.int64), 8, 5, 2)
    assert abs(mk - 1.0) < 1e-12 and abs(med - 1.0) < 1e-12
    # lower bounds hold for every policy: the ideal (all slots busy) and the longest chain
    rng = np.random.default_rng(0)
    cost = rng.uniform(0.5, 1.5, (64, 20))
    iters = np.zeros((64, 20), np.int64)
    cost[3] *= 6.0
    iters[3] = 10
    cost /= cost.sum() / 8
    for heavy in (1, 2, 1e9):
        mk = m.makespan(cost, iters, 8, 5, heavy)[0]
        assert mk >= max(1.0, cost[3].sum()) - 1e-12
    # one slot runs everything back to back: makespan = total work
    one = cost / cost.sum()
    assert abs(m.makespan(one, iters, 1, 5, 2)[0] - 1.0) < 1e-9


def test_tail_pmc_summary(tmp_path):
    t = _tool("tail_pmc")
    rows = {"mix": {"SQ_WAVES": 4, "SQ_INSTS_VALU": 1000, "SQ_INSTS_SALU": 400, "SQ_INSTS_LDS": 50, "SQ_INSTS_SMEM": 20,
                    "SQ_INSTS_VMEM": 30, "SQ_INSTS_BRANCH": 100, "SQ_WAVE_CYCLES": 800},
            "wait": {"SQ_INSTS_VALU_FMA_F64": 100, "SQ_INSTS_VALU_ADD_F64": 100, "SQ_INSTS_VALU_MUL_F64": 100,
                     "SQ_INSTS_VALU_TRANS_F64": 0, "SQ_WAIT_INST_ANY": 80, "SQ_WAIT_ANY": 400, "SQ_ACTIVE_INST_VALU": 240,
                     "SQ_BUSY_CYCLES": 900}}
    for p, counters in rows.items():
        d = tmp_path / p
        d.mkdir()
        with open(d / "tail_counter_collection.csv", "w", newline="") as f:
            w = csv.DictWriter(f, fieldnames=["Dispatch_Id", "Kernel_Name", "Counter_Name", "Counter_Value"])
            w.writeheader()
            for k, v in counters.items():
                # two SEs report halves of each counter: the summariser sums them
                w.writerow({"Dispatch_Id": 7, "Kernel_Name": "fks_simulate_linked", "Counter_Name": k, "Counter_Value": v / 2})
                w.writerow({"Dispatch_Id": 7, "Kernel_Name": "fks_simulate_linked", "Counter_Name": k, "Counter_Value": v / 2})
    out = tmp_path / "s.json"
    import sys

    argv = sys.argv
    sys.argv = ["tail_pmc.py", str(tmp_path), "--iterations", "10", "--json", str(out)]
    try:
        t.main()
    finally:
        sys.argv = argv
    s = json.load(open(out))
    d = s["dispatches"][0]
    assert d["valu_mix"]["f64"] == 0.3
    assert d["share_of_wave_cycles"]["valu_active"] == 0.3  # 4 x 240 / (4 x 800)
    assert d["share_of_wave_cycles"]["waiting_on_memory_lds_smem (s_waitcnt)"] == 0.5
    assert d["cycles_per_instruction"] == round(3200 / 1600, 2)
    assert s["lone_per_resolver_iteration"]["VALU"] == 100.0


@pytest.mark.gpu
def test_precompile_kernels_fills_the_disk_cache(tmp_path):
    """tools/precompile_kernels.py: the shapes of the named workloads are built
    into FKS_KERNEL_CACHE on the GPU host, so a planner's first large call finds them there."""
    import subprocess
    import sys

    env = dict(os.environ, FKS_KERNEL_CACHE=str(tmp_path / "cache"))
    p = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "precompile_kernels.py"), "--workload", "cfg2"],
                       stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, timeout=300, env=env)
    assert p.returncode == 0, p.stderr[-2000:]
    line = json.loads(p.stdout.strip().splitlines()[-1])
    assert line["active"] and not line["failed"] and line["shape"].startswith("t0-"), line
    assert len(list((tmp_path / "cache").glob(line["shape"] + "-*.hsaco"))) == 1
