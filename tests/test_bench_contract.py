"""bench.py keeps the driver's contract: one JSON line with the BASELINE.json metric,
whole-job value, roofline and cpu_baseline objects (GPU: a small run end to end)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_cli_parses():
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--help"], stdout=subprocess.PIPE,
                       stderr=subprocess.PIPE, text=True, timeout=120)
    assert p.returncode == 0 and "--workload" in p.stdout and "--gpus" in p.stdout


@pytest.mark.gpu
def test_bench_json_line():
    with open(os.path.join(ROOT, "BASELINE.json")) as f:
        metric = json.load(f)["metric"]
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--particles", "2048", "--steps", "1", "--warmup", "1",
                        "--cpu-sample", "16", "--no-config-check"], stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                       text=True, timeout=240, cwd=ROOT)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [l for l in p.stdout.splitlines() if l.strip()]
    assert len(lines) == 1
    d = json.loads(lines[0])
    assert d["metric"] == metric and d["n_gpus"] == 1 and d["steps"] == 1 and d["warmup"] == 1
    assert d["value"] > 0 and d["higher_is_better"] is True and d["scaling"] == "weak" and d["vs_baseline"] is None
    assert d["dtype"] == "f64" and "workload" in d["config"]
    r = d["roofline"]
    assert r["bound"] == "hbm" and r["unit"] == "GB/s" and abs(r["frac"] - r["achieved"] / r["peak"]) < 1e-12
    f = r["fp64"]
    assert f["unit"] == "TFLOP/s" and f["achieved"] > 0 and abs(f["frac"] - f["achieved"] / f["peak"]) < 1e-12
    c = d["cpu_baseline"]
    assert c["kind"] == "port" and c["cores"] >= 1 and c["value"] > 0 and c["sample"]
    assert c["host"]["nproc"] >= 1 and abs(c["per_core"] * c["cores"] - c["value"]) < 1e-6 * c["value"]
    assert d["statistics"]["successful_resolves"] > 0
    assert d["pcie_inclusive"]["value"] > 0


@pytest.mark.gpu
def test_bench_under_torchrun():
    """The driver's multi-GPU launch (torchrun, one rank per GPU, RCCL process group,
    outcome gather, max-over-ranks timing) at the world size one GPU allows."""
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    p = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1", "--master-addr",
                        "127.0.0.1", "--master-port", str(port), os.path.join(ROOT, "bench.py"), "--gpus", "1",
                        "--particles", "2048", "--steps", "1", "--warmup", "1", "--no-cpu-baseline", "--no-config-check"],
                       stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, timeout=300, cwd=ROOT, env=env)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [l for l in p.stdout.splitlines() if l.strip().startswith("{")]
    assert len(lines) == 1
    d = json.loads(lines[0])
    assert d["n_gpus"] == 1 and d["value"] > 0 and d["config"]["particles_total"] == 2048
    assert "process group" in p.stderr  # bench.py logs the RCCL group it joined
