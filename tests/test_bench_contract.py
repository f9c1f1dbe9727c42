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
    # one process, no launcher: no gather ran, and the line does not claim one
    assert d["config"]["outcome_gather"] is None and "RCCL" not in d["config"]["workload"]
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
@pytest.mark.parametrize("mode,kind", [("off", "throughput"), ("on", "shaped")])
def test_bench_specialize_flag_is_what_runs(mode, kind):
    """`--specialize off` times the generic kernel and `on` the shaped one, and the line names
    the kernel the timed launches actually ran (fks_get_launch_info), not the flag"""
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--particles", "8192", "--steps", "1", "--warmup", "1",
                        "--no-cpu-baseline", "--no-config-check", "--no-projection", "--pipeline-batches", "0",
                        "--specialize", mode], stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, timeout=240, cwd=ROOT)
    assert p.returncode == 0, p.stderr[-3000:]
    d = json.loads([l for l in p.stdout.splitlines() if l.strip()][-1])
    assert d["roofline"]["kernel_kind"] == kind, d["roofline"]
    assert d["roofline"]["kernel"].startswith("fks_simulate_shaped" if mode == "on" else "fks_simulate_linked"), d["roofline"]


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
    assert d["config"]["outcome_gather"] == "rccl"
    assert "process group" in p.stderr  # bench.py logs the RCCL group it joined


def _run_bench(args, timeout=240, env=None):
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], stdout=subprocess.PIPE,
                          stderr=subprocess.PIPE, text=True, timeout=timeout, cwd=ROOT, env=env)


def _json_lines(out):
    return [json.loads(l) for l in out.splitlines() if l.strip().startswith("{")]


def test_bench_spawns_its_own_ranks():
    """`bench.py --gpus 2` with no launcher starts two rank processes itself (RANK / WORLD_SIZE /
    MASTER_ADDR), which join one process group, shard the batch and gather the outcomes to
    rank 0 (gloo here, --dry-run: nothing is simulated without a GPU)."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    p = _run_bench(["--gpus", "2", "--particles", "64", "--no-cpu-baseline", "--dry-run"], env=env)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = _json_lines(p.stdout)
    assert len(lines) == 1, p.stdout
    d = lines[0]
    assert d["n_gpus"] == 2 and d["dry_run"] is True and d["value"] is None and d["gather_verified"] is True
    assert d["config"]["particles_total"] == 128 and d["config"]["particles_per_gpu"] == 64
    assert "started 2 rank processes" in p.stderr
    assert p.stderr.count("joined the gloo process group (world size 2") == 2


def test_bench_refuses_more_gpus_than_visible():
    """--gpus N beyond the visible devices fails (non-zero), it never times fewer GPUs."""
    import torch

    n = torch.cuda.device_count()
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    p = _run_bench(["--gpus", str(n + 1), "--particles", "64", "--no-cpu-baseline", "--no-config-check"], env=env)
    assert p.returncode != 0
    assert not _json_lines(p.stdout)
    assert f"needs GPU {n}" in p.stderr


def test_bench_refuses_world_size_mismatch():
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    p = _run_bench(["--gpus", "4", "--particles", "64", "--no-cpu-baseline", "--dry-run"], env=env)
    assert p.returncode == 2 and "WORLD_SIZE=2" in p.stderr


def test_bench_takes_world_size_without_gpus_flag():
    """A launcher that starts `bench.py` without --gpus: the rank count comes from WORLD_SIZE
    (only an explicit, different --gpus is refused)."""
    import socket

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    p = _run_bench(["--particles", "64", "--no-cpu-baseline", "--dry-run"], env=env)
    assert p.returncode == 0, p.stderr[-3000:]
    assert _json_lines(p.stdout)[0]["n_gpus"] == 1


@pytest.mark.gpu
def test_bench_spawns_ranks_on_gpus():
    """The real RCCL path of `bench.py --gpus 2` (two GPUs, one rank each)."""
    import torch

    if torch.cuda.device_count() < 2:
        pytest.skip("needs 2 GPUs")
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    p = _run_bench(["--gpus", "2", "--particles", "1024", "--steps", "1", "--warmup", "1", "--no-cpu-baseline",
                    "--no-config-check"], timeout=300, env=env)
    assert p.returncode == 0, p.stderr[-3000:]
    d = _json_lines(p.stdout)[0]
    assert d["n_gpus"] == 2 and d["value"] > 0 and d["config"]["outcome_gather"] == "rccl"
    assert d["config"]["particles_total"] == 2048


def test_bench_in_process_refuses_missing_devices():
    """`--in-process` lists devices for one fks_create_multi context: a device beyond the visible
    ones fails (non-zero) before anything is timed."""
    import torch

    n = torch.cuda.device_count()
    p = _run_bench(["--in-process", "--devices", f"0,{n}", "--particles", "64", "--no-cpu-baseline"])
    assert p.returncode == 1 and not _json_lines(p.stdout)
    assert "--in-process needs devices" in p.stderr


@pytest.mark.gpu
def test_bench_in_process_line():
    """The planner drop-in's multi-device path (one process, fks_create_multi, host buffers),
    here over device 0 listed twice: two shards, one line, the same contract keys."""
    p = _run_bench(["--in-process", "--devices", "0,0", "--particles", "2048", "--steps", "1", "--warmup", "1",
                    "--no-cpu-baseline"], timeout=300)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = _json_lines(p.stdout)
    assert len(lines) == 1
    d = lines[0]
    assert d["value"] > 0 and d["n_gpus"] == 1 and d["scaling"] == "weak" and d["dtype"] == "f64"
    c = d["config"]
    assert c["mode"] == "in-process" and c["devices"] == [0, 0] and c["particles_total"] == 4096 and c["error_particles"] == 0
    assert d["statistics"]["successful_resolves"] > 0 and d["roofline"]["avg_kernel_ms"] > 0
