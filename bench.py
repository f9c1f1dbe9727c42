"""Benchmark of the particle forward-simulation hot path (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N ...

`--gpus N` (N > 1) without a launcher starts the N rank processes itself (spawn_ranks);
under a launcher WORLD_SIZE must equal N.  A "step" is one ForwardSimulateRobots batch
(SPCS:788) of the headline workload cfg3 (7-DOF arm, 256^3 SDF @ 1 cm, 65,536 particles
x 200 controller steps) per GPU, inputs already resident in HBM, followed (with more than
one rank, or under a launcher) by the RCCL gather of every particle's outcome (reached
configuration, collided flag, microstep / resolver counts, error bits) to rank 0; a
single process without a launcher skips the gather and its line says so.
value = particle-microsteps executed by all ranks / max-over-ranks
wall time of the K timed steps (weak scaling: each GPU owns 65,536 particles; RNG
streams are keyed by global particle id so shards are independent).

Also reported: the dominant kernel's roofline (algorithmic SDF bytes per launch / the
launch's HIP-event duration, against the 8 TB/s HBM peak) and the CPU baseline (the
oracle, a C++ restatement of the reference's OpenMP path, timed on this host on a
bounded prefix of the same workload).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "particle-microsteps/sec, 7-DOF arm vs 256³ SDF, at 1/2/4/8 MI355X"
UNIT = "particle-microsteps/s"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak, /opt/skills/guides/MI355X_MICROARCH.md (8.0 TB/s spec)
FP64_VECTOR_PEAK_TFLOPS = 78.6  # MI355X FP64 vector peak, AMD's public spec (not in the container guide)
PARTICLES_PER_GPU = 65536
# the other BASELINE.json configs, runnable with --workload for side measurements
# (the headline line is cfg3): base particle count of the config, default per GPU, description
WORKLOADS = {
    "cfg1": (32, 32, "cfg1: SE(2) 3-DOF planar robot (64 points), 64^3 grid @ 0.0625 m, 50 controller steps"),
    "cfg2": (4096, 4096, "cfg2: 6-DOF UR5-style arm (7 links x 64 points), 128^3 SDF @ 0.02 m, 100 controller steps"),
    "cfg3": (65536, 65536, "cfg3: 7-DOF linked arm (8 links x 64 points), 256^3 SDF @ 0.01 m, 200 controller steps"),
    "cfg4": (1048576, 131072, "cfg4: SE(3) free flyer (256 points), 256^3 SDF @ 0.01 m, 100 controller steps"),
    "cfg5": (1048576, 131072, "cfg5: dual-arm 14-DOF linked robot (17 links x 64 points), 512^3 SDF @ 0.005 m, "
                              "200 controller steps"),
}
KERNELS = {0: "fks_simulate_linked", 1: "fks_simulate_se2", 2: "fks_simulate_se3"}


def log(msg):
    print(msg, file=sys.stderr, flush=True)


def host_cpu():
    """What the CPU baseline ran on: the host's logical CPUs (nproc), the ones this process
    may use (affinity), the OpenMP thread count and the lscpu model string."""
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        affinity = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        affinity = None
    return {"nproc": os.cpu_count(), "affinity_cpus": affinity, "omp_num_threads_env": os.environ.get("OMP_NUM_THREADS"),
            "model": model}


def cpu_baseline(wl, sample_particles: int):
    """The oracle in reference-RNG mode (per-OpenMP-thread mt19937_64, SPCS:431-441,
    #pragma omp parallel for over particles, SPCS:795) on a prefix of the batch, with
    every OpenMP thread the process is given (OMP_NUM_THREADS: 16 on the GPU box, its CPU
    share per GPU).  The particle loop is embarrassingly parallel, so the per-core rate
    is reported too."""
    import oracle

    threads = int(oracle.lib().oracle_max_threads())
    env = wl.environment()
    starts = wl.starts[:sample_particles]
    t0 = time.perf_counter()
    r = oracle.forward_simulate(env, wl.robot, wl.solver, wl.controller_frequency, wl.seed, starts, wl.targets, True,
                                rng_mode=oracle.RNG_REFERENCE, threads=threads)
    dt = time.perf_counter() - t0
    micro = int(r["counters"]["microsteps"])
    return {"value": micro / dt, "unit": UNIT, "cores": threads, "kind": "port", "per_core": micro / dt / threads,
            "host": host_cpu(),
            "sample": f"first {len(starts)} particles of {wl.name} x {wl.steps} controller steps ({micro} microsteps, "
                      f"{dt:.1f} s), oracle in reference-RNG mode (per-check robot clones, hash-map self-collision, "
                      f"dynamic-matrix QR as SPCS), OpenMP {threads} threads"}


def fp64_algorithmic_flops(robot, counters):
    """FP64 flops the reference's algorithm performs for the counted work:
    per microstep the FK (145 per moving joint: angle-axis matrix 19 + two 3x4 compositions
    63 each; 63 per fixed joint) and, for every point, the environment check (45: link
    transform 21, inverse grid origin 21, scaling 3) and the self-collision key (45,
    SPCS:1202-1236); per controller step two FKs and two workspace-motion maxima (50 per
    point); per resolver iteration a Jacobian (12 per point and dof, SPCS:1858), the
    distance estimate (45 per point), one FK and a motion maximum; per least-squares row
    2 D^2 for the Householder QR (SPCS:1994)."""
    P, D = robot.num_points, robot.num_dofs
    J = len(robot.joints)
    fk = 145 * D + 63 * (J - D) if robot.robot_type == 0 else 63
    return (counters["microsteps"] * (fk + 90 * P) + counters["controller_steps"] * (2 * fk + 100 * P)
            + counters["resolver_iterations"] * (P * (95 + 12 * D) + fk) + 2 * D * D * counters["least_squares_rows"])


def config_check_bench(sim, wl, dev, n=1 << 20, reps=3, cpu_sample=16384, threads=16, with_cpu=True):
    """Batched CheckConfigCollision (SPCS:1398-1416) on the cfg3 arm:
    n configurations uniform in the joint limits, inflation ratio 0.5, inputs in HBM.
    Reported beside the headline metric (not part of it)."""
    import numpy as np
    import torch

    lo, hi = wl.robot.dof_limits()
    rng = np.random.default_rng(21)
    cfgs = rng.uniform(lo, hi, size=(n, wl.robot.config_width))
    d_cfg = torch.from_numpy(cfgs).to(dev)
    d_out = torch.empty(n, dtype=torch.uint8, device=dev)
    stream = torch.cuda.current_stream(dev)
    sim.check_config_collisions_device(wl.robot, d_cfg.data_ptr(), n, 0.5, d_out.data_ptr(), stream=stream.cuda_stream,
                                       synchronize=True)
    ms = []
    for _ in range(reps):
        sim.check_config_collisions_device(wl.robot, d_cfg.data_ptr(), n, 0.5, d_out.data_ptr(), stream=stream.cuda_stream,
                                           synchronize=True)
        ms.append(sim.last_check_counters()["kernel_ms"])
    c = sim.last_check_counters()
    kernel_s = sum(ms) / len(ms) / 1e3
    out = {"metric": "configurations checked/s (batched CheckConfigCollision, cfg3 arm, 256^3 SDF, inflation 0.5)",
           "value": n / kernel_s, "unit": "configs/s", "configs": n, "kernel_ms": kernel_s * 1e3,
           "collided_fraction": float(d_out.float().mean().item()),
           "roofline": {"bound": "hbm", "achieved": c["sdf_bytes"] / kernel_s / 1e9, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": c["sdf_bytes"] / kernel_s / 1e9 / HBM_PEAK_GBS,
                        "algorithmic_bytes_per_launch": c["sdf_bytes"]}}
    if with_cpu:
        import oracle

        t0 = time.perf_counter()
        oracle.check_config_collision(wl.environment(), wl.robot, wl.solver, cfgs[:cpu_sample], 0.5, threads=threads)
        dt = time.perf_counter() - t0
        out["cpu_baseline"] = {"value": cpu_sample / dt, "unit": "configs/s", "cores": threads, "kind": "port",
                               "sample": f"first {cpu_sample} configurations, oracle CheckConfigCollision, OpenMP {threads} threads"}
    return out


def kernel_name(kind: str, robot_type: int, spec) -> str:
    """The simulation kernel the last timed launch ran (fks_get_launch_info's last_kernel),
    not the one the flags asked for."""
    if kind in ("shaped", "shaped_small_batch"):
        name = "fks_simulate_shaped" if kind == "shaped" else "fks_simulate_shaped_small"
        return name + " (" + (spec["shape"] if spec else "?") + ")"
    base = KERNELS.get(robot_type, "fks_simulate")
    return {"throughput": base, "small_batch": base + "_small", "cooperative": base + "_coop"}.get(kind, f"{base} ({kind})")


def kernel_source_sha16() -> str:
    """The hash tools/profile_pmc.py records: the kernel source and the headers it includes."""
    import hashlib

    from fast_kinematic_simulator_amd import build

    h = hashlib.sha256()
    for name, rel in build.EMBEDDED:
        h.update(name.encode() + b"\0")
        with open(os.path.join(build.PKG, rel), "rb") as f:
            h.update(f.read())
    return h.hexdigest()[:16]


def load_traffic(kernel: str):
    """HBM bytes per launch of the simulation kernel and the L2 hit rate from the committed
    rocprofv3 PMC summary (profiles/latest_pmc.json, written by tools/profile_pmc.py from
    separate FETCH_SIZE / WRITE_SIZE / TCC_HIT+MISS passes of this bench), or Nones.  It is
    the builder's profile of the same command, not a measurement of this run, so it is used
    only when the profile names the kernel (and shape) this run's timed launches ran."""
    path = os.path.join(ROOT, "profiles", "latest_pmc.json")
    if not os.path.exists(path):
        return None, None, None
    try:
        with open(path) as f:
            d = json.load(f)
        if d.get("kernel") != kernel:
            return None, None, (f"profiles/latest_pmc.json profiles {d.get('kernel')!r}, this run ran {kernel!r}: "
                                "traffic not quoted")
        sha = kernel_source_sha16()
        if d.get("kernel_source_sha16") != sha:
            return None, None, (f"profiles/latest_pmc.json profiles kernel sources {d.get('kernel_source_sha16')}, this tree's "
                                f"are {sha}: traffic not quoted")
        src = d.get("source", "profiles/latest_pmc.json")
        if d.get("note"):
            src = src + "; " + d["note"]
        return float(d["hbm_bytes_per_launch"]), d.get("l2_hit_rate"), src
    except Exception:
        return None, None, None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None, help="GPUs (ranks); default: WORLD_SIZE under a launcher, else 1")
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--workload", default="cfg3", choices=sorted(WORKLOADS),
                    help="BASELINE.json config (the headline metric is cfg3)")
    ap.add_argument("--particles", type=int, default=0, help="particles per GPU (default: the workload's)")
    ap.add_argument("--cpu-sample", type=int, default=4096, help="particles in the CPU-baseline sample (SURVEY §8d: 4096)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-config-check", action="store_true", help="skip the batched CheckConfigCollision line")
    ap.add_argument("--segment-steps", type=int, default=-1, help="A/B: fks_set_segment_steps (default: automatic)")
    ap.add_argument("--no-contacts", action="store_true",
                    help="A/B only: allow_contacts = false (particles stop at their first contact; no resolver)")
    ap.add_argument("--pipeline-batches", type=int, default=6,
                    help="one GPU: also time this many batches alternated over two contexts on two streams, so a "
                         "batch's tail overlaps the next batch's start (reported beside `value`, never as it; 0: off)")
    ap.add_argument("--specialize", choices=("on", "off"), default="on",
                    help="run the robot's shape-specialised kernel (fks_set_specialization: compiled at setup, outside the "
                         "timed region; results identical) or the generic one")
    ap.add_argument("--in-process", action="store_true",
                    help="one process driving --gpus devices through fks_create_multi: the planner drop-in's path "
                         "(HipParticleContactSimulator / MultiDeviceSimulator), host buffers in and out, as a planner's "
                         "ForwardSimulateRobots call gets it; no launcher, no collective")
    ap.add_argument("--devices", default=None, help="--in-process: comma-separated device ids (default 0..gpus-1; "
                                                      "a device may repeat)")
    ap.add_argument("--no-projection", action="store_true",
                    help="skip the strong-scaling projection (the batch's 2/4/8-way shards timed alone on this GPU)")
    ap.add_argument("--dry-run", action="store_true",
                    help="launcher / rendezvous / shard / gather check without a GPU (gloo): no simulation, value null")
    args = ap.parse_args()
    if args.gpus is None:
        args.gpus = int(os.environ.get("WORLD_SIZE", "1"))
    if args.gpus < 1:
        log("--gpus must be >= 1")
        return 2
    if args.in_process:
        return in_process(args)
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # no external launcher: start one rank process per GPU before anything touches a GPU
        return spawn_ranks(args.gpus)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        log(f"--gpus {args.gpus} but the launcher started WORLD_SIZE={world} ranks")
        return 2
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    import numpy as np
    import torch

    if args.dry_run:
        return dry_run(args, world, rank)
    if torch.cuda.device_count() <= local_rank:
        log(f"[rank {rank}] needs GPU {local_rank}, {torch.cuda.device_count()} visible")
        return 1
    torch.cuda.set_device(local_rank)
    dist = None
    # under a launcher (RANK/MASTER_ADDR set) the RCCL process group is used even at
    # world size 1, so the launched path is the one the multi-GPU runs take
    if world > 1 or ("RANK" in os.environ and "MASTER_ADDR" in os.environ):
        import torch.distributed as dist

        dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
        log(f"[rank {rank}] joined the RCCL process group (world size {world})")

    from fast_kinematic_simulator_amd import make_linked_simulator
    from fast_kinematic_simulator_amd import workloads as W

    from fast_kinematic_simulator_amd._capi import PHASE_COUNTS
    from fast_kinematic_simulator_amd.sharding import gather_outcomes, pack_outcomes, shard_bounds

    base, per_gpu, workload_desc = WORKLOADS[args.workload]
    n_total = (args.particles or per_gpu) * world
    lo, hi = shard_bounds(n_total, world, rank)
    n_local = hi - lo
    wl = W.WORKLOADS[args.workload](scale=n_total / float(base))
    t0 = time.perf_counter()
    env_stats = {}
    # the environment is built on this rank's GPU and handed to the simulator there
    # (fks_env_build_device + fks_create_from_device_env: the host build's bytes)
    denv = W.SCENES[args.workload](device=local_rank, stats=env_stats, resident=True)
    log(f"[rank {rank}] environment {env_stats['cells']} cells built on the GPU in {env_stats['gpu_ms']:.1f} ms device "
        f"time ({time.perf_counter() - t0:.2f}s call, {env_stats['normal_entries']} surface-normal entries)")
    sim = make_linked_simulator(denv, wl.solver, wl.controller_frequency, wl.seed, device=local_rank)
    if args.segment_steps >= 0:
        sim.set_segment_steps(args.segment_steps)
    sim.set_robot(wl.robot)
    spec = None
    if args.specialize == "on":
        t0 = time.perf_counter()
        sim.set_specialization(True)
        spec = sim.specialization()
        log(f"[rank {rank}] shape-specialised kernel {spec['shape']}: "
            + (f"compiled in {spec['compile_seconds']:.1f}s" if not spec["from_cache"] else "from the kernel cache")
            + f" ({time.perf_counter() - t0:.1f}s setup)")
    else:
        # the library specialises by default (lazily, at the first throughput launch): the
        # generic-kernel A/B leg has to switch it off, or it would time the shaped kernel
        sim.set_specialization(False)
    Wd = wl.robot.config_width
    dev = torch.device("cuda", local_rank)
    starts = torch.from_numpy(np.ascontiguousarray(wl.starts[lo:lo + n_local])).to(dev)
    targets = torch.from_numpy(np.ascontiguousarray(wl.targets)).to(dev)
    out_q = torch.empty((n_local, Wd), dtype=torch.float64, device=dev)
    out_coll = torch.empty(n_local, dtype=torch.uint8, device=dev)
    out_micro = torch.empty(n_local, dtype=torch.int32, device=dev)
    out_res = torch.empty(n_local, dtype=torch.int32, device=dev)
    out_err = torch.empty(n_local, dtype=torch.int32, device=dev)
    packed = torch.empty((n_local, Wd + 4), dtype=torch.float64, device=dev)
    gathered = [torch.empty_like(packed) for _ in range(world)] if (dist is not None and rank == 0) else None
    micro_total = torch.zeros((), dtype=torch.int64, device=dev)
    stream = torch.cuda.current_stream(dev)

    def step(call_index, timed_events=None):
        # every rank uses the same RNG call index for the same logical batch
        sim.set_call_index(call_index)
        if timed_events is not None:
            timed_events[0].record(stream)
        sim.forward_simulate_device(wl.robot, starts.data_ptr(), n_local, targets.data_ptr(), 1, lo, not args.no_contacts,
                                    out_q.data_ptr(), out_coll.data_ptr(), out_micro.data_ptr(), out_res.data_ptr(),
                                    out_err.data_ptr(), stream=stream.cuda_stream, synchronize=False)
        if timed_events is not None:
            timed_events[1].record(stream)
        micro_total.add_(out_micro.sum(dtype=torch.int64))
        # outcome of every particle -> rank 0 (RCCL gather over xGMI)
        pack_outcomes(out_q, out_coll, out_micro, out_res, out_err, out=packed)
        if dist is not None:
            gather_outcomes(packed, dist, n_total, world, rank, gathered)

    for w in range(args.warmup):
        step(1000 + w)
    torch.cuda.synchronize()
    sim.reset_total_counters()
    micro_total.zero_()
    spec_before = sim.specialization()["launches"] if spec else 0
    events = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    t_start = time.perf_counter()
    for k in range(args.steps):
        step(k, events[k])
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t_start
    kernel_ms = [a.elapsed_time(b) for a, b in events]
    ran_kernel = sim.launch_info()["last_kernel"]  # what the last timed launch actually ran
    tot = sim.total_counters()
    spec_launches = (sim.specialization()["launches"] - spec_before) if spec else 0
    phases = sim.phase_cycles(total=True)
    geom = sim.launch_geometry()
    local_micro = int(micro_total.item())
    assert local_micro == int(tot["microsteps"]), (local_micro, tot["microsteps"])
    stats = sim.get_statistics()  # this rank's SimpleParticleContactSimulator counters (SPCS:488-500)
    stat_names = sorted(stats)
    if dist is not None:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        m = torch.tensor([local_micro], dtype=torch.int64, device=dev)
        dist.all_reduce(m)
        all_micro = int(m.item())
        # GetStatistics of the whole job: every rank's counters summed (RCCL all-reduce)
        st = torch.tensor([stats[k] for k in stat_names], dtype=torch.float64, device=dev)
        dist.all_reduce(st)
        stats = {k: float(v) for k, v in zip(stat_names, st.tolist())}
    else:
        all_micro = local_micro

    if rank == 0:
        calls = max(1, int(tot["calls"]))
        avg_kernel_s = (sum(kernel_ms) / len(kernel_ms)) / 1e3
        bytes_per_launch = tot["sdf_bytes"] / calls
        achieved = bytes_per_launch / avg_kernel_s / 1e9
        traffic, l2_hit, traffic_src = (load_traffic(kernel_name(ran_kernel, wl.robot.robot_type, spec))
                                        if args.workload == "cfg3" else (None, None, None))  # cfg3 profile
        per_launch = {k: tot[k] / calls for k in ("microsteps", "controller_steps", "resolver_iterations", "least_squares_rows")}
        flops = fp64_algorithmic_flops(wl.robot, per_launch)
        cpu = None
        if not args.no_cpu_baseline:
            t0 = time.perf_counter()
            sample = min(args.cpu_sample, n_total)
            cwl = W.WORKLOADS[args.workload](scale=sample / float(base))
            cwl._env = denv.download()
            cpu = cpu_baseline(cwl, sample)
            log(f"cpu baseline {cpu['value']:.0f} {UNIT} in {time.perf_counter() - t0:.1f}s")
        value = all_micro / elapsed
        # the host-buffer entry (fks_forward_simulate: starts/targets over PCIe, outcomes
        # back) on the same batch: reported beside `value`, never as it
        sim.set_call_index(0)
        t0 = time.perf_counter()
        hr = sim.forward_simulate_arrays(wl.robot, wl.starts[lo:lo + n_local], wl.targets, True)
        host_s = time.perf_counter() - t0
        pcie = {"value": float(np.sum(hr["microsteps"], dtype=np.int64)) / host_s, "unit": UNIT, "ms": host_s * 1e3,
                "note": "one fks_forward_simulate call with host buffers (H2D starts/targets, kernel, D2H outcomes), rank 0"}
        pipe = None
        if world == 1 and not args.no_contacts:
            try:
                pipe = pipelined_batches(sim, denv, wl, dev, starts, targets, n_local, lo, args.pipeline_batches)
            except Exception as e:  # a side figure: never costs the headline line
                pipe = {"value": None, "error": f"{type(e).__name__}: {e}"}
        if pipe and pipe.get("value"):
            log(f"pipelined: {pipe['value']:.4e} {UNIT}, {pipe['ms_per_batch']:.1f} ms per batch, identical={pipe['identical_to_sequential']}")
        proj = None
        if world == 1 and not args.no_contacts and not args.no_projection:
            try:
                proj = strong_scaling_projection(sim, wl, dev, n_local, lo)
                log("strong-scaling projection: " + ", ".join(f"{r['devices']} dev {r['slowest_shard_ms']:.1f} ms "
                                                               f"(x{r['projected_speedup']:.2f})" for r in proj["rows"]))
            except Exception as e:  # a side figure: never costs the headline line
                proj = {"error": f"{type(e).__name__}: {e}"}
        cc = None
        if not args.no_config_check and args.workload == "cfg3":
            if not args.no_cpu_baseline:
                wl._env = denv.download()  # the oracle's CPU baseline reads the host copy
            cc = config_check_bench(sim, wl, dev, with_cpu=not args.no_cpu_baseline)
            log(f"config check {cc['value']:.3e} configs/s")
        line = {
            "metric": METRIC,
            "value": value,
            "unit": UNIT,
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": f"synthetic (seeded {args.workload} scene and start perturbations, workloads.py)",
            "config": {
                "workload": f"{workload_desc}, {n_local} particles per GPU, "
                            + ("allow_contacts = false (A/B only)" if args.no_contacts else "allow_contacts")
                            + (f", RCCL gather of outcomes to rank 0 over {world} ranks" if dist is not None else
                               ", one process (no gather: outcomes stay on this GPU)"),
                "outcome_gather": "rccl" if dist is not None else None,
                "particles_per_gpu": n_local,
                "particles_total": n_local * world,
                "controller_steps": wl.steps,
                "parallelism": f"dp{world} (particle shards)",
                "microsteps_per_step": all_micro / args.steps,
                "mean_microsteps_per_controller_step": tot["microsteps"] / max(1, tot["controller_steps"]),
                "resolver_iterations_per_step": tot["resolver_iterations"] / calls * world,
                "mean_least_squares_rows": tot["least_squares_rows"] / max(1, tot["resolver_iterations"]),
                "error_particles": tot["error_particles"],
            },
            "roofline": {
                "bound": "hbm",
                "achieved": achieved,
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBS,
                "traffic": traffic,
                "traffic_source": traffic_src,
                "l2_hit_rate": l2_hit,
                "kernel": kernel_name(ran_kernel, wl.robot.robot_type, spec),
                "kernel_kind": ran_kernel,
                "avg_kernel_ms": avg_kernel_s * 1e3,
                "algorithmic_bytes_per_launch": bytes_per_launch,
                # second entry: the kernel is FP64-VALU- and latency-bound, not HBM-bound
                "fp64": {"bound": "valu", "achieved": flops / avg_kernel_s / 1e12, "peak": FP64_VECTOR_PEAK_TFLOPS,
                         "unit": "TFLOP/s", "frac": flops / avg_kernel_s / 1e12 / FP64_VECTOR_PEAK_TFLOPS,
                         "algorithmic_flops_per_launch": flops},
            },
            "statistics": stats,
            # share of the persistent grid's wave slots that held a particle during the timed
            # launches (1.0 = no tail): wave residency in 100 MHz s_memrealtime ticks
            "wave_slots": {"resident_waves": geom["resident_waves"],
                           "busy_fraction": phases["wave_residency"] / 1e5 / max(1e-9, geom["resident_waves"] * sum(kernel_ms))},
            "cpu_baseline": cpu,
            # the robot-shape-specialised kernel (fks_set_specialization): compiled by hiprtc at
            # setup, before the warm-up; every timed launch ran it
            "specialization": ({"shape": spec["shape"], "compile_seconds": spec["compile_seconds"],
                                "from_cache": bool(spec["from_cache"]), "timed_launches": spec_launches,
                                "all_timed_launches": spec_launches == args.steps} if spec else None),
            "config_check": cc,
            "pcie_inclusive": pcie,
            "pipelined": pipe,
            # a fixed batch split over G devices, each shard timed alone on this GPU
            "strong_scaling_projection": proj,
            # share of wave time per phase of the hot path (s_memtime cycle sums, rank 0)
            # (only in profiling builds of the library: -DFKS_PHASE_TIMERS=1, see tools/variant_bench.py)
            "kernel_phases": ({k: (v if k in PHASE_COUNTS else round(v / max(1, phases["particle"]), 4))
                               for k, v in phases.items() if k not in ("particle", "wave_residency")}
                              if phases.get("control", 0) > 0 else None),
        }
        print(json.dumps(line), flush=True)
    sim.close()
    denv.close()
    if dist is not None:
        dist.barrier()  # rank 0 ran the CPU baseline and the config-check line after the timed region
        dist.destroy_process_group()
    return 0


def pipelined_batches(sim, denv, wl, dev, starts, targets, n, first_id, batches):
    """Consecutive batches alternated over two contexts (each with its own workspace) on two
    streams: the persistent grid of batch k + 1 takes the wave slots batch k frees during its
    tail, so the machine stays busy across batches.  Each batch is the full hot path over
    the same particles with its own RNG call index; the last batch's outcomes are compared
    bit for bit with a sequential call at that index.  Reported beside `value`, never as it:
    one batch's latency is still the kernel time of the sequential run."""
    import torch

    if batches < 2:
        return None
    from fast_kinematic_simulator_amd import make_linked_simulator

    sim2 = make_linked_simulator(denv, wl.solver, wl.controller_frequency, wl.seed, device=dev.index)
    sim2.set_robot(wl.robot)
    # the same kernel as the first context (the process cache holds the shaped code object)
    sim2.set_specialization(bool(sim.specialization()["active"]))
    sims = (sim, sim2)
    streams = (torch.cuda.Stream(dev), torch.cuda.Stream(dev))
    W = wl.robot.config_width

    def outs():
        return (torch.empty((n, W), dtype=torch.float64, device=dev), torch.empty(n, dtype=torch.uint8, device=dev),
                torch.empty(n, dtype=torch.int32, device=dev), torch.empty(n, dtype=torch.int32, device=dev),
                torch.empty(n, dtype=torch.int32, device=dev))

    bufs = (outs(), outs())
    totals = (torch.zeros((), dtype=torch.int64, device=dev), torch.zeros((), dtype=torch.int64, device=dev))

    def launch(k, call_index):
        j = k % 2
        q, c, m, r, e = bufs[j]
        sims[j].set_call_index(call_index)
        sims[j].forward_simulate_device(wl.robot, starts.data_ptr(), n, targets.data_ptr(), 1, first_id, True, q.data_ptr(),
                                        c.data_ptr(), m.data_ptr(), r.data_ptr(), e.data_ptr(), stream=streams[j].cuda_stream,
                                        synchronize=False)
        with torch.cuda.stream(streams[j]):
            totals[j].add_(m.sum(dtype=torch.int64))

    for k in range(2):
        launch(k, 2000 + k)
    torch.cuda.synchronize()
    for t in totals:
        t.zero_()
    t0 = time.perf_counter()
    for k in range(batches):
        launch(k, k)
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    micro = int(totals[0].item() + totals[1].item())
    # the last batch again, alone on the first context: the same outcomes bit for bit
    last = bufs[(batches - 1) % 2]
    ref = outs()
    sim.set_call_index(batches - 1)
    sim.forward_simulate_device(wl.robot, starts.data_ptr(), n, targets.data_ptr(), 1, first_id, True, ref[0].data_ptr(),
                                ref[1].data_ptr(), ref[2].data_ptr(), ref[3].data_ptr(), ref[4].data_ptr(),
                                stream=torch.cuda.current_stream(dev).cuda_stream, synchronize=True)
    torch.cuda.synchronize()
    same = all(bool(torch.equal(a, b)) for a, b in zip(last, ref))
    sim2.close()
    return {"value": micro / elapsed, "unit": UNIT, "ms_per_batch": elapsed / batches * 1e3, "batches": batches,
            "contexts": 2, "streams": 2, "identical_to_sequential": same,
            "note": "throughput of back-to-back batches whose tails overlap the next batch's start (two contexts, two "
                    "streams, fks_forward_simulate_device without synchronisation); `value` above is the one-stream figure"}


def strong_scaling_projection(sim, wl, dev, n, first_id=0, groups=(1, 2, 4, 8), call_index=0):
    """What one GPU can say about strong scaling a fixed batch (the planner's regime: one
    ForwardSimulateRobots call of n particles, SPCS:795-802) over G devices: the batch split as
    fks_shard_bounds splits it, every shard run alone on this GPU with its own first particle
    id (so each shard's particles are exactly those of the whole batch, the same trajectories),
    and the projected time on G devices = the slowest shard's kernel time.  speedup = T(n) /
    that.  A projection, not a measurement: it leaves out the per-device host staging and any
    interference between devices, and no multi-GPU run backs it."""
    import numpy as np
    import torch

    from fast_kinematic_simulator_amd.sharding import shard_bounds

    W = wl.robot.config_width
    d_starts = torch.from_numpy(np.ascontiguousarray(wl.starts[first_id:first_id + n])).to(dev)
    d_targets = torch.from_numpy(np.ascontiguousarray(wl.targets)).to(dev)
    out = torch.empty((n, W), dtype=torch.float64, device=dev)
    micro = torch.empty(n, dtype=torch.int32, device=dev)

    def shard_ms(lo, hi):
        k = hi - lo
        sim.set_call_index(call_index)
        sim.forward_simulate_device(wl.robot, d_starts[lo:].data_ptr(), k, d_targets.data_ptr(), 1, first_id + lo, True,
                                    out[lo:].data_ptr(), d_out_microsteps=micro[lo:].data_ptr(), synchronize=True)
        return sim.last_call_counters()["kernel_ms"], sim.launch_info()["last_kernel"]

    rows = []
    t1 = None
    for G in groups:
        times, kinds = [], set()
        for g in range(G):
            lo, hi = shard_bounds(n, G, g)
            ms, kind = shard_ms(lo, hi)
            times.append(ms)
            kinds.add(kind)
        t = max(times)
        if G == 1:
            t1 = t
        rows.append({"devices": G, "particles_per_device": n // G, "slowest_shard_ms": t, "mean_shard_ms": sum(times) / G,
                     "projected_speedup": t1 / t, "projected_efficiency": t1 / t / G, "kernels": sorted(kinds)})
    return {"particles": n, "rows": rows,
            "note": "each shard of the batch run alone on one GPU (same particle ids, same trajectories); projected time on G "
                    "devices = the slowest shard's kernel time; excludes host staging and inter-device effects; no multi-GPU "
                    "run measured it"}


def in_process(args) -> int:
    """`--in-process`: the planner drop-in's multi-device path timed as a planner sees it.  One
    process, one fks_create_multi context over the devices (Make*Simulator's default device list
    is every visible device); each step is one fks_multi_forward_simulate call on host arrays
    (starts H2D, the shards' kernels concurrently on their devices' streams, outcomes D2H into
    the caller's arrays), so `value` includes the PCIe copies, unlike the launcher path's
    device-resident `value`.  Weak scaling: 65,536 cfg3 particles per listed device, sharded
    contiguously by global particle id; every device runs the shape-specialised kernel."""
    import numpy as np
    import torch

    from fast_kinematic_simulator_amd import workloads as W
    from fast_kinematic_simulator_amd.simulator import MultiDeviceSimulator

    devices = [int(d) for d in args.devices.split(",")] if args.devices else list(range(args.gpus))
    visible = torch.cuda.device_count()
    if not devices or max(devices) >= visible or min(devices) < 0:
        log(f"--in-process needs devices {devices}, {visible} visible")
        return 1
    ndev = len(devices)
    base, per_gpu, workload_desc = WORKLOADS[args.workload]
    n_total = (args.particles or per_gpu) * ndev
    wl = W.WORKLOADS[args.workload](scale=n_total / float(base))
    t0 = time.perf_counter()
    env_stats = {}
    denv = W.SCENES[args.workload](device=devices[0], stats=env_stats, resident=True)
    henv = denv.download()  # the planner hands the simulator a host environment
    log(f"environment built on device {devices[0]} and downloaded in {time.perf_counter() - t0:.2f}s")
    sim = MultiDeviceSimulator(henv, wl.solver, wl.controller_frequency, wl.seed, devices)
    sim.set_robot(wl.robot)
    starts = np.ascontiguousarray(wl.starts[:n_total])
    for w in range(args.warmup):  # the first call builds each device's shape-specialised kernel
        sim.set_call_index(1000 + w)
        sim.forward_simulate_arrays(wl.robot, starts, wl.targets, not args.no_contacts)
    micro = 0
    kernel_ms = []
    totals = {k: 0 for k in ("calls", "sdf_bytes", "microsteps", "controller_steps", "resolver_iterations", "least_squares_rows",
                             "error_particles")}
    t_start = time.perf_counter()
    for k in range(args.steps):
        sim.set_call_index(k)
        r = sim.forward_simulate_arrays(wl.robot, starts, wl.targets, not args.no_contacts)
        micro += int(np.sum(r["microsteps"], dtype=np.int64))
        c = sim.last_call_counters()
        kernel_ms.append(c["kernel_ms"])
        for key in totals:
            totals[key] += c[key] if key != "calls" else 1
    elapsed = time.perf_counter() - t_start
    assert micro == totals["microsteps"], (micro, totals["microsteps"])
    avg_kernel_s = sum(kernel_ms) / len(kernel_ms) / 1e3
    bytes_per_device_launch = totals["sdf_bytes"] / totals["calls"] / ndev
    achieved = bytes_per_device_launch / avg_kernel_s / 1e9
    proj = None
    if not args.no_projection and not args.no_contacts:
        # the planner's fixed batch of one device's size, split as the multi-device path would
        # split it, every shard timed alone on devices[0]
        from fast_kinematic_simulator_amd import make_linked_simulator

        one = make_linked_simulator(henv, wl.solver, wl.controller_frequency, wl.seed, device=devices[0])
        one.set_robot(wl.robot)
        one.set_specialization(True)
        proj = strong_scaling_projection(one, wl, torch.device("cuda", devices[0]), n_total // ndev, 0)
        one.close()
    cpu = None
    if not args.no_cpu_baseline:
        sample = min(args.cpu_sample, n_total)
        cwl = W.WORKLOADS[args.workload](scale=sample / float(base))
        cwl._env = henv
        cpu = cpu_baseline(cwl, sample)
    line = {
        "metric": METRIC, "value": micro / elapsed, "unit": UNIT, "n_gpus": len(set(devices)), "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "f64",
        "data": f"synthetic (seeded {args.workload} scene and start perturbations, workloads.py)",
        "config": {
            "workload": f"{workload_desc}, {n_total // ndev} particles per listed device, "
                        + ("allow_contacts = false (A/B only)" if args.no_contacts else "allow_contacts")
                        + f", one process over devices {devices} (fks_create_multi, host buffers: PCIe included)",
            "mode": "in-process", "devices": devices, "particles_per_gpu": n_total // ndev, "particles_total": n_total,
            "controller_steps": wl.steps, "parallelism": f"in-process x{ndev} (particle shards, no collective)",
            "microsteps_per_step": micro / args.steps,
            "mean_microsteps_per_controller_step": totals["microsteps"] / max(1, totals["controller_steps"]),
            "resolver_iterations_per_step": totals["resolver_iterations"] / args.steps,
            "error_particles": totals["error_particles"],
        },
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS,
                     "traffic": None, "kernel": "fks_simulate_shaped (per device)", "avg_kernel_ms": avg_kernel_s * 1e3,
                     "note": "per device: algorithmic bytes of one shard's launch / the slowest shard's kernel time"},
        "statistics": sim.get_statistics(),
        "cpu_baseline": cpu,
        "strong_scaling_projection": proj,
        "active_devices": sim.active_devices(),
    }
    print(json.dumps(line), flush=True)
    sim.close()
    denv.close()
    return 0


def spawn_ranks(n: int) -> int:
    """`bench.py --gpus N` without a launcher: N child processes of this script, rank r on
    GPU r (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR=127.0.0.1 / MASTER_PORT), the same
    RCCL path torch.distributed.run gives.  No GPU is touched here; only rank 0 prints the
    line.  Any failed rank fails the run (the others are stopped by PID)."""
    import socket
    import subprocess

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__), *sys.argv[1:]], env=env))
    log(f"started {n} rank processes (MASTER_PORT {port})")
    rc = 0
    pending = list(procs)
    while pending:
        for p in list(pending):
            code = p.poll()
            if code is None:
                continue
            pending.remove(p)
            if code != 0 and rc == 0:
                rc = code if code > 0 else 1
                log(f"rank process {procs.index(p)} exited with {code}: stopping the others")
                for q in pending:
                    q.terminate()
        time.sleep(0.05)
    return rc


def dry_run(args, world: int, rank: int) -> int:
    """The multi-process plumbing without a GPU (CPU tests): gloo process group, this rank's
    shard of the batch, the outcome gather to rank 0 (each row carries its global particle id,
    so rank 0 checks that the concatenation is the whole batch in order), max-over-ranks
    timing.  Nothing is simulated: the line says so and its value is null."""
    import torch
    import torch.distributed as dist

    from fast_kinematic_simulator_amd.sharding import OUTCOME_EXTRA, gather_outcomes, shard_bounds

    base, per_gpu, workload_desc = WORKLOADS[args.workload]
    n_total = (args.particles or per_gpu) * world
    lo, hi = shard_bounds(n_total, world, rank)
    dist.init_process_group("gloo")
    log(f"[rank {rank}] joined the gloo process group (world size {world}, dry run)")
    W = 7
    packed = torch.zeros((hi - lo, W + OUTCOME_EXTRA), dtype=torch.float64)
    packed[:, 0] = torch.arange(lo, hi, dtype=torch.float64)
    dist.barrier()
    t0 = time.perf_counter()
    full = gather_outcomes(packed, dist, n_total, world, rank)
    dist.barrier()
    t = torch.tensor([time.perf_counter() - t0], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    ok = True
    if rank == 0:
        ok = full.shape[0] == n_total and bool(torch.equal(full[:, 0], torch.arange(n_total, dtype=torch.float64)))
        print(json.dumps({"metric": METRIC, "value": None, "unit": UNIT, "n_gpus": world, "steps": 0, "warmup": 0,
                          "dry_run": True, "gather_verified": ok, "gather_ms": float(t.item()) * 1e3,
                          "config": {"workload": f"{workload_desc}: dry run, nothing simulated",
                                     "particles_per_gpu": hi - lo, "particles_total": n_total,
                                     "parallelism": f"dp{world} (particle shards)", "outcome_gather": "gloo"}}), flush=True)
    dist.destroy_process_group()
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
