"""Discrete-event model of the kernel's segment scheduler, to reason about
scheduling policies on the CPU.  Input: per-particle, per-controller-step microsteps and
resolver iterations of a sample of cfg3 particles (the traced oracle, counter RNG = the GPU's
trajectories), written by `--profiles`; the batch is the sample resampled to n particles with
the listed heavy particles at their own indices.

Model: `slots` wave slots run tickets t = k * n + p (segment k of particle p) in order; a
segment costs sum over its steps of (a * microsteps + b * resolver_iterations) wave-time.  A
ticket whose predecessor segment is unfinished is skipped; the wave that finishes segment k
claims k + 1 if its ticket was already drawn, or at once if segment k was contact-heavy
(>= heavy * steps resolver iterations).  Issue priority and SIMD contention are not modelled.

    python tools/sched_model.py --profiles out.npz            # record (oracle, CPU)
    python tools/sched_model.py --model out.npz --heavy 2,8,14,20,28,1000000
"""
from __future__ import annotations

import argparse
import heapq
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def record(path, sample=1536, first=20000, heavy=(57934, 48094, 1036), batch=128):
    """The per-step profile of particles [first, first + sample) and of the heavy ones (each
    simulated with its own global id, so its own noise: the GPU's trajectory)."""
    import oracle
    from fast_kinematic_simulator_amd import workloads as W

    wl = W.cfg3(1.0)
    env = wl.environment()
    ids = np.concatenate([np.arange(first, first + sample), np.asarray(heavy)])
    micro = np.zeros((len(ids), wl.steps), np.int32)
    iters = np.zeros((len(ids), wl.steps), np.int32)
    chunks = [(b0, ids[b0:min(b0 + batch, sample)]) for b0 in range(0, sample, batch)]
    chunks += [(sample + j, ids[sample + j:sample + j + 1]) for j in range(len(heavy))]
    for b0, sel in chunks:
        _, buf = oracle.forward_simulate_traced(env, wl.robot, wl.solver, wl.controller_frequency, wl.seed, wl.starts[sel], wl.targets,
                                                True, config_capacity=16000, threads=os.cpu_count(), first_particle_id=int(sel[0]))
        for j in range(len(sel)):
            ns = int(buf.num_steps[j])
            micro[b0 + j, :ns] = buf.step_microsteps[j, :ns]
            tags = buf.config_tags[j, :min(int(buf.num_configs[j]), 16000)]
            m = tags[:, 2] == 1  # FKS_TRACE_RESOLVER_STEP
            np.add.at(iters[b0 + j], tags[m, 0], 1)
    np.savez(path, ids=ids, micro=micro, iters=iters, heavy=np.asarray(heavy))


def makespan(cost_steps, iters_steps, slots, seg_steps, heavy, carry_after=0):
    """cost_steps[p, s]: wave-time of step s of particle p; iters_steps: its resolver iterations.
    carry_after: heavy segments keep their wave only once that many rounds of tickets (n each)
    have been drawn (0: always)."""
    n, T = cost_steps.shape
    nseg = (T + seg_steps - 1) // seg_steps
    seg_cost = np.add.reduceat(cost_steps, np.arange(0, T, seg_steps), axis=1)
    seg_iters = np.add.reduceat(iters_steps, np.arange(0, T, seg_steps), axis=1)
    seg_len = np.diff(np.append(np.arange(0, T, seg_steps), T))
    done = np.zeros(n, np.int64)      # finished segments per particle
    running = np.zeros(n, bool)
    next_ticket = 0
    total = n * nseg
    events = []                       # (time, slot, particle, segment)
    end = np.zeros(n)
    free = list(range(slots))
    t_now = 0.0

    def draw(t):
        nonlocal next_ticket
        while next_ticket < total:
            k, p = divmod(next_ticket, n)
            next_ticket += 1
            if done[p] == k and not running[p]:
                return p, k
        return None

    def start(slot, t, p, k):
        running[p] = True
        heapq.heappush(events, (t + seg_cost[p, k], slot, p, k))

    for s in free:
        job = draw(0.0)
        if job is None:
            break
        start(s, 0.0, *job)
    while events:
        t_now, slot, p, k = heapq.heappop(events)
        running[p] = False
        done[p] = k + 1
        if k + 1 == nseg:
            end[p] = t_now
        else:
            is_heavy = seg_iters[p, k] >= heavy * seg_len[k] and next_ticket >= carry_after * n
            if is_heavy or next_ticket > (k + 1) * n + p:
                start(slot, t_now, p, k + 1)
                continue
        job = draw(t_now)
        if job is not None:
            start(slot, t_now, *job)
    return float(end.max()), float(np.median(end)), float(np.percentile(end, 99))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--profiles", default="")
    ap.add_argument("--model", default="")
    ap.add_argument("--n", type=int, default=65536)
    ap.add_argument("--slots", type=int, default=5120)
    ap.add_argument("--segments", default="14")
    ap.add_argument("--heavy", default="2,8,14,20,28,1000000")
    ap.add_argument("--b-over-a", type=float, default=3.0, help="cost of a resolver iteration in microsteps")
    ap.add_argument("--carry-after", default="0", help="comma list: rounds of tickets drawn before heavy segments keep their wave")
    a = ap.parse_args()
    if a.profiles:
        record(a.profiles)
        return
    z = np.load(a.model)
    ids, micro, iters, heavy_ids = z["ids"], z["micro"], z["iters"], z["heavy"]
    rng = np.random.default_rng(1)
    light = np.arange(len(ids) - len(heavy_ids))
    pick = rng.choice(light, a.n)
    for j, pid in enumerate(heavy_ids):
        if pid < a.n:
            pick[pid] = len(ids) - len(heavy_ids) + j
    cost = micro[pick].astype(np.float64) + a.b_over_a * iters[pick]
    cost /= cost.sum() / a.slots  # time unit: the ideal makespan (every slot busy) = 1
    rows = []
    for seg in [int(v) for v in a.segments.split(",")]:
        for h in [float(v) for v in a.heavy.split(",")]:
          for ca in [float(v) for v in a.carry_after.split(",")]:
            mk, med, p99 = makespan(cost, iters[pick], a.slots, seg, h, ca)
            rows.append({"segment_steps": seg, "heavy_per_step": h, "carry_after": ca, "makespan": round(mk, 4),
                         "median_end": round(med, 4), "p99_end": round(p99, 4)})
            print(json.dumps(rows[-1]), flush=True)


if __name__ == "__main__":
    main()
