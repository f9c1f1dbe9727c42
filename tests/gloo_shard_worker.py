"""One rank of the world_size-2 sharding test (tests/test_sharding.py).

Each rank simulates its contiguous particle range of a small seeded batch with the
CPU oracle (first_particle_id = range start, as the GPU ranks do), packs the
outcomes and gathers them to rank 0 over gloo with the same
fast_kinematic_simulator_amd.sharding code bench.py uses over RCCL.  Rank 0
compares the gathered batch with one unsharded run and writes a JSON verdict."""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rank", type=int, required=True)
    ap.add_argument("--world", type=int, required=True)
    ap.add_argument("--port", type=int, required=True)
    ap.add_argument("--particles", type=int, default=13)
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    import numpy as np
    import torch.distributed as dist

    import oracle
    from fast_kinematic_simulator_amd import workloads as W
    from fast_kinematic_simulator_amd.sharding import gather_outcomes, pack_outcomes, shard_bounds, unpack_outcomes

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{a.port}", rank=a.rank, world_size=a.world)
    wl = W.cfg1(a.particles / 32.0)
    env = wl.environment()
    lo, hi = shard_bounds(a.particles, a.world, a.rank)
    r = oracle.forward_simulate(env, wl.robot, wl.solver, wl.controller_frequency, wl.seed, wl.starts[lo:hi], wl.targets,
                                True, call_index=4, first_particle_id=lo, threads=1)
    packed = pack_outcomes(r["positions"], r["collided"], r["microsteps"], r["resolver_iterations"], r["error_flags"])
    full = gather_outcomes(packed, dist, a.particles, a.world, a.rank)
    if a.rank == 0:
        g = unpack_outcomes(full)
        ref = oracle.forward_simulate(env, wl.robot, wl.solver, wl.controller_frequency, wl.seed, wl.starts, wl.targets, True,
                                      call_index=4, threads=1)
        same = all(np.array_equal(np.asarray(g[k]), np.asarray(ref[k]))
                   for k in ("positions", "collided", "microsteps", "resolver_iterations", "error_flags"))
        with open(a.out, "w") as f:
            json.dump({"identical": bool(same), "rows": int(full.shape[0]),
                       "collided": int(np.asarray(ref["collided"]).sum())}, f)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
