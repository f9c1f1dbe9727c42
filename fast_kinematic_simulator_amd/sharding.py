"""Particle sharding across GPUs (one process per GPU) and the outcome gather.

ForwardSimulateRobots (SPCS:788-804) simulates independent particles that share
only read-only inputs, so a batch splits into contiguous particle ranges with no
data-path collective.  Every rank simulates its range with
``first_particle_id`` = the range start (the counter RNG is keyed by the global
particle id, so the union of the shards is bit-identical to a single-GPU call),
then the per-particle outcomes are gathered to rank 0, where the planner consumes
them (RCCL over xGMI on MI355X; gloo in the CPU tests).

Outcome rows are packed as float64 ``[q (W) | collided | microsteps |
resolver_iterations | error_flags]``; the integers are exact in float64.
"""
from __future__ import annotations

from typing import List, Optional, Tuple

import numpy as np

OUTCOME_EXTRA = 4


def shard_bounds(n_total: int, world: int, rank: int) -> Tuple[int, int]:
    """Contiguous, balanced [lo, hi) particle range of `rank` (the first
    n_total % world ranks get one extra particle)."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError("rank must be in [0, world)")
    base, extra = divmod(int(n_total), int(world))
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


def pack_outcomes(positions, collided, microsteps, resolver_iterations, error_flags, out=None):
    """Pack one shard's outcomes into a (n, W + 4) float64 array (torch tensor or
    numpy array, matching the type of `positions`)."""
    try:
        import torch

        is_torch = isinstance(positions, torch.Tensor)
    except ImportError:  # pragma: no cover
        is_torch = False
    n, w = positions.shape
    if is_torch:
        import torch

        packed = out if out is not None else torch.empty((n, w + OUTCOME_EXTRA), dtype=torch.float64, device=positions.device)
        packed[:, :w] = positions
        for k, col in enumerate((collided, microsteps, resolver_iterations, error_flags)):
            packed[:, w + k] = col.to(torch.float64)
        return packed
    packed = out if out is not None else np.empty((n, w + OUTCOME_EXTRA), dtype=np.float64)
    packed[:, :w] = positions
    for k, col in enumerate((collided, microsteps, resolver_iterations, error_flags)):
        packed[:, w + k] = np.asarray(col, dtype=np.float64)
    return packed


def unpack_outcomes(packed) -> dict:
    """Inverse of :func:`pack_outcomes` (numpy)."""
    p = np.asarray(packed.cpu() if hasattr(packed, "cpu") else packed)
    w = p.shape[1] - OUTCOME_EXTRA
    return {
        "positions": p[:, :w].copy(),
        "collided": p[:, w] != 0.0,
        "microsteps": p[:, w + 1].astype(np.uint32),
        "resolver_iterations": p[:, w + 2].astype(np.uint32),
        "error_flags": p[:, w + 3].astype(np.uint32),
    }


def gather_outcomes(packed, dist, n_total: int, world: int, rank: int, gather_buffers: Optional[List] = None):
    """Gather every rank's packed outcomes to rank 0 and return the (n_total, W+4)
    concatenation there (None on other ranks).  Shards may differ in size by one
    particle: each is padded to the largest shard for the collective."""
    import torch

    rows = shard_bounds(n_total, world, 0)[1]  # rank 0 holds the largest shard
    lo, hi = shard_bounds(n_total, world, rank)
    t = packed if isinstance(packed, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(packed))
    if hi - lo < rows:
        pad = torch.zeros((rows - (hi - lo), t.shape[1]), dtype=t.dtype, device=t.device)
        t = torch.cat([t, pad], dim=0)
    if rank == 0:
        bufs = gather_buffers if gather_buffers is not None else [torch.empty_like(t) for _ in range(world)]
        dist.gather(t, bufs, dst=0)
        parts = []
        for r in range(world):
            a, b = shard_bounds(n_total, world, r)
            parts.append(bufs[r][: b - a])
        return torch.cat(parts, dim=0)
    dist.gather(t, None, dst=0)
    return None
