"""Root sharding across ranks: one process per GPU, each owning a contiguous
range of the batch's independent roots.

Roots never interact (cnode.cpp:633-641, 663-669) and tree i is seeded with
random_seed*2333 + i (cnode.cpp:574); creating each rank's batch with root_offset = its first
global root therefore reproduces the unsharded batch bit-for-bit, with no collective on the data
path.  The only collectives are the barrier / max-over-ranks of the benchmark clock and the
periodic weight broadcast (mazero_amd.weights).
"""
from __future__ import annotations

from dataclasses import replace


def shard_bounds(total_roots: int, world: int, rank: int) -> tuple[int, int]:
    """Contiguous, balanced [lo, hi) root range of `rank` (the first total % world ranks get one more)."""
    q, r = divmod(total_roots, world)
    lo = rank * q + min(rank, r)
    return lo, lo + q + (1 if rank < r else 0)


def slice_inputs(inp, lo: int, hi: int):
    """The SearchInputs of roots [lo, hi) (root arrays [B, ...], per-simulation arrays [S, B, ...])."""
    return replace(
        inp,
        B=hi - lo,
        root_reward=inp.root_reward[lo:hi],
        root_value=inp.root_value[lo:hi],
        root_policy=inp.root_policy[lo:hi],
        root_beta=inp.root_beta[lo:hi],
        root_noise=inp.root_noise[lo:hi],
        reward=inp.reward[:, lo:hi],
        value=inp.value[:, lo:hi],
        policy=inp.policy[:, lo:hi],
        beta=inp.beta[:, lo:hi],
    )


def max_over_ranks(x: float, dist, device=None) -> float:
    """Max of a host float over all ranks (the benchmark's wall clock)."""
    import torch

    if dist is None or not dist.is_initialized() or dist.get_world_size() == 1:
        return float(x)
    t = torch.tensor([float(x)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())
