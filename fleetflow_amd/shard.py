"""Scenario sharding for the what-if batch.

Scenarios are independent, so rank g of G plans the contiguous block
``[g*S/G, (g+1)*S/G)`` with no data-path collective.  After planning, the one
exchange is an all-gather of the packed u64 costs (``SPEC.md`` 2.4), 8 B per
scenario, over RCCL (backend ``nccl``) on the GPU box or ``gloo`` in the CPU
tests.  Every rank then holds the same cost vector and picks the same winner.
The winner's plan stays with its owner, which alone writes it.

Costs travel as int64 tensors holding the u64 bit pattern.  Blocks of unequal
size are padded with ``PAD`` (all ones, the largest u64), which never wins.
"""
from __future__ import annotations

PAD = -1  # int64 bit pattern of 0xFFFF_FFFF_FFFF_FFFF


def block(rank: int, world: int, n_scen: int) -> tuple[int, int]:
    """(first scenario id, count) of this rank's contiguous block."""
    if not 0 <= rank < world:
        raise ValueError(f"rank {rank} outside world {world}")
    lo = rank * n_scen // world
    hi = (rank + 1) * n_scen // world
    return lo, hi - lo


def owner(scenario: int, world: int, n_scen: int) -> int:
    """Rank whose block holds global scenario id ``scenario``."""
    if not 0 <= scenario < n_scen:
        raise ValueError(f"scenario {scenario} outside 0..{n_scen - 1}")
    for r in range(world):
        lo, n = block(r, world, n_scen)
        if lo <= scenario < lo + n:
            return r
    raise AssertionError("unreachable")


def gather_costs(cost_local, world: int, n_scen: int, group=None):
    """All-gather every rank's packed costs into one [n_scen] int64 tensor, in
    global scenario order (the only collective of the batch path)."""
    import torch
    import torch.distributed as dist

    width = max(block(r, world, n_scen)[1] for r in range(world))
    if cost_local.numel() == width:
        send = cost_local
    else:
        send = torch.full((width,), PAD, dtype=torch.int64, device=cost_local.device)
        send[:cost_local.numel()] = cost_local
    out = torch.empty(width * world, dtype=torch.int64, device=cost_local.device)
    dist.all_gather_into_tensor(out, send, group=group)
    if width * world == n_scen:
        return out
    parts = [out[r * width:r * width + block(r, world, n_scen)[1]] for r in range(world)]
    return torch.cat(parts)


def unpack_cost(cost: int) -> tuple[int, int, int]:
    """(n_rejected, n_nodes_used, scenario_id & 0xFFFF) of a packed cost (SPEC.md 2.4)."""
    c = cost & 0xFFFF_FFFF_FFFF_FFFF
    return c >> 40, (c >> 16) & 0xFFFFFF, c & 0xFFFF
