"""Scenario sharding for the what-if batch.

Scenarios are independent, so rank g of G plans the contiguous block
``[g*S/G, (g+1)*S/G)`` with no data-path collective.  After planning, the one
exchange is an all-gather of the packed u64 costs (``SPEC.md`` 2.4), 8 B per
scenario, over RCCL (backend ``nccl``) on the GPU box or ``gloo`` in the CPU
tests.  Every rank then holds the same cost vector and picks the same winner.
The winner's plan is then fetched from its owner: the owner packs the winning
scenario's assignment and reasons into one buffer and broadcasts it (the only
data-bearing exchange, 5 B per container), so every rank -- the one that reports
the plan included -- holds the plan the owner computed.  This is the sharded
counterpart of routing one deploy request to the server that runs it
(``crates/fleetflow-controlplane/src/handlers/deploy.rs:441-451``).

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


def check_scenario_ids(n_scen: int) -> None:
    """The packed cost keeps 16 bits of the scenario id (SPEC.md 2.4): beyond 65536
    scenarios a wrapped id could win a tie it must lose (fp_dev_place_batch refuses
    them too, FP_EOVERFLOW)."""
    if n_scen > 65536:
        raise OverflowError(f"{n_scen} scenarios: the packed cost holds 16-bit scenario ids (<= 65536)")


def gather_costs(cost_local, world: int, n_scen: int, group=None):
    """All-gather every rank's packed costs into one [n_scen] int64 tensor, in
    global scenario order (the only collective of the batch path)."""
    import torch
    import torch.distributed as dist

    check_scenario_ids(n_scen)
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


def plan_words(C: int) -> int:
    """int32 words of one packed plan: C assignments + C reason bytes, padded."""
    return C + (C + 3) // 4


def pack_plan(assign_row, reason_row, out):
    """Pack one scenario's plan (int32 assign[C], uint8 reason[C]) into ``out``
    (int32 [plan_words(C)]) -- one buffer, so the hand-off is one broadcast."""
    C = assign_row.numel()
    out[:C].copy_(assign_row)
    out[C:].view(dtype=_uint8())[:C].copy_(reason_row)
    return out


def unpack_plan(buf, C: int):
    """(assign int32 [C], reason uint8 [C]) views of a packed plan."""
    return buf[:C], buf[C:].view(dtype=_uint8())[:C]


def _uint8():
    import torch
    return torch.uint8


def hand_off_plan(best: int, assign_local, reason_local, C: int, rank: int, world: int, n_scen: int,
                  out, group=None) -> int:
    """Fetch the winning scenario's plan from its owner.

    ``assign_local``/``reason_local`` hold this rank's block ([n_local * C]);
    ``out`` is an int32 [plan_words(C)] buffer on every rank.  The owner packs the
    winner's rows into ``out`` and broadcasts it (world > 1); afterwards every
    rank's ``out`` holds the owner's plan.  Returns the owner rank."""
    own = owner(best, world, n_scen)
    if rank == own:
        lo, _ = block(rank, world, n_scen)
        j = best - lo
        pack_plan(assign_local[j * C:(j + 1) * C], reason_local[j * C:(j + 1) * C], out)
    if world > 1:
        import torch.distributed as dist
        dist.broadcast(out, src=own, group=group)
    return own
