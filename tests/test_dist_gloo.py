"""Multi-rank host logic of the sharded what-if batch (fleetflow_amd/shard.py) on
CPU with gloo, world size 2: block split, cost all-gather, identical argmin on
every rank, owner of the winner.  Costs come from the oracle (the checker); the
GPU path computes the same packed costs (tests/test_gpu_parity.py)."""
import os
import socket

import numpy as np
import pytest


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, n_scen, C, N, seed):
    import torch
    import torch.distributed as dist

    from fleetflow_amd import shard
    from oracle import oracle as O

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        lo, n = shard.block(rank, world, n_scen)
        local = []
        for s in range(lo, lo + n):
            cont, nodes = O.gen_scenario(seed, s, C, N, 7)
            assign, _, _, _ = O.place(cont, nodes)
            local.append(O.cost(assign, N, s))
        t = torch.tensor(np.array(local, np.uint64).view(np.int64))
        allc = shard.gather_costs(t, world, n_scen).numpy().view(np.uint64)
        # expected: every scenario planned on one process
        exp = []
        for s in range(n_scen):
            cont, nodes = O.gen_scenario(seed, s, C, N, 7)
            exp.append(O.cost(O.place(cont, nodes)[0], N, s))
        assert allc.tolist() == exp
        best = int(np.argmin(allc))
        # every rank agrees on the winner
        b = torch.tensor([best], dtype=torch.int64)
        bs = [torch.empty(1, dtype=torch.int64) for _ in range(world)]
        dist.all_gather(bs, b)
        assert all(int(x.item()) == best for x in bs)
        assert shard.unpack_cost(int(allc[best]))[2] == best & 0xFFFF
        own = shard.owner(best, world, n_scen)
        assert (lo <= best < lo + n) == (own == rank)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("n_scen", [6, 7])
def test_sharded_costs_gloo_world2(n_scen):
    import torch.multiprocessing as mp
    mp.spawn(_worker, args=(2, _free_port(), n_scen, 300, 40, 0x5EED0004), nprocs=2, join=True)


def test_block_split_covers_every_scenario():
    from fleetflow_amd import shard
    for world in (1, 2, 3, 8):
        for n in (0, 1, 7, 4096):
            seen = []
            for r in range(world):
                lo, c = shard.block(r, world, n)
                seen.extend(range(lo, lo + c))
                assert all(shard.owner(s, world, n) == r for s in range(lo, lo + c))
            assert seen == list(range(n))
    with pytest.raises(ValueError):
        shard.block(2, 2, 10)
