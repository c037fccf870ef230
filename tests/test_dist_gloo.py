"""Multi-rank host logic of the sharded what-if batch (fleetflow_amd/shard.py) on
CPU with gloo, world size 2: block split, cost all-gather, identical argmin on
every rank, and the hand-off of the winner's plan from its owner (one broadcast;
every rank must then hold exactly the oracle's plan for the winning scenario).
Plans and costs come from the oracle (the checker); the GPU path computes the
same plans and packed costs (tests/test_gpu_parity.py)."""
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
        local, la, lr = [], [], []
        for s in range(lo, lo + n):
            cont, nodes = O.gen_scenario(seed, s, C, N, 7)
            assign, reason, _, _ = O.place(cont, nodes)
            local.append(O.cost(assign, N, s))
            la.append(assign)
            lr.append(reason)
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
        # hand-off: the owner broadcasts the winner's plan; every rank then holds the oracle's plan
        assign_local = torch.from_numpy(np.concatenate(la).view(np.int32)) if la else torch.empty(0, dtype=torch.int32)
        reason_local = torch.from_numpy(np.concatenate(lr)) if lr else torch.empty(0, dtype=torch.uint8)
        buf = torch.full((shard.plan_words(C),), -7, dtype=torch.int32)
        got_owner = shard.hand_off_plan(best, assign_local, reason_local, C, rank, world, n_scen, buf)
        assert got_owner == own
        cont, nodes = O.gen_scenario(seed, best, C, N, 7)
        ea, er, _, _ = O.place(cont, nodes)
        ga, gr = shard.unpack_plan(buf, C)
        assert np.array_equal(ga.numpy().view(np.uint32), ea)
        assert np.array_equal(gr.numpy(), er)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("n_scen,C", [(6, 300), (7, 301), (3, 64)])
def test_sharded_costs_gloo_world2(n_scen, C):
    import torch.multiprocessing as mp
    mp.spawn(_worker, args=(2, _free_port(), n_scen, C, 40, 0x5EED0004), nprocs=2, join=True)


def test_scenario_id_limit():
    from fleetflow_amd import shard
    shard.check_scenario_ids(65536)
    with pytest.raises(OverflowError):
        shard.check_scenario_ids(65537)


def test_pack_plan_roundtrip():
    import torch
    from fleetflow_amd import shard
    for C in (1, 2, 3, 4, 5, 50_001):
        a = torch.arange(C, dtype=torch.int32) * 7 - 3
        r = (torch.arange(C) % 3).to(torch.uint8)
        buf = torch.zeros(shard.plan_words(C), dtype=torch.int32)
        ga, gr = shard.unpack_plan(shard.pack_plan(a, r, buf), C)
        assert torch.equal(ga, a) and torch.equal(gr, r)


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
