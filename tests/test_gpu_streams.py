"""fp_ctx_set_stream waits for the context's previous work: the generator on one
stream, a switch, then the placement on another must see fully generated inputs.  The calls go
straight through the C ABI, so nothing but the library orders them (the Python Planner's own
torch stream ordering is bypassed on purpose)."""
import ctypes as ct

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SEED = 0x5EED0004 + 101


def test_gen_switch_stream_place(planner, O):
    import torch
    from fleetflow_amd import DevBatch
    from fleetflow_amd._lib import check
    S, C, N, base = 48, 20_000, 2_000, 5
    db = DevBatch.allocate(S, C, N, "cuda:0", scen_base=base)
    torch.cuda.synchronize()
    a, b = torch.cuda.Stream(), torch.cuda.Stream()
    L, ctx = planner._L, planner._ctx
    try:
        check(L.fp_ctx_set_stream(ctx, ct.c_void_p(a.cuda_stream)), "fp_ctx_set_stream")
        st = db.struct()
        check(L.fp_dev_gen_batch(ctx, ct.c_uint64(SEED), ct.byref(st), 7), "fp_dev_gen_batch")
        # the switch must wait for the generator (its last_ev), not for stream `a` by handle
        check(L.fp_ctx_set_stream(ctx, ct.c_void_p(b.cuda_stream)), "fp_ctx_set_stream")
        check(L.fp_dev_place_batch(ctx, ct.byref(st)), "fp_dev_place_batch")
        best = torch.empty(1, dtype=torch.int32, device="cuda:0")
        check(L.fp_dev_argmin_cost(ctx, db.cost.data_ptr(), S, best.data_ptr()), "fp_dev_argmin_cost")
        # and a switch back waits for the argmin recorded on `b`
        check(L.fp_ctx_set_stream(ctx, ct.c_void_p(a.cuda_stream)), "fp_ctx_set_stream")
        check(L.fp_ctx_sync(ctx), "fp_ctx_sync")
        costs = db.cost.cpu().numpy().view(np.uint64)
        arg = int(best.cpu().item())
    finally:
        planner.reset_stream()
    ecost = np.array([O.cost(O.place(*O.gen_scenario(SEED, base + s, C, N, 7))[0], N, base + s) for s in range(S)],
                     np.uint64)
    assert np.array_equal(costs, ecost)
    assert arg == int(np.argmin(ecost))
