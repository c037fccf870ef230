"""Error behaviour of the C ABI (include/fleetplace.h conventions) on the GPU:
kernel-side errors of asynchronous fp_dev_* calls are sticky until fp_ctx_sync
(or the next host-pointer call) reports them once and clears them, and the
host-pointer calls write nothing on error."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_pipeline_deadlock_guard_is_reported_by_sync(planner, opts):
    """Force the placement pipeline's wall-clock guard (FP_OPT_SPIN_TICKS = 1: any
    wait longer than ~2k spin iterations aborts): the launch drains, fp_dev_place_batch
    itself returns OK (asynchronous), fp_ctx_sync reports FP_EDEVICE exactly once, and a
    normal run afterwards is clean."""
    import torch
    from fleetflow_amd import DevBatch
    from fleetflow_amd._lib import FP_EDEVICE, FleetplaceError
    db = DevBatch.allocate(4, 50_000, 5_000, "cuda:0")
    planner.dev_gen_batch(0x5EED0004, db, 7)
    snap = db.node_snapshot()
    opts(spin_ticks=1)
    planner.dev_place_batch(db)
    with pytest.raises(FleetplaceError) as e:
        planner.sync()
    assert e.value.code == FP_EDEVICE
    planner.sync()  # reported once, then cleared
    planner.set_option("spin_ticks")
    db.restore_nodes(snap)
    planner.dev_place_batch(db)
    planner.sync()
    assert int((db.reason == 0).sum().item()) > 0
    del db
    torch.cuda.empty_cache()


@pytest.mark.parametrize("bad", ["col", "row_ptr"])
def test_dev_levelize_corrupt_csr_reported_once(bad, planner):
    """fp_dev_levelize is asynchronous (no read-back inside): a corrupt CSR is found on the
    device, every later kernel of the call does nothing, and fp_ctx_sync reports FP_ECORRUPT
    exactly once.  A valid call afterwards, asynchronous too, is exact."""
    import torch
    from fleetflow_amd._lib import FP_ECORRUPT, FleetplaceError
    dev = "cuda:0"
    rp = torch.tensor([0, 1, 2] if bad == "col" else [0, 2, 1], dtype=torch.int32, device=dev)
    col = torch.tensor([0, 7] if bad == "col" else [1, 0], dtype=torch.int32, device=dev)  # 7 >= V
    hd = torch.tensor([0, 1], dtype=torch.uint8, device=dev)
    lv = torch.empty(2, dtype=torch.int32, device=dev)
    od = torch.empty(2, dtype=torch.int32, device=dev)
    nc = torch.empty(1, dtype=torch.int32, device=dev)
    planner.dev_levelize(rp, col, hd, lv, od, nc)  # returns at once: the error is sticky
    with pytest.raises(FleetplaceError) as e:
        planner.sync()
    assert e.value.code == FP_ECORRUPT
    planner.sync()  # reported once, then cleared
    rp2 = torch.tensor([0, 1, 1], dtype=torch.int32, device=dev)
    col2 = torch.tensor([1], dtype=torch.int32, device=dev)
    planner.dev_levelize(rp2, col2, hd, lv, od, nc)
    planner.sync()
    assert lv.tolist() == [0, 1] and od.tolist() == [0, 1] and nc.item() == 0
    level, order, ncyc = planner.levelize([0, 1, 1], [1], [0, 1])
    assert level.tolist() == [0, 1] and order.tolist() == [0, 1] and ncyc == 0


def test_host_call_writes_nothing_on_error(planner):
    from fleetflow_amd._lib import FleetplaceError
    level = np.full(2, 12345, np.uint32)
    order = np.full(2, 54321, np.uint32)
    import ctypes as ct
    from fleetflow_amd import _lib
    rp = np.array([0, 1, 2], np.uint32)
    col = np.array([0, 7], np.uint32)
    hd = np.array([0, 1], np.uint8)
    g = _lib.FpGraph(2, 2, rp.ctypes.data, col.ctypes.data, hd.ctypes.data)
    ncyc = ct.c_uint32(777)
    rc = _lib.load().fp_levelize(planner._ctx, ct.byref(g), level.ctypes.data_as(_lib.u32p),
                                 order.ctypes.data_as(_lib.u32p), ct.byref(ncyc))
    assert rc == _lib.FP_ECORRUPT
    assert level.tolist() == [12345, 12345] and order.tolist() == [54321, 54321] and ncyc.value == 777
    with pytest.raises(FleetplaceError):
        planner.levelize([0, 2, 1], [1, 0], [0, 1])  # row_ptr not monotone
    planner.sync()


def test_pending_async_error_survives_unrelated_host_call(planner, opts):
    """an asynchronous call's kernel error is neither reported by, nor cleared by, a
    later unrelated host-pointer call (those have their own error word); fp_ctx_sync still
    reports it once."""
    import torch
    from fleetflow_amd import DevBatch
    from fleetflow_amd._lib import FP_EDEVICE, FleetplaceError
    db = DevBatch.allocate(4, 50_000, 5_000, "cuda:0")
    planner.dev_gen_batch(0x5EED0004, db, 7)
    opts(spin_ticks=1)
    planner.dev_place_batch(db)                              # fails asynchronously (guard)
    planner.set_option("spin_ticks")
    level, order, ncyc = planner.levelize([0, 1, 1], [1], [0, 1])   # unrelated host call: fine
    assert level.tolist() == [0, 1] and ncyc == 0
    with pytest.raises(FleetplaceError) as e:
        planner.sync()
    assert e.value.code == FP_EDEVICE
    planner.sync()
    del db
    torch.cuda.empty_cache()


def test_forced_bounded_links_without_residency_fail_promptly(planner, opts):
    """bounded links on a batch whose consumers cannot be resident must end in
    FP_EDEVICE from the deadlock guard, promptly, and leave the context usable.  Forced: lag = S
    hands out every scenario's segment-0 ticket before any segment-1 ticket, and the batch holds
    more scenarios than the device has segment slots, so the resident segment-0 producers fill
    their 8-slot rings and wait on segment-1 consumers that can never be dispatched.  (With
    every segment resident the same forced geometry completes: a consumer is always running.)"""
    import time
    import torch
    from fleetflow_amd import DevBatch
    from fleetflow_amd._lib import FP_EDEVICE, FleetplaceError
    C, N = 12_000, 5_000  # 7 segments of 12 groups; segment 0 (768 nodes) forwards ~4k per scenario
    S = planner.geometry(8192, C, N)["resident"] + 256  # the resident slots of a batch this large
    db = DevBatch.allocate(S, C, N, "cuda:0")
    planner.dev_gen_batch(0x5EED0004, db, 7)
    snap = db.node_snapshot()
    opts(pipe_lag=S, link_bounded=1, link_slots=8, spin_ticks=20_000_000)  # 0.2 s guard
    g = planner.geometry(S, C, N)
    assert g["bounded"] == 1 and g["lag"] == S and g["link_slots"] == 8, g
    assert S > g["resident"] and g["segments"] > 1, g
    t0 = time.perf_counter()
    planner.dev_place_batch(db)
    with pytest.raises(FleetplaceError) as e:
        planner.sync()
    assert e.value.code == FP_EDEVICE
    assert time.perf_counter() - t0 < 30
    planner.reset_options()
    db.restore_nodes(snap)
    planner.dev_place_batch(db)
    planner.sync()
    assert int((db.reason == 0).sum().item()) > 0
    del db
    torch.cuda.empty_cache()
