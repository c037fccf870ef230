"""ctypes binding of libfleetplace.so (include/fleetplace.h).

The product path has NO CPU fallback: if the HIP library is missing or no gfx950
device is present, calls raise.  The binding is the same one a Rust crate would
declare with ``extern "C"``.
"""
from __future__ import annotations

import ctypes as ct
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# FLEETPLACE_LIB selects another build of the same ABI (e.g. the diagnostics build
# libfleetplace_stats.so used by tools/pipe_stats.py); default is the release build.
LIB_PATH = os.environ.get("FLEETPLACE_LIB") or os.path.join(_HERE, "libfleetplace.so")

FP_OK, FP_EINVAL, FP_ENOMEM, FP_EDEVICE, FP_EOVERFLOW, FP_ECORRUPT = 0, -1, -2, -3, -4, -5
FP_NONE = 0xFFFFFFFF
REASON_OK, REASON_NOFIT, REASON_CYCLE = 0, 1, 2
FP_K_PLACE, FP_K_SORT, FP_K_FEAS, FP_K_LEVEL, FP_K_GEN = 0, 1, 2, 3, 4
# context options (fleetplace.h enum fp_option); FP_OPT_AUTO = the production default
# ("segsort" is ignored by the library and kept for ABI stability)
FP_OPT_AUTO = -1
OPTIONS = {"pipe_w": 0, "pipe_seg": 1, "pipe_r": 2, "pipe_lag": 3, "link_slots": 4, "link_bounded": 5,
           "pipe_flush": 6, "spin_ticks": 7, "kpack": 8, "scen_sort": 9, "segsort": 10, "systolic": 11,
           "levelize_sync": 12, "systolic_extra": 13, "screen": 14, "payload_lds": 15, "systolic_valu": 16, "link_publish": 17,
           "level_sort": 18, "level_small": 19, "pipe_prio": 20,
           "indeg_bin": 21, "packed": 22}
# fp_place_geometry out[] (fleetplace.h FP_GEOM_*)
GEOM_FIELDS = ("groups", "stages", "segments", "ring", "lag", "link_slots", "bounded", "resident", "systolic")

u8p = ct.POINTER(ct.c_uint8)
u32p = ct.POINTER(ct.c_uint32)
u64p = ct.POINTER(ct.c_uint64)
vp = ct.c_void_p


class FpGraph(ct.Structure):
    _fields_ = [("n_vertices", ct.c_uint32), ("n_edges", ct.c_uint32), ("row_ptr", vp), ("col", vp),
                ("has_deps", vp)]


class FpContainers(ct.Structure):
    _fields_ = [("n", ct.c_uint32), ("cpu_m", vp), ("mem_mib", vp), ("req_labels", vp), ("conflict", vp)]


class FpNodes(ct.Structure):
    _fields_ = [("n", ct.c_uint32), ("cpu_free", vp), ("mem_free", vp), ("labels", vp),
                ("conflict_used", vp), ("schedulable", vp)]


class FpBatch(ct.Structure):
    _fields_ = [("n_scen", ct.c_uint32), ("scen_base", ct.c_uint32), ("n_containers", ct.c_uint32),
                ("n_nodes", ct.c_uint32),
                ("cpu_m", vp), ("mem_mib", vp), ("req_labels", vp), ("conflict", vp), ("level", vp),
                ("cpu_free", vp), ("mem_free", vp), ("labels", vp), ("conflict_used", vp),
                ("schedulable", vp), ("assign", vp), ("reason", vp), ("cost", vp)]


class FleetplaceError(RuntimeError):
    def __init__(self, code, where):
        self.code = code
        msg = _lib_strerror(code) if _LIB is not None else str(code)
        super().__init__(f"{where}: {msg} ({code})")


_LIB = None

# name -> (restype, argtypes); the full export list of include/fleetplace.h
SIGNATURES = {
    "fp_ctx_create": (ct.c_int, [ct.POINTER(vp), ct.c_int]),
    "fp_ctx_destroy": (None, [vp]),
    "fp_ctx_set_stream": (ct.c_int, [vp, vp]),
    "fp_ctx_reset_stream": (ct.c_int, [vp]),
    "fp_ctx_sync": (ct.c_int, [vp]),
    "fp_strerror": (ct.c_char_p, [ct.c_int]),
    "fp_abi_version": (ct.c_int, []),
    "fp_ctx_profile": (ct.c_int, [vp, ct.c_int]),
    "fp_ctx_kernel_stats": (ct.c_int, [vp, ct.c_int, ct.POINTER(ct.c_double), ct.POINTER(ct.c_uint64)]),
    "fp_ctx_place_path": (ct.c_int, [vp, u32p]),
    "fp_ctx_set_option": (ct.c_int, [vp, ct.c_int, ct.c_int64]),
    "fp_ctx_get_option": (ct.c_int, [vp, ct.c_int, ct.POINTER(ct.c_int64)]),
    "fp_legacy_order": (ct.c_int, [vp, ct.POINTER(FpGraph), u32p]),
    "fp_levelize": (ct.c_int, [vp, ct.POINTER(FpGraph), u32p, u32p, u32p]),
    "fp_place": (ct.c_int, [vp, ct.POINTER(FpContainers), ct.POINTER(FpNodes), u32p, u32p, u8p]),
    "fp_place_batch": (ct.c_int, [vp, ct.POINTER(FpBatch)]),
    "fp_feasibility": (ct.c_int, [vp, ct.POINTER(FpContainers), ct.POINTER(FpNodes), u32p, u32p, u64p]),
    # output arrays as plain addresses (vp): a 3-service stage's call is on the config-1 clock
    "fp_plan_stage": (ct.c_int, [vp, ct.POINTER(FpGraph), ct.POINTER(FpContainers), ct.POINTER(FpNodes), vp, vp,
                                 vp, u32p, vp, vp, vp, vp]),
    "fp_dev_legacy_order": (ct.c_int, [vp, ct.POINTER(FpGraph), vp]),
    "fp_dev_levelize": (ct.c_int, [vp, ct.POINTER(FpGraph), vp, vp, vp]),
    "fp_dev_place_batch": (ct.c_int, [vp, ct.POINTER(FpBatch)]),
    "fp_place_ws_bytes": (ct.c_int, [vp, ct.c_uint32, ct.c_uint32, ct.c_uint32, u64p]),
    "fp_place_geometry": (ct.c_int, [vp, ct.c_uint32, ct.c_uint32, ct.c_uint32, u32p]),
    "fp_dev_feasibility": (ct.c_int, [vp, ct.POINTER(FpContainers), ct.POINTER(FpNodes), vp, vp, vp]),
    "fp_dev_feasibility_batch": (ct.c_int, [vp, ct.POINTER(FpBatch), vp, vp]),
    "fp_dev_argmin_cost": (ct.c_int, [vp, vp, ct.c_uint32, vp]),
    "fp_dev_gen_batch": (ct.c_int, [vp, ct.c_uint64, ct.POINTER(FpBatch), ct.c_uint32]),
}


def load():
    """Load libfleetplace.so; raise loudly if it has not been built."""
    global _LIB
    if _LIB is None:
        # One HIP runtime per process: PyTorch-ROCm ships its own libamdhip64.so.7.
        # Loading torch first makes our DT_NEEDED libamdhip64.so.7 bind to that same
        # runtime (same SONAME), so device pointers from torch tensors and from this
        # library live in one HIP context.  Loading ours first would leave torch with
        # a second runtime that finds no GPU.
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(
                f"{LIB_PATH} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
                "(there is no CPU fallback)")
        L = ct.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _LIB = L
    return _LIB


def raw_function(name):
    """A second handle to an export with no argtypes (no per-argument conversion on the call): the
    caller passes ctypes objects only.  For the per-plan fast path (Planner.plan_stage_lists)."""
    load()
    f = getattr(ct.CDLL(LIB_PATH), name)
    f.restype = ct.c_int
    f.argtypes = None
    return f


def _lib_strerror(code):
    return load().fp_strerror(code).decode()


def check(rc, where):
    if rc != FP_OK:
        raise FleetplaceError(rc, where)
