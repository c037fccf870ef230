"""CPU tests of the C-ABI boundary: libfleetplace.so loads and exports every
function include/fleetplace.h declares (no compute calls without a GPU)."""
import ctypes as ct
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_functions():
    src = open(os.path.join(ROOT, "include", "fleetplace.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(fp_[a-z_0-9]+)\s*\(", src)))


def test_header_declares_expected_entry_points():
    names = declared_functions()
    for must in ["fp_ctx_create", "fp_ctx_destroy", "fp_legacy_order", "fp_levelize", "fp_place",
                 "fp_place_batch", "fp_feasibility", "fp_dev_place_batch", "fp_dev_levelize"]:
        assert must in names


def test_library_exports_every_declared_symbol():
    from fleetflow_amd import _lib
    L = ct.CDLL(_lib.LIB_PATH)
    missing = [n for n in declared_functions() if not hasattr(L, n)]
    assert not missing, missing
    # the python binding covers the same list
    assert sorted(_lib.SIGNATURES) == declared_functions()


def test_no_cpu_backend_and_error_strings():
    from fleetflow_amd import _lib
    L = _lib.load()
    assert L.fp_abi_version() == 1
    h = ct.c_void_p()
    assert L.fp_ctx_create(ct.byref(h), -1) == _lib.FP_EINVAL  # device -1 (CPU) is refused
    rc = L.fp_ctx_create(ct.byref(h), 0)
    if rc == 0:  # running on the GPU box
        L.fp_ctx_destroy(h)
    else:
        assert rc == _lib.FP_EDEVICE
    for code in (0, -1, -2, -3, -4, -5):
        assert L.fp_strerror(code)
    assert L.fp_ctx_create(None, 0) == _lib.FP_EINVAL
