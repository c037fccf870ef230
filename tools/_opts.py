"""Diagnostics only: apply FLEETPLACE_<OPTION>=value environment variables (e.g.
FLEETPLACE_PIPE_W=4, FLEETPLACE_SYSTOLIC=24) to a Planner's context options.  The product
library and fleetflow_amd never read the environment (fleetplace.h fp_ctx_set_option)."""
import os

from fleetflow_amd import _lib


def apply_env(planner):
    applied = {}
    for name in _lib.OPTIONS:
        v = os.environ.get("FLEETPLACE_" + name.upper())
        if v is not None and v != "":
            planner.set_option(name, int(v))
            applied[name] = int(v)
    return applied
