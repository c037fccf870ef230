"""fleetflow_amd -- MI355X-native placement planner for FleetFlow's plan path.

The product is libfleetplace.so (HIP, gfx950) behind include/fleetplace.h;
this package is its host-side mirror of the reference interface.
"""
from .planner import NONE, DevBatch, Planner  # noqa: F401
from .flow import (Flow, Plan, Server, Service, Stage, order_by_dependencies,  # noqa: F401
                   plan_stage, resolve_target_server)

__all__ = ["NONE", "DevBatch", "Planner", "Flow", "Plan", "Server", "Service", "Stage",
           "order_by_dependencies", "plan_stage", "resolve_target_server"]
