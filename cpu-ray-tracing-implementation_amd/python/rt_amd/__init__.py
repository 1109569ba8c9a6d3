"""Python handle on the MI355X wavefront path tracer (C ABI: include/rt_hip.h)."""
from . import abi
from .render import Context, Multi, multi_plan
from .scene import SceneBuilder, perspective

__all__ = ["abi", "Context", "Multi", "multi_plan", "SceneBuilder", "perspective"]
