"""Python handle on the MI355X wavefront path tracer (C ABI: include/rt_hip.h)."""
from . import abi
from .render import Context
from .scene import SceneBuilder, perspective

__all__ = ["abi", "Context", "SceneBuilder", "perspective"]
