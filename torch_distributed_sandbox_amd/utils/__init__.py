"""Aux subsystems: fault injection, timing/roctx, checkpointing."""
from . import checkpoint, fault, timing

__all__ = ["checkpoint", "fault", "timing"]
