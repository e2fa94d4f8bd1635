"""tfhe_mi355 -- host-side mirror of the reference (tfhe-rs-odd) PBS interface over the MI355X
HIP engine's C ABI (include/tfhe_mi355.h, lib/libtfhe_mi355.so).

No CPU fallback: every compute call goes through the HIP engine.
"""
from . import parameters
from ._lib import EngineError, LIB_PATH, load
from .engine import Engine, device_count, fill_accumulator, pinned_empty

__all__ = ["parameters", "Engine", "EngineError", "LIB_PATH", "load", "device_count", "fill_accumulator"]
