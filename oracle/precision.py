"""ORACLE (test infrastructure only): the oracle's floating-point type.

float64 (the reference's configs/*.json "dtype", main.py:35) unless bench.py's CPU
baseline sets float32 for its single-precision timing; the parity checks always run it
in float64.
"""
import torch

_STATE = {"dtype": torch.float64}


def dtype() -> torch.dtype:
    return _STATE["dtype"]


def set_dtype(dt: torch.dtype) -> None:
    if dt not in (torch.float32, torch.float64):
        raise ValueError(f"oracle dtype must be float32 or float64, got {dt}")
    _STATE["dtype"] = dt
