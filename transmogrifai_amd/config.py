"""Process-wide engine configuration.

* feature vectors are ``float64`` on the host (bit-for-bit parity with the reference's doubles on
  small data) and ``float32`` on the GPU (HBM bandwidth; statistics that need it accumulate in fp64);
* ``default_device()`` is where readers place raw columns when the caller does not say.
"""
from __future__ import annotations

import os

import torch

_DEVICE = None


def default_device() -> torch.device:
    global _DEVICE
    if _DEVICE is None:
        env = os.environ.get("TMOG_DEVICE")
        if env:
            _DEVICE = torch.device(env)
        else:
            _DEVICE = torch.device("cpu")
    return _DEVICE


def set_default_device(dev) -> None:
    global _DEVICE
    _DEVICE = torch.device(dev)


def vector_dtype(device) -> torch.dtype:
    device = torch.device(device)
    return torch.float32 if device.type == "cuda" else torch.float64


_LINEAR_DTYPE = None


def linear_dtype() -> str:
    """Storage / matrix-core precision of the linear learners' design matrix on the GPU: ``"fp32"`` (default) or
    ``"bf16"`` (X rounded to bf16 once per fit, products on the bf16 MFMA: ``ops/csrc/hip/linear_bf16_kernels.hip``;
    coefficients, margins and sums stay fp32 / fp64). ``TMOG_LINEAR_DTYPE`` or ``set_linear_dtype``."""
    global _LINEAR_DTYPE
    if _LINEAR_DTYPE is None:
        v = os.environ.get("TMOG_LINEAR_DTYPE", "fp32").lower()
        if v not in ("fp32", "bf16"):
            raise ValueError(f"TMOG_LINEAR_DTYPE must be fp32 or bf16, not {v!r}")
        _LINEAR_DTYPE = v
    return _LINEAR_DTYPE


def set_linear_dtype(v: str) -> None:
    global _LINEAR_DTYPE
    if v not in ("fp32", "bf16"):
        raise ValueError(f"linear dtype must be fp32 or bf16, not {v!r}")
    _LINEAR_DTYPE = v
