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
