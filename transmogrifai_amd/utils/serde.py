"""JSON (de)serialization of learned state: nested dicts/lists with numpy arrays and tensors.

Arrays are stored as ``{"__ndarray__": dtype, "shape": [...], "b64": <little-endian bytes>}`` so a
checkpoint stays one text file (the reference writes MLeap bundle JSON next to ``op-model.json``,
``SparkStageParam.scala:89-107``); nothing in a checkpoint is ever unpickled.
"""
from __future__ import annotations

import base64
import math

import numpy as np
import torch


def encode(obj):
    if isinstance(obj, torch.Tensor):
        obj = obj.detach().cpu().numpy()
    if isinstance(obj, np.ndarray):
        a = np.ascontiguousarray(obj)
        if a.dtype == object:
            return {"__list__": [encode(x) for x in a.tolist()]}
        return {"__ndarray__": a.dtype.str, "shape": list(a.shape), "b64": base64.b64encode(a.tobytes()).decode()}
    if isinstance(obj, dict):
        return {str(k): encode(v) for k, v in obj.items()}
    if isinstance(obj, (list, tuple)):
        return [encode(x) for x in obj]
    if isinstance(obj, (np.floating,)):
        return special_float(float(obj))
    if isinstance(obj, float):
        return special_float(obj)
    if isinstance(obj, (np.integer,)):
        return int(obj)
    if isinstance(obj, (np.bool_,)):
        return bool(obj)
    return obj


def special_float(x: float):
    if math.isnan(x):
        return "NaN"
    if math.isinf(x):
        return "Infinity" if x > 0 else "-Infinity"
    return x


def decode(obj):
    if isinstance(obj, dict):
        if "__ndarray__" in obj:
            a = np.frombuffer(base64.b64decode(obj["b64"]), dtype=np.dtype(obj["__ndarray__"]))
            return a.reshape(obj["shape"]).copy()
        if "__list__" in obj:
            return [decode(x) for x in obj["__list__"]]
        return {k: decode(v) for k, v in obj.items()}
    if isinstance(obj, list):
        return [decode(x) for x in obj]
    if not isinstance(obj, str):     # already-decoded values (decode is idempotent)
        return obj
    if obj == "NaN":
        return float("nan")
    if obj == "Infinity":
        return float("inf")
    if obj == "-Infinity":
        return float("-inf")
    return obj
