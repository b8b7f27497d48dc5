"""Host->device staging without queue drains.

``torch.tensor(x, device=cuda)`` / ``torch.as_tensor(np_array, device=cuda)`` copy from pageable memory
with a synchronous ``hipMemcpy``: the host waits for every kernel already queued on the stream. In
loops that queue GPU work and then upload small arrays (tree levels, optimizer steps, vectorizer
fill values) that serialises host and device. ``Pack`` stages several arrays in a ring of pinned
buffers and ships them with one asynchronous copy; ``to_device`` is the one-array shorthand.
"""
from __future__ import annotations

import threading
from typing import List

import numpy as np
import torch


_TORCH_OF_NP = {np.dtype(np.int64): torch.int64, np.dtype(np.int32): torch.int32,
                np.dtype(np.float32): torch.float32, np.dtype(np.float64): torch.float64,
                np.dtype(np.uint8): torch.uint8, np.dtype(np.bool_): torch.bool}


class Pack:
    """Ships several small host arrays with ONE host->device copy through a pinned staging ring
    (each ``torch.as_tensor(a, device=cuda)`` is its own blocking hipMemcpy: ~10 per tree level)."""
    _ring: dict = {}
    _RING = 16
    _lock = threading.Lock()        # host threads of concurrent learners / boosting parts share the ring

    def __init__(self, dev):
        self.dev = dev
        self.arrs: List[np.ndarray] = []

    def add(self, a) -> int:
        self.arrs.append(np.ascontiguousarray(a))
        return len(self.arrs) - 1

    def ship(self) -> List[torch.Tensor]:
        if self.dev.type != "cuda":
            return [torch.from_numpy(a) for a in self.arrs]
        offs, tot = [], 0
        for a in self.arrs:
            offs.append(tot)
            tot += (a.nbytes + 15) & ~15
        tot = max(tot, 16)
        key = self.dev.index if self.dev.index is not None else torch.cuda.current_device()
        d = torch.empty(tot, dtype=torch.uint8, device=self.dev)
        with Pack._lock:
            slots = Pack._ring.setdefault(key, {"i": 0, "bufs": [None] * self._RING, "ev": [None] * self._RING})
            k = slots["i"] = (slots["i"] + 1) % self._RING
            buf, ev = slots["bufs"][k], slots["ev"][k]
            if ev is not None:
                ev.synchronize()                 # the copy that last used this slot has finished
            if buf is None or buf.numel() < tot:
                buf = torch.empty(max(tot, 1 << 16), dtype=torch.uint8, pin_memory=True)
                slots["bufs"][k] = buf
            hb = buf.numpy()
            for a, o in zip(self.arrs, offs):
                hb[o:o + a.nbytes] = a.reshape(-1).view(np.uint8)
            d.copy_(buf[:tot], non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(torch.cuda.current_stream(self.dev))
            slots["ev"][k] = ev
        return [d[o:o + a.nbytes].view(_TORCH_OF_NP[a.dtype]).reshape(a.shape) if a.dtype in _TORCH_OF_NP
                else d[o:o + a.nbytes] for a, o in zip(self.arrs, offs)]


def to_device(a, dev, dtype=None) -> torch.Tensor:
    """Asynchronous host->device copy of a small array / list (see module docstring)."""
    arr = np.asarray(a) if dtype is None else np.asarray(a, dtype=dtype)
    if arr.dtype == np.float16 or arr.dtype not in _TORCH_OF_NP:
        arr = arr.astype(np.float64)
    pk = Pack(torch.device(dev) if not isinstance(dev, torch.device) else dev)
    i = pk.add(arr)
    return pk.ship()[i]
