"""Sequential UID generator.

Mirrors the identity rules of the reference (``utils/src/main/scala/com/salesforce/op/UID.scala:40-108``):
a UID is ``<Prefix>_<12 hex digits>`` drawn from a process-global counter that tests can ``reset``
so generated workflows (and therefore checkpoints) are deterministic.
"""
from __future__ import annotations

import itertools
import threading

_lock = threading.Lock()
_counter = 0


def make_uid(prefix) -> str:
    """Return ``prefix_%012x`` using the global sequential counter.

    ``prefix`` may be a string or a class (its ``__name__`` is used, like ``getSimpleName``).
    """
    global _counter
    if not isinstance(prefix, str):
        prefix = prefix.__name__
    with _lock:
        _counter += 1
        v = _counter
    return f"{prefix}_{v:012x}"


def reset(v: int = 0) -> None:
    """Reset the counter (reference ``UID.reset``)."""
    global _counter
    with _lock:
        _counter = v


def count() -> int:
    return _counter


def from_string(uid: str):
    """Split a UID into ``(prefix, suffix)``; raises ``ValueError`` on malformed input."""
    parts = uid.split("_")
    if len(parts) != 2:
        raise ValueError(f"Invalid UID: {uid}")
    return parts[0], parts[1]
