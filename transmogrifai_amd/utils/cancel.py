"""Cooperative cancellation of a running fit (``maxWait``, OpValidator.scala:348).

The reference abandons a timed-out fit's future while Spark keeps running it; here a fit that outlives the
model selector's deadline is asked to stop: :func:`scope` installs a per-thread token, the learners call
:func:`check` between iterations (boosting rounds, optimizer iterations, forest batches) and a set token
raises :class:`FitCancelled`. The selector then joins the worker thread, so no abandoned fit keeps using
the GPU, its stream or the native tree-grower slots while the next learner runs. Threads a learner starts
for itself (the boosting parts) inherit the token with :func:`current` / :func:`scope`.
"""
from __future__ import annotations

import contextlib
import threading
from typing import Optional

from . import watchdog as _watchdog

_local = threading.local()


class FitCancelled(BaseException):
    """Raised inside a fit whose deadline passed (a BaseException: the per-grid-point retry of the
    validator, which catches Exception, must not retry a cancelled fit)."""


def current() -> Optional[threading.Event]:
    return getattr(_local, "token", None)


@contextlib.contextmanager
def scope(token: Optional[threading.Event]):
    prev = current()
    _local.token = token
    try:
        yield token
    finally:
        _local.token = prev


def check() -> None:
    """Raise :class:`FitCancelled` when this thread's token is set; also the fits' progress heartbeat
    (utils/watchdog.py)."""
    _watchdog.beat()
    tok = current()
    if tok is not None and tok.is_set():
        raise FitCancelled("fit cancelled: maxWait deadline passed")
