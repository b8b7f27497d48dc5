"""Process-wide GIL switch interval override shared by concurrent users.

Host threads returning from native calls (tree grower, boosting parts, concurrent learner lanes) must win the
GIL back promptly from a thread running Python; the default 5 ms switch interval would stall them. Several
such sections can run at once on different threads, so the override is reference-counted: the first entrant
saves the interval, every entrant may only lower it, and the LAST one out restores the original."""
from __future__ import annotations

import contextlib
import sys
import threading

_lock = threading.Lock()
_depth = 0
_saved = None


@contextlib.contextmanager
def fast_switch(seconds: float):
    global _depth, _saved
    with _lock:
        if _depth == 0:
            _saved = sys.getswitchinterval()
        _depth += 1
        sys.setswitchinterval(min(sys.getswitchinterval(), float(seconds)))
    try:
        yield
    finally:
        with _lock:
            _depth -= 1
            if _depth == 0:
                sys.setswitchinterval(_saved)
                _saved = None
