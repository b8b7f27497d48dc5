"""Stall detector for the concurrent parts of a fit (lanes, boosting parts).

Every learner calls :func:`utils.cancel.check` between iterations / rounds / tree batches; that call also
records a heartbeat here. While a :class:`Watchdog` is active, a monitor thread watches the heartbeat: when no
fit has made progress for ``after`` seconds it dumps every thread's Python stack (``faulthandler``: a thread
blocked in a native call shows the ctypes / torch call it is in) to stderr once per stall and records the stall
in :data:`STALLS` (bench.py reports them). This is the instrument for the round-3 lanes stalls, which left no
trace beyond a slow step (docs/ROUND4.md)."""
from __future__ import annotations

import faulthandler
import os
import sys
import threading
import time
from typing import List

_last = time.monotonic()
_where = ""
STALLS: List[dict] = []
_active = 0
_alock = threading.Lock()


def beat(where: str = "") -> None:
    global _last, _where
    _last = time.monotonic()
    if where:
        _where = where


def default_after() -> float:
    return float(os.environ.get("TMOG_WATCHDOG_S", "15"))


class Watchdog:
    """``with Watchdog(label):`` -- monitor the heartbeat while the block runs (nested uses share one monitor)."""

    def __init__(self, label: str = "", after: float = None):
        self.label = label
        self.after = default_after() if after is None else float(after)
        self._stop = threading.Event()
        self._th = None

    def _run(self):
        stalled_since = None
        while not self._stop.wait(min(1.0, self.after / 4)):
            idle = time.monotonic() - _last
            if idle < self.after:
                if stalled_since is not None:
                    STALLS[-1]["resolved_after_s"] = round(time.monotonic() - stalled_since, 3)
                stalled_since = None
                continue
            if stalled_since is None:
                stalled_since = _last
                rec = {"label": self.label, "idle_s": round(idle, 3), "last_beat": _where,
                       "threads": [t.name for t in threading.enumerate()]}
                STALLS.append(rec)
                sys.stderr.write(f"\n[tmog watchdog] no fit progress for {idle:.1f} s ({self.label}; last beat: "
                                 f"{_where}); thread stacks:\n")
                sys.stderr.flush()
                try:
                    faulthandler.dump_traceback(file=sys.stderr, all_threads=True)
                except Exception:          # noqa: BLE001  (stderr without a file descriptor)
                    pass
                sys.stderr.flush()

    def __enter__(self):
        global _active
        beat(f"enter {self.label}")
        with _alock:
            _active += 1
            start = _active == 1
        if start and self.after > 0:
            self._th = threading.Thread(target=self._run, name="tmog-watchdog", daemon=True)
            self._th.start()
        return self

    def __exit__(self, *exc):
        global _active
        self._stop.set()
        if self._th is not None:
            self._th.join()
        with _alock:
            _active -= 1
        return False
