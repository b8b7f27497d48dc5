"""Classifying GPU failures: ordinary errors vs faults that leave the device context dead.

The model selector drops a failing (estimator, ParamMap) fit and goes on (``OpValidator.scala:324-353``).
That is right for an ordinary failure -- a bad parameter, a singular system, a recoverable out-of-memory --
but not after the device itself faulted (an illegal address, a kernel that aborted): HIP errors of that kind
are sticky, every later launch on the context fails, and retrying the remaining grid points only produces
pages of errors and, at exit, a core dump from runtime teardown on a dead context. Such a failure is raised
as :class:`DeviceFault`; the selector re-raises it at once, and the entry points (``bench.py``,
``app.py``) report it and leave the process with :data:`EXIT_DEVICE_FAULT` without running teardown.
"""
from __future__ import annotations

import os
import sys
from typing import Optional

import torch

EXIT_DEVICE_FAULT = 70

# message fragments of the sticky HIP / HSA failures (hipGetErrorString texts and the runtime's aborts)
_STICKY = ("illegal memory access", "illegal address", "hiperrorillegaladdress", "hiperrorlaunchfailure",
           "unspecified launch failure", "device-side assert", "memory access fault",
           "hsa_status_error", "gpu hang", "hiperrorecc", "ecc error", "hardware exception",
           "an illegal instruction")


class DeviceFault(RuntimeError):
    """The GPU context is no longer usable; nothing after this can run on it."""


def is_device_fault(err: BaseException, device: Optional[torch.device] = None, probe: bool = True) -> bool:
    """True when ``err`` is (or left behind) a sticky device error. Out-of-memory is not one. With ``probe``
    and a CUDA ``device``, a synchronisation of the calling thread's current stream tells a context that is still
    healthy from a dead one whatever the message said (only that stream: a learner lane must not wait for -- or
    be blamed for -- the other lanes' queued work; a sticky error fails every synchronisation on the context)."""
    if isinstance(err, DeviceFault):
        return True
    msg = f"{type(err).__name__}: {err}".lower()
    if "out of memory" in msg and not any(s in msg for s in _STICKY):
        return False
    if any(s in msg for s in _STICKY):
        return True
    if probe and device is not None and torch.device(device).type == "cuda":
        try:
            torch.cuda.current_stream(device).synchronize()
        except Exception:  # noqa: BLE001 - any failure of a bare synchronise means the context is gone
            return True
    return False


def fault_in_chain(err: BaseException) -> bool:
    """A :class:`DeviceFault` (or a sticky error message) anywhere in ``err``'s cause / context chain."""
    seen = set()
    while err is not None and id(err) not in seen:
        seen.add(id(err))
        if not isinstance(err, (SystemExit, KeyboardInterrupt)) and is_device_fault(err, probe=False):
            return True
        err = err.__cause__ or err.__context__
    return False


def run_main(fn, what: str):
    """Run an entry point; a device fault ends the process with :data:`EXIT_DEVICE_FAULT` (no teardown)."""
    try:
        return fn()
    except BaseException as e:  # noqa: BLE001 - re-raised unless it is a device fault
        if fault_in_chain(e):
            import traceback
            traceback.print_exc()
            fatal_exit(e, what)
        raise


def fatal_exit(err: BaseException, what: str = "tmog") -> None:
    """Report a device fault and end the process without interpreter / HIP runtime teardown (which can
    crash on a dead context and dump core instead of exiting with a status)."""
    try:
        sys.stdout.flush()
    finally:
        sys.stderr.write(f"{what}: fatal device fault, exiting with status {EXIT_DEVICE_FAULT}: {err!r}\n")
        sys.stderr.flush()
        os._exit(EXIT_DEVICE_FAULT)
