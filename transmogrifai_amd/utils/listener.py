"""Stage metrics listener: the MI355X counterpart of ``OpSparkListener`` (``utils/.../spark/OpSparkListener.scala:62-418``).

Spark reports per-stage task metrics (run time, GC, spill) to the listener; here the unit of work is a
pipeline stage's fit or transform on the device, so the workflow's DAG executor reports each one with
its wall time, the rows it processed, the device memory allocated before / after it and the device
high-water mark so far (HIP caching allocator statistics). Metrics are accumulated like
``CumulativeStageMetrics`` and, with ``log_stage_metrics``, logged with the reference's prefix format.
A listener is activated for a block with :func:`listening` (the runner does this for every run type).
"""
from __future__ import annotations

import contextlib
import logging
import threading
import time
from dataclasses import asdict, dataclass, field
from typing import Dict, Iterator, List, Optional

log = logging.getLogger(__name__)
_ACTIVE = threading.local()


@dataclass
class StageMetrics:
    stageName: str
    phase: str                    # "fit" | "transform"
    jobGroup: str                 # OpStep of the enclosing workflow step
    startTime: float
    endTime: float
    durationSecs: float
    numRows: int
    deviceAllocatedBeforeBytes: int = 0
    deviceAllocatedAfterBytes: int = 0
    devicePeakBytes: int = 0


@dataclass
class CumulativeStageMetrics:
    numStages: int = 0
    totalDurationSecs: float = 0.0
    maxDevicePeakBytes: int = 0
    byJobGroup: Dict[str, float] = field(default_factory=dict)

    def plus(self, sm: StageMetrics) -> None:
        self.numStages += 1
        self.totalDurationSecs += sm.durationSecs
        self.maxDevicePeakBytes = max(self.maxDevicePeakBytes, sm.devicePeakBytes)
        self.byJobGroup[sm.jobGroup] = self.byJobGroup.get(sm.jobGroup, 0.0) + sm.durationSecs


def _device_mem():
    try:
        import torch
        if torch.cuda.is_available() and torch.cuda.is_initialized():
            return int(torch.cuda.memory_allocated()), int(torch.cuda.max_memory_allocated())
    except Exception:  # pragma: no cover - metrics must never break a run
        pass
    return 0, 0


class OpDeviceListener:
    def __init__(self, app_name: str, run_type: str, custom_tag_name: Optional[str] = None,
                 custom_tag_value: Optional[str] = None, log_stage_metrics: bool = False,
                 collect_stage_metrics: bool = True):
        self.app_name, self.run_type = app_name, run_type
        self.custom_tag_name, self.custom_tag_value = custom_tag_name, custom_tag_value
        self.log_stage_metrics, self.collect_stage_metrics = log_stage_metrics, collect_stage_metrics
        self.job_group = "Other"
        self.stage_metrics: List[StageMetrics] = []
        self.cumulative = CumulativeStageMetrics()
        self.log_prefix = "%s:%s,RUN_TYPE:%s,APP:%s" % (custom_tag_name or "APP_NAME",
                                                          custom_tag_value or app_name, run_type, app_name)

    @contextlib.contextmanager
    def stage(self, name: str, phase: str, rows: int) -> Iterator[None]:
        a0, _ = _device_mem()
        t0 = time.time()
        try:
            yield
        finally:
            t1 = time.time()
            a1, peak = _device_mem()
            sm = StageMetrics(name, phase, self.job_group, t0, t1, t1 - t0, int(rows), a0, a1, peak)
            if self.collect_stage_metrics:
                self.stage_metrics.append(sm)
            self.cumulative.plus(sm)
            if self.log_stage_metrics:
                log.info("%s,STAGE:%s,PHASE:%s,ROWS:%d,DEVICE_PEAK_BYTES:%d,STAGE_TIME_MS:%d,JOB_GROUP:%s",
                         self.log_prefix, name, phase, rows, peak, int(1000 * sm.durationSecs), self.job_group)

    def to_json(self) -> Dict:
        return {"stageMetrics": [asdict(s) for s in self.stage_metrics],
                "cumulativeStageMetrics": asdict(self.cumulative)}


def active() -> Optional[OpDeviceListener]:
    return getattr(_ACTIVE, "listener", None)


@contextlib.contextmanager
def listening(listener: Optional[OpDeviceListener]) -> Iterator[Optional[OpDeviceListener]]:
    prev = active()
    _ACTIVE.listener = listener
    try:
        yield listener
    finally:
        _ACTIVE.listener = prev


@contextlib.contextmanager
def job_group(name: str) -> Iterator[None]:
    """The OpStep the stages inside the block belong to (Spark job groups of ``OpStep``)."""
    lst = active()
    if lst is None:
        yield
        return
    prev = lst.job_group
    lst.job_group = name
    try:
        yield
    finally:
        lst.job_group = prev


@contextlib.contextmanager
def stage(name: str, phase: str, rows: int) -> Iterator[None]:
    lst = active()
    if lst is None:
        yield
        return
    with lst.stage(name, phase, rows):
        yield
