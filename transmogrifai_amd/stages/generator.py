"""Origin stage of raw features (``features/.../stages/FeatureGeneratorStage.scala:66-210``).

Holds the extract function (record -> value), the monoid aggregator used by aggregate readers,
the aggregation window and the response flag. When the raw data is already columnar (a
DataFrame / :class:`Dataset` / CSV with named columns) ``extract_fn`` is ``None`` and the column
of the same name is used directly -- the fast path used by every large-data run.
"""
from __future__ import annotations

import logging
from typing import Any, Callable, Dict, Optional

from ..features import types as T
from ..features.feature import FeatureLike
from .base import OpPipelineStage, register_stage

log = logging.getLogger(__name__)


@register_stage
class FeatureGeneratorStage(OpPipelineStage):
    operation_name = "FeatureGenerator"
    arity = "0N"

    def __init__(self, name: str, output_type, extract_fn: Optional[Callable] = None, aggregator=None,
                 aggregate_window=None, output_is_response: bool = False, extract_source: Optional[str] = None,
                 uid: Optional[str] = None, column: Optional[str] = None):
        super().__init__(uid=uid, output_type=output_type)
        self.name = name
        self.extract_fn = extract_fn
        if extract_fn is not None:
            _fn_name(extract_fn)         # registers module-level functions for checkpoint reloads
        self.aggregator = aggregator
        self.aggregate_window = aggregate_window
        self.output_is_response = output_is_response
        self.extract_source = extract_source
        self.column = column if column is not None else (name if extract_fn is None else None)
        self._output_name = name

    def output_is_response_fn(self):
        return self.output_is_response

    def get_output(self) -> FeatureLike:
        if self._output is None:
            self._output = FeatureLike(self.name, self.output_type, self.output_is_response, self, [],
                                       self.output_feature_uid())
        return self._output

    def extract(self, record) -> Any:
        """Apply the extract function to a record (dict, object or pandas row)."""
        col = self.column if self.column is not None else self.name
        if self.extract_fn is not None:
            v = self.extract_fn(record)
        elif isinstance(record, dict):
            v = record.get(col)
        else:
            v = getattr(record, col, None)
        if isinstance(v, T.FeatureType):
            v = v.value
        return v

    def aggregate_records(self, records, time_fn=None, cutoff=None, response_window: Optional[int] = None,
                          predictor_window: Optional[int] = None):
        """``FeatureAggregator.extract`` (FeatureAggregator.scala:48-130): fold one key's records into this
        feature's value -- each record becomes an event (``time_fn(record)`` ms, 0 without one) and is kept by
        ``filter_by_date_with_cutoff`` with the response window for a response feature and the predictor
        window otherwise (the stage's own ``aggregate_window`` when it has one); returns a FeatureType."""
        from ..features.aggregators import CutOffTime, Event, default_aggregator, filter_by_date_with_cutoff
        agg = self.aggregator if self.aggregator is not None else default_aggregator(self.output_type)
        cutoff = cutoff if cutoff is not None else CutOffTime.no_cutoff()
        resp = bool(self.output_is_response)
        win = self.aggregate_window if self.aggregate_window is not None else \
            (response_window if resp else predictor_window)
        evs = []
        for r in records:
            d = int(time_fn(r)) if time_fn is not None else 0
            if filter_by_date_with_cutoff(d, cutoff, resp, win):
                evs.append(Event(d, self.extract(r), resp))
        return self.output_type(agg.aggregate(evs)) if self.output_type.nullable or evs else self.output_type.empty()

    def ctor_args(self):
        agg = None
        if self.aggregator is not None:
            agg = {"className": type(self.aggregator).__name__, "value": getattr(self.aggregator, "to_json",
                                                                               lambda: {})()}
        return {"tti": "Record", "tto": self.output_type.type_name(), "aggregator": agg,
                "extractFn": {"className": _fn_name(self.extract_fn), "column": self.column},
                "outputName": self.name, "uid": self.uid,
                "extractSource": self.extract_source or "",
                "outputIsResponse": self.output_is_response,
                "aggregateWindow": self.aggregate_window}


# Functions a checkpoint may name (extract functions, predicate / map functions of _FnStage). A
# checkpoint is data: loading one never imports a module or resolves an arbitrary attribute path; it can
# only select a function that this process registered -- explicitly with ``register_function`` or
# implicitly by handing it to a FeatureBuilder / stage (user code that the process already runs).
_FUNCTIONS: Dict[str, Callable] = {}


def register_function(fn: Callable = None, name: Optional[str] = None):
    """Make ``fn`` loadable by name from checkpoints (decorator or call). Returns ``fn``."""
    def reg(f):
        key = name or _qual_name(f)
        if key is None:
            raise ValueError("only module-level functions (or an explicit name) can be registered")
        _FUNCTIONS[key] = f
        return f
    return reg(fn) if fn is not None else reg


def registered_functions() -> Dict[str, Callable]:
    return dict(_FUNCTIONS)


def _qual_name(fn) -> Optional[str]:
    mod, qn = getattr(fn, "__module__", None), getattr(fn, "__qualname__", "")
    if mod and qn and "<" not in qn:
        return f"{mod}.{qn}"
    return None


def _fn_name(fn) -> str:
    """Registry name of a user function (``module.qualname``; registered as a side effect so the model
    reloads in this process); ``ColumnExtract`` for column extraction; ``PythonFunction`` for lambdas /
    closures, which cannot be restored."""
    if fn is None:
        return "ColumnExtract"
    for k, v in _FUNCTIONS.items():
        if v is fn:
            return k
    q = _qual_name(fn)
    if q is None:
        return "PythonFunction"
    _FUNCTIONS.setdefault(q, fn)
    return q


def load_extract_fn(name: Optional[str]):
    """Resolve a checkpoint function name through the registry only (no imports, no attribute walks).
    Unknown names resolve to None: column-extract stages fall back to the column of the feature's name;
    a stage that needs the function raises when it is applied (see ``require_function``)."""
    if not name or name in ("ColumnExtract", "PythonFunction"):
        return None
    fn = _FUNCTIONS.get(name)
    if fn is None:
        log.warning("checkpoint names function %r which is not registered in this process; register it with "
                    "transmogrifai_amd.register_function before loading the model to restore it", name)
    return fn


def require_function(fn, name: Optional[str]):
    if fn is None:
        raise RuntimeError(f"function {name!r} is not registered; call register_function on it before loading")
    return fn
