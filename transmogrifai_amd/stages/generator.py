"""Origin stage of raw features (``features/.../stages/FeatureGeneratorStage.scala:66-210``).

Holds the extract function (record -> value), the monoid aggregator used by aggregate readers,
the aggregation window and the response flag. When the raw data is already columnar (a
DataFrame / :class:`Dataset` / CSV with named columns) ``extract_fn`` is ``None`` and the column
of the same name is used directly -- the fast path used by every large-data run.
"""
from __future__ import annotations

from typing import Any, Callable, Optional

from ..features import types as T
from ..features.feature import FeatureLike
from .base import OpPipelineStage, register_stage


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


def _fn_name(fn) -> str:
    """Importable ``module.qualname`` of a module-level extract function (reloaded on model load, the
    analogue of the reference's reflective ``extractFn`` class instances); ``ColumnExtract`` for
    column extraction; ``PythonFunction`` for lambdas / closures, which cannot be restored."""
    if fn is None:
        return "ColumnExtract"
    mod, qn = getattr(fn, "__module__", None), getattr(fn, "__qualname__", "")
    if mod and qn and "<" not in qn:
        return f"{mod}.{qn}"
    return "PythonFunction"


def load_extract_fn(name: Optional[str]):
    if not name or name in ("ColumnExtract", "PythonFunction"):
        return None
    import importlib
    mod, _, qn = name.rpartition(".")
    while mod:
        try:
            obj = importlib.import_module(mod)
            break
        except ImportError:
            mod, _, head = mod.rpartition(".")
            qn = head + "." + qn
    else:
        return None
    for part in qn.split("."):
        obj = getattr(obj, part, None)
        if obj is None:
            return None
    return obj if callable(obj) else None
