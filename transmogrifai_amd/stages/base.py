"""Stage ABI: pipeline stages, transformers and estimators.

Reference: ``OpPipelineStageBase`` / ``OpPipelineStage1..N`` (``features/.../stages/OpPipelineStages.scala:50-552``),
output naming (``stages/package.scala:42-57``), the ``OpTransformer`` row interface
(``transformRow``/``transformMap``/``transformKeyValue``) and the unary..sequence estimator/transformer
bases (``stages/base/**``).

Design (MI355X-first): a transformer's primary entry point is :meth:`OpTransformer.transform_columns`,
a *batch* kernel over whole device-resident columns; the row path (:meth:`transform_row`,
:meth:`transform_key_value`) is derived from it so batch == row == reloaded-checkpoint by
construction. Estimators reduce whole columns (:meth:`OpEstimator.fit_columns`) and return a
fitted model that shares their uid.
"""
from __future__ import annotations

import logging

import copy as _copy
import re
from typing import Any, Callable, Dict, List, Optional, Sequence

from ..data.columns import Column, column_from_values
from ..data.dataset import Dataset
from ..features import types as T
from ..features.feature import FeatureLike, TransientFeature, feature_uid
from ..uid import make_uid

log = logging.getLogger(__name__)

_STAGE_REGISTRY: Dict[str, type] = {}


def register_stage(cls):
    """Class decorator: make a stage class loadable from checkpoints by name. Reference checkpoints name
    stages by their JVM class (``com.salesforce.op...OpIndexToString``) and resolve by the short name, so
    two different classes may not share one: that would make loading depend on import order."""
    prev = _STAGE_REGISTRY.get(cls.__name__)
    if prev is not None and (prev.__module__, prev.__qualname__) != (cls.__module__, cls.__qualname__):
        raise TypeError(f"stage class name {cls.__name__!r} registered twice: {prev.__module__} and {cls.__module__}")
    _STAGE_REGISTRY[cls.__name__] = cls
    _STAGE_REGISTRY[f"{cls.__module__}.{cls.__qualname__}"] = cls
    return cls


# every module of this package that defines checkpoint-loadable stages: a fresh process that loads a
# model imports them on the first lookup miss (the registry is filled by the @register_stage decorators)
_STAGE_MODULES = (
    "transmogrifai_amd.stages.generator", "transmogrifai_amd.stages.feature.vectorizers",
    "transmogrifai_amd.stages.feature.bucketizers", "transmogrifai_amd.stages.feature.indexers",
    "transmogrifai_amd.stages.feature.maps", "transmogrifai_amd.stages.feature.math_stages",
    "transmogrifai_amd.stages.feature.misc_stages", "transmogrifai_amd.stages.feature.nlp_stages",
    "transmogrifai_amd.stages.feature.text_stages", "transmogrifai_amd.stages.feature.vector_stages",
    "transmogrifai_amd.stages.feature.vector_scalers",
    "transmogrifai_amd.stages.insights.record_insights", "transmogrifai_amd.stages.preparators.min_variance",
    "transmogrifai_amd.stages.preparators.sanity_checker", "transmogrifai_amd.models.base",
    "transmogrifai_amd.models.linear", "transmogrifai_amd.models.glm", "transmogrifai_amd.models.mlp",
    "transmogrifai_amd.models.trees", "transmogrifai_amd.selector.model_selector",
    "transmogrifai_amd.selector.extras",
)
_ALL_IMPORTED = False


def import_stage_modules() -> None:
    """Import every stage-defining module of this package (a fixed list: checkpoint contents never
    choose what is imported)."""
    global _ALL_IMPORTED
    if _ALL_IMPORTED:
        return
    import importlib
    for m in _STAGE_MODULES:
        importlib.import_module(m)
    _ALL_IMPORTED = True


def _lookup(name: str) -> Optional[type]:
    return _STAGE_REGISTRY.get(name) or _STAGE_REGISTRY.get(name.rsplit(".", 1)[-1].rstrip("$"))


def stage_class(name: str) -> type:
    cls = _lookup(name)
    if cls is None:
        import_stage_modules()
        cls = _lookup(name)
    if cls is None:
        raise ValueError(f"Unknown stage class '{name}'")
    return cls


def make_output_name(output_feature_uid: str, inputs: Sequence[TransientFeature], num_ops: int = 1) -> str:
    """``<sorted origins joined by ->_<n>-stagesApplied_<FeatureUID>`` (``stages/package.scala:42-49``)."""
    origins = sorted({o for t in inputs for o in t.origin_features})
    origins = re.sub(r"[^A-Za-z\-_0-9]+", "", "-".join(origins))
    n_stages = len({s for t in inputs for s in t.stages}) + num_ops
    return f"{origins}_{n_stages}-stagesApplied_{output_feature_uid}"


def _in_domain(value, dom) -> bool:
    """``dom`` = (lo, hi, lo_inclusive, hi_inclusive); None bounds are open (Spark ``ParamValidators``)."""
    lo, hi, lo_in, hi_in = dom
    v = float(value)
    if lo is not None and not (v >= lo if lo_in else v > lo):
        return False
    return hi is None or (v <= hi if hi_in else v < hi)


def _fmt_domain(dom) -> str:
    lo, hi, lo_in, hi_in = dom
    return f"{'[' if lo_in else '('}{'-inf' if lo is None else lo}, {'inf' if hi is None else hi}{']' if hi_in else ')'}"


# common domains of the reference's param validators
GT0 = (0, None, False, False)
GTEQ0 = (0, None, True, False)
UNIT = (0.0, 1.0, True, True)


class OpPipelineStage:
    """Base of every stage. Subclasses set ``operation_name``, ``output_type`` and ``_defaults``; numeric
    params with a domain (``_param_domains``: name -> (lo, hi, lo_inclusive, hi_inclusive)) are checked on
    ``set`` the way Spark's ``ParamValidators`` reject an out-of-range ``setX``."""

    operation_name: str = "stage"
    output_type = T.FeatureType
    arity: Any = 1                # 1, 2, 3, 4, "N" (sequence), "1N" (one + sequence)
    allow_label_as_input = False
    is_estimator = False
    _defaults: Dict[str, Any] = {}

    def __init__(self, uid: Optional[str] = None, operation_name: Optional[str] = None, output_type=None,
                 **params):
        self.uid = uid or make_uid(type(self).__name__)
        if operation_name is not None:
            self.operation_name = operation_name
        if output_type is not None:
            self.output_type = output_type
        self.params: Dict[str, Any] = {}
        for klass in reversed(type(self).__mro__):
            self.params.update(getattr(klass, "_defaults", {}) or {})
        for k, v in params.items():
            self.set(k, v)
        self._inputs: List[FeatureLike] = []
        self._transient: Optional[List[TransientFeature]] = None
        self._output: Optional[FeatureLike] = None
        self._output_name: Optional[str] = None
        self.metadata: Dict[str, Any] = {}
        self.parent = None

    # ----------------------------------------------------------------------------------- params
    def set(self, name: str, value) -> "OpPipelineStage":
        if name not in self.params and not self._accepts_param(name):
            raise ValueError(f"{type(self).__name__} has no param '{name}'")
        dom = getattr(type(self), "_param_domains", {}).get(name)
        if dom is not None and value is not None and not _in_domain(value, dom):
            raise ValueError(f"{type(self).__name__} param {name} = {value!r} outside {_fmt_domain(dom)}")
        self.params[name] = value
        return self

    def _accepts_param(self, name) -> bool:
        return False

    def get(self, name: str, default=None):
        return self.params.get(name, default)

    def __getattr__(self, item):
        # set_foo(v) / get_foo() sugar over the params dict (Spark ML ``setX``/``getX``)
        if item.startswith("set_"):
            key = item[4:]
            params = self.__dict__.get("params", {})
            if key in params or self._accepts_param(key):
                return lambda v: self.set(key, v)
        if item.startswith("get_"):
            key = item[4:]
            params = self.__dict__.get("params", {})
            if key in params:
                return lambda: params[key]
        raise AttributeError(f"'{type(self).__name__}' object has no attribute '{item}'")

    # ----------------------------------------------------------------------------------- inputs
    def set_input(self, *features) -> "OpPipelineStage":
        flat: List[FeatureLike] = []
        for f in features:
            if isinstance(f, (list, tuple)):
                flat.extend(f)
            else:
                flat.append(f)
        if not self.check_input_length(flat):
            raise ValueError(f"{type(self).__name__}: wrong number of inputs {len(flat)} (arity {self.arity})")
        if not all(isinstance(f, FeatureLike) for f in flat):
            raise TypeError("inputs must be features")
        if len({f.uid for f in flat}) != len(flat) and self.arity not in (2, 3, 4):
            raise ValueError("input features must be distinct")
        self.check_input_types(flat)
        self._inputs = flat
        self._transient = None
        self._output = None
        return self

    def check_input_length(self, feats) -> bool:
        a = self.arity
        if a == "N":
            return len(feats) >= 1
        if a == "1N":
            return len(feats) >= 1
        if a == "0N":
            return True
        return len(feats) == a

    def check_input_types(self, feats):
        pass

    def get_input_features(self) -> List[FeatureLike]:
        return list(self._inputs)

    def get_transient_features(self) -> List[TransientFeature]:
        if self._transient is None:
            self._transient = [TransientFeature.of(f) for f in self._inputs]
        return self._transient

    @property
    def input_names(self) -> List[str]:
        return [f.name for f in self._inputs]

    # ---------------------------------------------------------------------------------- outputs
    def output_feature_uid(self) -> str:
        return feature_uid(self.output_type, self.uid)

    def output_is_response(self) -> bool:
        ins = self._inputs
        if self.allow_label_as_input:
            return bool(ins) and all(f.is_response for f in ins)
        return any(f.is_response for f in ins)

    def set_output_feature_name(self, name: str) -> "OpPipelineStage":
        self._output_name = name
        self._output = None
        return self

    def get_output_feature_name(self) -> str:
        if self._output_name:
            return self._output_name
        return make_output_name(self.output_feature_uid(), self.get_transient_features())

    def get_output(self) -> FeatureLike:
        if not self._inputs and self.arity != "0N":
            raise ValueError(f"Stage {self.uid} has no inputs set")
        if self._output is None:
            self._output = FeatureLike(self.get_output_feature_name(), self.output_type, self.output_is_response(),
                                       self, self._inputs, self.output_feature_uid())
        return self._output

    def stage_name(self) -> str:
        return f"{self.operation_name}_{self.uid}"

    # ------------------------------------------------------------------------------------- misc
    def copy(self) -> "OpPipelineStage":
        c = _copy.copy(self)
        c.params = dict(self.params)
        c.metadata = _copy.deepcopy(self.metadata)
        return c

    def ctor_args(self) -> Dict[str, Any]:
        """Learned / constructor state to serialize (``ctorArgs``)."""
        return {}

    def load_ctor_args(self, args: Dict[str, Any]) -> None:
        pass

    def __repr__(self):
        return f"{type(self).__name__}({self.uid})"


class OpTransformer(OpPipelineStage):
    """A stage that maps input columns to one output column."""

    def transform_columns(self, *cols: Column, ds: Optional[Dataset] = None) -> Column:
        raise NotImplementedError(type(self).__name__)

    def transform(self, ds: Dataset) -> Dataset:
        cols = [ds[f.name] for f in self._inputs]
        out = self.transform_columns(*cols, ds=ds)
        return ds.with_column(self.get_output_feature_name(), out)

    # row interface (``OpTransformer.transformRow/transformMap/transformKeyValue``)
    def transform_row(self, *values) -> Any:
        cols = [column_from_values(f.wtype, [v], "cpu") for f, v in zip(self._inputs, values)]
        out = self.transform_columns(*cols, ds=None)
        return out.row(0)

    def transform_key_value(self, getter: Callable[[str], Any]) -> Any:
        return self.transform_row(*[getter(f.name) for f in self._inputs])

    def transform_map(self, row: Dict[str, Any]) -> Any:
        return self.transform_key_value(row.get)


class OpEstimator(OpPipelineStage):
    """A stage that is fit on data and produces an :class:`OpTransformer` model sharing its uid."""

    is_estimator = True
    model_class: type = None
    # True when fit_columns reduces its own statistics over the ranks of a row-sharded fit
    # (parallel/dp.py); other estimators see their inputs gathered from every rank
    dp_aware = False

    def fit_columns(self, *cols: Column, ds: Optional[Dataset] = None) -> OpTransformer:
        raise NotImplementedError(type(self).__name__)

    def fit(self, ds: Dataset) -> OpTransformer:
        from ..parallel import dp
        if dp.active() and not self.dp_aware:
            # generic fallback: correct, but every rank receives every row of the inputs -- logged and
            # recorded (parallel/dp.py GATHER_FALLBACKS) so benchmarks and tests can assert it never fires
            log.warning("%s (%s) has no data-parallel fit: gathering its %d input column(s) from every rank",
                        type(self).__name__, self.uid, len(self._inputs))
            dp.GATHER_FALLBACKS.append(type(self).__name__)
            ds = dp.gather_dataset(ds, dict.fromkeys(f.name for f in self._inputs))
            with dp.local_only():
                model = self.fit_columns(*[ds[f.name] for f in self._inputs], ds=ds)
            return self._finish_model(model)
        cols = [ds[f.name] for f in self._inputs]
        model = self.fit_columns(*cols, ds=ds)
        return self._finish_model(model)

    def _finish_model(self, model: OpTransformer) -> OpTransformer:
        model.uid = self.uid
        model.operation_name = self.operation_name
        model.output_type = self.output_type
        for k, v in self.params.items():
            if k in model.params or model._accepts_param(k):
                model.params.setdefault(k, v)
        model._inputs = list(self._inputs)
        model._transient = self._transient
        model._output_name = self.get_output_feature_name()
        model._output = self.get_output()
        merged = dict(self.metadata)
        merged.update(model.metadata)
        model.metadata = merged
        model.parent = self
        return model


class UnaryTransformer(OpTransformer):
    """Elementwise transformer defined by a row function (``UnaryTransformer.scala:58-113``)."""
    arity = 1

    def __init__(self, fn: Optional[Callable] = None, uid=None, operation_name=None, output_type=None, **params):
        super().__init__(uid=uid, operation_name=operation_name, output_type=output_type, **params)
        self.fn = fn

    def transform_fn(self, v):
        return self.fn(v)

    def transform_columns(self, *cols, ds=None):
        vals = cols[0].to_list()
        out = [self.transform_fn(v) for v in vals]
        return column_from_values(self.output_type, out, cols[0].device)

    def transform_row(self, *values):
        if self.fn is None and type(self).transform_fn is UnaryTransformer.transform_fn:
            return OpTransformer.transform_row(self, *values)   # columnar-only model: one-row batch
        return _unwrap(self.transform_fn(values[0]))


class BinaryTransformer(OpTransformer):
    arity = 2

    def __init__(self, fn: Optional[Callable] = None, uid=None, operation_name=None, output_type=None, **params):
        super().__init__(uid=uid, operation_name=operation_name, output_type=output_type, **params)
        self.fn = fn

    def transform_fn(self, a, b):
        return self.fn(a, b)

    def transform_columns(self, *cols, ds=None):
        a, b = cols[0].to_list(), cols[1].to_list()
        out = [self.transform_fn(x, y) for x, y in zip(a, b)]
        return column_from_values(self.output_type, out, cols[0].device)

    def transform_row(self, *values):
        if self.fn is None and type(self).transform_fn is BinaryTransformer.transform_fn:
            return OpTransformer.transform_row(self, *values)
        return _unwrap(self.transform_fn(values[0], values[1]))


class SequenceTransformer(OpTransformer):
    arity = "N"


class SequenceEstimator(OpEstimator):
    arity = "N"


class UnaryEstimator(OpEstimator):
    arity = 1


class BinaryEstimator(OpEstimator):
    arity = 2


def _unwrap(v):
    return v.value if isinstance(v, T.FeatureType) else v
