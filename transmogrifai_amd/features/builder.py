"""Raw feature definitions (``features/.../features/FeatureBuilder.scala:48-351``).

Usage mirrors the reference DSL::

    survived = FeatureBuilder.RealNN("survived").extract(lambda p: p["survived"]).as_response()
    age      = FeatureBuilder.Real("age").as_predictor()           # column extract by name
    label, predictors = FeatureBuilder.from_dataframe(df, response="survived")

A builder without ``extract`` reads the column of the same name from columnar input (the fast
path for DataFrames, Parquet/CSV and device-resident datasets).
"""
from __future__ import annotations

from typing import Callable, Iterable, Optional, Sequence, Tuple

from . import types as T
from .feature import FeatureLike


class FeatureBuilderWithExtract:
    def __init__(self, name: str, wtype, extract_fn: Optional[Callable] = None, extract_source: str = ""):
        self.name = name
        self.wtype = wtype
        self.extract_fn = extract_fn
        self.extract_source = extract_source
        self._aggregator = None
        self._window = None

    def extract(self, fn: Callable, source: str = "") -> "FeatureBuilderWithExtract":
        self.extract_fn = fn
        self.extract_source = source or getattr(fn, "__name__", "")
        return self

    def aggregate(self, aggregator) -> "FeatureBuilderWithExtract":
        self._aggregator = aggregator
        return self

    def window(self, duration_ms: int) -> "FeatureBuilderWithExtract":
        self._window = duration_ms
        return self

    def _make(self, is_response: bool) -> FeatureLike:
        from ..stages.generator import FeatureGeneratorStage
        from .aggregators import default_aggregator
        agg = self._aggregator if self._aggregator is not None else default_aggregator(self.wtype)
        stage = FeatureGeneratorStage(self.name, self.wtype, extract_fn=self.extract_fn, aggregator=agg,
                                      aggregate_window=self._window, output_is_response=is_response,
                                      extract_source=self.extract_source)
        return stage.get_output()

    def as_predictor(self) -> FeatureLike:
        return self._make(False)

    def as_response(self) -> FeatureLike:
        return self._make(True)


class _FeatureBuilderMeta(type):
    def __getattr__(cls, item):
        try:
            t = T.feature_type_from_name(item)
        except ValueError:
            raise AttributeError(item) from None
        return lambda name, extract=None: FeatureBuilderWithExtract(name, t, extract)


class FeatureBuilder(metaclass=_FeatureBuilderMeta):
    """``FeatureBuilder.<Type>(name)`` for each of the 53 feature types, plus schema inference."""

    @staticmethod
    def of(wtype, name: str, extract: Optional[Callable] = None) -> FeatureBuilderWithExtract:
        return FeatureBuilderWithExtract(name, wtype, extract)

    @staticmethod
    def from_schema(schema: Sequence[Tuple[str, str]], response: str, non_nullable: Iterable[str] = (),
                    response_type=None):
        """``schema`` = ``[(name, kind)]`` with kinds ``double|float|long|int|string|bool|date|timestamp|
        array<string>|array<long>|array<double>|map<string,...>|vector`` (``FeatureSparkTypes.scala:202-226``)."""
        nn = set(non_nullable)
        feats = []
        for name, kind in schema:
            is_resp = name == response
            nullable = not is_resp and name not in nn
            t = _type_of_kind(kind, nullable)
            b = FeatureBuilderWithExtract(name, t)
            feats.append(b.as_response() if is_resp else b.as_predictor())
        resp = [f for f in feats if f.name == response]
        if not resp:
            raise RuntimeError(f"Response feature '{response}' was not found in dataframe schema")
        r = resp[0]
        if response_type is not None and not issubclass(r.wtype, response_type):
            raise RuntimeError(f"Response feature '{response}' is of type {r.type_name}, "
                               f"but expected {response_type.type_name()}")
        return r, [f for f in feats if f.name != response]

    @staticmethod
    def from_dataframe(df, response: str, non_nullable: Iterable[str] = (), response_type=None):
        """Infer features from a pandas DataFrame's dtypes."""
        import numpy as np
        schema = []
        for name in df.columns:
            if name == "key":
                continue
            dt = df[name].dtype
            if dt.kind == "f":
                kind = "double"
            elif dt.kind in "iu":
                kind = "long"
            elif dt.kind == "b":
                kind = "bool"
            elif dt.kind == "M":
                kind = "timestamp"
            else:
                sample = next((v for v in df[name] if v is not None and not (isinstance(v, float) and v != v)), None)
                if isinstance(sample, (list, tuple, np.ndarray)):
                    kind = "array<string>" if (len(sample) == 0 or isinstance(sample[0], str)) else "array<long>"
                elif isinstance(sample, dict):
                    v0 = next(iter(sample.values()), "")
                    kind = "map<string,double>" if isinstance(v0, float) else (
                        "map<string,long>" if isinstance(v0, int) and not isinstance(v0, bool) else
                        "map<string,bool>" if isinstance(v0, bool) else "map<string,string>")
                elif isinstance(sample, bool):
                    kind = "bool"
                else:
                    kind = "string"
            if name == response and kind == "long":
                kind = "double"
            schema.append((name, kind))
        return FeatureBuilder.from_schema(schema, response, non_nullable, response_type)

    @staticmethod
    def from_dataset(ds, response: str, types: Optional[dict] = None):
        """Features for every column of a columnar :class:`Dataset` using the column types."""
        feats = []
        for name, col in ds.columns.items():
            t = (types or {}).get(name, col.ftype)
            b = FeatureBuilderWithExtract(name, t)
            feats.append(b.as_response() if name == response else b.as_predictor())
        resp = [f for f in feats if f.name == response]
        if not resp:
            raise RuntimeError(f"Response feature '{response}' was not found")
        return resp[0], [f for f in feats if f.name != response]


def _type_of_kind(kind: str, nullable: bool):
    k = kind.lower().replace(" ", "")
    if k in ("double", "float"):
        return T.Real if nullable else T.RealNN
    if k in ("long", "int", "integer", "short", "byte"):
        return T.Integral
    if k == "date":
        return T.Date
    if k == "timestamp":
        return T.DateTime
    if k == "array<string>":
        return T.TextList
    if k == "string":
        return T.Text
    if k in ("bool", "boolean"):
        return T.Binary
    if k == "array<long>":
        return T.DateList
    if k == "array<double>":
        return T.Geolocation
    if k == "map<string,string>":
        return T.TextMap
    if k == "map<string,double>":
        return T.RealMap
    if k == "map<string,long>":
        return T.IntegralMap
    if k in ("map<string,bool>", "map<string,boolean>"):
        return T.BinaryMap
    if k == "map<string,array<string>>":
        return T.MultiPickListMap
    if k == "map<string,array<double>>":
        return T.GeolocationMap
    if k == "vector":
        return T.OPVector
    raise ValueError(f"No feature type mapping for type {kind}")
