"""Feature type system.

The 53 concrete feature types of the reference
(``features/src/main/scala/com/salesforce/op/features/types/FeatureType.scala:265-325`` registry;
numerics ``Numerics.scala:40-155``, text ``Text.scala:48-305``, lists ``Lists.scala:40-80``,
sets ``Sets.scala:38``, geolocation ``Geolocation.scala:47-206``, vector ``OPVector.scala:41-91``,
maps ``Maps.scala:40-461``).

Each class is a small value container used on the *row* path (local scoring, test kits). On the
batch path a feature is stored as a column whose storage ``kind`` is a class attribute here
(see :mod:`transmogrifai_amd.data.columns`): numeric → values tensor + validity mask, text →
dictionary codes + vocabulary, vector → dense tensor + column metadata, and so on.
"""
from __future__ import annotations

import math
from typing import Any, Dict, Optional

import numpy as np


class NonNullableEmptyException(ValueError):
    pass


class FeatureType:
    """Root of the hierarchy (reference ``FeatureType.scala:44-116``)."""

    kind = "abstract"          # column storage kind
    nullable = True
    categorical = False
    single_response = False
    multi_response = False
    location = False

    __slots__ = ("value",)

    def __init__(self, value=None):
        self.value = self._convert(value)

    @classmethod
    def _convert(cls, v):
        return v

    @property
    def is_empty(self) -> bool:
        v = self.value
        if v is None:
            return True
        if isinstance(v, (list, tuple, set, frozenset, dict)):
            return len(v) == 0
        return False

    @property
    def non_empty(self) -> bool:
        return not self.is_empty

    @classmethod
    def type_name(cls) -> str:
        return f"com.salesforce.op.features.types.{cls.__name__}"

    @classmethod
    def short_name(cls) -> str:
        return cls.__name__

    @classmethod
    def empty(cls):
        return cls(None)

    def __eq__(self, other):
        return type(self) is type(other) and _values_equal(self.value, other.value)

    def __hash__(self):
        v = self.value
        if isinstance(v, dict):
            v = tuple(sorted(v.items()))
        elif isinstance(v, (list, set, frozenset)):
            v = tuple(v)
        elif isinstance(v, np.ndarray):
            v = tuple(v.tolist())
        return hash((type(self).__name__, v))

    def __repr__(self):
        return f"{type(self).__name__}({self.value!r})"


def _values_equal(a, b):
    if isinstance(a, np.ndarray) or isinstance(b, np.ndarray):
        return np.array_equal(np.asarray(a), np.asarray(b))
    if isinstance(a, float) and isinstance(b, float) and math.isnan(a) and math.isnan(b):
        return True
    return a == b


# ----------------------------------------------------------------------------------------- numerics
class OPNumeric(FeatureType):
    kind = "numeric"
    dtype = "float64"

    def to_double(self) -> Optional[float]:
        return None if self.value is None else float(self.value)


class Real(OPNumeric):
    @classmethod
    def _convert(cls, v):
        if v is None:
            return None
        if isinstance(v, float) and math.isnan(v):
            return None
        return float(v)


class RealNN(Real):
    """Non-nullable real: constructing an empty value throws (``Numerics.scala:59``)."""
    nullable = False

    def __init__(self, value=None):
        if value is None or (isinstance(value, float) and math.isnan(value)):
            raise NonNullableEmptyException("RealNN cannot be empty")
        super().__init__(value)


class Percent(Real):
    pass


class Currency(Real):
    pass


class Binary(OPNumeric):
    single_response = True
    categorical = True
    dtype = "bool"

    @classmethod
    def _convert(cls, v):
        if v is None:
            return None
        if isinstance(v, float) and math.isnan(v):
            return None
        return bool(v)

    def to_double(self):
        return None if self.value is None else (1.0 if self.value else 0.0)


class Integral(OPNumeric):
    dtype = "int64"

    @classmethod
    def _convert(cls, v):
        if v is None:
            return None
        if isinstance(v, float) and math.isnan(v):
            return None
        return int(v)


class Date(Integral):
    """Milliseconds since epoch (UTC)."""


class DateTime(Date):
    pass


# --------------------------------------------------------------------------------------------- text
class Text(FeatureType):
    kind = "text"

    @classmethod
    def _convert(cls, v):
        if v is None:
            return None
        if isinstance(v, float) and math.isnan(v):
            return None
        return str(v)


class Email(Text):
    """``Email`` (types/Text.scala:60-95): prefix / domain are the groups of ``Email.pattern``, None when the
    value does not parse."""

    def prefix(self):
        from ..utils.text import email_prefix
        return email_prefix(self.value)

    def domain(self):
        from ..utils.text import email_domain
        return email_domain(self.value)


class Base64(Text):
    """``Base64`` (types/Text.scala:100-140): the decoded bytes / UTF-8 string, None when empty."""

    def as_bytes(self) -> Optional[bytes]:
        import base64
        return None if self.value is None else base64.b64decode(self.value)

    def as_string(self) -> Optional[str]:
        b = self.as_bytes()
        return None if b is None else b.decode("utf-8")

    def map_input_stream(self, fn):
        import io
        b = self.as_bytes()
        return None if b is None else fn(io.BytesIO(b))


class Phone(Text):
    pass


class ID(Text):
    pass


class URL(Text):
    """``URL`` (types/Text.scala:160-190): validity per Apache UrlValidator's default schemes (or the given
    ``protocols``), host and protocol of the parsed URL."""

    def is_valid(self, protocols=None) -> bool:
        from ..utils.text import is_valid_url
        if self.value is None:
            return False
        return is_valid_url(self.value) if protocols is None else is_valid_url(self.value, tuple(protocols))

    def domain(self):
        from ..utils.text import url_domain
        return None if self.value is None else url_domain(self.value)

    def protocol(self):
        from ..utils.text import url_protocol
        return None if self.value is None else url_protocol(self.value)


class TextArea(Text):
    pass


class PickList(Text):
    single_response = True
    categorical = True


class ComboBox(Text):
    pass


class Country(Text):
    location = True


class State(Text):
    location = True


class PostalCode(Text):
    location = True


class City(Text):
    location = True


class Street(Text):
    location = True


# ---------------------------------------------------------------------------------------- collections
class OPCollection(FeatureType):
    pass


class OPList(OPCollection):
    kind = "list"

    @classmethod
    def _convert(cls, v):
        if v is None:
            return []
        return list(v)


class TextList(OPList):
    elem = str


class DateList(OPList):
    elem = int

    @classmethod
    def _convert(cls, v):
        return [] if v is None else [int(x) for x in v]


class DateTimeList(DateList):
    pass


class Geolocation(OPList):
    """(lat, lon, accuracy) triple (``Geolocation.scala:47-206``)."""
    kind = "geo"
    location = True

    @classmethod
    def _convert(cls, v):
        if v is None:
            return []
        v = [float(x) for x in v]
        if v and len(v) != 3:
            raise ValueError("Geolocation must have lat, lon, and accuracy, or be empty")
        if v:
            lat, lon = v[0], v[1]
            if not (-90.0 <= lat <= 90.0) or not (-180.0 <= lon <= 180.0):
                raise ValueError(f"Invalid geolocation {v}")
            if v[2] != int(v[2]) or not 0 <= int(v[2]) <= 10:      # a GeolocationAccuracy value
                raise ValueError(f"Invalid geolocation accuracy {v[2]}")
        return v

    @property
    def lat(self) -> float:
        """Latitude; NaN when empty (``Geolocation.lat``)."""
        return self.value[0] if self.value else float("nan")

    @property
    def lon(self) -> float:
        return self.value[1] if self.value else float("nan")

    @property
    def accuracy(self) -> int:
        """GeolocationAccuracy value; Unknown (0) when empty."""
        return int(self.value[2]) if self.value else 0

    def to_geo_point(self):
        """The spatial3d WGS84 ``GeoPoint`` (x, y, z) of the location; (0, 0, 0) when empty."""
        if not self.value:
            return (0.0, 0.0, 0.0)
        import torch
        from .geo import prepare
        return tuple(prepare(torch.tensor([self.value], dtype=torch.float64))[0, :3].tolist())


class OrderedSet(frozenset):
    """A ``frozenset`` that iterates in a fixed order: the order of the sequence it was built from (Scala's small
    immutable sets Set1..Set4 iterate in insertion order, which ``SetNGramSimilarity``'s ``mkString(" ")``
    exposes, NGramSimilarity.scala:53), or sorted when built from an unordered set -- never Python's
    per-process string-hash order. Equality and hashing are the plain set's."""

    def __new__(cls, items=()):
        if isinstance(items, OrderedSet):
            return items
        if isinstance(items, (set, frozenset)):
            seq = sorted(items, key=lambda e: (type(e).__name__, str(e)))
        else:
            seq = list(dict.fromkeys(items))
        o = super().__new__(cls, seq)
        o._order = tuple(seq)
        return o

    def __iter__(self):
        return iter(self._order)

    def __reduce__(self):
        return (OrderedSet, (list(self._order),))

    def __repr__(self):
        return f"OrderedSet({list(self._order)!r})"


class OPSet(OPCollection):
    kind = "set"
    multi_response = True
    categorical = True

    @classmethod
    def _convert(cls, v):
        if v is None:
            return OrderedSet()
        return OrderedSet(v)


class MultiPickList(OPSet):
    pass


class OPVector(OPCollection):
    kind = "vector"

    @classmethod
    def _convert(cls, v):
        if v is None:
            return np.zeros(0)
        return np.asarray(v, dtype=np.float64)

    @property
    def is_empty(self):
        return self.value.size == 0


# ----------------------------------------------------------------------------------------------- maps
class OPMap(OPCollection):
    kind = "map"
    value_kind = "text"

    @classmethod
    def _convert(cls, v):
        if v is None:
            return {}
        return dict(v)


class TextMap(OPMap):
    pass


class EmailMap(TextMap):
    pass


class Base64Map(TextMap):
    pass


class PhoneMap(TextMap):
    pass


class IDMap(TextMap):
    pass


class URLMap(TextMap):
    pass


class TextAreaMap(TextMap):
    pass


class PickListMap(TextMap):
    single_response = True
    categorical = True


class ComboBoxMap(TextMap):
    pass


class CountryMap(TextMap):
    location = True


class StateMap(TextMap):
    location = True


class CityMap(TextMap):
    location = True


class PostalCodeMap(TextMap):
    location = True


class StreetMap(TextMap):
    location = True


class NameStats(TextMap):
    pass


class NumericMap(OPMap):
    pass


class BinaryMap(NumericMap):
    value_kind = "binary"
    single_response = True
    categorical = True


class IntegralMap(NumericMap):
    value_kind = "integral"


class RealMap(NumericMap):
    value_kind = "real"


class PercentMap(RealMap):
    pass


class CurrencyMap(RealMap):
    pass


class DateMap(IntegralMap):
    pass


class DateTimeMap(DateMap):
    pass


class MultiPickListMap(OPMap):
    value_kind = "set"
    multi_response = True
    categorical = True


class GeolocationMap(OPMap):
    value_kind = "geo"
    location = True


class Prediction(RealMap):
    """Non-nullable prediction map with keys ``prediction``, ``rawPrediction_i``, ``probability_i``
    (``Maps.scala:339-435``)."""
    kind = "prediction"
    nullable = False
    PredictionName = "prediction"
    RawPredictionName = "rawPrediction"
    ProbabilityName = "probability"

    def __init__(self, value=None, prediction=None, raw_prediction=None, probability=None):
        if value is None or (isinstance(value, dict) and not value and prediction is not None):
            if prediction is None:
                raise NonNullableEmptyException("Prediction cannot be empty")
            value = {self.PredictionName: float(prediction)}
            for i, r in enumerate([] if raw_prediction is None else list(raw_prediction)):
                value[f"{self.RawPredictionName}_{i}"] = float(r)
            for i, p in enumerate([] if probability is None else list(probability)):
                value[f"{self.ProbabilityName}_{i}"] = float(p)
        if not isinstance(value, dict) or not value:
            raise NonNullableEmptyException("Prediction cannot be empty")
        if self.PredictionName not in value:        # Maps.scala:350-362
            raise NonNullableEmptyException(
                f"Prediction cannot be empty: value map must contain '{self.PredictionName}' key")
        bad = [k for k in value if k != self.PredictionName and not k.startswith(self.RawPredictionName)
               and not k.startswith(self.ProbabilityName)]
        if bad:
            raise ValueError(f"requirement failed: value map must only contain valid keys: '{self.PredictionName}' "
                             f"or starting with '{self.RawPredictionName}' or '{self.ProbabilityName}'")
        FeatureType.__init__(self, value)

    def __str__(self):
        def arr(v):
            return "Array(" + ", ".join(repr(float(x)) for x in v) + ")"
        return (f"Prediction(prediction = {float(self.prediction)!r}, rawPrediction = {arr(self.raw_prediction)}, "
                f"probability = {arr(self.probability)})")

    @property
    def prediction(self) -> float:
        return self.value[self.PredictionName]

    def _vec(self, prefix):
        ks = sorted((k for k in self.value if k.startswith(prefix + "_")),
                    key=lambda k: int(k.rsplit("_", 1)[1]))
        return [self.value[k] for k in ks]

    @property
    def raw_prediction(self):
        return self._vec(self.RawPredictionName)

    @property
    def probability(self):
        return self._vec(self.ProbabilityName)

    @property
    def score(self):
        p = self.probability
        return p if p else [self.prediction]


# ------------------------------------------------------------------------------------------ registry
ALL_TYPES = [
    OPVector, TextList, DateList, DateTimeList, Geolocation,
    Base64Map, BinaryMap, ComboBoxMap, CurrencyMap, DateMap, DateTimeMap, EmailMap, IDMap,
    IntegralMap, MultiPickListMap, PercentMap, PhoneMap, PickListMap, RealMap, TextAreaMap, TextMap,
    URLMap, CountryMap, StateMap, CityMap, PostalCodeMap, StreetMap, NameStats, GeolocationMap,
    Prediction,
    Binary, Currency, Date, DateTime, Integral, Percent, Real, RealNN,
    MultiPickList,
    Base64, ComboBox, Email, ID, Phone, PickList, Text, TextArea, URL, Country, State, City,
    PostalCode, Street,
]
assert len(ALL_TYPES) == 53, len(ALL_TYPES)

_BY_NAME: Dict[str, type] = {}
for _t in ALL_TYPES:
    _BY_NAME[_t.__name__] = _t
    _BY_NAME[_t.type_name()] = _t


def feature_type_from_name(name: str) -> type:
    """Resolve a short (``Real``) or fully-qualified (``com.salesforce...Real``) type name."""
    t = _BY_NAME.get(name) or _BY_NAME.get(name.rsplit(".", 1)[-1])
    if t is None:
        raise ValueError(f"Unknown feature type '{name}'")
    return t


def is_subtype(t: type, parent: type) -> bool:
    return isinstance(t, type) and issubclass(t, parent)


TEXT_TYPES = [t for t in ALL_TYPES if issubclass(t, Text)]
NUMERIC_TYPES = [t for t in ALL_TYPES if issubclass(t, OPNumeric)]
MAP_TYPES = [t for t in ALL_TYPES if issubclass(t, OPMap)]


def default_value(t: type) -> Any:
    """Empty python value for a type (reference ``FeatureTypeDefaults.scala``)."""
    if issubclass(t, Prediction):
        return None
    if issubclass(t, (OPNumeric, Text)):
        return None
    if issubclass(t, OPVector):
        return np.zeros(0)
    if issubclass(t, OPSet):
        return frozenset()
    if issubclass(t, OPList):
        return []
    if issubclass(t, OPMap):
        return {}
    return None
