"""Per-column provenance of a feature vector.

Equivalent of ``OpVectorColumnMetadata`` (``features/.../utils/spark/OpVectorColumnMetadata.scala:40-216``)
and ``OpVectorMetadata`` (``OpVectorMetadata.scala:51-277``, keys ``vector_columns``,
``vector_history``, ``vector_detected_sensitive`` at ``:187-189``). The metadata lives on the host
and drives column offsets of the device-resident feature matrix.
"""
from __future__ import annotations

from functools import lru_cache

from dataclasses import dataclass, field, replace
from typing import Dict, List, Optional, Sequence

NULL_STRING = "NullIndicatorValue"
TEXT_LEN_STRING = "TextLenValue"
OTHER_STRING = "OTHER"


@dataclass(frozen=True)
class FeatureHistory:
    origin_features: tuple
    stages: tuple

    def merge(self, *others: "FeatureHistory") -> "FeatureHistory":
        of = list(self.origin_features)
        st = list(self.stages)
        for o in others:
            of += list(o.origin_features)
            st += list(o.stages)
        return FeatureHistory(tuple(sorted(set(of))), tuple(sorted(set(st))))

    def to_json(self):
        return {"originFeatures": list(self.origin_features), "stages": list(self.stages)}

    @staticmethod
    def from_json(d):
        return FeatureHistory(tuple(d.get("originFeatures", [])), tuple(d.get("stages", [])))

    @staticmethod
    def map_to_json(m: dict) -> dict:
        """``FeatureHistory.toMetadata(map)`` (FeatureHistory.scala:81-91): one entry per feature name."""
        return {k: v.to_json() for k, v in m.items()}

    @staticmethod
    def map_from_json(d: dict) -> dict:
        """``FeatureHistory.fromMetadataMap`` (FeatureHistory.scala:93-102)."""
        return {k: FeatureHistory.from_json(v) for k, v in d.items()}


@lru_cache(maxsize=4096)
def _has_subtype(type_names: tuple, t) -> bool:
    """Any of the parent type names a subclass of ``t`` (memoised: the SanityChecker asks for every column of
    wide text vectors, whose columns share a few parent-type tuples)."""
    from ..features.types import feature_type_from_name
    return any(issubclass(feature_type_from_name(n), t) for n in type_names)


@dataclass(frozen=True)
class OpVectorColumnMetadata:
    parent_feature_name: tuple
    parent_feature_type: tuple
    grouping: Optional[str] = None
    indicator_value: Optional[str] = None
    descriptor_value: Optional[str] = None
    index: int = 0

    def __post_init__(self):
        # sequences are stored as tuples: the metadata is hashed / grouped by its (name, type) key
        if not isinstance(self.parent_feature_name, tuple):
            object.__setattr__(self, "parent_feature_name", tuple(self.parent_feature_name))
        if not isinstance(self.parent_feature_type, tuple):
            object.__setattr__(self, "parent_feature_type", tuple(self.parent_feature_type))
        if not self.parent_feature_name:
            raise ValueError("must provide parent feature name")
        if len(self.parent_feature_name) != len(self.parent_feature_type):
            raise ValueError("must provide both type and name for every parent feature")
        if self.indicator_value is not None and self.descriptor_value is not None:
            raise ValueError("cannot have both indicatorValue and descriptorValue")

    @property
    def is_null_indicator(self) -> bool:
        return self.indicator_value == NULL_STRING

    @property
    def is_other_indicator(self) -> bool:
        return self.indicator_value == OTHER_STRING

    def make_col_name(self) -> str:
        s = "_".join(self.parent_feature_name)
        if self.grouping is not None:
            s += "_" + self.grouping
        if self.indicator_value is not None:
            s += "_" + self.indicator_value
        if self.descriptor_value is not None:
            s += "_" + self.descriptor_value
        return f"{s}_{self.index}"

    def has_parent_of_subtype(self, t) -> bool:
        return _has_subtype(self.parent_feature_type, t)

    def parent_names_with_map_keys(self) -> List[str]:
        from ..features.types import OPMap
        if self.has_parent_of_subtype(OPMap):
            return [p + "_" + self.grouping if self.grouping is not None else p
                    for p in self.parent_feature_name]
        return list(self.parent_feature_name)

    def feature_group(self) -> Optional[str]:
        return None if self.grouping is None else "_".join(self.parent_feature_name) + "_" + self.grouping

    def with_index(self, i: int) -> "OpVectorColumnMetadata":
        return replace(self, index=i)

    def key(self):
        return (self.parent_feature_name, self.parent_feature_type, self.grouping,
                self.indicator_value, self.descriptor_value)

    def to_json(self, indices=None):
        d = {"parent_feature": list(self.parent_feature_name),
             "parent_feature_type": list(self.parent_feature_type),
             "indices": list(indices) if indices is not None else [self.index]}
        if self.grouping is not None:
            d["grouping"] = self.grouping
        if self.indicator_value is not None:
            d["indicator_value"] = self.indicator_value
        if self.descriptor_value is not None:
            d["descriptor_value"] = self.descriptor_value
        return d

    @staticmethod
    def from_json(d) -> List["OpVectorColumnMetadata"]:
        base = OpVectorColumnMetadata(
            tuple(d["parent_feature"]), tuple(d["parent_feature_type"]),
            d.get("grouping", d.get("indicator_group")),     # pre-0.5 checkpoints: indicator_group
            d.get("indicator_value"), d.get("descriptor_value"), 0)
        return [base.with_index(int(i)) for i in d.get("indices", [0])]


@dataclass
class OpVectorMetadata:
    name: str
    columns: List[OpVectorColumnMetadata]
    history: Dict[str, FeatureHistory] = field(default_factory=dict)
    sensitive: Dict[str, list] = field(default_factory=dict)

    def __post_init__(self):
        self.columns = [c if c.index == i else c.with_index(i) for i, c in enumerate(self.columns)]

    @property
    def size(self) -> int:
        return len(self.columns)

    def column_names(self) -> List[str]:
        return [c.make_col_name() for c in self.columns]

    def select(self, indices: Sequence[int], name: Optional[str] = None) -> "OpVectorMetadata":
        cols = [self.columns[i] for i in indices]
        return OpVectorMetadata(name or self.name, cols, dict(self.history), dict(self.sensitive))

    def with_name(self, name) -> "OpVectorMetadata":
        return OpVectorMetadata(name, list(self.columns), dict(self.history), dict(self.sensitive))

    def index_of(self, column: OpVectorColumnMetadata) -> int:
        m = [i for i, c in enumerate(self.columns) if c == column]
        if not m:
            raise ValueError(f"No instance of {column} found")
        if len(m) > 1:
            raise ValueError(f"Multiple instances of {column} found at {m}")
        return m[0]

    def column_history(self):
        out = []
        for c in self.columns:
            hs = [self.history.get(p) for p in c.parent_feature_name]
            hs = [h for h in hs if h is not None]
            comb = hs[0].merge(*hs[1:]) if hs else FeatureHistory((), ())
            out.append({
                "columnName": c.make_col_name(),
                "parentFeatureName": list(c.parent_feature_name),
                "parentFeatureOrigins": list(comb.origin_features),
                "parentFeatureStages": list(comb.stages),
                "parentFeatureType": list(c.parent_feature_type),
                "grouping": c.grouping, "indicatorValue": c.indicator_value,
                "descriptorValue": c.descriptor_value, "index": c.index})
        return out

    def to_json(self):
        groups: Dict[tuple, list] = {}
        order = []
        for c in self.columns:
            k = c.key()
            if k not in groups:
                groups[k] = []
                order.append((k, c))
            groups[k].append(c.index)
        return {
            "vector_columns": [c.to_json(groups[k]) for k, c in order],
            "vector_history": {k: v.to_json() for k, v in self.history.items()},
            "vector_detected_sensitive": dict(self.sensitive),
        }

    @staticmethod
    def from_json(name: str, d) -> "OpVectorMetadata":
        cols = []
        for cd in d.get("vector_columns", []):
            cols.extend(OpVectorColumnMetadata.from_json(cd))
        cols.sort(key=lambda c: c.index)
        hist = {k: FeatureHistory.from_json(v) for k, v in d.get("vector_history", {}).items()}
        return OpVectorMetadata(name, cols, hist, dict(d.get("vector_detected_sensitive", {})))

    @staticmethod
    def flatten(output_name: str, vectors: Sequence["OpVectorMetadata"]) -> "OpVectorMetadata":
        cols = [c for v in vectors for c in v.columns]
        hist = {}
        sens = {}
        for v in vectors:
            hist.update(v.history)
            sens.update(v.sensitive)
        return OpVectorMetadata(output_name, cols, hist, sens)
