"""``TestFeatureBuilder`` (``testkit/.../test/TestFeatureBuilder.scala:65-416``): a dataset plus typed
raw features from in-memory columns, for stage tests.

    ds, (age, name) = TestFeatureBuilder.of(("age", T.Real, [1.0, None, 3.0]),
                                            ("name", T.Text, ["a", "b", None]))
    ds, feats = TestFeatureBuilder.random(100)   # one column of every common feature type
"""
from __future__ import annotations

from collections import OrderedDict
from typing import Sequence, Tuple

from ..data.columns import column_from_values
from ..data.dataset import Dataset
from ..features import types as T
from ..features.builder import FeatureBuilder
from .random_data import (RandomBinary, RandomIntegral, RandomList, RandomMap, RandomReal, RandomSet,
                          RandomText, RandomVector)


class TestFeatureBuilder:
    __test__ = False     # not a pytest test class

    @staticmethod
    def of(*columns: Tuple[str, type, Sequence], device="cpu", response: str = None):
        """``columns`` = ``(name, feature type, values)`` triples of equal length."""
        cols = OrderedDict()
        feats = []
        n = None
        for name, ftype, values in columns:
            values = list(values)
            if n is None:
                n = len(values)
            elif len(values) != n:
                raise ValueError("all columns must have the same number of rows")
            cols[name] = column_from_values(ftype, values, device)
            b = FeatureBuilder.of(ftype, name)
            feats.append(b.as_response() if name == response else b.as_predictor())
        return Dataset(cols, None, n or 0), feats

    @staticmethod
    def random(n_rows: int = 10, seed: int = 42, device="cpu"):
        """One column per commonly used feature type (``TestFeatureBuilder.random``, ``:298``)."""
        gens = [
            ("real", RandomReal.normal()),
            ("realNN", RandomReal.uniform(ftype=T.RealNN)),
            ("currency", RandomReal.log_normal(ftype=T.Currency)),
            ("percent", RandomReal.uniform(ftype=T.Percent)),
            ("integral", RandomIntegral.integrals(0, 100)),
            ("binary", RandomBinary(0.5)),
            ("date", RandomIntegral.dates(1_500_000_000_000, 86_400_000)),
            ("text", RandomText.strings(0, 20)),
            ("email", RandomText.emails("example.com")),
            ("phone", RandomText.phones()),
            ("picklist", RandomText.pick_lists(["a", "b", "c", "d"])),
            ("country", RandomText.countries()),
            ("city", RandomText.cities()),
            ("textlist", RandomList.of_texts(RandomText.strings(1, 5), 0, 3)),
            ("multipicklist", RandomSet.of(["x", "y", "z", "w"])),
            ("realmap", RandomMap.of(RandomReal.normal(), 0, 3)),
            ("vector", RandomVector.dense(RandomReal.normal(), 3)),
        ]
        columns = []
        for k, (name, g) in enumerate(gens):
            g.reset(seed + 17 * k)
            if name not in ("realNN", "vector"):
                g.with_probability_of_empty(0.2)
            columns.append((name, g.ftype, g.take(n_rows)))
        return TestFeatureBuilder.of(*columns, device=device)
