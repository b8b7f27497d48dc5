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
from .random_data import (RandomBinary, RandomData, RandomIntegral, RandomList, RandomMap, RandomReal, RandomSet,
                          RandomText, RandomVector)

_INIT_DATE_MS = 1_500_000_000_000


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
            resp = name in response if isinstance(response, (list, tuple, set)) else name == response
            feats.append(b.as_response() if resp else b.as_predictor())
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

    @staticmethod
    def random_all(n_rows: int = 10, seed: int = 42, device="cpu", text_list_min_len: int = 0):
        """One column of EVERY feature type the reference's ``TestFeatureBuilder.random`` generates
        (``TestFeatureBuilder.scala:298-397``: 52 columns -- vectors, lists, geolocations, all the typed maps,
        name stats and every scalar type), named after the type. The reference's generators are mirrored in
        kind (Poisson currencies, N(50, 5) percents, three-choice pick lists / combo boxes, country multi-pick
        lists); the draws are this package's own seeded streams."""
        d0 = _INIT_DATE_MS
        dates = lambda: RandomIntegral.dates(d0, 1000, 1000)                           # noqa: E731
        datetimes = lambda: RandomIntegral.datetimes(d0, d0 + 1000 * 1000)             # noqa: E731
        picks = ["pick1", "pick2", "pick3"]
        combos = ["choice1", "choice2", "choice3"]
        countries = RandomText.countries()._producer

        def mpl(r):
            n = int(r.integers(0, 6))
            return {countries(r) for _ in range(n)}

        def name_stats(r):
            return {"isName": "true" if r.random() < 0.5 else "false", "gender": ["Male", "Female", "GenderNA"][
                int(r.integers(0, 3))]}

        def tmap(gen, ftype):
            return RandomMap.of(gen, 0, 5, ftype=ftype)

        gens = [
            ("vector", RandomVector.sparse(RandomReal.normal(), 10)),
            ("textList", RandomList.of_texts(RandomText.strings(0, 10), text_list_min_len, 10)),
            ("dateList", RandomList.of_dates(dates(), 0, 10)),
            ("dateTimeList", RandomList.of_dates(datetimes(), 0, 10, ftype=T.DateTimeList)),
            ("geolocation", RandomList.of_geolocations()),
            ("base64Map", tmap(RandomText.base64(5, 10), T.Base64Map)),
            ("binaryMap", tmap(RandomBinary(0.5), T.BinaryMap)),
            ("comboBoxMap", tmap(RandomText.combo_boxes(combos), T.ComboBoxMap)),
            ("currencyMap", tmap(RandomReal.poisson(5.0, ftype=T.Currency), T.CurrencyMap)),
            ("dateMap", tmap(dates(), T.DateMap)),
            ("dateTimeMap", tmap(datetimes(), T.DateTimeMap)),
            ("emailMap", tmap(RandomText.emails_on(lambda r: ["example.com", "test.com"][int(r.integers(0, 2))]),
                              T.EmailMap)),
            ("idMap", tmap(RandomText.ids(), T.IDMap)),
            ("integralMap", tmap(RandomIntegral.integrals(0, 100), T.IntegralMap)),
            ("multiPickListMap", tmap(RandomData(mpl, T.MultiPickList), T.MultiPickListMap)),
            ("percentMap", tmap(RandomReal.normal(50, 5, ftype=T.Percent), T.PercentMap)),
            ("phoneMap", tmap(RandomText.phones(), T.PhoneMap)),
            ("pickListMap", tmap(RandomText.pick_lists(picks), T.PickListMap)),
            ("realMap", tmap(RandomReal.normal(), T.RealMap)),
            ("textAreaMap", tmap(RandomText.text_areas(0, 50), T.TextAreaMap)),
            ("textMap", tmap(RandomText.strings(0, 10), T.TextMap)),
            ("urlMap", tmap(RandomText.urls(), T.URLMap)),
            ("countryMap", tmap(RandomText.countries(), T.CountryMap)),
            ("stateMap", tmap(RandomText.states(), T.StateMap)),
            ("cityMap", tmap(RandomText.cities(), T.CityMap)),
            ("postalCodeMap", tmap(RandomText.postal_codes(), T.PostalCodeMap)),
            ("streetMap", tmap(RandomText.streets(), T.StreetMap)),
            ("nameStats", RandomData(name_stats, T.NameStats)),
            ("geolocationMap", tmap(RandomList.of_geolocations(), T.GeolocationMap)),
            ("binary", RandomBinary(0.5)),
            ("currency", RandomReal.poisson(5.0, ftype=T.Currency)),
            ("date", dates()),
            ("dateTime", datetimes()),
            ("integral", RandomIntegral.integrals(0, 100)),
            ("percent", RandomReal.normal(50, 5, ftype=T.Percent)),
            ("real", RandomReal.normal()),
            ("realNN", RandomReal.normal(ftype=T.RealNN)),
            ("multiPickList", RandomData(mpl, T.MultiPickList)),
            ("base64", RandomText.base64(5, 10)),
            ("comboBox", RandomText.combo_boxes(combos)),
            ("email", RandomText.emails_on(lambda r: ["example.com", "test.com"][int(r.integers(0, 2))])),
            ("id", RandomText.ids()),
            ("phone", RandomText.phones()),
            ("pickList", RandomText.pick_lists(picks)),
            ("text", RandomData(RandomText.base64(5, 10)._producer, T.Text)),
            ("textArea", RandomText.text_areas(0, 50)),
            ("url", RandomText.urls()),
            ("country", RandomText.countries()),
            ("state", RandomText.states()),
            ("city", RandomText.cities()),
            ("postalCode", RandomText.postal_codes()),
            ("street", RandomText.streets()),
        ]
        columns = []
        for k, (name, g) in enumerate(gens):
            g.reset(seed + 31 * k)
            if g.ftype.kind in ("map", "vector") or g.ftype in (T.RealNN,) or name in ("textList", "dateList",
                                                                                      "dateTimeList", "geolocation",
                                                                                      "multiPickList", "nameStats"):
                pass
            else:
                g.with_probability_of_empty(0.1)
            columns.append((name, g.ftype, g.take(n_rows)))
        return TestFeatureBuilder.of(*columns, device=device)
