"""Seeded random feature-value generators (``testkit/src/main/scala/com/salesforce/op/testkit/*``).

Each generator yields values of one feature type: ``RandomReal.normal()``, ``RandomText.emails("x.com")``,
``RandomIntegral.integrals(0, 10)``, ``RandomBinary(0.3)``, ``RandomList.of_texts(...)``,
``RandomSet.of(...)``, ``RandomMap.of(...)``, ``RandomVector.dense(...)``, all with
``with_probability_of_empty(p)`` (``ProbabilityOfEmpty.scala:44-66``) and ``reset(seed)``
(``RandomData.scala:53-70``). A generator is an infinite iterator (``InfiniteStream.scala``);
``take(n)`` returns a list and ``limit(n)`` an iterator. Values are plain Python values (``None`` =
empty) so they feed ``Dataset.from_rows`` / ``TestFeatureBuilder`` directly.
"""
from __future__ import annotations

import base64 as _b64
import itertools
import math
import string
from typing import Callable, Dict, Iterator, List, Optional, Sequence

import numpy as np

from ..features import types as T


class RandomData:
    """Base infinite stream of optional values of ``ftype``."""
    ftype = T.FeatureType

    def __init__(self, producer: Callable[[np.random.Generator], object], ftype=None, seed: int = 42):
        self._producer = producer
        if ftype is not None:
            self.ftype = ftype
        self.p_empty = 0.0
        self.reset(seed)

    def reset(self, seed: int) -> "RandomData":
        self.seed = int(seed)
        self.rng = np.random.default_rng(self.seed)
        self.empty_rng = np.random.default_rng(self.seed + 1_000_003)
        return self

    def with_probability_of_empty(self, p: float) -> "RandomData":
        if not 0.0 <= p <= 1.0:
            raise ValueError("probability of empty must be in [0, 1]")
        self.p_empty = float(p)
        return self

    def __iter__(self) -> Iterator:
        return self

    def __next__(self):
        if self.p_empty > 0 and self.empty_rng.random() < self.p_empty:
            return None
        return self._producer(self.rng)

    next = __next__

    def take(self, n: int) -> List:
        return [next(self) for _ in range(n)]

    def limit(self, n: int) -> Iterator:
        return itertools.islice(self, n)


# --------------------------------------------------------------------------------------------- numeric
class RandomReal(RandomData):
    ftype = T.Real

    @staticmethod
    def uniform(min_value: float = 0.0, max_value: float = 1.0, ftype=T.Real):
        return RandomReal(lambda r: float(r.uniform(min_value, max_value)), ftype)

    @staticmethod
    def normal(mean: float = 0.0, sigma: float = 1.0, ftype=T.Real):
        return RandomReal(lambda r: float(r.normal(mean, sigma)), ftype)

    @staticmethod
    def poisson(mean: float = 0.0, ftype=T.Real):
        return RandomReal(lambda r: float(r.poisson(mean)), ftype)

    @staticmethod
    def exponential(mean: float = 1.0, ftype=T.Real):
        return RandomReal(lambda r: float(r.exponential(mean)), ftype)

    @staticmethod
    def gamma(shape: float = 1.0, scale: float = 1.0, ftype=T.Real):
        return RandomReal(lambda r: float(r.gamma(shape, scale)), ftype)

    @staticmethod
    def log_normal(mean: float = 0.0, sigma: float = 1.0, ftype=T.Real):
        return RandomReal(lambda r: float(r.lognormal(mean, sigma)), ftype)

    @staticmethod
    def weibull(alpha: float = 1.0, beta: float = 5.0, ftype=T.Real):
        return RandomReal(lambda r: float(beta * r.weibull(alpha)), ftype)


class RandomIntegral(RandomData):
    ftype = T.Integral

    @staticmethod
    def integrals(lo: int = 0, hi: int = 100, ftype=T.Integral):
        return RandomIntegral(lambda r: int(r.integers(lo, hi)), ftype)

    @staticmethod
    def dates(start_ms: int, step_ms: int, count: int = 1 << 20):
        return RandomIntegral(lambda r: int(start_ms + step_ms * int(r.integers(0, count))), T.Date)

    @staticmethod
    def datetimes(start_ms: int, end_ms: int):
        return RandomIntegral(lambda r: int(r.integers(start_ms, end_ms)), T.DateTime)


class RandomBinary(RandomData):
    ftype = T.Binary

    def __init__(self, probability_of_success: float = 0.5, seed: int = 42):
        super().__init__(lambda r: bool(r.random() < probability_of_success), T.Binary, seed)


# ------------------------------------------------------------------------------------------------ text
_ALNUM = string.ascii_letters + string.digits
_COUNTRIES = ["United States", "Canada", "Mexico", "France", "Germany", "Italy", "Spain", "Japan", "China",
              "India", "Brazil", "Argentina", "Australia", "Egypt", "Kenya", "Norway", "Sweden", "Poland",
              "Portugal", "Ireland", "Netherlands", "Belgium", "Switzerland", "Austria", "Denmark", "Finland",
              "Greece", "Turkey", "Russia", "Ukraine", "Romania", "Hungary", "Czech Republic", "Chile", "Peru",
              "Colombia", "Venezuela", "Cuba", "Nigeria", "Ghana", "Morocco", "Algeria", "Ethiopia", "South Africa",
              "Israel", "Saudi Arabia", "Iran", "Iraq", "Pakistan", "Bangladesh", "Thailand", "Vietnam",
              "Indonesia", "Philippines", "Malaysia", "Singapore", "South Korea", "New Zealand", "Iceland", "Estonia"]
_STATES = ["AL", "AK", "AZ", "AR", "CA", "CO", "CT", "DE", "FL", "GA", "HI", "ID", "IL", "IN", "IA", "KS", "KY",
           "LA", "ME", "MD", "MA", "MI", "MN", "MS", "MO", "MT", "NE", "NV", "NH", "NJ", "NM", "NY", "NC", "ND",
           "OH", "OK", "OR", "PA", "RI", "SC", "SD", "TN", "TX", "UT", "VT", "VA", "WA", "WV", "WI", "WY"]
_CITIES = ["San Jose", "San Francisco", "Los Angeles", "San Diego", "Sacramento", "Oakland", "Fresno",
           "Palo Alto", "Berkeley", "Santa Clara", "Sunnyvale", "Mountain View", "Cupertino", "Irvine", "Seattle",
           "Portland", "Boston", "New York", "Chicago", "Austin", "Denver", "Phoenix", "Dallas", "Houston",
           "Atlanta", "Miami", "Detroit", "Minneapolis", "Philadelphia", "Pittsburgh", "Baltimore", "Nashville",
           "Las Vegas", "Salt Lake City", "Albuquerque", "Tucson", "Omaha", "Kansas City", "St. Louis", "Cleveland"]
_STREETS = ["Almaden Blvd", "Santa Clara St", "First St", "Market St", "Park Ave", "Story Rd", "Tully Rd",
            "King Rd", "Capitol Expy", "Meridian Ave", "Winchester Blvd", "Bascom Ave"]


def _rand_string(r: np.random.Generator, alphabet: str, lo: int, hi: int) -> str:
    """A string of length in [lo, hi) (``RandomText.strings``: minLen inclusive, maxLen exclusive)."""
    n = int(r.integers(lo, hi)) if hi > lo else lo
    idx = r.integers(0, len(alphabet), n)
    return "".join(alphabet[i] for i in idx)


def _between(r, lo: int, hi: int) -> int:
    """The reference's ``RandomStream.randomBetween``: uniform in [lo, hi) (hi exclusive; lo when hi <= lo)."""
    lo = max(0, lo)
    hi = max(1, max(lo, hi))
    return lo if lo == hi else lo + int(r.integers(0, hi - lo))


def _select(domain: Sequence[str], dist: Sequence[float] = ()):
    dom = list(domain)
    if dist:
        p = np.asarray(dist, np.float64)
        p = p / p.sum()
        return lambda r: dom[int(r.choice(len(dom), p=p))]
    return lambda r: dom[int(r.integers(0, len(dom)))]


class RandomText(RandomData):
    ftype = T.Text

    @staticmethod
    def strings(min_len: int = 0, max_len: int = 10):
        return RandomText(lambda r: _rand_string(r, _ALNUM + " ", min_len, max_len), T.Text)

    @staticmethod
    def text_areas(min_len: int = 0, max_len: int = 100):
        return RandomText(lambda r: _rand_string(r, _ALNUM + " ", min_len, max_len), T.TextArea)

    @staticmethod
    def emails(domain: str):
        return RandomText(lambda r: _rand_string(r, string.ascii_lowercase + string.digits, 1, 10) + "@" + domain,
                          T.Email)

    @staticmethod
    def emails_on(domains: Callable[[np.random.Generator], str]):
        return RandomText(lambda r: _rand_string(r, string.ascii_lowercase, 1, 10) + "@" + domains(r), T.Email)

    @staticmethod
    def text_from_domain(domain: Sequence[str], distribution: Sequence[float] = ()):
        return RandomText(_select(domain, distribution), T.Text)

    @staticmethod
    def text_area_from_domain(domain: Sequence[str], distribution: Sequence[float] = ()):
        return RandomText(_select(domain, distribution), T.TextArea)

    @staticmethod
    def pick_lists(domain: Sequence[str], distribution: Sequence[float] = ()):
        return RandomText(_select(domain, distribution), T.PickList)

    @staticmethod
    def combo_boxes(domain: Sequence[str], distribution: Sequence[float] = ()):
        return RandomText(_select(domain, distribution), T.ComboBox)

    @staticmethod
    def countries():
        return RandomText(_select(_COUNTRIES), T.Country)

    @staticmethod
    def states():
        return RandomText(_select(_STATES), T.State)

    @staticmethod
    def cities():
        return RandomText(_select(_CITIES), T.City)

    @staticmethod
    def streets():
        return RandomText(lambda r: f"{int(r.integers(1, 9999))} {_STREETS[int(r.integers(0, len(_STREETS)))]}",
                          T.Street)

    @staticmethod
    def base64(min_len: int = 0, max_len: int = 100):
        def prod(r):
            n = int(r.integers(min_len, max_len + 1)) if max_len > min_len else min_len
            return _b64.b64encode(r.integers(0, 256, n, dtype=np.uint8).tobytes()).decode("ascii")
        return RandomText(prod, T.Base64)

    @staticmethod
    def phones():
        return RandomText(lambda r: f"{int(r.integers(200, 999))}{int(r.integers(200, 999))}{int(r.integers(0, 9999)):04d}",
                          T.Phone)

    @staticmethod
    def phones_with_errors(probability_of_error: float):
        good = RandomText.phones()._producer

        def prod(r):
            if r.random() < probability_of_error:
                return _rand_string(r, string.digits, 1, 8)
            return good(r)
        return RandomText(prod, T.Phone)

    @staticmethod
    def postal_codes():
        return RandomText(lambda r: str(101000 + int(r.integers(0, 99000)))[1:], T.PostalCode)

    @staticmethod
    def ids():
        return RandomText(lambda r: _rand_string(r, _ALNUM, 1, 12), T.ID)

    @staticmethod
    def unique_ids():
        counter = itertools.count(1)
        return RandomText(lambda r: f"{next(counter):x}_{_rand_string(r, _ALNUM, 4, 4)}", T.ID)

    @staticmethod
    def urls():
        def prod(r):
            host = _rand_string(r, string.ascii_lowercase, 3, 10)
            tld = ["com", "org", "net", "io", "edu"][int(r.integers(0, 5))]
            path = _rand_string(r, string.ascii_lowercase, 0, 8)
            return f"https://{host}.{tld}/{path}"
        return RandomText(prod, T.URL)

    @staticmethod
    def urls_on(domains: Callable[[np.random.Generator], str]):
        return RandomText(lambda r: f"http://{domains(r)}/{_rand_string(r, string.ascii_lowercase, 0, 8)}", T.URL)


# ----------------------------------------------------------------------------------------- collections
class RandomList(RandomData):
    ftype = T.TextList

    @staticmethod
    def of_texts(texts: RandomData, min_len: int = 0, max_len: int = 5):
        def prod(r):
            n = _between(r, min_len, max_len)
            return [v for v in texts.take(n) if v is not None]
        return RandomList(prod, T.TextList)

    @staticmethod
    def of_dates(dates: RandomIntegral, min_len: int = 0, max_len: int = 5, ftype=T.DateList):
        def prod(r):
            n = _between(r, min_len, max_len)
            return sorted(v for v in dates.take(n) if v is not None)
        return RandomList(prod, ftype)

    @staticmethod
    def of_geolocations():
        def prod(r):
            return [float(r.uniform(-90, 90)), float(r.uniform(-180, 180)), float(int(r.integers(1, 10)))]
        return RandomList(prod, T.Geolocation)


class RandomSet(RandomData):
    ftype = T.MultiPickList

    @staticmethod
    def of(values, min_len: int = 0, max_len: int = 3):
        """``RandomSet.of`` (``RandomSet.scala``): ``values`` is a domain sequence or, as in the reference, a
        generator whose draws fill the set (``max_len`` exclusive; a generator with a small domain gives up
        after a bounded number of draws rather than looping)."""
        if isinstance(values, RandomData):
            def prod_gen(r):
                n = _between(r, min_len, max_len)
                out: set = set()
                for _ in range(max(8 * n, 16)):
                    if len(out) >= n:
                        break
                    v = next(values)
                    if v is not None:
                        out.add(v)
                return out
            return RandomSet(prod_gen, T.MultiPickList)
        vals = list(values)

        def prod(r):
            n = min(_between(r, min_len, max_len), len(vals))
            return set(vals[i] for i in r.choice(len(vals), n, replace=False))
        return RandomSet(prod, T.MultiPickList)


class RandomMap(RandomData):
    ftype = T.RealMap

    @staticmethod
    def of(values: RandomData, min_size: int = 0, max_size: int = 5, ftype=T.RealMap,
           key_prefix: str = "k"):
        def prod(r):
            # keys "k0", "k1", ... by position, as the reference's RandomMap (RandomMap.scala asMap)
            n = _between(r, min_size, max_size)
            out = {}
            for k in range(n):
                v = next(values)
                if v is not None:
                    out[f"{key_prefix}{k}"] = v
            return out
        return RandomMap(prod, ftype)


class RandomVector(RandomData):
    ftype = T.OPVector

    @staticmethod
    def dense(values: RandomReal, length: int):
        return RandomVector(lambda r: [float(v) if v is not None else 0.0 for v in values.take(length)], T.OPVector)

    @staticmethod
    def sparse(values: RandomReal, length: int, density: Optional[float] = None):
        """``RandomVector.sparse`` (``RandomVector.scala:73``, ``asSparse`` :151): ``length`` draws of ``values``,
        an empty draw leaving its position zero -- the sparsity comes from ``values.with_probability_of_empty``.
        ``density`` additionally keeps each position with that probability."""
        def prod(r):
            out = [0.0] * length
            for i in range(length):
                if density is None or r.random() < density:
                    v = next(values)
                    out[i] = float(v) if v is not None else 0.0
            return out
        return RandomVector(prod, T.OPVector)

    @staticmethod
    def normal(mean: Sequence[float], sigma: float = 1.0):
        mu = np.asarray(mean, np.float64)
        return RandomVector(lambda r: (mu + sigma * r.standard_normal(mu.size)).tolist(), T.OPVector)

    @staticmethod
    def binary(length: int, probability_of_success: float = 0.5):
        return RandomVector(lambda r: (r.random(length) < probability_of_success).astype(np.float64).tolist(),
                            T.OPVector)


class InfiniteStream:
    """``InfiniteStream.scala``: ``map`` over an endless producer."""

    def __init__(self, producer: Callable[[], object]):
        self._p = producer

    def __iter__(self):
        return self

    def __next__(self):
        return self._p()

    def map(self, fn: Callable) -> "InfiniteStream":
        return InfiniteStream(lambda: fn(self._p()))

    def take(self, n: int) -> List:
        return [self._p() for _ in range(n)]
