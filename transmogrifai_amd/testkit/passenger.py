"""The reference's passenger test fixture (``PassengerFeaturesTest.scala`` + ``PassengerSparkFixtureTest.scala``):
the raw features every workflow-level reference test builds on, and the readers over ``PassengerData.avro``.

``age`` is max-aggregated, ``height`` (RealNN, 0.0 when missing) has a 300 ms window, ``gender`` is a one-element
MultiPickList (``genderPL`` the PickList twin), ``boarded`` a one-element DateList, the three maps are read as they
are, ``survived`` is the Binary response. ``data_reader`` aggregates the 8 event records of the avro file per
passenger id with the fixture's cutoff (unix 1471046600), ``simple_reader`` reads them one row per record.
"""
from __future__ import annotations

import os
from typing import List, Optional

from ..features.builder import FeatureBuilder

TEST_DATA = os.environ.get("TMOG_REFERENCE_TEST_DATA", "/root/reference/test-data")
CUTOFF_S = 1471046600
PASSENGER_TYPE = "com.salesforce.op.test.Passenger"     # the record type name reader params are keyed by


def passenger_avro_path() -> str:
    return os.path.join(TEST_DATA, "PassengerData.avro")


def available() -> bool:
    return os.path.exists(passenger_avro_path())


def _opt_float(v):
    return None if v is None else float(v)


class PassengerFeatures:
    """``PassengerFeaturesTest``: one instance = one fresh set of raw features (fresh uids)."""

    def __init__(self):
        from ..features.aggregators import MaxNumeric
        FB = FeatureBuilder
        self.age = FB.Real("age").extract(lambda p: _opt_float(p.get("age"))).aggregate(MaxNumeric()).as_predictor()
        self.gender = FB.MultiPickList("gender").extract(
            lambda p: {p["gender"]} if p.get("gender") is not None else set()).as_predictor()
        self.genderPL = FB.PickList("genderPL").extract(lambda p: p.get("gender")).as_predictor()
        self.height = FB.RealNN("height").extract(
            lambda p: float(p["height"]) if p.get("height") is not None else 0.0).window(300).as_predictor()
        self.heightNoWindow = FB.Real("heightNoWindow").extract(lambda p: _opt_float(p.get("height"))).as_predictor()
        self.weight = FB.Real("weight").extract(lambda p: _opt_float(p.get("weight"))).as_predictor()
        self.description = FB.Text("description").extract(lambda p: p.get("description")).as_predictor()
        self.boarded = FB.DateList("boarded").extract(
            lambda p: [int(p["boarded"])] if p.get("boarded") is not None else []).as_predictor()
        self.stringMap = FB.TextMap("stringMap").extract(lambda p: p.get("stringMap") or {}).as_predictor()
        self.numericMap = FB.RealMap("numericMap").extract(lambda p: p.get("numericMap") or {}).as_predictor()
        self.booleanMap = FB.BinaryMap("booleanMap").extract(lambda p: p.get("booleanMap") or {}).as_predictor()
        self.survived = FB.Binary("survived").extract(
            lambda p: None if p.get("survived") is None else p["survived"] == 1).as_response()
        self.boardedTime = FB.Date("boardedTime").extract(
            lambda p: None if p.get("boarded") is None else int(p["boarded"])).as_predictor()
        self.boardedTimeAsDateTime = FB.DateTime("boardedTimeAsDateTime").extract(
            lambda p: None if p.get("boarded") is None else int(p["boarded"])).as_predictor()

    @property
    def raw_features(self) -> List:
        return [self.survived, self.age, self.gender, self.height, self.weight, self.description, self.boarded,
                self.stringMap, self.numericMap, self.booleanMap]


def passenger_records() -> List[dict]:
    from ..readers.avro import read_avro
    return read_avro(passenger_avro_path())


def data_reader(records: Optional[List[dict]] = None):
    """``DataReaders.Aggregate.avro[Passenger]`` keyed by passenger id with the fixture's cutoff."""
    from ..features.aggregators import CutOffTime
    from ..readers.aggregate import AggregateParams
    from ..readers.files import DataReaders
    params = AggregateParams(lambda r: int(r["recordDate"]), CutOffTime.unix_epoch(CUTOFF_S))
    if records is not None:
        r = DataReaders.Aggregate.custom(records, key=lambda r: str(r["passengerId"]), aggregate_params=params)
    else:
        r = DataReaders.Aggregate.avro(passenger_avro_path(), key=lambda r: str(r["passengerId"]),
                                       aggregate_params=params)
    r.type_name = PASSENGER_TYPE
    return r


def simple_reader(records: Optional[List[dict]] = None):
    """``DataReaders.Simple.avro[Passenger]`` keyed by passenger id."""
    from ..readers.files import DataReaders
    if records is not None:
        r = DataReaders.Simple.custom(records, key=lambda r: str(r["passengerId"]))
    else:
        r = DataReaders.Simple.avro(passenger_avro_path(), key=lambda r: str(r["passengerId"]))
    r.type_name = PASSENGER_TYPE
    return r
