"""TimeBasedAggregatorTest.scala (features/src/test/.../aggregators/): Last / First aggregators through the
feature generator's event extraction with cutoffs and windows."""
from dataclasses import dataclass

from transmogrifai_amd.features import types as T
from transmogrifai_amd.features.aggregators import CutOffTime, FirstAggregator, LastAggregator
from transmogrifai_amd.features.builder import FeatureBuilder


@dataclass
class Rec:
    time: int
    real: float
    string: str
    map: dict


DATA = [Rec(100, 1.0, "a", {"a": "a"}), Rec(200, 2.0, "b", {"b": "b"}), Rec(300, 3.0, "c", {"c": "c"}),
        Rec(400, 4.0, "d", {"d": "d"}), Rec(500, 5.0, "e", {"e": "e"}), Rec(600, 6.0, "f", {"f": "f"})]


def _time(r):
    return r.time


def test_last_returns_the_most_recent_event():
    f = FeatureBuilder.Real("real").extract(lambda r: r.real).aggregate(LastAggregator("LastReal")).as_predictor()
    assert f.origin_stage.aggregate_records(DATA, _time, CutOffTime.no_cutoff()) == T.Real(6.0)


def test_last_within_the_response_window():
    f = FeatureBuilder.Text("s").extract(lambda r: r.string).aggregate(LastAggregator("LastText")).as_response()
    got = f.origin_stage.aggregate_records(DATA, _time, CutOffTime.unix_epoch(300), response_window=201)
    assert got == T.Text("e")


def test_last_without_events_is_empty():
    f = FeatureBuilder.TextMap("m").extract(lambda r: r.map).aggregate(LastAggregator("LastTextMap")).as_predictor()
    assert f.origin_stage.aggregate_records([], _time, CutOffTime.no_cutoff()) == T.TextMap.empty()


def test_first_returns_the_first_event_after_the_cutoff():
    f = FeatureBuilder.TextAreaMap("m").extract(lambda r: r.map).aggregate(
        FirstAggregator("FirstTextAreaMap")).as_response()
    assert f.origin_stage.aggregate_records(DATA, _time, CutOffTime.unix_epoch(301)) == T.TextAreaMap({"d": "d"})


def test_first_within_the_predictor_window():
    f = FeatureBuilder.Currency("c").extract(lambda r: r.real).aggregate(FirstAggregator("FirstCurrency")).as_predictor()
    got = f.origin_stage.aggregate_records(DATA, _time, CutOffTime.unix_epoch(400), predictor_window=201)
    assert got == T.Currency(2.0)


def test_first_without_events_is_empty():
    f = FeatureBuilder.State("s").extract(lambda r: r.string).aggregate(FirstAggregator("FirstState")).as_predictor()
    assert f.origin_stage.aggregate_records([], _time, CutOffTime.no_cutoff()) == T.State.empty()


def test_ties_and_json():
    from transmogrifai_amd.features.aggregators import Event, aggregator_from_json
    last, first = LastAggregator("LastReal"), FirstAggregator("FirstReal")
    evs = [Event(5, 1.0), Event(5, 2.0)]
    assert last.aggregate(evs) == 1.0 and first.aggregate(evs) == 2.0
    for a in (last, first):
        b = aggregator_from_json({"value": a.to_json()})
        assert b.to_json() == a.to_json()
