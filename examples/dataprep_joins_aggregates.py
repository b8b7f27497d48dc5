"""Aggregate + joined readers, mirroring ``helloworld/.../dataprep/JoinsAndAggregates.scala``.

Two event tables (email sends and clicks) are aggregated per user around a cutoff time (04/09/2017):
predictors fold the events of a window *before* the cutoff, the response folds the day *after* it, and
the two aggregate readers are left-outer joined on the user key. ``ctr`` is derived from two features of
different readers.

The reference's "Expected Output" comment shows 0.0 where this prints None (user 456's yday clicks and
last-week sends, and ``ctr`` of users 456 / 789): under the reference code ``SumReal``'s zero is empty
(``aggregators/Numerics.scala:45,51``) and ``DivideTransformer`` yields empty for an empty operand
(``MathTransformers.scala:192-199``), which is what is implemented here; the rows with events agree.

Run: ``python examples/dataprep_joins_aggregates.py [Clicks.csv Sends.csv]``
"""
from __future__ import annotations

import datetime as _dt
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from transmogrifai_amd.dsl import core  # noqa: E402,F401  (DSL operators)
from transmogrifai_amd.features import aggregators as A  # noqa: E402
from transmogrifai_amd.features.builder import FeatureBuilder  # noqa: E402
from transmogrifai_amd.readers.aggregate import AggregateParams  # noqa: E402
from transmogrifai_amd.readers.files import DataReaders  # noqa: E402
from transmogrifai_amd.readers.joined import JoinedReader, JoinTypes  # noqa: E402
from transmogrifai_amd.workflow.workflow import OpWorkflow  # noqa: E402

DATA = "/root/reference/helloworld/src/main/resources/EmailDataset"
DAY = 86_400_000
CLICK = [("clickId", "int"), ("userId", "int"), ("emailId", "int"), ("timeStamp", "string")]
SEND = [("sendId", "int"), ("userId", "int"), ("emailId", "int"), ("timeStamp", "string")]


def parse_ts(s: str) -> int:
    t = _dt.datetime.strptime(s, "%Y-%m-%d::%H:%M:%S").replace(tzinfo=_dt.timezone.utc)
    return int(t.timestamp() * 1000)


def build():
    num_clicks_yday = FeatureBuilder.Real("numClicksYday").extract(lambda r: 1.0).aggregate(A.SumNumeric()) \
        .window(DAY).as_predictor()
    num_sends_last_week = FeatureBuilder.Real("numSendsLastWeek").extract(lambda r: 1.0) \
        .aggregate(A.SumNumeric()).window(7 * DAY).as_predictor()
    num_clicks_tomorrow = FeatureBuilder.Real("numClicksTomorrow").extract(lambda r: 1.0) \
        .aggregate(A.SumNumeric()).window(DAY).as_response()
    ctr = (num_clicks_yday / (num_sends_last_week + 1)).alias("ctr")
    return num_clicks_yday, num_sends_last_week, num_clicks_tomorrow, ctr


def main(argv):
    clicks = argv[0] if len(argv) > 0 else f"{DATA}/Clicks.csv"
    sends = argv[1] if len(argv) > 1 else f"{DATA}/Sends.csv"
    yday, sends_w, tomorrow, ctr = build()
    cutoff = A.CutOffTime.ddmmyyyy("04092017")
    clicks_reader = DataReaders.Aggregate.csv(clicks, CLICK, key=lambda r: str(r["userId"]),
                                              aggregate_params=AggregateParams(lambda r: parse_ts(r["timeStamp"]),
                                                                               cutoff))
    sends_reader = DataReaders.Aggregate.csv(sends, SEND, key=lambda r: str(r["userId"]),
                                             aggregate_params=AggregateParams(lambda r: parse_ts(r["timeStamp"]),
                                                                              cutoff))
    reader = JoinedReader(sends_reader, clicks_reader, JoinTypes.LeftOuter,
                          right_features=["numClicksYday", "numClicksTomorrow"])
    model = OpWorkflow().set_reader(reader).set_result_features(yday, tomorrow, sends_w, ctr).train()
    scores = model.score()
    rows = {}
    for i, k in enumerate(scores.key):
        rows[k] = {f.name: scores[f.name].to_list()[i] for f in (ctr, tomorrow, yday, sends_w)}
    for k in sorted(rows, reverse=True):
        print(k, rows[k])
    return rows


if __name__ == "__main__":
    main(sys.argv[1:])
