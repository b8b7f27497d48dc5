"""Conditional aggregation reader, mirroring ``helloworld/.../dataprep/ConditionalAggregation.scala``.

Each user's web visits are aggregated around the first visit that meets a target condition (a visit to
``/SaveBig``): visits in the week before it are the predictor, purchases in the day after it the response;
users that never meet the condition are dropped.

Run: ``python examples/dataprep_conditional_aggregation.py [WebVisits.csv]``
"""
from __future__ import annotations

import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from transmogrifai_amd.features import aggregators as A  # noqa: E402
from transmogrifai_amd.features.builder import FeatureBuilder  # noqa: E402
from transmogrifai_amd.readers.aggregate import ConditionalParams  # noqa: E402
from transmogrifai_amd.readers.files import DataReaders  # noqa: E402
from transmogrifai_amd.workflow.workflow import OpWorkflow  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from dataprep_joins_aggregates import DAY, parse_ts  # noqa: E402

DATA = "/root/reference/helloworld/src/main/resources/WebVisitsDataset/WebVisits.csv"
VISIT = [("userId", "string"), ("url", "string"), ("productId", "int"), ("price", "double"),
         ("timestamp", "string")]


def main(argv):
    path = argv[0] if argv else DATA
    visits_week_prior = FeatureBuilder.RealNN("numVisitsWeekPrior").extract(lambda r: 1.0) \
        .aggregate(A.SumRealNN()).window(7 * DAY).as_predictor()
    purchases_next_day = FeatureBuilder.RealNN("numPurchasesNextDay").extract(
        lambda r: 0.0 if r["productId"] is None or r["productId"] != r["productId"] else 1.0) \
        .aggregate(A.SumRealNN()).window(DAY).as_response()
    params = ConditionalParams(timestamp_fn=lambda r: parse_ts(r["timestamp"]),
                               target_condition=lambda r: r["url"] == "http://www.amazon.com/SaveBig",
                               response_window_ms=DAY, drop_if_target_condition_not_met=True)
    reader = DataReaders.Conditional.csv(path, VISIT, key=lambda r: r["userId"], conditional_params=params)
    model = OpWorkflow().set_reader(reader).set_result_features(visits_week_prior, purchases_next_day).train()
    scores = model.score()
    rows = {k: {"numPurchasesNextDay": scores["numPurchasesNextDay"].to_list()[i],
                "numVisitsWeekPrior": scores["numVisitsWeekPrior"].to_list()[i]} for i, k in enumerate(scores.key)}
    for k in sorted(rows, reverse=True):
        print(k, rows[k])
    return rows


if __name__ == "__main__":
    main(sys.argv[1:])
