"""Boston housing regression, mirroring ``helloworld/.../boston/OpBoston.scala`` (GBT + RF regressors)."""
from __future__ import annotations

import os
import re
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from transmogrifai_amd.dsl import transmogrify  # noqa: E402
from transmogrifai_amd.evaluators.evaluators import Evaluators  # noqa: E402
from transmogrifai_amd.features.builder import FeatureBuilder  # noqa: E402
from transmogrifai_amd.selector.factories import RegressionModelSelector  # noqa: E402
from transmogrifai_amd.tuning.splitters import DataSplitter  # noqa: E402
from transmogrifai_amd.workflow.workflow import OpWorkflow  # noqa: E402

DEFAULT = "/root/reference/helloworld/src/main/resources/BostonDataset/housing.data"
COLS = ["crim", "zn", "indus", "chas", "nox", "rm", "age", "dis", "rad", "tax", "ptratio", "b", "lstat", "medv"]


def read(path):
    recs = []
    with open(path) as f:
        for i, line in enumerate(l for l in f if l.strip()):
            w = re.split(r"\s+", line.strip())
            r = {c: float(v) for c, v in zip(COLS, w)}
            r["chas"] = w[3]
            r["rad"] = int(w[8])
            r["rowId"] = i
            recs.append(r)
    return recs


def build(seed: int = 42, models=("OpGBTRegressor", "OpRandomForestRegressor")):
    medv = FeatureBuilder.RealNN("medv").as_response()
    feats = []
    for c in COLS[:-1]:
        if c == "chas":
            feats.append(FeatureBuilder.PickList(c).as_predictor())
        elif c == "rad":
            feats.append(FeatureBuilder.Integral(c).as_predictor())
        else:
            feats.append(FeatureBuilder.RealNN(c).as_predictor())
    house = transmogrify(feats)
    prediction = RegressionModelSelector.with_cross_validation(
        splitter=DataSplitter(seed=seed), seed=seed, model_types_to_use=list(models)).set_input(medv, house).get_output()
    return medv, prediction


def main(argv):
    recs = read(argv[0] if argv else DEFAULT)
    medv, prediction = build()
    model = OpWorkflow().set_result_features(prediction, medv).set_input_dataset(recs, key=lambda r: r["rowId"]).train()
    print(model.summary_pretty())
    ev = Evaluators.Regression().set_label_col(medv).set_prediction_col(prediction)
    _, metrics = model.score_and_evaluate(ev)
    print({k: v for k, v in metrics.items() if not isinstance(v, (dict, list))})
    return model, metrics


if __name__ == "__main__":
    main(sys.argv[1:])
