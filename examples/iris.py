"""Iris multiclass, mirroring ``helloworld/.../iris/OpIris.scala`` (MultiClassificationModelSelector + DataCutter)."""
from __future__ import annotations

import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from transmogrifai_amd.dsl import transmogrify  # noqa: E402
from transmogrifai_amd.evaluators.evaluators import Evaluators  # noqa: E402
from transmogrifai_amd.features.builder import FeatureBuilder  # noqa: E402
from transmogrifai_amd.readers.files import CSVReader  # noqa: E402
from transmogrifai_amd.selector.factories import MultiClassificationModelSelector  # noqa: E402
from transmogrifai_amd.tuning.splitters import DataCutter  # noqa: E402
from transmogrifai_amd.workflow.workflow import OpWorkflow  # noqa: E402

DEFAULT = "/root/reference/helloworld/src/main/resources/IrisDataset/iris.data"
SCHEMA = [("sepalLength", "double"), ("sepalWidth", "double"), ("petalLength", "double"),
          ("petalWidth", "double"), ("irisClass", "string")]


def build(seed: int = 42):
    sl = FeatureBuilder.Real("sepalLength").as_predictor()
    sw = FeatureBuilder.Real("sepalWidth").as_predictor()
    pl = FeatureBuilder.Real("petalLength").as_predictor()
    pw = FeatureBuilder.Real("petalWidth").as_predictor()
    iris_class = FeatureBuilder.Text("irisClass").as_response()
    labels = iris_class.indexed()
    features = transmogrify([sl, sw, pl, pw])
    cutter = DataCutter(reserve_test_fraction=0.2, seed=seed)
    prediction = MultiClassificationModelSelector.with_cross_validation(splitter=cutter, seed=seed) \
        .set_input(labels, features).get_output()
    return labels, prediction


def main(argv):
    path = argv[0] if argv else DEFAULT
    labels, prediction = build()
    wf = OpWorkflow().set_result_features(prediction, labels).set_reader(CSVReader(path, SCHEMA))
    model = wf.train()
    print(model.summary_pretty())
    ev = Evaluators.MultiClassification.f1().set_label_col(labels).set_prediction_col(prediction)
    _, metrics = model.score_and_evaluate(ev)
    print({k: v for k, v in metrics.items() if not isinstance(v, dict)})
    return model, metrics


if __name__ == "__main__":
    main(sys.argv[1:])
