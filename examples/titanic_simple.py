"""Titanic binary classification, mirroring ``helloworld/.../OpTitanicSimple.scala:60-177``.

The reference example restricts the selector to ``OpLogisticRegression`` (``OpTitanicSimple.scala:134-136``)
and that is the default here too; ``--all`` runs the full default binary grid (LR, RF, XGBoost), the
setting of the README's model summary (RF selected, hold-out AuPR 0.8225, ``README.md:61-126``).

Run: ``python examples/titanic_simple.py [path/to/PassengerDataAll.csv] [--all] [--quiet] [--seed=N]``
"""
from __future__ import annotations

import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from transmogrifai_amd.features.builder import FeatureBuilder  # noqa: E402
from transmogrifai_amd.features import types as T  # noqa: E402
from transmogrifai_amd.dsl import transmogrify  # noqa: E402
from transmogrifai_amd.readers.files import CSVReader  # noqa: E402
from transmogrifai_amd.selector.factories import BinaryClassificationModelSelector  # noqa: E402
from transmogrifai_amd.evaluators.evaluators import Evaluators  # noqa: E402
from transmogrifai_amd.workflow.workflow import OpWorkflow  # noqa: E402

SCHEMA = [("id", "int"), ("survived", "int"), ("pClass", "int"), ("name", "string"), ("sex", "string"),
          ("age", "double"), ("sibSp", "int"), ("parCh", "int"), ("ticket", "string"), ("fare", "double"),
          ("cabin", "string"), ("embarked", "string")]

DEFAULT_CSV = "/root/reference/test-data/PassengerDataAll.csv"


def build(lr_only: bool = True, seed=None):
    survived = FeatureBuilder.RealNN("survived").extract(lambda r: float(r["survived"])).as_response()
    p_class = FeatureBuilder.PickList("pClass").extract(
        lambda r: None if r["pClass"] != r["pClass"] else str(int(r["pClass"]))).as_predictor()
    name = FeatureBuilder.Text("name").as_predictor()
    sex = FeatureBuilder.PickList("sex").as_predictor()
    age = FeatureBuilder.Real("age").as_predictor()
    sib_sp = FeatureBuilder.Integral("sibSp").as_predictor()
    par_ch = FeatureBuilder.Integral("parCh").as_predictor()
    ticket = FeatureBuilder.PickList("ticket").as_predictor()
    fare = FeatureBuilder.Real("fare").as_predictor()
    cabin = FeatureBuilder.PickList("cabin").as_predictor()
    embarked = FeatureBuilder.PickList("embarked").as_predictor()

    family_size = sib_sp + par_ch + 1
    estimated_cost = family_size * fare
    pivoted_sex = sex.pivot()
    normed_age = age.fill_missing_with_mean().z_normalize()
    age_group = age.map(lambda v: None if v is None else ("adult" if v > 18 else "child"), output_type=T.PickList)

    passenger_features = transmogrify([p_class, name, age, sib_sp, par_ch, ticket, cabin, embarked,
                                       family_size, estimated_cost, pivoted_sex, age_group, normed_age])
    checked = survived.sanity_check(passenger_features, remove_bad_features=True)
    types = ["OpLogisticRegression"] if lr_only else None
    prediction = BinaryClassificationModelSelector.with_train_validation_split(
        model_types_to_use=types, seed=seed).set_input(survived, checked).get_output()
    return survived, prediction


LAST_PREDICTION = None


def main(argv):
    global LAST_PREDICTION
    path = next((a for a in argv if not a.startswith("--")), DEFAULT_CSV)
    quiet = "--quiet" in argv
    seed = next((int(a.split("=", 1)[1]) for a in argv if a.startswith("--seed=")), None)
    survived, prediction = build(lr_only="--all" not in argv, seed=seed)
    LAST_PREDICTION = prediction
    evaluator = Evaluators.BinaryClassification().set_label_col(survived).set_prediction_col(prediction)
    reader = CSVReader(path=path, schema=SCHEMA, key=lambda r: str(r["id"]))
    wf = OpWorkflow().set_result_features(survived, prediction).set_reader(reader)
    model = wf.train()
    if not quiet:
        print("Model summary:\n" + model.summary_pretty())
        # feature contributions via model insights (OpTitanicSimple.scala:156-166)
        insights = model.model_insights(prediction)
        contrib = []
        for feat in insights.features:
            for d in feat.derivedFeatures:
                c = max((abs(x) for x in (d.contribution or [])), default=0.0)
                contrib.append((d.derivedFeatureName, c))
        contrib.sort(key=lambda x: -x[1])
        print(f"Top {min(20, len(contrib))} feature contributions:")
        for name, c in contrib[:20]:
            print(f"{name}: {c}")
    scores, metrics = model.score_and_evaluate(evaluator)
    if not quiet:
        print("Metrics:\n", metrics)
    return model, metrics


if __name__ == "__main__":
    main(sys.argv[1:])
