"""Every stand-alone predictor estimator stage in one namespace (the reference's
``stages/impl/classification`` and ``stages/impl/regression`` packages): ``OpXGBoostClassifier().set_input(label,
features).get_output()`` outside a model selector, as ``ModelInsightsTest.scala:77-83`` uses them."""
from .glm import OpGeneralizedLinearRegression  # noqa: F401
from .linear import OpLinearRegression, OpLinearSVC, OpLogisticRegression, OpNaiveBayes  # noqa: F401
from .mlp import OpMultilayerPerceptronClassifier  # noqa: F401
from .trees import (OpDecisionTreeClassifier, OpDecisionTreeRegressor, OpGBTClassifier,  # noqa: F401
                    OpGBTRegressor, OpRandomForestClassifier, OpRandomForestRegressor, OpXGBoostClassifier,
                    OpXGBoostRegressor)
