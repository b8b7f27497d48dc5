"""Problem-specific model selector factories and default grids.

Reference: ``DefaultSelectorParams`` (``core/.../impl/selector/DefaultSelectorParams.scala:35-76``),
``BinaryClassificationModelSelector`` (``classification/BinaryClassificationModelSelector.scala:54-272``:
defaults LR + RF + XGB, AuPR, DataSplitter), ``MultiClassificationModelSelector`` (LR + RF, Error,
DataCutter), ``RegressionModelSelector`` (LR + RF + GBT, RMSE, DataSplitter) and ``ModelSelectorFactory``
(``selector/ModelSelectorFactory.scala:75-104``: filter grids by ``modelTypesToUse``).
"""
from __future__ import annotations

import itertools
from typing import Dict, List, Optional, Sequence

from ..evaluators.evaluators import (Evaluators, OpBinaryClassificationEvaluator, OpBinScoreEvaluator,
                                     OpMultiClassificationEvaluator, OpRegressionEvaluator)
from ..tuning.splitters import DataCutter, DataSplitter
from ..tuning.validators import OpCrossValidation, OpTrainValidationSplit
from .model_selector import ModelSelector


class DefaultSelectorParams:
    MaxDepth = [3, 6, 12]
    MaxBin = [32]
    MinInstancesPerNode = [10, 100]
    MinInfoGain = [0.001, 0.01, 0.1]
    Regularization = [0.001, 0.01, 0.1, 0.2]
    MaxIterLin = [50]
    MaxIterTree = [20]
    SubsampleRate = [1.0]
    StepSize = [0.1]
    ImpurityReg = ["variance"]
    ImpurityClass = ["gini"]
    ElasticNet = [0.1, 0.5]
    MaxTrees = [50]
    Standardized = [True]
    Tol = [1e-6]
    TreeLossType = ["squared"]
    RegSolver = ["auto"]
    FitIntercept = [True]
    NbSmoothing = [1.0]
    DistFamily = ["gaussian", "binomial", "poisson", "gamma", "tweedie"]
    LinkFunction = ["identity", "log", "inverse", "logit", "probit", "cloglog", "sqrt"]
    NumRound = [200]
    Eta = [0.02]
    MinChildWeight = [1.0, 10.0]
    BinaryClassMaxDepthXGB = [10]
    MissingValPad = [0.0]
    BinaryClassXGBEvaluationMetric = ["aucpr"]
    BinaryClassXGBObjective = ["binary:logistic"]
    EarlyStopping = [20]
    MaximizeEvaluationMetrics = [True]
    BinaryClassXGBGamma = [0.8]


def param_grid(**axes) -> List[Dict]:
    """``ParamGridBuilder().addGrid(...).build()``: cartesian product of the axes."""
    keys = list(axes)
    return [dict(zip(keys, vals)) for vals in itertools.product(*[axes[k] for k in keys])]


D = DefaultSelectorParams


def _lr_grid():
    return param_grid(fit_intercept=D.FitIntercept, elastic_net_param=D.ElasticNet, max_iter=D.MaxIterLin,
                      reg_param=D.Regularization, standardization=D.Standardized, tol=D.Tol)


def _rf_grid(impurity):
    return param_grid(max_depth=D.MaxDepth, impurity=impurity, max_bins=D.MaxBin, min_info_gain=D.MinInfoGain,
                      min_instances_per_node=D.MinInstancesPerNode, num_trees=D.MaxTrees,
                      subsampling_rate=D.SubsampleRate)


def _gbt_grid(impurity):
    return param_grid(max_depth=D.MaxDepth, impurity=impurity, max_bins=D.MaxBin, min_info_gain=D.MinInfoGain,
                      min_instances_per_node=D.MinInstancesPerNode, max_iter=D.MaxIterTree,
                      subsampling_rate=D.SubsampleRate, step_size=D.StepSize)


def _dt_grid(impurity):
    return param_grid(max_depth=D.MaxDepth, impurity=impurity, max_bins=D.MaxBin, min_info_gain=D.MinInfoGain,
                      min_instances_per_node=D.MinInstancesPerNode)


def _svc_grid():
    return param_grid(reg_param=D.Regularization, max_iter=D.MaxIterLin, fit_intercept=D.FitIntercept, tol=D.Tol,
                      standardization=D.Standardized)


def _xgb_bin_grid():
    return param_grid(num_round=D.NumRound, num_early_stopping_rounds=D.EarlyStopping, eta=D.Eta,
                      gamma=D.BinaryClassXGBGamma, max_depth=D.BinaryClassMaxDepthXGB,
                      min_child_weight=D.MinChildWeight, missing=D.MissingValPad,
                      maximize_evaluation_metrics=D.MaximizeEvaluationMetrics,
                      eval_metric=D.BinaryClassXGBEvaluationMetric, objective=D.BinaryClassXGBObjective)


class _SelectorFactory:
    defaults: List[str] = []
    problem = "binary"

    @classmethod
    def models_and_params(cls) -> Dict[str, List[Dict]]:
        raise NotImplementedError

    @classmethod
    def _select_models(cls, model_types_to_use, models_and_parameters):
        if models_and_parameters:
            return [(n if isinstance(n, str) else n.name, list(g)) for n, g in models_and_parameters]
        mp = cls.models_and_params()
        types = model_types_to_use or cls.defaults
        out = []
        for t in types:
            t = t if isinstance(t, str) else t.__name__
            if t not in mp:
                raise ValueError(f"model type {t} not supported for {cls.__name__}")
            out.append((t, mp[t]))
        return out


class BinaryClassificationModelSelector(_SelectorFactory):
    defaults = ["OpLogisticRegression", "OpRandomForestClassifier", "OpXGBoostClassifier"]

    @classmethod
    def models_and_params(cls):
        return {"OpLogisticRegression": _lr_grid(), "OpRandomForestClassifier": _rf_grid(D.ImpurityClass),
                "OpGBTClassifier": _gbt_grid(D.ImpurityClass), "OpLinearSVC": _svc_grid(),
                "OpNaiveBayes": param_grid(smoothing=D.NbSmoothing),
                "OpDecisionTreeClassifier": _dt_grid(D.ImpurityClass), "OpXGBoostClassifier": _xgb_bin_grid()}

    def __new__(cls, *a, **kw):
        return cls.with_cross_validation(*a, **kw)

    @classmethod
    def with_cross_validation(cls, splitter="default", num_folds: int = 3, validation_metric=None,
                              train_test_evaluators: Sequence = (), seed: Optional[int] = None,
                              stratify: bool = False, parallelism: int = 8, model_types_to_use=None,
                              models_and_parameters=None, max_wait: float = 86400.0) -> ModelSelector:
        ev = validation_metric or Evaluators.BinaryClassification.auPR()
        val = OpCrossValidation(num_folds=num_folds, evaluator=ev, seed=seed, stratify=stratify,
                                parallelism=parallelism, max_wait=max_wait)
        return cls._make(val, splitter, train_test_evaluators, model_types_to_use, models_and_parameters, seed)

    @classmethod
    def with_train_validation_split(cls, splitter="default", train_ratio: float = 0.75, validation_metric=None,
                                    train_test_evaluators: Sequence = (), seed: Optional[int] = None,
                                    stratify: bool = False, parallelism: int = 8, model_types_to_use=None,
                                    models_and_parameters=None, max_wait: float = 86400.0) -> ModelSelector:
        ev = validation_metric or Evaluators.BinaryClassification.auPR()
        val = OpTrainValidationSplit(train_ratio=train_ratio, evaluator=ev, seed=seed, stratify=stratify,
                                     parallelism=parallelism, max_wait=max_wait)
        return cls._make(val, splitter, train_test_evaluators, model_types_to_use, models_and_parameters, seed)

    @classmethod
    def _evals(cls, extra):
        evs = [OpBinaryClassificationEvaluator(), OpBinScoreEvaluator()]
        names = {type(e).__name__ for e in evs}
        return evs + [e for e in extra if type(e).__name__ not in names]

    @classmethod
    def _default_splitter(cls, seed):
        return DataSplitter(seed=seed)

    @classmethod
    def _make(cls, val, splitter, evs, types, mp, seed):
        sp = cls._default_splitter(seed) if splitter == "default" else splitter
        return ModelSelector(val, sp, cls._select_models(types, mp), cls._evals(list(evs)))


class MultiClassificationModelSelector(BinaryClassificationModelSelector):
    defaults = ["OpLogisticRegression", "OpRandomForestClassifier"]

    @classmethod
    def models_and_params(cls):
        return {"OpLogisticRegression": _lr_grid(), "OpRandomForestClassifier": _rf_grid(D.ImpurityClass),
                "OpNaiveBayes": param_grid(smoothing=D.NbSmoothing),
                "OpDecisionTreeClassifier": _dt_grid(D.ImpurityClass)}

    @classmethod
    def with_cross_validation(cls, splitter="default", num_folds: int = 3, validation_metric=None,
                              train_test_evaluators=(), seed=None, stratify=False, parallelism=8,
                              model_types_to_use=None, models_and_parameters=None, max_wait=86400.0):
        ev = validation_metric or Evaluators.MultiClassification.error()
        val = OpCrossValidation(num_folds=num_folds, evaluator=ev, seed=seed, stratify=stratify,
                                parallelism=parallelism, max_wait=max_wait)
        return cls._make(val, splitter, train_test_evaluators, model_types_to_use, models_and_parameters, seed)

    @classmethod
    def with_train_validation_split(cls, splitter="default", train_ratio=0.75, validation_metric=None,
                                    train_test_evaluators=(), seed=None, stratify=False, parallelism=8,
                                    model_types_to_use=None, models_and_parameters=None, max_wait=86400.0):
        ev = validation_metric or Evaluators.MultiClassification.error()
        val = OpTrainValidationSplit(train_ratio=train_ratio, evaluator=ev, seed=seed, stratify=stratify,
                                     parallelism=parallelism, max_wait=max_wait)
        return cls._make(val, splitter, train_test_evaluators, model_types_to_use, models_and_parameters, seed)

    @classmethod
    def _evals(cls, extra):
        evs = [OpMultiClassificationEvaluator()]
        return evs + [e for e in extra if type(e).__name__ != "OpMultiClassificationEvaluator"]

    @classmethod
    def _default_splitter(cls, seed):
        return DataCutter(seed=seed)


class RegressionModelSelector(BinaryClassificationModelSelector):
    defaults = ["OpLinearRegression", "OpRandomForestRegressor", "OpGBTRegressor"]

    @classmethod
    def models_and_params(cls):
        glm = param_grid(fit_intercept=D.FitIntercept, family=D.DistFamily, link=D.LinkFunction,
                         max_iter=D.MaxIterLin, reg_param=D.Regularization, tol=D.Tol)
        return {"OpLinearRegression": param_grid(fit_intercept=D.FitIntercept, elastic_net_param=D.ElasticNet,
                                                 max_iter=D.MaxIterLin, reg_param=D.Regularization,
                                                 solver=D.RegSolver, standardization=D.Standardized, tol=D.Tol),
                "OpRandomForestRegressor": _rf_grid(D.ImpurityReg), "OpGBTRegressor": _gbt_grid(D.ImpurityReg),
                "OpDecisionTreeRegressor": _dt_grid(D.ImpurityReg),
                "OpGeneralizedLinearRegression": glm,
                "OpXGBoostRegressor": param_grid(num_round=D.NumRound, eta=D.Eta, max_depth=[3, 6, 12],
                                                 min_child_weight=D.MinChildWeight, missing=D.MissingValPad)}

    @classmethod
    def with_cross_validation(cls, splitter="default", num_folds: int = 3, validation_metric=None,
                              train_test_evaluators=(), seed=None, stratify=False, parallelism=8,
                              model_types_to_use=None, models_and_parameters=None, max_wait=86400.0):
        ev = validation_metric or Evaluators.Regression.rmse()
        val = OpCrossValidation(num_folds=num_folds, evaluator=ev, seed=seed, stratify=False,
                                parallelism=parallelism, max_wait=max_wait, is_classification=False)
        return cls._make(val, splitter, train_test_evaluators, model_types_to_use, models_and_parameters, seed)

    @classmethod
    def with_train_validation_split(cls, splitter="default", train_ratio=0.75, validation_metric=None,
                                    train_test_evaluators=(), seed=None, stratify=False, parallelism=8,
                                    model_types_to_use=None, models_and_parameters=None, max_wait=86400.0):
        ev = validation_metric or Evaluators.Regression.rmse()
        val = OpTrainValidationSplit(train_ratio=train_ratio, evaluator=ev, seed=seed, parallelism=parallelism,
                                     max_wait=max_wait, is_classification=False)
        return cls._make(val, splitter, train_test_evaluators, model_types_to_use, models_and_parameters, seed)

    @classmethod
    def _evals(cls, extra):
        evs = [OpRegressionEvaluator()]
        return evs + [e for e in extra if type(e).__name__ != "OpRegressionEvaluator"]
