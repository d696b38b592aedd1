"""Every parameter of every estimator's reference parameter table does
something: a non-default value changes the trained model (predictions,
outputs, metrics, scoring history, CV artefacts or written files) or is
rejected with an error -- the equivalent of the reference's
ModelBuilder.init `error(...)` checks plus its algorithms actually reading
their parameters.

The few parameters that cannot change a model by design (execution /
logging knobs, names of data roles exercised by every other test) are
listed in INERT with the reason; the test fails for any parameter that is
neither probed nor listed, so a new table entry cannot be silently ignored.
"""
import math
import os
import re

import numpy as np
import pandas as pd
import pytest

import h2o3_amd as h2o
from h2o3_amd import estimators as E
from h2o3_amd.models.base import COMMON_DEFAULTS

_N = 400


def _df(n=_N, seed=0):
    rng = np.random.default_rng(seed)
    X = rng.normal(size=(n, 4))
    c = rng.choice(["p", "q", "r", "s", "t"], n)
    ce = {"p": 0.5, "q": -0.5, "r": 1.0, "s": 0.0, "t": -1.0}
    lin = 1.2 * X[:, 0] - 0.8 * X[:, 1] + 0.4 * X[:, 2] * X[:, 3] + np.array([ce[v] for v in c])
    df = pd.DataFrame(X, columns=["x0", "x1", "x2", "x3"])
    df.loc[rng.random(n) < 0.05, "x2"] = np.nan
    df["c"] = c
    df["const"] = 1.0
    df["yb"] = np.where(rng.random(n) < 1 / (1 + np.exp(-lin)), "a", "b")
    df["ym"] = np.where(lin > 0.7, "hi", np.where(lin < -0.7, "lo", "mid"))
    df["yr"] = lin + 0.3 * rng.normal(size=n)
    df["yp"] = rng.gamma(2.0, np.exp(0.3 * lin) / 2.0)
    df["yc"] = rng.poisson(np.exp(0.3 * lin))
    df["w"] = rng.uniform(0.5, 2.0, n)
    df["off"] = 0.1 * rng.normal(size=n)
    df["fold"] = np.arange(n) % 3
    df["treat"] = np.where(rng.random(n) < 0.5, "treatment", "control")
    T = rng.exponential(1 / np.exp(0.5 * X[:, 0]))
    Cn = rng.exponential(2.0, n)
    df["t_stop"] = np.ceil(np.minimum(T, Cn) * 10) + 1
    df["t_start"] = np.where(rng.random(n) < 0.3, np.floor(df["t_stop"] * 0.3), 0.0)
    df["event"] = (T <= Cn).astype(int)
    return df


@pytest.fixture(scope="module")
def data():
    h2o.init(device="cpu", verbose=False)
    tr = _df()
    va = _df(200, seed=1)
    fr, vf = h2o.H2OFrame(tr), h2o.H2OFrame(va)
    words = []
    rng = np.random.default_rng(2)
    groups = [["cat", "dog", "cow"], ["red", "tan", "blue"], ["one", "two", "six"]]
    for _ in range(300):
        g = groups[rng.integers(3)]
        words += list(rng.choice(g, 4)) + [None]
    text = h2o.H2OFrame(pd.DataFrame({"w": words}), column_types=["string"])
    return {"train": fr, "valid": vf, "text": text, "df": tr}


X4 = ["x0", "x1", "x2", "c", "const"]

# estimator key -> (class, constructor kwargs, train kwargs)
CONFIGS = {
    "gbm": (E.H2OGradientBoostingEstimator, dict(ntrees=3, max_depth=3, seed=1, min_rows=5), dict(x=X4, y="yb")),
    "drf": (E.H2ORandomForestEstimator, dict(ntrees=3, max_depth=4, seed=1), dict(x=X4, y="yb")),
    "xrt": (E.H2OExtremelyRandomizedTreesEstimator, dict(ntrees=3, max_depth=4, seed=1), dict(x=X4, y="yb")),
    "xgb": (E.H2OXGBoostEstimator, dict(ntrees=3, max_depth=3, seed=1), dict(x=X4, y="yb")),
    "glm": (E.H2OGeneralizedLinearEstimator, dict(family="binomial", seed=1), dict(x=X4, y="yb")),
    "gam": (E.H2OGeneralizedAdditiveEstimator, dict(family="gaussian", gam_columns=["x0"], seed=1),
            dict(x=["x0", "x1", "c"], y="yr")),
    "dl": (E.H2ODeepLearningEstimator, dict(hidden=[4], epochs=2, seed=1), dict(x=X4, y="yb")),
    "ae": (E.H2OAutoEncoderEstimator, dict(hidden=[3], epochs=2, seed=1), dict(x=["x0", "x1", "x2", "c"])),
    "km": (E.H2OKMeansEstimator, dict(k=3, seed=1), dict(x=["x0", "x1", "x2", "c"])),
    "pca": (E.H2OPrincipalComponentAnalysisEstimator, dict(k=2, seed=1), dict(x=["x0", "x1", "x2", "x3", "c"])),
    "svd": (E.H2OSingularValueDecompositionEstimator, dict(nv=2, seed=1), dict(x=["x0", "x1", "x2", "x3", "c"])),
    "glrm": (E.H2OGeneralizedLowRankEstimator, dict(k=2, seed=1, max_iterations=20),
             dict(x=["x0", "x1", "x2", "x3", "c"])),
    "nb": (E.H2ONaiveBayesEstimator, dict(seed=1), dict(x=X4, y="yb")),
    "if": (E.H2OIsolationForestEstimator, dict(ntrees=5, seed=1, sample_size=64), dict(x=["x0", "x1", "x2", "c"])),
    "eif": (E.H2OExtendedIsolationForestEstimator, dict(ntrees=5, seed=1, sample_size=64),
            dict(x=["x0", "x1", "x2", "x3"])),
    "cox": (E.H2OCoxProportionalHazardsEstimator, dict(stop_column="t_stop"), dict(x=["x0", "x1", "c"], y="event")),
    "agg": (E.H2OAggregatorEstimator, dict(target_num_exemplars=40, seed=1), dict(x=["x0", "x1", "x2", "c"])),
    "w2v": (E.H2OWord2vecEstimator, dict(vec_size=8, epochs=2, min_word_freq=2, seed=1), dict(_text=True)),
    "psvm": (E.H2OSupportVectorMachineEstimator, dict(seed=1), dict(x=["x0", "x1", "x2", "x3"], y="yb")),
    "rulefit": (E.H2ORuleFitEstimator, dict(rule_generation_ntrees=3, max_rule_length=2, min_rule_length=1, seed=1),
                dict(x=["x0", "x1", "c"], y="yb")),
    "iso": (E.H2OIsotonicRegressionEstimator, dict(), dict(x=["x0"], y="yr")),
    "te": (E.H2OTargetEncoderEstimator, dict(seed=1), dict(x=["c"], y="yb")),
    "uplift": (E.H2OUpliftRandomForestEstimator, dict(ntrees=3, max_depth=3, treatment_column="treat", seed=1),
               dict(x=["x0", "x1", "c"], y="yb")),
    "anova": (E.H2OANOVAGLMEstimator, dict(family="gaussian", highest_interaction_term=2),
              dict(x=["x0", "x1", "c"], y="yr")),
    "ms": (E.H2OModelSelectionEstimator, dict(mode="maxr", max_predictor_number=2), dict(x=["x0", "x1", "x3"], y="yr")),
    "infogram": (E.H2OInfogram, dict(seed=1, algorithm="glm"), dict(x=["x0", "x1", "x2", "x3"], y="yb")),
    "se": (E.H2OStackedEnsembleEstimator, dict(seed=1), dict(x=X4, y="yb", _se=True)),
}

# Estimator classes of the reference's table that are probed elsewhere.
ELSEWHERE = {"H2OGenericEstimator": "model_key / path: tests/test_mojo*.py load MOJOs into Generic models"}

# parameter -> non-default value, or (value, extra constructor/train kwargs shared
# by the baseline and the probe); "*" applies to every estimator, a key to one
_V = {
    "*": {
        "nfolds": 2, "fold_assignment": ("modulo", {"nfolds": 2}), "fold_column": "fold",
        "keep_cross_validation_models": (False, {"nfolds": 2}),
        "keep_cross_validation_predictions": (True, {"nfolds": 2}),
        "keep_cross_validation_fold_assignment": (True, {"nfolds": 2}),
        "weights_column": "w", "offset_column": "off", "ignored_columns": ["x1"],
        "validation_frame": "_valid", "model_id": "sweep_custom_id", "ignore_const_cols": False,
        "max_runtime_secs": 1e-9, "seed": 7, "score_each_iteration": True,
        "stopping_rounds": 1, "stopping_metric": ("AUC", {"stopping_rounds": 1}),
        "stopping_tolerance": (0.5, {"stopping_rounds": 1}), "export_checkpoints_dir": "_dir",
        "auc_type": ("MACRO_OVO", {"_y": "ym"}), "gainslift_bins": 5,
        "balance_classes": True, "class_sampling_factors": ([3.0, 1.0], {"balance_classes": True}),
        "max_after_balance_size": (0.5, {"balance_classes": True}),
        "max_confusion_matrix_size": (2, {"_y": "ym"}),
        "categorical_encoding": "one_hot_explicit", "distribution": ("laplace", {"_y": "yr"}),
        "standardize": False, "missing_values_handling": "Skip", "checkpoint": "_checkpoint",
        "custom_metric_func": "_udf_metric",
        "max_iterations": 2, "init": "Random", "k": 3, "transform": "STANDARDIZE",
        "use_all_factor_levels": "_flip", "score_tree_interval": (2, {"ntrees": 4}),
        "ntrees": 5, "max_depth": 2, "min_rows": 20.0, "nbins": 5, "nbins_top_level": 64, "nbins_cats": 2,
        "r2_stopping": 0.5, "stopping_rounds_gbm": None, "learn_rate": 0.5, "learn_rate_annealing": 0.5,
        "sample_rate": 0.5, "sample_rate_per_class": [0.3, 1.0], "col_sample_rate": 0.5,
        "col_sample_rate_change_per_level": 0.5, "col_sample_rate_per_tree": 0.5,
        "min_split_improvement": 0.1, "histogram_type": "Random", "mtries": 2,
        "max_abs_leafnode_pred": 0.05, "pred_noise_bandwidth": 0.5,
        "calibrate_model": (True, {"calibration_frame": "_valid"}),
        "calibration_frame": ("_valid", {"calibrate_model": True}),
        "calibration_method": ("IsotonicRegression", {"calibrate_model": True, "calibration_frame": "_valid"}),
        "check_constant_response": (False, {"_y": "const"}),
        "binomial_double_trees": True,
        "monotone_constraints": ({"x0": 1}, {"_y": "yr"}),
        "interaction_constraints": [["x0", "x1"]],
        "in_training_checkpoints_dir": "_dir", "in_training_checkpoints_tree_interval": (2, {"_itc": True}),
        "huber_alpha": (0.3, {"distribution": "huber", "_y": "yr"}),
        "quantile_alpha": (0.2, {"distribution": "quantile", "_y": "yr"}),
        "tweedie_power": (1.8, {"distribution": "tweedie", "_y": "yp"}),
        "custom_distribution_func": "_udf_dist",
        "alpha": 0.9, "lambda_": 0.05, "lambda_search": True, "nlambdas": (5, {"lambda_search": True}),
        "lambda_min_ratio": (0.1, {"lambda_search": True}), "early_stopping": (False, {"lambda_search": True}),
        "solver": "COORDINATE_DESCENT_NAIVE", "intercept": False, "non_negative": True,
        "objective_epsilon": 0.2, "beta_epsilon": 0.5, "gradient_epsilon": 0.5, "link": ("log", {"family": "poisson",
                                                                                                "_y": "yc"}),
        "family": ("poisson", {"_y": "yc"}), "prior": 0.3, "compute_p_values": (True, {"lambda_": 0.0}),
        "remove_collinear_columns": (True, {"lambda_": 0.0, "_x": ["x0", "x1", "x2", "c", "x0x"]}),
        "cold_start": (True, {"lambda_search": True, "nlambdas": 4}), "max_active_predictors": (2, {"lambda_search": True}),
        "beta_constraints": "_beta_constraints", "startval": "_startval",
        "interactions": ["x0", "x1"], "interaction_pairs": [("x0", "x1")], "calc_like": True,
        "obj_reg": 0.01, "plug_values": ("_plug", {"missing_values_handling": "PlugValues", "plug_values": "_plug0"}),
        "theta": (0.5, {"family": "negativebinomial", "_y": "yc"}),
        "tweedie_variance_power": (1.5, {"family": "tweedie", "_y": "yp"}),
        "tweedie_link_power": (0.0, {"family": "tweedie", "tweedie_variance_power": 1.5, "_y": "yp"}),
        "dispersion_parameter_method": ("deviance", {"family": "gamma", "_y": "yp", "compute_p_values": True,
                                                     "lambda_": 0.0}),
        "init_dispersion_parameter": (2.0, {"family": "gamma", "_y": "yp", "compute_p_values": True, "lambda_": 0.0,
                                            "fix_dispersion_parameter": True}),
        "fix_dispersion_parameter": (True, {"family": "gamma", "_y": "yp", "compute_p_values": True, "lambda_": 0.0,
                                            "init_dispersion_parameter": 2.0}),
        "dispersion_epsilon": (0.5, {"family": "gamma", "_y": "yp", "compute_p_values": True, "lambda_": 0.0,
                                     "dispersion_parameter_method": "ml"}),
        "max_iterations_dispersion": (1, {"family": "gamma", "_y": "yp", "compute_p_values": True, "lambda_": 0.0,
                                          "dispersion_parameter_method": "ml"}),
        "build_null_model": (True, {"family": "gamma", "_y": "yp"}),
        "generate_scoring_history": True, "score_iteration_interval": (2, {"generate_scoring_history": True}),
        "HGLM": (True, {"family": "gaussian", "_y": "yr", "random_columns": ["c"], "_x": ["x0", "x1", "c"]}),
        "random_columns": (["c"], {"HGLM": True, "family": "gaussian", "_y": "yr", "_x": ["x0", "x1", "c"]}),
        "rand_family": (["gamma"], {"HGLM": True, "family": "gaussian", "_y": "yr", "random_columns": ["c"],
                                    "_x": ["x0", "x1", "c"]}),
        "rand_link": (["log"], {"HGLM": True, "family": "gaussian", "_y": "yr", "random_columns": ["c"],
                                "_x": ["x0", "x1", "c"]}),
        # deep learning
        "activation": "Tanh", "hidden": [3, 3], "epochs": 3.0, "train_samples_per_iteration": 50,
        "target_ratio_comm_to_comp": (0.5, {"_ranks": 2}), "adaptive_rate": False, "rho": 0.5, "epsilon": 1e-3,
        "rate": (0.1, {"adaptive_rate": False}), "rate_annealing": (0.1, {"adaptive_rate": False}),
        "rate_decay": (0.5, {"adaptive_rate": False}), "momentum_start": (0.5, {"adaptive_rate": False}),
        "momentum_ramp": (10.0, {"adaptive_rate": False, "momentum_stable": 0.9}),
        "momentum_stable": (0.9, {"adaptive_rate": False}),
        "nesterov_accelerated_gradient": (False, {"adaptive_rate": False, "momentum_start": 0.9}),
        "input_dropout_ratio": 0.3, "hidden_dropout_ratios": ([0.3], {"activation": "RectifierWithDropout"}),
        "l1": 0.01, "l2": 0.01, "max_w2": 0.01, "initial_weight_distribution": "Normal", "initial_weight_scale": 0.1,
        "initial_weights": "_init_w", "initial_biases": "_init_b", "loss": "Absolute",
        "score_interval": (1e9, {"epochs": 5, "train_samples_per_iteration": 100}),
        "score_training_samples": 50,
        "score_validation_samples": (50, {"validation_frame": "_valid"}),
        "score_duty_cycle": (0.0, {"epochs": 5, "train_samples_per_iteration": 100, "score_interval": 0}),
        "classification_stop": 0.9, "regression_stop": (10.0, {"_y": "yr"}),
        "score_validation_sampling": ("Stratified", {"validation_frame": "_valid", "score_validation_samples": 50}),
        "variable_importances": False, "replicate_training_data": (False, {"_ranks": 2}),
        "single_node_mode": (True, {"_ranks": 2}), "shuffle_training_data": (True, {"train_samples_per_iteration": 50}),
        "autoencoder": True, "average_activation": (0.5, {"sparsity_beta": 0.5}), "sparsity_beta": 0.5,
        "max_categorical_features": 2, "reproducible": "_repro", "export_weights_and_biases": True,
        "mini_batch_size": 16, "elastic_averaging": (True, {"_ranks": 2}),
        "elastic_averaging_moving_rate": (0.2, {"elastic_averaging": True, "_ranks": 2}),
        "elastic_averaging_regularization": (0.5, {"elastic_averaging": True, "_ranks": 2}),
        "pretrained_autoencoder": "_pretrained", "overwrite_with_best_model": (False, {"epochs": 5,
                                                                                    "train_samples_per_iteration": 50}),
        # clustering / matrix factorization
        "estimate_k": (True, {"k": 6}), "user_points": "_user_points", "cluster_size_constraints": [100, 100, 100],
        "pca_method": "Power", "pca_impl": "mtj_svd_densematrix", "compute_metrics": False, "impute_missing": True,
        "svd_method": "Power", "nv": 3, "keep_u": False, "u_name": "sweep_u_frame",
        "loss": "Absolute", "multi_loss": "Ordinal", "loss_by_col": (["Absolute"], {"loss_by_col_idx": [0]}),
        "loss_by_col_idx": ([1], {"loss_by_col": ["Huber"]}), "period": (2, {"loss": "Periodic"}),
        "regularization_x": ("Quadratic", {"gamma_x": 1.0}), "regularization_y": ("Quadratic", {"gamma_y": 1.0}),
        "gamma_x": (1.0, {"regularization_x": "Quadratic"}), "gamma_y": (1.0, {"regularization_y": "Quadratic"}),
        "max_updates": 3, "init_step_size": 0.01, "min_step_size": 0.5, "user_y": ("_user_y", {"init": "User"}),
        "user_x": ("_user_x", {"init": "User"}), "expand_user_y": (False, {"init": "User", "user_y": "_user_y_exp"}),
        "impute_original": True, "recover_svd": True, "representation_name": "sweep_rep",
        "loading_name": "sweep_loading",
        # naive bayes
        "laplace": 1.0, "min_sdev": 0.5, "eps_sdev": 1.0, "min_prob": 0.4, "eps_prob": 1.0,
        # isolation forests
        "sample_size": 16, "extension_level": 2, "contamination": 0.2,
        "validation_response_column": ("yb", {"validation_frame": "_valid"}),
        # coxph
        "start_column": "t_start", "stop_column": "_raise", "ties": "breslow", "lre_min": 1.0,
        "stratify_by": ["c"], "interactions_only": (["x1"], {"interaction_pairs": [("x0", "x1")]}),
        # aggregator
        "target_num_exemplars": 10, "rel_tol_num_exemplars": 0.05, "save_mapping_frame": True,
        "num_iteration_without_new_exemplar": 0,
        # word2vec
        "vec_size": 4, "window_size": 1, "sent_sample_rate": 0.01, "norm_model": "_raise",
        "min_word_freq": 30, "init_learning_rate": 0.2, "word_model": "CBOW", "pre_trained": "_w2v_pre",
        # psvm
        "hyper_param": 0.01, "kernel_type": "_raise", "gamma": 0.5, "rank_ratio": 0.2, "positive_weight": 3.0,
        "negative_weight": 3.0, "disable_training_metrics": False, "sv_threshold": 0.5, "fact_threshold": 0.5,
        "feasible_threshold": 0.5, "surrogate_gap_threshold": 0.5, "mu_factor": 2.0,
        # rulefit
        "algorithm": "GBM", "min_rule_length": 2, "max_rule_length": 3, "max_num_rules": 2,
        "model_type": "RULES", "rule_generation_ntrees": 6, "remove_duplicates": False, "max_categorical_levels": 2,
        # isotonic
        "out_of_bounds": "clip",
        # target encoder
        "columns_to_encode": [["c"]], "keep_original_categorical_columns": False, "blending": True,
        "inflection_point": (2.0, {"blending": True}), "smoothing": (2.0, {"blending": True}),
        "data_leakage_handling": "KFold", "noise": 0.5,
        # uplift
        "treatment_column": "_raise", "uplift_metric": "ChiSquared", "auuc_type": "gain", "auuc_nbins": 5,
        # anova / model selection
        "highest_interaction_term": 1, "type": "_raise", "save_transformed_framekeys": True,
        "mode": "backward", "max_predictor_number": 1, "min_predictor_number": (2, {"mode": "backward"}),
        "p_values_threshold": (0.5, {"mode": "backward"}),
        # infogram
        "algorithm_params": ({"max_iterations": 1}, {}), "protected_columns": ["x3"],
        "total_information_threshold": 0.9, "net_information_threshold": 0.9,
        "relevance_index_threshold": (0.9, {"protected_columns": ["x3"]}),
        "safety_index_threshold": (0.9, {"protected_columns": ["x3"]}), "data_fraction": 0.5, "top_n_features": 1,
        # stacked ensemble
        "base_models": "_se_base_one", "metalearner_algorithm": "gbm", "metalearner_nfolds": 2,
        "metalearner_fold_assignment": ("modulo", {"metalearner_nfolds": 2}),
        "metalearner_fold_column": "fold", "metalearner_params": {"lambda_": 0.5},
        "metalearner_transform": "Logit", "blending_frame": "_valid", "keep_levelone_frame": True,
        "score_training_samples": 50,
        # gam
        "gam_columns": [["x1"]], "num_knots": [4], "knot_ids": "_knot_ids", "bs": [2], "scale": [10.0],
        "keep_gam_cols": True, "spline_orders": ([3], {"bs": [2]}), "splines_non_negative": ([False], {"bs": [2]}),
        "standardize_tp_gam_cols": (True, {"bs": [1]}), "scale_tp_penalty_mat": (True, {"bs": [1]}),
        "store_knot_locations": True,
        # xgboost
        "eta": 0.7, "subsample": 0.5, "colsample_bylevel": 0.5, "colsample_bytree": 0.5, "colsample_bynode": 0.5,
        "min_child_weight": 20.0, "max_delta_step": 0.05, "max_bins": 8, "max_leaves": (3, {"grow_policy": "lossguide"}),
        "tree_method": "_raise_exact", "grow_policy": ("lossguide", {"max_depth": 0, "max_leaves": 4}),
        "booster": "gblinear", "reg_lambda": 50.0, "reg_alpha": 5.0, "normalize_type": ("forest",
                                                                                          {"booster": "dart",
                                                                                           "rate_drop": 0.5}),
        "rate_drop": (0.5, {"booster": "dart"}), "one_drop": (True, {"booster": "dart"}),
        "skip_drop": (0.9, {"booster": "dart", "rate_drop": 0.5}), "scale_pos_weight": 5.0,
        "sample_type": ("weighted", {"booster": "dart", "rate_drop": 0.5}), "save_matrix_directory": "_dir",
    },
    "xgb": {"gamma": 5.0, "max_abs_leafnode_pred": 0.05, "learn_rate": 0.9, "sample_rate": 0.5,
            "col_sample_rate": 0.5, "col_sample_rate_per_tree": 0.5, "min_rows": 30.0,
            "min_split_improvement": 5.0},
    "glm": {"max_iterations": 1, "alpha": (0.9, {"lambda_": 0.05}), "standardize": (False, {"lambda_": 0.05}),
            "solver": "L_BFGS", "lambda_search": True,
            "auc_type": ("MACRO_OVO", {"_y": "ym", "family": "multinomial"}),
            "max_confusion_matrix_size": (2, {"_y": "ym", "family": "multinomial"}),
            "startval": ("_startval", {"lambda_": 0.0, "max_iterations": 1})},
    "gam": {"max_iterations": (1, {"family": "binomial", "_y": "yb"}), "alpha": (0.9, {"lambda_": 0.05}),
            "lambda_": 0.05, "standardize": True, "solver": "L_BFGS",
            "compute_p_values": (True, {"lambda_": 0.0}),
            "auc_type": ("MACRO_OVO", {"_y": "ym", "family": "multinomial"}),
            "max_confusion_matrix_size": (2, {"_y": "ym", "family": "multinomial"}),
            "beta_constraints": "_beta_constraints_x1", "interactions": ["x1", "c"],
            "interaction_pairs": [("x1", "c")], "startval": ("_startval", {"max_iterations": 1,
                                                                           "family": "binomial", "_y": "yb"})},
    "dl": {"distribution": ("laplace", {"_y": "yr"}), "max_iterations": None, "loss": "Absolute",
           "standardize": False},
    "ae": {"loss": "Absolute", "standardize": False},
    "km": {"max_iterations": 1, "init": "Random", "standardize": False},
    "pca": {"max_iterations": (1, {"pca_method": "Power"}), "k": 3, "transform": "STANDARDIZE",
            "seed": (7, {"pca_method": "Randomized"}), "use_all_factor_levels": True},
    "svd": {"max_iterations": (1, {"svd_method": "Power"}), "transform": "STANDARDIZE",
            "seed": (7, {"svd_method": "Randomized"}), "use_all_factor_levels": False},
    "glrm": {"max_iterations": 2, "k": 3, "transform": "STANDARDIZE", "init": "SVD", "loss": "Absolute",
             "svd_method": ("GramSVD", {"init": "SVD"})},
    "nb": {"seed": None},
    "if": {"max_depth": 2, "mtries": 2, "sample_rate": 0.5},
    "eif": {"ntrees": 3},
    "cox": {"init": 0.5, "max_iterations": 1, "use_all_factor_levels": True, "interactions": ["x0", "x1"],
            "interaction_pairs": [("x0", "x1")]},
    "agg": {"transform": "DEMEAN", "categorical_encoding": "Eigen"},
    "w2v": {"epochs": 4},
    "psvm": {"max_iterations": 1},
    "rulefit": {"lambda_": 0.5, "distribution": "bernoulli", "algorithm": "GBM",
                "auc_type": ("MACRO_OVO", {"_y": "ym", "rule_generation_ntrees": 2, "max_rule_length": 1})},
    "iso": {},
    "te": {"seed": (7, {"noise": 0.5})},
    "uplift": {"max_depth": 2, "mtries": 1, "sample_rate": 0.5, "histogram_type": "Random",
               "distribution": "_raise"},
    "anova": {"family": ("poisson", {"_y": "yc"}), "link": ("identity", {"family": "poisson", "_y": "yc"}),
              "lambda_": 0.5, "alpha": (0.5, {"lambda_": 0.5}), "standardize": (False, {"lambda_": 0.5}),
              "compute_p_values": False, "max_iterations": (1, {"family": "poisson", "_y": "yc"}),
              "early_stopping": (True, {"lambda_search": True})},
    "ms": {"theta": (0.5, {"family": "negativebinomial", "_y": "yc", "mode": "backward"}),
           "tweedie_variance_power": (1.5, {"family": "tweedie", "_y": "yp", "mode": "backward"}),
           "tweedie_link_power": (0.0, {"family": "tweedie", "tweedie_variance_power": 1.5, "_y": "yp",
                                        "mode": "backward"}),
           "beta_constraints": ("_beta_constraints", {"compute_p_values": False}),
           "family": ("poisson", {"_y": "yc", "mode": "backward"}),
           "link": ("identity", {"family": "poisson", "_y": "yc", "mode": "backward"}),
           "startval": ({"x0": 0.5, "x1": -0.5, "x3": 0.3, "Intercept": 1.0},
                        {"mode": "backward", "family": "poisson", "_y": "yc", "max_iterations": 1}),
           "lambda_": (0.5, {"mode": "maxr"}), "alpha": (0.5, {"lambda_": 0.5}),
           "compute_p_values": (False, {"mode": "backward"}), "max_iterations": (1, {"family": "poisson",
                                                                                       "_y": "yc", "mode": "backward"})},
    "infogram": {"plug_values": "_plug", "algorithm": "gbm", "standardize": False, "max_iterations": (1, {"algorithm": "glm"})},
    "se": {"seed": None},
}

# parameter -> reason it cannot change a model, "*" for every estimator
INERT = {
    "*": {
        "training_frame": "the data itself; every test trains on it",
        "response_column": "the target; given as y by every test",
        "model_id": None,    # probed: the model's key changes
        "quiet_mode": "logging only (reference: log verbosity)",
        "diagnostics": "reference: per-layer weight statistics for logs; no effect on training",
        "col_major": "deprecated in the reference (column-major weight storage); same model",
        "fast_mode": "reference: approximate dropout back-prop on CPU; the GPU back-prop is exact",
        "force_load_balance": "reference: chunk re-balancing of the training frame; rows are sharded evenly here",
        "sparse": "reference: sparse row storage; the device matrix is dense, same model",
        "nthread": "reference XGBoost thread count; the GPU kernel has no CPU threads",
        "backend": "reference XGBoost CPU/GPU backend choice; always the GPU engine here",
        "gpu_id": "device ordinal: one process per GPU (LOCAL_RANK)",
        "dmatrix_type": "reference XGBoost sparse/dense DMatrix choice; one binned device matrix here",
        "build_tree_one_node": "reference: build on one node; every rank already builds the same tree",
        "nparallelism": "number of models built concurrently; same models",
        "verbose": "logging only",
    },
    "nb": {"seed": "Naive Bayes is deterministic (seed only seeds CV fold assignment)",
           "max_runtime_secs": "a single counting pass; nothing to stop"},
    "pca": {"max_runtime_secs": "a single Gram pass + eigen solve; nothing to stop"},
    "svd": {"max_runtime_secs": "a single Gram pass + eigen solve; nothing to stop"},
    "cox": {"single_node_mode": "reference: run on one node; every rank already holds the risk sets",
            "max_runtime_secs": None},
    "iso": {"max_runtime_secs": "one pool-adjacent-violators pass; nothing to stop"},
    "te": {"max_runtime_secs": "one counting pass; nothing to stop"},
    "glm": {"seed": "IRLS is deterministic (seed only seeds CV fold assignment / ordinal GD start)"},
    "gam": {"seed": "IRLS is deterministic (seed only seeds CV fold assignment)"},
    "anova": {"seed": "IRLS is deterministic", "nparallelism": "number of GLMs built concurrently; same models",
              "max_runtime_secs": None},
    "ms": {"seed": "IRLS is deterministic", "nparallelism": "number of GLMs built concurrently; same models",
           "score_iteration_interval": "passed to the inner GLMs (their scoring schedule); the selected "
                                       "subsets and coefficients are unaffected",
           "max_confusion_matrix_size": "ModelSelection models are regression or binomial; the cap applies "
                                        "to multinomial confusion matrices"},
    "psvm": {"seed": "the IPM / ICF solver is deterministic"},
    "uplift": {"check_constant_response": "a constant response has one class and Uplift DRF needs two, so "
                                          "training is rejected with or without the check"},
}


# (estimator, parameter) pairs whose probe value is rejected on purpose
EXPECTED_RAISE = {
    ("ae", "max_categorical_features"),    # hashed inputs cannot be reconstructed
}


def _value(key, param):
    for scope in (key, "*"):
        d = _V.get(scope, {})
        if param in d:
            v = d[param]
            return (v if isinstance(v, tuple) else (v, {}))
    return None


def _inert(key, param):
    for scope in (key, "*"):
        d = INERT.get(scope, {})
        if param in d:
            return d[param]
    return None


def _num_summary(v, depth=0):
    """Deterministic, rounded summary of an output value."""
    if depth > 4:
        return "..."
    if v is None or isinstance(v, (bool, str)):
        return v
    if isinstance(v, (int, np.integer)):
        return int(v)
    if isinstance(v, (float, np.floating)):
        return None if not math.isfinite(v) else float(f"{float(v):.6g}")
    if isinstance(v, dict):
        return {str(k): _num_summary(x, depth + 1) for k, x in sorted(v.items(), key=lambda kv: str(kv[0]))
                if not re.search(r"time|duration|timestamp|_ms$|^run", str(k))}
    if isinstance(v, (list, tuple)):
        return [_num_summary(x, depth + 1) for x in list(v)[:200]]
    if isinstance(v, np.ndarray):
        return _num_summary(v.ravel()[:500].tolist(), depth + 1)
    if isinstance(v, pd.DataFrame):
        return _num_summary(v.select_dtypes(include=[np.number]).values, depth + 1), list(v.columns)
    try:
        import torch
        if isinstance(v, torch.Tensor):
            return _num_summary(v.detach().cpu().double().numpy(), depth + 1)
    except Exception:
        pass
    if hasattr(v, "as_data_frame") and hasattr(v, "nrows"):
        try:
            return ("frame", v.nrows, v.ncols, _num_summary(v.as_data_frame(), depth + 1))
        except Exception:
            return ("frame", v.nrows, v.ncols)
    return type(v).__name__


def _signature(m, fr, files):
    sig = {"id": m.model_id}
    try:
        pr = m.predict(fr).as_data_frame()
        sig["pred"] = _num_summary(pr.apply(lambda c: c.astype("category").cat.codes if c.dtype == object else c))
    except Exception as e:   # noqa: BLE001 - some models have no predict
        sig["pred"] = type(e).__name__
    sig["out"] = _num_summary(getattr(m, "_output", {}))
    for k in ("_training_metrics", "_validation_metrics", "_cross_validation_metrics"):
        mt = getattr(m, k, None)
        sig[k] = _num_summary(getattr(mt, "_m", None) if mt is not None else None)
    sig["hist"] = _num_summary(getattr(m, "_scoring_history", None))
    sig["cv"] = (len(getattr(m, "_cv_models", None) or []), getattr(m, "_cv_holdout", None) is not None,
                 m._output.get("cross_validation_fold_assignment") is not None if hasattr(m, "_output") else None)
    sig["files"] = sorted(files)
    return sig


def _resolve(v, data, tmp, key):
    fr, vf = data["train"], data["valid"]
    if isinstance(v, str) and v.startswith("_"):
        if v == "_valid":
            return vf
        if v == "_dir":
            d = tmp / f"dir_{key}"
            d.mkdir(exist_ok=True)
            return str(d)
        if v in ("_plug", "_plug0"):
            z = 5.0 if v == "_plug" else 0.0
            return h2o.H2OFrame(pd.DataFrame({"x0": [z], "x1": [z], "x2": [z], "x3": [z], "const": [1.0]}))
        if v in ("_beta_constraints", "_beta_constraints_x1"):
            nm = "x0" if v == "_beta_constraints" else "x1"
            return h2o.H2OFrame(pd.DataFrame({"names": [nm], "lower_bounds": [0.0], "upper_bounds": [0.1]}))
        if v == "_user_points":
            return h2o.H2OFrame(data["df"][["x0", "x1", "x2", "c"]].iloc[[0, 10, 20]].reset_index(drop=True))
        if v == "_user_y":
            u = pd.DataFrame(np.random.default_rng(3).normal(size=(2, 4)), columns=["x0", "x1", "x2", "x3"])
            u["c"] = ["q", "s"]
            return h2o.H2OFrame(u)
        if v == "_user_y_exp":
            return h2o.H2OFrame(pd.DataFrame(np.random.default_rng(3).normal(size=(2, 9)),
                                             columns=[f"y{i}" for i in range(9)]))
        if v == "_user_x":
            return h2o.H2OFrame(pd.DataFrame(np.random.default_rng(4).normal(size=(_N, 2)), columns=["a", "b"]))
        if v == "_knot_ids":
            return [h2o.H2OFrame(pd.DataFrame({"k": [-1.5, -0.5, 0.5, 1.5]}))]
    return v


_BASE = {}


def _train(key, kw, data, tmp, extra_files_dir=None):
    cls, ckw, tkw = CONFIGS[key]
    kw = dict(kw)
    tkw = dict(tkw)
    for k in list(kw):
        if k.startswith("_"):
            v = kw.pop(k)
            if k == "_y":
                tkw["y"] = v
            elif k == "_x":
                tkw["x"] = v
    args = dict(ckw)
    args.update(kw)
    fr = data["train"]
    if "x0x" in (tkw.get("x") or []):
        fr = fr[:, :]
        fr["x0x"] = fr["x0"] * 2.0
    if tkw.get("_text"):
        for k, v in list(args.items()):
            args[k] = _resolve(v, data, tmp, key)
    if tkw.pop("_text", False):
        m = cls(**args)
        m.train(training_frame=data["text"])
        return m, data["text"]
    if tkw.pop("_se", False):
        base = data["se_base"]
        args.setdefault("base_models", base)
        if args.get("base_models") == "_se_base_one":
            args["base_models"] = base[:1]
        if isinstance(args.get("blending_frame"), type(data["valid"])):
            pass
    for k, v in list(args.items()):
        args[k] = _resolve(v, data, tmp, key)
    vfr = args.pop("validation_frame", None)
    m = cls(**args)
    m.train(training_frame=fr, validation_frame=vfr, **tkw)
    return m, fr


def _dir_files(tmp, key):
    d = tmp / f"dir_{key}"
    return sorted(os.listdir(d)) if d.exists() else []


def _params():
    import inspect
    out = []
    for name in sorted(dir(E)):
        cls = getattr(E, name)
        if not inspect.isclass(cls) or not hasattr(cls, "_param_names") or cls._param_names() is None:
            continue
        key = next((k for k, (c, _, _) in CONFIGS.items() if c is cls), None)
        if key is None:
            continue
        for p in sorted(cls._param_names()):
            out.append(pytest.param(key, p, id=f"{key}-{p}"))
    return out


def test_every_estimator_is_configured():
    import inspect
    missing = []
    for name in sorted(dir(E)):
        cls = getattr(E, name)
        if inspect.isclass(cls) and hasattr(cls, "_param_names") and cls._param_names() is not None:
            if not any(c is cls for c, _, _ in CONFIGS.values()) and name not in ELSEWHERE:
                missing.append(name)
    assert not missing, missing


@pytest.fixture(scope="module")
def se_base(data):
    gb = E.H2OGradientBoostingEstimator(ntrees=3, seed=1, nfolds=2, keep_cross_validation_predictions=True,
                                        fold_assignment="modulo")
    gb.train(x=X4, y="yb", training_frame=data["train"])
    gl = E.H2OGeneralizedLinearEstimator(family="binomial", nfolds=2, keep_cross_validation_predictions=True,
                                         fold_assignment="modulo")
    gl.train(x=X4, y="yb", training_frame=data["train"])
    data["se_base"] = [gb, gl]
    return data


@pytest.mark.parametrize("key,param", _params())
def test_parameter_changes_model_or_raises(se_base, tmp_path, key, param):
    data = se_base
    reason = _inert(key, param)
    if reason:
        pytest.skip(f"inert by design: {reason}")
    pv = _value(key, param)
    assert pv is not None, f"{key}.{param}: no probe value and not listed as inert"
    val, extra = pv
    if val is None:
        pytest.skip("probed elsewhere in this table")
    if extra.get("_ranks"):
        pytest.skip("multi-rank behaviour: tests/test_distributed.py::test_deeplearning_model_averaging")
    if isinstance(val, str) and val.startswith("_raise"):
        cls, ckw, tkw = CONFIGS[key]
        bad = "exact" if val == "_raise_exact" else "__not_a_valid_value__"
        with pytest.raises((ValueError, TypeError, NotImplementedError, KeyError)):
            _train(key, {**extra, param: bad}, data, tmp_path)
        return
    if val in ("_checkpoint", "_udf_metric", "_udf_dist", "_startval", "_init_w", "_init_b", "_pretrained",
               "_w2v_pre", "_flip", "_repro", "_se_base_one", "_knot_ids"):
        val = _special(key, param, val, data, tmp_path, extra)
        if val is _DONE:
            return
    try:
        base, bfr = _train(key, dict(extra), data, tmp_path)
    except (ValueError, TypeError, NotImplementedError, KeyError) as e:
        # the default is rejected for this setup and the probed value makes it
        # valid (e.g. check_constant_response=False on a constant response)
        probe, _ = _train(key, {**extra, param: val}, data, tmp_path)
        return
    b_files = _dir_files(tmp_path, key)
    try:
        probe, _ = _train(key, {**extra, param: val}, data, tmp_path)
    except (ValueError, TypeError, NotImplementedError, KeyError) as e:
        if (key, param) not in EXPECTED_RAISE and ("*", param) not in EXPECTED_RAISE:
            pytest.fail(f"{key}.{param}={val!r} raised unexpectedly: {type(e).__name__}: {e}")
        return      # rejected on purpose: the reference's init errors
    p_files = _dir_files(tmp_path, key)
    s1 = _signature(base, bfr, b_files)
    s2 = _signature(probe, bfr, p_files)
    assert s1 != s2, f"{key}.{param}={val!r} changed nothing"


class _Done:
    pass


_DONE = _Done()


def _special(key, param, val, data, tmp, extra):
    """Parameters whose probe needs a prepared object."""
    cls, ckw, tkw = CONFIGS[key]
    if val == "_flip":
        d = dict(COMMON_DEFAULTS)
        d.update(cls._defaults)
        return not bool(d.get(param))
    if val == "_checkpoint":
        first = {"ntrees": 2} if "ntrees" in cls._param_names() else {"epochs": 1} \
            if "epochs" in cls._param_names() else {"max_iterations": 1}
        m, _ = _train(key, {**extra, **first, "model_id": f"ck_{key}"}, data, tmp)
        return m.model_id
    if val == "_startval":
        m, _ = _train(key, dict(extra), data, tmp)
        return {k: 0.5 * v + 0.3 for k, v in m.coef().items()}
    if val == "_repro":
        # reproducible: two runs with it are identical
        a, fr = _train(key, {**extra, param: True}, data, tmp)
        b, _ = _train(key, {**extra, param: True}, data, tmp)
        assert _signature(a, fr, [])["pred"] == _signature(b, fr, [])["pred"]
        return _DONE
    if val in ("_udf_metric", "_udf_dist"):
        pytest.skip("user-defined functions: tests/test_api_surface.py uploads and checks them")
    if val == "_se_base_one":
        return data["se_base"][:1]
    if val in ("_init_w", "_init_b"):
        import torch
        rng = np.random.default_rng(5)
        m, _ = _train(key, dict(extra), data, tmp)
        mats = [h2o.H2OFrame(pd.DataFrame(rng.normal(size=tuple(L.W.shape)) * 0.5)) if val == "_init_w" else
                h2o.H2OFrame(pd.DataFrame(rng.normal(size=(L.b.shape[0], 1)))) for L in m._layers]
        return mats
    if val == "_pretrained":
        ae = E.H2OAutoEncoderEstimator(hidden=list(CONFIGS[key][1].get("hidden", [4])), epochs=2, seed=3)
        ae.train(x=X4, training_frame=data["train"])
        return ae
    if val == "_w2v_pre":
        pre = CONFIGS["w2v"][0](vec_size=8, epochs=1, min_word_freq=2, seed=9)
        pre.train(training_frame=data["text"])
        return pre.to_frame()
    if val == "_knot_ids":
        return val
    pytest.skip(f"no special probe for {val}")
