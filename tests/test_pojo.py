"""POJO export: the generated Java is translated line-by-line into Python
(the generator emits a small fixed grammar: if/else, returns, arithmetic on
doubles, Math.exp) and executed, so the POJO's score0 is checked numerically
against in-memory predictions.  No JVM in this environment."""
import math
import re

import numpy as np
import pandas as pd
import pytest

import h2o3_amd as h2o
from h2o3_amd.estimators import (H2OGeneralizedLinearEstimator, H2OGradientBoostingEstimator,
                                 H2ORandomForestEstimator)
from h2o3_amd.mojo.pojo import to_java


def _expr(e):
    e = re.sub(r"\(float\) (data\[\d+\])", r"f32(\1)", e)
    e = re.sub(r"(?<![\w.])(-?\d+\.\d+(e-?\d+)?|-?\d+e-?\d+)f\b", r"f32(\1)", e)
    e = re.sub(r"\(int\) (\w+(?:\[[^\]]*\])?)", r"int(\1)", e)
    for a_, b_ in (("!Double.isNaN", "not math.isnan"), ("Double.isNaN", "math.isnan"),
                   ("Double.POSITIVE_INFINITY", "math.inf"), ("Double.NEGATIVE_INFINITY", "-math.inf"),
                   ("Math.exp", "math.exp"), ("Math.log", "math.log"), ("Math.sqrt", "math.sqrt"),
                   ("Math.abs", "abs"), ("Math.max", "max"), ("Math.min", "min"), ("||", " or "), ("&&", " and ")):
        e = e.replace(a_, b_)
    return e


def _java_to_python(src):
    """Translate the POJO's constant arrays, static tree methods and score0
    (the generator's fixed grammar: declarations, for loops over int ranges,
    if / else blocks, arithmetic, Math.* calls, ternary labels)."""
    py = ["import math", "import numpy as _np", "def f32(x):", "    return float(_np.float32(x))",
          "def inBits(bits, v):", "    c = int(v)", "    return 0 <= c < len(bits) and bits[c] != 0",
          "def nz(v, plug):", "    return plug if math.isnan(v) else v",
          "def level(v, mode, lvl):", "    c = mode if math.isnan(v) else int(v)", "    return 1.0 if c == lvl else 0.0"]
    ind = 0
    in_fn = False
    for raw in src.splitlines():
        ln = raw.strip()
        m = re.match(r"static final (?:byte|int|double)\[\] (\w+) = new \w+\[\] \{(.*)\};", ln)
        if m:
            py.append(f"{m.group(1)} = [{_expr(m.group(2))}]")
            continue
        m = re.match(r"static final double\[\]\[\] (\w+) = new double\[\]\[\] \{(.*)\};", ln)
        if m:
            py.append(f"{m.group(1)} = [{_expr(m.group(2)).replace('{', '[').replace('}', ']')}]")
            continue
        m = re.match(r"static double (tree_\d+)\(double\[\] data\) \{", ln)
        if m or ln.startswith("public final double[] score0"):
            name = m.group(1) if m else "score0"
            args = "data" if m else "data, preds"
            py.append(f"def {name}({args}):")
            ind, in_fn = 1, True
            continue
        if not in_fn:
            continue
        if ln == "}" and ind == 1:
            in_fn = False
            continue
        e = _expr(ln)
        m = re.match(r"for \(int (\w+) = (.+); \1 < (.+); \1\+\+\) \{$", e)
        if m:
            py.append("    " * ind + f"for {m.group(1)} in range({m.group(2)}, {m.group(3)}):")
            ind += 1
            continue
        if e.startswith("if (") and e.endswith(") {"):
            cond = e[4:-3]
            if " ? " in cond:
                a, rest = cond.split(" ? ", 1)
                t, f = rest.split(" : ", 1)
                cond = f"({t.replace('true', 'True').replace('false', 'False')} if {a} else {f})"
            py.append("    " * ind + f"if {cond}:")
            ind += 1
        elif e == "} else {":
            py.append("    " * (ind - 1) + "else:")
        elif e == "}":
            ind -= 1
        elif e.startswith("return"):
            py.append("    " * ind + e.rstrip(";"))
        else:
            m = re.match(r"(?:double|int)\[\] (\w+) = new (?:double|int)\[(.+)\];", e)
            if m:
                py.append("    " * ind + f"{m.group(1)} = [0.0] * ({m.group(2)})")
                continue
            stmt = re.sub(r"^(?:double|int) ", "", e.rstrip(";"))
            stmt = re.sub(r"(\S+) >= (\S+) \? 1 : 0", r"(1 if \1 >= \2 else 0)", stmt)
            for part in stmt.split("; "):
                py.append("    " * ind + part.strip().rstrip(";"))
    ns = {}
    exec("\n".join(py), ns)
    return ns["score0"]


def _names_domains(src):
    names = re.findall(r'"((?:[^"\\]|\\.)*)"', re.search(r"NAMES = new String\[\] \{(.*)\};", src).group(1))
    dl = re.search(r"DOMAINS = new String\[\]\[\] \{(.*)\};", src).group(1)
    doms = []
    for part in re.findall(r"null|new String\[\] \{[^}]*\}", dl):
        doms.append(None if part == "null" else re.findall(r'"((?:[^"\\]|\\.)*)"', part))
    return names, doms


@pytest.fixture(scope="module")
def data():
    h2o.init(verbose=False)
    rng = np.random.RandomState(0)
    n = 600
    df = pd.DataFrame({"a": rng.randn(n), "b": rng.randn(n), "c": rng.choice(["u", "v", "w"], n)})
    df.loc[::17, "a"] = np.nan
    df["y"] = np.where(df.a.fillna(0) + (df.c == "v") * 1.0 + 0.3 * rng.randn(n) > 0.4, "yes", "no")
    df["r"] = df.a.fillna(0) * 2 + df.b
    return df


def _rows(df, names, doms):
    X = np.full((len(df), len(names)), np.nan)
    for j, c in enumerate(names):
        if doms.get(c):
            idx = {d: i for i, d in enumerate(doms[c])}
            X[:, j] = [idx.get(v, np.nan) for v in df[c]]
        else:
            X[:, j] = df[c].values
    return X


@pytest.mark.parametrize("algo", ["gbm", "drf", "glm"])
def test_pojo_scores_like_the_model(data, algo):
    fr = h2o.H2OFrame(data)
    if algo == "gbm":
        m = H2OGradientBoostingEstimator(ntrees=5, max_depth=3, seed=1)
    elif algo == "drf":
        m = H2ORandomForestEstimator(ntrees=4, max_depth=4, seed=1)
    else:
        m = H2OGeneralizedLinearEstimator(family="binomial", lambda_=0)
    m.train(x=["a", "b", "c"], y="y", training_frame=fr)
    src = to_java(m)
    assert "extends GenModel" in src and src.count("{") == src.count("}")
    score0 = _java_to_python(src)
    doms = getattr(m, "_x_domains", None) or {c: d for c, d in m._dinfo.domains.items()}
    X = _rows(data, ["a", "b", "c"], doms)
    ref = m.predict(fr).as_data_frame()["yes"].values
    got = np.array([score0(list(x), [0.0, 0.0, 0.0])[2] for x in X])
    np.testing.assert_allclose(got, ref, atol=1e-5)


@pytest.mark.parametrize("algo", ["kmeans", "pca", "deeplearning", "naivebayes", "dl_reg"])
def test_pojo_more_algos(data, algo):
    """K-Means / PCA / Deep Learning / Naive Bayes POJOs score like the model."""
    from h2o3_amd.estimators import (H2ODeepLearningEstimator, H2OKMeansEstimator, H2ONaiveBayesEstimator,
                                     H2OPrincipalComponentAnalysisEstimator)
    fr = h2o.H2OFrame(data)
    x = ["a", "b", "c"]
    if algo == "kmeans":
        m = H2OKMeansEstimator(k=3, seed=1, standardize=True)
        m.train(x=x, training_frame=fr)
    elif algo == "pca":
        m = H2OPrincipalComponentAnalysisEstimator(k=2, transform="STANDARDIZE", seed=1)
        m.train(x=x, training_frame=fr)
    elif algo == "deeplearning":
        m = H2ODeepLearningEstimator(hidden=[6, 5], epochs=3, seed=1, reproducible=True, activation="Tanh")
        m.train(x=x, y="y", training_frame=fr)
    elif algo == "dl_reg":
        m = H2ODeepLearningEstimator(hidden=[4], epochs=3, seed=1, reproducible=True, activation="RectifierWithDropout",
                                     hidden_dropout_ratios=[0.2])
        m.train(x=x, y="r", training_frame=fr)
    else:
        m = H2ONaiveBayesEstimator(laplace=0.5)
        m.train(x=x, y="y", training_frame=fr)
    src = to_java(m)
    assert "extends GenModel" in src and src.count("{") == src.count("}")
    score0 = _java_to_python(src)
    names, doms = _names_domains(src)
    X = _rows(data, names[:len([n for n in names if n in data.columns and n not in ("y", "r")])],
              {n: d for n, d in zip(names, doms) if d})
    pred = m.predict(fr).as_data_frame()
    if algo == "kmeans":
        got = np.array([score0(list(r), [0.0])[0] for r in X])
        np.testing.assert_array_equal(got.astype(int), pred["predict"].values.astype(int))
    elif algo == "pca":
        got = np.array([score0(list(r), [0.0, 0.0]) for r in X])
        # PCAModel.toJavaPredictBody lets a missing numeric propagate (the
        # in-cluster predict mean-imputes it)
        na = data["a"].isna().values
        assert np.isnan(got[na]).all()
        np.testing.assert_allclose(got[~na], pred[["PC1", "PC2"]].values[~na], rtol=1e-5, atol=1e-5)
    elif algo == "dl_reg":
        got = np.array([score0(list(r), [0.0])[0] for r in X])
        np.testing.assert_allclose(got, pred["predict"].values, rtol=1e-4, atol=1e-4)
    else:
        got = np.array([score0(list(r), [0.0, 0.0, 0.0])[2] for r in X])
        np.testing.assert_allclose(got, pred["yes"].values, rtol=1e-4, atol=1e-5)


@pytest.mark.parametrize("family", ["multinomial", "ordinal"])
def test_pojo_glm_multinomial_ordinal(data, family):
    """Multinomial / ordinal GLM POJO (GLMModel.java:1827-1865): class
    probabilities of the generated score0 equal the model's."""
    df = data.copy()
    df["k"] = np.where(df.a.fillna(0) < -0.4, "lo", np.where(df.a.fillna(0) > 0.5, "hi", "mid"))
    fr = h2o.H2OFrame(df)
    fr["k"] = fr["k"].asfactor()
    m = H2OGeneralizedLinearEstimator(family=family, lambda_=0 if family == "multinomial" else 1e-4)
    m.train(x=["a", "b", "c"], y="k", training_frame=fr)
    src = to_java(m)
    assert "extends GenModel" in src and src.count("{") == src.count("}")
    score0 = _java_to_python(src)
    doms = {c: d for c, d in m._dinfo.domains.items()}
    X = _rows(df, ["a", "b", "c"], doms)
    pred = m.predict(fr).as_data_frame()
    lv = list(fr["k"]._vecs[0].domain) if hasattr(fr["k"], "_vecs") else ["hi", "lo", "mid"]
    got = np.array([score0(list(x), [0.0] * 4)[1:] for x in X])
    np.testing.assert_allclose(got, pred[lv].values, atol=1e-6)
