"""Reference h2o-py calls that use the inspection / persistence / session
routes of server/rest_more.py: H2OTree (GET /3/Tree), Word2Vec synonyms and
transform, feature_interaction, h(), RuleFit rule_importance, TargetEncoder
transform, makeGLMModel, save_frame / load_frame, save_grid / load_grid,
column domains, session properties, Ping, S3 credentials, sparse-matrix
upload (ParseSVMLight).
Run by tests/test_rest_wire.py as `python wire_client_more.py <url> <h2o-py dir>`."""
import json
import os
import sys
import tempfile

sys.path[:0] = [os.path.join(os.path.dirname(os.path.abspath(__file__)), "refclient_shim"), sys.argv[2]]
import h2o  # noqa: E402  (the reference client)
import numpy as np  # noqa: E402
import pandas as pd  # noqa: E402
from h2o.estimators import *  # noqa: E402,F401,F403
from h2o.tree import H2OTree  # noqa: E402

h2o.connect(url=sys.argv[1], verbose=False)
rng = np.random.default_rng(0)
df = pd.DataFrame({"a": rng.normal(size=400), "b": rng.normal(size=400), "c": rng.choice(["u", "v", "w"], 400)})
df["y"] = np.where(df.a + df.b + (df.c == "u") > 0.3, "yes", "no")
fr = h2o.H2OFrame(df)
ok, bad = [], []


def t(name, f):
    try:
        v = f(); ok.append(name); print("OK ", name, str(v)[:100].replace("\n", " "))
    except Exception as e:
        bad.append(name); print("BAD", name, type(e).__name__, " | ".join(str(e).splitlines()[:5])[:600])


gbm = H2OGradientBoostingEstimator(ntrees=3, max_depth=3, seed=1)
gbm.train(x=["a", "b", "c"], y="y", training_frame=fr)


def tree_check():
    tr = H2OTree(gbm, 0, "yes")
    assert len(tr) >= 3 and tr.root_node is not None
    assert tr.left_children[0] == 1 and tr.right_children[0] == 2
    return len(tr), tr.features[0], tr.thresholds[0]
t("h2o_tree", tree_check)
t("feature_interaction", lambda: len(gbm.feature_interaction()))
t("h_stat", lambda: gbm.h(fr, ["a", "b"]))
words = h2o.H2OFrame(pd.DataFrame({"w": (["king", "queen", "man", "woman", "apple", None] * 60)}))
words = words.ascharacter()
w2v = H2OWord2vecEstimator(vec_size=8, epochs=3, min_word_freq=1)
w2v.train(training_frame=words)
t("w2v_synonyms", lambda: len(w2v.find_synonyms("king", 3)))
t("w2v_transform", lambda: w2v.transform(words, aggregate_method="NONE").ncols)
rf = H2ORuleFitEstimator(min_rule_length=1, max_rule_length=2, max_num_rules=5, seed=1)
rf.train(x=["a", "b"], y="y", training_frame=fr)
t("rule_importance", lambda: rf.rule_importance().as_data_frame().shape)
te = H2OTargetEncoderEstimator()
te.train(x=["c"], y="y", training_frame=fr)
t("te_transform", lambda: te.transform(fr, as_training=True).ncols)
glm = H2OGeneralizedLinearEstimator(family="binomial")
glm.train(x=["a", "b"], y="y", training_frame=fr)


def make_glm():
    c = glm.coef()
    c["a"] = 0.0
    m = H2OGeneralizedLinearEstimator.makeGLMModel(glm, c)
    return m.coef()["a"]
t("make_glm_model", make_glm)
d = tempfile.mkdtemp()


def save_load_frame():
    fr.save(d + "/fr", force=True)
    back = h2o.load_frame(fr.frame_id, d + "/fr", force=True)
    assert back.nrows == fr.nrows
    return back.dim
t("save_load_frame", save_load_frame)
from h2o.grid.grid_search import H2OGridSearch  # noqa: E402
gs = H2OGridSearch(H2OGradientBoostingEstimator(ntrees=2, seed=1), {"max_depth": [2, 3]}, grid_id="wgrid")
gs.train(x=["a", "b"], y="y", training_frame=fr)


def save_load_grid():
    p = h2o.save_grid(d, "wgrid")
    g = h2o.load_grid(p)
    return len(g.model_ids)
t("save_load_grid", save_load_grid)
t("levels_domain", lambda: h2o.api("GET /3/Frames/%s/columns/c/domain" % fr.frame_id)["domain"])
t("ping", lambda: h2o.api("GET /3/Ping")["cloud_healthy"])
t("session_prop", lambda: (h2o.api("POST /3/SessionProperties", data={"key": "k", "value": "v"}),
                           h2o.api("GET /3/SessionProperties", data={"key": "k"})["value"])[1])
t("model_builders", lambda: len(h2o.api("GET /3/ModelBuilders")["model_builders"]))


def s3():
    from h2o.persist import set_s3_credentials, remove_s3_credentials
    set_s3_credentials("AKID", "SECRET")
    remove_s3_credentials()
    return True
t("s3_credentials", s3)


def sparse_upload():
    import scipy.sparse as sp
    m = sp.random(50, 6, density=0.3, format="csr", random_state=1)
    f = h2o.H2OFrame(m)
    return f.dim
t("sparse_upload", sparse_upload)


def assembly():
    from h2o.assembly import H2OAssembly
    from h2o.transforms.preprocessing import H2OColOp, H2OColSelect
    asm = H2OAssembly(steps=[("select", H2OColSelect(["a", "b", "c"])),
                             ("cos_a", H2OColOp(op=h2o.H2OFrame.cos, col="a", inplace=True)),
                             ("cnt_c", H2OColOp(op=h2o.H2OFrame.countmatches, col="c", inplace=False, pattern="u"))])
    out = asm.fit(fr)
    got = out.as_data_frame()
    assert abs(got["a"].values - np.cos(df.a.values)).max() < 1e-5 and out.ncols == 4
    return out.dim
t("assembly", assembly)
print("SUMMARY " + json.dumps({"ok": len(ok), "bad": bad}))
