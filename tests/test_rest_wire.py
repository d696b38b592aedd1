"""Wire compatibility: the reference's own h2o-py client drives the h2o3_amd
REST server.

tests/wire_client.py loads h2o-py from the reference tree (when it is
present: /root/reference/h2o-py, or $H2O_PY_REFERENCE) with a tiny stand-in
for the `future` package, connects with h2o.connect(url=...), uploads a
pandas frame (PostFile -> ParseSetup -> Parse -> Jobs -> Frames), munges it
through Rapids (append, row filter, split_frame, table, group_by, quantile,
cbind, as.character, levels, ls), trains GBM / GLM / K-Means / DRF / DL /
XGBoost models (ModelBuilders -> Jobs -> Models with the metrics and table
schemas), predicts, scores a held-out frame, downloads a MOJO, runs a grid
search sorted by AUC and a small AutoML.  Every value the client computes
comes from this server, so the assertions check both the protocol and the
numbers (e.g. GLM coefficients of y = 2a - b).
"""
import json
import os
import socket
import subprocess
import sys
import threading
import time

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
REF_PY = os.environ.get("H2O_PY_REFERENCE", "/root/reference/h2o-py")


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.fixture(scope="module")
def server_url():
    import uvicorn
    from h2o3_amd.server import create_app
    port = _free_port()
    srv = uvicorn.Server(uvicorn.Config(create_app(), host="127.0.0.1", port=port, log_level="warning"))
    th = threading.Thread(target=srv.run, daemon=True)
    th.start()
    t0 = time.time()
    while not srv.started and time.time() - t0 < 30:
        time.sleep(0.05)
    assert srv.started
    yield f"http://127.0.0.1:{port}"
    srv.should_exit = True
    th.join(timeout=10)


@pytest.mark.skipif(not os.path.isdir(os.path.join(REF_PY, "h2o")), reason="reference h2o-py client not present")
@pytest.mark.timeout(300)
def test_reference_python_client_end_to_end(server_url):
    env = dict(os.environ, PYTHONPATH="", OMP_NUM_THREADS="2")
    r = subprocess.run([sys.executable, "-u", os.path.join(HERE, "wire_client.py"), server_url, REF_PY],
                       capture_output=True, text=True, timeout=280, env=env, cwd=HERE)
    assert r.returncode == 0, (r.stdout[-3000:], r.stderr[-3000:])
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("RESULT ")]
    assert line, r.stdout[-3000:]
    out = json.loads(line[-1][len("RESULT "):])
    assert out["shape"] == [400, 5]
    assert abs(out["a2_sum"] - 2 * 400 * out["mean_a"]) < 1e-3
    assert 150 < out["sub_rows"] < 250
    assert out["levels"] == [["u", "v", "w"]]
    assert sum(out["split"]) == 400 and out["as_df"] == [400, 6]
    tr_auc, va_auc = out["auc"]
    assert tr_auc > 0.95 and va_auc > 0.9 and abs(out["perf_auc"] - va_auc) < 1e-9
    cm = out["cm"]                        # [[tn, fp], [fn, tp]] of the training frame
    assert int(np.sum(cm)) == out["split"][0]
    assert out["varimp"][0][0] in ("a", "b")
    assert out["sh"][0] >= 5 and out["pred"] == [out["split"][1], 3]
    coef = out["glm_coef"]
    assert abs(coef["a"] - 2.0) < 0.05 and abs(coef["b"] + 1.0) < 0.05 and out["glm_r2"] > 0.99
    assert out["km"] > 0 and out["km_centers"] == 3
    assert out["mojo"].endswith(".zip") and out["get_model"]
    assert out["drf_auc"] > 0.85 and out["xgb_auc"] > 0.9 and np.isfinite(out["dl_rmse"])
    assert out["grid"] == 2 and len(out["grid_sorted"]) == 2
    assert out["table"] == [3, 2] and out["group_by"] == [3, 2] and out["cbind"] == 7
    assert out["nunique"] == [3] and out["isna"] == 0 and out["ascharacter"] == "string"
    assert out["aml_leader"] and out["aml_lb"][0] == 2
    assert out["saved"] and abs(out["loaded_auc"] - va_auc) < 1e-9
    assert out["exported_rows"] == out["split"][0]
    assert abs(out["make_metrics_auc"] - va_auc) < 1e-6
    assert out["pdp_rows"] >= 2 and 5 <= out["missing"] <= 40


@pytest.mark.skipif(not os.path.isdir(os.path.join(REF_PY, "h2o")), reason="reference h2o-py client not present")
@pytest.mark.timeout(300)
def test_reference_python_client_munging(server_url):
    """~45 H2OFrame operations of the reference client (merge, sort, impute,
    cut, string ops, apply, ifelse, group_by, kfold, isin, topN, which, ...)
    each evaluate on this server without error."""
    env = dict(os.environ, PYTHONPATH="", OMP_NUM_THREADS="2")
    r = subprocess.run([sys.executable, "-u", os.path.join(HERE, "wire_client_munging.py"), server_url, REF_PY],
                       capture_output=True, text=True, timeout=280, env=env, cwd=HERE)
    assert r.returncode == 0, (r.stdout[-3000:], r.stderr[-3000:])
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("SUMMARY ")]
    assert line, r.stdout[-3000:]
    out = json.loads(line[-1][len("SUMMARY "):])
    bad = [ln for ln in r.stdout.splitlines() if ln.startswith("BAD")]
    assert out["bad"] == [], bad
    assert out["ok"] >= 45


@pytest.mark.skipif(not os.path.isdir(os.path.join(REF_PY, "h2o")), reason="reference h2o-py client not present")
@pytest.mark.timeout(300)
def test_reference_python_client_models(server_url):
    """Model-level accessors of the reference client (tests/wire_client_models.py)."""
    env = dict(os.environ, PYTHONPATH="", OMP_NUM_THREADS="2")
    r = subprocess.run([sys.executable, "-u", os.path.join(HERE, "wire_client_models.py"), server_url, REF_PY],
                       capture_output=True, text=True, timeout=280, env=env, cwd=HERE)
    assert r.returncode == 0, (r.stdout[-3000:], r.stderr[-3000:])
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("SUMMARY ")]
    assert line, r.stdout[-3000:]
    out = json.loads(line[-1][len("SUMMARY "):])
    bad = [ln for ln in r.stdout.splitlines() if ln.startswith("BAD")]
    assert out["bad"] == [], bad
    assert out["ok"] >= 30


@pytest.mark.skipif(not os.path.isdir(os.path.join(REF_PY, "h2o")), reason="reference h2o-py client not present")
@pytest.mark.timeout(300)
def test_reference_python_client_inspection_and_persistence(server_url):
    """H2OTree, Word2Vec, feature interactions, H, rules, TE transform,
    makeGLMModel, frame / grid save-load, sessions (tests/wire_client_more.py)."""
    env = dict(os.environ, PYTHONPATH="", OMP_NUM_THREADS="2")
    r = subprocess.run([sys.executable, "-u", os.path.join(HERE, "wire_client_more.py"), server_url, REF_PY],
                       capture_output=True, text=True, timeout=280, env=env, cwd=HERE)
    assert r.returncode == 0, (r.stdout[-3000:], r.stderr[-3000:])
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("SUMMARY ")]
    assert line, r.stdout[-3000:]
    out = json.loads(line[-1][len("SUMMARY "):])
    bad = [ln for ln in r.stdout.splitlines() if ln.startswith("BAD")]
    assert out["bad"] == [], bad
    assert out["ok"] >= 16


@pytest.mark.skipif(not os.path.isdir(os.path.join(REF_PY, "h2o")), reason="reference h2o-py client not present")
@pytest.mark.timeout(200)
def test_reference_python_client_basic_auth(tmp_path):
    """The reference client with auth=(user, password) against a server
    started with a realm file; without credentials the connect fails."""
    import uvicorn
    from h2o3_amd.server import create_server_app
    realm = tmp_path / "realm.properties"
    realm.write_text("ana: s3cret,user\n")
    port = _free_port()
    srv = uvicorn.Server(uvicorn.Config(create_server_app(str(realm)), host="127.0.0.1", port=port,
                                        log_level="warning"))
    th = threading.Thread(target=srv.run, daemon=True)
    th.start()
    t0 = time.time()
    while not srv.started and time.time() - t0 < 30:
        time.sleep(0.05)
    code = ("import sys, os; sys.path[:0] = [os.path.join(%r, 'refclient_shim'), %r]\n"
            "import h2o\n"
            "h2o.connect(url=%r, auth=('ana', 's3cret'), verbose=False)\n"
            "fr = h2o.H2OFrame({'a': [1, 2, 3]})\n"
            "print('ROWS', fr.nrows)\n"
            "try:\n"
            "    h2o.connect(url=%r, verbose=False)\n"
            "    print('NOAUTH ok')\n"
            "except Exception as e:\n"
            "    print('NOAUTH rejected', type(e).__name__)\n") % (HERE, REF_PY, f"http://127.0.0.1:{port}",
                                                                 f"http://127.0.0.1:{port}")
    try:
        r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=150,
                           env=dict(os.environ, PYTHONPATH=""), cwd=HERE)
    finally:
        srv.should_exit = True
        th.join(timeout=10)
    assert "ROWS 3" in r.stdout, (r.stdout[-2000:], r.stderr[-2000:])
    assert "NOAUTH rejected" in r.stdout, r.stdout[-2000:]
