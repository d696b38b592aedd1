"""Flow notebooks (h2o-web): the cell language parser, the routine runner,
the server's /flow/cell endpoint and NodePersistentStorage, and the
reference's own Flow test-pack notebooks run on synthetic data of their
declared layout (h2o3_amd/server/flow_packs.py)."""
import glob
import json
import os

import numpy as np
import pytest

from h2o3_amd.server.flow import (Assign, Call, FlowError, FlowRunner, FlowSyntaxError, HttpTransport, If,
                                  LocalTransport, ROUTINES, Symbol, parse_cell)
from h2o3_amd.server.flow_packs import PACKS, run_pack

HAVE_PACKS = os.path.isdir(PACKS)


def test_parse_implicit_calls_and_objects():
    assert parse_cell('importFiles [ "../a.csv" ]') == [Call("importFiles", [["../a.csv"]])]
    assert parse_cell("getFrames") == [Call("getFrames", [])]
    # implicit calls nest to the right, trailing pairs form one object
    assert parse_cell("grid inspect 'summary', getGrid \"g\", sort_by:\"auc\", decreasing:true") == [
        Call("grid", [Call("inspect", ["summary", Call("getGrid", ["g", {"sort_by": "auc", "decreasing": True}])])])]
    assert parse_cell('assist buildModel, null, training_frame: "ad.hex"') == [
        Call("assist", [Symbol("buildModel"), None, {"training_frame": "ad.hex"}])]
    src = 'parseFiles\n  paths: ["x.csv"]\n  destination_frame: "x.hex"\n  separator: 44\n  check_header: -1'
    assert parse_cell(src) == [Call("parseFiles", [{"paths": ["x.csv"], "destination_frame": "x.hex",
                                                    "separator": 44, "check_header": -1}])]
    assert parse_cell('buildModel \'gbm\', {"seed":-4147985762995881000,"s":0xDECAF,"h":{"a":["1";"2",null]}}') == [
        Call("buildModel", ["gbm", {"seed": -4147985762995881000, "s": 0xDECAF, "h": {"a": ["1", "2", None]}}])]
    assert parse_cell("# only a comment") == []
    assert parse_cell("predict model: 'm', frame: \"f\"") == [Call("predict", [{"model": "m", "frame": "f"}])]
    assert parse_cell('f "a\\"b\\n"') == [Call("f", ['a"b\n'])]


def test_parse_statements_blocks():
    src = 'x = false\nloc = "d/"\nif x\n  f = loc + "a"\nelse\n  f = "b"\nimportFiles [f]'
    st = parse_cell(src)
    assert st[0] == Assign("x", False)
    assert isinstance(st[2], If) and st[2].other == [Assign("f", "b")]
    assert st[3] == Call("importFiles", [[Symbol("f")]])
    with pytest.raises(FlowSyntaxError):
        parse_cell('f "unterminated')
    with pytest.raises(FlowSyntaxError):
        parse_cell("f a b %")


@pytest.mark.skipif(not HAVE_PACKS, reason="reference Flow packs not present")
def test_every_reference_flow_cell_parses_and_names_known_routines():
    n, unknown = 0, set()

    def walk(x):
        if isinstance(x, Call):
            if x.name not in ROUTINES:
                unknown.add(x.name)
            for a in x.args:
                walk(a)
        elif isinstance(x, (list, tuple)):
            for a in x:
                walk(a)
        elif isinstance(x, dict):
            for a in x.values():
                walk(a)
    for f in glob.glob(os.path.join(PACKS, "*", "*.flow")):
        with open(f) as fh:
            for cell in json.load(fh)["cells"]:
                if cell["type"] == "cs":
                    n += 1
                    st = parse_cell(cell["input"])
                    assigned = {s.name for s in st if isinstance(s, Assign)}
                    walk([s for s in st if not isinstance(s, Assign)])
                    unknown -= assigned
    assert n > 3800
    # bare variables of the KDD example are Calls at statement level only when unassigned in-cell
    assert unknown <= {"hasLocalData"}, unknown


@pytest.fixture(scope="module")
def app(tmp_path_factory):
    from h2o3_amd.server.rest import create_app
    return create_app(flow_dir=str(tmp_path_factory.mktemp("nps")))


def _write_csv(path, n=150, seed=0):
    rng = np.random.default_rng(seed)
    x1, x2 = rng.normal(size=n), rng.normal(size=n)
    y = (x1 + 0.5 * x2 + 0.3 * rng.normal(size=n) > 0).astype(int)
    c = rng.choice(["a", "b", "c"], n)
    with open(path, "w") as f:
        f.write("x1,x2,c,y\n")
        for i in range(n):
            f.write(f"{x1[i]:.4f},{x2[i]:.4f},{c[i]},{y[i]}\n")


def test_notebook_end_to_end_local(app, tmp_path):
    _demo_notebook(app, tmp_path)


@pytest.mark.gpu
def test_notebook_end_to_end_gpu(app, tmp_path):
    """The same notebook with the cloud on the GPU: every routine's model
    build / predict / munging runs through the device paths."""
    import torch
    from h2o3_amd.parallel import cloud
    assert torch.cuda.is_available() and cloud.device().type == "cuda"
    _demo_notebook(app, tmp_path)


def _demo_notebook(app, tmp_path):
    csv = tmp_path / "d.csv"
    _write_csv(csv)
    nb = {"version": "1.0.0", "cells": [
        {"type": "md", "input": "# demo"},
        {"type": "cs", "input": f'path = "{csv}"\nimportFiles [path]'},
        {"type": "cs", "input": "setupParse paths: [path]"},
        {"type": "cs", "input": 'parseFiles\n  paths: [path]\n  destination_frame: "d.hex"\n'
                                '  column_types: ["Numeric","Numeric","Enum","Enum"]\n  check_header: 1'},
        {"type": "cs", "input": 'getFrameSummary "d.hex"'},
        {"type": "cs", "input": 'splitFrame "d.hex", [0.7], ["tr.hex","te.hex"], 42'},
        {"type": "cs", "input": 'buildModel "gbm"'},
        {"type": "cs", "input": 'buildModel \'gbm\', {"model_id":"g1","training_frame":"tr.hex",'
                                '"validation_frame":"te.hex","response_column":"y","ntrees":5,"max_depth":3,'
                                '"checkpoint":"","seed":-1}'},
        {"type": "cs", "input": 'getModel "g1"'},
        {"type": "cs", "input": 'inspect getModel "g1"'},
        {"type": "cs", "input": 'predict model: "g1", frame: "te.hex", predictions_frame: "p1"'},
        {"type": "cs", "input": 'bindFrames "both", [ "p1", "te.hex" ]'},
        {"type": "cs", "input": 'changeColumnType frame: "both", column: "x1", type: \'enum\''},
        {"type": "cs", "input": 'buildModel \'glm\', {"model_id":"gl","training_frame":"tr.hex","response_column":"y",'
                                '"family":"binomial","lambda":[],"hyper_parameters":{"alpha":[[0.0],[0.5],null]},'
                                '"grid_id":"glm_grid"}'},
        {"type": "cs", "input": 'grid inspect "summary", getGrid "glm_grid", sort_by:"auc", decreasing:true'},
        {"type": "cs", "input": "getJobs"},
        {"type": "cs", "input": 'deleteModel "g1"'},
        {"type": "cs", "input": "getModels"},
    ]}
    runner = FlowRunner(LocalTransport(app))
    res = runner.run_notebook(nb)
    kinds = [r.get("kind") for _, _, r in res]
    assert kinds[0] == "markup" and kinds[6] == "form"
    fr = res[4][2]["data"]["frames"][0]
    assert fr["rows"] == 150 and [c["type"] for c in fr["columns"]][2:] == ["enum", "enum"]
    assert res[5][2]["keys"] == ["tr.hex", "te.hex"]
    m = res[8][2]["data"]["models"][0]
    assert m["algo"] == "gbm" and m["output"]["validation_metrics"]["AUC"] > 0.7
    assert res[9][2]["kind"] == "tables" and res[9][2]["data"]
    from h2o3_amd.core import dkv
    both = dkv.get("both")
    assert both.ncol == 3 + 4 and both.vec("x1").type == "enum"
    assert res[14][2]["kind"] == "table"
    assert "g1" not in [x["model_id"]["name"] for x in res[-1][2]["data"]["models"]]
    with pytest.raises(FlowError, match="unknown Flow routine"):
        runner.run_cell("noSuchRoutine 1")
    with pytest.raises(FlowError):
        runner.run_cell('getFrame "missing.hex"')


def test_flow_cell_endpoint_and_node_persistent_storage(app):
    from fastapi.testclient import TestClient
    c = TestClient(app)
    assert "Flow" in c.get("/flow/index.html").text
    assert "buildModel" in c.get("/flow/routines").json()["routines"]
    r = c.post("/flow/cell", json={"input": 'v = "x" + 1'}).json()
    assert r["ok"] and r["result"]["data"] == "x1"
    r = c.post("/flow/cell", json={"input": "v"}).json()       # variables persist across cells
    assert r["result"]["data"] == "x1"
    r = c.post("/flow/cell", json={"input": "getFrame"})
    assert r.status_code == 400 and not r.json()["ok"]
    assert c.get("/3/NodePersistentStorage/configured").json()["configured"] is True
    doc = json.dumps({"version": "1.0.0", "cells": [{"type": "cs", "input": "getFrames"}]})
    assert c.post("/3/NodePersistentStorage/notebook/My Flow (1)", json={"value": doc}).status_code == 200
    assert c.get("/3/NodePersistentStorage/categories/notebook/names/My Flow (1)/exists").json()["exists"]
    assert c.get("/3/NodePersistentStorage/categories/notebook/exists").json()["exists"]
    lst = c.get("/3/NodePersistentStorage/notebook").json()["entries"]
    assert [e["name"] for e in lst] == ["My Flow (1)"] and lst[0]["size"] == len(doc)
    assert json.loads(c.get("/3/NodePersistentStorage/notebook/My Flow (1)").json()["value"]) == json.loads(doc)
    anon = c.post("/3/NodePersistentStorage/notebook", data={"value": "abc"}).json()["name"]
    assert c.get(f"/3/NodePersistentStorage/notebook/{anon}").json()["value"] == "abc"
    assert c.post("/3/NodePersistentStorage/bad.cat/x", json={"value": "1"}).status_code == 400
    assert c.post("/3/NodePersistentStorage/notebook/..", json={"value": "1"}).status_code in (400, 404, 405)
    assert c.post("/3/NodePersistentStorage/notebook/a.b", json={"value": "1"}).status_code == 400
    c.delete("/3/NodePersistentStorage/notebook/My Flow (1)")
    assert not c.get("/3/NodePersistentStorage/categories/notebook/names/My Flow (1)/exists").json()["exists"]


def test_http_transport_runs_a_notebook(app, tmp_path):
    from fastapi.testclient import TestClient
    csv = tmp_path / "h.csv"
    _write_csv(csv, seed=3)
    runner = FlowRunner(HttpTransport("http://testserver", session=TestClient(app)))
    runner.run_cell(f'importFiles ["{csv}"]')
    runner.run_cell(f'parseFiles\n  paths: ["{csv}"]\n  destination_frame: "h.hex"')
    out = runner.run_cell('buildModel \'glm\', {"model_id":"hg","training_frame":"h.hex","response_column":"y",'
                          '"family":"gaussian"}')
    assert out["key"] == "hg"
    assert runner.run_cell('getModel "hg"')["data"]["models"][0]["algo"] == "glm"


@pytest.mark.skipif(not HAVE_PACKS, reason="reference Flow packs not present")
def test_reference_flow_packs_run_on_synthetic_data(app, tmp_path):
    nbs = [os.path.join(PACKS, "test-small", f) for f in (
        "gbm_junit_cars.flow", "glm_test_poisson_tst1.flow", "dl_iris.flow", "impute.flow", "export_frame.flow",
        "automl_prostate.flow", "dl_junit_arff_time.flow")]
    t = LocalTransport(app)
    cwd = os.getcwd()
    os.chdir(tmp_path)                       # export_frame writes a relative path
    try:
        res = run_pack(nbs, str(tmp_path / "data"), t, rows=150, automl_secs=15)
    finally:
        os.chdir(cwd)
    bad = [(r["notebook"], r["errors"]) for r in res if r.get("failed")]
    assert not bad, bad
    assert sum(r["cells"] for r in res) > 50


def test_flow_page_script_and_charts(tmp_path):
    """The Flow page's script parses (node --check) and its inline-SVG charts
    render a scoring-history polyline, variable-importance bars and a ROC
    curve from ModelSchemaV3-shaped tables."""
    import re
    import shutil
    import subprocess
    from pathlib import Path
    node = shutil.which("node")
    if node is None:
        pytest.skip("no node.js")
    src = (Path(__file__).resolve().parents[1] / "h2o3_amd" / "server" / "static" / "flow.html").read_text()
    js = re.search(r"<script>(.*)</script>", src, re.S).group(1)
    (tmp_path / "flow.js").write_text(js)
    subprocess.run([node, "--check", str(tmp_path / "flow.js")], check=True)
    body = js[:js.rindex("(async () => {")]               # function definitions, not the page bootstrap
    harness = body + r'''
const T = (name, cols) => ({__meta: {schema_type: "TwoDimTable"}, name,
  columns: Object.keys(cols).map(n => ({name: n})), data: Object.values(cols)});
const host = {innerHTML: "", appendChild() {}};
global.document = {createElement: () => ({append() {}, appendChild() {}, set onclick(f) {}, className: ""})};
const m = {model_id: {name: "m1"}, output: {
  scoring_history: T("sh", {number_of_trees: [0, 1, 2, 3], training_logloss: [0.69, 0.5, 0.4, 0.35],
                            validation_logloss: [0.69, 0.55, 0.47, 0.44]}),
  variable_importances: T("vi", {variable: ["a", "b"], scaled_importance: [1.0, 0.4]}),
  training_metrics: {AUC: 0.9, thresholds_and_metric_scores: T("thr", {fpr: [0, 0.1, 0.5, 1], tpr: [0, 0.6, 0.9, 1]})}}};
modelCharts(host, m);
console.log(JSON.stringify({poly: (host.innerHTML.match(/<polyline/g) || []).length,
                            rect: (host.innerHTML.match(/<rect/g) || []).length,
                            roc: host.innerHTML.includes("ROC (AUC 0.900000)")}));
'''
    (tmp_path / "h.js").write_text(harness)
    out = subprocess.run([node, str(tmp_path / "h.js")], check=True, capture_output=True, text=True).stdout
    import json
    r = json.loads(out.strip().splitlines()[-1])
    assert r == {"poly": 3, "rect": 2, "roc": True}


def test_model_builder_parameter_metadata(app):
    """/3/ModelBuilders/{algo}: the reference client's parameter list with
    typed entries (enum values, help, critical / secondary / expert levels)
    that Flow's buildModel form renders."""
    from fastapi.testclient import TestClient
    c = TestClient(app)
    ps = c.get("/3/ModelBuilders/gbm").json()["model_builders"]["gbm"]["parameters"]
    by = {p["name"]: p for p in ps}
    assert by["distribution"]["type"] == "enum" and "bernoulli" in by["distribution"]["values"]
    assert by["ntrees"]["type"] == "int" and by["ntrees"]["level"] == "critical"
    assert by["training_frame"]["type"] == "Key<Frame>"
    assert by["sample_rate"]["help"].startswith("Row sample rate")
    assert {p["level"] for p in ps} == {"critical", "secondary", "expert"}
