"""REST API round trip: upload -> build -> predict -> jobs -> delete."""
import numpy as np
import pandas as pd
from fastapi.testclient import TestClient

import h2o3_amd as h2o
from h2o3_amd.server import create_app


def _wait(c, job, timeout=120):
    """Poll /3/Jobs/{key} like h2o-py's H2OJob.poll until the job leaves RUNNING."""
    import time
    t0 = time.time()
    while job["status"] in ("CREATED", "RUNNING") and time.time() - t0 < timeout:
        time.sleep(0.05)
        job = c.get(f"/3/Jobs/{job['key']['name']}").json()["jobs"][0]
    return job


def test_rest_roundtrip():
    h2o.init()
    c = TestClient(create_app())
    assert c.get("/3/Cloud").json()["cloud_healthy"]
    rng = np.random.default_rng(0)
    df = pd.DataFrame({"a": rng.normal(size=200), "b": rng.normal(size=200)})
    df["y"] = np.where(df.a + df.b > 0, "p", "n")
    r = c.post("/3/PostFile", json={"data": df.to_dict(orient="list"), "destination_frame": "train.hex"})
    assert r.json()["destination_frame"] == "train.hex"
    fj = c.get("/3/Frames/train.hex").json()["frames"][0]
    assert fj["rows"] == 200 and fj["column_count"] == 3
    r = c.post("/3/ModelBuilders/gbm", json={"training_frame": "train.hex", "response_column": "y", "ntrees": 5,
                                              "model_id": "gbm_rest"})
    job = _wait(c, r.json()["job"])
    assert job["status"] == "DONE" and job["dest"]["name"] == "gbm_rest"
    mj = c.get("/3/Models/gbm_rest").json()["models"][0]
    assert mj["algo"] == "gbm" and mj["output"]["training_metrics"]["AUC"] > 0.9
    pr = c.post("/3/Predictions/models/gbm_rest/frames/train.hex").json()
    assert pr["predictions_frame"]["name"] and pr["model_metrics"][0]["AUC"] > 0.9
    assert any(j["dest"]["name"] == "gbm_rest" for j in c.get("/3/Jobs").json()["jobs"])
    assert c.delete("/3/DKV/train.hex").status_code == 200
    assert c.get("/3/Frames/train.hex").status_code == 404
    assert len(c.get("/3/Metadata/endpoints").json()["routes"]) > 10


def test_rest_parse_grid_automl_mojo(tmp_path):
    h2o.init()
    c = TestClient(create_app())
    rng = np.random.default_rng(1)
    df = pd.DataFrame({"a": rng.normal(size=300), "b": rng.normal(size=300)})
    df["y"] = np.where(df.a - df.b > 0, "p", "n")
    p = tmp_path / "d.csv"
    df.to_csv(p, index=False)
    st = c.post("/3/ParseSetup", json={"source_frames": [str(p)]}).json()
    assert st["separator"] == ord(",")
    r = c.post("/3/Parse", json={"source_frames": [str(p)], "destination_frame": "d.hex", "separator": 44}).json()
    assert r["destination_frame"]["name"] == "d.hex"
    assert "a,b,y" in c.get("/3/DownloadDataset", params={"frame_id": "d.hex"}).text
    g = c.post("/99/Grid/gbm", json={"training_frame": "d.hex", "response_column": "y", "ntrees": 3,
                                      "hyper_parameters": {"max_depth": [2, 3]}, "grid_id": "g_rest"}).json()
    assert _wait(c, g["job"])["status"] == "DONE"
    gj = c.get("/99/Grids/g_rest").json()
    assert len(gj["model_ids"]) == 2
    mid = gj["model_ids"][0]["name"]
    z = c.get(f"/3/Models/{mid}/mojo")
    assert z.status_code == 200 and z.content[:2] == b"PK"
    assert "extends GenModel" in c.get(f"/3/Models.java/{mid}").text
    mm = c.post(f"/3/ModelMetrics/models/{mid}/frames/d.hex").json()
    assert mm["model_metrics"][0]["AUC"] > 0.8
    a = c.post("/99/AutoMLBuilder", json={"build_control": {"project_name": "aml_rest", "nfolds": 2,
                                                            "stopping_criteria": {"max_models": 2, "seed": 1}},
                                          "input_spec": {"training_frame": "d.hex", "response_column": "y"},
                                          "build_models": {"include_algos": ["GLM", "GBM"]}}).json()
    assert a["job"]["dest"]["name"] == "aml_rest"
    assert _wait(c, a["job"], timeout=300)["status"] == "DONE"
    lb = c.get("/99/Leaderboards/aml_rest").json()
    assert len(lb["models"]) >= 2
    assert c.get("/3/About").status_code == 200


def test_rest_basic_auth_realm_file(tmp_path):
    """-hash_login: Basic auth against a Jetty realm file (plain, MD5:, OBF:)."""
    import base64
    import hashlib
    from h2o3_amd.server import create_server_app
    from h2o3_amd.server.auth import deobfuscate
    realm = tmp_path / "realm.properties"
    realm.write_text("# users\nalice: wonderland,admin\nbob: MD5:%s\ncarol: OBF:1yta1t331v8w1v9q1t331ytc,user\n"
                     % hashlib.md5(b"builder").hexdigest())
    assert deobfuscate("OBF:1yta1t331v8w1v9q1t331ytc") == "secret"
    h2o.init()
    c = TestClient(create_server_app(str(realm)))

    def hdr(u, p):
        return {"Authorization": "Basic " + base64.b64encode(f"{u}:{p}".encode()).decode()}
    r = c.get("/3/Cloud")
    assert r.status_code == 401 and "Basic" in r.headers["www-authenticate"]
    assert c.get("/3/Cloud", headers=hdr("alice", "nope")).status_code == 401
    for u, p in (("alice", "wonderland"), ("bob", "builder"), ("carol", "secret")):
        assert c.get("/3/Cloud", headers=hdr(u, p)).json()["cloud_healthy"]


def test_flow_page_served():
    h2o.init()
    c = TestClient(create_app())
    r = c.get("/", follow_redirects=True)
    assert r.status_code == 200 and "h2o3_amd Flow" in r.text
    # the notebook page runs cells through /flow/cell and keeps notebooks in NodePersistentStorage
    for ep in ("/3/Cloud", "/3/Frames", "/3/Models", "/flow/cell", "/flow/routines",
               "/3/NodePersistentStorage/notebook"):
        assert ep in r.text
