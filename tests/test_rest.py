"""REST API round trip: upload -> build -> predict -> jobs -> delete."""
import numpy as np
import pandas as pd
from fastapi.testclient import TestClient

import h2o3_amd as h2o
from h2o3_amd.server import create_app


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
    job = r.json()["job"]
    assert job["status"] == "DONE" and job["dest"]["name"] == "gbm_rest"
    mj = c.get("/3/Models/gbm_rest").json()["models"][0]
    assert mj["algo"] == "gbm" and mj["output"]["training_metrics"]["AUC"] > 0.9
    pr = c.post("/3/Predictions/models/gbm_rest/frames/train.hex").json()
    assert pr["predictions_frame"]["name"] and pr["model_metrics"][0]["AUC"] > 0.9
    assert any(j["dest"]["name"] == "gbm_rest" for j in c.get("/3/Jobs").json()["jobs"])
    assert c.delete("/3/DKV/train.hex").status_code == 200
    assert c.get("/3/Frames/train.hex").status_code == 404
    assert len(c.get("/3/Metadata/endpoints").json()["routes"]) > 10
