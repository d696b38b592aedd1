"""Utility routes of server/rest_more.py over the REST app: Tabulate,
DataInfoFrame, ComputeGram (vs numpy), DCTTransformer (vs scipy), Find,
ModelMetrics listings, monitoring (WaterMeter, Profiler, KillMinus3,
SteamMetrics), POJO preview, endpoint metadata, Ping, Typeahead."""
import numpy as np
import pandas as pd
import scipy.fft as sfft
from fastapi.testclient import TestClient

import h2o3_amd as h2o
from h2o3_amd.core import dkv
from h2o3_amd.server import create_app


def test_rest_more_routes():
    h2o.init()
    c = TestClient(create_app())
    rng = np.random.default_rng(0)
    n = 300
    df = pd.DataFrame({"a": rng.normal(size=n), "b": rng.normal(size=n), "c": rng.choice(list("xyz"), n)})
    df["y"] = np.where(df.a + df.b > 0, "p", "n")
    c.post("/3/PostFile", json={"data": df.to_dict(orient="list"), "destination_frame": "t.hex"})
    assert c.post("/3/ModelBuilders/gbm", json={"training_frame": "t.hex", "response_column": "y", "ntrees": 3,
                                                "model_id": "g1"}).status_code == 200
    tab = c.post("/99/Tabulate", json={"dataset": "t.hex", "predictor": "a", "response": "y", "nbins_predictor": 5,
                                       "nbins_response": 2}).json()
    assert sum(tab["count_table"]["data"][2]) == n
    di = c.post("/3/DataInfoFrame", json={"frame": "t.hex", "use_all": True}).json()
    X = dkv.get(di["result"]["name"]).as_data_frame()
    assert X.shape[1] == 3 + 2 + 2                     # c (3 levels) + y (2) one-hot, a, b
    g = c.get("/3/ComputeGram", params={"X": "t.hex"}).json()
    G = dkv.get(g["destination_frame"]["name"]).as_data_frame().values
    Xd = c.post("/3/DataInfoFrame", json={"frame": "t.hex"}).json()
    Xm = dkv.get(Xd["result"]["name"]).as_data_frame().values
    np.testing.assert_allclose(G, Xm.T @ Xm, rtol=1e-5, atol=1e-4)
    f = c.get("/3/Find", params={"key": "t.hex", "column": "c", "row": 5, "match": "x"}).json()
    xs = np.nonzero(df.c.values == "x")[0]
    assert f["next"] == xs[xs > 5][0] and f["prev"] == (xs[xs < 5][-1] if (xs < 5).any() else -1)
    assert c.get("/3/ModelMetrics/models/g1").json()["model_metrics"]
    assert c.delete("/3/ModelMetrics").status_code == 200
    for url in ("/3/WaterMeterCpuTicks/0", "/3/WaterMeterIo", "/3/SteamMetrics", "/3/Profiler", "/3/Ping",
                "/3/Metadata/endpoints/Frames"):
        assert c.get(url).status_code == 200, url
    assert c.post("/3/KillMinus3").status_code == 200
    assert "score0" in c.get("/3/Models.java/g1/preview").text
    d2 = pd.DataFrame({f"c{i}": rng.normal(size=10) for i in range(8)})
    c.post("/3/PostFile", json={"data": d2.to_dict(orient="list"), "destination_frame": "d.hex"})
    r = c.post("/99/DCTTransformer", json={"dataset": "d.hex", "dimensions": [8, 1, 1]}).json()
    out = dkv.get(r["destination_frame"]["name"]).as_data_frame().values
    np.testing.assert_allclose(out, sfft.dct(d2.values, type=2, axis=1, norm="ortho"), atol=1e-5)
    assert c.post("/99/DCTTransformer", json={"dataset": "d.hex", "dimensions": [3, 1, 1]}).status_code == 400
