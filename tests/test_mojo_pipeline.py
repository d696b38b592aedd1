"""MOJO pipelines (hex/genmodel/MojoPipelineBuilder.java, MojoPipelineWriter,
algos/pipeline/MojoPipelineReader + MojoPipeline): the reference's own
pipeline test (MojoPipelineBuilderTest) assembles its K-Means fixture, whose
cluster feeds the GLM fixture's CLUSTER input, and pins two prostate rows;
the same assembly here, read back by the reference-layout reader, must give
those numbers."""
import os

import numpy as np
import pandas as pd
import pytest

D = "/root/reference/h2o-genmodel/src/test/resources/hex/genmodel/algos/pipeline"


@pytest.mark.skipif(not os.path.exists(os.path.join(D, "glm_model.zip")), reason="reference fixtures not available")
def test_reference_pipeline_fixture_predictions(tmp_path):
    from h2o3_amd.mojo import h2o_mojo
    from h2o3_amd.mojo.h2o_writer import build_mojo_pipeline
    z = build_mojo_pipeline({"clustering": os.path.join(D, "kmeans_model.zip"),
                             "regression": os.path.join(D, "glm_model.zip")},
                            {"CLUSTER": "clustering:0"}, "regression")
    path = tmp_path / "mojo-pipeline.zip"
    path.write_bytes(z)
    mj = h2o_mojo.load(str(path))
    assert mj.algo == "pipeline" and mj.columns[:2] == ["AGE", "RACE"] and "CLUSTER" not in mj.columns
    rows = pd.DataFrame({"AGE": [71.0, 76.0], "RACE": ["1", "2"], "DPROS": [3.0, 2.0], "DCAPS": [2.0, 1.0],
                         "PSA": [3.3, 51.2], "VOL": [0.0, 20.0], "GLEASON": [8.0, 7.0]})
    got = mj.predict(rows)["predict"].values
    np.testing.assert_allclose(got, [0.7812266, 0.5690164], atol=1e-7)
    # the pipeline equals scoring the two models by hand
    km = h2o_mojo.load(os.path.join(D, "kmeans_model.zip"))
    gl = h2o_mojo.load(os.path.join(D, "glm_model.zip"))
    cl = km.predict(rows[["AGE", "RACE"]])["predict"].values
    man = rows.copy()
    man["CLUSTER"] = [str(int(c)) if gl.domains[0] and str(int(c)) in gl.domains[0] else gl.domains[0][int(c)]
                      for c in cl]
    np.testing.assert_allclose(gl.predict(man)["predict"].values, got, rtol=1e-12)


def test_pipeline_rejects_missing_main_model():
    from h2o3_amd.mojo.h2o_writer import build_mojo_pipeline
    if not os.path.exists(os.path.join(D, "glm_model.zip")):
        pytest.skip("reference fixtures not available")
    with pytest.raises(ValueError, match="Main model is missing"):
        build_mojo_pipeline({"a": os.path.join(D, "glm_model.zip")}, {}, "b")
