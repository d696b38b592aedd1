"""One REST endpoint drives a 2-rank cloud (server/spmd.py), with asynchronous
jobs: live progress, cancel, and models equal to the 1-rank cloud's.

Each server is `python -m h2o3_amd.server` started as RANK 0 / 1 of a gloo
cloud on the CPU (the GPU cloud runs the same code under torchrun with
RCCL for the data plane).  The reference's own h2o-py client drives it end
to end (tests/wire_client.py)."""
import os
import signal
import socket
import subprocess
import sys
import time

import numpy as np
import pytest
import requests

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _launch(world, gpu=False):
    http = _free_port()
    mport = _free_port()
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), LOCAL_RANK=str(r), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(mport), OMP_NUM_THREADS="2", PYTHONPATH=ROOT, H2O3_SPMD_IDLE_S="5", H2O3_REST_DEBUG="1")
        if gpu:
            env["H2O3_DIST_BACKEND"] = "gloo"      # N ranks share the box's one GPU: gloo data plane
        else:
            env["CUDA_VISIBLE_DEVICES"] = ""
        procs.append(subprocess.Popen([sys.executable, "-u", "-m", "h2o3_amd.server", "--port", str(http)],
                                      env=env, cwd=ROOT, stdout=subprocess.PIPE, stderr=subprocess.STDOUT,
                                      start_new_session=True))
    url = f"http://127.0.0.1:{http}"
    t0 = time.time()
    while time.time() - t0 < 180:
        try:
            if requests.get(url + "/3/Cloud", timeout=2).status_code == 200:
                return url, procs
        except requests.RequestException:
            pass
        if any(p.poll() is not None for p in procs):
            break
        time.sleep(0.3)
    _stop(url, procs)
    raise RuntimeError("server did not come up: " + "".join(
        (p.stdout.read() or b"").decode(errors="replace")[-2000:] for p in procs))


def _stop(url, procs):
    try:
        requests.post(url + "/3/Shutdown", timeout=10)
    except requests.RequestException:
        pass
    for p in procs:
        try:
            p.wait(timeout=60)
        except subprocess.TimeoutExpired:
            os.killpg(p.pid, signal.SIGKILL)
            p.wait()


@pytest.fixture(scope="module")
def cloud2():
    url, procs = _launch(2)
    yield url
    _stop(url, procs)
    assert all(p.returncode == 0 for p in procs), [p.returncode for p in procs]


@pytest.fixture(scope="module")
def cloud1():
    url, procs = _launch(1)
    yield url
    _stop(url, procs)


def _upload(url, df, name):
    r = requests.post(url + "/3/PostFile", json={"data": df.to_dict(orient="list"), "destination_frame": name})
    assert r.status_code == 200, r.text
    return name


def _wait(url, job, timeout=240, seen=None):
    t0 = time.time()
    while job["status"] in ("CREATED", "RUNNING") and time.time() - t0 < timeout:
        if seen is not None:
            seen.append((job["status"], job["progress"]))
        time.sleep(0.02)
        job = requests.get(url + f"/3/Jobs/{job['key']['name']}").json()["jobs"][0]
    return job


def _data(n=3000, seed=0):
    import pandas as pd
    rng = np.random.default_rng(seed)
    df = pd.DataFrame({"a": rng.normal(size=n), "b": rng.normal(size=n), "c": rng.normal(size=n)})
    df["y"] = np.where(df.a - 0.5 * df.b + 0.3 * rng.normal(size=n) > 0, "p", "n")
    df["r"] = 2 * df.a - df.b + 0.1 * rng.normal(size=n)
    return df


def _build(url, algo, body):
    r = requests.post(url + f"/3/ModelBuilders/{algo}", json=body)
    assert r.status_code == 200, r.text
    job = _wait(url, r.json()["job"])
    assert job["status"] == "DONE", job
    return requests.get(url + f"/3/Models/{body['model_id']}").json()["models"][0]["output"]


def test_cloud_size_is_two(cloud2):
    j = requests.get(cloud2 + "/3/Cloud").json()
    assert j["cloud_size"] == 2 and j["cloud_healthy"]


def test_models_equal_one_rank_cloud(cloud1, cloud2):
    """GBM / GLM / K-Means built through one REST endpoint on 2 ranks equal
    the 1-rank models (same trees / coefficients / centers)."""
    df = _data()
    out = {}
    for name, url in (("one", cloud1), ("two", cloud2)):
        _upload(url, df, "eq.hex")
        g = _build(url, "gbm", {"training_frame": "eq.hex", "response_column": "y", "ntrees": 8, "max_depth": 4,
                                "seed": 7, "model_id": "gbm_eq", "ignored_columns": ["r"]})
        l = _build(url, "glm", {"training_frame": "eq.hex", "response_column": "r", "lambda_": 0, "seed": 1,
                                "model_id": "glm_eq", "ignored_columns": ["y"]})
        k = _build(url, "kmeans", {"training_frame": "eq.hex", "k": 3, "seed": 5, "model_id": "km_eq",
                                   "ignored_columns": ["y", "r"]})
        out[name] = (g["training_metrics"]["logloss"], l["coefficients_table"]["data"],
                     k["centers"]["data"])
    assert abs(out["one"][0] - out["two"][0]) < 1e-6
    np.testing.assert_allclose(np.array(out["one"][1][1], float), np.array(out["two"][1][1], float), rtol=1e-6,
                               atol=1e-7)
    np.testing.assert_allclose(np.array(out["one"][2][1:], float), np.array(out["two"][2][1:], float),
                               rtol=1e-6, atol=1e-8)


def test_job_poll_sees_running_then_done(cloud2):
    _upload(cloud2, _data(20000, 1), "poll.hex")
    r = requests.post(cloud2 + "/3/ModelBuilders/gbm", json={"training_frame": "poll.hex", "response_column": "y",
                                                              "ntrees": 150, "max_depth": 5, "model_id": "gbm_poll",
                                                              "score_tree_interval": 50})
    job = r.json()["job"]
    assert job["status"] == "RUNNING"
    seen = []
    job = _wait(cloud2, job, seen=seen)
    assert job["status"] == "DONE" and job["progress"] == 1.0
    assert any(s == "RUNNING" and 0 < p < 1 for s, p in seen), seen[:20]
    m = requests.get(cloud2 + "/3/Models/gbm_poll").json()["models"][0]
    assert m["output"]["model_summary"]["data"][1][0] == 150 or m["algo"] == "gbm"


def test_cancel_stops_a_long_gbm(cloud2):
    _upload(cloud2, _data(20000, 2), "cancel.hex")
    r = requests.post(cloud2 + "/3/ModelBuilders/gbm", json={"training_frame": "cancel.hex", "response_column": "y",
                                                              "ntrees": 10000, "max_depth": 5,
                                                              "model_id": "gbm_cancel"})
    job = r.json()["job"]
    key = job["key"]["name"]
    t0 = time.time()
    while time.time() - t0 < 120:
        job = requests.get(cloud2 + f"/3/Jobs/{key}").json()["jobs"][0]
        if job["progress"] > 0:
            break
        time.sleep(0.05)
    assert job["status"] == "RUNNING" and 0 < job["progress"] < 0.5
    assert requests.post(cloud2 + f"/3/Jobs/{key}/cancel").status_code == 200
    job = _wait(cloud2, job, timeout=60)
    assert job["status"] == "CANCELLED", job
    assert time.time() - t0 < 120
    # both ranks stopped at the same tree: the cloud still runs collectives
    fr = requests.get(cloud2 + "/3/Frames/cancel.hex").json()["frames"][0]
    assert fr["rows"] == 20000
    assert requests.get(cloud2 + "/3/Models/gbm_cancel").status_code == 404


def test_reads_and_queued_builds_during_a_build(cloud2):
    """While a 10k-tree GBM runs on the 2-rank cloud, frame / model /
    leaderboard / AutoML-event-log reads answer within 1 s each (served off
    the executor, collectives refused), and a second build is accepted at
    once as a CREATED job that runs after the first one."""
    _upload(cloud2, _data(3000, 4), "aml.hex")
    r = requests.post(cloud2 + "/99/AutoMLBuilder", json={
        "build_control": {"project_name": "aml_conc", "nfolds": 0, "stopping_criteria": {"max_models": 1, "seed": 1}},
        "input_spec": {"training_frame": "aml.hex", "response_column": "y", "ignored_columns": ["r"]},
        "build_models": {"include_algos": ["GLM"]}})
    assert r.status_code == 200, r.text
    assert _wait(cloud2, r.json()["job"])["status"] == "DONE"
    _upload(cloud2, _data(20000, 5), "long.hex")
    r = requests.post(cloud2 + "/3/ModelBuilders/gbm", json={"training_frame": "long.hex", "response_column": "y",
                                                              "ntrees": 10000, "max_depth": 5, "model_id": "gbm_long"})
    job = r.json()["job"]
    key = job["key"]["name"]
    t0 = time.time()
    while time.time() - t0 < 120:
        job = requests.get(cloud2 + f"/3/Jobs/{key}").json()["jobs"][0]
        if job["progress"] > 0:
            break
        time.sleep(0.05)
    assert job["status"] == "RUNNING"
    for path in ("/3/Frames", "/3/Frames/aml.hex", "/3/Models", "/99/Leaderboards/aml_conc", "/99/AutoML/aml_conc"):
        t1 = time.time()
        rr = requests.get(cloud2 + path, timeout=30)
        dt = time.time() - t1
        assert rr.status_code == 200, (path, rr.text[:300])
        assert dt < 1.0, (path, dt)
    assert any(f["frame_id"]["name"] == "long.hex" for f in requests.get(cloud2 + "/3/Frames").json()["frames"])
    ev = requests.get(cloud2 + "/99/AutoML/aml_conc").json()
    assert ev.get("event_log") is not None or ev.get("leaderboard") is not None
    # a second build while the first runs: CREATED at once, runs afterwards
    t1 = time.time()
    r2 = requests.post(cloud2 + "/3/ModelBuilders/glm", json={"training_frame": "aml.hex", "response_column": "r",
                                                               "model_id": "glm_queued", "ignored_columns": ["y"]},
                       timeout=30)
    assert time.time() - t1 < 1.0 and r2.status_code == 200, r2.text
    j2 = r2.json()["job"]
    assert j2["status"] == "CREATED"
    assert requests.get(cloud2 + f"/3/Jobs/{j2['key']['name']}").json()["jobs"][0]["status"] == "CREATED"
    assert requests.post(cloud2 + f"/3/Jobs/{key}/cancel").status_code == 200
    assert _wait(cloud2, job, timeout=60)["status"] == "CANCELLED"
    j2 = _wait(cloud2, j2, timeout=120)
    assert j2["status"] == "DONE", j2
    assert requests.get(cloud2 + "/3/Models/glm_queued").status_code == 200


@pytest.mark.skipif(not os.path.isdir("/root/reference/h2o-py/h2o") and not os.environ.get("H2O_PY_REFERENCE"),
                    reason="reference h2o-py client not present")
@pytest.mark.timeout(400)
def test_reference_python_client_on_two_ranks(cloud2):
    """tests/wire_client.py (the reference h2o-py client: upload, Rapids
    munging, GBM/GLM/K-Means/DRF/DL/XGBoost, predict, MOJO, grid, AutoML)
    against the 2-rank cloud, with the 1-rank assertions."""
    sys.path.insert(0, HERE)
    import test_rest_wire
    test_rest_wire.test_reference_python_client_end_to_end(cloud2)


@pytest.mark.skipif(not os.path.isdir("/root/reference/h2o-py/h2o") and not os.environ.get("H2O_PY_REFERENCE"),
                    reason="reference h2o-py client not present")
@pytest.mark.timeout(900)
def test_reference_python_client_munging_models_more_on_two_ranks(cloud2):
    """The munging (~47 H2OFrame ops), model-accessor and inspection /
    persistence clients of the reference h2o-py against the 2-rank cloud:
    every replayed command keeps the ranks' collective sequences and keys
    aligned (H2O3_TRACE_COLL diffs them when one does not)."""
    sys.path.insert(0, HERE)
    import test_rest_wire
    test_rest_wire.test_reference_python_client_munging(cloud2)
    test_rest_wire.test_reference_python_client_models(cloud2)
    test_rest_wire.test_reference_python_client_inspection_and_persistence(cloud2)


@pytest.mark.gpu
@pytest.mark.timeout(600)
def test_two_rank_gpu_cloud_over_rest():
    """Both ranks on the GPU (sharing the box's one device): the executor
    thread binds the rank's HIP device, a GBM built over REST equals the
    1-rank GPU model, and a long build cancels cleanly."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    df = _data(20000, 3)
    out = {}
    for world in (1, 2):
        url, procs = _launch(world, gpu=True)
        try:
            j = requests.get(url + "/3/Cloud").json()
            assert j["cloud_size"] == world
            _upload(url, df, "g.hex")
            g = _build(url, "gbm", {"training_frame": "g.hex", "response_column": "y", "ntrees": 10,
                                    "max_depth": 5, "seed": 3, "model_id": "gbm_gpu", "ignored_columns": ["r"]})
            out[world] = g["training_metrics"]["logloss"]
            if world == 2:
                r = requests.post(url + "/3/ModelBuilders/gbm", json={"training_frame": "g.hex",
                                                                      "response_column": "y", "ntrees": 100000,
                                                                      "model_id": "gbm_long"})
                job = r.json()["job"]
                t0 = time.time()
                while time.time() - t0 < 60:
                    job = requests.get(url + f"/3/Jobs/{job['key']['name']}").json()["jobs"][0]
                    if job["progress"] > 0:
                        break
                    time.sleep(0.05)
                requests.post(url + f"/3/Jobs/{job['key']['name']}/cancel")
                assert _wait(url, job, timeout=60)["status"] == "CANCELLED"
                assert requests.get(url + "/3/Frames/g.hex").json()["frames"][0]["rows"] == 20000
        finally:
            _stop(url, procs)
    assert abs(out[1] - out[2]) < 1e-5
