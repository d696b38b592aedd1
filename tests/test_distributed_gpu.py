"""Two ranks sharing one GPU (gloo) grow the same trees as one rank.

Covers the multi-rank GPU tree path on the one-GPU test box: the
feature-sharded reduce-scatter of level histograms (GBM) and the
node-sharded pair path of DRF with mtries (reduce-scatter of pair
histograms by node, per-rank pair scoring and selection, all-gather of the
records).  Reference parity: the reference's multi-JVM runs build the same
model as one JVM (h2o-algos tests under a multi-node cloud).
"""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest
import torch

HERE = os.path.dirname(os.path.abspath(__file__))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(world, out):
    port = _free_port()
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), H2O3_DIST_BACKEND="gloo", H2O3_PAIR_DIRECT="1", OMP_NUM_THREADS="2")
        procs.append(subprocess.Popen([sys.executable, "-u", os.path.join(HERE, "dist_gpu_worker.py"), out], env=env,
                                      stdout=subprocess.PIPE, stderr=subprocess.STDOUT))
    outs = []
    for p in procs:
        try:
            o, _ = p.communicate(timeout=100)
        except subprocess.TimeoutExpired:
            p.kill()
            o, _ = p.communicate()
        outs.append(o.decode(errors="replace"))
    for p, o in zip(procs, outs):
        # the head holds the Python traceback / error line, the tail the exit
        assert p.returncode == 0, o[:6000] + "\n...\n" + o[-2000:]
    with open(out) as f:
        return json.load(f)


@pytest.mark.gpu
@pytest.mark.timeout(400)
def test_two_ranks_one_gpu_grow_same_trees(tmp_path):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    one = _run(1, str(tmp_path / "w1.json"))
    two = _run(2, str(tmp_path / "w2.json"))
    assert one["world"] == 1 and two["world"] == 2 and two["backend"] == "gloo"
    assert any("libtree_hist.so" in s for s in two["native"]) and any("libtree_split.so" in s for s in two["native"])
    # the device-resident tree ran in both clouds (stream-ordered collectives
    # at W = 2), the level loop where forced
    for w in (one, two):
        assert w["gbm3_devtree"] and w["gbm4_devtree"] and not w["gbm5_devtree"]
    ll = {k: (one[k + "_logloss"], two[k + "_logloss"]) for k in ("gbm3", "gbm4", "gbm5")}
    print("logloss (1 rank, 2 ranks):", ll)
    # without sampling the cloud size does not change the model
    assert abs(ll["gbm3"][0] - ll["gbm3"][1]) < 1e-5, ll
    # row sampling draws from a per-rank stream (like the reference's
    # per-chunk seeds, the sample depends on the row layout), so at each
    # cloud size the device tree must grow the level loop's trees
    for w in (one, two):
        assert abs(w["gbm4_logloss"] - w["gbm5_logloss"]) < 1e-6, ll
        for t4, t5 in zip(w["gbm4_trees"], w["gbm5_trees"]):
            assert t4["feat"] == t5["feat"] and t4["left"] == t5["left"]
            np.testing.assert_allclose(t4["thr"], t5["thr"], rtol=1e-6, atol=1e-9)
    for key in ("drf_trees", "drf2_trees", "gbm_trees", "gbm2_trees", "gbm3_trees"):
        assert len(one[key]) == len(two[key])
        for t1, t2 in zip(one[key], two[key]):
            assert t1["feat"] == t2["feat"], key
            assert t1["left"] == t2["left"], key
            np.testing.assert_allclose(t1["thr"], t2["thr"], rtol=1e-6, atol=1e-9)
    np.testing.assert_allclose(one["drf_pred"], two["drf_pred"], rtol=1e-5, atol=1e-5)
    assert abs(one["gbm_logloss"] - two["gbm_logloss"]) < 1e-5
    assert abs(one["gbm2_logloss"] - two["gbm2_logloss"]) < 1e-5
