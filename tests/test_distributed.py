"""Multi-process (gloo, CPU) runs must reproduce the single-process models.

Reference: the reference's multi-node tests (h2o-core/src/test MRTask /
cloud tests run with 1..N JVMs) — here the SPMD row-sharded path with
torch.distributed collectives (all_reduce / reduce_scatter / all_gather).
"""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run_ranks(world, out):
    port = _free_port()
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), LOCAL_RANK=str(r), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), CUDA_VISIBLE_DEVICES="", OMP_NUM_THREADS="2")
        procs.append(subprocess.Popen([sys.executable, os.path.join(HERE, "dist_worker.py"), out], env=env,
                                      stdout=subprocess.PIPE, stderr=subprocess.STDOUT))
    outs = []
    for p in procs:
        try:
            o, _ = p.communicate(timeout=600)
        except subprocess.TimeoutExpired:
            p.kill()
            o, _ = p.communicate()
        outs.append(o.decode(errors="replace"))
    for p, o in zip(procs, outs):
        assert p.returncode == 0, o[-3000:]
    with open(out) as f:
        return json.load(f)


@pytest.fixture(scope="module")
def results(tmp_path_factory):
    d = tmp_path_factory.mktemp("dist")
    one = _run_ranks(1, str(d / "w1.json"))
    two = _run_ranks(2, str(d / "w2.json"))
    return one, two


@pytest.mark.parametrize("op", ["quantile", "quantile_w", "table1", "table2", "table_sparse", "unique", "hist", "cor",
                                "spearman", "dedup", "pivot", "melt", "rank", "inter", "gb_med_mode", "sort_dups",
                                "topn", "bottomn", "impute_mean", "impute_median", "impute_mode", "apply_num",
                                "apply_str", "fill_fwd", "fill_bwd", "distance"])
def test_dist_ops_match_one_rank(results, op):
    """Quantile / table / unique / hist / cor / pivot / melt / rank-within-group /
    interaction / drop_duplicates / median-mode / sort computed shard-locally
    on 2 ranks equal the one-rank results (no frame gathers on either)."""
    one, two = results
    assert one["dist_ops"][op] == two["dist_ops"][op]


def test_drf_pair_exchange_same_trees(results):
    """DRF on the pair path (mtries 6 of 44 features, 4 categoricals of
    cardinality 60): identical trees at 1 and 2 ranks with the packed /
    sparse pair exchange; the deep levels took the sparse all_to_all."""
    one, two = results
    assert one["drf_pairs"]["trees"] == two["drf_pairs"]["trees"]
    assert one["drf_pairs"]["rmse"] == two["drf_pairs"]["rmse"]
    assert two["drf_pairs"]["a2a_levels"], "no level used the sparse exchange"
    # classification (whole-number histograms: the int32 transport)
    assert one["drf_pairs"]["trees_c"] == two["drf_pairs"]["trees_c"]
    assert one["drf_pairs"]["logloss_c"] == two["drf_pairs"]["logloss_c"]


def test_persist_sharded_state(results):
    """save_model / load_model of models with row-sharded state (CV holdout
    predictions, GLRM X) on 2 ranks: the archive holds all rows, each loaded
    rank holds its shard, and the values equal the saved ones."""
    one, two = results
    for r in (one, two):
        p = r["persist"]
        assert p["cv_holdout_equal"] and p["cv_holdout_local_rows_ok"] and p["glrm_x_equal"], p
        assert p["cv_pred_rows"] == 4000 and p["glrm_x_rows"] == 4000, p
    assert abs(one["persist"]["cv_holdout_sum"] - two["persist"]["cv_holdout_sum"]) < 1e-6


def test_rows_sharded(results):
    one, two = results
    assert one["nrow"] == two["nrow"] == 4000


def test_gbm_matches_single_process(results):
    one, two = results
    assert abs(one["gbm_auc"] - two["gbm_auc"]) < 1e-5
    assert abs(one["gbm_logloss"] - two["gbm_logloss"]) < 1e-5
    assert abs(one["gbm_ua_logloss"] - two["gbm_ua_logloss"]) < 1e-5


def test_metrics_from_merged_sketches_match_single_process(results):
    """Binomial metrics at W > 1 come from the merged logit histogram (AUC2's
    role), multinomial ones from sums + the [K, K, bins] AUC sketch: no rows
    gathered, and the values equal the single-process ones."""
    one, two = results
    a, b = one["multi"], two["multi"]
    assert abs(a["logloss"] - b["logloss"]) < 1e-6
    assert a["cm"] == b["cm"] and np.allclose(a["hr"], b["hr"], atol=1e-12)
    assert abs(a["auc"] - b["auc"]) < 1e-9 and abs(a["wovr"] - b["wovr"]) < 1e-9 and a["auc"] > 0.8
    assert abs(a["aucpr"] - b["aucpr"]) < 1e-9
    assert abs(one["bin_prauc"] - two["bin_prauc"]) < 2e-3
    assert 50 < two["bin_tab_rows"] <= 400


def test_glm_matches_single_process(results):
    one, two = results
    for k, v in one["glm_coef"].items():
        assert abs(v - two["glm_coef"][k]) < 1e-6 * max(1, abs(v)), k
    for k, v in one["glmr_coef"].items():
        assert abs(v - two["glmr_coef"][k]) < 1e-6 * max(1, abs(v)), k


def test_drf_and_kmeans_close(results):
    one, two = results
    # DRF row sampling / kmeans++ seeding are rank-local streams: same quality, not bitwise
    assert abs(one["drf_rmse"] - two["drf_rmse"]) < 0.1 * one["drf_rmse"]
    assert abs(one["km_tot_withinss"] - two["km_tot_withinss"]) < 0.05 * one["km_tot_withinss"]


def test_deeplearning_model_averaging(results):
    """DeepLearningTask model averaging at W=2: one all-reduce per iteration,
    identical models on every rank, and a useful model for every mode."""
    for res in results:
        for tag, d in res["dl"].items():
            assert d["same"], tag
            assert d["auc"] > 0.8, (tag, d["auc"])


def test_munging_without_gathers_matches_single_process(results):
    """dist_munge: sort by range exchange, group-by by reduced partials,
    merge by range-partitioned local joins -- identical rows in identical
    order to the one-rank run."""
    one, two = results
    for k in ("mung_sort", "mung_gb", "mung_merge_inner", "mung_merge_left", "mung_merge_right"):
        assert one[k] == two[k], k


def test_failed_rank_exits_fast():
    """A rank that dies on an exception exits without an exit-time barrier,
    and its peer's pending collective fails on the broken connection instead
    of waiting out the 30-minute collective timeout."""
    import time
    port = _free_port()
    procs = []
    t0 = time.time()
    for r in range(2):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE="2", LOCAL_RANK=str(r), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), CUDA_VISIBLE_DEVICES="", OMP_NUM_THREADS="1")
        procs.append(subprocess.Popen([sys.executable, os.path.join(HERE, "dist_fail_worker.py")], env=env,
                                      stdout=subprocess.PIPE, stderr=subprocess.STDOUT))
    outs = []
    for p in procs:
        try:
            o, _ = p.communicate(timeout=240)
        except subprocess.TimeoutExpired:
            p.kill()
            o, _ = p.communicate()
            outs.append(None)
            continue
        outs.append(o.decode(errors="replace"))
    assert all(o is not None for o in outs), "a rank hung after its peer failed"
    assert procs[1].returncode != 0 and "simulated failure" in outs[1]
    assert procs[0].returncode != 0 and "unexpected" not in outs[0]
    assert time.time() - t0 < 200


def test_heartbeat_reports_hung_rank():
    """A frozen rank (SIGSTOP: its connections stay open, so the collective
    never errors) is named by the survivor's heartbeat within the suspect
    window, and the survivor leaves its pending collective with status 3
    instead of waiting out the 1800 s collective timeout
    (water/HeartBeatThread.java TIMEOUT)."""
    import signal
    import time
    port = _free_port()
    procs = []
    t0 = time.time()
    for r in range(2):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE="2", LOCAL_RANK=str(r), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), CUDA_VISIBLE_DEVICES="", OMP_NUM_THREADS="1", H2O3_HB_INTERVAL="1",
                   H2O3_HB_SUSPECT="8")
        procs.append(subprocess.Popen([sys.executable, os.path.join(HERE, "dist_hang_worker.py")], env=env,
                                      stdout=subprocess.PIPE, stderr=subprocess.STDOUT))
    try:
        o0, _ = procs[0].communicate(timeout=90)
    finally:
        for p in procs:
            if p.poll() is None:
                p.send_signal(signal.SIGKILL)
                p.wait()
    out = o0.decode(errors="replace")
    assert procs[0].returncode == 3, out[-2000:]
    assert "rank(s) [1] missed heartbeats" in out, out[-2000:]
    assert "unexpected" not in out
    assert time.time() - t0 < 90
