import numpy as np
import pandas as pd
import pytest

import h2o3_amd as h2o


def _df():
    return pd.DataFrame({"a": [1.0, 2.0, np.nan, 4.0, 5.0, 6.0], "b": ["x", "y", "x", "z", None, "y"],
                         "c": [10, 20, 30, 40, 50, 60]})


def test_construct_types_and_rollups():
    fr = h2o.H2OFrame(_df())
    assert fr.shape == (6, 3)
    assert fr.types == {"a": "int", "b": "enum", "c": "int"}  # integral floats are "int" (as in H2O)
    assert fr["a"].mean() == pytest.approx(np.nanmean(_df()["a"]))
    assert fr.vec("a").nacnt() == 1
    assert fr["b"].levels()[0] == ["x", "y", "z"]
    assert fr.vec("b").nacnt() == 1


def test_indexing_and_ops():
    fr = h2o.H2OFrame(_df())
    sub = fr[fr["c"] > 25, :]
    assert sub.nrows == 4
    assert (fr["c"] * 2 + 1)[0, 0] == 21
    assert fr[1, "b"] == "y"
    fr["d"] = fr["c"] / 10
    assert fr.ncols == 4
    assert fr[fr["b"] == "x", "c"].as_data_frame()["c"].tolist() == [10, 30]
    assert fr[[0, 2], :].nrows == 2
    assert fr[:, ["a", "c"]].names == ["a", "c"]


def test_munging_group_by_merge_sort_split():
    fr = h2o.H2OFrame(_df())
    g = fr.group_by("b").sum("c").count().get_frame().as_data_frame()
    assert set(g.columns) >= {"b", "sum_c", "nrow"}
    srt = fr.sort("c", ascending=False)
    assert srt[0, "c"] == 60
    right = h2o.H2OFrame(pd.DataFrame({"b": ["x", "y"], "val": [1.5, 2.5]}))
    m = fr.merge(right)
    assert m.nrows == 4
    tr, te = fr.split_frame([0.5], seed=1)
    assert tr.nrows + te.nrows == 6
    q = fr["c"].quantile([0.5]).as_data_frame()
    assert q.iloc[0, 1] == pytest.approx(35.0)
    assert fr["c"].asfactor().types["c"] == "enum"
    assert fr.cbind(fr["a"]).ncols == 4
    assert fr.rbind(fr).nrows == 12


def test_csv_parse(tmp_path):
    p = tmp_path / "x.csv"
    p.write_text("id,name,score,when\n1,alpha,1.5,2020-01-02\n2,beta,NA,2021-03-04 10:11:12\n3,alpha,3.25,\n")
    fr = h2o.import_file(str(p))
    assert fr.names == ["id", "name", "score", "when"]
    assert fr.types["name"] == "enum" and fr.types["when"] == "time"
    assert fr.vec("score").nacnt() == 1
    assert fr["score"].max() == 3.25
    assert h2o.import_file(str(p), col_types={"id": "enum"}).types["id"] == "enum"


def test_strings_and_time():
    fr = h2o.H2OFrame(pd.DataFrame({"s": ["Ab", "cD", "Ab"]}))
    assert fr["s"].tolower().levels()[0] == ["ab", "cd"]
    t = h2o.H2OFrame(pd.DataFrame({"t": pd.to_datetime(["2020-05-17", "2021-12-31"])}))
    assert t["t"].year().as_data_frame()["t"].tolist() == [2020, 2021]


def test_uuid_column_guess(tmp_path):
    import uuid
    import h2o3_amd as h2o
    h2o.init()
    p = tmp_path / "u.csv"
    p.write_text("id,x\n" + "".join(f"{uuid.UUID(int=i * 7919 + 12345)},{i}\n" for i in range(50)))
    fr = h2o.import_file(str(p))
    assert fr.types["id"] == "uuid"
    assert fr["id"].as_data_frame().iloc[0, 0] == str(uuid.UUID(int=12345))


def test_fillna_forward_backward_both_axes():
    """AstFillNA: at most maxlen consecutive NAs filled, down columns or along rows."""
    import numpy as np
    import pandas as pd
    import h2o3_amd as h
    nan = float("nan")
    df = pd.DataFrame({"a": [1, nan, nan, nan, 5, nan], "b": [nan, 2, nan, 4, nan, nan],
                       "c": [nan, nan, 3, nan, nan, 6]})
    fr = h.H2OFrame(df)

    def same(got, want):
        np.testing.assert_array_equal(np.asarray(got, dtype=float), np.asarray(want, dtype=float))
    same(fr.fillna("forward", 0, 2).as_data_frame().values,
         [[1, nan, nan], [1, 2, nan], [1, 2, 3], [nan, 4, 3], [5, 4, 3], [5, 4, 6]])
    same(fr.fillna("backward", 0, 1).as_data_frame().values,
         [[1, 2, nan], [nan, 2, 3], [nan, 4, 3], [5, 4, nan], [5, nan, 6], [nan, nan, 6]])
    same(fr.fillna("forward", 1, 1).as_data_frame().values,
         [[1, 1, nan], [nan, 2, 2], [nan, nan, 3], [nan, 4, 4], [5, 5, nan], [nan, nan, 6]])
    same(fr.fillna("backward", 1, 5).as_data_frame().values,
         [[1, nan, nan], [2, 2, nan], [3, 3, 3], [4, 4, nan], [5, nan, nan], [6, 6, 6]])


@pytest.mark.parametrize("how", ["inner", "left", "right"])
def test_merge_sort_join_matches_pandas(how):
    """Device sort-join vs pandas on the same keys (categorical keys with
    different domains on each side, a numeric second key, duplicates on both
    sides, NA keys that never match -- Merge.java drops NA-key right rows)."""
    import numpy as np
    import pandas as pd
    import h2o3_amd as h
    rng = np.random.default_rng(7)
    n, m = 300, 80
    lx = pd.DataFrame({"k": rng.choice(["a", "b", "c", "d", None], n), "j": rng.integers(0, 3, n).astype(float),
                       "v": rng.normal(size=n)})
    ry = pd.DataFrame({"k": rng.choice(["b", "c", "d", "e", None], m), "j": rng.integers(0, 3, m).astype(float),
                       "w": rng.normal(size=m)})
    lx.loc[::17, "j"] = np.nan
    fx, fy = h.H2OFrame(lx), h.H2OFrame(ry)
    got = fx.merge(fy, all_x=how == "left", all_y=how == "right").as_data_frame()
    ref = lx.dropna(subset=["k", "j"]) if how == "inner" else lx
    refy = ry.dropna(subset=["k", "j"])
    if how == "inner":
        want = ref.merge(refy, on=["k", "j"], how="inner", sort=True)
    elif how == "left":
        want = lx.assign(_na=lx[["k", "j"]].isna().any(axis=1))
        a = want[~want._na].merge(refy, on=["k", "j"], how="left", sort=True)
        b = want[want._na].assign(w=np.nan)
        want = pd.concat([a, b]).drop(columns="_na")
    else:
        # all_y = a left join from the right frame's side (AstMerge swaps the frames):
        # its NA-key rows are kept unmatched, the left frame's NA-key rows dropped
        want = lx.dropna(subset=["k", "j"]).merge(ry, on=["k", "j"], how="right")
    cols = ["k", "j", "v", "w"]
    g = got[cols].reset_index(drop=True)
    w = want[cols].reset_index(drop=True)
    assert len(g) == len(w)
    if how == "right":
        key = lambda d: d.fillna(-999).sort_values(cols).reset_index(drop=True)   # noqa: E731
        pd.testing.assert_frame_equal(key(g), key(w), check_dtype=False, atol=1e-6)
    else:
        pd.testing.assert_frame_equal(g.fillna(-999), w.fillna(-999), check_dtype=False, atol=1e-6)


def test_cor_use_modes():
    """AstCorrelation use=: everything propagates NAs, complete.obs drops NA rows,
    all.obs rejects them; na_rm=True means complete.obs."""
    import numpy as np
    import pandas as pd
    import h2o3_amd as h
    df = pd.DataFrame({"a": [1, 2, np.nan, 4, 5.0], "b": [2, 1, 3, 5, 4.0], "c": [1, 3, 2, 5, 4.0]})
    fr = h.H2OFrame(df)
    assert np.isnan(fr.cor().as_data_frame().iloc[0, 1])
    got = fr.cor(na_rm=True).as_data_frame().values
    np.testing.assert_allclose(got, df.dropna().corr().values, rtol=1e-6)
    with pytest.raises(ValueError):
        fr.cor(use="all.obs")
    assert abs(fr["b"].cor(fr["c"]) - df.b.corr(df.c)) < 1e-9
