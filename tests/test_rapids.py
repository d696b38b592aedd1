"""Rapids interpreter (water/rapids/Rapids.java grammar + prims) on CPU."""
import math

import pytest
from fastapi.testclient import TestClient

import h2o
import h2o3_amd
from h2o3_amd.core.rapids import RapidsError, parse


@pytest.fixture()
def fr():
    h2o3_amd.init(verbose=False)
    return h2o.H2OFrame({"a": [1.0, 2, 3, None, 5], "b": ["x", "y", "x", "z", "x"], "c": [0, 0, 1, 1, 0]},
                        destination_frame="rap1")


def test_parser_forms():
    assert parse("[0:3]") == ("numlist", [0.0, 1.0, 2.0])
    assert parse("[1 5:2:2]") == ("numlist", [1.0, 5.0, 7.0])
    assert parse("['a' \"b\"]") == ("strlist", ["a", "b"])
    with pytest.raises(RapidsError):
        parse("(+ 1 2")
    with pytest.raises(RapidsError):
        parse("[1:0]")


def test_scalar_math_and_scopes(fr):
    R = h2o.rapids
    assert R("(+ 1 2)") == 3.0
    assert R("(^ 2 10)") == 1024.0
    assert R("(%/% 7 2)") == 3.0
    assert R("(, (tmp= rq (* 2 3)) (+ rq 1))") == 7.0
    assert R("(ifelse (> 3 2) 'y' 'n')") == "y"
    assert math.isnan(R("(/ 0 0)"))


def test_frame_prims(fr):
    R = h2o.rapids
    assert math.isnan(R("(sum (cols rap1 [0]))"))
    assert R("(sumNA (cols rap1 [0]))") == 11.0
    assert R("(nrow rap1)") == 5.0 and R("(ncol rap1)") == 3.0
    assert R("(cols rap1 ['c' 'a'])").names == ["c", "a"]
    assert R("(cols rap1 [-2])").names == ["a", "c"]
    assert R("(rows rap1 (> (cols rap1 'c') 0))").nrows == 2
    g = R("(GB rap1 [1] 'mean' 0 'all' 'nrow' 0 'all')").as_data_frame()
    assert g["nrow"].tolist() == [3, 1, 1]
    ap = R("(apply (cols rap1 [0 2]) 2 {x . (sumNA x)})").as_data_frame()
    assert ap.iloc[0].tolist() == [11, 2]
    assert R("(toupper (cols rap1 'b'))").levels()[0] == ["X", "Y", "Z"]
    lv = R("(levels (cols rap1 'b'))")   # AstLevels: a categorical column of the domain
    assert lv.as_data_frame()["C1"].tolist() == ["x", "y", "z"]
    assert R("(sort rap1 [0] [0])").as_data_frame()["a"].tolist()[:3] == [5.0, 3.0, 2.0]
    assert R("(year (mktime 2021 5 3 0 0 0 0))").as_data_frame().iloc[0, 0] == 2021
    # a global frame is looked up as a defensive copy (Env.addGlobals): := and
    # colnames= change the result, the stored frame only through assign / tmp=
    assert R("(:= rap1 99 [0] [1])").as_data_frame()["a"].tolist()[1] == 99.0
    assert h2o.get_frame("rap1").as_data_frame()["a"].tolist()[1] != 99.0
    R("(assign rap1 (:= rap1 99 [0] [1]))")
    assert h2o.get_frame("rap1").as_data_frame()["a"].tolist()[1] == 99.0
    assert R("(colnames= rap1 [0] ['A'])").names[0] == "A" and h2o.get_frame("rap1").names[0] == "a"
    R("(tmp= rap1 (colnames= rap1 [0] ['A']))")
    assert h2o.get_frame("rap1").names[0] == "A"


def test_rest_rapids(fr):
    from h2o3_amd.server import create_app
    c = TestClient(create_app())
    r = c.post("/99/Rapids", json={"ast": "(tmp= rq2 (cols rap1 [0 2]))"}).json()
    assert r["key"]["name"] == "rq2" and r["num_cols"] == 2
    assert c.post("/99/Rapids", json={"ast": "(nrow rq2)"}).json()["scalar"] == 5.0
    assert c.post("/99/Rapids", json={"ast": "(nosuchprim 1)"}).status_code == 400
