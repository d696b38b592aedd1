"""Avro import (h2o-parsers/h2o-avro-parser parity) through the built-in
object-container reader: null and deflate codecs, unions with null, enums."""
import math

import numpy as np
import pytest

import h2o3_amd as h2o
from h2o3_amd.core.avro import read_avro, write_avro

SCHEMA = {"type": "record", "name": "R", "fields": [
    {"name": "i", "type": "int"}, {"name": "l", "type": ["null", "long"]}, {"name": "d", "type": "double"},
    {"name": "f", "type": "float"}, {"name": "b", "type": "boolean"}, {"name": "s", "type": ["string", "null"]},
    {"name": "e", "type": {"type": "enum", "name": "Color", "symbols": ["red", "green", "blue"]}},
    {"name": "arr", "type": {"type": "array", "items": "int"}}]}


def _records(n=2500):
    rng = np.random.RandomState(0)
    out = []
    for k in range(n):
        out.append({"i": int(k - 1000), "l": None if k % 7 == 0 else int(k) * 10 ** 10, "d": float(rng.randn()),
                    "f": float(np.float32(k / 4)), "b": bool(k % 2), "s": None if k % 11 == 0 else f"s{k % 5}",
                    "e": ["red", "green", "blue"][k % 3], "arr": [1, 2, 3]})
    return out


@pytest.mark.parametrize("codec", ["null", "deflate"])
def test_avro_roundtrip_and_import(tmp_path, codec):
    h2o.init(verbose=False)
    recs = _records()
    p = write_avro(str(tmp_path / f"t_{codec}.avro"), SCHEMA, recs, codec=codec, block_size=700)
    schema, rows = read_avro(p)
    assert rows[5] == recs[5] and len(rows) == len(recs)
    fr = h2o.import_file(p)
    assert fr.names == ["i", "l", "d", "f", "b", "s", "e"]      # the array field is not flat: skipped
    assert fr.nrows == 2500
    df = fr.as_data_frame()
    assert df["i"].iloc[3] == -997
    assert math.isnan(df["l"].iloc[0]) and df["l"].iloc[1] == 1e10
    assert fr.types["e"] == "enum" and fr["e"].levels()[0] == ["red", "green", "blue"]
    assert df["b"].sum() == 1250
    assert df["s"].isna().sum() == len([k for k in range(2500) if k % 11 == 0])
