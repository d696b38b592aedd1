"""Word2Vec skip-gram/HSM learns co-occurrence structure."""
import numpy as np
import pandas as pd

import h2o3_amd as h2o
from h2o3_amd.estimators import H2OWord2vecEstimator
from h2o3_amd.models.word2vec import _huffman


def test_huffman_prefix_free():
    codes, points = _huffman([50, 30, 10, 5, 5])
    s = ["".join(map(str, c)) for c in codes]
    for i, a in enumerate(s):
        for j, b in enumerate(s):
            if i != j:
                assert not b.startswith(a)
    assert len(codes[0]) <= len(codes[-1])


def test_word2vec_synonyms_and_transform():
    h2o.init()
    rng = np.random.default_rng(0)
    groups = [["cat", "dog", "mouse", "horse"], ["red", "green", "blue", "yellow"], ["one", "two", "three", "four"]]
    toks = []
    for _ in range(1500):
        g = groups[rng.integers(3)]
        toks += list(rng.choice(g, 5)) + [None]
    fr = h2o.H2OFrame(pd.DataFrame({"w": toks}), column_types=["string"])
    m = H2OWord2vecEstimator(vec_size=16, window_size=3, epochs=10, min_word_freq=5, seed=1, sent_sample_rate=0.0,
                             init_learning_rate=0.05)
    m.train(training_frame=fr)
    syn = m.find_synonyms("cat", 3)
    assert set(syn) <= {"dog", "mouse", "horse"}, syn
    syn = m.find_synonyms("red", 3)
    assert set(syn) <= {"green", "blue", "yellow"}, syn
    t = m.transform(h2o.H2OFrame(pd.DataFrame({"w": ["cat", "dog", None, "red", "zzz"]}), column_types=["string"]),
                    aggregate_method="AVERAGE")
    assert t.nrow == 2 and t.ncol == 16
    wf = m.to_frame()
    assert wf.nrow == 12 and wf.ncol == 17


def test_word2vec_cbow_and_model_checks():
    """word_model=CBOW (WordVectorTrainer.CBOW): window mean -> centre word."""
    import pytest
    h2o.init()
    rng = np.random.default_rng(1)
    groups = [["cat", "dog", "mouse", "horse"], ["red", "green", "blue", "yellow"], ["one", "two", "three", "four"]]
    toks = []
    for _ in range(1500):
        g = groups[rng.integers(3)]
        toks += list(rng.choice(g, 5)) + [None]
    fr = h2o.H2OFrame(pd.DataFrame({"w": toks}), column_types=["string"])
    kw = dict(vec_size=16, window_size=3, epochs=10, min_word_freq=5, seed=1, sent_sample_rate=0.0,
              init_learning_rate=0.05)
    cb = H2OWord2vecEstimator(word_model="CBOW", **kw)
    cb.train(training_frame=fr)
    assert set(cb.find_synonyms("cat", 3)) <= {"dog", "mouse", "horse"}
    sg = H2OWord2vecEstimator(**kw)
    sg.train(training_frame=fr)
    a = cb.to_frame().as_data_frame().iloc[:, 1:].values
    b = sg.to_frame().as_data_frame().iloc[:, 1:].values
    assert not np.allclose(a, b)
    with pytest.raises(ValueError, match="word_model"):
        H2OWord2vecEstimator(word_model="glove", **kw).train(training_frame=fr)
