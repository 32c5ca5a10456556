"""Model persistence in the reference's layout (LanguageDetectorModel.scala:27-105),
incl. the reference's integration test (LanguageDetectionModelItSpecs.scala:15-47).
Host-only: the device table is built lazily, so no GPU is needed here."""
import json
import os

import numpy as np
import pyarrow.parquet as pq
import pytest

from languagedetection import LanguageDetectorModel


def test_reference_it_save_and_load(tmp_path):
    """LanguageDetectionModelItSpecs.scala:15-47: save a dummy model, the path
    exists, load it back (the reference never checks the loaded model; we do)."""
    path = str(tmp_path / "model")
    model = LanguageDetectorModel({"a".encode(): [1.0]}, [1], ["a"])
    model.write().save(path)
    assert os.path.exists(path)
    model2 = LanguageDetectorModel.load(path)
    assert model.gramLenghts == [1] and len(model.gramLenghts) == 1
    assert model2.gramProbabilities == {b"a": [1.0]}
    assert model2.gramLenghts == [1] and model2.supportedLanguages == ["a"]
    assert model2.uid == model.uid


def test_layout_matches_reference_schema(tmp_path):
    path = str(tmp_path / "m")
    table = {b"Die": [1.0, 0.0], "ö".encode("utf-8"): [0.25, -3.5], b"\xff\x00": [0.0, 1e-300]}
    m = LanguageDetectorModel(table, [3, 1, 3], ["de", "en"]).setOutputCol("label")
    m.save(path)
    meta = json.loads(open(os.path.join(path, "metadata", "part-00000")).readline())
    assert meta["class"] == "org.apache.spark.ml.feature.languagedetection.LanguageDetectorModel"
    assert meta["paramMap"] == {"inputCol": "fulltext", "outputCol": "label"}
    probs = pq.read_table(os.path.join(path, "probabilities"))
    assert str(probs.schema.field("_1").type.value_type) == "int8"      # array<tinyint>
    assert str(probs.schema.field("_2").type.value_type) == "double"    # array<double>
    assert [bytes(np.array(k, dtype=np.int8).view(np.uint8)) for k in probs.column("_1").to_pylist()] == list(table)
    assert pq.read_table(os.path.join(path, "supportedLanguages")).column("value").to_pylist() == ["de", "en"]
    assert pq.read_table(os.path.join(path, "gramLengths")).column("value").to_pylist() == [3, 1, 3]
    back = LanguageDetectorModel.load(path)
    assert back.gramProbabilities == table and back.getOutputCol() == "label"


def test_save_refuses_existing_path_without_overwrite(tmp_path):
    path = str(tmp_path / "m")
    m = LanguageDetectorModel({b"x": [1.0]}, [1], ["x"])
    m.save(path)
    with pytest.raises(IOError, match="already exists"):
        m.save(path)
    m.write().overwrite().save(path)


@pytest.mark.gpu
def test_saved_fitted_model_loads_and_scores_like_oracle(tmp_path):
    """Fit on the GPU, save in the reference layout, load back, score on the
    GPU: labels and fp64 scores equal the oracle's on the loaded table, and the
    table / languages / gram lengths survive the round trip exactly."""
    import ldoracle as O
    import pandas as pd
    from languagedetection import LanguageDetector, LanguageDetectorModel, synth
    ls = synth.make_languages(7, seed=61)
    tdata, toff, tlang = synth.generate(ls, 700, 100, 500, seed=62)
    df = pd.DataFrame({"lang": [ls.names[i] for i in tlang], "fulltext": synth.texts(tdata, toff)})
    model = LanguageDetector(ls.names, [1, 2, 3, 4], 150).fit(df)
    path = str(tmp_path / "model")
    model.write().overwrite().save(path)
    loaded = LanguageDetectorModel.load(path)
    assert loaded.supportedLanguages == ls.names and loaded.gramLenghts == [1, 2, 3, 4]
    assert loaded.gramProbabilities == model.gramProbabilities
    data, off, _ = synth.generate(ls, 400, 0, 300, seed=63)
    texts = synth.texts(data, off)
    labels, scores = loaded.predict_indices(texts, want_scores=True)
    for i, t in enumerate(texts):
        s = O.detect_scores(O.score_encode(t), loaded.gramProbabilities, 7, [1, 2, 3, 4])
        assert scores[i].tolist() == s
        assert int(labels[i]) == O.argmax_first(s)


def test_language_order_pinned_by_metadata(tmp_path):
    """SURVEY §3.4 hazard (LanguageDetectorModel.scala:82-87): a multi-part
    supportedLanguages dataset can come back permuted.  Our writer pins the
    order in the metadata's top-level languageOrder; the parquet schema stays
    the reference's single `value` column."""
    import pyarrow as pa
    from languagedetection.persistence import load_model_parts
    m = LanguageDetectorModel({"ab": [1.0, 0.0, 0.5]}, [2], ["de", "en", "fr"])
    path = str(tmp_path / "m")
    m.save(path)
    d = os.path.join(path, "supportedLanguages")
    assert pq.read_table(os.path.join(d, "part-00000.snappy.parquet")).column_names == ["value"]
    # re-split the dataset into two part files whose name order permutes the languages
    os.remove(os.path.join(d, "part-00000.snappy.parquet"))
    pq.write_table(pa.table({"value": ["fr"]}), os.path.join(d, "part-00000.snappy.parquet"))
    pq.write_table(pa.table({"value": ["de", "en"]}), os.path.join(d, "part-00001.snappy.parquet"))
    meta, table, langs, grams = load_model_parts(path)
    assert langs == ["de", "en", "fr"] and meta["languageOrder"] == langs
    # a model written without the pin (e.g. by the reference) keeps part order
    mp_ = os.path.join(path, "metadata", "part-00000")
    meta.pop("languageOrder")
    with open(mp_, "w") as f:
        f.write(json.dumps(meta) + "\n")
    assert load_model_parts(path)[2] == ["fr", "de", "en"]
    # a pin that names other languages is an error, not a silent relabelling
    meta["languageOrder"] = ["de", "en", "es"]
    with open(mp_, "w") as f:
        f.write(json.dumps(meta) + "\n")
    with pytest.raises(ValueError, match="languageOrder"):
        load_model_parts(path)
