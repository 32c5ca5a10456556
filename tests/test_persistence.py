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
