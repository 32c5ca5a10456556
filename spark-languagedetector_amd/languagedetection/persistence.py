"""Model persistence in the reference's on-disk layout (SURVEY.md §8f "next" #2).

LanguageDetectorModelWriter.saveImpl (LanguageDetectorModel.scala:30-59) writes
  path/metadata/part-00000        DefaultParamsWriter.saveMetadata: one JSON line
                                  {class, timestamp, sparkVersion, uid, paramMap}
  path/probabilities/*.parquet    Dataset[(Seq[Byte], Array[Double])]:
                                  _1 array<tinyint> (signed bytes), _2 array<double>
  path/supportedLanguages/*.parquet  Dataset[String]: column `value`
  path/gramLengths/*.parquet      Dataset[Int]: column `value`
and LanguageDetectorModelReader.load (:68-104) reads them back.

The reference collects supportedLanguages without an ordering key (:82-87);
with several part files Spark may return them permuted relative to the
probability rows.  The writer therefore pins the order explicitly: the
metadata JSON carries a top-level "languageOrder" list (DefaultParamsWriter's
extraMetadata slot: the reference's reader, DefaultParamsReader.loadMetadata,
ignores unknown top-level fields, and the parquet datasets keep exactly the
reference's schema, so a reference Spark job can still read the model).  The
reader uses it when present (after checking it names the same languages as
the parquet dataset) and otherwise reads part files in name order, the order
Spark lists them in.
"""
from __future__ import annotations

import glob
import json
import os
import shutil
import time
from typing import Dict, List, Tuple

import numpy as np

MODEL_CLASS = "org.apache.spark.ml.feature.languagedetection.LanguageDetectorModel"
SPARK_VERSION = "2.2.0"


def _write_parquet(dirpath: str, table) -> None:
    import pyarrow.parquet as pq
    os.makedirs(dirpath, exist_ok=True)
    pq.write_table(table, os.path.join(dirpath, "part-00000.snappy.parquet"), compression="snappy")
    open(os.path.join(dirpath, "_SUCCESS"), "w").close()


def _read_parquet_dir(dirpath: str):
    import pyarrow as pa
    import pyarrow.parquet as pq
    parts = sorted(p for p in glob.glob(os.path.join(dirpath, "*.parquet")))
    if not parts:
        raise FileNotFoundError(f"no parquet part files under {dirpath}")
    return pa.concat_tables([pq.read_table(p) for p in parts])


def save_model(model, path: str, overwrite: bool = True) -> None:
    """MLWriter.save(path) for LanguageDetectorModel (:30-59)."""
    import pyarrow as pa
    if os.path.exists(path):
        if not overwrite:
            raise IOError(f"Path {path} already exists. To overwrite it, please use write.overwrite().save(path)")
        shutil.rmtree(path)
    meta = {"class": MODEL_CLASS, "timestamp": int(time.time() * 1000), "sparkVersion": SPARK_VERSION,
            "uid": model.uid, "paramMap": model.extractParamMap(),
            "languageOrder": list(model.supportedLanguages)}
    os.makedirs(os.path.join(path, "metadata"), exist_ok=True)
    with open(os.path.join(path, "metadata", "part-00000"), "w") as f:
        f.write(json.dumps(meta, separators=(",", ":")) + "\n")
    open(os.path.join(path, "metadata", "_SUCCESS"), "w").close()

    keys = [np.frombuffer(k, dtype=np.int8).tolist() for k in model.gramProbabilities]
    rows = [list(map(float, v)) for v in model.gramProbabilities.values()]
    _write_parquet(os.path.join(path, "probabilities"),
                   pa.table({"_1": pa.array(keys, type=pa.list_(pa.int8())),
                             "_2": pa.array(rows, type=pa.list_(pa.float64()))}))
    _write_parquet(os.path.join(path, "supportedLanguages"),
                   pa.table({"value": pa.array(list(model.supportedLanguages), type=pa.string())}))
    _write_parquet(os.path.join(path, "gramLengths"),
                   pa.table({"value": pa.array(list(model.gramLenghts), type=pa.int32())}))


def load_model_parts(path: str) -> Tuple[dict, Dict[bytes, List[float]], List[str], List[int]]:
    """LanguageDetectorModelReader.load (:68-104): metadata, map, languages, gram lengths."""
    with open(sorted(glob.glob(os.path.join(path, "metadata", "part-*")))[0]) as f:
        meta = json.loads(f.readline())
    if meta.get("class") != MODEL_CLASS:
        raise ValueError(f"Error loading metadata: Expected class name {MODEL_CLASS} but found class name "
                         f"{meta.get('class')}")
    probs = _read_parquet_dir(os.path.join(path, "probabilities"))
    table: Dict[bytes, List[float]] = {}
    for k, v in zip(probs.column("_1").to_pylist(), probs.column("_2").to_pylist()):
        table[bytes((int(x) & 0xFF) for x in k)] = list(v)   # .toMap: a later duplicate wins
    langs = [str(x) for x in _read_parquet_dir(os.path.join(path, "supportedLanguages")).column("value").to_pylist()]
    order = meta.get("languageOrder")
    if order is not None:
        if sorted(map(str, order)) != sorted(langs):
            raise ValueError(f"metadata languageOrder {order} does not match the supportedLanguages dataset {langs}")
        langs = [str(x) for x in order]
    grams = [int(x) for x in _read_parquet_dir(os.path.join(path, "gramLengths")).column("value").to_pylist()]
    return meta, table, langs, grams
