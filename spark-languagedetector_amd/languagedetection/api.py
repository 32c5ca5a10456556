"""Host mirror of the reference's Spark ML surface, over pandas DataFrames.

Reference (org.apache.spark.ml.feature.languagedetection):
  class LanguageDetector(uid, supportedLanguages, gramLengths, languageProfileSize)
      LanguageDetector.scala:176-264  (Estimator; params inputCol="fulltext",
      labelCol="lang", saveGramsToHDFS=None; fit)
  object LanguageDetector.computeGramProbabilities   LanguageDetector.scala:145-165
  class LanguageDetectorModel(uid, gramProbabilities, gramLenghts, supportedLanguages)
      LanguageDetectorModel.scala:178-242  (Model; params inputCol="fulltext",
      outputCol="lang"; transformSchema; transform)
  object LanguageDetectorModel.detect(String | Array[Byte], map, langs, grams)
      LanguageDetectorModel.scala:131-165

Names, argument meaning, defaults and error behaviour follow the reference
(including the ``gramLenghts`` field name and the "contians" typo of the fit
validation message).  The arithmetic runs on the GPU through libldgpu.so;
there is no CPU fallback.
"""
from __future__ import annotations

import threading
import uuid
from collections.abc import Mapping
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

from . import encoding
from .runtime import DeviceCounts, DeviceModel


class NullPointerException(Exception):
    """A null text, as the JVM raises in detect/computeGrams."""


def _random_uid(prefix: str) -> str:
    return f"{prefix}_{uuid.uuid4().hex[:12]}"


class _Params:
    _defaults: Dict[str, object] = {}

    def __init__(self):
        self._values: Dict[str, object] = {}

    def _set(self, name: str, value):
        self._values[name] = value
        return self

    def getOrDefault(self, name: str):
        return self._values.get(name, self._defaults[name])

    def extractParamMap(self) -> Dict[str, object]:
        return {**self._defaults, **self._values}


def _rows_of(dataset, *cols: str):
    """Columns of a pandas DataFrame (or a mapping of column -> sequence)."""
    missing = [c for c in cols if c not in dataset]
    if missing:
        raise ValueError(f"Field \"{missing[0]}\" does not exist.")
    return [list(dataset[c]) for c in cols]


# ----------------------------------------------------------------------- SCORE
class LanguageDetectorModel(_Params):
    """LanguageDetectorModel (LanguageDetectorModel.scala:178-242)."""

    _defaults = {"inputCol": "fulltext", "outputCol": "lang"}

    def __init__(self, gramProbabilities: Dict, gramLengths: Sequence[int], languages: Sequence[str],
                 uid: Optional[str] = None, device: Optional[int] = None):
        super().__init__()
        self.uid = uid or _random_uid("LanguageDetectorModel")
        self.gramProbabilities = {encoding.gram_key(k): list(v) for k, v in gramProbabilities.items()}
        self.gramLenghts = list(gramLengths)       # field name as in the reference (:180)
        self.supportedLanguages = list(languages)
        self._device = device
        self._dev: Optional[DeviceModel] = None

    # params
    def setInputCol(self, value: str):
        return self._set("inputCol", value)

    def setOutputCol(self, value: str):
        return self._set("outputCol", value)

    def getInputCol(self) -> str:
        return self.getOrDefault("inputCol")

    def getOutputCol(self) -> str:
        return self.getOrDefault("outputCol")

    # the device table is built on first use, as the reference broadcasts the
    # map at transform time (:222); errors of the map surface there too
    def device_model(self) -> DeviceModel:
        if self._dev is None:
            self._dev = DeviceModel(self.gramProbabilities, len(self.supportedLanguages), self.gramLenghts,
                                    device=self._device)
        return self._dev

    def transformSchema(self, schema: Dict[str, str]) -> Dict[str, str]:
        """schema: column name -> type name ("string", ...) (:206-210)."""
        in_type = schema.get(self.getInputCol())
        if in_type is None:
            raise ValueError(f"Field \"{self.getInputCol()}\" does not exist.")
        if in_type != "string":
            raise ValueError(f"requirement failed: Input type must be StringType but got {in_type}.")
        if self.getOutputCol() in schema:
            raise ValueError(f"requirement failed: Column {self.getOutputCol()} already exists.")
        return {**schema, self.getOutputCol(): "string"}

    @staticmethod
    def _schema_of(df) -> Dict[str, str]:
        out = {}
        for c in df.columns:
            vals = [v for v in df[c] if v is not None]
            out[c] = "string" if all(isinstance(v, str) for v in vals) else str(df[c].dtype)
        return out

    def predict_indices(self, texts: Sequence[str], want_scores: bool = False
                        ) -> Tuple[np.ndarray, Optional[np.ndarray]]:
        for t in texts:
            if t is None:
                raise NullPointerException("text is null")
        data, offsets = encoding.pack_score(texts)
        return self.device_model().score(data, offsets, want_scores)

    def transform(self, dataset):
        """Append outputCol = detected language for every row (:219-240)."""
        import pandas as pd
        df = dataset if isinstance(dataset, pd.DataFrame) else pd.DataFrame(dataset)
        self.transformSchema(self._schema_of(df))
        labels, _ = self.predict_indices(list(df[self.getInputCol()]))
        out = df.copy()
        out[self.getOutputCol()] = [self.supportedLanguages[i] for i in labels]
        return out

    # persistence (LanguageDetectorModel.scala:24-105): the reference's layout
    def write(self) -> "LanguageDetectorModelWriter":
        return LanguageDetectorModelWriter(self)

    def save(self, path: str) -> None:
        self.write().save(path)

    @classmethod
    def read(cls) -> "LanguageDetectorModelReader":
        return LanguageDetectorModelReader()

    @classmethod
    def load(cls, path: str) -> "LanguageDetectorModel":
        return cls.read().load(path)

    @staticmethod
    def detect(text, probabilityMap: Dict, supportedLanguages: Sequence[str], gramLengths: Sequence[int]) -> str:
        """detect(String | Array[Byte], ...) (:131-165); a str is encoded by the
        low byte of each UTF-16 unit, bytes are used as they are."""
        if text is None:
            raise NullPointerException("text is null")
        raw = text if isinstance(text, (bytes, bytearray)) else encoding.score_bytes(text)
        m = _detect_model(probabilityMap, len(supportedLanguages), gramLengths)
        data, offsets = encoding.pack([bytes(raw)])
        labels, _ = m.score(data, offsets)
        return supportedLanguages[int(labels[0])]


class FrozenTable(Mapping):
    """An immutable gram -> probability-row map (keys bytes, rows tuples of
    floats).  detect() reuses its device table by identity alone; any other
    mapping is compared with a snapshot of its contents on every call."""

    __slots__ = ("_d",)

    def __init__(self, table):
        self._d = {encoding.gram_key(k): tuple(float(x) for x in v) for k, v in table.items()}

    def __getitem__(self, k):
        return self._d[k]

    def __iter__(self):
        return iter(self._d)

    def __len__(self):
        return len(self._d)


def freeze_table(table) -> FrozenTable:
    """The table as a FrozenTable: detect() over it skips the content check."""
    return table if isinstance(table, FrozenTable) else FrozenTable(table)


# The device tables of recent detect() calls (the Scala drop-in's
# detectAcquire): callers score row after row with the same map, so its
# table is kept.  The reference builds its lookups from the map on every
# call, so a cached table may serve a call only if the map's contents are
# those it was built from: a FrozenTable cannot change, and any other mapping
# (a dict and its value lists can be edited in place) is compared with a copy
# of its contents taken at build time (one C-level dict compare, ~0.7 ms for
# 10k rows of 20 values); a mapping whose values cannot be compared that way
# (e.g. numpy rows) is never cached.
_DETECT_CACHE: list = []
_DETECT_CACHE_SIZE = 4


_DETECT_LOCK = threading.Lock()


def _snapshot(probabilityMap):
    """A copy of the map's contents to compare later calls with, or None."""
    if isinstance(probabilityMap, FrozenTable):
        return probabilityMap
    if not all(isinstance(v, (list, tuple)) for v in probabilityMap.values()):
        return None
    return {k: (list(v) if isinstance(v, list) else v) for k, v in probabilityMap.items()}


def _unchanged(probabilityMap, snap) -> bool:
    if isinstance(probabilityMap, FrozenTable):
        return snap is probabilityMap
    try:
        return type(probabilityMap) is dict and probabilityMap == snap
    except (TypeError, ValueError):
        return False


def _detect_model(probabilityMap, n_langs: int, gramLengths):
    key = (id(probabilityMap), n_langs, tuple(gramLengths))
    with _DETECT_LOCK:
        for i, (k, ref, snap, m) in enumerate(_DETECT_CACHE):
            if k == key and ref is probabilityMap and _unchanged(probabilityMap, snap):
                _DETECT_CACHE.insert(0, _DETECT_CACHE.pop(i))
                return m
    snap = _snapshot(probabilityMap)
    m = DeviceModel({encoding.gram_key(k): v for k, v in probabilityMap.items()}, n_langs, gramLengths)
    if snap is not None:
        with _DETECT_LOCK:
            # (a stale entry of the same map object is replaced; an evicted
            # table is released when its last caller drops it)
            _DETECT_CACHE[:] = [e for e in _DETECT_CACHE if e[0] != key]
            _DETECT_CACHE.insert(0, (key, probabilityMap, snap, m))
            del _DETECT_CACHE[_DETECT_CACHE_SIZE:]
    return m


class LanguageDetectorModelWriter:
    """LanguageDetectorModelWriter (LanguageDetectorModel.scala:27-60) with
    MLWriter's save/overwrite behaviour."""

    def __init__(self, instance: LanguageDetectorModel):
        self.instance = instance
        self._overwrite = False

    def overwrite(self) -> "LanguageDetectorModelWriter":
        self._overwrite = True
        return self

    def save(self, path: str) -> None:
        from .persistence import save_model
        save_model(self.instance, path, overwrite=self._overwrite)


class LanguageDetectorModelReader:
    """LanguageDetectorModelReader (LanguageDetectorModel.scala:62-105)."""

    def load(self, path: str) -> LanguageDetectorModel:
        from .persistence import load_model_parts
        meta, table, langs, grams = load_model_parts(path)
        m = LanguageDetectorModel(table, grams, langs, uid=meta.get("uid"))
        for k, v in (meta.get("paramMap") or {}).items():   # DefaultParamsReader.getAndSetParams
            if k in m._defaults:
                m._set(k, v)
        return m


# ------------------------------------------------------------------------- FIT
class FitValidationError(Exception):
    """java.lang.Exception raised by LanguageDetector.fit's input checks."""


class LanguageDetector(_Params):
    """LanguageDetector (LanguageDetector.scala:176-264)."""

    _defaults = {"inputCol": "fulltext", "labelCol": "lang", "saveGrams": None}

    def __init__(self, supportedLanguages: Sequence[str], gramLengths: Sequence[int], languageProfileSize: int,
                 uid: Optional[str] = None, device: Optional[int] = None):
        super().__init__()
        self.uid = uid or _random_uid("LanguageDetector")
        self.supportedLanguages = list(supportedLanguages)
        self.gramLengths = list(gramLengths)
        self.languageProfileSize = int(languageProfileSize)
        self._device = device

    def setInputCol(self, value: str):
        return self._set("inputCol", value)

    def setLabelCol(self, value: str):
        return self._set("labelCol", value)

    def setSaveGramsToHDFS(self, value: Optional[str]):
        return self._set("saveGrams", value)

    def getInputCol(self) -> str:
        return self.getOrDefault("inputCol")

    def getLabelCol(self) -> str:
        return self.getOrDefault("labelCol")

    def transformSchema(self, schema):
        return schema

    @staticmethod
    def validate(labels: Sequence[str], supportedLanguages: Sequence[str]) -> None:
        """LanguageDetector.scala:221-238 in code order: an unsupported label
        first (first in input order here; Spark's `distinct` order is
        unspecified), then a supported language without rows."""
        sup = set(supportedLanguages)
        seen = set()
        for lang in labels:
            if lang in seen:
                continue
            seen.add(lang)
            if lang not in sup:
                raise FitValidationError(
                    f"Input data contians {lang}, but it is not in the list of supported languages")
        for lang in supportedLanguages:
            if lang not in seen:
                raise FitValidationError(
                    f"No training examples found for language {lang}. Provide examples for each language")

    @staticmethod
    def count_grams(data: Sequence[Tuple[str, str]], gramLengths: Sequence[int], supportedLanguages: Sequence[str],
                    device: Optional[int] = None) -> DeviceCounts:
        """computeGrams + reduceGrams on the GPU (LanguageDetector.scala:25-66)."""
        index = {l: i for i, l in enumerate(supportedLanguages)}
        langs = np.asarray([index.get(l, -1) for l, _ in data], dtype=np.int32)
        for _, t in data:
            if t is None:
                raise NullPointerException("training text is null")
        bytes_, offsets = encoding.pack_fit([t for _, t in data])
        counts = DeviceCounts(len(supportedLanguages), gramLengths, device=device)
        counts.count(bytes_, offsets, langs)
        return counts

    @staticmethod
    def computeGramProbabilities(data: Sequence[Tuple[str, str]], gramLengths: Sequence[int],
                                 languageProfileSize: int, supportedLanguages: Sequence[str],
                                 device: Optional[int] = None) -> Dict[bytes, List[float]]:
        """computeGramProbabilities (LanguageDetector.scala:145-165) -> {gram: row}."""
        counts = LanguageDetector.count_grams(data, gramLengths, supportedLanguages, device)
        try:
            return counts.fit_table(languageProfileSize)
        finally:
            counts.close()

    def fit(self, dataset) -> LanguageDetectorModel:
        labels, texts = _rows_of(dataset, self.getLabelCol(), self.getInputCol())
        self.validate(labels, self.supportedLanguages)
        table = self.computeGramProbabilities(list(zip(labels, texts)), self.gramLengths,
                                              self.languageProfileSize, self.supportedLanguages, self._device)
        save = self.getOrDefault("saveGrams")
        if save:
            save_grams(save, table)
        return LanguageDetectorModel(table, self.gramLengths, self.supportedLanguages, device=self._device)


def save_grams(path: str, table: Dict[bytes, List[float]]) -> None:
    """LanguageDetector.save (LanguageDetector.scala:167-171): the gram table
    as parquet columns _1 array<tinyint> (signed bytes), _2 array<double>."""
    import pyarrow as pa
    import pyarrow.parquet as pq
    keys = [np.frombuffer(k, dtype=np.int8).tolist() for k in table]
    rows = [list(v) for v in table.values()]
    t = pa.table({"_1": pa.array(keys, type=pa.list_(pa.int8())), "_2": pa.array(rows, type=pa.list_(pa.float64()))})
    import os
    os.makedirs(path, exist_ok=True)
    pq.write_table(t, os.path.join(path, "part-00000.parquet"))
