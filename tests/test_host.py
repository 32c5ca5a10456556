"""CPU: host logic of the drop-in (encodings, packing, validation, params) and
the C-ABI library: it loads and exports every symbol include/ldgpu.h declares.
No compute call is made here (no GPU)."""
import ctypes
import os
import re

import numpy as np
import pytest

import ldoracle as O
from conftest import ROOT
from languagedetection import _lib, encoding, synth
from languagedetection.api import FitValidationError, LanguageDetector, LanguageDetectorModel

HEADER = os.path.join(ROOT, "include", "ldgpu.h")


def header_symbols():
    src = open(HEADER).read()
    return sorted(set(re.findall(r"\b(ldgpu_[a-z_]+)\s*\(", src)))


def test_library_exports_every_header_symbol():
    lib = _lib.load()
    syms = header_symbols()
    assert len(syms) >= 20
    for s in syms:
        assert hasattr(lib, s), s
    assert sorted(_lib.exported_symbols()) == syms
    assert lib.ldgpu_version().decode().startswith("ldgpu")


def test_libraries_are_built_from_this_tree():
    # build provenance: the hash of the sources compiled into each library
    # (ldgpu_build_id) equals the hash of the sources in this tree
    for variant in ("product", "diag"):
        prov = _lib.provenance(variant)
        assert prov["match"], (variant, prov)
    # ... and the compile flags: a diagnostics (or any non-product) build
    # reports its own id, never the product's
    prod = _lib.load().ldgpu_build_id().decode()
    diag = _lib.load(variant="diag").ldgpu_build_id().decode()
    assert "+" not in prod and diag.startswith(prod + "+") and diag != prod


def test_library_is_gfx950_code_object():
    so = _lib.LIB_PATH
    blob = open(so, "rb").read()
    assert b"gfx950" in blob


def test_encodings_match_oracle():
    texts = ["plain ascii", "schön", "日本語", "😀 x", "\ud800 lone", "\udfff", "", "Ärger über Öl"]
    for t in texts:
        assert encoding.fit_bytes(t) == O.fit_encode(t), t
        assert encoding.score_bytes(t) == O.score_encode(t), t


def test_pack_padding_and_offsets():
    data, off = encoding.pack([b"ab", b"", b"cde"])
    assert off.tolist() == [0, 2, 2, 5]
    assert len(data) % 4 == 0 and len(data) >= 5 + 4
    assert data[:5].tobytes() == b"abcde"


def test_gram_key_forms():
    assert encoding.gram_key("Die") == b"Die"
    assert encoding.gram_key([-61, -74]) == b"\xc3\xb6"   # Scala signed bytes
    assert encoding.gram_key(b"x") == b"x"


def test_pack_table_marks_wrong_length_rows():
    kb, ko, rows, ok = encoding.pack_table({b"a": [1.0, 2.0], b"b": [1.0]}, 2)
    assert ok.tolist() == [1, 0]
    assert rows[0].tolist() == [1.0, 2.0]


def test_fit_validation_messages_follow_code_order():
    with pytest.raises(FitValidationError) as e:
        LanguageDetector.validate(["de", "de", "es"], ["de", "en"])
    assert str(e.value) == "Input data contians es, but it is not in the list of supported languages"
    with pytest.raises(FitValidationError) as e:
        LanguageDetector.validate(["de"], ["de", "en"])
    assert str(e.value) == "No training examples found for language en. Provide examples for each language"
    LanguageDetector.validate(["en", "de"], ["de", "en"])


def test_params_defaults_and_setters():
    d = LanguageDetector(["de", "en"], [3], 5)
    assert d.getInputCol() == "fulltext" and d.getLabelCol() == "lang"
    assert d.uid.startswith("LanguageDetector_")
    d.setInputCol("text").setLabelCol("label")
    assert d.getInputCol() == "text" and d.getLabelCol() == "label"
    m = LanguageDetectorModel({"Die": [1.0, 0.0]}, [3], ["de", "en"])
    assert m.getInputCol() == "fulltext" and m.getOutputCol() == "lang"
    assert m.gramLenghts == [3] and m.supportedLanguages == ["de", "en"]
    assert m.gramProbabilities == {b"Die": [1.0, 0.0]}


def test_transform_schema_rules():
    m = LanguageDetectorModel({}, [3], ["de"])
    assert m.transformSchema({"fulltext": "string"}) == {"fulltext": "string", "lang": "string"}
    with pytest.raises(ValueError, match="Input type must be StringType"):
        m.transformSchema({"fulltext": "int64"})
    with pytest.raises(ValueError, match="Column lang already exists"):
        m.transformSchema({"fulltext": "string", "lang": "string"})


def test_synth_is_deterministic_ascii():
    ls = synth.make_languages(5, seed=11)
    a = synth.generate(ls, 50, 10, 40, seed=3)
    b = synth.generate(synth.make_languages(5, seed=11), 50, 10, 40, seed=3)
    for x, y in zip(a, b):
        assert np.array_equal(x, y)
    data, off, lang = a
    assert data.max() < 128 and len(off) == 51 and off[-1] == len(data)
    assert synth.language_names(3) == ["en", "de", "fr"]
    assert len(set(synth.language_names(200))) == 200


def test_no_gpu_fails_loudly():
    """Without a visible GPU the product path raises; there is no fallback."""
    if _lib.device_count() > 0:
        pytest.skip("a GPU is visible")
    with pytest.raises(Exception):
        _lib.context(0)


def test_product_library_reads_no_env_switches():
    """The LDGPU_* path / ablation switches live only in the diagnostics build
    (lib/libldgpu_diag.so): no such name appears in the product library."""
    from languagedetection import _lib
    blob = open(_lib.LIB_PATH, "rb").read()
    assert b"LDGPU_" not in blob
    assert b"LDGPU_ABLATE" in open(_lib.DIAG_LIB_PATH, "rb").read()


def test_bench_traffic_lookup_scales_profiled_launch():
    """bench.py reports the committed PMC traffic of its exact workload, or of
    the same workload profiled over fewer documents scaled to its own count
    (roofline.traffic_scaled_from says so); another shape gets none."""
    import importlib.util
    import json
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(root, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    prof = json.load(open(os.path.join(root, "profiles", "pmc_traffic_config5.json")))
    key = prof["workload_key"]
    assert bench.traffic_from_profiles(key)["traffic_bytes_per_launch"] == prof["traffic_bytes_per_launch"]
    docs = int(key.split(":docs=")[1].split(":")[0])
    scaled = bench.traffic_from_profiles(key.replace(f":docs={docs}:", f":docs={5 * docs}:"))
    assert scaled["traffic_bytes_per_launch"] == round(5 * prof["traffic_bytes_per_launch"])
    assert "x5" in scaled["traffic_scaled_from"]
    assert bench.traffic_from_profiles(key.replace(":L=200:", ":L=201:")) is None


def test_detect_cache_reuses_only_unchanged_maps():
    """The detect() cache (api._detect_model) may reuse a device table only
    while the map's contents equal the snapshot it was built from."""
    from languagedetection.api import FrozenTable, _snapshot, _unchanged, freeze_table
    t = {"ab": [1.0, 0.0], "cd": [0.0, 1.0]}
    s = _snapshot(t)
    assert _unchanged(t, s)
    t["ab"][0] = 0.5                      # value list edited in place
    assert not _unchanged(t, s)
    t["ab"][0] = 1.0
    assert _unchanged(t, s)
    t["cd"] = [0.0, 2.0]                  # non-first entry replaced, same length
    assert not _unchanged(t, s)
    assert _snapshot({"ab": np.zeros(2)}) is None   # rows not comparable: never cached
    f = freeze_table(t)
    assert isinstance(f, FrozenTable) and freeze_table(f) is f
    assert _unchanged(f, _snapshot(f)) and dict(f) == {b"ab": (1.0, 0.0), b"cd": (0.0, 2.0)}


def test_round_bench_lines_follow_from_committed_profiles():
    """Every round-6 bench line's roofline.traffic is what bench.py computes
    from the committed PMC file of its workload (profiles/pmc_traffic*.json),
    FIT lines charged with the count's own kernels only; config 5's frac is
    priced on the bytes its design moves (<= 1)."""
    import glob
    import json
    import sys
    sys.path.insert(0, ROOT)
    import bench
    lines = sorted(glob.glob(os.path.join(ROOT, "profiles", "r06_bench*.json")))
    assert len(lines) >= 6
    for f in lines:
        d = json.load(open(f))
        r = d["roofline"]
        if r.get("workload_key"):
            want = (bench.traffic_from_profiles(r["workload_key"]) or {}).get("traffic_bytes_per_launch")
        else:
            wl = d["config"]
            L = int(re.search(r"(\d+) languages", wl["workload"]).group(1))
            G = [int(x) for x in re.search(r"grams ([\d,]+),", wl["workload"]).group(1).split(",")]
            want = bench.count_traffic(
                bench.traffic_from_profiles(f"fit:bytes={wl['corpus_bytes_per_gpu']}:L={L}:G={','.join(map(str, G))}"),
                L, G)
        assert r["traffic"] == want, (f, r["traffic"], want)   # (None: no PMC profile, no claim)
        assert 0 < r["frac"] <= 1, (f, r["frac"])
        assert d["build"]["match"], f
    # one library build for every line of the round
    assert len({json.load(open(f))["build"]["library_source_hash"] for f in lines}) == 1


def test_fit_pmc_calibration_follows_from_its_raw_counters():
    """The FIT PMC files' read / write factors are the calibration kernels'
    known bytes over their raw counters (tools/fit_pmc.py): FIT v4 part2's
    8 B per record read and written; FIT v5 sort_emit's 8 B written per
    position and runs_count's 8 B read per sorted key (one pass)."""
    import json
    for name, line in (("pmc_traffic_fit.json", "r06_bench_fit.json"),
                       ("pmc_traffic_fit_L200.json", "r06_bench_fit_L200_1GB.json")):
        prof = json.load(open(os.path.join(ROOT, "profiles", name)))
        cfg = json.load(open(os.path.join(ROOT, "profiles", line)))["config"]
        raw = prof["per_kernel_raw_bytes_per_count"]
        rec = 8 * cfg["corpus_bytes_per_gpu"]
        p2 = next((v for k, v in raw.items() if k.startswith("part2_kernel")), None)
        if p2:
            rf, wf = rec / p2["FETCH_SIZE"], rec / p2["WRITE_SIZE"]
        else:
            G = [int(x) for x in re.search(r"grams ([\d,]+),", cfg["workload"]).group(1).split(",")]
            em = next(v for k, v in raw.items() if k.startswith("sort_emit_kernel"))
            rc = next(v for k, v in raw.items() if k.startswith("runs_count_kernel"))
            rf, wf = 8 * cfg["windows_per_gpu"] / len(G) / rc["FETCH_SIZE"], rec / em["WRITE_SIZE"]
        assert abs(prof["read_factor"] - rf) < 1e-3 and abs(prof["write_factor"] - wf) < 1e-3, (name, rf, wf)
        # streaming counters undercount reads about 2x on gfx950 (MI355X guide): the factors say so
        assert 1.2 < prof["read_factor"] < 2.5 and 0.8 < prof["write_factor"] < 1.2, name
