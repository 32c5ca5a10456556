"""GPU parity of FIT (LanguageDetector.scala:25-132): counts bit-exact, the
probability rows and the deterministic top-K table equal to the oracle's."""
import json
import os

import numpy as np
import pytest

import ldoracle as O
import ldoracle_c as OC
from conftest import GOLDEN
from languagedetection import LanguageDetector, LanguageDetectorModel, encoding, synth
from languagedetection.runtime import DeviceCounts

pytestmark = pytest.mark.gpu


def load(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


def dec_table(enc):
    return {bytes.fromhex(k): [float.fromhex(v) for v in row] for k, row in enc}


@pytest.mark.parametrize("case", load("fit_cases.json"), ids=lambda c: c["name"])
def test_golden_fit_cases(case):
    rows = [tuple(r) for r in case["rows"]]
    langs = case["languages"]
    counts = LanguageDetector.count_grams(rows, case["gram_lengths"], langs)
    keys, cnt = counts.export()
    got = {}
    for i, k in enumerate(keys):
        for l, lang in enumerate(langs):
            if cnt[i, l]:
                got.setdefault(k.hex(), {})[lang] = int(O.int32_wrap(int(cnt[i, l])))
    assert got == case["counts"]
    table = counts.fit_table(case["profile_size"])
    assert table == dec_table(case["table"])


def test_reference_fit_kat():
    """LanguageDetectorSpecs.scala:15-40 through the Estimator API."""
    import pandas as pd
    k = load("reference_kats.json")["fit_kat"]
    df = pd.DataFrame(k["rows"], columns=["lang", "fulltext"])
    det = LanguageDetector(supportedLanguages=k["languages"], gramLengths=k["gram_lengths"],
                           languageProfileSize=k["profile_size"])
    model = det.fit(df)
    assert len(model.gramProbabilities) == k["expect_table_size"]
    assert all(len(r) == k["expect_row_length"] for r in model.gramProbabilities.values())
    probs = O.fit_probabilities([tuple(r) for r in k["rows"]], k["languages"], k["gram_lengths"])
    assert O.topk_contract_violations(model.gramProbabilities, probs, k["languages"], k["profile_size"]) == []


def test_validation_order_kat():
    import pandas as pd
    k = load("reference_kats.json")["validation_kat"]
    det = LanguageDetector(k["languages"], k["gram_lengths"], k["profile_size"])
    with pytest.raises(Exception) as e:
        det.fit(pd.DataFrame(k["rows"], columns=["lang", "fulltext"]))
    assert str(e.value) == k["code_order_raises"]


@pytest.mark.parametrize("L,grams,n_docs", [(3, [1, 2, 3], 300), (20, [1, 2, 3, 4, 5], 2000),
                                            (70, [7, 1, 4, 4], 1500), (200, [1, 2, 3], 1200),
                                            (300, [1, 2, 3, 4], 1500)])
def test_counts_match_c_oracle(L, grams, n_docs):
    ls = synth.make_languages(L, seed=L)
    data, off, lang = synth.generate(ls, n_docs, 0, 700, seed=L + 1)
    counts = DeviceCounts(L, grams)
    counts.count(data, off, lang)
    keys, cnt = counts.export()
    okeys, ocnt = OC.count(data, off, lang, L, grams)
    assert keys == okeys
    assert np.array_equal(cnt, ocnt)


def test_counts_growth_and_overflow_path():
    """A tiny capacity hint forces overflow entries and device re-hashing."""
    rng = np.random.default_rng(4)
    docs = [bytes(rng.integers(0, 256, size=int(n), dtype=np.uint8)) for n in rng.integers(0, 2000, size=400)]
    data, off = encoding.pack(docs)
    lang = rng.integers(0, 4, size=len(docs)).astype(np.int32)
    lang[::37] = -1   # unsupported labels are skipped (reduceGrams filter)
    counts = DeviceCounts(4, [3, 5, 2], capacity_hint=16)
    counts.count(data, off, lang)
    counts.count(data, off, lang)  # second batch accumulates
    keys, cnt = counts.export()
    okeys, ocnt = OC.count(data, off, lang, 4, [3, 5, 2])
    assert keys == okeys
    assert np.array_equal(cnt, 2 * ocnt)


def test_counts_add_merges_blocks():
    ls = synth.make_languages(5, seed=3)
    data, off, lang = synth.generate(ls, 400, 10, 300, seed=4)
    a = DeviceCounts(5, [1, 2, 3])
    a.count(data, off, lang)
    keys, cnt = a.export()
    b = DeviceCounts(5, [1, 2, 3])
    b.add(keys[::2], cnt[::2])
    b.add(keys, cnt)
    k2, c2 = b.export()
    assert k2 == keys
    extra = np.zeros_like(cnt)
    extra[::2] = cnt[::2]
    assert np.array_equal(c2, cnt + extra)


@pytest.mark.parametrize("L,grams,K", [(3, [1, 2, 3], 50), (20, [1, 2, 3, 4, 5], 500), (8, [2, 3], 100000),
                                       (5, [3], 0)])
def test_fit_table_matches_oracle(L, grams, K):
    ls = synth.make_languages(L, seed=100 + L)
    data, off, lang = synth.generate(ls, 60 * L, 20, 200, seed=L)
    rows = list(zip([ls.names[i] for i in lang], synth.texts(data, off)))
    table = LanguageDetector.computeGramProbabilities(rows, grams, K, ls.names)
    probs = O.fit_probabilities(rows, ls.names, grams)
    expect = O.filter_top_grams(probs, ls.names, K)
    assert table.keys() == expect.keys()
    for g in expect:
        assert table[g] == expect[g]  # log(1+1/k) computed by the same libm formula
    assert O.topk_contract_violations(table, probs, ls.names, K) == []


def test_fit_then_transform_end_to_end():
    import pandas as pd
    ls = synth.make_languages(6, seed=9)
    tdata, toff, tlang = synth.generate(ls, 600, 100, 400, seed=10)
    df = pd.DataFrame({"lang": [ls.names[i] for i in tlang], "fulltext": synth.texts(tdata, toff)})
    model = LanguageDetector(ls.names, [1, 2, 3], 200).fit(df)
    data, off, lang = synth.generate(ls, 500, 50, 300, seed=11)
    texts = synth.texts(data, off)
    out = model.transform(pd.DataFrame({"fulltext": texts}))
    expect = O.transform(texts, model.gramProbabilities, ls.names, [1, 2, 3])
    assert list(out["lang"]) == expect
    acc = np.mean([ls.names[l] == p for l, p in zip(lang, out["lang"])])
    assert acc > 0.9


def test_device_export_add_roundtrip_and_device_top_k():
    """ldgpu_counts_export_device / _add_device keep counts in HBM; the device
    top-K path (no zero fill needed) equals the oracle's deterministic table."""
    import torch
    ls = synth.make_languages(12, seed=31)
    data, off, lang = synth.generate(ls, 1500, 100, 800, seed=32)
    a = DeviceCounts(12, [1, 2, 3, 4])
    a.count(data, off, lang)
    k, c = a.export_device()
    b = DeviceCounts(12, [1, 2, 3, 4])
    b.add_device(k, c)
    b.add_device(k, c)
    ka, ca = a.export()
    kb, cb = b.export()
    assert ka == kb and np.array_equal(2 * ca, cb)
    rows = list(zip([ls.names[i] for i in lang], synth.texts(data, off)))
    probs = O.fit_probabilities(rows, ls.names, [1, 2, 3, 4])
    expect = O.filter_top_grams(probs, ls.names, 300)
    assert a.fit_table(300) == expect


@pytest.mark.parametrize("L,grams,K", [(20, [1, 2, 3, 4, 5], 300), (70, [1, 2, 3], 50), (8, [2, 3], 100000)])
def test_fit_table_mask_form_and_model_from_masks(L, grams, K):
    """ldgpu_fit_table_export_masks carries the same table as the dense export
    (row = val at the mask's languages), and a model built from it
    (ldgpu_model_create_masks) scores bit-identically to the dense-built one."""
    from languagedetection.runtime import DeviceModel
    ls = synth.make_languages(L, seed=300 + L)
    data, off, lang = synth.generate(ls, 40 * L, 50, 300, seed=L + 1)
    counts = DeviceCounts(L, grams)
    counts.count(data, off, lang)
    dense = counts.fit_table(K)
    kb, ko, masks, vals = counts.fit_table_masks(K)
    b = kb.tobytes()
    assert len(ko) - 1 == len(dense)
    for i in range(len(ko) - 1):
        row = dense[b[ko[i]:ko[i + 1]]]
        exp = [vals[i] if (int(masks[i, l // 64]) >> (l % 64)) & 1 else 0.0 for l in range(L)]
        assert row == exp
    counts.close()
    sdata, soff, _ = synth.generate(ls, 3000, 0, 300, seed=L + 2)
    m1 = DeviceModel(dense, L, grams)
    m2 = DeviceModel.from_masks(kb, ko, masks, vals, L, grams)
    assert m1.info()["mode"] == m2.info()["mode"]
    l1, s1 = m1.score(sdata, soff, want_scores=True)
    l2, s2 = m2.score(sdata, soff, want_scores=True)
    assert np.array_equal(l1, l2) and np.array_equal(s1.view(np.uint64), s2.view(np.uint64))


def test_fit_tables_of_two_count_tables_on_one_context():
    """A single-rank device top-K leaves its rows in the context's pinned
    buffer until exported; a second table's build on the same context first
    moves them into the first table's own storage: both tables export what
    they built, in mask and dense form, in any order."""
    L, grams = 12, [1, 2, 3]
    ls = synth.make_languages(L, seed=41)
    d1, o1, l1 = synth.generate(ls, 800, 50, 400, seed=42)
    d2, o2, l2 = synth.generate(ls, 800, 50, 400, seed=43)
    a = DeviceCounts(L, grams)
    a.count(d1, o1, l1)
    b = DeviceCounts(L, grams)
    b.count(d2, o2, l2)
    ta = a.fit_table_masks(150)
    tb = b.fit_table_masks(150)          # a's rows leave the pinned buffer first
    ta2 = a.cached_table_masks()
    tb2 = b.cached_table_masks()
    for x, y in ((ta, ta2), (tb, tb2)):
        assert all(np.array_equal(u, v) for u, v in zip(x, y))
    dense_a = a.fit_table(150)           # rebuilt: pinned again, b's moved out
    assert dense_a == _topk_table_from_counts(*OC.count(d1, o1, l1, L, grams), L, 150)
    assert all(np.array_equal(u, v) for u, v in zip(tb, b.cached_table_masks()))
    a.close()
    assert all(np.array_equal(u, v) for u, v in zip(tb, b.cached_table_masks()))
    b.close()


def _topk_table_from_counts(keys, cnt, L, K):
    """filterTopGrams (LanguageDetector.scala:100-132) over oracle counts,
    vectorised: v_l = log(1 + [l] / k); per language the K largest v_l, ties
    by ascending (length, bytes) = index order of the sorted keys."""
    pres = cnt > 0
    k = pres.sum(axis=1)
    w = np.zeros(len(keys))
    w[k > 0] = np.log(1.0 + 1.0 / k[k > 0])
    chosen = np.zeros(len(keys), dtype=bool)
    idx = np.arange(len(keys))
    for l in range(L):
        v = np.where(pres[:, l], w, 0.0)
        order = np.lexsort((idx, -v))
        chosen[order[:K]] = True
    return {keys[i]: [float(w[i]) if pres[i, l] else 0.0 for l in range(L)] for i in np.nonzero(chosen)[0]}


def test_fit_and_score_more_than_256_languages():
    """L > 256: FIT counts / top-K unchanged in form (mask words ceil(L/64)),
    and the model scores in language blocks of 256 (one launch per block,
    first maximum across blocks): labels and fp64 scores bit-identical to the
    oracle, dense-built and mask-built, labels-only too."""
    from languagedetection.runtime import DeviceModel
    L, grams, K = 300, [1, 2, 3], 25
    ls = synth.make_languages(L, seed=77)
    data, off, lang = synth.generate(ls, 8 * L, 50, 300, seed=78)
    counts = DeviceCounts(L, grams)
    counts.count(data, off, lang)
    keys, cnt = counts.export()
    okeys, ocnt = OC.count(data, off, lang, L, grams)
    assert keys == okeys and np.array_equal(cnt, ocnt)
    dense = counts.fit_table(K)
    assert dense == _topk_table_from_counts(okeys, ocnt, L, K)
    kb, ko, masks, vals = counts.fit_table_masks(K)
    counts.close()
    sdata, soff, _ = synth.generate(ls, 3000, 0, 300, seed=79)
    ol, osc = OC.Table(dense, L).score(grams, sdata, soff, want_scores=True, nthreads=8)
    for m in (DeviceModel(dense, L, grams), DeviceModel.from_masks(kb, ko, masks, vals, L, grams)):
        labels, scores = m.score(sdata, soff, want_scores=True)
        assert np.array_equal(labels, ol)
        assert np.array_equal(scores.view(np.uint64), osc.view(np.uint64))
        only, _ = m.score(sdata, soff, want_scores=False)
        assert np.array_equal(only, ol)


def test_config3_shape_counts_and_table():
    """Config 3's shape at test size: documents of 1-7 KB (U[1024, 7168]),
    20 languages, grams 1-5, ~40 MB of corpus through the device-resident
    path (ldgpu_count_device, as bench.py --mode fit).  Counts bit-exact
    against the C restatement, the K=500 table equal to the top-K rule
    applied to the oracle's counts."""
    import torch
    L, grams, K = 20, [1, 2, 3, 4, 5], 500
    ls = synth.make_languages(L)
    data, off, lang = synth.generate(ls, 10000, 1024, 7168, seed=synth.SEED_BASE + 3)
    dev = torch.device("cuda", 0)
    n = int(off[-1])
    d_bytes = torch.zeros(((n + 3) // 4) * 4 + 16, dtype=torch.uint8, device=dev)
    d_bytes[:n].copy_(torch.from_numpy(data))
    d_off = torch.from_numpy(off).to(dev)
    d_lang = torch.from_numpy(lang).to(dev)
    counts = DeviceCounts(L, grams, capacity_hint=1 << 16)
    counts.count_device(d_bytes.data_ptr(), n, d_off.data_ptr(), d_lang.data_ptr(), len(off) - 1,
                        torch.cuda.current_stream(dev).cuda_stream)
    torch.cuda.synchronize(dev)
    keys, cnt = counts.export()
    okeys, ocnt = OC.count(data, off, lang, L, grams)
    assert len(keys) == len(okeys) and keys == okeys
    assert np.array_equal(cnt, ocnt)
    table = counts.fit_table(K)
    expect = _topk_table_from_counts(okeys, ocnt, L, K)
    assert table.keys() == expect.keys()
    assert all(table[g] == expect[g] for g in expect)


@pytest.mark.parametrize("variant,env", [
    ("product", {}),                                         # FIT v4, the table's own record form: one batch
    ("diag", {"LDGPU_FIT_BATCH_WINDOWS": "20000"}),          # FIT v4: many small batches
    ("diag", {"LDGPU_FIT_K": "2"}),                          # two-word records: FIT v5 (sort + runs)
    ("diag", {"LDGPU_FIT_K": "2", "LDGPU_FIT_SORT_BATCH": "5000"}),  # ... many sort batches
    ("diag", {"LDGPU_FIT_K": "2", "LDGPU_FIT_NO_SORT": "1"}),  # ... FIT v4: T1 of two-word pairs + derive
    ("diag", {"LDGPU_FIT_K": "2", "LDGPU_FIT_NO_SORT": "1", "LDGPU_FIT_DERIVE_INPLACE": "1"}),  # ... one T1
    ("diag", {"LDGPU_FIT_K": "3", "LDGPU_FIT_BATCH_WINDOWS": "50000"}),  # three-word records, several batches
    ("diag", {"LDGPU_FIT_BATCH_WINDOWS": "700"}),            # batches of one document (most are longer)
    ("diag", {"LDGPU_FIT_LEGACY": "1"}),                     # round-1 single-pass atomic kernels (A/B only)
])
@pytest.mark.parametrize("L,grams", [(20, [1, 2, 3, 4, 5]), (100, [1, 2, 6]), (256, [3, 1, 3]), (2, [5, 4]),
                                     (200, [1, 2, 3, 4, 5, 6, 7]), (20, [7]), (5, [2, 9, 15]), (30, [8, 1])])
def test_count_paths_match_oracle(L, grams, variant, env, monkeypatch):
    """Every counting path, bit-exact against the C restatement over two
    calls: FIT v5 for two-word records (every full maximal window's sort key
    lang << 8N | bytes big-endian, radix-sorted, one run pass per gram length;
    tail positions added directly), in one and in many sort batches; FIT v4 (documents grouped by language, one record per byte
    position -- its maximal window of min(max(G), rest) bytes --, records
    bucketed twice and LDS-aggregated into the call's table of maximal
    windows, which derives every gram length as prefixes) in the table's own
    record form -- one word when it fits (L=20, grams 1-5), two for grams of
    <= 7 bytes with many languages (L=200, grams 1-7; L=4096), three with
    grams of 8..15 bytes -- in one and in many batches, the wider forms forced
    on small tables, and the legacy kernels.  Duplicate lengths count twice
    (256, [3, 1, 3]); unsupported labels (-1) are skipped; documents shorter
    than n count their whole text (partial windows, also of 8..14 bytes)."""
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    rng = np.random.default_rng(L + len(grams))
    ls = synth.make_languages(L, seed=L + 7)
    data, off, lang = synth.generate(ls, 900, 0, 900, seed=L + 8)
    docs = [bytes(data[off[i]:off[i + 1]]) for i in range(len(off) - 1)]
    docs += [b"a" * 3000, b"ab" * 1500, b"abc" * 700, b"", b"x", b"xy", b"abcdefghijklmnopq" * 20]
    dl = np.concatenate([lang, rng.integers(0, L, size=7).astype(np.int32)])
    dl[::29] = -1
    d, o = encoding.pack(docs)
    counts = DeviceCounts(L, grams, variant=variant)
    counts.count(d, o, dl)
    counts.count(d[:int(o[300])], o[:301], dl[:300])   # a second call accumulates
    keys, cnt = counts.export()
    okeys, ocnt = OC.count(d, o, dl, L, grams)
    okeys2, ocnt2 = OC.count(d[:int(o[300])], o[:301], dl[:300], L, grams)
    extra = dict(zip(okeys2, ocnt2))
    expect = np.array([ocnt[i] + extra.get(k, 0) for i, k in enumerate(okeys)])
    assert keys == okeys
    assert np.array_equal(cnt, expect)


@pytest.mark.parametrize("variant", ["product", "diag"])
def test_count_4096_languages(variant, monkeypatch):
    """The largest language count: two-word records (12 language bits leave
    a one-word record no count bits at grams up to 6), a few short documents
    per language id spread over all 4096 (dense export rows stay small)."""
    if variant == "diag":
        monkeypatch.setenv("LDGPU_FIT_BATCH_WINDOWS", "3000")
        monkeypatch.setenv("LDGPU_FIT_SORT_BATCH", "300")
    L, grams = 4096, [2, 6, 1]
    rng = np.random.default_rng(4096)
    alphabet = np.frombuffer(b"abcdefgh ", dtype=np.uint8)
    docs = [bytes(rng.choice(alphabet, size=int(n))) for n in rng.integers(0, 60, size=40)]
    dl = rng.integers(0, L, size=len(docs)).astype(np.int32)
    dl[-1] = L - 1
    d, o = encoding.pack(docs)
    counts = DeviceCounts(L, grams, variant=variant)
    counts.count(d, o, dl)
    keys, cnt = counts.export()
    okeys, ocnt = OC.count(d, o, dl, L, grams)
    assert keys == okeys
    assert np.array_equal(cnt, ocnt)


def test_count_single_language_long_corpus():
    """One language, long documents: the reduce buckets' LDS hashes fill
    (random bytes: many distinct windows, some go out unaggregated) and hot
    grams count far past a record's count field; counts bit-exact."""
    rng = np.random.default_rng(12)
    ls = synth.make_languages(3, seed=12)
    lang = np.zeros(400, np.int32)
    data, off, lang = synth.generate(ls, 400, 3000, 9000, seed=13, doc_lang=lang)
    rnd = [bytes(rng.integers(0, 256, size=20000, dtype=np.uint8)) for _ in range(20)]  # many distinct 3-grams
    docs = [bytes(data[off[i]:off[i + 1]]) for i in range(len(off) - 1)] + rnd
    d, o = encoding.pack(docs)
    dl = np.zeros(len(docs), np.int32)
    counts = DeviceCounts(3, [1, 2, 3, 4, 5])
    counts.count(d, o, dl)
    keys, cnt = counts.export()
    okeys, ocnt = OC.count(d, o, dl, 3, [1, 2, 3, 4, 5])
    assert keys == okeys
    assert np.array_equal(cnt, ocnt)


def _wide_corpus(grams, L, seed):
    rng = np.random.default_rng(seed)
    alphabet = np.frombuffer(b"abcd ", dtype=np.uint8)
    lens = rng.integers(0, 60, size=600)
    lens[:12] = [0, 1, 2, 7, 8, 9, 11, 14, 15, 16, 17, 30]
    docs = [bytes(rng.choice(alphabet, size=int(n))) for n in lens]
    data, off = encoding.pack(docs)
    lang = rng.integers(0, L, size=len(docs)).astype(np.int32)
    lang[::41] = -1
    return data, off, lang


@pytest.mark.parametrize("grams", [[8], [1, 3, 9, 12], [15, 2, 9, 9], [5, 10], [7, 8], [16], [3, 20], [31],
                                   [2, 17, 9, 17]])
def test_wide_gram_counts_table_and_model(grams):
    """Gram lengths 8..15 (computeGrams, LanguageDetector.scala:32-43, any n):
    windows of 8..15 bytes count in a two-word-key table of their own; the
    partial window of a document shorter than n is its whole text, so a wide
    length also makes keys of every length below n (those under 8 bytes in
    the one-word table).  Counts bit-exact against the C restatement over two
    calls, the top-K table (host selection over the pulled table, ties by
    (length, bytes)) equal to the rule applied to the oracle's counts, and the
    model built from it scoring like the oracle."""
    from languagedetection.runtime import DeviceModel
    L = 5
    data, off, lang = _wide_corpus(grams, L, sum(grams))
    counts = DeviceCounts(L, grams, capacity_hint=16)
    counts.count(data, off, lang)
    counts.count(data[:int(off[100])], off[:101], lang[:100])   # a second call accumulates
    keys, cnt = counts.export()
    okeys, ocnt = OC.count(data, off, lang, L, grams)
    okeys2, ocnt2 = OC.count(data[:int(off[100])], off[:101], lang[:100], L, grams)
    extra = dict(zip(okeys2, ocnt2))
    expect = np.array([ocnt[i] + extra.get(k, 0) for i, k in enumerate(okeys)])
    assert keys == okeys
    assert np.array_equal(cnt, expect)
    assert max(len(k) for k in keys) == max(grams) or max(grams) <= 7
    st = counts.stats()
    assert st == {"grams": len(okeys), "pairs": int((expect > 0).sum()), "total": int(expect.sum())}
    for K in (20, 100000):   # 100000: every gram, zero-valued fill included
        table = counts.fit_table(K)
        assert table == _topk_table_from_counts(okeys, expect, L, K)
    table = counts.fit_table(30)
    counts.close()
    sdata, soff, _ = _wide_corpus(grams, L, sum(grams) + 1)
    ol, osc = OC.Table(table, L).score(grams, sdata, soff, want_scores=True, nthreads=8)
    labels, scores = DeviceModel(table, L, grams).score(sdata, soff, want_scores=True)
    assert np.array_equal(labels, ol)
    assert np.array_equal(scores.view(np.uint64), osc.view(np.uint64))


def test_wide_gram_counts_add_and_limits():
    """ldgpu_counts_add takes keys of 1..15 bytes (wide ones into the two-word
    table); the packed-u64 device export has no form for them and says so."""
    L, grams = 4, [2, 9]
    data, off, lang = _wide_corpus(grams, L, 5)
    a = DeviceCounts(L, grams)
    a.count(data, off, lang)
    keys, cnt = a.export()
    assert any(len(k) > 7 for k in keys)
    b = DeviceCounts(L, [1])
    b.add(keys[::2], cnt[::2])
    b.add(keys, cnt)
    k2, c2 = b.export()
    extra = np.zeros_like(cnt)
    extra[::2] = cnt[::2]
    assert k2 == keys and np.array_equal(c2, cnt + extra)
    with pytest.raises(NotImplementedError, match="8 or more bytes"):
        a.export_device()
    # gram lengths beyond 15: the long-key table; its keys take counts_add too
    c = DeviceCounts(L, [2, 18])
    c.count(data, off, lang)
    lk, lc = c.export()
    okeys, ocnt = OC.count(data, off, lang, L, [2, 18])
    assert lk == okeys and np.array_equal(lc, ocnt)
    d = DeviceCounts(L, [1])
    d.add(lk, lc)
    d.add(lk[::3], lc[::3])
    dk, dc = d.export()
    extra = np.zeros_like(lc)
    extra[::3] = lc[::3]
    assert dk == lk and np.array_equal(dc, lc + extra)
    with pytest.raises(NotImplementedError, match="8 or more bytes"):
        c.export_device()


@pytest.mark.parametrize("grams", [[1, 2, 3], [2, 9]])
def test_sparse_export_ranges_and_add(grams):
    """ldgpu_counts_export_sparse / _add_sparse (the Scala shuffle payload):
    ranges of the (length, bytes) order carry each gram's nonzero (language,
    count) pairs; concatenated they equal the dense export, and adding them
    (twice, in ranges) into a fresh table doubles every count."""
    L = 7
    data, off, lang = _wide_corpus(grams, L, 99)
    a = DeviceCounts(L, grams)
    a.count(data, off, lang)
    keys, cnt = a.export()
    n = len(keys)
    b = DeviceCounts(L, grams)
    cuts = [0, 1, n // 3, n // 2, n]
    for first, last in zip(cuts[:-1], cuts[1:]):
        kb, ko, po, pl, pc = a.export_sparse(first, last - first)
        got = [kb[ko[i]:ko[i + 1]].tobytes() for i in range(last - first)]
        assert got == keys[first:last]
        for i in range(last - first):
            row = np.zeros(L, dtype=np.int64)
            row[pl[po[i]:po[i + 1]]] = pc[po[i]:po[i + 1]]
            assert np.array_equal(row, cnt[first + i])
            assert np.all(np.diff(pl[po[i]:po[i + 1]]) > 0)   # language order, no zero pairs
            assert np.all(pc[po[i]:po[i + 1]] > 0)
        b.add_sparse(kb, ko, po, pl, pc)
        b.add_sparse(kb, ko, po, pl, pc)
    k2, c2 = b.export()
    assert k2 == keys and np.array_equal(c2, 2 * cnt)
    with pytest.raises(ValueError, match="outside"):
        a.export_sparse(n, 1)


def test_bench_fit_two_ranks_merged_table_matches_oracle():
    """bench.py --mode fit --gpus 2 over the host transport (gloo; two ranks
    on this box's GPU): each rank counts its own GPU-drawn shard, the owner
    exchange sends sparse (gram, language, count) pairs, the distributed top-K
    builds the table; the merged table equals the top-K rule over the
    oracle's counts of both shards together."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, LDGPU_BENCH_BACKEND="gloo")
    out = os.path.join(root, "gpurun_out", "test_fit_world2.json")
    os.makedirs(os.path.dirname(out), exist_ok=True)
    cmd = [sys.executable, os.path.join(root, "bench.py"), "--mode", "fit", "--gpus", "2", "--fit-bytes", "3000000",
           "--steps", "1", "--warmup", "0", "--profile-size", "200", "--check-merge", "--json-out", out]
    r = subprocess.run(cmd, env=env, cwd=root, timeout=240, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads(open(out).read())
    assert line["n_gpus"] == 2
    assert line["merged_table_matches_oracle"] is True, line.get("merge_check")
    assert line["windows_counted_exactly_once"] is True


def _sparse_topk_masks(expect, L, K):
    """filterTopGrams over the oracle's sparse counts (kb, ko, po, pl, pc in
    (length, bytes, language) order): every gram in some language's top K by
    (v_l desc, index asc), as (keys, mask words [n][ceil(L/64)], values)."""
    kb, ko, po, pl, pc = expect
    n = len(ko) - 1
    k = np.diff(po)
    w = np.zeros(n)
    w[k > 0] = np.log(1.0 + 1.0 / k[k > 0])
    g = np.repeat(np.arange(n), k)
    order = np.lexsort((g, -w[g], pl))
    sl = pl[order]
    chosen = np.zeros(n, dtype=bool)
    starts = np.searchsorted(sl, np.arange(L + 1))
    for l in range(L):
        chosen[g[order[starts[l]:min(starts[l + 1], starts[l] + K)]]] = True
    idx = np.nonzero(chosen)[0]
    b = kb.tobytes()
    keys = [b[ko[i]:ko[i + 1]] for i in idx]
    words = (L + 63) // 64
    masks = np.zeros((len(idx), words), dtype=np.uint64)
    for j, i in enumerate(idx):
        for l in pl[po[i]:po[i + 1]]:
            masks[j, l // 64] |= np.uint64(1) << np.uint64(l % 64)
    return keys, masks, w[idx]


def test_config5_shape_fit_counts_table_and_scores():
    """Config 5's fit shape at test size -- L = 200, grams 1-7 (two-word
    records: the radix-sort + run-pass count), a ~10 MB corpus of 1-5 KB
    documents, K = 2000 -- through the product library: the sparse counts equal
    the C restatement's pair for pair, the mask-form top-K table equals the
    rule over those counts, and the model built from it labels (labels-only:
    class or replay mode) and scores (fp64 bits) like the oracle."""
    from languagedetection.runtime import DeviceModel
    L, grams, K = 200, [1, 2, 3, 4, 5, 6, 7], 2000
    ls = synth.make_languages(L)
    data, off, lang = synth.generate(ls, 3400, 1024, 5120, seed=synth.SEED_BASE + 5)
    counts = DeviceCounts(L, grams)
    counts.count(data, off, lang)
    got = counts.export_sparse()
    expect = OC.count_sparse(data, off, lang, L, grams, nthreads=8)
    assert len(got) == len(expect) and all(np.array_equal(a, b) for a, b in zip(got, expect))
    kb, ko, masks, vals = counts.fit_table_masks(K)
    counts.close()
    b = kb.tobytes()
    gkeys = [b[ko[i]:ko[i + 1]] for i in range(len(ko) - 1)]
    order = sorted(range(len(gkeys)), key=lambda i: (len(gkeys[i]), gkeys[i]))
    ekeys, emasks, evals = _sparse_topk_masks(expect, L, K)
    assert [gkeys[i] for i in order] == ekeys
    assert np.array_equal(masks[order], emasks)
    assert np.array_equal(np.asarray(vals)[order], evals)
    sdata, soff, _ = synth.generate(ls, 20000, 0, 300, seed=synth.SEED_BASE + 6)
    m = DeviceModel.from_masks(kb, ko, masks, vals, L, grams)
    t = OC.Table.from_masks(kb[:max(int(ko[-1]), 1)], ko, masks, vals, L)
    labels, _ = m.score(sdata, soff)
    ol, _ = t.score(grams, sdata, soff, nthreads=8)
    assert np.array_equal(labels, ol)
    n2 = 2000
    lab2, sc2 = m.score(sdata[:int(soff[n2])], soff[:n2 + 1], want_scores=True)
    ol2, os2 = t.score(grams, sdata[:int(soff[n2])], soff[:n2 + 1], want_scores=True, nthreads=8)
    assert np.array_equal(lab2, ol2) and np.array_equal(sc2.view(np.uint64), os2.view(np.uint64))
