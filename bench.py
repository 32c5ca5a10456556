"""Headline benchmark: SCORE throughput (BASELINE.json metric, config 2).

    python bench.py [--gpus N --steps K --warmup W]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

Workload (config 2 of BASELINE.json): 10M synthetic 256-byte documents per GPU,
20 languages, gram lengths 1-5, scored against a K=500 profile table that this
script first FITs on the GPU from a synthetic training corpus.  A step = one
pass of the SCORE kernel over the GPU's 10M resident documents (inputs already
in HBM).  Documents shard across ranks with no collective (weak scaling);
value = documents scored by all ranks / max-over-ranks time.

Also reported: the SCORE kernel's roofline position (algorithmic bytes / HIP
event time on the launch stream) and a CPU baseline (the oracle's C
restatement, multithreaded, on a bounded sample; kind "port" -- the Scala
reference cannot run without a JVM).
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "spark-languagedetector_amd"))

from languagedetection import _lib, synth  # noqa: E402
from languagedetection.runtime import DeviceCounts, DeviceModel  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
METRIC = "documents/sec scored (whole node, 1/2/4/8 GPU) + achieved HBM GB/s vs roofline"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", type=int, choices=[1, 2, 4, 5], default=2,
                    help="BASELINE.json config: 2 = headline (default), 4 = short text, 5 = large profile, "
                         "1 = the reference's own CPU-sized case (3 languages, 10k documents)")
    ap.add_argument("--docs", type=int, default=None, help="documents per GPU")
    ap.add_argument("--doc-bytes", type=int, default=None, help="fixed document length (sets min = max)")
    ap.add_argument("--doc-min", type=int, default=None)
    ap.add_argument("--doc-max", type=int, default=None)
    ap.add_argument("--langs", type=int, default=None)
    ap.add_argument("--grams", type=str, default=None)
    ap.add_argument("--profile-size", type=int, default=None)
    ap.add_argument("--pool", type=int, default=None,
                    help="distinct docs generated on the host and tiled to --docs (default: every document "
                         "distinct, drawn on the GPU)")
    ap.add_argument("--train-docs", type=int, default=None, help="training docs per language for the table")
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="target CPU-baseline sample time")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-host-path", action="store_true", help="skip the host-buffer (PCIe-inclusive) measurement")
    ap.add_argument("--no-alt-paths", action="store_true",
                    help="skip timing the same table on the ordered mask-replay path (diagnostics library)")
    ap.add_argument("--empty-table", action="store_true", help="calibration: table with no keys")
    ap.add_argument("--path", choices=["product", "replay"], default="product",
                    help="replay: time the ordered mask-replay path on the same table (diagnostics library, "
                         "LDGPU_NO_COUNT_MODE) instead of the product path -- for profiling, never the headline")
    ap.add_argument("--json-out", type=str, default="")
    ap.add_argument("--mode", choices=["score", "fit"], default="score",
                    help="score = the headline metric (config 2); fit = config 3's count + table build")
    ap.add_argument("--fit-bytes", type=int, default=6_250_000_000,
                    help="fit mode: corpus bytes per GPU (default: config 3's 50 GB over 8 GPUs)")
    ap.add_argument("--count-only", action="store_true",
                    help="fit mode: time the count alone, no top-K table (PMC passes of the count kernels)")
    ap.add_argument("--check-merge", action="store_true",
                    help="fit mode, N > 1: check the merged table against the oracle over every rank's corpus")
    args = ap.parse_args()
    # SURVEY §8d shapes; explicit flags override
    preset = {1: dict(docs=10_000, doc_min=128, doc_max=384, langs=3, grams="1,2,3", profile_size=1000,
                      train_docs=1000),
              2: dict(docs=10_000_000, doc_min=256, doc_max=256, langs=20, grams="1,2,3,4,5", profile_size=500,
                      train_docs=1000),
              4: dict(docs=125_000_000, doc_min=32, doc_max=96, langs=100, grams="1,2,3,4,5", profile_size=1000,
                      train_docs=300),
              5: dict(docs=10_000_000, doc_min=256, doc_max=256, langs=200, grams="1,2,3,4,5,6,7",
                      profile_size=50_000, train_docs=80)}[args.config]
    if args.doc_bytes is not None:
        args.doc_min = args.doc_max = args.doc_bytes
    for k, v in preset.items():
        if getattr(args, k) is None:
            setattr(args, k, v)
    args.doc_bytes = args.doc_min
    return args


def build_table(args, ls, device):
    """FIT on the GPU (the reference's LanguageDetector.fit path) -> the
    profile table in mask form (packed arrays), plus it as a {gram: row} dict
    when small enough for the CPU baseline."""
    grams = [int(x) for x in args.grams.split(",")]
    lang = np.repeat(np.arange(args.langs, dtype=np.int32), args.train_docs)
    data, off, lang = synth.generate(ls, len(lang), 200, 2000, seed=synth.SEED_BASE + 100, doc_lang=lang)
    t0 = time.perf_counter()
    counts = DeviceCounts(args.langs, grams, capacity_hint=1 << 20, device=device)
    counts.count(data, off, lang)
    n_distinct = counts.size()
    kb, ko, masks, vals = counts.fit_table_masks(args.profile_size)
    fit_s = time.perf_counter() - t0
    counts.close()
    n = len(ko) - 1
    table = None
    if n * args.langs <= 1_000_000:  # larger tables reach the CPU baseline as the packed arrays
        b = kb.tobytes()
        table = {}
        for i in range(n):
            row = [0.0] * args.langs
            for l in range(args.langs):
                if (int(masks[i, l // 64]) >> (l % 64)) & 1:
                    row[l] = float(vals[i])
            table[b[ko[i]:ko[i + 1]]] = row
    fit_info = {"train_docs": int(len(lang)), "train_bytes": int(off[-1]), "distinct_grams": int(n_distinct),
                "table_rows": int(n), "host_wall_s": round(fit_s, 3)}
    return (kb, ko, masks, vals), table, grams, fit_info


def host_cores() -> int:
    """The host cores this process may use (N = nproc of the
    allocation).  On the GPU pool the machine is shared and the allocation's
    share is published as OMP_NUM_THREADS (16 per GPU); elsewhere the CPU
    affinity mask."""
    env = os.environ.get("OMP_NUM_THREADS")
    if env and env.isdigit() and int(env) > 0:
        return int(env)
    try:
        return len(os.sched_getaffinity(0))
    except Exception:
        return int(os.cpu_count() or 1)


def cpu_baseline(args, table, grams, data, off, packed=None):
    """The oracle's C restatement (kind 'port'), on rank 0, bounded sample.
    The table comes as a {gram: row} dict, or (tables too large for one, as
    config 5's 10M rows x 200 languages) as the packed mask-form arrays."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import ldoracle_c as OC
    threads = host_cores()
    if table:
        t = OC.Table(table, args.langs)
    else:
        kb, ko, masks, vals = packed
        t = OC.Table.from_masks(kb[:max(int(ko[-1]), 1)], ko, masks, vals, args.langs)
    probe = min(20_000, len(off) - 1)
    t0 = time.perf_counter()
    t.score(grams, data, off[:probe + 1], nthreads=threads)
    rate = probe / max(time.perf_counter() - t0, 1e-9)
    n = int(min(len(off) - 1, max(probe, rate * args.cpu_seconds)))
    t0 = time.perf_counter()
    labels, _ = t.score(grams, data, off[:n + 1], nthreads=threads)
    dt = time.perf_counter() - t0
    # config 5's bytes model: the table hits per document (windows whose key
    # is in the table), from the first documents of the sample
    hits = None
    if args.config == 5:
        k = min(5000, len(off) - 1)
        hits = {"docs": k, "hits_per_doc": t.hits(grams, data, off[:k + 1]) / max(k, 1)}
    return {"value": round(n / dt, 1), "unit": "docs/s", "cores": threads, "kind": "port",
            "sample": f"first {n} of the GPU's documents ({args.doc_min}-{args.doc_max} B), same table, "
                      f"{threads} pthreads, {dt:.1f} s"}, labels, hits


def cpu_baseline_fit(args, grams, data, off, lang):
    """FIT on the oracle's C restatement (computeGrams per thread into private
    host hash tables, then reduceGrams as a hash-partitioned merge: kind
    'port', host_cores() pthreads, as the SCORE baseline), rank 0, bounded
    sample of the same corpus; unit = corpus bytes/s like the line's value.
    Also returns the sample's oracle counts in sparse form (key bytes, key
    offsets, pair offsets, languages, counts) for the parity check of the GPU
    path on the same documents."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import ldoracle_c as OC
    L = OC.lib()
    g = np.asarray(grams, dtype=np.int32)
    threads = host_cores()

    def run(n, keep=False):
        o = np.ascontiguousarray(off[:n + 1], dtype=np.int64)
        t0 = time.perf_counter()
        h = L.ldo_count_mt(OC._ptr(data), OC._ptr(o), OC._ptr(lang), n, args.langs, OC._ptr(g), len(g), threads)
        dt = time.perf_counter() - t0
        out = OC.export_sparse(h) if keep else None   # (gram, language) pairs: no dense row of L per gram
        L.ldo_counts_destroy(h)
        return dt, out

    probe = min(200 * threads, len(off) - 1)
    rate = int(off[probe]) / max(run(probe)[0], 1e-9)
    target = rate * args.cpu_seconds
    n = int(min(len(off) - 1, max(probe, np.searchsorted(off, target))))
    n = int(min(n, np.searchsorted(off, len(data), side="right") - 1))  # within the host copy of the corpus
    dt, exported = run(n, keep=True)
    return {"value": round(int(off[n]) / dt, 1), "unit": "bytes/s", "cores": threads, "kind": "port",
            "sample": f"first {n} documents ({int(off[n])} corpus bytes) of the GPU's corpus, "
                      f"oracle/ldoracle.c ldo_count_mt, {threads} pthreads, {dt:.1f} s"}, n, exported


def host_path(model, data, off, acc_labels):
    """The host-buffer boundary (ldgpu_score: the JNI shim's call), PCIe
    copies included -- reported beside `value`, never as it.  Pageable numpy
    buffers (staged through pinned memory) and ldgpu_host_alloc buffers."""
    from languagedetection.runtime import PinnedArray
    n = len(off) - 1
    res = {"note": "ldgpu_score over the same documents: H2D + score + D2H, 64 MiB chunks pipelined on two streams"}
    model.score(data[: int(off[min(n, 100000)])], off[: min(n, 100000) + 1])  # warm the staging buffers
    t0 = time.perf_counter()
    lab, _ = model.score(data, off)
    res["pageable_docs_per_s"] = round(n / (time.perf_counter() - t0), 1)
    pin = PinnedArray(len(data), np.uint8)
    pin.array[:] = data
    pout = PinnedArray(n, np.int32)
    model.score(pin.array, off, out=pout.array)
    t0 = time.perf_counter()
    model.score(pin.array, off, out=pout.array)
    res["pinned_docs_per_s"] = round(n / (time.perf_counter() - t0), 1)
    res["labels_match_device_path"] = bool(np.array_equal(lab, acc_labels) and np.array_equal(pout.array, acc_labels))
    pin.close()
    pout.close()
    return res


def mask_replay_path(args, packed, grams, local, d_bytes, n_bytes, d_off, n_docs, d_lab, stream):
    """Config 2's documents on the paths a table whose rows do NOT share one
    value takes (every mixed-presence-class fit table, every user mask
    table), each timed like `value` and reported beside it, never as it:
      - kernel_ms: the same table forced off count mode (diagnostics library,
        LDGPU_NO_COUNT_MODE): its labels-only call takes class mode (per-
        (value, language) hit counts + a rounding bound, ambiguous documents
        replayed in order); labels must equal count mode's;
      - ordered_kernel_ms: also LDGPU_NO_CLASS_MODE: the full ordered fp64
        replay of every verified hit (LanguageDetectorModel.scala:139-154);
      - two_values: the product library on the same table with every second
        row's value halved (two presence classes): class mode, its ambiguous
        share, labels against the C oracle on a sample."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    d_alt = torch.empty_like(d_lab)

    def timed(model):
        def step():
            model.score_device(d_bytes.data_ptr(), n_bytes, d_off.data_ptr(), n_docs, d_alt.data_ptr(), 0,
                               stream.cuda_stream)
        for _ in range(max(1, args.warmup)):
            step()
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
        for s_, e_ in ev:
            s_.record(stream)
            step()
            e_.record(stream)
        torch.cuda.synchronize()
        return float(np.mean([s_.elapsed_time(e_) for s_, e_ in ev]))

    def diag_model(env):
        os.environ.update(env)
        try:
            return DeviceModel.from_masks(*packed, args.langs, grams, device=local, variant="diag")
        finally:
            for k in env:
                del os.environ[k]

    res = {"library": "libldgpu_diag.so (LDGPU_NO_COUNT_MODE=1)"}
    alt = diag_model({"LDGPU_NO_COUNT_MODE": "1"})
    ms = timed(alt)
    res.update(table_mode={0: "mask", 1: "mask, finite values (fma replay)", 2: "dense"}.get(alt.info()["mode"]),
               layout=alt.info()["layout"], kernel_ms=round(ms, 4), docs_per_s=round(n_docs / (ms * 1e-3), 1),
               labels_match_count_mode=bool(torch.equal(d_alt, d_lab)))
    alt.close()
    alt = diag_model({"LDGPU_NO_COUNT_MODE": "1", "LDGPU_NO_CLASS_MODE": "1"})
    ms = timed(alt)
    res.update(ordered_kernel_ms=round(ms, 4), ordered_labels_match_count_mode=bool(torch.equal(d_alt, d_lab)))
    alt.close()
    # two presence classes on the product library
    import ldoracle_c as OC
    kb, ko, masks, vals = packed
    vals2 = np.array(vals, dtype=np.float64, copy=True)
    vals2[1::2] *= 0.5
    two = DeviceModel.from_masks(kb, ko, masks, vals2, args.langs, grams, device=local)
    ms = timed(two)
    sample = min(n_docs, 200_000)
    lab = d_alt[:sample].cpu().numpy()
    off_h = d_off[:sample + 1].cpu().numpy()
    data_h = d_bytes[:int(off_h[-1])].cpu().numpy()
    t = OC.Table.from_masks(kb[:max(int(ko[-1]), 1)], ko, masks, vals2, args.langs)
    ol, _ = t.score(grams, data_h, off_h, nthreads=host_cores())
    res["two_values"] = {"layout": two.info()["layout"], "kernel_ms": round(ms, 4),
                         "docs_per_s": round(n_docs / (ms * 1e-3), 1),
                         "labels_match_oracle": bool(np.array_equal(lab, ol)), "docs_checked": sample,
                         "note": "every second row's value halved: two distinct values, product library"}
    two.close()
    return res


def general_key_path(args, table, grams, local, d_bytes, d_off, n_docs, d_lab, stream):
    """A mixed table (a gram length beyond 15 bytes next to shorter ones):
    config 2's table plus one 16-byte key that valid UTF-8 never holds (0xff
    bytes), gram lengths + [16], over the first 1M documents -- lengths 1-5 on
    the count-mode kernel, the long-gram pass (ldgpu_general.hip) listing the
    documents a 16-byte window hits, those rescored by the general kernel: its
    time and whether its labels equal the count-mode launch's.  Reported
    beside `value`."""
    from languagedetection import LanguageDetectorModel
    t2 = dict(table)
    t2[b"\xff" * 16] = [next(iter(table.values()))[0] or 1.0] + [0.0] * (args.langs - 1)
    m = DeviceModel(t2, args.langs, grams + [16], device=local)
    n = min(n_docs, 1_000_000)
    nb = int(d_off[n].item())
    d_out = torch.empty(n, dtype=torch.int32, device=d_lab.device)

    def step():
        m.score_device(d_bytes.data_ptr(), nb, d_off.data_ptr(), n, d_out.data_ptr(), 0, stream.cuda_stream)
    step()
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(3)]
    for s_, e_ in ev:
        s_.record(stream)
        step()
        e_.record(stream)
    torch.cuda.synchronize()
    ms = float(np.mean([s_.elapsed_time(e_) for s_, e_ in ev]))
    res = {"layout": m.info()["layout"], "docs": n, "kernel_ms": round(ms, 4),
           "docs_per_s": round(n / (ms * 1e-3), 1), "labels_match_count_mode": bool(torch.equal(d_out, d_lab[:n])),
           "note": "config 2's table + one 16-byte key, gram lengths 1-5 and 16: lengths 1-5 on the LDS kernels, "
                   "the long-gram pass, documents with a long hit rescored on the general kernel"}
    m.close()
    # the static detect (LanguageDetectorModel.detect, one document per call,
    # the table cached across calls with the same map)
    lang_names = [f"l{i}" for i in range(args.langs)]
    k = 2000
    off_h = d_off[:k + 1].cpu().numpy()
    raw = d_bytes[:int(off_h[-1])].cpu().numpy().tobytes()
    docs = [raw[off_h[i]:off_h[i + 1]] for i in range(k)]
    t0 = time.perf_counter()
    first = LanguageDetectorModel.detect(docs[0], table, lang_names, grams)
    t_first = time.perf_counter() - t0
    t0 = time.perf_counter()
    got = [LanguageDetectorModel.detect(d, table, lang_names, grams) for d in docs]
    dt = time.perf_counter() - t0
    from languagedetection.api import freeze_table
    frozen = freeze_table(table)
    LanguageDetectorModel.detect(docs[0], frozen, lang_names, grams)
    t0 = time.perf_counter()
    got_f = [LanguageDetectorModel.detect(d, frozen, lang_names, grams) for d in docs]
    dt_f = time.perf_counter() - t0
    want = [lang_names[int(x)] for x in d_lab[:k].cpu().numpy()]
    res["static_detect"] = {"calls": k, "calls_per_s": round(k / dt, 1), "first_call_s": round(t_first, 4),
                            "frozen_calls_per_s": round(k / dt_f, 1),
                            "labels_match_count_mode": got == want and got_f == want and first == want[0],
                            "note": "LanguageDetectorModel.detect(bytes, map, languages, grams) per document; "
                                    "the device table is built on the first call and reused while the map's "
                                    "contents equal a snapshot (a dict compare per call); frozen_calls_per_s: "
                                    "the same map as a FrozenTable (reused by identity)"}
    return res


def traffic_from_profiles(workload_key):
    """HBM bytes per launch (per count, for FIT) from the committed rocprofv3
    PMC passes (profiles/pmc_traffic*.json), if they were collected for this
    exact workload (tools/pmc_traffic.py, tools/pmc_profile.sh)."""
    import glob
    import re
    docs_re = re.compile(r":docs=(\d+):")
    same_shape = None
    for p in sorted(glob.glob(os.path.join(ROOT, "profiles", "pmc_traffic*.json"))):
        try:
            d = json.load(open(p))
        except Exception:
            continue
        k = d.get("workload_key") or ""
        if k == workload_key:
            return d
        # the same score workload profiled over fewer documents: traffic
        # scales with the documents (the table is read once per launch and
        # is counted in the profiled launch's bytes, a slight overestimate)
        a, b = docs_re.search(k), docs_re.search(workload_key)
        if a and b and docs_re.sub(":", k) == docs_re.sub(":", workload_key):
            scale = int(b.group(1)) / int(a.group(1))
            same_shape = dict(d, traffic_bytes_per_launch=round(d["traffic_bytes_per_launch"] * scale),
                              traffic_scaled_from=f"{os.path.basename(p)} ({a.group(1)} docs, x{scale:g})")
    return same_shape


# the kernels of one count call (ldgpu_count): the traffic the count's time covers
COUNT_KERNELS = ("emit_kernel", "fit_offsets_kernel", "part2_kernel", "reduce_kernel", "merge_kernel",
                 "derive_level_kernel", "derive_pairs_level_kernel", "derive_pairs2_level_kernel", "len_hist_kernel",
                 "partial_kernel", "rehash_kernel", "wide_rehash_kernel", "sparse_rehash_kernel", "pair_rehash_kernel",
                 "counts_add_kernel", "sort_emit_kernel", "runs_count_kernel", "sort_runs_kernel", "runs_add_kernel")


def fit_sort_path(L, grams):
    """Whether the library counts (L, grams) by FIT v5 (ldgpu_api.hip
    counts_new / sort_path: two-word records whose sort key fits 64 bits --
    the radix sorts are then the count's own) or FIT v4 (no sort)."""
    maxg = max([g for g in grams if g <= 15] or [0])
    lb = max(1, (L - 1).bit_length())
    two_word = maxg <= 7 and 64 - (8 * maxg + 1) - lb < 8
    return bool(two_word and 8 * maxg + L.bit_length() <= 64)


def fit_count_kernels(L, grams):
    if fit_sort_path(L, grams):
        return "count (FIT v5: sort_emit + radix sort + runs_count + sort_runs per length group + runs_add into T)"
    return "count (FIT v4: emit + part2 + reduce + merge + derive)"


def is_count_kernel(name, L, grams):
    """A profiled kernel belongs to the count: one of COUNT_KERNELS, or a
    radix sort when the count is FIT v5's (FIT v4 sorts nothing; any other
    sort of a profiled run is an export's: sort_pairs_u64 in counts_pull)."""
    base = name.split("(")[0].split("<")[0]
    return base in COUNT_KERNELS or (base == "rocprim_radix_sort" and fit_sort_path(L, grams))


def count_traffic(prof, L, grams):
    """Calibrated HBM bytes per count from a FIT PMC profile
    (tools/fit_pmc.py), summed over the count's own kernels only."""
    if not prof:
        return None
    pk = prof.get("per_kernel_raw_bytes_per_count")
    if not pk:
        return prof.get("traffic_bytes_per_launch")
    rf, wf = prof.get("read_factor", 1.0), prof.get("write_factor", 1.0)
    tot = 0.0
    for k, v in pk.items():
        if is_count_kernel(k, L, grams):
            tot += rf * v.get("FETCH_SIZE", 0.0) + wf * v.get("WRITE_SIZE", 0.0)
    return int(round(tot))


def fit_corpus(args, ls, rank, dev):
    """This rank's config-3 shard: fit_bytes of 1-7 KB synthetic documents
    drawn on the GPU (synth.generate_device, seed per rank), untiled."""
    from languagedetection import synth as S
    n_docs = max(1, int(args.fit_bytes // 4096))  # U[1024, 7168]: 4096 B per document on average
    return S.generate_device(ls, n_docs, 1024, 7168, seed=S.SEED_BASE + 3 + 1000 * rank, device=dev)


def masks_to_table(kb, ko, masks, vals, L):
    """A mask-form fit table (DeviceCounts.fit_table_masks) as {gram: row}."""
    b = kb.tobytes()
    return {b[ko[i]:ko[i + 1]]: [float(vals[i]) if (int(masks[i, l // 64]) >> (l % 64)) & 1 else 0.0
                                 for l in range(L)] for i in range(len(ko) - 1)}


def topk_table_from_counts(kb, ko, cnt, K):
    """filterTopGrams (LanguageDetector.scala:100-132) over oracle counts (keys
    in (length, bytes) order): v_l = log(1 + [l] / k), per language the K
    largest v_l, ties by the key order -> {gram: row}."""
    pres = cnt > 0
    k = pres.sum(axis=1)
    w = np.zeros(len(k))
    w[k > 0] = np.log(1.0 + 1.0 / k[k > 0])
    chosen = np.zeros(len(k), dtype=bool)
    idx = np.arange(len(k))
    for l in range(cnt.shape[1]):
        v = np.where(pres[:, l], w, 0.0)
        chosen[np.lexsort((idx, -v))[:K]] = True
    b = kb.tobytes()
    return {b[ko[i]:ko[i + 1]]: [float(w[i]) if pres[i, l] else 0.0 for l in range(cnt.shape[1])]
            for i in np.nonzero(chosen)[0]}


def fit_main(args, world, rank, local, dev, backend):
    """Config 3 (FIT): count every window of a synthetic multilingual corpus
    (docs of 1-7 KB, drawn on the GPU, resident in HBM), merge across ranks
    (owner exchange of sparse (gram, language, count) pairs), build the
    K-profile table.  A step = one full fit."""
    from languagedetection.distributed import Communicator, merge_counts_device
    grams = [int(x) for x in args.grams.split(",")]
    comm = Communicator(device=local) if world > 1 else None
    ls = synth.make_languages(args.langs)
    d_bytes, d_off, d_lang = fit_corpus(args, ls, rank, dev)
    n_docs = len(d_off) - 1
    n_bytes = int(d_off[-1].item())
    off = d_off.cpu().numpy()
    stream = torch.cuda.current_stream(dev)
    torch.cuda.synchronize(dev)

    def step():
        t = {}
        t0 = time.perf_counter()
        c = DeviceCounts(args.langs, grams, capacity_hint=1 << 22, device=local)
        torch.cuda.synchronize(dev)
        t["create_s"] = time.perf_counter() - t0
        c.count_device(d_bytes.data_ptr(), n_bytes, d_off.data_ptr(), d_lang.data_ptr(), n_docs, stream.cuda_stream)
        torch.cuda.synchronize(dev)
        t["count_s"] = time.perf_counter() - t0 - t["create_s"]
        if world > 1:
            merge_counts_device(c, comm)   # owner exchange (RCCL with backend nccl)
            torch.cuda.synchronize(dev)
            t["merge_s"] = time.perf_counter() - t0 - t["create_s"] - t["count_s"]
        distinct = c.size()
        t1 = time.perf_counter()
        table = None if args.count_only else c.fit_table_masks(args.profile_size)  # packed mask form
        t["table_s"] = time.perf_counter() - t1
        t2 = time.perf_counter()
        c.close()
        t["close_s"] = time.perf_counter() - t2
        t["total_s"] = time.perf_counter() - t0
        return t, distinct, table

    def logged(tag):
        r = step()
        if rank == 0:  # progress on stderr (a long fit prints nothing else until its line)
            print(f"fit {tag}: count {r[0]['count_s']:.3f} s, total {r[0]['total_s']:.3f} s", file=sys.stderr, flush=True)
        return r

    for i in range(args.warmup):
        logged(f"warmup {i}")
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    parts = [logged(f"step {i}") for i in range(args.steps)]
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        tt = torch.tensor([elapsed], dtype=torch.float64, device=dev if backend == "nccl" else "cpu")
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
    count_s = float(np.mean([p[0]["count_s"] for p in parts]))
    windows = sum(int(synth_windows(off, n)) for n in grams)
    # one more count, untimed, for the table statistics: SURVEY §8d charges the
    # corpus byte, 12 B per document (offset + language id) and 16 B per
    # distinct (gram, language) count written
    c = DeviceCounts(args.langs, grams, capacity_hint=1 << 22, device=local)
    c.count_device(d_bytes.data_ptr(), n_bytes, d_off.data_ptr(), d_lang.data_ptr(), n_docs, stream.cuda_stream)
    torch.cuda.synchronize(dev)
    st = c.stats()
    c.close()
    windows_ok = st["total"] == windows   # every window counted exactly once
    algo = n_bytes + 12 * n_docs + 16 * st["pairs"]
    line = {
        "metric": "corpus bytes/sec fitted (config 3: count + merge + probability/top-K table)",
        "value": round(n_bytes * world * args.steps / elapsed, 1), "unit": "bytes/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(elapsed * 1e3 / args.steps, 3),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u64 (integer counts)",
        "data": "synthetic (Markov-chain text per language, docs 1-7 KB, drawn on the GPU, untiled)",
        "config": {"workload": f"config3: fit {n_bytes} corpus bytes per GPU, {args.langs} languages, "
                               f"grams {args.grams}, profile size {args.profile_size}",
                   "docs_per_gpu": n_docs, "corpus_bytes_per_gpu": n_bytes, "windows_per_gpu": windows,
                   "distinct_grams": parts[-1][1], "distinct_gram_language_pairs": st["pairs"],
                   "table_rows": None if args.count_only else len(parts[-1][2][1]) - 1,
                   "parallelism": f"dp{world} (corpus sharded; owner-exchange merge + distributed top-K)"},
        "phases_s": {k: round(float(np.mean([p[0].get(k, 0.0) for p in parts])), 4)
                     for k in ("create_s", "count_s", "merge_s", "table_s", "close_s", "total_s")},
        "count_s_per_step": [round(float(p[0].get("count_s", 0.0)), 4) for p in parts],
        "table_s_per_step": [round(float(p[0].get("table_s", 0.0)), 4) for p in parts],
        "count_windows_per_s": round(windows / count_s, 1),
        "count_ms_per_gib": round(count_s * 1e3 * (1 << 30) / n_bytes, 2),
        "windows_counted_exactly_once": windows_ok,
        "roofline": {"bound": "hbm", "achieved": round(algo / count_s / 1e9, 3), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(algo / count_s / 1e9 / HBM_PEAK_GBS, 6),
                     "traffic": count_traffic(traffic_from_profiles(f"fit:bytes={n_bytes}:L={args.langs}:G={args.grams}"),
                                              args.langs, grams),
                     "kernel": fit_count_kernels(args.langs, grams), "count_ms": round(count_s * 1e3, 3),
                     "algorithmic_bytes_per_count": int(algo)},
    }
    if line["roofline"]["traffic"]:  # the counters' view: calibrated HBM bytes per count over the count time
        tgbs = line["roofline"]["traffic"] / count_s / 1e9
        line["roofline"]["traffic_GBps"] = round(tgbs, 1)
        line["roofline"]["traffic_frac"] = round(tgbs / HBM_PEAK_GBS, 4)
    if world > 1 and args.check_merge:
        # every rank's corpus regenerated on this GPU (same seeds), counted by
        # the oracle; the merged table (the same on every rank) must equal the
        # top-K rule over those global counts
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import ldoracle_c as OC
        datas, offs, langs = [], [], []
        base = 0
        for r in range(world):
            b_, o_, l_ = fit_corpus(args, ls, r, dev)
            o_ = o_.cpu().numpy()
            datas.append(b_[:int(o_[-1])].cpu().numpy())
            offs.append(o_[1:] + base if r else o_ + base)
            base += int(o_[-1])
            langs.append(l_.cpu().numpy())
        okeys, ocnt = OC.count(np.concatenate(datas), np.concatenate(offs), np.concatenate(langs), args.langs, grams)
        kb = np.frombuffer(b"".join(okeys), dtype=np.uint8)
        ko = np.zeros(len(okeys) + 1, dtype=np.int64)
        np.cumsum([len(k) for k in okeys], out=ko[1:])
        expect = topk_table_from_counts(kb, ko, ocnt, args.profile_size)
        line["merged_table_matches_oracle"] = bool(masks_to_table(*parts[-1][2], args.langs) == expect)
        line["merge_check"] = {"ranks": world, "global_grams": len(okeys), "table_rows": len(expect)}
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        data_h = d_bytes[:min(n_bytes, 256 << 20)].cpu().numpy()
        lang_h = d_lang.cpu().numpy()
        line["cpu_baseline"], n_s, expect = cpu_baseline_fit(args, grams, data_h, off, lang_h)
        # the GPU count of the same sample documents against the oracle's, as
        # sorted (gram, language, count) pairs
        c = DeviceCounts(args.langs, grams, device=local)
        c.count_device(d_bytes.data_ptr(), n_bytes, d_off.data_ptr(), d_lang.data_ptr(), n_s, stream.cuda_stream)
        torch.cuda.synchronize(dev)
        got = c.export_sparse()
        c.close()
        ok = len(got) == len(expect) and all(np.array_equal(a, b) for a, b in zip(got, expect))
        line["counts_match_oracle"] = bool(ok)
        line["oracle_check"] = {"docs_checked": int(n_s), "grams_checked": int(len(expect[1]) - 1),
                                "pairs_checked": int(len(expect[3]))}
    line["build"] = _lib.provenance()  # the loaded library's source hash against this tree's
    if rank == 0:
        print(json.dumps(line), flush=True)
        if args.json_out:
            with open(args.json_out, "w") as f:
                f.write(json.dumps(line) + "\n")
    if world > 1:
        dist.destroy_process_group()


def synth_windows(off, n):
    lens = np.diff(off)
    return np.where(lens == 0, 0, np.where(lens < n, 1, lens - n + 1)).sum()


def launch_ranks(args):
    """`--gpus N` without a launcher: start N rank processes (one per GPU,
    torch.distributed.run on 127.0.0.1) as CHILDREN -- before this process
    touches the GPU -- and exit with their status.  Under a launcher the
    world size must equal --gpus."""
    world_env = os.environ.get("WORLD_SIZE")
    if world_env is not None:
        if int(world_env) != args.gpus:
            sys.exit(f"bench.py: --gpus {args.gpus} but the launcher started WORLD_SIZE={world_env} ranks")
        return
    if args.gpus <= 1:
        return
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    sys.exit(subprocess.call(cmd))


def main():
    args = parse()
    launch_ranks(args)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # one process per GPU; the modulo only matters when rehearsing several
    # ranks on a one-GPU box (with LDGPU_BENCH_BACKEND=gloo)
    local = local % max(torch.cuda.device_count(), 1)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    backend = os.environ.get("LDGPU_BENCH_BACKEND", "nccl")
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)
    if args.mode == "fit":
        return fit_main(args, world, rank, local, dev, backend)

    ls = synth.make_languages(args.langs)
    packed = None
    if args.empty_table:
        table, grams, fit_info = {}, [int(x) for x in args.grams.split(",")], {}
        model = DeviceModel(table, args.langs, grams, device=local)
    else:
        packed, table, grams, fit_info = build_table(args, ls, local)
        if args.path == "replay":
            os.environ["LDGPU_NO_COUNT_MODE"] = "1"
            model = DeviceModel.from_masks(*packed, args.langs, grams, device=local, variant="diag")
            del os.environ["LDGPU_NO_COUNT_MODE"]
        else:
            model = DeviceModel.from_masks(*packed, args.langs, grams, device=local)

    # this rank's documents, resident in HBM: every one distinct, drawn on the
    # GPU (synth.generate_device), or (--pool) a host-generated pool tiled
    if args.pool is None:
        pool = args.docs
        d_bytes, d_off, d_plang = synth.generate_device(ls, args.docs, args.doc_min, args.doc_max,
                                                        seed=synth.SEED_BASE + args.config + 1000 * rank, device=dev,
                                                        chunk_docs=1 << 20)
        off = d_off.cpu().numpy()
        n_bytes = int(off[-1])
        data = d_bytes[:n_bytes].cpu().numpy()
        plang = d_plang.cpu().numpy()
        del d_plang
    else:
        pool = min(args.pool, args.docs)
        pdata, poff, plang = synth.generate(ls, pool, args.doc_min, args.doc_max,
                                            seed=synth.SEED_BASE + args.config + 1000 * rank)
        data, off, _ = synth.tile(pdata, poff, plang, args.docs)
        n_bytes = int(off[-1])
        d_bytes = torch.empty(((n_bytes + 3) // 4) * 4 + 16, dtype=torch.uint8, device=dev)
        d_bytes[:n_bytes].copy_(torch.from_numpy(data))
        d_off = torch.from_numpy(off).to(dev)
    n_docs = len(off) - 1
    d_lab = torch.empty(n_docs, dtype=torch.int32, device=dev)
    stream = torch.cuda.current_stream(dev)

    def step():
        model.score_device(d_bytes.data_ptr(), n_bytes, d_off.data_ptr(), n_docs, d_lab.data_ptr(), 0,
                           stream.cuda_stream)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    t0 = time.perf_counter()
    for s, e in ev:
        s.record(stream)
        step()
        e.record(stream)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    kernel_ms = float(np.mean([s.elapsed_time(e) for s, e in ev]))
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev if backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    # labels sanity (synthetic docs carry their generating language)
    acc = float((d_lab[:pool].cpu().numpy() == plang[:pool]).mean()) if (table or packed) else None

    info = model.info()
    doc_b = n_bytes / max(n_docs, 1)                      # mean document bytes
    windows = int(sum(synth_windows(off, n) for n in grams))

    cpu = None
    oracle_check = None
    hits = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline and (table or packed):
        cpu, ol, hits = cpu_baseline(args, table, grams, data, off, packed)
        # the timed kernel's own labels (the last step's) against the oracle's
        # on the CPU sample: the exact code path the value measures
        dl = d_lab[:len(ol)].cpu().numpy()
        oracle_check = {"labels_match_oracle": bool(np.array_equal(dl, ol)), "docs_checked": int(len(ol)),
                        "mismatches": int((dl != ol).sum())}

    algo_per_launch = n_bytes + 12 * n_docs               # bytes + int64 offset + int32 label
    algo_per_launch += info["device_bytes"]               # the table, read once per launch (amortised)
    survey_algo = algo_per_launch + 64 * windows          # SURVEY §8d's notional 64-B sector per window probe
    model_note = None
    if args.config == 5:
        # table far beyond LDS / L2: the bytes THIS design must move (keyed
        # bloom, line layout: one 64-B line per window position for length 3's
        # word and one for lengths 4..7 together; the 1-/2-byte tests are LDS
        # bitmaps) plus one 64-B bucket line per table hit (a hit must be
        # verified; false candidates are the filter's waste, not counted)
        lens = set(grams)
        lines = 0
        if 3 in lens:
            lines += synth_windows(off, 3)
        g47 = [n for n in lens if 4 <= n <= 7]
        if g47:
            lines += synth_windows(off, min(g47))
        algo_per_launch += 64 * int(lines)
        if hits:
            algo_per_launch += int(64 * hits["hits_per_doc"] * n_docs)
        model_note = (f"algorithmic bytes: corpus + 12 B/doc + the table once + one 64-B bloom line per window "
                      f"position per length group ({int(lines)} lines) + one 64-B bucket line per table hit "
                      f"({'%.1f' % hits['hits_per_doc'] if hits else 'not measured'} per doc, C oracle on the first "
                      f"{hits['docs'] if hits else 0} docs); survey_frac: SURVEY 8d's 64 B per window probe")
    achieved = algo_per_launch / (kernel_ms * 1e-3) / 1e9
    workload_key = (f"score:docs={n_docs}:bytes={args.doc_min}-{args.doc_max}:L={args.langs}:G={args.grams}"
                    f":K={args.profile_size}")
    if args.config == 2:
        workload_key = f"score:docs={n_docs}:bytes={args.doc_min}:L={args.langs}:G={args.grams}:K={args.profile_size}"
    prof = traffic_from_profiles(workload_key) or {}
    roofline = {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": prof.get("traffic_bytes_per_launch"),
                # TCC hit / (hit + miss) of the same launch (tools/pmc_traffic.sh)
                "l2_hit_rate": (prof.get("l2") or {}).get("hit_rate"), "workload_key": workload_key,
                "traffic_scaled_from": prof.get("traffic_scaled_from"),
                "kernel_ms": round(kernel_ms, 4), "algorithmic_bytes_per_launch": int(algo_per_launch),
                "lookups_per_s": round(windows / (kernel_ms * 1e-3), 1)}
    if args.config == 5:
        roofline["note"] = model_note
        roofline["survey_algorithmic_bytes_per_launch"] = int(survey_algo)
        roofline["survey_frac"] = round(survey_algo / (kernel_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 5)
        roofline["table_hits_per_doc"] = hits["hits_per_doc"] if hits else None
    # the counters' view beside SURVEY's algorithmic one: calibrated HBM bytes
    # per launch over the kernel time, as a fraction of the same peak
    if roofline["traffic"]:
        tgbs = roofline["traffic"] / (kernel_ms * 1e-3) / 1e9
        roofline["traffic_GBps"] = round(tgbs, 1)
        roofline["traffic_frac"] = round(tgbs / HBM_PEAK_GBS, 4)

    alt = None
    if rank == 0 and world == 1 and args.config == 2 and not args.no_alt_paths and not args.empty_table:
        alt = mask_replay_path(args, packed, grams, local, d_bytes, n_bytes, d_off, n_docs, d_lab, stream)
    general = None
    if rank == 0 and world == 1 and args.config == 2 and not args.no_alt_paths and table:
        general = general_key_path(args, table, grams, local, d_bytes, d_off, n_docs, d_lab, stream)
    host = None
    if rank == 0 and world == 1 and not args.no_host_path and not args.empty_table:
        host = host_path(model, data, off, acc_labels=d_lab.cpu().numpy())

    total_docs = n_docs * world * args.steps
    doc_desc = f"{args.doc_min} B" if args.doc_min == args.doc_max else f"U[{args.doc_min},{args.doc_max}] B"
    if args.path == "replay":
        line_note = "profiling run: the ordered mask-replay path (diagnostics library), not the product path"
    elif args.config != 2:
        line_note = {1: "config 1: the reference's CPU-sized case (SURVEY §8d), timed beside its CPU restatement",
                     4: "config 4 is quoted on 1B docs over 8 GPUs (1.25e8 per GPU); --docs sets this run's count",
                     5: "config 5: table of up to L*K rows far beyond LDS: bloom in L2/MALL, slots in HBM"}[args.config]
    else:
        line_note = None
    line = {
        "metric": METRIC,
        "value": round(total_docs / elapsed, 1),
        "unit": "docs/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed * 1e3 / args.steps, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": ("synthetic (Markov-chain text per language, SURVEY.md §8d generator; table FIT on the GPU; "
                 + ("every document distinct, drawn on the GPU)" if args.pool is None
                    else f"a pool of {pool} documents tiled)")),
        "config": {"workload": f"config{args.config}: score {n_docs} x {doc_desc} docs per GPU, {args.langs} "
                               f"languages, grams {args.grams}, profile size {args.profile_size}",
                   "docs_per_gpu": n_docs, "doc_bytes": round(doc_b, 2), "languages": args.langs,
                   "gram_lengths": grams,
                   "profile_size": args.profile_size, "table_rows": info["n_keys"],
                   "table_mode": {0: "mask", 1: "dense", 2: "mask, one shared value (hit counts)"}[info["mode"]],
                   "parallelism": f"dp{world} (documents sharded, no collective)"},
        "roofline": roofline,
        "cpu_baseline": cpu,
        "labels_match_oracle": None if oracle_check is None else oracle_check["labels_match_oracle"],
        "oracle_check": oracle_check,
        "host_path": host,
        "mask_replay_path": alt,
        "general_keys_path": general,
        "fit_setup": fit_info,
        "label_accuracy_vs_generator": acc,
    }
    if line_note:
        line["note"] = line_note
    # build provenance: the loaded library's source hash against this tree's
    line["build"] = _lib.provenance()
    model.close()
    if rank == 0:
        s = json.dumps(line)
        print(s, flush=True)
        if args.json_out:
            with open(args.json_out, "w") as f:
                f.write(s + "\n")
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
