"""Multi-process paths (world size 2, gloo on 127.0.0.1): the FIT merge
(owner exchange, ldgpu_counts_merge) and sharded scoring.  The CPU test runs
the owner-exchange protocol on the C oracle's per-shard counts; the gpu tests
run the library's merge + distributed top-K from two ranks on cuda:0 (host
transport over gloo) and the RCCL transport at world size 1."""
import os
import socket
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

from conftest import ROOT


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _init(rank, world, port):
    import torch.distributed as dist
    for p in (os.path.join(ROOT, "spark-languagedetector_amd"), os.path.join(ROOT, "oracle")):
        if p not in sys.path:
            sys.path.insert(0, p)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    return dist


def _corpus():
    from languagedetection import synth
    ls = synth.make_languages(6, seed=21)
    return ls, synth.generate(ls, 500, 0, 300, seed=22)


def _merge_worker(rank, world, port, out_dir):
    dist = _init(rank, world, port)
    import ldoracle_c as OC
    from languagedetection.distributed import merge_counts, shard_range
    ls, (data, off, lang) = _corpus()
    lo, hi = shard_range(len(off) - 1, rank, world)
    sub_off = off[lo:hi + 1] - off[lo]
    sub = data[off[lo]:off[hi]]
    keys, cnt = OC.count(sub, sub_off, lang[lo:hi], 6, [1, 2, 3])
    gk, gc = merge_counts(keys, cnt, 6)   # this rank's owned grams, global counts
    np.save(os.path.join(out_dir, f"counts{rank}.npy"), gc)
    with open(os.path.join(out_dir, f"keys{rank}.bin"), "wb") as f:
        for k in gk:
            f.write(bytes([len(k)]) + k)
    dist.barrier()
    dist.destroy_process_group()


def _read_keys(path):
    b = open(path, "rb").read()
    out, i = [], 0
    while i < len(b):
        n = b[i]
        out.append(b[i + 1:i + 1 + n])
        i += 1 + n
    return out


def test_merge_counts_two_ranks(tmp_path):
    """The ranks' owned shards partition the global table: disjoint, every
    gram on its owner (distributed.owner_of), counts equal to the oracle's
    single-process counts."""
    import ldoracle_c as OC
    from languagedetection.distributed import owner_of, packed_keys
    mp.spawn(_merge_worker, args=(2, free_port(), str(tmp_path)), nprocs=2, join=True)
    ls, (data, off, lang) = _corpus()
    keys, cnt = OC.count(data, off, lang, 6, [1, 2, 3])
    got = {}
    for r in range(2):
        rk = _read_keys(os.path.join(tmp_path, f"keys{r}.bin"))
        rc = np.load(os.path.join(tmp_path, f"counts{r}.npy"))
        assert (owner_of(packed_keys(rk), 2) == r).all()
        for k, row in zip(rk, rc):
            assert k not in got
            got[k] = row
    assert sorted(got, key=lambda k: (len(k), k)) == keys
    assert np.array_equal(np.array([got[k] for k in keys]), cnt)


def test_sort_keys_roundtrip_and_order():
    from languagedetection.distributed import keys_of, shard_range, sort_keys
    ks = [b"b", b"a", b"ab", b"\xff", b"zzzzzzz", b"\x00\x01"]
    codes = sort_keys(ks)
    assert keys_of(codes) == ks
    order = [ks[i] for i in np.argsort(codes, kind="stable")]
    assert order == sorted(ks, key=lambda k: (len(k), k))
    cover = [shard_range(10, r, 3) for r in range(3)]
    assert cover == [(0, 3), (3, 6), (6, 10)]


def _fit_worker(rank, world, port, out_dir, K, grams, transport):
    dist = _init(rank, world, port)
    from languagedetection import synth
    from languagedetection.api import LanguageDetector
    from languagedetection.distributed import Communicator, merge_counts_device, shard_range
    ls, (data, off, lang) = _corpus()
    rows = list(zip([ls.names[i] for i in lang], synth.texts(data, off)))
    lo, hi = shard_range(len(rows), rank, world)
    local = LanguageDetector.count_grams(rows[lo:hi], grams, ls.names, device=0)
    comm = Communicator(device=0, transport=transport)
    merge_counts_device(local, comm)
    keys, cnt = local.export()      # this rank's owned shard, global counts
    table = local.fit_table(K)      # collective: the global table on every rank
    local.close()
    comm.close()
    import json
    with open(os.path.join(out_dir, f"table{rank}.json"), "w") as f:
        json.dump({"table": {k.hex(): v for k, v in table.items()},
                   "counts": {k.hex(): c.tolist() for k, c in zip(keys, cnt)}}, f)
    dist.barrier()
    dist.destroy_process_group()


def _check_fit(tmp_path, world, K, grams):
    import json
    import ldoracle as O
    import ldoracle_c as OC
    from languagedetection import synth
    ls, (data, off, lang) = _corpus()
    rows = list(zip([ls.names[i] for i in lang], synth.texts(data, off)))
    expect = O.filter_top_grams(O.fit_probabilities(rows, ls.names, grams), ls.names, K)
    okeys, ocnt = OC.count(data, off, lang, 6, grams)
    counts = {}
    for r in range(world):
        d = json.load(open(os.path.join(tmp_path, f"table{r}.json")))
        got = {bytes.fromhex(k): v for k, v in d["table"].items()}
        assert got == expect
        for k, c in d["counts"].items():
            assert k not in counts      # owned shards are disjoint
            counts[k] = c
    assert len(counts) == len(okeys)
    assert all(counts[k.hex()] == ocnt[i].tolist() for i, k in enumerate(okeys))


@pytest.mark.gpu
@pytest.mark.parametrize("K,grams", [(80, [1, 2, 3]), (5000, [2, 3]), (60, [2, 9]), (5000, [1, 8, 12]),
                                     (60, [2, 17]), (5000, [1, 16, 9])])
def test_fit_distributed_matches_single_process(tmp_path, K, grams):
    """Two ranks (cuda:0 each), host transport over gloo: the library's owner
    exchange leaves disjoint shards with the oracle's global counts, and the
    distributed top-K gives every rank the oracle's table -- also with K above
    some language's present grams (the zero-valued fill), and with gram
    lengths 8..15 (wide grams) or beyond (long grams): every rank's entries
    all-gathered, each rank keeping those it owns; the top-K over every rank's
    presence rows."""
    mp.spawn(_fit_worker, args=(2, free_port(), str(tmp_path), K, grams, "host"), nprocs=2, join=True)
    _check_fit(tmp_path, 2, K, grams)


@pytest.mark.gpu
@pytest.mark.parametrize("grams", [[1, 2, 3], [2, 9]])
def test_fit_merge_rccl_transport_world1(tmp_path, grams):
    """The RCCL transport (ncclCommInitRank, grouped ncclSend/ncclRecv,
    ncclAllGather) at world size 1, the only size one GPU allows."""
    mp.spawn(_fit_worker, args=(1, free_port(), str(tmp_path), 80, grams, "rccl"), nprocs=1, join=True)
    _check_fit(tmp_path, 1, 80, grams)


def _fail_worker(rank, world, port, out_dir, K, grams, point):
    """A merged table's top-K with rank 1 failing at `point` (diagnostics
    library, LDGPU_FAIL_AT): every rank must return an error, none may wait."""
    dist = _init(rank, world, port)
    from languagedetection import synth
    from languagedetection.distributed import Communicator, merge_counts_device, shard_range
    from languagedetection.runtime import DeviceCounts
    ls, (data, off, lang) = _corpus()
    lo, hi = shard_range(len(off) - 1, rank, world)
    local = DeviceCounts(6, grams, device=0, variant="diag")
    local.count(data[off[lo]:off[hi]], off[lo:hi + 1] - off[lo], lang[lo:hi])
    comm = Communicator(device=0, transport="host", variant="diag")
    merge_counts_device(local, comm)
    if rank == 1:
        os.environ["LDGPU_FAIL_AT"] = point
    try:
        local.fit_table(K)
        msg = "no error"
    except Exception as e:  # noqa: BLE001 -- the test reads the message
        msg = f"{type(e).__name__}: {e}"
    os.environ.pop("LDGPU_FAIL_AT", None)
    with open(os.path.join(out_dir, f"err{rank}.txt"), "w") as f:
        f.write(msg)
    local.close()
    comm.close()
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.parametrize("point,K,grams", [("table_hist", 80, [1, 2, 3]), ("table_select", 80, [1, 2, 3]),
                                           ("table_rows", 80, [1, 2, 3]), ("table_fallback", 5000, [2, 3]),
                                           ("table_wide", 60, [2, 9])])
def test_fit_table_rank_failure_ends_every_rank(tmp_path, point, K, grams):
    """The distributed top-K (LanguageDetector.scala:107-130 across ranks)
    agrees every rank's status before each of its collectives: rank 1 fails
    inside ldgpu_fit_table_size (injected at each phase: histogram, select,
    chosen rows; the zero-fill and wide-gram host selections), and both ranks
    return an error -- rank 1 its own, rank 0 naming rank 1 -- with no hang
    (a 120 s bound here; a rank left waiting in an all-gather would hold it)."""
    import time
    ctx = mp.spawn(_fail_worker, args=(2, free_port(), str(tmp_path), K, grams, point), nprocs=2, join=False)
    deadline = time.time() + 120
    while not ctx.join(timeout=5):
        if time.time() > deadline:
            for p in ctx.processes:
                p.kill()
            pytest.fail(f"ranks still running 120 s after a failure at {point}")
    e0 = open(os.path.join(tmp_path, "err0.txt")).read()
    e1 = open(os.path.join(tmp_path, "err1.txt")).read()
    assert f"injected failure at {point}" in e1, e1
    assert "fit table: rank 1 failed" in e0, e0


def _score_worker(rank, world, port, out_dir):
    dist = _init(rank, world, port)
    from languagedetection import LanguageDetectorModel, synth
    from languagedetection.distributed import score_sharded
    ls = synth.make_languages(5, seed=71)
    data, off, _ = synth.generate(ls, 3001, 0, 300, seed=72)
    table = {b"a": [0.5, 0.0, 0.0, 0.0, 0.1], b"th": [0.0, 1.0, 0.0, 0.0, 0.0], b"ing": [0.0, 0.0, 0.3, 0.3, 0.0]}
    model = LanguageDetectorModel(table, [1, 2, 3], ls.names, device=0)
    labels = score_sharded(model, synth.texts(data, off))
    np.save(os.path.join(out_dir, f"labels{rank}.npy"), labels)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.gpu
def test_score_sharded_two_ranks(tmp_path):
    """SCORE data parallelism: each rank scores its contiguous
    share, no collective on the data path; the all_gathered labels equal the
    oracle's over the whole (odd-sized) set on every rank."""
    import ldoracle as O
    from languagedetection import synth
    mp.spawn(_score_worker, args=(2, free_port(), str(tmp_path)), nprocs=2, join=True)
    ls = synth.make_languages(5, seed=71)
    data, off, _ = synth.generate(ls, 3001, 0, 300, seed=72)
    table = {b"a": [0.5, 0.0, 0.0, 0.0, 0.1], b"th": [0.0, 1.0, 0.0, 0.0, 0.0], b"ing": [0.0, 0.0, 0.3, 0.3, 0.0]}
    expect = [O.argmax_first(O.detect_scores(O.score_encode(t), table, 5, [1, 2, 3])) for t in synth.texts(data, off)]
    for r in range(2):
        assert np.load(os.path.join(tmp_path, f"labels{r}.npy")).tolist() == expect


def test_bench_refuses_mismatched_world_size():
    """--gpus must equal the launcher's WORLD_SIZE (no silent one-GPU run)."""
    import subprocess
    env = dict(os.environ, WORLD_SIZE="3", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"], env=env,
                       capture_output=True, text=True, timeout=120)
    assert r.returncode != 0 and "WORLD_SIZE=3" in r.stderr


@pytest.mark.gpu
def test_bench_gpus2_launches_two_ranks():
    """bench.py --gpus 2 without a launcher starts two rank processes (gloo
    rehearsal on one GPU: both ranks on cuda:0) and reports n_gpus 2 with
    weak-scaling accounting (value = docs of both ranks / max-rank time)."""
    import json
    import subprocess
    env = dict(os.environ, LDGPU_BENCH_BACKEND="gloo")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "3",
                        "--warmup", "1", "--docs", "200000", "--pool", "20000", "--no-cpu-baseline",
                        "--no-host-path"], env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    line = json.loads([x for x in r.stdout.splitlines() if x.startswith("{")][-1])
    assert line["n_gpus"] == 2 and line["scaling"] == "weak"
    assert line["config"]["docs_per_gpu"] == 200000
    assert abs(line["value"] - 2 * 200000 * 3 / (line["ms_per_step"] * 3 / 1e3)) / line["value"] < 1e-3
