"""Multi-GPU plumbing on CPU (no GPU needed):

* bench.py --gpus N is a launcher: it starts N ranks as child processes
  (torch.distributed.run) and the ranks report n_gpus = N; --dry-run runs the
  ranks' control plane and bitmap gather over gloo without a GPU;
* libstl's shard functions (stl_shard_range / stl_shard_range_bytes, which
  the host batch calls and the RCCL gather use) equal the Python mirror;
* byte-balanced shards of variable-length rows (config 5) over 2 gloo ranks
  reassemble exactly the single-rank bitmap (oracle as the per-rank checker:
  this box has no GPU);
* stl_init checks its configuration before it looks for a device.
Reference parallelism being replaced: the JobQueue thread pool,
src/ripple_core/functional/JobQueue.cpp:217-243."""
import ctypes
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np
import pytest
import torch.multiprocessing as mp

from stellard_amd import shard

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _last_json(out):
    for line in reversed(out.strip().splitlines()):
        line = line.strip()
        if line.startswith("{"):
            return json.loads(line)
    raise AssertionError(f"no JSON line in output:\n{out}")


@pytest.mark.parametrize("gpus", [1, 2])
def test_bench_launcher_dry_run(gpus):
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(gpus), "--dry-run",
                        "--steps", "2", "--warmup", "1", "--per-gpu", "4160"],
                       capture_output=True, text=True, timeout=240, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    line = _last_json(r.stdout)
    assert line["n_gpus"] == gpus and line["dry_run"] is True
    assert line["steps"] == 2 and line["warmup"] == 1 and line["scaling"] == "weak"
    assert line["config"]["gathered_all_ones"] is True
    assert line["config"]["rank0_shard"] == [0, 4160]
    assert line["config"]["rccl_nranks"] == gpus  # the GPU run reads it from libstl's stl_comm_info
    assert line["metric"].startswith("DRY RUN")


@pytest.mark.parametrize("gpus,fault", [(1, None), (2, None), (4, None), (2, "shift"), (2, "dup"), (4, "zero")])
def test_bench_digest_rehearsal_catches_bad_gather(gpus, fault):
    """the multi-rank legs must be able to FAIL.  The dry run
    runs tools/bench_legs.py's sharding (whole 65,536-row blocks, unequal at
    10M rows), gather and digest check over gloo with a fixed accept pattern;
    shifting rank 1's words, replacing them with rank 0's slice or zeroing them
    must turn digest_equal false, the clean run must keep it true."""
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(gpus), "--dry-run", "--steps", "1",
           "--warmup", "0", "--per-gpu", "4096"]
    if fault:
        cmd += ["--dry-run-fault", fault]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=240, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    leg = _last_json(r.stdout)["extra_configs"]["digest_rehearsal"]
    assert leg["n_ranks"] == gpus and leg["rows"] == 10_000_000
    assert leg["unequal_shards"] == (gpus > 1)
    assert leg["digest_equal"] is (fault is None or gpus == 1), leg


def test_block_shards_cover_and_align():
    """datasets.block_shard: contiguous, covering, whole 65,536-row blocks
    (word aligned), and the word offsets bench_legs gathers at."""
    from tests import datasets
    for n in (1 << 20, 10_000_000, 1 << 26, 65_536 * 3 + 17):
        for world in (1, 2, 3, 4, 8):
            prev = 0
            for r in range(world):
                lo, hi, b0, b1 = datasets.block_shard(n, r, world)
                assert lo == prev and lo % datasets.BLOCK == 0 and lo % 64 == 0
                assert hi == min(n, b1 * datasets.BLOCK) and lo == min(n, b0 * datasets.BLOCK)
                prev = hi
            assert prev == n


def test_block_digests_committed_and_consistent():
    """tests/golden/block_digests.json (libsodium-built, make_digests.py)
    covers every block of configs 2-4 and agrees with the whole-config
    digests' row counts; config 5's ledger digest is committed too."""
    from tests import datasets
    with open(datasets.BLOCK_DIGESTS) as f:
        blocks = json.load(f)
    with open(datasets.DIGESTS) as f:
        whole = json.load(f)
    for name in ("config2", "config4", "config3"):
        nb = -(-datasets.CONFIGS[name]["n"] // datasets.BLOCK)
        assert blocks[name]["block_rows"] == datasets.BLOCK
        assert len(blocks[name]["inputs_h16"]) == len(blocks[name]["bitmap_h16"]) == nb
        assert whole[name]["rows"] == datasets.CONFIGS[name]["n"]
    c5 = whole["config5"]
    assert c5["rows"] == datasets.CONFIG5["n"] and c5["accepted"] == c5["rows"] - c5["invalid_rows"]


def test_ledger_plan_and_mutations():
    """datasets.ledger_plan is deterministic; the invalid rows' flips land
    inside their own preimage (after the 4-byte prefix) or signature."""
    from tests import datasets
    cfg = dict(datasets.CONFIG5, n=4096)
    a, b = datasets.ledger_plan(cfg), datasets.ledger_plan(cfg)
    assert all(np.array_equal(a[k], b[k]) for k in ("pre", "offs", "lens", "who", "bad", "param"))
    assert (a["lens"] >= 113).all() and (a["lens"] <= 4096).all()
    assert all(bytes(a["pre"][o:o + 4]) == b"STX\x00" for o in a["offs"][:50])
    (pos, pbit), (srow, scol, sbit) = datasets.ledger_mutations(a)
    rows = np.searchsorted(a["offs"], pos, side="right") - 1
    assert set(rows.tolist()) <= set(a["bad"].tolist())
    assert ((pos - a["offs"][rows]) >= 4).all() and (pos < a["offs"][rows] + a["lens"][rows]).all()
    assert (scol >= 0).all() and (scol < 64).all() and (pbit > 0).all() and (sbit > 0).all()
    assert pos.size + srow.size == a["bad"].size


def test_bench_rank_count_must_match():
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dry-run"],
                       capture_output=True, text=True, timeout=120, env=env, cwd=ROOT)
    assert r.returncode != 0 and "one rank per GPU" in (r.stdout + r.stderr)


def _c_shard(lib, n, r, g):
    lo, hi = ctypes.c_size_t(0), ctypes.c_size_t(0)
    lib.stl_shard_range(n, r, g, ctypes.byref(lo), ctypes.byref(hi))
    return lo.value, hi.value


def _c_shard_bytes(lib, lens, r, g):
    lens = np.ascontiguousarray(lens, np.uint32)
    lo, hi = ctypes.c_size_t(0), ctypes.c_size_t(0)
    lib.stl_shard_range_bytes(lens.ctypes.data_as(ctypes.c_void_p), lens.shape[0], r, g, ctypes.byref(lo),
                              ctypes.byref(hi))
    return lo.value, hi.value


def test_c_shards_equal_python_mirror():
    from stellard_amd import _native
    lib = _native.load()
    rng = np.random.default_rng(5)
    for n in (0, 1, 63, 64, 65, 1000, 4097, 1 << 20, 67108864):
        for g in (1, 2, 3, 4, 7, 8):
            for r in range(g):
                assert _c_shard(lib, n, r, g) == shard.shard_range(n, r, g)
    for trial in range(60):
        n = int(rng.integers(0, 5000))
        g = int(rng.integers(1, 9))
        if trial % 3 == 0:
            lens = np.exp(rng.uniform(np.log(100), np.log(4096), n)).astype(np.uint32)  # config 5 shape
        elif trial % 3 == 1:
            lens = rng.integers(0, 3, n).astype(np.uint32)  # zeros and tiny rows
        else:
            lens = np.where(rng.random(n) < 0.01, 1 << 20, 113).astype(np.uint32)  # a few huge rows
        for r in range(g):
            assert _c_shard_bytes(lib, lens, r, g) == shard.shard_range_bytes(lens, r, g), (n, g, r)


def test_byte_shards_snap_to_the_verify_step():
    """verify time steps every shard.QUANTUM rows (one
    main-kernel wave per SIMD), so a byte-balanced boundary within 2.5 % of a
    rank's bytes of a multiple of it moves there: config 5's ledgers
    (log-uniform 113 B - 4 KB rows) over 2, 4 and 8 ranks get exactly 2^20 / g
    rows per rank, bytes within 2 % of the share; the C function equals the
    mirror; a boundary far from any multiple keeps its byte balance."""
    from stellard_amd import _native
    lib = _native.load()
    rng = np.random.default_rng(0x5A1)
    q = shard.QUANTUM
    for trial in range(3):
        n = 1 << 20
        lens = np.exp(rng.uniform(np.log(113), np.log(4096), n)).astype(np.uint32)
        total = int(lens.sum())
        for g in (2, 4, 8):
            b = [shard.shard_range_bytes(lens, r, g) for r in range(g)]
            assert [hi - lo for lo, hi in b] == [n // g] * g, (trial, g)
            per = [int(lens[lo:hi].sum()) for lo, hi in b]
            assert max(abs(p - total / g) for p in per) <= 0.02 * total / g
            for r in range(g):
                assert _c_shard_bytes(lib, lens, r, g) == b[r], (trial, g, r)
        # 3 ranks: boundaries near 349,525 rows, far from any multiple of q
        b = [shard.shard_range_bytes(lens, r, 3) for r in range(3)]
        assert all(lo % q for lo, _ in b[1:])
        assert [_c_shard_bytes(lib, lens, r, 3) for r in range(3)] == b
    # a heavy head: the snap would move too many bytes, so it stays put
    lens = np.full(1 << 18, 200, np.uint32)
    lens[: 1 << 16] = 4000
    b = [shard.shard_range_bytes(lens, r, 2) for r in range(2)]
    assert b[0][1] % q != 0 and [_c_shard_bytes(lib, lens, r, 2) for r in range(2)] == b


def test_byte_shards_cover_align_and_balance():
    rng = np.random.default_rng(6)
    lens = np.exp(rng.uniform(np.log(100), np.log(4096), 200000)).astype(np.uint32)
    total = int(lens.sum())
    for g in (2, 4, 8):
        b = [shard.shard_range_bytes(lens, r, g) for r in range(g)]
        assert b[0][0] == 0 and b[-1][1] == lens.shape[0]
        for (lo, hi), (lo2, _) in zip(b, b[1:]):
            assert hi == lo2 and lo % 64 == 0
        per = [int(lens[lo:hi].sum()) for lo, hi in b]
        # every shard within one 64-row word of bytes of the ideal split
        assert max(abs(p - total / g) for p in per) <= 2 * 64 * 4096
        # whereas equal-count shards of a length-sorted batch are badly skewed
    srt = np.sort(lens)
    b = [shard.shard_range_bytes(srt, r, 2) for r in range(2)]
    assert b[0][1] > srt.shape[0] // 2  # more short rows in the first shard


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _tx_worker(rank, world, port, q):
    import torch
    import torch.distributed as dist

    from tests import oracle_bind, txblob
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    o = oracle_bind.load_oracle()
    blobs, pres = txblob.valid_corpus(o, 300, 11, with_preimages=True)
    rng = np.random.default_rng(12)
    lens = np.array([len(b) for b in blobs], np.uint32)
    bounds = [shard.shard_range_bytes(lens, r, world)[0] for r in range(world)] + [len(blobs)]
    lo, hi = bounds[rank], bounds[rank + 1]
    bad = rng.random(len(blobs)) < 0.3
    blobs = [b[:-1] + bytes([b[-1] ^ 1]) if x else b for b, x in zip(blobs, bad)]
    bits = o.tx_blob_verify_batch(blobs[lo:hi], threads=2)
    full = shard.gather_bitmap_words_v(torch.from_numpy(shard.bool_to_words(bits)), bounds, dist)
    if rank == 0:
        ref = o.tx_blob_verify_batch(blobs, threads=2)
        q.put((shard.words_to_bool(full, len(blobs)).tolist(), ref.tolist(), [lo, hi]))
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_byte_shards_reassemble_tx_bitmap():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_tx_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got, ref, rank0 = q.get(timeout=180)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert got == ref
    assert 0 < rank0[1] < 300 and rank0[1] % 64 == 0


class Cfg(ctypes.Structure):
    _fields_ = [("struct_size", ctypes.c_uint32), ("device_count", ctypes.c_int32),
                ("first_device", ctypes.c_int32), ("flags", ctypes.c_uint32),
                ("shards_per_device", ctypes.c_int32), ("reserved", ctypes.c_uint32)]


def test_init_checks_config_before_devices():
    import torch
    from stellard_amd import _native as N
    lib = N.load()
    sz = ctypes.sizeof(Cfg)
    assert sz == 24
    bad = [Cfg(20, 0, 0, 0, 1, 0), Cfg(sz, 0, 0, N.STL_CFG_RCCL_GATHER | N.STL_CFG_NO_RCCL, 1, 0),
           Cfg(sz, 0, 0, 0x80, 1, 0), Cfg(sz, 0, -1, 0, 1, 0), Cfg(sz, 0, 0, 0, 1, 7)]
    for c in bad:
        assert lib.stl_init(ctypes.byref(c)) == N.STL_EINVAL
    if torch.cuda.is_available():
        pytest.skip("GPU present: the valid configurations are exercised by the gpu tests")
    for c in (Cfg(sz, 0, 0, 0, 3, 0), Cfg(16, 0, 0, 0, 0, 0), Cfg(sz, 2, 0, N.STL_CFG_RCCL_GATHER, 1, 0)):
        assert lib.stl_init(ctypes.byref(c)) == N.STL_ENODEV
    assert lib.stl_comm_init_rank(2, 0, bytes(128)) == N.STL_ENODEV
    assert lib.stl_bitmap_gather_device(None, 1, None, 0, None) == N.STL_ERCCL  # no communicator


def test_batcher_flush_with_nothing_pending_keeps_the_delay():
    """stl_batcher_flush on an idle aggregator must not make the next request
    skip its max_delay wait (the old flag stayed set)."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present: covered by the gpu tests")
    from stellard_amd import verify as V
    with V.Batcher(max_batch=64, max_delay_us=400_000) as b:
        b.flush()
        t0 = time.perf_counter()
        h = b.submit(bytes(64), bytes(32), bytes(32))
        v = h.result(timeout=10)
        waited = time.perf_counter() - t0
        assert v < 0
        assert waited >= 0.3, waited


def test_stats_without_gpu():
    """stl_get_stats on a GPU-less host: host counters only; a failed call is
    counted as an error (ENODEV), nothing as verified-and-accepted."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present: covered by the gpu tests")
    from stellard_amd import _native as N
    from stellard_amd import verify as V
    V.reset_stats()
    sig = np.zeros((64, 64), np.uint8)
    msg = np.zeros((64, 32), np.uint8)
    with pytest.raises(N.StlError):
        V.verify_batch(sig, msg, msg)
    st = V.get_stats()
    assert st["batches"] == 1 and st["signatures"] == 64 and st["errors"] == 1 and st["accepted"] == 0
    bad = V.Stats()
    bad.struct_size = 8
    assert N.load().stl_get_stats(ctypes.byref(bad)) == N.STL_EINVAL
    assert st["phase_chunks"] == 0 and set(st["phase_ns"]) == {"phase1", "point", "main", "fallback"}
    # the phase-timing switch returns the previous setting
    assert V.set_phase_timing(True) is False
    assert V.set_phase_timing(False) is True


def test_fallback_verify_without_gpu(oracle, golden):
    """stl_config.fallback_verify on a host without a gfx950 device: stl_init
    fails (ENODEV) but registers the caller's check, and the single call then
    answers every signature with it (composed with S < L) -- 0 / -1 only, the
    exact golden bits.  Registering NULL again restores the error code."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present: covered by the gpu tests")
    from stellard_amd import _native as N
    from stellard_amd import verify as V

    def fb(s, m, mlen, p):
        return 0 if oracle.verify_raw(ctypes.string_at(s, 64), ctypes.string_at(m, mlen), ctypes.string_at(p, 32),
                                      policy=0) else -1

    fn = V.VERIFY_FN(fb)
    lib = N.load()
    try:
        with pytest.raises(N.StlError) as e:
            V.init(fallback_verify=fn)
        assert e.value.rc == N.STL_ENODEV
        exp = golden["expected_sodium_1_0_18"].astype(bool)
        idx = np.random.default_rng(4).choice(exp.shape[0], 300, replace=False)
        for i in idx:
            rc = lib.stl_ed25519_verify_detached(golden["sig"][i].tobytes(), golden["msg"][i].tobytes(), 32,
                                                 golden["pk"][i].tobytes())
            assert rc in (0, -1) and (rc == 0) == bool(exp[i]), (i, rc)
    finally:
        with pytest.raises(N.StlError):
            V.init()  # registers NULL
    assert lib.stl_ed25519_verify_detached(golden["sig"][0].tobytes(), golden["msg"][0].tobytes(), 32,
                                           golden["pk"][0].tobytes()) == N.STL_ENODEV


def test_comm_info_without_communicator():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present: covered by the gpu tests")
    from stellard_amd import _native as N
    nr, r = ctypes.c_int(-5), ctypes.c_int(-5)
    assert N.load().stl_comm_info(ctypes.byref(nr), ctypes.byref(r)) == N.STL_ERCCL
    assert N.load().stl_comm_info(None, None) == N.STL_EINVAL
