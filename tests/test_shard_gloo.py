"""Multi-rank path on CPU (gloo, world_size 2): index sharding + the bitmap
all-gather reassemble exactly the single-rank accept bitmap.  The per-shard
checker here is the CPU oracle (this box has no GPU); on MI355X the same
functions run with backend "nccl" (RCCL) around the HIP kernel (bench.py)."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from stellard_amd import shard


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n, q):
    import torch
    import torch.distributed as dist

    from tests import oracle_bind
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    g = np.load(os.path.join(os.path.dirname(__file__), "golden", "ed25519_golden.npz"), allow_pickle=False)
    idx = np.arange(n) % g["sig"].shape[0]
    lo, hi = shard.shard_range(n, rank, world)
    o = oracle_bind.load_oracle()
    bits = o.verify_batch(g["sig"][idx][lo:hi], g["msg"][idx][lo:hi], g["pk"][idx][lo:hi], threads=2)
    local = torch.from_numpy(shard.bool_to_words(bits))
    full = shard.gather_bitmap_words(local, n, world, dist)
    if rank == 0:
        q.put(shard.words_to_bool(full, n).tolist())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("n", [64, 1000, 2163])
def test_two_rank_gather_matches_single_rank(n, golden):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = np.array(q.get(timeout=120), dtype=bool)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    idx = np.arange(n) % golden["sig"].shape[0]
    assert np.array_equal(got, golden["expected_sodium_1_0_18"][idx].astype(bool))


@pytest.mark.parametrize("n,world", [(1, 2), (63, 2), (64, 2), (65, 2), (1 << 20, 8), (67108864, 8), (1000, 3)])
def test_shard_ranges_cover_and_align(n, world):
    ranges = [shard.shard_range(n, r, world) for r in range(world)]
    assert ranges[0][0] == 0 and ranges[-1][1] == n
    for (a, b), (c, d) in zip(ranges, ranges[1:]):
        assert b == c
    for lo, hi in ranges:
        assert lo <= hi and (lo % 64 == 0 or lo == hi == n)
        assert (hi - lo + 63) // 64 <= shard.words_per_rank(n, world)


def test_word_roundtrip():
    rng = np.random.default_rng(0)
    for n in (1, 63, 64, 65, 1000):
        b = rng.random(n) < 0.5
        assert np.array_equal(shard.words_to_bool(shard.bool_to_words(b), n), b)
