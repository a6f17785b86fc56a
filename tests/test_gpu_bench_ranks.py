"""The multi-rank bench flow on the GPU box (-m gpu): `bench.py --gpus 2
--gather gloo` starts two ranks (torch.distributed.run) that both use the one
visible MI355X -- RCCL refuses two ranks on one device, so the bitmap words are
gathered through host memory with gloo -- and runs everything else of the
driver's SCALE path: per-rank shards, barriers, max-over-ranks timing, the
digest-checked configs[2] / configs[3] / configs[4] legs (extra_configs:
each rank rebuilds its block shard of the committed datasets, rank 0 checks
the gathered bitmap's SHA-256 against libsodium's; config 5 is one ledger
split by preimage bytes, and again as serialized blobs split by blob bytes,
with status bytes and transaction ids gathered too) and rank 0's JSON line.  The
reference parallelism this replaces is the JobQueue pool,
src/ripple_core/functional/JobQueue.cpp:217-243."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.timeout(600)
def test_bench_two_ranks_gloo_rehearsal():
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--gather", "gloo",
                        "--steps", "2", "--warmup", "1", "--per-gpu", "65536", "--no-cpu-baseline"],
                       capture_output=True, text=True, timeout=540, env=env, cwd=ROOT)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-3000:])
    line = None
    for s in reversed(r.stdout.strip().splitlines()):
        if s.strip().startswith("{"):
            line = json.loads(s)
            break
    assert line is not None, r.stdout[-2000:]
    assert line["n_gpus"] == 2 and line["value"] > 0 and line["steps"] == 2
    assert "gloo" in line["config"]["gather"]
    assert line["stats"]["accepted"] == line["stats"]["verifies"] == 65536 * 2
    assert line["config"]["gather_check"]["slices_equal_rank_words"] is True
    extra = line["extra_configs"]
    for key in ("config3_64M_digest", "config4_10M_digest", "config5_ledger_split", "config5_blob_split"):
        assert "error" not in extra[key], (key, extra[key])
    c3, c4, c5 = extra["config3_64M_digest"], extra["config4_10M_digest"], extra["config5_ledger_split"]
    assert c3["rows"] == 1 << 26 and c3["n_ranks"] == 2 and c3["digest_equal"] is True
    assert c3["accepted"] == c3["accepted_expected"]
    assert all(r["slice_bitmap_blocks_equal"] for r in c3["rank_slices"] + c4["rank_slices"])
    assert c4["rows"] == 10_000_000 and c4["digest_equal"] is True and "unequal" in c4["shards"]
    assert c5["n_ranks"] == 2 and c5["digest_equal"] is True and c5["digest_equal_dedup_keys"] is True
    assert c5["digest_equal_no_dedup"] is True
    assert c5["byte_shards"][0][0] == 0 and c5["byte_shards"][1][1] == 1 << 20
    sl = c5["small_ledgers"]
    assert sl["bits_equal_expected"] is True and sl["transactions"] == 1 << 20
    assert 1000 <= sl["ledger_size"]["median"] <= 20000 and sl["latency_ms"]["p50"] > 0
    cb = extra["config5_blob_split"]  # serialized blobs split by bytes: bits, statuses and ids gathered
    assert cb["n_ranks"] == 2 and cb["transactions"] == 1 << 20
    assert cb["digest_equal"] is True and cb["digest_equal_no_dedup"] is True and cb["digest_equal_two_step"] is True
    assert cb["status_digest_equal"] is True and cb["ids_digest_equal"] is True
    assert cb["accepted"] == cb["accepted_expected"]
    assert cb["byte_shards"][0][0] == 0 and cb["byte_shards"][1][1] == 1 << 20
