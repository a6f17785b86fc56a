"""The multi-rank bench flow on the GPU box (-m gpu): `bench.py --gpus 2
--gather gloo` starts two ranks (torch.distributed.run) that both use the one
visible MI355X -- RCCL refuses two ranks on one device, so the bitmap words are
gathered through host memory with gloo -- and runs everything else of the
driver's SCALE path: per-rank shards, barriers, max-over-ranks timing, the
configs[2] / configs[4] legs (extra_configs) and rank 0's JSON line.  The
reference parallelism this replaces is the JobQueue pool,
src/ripple_core/functional/JobQueue.cpp:217-243."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_two_ranks_gloo_rehearsal():
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--gather", "gloo",
                        "--steps", "2", "--warmup", "1", "--per-gpu", "65536", "--no-cpu-baseline"],
                       capture_output=True, text=True, timeout=300, env=env, cwd=ROOT)
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
    extra = line["extra_configs"]
    assert "error" not in extra, extra
    c3, c5 = extra["config3_64M"], extra["config5_ledger_replay"]
    assert c3["signatures_total"] == 1 << 26 and c3["signatures_per_rank"] == 1 << 25
    assert c3["all_accepted_every_rank"] is True and c3["gathered_all_accepted"] is True
    assert c5["transactions_total"] == 2 << 20 and c5["gathered_all_accepted"] is True
