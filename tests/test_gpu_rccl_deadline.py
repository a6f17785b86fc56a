"""The RCCL bring-up under a deadline.

stl_comm_init_rank builds the one-process-per-GPU communicator nonblocking
(ncclCommInitRankConfig, blocking = 0) and polls it against the deadline, so a
rank whose peers never join gets STL_ERCCL instead of hanging the driver's
first 1/2/4/8 run; a later bring-up then succeeds.  The replaced parallelism is
stellard's JobQueue pool (/root/reference/src/ripple_core/functional/
JobQueue.cpp:217-243).  On the one-GPU pool the only bring-up that can never
complete is a two-rank communicator whose second rank does not exist.

Run in a child process: an aborted bring-up must not leave RCCL state in the
pytest process that the other GPU tests share.
"""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import json, os, sys, time
sys.path.insert(0, os.environ["STL_ROOT"])
import torch
from stellard_amd import verify as V, _native as N
V.init(device_count=1)
V.debug_tuning(V.TUNE_RCCL_TIMEOUT_MS, 5000)
out = {}
uid = V.comm_unique_id()
t0 = time.time()
try:
    V.comm_init_rank(2, 0, uid)
    out["rc"] = 0
except N.StlError as e:
    out["rc"] = e.rc
out["dt"] = time.time() - t0
V.comm_init_rank(1, 0, V.comm_unique_id())
out["info"] = list(V.comm_info())
w = torch.arange(1, 5, dtype=torch.int64, device="cuda")
full = torch.zeros(4, dtype=torch.int64, device="cuda")
V.bitmap_gather_device(w, full, root=0)
V.comm_sync(None, 5000)
out["gather_ok"] = bool(torch.equal(w, full))
V.comm_destroy()
print("RESULT " + json.dumps(out), flush=True)
"""


@pytest.mark.timeout(150)
def test_comm_init_rank_times_out_then_recovers():
    env = dict(os.environ, STL_ROOT=ROOT, NCCL_SOCKET_IFNAME="lo")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, "-c", CHILD], capture_output=True, text=True, timeout=120, env=env,
                       cwd=ROOT)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-3000:])
    res = json.loads(next(s for s in r.stdout.splitlines() if s.startswith("RESULT "))[7:])
    assert res["rc"] == -1001, res  # STL_ERCCL
    assert 4.0 <= res["dt"] <= 40.0, res
    assert res["info"] == [1, 0] and res["gather_ok"] is True, res


CHILD_SYNC = r"""
import json, os, sys, time
sys.path.insert(0, os.environ["STL_ROOT"])
import numpy as np
import torch
from stellard_amd import verify as V, _native as N
V.init(device_count=1)
out = {}
V.comm_init_rank(1, 0, V.comm_unique_id())
n = 1 << 20
rng = np.random.default_rng(5)
seeds = torch.from_numpy(rng.integers(0, 256, (n, 32), dtype=np.uint8)).cuda()
msgs = torch.from_numpy(rng.integers(0, 256, (n, 32), dtype=np.uint8)).cuda()
pk, sig = V.sign_batch_device(seeds, msgs)
torch.cuda.synchronize()
s = torch.cuda.current_stream()
w = torch.empty(n // 64, dtype=torch.int64, device="cuda")
full = torch.zeros(n // 64, dtype=torch.int64, device="cuda")
V.bitmap_gather_device(w, full, root=0, stream=s)  # warm: RCCL's first collective sets itself up
V.comm_sync(s, 5000)
# ~25 ms of verify work queued ahead of the gather, then a 1-ms deadline: the
# deadline covers the gather only, so the healthy communicator survives
for _ in range(3):
    V.verify_batch_device(sig, msgs, pk, out_words=w, stream=s)
V.bitmap_gather_device(w, full, root=0, stream=s)
t0 = time.time()
try:
    V.comm_sync(s, 1)
    out["sync_rc"] = 0
except N.StlError as e:
    out["sync_rc"] = e.rc
out["sync_s"] = time.time() - t0
out["gathered_all_ones"] = bool(V.words_to_bool(full, n).all())
out["info_after_sync"] = list(V.comm_info())
# the abort path: a fault injected into comm_sync is a failed collective
V.debug_fault_after(0)
try:
    V.comm_sync(s, 5000)
    out["fault_rc"] = 0
except N.StlError as e:
    out["fault_rc"] = e.rc
V.debug_fault_after(-1)
try:
    V.bitmap_gather_device(w, full, root=0, stream=s)
    out["gather_after_abort_rc"] = 0
except N.StlError as e:
    out["gather_after_abort_rc"] = e.rc
# a new communicator after the abort works
V.comm_init_rank(1, 0, V.comm_unique_id())
full.zero_()
V.bitmap_gather_device(w, full, root=0, stream=s)
V.comm_sync(s, 5000)
out["regather_ok"] = bool(torch.equal(w, full))
V.comm_destroy()
print("RESULT " + json.dumps(out), flush=True)
"""


@pytest.mark.timeout(150)
def test_comm_sync_deadline_covers_the_gather_and_abort_path():
    """stl_comm_sync's deadline starts when the gather starts (work
    queued ahead of it does not count), and the abort path (here a fault
    injected into comm_sync) aborts and forgets the communicator -- the next
    gather is STL_ERCCL, a new bring-up works."""
    env = dict(os.environ, STL_ROOT=ROOT, NCCL_SOCKET_IFNAME="lo")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, "-c", CHILD_SYNC], capture_output=True, text=True, timeout=120, env=env,
                       cwd=ROOT)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-3000:])
    res = json.loads(next(s for s in r.stdout.splitlines() if s.startswith("RESULT "))[7:])
    assert res["sync_rc"] == 0 and res["gathered_all_ones"], res
    assert res["info_after_sync"] == [1, 0], res
    assert res["fault_rc"] == -1001 and res["gather_after_abort_rc"] == -1001, res
    assert res["regather_ok"] is True, res
