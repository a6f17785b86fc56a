#!/usr/bin/env python3
"""Does splitting one verify batch over concurrent streams fill the kernel-
boundary drains?  1,048,576 GPU-signed signatures: one
stl_ed25519_verify_batch_device call on one stream vs S calls of n/S
signatures on S streams (forked from / joined to the main stream), K launches
back to back, interleaved repetitions, median ms per 1M."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from stellard_amd import verify as V  # noqa: E402

n, K = 1 << 20, 10
torch.cuda.set_device(0)
V.init(device_count=1)
rng = np.random.default_rng(3)
seeds = torch.from_numpy(rng.integers(0, 256, (n, 32), dtype=np.uint8)).cuda()
msgs = torch.from_numpy(rng.integers(0, 256, (n, 32), dtype=np.uint8)).cuda()
pk, sig = V.sign_batch_device(seeds, msgs)
words = torch.empty((n + 63) // 64, dtype=torch.int64, device="cuda")
main = torch.cuda.current_stream()
streams = [main] + [torch.cuda.Stream() for _ in range(3)]


def run(S):
    if S == 1:
        V.verify_batch_device(sig, msgs, pk, out_words=words, stream=main)
        return
    ev = torch.cuda.Event()
    ev.record(main)
    step = (n // S + 63) // 64 * 64  # whole bitmap words per stream
    for j in range(S):
        s = streams[j]
        if j:
            s.wait_event(ev)
        lo, hi = j * step, (j + 1) * step if j + 1 < S else n
        V.verify_batch_device(sig[lo:hi], msgs[lo:hi], pk[lo:hi], out_words=words[lo // 64:(hi + 63) // 64], stream=s)
    for j in range(1, S):
        e = torch.cuda.Event()
        e.record(streams[j])
        main.wait_event(e)


for S in (1, 2, 3, 4):
    run(S)
torch.cuda.synchronize()
assert V.words_to_bool(words, n).all()
res = {1: [], 2: [], 3: [], 4: []}
for rep in range(5):
    for S in (1, 2, 3, 4):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(K):
            run(S)
        torch.cuda.synchronize()
        res[S].append((time.perf_counter() - t0) / K * 1e3)
print({f"streams={S}": round(float(np.median(v)), 3) for S, v in res.items()})
