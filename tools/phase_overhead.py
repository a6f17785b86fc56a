#!/usr/bin/env python3
"""Cost of libstl's phase clock (stl_set_phase_timing) on the bench workload:
wall time of K back-to-back verify launches of 1,048,576 signatures with the
phase events off and on, interleaved (ABAB), median per launch."""
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
rng = np.random.default_rng(2)
seeds = torch.from_numpy(rng.integers(0, 256, (n, 32), dtype=np.uint8)).cuda()
msgs = torch.from_numpy(rng.integers(0, 256, (n, 32), dtype=np.uint8)).cuda()
pk, sig = V.sign_batch_device(seeds, msgs)
words = torch.empty((n + 63) // 64, dtype=torch.int64, device="cuda")
s = torch.cuda.current_stream()
for _ in range(3):
    V.verify_batch_device(sig, msgs, pk, out_words=words, stream=s)
torch.cuda.synchronize()
res = {False: [], True: []}
for rep in range(6):
    for on in (False, True):
        V.set_phase_timing(on)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(K):
            V.verify_batch_device(sig, msgs, pk, out_words=words, stream=s)
        torch.cuda.synchronize()
        res[on].append((time.perf_counter() - t0) / K * 1e3)
V.set_phase_timing(False)
print({("on" if k else "off"): round(float(np.median(v)), 4) for k, v in res.items()})
