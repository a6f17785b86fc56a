#!/usr/bin/env python3
"""A/B timing of a libstl build variant (STL_LIB_PATH=<.so>): verify-kernel
time on 1,048,576 GPU-signed signatures, HIP events on the launch stream,
median of 10 launches; fails if any valid signature is rejected."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from stellard_amd import verify as V  # noqa: E402

n = int(os.environ.get("N", 1 << 20))
torch.cuda.set_device(0)
V.init(device_count=1)
rng = np.random.default_rng(1)
seeds = torch.from_numpy(rng.integers(0, 256, (n, 32), dtype=np.uint8)).cuda()
msgs = torch.from_numpy(rng.integers(0, 256, (n, 32), dtype=np.uint8)).cuda()
pk, sig = V.sign_batch_device(seeds, msgs)
words = torch.empty((n + 63) // 64, dtype=torch.int64, device="cuda")
s = torch.cuda.current_stream()
V.verify_batch_device(sig, msgs, pk, out_words=words)
torch.cuda.synchronize()
if not os.environ.get("STL_NOCHECK"):  # timing-only experiments may break results on purpose
    assert V.words_to_bool(words, n).all(), "parity failure"
ts = []
for _ in range(10):
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(s)
    V.verify_batch_device(sig, msgs, pk, out_words=words, stream=s)
    b.record(s)
    torch.cuda.synchronize()
    ts.append(a.elapsed_time(b))
ms = float(np.median(ts))
print(f"{os.path.basename(os.environ.get('STL_LIB_PATH', 'libstl.so'))}: {ms:.3f} ms  {n / ms / 1e3:.2f} M verifies/s")
