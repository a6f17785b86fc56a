#!/usr/bin/env python3
"""Host-API (PCIe-inclusive) rate of a libstl variant (STL_LIB_PATH):
stl_ed25519_verify_batch on 1,048,576 host-resident signatures (pageable numpy
arrays, and pinned torch tensors as bench.py's end_to_end leg), median of 7."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from stellard_amd import verify as V  # noqa: E402

n = int(os.environ.get("N", 1 << 20))
torch.cuda.set_device(0)
V.init(device_count=1)
rng = np.random.default_rng(2)
seeds = torch.from_numpy(rng.integers(0, 256, (n, 32), dtype=np.uint8)).cuda()
msgs = torch.from_numpy(rng.integers(0, 256, (n, 32), dtype=np.uint8)).cuda()
pk, sig = V.sign_batch_device(seeds, msgs)
s, m, p = sig.cpu().numpy(), msgs.cpu().numpy(), pk.cpu().numpy()
V.verify_batch(s, m, p)
ts = []
for _ in range(7):
    t0 = time.perf_counter()
    ok = V.verify_batch(s, m, p)
    ts.append(time.perf_counter() - t0)
assert ok.all()
t = float(np.median(ts))
sp, mp, pp = (torch.from_numpy(a).pin_memory().numpy() for a in (s, m, p))
tp = []
for _ in range(7):
    t0 = time.perf_counter()
    ok = V.verify_batch(sp, mp, pp)
    tp.append(time.perf_counter() - t0)
assert ok.all()
t2 = float(np.median(tp))
print(f"{os.path.basename(os.environ.get('STL_LIB_PATH', 'libstl.so'))}: host API {t * 1e3:.2f} ms  {n / t / 1e6:.1f} M/s"
      f"  pinned {t2 * 1e3:.2f} ms  {n / t2 / 1e6:.1f} M/s")
