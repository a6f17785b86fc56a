#!/usr/bin/env python3
"""Per-phase kernel time of 1M-signature device-resident launches (phase
clock on, kernels serial on one stream): the prep / main split of a libstl
build (STL_LIB_PATH selects it; timing-only builds may give wrong bits).
    STL_STREAMS=1 python3 tools/prep_probe.py [K]"""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from stellard_amd import verify as V  # noqa: E402


def main():
    K = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    n = 1 << 20
    V.init(device_count=1)
    rng = np.random.default_rng(11)
    seeds = torch.from_numpy(rng.integers(0, 256, (n, 32), dtype=np.uint8)).cuda()
    msgs = torch.from_numpy(rng.integers(0, 256, (n, 32), dtype=np.uint8)).cuda()
    pk, sig = V.sign_batch_device(seeds, msgs)
    V.verify_batch_device(sig, msgs, pk)
    torch.cuda.synchronize()
    V.set_phase_timing(True)
    before = V.get_stats()["phase_ns"]
    for _ in range(K):
        V.verify_batch_device(sig, msgs, pk)
    torch.cuda.synchronize()
    after = V.get_stats()["phase_ns"]
    V.set_phase_timing(False)
    out = {k: (after[k] - before[k]) / K / 1e6 for k in after}
    out["lib"] = os.environ.get("STL_LIB_PATH") or "product"
    print(json.dumps(out))


if __name__ == "__main__":
    main()
