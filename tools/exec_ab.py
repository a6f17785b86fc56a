#!/usr/bin/env python3
"""Same-process A/B of libstl's execution settings (stl_debug_tuning): fused
phase-1 kernel, the main kernel's unit queue, concurrent streams per call and
their chunk size.  1,048,576 GPU-signed signatures (1 % with a flipped message
byte), K back-to-back stl_ed25519_verify_batch_device launches per
measurement (as bench.py's timed region), settings interleaved in rotating
order over R repetitions; median ms per launch.  Every setting's bitmap must
equal the first setting's.

    python tools/exec_ab.py [K] [R] [name=fused,queue,streams,log2[,first] ...]
"""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from stellard_amd import verify as V  # noqa: E402

DEFAULT = ["base=0,0,1,18", "fq=1,1,1,18", "q_s2_18=0,1,2,18", "fq_s2_18=1,1,2,18", "fq_s2_19=1,1,2,19",
           "fq_s3_18=1,1,3,18", "fq_s4_18=1,1,4,18", "fq_s2_17=1,1,2,17", "fq_s3_17=1,1,3,17", "fq_s4_16=1,1,4,16"]


def main():
    args = sys.argv[1:]
    K = int(args.pop(0)) if args and args[0].isdigit() else 20
    R = int(args.pop(0)) if args and args[0].isdigit() else 5
    specs = args or DEFAULT
    cfgs = []
    for s in specs:
        name, vals = s.split("=")
        cfgs.append((name, [int(v) for v in vals.split(",")]))
    n = int(os.environ.get("N", 1 << 20))
    torch.cuda.set_device(0)
    V.init(device_count=1)
    rng = np.random.default_rng(7)
    seeds = torch.from_numpy(rng.integers(0, 256, (n, 32), dtype=np.uint8)).cuda()
    msgs = torch.from_numpy(rng.integers(0, 256, (n, 32), dtype=np.uint8)).cuda()
    pk, sig = V.sign_batch_device(seeds, msgs)
    bad = torch.from_numpy(rng.choice(n, n // 100, replace=False)).cuda()
    msgs[bad, 0] ^= 1
    words = torch.empty((n + 63) // 64, dtype=torch.int64, device="cuda")
    s = torch.cuda.current_stream()

    def apply(v):
        V.debug_tuning(V.TUNE_FUSED_PREP, v[0])
        V.debug_tuning(V.TUNE_MAIN_QUEUE, v[1])
        V.debug_tuning(V.TUNE_STREAMS, v[2])
        V.debug_tuning(V.TUNE_CHUNK_LOG2, v[3])
        V.debug_tuning(V.TUNE_FIRST_CHUNK, v[4] if len(v) > 4 else 0)  # rows of a smaller first chunk

    ref = None
    for name, v in cfgs:  # warm-up and parity
        apply(v)
        words.fill_(0)
        V.verify_batch_device(sig, msgs, pk, out_words=words, stream=s)
        torch.cuda.synchronize()
        bits = V.words_to_bool(words, n)
        if os.environ.get("STL_AB_TIMING_ONLY"):  # timing-only builds (STL_EXP_*): results are wrong by design
            continue
        if ref is None:
            ref = bits
            assert int(bits.sum()) == n - n // 100, "parity failure"
        assert (bits == ref).all(), f"{name}: bitmap differs from {cfgs[0][0]}"
    res = {name: [] for name, _ in cfgs}
    for r in range(R):
        order = cfgs[r % len(cfgs):] + cfgs[:r % len(cfgs)]
        if r % 2:
            order = order[::-1]
        for name, v in order:
            apply(v)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(K):
                V.verify_batch_device(sig, msgs, pk, out_words=words, stream=s)
            torch.cuda.synchronize()
            res[name].append((time.perf_counter() - t0) / K * 1e3)
    out = {name: {"ms": round(float(np.median(v)), 4), "M_per_s": round(n / np.median(v) / 1e3, 2),
                  "all": [round(x, 3) for x in v]} for name, v in res.items()}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
