#!/usr/bin/env python3
"""Per-phase kernel time of small device batches (stl_set_phase_timing: HIP
events between libstl's launches), two lanes per signature vs STL_ONE_LANE.

    python tools/phase_small.py --out gpurun_out/phase_small.json
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=None)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--signers", type=int, default=0, help="distinct keys (0 = every row its own)")
    args = ap.parse_args()
    import torch
    torch.cuda.set_device(0)
    from stellard_amd import verify as V
    V.init(device_count=1)
    n = 1 << 16
    rng = np.random.default_rng(0x1A7)
    seeds_np = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    if args.signers:
        seeds_np = seeds_np[rng.integers(0, args.signers, n)]
    seeds = torch.from_numpy(seeds_np).cuda()
    msgs = torch.from_numpy(rng.integers(0, 256, (n, 32), dtype=np.uint8)).cuda()
    pk, sig = V.sign_batch_device(seeds, msgs)
    torch.cuda.synchronize()
    rep = {}
    V.set_phase_timing(True)
    modes = [("pair", 0), ("one_lane", V.ONE_LANE)]
    if args.signers:
        modes += [("dedup", V.DEDUP_KEYS), ("dedup_one_lane", V.DEDUP_KEYS | V.ONE_LANE)]
    for label, pol in modes:
        for m in (1, 1024, 16384, 32768, 49152, 65536):
            w = torch.empty((m + 63) // 64, dtype=torch.int64, device="cuda")
            V.verify_batch_device(sig[:m], msgs[:m], pk[:m], out_words=w, policy=pol)
            torch.cuda.synchronize()
            V.reset_stats()
            for _ in range(args.reps):
                V.verify_batch_device(sig[:m], msgs[:m], pk[:m], out_words=w, policy=pol)
            torch.cuda.synchronize()
            st = V.get_stats()
            assert V.words_to_bool(w, m).all()
            rep[f"{label}_{m}"] = {k: v / 1e3 / args.reps for k, v in st["phase_ns"].items()}  # us per call
            rep[f"{label}_{m}"]["total"] = sum(rep[f"{label}_{m}"].values())
            print(label, m, {k: round(v, 1) for k, v in rep[f"{label}_{m}"].items()}, flush=True)
    V.set_phase_timing(False)
    if args.out:
        with open(args.out, "w") as f:
            json.dump(rep, f, indent=1)


if __name__ == "__main__":
    main()
