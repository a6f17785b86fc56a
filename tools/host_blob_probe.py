#!/usr/bin/env python3
"""Config-1 host API timeline probe: 100,000 Payment blobs (bench.py
config1_leg's construction) through stl_tx_blob_verify_batch, K timed calls;
run under rocprofv3 --kernel-trace --memory-copy-trace to see where a call's
time goes.  Prints the median ms and the per-call host times.
    python3 tools/host_blob_probe.py [K] [n] [device]
With `device`: the device-resident one call (stl_signed_blob_verify_batch_device)
on blobs already in HBM instead."""
import ctypes
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from stellard_amd import _native as N  # noqa: E402
from stellard_amd import verify as V  # noqa: E402
from tools.payments import blobs_from_preimages, pack, payment_preimages  # noqa: E402


def main():
    K = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 100_000
    V.init(device_count=1)
    rng = np.random.default_rng(0x5EED0001)
    nacc = 1000
    acc_seeds = rng.integers(0, 256, (nacc, 32), dtype=np.uint8)
    apk, _ = V.sign_batch_device(torch.from_numpy(acc_seeds).cuda(), torch.zeros((nacc, 32), dtype=torch.uint8,
                                                                                   device="cuda"))
    apk = apk.cpu().numpy()
    pre = payment_preimages(apk, n, rng)
    pbuf, poff, plen = pack(pre)
    d_msg = V.tx_hash_batch_device(torch.from_numpy(pbuf).cuda(), torch.from_numpy(poff.view(np.int64)).cuda(),
                                   torch.from_numpy(plen.view(np.int32)).cuda())
    seeds = torch.from_numpy(acc_seeds[np.arange(n) % nacc]).cuda()
    tpk, tsig = V.sign_batch_device(seeds, d_msg)
    torch.cuda.synchronize()
    blobs = blobs_from_preimages(pre, tsig.cpu().numpy(), tpk.cpu().numpy())
    buf, offs, lens = pack(blobs)
    buf = np.concatenate([buf, np.zeros(4, np.uint8)])
    if len(sys.argv) > 3 and sys.argv[3] == "device":
        d_buf = torch.from_numpy(buf).cuda()
        d_off = torch.from_numpy(offs.view(np.int64)).cuda()
        d_len = torch.from_numpy(lens.view(np.int32)).cuda()
        words = torch.empty((n + 63) // 64, dtype=torch.int64, device="cuda")
        ts = []
        for _ in range(K + 1):
            t0 = time.perf_counter()
            V.signed_blob_verify_batch_device(d_buf, d_off, d_len, out_words=words)
            torch.cuda.synchronize()
            ts.append((time.perf_counter() - t0) * 1e3)
        print(json.dumps({"n": n, "mode": "device", "ms_median": float(np.median(ts[1:])),
                          "ms": [round(t, 3) for t in ts], "accepted": int(V.words_to_bool(words, n).sum())}))
        return
    B = lambda a: a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
    bm = np.zeros((n + 7) // 8, np.uint8)
    st = np.zeros(n, np.uint8)
    lib = N.load()
    ts = []
    for _ in range(K + 1):
        t0 = time.perf_counter()
        N.check(lib.stl_tx_blob_verify_batch(B(buf), B(offs), B(lens), n, B(bm), B(st), None, 0), "host")
        ts.append((time.perf_counter() - t0) * 1e3)
    bits = np.unpackbits(bm, bitorder="little")[:n].astype(bool)
    print(json.dumps({"n": n, "bytes": int(lens.sum()), "ms_median": float(np.median(ts[1:])),
                      "ms": [round(t, 3) for t in ts], "accepted": int(bits.sum())}))


if __name__ == "__main__":
    main()
