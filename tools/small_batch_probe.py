"""Latency of one synchronous device-resident call on small ledgers (1k-20k
transactions of the config-5 plan), split by path: the one-call checkSign
(stl_tx_verify_batch_device) under each dedup choice, the two-step path
(tx_hash_batch_device + verify_batch_device), the verify alone on hashes
already in HBM, and the hash alone.  Median of R calls, host clock around
call + stream sync.  GPU only; prints one JSON document.

    python3 tools/small_batch_probe.py [R]
"""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tests import datasets  # noqa: E402


def main():
    import torch
    from stellard_amd import verify as V
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    V.init()
    if os.environ.get("PROBE_QUAD"):  # A/B of the quad main kernel (STL_TUNE_QUAD)
        V.debug_tuning(V.TUNE_QUAD, int(os.environ["PROBE_QUAD"]))
    if os.environ.get("PROBE_LONG"):  # A/B of the hash kernel's long mode (STL_TUNE_LONG_HASH)
        V.debug_tuning(V.TUNE_LONG_HASH, int(os.environ["PROBE_LONG"]))
    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream()
    lp = datasets.ledger_plan()
    d_pre = torch.from_numpy(lp["pre"]).to(dev)
    d_off = torch.from_numpy(lp["offs"]).to(dev)
    d_len = torch.from_numpy(lp["lens"]).to(dev)
    seeds = torch.from_numpy(np.ascontiguousarray(lp["signers"][lp["who"]])).to(dev)
    msgs = V.tx_hash_batch_device(d_pre, d_off, d_len, stream=stream)
    pk, sig = V.sign_batch_device(seeds, msgs)
    torch.cuda.synchronize()
    out = {}
    sizes = [int(x) for x in os.environ.get("PROBE_SIZES", "1000,4000,8000,19000,40000").split(",")]
    for n in sizes:
        w = torch.zeros((n + 63) // 64, dtype=torch.int64, device=dev)
        m = torch.empty((n, 32), dtype=torch.uint8, device=dev)
        sl = slice(4096, 4096 + n)
        paths = {
            "one_call_auto": lambda: V.tx_verify_batch_device(d_pre, d_off[sl], d_len[sl], sig[sl], pk[sl],
                                                              out_words=w, stream=stream),
            "one_call_no_dedup": lambda: V.tx_verify_batch_device(d_pre, d_off[sl], d_len[sl], sig[sl], pk[sl],
                                                                  out_words=w, policy=V.NO_AUTO_DEDUP,
                                                                  stream=stream),
            "one_call_dedup": lambda: V.tx_verify_batch_device(d_pre, d_off[sl], d_len[sl], sig[sl], pk[sl],
                                                               out_words=w, policy=V.DEDUP_KEYS, stream=stream),
            "two_step": lambda: (V.tx_hash_batch_device(d_pre, d_off[sl], d_len[sl], out_msg=m, stream=stream),
                                 V.verify_batch_device(sig[sl], m, pk[sl], out_words=w, stream=stream)),
            "verify_only_auto": lambda: V.verify_batch_device(sig[sl], msgs[sl], pk[sl], out_words=w,
                                                              stream=stream),
            "verify_only_no_dedup": lambda: V.verify_batch_device(sig[sl], msgs[sl], pk[sl], out_words=w,
                                                                  policy=V.NO_AUTO_DEDUP, stream=stream),
            "hash_only": lambda: V.tx_hash_batch_device(d_pre, d_off[sl], d_len[sl], out_msg=m, stream=stream),
        }
        res = {}
        for name, fn in paths.items():
            for _ in range(3):
                fn()
            stream.synchronize()
            ts = []
            for _ in range(reps):
                t0 = time.perf_counter()
                fn()
                stream.synchronize()
                ts.append(time.perf_counter() - t0)
            res[name] = round(float(np.median(ts)) * 1e3, 4)
        V.reset_stats()
        V.tx_verify_batch_device(d_pre, d_off[sl], d_len[sl], sig[sl], pk[sl], out_words=w, stream=stream)
        stream.synchronize()
        res["auto_dedup_chunks_after_warm_call"] = V.get_stats()["auto_dedup_chunks"]
        out[str(n)] = res
        print(n, res, flush=True)
    # the whole 2^20-row config-5 ledger: hash alone, one call (throughput side)
    n = lp["n"]
    m = torch.empty((n, 32), dtype=torch.uint8, device=dev)
    ts = []
    for i in range(6):
        t0 = time.perf_counter()
        V.tx_hash_batch_device(d_pre, d_off, d_len, out_msg=m, stream=stream)
        stream.synchronize()
        if i:
            ts.append(time.perf_counter() - t0)
    assert torch.equal(m, msgs)
    out["ledger_hash_1M_ms"] = round(float(np.median(ts)) * 1e3, 4)
    print("ledger hash", out["ledger_hash_1M_ms"], flush=True)
    print(json.dumps({"ms_median": out, "reps": reps}))


if __name__ == "__main__":
    main()
