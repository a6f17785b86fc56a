#!/usr/bin/env python3
"""Single-call drop-in latency on one MI355X.

stellard calls RippleAddress::verifySignature one signature at a time from
its JobQueue workers (RippleAddress.cpp:190-200; min(ncpu,4)+2 = 6 workers,
JobQueue.cpp:223-236).  This measures, on the GPU box's host cores:

  * stl_ed25519_verify_detached per call (the C-ABI drop-in for
    crypto_sign_verify_detached) at T = 1 and T = 6 calling threads;
  * libsodium 1.0.18 crypto_sign_verify_detached + S<L (the reference call
    path, oracle/_ref/libsodium_ref.so) the same way;
  * the request aggregator (stl_batcher_*) with T = 6 submitting threads that
    each wait for their verdict (the JobQueue integration of INTEGRATION.md);
  * stl_ed25519_verify_batch latency against batch size (host buffers,
    PCIe included): where one batch call overtakes T CPU threads.

    python tools/latency.py --out gpurun_out/latency.json
"""
import argparse
import ctypes
import json
import os
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def threaded(fn, threads, per):
    """fn(i) per thread `per` times; returns calls/s and latency percentiles (us)."""
    lat = [[] for _ in range(threads)]
    bar = threading.Barrier(threads + 1)

    def work(t):
        bar.wait()
        for j in range(per):
            i = (t * per + j)
            t0 = time.perf_counter()
            fn(i)
            lat[t].append(time.perf_counter() - t0)

    ts = [threading.Thread(target=work, args=(t,)) for t in range(threads)]
    for x in ts:
        x.start()
    bar.wait()
    t0 = time.perf_counter()
    for x in ts:
        x.join()
    wall = time.perf_counter() - t0
    a = np.concatenate([np.array(x) for x in lat]) * 1e6
    return {"threads": threads, "calls": int(a.size), "calls_per_s": a.size / wall,
            "p50_us": float(np.percentile(a, 50)), "p99_us": float(np.percentile(a, 99)),
            "mean_us": float(a.mean())}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    import torch
    torch.cuda.set_device(0)
    from stellard_amd import _native as N
    from stellard_amd import verify as V
    from tests import oracle_bind
    V.init(device_count=1)
    n = 1 << 16
    rng = np.random.default_rng(0x1A7)
    seeds = torch.from_numpy(rng.integers(0, 256, (n, 32), dtype=np.uint8)).cuda()
    msgs = torch.from_numpy(rng.integers(0, 256, (n, 32), dtype=np.uint8)).cuda()
    pk_d, sig_d = V.sign_batch_device(seeds, msgs)
    sig, msg, pk = sig_d.cpu().numpy(), msgs.cpu().numpy(), pk_d.cpu().numpy()
    sb = [sig[i].tobytes() for i in range(n)]
    mb = [msg[i].tobytes() for i in range(n)]
    pb = [pk[i].tobytes() for i in range(n)]
    lib = N.load()
    rep = {"gpu": "1 x MI355X", "host_cpus_used": "threads as listed"}

    def stl_call(i):
        i %= n
        rc = lib.stl_ed25519_verify_detached(sb[i], mb[i], 32, pb[i])
        assert rc == 0, rc

    stl_call(0)
    rep["stl_ed25519_verify_detached"] = [threaded(stl_call, 1, 400), threaded(stl_call, 6, 150)]
    sod = oracle_bind.load_sodium_ref()
    if sod is not None:
        def sod_call(i):
            i %= n
            assert sod.ref_verify_signature(sb[i], mb[i], pb[i]) == 1

        rep["libsodium_" + sod.ref_sodium_version().decode()] = [threaded(sod_call, 1, 4000),
                                                                  threaded(sod_call, 6, 4000)]
    for delay in (200, 1000):
        with V.Batcher(max_batch=4096, max_delay_us=delay) as b:
            def bat_call(i):
                i %= n
                assert b.submit(sb[i], mb[i], pb[i]).result(timeout=30) == V.VERDICT_ACCEPT

            bat_call(0)
            rep[f"stl_batcher_max_delay_{delay}us"] = [threaded(bat_call, 6, 300), threaded(bat_call, 64, 200)]
    # batches below half the resident lanes run two lanes per signature;
    # STL_ONE_LANE is the one-lane A/B of the same call
    for label, pol in (("", 0), ("_one_lane", V.ONE_LANE)):
        sizes = {}
        for m in (1, 64, 1024, 16384, 65536):
            V.verify_batch(sig[:m], msg[:m], pk[:m], policy=pol)
            ts = []
            for _ in range(5):
                t0 = time.perf_counter()
                ok = V.verify_batch(sig[:m], msg[:m], pk[:m], policy=pol)
                ts.append(time.perf_counter() - t0)
            assert ok.all()
            t = float(np.median(ts))
            sizes[str(m)] = {"ms": t * 1e3, "verifies_per_s": m / t}
        rep["stl_ed25519_verify_batch_by_size" + label] = sizes
        dev = {}  # device-resident inputs: kernels only (HIP events on the call's stream)
        for m in (1, 1024, 16384, 32768, 65536):
            w = torch.empty((m + 63) // 64, dtype=torch.int64, device="cuda")
            V.verify_batch_device(sig_d[:m], msgs[:m], pk_d[:m], out_words=w, policy=pol)
            ts = []
            for _ in range(9):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                V.verify_batch_device(sig_d[:m], msgs[:m], pk_d[:m], out_words=w, policy=pol,
                                      stream=torch.cuda.current_stream())
                e1.record()
                e1.synchronize()
                ts.append(e0.elapsed_time(e1))
            assert V.words_to_bool(w, m).all()
            dev[str(m)] = {"ms": float(np.median(ts))}
        rep["stl_ed25519_verify_batch_device_by_size" + label] = dev
    doc = json.dumps(rep, indent=1)
    print(doc)
    if args.out:
        with open(args.out, "w") as f:
            f.write(doc)


if __name__ == "__main__":
    main()
