#!/usr/bin/env python3
"""Timing harness for the hashing kernels on config-5-shaped data (1,048,576
transactions, blob lengths log-uniform in 100 B - 4 KB):

  tx_hash   stl_tx_hash_batch_device over signing preimages
  tx_blob   stl_tx_blob_prepare_device over whole serialized transactions
            (canonical pass + signing hash + transaction ID)

Signatures are random bytes (the hashing kernels do not verify).  Prints one
JSON line; used for A/B runs and under rocprofv3.
  python3 tools/hash_bench.py [--n N] [--reps R] [--no-ids]
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def make_blobs(n, seed, uniform=0):
    """Payment transactions (tools/payments.py: the Payment template, a Memos
    array as the pad) with preimage lengths log-uniform in 100 B - 4 KB, or
    all `uniform` bytes: (signing preimages, serialized transactions)."""
    from tools.payments import blobs_from_preimages, payment_preimages
    rng = np.random.default_rng(seed)
    target = np.exp(rng.uniform(np.log(100), np.log(4096), n)).astype(np.int64)
    if uniform:
        target[:] = uniform
    pks = np.frombuffer(rng.bytes(1000 * 32), np.uint8).reshape(1000, 32)
    pres = payment_preimages(pks, n, rng, pad_lens=target)
    sig = np.frombuffer(rng.bytes(n * 64), np.uint8).reshape(n, 64)
    pk = pks[np.arange(n) % 1000]
    return pres, blobs_from_preimages(pres, sig, pk)


def pack(chunks):
    lens = np.array([len(c) for c in chunks], np.uint32)
    offs = np.zeros(len(chunks), np.uint64)
    offs[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
    buf = np.frombuffer(b"".join(chunks) + b"\0" * 4, np.uint8).copy()
    return buf, offs, lens


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1 << 20)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--no-ids", action="store_true")
    ap.add_argument("--uniform", type=int, default=0, help="all blobs this many bytes")
    ap.add_argument("--timing-only", action="store_true", help="skip the hash check (timing-only A/B builds)")
    args = ap.parse_args()
    import ctypes

    import torch
    from stellard_amd import _native as N
    from stellard_amd import verify as V
    V.init(device_count=1)
    n = args.n
    pres, blobs = make_blobs(n, 0x5EED0005, args.uniform)
    out = {"n": n}
    s = torch.cuda.current_stream()
    for name, chunks in (("tx_hash", pres), ("tx_blob", blobs)):
        buf, offs, lens = pack(chunks)
        d_buf = torch.from_numpy(buf).cuda()
        d_off = torch.from_numpy(offs.view(np.int64)).cuda()
        d_len = torch.from_numpy(lens.view(np.int32)).cuda()
        d_msg = torch.empty((n, 32), dtype=torch.uint8, device="cuda")

        def run():
            if name == "tx_hash":
                N.check(N.load().stl_tx_hash_batch_device(
                    ctypes.c_void_p(d_buf.data_ptr()), ctypes.c_void_p(d_off.data_ptr()),
                    ctypes.c_void_p(d_len.data_ptr()), n, ctypes.c_void_p(d_msg.data_ptr()),
                    ctypes.c_void_p(s.cuda_stream)), "tx_hash")
                return None
            return V.tx_blob_prepare_device(d_buf, d_off, d_len, tx_ids=not args.no_ids, stream=s)

        o = run()
        torch.cuda.synchronize()
        ts = []
        for _ in range(args.reps):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(s)
            run()
            b.record(s)
            torch.cuda.synchronize()
            ts.append(a.elapsed_time(b))
        ms = float(np.median(ts))
        # the signing preimages are the same bytes on both legs (the blob leg
        # splices them out of the blobs); plus each blob's ID pass
        pl = np.array([len(x) for x in pres], dtype=np.int64)
        blocks = int(((pl + 17 + 127) // 128).sum())
        if name == "tx_blob" and not args.no_ids:
            blocks += int(((lens.astype(np.int64) + 4 + 17 + 127) // 128).sum())
        out[name] = {"ms": ms, "tx_per_s": n / ms * 1e3, "bytes": int(lens.sum()),
                     "GB_per_s": float(lens.sum()) / ms / 1e6, "sha512_blocks": blocks,
                     "blocks_per_s": blocks / ms * 1e3}
        if o is not None:
            st = o["status"].cpu().numpy()
            out[name]["status_counts"] = {str(k): int((st == k).sum()) for k in (0, 1, 2)}
            if name == "tx_blob" and not args.timing_only:
                import hashlib
                m = o["msg"].cpu().numpy()
                for i in (0, n // 2, n - 1):
                    assert bytes(m[i]) == hashlib.sha512(pres[i]).digest()[:32]
    print(json.dumps(out))


if __name__ == "__main__":
    main()
