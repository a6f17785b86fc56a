"""Verify time against row count around the main kernel's round of resident
lanes.  One JSON document:

  verify       device-resident stl_ed25519_verify_batch_device over n valid
               signatures, n in PROBE_SIZES (default: 100,000; 130,304;
               131,072; 131,584; 140,000; 263,040; 525,952), ms and M/s;
  config1      the bench's config-1 leg: 100k Payment blobs, one
               stl_signed_blob_verify_batch_device call (M tx/s);
  shards_*     configs[4]'s one ledger split into N = 2, 4, 8 byte shards
               (stl_shard_range_bytes) as the bench's config5_ledger_split
               (preimages, stl_tx_verify_batch_device) and config5_blob_split
               (blobs, stl_signed_blob_verify_batch_device) legs cut it, each
               rank's shard timed one after another on this GPU: per-shard ms
               and max / mean.

Median of R calls, host clock around call + sync.

    python3 tools/round_probe.py [R]
"""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tests import datasets  # noqa: E402


def med(torch, fn, reps):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    return float(np.median(ts))


def main():
    import torch
    from stellard_amd import verify as V
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 9
    V.init()
    dev = torch.device("cuda", 0)
    s = torch.cuda.current_stream()
    out = {}
    sizes = [int(x) for x in os.environ.get(
        "PROBE_SIZES", "100000,130304,131072,131584,140000,263040,525952").split(",")]
    nmax = max(sizes)
    rng = np.random.default_rng(7)
    seeds = torch.from_numpy(rng.integers(0, 256, (nmax, 32), dtype=np.uint8)).to(dev)
    msgs = torch.from_numpy(rng.integers(0, 256, (nmax, 32), dtype=np.uint8)).to(dev)
    pk, sig = V.sign_batch_device(seeds, msgs)
    w = torch.empty((nmax + 63) // 64, dtype=torch.int64, device=dev)
    ver = {}
    for n in sizes:
        dt = med(torch, lambda: V.verify_batch_device(sig[:n], msgs[:n], pk[:n], out_words=w, stream=s), reps)  # noqa: B023
        ok = bool(V.words_to_bool(w, n).all())
        ver[n] = {"ms": dt * 1e3, "M_per_s": n / dt / 1e6, "all_accepted": ok}
        print(f"verify {n}: {dt * 1e3:.3f} ms {n / dt / 1e6:.1f} M/s", file=sys.stderr, flush=True)
    out["verify"] = ver
    only = os.environ.get("PROBE_ONLY", "")
    if "config1" in only or not only:
        from bench import config1_leg
        c1 = config1_leg(V, torch, dev, s, 16)
        out["config1"] = {k: c1.get(k) for k in ("gpu_device_resident_tx_per_s", "gpu_device_ms",
                                                 "gpu_device_two_step_tx_per_s", "bitmap_parity")}
        print(f"config1: {out['config1']}", file=sys.stderr, flush=True)
    if "shards" in only or not only:
        lp = datasets.ledger_plan()
        d_pre = torch.from_numpy(lp["pre"]).to(dev)
        d_off = torch.from_numpy(lp["offs"]).to(dev)
        d_len = torch.from_numpy(lp["lens"]).to(dev)
        sd = torch.from_numpy(np.ascontiguousarray(lp["signers"][lp["who"]])).to(dev)
        m5 = V.tx_hash_batch_device(d_pre, d_off, d_len, stream=s)
        lpk, lsig = V.sign_batch_device(sd, m5)

        def signer_pks(seeds_):
            z = torch.zeros((seeds_.shape[0], 32), dtype=torch.uint8, device=dev)
            return V.sign_batch_device(torch.from_numpy(np.ascontiguousarray(seeds_)).to(dev), z)[0].cpu().numpy()
        bp = datasets.blob_ledger_plan(signer_pks)
        bm = torch.from_numpy(datasets.blob_signing_hashes(bp)).to(dev)
        _, bsig = V.sign_batch_device(torch.from_numpy(np.ascontiguousarray(bp["seeds"][bp["who"]])).to(dev), bm)
        datasets.blob_ledger_finish(bp, bsig.cpu().numpy())
        b_buf = torch.from_numpy(bp["buf"]).to(dev)
        b_off = torch.from_numpy(bp["offs"]).to(dev)
        b_len = torch.from_numpy(bp["lens"]).to(dev)
        n = lp["n"]
        wl = torch.zeros((n + 63) // 64, dtype=torch.int64, device=dev)
        stt = torch.zeros(n + 64, dtype=torch.uint8, device=dev)
        for world in (2, 4, 8):
            for kind, lens in (("ledger", lp["lens"]), ("blob", bp["lens"])):
                bounds = [V.shard_range_bytes(lens, r, world) for r in range(world)]
                ms = []
                for lo, hi in bounds:
                    if kind == "ledger":
                        fn = lambda lo=lo, hi=hi: V.tx_verify_batch_device(  # noqa: E731
                            d_pre, d_off[lo:hi], d_len[lo:hi], lsig[lo:hi], lpk[lo:hi], out_words=wl, stream=s)
                    else:
                        fn = lambda lo=lo, hi=hi: V.signed_blob_verify_batch_device(  # noqa: E731
                            b_buf, b_off[lo:hi], b_len[lo:hi], out_words=wl, out_status=stt, stream=s)
                    ms.append(med(torch, fn, reps) * 1e3)
                rows = [hi - lo for lo, hi in bounds]
                out[f"shards_{kind}_n{world}"] = {"rows": rows, "ms": ms, "max_over_mean": max(ms) / float(np.mean(ms))}
                print(f"{kind} N={world}: rows {rows} ms {[round(x, 3) for x in ms]} max/mean "
                      f"{max(ms) / float(np.mean(ms)):.3f}", file=sys.stderr, flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
