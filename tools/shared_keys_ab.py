"""A/B of the launch-wide key domain (STL_TUNE_SHARED_KEYS 1) against one
key domain per chunk (0), and of the wide key tables' row minimum
(STL_TUNE_WIDE_MIN_ROWS), interleaved in one process: configs[0]'s 100k
Payment blobs in one stl_signed_blob_verify_batch_device call (automatic
dedup: 1,000 accounts), config 5's 2^20-preimage ledger in one
stl_tx_verify_batch_device call, and a 1M / 300k verify with forced dedup.
Median of R calls per setting and size, host clock around call + sync;
prints one JSON document.

    python3 tools/shared_keys_ab.py [R]
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
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 9
    V.init()
    dev = torch.device("cuda", 0)
    s = torch.cuda.current_stream()

    def signer_pks(seeds):
        z = torch.zeros((seeds.shape[0], 32), dtype=torch.uint8, device=dev)
        return V.sign_batch_device(torch.from_numpy(np.ascontiguousarray(seeds)).to(dev), z)[0].cpu().numpy()
    plan = datasets.config1_plan(signer_pks)
    n1 = plan["n"]
    m1 = torch.from_numpy(datasets.config1_signing_hashes(plan)).to(dev)
    _, s1 = V.sign_batch_device(torch.from_numpy(np.ascontiguousarray(plan["seeds"][plan["who"]])).to(dev), m1)
    buf, offs, lens = datasets.config1_finish(plan, s1.cpu().numpy())
    b_buf, b_off, b_len = (torch.from_numpy(a).to(dev) for a in (buf, offs, lens))
    w1 = torch.empty((n1 + 63) // 64, dtype=torch.int64, device=dev)
    st1 = torch.empty(n1, dtype=torch.uint8, device=dev)
    lp = datasets.ledger_plan()
    d_pre, d_off, d_len = (torch.from_numpy(lp[k]).to(dev) for k in ("pre", "offs", "lens"))
    m5 = V.tx_hash_batch_device(d_pre, d_off, d_len, stream=s)
    pk5, sig5 = V.sign_batch_device(torch.from_numpy(np.ascontiguousarray(lp["signers"][lp["who"]])).to(dev), m5)
    n5 = lp["n"]
    w5 = torch.empty((n5 + 63) // 64, dtype=torch.int64, device=dev)
    cases = {
        "config1_blob_one_call_auto": lambda: V.signed_blob_verify_batch_device(b_buf, b_off, b_len, out_words=w1,
                                                                               out_status=st1, stream=s),
        "config1_blob_one_call_dedup": lambda: V.signed_blob_verify_batch_device(
            b_buf, b_off, b_len, out_words=w1, out_status=st1, policy=V.DEDUP_KEYS, stream=s),
        "config1_blob_one_call_no_dedup": lambda: V.signed_blob_verify_batch_device(
            b_buf, b_off, b_len, out_words=w1, out_status=st1, policy=V.NO_AUTO_DEDUP, stream=s),
        "config5_one_call_dedup": lambda: V.tx_verify_batch_device(d_pre, d_off, d_len, sig5, pk5, out_words=w5,
                                                                   policy=V.DEDUP_KEYS, stream=s),
        "config5_verify_1M_dedup": lambda: V.verify_batch_device(sig5, m5, pk5, out_words=w5, policy=V.DEDUP_KEYS,
                                                                 stream=s),
        "config5_verify_300k_dedup": lambda: V.verify_batch_device(sig5[:300000], m5[:300000], pk5[:300000],
                                                                   out_words=w5, policy=V.DEDUP_KEYS, stream=s),
        "config5_verify_100k_dedup": lambda: V.verify_batch_device(sig5[:100000], m5[:100000], pk5[:100000],
                                                                   out_words=w5, policy=V.DEDUP_KEYS, stream=s),
    }
    # settings: (shared key domain, wide-table minimum rows, R decoded ahead)
    settings = {"shared": (1, 0, 1), "shared_r_inline": (1, 0, 0), "per_chunk": (0, 0, 0)}
    if os.environ.get("AB_SETTINGS"):
        settings = {k: v for k, v in settings.items() if k in os.environ["AB_SETTINGS"].split(",")}

    def apply(v):
        V.debug_tuning(V.TUNE_SHARED_KEYS, v[0])
        V.debug_tuning(V.TUNE_WIDE_MIN_ROWS, v[1])
        V.debug_tuning(V.TUNE_R_AHEAD, v[2])
    out = {}
    names = list(settings)
    for name, fn in cases.items():
        ts = {k: [] for k in names}
        for k in names:
            apply(settings[k])
            fn()
            fn()
        torch.cuda.synchronize()
        for r in range(reps):
            order = names[r % len(names):] + names[:r % len(names)]
            for k in (order if r % 2 == 0 else order[::-1]):
                apply(settings[k])
                fn()  # the automatic dedup follows the previous call's sample
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                fn()
                torch.cuda.synchronize()
                ts[k].append(time.perf_counter() - t0)
        out[name] = {f"{k}_ms": float(np.median(v)) * 1e3 for k, v in ts.items()}
        print(name, {k: round(v, 3) for k, v in out[name].items()}, file=sys.stderr, flush=True)
    apply((1, 0, 1))
    print(json.dumps(out))


if __name__ == "__main__":
    main()
