"""configs[0]'s 100k Payment blobs (tests/datasets.py config1_plan) through
one stl_signed_blob_verify_batch_device call, R times (median ms, M tx/s;
bits checked against the committed digest).  For kernel traces:
tools/gpujob.sh OUT trace:config1_probe.py:R.  PROBE_FLAGS: policy flags
(e.g. 32 = STL_NO_AUTO_DEDUP, 8 = STL_DEDUP_KEYS).

    python3 tools/config1_probe.py [R]
"""
import hashlib
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
    flags = int(os.environ.get("PROBE_FLAGS", "0"))
    V.init()
    dev = torch.device("cuda", 0)
    s = torch.cuda.current_stream()
    with open(datasets.DIGESTS) as f:
        want = json.load(f)["config1"]

    def signer_pks(seeds):
        z = torch.zeros((seeds.shape[0], 32), dtype=torch.uint8, device=dev)
        return V.sign_batch_device(torch.from_numpy(np.ascontiguousarray(seeds)).to(dev), z)[0].cpu().numpy()
    plan = datasets.config1_plan(signer_pks)
    n = plan["n"]
    m = torch.from_numpy(datasets.config1_signing_hashes(plan)).to(dev)
    _, sig = V.sign_batch_device(torch.from_numpy(np.ascontiguousarray(plan["seeds"][plan["who"]])).to(dev), m)
    buf, offs, lens = datasets.config1_finish(plan, sig.cpu().numpy())
    b_buf, b_off, b_len = (torch.from_numpy(a).to(dev) for a in (buf, offs, lens))
    w = torch.empty((n + 63) // 64, dtype=torch.int64, device=dev)
    st = torch.empty(n, dtype=torch.uint8, device=dev)

    def call():
        V.signed_blob_verify_batch_device(b_buf, b_off, b_len, out_words=w, out_status=st, policy=flags, stream=s)
    call()
    torch.cuda.synchronize()
    ts, enq = [], []
    for _ in range(reps):
        t0 = time.perf_counter()
        call()
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
        enq.append(t1 - t0)
    bits = np.packbits(V.words_to_bool(w, n), bitorder="little")
    ok = hashlib.sha256(bits.tobytes()).hexdigest() == want["bitmap_sha256"]
    med = float(np.median(ts))
    print(json.dumps({"n": n, "flags": flags, "ms": med * 1e3, "M_tx_per_s": n / med / 1e6, "digest_equal": ok,
                      "enqueue_ms": float(np.median(enq)) * 1e3, "all_ms": [round(t * 1e3, 3) for t in ts]}))


if __name__ == "__main__":
    main()
