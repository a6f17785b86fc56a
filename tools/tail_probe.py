"""A/B of STL_TUNE_TAIL_PAIRS (a lane-pair remainder chunk past three
lane-pair chunks' rows) interleaved in one process: device-resident verify at
PROBE_SIZES rows and configs[0]'s 100k Payment blobs through one
stl_signed_blob_verify_batch_device call; median ms of R calls per setting and
rotation, bits checked (verify: all accepted; blobs: the committed digest).

    python3 tools/tail_probe.py [R] [ROTATIONS]
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
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 11
    rots = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    V.init()
    dev = torch.device("cuda", 0)
    s = torch.cuda.current_stream()
    sizes = [int(x) for x in os.environ.get("PROBE_SIZES", "98304,100000,110000,120000,131072").split(",")]
    settings = [int(x) for x in os.environ.get("PROBE_TAILS", "0,32768").split(",")]
    nmax = max(sizes)
    rng = np.random.default_rng(7)
    seeds = torch.from_numpy(rng.integers(0, 256, (nmax, 32), dtype=np.uint8)).to(dev)
    msgs = torch.from_numpy(rng.integers(0, 256, (nmax, 32), dtype=np.uint8)).to(dev)
    pk, sig = V.sign_batch_device(seeds, msgs)
    w = torch.empty((nmax + 63) // 64, dtype=torch.int64, device=dev)
    with open(datasets.DIGESTS) as f:
        want = json.load(f)["config1"]

    def signer_pks(sd):
        z = torch.zeros((sd.shape[0], 32), dtype=torch.uint8, device=dev)
        return V.sign_batch_device(torch.from_numpy(np.ascontiguousarray(sd)).to(dev), z)[0].cpu().numpy()
    plan = datasets.config1_plan(signer_pks)
    n1 = plan["n"]
    m1 = torch.from_numpy(datasets.config1_signing_hashes(plan)).to(dev)
    _, s1 = V.sign_batch_device(torch.from_numpy(np.ascontiguousarray(plan["seeds"][plan["who"]])).to(dev), m1)
    buf, offs, lens = datasets.config1_finish(plan, s1.cpu().numpy())
    b_buf, b_off, b_len = (torch.from_numpy(a).to(dev) for a in (buf, offs, lens))
    w1 = torch.empty((n1 + 63) // 64, dtype=torch.int64, device=dev)
    st = torch.empty(n1, dtype=torch.uint8, device=dev)

    def timed(fn):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        ts = []
        for _ in range(reps):
            t0 = time.perf_counter()
            fn()
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
        return float(np.median(ts)) * 1e3

    res = {t: {} for t in settings}
    order = []
    for r in range(rots):
        order += settings if r % 2 == 0 else settings[::-1]
    for t in order:
        V.debug_tuning(V.TUNE_TAIL_PAIRS, t)
        row = res[t]
        for n in sizes:
            ms = timed(lambda: V.verify_batch_device(sig[:n], msgs[:n], pk[:n], out_words=w, stream=s))  # noqa: B023
            ok = bool(V.words_to_bool(w, n).all())
            row.setdefault(f"verify_{n}", []).append((round(ms, 4), ok))
        ms = timed(lambda: V.signed_blob_verify_batch_device(b_buf, b_off, b_len, out_words=w1, out_status=st,
                                                             stream=s))
        bits = np.packbits(V.words_to_bool(w1, n1), bitorder="little")
        ok = hashlib.sha256(bits.tobytes()).hexdigest() == want["bitmap_sha256"]
        row.setdefault("config1", []).append((round(ms, 4), ok))
        print(json.dumps({"tail": t, **{k: v[-1] for k, v in row.items()}}), file=sys.stderr, flush=True)
    V.debug_tuning(V.TUNE_TAIL_PAIRS, 0)
    print(json.dumps({str(t): v for t, v in res.items()}))


if __name__ == "__main__":
    main()
