"""Hash-kernel long mode (STL_TUNE_LONG_HASH) probe: one small call at a time,
progress printed after each, hashlib-checked.  GPU only.
    python3 tools/long_hash_probe.py"""
import hashlib
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from stellard_amd import verify as V
    V.init()
    rng = np.random.default_rng(3)
    for n in (1, 64, 1000, 4000):
        lens = np.exp(rng.uniform(np.log(113), np.log(4096), n)).astype(np.int64)
        offs = np.zeros(n, np.int64)
        offs[1:] = np.cumsum(lens[:-1])
        buf = rng.integers(0, 256, int(offs[-1] + lens[-1] + 16), dtype=np.uint8)
        want = np.array([np.frombuffer(hashlib.sha512(buf[o:o + ln].tobytes()).digest()[:32], np.uint8)
                         for o, ln in zip(offs, lens)])
        d = [torch.from_numpy(buf).cuda(), torch.from_numpy(offs).cuda(), torch.from_numpy(lens.astype(np.int32)).cuda()]
        for lm in (0, 8):
            V.debug_tuning(V.TUNE_LONG_HASH, lm)
            t0 = time.perf_counter()
            got = V.tx_hash_batch_device(*d)
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            ok = np.array_equal(got.cpu().numpy(), want)
            print(f"n={n} long_min={lm} ms={dt * 1e3:.3f} ok={ok} max_len={lens.max()}", flush=True)


if __name__ == "__main__":
    main()
