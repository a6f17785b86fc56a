"""What s_memtime counts on this box (a shader clock beside the
bench line).  stl_debug_clock_stamp runs one-wave workgroups that record the
shader cycle counter, the 100 MHz counter and their XCD / SE / CU.  Three
checks, one JSON document:

  idle_2048     one stamp of 2,048 workgroups on an idle chip: per XCD, the
                spread of the cycle counter across CUs at (almost) one instant
                -- small means one counter per XCD, so start and end stamps
                taken on different CUs of an XCD can be compared;
  loaded        stamps before and after K back-to-back 1M-signature verifies
                (the bench's timed region): the average clock per XCD;
  idle_gap      stamps around 50 ms of host sleep: the counter's idle rate.

    python3 tools/clock_probe.py [K]
"""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from stellard_amd import verify as V
    k = int(sys.argv[1]) if len(sys.argv) > 1 else 40
    V.init()
    s = torch.cuda.current_stream()
    out = {}
    a = V.clock_stamp(2048, s).cpu().numpy()
    per = {}
    for x in sorted(set((a[:, 2] & 0xF).tolist())):
        r = a[(a[:, 2] & 0xF) == x]
        # cycles relative to the earliest stamp, minus the realtime elapsed x 2.4 GHz
        t = r[:, 0].astype(np.float64)
        rt = r[:, 1].astype(np.float64)
        resid = (t - t.min()) - (rt - rt.min()) * 24.0
        se = (r[:, 3] >> 13) & 0x7
        per[int(x)] = {"wgs": int(r.shape[0]), "cycle_span": float(t.max() - t.min()),
                       "realtime_span_10ns": float(rt.max() - rt.min()),
                       "resid_min": float(resid.min()), "resid_max": float(resid.max()),
                       "ses": sorted(set(se.tolist())),
                       "first_cycles": int(t.min()), "first_realtime": int(rt.min())}
    out["idle_2048"] = per
    cu = {}
    for t, rt, x, hw in a.tolist():
        cu.setdefault((int(x) & 0xF, (int(hw) >> 8) & 0xFF), []).append((t, rt))
    spans = [max(v[0] for v in vs) - min(v[0] for v in vs) for vs in cu.values() if len(vs) > 1]
    rts = [max(v[1] for v in vs) - min(v[1] for v in vs) for vs in cu.values() if len(vs) > 1]
    out["idle_2048_per_cu"] = {"cus": len(cu), "max_cycle_span_within_cu": max(spans) if spans else None,
                               "max_realtime_span_within_cu_10ns": max(rts) if rts else None}
    n = 1 << 20
    rng = np.random.default_rng(1)
    seeds = torch.from_numpy(rng.integers(0, 256, (n, 32), dtype=np.uint8)).cuda()
    msgs = torch.from_numpy(rng.integers(0, 256, (n, 32), dtype=np.uint8)).cuda()
    pk, sig = V.sign_batch_device(seeds, msgs)
    w = torch.empty(n // 64, dtype=torch.int64, device="cuda")
    for _ in range(10):
        V.verify_batch_device(sig, msgs, pk, out_words=w, stream=s)
    torch.cuda.synchronize()
    for nwg in (64, 256):
        t0 = time.perf_counter()
        st0 = V.clock_stamp(nwg, s)
        for _ in range(k):
            V.verify_batch_device(sig, msgs, pk, out_words=w, stream=s)
        st1 = V.clock_stamp(nwg, s)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        ghz, per, ncu = V.clock_ghz(st0, st1)
        out[f"loaded_{nwg}"] = {"ghz": ghz, "per_xcc": per, "cus_matched": ncu, "ms_per_launch": dt * 1e3 / k,
                                "cycles_per_verify": (dt / k) * ghz * 1e9 / n if ghz else None}
    st0 = V.clock_stamp(256, s)
    torch.cuda.synchronize()
    time.sleep(0.05)
    st1 = V.clock_stamp(256, s)
    torch.cuda.synchronize()
    out["idle_gap"] = dict(zip(("ghz", "per_xcc", "cus_matched"), V.clock_ghz(st0, st1)))
    print(json.dumps(out))


if __name__ == "__main__":
    main()
