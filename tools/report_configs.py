#!/usr/bin/env python3
"""BASELINE.json configs 1-5 on one MI355X, next to the reference's CPU path.

CPU reference = oracle/_ref/libsodium_ref.so: the calls stellard makes
(SerializedTransaction::checkSign -> SHA512Half via OpenSSL SHA512,
RippleAddress::verifySignature -> libsodium 1.0.18 crypto_sign_verify_detached
&& S < L), timed at T = 16 (the GPU box's CPU share), 6 (stellard's JobQueue
default min(ncpu,4)+2, JobQueue.cpp:223-236) and 1 thread.  GPU = libstl.

  config 1  100,000 Payment txs (Appendix C blobs, 1,000 accounts), checkSign
            path: GPU SHA512Half + verify vs CPU SHA512 + libsodium
  config 2  1,048,576 signatures: device-resident and PCIe-inclusive (host
            API) rates; CPU rates on bounded samples
  config 4  10,000,000 signatures, 2 % adversarial rows (every golden
            Appendix-B class): GPU bitmap diffed against libsodium on all rows
  config 5  ledger replay: 1,048,576 txs with preimages log-uniform in
            100 B - 4 KB (Memo padding), checkSign path as config 1
  config 3  (--parity64m) 67,108,864 signatures with 2 % adversarial rows in
            4M chunks, every GPU bit diffed against libsodium (the multi-GPU
            throughput of config 3 is the driver's 1/2/4/8-GPU bench.py run)

Writes one JSON document to stdout (and --out).  Run on the GPU box:
  python3 tools/report_configs.py --out gpurun_out/report_configs.json
"""
import argparse
import ctypes
import hashlib
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from tools.payments import blobs_from_preimages, pack, payment_preimages  # noqa: E402

L = 2**252 + 27742317777372353535851937790883648493


def log(*a):
    print(*a, file=sys.stderr, flush=True)


# ---------------------------------------------------------------- CPU side
class CpuRef:
    def __init__(self):
        from tests import oracle_bind
        self.lib = oracle_bind.load_sodium_ref()
        if self.lib is None:
            raise SystemExit("libsodium reference harness unavailable")
        self.version = self.lib.ref_sodium_version().decode()
        self.ob = oracle_bind

    def verify(self, sig, msg, pk, threads):
        return self.ob.sodium_verify_batch(self.lib, sig, msg, pk, threads=threads)

    def tx_blob_verify(self, buf, offs, lens, threads):
        n = lens.shape[0]
        bm = np.zeros((n + 7) // 8, np.uint8)
        B = lambda a: np.ascontiguousarray(a).ctypes.data_as(ctypes.c_void_p)  # noqa: E731
        self.lib.ref_tx_blob_verify_batch(B(buf), B(offs), B(lens), n, B(bm), None, 0, threads)
        return np.unpackbits(bm, bitorder="little")[:n].astype(bool)

    def tx_verify(self, blob, offs, lens, sig, pk, threads):
        n = sig.shape[0]
        bm = np.zeros((n + 7) // 8, np.uint8)
        B = lambda a: np.ascontiguousarray(a).ctypes.data_as(ctypes.c_void_p)  # noqa: E731
        self.lib.ref_tx_verify_batch(B(blob), B(offs), B(lens), B(sig), B(pk), n, B(bm), threads)
        return np.unpackbits(bm, bitorder="little")[:n].astype(bool)


def timed(fn):
    t0 = time.perf_counter()
    r = fn()
    return r, time.perf_counter() - t0


def cpu_rates(run, n_total, samples):
    """run(lo, hi, threads) over a bounded prefix; returns {T: rate}."""
    out = {}
    for threads, cap in samples:
        m = min(n_total, cap)
        run(0, min(m, 2048), threads)  # warm
        _, dt = timed(lambda: run(0, m, threads))
        out[str(threads)] = {"verifies_per_s": m / dt, "sample": m, "seconds": dt}
    return out


# ---------------------------------------------------------------- GPU side
class Gpu:
    def __init__(self):
        import torch
        self.torch = torch
        torch.cuda.set_device(0)
        from stellard_amd import _native as N
        from stellard_amd import verify as V
        self.V, self.N = V, N
        V.init(device_count=1, first_device=0)
        self.stream = torch.cuda.current_stream()

    def sign(self, seeds, msgs):
        t = self.torch
        pk, sig = self.V.sign_batch_device(t.from_numpy(seeds).cuda(), t.from_numpy(msgs).cuda())
        return pk, sig

    def verify_dev(self, sig, msg, pk, reps=5, policy=0):
        t = self.torch
        words = self.V.verify_batch_device(sig, msg, pk, stream=self.stream, policy=policy)
        t.cuda.synchronize()
        times = []
        for _ in range(reps):
            a, b = t.cuda.Event(enable_timing=True), t.cuda.Event(enable_timing=True)
            a.record(self.stream)
            self.V.verify_batch_device(sig, msg, pk, out_words=words, stream=self.stream, policy=policy)
            b.record(self.stream)
            t.cuda.synchronize()
            times.append(a.elapsed_time(b) * 1e-3)
        return self.V.words_to_bool(words, sig.shape[0]), float(np.median(times))

    def phase_split(self, fn, reps=3):
        """ms per verify chunk (<= 2^20 signatures) of each verify phase, from
        libstl's phase clock (HIP events between the kernels) over `reps` calls."""
        V = self.V
        V.set_phase_timing(True)
        V.reset_stats()
        try:
            for _ in range(reps):
                fn()
            self.torch.cuda.synchronize()
            st = V.get_stats()
        finally:
            V.set_phase_timing(False)
        c = max(1, st["phase_chunks"])
        return {k: v / c / 1e6 for k, v in st["phase_ns"].items()}

    def tx_hash_dev(self, d_blob, d_off, d_len, n, d_msg):
        N = self.N
        N.check(N.load().stl_tx_hash_batch_device(
            ctypes.c_void_p(d_blob.data_ptr()), ctypes.c_void_p(d_off.data_ptr()), ctypes.c_void_p(d_len.data_ptr()),
            n, ctypes.c_void_p(d_msg.data_ptr()), ctypes.c_void_p(self.stream.cuda_stream)), "tx_hash")


# ------------------------------------------------------------ data shapes
def adversarial_pool():
    g = np.load(os.path.join(ROOT, "tests", "golden", "ed25519_golden.npz"), allow_pickle=False)
    names = [str(x) for x in g["class_names"]]
    valid = names.index("valid")
    idx = np.nonzero(g["cls"] != valid)[0]
    return g["sig"][idx], g["msg"][idx], g["pk"][idx], g["cls"][idx], names


def mutated_batch(gpu, n, seed, frac=0.02):
    """n GPU-signed valid signatures; a fraction replaced by golden adversarial rows."""
    rng = np.random.default_rng(seed)
    seeds = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    msgs = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    pk, sig = gpu.sign(seeds, msgs)
    sig, pk = sig.cpu().numpy(), pk.cpu().numpy()
    asig, amsg, apk, acls, names = adversarial_pool()
    rows = rng.choice(n, int(n * frac), replace=False)
    pick = rng.integers(0, asig.shape[0], rows.size)
    sig[rows], msgs[rows], pk[rows] = asig[pick], amsg[pick], apk[pick]
    classes = {names[c]: int((acls[pick] == c).sum()) for c in np.unique(acls[pick])}
    return sig, msgs, pk, classes


# ------------------------------------------------------------------ configs
def tx_config(gpu, cpu, n, rng, pad_lens, cpu_samples):
    t = gpu.torch
    nacc = 1000
    acc_seeds = rng.integers(0, 256, (nacc, 32), dtype=np.uint8)
    apk, _ = gpu.sign(acc_seeds, np.zeros((nacc, 32), np.uint8))
    apk = apk.cpu().numpy()
    pre = payment_preimages(apk, n, rng, pad_lens)
    blob, offs, lens = pack(pre)
    d_blob = t.from_numpy(blob).cuda()
    d_off = t.from_numpy(offs.view(np.int64)).cuda()
    d_len = t.from_numpy(lens.view(np.int32)).cuda()
    d_msg = t.empty((n, 32), dtype=t.uint8, device="cuda")
    gpu.tx_hash_dev(d_blob, d_off, d_len, n, d_msg)
    seeds = acc_seeds[np.arange(n) % nacc]
    pk, sig = gpu.V.sign_batch_device(t.from_numpy(seeds).cuda(), d_msg)
    t.cuda.synchronize()
    sig_np, pk_np = sig.cpu().numpy(), pk.cpu().numpy()
    # device-resident checkSign: SHA512Half kernel + verify kernels, one stream
    words = t.empty((n + 63) // 64, dtype=t.int64, device="cuda")
    times = []
    for _ in range(6):
        a, b = t.cuda.Event(enable_timing=True), t.cuda.Event(enable_timing=True)
        a.record(gpu.stream)
        gpu.tx_hash_dev(d_blob, d_off, d_len, n, d_msg)
        gpu.V.verify_batch_device(sig, d_msg, pk, out_words=words, stream=gpu.stream)
        b.record(gpu.stream)
        t.cuda.synchronize()
        times.append(a.elapsed_time(b) * 1e-3)
    dev_bits = gpu.V.words_to_bool(words, n)
    dev_s = float(np.median(times[1:]))
    # the same with STL_DEDUP_KEYS (1,000 signers: each key decoded once per batch)
    times = []
    for _ in range(6):
        a, b = t.cuda.Event(enable_timing=True), t.cuda.Event(enable_timing=True)
        a.record(gpu.stream)
        gpu.tx_hash_dev(d_blob, d_off, d_len, n, d_msg)
        gpu.V.verify_batch_device(sig, d_msg, pk, out_words=words, stream=gpu.stream, policy=gpu.V.DEDUP_KEYS)
        b.record(gpu.stream)
        t.cuda.synchronize()
        times.append(a.elapsed_time(b) * 1e-3)
    dedup_bits = gpu.V.words_to_bool(words, n)
    dedup_s = float(np.median(times[1:]))
    phase = gpu.phase_split(lambda: gpu.V.verify_batch_device(sig, d_msg, pk, out_words=words, stream=gpu.stream))
    phase_dd = gpu.phase_split(lambda: gpu.V.verify_batch_device(sig, d_msg, pk, out_words=words, stream=gpu.stream,
                                                                 policy=gpu.V.DEDUP_KEYS))
    # host API (PCIe-inclusive): one stl_tx_verify_batch call on packed host buffers
    bm = np.zeros((n + 7) // 8, np.uint8)
    B = lambda a: a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
    call = lambda: gpu.N.check(gpu.N.load().stl_tx_verify_batch(  # noqa: E731
        B(blob), B(offs), B(lens), B(sig_np), B(pk_np), n, B(bm), 0), "stl_tx_verify_batch")
    call()
    _, host_s = timed(call)
    host_bits = np.unpackbits(bm, bitorder="little")[:n].astype(bool)
    ref_bits, ref_s = timed(lambda: cpu.tx_verify(blob, offs, lens, sig_np, pk_np, 16))

    def run(lo, hi, threads):
        return cpu.tx_verify(blob, offs[lo:hi], lens[lo:hi], sig_np[lo:hi], pk_np[lo:hi], threads)

    log("  from serialized transactions")
    from_blobs = blob_leg(gpu, cpu, blobs_from_preimages(pre, sig_np, pk_np), cpu_samples)
    return {
        "from_serialized_transactions": from_blobs,
        "n": n, "preimage_bytes": {"min": int(lens.min()), "median": int(np.median(lens)), "max": int(lens.max()),
                                   "total": int(lens.sum())},
        "gpu_device_resident_tx_per_s": n / dev_s, "gpu_device_ms": dev_s * 1e3,
        "gpu_device_resident_dedup_keys_tx_per_s": n / dedup_s, "gpu_device_dedup_keys_ms": dedup_s * 1e3,
        "gpu_phase_ms": phase, "gpu_phase_ms_dedup_keys": phase_dd,
        "gpu_host_api_tx_per_s": n / host_s,
        "cpu_reference": cpu_rates(run, n, cpu_samples),
        "bitmap_parity": {"rows": n, "mismatches_device": int((dev_bits != ref_bits).sum()),
                          "mismatches_device_dedup_keys": int((dedup_bits != ref_bits).sum()),
                          "mismatches_host_api": int((host_bits != ref_bits).sum()),
                          "accepted": int(ref_bits.sum())},
        "cpu_full_run_16_threads_s": ref_s,
    }


def blob_leg(gpu, cpu, blobs, cpu_samples):
    """checkSign from serialized transactions: libstl's canonical-form pass +
    spliced signing hash + transaction ID + verify, vs the reference path
    (parse, re-serialise, OpenSSL SHA512, libsodium) on the CPU."""
    t = gpu.torch
    buf, offs, lens = pack(blobs)
    buf = np.concatenate([buf, np.zeros(4, np.uint8)])
    n = len(blobs)
    d_buf = t.from_numpy(buf).cuda()
    d_off = t.from_numpy(offs.view(np.int64)).cuda()
    d_len = t.from_numpy(lens.view(np.int32)).cuda()
    words = t.empty((n + 63) // 64, dtype=t.int64, device="cuda")
    times = []
    for _ in range(6):
        a, b = t.cuda.Event(enable_timing=True), t.cuda.Event(enable_timing=True)
        a.record(gpu.stream)
        o = gpu.V.tx_blob_prepare_device(d_buf, d_off, d_len, tx_ids=True, stream=gpu.stream)
        gpu.V.verify_batch_device(o["sig"], o["msg"], o["pk"], out_words=words, stream=gpu.stream)
        b.record(gpu.stream)
        t.cuda.synchronize()
        times.append(a.elapsed_time(b) * 1e-3)
    dev_bits = gpu.V.words_to_bool(words, n)
    status = o["status"].cpu().numpy()
    dev_s = float(np.median(times[1:]))
    # prepare kernel alone (canonical pass + both hashes)
    ptimes = []
    for _ in range(4):
        a, b = t.cuda.Event(enable_timing=True), t.cuda.Event(enable_timing=True)
        a.record(gpu.stream)
        gpu.V.tx_blob_prepare_device(d_buf, d_off, d_len, tx_ids=True, stream=gpu.stream)
        b.record(gpu.stream)
        t.cuda.synchronize()
        ptimes.append(a.elapsed_time(b) * 1e-3)
    # host API (PCIe-inclusive): one stl_tx_blob_verify_batch call on packed host buffers
    bm = np.zeros((n + 7) // 8, np.uint8)
    hst = np.zeros(n, np.uint8)
    B = lambda a: a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
    call = lambda: gpu.N.check(gpu.N.load().stl_tx_blob_verify_batch(  # noqa: E731
        B(buf), B(offs), B(lens), n, B(bm), B(hst), None, 0), "stl_tx_blob_verify_batch")
    call()
    _, host_s = timed(call)
    hbits = np.unpackbits(bm, bitorder="little")[:n].astype(bool)
    ref_bits, ref_s = timed(lambda: cpu.tx_blob_verify(buf, offs, lens, 16))

    def run(lo, hi, threads):
        return cpu.tx_blob_verify(buf, offs[lo:hi], lens[lo:hi], threads)

    return {"n": n, "blob_bytes": {"min": int(lens.min()), "median": int(np.median(lens)), "max": int(lens.max())},
            "gpu_device_resident_tx_per_s": n / dev_s, "gpu_device_ms": dev_s * 1e3,
            "gpu_prepare_kernel_ms": float(np.median(ptimes[1:])) * 1e3,
            "gpu_host_api_tx_per_s": n / host_s,
            "status_counts": {str(k): int((status == k).sum()) for k in (0, 1, 2)},
            "cpu_reference": cpu_rates(run, n, cpu_samples),
            "bitmap_parity": {"rows": n, "mismatches_device": int((dev_bits != ref_bits).sum()),
                              "mismatches_host_api": int((hbits != ref_bits).sum()), "accepted": int(ref_bits.sum())}}


def config2(gpu, cpu):
    t = gpu.torch
    n = 1 << 20
    rng = np.random.default_rng(0x5EED0002)
    seeds = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    msgs = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    pk, sig = gpu.sign(seeds, msgs)
    d_msg = t.from_numpy(msgs).cuda()
    bits, dev_s = gpu.verify_dev(sig, d_msg, pk)
    dbits, dedup_s = gpu.verify_dev(sig, d_msg, pk, policy=gpu.V.DEDUP_KEYS)  # all keys distinct: overhead only
    phase = gpu.phase_split(lambda: gpu.V.verify_batch_device(sig, d_msg, pk, stream=gpu.stream))
    phase_dd = gpu.phase_split(lambda: gpu.V.verify_batch_device(sig, d_msg, pk, stream=gpu.stream,
                                                                 policy=gpu.V.DEDUP_KEYS))
    s_np, p_np = sig.cpu().numpy(), pk.cpu().numpy()
    hb, host_s = timed(lambda: gpu.V.verify_batch(s_np, msgs, p_np))
    hb, host_s = timed(lambda: gpu.V.verify_batch(s_np, msgs, p_np))

    def run(lo, hi, threads):
        return cpu.verify(s_np[lo:hi], msgs[lo:hi], p_np[lo:hi], threads)

    sample = 1 << 18
    ref = run(0, sample, 16)
    return {"n": n, "gpu_device_resident_verifies_per_s": n / dev_s, "gpu_device_ms": dev_s * 1e3,
            "gpu_device_dedup_keys_ms_all_distinct": dedup_s * 1e3, "dedup_bits_equal": bool((dbits == bits).all()),
            "gpu_phase_ms": phase, "gpu_phase_ms_dedup_keys_all_distinct": phase_dd,
            "gpu_host_api_verifies_per_s": n / host_s,
            "cpu_reference": cpu_rates(run, n, [(16, 1 << 19), (6, 1 << 18), (1, 1 << 15)]),
            "bitmap_parity": {"rows": sample, "mismatches": int((bits[:sample] != ref).sum()),
                              "all_gpu_accepted": bool(bits.all()), "host_api_equal": bool((hb == bits).all())}}


def adversarial(gpu, cpu, n, seed, chunk):
    t = gpu.torch
    tot_mis, tot_acc, tot_rows, gpu_s, cpu_s = 0, 0, 0, 0.0, 0.0
    classes = {}
    for c0 in range(0, n, chunk):
        m = min(chunk, n - c0)
        sig, msg, pk, cls = mutated_batch(gpu, m, seed + c0)
        for k, v in cls.items():
            classes[k] = classes.get(k, 0) + v
        d = [t.from_numpy(np.ascontiguousarray(a)).cuda() for a in (sig, msg, pk)]
        bits, s = gpu.verify_dev(*d, reps=3)
        gpu_s += s
        ref, dt = timed(lambda: cpu.verify(sig, msg, pk, 16))
        cpu_s += dt
        tot_mis += int((bits != ref).sum())
        tot_acc += int(ref.sum())
        tot_rows += m
        log(f"  rows {tot_rows}: mismatches {tot_mis}")
    return {"n": tot_rows, "adversarial_rows_by_class": classes, "mismatches": tot_mis, "accepted": tot_acc,
            "gpu_device_resident_verifies_per_s": tot_rows / gpu_s, "cpu_16_threads_verifies_per_s": tot_rows / cpu_s}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=None)
    ap.add_argument("--parity64m", action="store_true")
    ap.add_argument("--skip", default="", help="comma list of configs to skip (1,2,4,5)")
    args = ap.parse_args()
    skip = set(args.skip.split(",")) - {""}
    gpu, cpu = Gpu(), CpuRef()
    rep = {"cpu_reference": f"libsodium {cpu.version} crypto_sign_verify_detached + S<L, OpenSSL SHA512 "
                            "(oracle/_ref/libsodium_ref.so)", "cpu_threads_box_share": 16,
           "gpu": "1 x MI355X (gfx950), libstl"}
    if "1" not in skip:
        log("config 1")
        rep["config1_payment_checksign_100k"] = tx_config(
            gpu, cpu, 100000, np.random.default_rng(0x5EED0001), None, [(16, 100000), (6, 100000), (1, 20000)])
    if "2" not in skip:
        log("config 2")
        rep["config2_1M_signatures"] = config2(gpu, cpu)
    if "4" not in skip:
        log("config 4")
        rep["config4_10M_adversarial"] = adversarial(gpu, cpu, 10_000_000, 0x5EED0004, 2_000_000)
    if "5" not in skip:
        log("config 5")
        rng = np.random.default_rng(0x5EED0005)
        n5 = 1 << 20
        pads = np.exp(rng.uniform(np.log(100), np.log(4096), n5))
        rep["config5_ledger_replay_1M"] = tx_config(gpu, cpu, n5, rng, pads, [(16, 1 << 20), (6, 1 << 18), (1, 1 << 14)])
    if args.parity64m:
        log("config 3 parity (64M)")
        rep["config3_64M_parity"] = adversarial(gpu, cpu, 1 << 26, 0x5EED0003, 1 << 22)
    doc = json.dumps(rep, indent=1)
    print(doc)
    if args.out:
        with open(args.out, "w") as f:
            f.write(doc)


if __name__ == "__main__":
    main()
