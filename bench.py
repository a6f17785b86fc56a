#!/usr/bin/env python3
"""bench.py -- Ed25519 tx-signature verifies/s on MI355X (BASELINE.json metric).

Workload (BASELINE.json configs[1]): 1,048,576 fixed-size Payment-tx
signatures per GPU -- (R||S, 32-byte signing hash, pk) in SoA HBM buffers,
all valid, signed on the GPU from seeded random keys/hashes before timing.
One "step" = one stl_ed25519_verify_batch_device call over the whole batch
(SHA-512(R||A||M), decompress, [k](-A)+[S]B, encode/compare, ballot bitmap),
plus -- at N > 1 -- the RCCL all-gather of every rank's accept bitmap (the
path's only exchange step).  Shards are independent per rank
(weak scaling: every rank verifies its own 1,048,576 signatures).

  python bench.py [--gpus N] [--steps K] [--warmup W] [--n PER_GPU]
  (N > 1: launched by torch.distributed.run, one process per GPU, RCCL)

Prints ONE JSON line on rank 0.  roofline: integer-VALU bound; achieved =
W_VERIFY int ops per verify (frozen) x verifies per kernel launch /
average kernel time measured with HIP events on the launch stream.
cpu_baseline: the reference's verify call path (libsodium 1.0.18
crypto_sign_verify_detached + stellard S<L, oracle/_ref/libsodium_ref.so) --
or the oracle port when libsodium is absent -- on a bounded sample, rank 0 only.
"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

# Frozen work model (DESIGN.md "Roofline"): 64*N_M + 36*N_S + 5520*B_k with the
# ref10 operation counts N_M = 1520, N_S = 1525 measured by instrumenting the
# oracle's restatement of libsodium's verify (oracle_op_counts), B_k = 1.
W_VERIFY = 64 * 1520 + 36 * 1525 + 5520
# gfx950 full-rate 32-bit VALU peak: 256 CU x 4 SIMD x 32 lanes x 2.4 GHz
PEAK_INT_OPS = 256 * 4 * 32 * 2.4e9
HBM_PEAK_GBS = 8000.0
BYTES_PER_VERIFY = 64 + 32 + 32 + 1.0 / 8  # algorithmic HBM bytes (sig, msg, pk in; 1 bit out)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--n", type=int, default=1 << 20, help="signatures per GPU")
    ap.add_argument("--cpu-sample", type=int, default=1 << 19)
    ap.add_argument("--cpu-threads", type=int, default=16)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    return ap.parse_args()


def cpu_baseline(sig, msg, pk, sample, threads):
    """Host-core baseline on a bounded sample of the same workload."""
    from tests import oracle_bind
    n = min(sample, sig.shape[0])
    s, m, p = (np.ascontiguousarray(a[:n]) for a in (sig, msg, pk))
    threads = max(1, min(threads, os.cpu_count() or 1))
    lib = oracle_bind.load_sodium_ref()
    if lib is not None:
        kind = "reference"
        run = lambda: oracle_bind.sodium_verify_batch(lib, s, m, p, threads=threads)  # noqa: E731
        what = (f"libsodium {lib.ref_sodium_version().decode()} crypto_sign_verify_detached + S<L "
                "(RippleAddress::verifySignature call path)")
    else:
        o = oracle_bind.load_oracle()
        kind = "port"
        run = lambda: o.verify_batch(s, m, p, threads=threads)  # noqa: E731
        what = "oracle/stl_oracle.c restatement"
    run()  # warm
    t0 = time.perf_counter()
    bits = run()
    dt = time.perf_counter() - t0
    return {"value": n / dt, "unit": "verifies/s", "cores": threads, "kind": kind,
            "sample": f"{n} signatures of the bench batch, {threads} threads, {what}; "
                      f"{int(bits.sum())}/{n} accepted; {dt:.2f} s wall"}


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(0)
    from stellard_amd import shard
    from stellard_amd import verify as V

    V.init(device_count=1, first_device=torch.cuda.current_device())
    dev = torch.device("cuda", torch.cuda.current_device())
    n = args.n

    # ---- synthetic data (outside the timed region) ----
    rng = np.random.default_rng(0x5EED0002 + rank)
    seeds = torch.from_numpy(rng.integers(0, 256, (n, 32), dtype=np.uint8)).to(dev)
    msgs = torch.from_numpy(rng.integers(0, 256, (n, 32), dtype=np.uint8)).to(dev)
    pk, sig = V.sign_batch_device(seeds, msgs)
    torch.cuda.synchronize()
    words = torch.empty((n + 63) // 64, dtype=torch.int64, device=dev)
    full_words = None
    stream = torch.cuda.current_stream()

    def gather():
        # rank r holds global indices [r*n, (r+1)*n): shard.shard_range(n*world, r, world)
        return shard.gather_bitmap_words(words, n * world, world, dist)

    def step():
        V.verify_batch_device(sig, msgs, pk, out_words=words, stream=stream)
        if world > 1:
            gather()

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    ok = V.words_to_bool(words, n)
    if not ok.all():
        raise SystemExit(f"rank {rank}: {int((~ok).sum())} valid signatures rejected -- parity failure")

    # ---- timed region: exactly K steps between barrier+sync on both sides ----
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    t0 = time.perf_counter()
    for k in range(args.steps):
        ev[k][0].record(stream)
        V.verify_batch_device(sig, msgs, pk, out_words=words, stream=stream)
        ev[k][1].record(stream)
        if world > 1:
            full_words = gather()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    kern_ms = float(np.mean([a.elapsed_time(b) for a, b in ev]))
    t = torch.tensor([dt, kern_ms], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    dt, kern_ms = float(t[0]), float(t[1])
    if world > 1:
        assert V.words_to_bool(full_words, n * world).all()

    if rank == 0:
        total = n * world * args.steps
        value = total / dt
        per_launch = n / (kern_ms * 1e-3)
        achieved = W_VERIFY * per_launch / 1e12
        traffic = None
        tp = os.path.join(ROOT, "profiles", "traffic_latest.json")
        if os.path.exists(tp):
            with open(tp) as f:
                traffic = json.load(f).get("hbm_bytes_per_launch")
        valu_busy = None
        vp = os.path.join(ROOT, "profiles", "valu_latest.json")
        if os.path.exists(vp):
            with open(vp) as f:
                vd = json.load(f)
            valu_busy = {"launch_pct": vd.get("launch_valu_busy_pct"),
                         "per_kernel_pct": {k: v.get("VALUBusy") for k, v in vd.get("kernels", {}).items()},
                         "source": "rocprofv3 --pmc VALUBusy of this build, profiles/valu_latest.json"}
        line = {
            "metric": "Ed25519 tx verifies/sec",
            "value": value,
            "unit": "verifies/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": dt * 1e3 / args.steps,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u32",
            "data": "synthetic: GPU-signed RFC 8032 signatures over seeded random keys and 32-byte signing hashes",
            "config": {"workload": "configs[1]: 1,048,576 fixed-size Payment-tx signatures per GPU "
                                   "(stl_ed25519_verify_batch_device, policy libsodium-1.0.18 + S<L)",
                       "signatures_per_gpu": n, "parallelism": f"dp{world} (index shards, RCCL bitmap all-gather)"},
            "roofline": {"bound": "valu", "achieved": achieved, "peak": PEAK_INT_OPS / 1e12, "unit": "Tops/s",
                         "frac": achieved * 1e12 / PEAK_INT_OPS, "traffic": traffic,
                         "kernel_ms": kern_ms, "work_per_verify": W_VERIFY,
                         "kernels": "verify_scalar + verify_point + verify_main + verify_fallback, one stream, HIP events around "
                                    "each stl_ed25519_verify_batch_device call",
                         "hbm_frac": BYTES_PER_VERIFY * per_launch / (HBM_PEAK_GBS * 1e9),
                         "valu_busy_pmc": valu_busy},
            "cpu_baseline": None,
        }
        if world == 1 and not args.no_cpu_baseline:
            try:
                line["cpu_baseline"] = cpu_baseline(sig.cpu().numpy(), msgs.cpu().numpy(), pk.cpu().numpy(),
                                                    args.cpu_sample, args.cpu_threads)
            except Exception as e:  # noqa: BLE001 - the baseline must not kill the GPU number
                line["cpu_baseline"] = {"error": repr(e)}
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
