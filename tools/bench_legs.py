"""Sharded, digest-checked legs of bench.py (BASELINE.json configs[2]-[4]).

Each leg runs at every N with one rank per GPU and proves bit-exactness of
the *gathered* result, not only of each rank's own slice:

  config3_64M_digest       configs[2]: the 67,108,864-row dataset of
                           tests/datasets.py (2 % adversarial rows over the
                           Appendix-B classes B1-B11), index shards of whole
                           65,536-row blocks, ncclGather to rank 0
                           (stl_bitmap_gather_device);
  config4_10M_digest       configs[3]: the 10,000,000-row adversarial set, the
                           same block shards -- unequal at N = 2, 4, 8 (153
                           blocks, the last one partial) -- gathered with
                           stl_bitmap_gatherv_device;
  config5_ledger_split     configs[4]: ONE ledger of 2^20 signed preimages
                           (113 B - 4 KB, 1,000 signers, 2 % invalid rows) split
                           by preimage bytes (stl_shard_range_bytes), SHA512Half +
                           verify per rank, stl_bitmap_gatherv_device;
  config5_blob_split       configs[4] from serialized transactions: ONE ledger of
                           2^20 canonical Payment blobs (100 B - 4 KB, 2 % invalid,
                           deferred and malformed rows) split by blob bytes,
                           stl_signed_blob_verify_batch_device per rank, accept
                           words and status bytes gathered, both digests checked.

Every rank rebuilds only its own rows (the device signer and adversarial-row
builder, stl_debug_sign_adversarial_device, from the seeded plans), checks its
inputs against the committed per-block digests (tests/golden/
block_digests.json, made with libsodium by tests/golden/make_digests.py),
verifies, checks its slice's per-block bitmap digests, and rank 0 compares
the SHA-256 of the gathered bitmap with libsodium's
(tests/golden/bitmap_digests.json).  A misplaced, duplicated, missing or
stale rank slice changes that digest (tests/test_multigpu_host.py shifts one
rank's words in the CPU rehearsal and expects digest_equal false).

The predicate sharded here is RippleAddress::verifySignature
(/root/reference/src/ripple_data/protocol/RippleAddress.cpp:190-200); the
batch split over ranks replaces the JobQueue worker pool
(src/ripple_core/functional/JobQueue.cpp:217-243) and, for config 5, one
ledger's transaction set (src/ripple_app/consensus/LedgerConsensus.cpp:1934-1958).
"""
import hashlib
import json
import time
from concurrent.futures import ThreadPoolExecutor

import numpy as np

from tests import datasets


def bitmap_sha256(full_words, n):
    """SHA-256 of the first n accept bits as packed bytes (LSB first), the
    form of tests/golden/bitmap_digests.json."""
    arr = full_words.cpu().numpy() if hasattr(full_words, "cpu") else np.asarray(full_words)
    b = arr.astype("<i8").view(np.uint8)[:(n + 7) // 8].copy()
    if n % 8:
        b[-1] &= (1 << (n % 8)) - 1
    return hashlib.sha256(b.tobytes()).hexdigest()


def words_h16(words):
    arr = words.cpu().numpy() if hasattr(words, "cpu") else np.asarray(words)
    return datasets.h16(arr.astype("<i8"))


class Gather:
    """Accept-bitmap words of every rank into one buffer on rank 0.

    mode "rccl": libstl (ncclGather when every slice has the same word count,
    grouped send / recv -- stl_bitmap_gatherv_device -- otherwise); "nccl":
    torch.distributed's RCCL all_gather of padded slices (used only if libstl's
    communicator could not be built); "gloo": through host memory (the
    multi-rank rehearsal on a 1-GPU box and the CPU dry run); world 1: the
    rank's own words."""

    def __init__(self, world, rank, dist, mode, V=None, stream=None, group=None):
        self.world, self.rank, self.dist, self.mode = world, rank, dist, mode
        self.V, self.stream, self.group = V, stream, group

    def __call__(self, words, offs, full):
        """words: this rank's slice (offs[rank+1] - offs[rank] int64 words);
        offs: world+1 word offsets; full: offs[-1] words on rank 0 (else None)."""
        import torch
        if self.world == 1:
            if full is not None and full.data_ptr() != words.data_ptr():
                full[:words.numel()].copy_(words)
            return
        sizes = [int(offs[r + 1] - offs[r]) for r in range(self.world)]
        equal = len(set(sizes)) == 1
        if self.mode == "rccl":
            if equal:
                self.V.bitmap_gather_device(words, full, root=0, stream=self.stream)
            else:
                self.V.bitmap_gatherv_device(words, offs, full, root=0, stream=self.stream)
            return
        mx = max(sizes)
        pad = torch.zeros(mx, dtype=torch.int64, device=words.device if self.mode == "nccl" else "cpu")
        pad[:words.numel()].copy_(words)
        parts = [torch.empty_like(pad) for _ in range(self.world)]
        if self.mode == "nccl":
            self.dist.all_gather(parts, pad, group=self.group)
        else:
            self.dist.all_gather(parts, pad)
        if self.rank == 0:
            for r in range(self.world):
                full[int(offs[r]):int(offs[r + 1])].copy_(parts[r][:sizes[r]])


def _all(dist, world, obj):
    if world == 1:
        return [obj]
    out = [None] * world
    dist.all_gather_object(out, obj)
    return out


def timed(ctx, fn, reps):
    """Median over reps of (barrier, fn, sync, barrier) on this rank, max over
    ranks (seconds)."""
    import torch
    world, dist = ctx["world"], ctx["dist"]
    ts = []
    for _ in range(reps):
        ctx["sync"]()
        if world > 1:
            dist.barrier()
        t0 = time.perf_counter()
        fn()
        ctx["sync"]()
        if world > 1:
            dist.barrier()
        ts.append(time.perf_counter() - t0)
    t = torch.tensor([float(np.median(ts))], dtype=torch.float64)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t[0])


class _BlockInputs:
    """Streams rows (from row `lo`, block aligned) into per-block input
    digests, hashed on a thread pool (hashlib releases the GIL)."""

    def __init__(self, pool):
        self.pool, self.pending, self.n, self.futs = pool, [], 0, []

    def add(self, sig, msg, pk):
        i, n = 0, sig.shape[0]
        while i < n:
            take = min(datasets.BLOCK - self.n, n - i)
            self.pending.append((sig[i:i + take], msg[i:i + take], pk[i:i + take]))
            self.n += take
            i += take
            if self.n == datasets.BLOCK:
                self._emit()

    def _emit(self):
        if self.n:
            s, m, p = (np.concatenate(x) for x in zip(*self.pending))
            self.futs.append(self.pool.submit(datasets.h16, s, m, p))
        self.pending, self.n = [], 0

    def result(self):
        self._emit()
        return [f.result() for f in self.futs]


def _gather_label(ctx, offs):
    """How the leg's bitmap slices reached rank 0 (the gloo
    rehearsal is not labelled as RCCL)."""
    equal = len(set(np.diff(offs.astype(np.int64)).tolist())) == 1
    if ctx["world"] == 1:
        return "one rank: no gather"
    if ctx["gather"].mode == "rccl":
        return "equal: ncclGather" if equal else "unequal: grouped send/recv (stl_bitmap_gatherv_device)"
    return ("equal" if equal else "unequal") + f": {ctx['gather'].mode} through host memory (not RCCL)"


def digest_leg(ctx, name, reps=3):
    """configs[2] / configs[3] on this rank's block shard; see the module
    docstring.  ctx: world, rank, dist, V, torch, dev, stream, sync, gather."""
    torch, V, dev, stream = ctx["torch"], ctx["V"], ctx["dev"], ctx["stream"]
    world, rank = ctx["world"], ctx["rank"]
    n = datasets.CONFIGS[name]["n"]
    with open(datasets.DIGESTS) as f:
        want = json.load(f)[name]
    with open(datasets.BLOCK_DIGESTS) as f:
        blocks = json.load(f)[name]
    lo, hi, b0, b1 = datasets.block_shard(n, rank, world)
    offs = np.array([datasets.block_shard(n, r, world)[0] // 64 for r in range(world)] + [(n + 63) // 64],
                    np.uint64)
    m = hi - lo
    err, inputs_ok = None, False
    try:
        sig = torch.empty((m, 64), dtype=torch.uint8, device=dev)
        msg = torch.empty((m, 32), dtype=torch.uint8, device=dev)
        pk = torch.empty((m, 32), dtype=torch.uint8, device=dev)
        t0 = time.time()
        with ThreadPoolExecutor(8) as pool:
            bi = _BlockInputs(pool)
            for a, seeds, msgs, cls, param in datasets.rows_plan(name, lo, hi):
                k = seeds.shape[0]
                t = [torch.from_numpy(np.ascontiguousarray(x)).to(dev)
                     for x in (seeds, msgs, cls, param.view(np.int32))]
                p_, s_, m_ = V.sign_adversarial_device(*t)
                sig[a - lo:a - lo + k] = s_
                msg[a - lo:a - lo + k] = m_
                pk[a - lo:a - lo + k] = p_
                bi.add(s_.cpu().numpy(), m_.cpu().numpy(), p_.cpu().numpy())
            got_in = bi.result()
        build_s = time.time() - t0
        inputs_ok = got_in == blocks["inputs_h16"][b0:b1]
        words = torch.zeros((m + 63) // 64, dtype=torch.int64, device=dev)
        full = torch.zeros(int(offs[-1]), dtype=torch.int64, device=dev) if rank == 0 else None
        if world > 1 and ctx["gather"].mode == "gloo" and rank == 0:
            full = full.cpu()
        V.verify_batch_device(sig, msg, pk, out_words=words, stream=stream)
        ctx["sync"]()
        bits = V.words_to_bool(words, m)
        got_bits = [datasets.h16(np.packbits(bits[i:i + datasets.BLOCK], bitorder="little"))
                    for i in range(0, m, datasets.BLOCK)]
        slice_ok = got_bits == blocks["bitmap_h16"][b0:b1]
    except Exception as e:  # noqa: BLE001 - every rank learns of it before the leg's collectives
        err = f"rank {rank}: {e!r}"
    fault = ctx.get("fault")
    st = _all(ctx["dist"], world, (err, bool(inputs_ok)))
    if any(e for e, _ in st):
        return {"error": "; ".join(e for e, _ in st if e)}
    if not all(o for _, o in st):
        return {"error": f"input block digests differ on ranks {[r for r, (_, o) in enumerate(st) if not o]}"}

    def step():
        V.verify_batch_device(sig, msg, pk, out_words=words, stream=stream)
        if fault:
            fault(words)
        ctx["gather"](words, offs, full)

    dt = timed(ctx, step, reps)
    slices = _all(ctx["dist"], world, {"rank": rank, "rows": [lo, hi], "slice_bitmap_blocks_equal": bool(slice_ok),
                                       "accepted": int(bits.sum())})
    out = {"rows": n, "n_ranks": world, "verifies_per_s": n / dt, "ms": dt * 1e3, "median_of": reps,
           "shards": "whole 65,536-row blocks per rank (datasets.block_shard), " + _gather_label(ctx, offs),
           "rank_slices": slices, "build_s": build_s,
           "data": "tests/datasets.py %s, rows rebuilt per rank by the device signer + adversarial-row builder, "
                   "inputs checked per 65,536-row block against libsodium-built digests" % name,
           "timing": "barrier, one verify call per rank over its resident rows + gather to rank 0, sync, "
                     "barrier; median, max over ranks"}
    if rank == 0:
        dg = bitmap_sha256(full, n)
        acc = int(np.unpackbits(full.cpu().numpy().astype("<i8").view(np.uint8), bitorder="little")[:n].sum())
        out.update({"accepted": acc, "accepted_expected": want["accepted"],
                    "bitmap_sha256": dg, "digest_equal": dg == want["bitmap_sha256"],
                    "expected_from": want.get("expected_from")})
    return out


def ledger_leg(ctx, reps=5):
    """configs[4]: one ledger split across the ranks by preimage bytes."""
    torch, V, dev, stream = ctx["torch"], ctx["V"], ctx["dev"], ctx["stream"]
    world, rank = ctx["world"], ctx["rank"]
    with open(datasets.DIGESTS) as f:
        want = json.load(f)["config5"]
    err, inputs = None, None
    try:
        t0 = time.time()
        lp = datasets.ledger_plan()
        n = lp["n"]
        d_pre = torch.from_numpy(lp["pre"]).to(dev)
        d_off = torch.from_numpy(lp["offs"]).to(dev)
        d_len = torch.from_numpy(lp["lens"]).to(dev)
        seeds = torch.from_numpy(np.ascontiguousarray(lp["signers"][lp["who"]])).to(dev)
        msgs = V.tx_hash_batch_device(d_pre, d_off, d_len, stream=stream)
        pk, sig = V.sign_batch_device(seeds, msgs)
        (pos, pbit), (srow, scol, sbit) = datasets.ledger_mutations(lp)
        d_pre[torch.from_numpy(pos).to(dev)] ^= torch.from_numpy(pbit).to(dev)
        sig[torch.from_numpy(srow).to(dev), torch.from_numpy(scol).to(dev)] ^= torch.from_numpy(sbit).to(dev)
        ctx["sync"]()
        inputs = datasets.ledger_input_digest(d_pre.cpu().numpy(), lp["total"], lp["lens"], sig.cpu().numpy(),
                                              pk.cpu().numpy())
        build_s = time.time() - t0
        bounds = [V.shard_range_bytes(lp["lens"], r, world) for r in range(world)]
        lo, hi = bounds[rank]
        offs = np.array([b[0] // 64 for b in bounds] + [(n + 63) // 64], np.uint64)
        m = hi - lo
        m5 = torch.empty((n, 32), dtype=torch.uint8, device=dev)
        words = torch.zeros((m + 63) // 64, dtype=torch.int64, device=dev)
        full = torch.zeros(int(offs[-1]), dtype=torch.int64, device=dev) if rank == 0 else None
        if world > 1 and ctx["gather"].mode == "gloo" and rank == 0:
            full = full.cpu()
    except Exception as e:  # noqa: BLE001 - every rank learns of it before the leg's collectives
        err = f"rank {rank}: {e!r}"
    st = _all(ctx["dist"], world, (err, inputs == want["inputs_h16"]))
    if any(e for e, _ in st):
        return {"error": "; ".join(e for e, _ in st if e)}
    if not all(o for _, o in st):
        return {"error": f"ledger input digest differs on ranks {[r for r, (_, o) in enumerate(st) if not o]}"}

    def step(flags, fused=True):
        if m and fused:  # one call: hashing and verify chunk by chunk over two streams
            V.tx_verify_batch_device(d_pre, d_off[lo:hi], d_len[lo:hi], sig[lo:hi], pk[lo:hi], out_words=words,
                                     policy=flags, stream=stream)
        elif m:
            V.tx_hash_batch_device(d_pre, d_off[lo:hi], d_len[lo:hi], out_msg=m5[lo:hi], stream=stream)
            V.verify_batch_device(sig[lo:hi], m5[lo:hi], pk[lo:hi], out_words=words, policy=flags, stream=stream)
        ctx["gather"](words, offs, full)

    step(V.DEDUP_KEYS)  # warm: the dedup workspaces are allocated outside the timed reps
    step(0)
    ctx["sync"]()
    res = {}
    # default flags: the device API's automatic dedup follows the previous
    # call's key sample (the warm-up call above sampled this ledger's 1,000
    # signers); forced on; forced off
    for label, flags in (("", 0), ("_dedup_keys", V.DEDUP_KEYS), ("_no_dedup", V.NO_AUTO_DEDUP)):
        dt = timed(ctx, lambda: step(flags), reps)  # noqa: B023 - called right here
        res["tx_per_s" + label] = n / dt
        res["ms" + label] = dt * 1e3
        if rank == 0:
            res["digest_equal" + label] = bitmap_sha256(full, n) == want["bitmap_sha256"]
    # the two-step path (tx_hash_batch_device, then verify_batch_device) for comparison
    dt = timed(ctx, lambda: step(0, fused=False), reps)
    res["tx_per_s_two_step"] = n / dt
    if rank == 0:
        res["digest_equal_two_step"] = bitmap_sha256(full, n) == want["bitmap_sha256"]
    small = small_ledgers(ctx, lp, d_pre, d_off, d_len, sig, pk)
    pre_bytes = [int(lp["offs"][b[1] - 1] + lp["lens"][b[1] - 1] - lp["offs"][b[0]]) if b[1] > b[0] else 0
                 for b in bounds]
    out = {"transactions": n, "n_ranks": world, "scaling": "strong (one ledger split across the ranks)",
           "preimage_bytes": lp["total"], "byte_shards": [list(map(int, b)) for b in bounds],
           "preimage_bytes_per_rank": pre_bytes, "median_of": reps, "build_s": build_s, **res,
           "invalid_rows": int(lp["bad"].size),
           "data": "tests/datasets.py ledger_plan: 'STX\\0' + random bytes, lengths log-uniform in [113, 4096], "
                   "1,000 signers, GPU-signed over SHA512Half, 2 % of the rows with a preimage / R / S bit "
                   "flipped after signing; every rank builds the whole ledger and checks its input digest",
           "timing": "barrier, SHA512Half + verify of the rank's byte shard (stl_tx_verify_batch_device; "
                     "tx_per_s_two_step: tx_hash_batch_device then verify_batch_device) + gather to rank 0 "
                     "(stl_bitmap_gatherv_device), sync, barrier; median, max over ranks"}
    if rank == 0:
        out.update({"accepted_expected": want["accepted"], "bitmap_sha256_expected": want["bitmap_sha256"]})
    out["small_ledgers"] = small
    return out


def blob_ledger_leg(ctx, reps=5):
    """configs[4] as a ledger close feeds it: ONE ledger of
    2^20 serialized Payment transactions (tests/datasets.py blob_ledger_plan:
    canonical blobs memo-padded to log-uniform 100 B - 4 KB, 1,000 signers, 2 %
    invalid -- payload / R / S bits flipped after signing, Flags and Sequence
    swapped (deferred), 33-byte keys (malformed)) split by blob bytes
    (stl_shard_range_bytes); each rank runs stl_signed_blob_verify_batch_device
    over its shard -- the canonical-form walk, TxFormats check, splice,
    SHA512Half and verify -- and the accept words and per-row status bytes are
    gathered to rank 0 (stl_bitmap_gatherv_device), which compares their
    SHA-256 with the committed reference digests (tests/golden/make_digests.py
    config5b: re-serialise + OpenSSL + libsodium per row).  The reference path
    replaced: LedgerConsensus.cpp:1947-1958 -> SerializedTransaction.cpp:65-92,
    220-230."""
    torch, V, dev, stream = ctx["torch"], ctx["V"], ctx["dev"], ctx["stream"]
    world, rank = ctx["world"], ctx["rank"]
    with open(datasets.DIGESTS) as f:
        want = json.load(f)["config5b"]
    err, inputs = None, None
    try:
        t0 = time.time()

        def signer_pks(seeds):
            z = torch.zeros((seeds.shape[0], 32), dtype=torch.uint8, device=dev)
            return V.sign_batch_device(torch.from_numpy(np.ascontiguousarray(seeds)).to(dev), z)[0].cpu().numpy()
        bp = datasets.blob_ledger_plan(signer_pks)
        n = bp["n"]
        msgs = torch.from_numpy(datasets.blob_signing_hashes(bp)).to(dev)
        _, sig = V.sign_batch_device(torch.from_numpy(np.ascontiguousarray(bp["seeds"][bp["who"]])).to(dev), msgs)
        datasets.blob_ledger_finish(bp, sig.cpu().numpy())
        inputs = datasets.blob_ledger_inputs_h16(bp)
        build_s = time.time() - t0
        d_buf = torch.from_numpy(bp["buf"]).to(dev)
        d_off = torch.from_numpy(bp["offs"]).to(dev)
        d_len = torch.from_numpy(bp["lens"]).to(dev)
        bounds = [V.shard_range_bytes(bp["lens"], r, world) for r in range(world)]
        lo, hi = bounds[rank]
        m = hi - lo
        offs = np.array([b[0] // 64 for b in bounds] + [(n + 63) // 64], np.uint64)
        words = torch.zeros((m + 63) // 64, dtype=torch.int64, device=dev)
        # status bytes and ids ride the same gatherv as int64 words: shards
        # start on 64-row boundaries, so a rank's status bytes are whole words
        status = torch.zeros(((m + 63) // 64) * 64, dtype=torch.uint8, device=dev)
        ids = torch.zeros((max(m, 1), 32), dtype=torch.uint8, device=dev)
        full, full_st, full_id = None, None, None
        if rank == 0:
            full = torch.zeros(int(offs[-1]), dtype=torch.int64, device=dev)
            full_st = torch.zeros(int(offs[-1]) * 8, dtype=torch.int64, device=dev)
            full_id = torch.zeros(n * 4, dtype=torch.int64, device=dev)
            if world > 1 and ctx["gather"].mode == "gloo":
                full, full_st, full_id = full.cpu(), full_st.cpu(), full_id.cpu()
    except Exception as e:  # noqa: BLE001 - every rank learns of it before the leg's collectives
        err = f"rank {rank}: {e!r}"
    st = _all(ctx["dist"], world, (err, inputs == want["inputs_h16"]))
    if any(e for e, _ in st):
        return {"error": "; ".join(e for e, _ in st if e)}
    if not all(o for _, o in st):
        return {"error": f"blob ledger input digest differs on ranks {[r for r, (_, o) in enumerate(st) if not o]}"}

    def step(flags=0, fused=True):
        if m and fused:  # one call: blob pass and verify chunk by chunk over two streams
            V.signed_blob_verify_batch_device(d_buf, d_off[lo:hi], d_len[lo:hi], out_words=words,
                                              out_status=status, policy=flags, stream=stream)
        elif m:
            o = V.tx_blob_prepare_device(d_buf, d_off[lo:hi], d_len[lo:hi], tx_ids=False, stream=stream)
            V.verify_batch_device(o["sig"], o["msg"], o["pk"], out_words=words, policy=flags, stream=stream)
        ctx["gather"](words, offs, full)

    step()  # warm: workspaces, and the key sample the automatic dedup follows
    ctx["sync"]()
    res = {}
    for label, flags in (("", 0), ("_no_dedup", V.NO_AUTO_DEDUP)):
        dt = timed(ctx, lambda: step(flags), reps)  # noqa: B023 - called right here
        res["tx_per_s" + label] = n / dt
        res["ms" + label] = dt * 1e3
        if rank == 0:
            res["digest_equal" + label] = bitmap_sha256(full, n) == want["bitmap_sha256"]
    dt = timed(ctx, lambda: step(0, fused=False), reps)
    res["tx_per_s_two_step"] = n / dt
    if rank == 0:
        res["digest_equal_two_step"] = bitmap_sha256(full, n) == want["bitmap_sha256"]
    # untimed: one call with transaction ids, then status bytes and ids gathered
    if m:
        V.signed_blob_verify_batch_device(d_buf, d_off[lo:hi], d_len[lo:hi], out_words=words, out_status=status,
                                          out_ids=ids, stream=stream)
    ctx["sync"]()
    ctx["gather"](status.view(torch.int64), offs * 8, full_st)
    ctx["gather"](ids[:m].reshape(-1).view(torch.int64) if m else ids.reshape(-1).view(torch.int64)[:0],
                  np.array([b[0] * 4 for b in bounds] + [n * 4], np.uint64), full_id)
    ctx["sync"]()
    out = {"transactions": n, "n_ranks": world, "scaling": "strong (one ledger split across the ranks)",
           "blob_bytes": bp["total"], "byte_shards": [list(map(int, b)) for b in bounds],
           "blob_bytes_per_rank": [int(bp["offs"][b[1] - 1] + bp["lens"][b[1] - 1] - bp["offs"][b[0]])
                                   if b[1] > b[0] else 0 for b in bounds],
           "median_of": reps, "build_s": build_s, **res,
           "invalid_rows": int(bp["bad"].size),
           "invalid_by_kind": want.get("invalid_by_kind"),
           "data": "tests/datasets.py blob_ledger_plan: canonical serialized Payment blobs (TransactionType .. "
                   "Destination, optional DestinationTag / IOU Amount, Memos padding to log-uniform 100 B - 4 KB), "
                   "1,000 signers, GPU-signed over hashlib SHA512Half of each signing preimage; 2 % invalid "
                   "(payload / R / S bit flips, Flags-Sequence swap -> deferred, 33-byte key -> malformed); every "
                   "rank builds the whole ledger and checks its input digest",
           "timing": "barrier, stl_signed_blob_verify_batch_device over the rank's byte shard (blob pass + verify "
                     "in one call; tx_per_s_two_step: stl_tx_blob_prepare_device then verify_batch_device) + "
                     "gather of the accept words to rank 0 (stl_bitmap_gatherv_device), sync, barrier; median, max "
                     "over ranks; status bytes and transaction ids gathered after the timed reps"}
    if rank == 0:
        stb = full_st.cpu().numpy().astype("<i8").view(np.uint8)[:n]
        idb = full_id.cpu().numpy().astype("<i8").view(np.uint8)[:n * 32]
        out.update({"accepted": int(np.unpackbits(full.cpu().numpy().astype("<i8").view(np.uint8),
                                                  bitorder="little")[:n].sum()),
                    "accepted_expected": want["accepted"], "bitmap_sha256_expected": want["bitmap_sha256"],
                    "status_counts": {str(k): int((stb == k).sum()) for k in (0, 1, 2)},
                    "status_digest_equal": hashlib.sha256(stb.tobytes()).hexdigest() == want["status_sha256"],
                    "ids_digest_equal": hashlib.sha256(idb.tobytes()).hexdigest() == want["ids_sha256"],
                    "deferred_rows_reference_accepts": "every deferred row (Flags/Sequence swapped) is accepted by "
                                                       "the reference's re-serialising checkSign -- the caller's "
                                                       "serial check answers them (STL_TX_DEFERRED)",
                    "expected_from": want.get("expected_from")})
    return out


def ledger_cuts(n, lo=1000, hi=20000):
    """Row bounds of consecutive ledgers of log-uniform size in [lo, hi]
    (ledgers of 1k-20k transactions) over n rows."""
    rng = np.random.default_rng(0x5EED0005 ^ 0x5A11)
    cuts = [0]
    while cuts[-1] < n:
        cuts.append(min(n, cuts[-1] + int(np.exp(rng.uniform(np.log(lo), np.log(hi + 1))))))
    return cuts


def small_ledgers(ctx, lp, d_pre, d_off, d_len, sig, pk, reps=3):
    """configs[4] as SURVEY 8d words it: the config-5 rows cut into ledgers of
    1k-20k transactions, each verified by ONE synchronous call (ledger close
    waits for its verdicts): stl_tx_verify_batch_device, then a stream sync.
    Ledger i goes to rank i % N.  Every ledger's bits are checked against the
    plan's invalid rows (the rows whose bits the committed libsodium digest
    rejects)."""
    torch, V, dev, stream = ctx["torch"], ctx["V"], ctx["dev"], ctx["stream"]
    world, rank = ctx["world"], ctx["rank"]
    n = lp["n"]
    cuts = ledger_cuts(n)
    mine = [(cuts[i], cuts[i + 1]) for i in range(len(cuts) - 1) if i % world == rank]
    outs = [torch.zeros((b - a + 63) // 64, dtype=torch.int64, device=dev) for a, b in mine]
    lat = []

    def run_all(record):
        for (a, b), w in zip(mine, outs):
            t0 = time.perf_counter()
            V.tx_verify_batch_device(d_pre, d_off[a:b], d_len[a:b], sig[a:b], pk[a:b], out_words=w, stream=stream)
            stream.synchronize()
            if record:
                lat.append(time.perf_counter() - t0)

    run_all(False)  # warm: workspaces, the key sample of the device API's automatic dedup
    dt = timed(ctx, lambda: run_all(True), reps)
    expect = np.ones(n, dtype=bool)
    expect[lp["bad"]] = False
    ok = all(np.array_equal(V.words_to_bool(w, b - a), expect[a:b]) for (a, b), w in zip(mine, outs))
    st = _all(ctx["dist"], world, (ok, lat))
    sizes = np.diff(np.array(cuts))
    all_lat = np.array([x for _, l in st for x in l]) * 1e3
    return {"ledgers": len(sizes), "transactions": n,
            "ledger_size": {"min": int(sizes.min()), "median": int(np.median(sizes)), "max": int(sizes.max())},
            "tx_per_s": n / dt, "ms": dt * 1e3, "median_of": reps,
            "latency_ms": {"p50": float(np.percentile(all_lat, 50)), "p99": float(np.percentile(all_lat, 99)),
                           "max": float(all_lat.max())},
            "bits_equal_expected": all(o for o, _ in st),
            "timing": "per ledger: host clock around one stl_tx_verify_batch_device call + stream sync (a "
                      "ledger close waits for its verdicts); ledgers one after another on each rank, ledger i "
                      "on rank i % N; total = barrier to barrier, median, max over ranks",
            "data": "the config-5 rows (above) cut into consecutive ledgers of log-uniform size in [1,000, "
                    "20,000] (tools/bench_legs.ledger_cuts)"}


def _pattern_bits(lo, hi):
    """Dry-run stand-in for a verifier: a fixed, irregular accept pattern of
    rows [lo, hi) (about 2 % rejects), identical whoever computes it."""
    i = np.arange(lo, hi, dtype=np.uint64)
    h = (i * np.uint64(0x9E3779B97F4A7C15)) >> np.uint64(57)
    return h >= np.uint64(3)


def _pack_words(bits):
    b = np.packbits(bits, bitorder="little")
    b = np.concatenate([b, np.zeros(-len(b) % 8, np.uint8)])
    return b.view("<i8")


def dry_digest_leg(ctx, n=10_000_000, fault=None):
    """CPU rehearsal of digest_leg's sharding, gather and digest check (no GPU,
    no verification): every rank packs the fixed pattern of its block shard,
    `fault` ("shift" / "dup" / "zero") corrupts rank 1's slice the way a wrong
    gather offset, a duplicated rank-0 slice or a skipped rank would, and rank
    0 compares the gathered digest with the pattern's over all n rows."""
    import torch
    world, rank = ctx["world"], ctx["rank"]
    lo, hi, b0, b1 = datasets.block_shard(n, rank, world)
    offs = np.array([datasets.block_shard(n, r, world)[0] // 64 for r in range(world)] + [(n + 63) // 64],
                    np.uint64)
    words = torch.from_numpy(_pack_words(_pattern_bits(lo, hi)).copy())
    if fault and rank == min(1, world - 1):
        if fault == "shift":
            words = torch.roll(words, 1)
        elif fault == "dup":
            words = torch.from_numpy(_pack_words(_pattern_bits(0, hi - lo)).copy())
        elif fault == "zero":
            words = torch.zeros_like(words)
    full = torch.zeros(int(offs[-1]), dtype=torch.int64) if rank == 0 else None
    dt = timed(ctx, lambda: ctx["gather"](words, offs, full), 3)
    out = {"rows": n, "n_ranks": world, "ms": dt * 1e3, "fault": fault,
           "unequal_shards": len(set(np.diff(offs.astype(np.int64)).tolist())) > 1}
    if rank == 0:
        want = hashlib.sha256(np.packbits(_pattern_bits(0, n), bitorder="little").tobytes()).hexdigest()
        out["digest_equal"] = bitmap_sha256(full, n) == want
    return out
