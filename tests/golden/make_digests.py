#!/usr/bin/env python3
"""Generates tests/golden/bitmap_digests.json: SHA-256 digests of the accept
bitmaps libsodium 1.0.18 gives the seeded datasets of BASELINE.json configs 2,
4, 3 and 5 (tests/datasets.py), with the digests of the inputs; and
tests/golden/block_digests.json: the same per 65,536-row block (inputs and
expected bitmap, first 16 bytes of SHA-256), which each rank of a sharded
bench run checks its own slice against.  Where a config's whole-input or
bitmap digest is already committed the regenerated one must equal it.

Run here (the build container: libsodium at /opt/conda/lib), never on the GPU
box.  Signing and verification both go through oracle/_ref/libsodium_ref.so
(crypto_sign_seed_keypair + crypto_sign_detached, and the reference's
verifySignature = crypto_sign_verify_detached && S < L).

    python tests/golden/make_digests.py [config2 config4 config3 config5 config5b config1]
"""
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from tests import datasets, oracle_bind  # noqa: E402


def _store_block(name, blocks):
    doc = {}
    if os.path.exists(datasets.BLOCK_DIGESTS):
        with open(datasets.BLOCK_DIGESTS) as f:
            doc = json.load(f)
    doc[name] = blocks
    with open(datasets.BLOCK_DIGESTS, "w") as f:
        json.dump(doc, f, indent=0, sort_keys=True)


def _check_same(out, name, got):
    old = out.get(name)
    if old:
        for k in ("inputs_sha256", "bitmap_sha256", "accepted", "rows"):
            if k in old and k in got:
                assert old[k] == got[k], (name, k, old[k], got[k])


def config5(lib, threads):
    """The ledger of datasets.ledger_plan: SHA512Half of every preimage
    (hashlib), libsodium signing by each row's signer, the invalid rows'
    bit flips, SHA512Half again where a preimage changed, libsodium's
    verifySignature."""
    import hashlib
    lp = datasets.ledger_plan()
    n, pre, offs, lens = lp["n"], lp["pre"], lp["offs"], lp["lens"]
    mv = memoryview(pre)

    def half(rows):
        return np.frombuffer(b"".join(hashlib.sha512(mv[int(offs[i]):int(offs[i] + lens[i])]).digest()[:32]
                                      for i in rows), np.uint8).reshape(-1, 32)
    msgs = half(range(n)).copy()
    pk, sig = oracle_bind.sodium_sign_batch(lib, np.ascontiguousarray(lp["signers"][lp["who"]]), msgs, threads)
    (pos, pbit), (srow, scol, sbit) = datasets.ledger_mutations(lp)
    pre[pos] ^= pbit
    sig[srow, scol] ^= sbit
    changed = np.unique(np.searchsorted(offs, pos, side="right") - 1)
    msgs[changed] = half(changed)
    bits = oracle_bind.sodium_verify_batch(lib, sig, msgs, pk, threads)
    bm = np.packbits(bits.astype(bool), bitorder="little")
    import hashlib as hl
    return {"rows": n, "accepted": int(bits.sum()), "bitmap_sha256": hl.sha256(bm.tobytes()).hexdigest(),
            "inputs_h16": datasets.ledger_input_digest(pre, lp["total"], lens, sig, pk),
            "preimage_bytes": lp["total"], "invalid_rows": int(lp["bad"].size),
            "invalid_by_kind": {k: int((lp["kind"] == i).sum()) for i, k in
                                enumerate(("preimage_bit", "R_bit", "S_bit"))},
            **{k: v for k, v in datasets.CONFIG5.items()},
            "construction": "datasets.ledger_plan: one ledger, signed over SHA512Half(preimage), invalid rows' "
                            "bits flipped after signing",
            "expected_from": f"libsodium {lib.ref_sodium_version().decode()} crypto_sign_verify_detached && S < L "
                             "over SHA512Half (hashlib) of each preimage"}


def config5b(lib, threads):
    """The serialized-blob ledger of datasets.blob_ledger_plan: signer keys and
    signatures from libsodium over hashlib's SHA512Half of each blob's signing
    preimage, the invalid rows made, then the reference's checkSign of every
    row -- parse, re-serialise (oracle/stl_oracle_tx.c, the STObject::set / add
    restatement), OpenSSL SHA-512, libsodium verify && S < L
    (ref_tx_blob_verify_batch) -- and each row's status under the device
    contract (include/stl.h STL_TX_*) from the same re-serialiser: DEFERRED
    unless the blob re-serialises to itself, MALFORMED when SigningPubKey is
    not 32 B or TxnSignature not 64 B."""
    import ctypes
    import hashlib
    zeros = lambda s: oracle_bind.sodium_sign_batch(lib, s, np.zeros((s.shape[0], 32), np.uint8), threads)[0]  # noqa: E731
    bp = datasets.blob_ledger_plan(zeros)
    n = bp["n"]
    msgs = datasets.blob_signing_hashes(bp)
    pk, sig = oracle_bind.sodium_sign_batch(lib, np.ascontiguousarray(bp["seeds"][bp["who"]]), msgs, threads)
    assert np.array_equal(pk, bp["pks"][bp["who"]])
    datasets.blob_ledger_finish(bp, sig)
    buf, offs, lens = bp["buf"], bp["offs"].astype(np.uint64), bp["lens"].astype(np.uint32)
    B = oracle_bind._buf
    bm = np.zeros((n + 7) // 8, np.uint8)
    ids = np.zeros((n, 32), np.uint8)
    lib.ref_tx_blob_verify_batch(B(buf), B(offs), B(lens), n, B(bm), B(ids), 0, threads)
    ref_bits = np.unpackbits(bm, bitorder="little")[:n].astype(bool)
    orc = oracle_bind.load_oracle()
    mv = memoryview(buf)
    status = np.zeros(n, np.uint8)
    cap = int(lens.max()) + 64
    sb, fb = ctypes.create_string_buffer(cap), ctypes.create_string_buffer(cap)
    info = oracle_bind.TxInfo()
    for i in range(n):
        b = mv[int(offs[i]):int(offs[i]) + int(lens[i])].tobytes()
        ok = orc.lib.oracle_tx_blob(b, len(b), sb, fb, cap, ctypes.byref(info)) == 0
        assert ok, ("reference cannot construct row", i)
        if fb.raw[:info.full_len] != b:
            status[i] = 1
        elif info.pk_len != 32 or info.sig_len != 64:
            status[i] = 2
    want_st = datasets.blob_expected_status(bp)
    assert np.array_equal(status, want_st), np.nonzero(status != want_st)[0][:10]
    kinds = {k: bp["bad"][bp["kind"] == i] for i, k in enumerate(datasets.BLOB_KINDS)}
    for k in ("payload_bit", "R_bit", "S_bit", "malformed_pk33"):
        assert not ref_bits[kinds[k]].any(), k
    assert ref_bits[kinds["deferred_order"]].all()
    assert ref_bits.sum() == n - bp["bad"].size + kinds["deferred_order"].size
    dev_bits = ref_bits & (status == 0)
    ids[status == 1] = 0  # the device writes no id for a deferred row
    sha = lambda a: hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()  # noqa: E731
    return {"rows": n, "accepted": int(dev_bits.sum()),
            "bitmap_sha256": sha(np.packbits(dev_bits, bitorder="little")),
            "ref_accepted": int(ref_bits.sum()), "ref_bitmap_sha256": sha(np.packbits(ref_bits, bitorder="little")),
            "status_sha256": sha(status), "status_counts": {str(k): int((status == k).sum()) for k in (0, 1, 2)},
            "ids_sha256": sha(ids), "inputs_h16": datasets.blob_ledger_inputs_h16(bp),
            "blob_bytes": bp["total"], "invalid_rows": int(bp["bad"].size),
            "invalid_by_kind": {k: int(v.size) for k, v in kinds.items()},
            **{k: v for k, v in datasets.CONFIG5B.items()},
            "construction": "datasets.blob_ledger_plan: one ledger of canonical serialized Payment blobs, signed "
                            "over SHA512Half('STX\\0' || blob minus TxnSignature), invalid rows made after "
                            "signing (datasets.BLOB_KINDS)",
            "expected_from": f"reference checkSign per row: oracle/stl_oracle_tx.c parse + re-serialise, OpenSSL "
                             f"SHA-512, libsodium {lib.ref_sodium_version().decode()} crypto_sign_verify_detached "
                             "&& S < L (ref_tx_blob_verify_batch); bitmap_sha256 = that && status OK (the device "
                             "contract: deferred and malformed rows carry accept bit 0); ids_sha256 = "
                             "SHA512Half('TXN\\0' || blob), zero for deferred rows"}


def config1(lib, threads):
    """configs[0]: the 100k Payment blobs of
    datasets.config1_plan -- bench.py's config-1 rows plus 2 % invalid rows
    (datasets.BLOB_KINDS) -- signed with libsodium over hashlib's SHA512Half of
    each signing preimage, then the reference's checkSign of every row: parse,
    re-serialise (oracle/stl_oracle_tx.c), OpenSSL SHA-512, libsodium verify &&
    S < L (ref_tx_blob_verify_batch), each row's status from the same
    re-serialiser, and the transaction ids."""
    import ctypes
    import hashlib
    zeros = lambda s: oracle_bind.sodium_sign_batch(lib, s, np.zeros((s.shape[0], 32), np.uint8), threads)[0]  # noqa: E731
    plan = datasets.config1_plan(zeros)
    n = plan["n"]
    msgs = datasets.config1_signing_hashes(plan)
    pk, sig = oracle_bind.sodium_sign_batch(lib, np.ascontiguousarray(plan["seeds"][plan["who"]]), msgs, threads)
    assert np.array_equal(pk, plan["pks"][plan["who"]])
    buf, offs, lens = datasets.config1_finish(plan, sig)
    offs, lens = offs.astype(np.uint64), lens.astype(np.uint32)
    B = oracle_bind._buf
    bm = np.zeros((n + 7) // 8, np.uint8)
    ids = np.zeros((n, 32), np.uint8)
    lib.ref_tx_blob_verify_batch(B(buf), B(offs), B(lens), n, B(bm), B(ids), 0, threads)
    ref_bits = np.unpackbits(bm, bitorder="little")[:n].astype(bool)
    orc = oracle_bind.load_oracle()
    mv = memoryview(buf)
    status = np.zeros(n, np.uint8)
    cap = int(lens.max()) + 64
    sb, fb = ctypes.create_string_buffer(cap), ctypes.create_string_buffer(cap)
    info = oracle_bind.TxInfo()
    for i in range(n):
        b = mv[int(offs[i]):int(offs[i]) + int(lens[i])].tobytes()
        ok = orc.lib.oracle_tx_blob(b, len(b), sb, fb, cap, ctypes.byref(info)) == 0
        assert ok, ("reference cannot construct row", i)
        if fb.raw[:info.full_len] != b:
            status[i] = 1
        elif info.pk_len != 32 or info.sig_len != 64:
            status[i] = 2
    want_st = datasets.config1_expected_status(plan)
    assert np.array_equal(status, want_st), np.nonzero(status != want_st)[0][:10]
    kinds = {k: plan["bad"][plan["kind"] == i] for i, k in enumerate(datasets.BLOB_KINDS)}
    for k in ("payload_bit", "R_bit", "S_bit", "malformed_pk33"):
        assert not ref_bits[kinds[k]].any(), k
    assert ref_bits[kinds["deferred_order"]].all()
    assert ref_bits.sum() == n - plan["bad"].size + kinds["deferred_order"].size
    dev_bits = ref_bits & (status == 0)
    ids[status == 1] = 0  # the device writes no id for a deferred row
    sha = lambda a: hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()  # noqa: E731
    return {"rows": n, "accepted": int(dev_bits.sum()),
            "bitmap_sha256": sha(np.packbits(dev_bits, bitorder="little")),
            "ref_accepted": int(ref_bits.sum()), "ref_bitmap_sha256": sha(np.packbits(ref_bits, bitorder="little")),
            "status_sha256": sha(status), "status_counts": {str(k): int((status == k).sum()) for k in (0, 1, 2)},
            "ids_sha256": sha(ids), "inputs_h16": datasets.config1_inputs_h16(buf, lens),
            "blob_bytes": int(lens.astype(np.int64).sum()),
            "blob_len": {"min": int(lens.min()), "median": int(np.median(lens)), "max": int(lens.max())},
            "invalid_rows": int(plan["bad"].size),
            "invalid_by_kind": {k: int(v.size) for k, v in kinds.items()},
            **{k: v for k, v in datasets.CONFIG1.items()},
            "construction": "datasets.config1_plan: bench.py's config-1 Payment transactions (tools/payments.py, "
                            "1,000 accounts signing in turn) as serialized blobs, signed over SHA512Half('STX\\0' "
                            "|| preimage fields), 2 % invalid rows made after signing (datasets.BLOB_KINDS; the "
                            "33-byte keys before it)",
            "expected_from": f"reference checkSign per row: oracle/stl_oracle_tx.c parse + re-serialise, OpenSSL "
                             f"SHA-512, libsodium {lib.ref_sodium_version().decode()} crypto_sign_verify_detached "
                             "&& S < L (ref_tx_blob_verify_batch); bitmap_sha256 = that && status OK; ids_sha256 = "
                             "SHA512Half('TXN\\0' || blob), zero for deferred rows"}


def main(names):
    lib = oracle_bind.load_sodium_ref()
    assert lib is not None, "needs libsodium"
    threads = os.cpu_count() or 8
    out = {}
    if os.path.exists(datasets.DIGESTS):
        with open(datasets.DIGESTS) as f:
            out = json.load(f)
    group = datasets.sodium_group(lib)
    for name in names:
        t0 = time.time()
        if name in ("config5", "config5b", "config1"):
            got = {"config5": config5, "config5b": config5b, "config1": config1}[name](lib, threads)
            _check_same(out, name, got)
            out[name] = got
            with open(datasets.DIGESTS, "w") as f:
                json.dump(out, f, indent=1, sort_keys=True)
            print(f"{name}: {got['accepted']} accepted ({time.time() - t0:.0f} s)", flush=True)
            continue
        dg = datasets.Digest()
        blk = datasets.BlockDigest()
        classes, keys = {}, []

        def make(seeds, msgs, cls, param):
            pk, sig = oracle_bind.sodium_sign_batch(lib, seeds, msgs, threads)
            msgs = msgs.copy()
            datasets.mutate(seeds, msgs, pk, sig, cls, param, group)
            return pk, sig, msgs

        for c0, seed, n, frac in datasets.chunks(name):
            sig, msg, pk, cls = datasets.chunk(seed, n, frac, make)
            bits = oracle_bind.sodium_verify_batch(lib, sig, msg, pk, threads)
            dg.add(sig, msg, pk, bits)
            blk.add(sig, msg, pk, bits)
            for k, v in datasets.class_counts(cls).items():
                classes[k] = classes.get(k, 0) + v
            adv = np.nonzero(cls)[0]
            keys.append(datasets.row_keys(sig[adv], msg[adv], pk[adv]))
            print(f"{name}: rows {c0 + n} accepted {dg.accepted} ({time.time() - t0:.0f} s)", flush=True)
        keys = np.concatenate(keys) if keys else np.zeros(0, "S16")
        got = dict(dg.result(), **datasets.CONFIGS[name], adversarial_rows_by_class=classes,
                   adversarial_rows_distinct=int(np.unique(keys).size),
                   construction="each adversarial row mutated from its own honest row, classes B1-B11 "
                                "evenly (tests/datasets.py)",
                   expected_from=f"libsodium {lib.ref_sodium_version().decode()} "
                                 "crypto_sign_verify_detached && S < L")
        _check_same(out, name, got)
        out[name] = got
        with open(datasets.DIGESTS, "w") as f:
            json.dump(out, f, indent=1, sort_keys=True)
        _store_block(name, blk.result())
    print(json.dumps({k: {kk: vv for kk, vv in v.items() if kk != "adversarial_rows_by_class"}
                      for k, v in out.items()}, indent=1))


if __name__ == "__main__":
    main(sys.argv[1:] or ["config2", "config4", "config3", "config5", "config5b", "config1"])
