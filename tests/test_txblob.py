"""Serialized-transaction path (stellard_amd/csrc/stl_txblob.h)
on the CPU: the C re-serialiser (oracle/stl_oracle_tx.c, the reference's
parse + STObject::add) against an independent Python serializer, and the
device pass compiled for the host (tests/native/hostemu.cpp) against the
oracle -- status, signing hash, transaction ID -- on the named special cases
and on randomly mutated blobs.

Parity anchor: the reference holds no serialized-transaction fixtures (its
SerializedTransaction_test builds a transaction, signs it and round-trips it:
SerializedTransaction.cpp:374-400); the two restatements here, plus
signatures made over the Python preimages and accepted by libsodium, are what
pin it."""
import hashlib

import numpy as np
import pytest

from tests import txblob as T
from tests.oracle_bind import (hostemu_tx_blob, load_hostemu, load_oracle, load_sodium_ref,
                               sodium_tx_blob_verify_batch)

OK, DEFERRED, MALFORMED = 0, 1, 2
MAX_DEPTH = 8


@pytest.fixture(scope="module")
def oracle():
    return load_oracle()


@pytest.fixture(scope="module")
def emu():
    return load_hostemu()


@pytest.fixture(scope="module")
def corpus(oracle):
    return T.valid_corpus(oracle, 240, seed=11, with_preimages=True)


def h512half(b):
    return hashlib.sha512(b).digest()[:32]


def test_oracle_reserialises_python_blobs(oracle, corpus):
    blobs, pres = corpus
    for b, p in zip(blobs, pres):
        ok, info, signing, full = oracle.tx_blob(b)
        assert ok
        assert full == b
        assert signing == p
        assert info.pk_len == 32 and info.sig_len == 64


def test_corpus_signatures_accepted(oracle, corpus):
    blobs, _ = corpus
    bits, ids = oracle.tx_blob_verify_batch(blobs, tx_ids=True)
    assert bits.all()
    for b, i in zip(blobs, ids):
        assert bytes(i) == T.tx_id(b)
    ref = load_sodium_ref()
    if ref is not None:
        rbits, rids = sodium_tx_blob_verify_batch(ref, blobs, tx_ids=True)
        assert rbits.all()
        assert (rids == ids).all()


def _check_device_vs_oracle(oracle, emu, blob):
    """Invariants between the device pass and the reference re-serialisation.
    Returns (device status, oracle-constructible)."""
    st, msg, tid, lay = hostemu_tx_blob(emu, blob)
    ok, info, signing, full = oracle.tx_blob(blob)
    if not ok:
        return st, False  # the reference never builds this transaction: no claim
    canonical = full == blob and not info.stopped_early
    if st != DEFERRED:
        # the device only decides blobs the reference re-serialises unchanged
        assert canonical, blob.hex()
        assert tid == h512half(b"TXN\x00" + full)
        shaped = info.pk_len == 32 and info.sig_len == 64
        assert st == (OK if shaped else MALFORMED)
        if st == OK:
            assert msg == h512half(signing)
    elif canonical and info.all_declared and info.max_depth <= MAX_DEPTH:
        pytest.fail("deferred a canonical blob: " + blob.hex())
    return st, True


def test_device_pass_on_corpus(oracle, emu, corpus):
    blobs, pres = corpus
    for b, p in zip(blobs, pres):
        st, msg, tid, lay = hostemu_tx_blob(emu, b)
        assert st == OK
        assert msg == h512half(p)
        assert tid == T.tx_id(b)
        pk_off, pk_len, sig_off, sig_len = lay[:4]
        assert pk_len == 32 and sig_len == 64
        assert b[pk_off - 2:pk_off] == b"\x73\x20" and b[sig_off - 2:sig_off] == b"\x74\x40"


@pytest.mark.parametrize("case", range(len(T.special_cases(load_oracle()))))
def test_special_cases(oracle, emu, case):
    name, blob, expect = T.special_cases(oracle)[case]
    st, constructible = _check_device_vs_oracle(oracle, emu, blob)
    if expect == "unconstructible":
        assert not constructible, name
        return
    assert constructible, name
    want = {"ok": OK, "reject": OK, "malformed": MALFORMED, "defer": DEFERRED}[expect]
    assert st == want, name
    bit = oracle.tx_blob_verify_batch([blob])[0]
    if expect != "defer":  # a deferred blob gets the caller's own checkSign, whatever it says
        assert bit == (expect == "ok"), name
    if expect == "defer" and name not in ("depth_too_deep", "dynamic_field"):
        ok, info, signing, full = oracle.tx_blob(blob)
        assert full != blob or info.stopped_early, name  # deferral was necessary


def test_fuzz_invariants(oracle, emu, corpus):
    blobs, _ = corpus
    rng = np.random.default_rng(2024)
    counts = {OK: 0, DEFERRED: 0, MALFORMED: 0}
    built = 0
    for _ in range(4000):
        b = blobs[int(rng.integers(len(blobs)))]
        if int(rng.integers(0, 10)) == 0:  # TxnSignature (optional) cut out: B12, checkSign false
            i = b.index(b"\x74\x40")
            m = b[:i] + b[i + 66:]
            if int(rng.integers(0, 2)):
                m = T.mutate(rng, m)
        else:
            m = T.mutate(rng, b)
        if int(rng.integers(0, 4)) == 0:
            m = T.mutate(rng, m)
        st, constructible = _check_device_vs_oracle(oracle, emu, m)
        counts[st] += 1
        built += constructible
    # the mutations reach every outcome
    assert counts[OK] > 100 and counts[DEFERRED] > 100 and counts[MALFORMED] > 5, counts
    assert built > 500


@pytest.mark.parametrize("off", range(0, 9))
def test_blob_words_unaligned(emu, off):
    import ctypes
    rng = np.random.default_rng(off)
    buf = np.frombuffer(rng.bytes(128), np.uint8).copy()
    for n, ln in ((16, 128), (8, off + 32), (8, 128)):
        if off + 4 * n > ln:
            continue
        out = (ctypes.c_uint32 * n)()
        emu.hostemu_blob_words(buf.ctypes.data_as(ctypes.c_void_p), off, n, ln, out)
        assert bytes(np.array(out, np.uint32).tobytes()) == buf[off:off + 4 * n].tobytes()


# ---- serialized validations -------------------------------
VALIDATION = 1


@pytest.fixture(scope="module")
def val_corpus(oracle):
    rng = np.random.default_rng(77)
    keys = [oracle.keypair(rng.bytes(32)) for _ in range(4)]
    out = []
    for i in range(160):
        pk, sk = keys[i % 4]
        fs = T.validation_fields(rng, pk, full=bool(i % 3))
        blob, h, _ = T.signed_validation(fs, sk, oracle.sign)
        out.append((blob, T.validation_preimage(fs), h))
    return out


def test_oracle_reserialises_validations(oracle, val_corpus):
    """SerializedValidation(sit) + getSigningHash (SerializedValidation.cpp:22-34,
    70-73): the C re-serialiser gives back the Python blob and "VAL\\0" ||
    fields without Signature; libsodium accepts the signatures over it."""
    from tests.oracle_bind import sodium_signed_blob_verify_batch
    for blob, pre, h in val_corpus:
        ok, info, signing, full = oracle.signed_blob(VALIDATION, blob)
        assert ok and full == blob and signing == pre
        assert h512half(signing) == h
        assert info.pk_len == 32 and info.sig_len == 64
    blobs = [b for b, _, _ in val_corpus]
    bits, ids = oracle.signed_blob_verify_batch(VALIDATION, blobs, ids=True)
    assert bits.all()
    assert all(bytes(i) == h512half(b) for i, b in zip(ids, blobs))  # PeerImp.cpp:1155 suppression key
    ref = load_sodium_ref()
    if ref is not None:
        assert sodium_signed_blob_verify_batch(ref, VALIDATION, blobs).all()
    # as transactions they do not verify (no TransactionType, no TxnSignature)
    assert not oracle.tx_blob_verify_batch(blobs).any()


def test_device_pass_on_validations_and_fuzz(oracle, emu, val_corpus):
    """The device pass for validations (BlobKind: "VAL\\0", sfSignature, id =
    SHA512Half(raw), 50-byte floor) against the oracle on the corpus and on
    3,000 mutated blobs: wherever the device decides, the reference
    re-serialises unchanged and the signing hash / id / status agree."""
    from tests.oracle_bind import hostemu_signed_blob
    blobs = [b for b, _, _ in val_corpus]
    for blob, pre, h in val_corpus:
        st, msg, idb = hostemu_signed_blob(emu, VALIDATION, blob)
        assert st == OK and msg == h and idb == h512half(blob)
    rng = np.random.default_rng(78)
    counts = {OK: 0, DEFERRED: 0, MALFORMED: 0}
    for _ in range(3000):
        m = T.mutate(rng, blobs[int(rng.integers(len(blobs)))])
        st, msg, idb = hostemu_signed_blob(emu, VALIDATION, m)
        counts[st] += 1
        ok, info, signing, full = oracle.signed_blob(VALIDATION, m)
        if st == DEFERRED or not ok:
            continue
        assert full == m and not info.stopped_early, m.hex()
        assert idb == h512half(m)
        assert st == (OK if (info.pk_len == 32 and info.sig_len == 64) else MALFORMED)
        if st == OK:
            assert msg == h512half(signing)
    assert counts[OK] > 100 and counts[DEFERRED] > 100, counts
    # below PeerImp::recvValidation's 50-byte floor: deferred
    short = blobs[0][:49]
    assert hostemu_signed_blob(emu, VALIDATION, short)[0] == DEFERRED


def test_validation_template_drops_foreign_fields(oracle, emu):
    """SerializedValidation(sit) is STObject(getFormat(), sit, sfValidation):
    set() then setType() with its result ignored (SerializedObject.h:54-58), so
    a top-level field outside the validation template (SerializedValidation.cpp:
    134-159) is dropped from the object and from the signing hash.  The oracle
    restates that (a signature over the template fields alone verifies); the
    device cannot splice such a blob and defers it; a duplicate template field
    is dropped too (setType moves the first)."""
    from tests.oracle_bind import hostemu_signed_blob
    rng = np.random.default_rng(79)
    pk, sk = oracle.keypair(rng.bytes(32))
    for extra in ([T.Field(T.TransactionType, T.u16(0))], [T.Field(T.Memos, T.array_value(
            [(T.Memo, [T.Field(T.MemoData, T.vl(b"hi"))])]))], [T.Field(T.TxnSignature, T.vl(bytes(64)))]):
        fs = T.validation_fields(rng, pk)
        h = h512half(T.validation_preimage(fs))
        blob = T.serialize(fs + extra + [T.Field(T.Signature, T.vl(oracle.sign(h, sk)))])
        ok, info, signing, full = oracle.signed_blob(VALIDATION, blob)
        assert ok and signing == T.validation_preimage(fs) and full != blob
        assert oracle.signed_blob_verify_batch(VALIDATION, [blob])[0].all()
        assert hostemu_signed_blob(emu, VALIDATION, blob)[0] == DEFERRED
        ref = load_sodium_ref()
        if ref is not None:
            from tests.oracle_bind import sodium_signed_blob_verify_batch
            assert sodium_signed_blob_verify_batch(ref, VALIDATION, [blob]).all()
    # the same validation without the extra field is decided on the device
    fs = T.validation_fields(rng, pk)
    blob, h, _ = T.signed_validation(fs, sk, oracle.sign)
    assert hostemu_signed_blob(emu, VALIDATION, blob)[0] == OK


def test_transaction_templates(oracle, emu):
    """TxFormats (TxFormats.cpp:22-130) + SerializedTransaction's constructor
    (SerializedTransaction.cpp:79-91): the device decides exactly the
    constructible, canonical blobs of every transaction type; template
    violations (missing required, foreign or duplicate fields, types without a
    format) are unconstructible and deferred.  Covered case by case in
    test_special_cases; here a sweep over every TransactionType value and
    every template field added to a Payment."""
    rng = np.random.default_rng(80)
    pk, sk = oracle.keypair(rng.bytes(32))
    base = T.payment_fields(rng, pk, 3)
    rest = [x for x in base if x.fid != T.TransactionType]
    decided = 0
    for tt in list(range(0, 24)) + [99, 100, 101, 102, 255, 256, 0x7FFF, 0xFFFF]:
        blob = T.signed_blob(rest + [T.Field(T.TransactionType, T.u16(tt))], sk, oracle.sign)[0]
        st, constructible = _check_device_vs_oracle(oracle, emu, blob)
        assert constructible == (tt == 0), tt  # Payment's fields fit no other template
        decided += st != DEFERRED
    assert decided == 1


def test_txnsignatures_always_deferred(oracle, emu):
    """TxnSignatures (ARRAY 3, FieldNames.cpp:49-51) lies outside
    every TxFormats template and SerializedValidation's template, so a blob
    that carries it is always DEFERRED under the product's template checks
    (the TxnSignatures cut of the bare pass only runs in host tests without a
    template); the reference does not construct such a transaction either."""
    from tests.oracle_bind import hostemu_signed_blob
    blob = dict((n, b) for n, b, _ in T.special_cases(oracle))["with_TxnSignatures"]
    assert not oracle.tx_blob(blob)[0]  # unconstructible in the reference
    assert hostemu_tx_blob(emu, blob)[0] == DEFERRED
    assert hostemu_signed_blob(emu, 0, blob)[0] == DEFERRED
    assert hostemu_signed_blob(emu, 1, blob)[0] == DEFERRED


def test_blob_ledger_construction(oracle, emu):
    """The config-5 blob ledger's construction (tests/datasets.py
    blob_ledger_plan, here 3,000 rows with 5 % invalid): every row is built
    by the reference re-serialiser; canonical rows re-serialise to themselves
    and their signing preimage hashes to the construction's signing hash;
    the statuses by the reference's rules equal the construction's
    (deferred = Flags / Sequence swapped, malformed = 33-byte key) and the
    device pass's on the host; the reference accepts exactly the honest and
    the deferred rows."""
    from tests import datasets as D
    bp, blobs = D.blob_ledger_cpu(oracle, 3000)
    want = D.blob_expected_status(bp)
    msgs = D.blob_signing_hashes(bp)
    kinds = {k: set(bp["bad"][bp["kind"] == i].tolist()) for i, k in enumerate(D.BLOB_KINDS)}
    assert all(len(v) >= 25 for v in kinds.values())
    ref_st = np.zeros(len(blobs), np.uint8)
    for i, b in enumerate(blobs):
        ok, info, signing, full = oracle.tx_blob(b)
        assert ok, i
        if full != b:
            ref_st[i] = DEFERRED
        elif info.pk_len != 32 or info.sig_len != 64:
            ref_st[i] = MALFORMED
        else:
            assert h512half(signing) == bytes(msgs[i]) or i in kinds["payload_bit"], i
        st, msg, tid, _ = hostemu_tx_blob(emu, b)
        assert st == want[i], (i, st, want[i])
        if st == OK:
            assert msg == h512half(signing) and tid == T.tx_id(b)
    assert np.array_equal(ref_st, want)
    bits = oracle.tx_blob_verify_batch(blobs)
    expect = np.ones(len(blobs), bool)
    for k in ("payload_bit", "R_bit", "S_bit", "malformed_pk33"):
        expect[list(kinds[k])] = False
    assert np.array_equal(bits, expect)
    assert 100 <= min(bp["lens"]) and max(bp["lens"]) <= 4100


def test_splice_word_assembly_equals_stream(emu):
    """The word-wise one-cut splice (stl_txblob.h splice1_block) and
    tx_blob_kernel's block schedule (the parse kernel's spliced block between
    plain windows, hostemu_splice_kernel) against SpliceStream and hashlib: SHA512Half(prefix || blob[0, xs) ||
    blob[xe, len)) over random lengths, cut positions and buffer alignments,
    including cuts at the blob's edges and preimages ending in every byte of a
    block."""
    import ctypes
    from tests.oracle_bind import _buf
    emu.hostemu_splice_pair.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                        ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p]
    rng = np.random.default_rng(0x5911CE)
    cases = [(L, xs, xe) for L in (32, 66, 67, 100, 127, 128, 129, 200) for xs in (0, 1, 3, 5) for xe in (xs, xs + 66)
             if xe <= L]
    for _ in range(3000):
        L = int(rng.integers(32, 5000))
        xs = int(rng.integers(0, L))
        xe = int(rng.integers(xs, min(L, xs + 300) + 1))
        cases.append((L, xs, xe))
    for L in range(160, 420):  # every preimage length across two block edges
        cases.append((L, 80, 146))
    emu.hostemu_splice_kernel.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                          ctypes.c_uint32, ctypes.c_void_p]
    a, w, k = ctypes.create_string_buffer(32), ctypes.create_string_buffer(32), ctypes.create_string_buffer(32)
    for i, (L, xs, xe) in enumerate(cases):
        sh = i % 16
        arr = np.zeros(L + 64, np.uint8)
        arr[sh:sh + L] = rng.integers(0, 256, L, dtype=np.uint8)
        blob = arr[sh:sh + L].tobytes()
        ptr = ctypes.c_void_p(arr.ctypes.data + sh)
        emu.hostemu_splice_pair(ptr, L, 0x53545800, xs, xe, a, w)
        emu.hostemu_splice_kernel(ptr, L, 0x53545800, xs, xe, k)
        want = hashlib.sha512(b"STX\x00" + blob[:xs] + blob[xe:]).digest()[:32]
        assert a.raw == want and w.raw == want and k.raw == want, (L, xs, xe, sh)
