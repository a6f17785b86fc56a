"""GPU parity tests: the gfx950 kernels, called through the C ABI (libstl.so),
against the golden vectors (expected bits from libsodium 1.0.18) and the CPU
oracle (oracle/stl_oracle.c) on the same seeded inputs.  Bit-exact: any
differing accept bit fails.

Run on an MI355X:  python -u -m pytest tests -m gpu -x -v --timeout 120
"""
import hashlib

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

L = 2**252 + 27742317777372353535851937790883648493


@pytest.fixture(scope="module")
def torch_cuda():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch


@pytest.fixture(scope="module")
def stl(torch_cuda):
    from stellard_amd import verify
    verify.init()
    return verify


def _golden_arrays(golden):
    return golden["sig"], golden["msg"], golden["pk"]


@pytest.mark.parametrize("policy,key", [(0, "expected_sodium_1_0_18"), (1, "expected_stellard_1_0_0_unpinned")])
def test_golden_host_batch(stl, golden, policy, key):
    sig, msg, pk = _golden_arrays(golden)
    got = stl.verify_batch(sig, msg, pk, policy=policy)
    exp = golden[key].astype(bool)
    bad = np.nonzero(got != exp)[0]
    names = golden["class_names"]
    assert bad.size == 0, [(int(i), str(names[golden["cls"][i]]), bool(got[i])) for i in bad[:20]]


def test_golden_device_batch(stl, golden, torch_cuda):
    torch = torch_cuda
    sig, msg, pk = _golden_arrays(golden)
    n = sig.shape[0]
    d = [torch.from_numpy(np.ascontiguousarray(a)).cuda() for a in (sig, msg, pk)]
    words = stl.verify_batch_device(*d)
    torch.cuda.synchronize()
    got = stl.words_to_bool(words, n)
    assert np.array_equal(got, golden["expected_sodium_1_0_18"].astype(bool))


def test_golden_per_class_counts(stl, golden):
    """Adversarial classes reject exactly as libsodium does."""
    sig, msg, pk = _golden_arrays(golden)
    got = stl.verify_batch(sig, msg, pk)
    exp = golden["expected_sodium_1_0_18"].astype(bool)
    for c, name in enumerate(golden["class_names"]):
        m = golden["cls"] == c
        assert int(got[m].sum()) == int(exp[m].sum()), str(name)


def test_single_verify_detached(stl, golden, oracle):
    sig, msg, pk = _golden_arrays(golden)
    exp = golden["expected_sodium_1_0_18"].astype(bool)
    for i in list(range(0, sig.shape[0], 97)) + [sig.shape[0] - 1]:
        assert stl.verify_signature(msg[i].tobytes(), sig[i].tobytes(), pk[i].tobytes()) == bool(exp[i])
    with pytest.raises(stl.BadInputs):
        stl.verify_signature(bytes(32), bytes(63), bytes(32))
    with pytest.raises(stl.BadInputs):
        stl.verify_signature(bytes(32), bytes(64), bytes(33))


def test_verify_detached_variable_length(stl, oracle):
    rng = np.random.default_rng(7)
    for mlen in (0, 1, 31, 33, 64, 111, 112, 128, 239, 1000):
        seed = rng.bytes(32)
        pkb, sk = oracle.keypair(seed)
        m = rng.bytes(mlen)
        s = oracle.sign(m, sk)
        assert stl.crypto_sign_verify_detached(s, m, pkb) == 0, mlen
        bad = bytearray(s)
        bad[5] ^= 4
        assert stl.crypto_sign_verify_detached(bytes(bad), m, pkb) == -1, mlen


def test_sign_kernel_matches_oracle(stl, oracle, torch_cuda):
    """GPU RFC 8032 signer (synthetic-data generator) is byte-identical to the
    oracle signer (deterministic signatures)."""
    torch = torch_cuda
    rng = np.random.default_rng(11)
    n = 300
    seeds = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    msgs = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    pk, sig = stl.sign_batch_device(torch.from_numpy(seeds).cuda(), torch.from_numpy(msgs).cuda())
    pk, sig = pk.cpu().numpy(), sig.cpu().numpy()
    for i in range(0, n, 7):
        opk, osk = oracle.keypair(seeds[i].tobytes())
        assert pk[i].tobytes() == opk
        assert sig[i].tobytes() == oracle.sign(msgs[i].tobytes(), osk)


def _gpu_signed(stl, torch, n, seed):
    rng = np.random.default_rng(seed)
    seeds = torch.from_numpy(rng.integers(0, 256, (n, 32), dtype=np.uint8)).cuda()
    msgs = torch.from_numpy(rng.integers(0, 256, (n, 32), dtype=np.uint8)).cuda()
    pk, sig = stl.sign_batch_device(seeds, msgs)
    return sig, msgs, pk


def _mutate(sig, msg, pk, rng):
    """Mix of SURVEY App. B mutations on ~30% of the rows (host numpy arrays)."""
    n = sig.shape[0]
    sig, msg, pk = sig.copy(), msg.copy(), pk.copy()
    kinds = rng.integers(0, 10, n)
    for i in np.nonzero(rng.random(n) < 0.3)[0]:
        k = kinds[i]
        if k == 0:
            msg[i, rng.integers(32)] ^= 1 << rng.integers(8)
        elif k == 1:
            sig[i, rng.integers(32)] ^= 1 << rng.integers(8)
        elif k == 2:
            sig[i, 32 + rng.integers(31)] ^= 1 << rng.integers(8)
        elif k == 3:  # S + L
            S = int.from_bytes(sig[i, 32:].tobytes(), "little") + L
            sig[i, 32:] = np.frombuffer(S.to_bytes(32, "little"), np.uint8)
        elif k == 4:
            sig[i, 63] |= 0xE0
        elif k == 5:
            pk[i, 31] ^= 0x80
        elif k == 6:
            pk[i] = np.frombuffer(bytes([1]) + bytes(31), np.uint8)
        elif k == 7:
            sig[i, :32] = np.frombuffer(bytes([1]) + bytes(31), np.uint8)
        elif k == 8:
            pk[i, rng.integers(32)] ^= 1 << rng.integers(8)
        else:
            pk[i] = rng.integers(0, 256, 32, dtype=np.uint8)
    return sig, msg, pk


@pytest.mark.parametrize("policy", [0, 1])
def test_random_mutations_vs_oracle(stl, oracle, torch_cuda, policy):
    torch = torch_cuda
    n = 12288
    sig, msg, pk = _gpu_signed(stl, torch, n, 1234)
    rng = np.random.default_rng(99)
    sig, msg, pk = _mutate(sig.cpu().numpy(), msg.cpu().numpy(), pk.cpu().numpy(), rng)
    exp = oracle.verify_batch(sig, msg, pk, policy=policy, threads=16)
    got = stl.verify_batch(sig, msg, pk, policy=policy)
    bad = np.nonzero(got != exp)[0]
    assert bad.size == 0, bad[:20]
    assert 0.5 < exp.mean() < 0.95


@pytest.mark.parametrize("n", [1, 2, 63, 64, 65, 255, 256, 257, 1023, 4097])
def test_ragged_sizes(stl, golden, n):
    sig, msg, pk = _golden_arrays(golden)
    idx = np.arange(n) % sig.shape[0]
    got = stl.verify_batch(sig[idx], msg[idx], pk[idx])
    assert np.array_equal(got, golden["expected_sodium_1_0_18"][idx].astype(bool))


@pytest.mark.parametrize("quad", [3, 1, 0])
def test_pair_lanes_same_bits(stl, oracle, torch_cuda, quad):
    """Batches up to a quarter of the resident lanes run each signature on two lanes
    (verify_main_pair_kernel), the smallest (one wave per SIMD at eight lanes
    per signature, STL_TUNE_QUAD 1) on lane quads (verify_main_quad_kernel);
    STL_ONE_LANE forces one lane.  All give the oracle's bits on mutated rows
    at ragged sizes either side of the switches (the point kernel pairs up to
    twice the main kernel's limit), on the host and device APIs; the accept
    counter counts the bits once.  Pre-filled output words show that every
    word of the batch is written (bits past n included)."""
    torch = torch_cuda
    n = 70000
    sig, msg, pk = _gpu_signed(stl, torch, n, 4711)
    rng = np.random.default_rng(17)
    s, m, p = _mutate(sig.cpu().numpy(), msg.cpu().numpy(), pk.cpu().numpy(), rng)
    exp = oracle.verify_batch(s, m, p, threads=16)
    ds, dm, dp = (torch.from_numpy(a).cuda() for a in (s, m, p))
    old = stl.debug_tuning(stl.TUNE_QUAD, quad)
    try:
        _pair_sizes(stl, torch, s, m, p, ds, dm, dp, exp)
    finally:
        stl.debug_tuning(stl.TUNE_QUAD, old)


def _pair_sizes(stl, torch, s, m, p, ds, dm, dp, exp):
    for k in (1, 31, 33, 95, 4097, 8191, 8192, 8193, 12000, 16384, 16385, 32767, 32768, 32769, 49153, 65536, 65537,
              70000):
        two = stl.verify_batch(s[:k], m[:k], p[:k])
        one = stl.verify_batch(s[:k], m[:k], p[:k], policy=stl.ONE_LANE)
        assert np.array_equal(two, exp[:k]), (k, np.nonzero(two != exp[:k])[0][:10])
        assert np.array_equal(one, exp[:k]), k
        w = torch.full(((k + 63) // 64,), -1, dtype=torch.int64, device="cuda")
        stl.reset_stats()
        stl.verify_batch_device(ds[:k], dm[:k], dp[:k], out_words=w)
        torch.cuda.synchronize()
        assert stl.get_stats()["accepted"] == int(exp[:k].sum()), k
        bits = np.unpackbits(w.cpu().numpy().astype("<i8").view(np.uint8), bitorder="little")
        assert np.array_equal(bits[:k].astype(bool), exp[:k]), k
        assert not bits[k:].any(), k


def test_empty_batch(stl):
    z = np.zeros((0, 64), np.uint8)
    assert stl.verify_batch(z, np.zeros((0, 32), np.uint8), np.zeros((0, 32), np.uint8)).size == 0


def test_full_size_valid_batch(stl, oracle, torch_cuda):
    """configs[1]: 1,048,576 signatures, all valid -> every bit set; a seeded
    sample of 8192 rows re-checked by the oracle; the bitmap is independent of
    how the batch is split (device API, one call vs. 4 calls)."""
    torch = torch_cuda
    n = 1 << 20
    sig, msg, pk = _gpu_signed(stl, torch, n, 0x5EED0002)
    words = stl.verify_batch_device(sig, msg, pk)
    torch.cuda.synchronize()
    got = stl.words_to_bool(words, n)
    assert got.all(), int((~got).sum())
    # a mutated copy: flip one S bit in every 97th row
    sig2 = sig.clone()
    sig2[::97, 40] ^= 1
    w2 = stl.verify_batch_device(sig2, msg, pk)
    q = n // 4
    parts = [stl.verify_batch_device(sig2[i * q:(i + 1) * q].contiguous(), msg[i * q:(i + 1) * q].contiguous(),
                                     pk[i * q:(i + 1) * q].contiguous()) for i in range(4)]
    torch.cuda.synchronize()
    b2 = stl.words_to_bool(w2, n)
    assert np.array_equal(b2, np.concatenate([stl.words_to_bool(p, q) for p in parts]))
    expect = np.ones(n, bool)
    expect[::97] = False
    assert np.array_equal(b2, expect)
    rng = np.random.default_rng(5)
    sample = rng.choice(n, 8192, replace=False)
    s_np, m_np, p_np = sig2.cpu().numpy()[sample], msg.cpu().numpy()[sample], pk.cpu().numpy()[sample]
    assert np.array_equal(b2[sample], oracle.verify_batch(s_np, m_np, p_np, threads=16))


def test_tx_verify_batch_vs_oracle(stl, oracle):
    """checkSign path: SHA512Half(preimage) on the GPU, then verify."""
    rng = np.random.default_rng(21)
    n = 600
    pre, sigs, pks = [], [], []
    seed_keys = [oracle.keypair(rng.bytes(32)) for _ in range(16)]
    for i in range(n):
        ln = int(np.exp(rng.uniform(np.log(100), np.log(4096))))
        p = b"STX\x00" + rng.bytes(ln - 4)
        pkb, sk = seed_keys[i % 16]
        h = hashlib.sha512(p).digest()[:32]
        s = bytearray(oracle.sign(h, sk))
        if i % 5 == 0:
            s[rng.integers(64)] ^= 1 << int(rng.integers(8))
        if i % 7 == 0:
            p = p[:-1] + bytes([p[-1] ^ 1])
        pre.append(p)
        sigs.append(bytes(s))
        pks.append(pkb)
    sig = np.frombuffer(b"".join(sigs), np.uint8).reshape(n, 64)
    pk = np.frombuffer(b"".join(pks), np.uint8).reshape(n, 32)
    exp = oracle.tx_verify_batch(pre, sig, pk, threads=16)
    got = stl.tx_verify_batch(pre, sig, pk)
    assert np.array_equal(got, exp)
    assert 0.5 < exp.mean() < 0.9


@pytest.mark.parametrize("policy", [0, 1])
def test_full_length_flag_same_bits(stl, golden, oracle, torch_cuda, policy):
    """STL_FULL_LENGTH routes every lane through the full-length fallback
    kernel ([S]B - [k]A, 253-bit chain); the default half-size-scalar path
    must give the same bits, and both the golden / oracle bits."""
    torch = torch_cuda
    sig, msg, pk = _golden_arrays(golden)
    key = "expected_sodium_1_0_18" if policy == 0 else "expected_stellard_1_0_0_unpinned"
    full = stl.verify_batch(sig, msg, pk, policy=policy | stl.FULL_LENGTH)
    assert np.array_equal(full, golden[key].astype(bool))
    n = 4096
    s2, m2, p2 = _gpu_signed(stl, torch, n, 77 + policy)
    rng = np.random.default_rng(3 + policy)
    s2, m2, p2 = _mutate(s2.cpu().numpy(), m2.cpu().numpy(), p2.cpu().numpy(), rng)
    half = stl.verify_batch(s2, m2, p2, policy=policy)
    full = stl.verify_batch(s2, m2, p2, policy=policy | stl.FULL_LENGTH)
    assert np.array_equal(half, full)
    assert np.array_equal(half, oracle.verify_batch(s2, m2, p2, policy=policy, threads=16))


def test_chunk_boundary(stl, oracle, torch_cuda):
    """n just above the phase-1 chunk (2^20): two chunks, bitmap words of the
    second chunk land after the first; mutated rows straddle the boundary."""
    torch = torch_cuda
    n = (1 << 20) + 4097
    sig, msg, pk = _gpu_signed(stl, torch, n, 4242)
    sig = sig.clone()
    bad_rows = torch.tensor([0, 5, (1 << 20) - 1, 1 << 20, (1 << 20) + 63, (1 << 20) + 64, n - 1], device=sig.device)
    sig[bad_rows, 33] ^= 1
    words = stl.verify_batch_device(sig, msg, pk)
    torch.cuda.synchronize()
    got = stl.words_to_bool(words, n)
    exp = np.ones(n, bool)
    exp[bad_rows.cpu().numpy()] = False
    assert np.array_equal(got, exp)


def test_tx_hash_device_config5(stl, torch_cuda):
    """SHA512Half over 20,000 preimages of log-uniform length 100 B - 4 KB at
    arbitrary byte offsets (config 5 shape), device entry point, against
    hashlib; lanes of one wave see very different block counts (work queue)."""
    import ctypes

    from stellard_amd import _native as N
    torch = torch_cuda
    rng = np.random.default_rng(31)
    n = 20000
    lens = np.exp(rng.uniform(np.log(100), np.log(4096), n)).astype(np.uint32)
    gaps = rng.integers(0, 7, n).astype(np.uint64)  # odd alignments
    offs = np.zeros(n, np.uint64)
    offs[1:] = np.cumsum(lens[:-1].astype(np.uint64) + gaps[:-1])
    total = int(offs[-1] + lens[-1])
    blob = rng.integers(0, 256, total, dtype=np.uint8)
    d_blob, d_off, d_len = (torch.from_numpy(a).cuda() for a in (blob, offs.view(np.int64), lens.view(np.int32)))
    d_msg = torch.empty((n, 32), dtype=torch.uint8, device="cuda")
    s = torch.cuda.current_stream()
    N.check(N.load().stl_tx_hash_batch_device(ctypes.c_void_p(d_blob.data_ptr()), ctypes.c_void_p(d_off.data_ptr()),
                                              ctypes.c_void_p(d_len.data_ptr()), n, ctypes.c_void_p(d_msg.data_ptr()),
                                              ctypes.c_void_p(s.cuda_stream)), "stl_tx_hash_batch_device")
    torch.cuda.synchronize()
    got = d_msg.cpu().numpy()
    for i in range(n):
        o, ln = int(offs[i]), int(lens[i])
        assert got[i].tobytes() == hashlib.sha512(blob[o:o + ln].tobytes()).digest()[:32], i


def test_check_sign_batch_mixed(stl, oracle):
    """SerializedTransaction::checkSign mirror over a mixed batch: well-formed
    rows through stl_tx_verify_batch (bits == CPU oracle), B12 malformed rows
    rejected on the host, cache flags set like the serial path."""
    rng = np.random.default_rng(44)
    keys = [oracle.keypair(rng.bytes(32)) for _ in range(8)]
    txs, exp = [], []
    for i in range(300):
        pkb, sk = keys[i % 8]
        pre = b"STX\x00" + rng.bytes(int(rng.integers(100, 600)))
        s = bytearray(oracle.sign(hashlib.sha512(pre).digest()[:32], sk))
        kind = i % 6
        if kind == 1:
            s[int(rng.integers(64))] ^= 1 << int(rng.integers(8))
        if kind == 2:
            txs.append(stl.SignedTx(pkb + b"\x00", bytes(s), pre))
            exp.append(False)
            continue
        if kind == 3:
            txs.append(stl.SignedTx(pkb, None, pre))
            exp.append(False)
            continue
        txs.append(stl.SignedTx(pkb, bytes(s), pre))
        sig = np.frombuffer(bytes(s), np.uint8).reshape(1, 64)
        exp.append(bool(oracle.tx_verify_batch([pre], sig, np.frombuffer(pkb, np.uint8).reshape(1, 32))[0]))
    got = stl.check_sign_batch(txs)
    assert got == exp
    assert all(t.sig_good == e and t.sig_bad == (not e) for t, e in zip(txs, exp))
    assert stl.check_sign_batch(txs) == exp  # cached verdicts


# ---- serialized transactions (stl_tx_blob_*; stl_txblob.h) ----

def _blob_expectations(oracle, blobs):
    """Reference bits / ids (oracle re-serialisation), whether the reference
    constructs the transaction at all, and the device pass compiled for the
    host (status, tx id) for each blob."""
    from tests.oracle_bind import hostemu_tx_blob, load_hostemu
    emu = load_hostemu()
    bits, ids = oracle.tx_blob_verify_batch(blobs, tx_ids=True)
    built = np.array([oracle.tx_blob(b)[0] for b in blobs], bool)
    em = [hostemu_tx_blob(emu, b) for b in blobs]
    st = np.array([e[0] for e in em], np.uint8)
    emu_ids = np.array([np.frombuffer(e[2], np.uint8) for e in em]).reshape(-1, 32)
    return dict(bits=bits, ids=ids, built=built, status=st, emu_ids=emu_ids)


def _check_blob_results(got_bits, got_status, got_ids, exp):
    # the GPU runs the same pass as its host build, bit for bit
    assert np.array_equal(got_status, exp["status"]), np.nonzero(got_status != exp["status"])[0][:10]
    assert np.array_equal(got_ids, exp["emu_ids"])
    decided = got_status != 1
    # decided rows the reference constructs: exactly its checkSign and transaction ID
    chk = decided & exp["built"]
    assert np.array_equal(got_bits[chk], exp["bits"][chk]), np.nonzero((got_bits != exp["bits"]) & chk)[0][:10]
    assert (got_ids[chk] == exp["ids"][chk]).all()
    # deferred rows: never accepted, id zero
    assert not got_bits[~decided].any()
    assert not got_ids[~decided].any()


def test_tx_blob_special_cases_and_corpus(stl, oracle):
    from tests import txblob as T
    blobs = [b for _, b, _ in T.special_cases(oracle)] + T.valid_corpus(oracle, 400, seed=21)
    exp = _blob_expectations(oracle, blobs)
    for policy in (0, 1):
        bits, st, ids = stl.tx_blob_verify_batch(blobs, policy=policy, tx_ids=True)
        _check_blob_results(bits, st, ids, exp)
    assert (exp["status"] == 0).sum() > 400


def test_tx_blob_cut_in_later_blocks(stl, oracle, torch_cuda):
    """Payments whose TxnSignature starts past the first SHA-512 block of the
    signing preimage (every optional field before it: tags, the last ledger
    sequence, PreviousTxnID / AccountTxnID / InvoiceID, IOU Amount and SendMax
    -- up to 4 + 270 bytes): the parse kernel assembles block 1 or 2 as the
    spliced block and the hash kernel reads the blocks around it as plain
    windows.  Bits, statuses and IDs equal the oracle's, through the host API
    and the device-resident one call."""
    torch = torch_cuda
    from tests import txblob as T
    from tests.oracle_bind import pack_blobs
    rng = np.random.default_rng(0xC075)
    ks = T.keys(oracle, 4, 0xC075)
    cur = b"\0" * 12 + b"USD" + b"\0" * 5
    blobs, xs = [], []
    for i in range(600):
        pk, sk = ks[i % 4]
        fs = [T.Field(T.TransactionType, T.u16(0)), T.Field(T.Flags, T.u32(0x80000000)),
              T.Field(T.Sequence, T.u32(i + 1)), T.Field(T.Fee, T.amount_native(10)),
              T.Field(T.SigningPubKey, T.vl(pk)), T.Field(T.Account, T.vl(T.account_id(pk))),
              T.Field(T.Destination, T.vl(rng.bytes(20)))]
        if rng.random() < 0.8:
            fs.append(T.Field(T.Amount, T.amount_iou(int(rng.integers(10**15, 10**16)), 0, cur, rng.bytes(20))))
        else:
            fs.append(T.Field(T.Amount, T.amount_native(int(rng.integers(1, 10**11)))))
        opt = [(T.SourceTag, T.u32(int(rng.integers(0, 2**32)))), (T.DestinationTag, T.u32(7)),
               (T.LastLedgerSequence, T.u32(99)), ((T.HASH256, 5), rng.bytes(32)),  # PreviousTxnID
               (T.AccountTxnID, rng.bytes(32)), (T.InvoiceID, rng.bytes(32)),
               (T.SendMax, T.amount_iou(int(rng.integers(10**15, 10**16)), 0, cur, rng.bytes(20)))]
        for fid, v in opt:
            if rng.random() < 0.85:
                fs.append(T.Field(fid, v))
        if rng.random() < 0.3:
            fs.append(T.Field(T.Memos, T.array_value([(T.Memo, [T.Field(T.MemoData, T.vl(rng.bytes(int(rng.integers(0, 600)))))])])))
        blob, _, sig = T.signed_blob(fs, sk, oracle.sign)
        blobs.append(blob)
        xs.append(blob.find(b"\x74\x40" + bytes(sig)))
    xs = np.array(xs)
    assert (xs >= 0).all() and ((4 + xs) // 128 >= 1).sum() > 300 and ((4 + xs) // 128 == 2).sum() > 50, \
        np.bincount((4 + xs) // 128)
    exp = _blob_expectations(oracle, blobs)
    assert (exp["status"] == 0).all()
    bits, st, ids = stl.tx_blob_verify_batch(blobs, tx_ids=True)
    _check_blob_results(bits, st, ids, exp)
    assert bits.all()
    buf, offs, lens = pack_blobs(blobs)
    out = stl.signed_blob_verify_batch_device(torch.from_numpy(buf).cuda(), torch.from_numpy(offs.astype(np.int64)).cuda(),
                                              torch.from_numpy(lens.astype(np.int32)).cuda())
    torch.cuda.synchronize()
    assert stl.words_to_bool(out["words"], len(blobs)).all()
    assert np.array_equal(out["status"].cpu().numpy(), st)


def test_tx_blob_fuzz(stl, oracle):
    from tests import txblob as T
    base = T.valid_corpus(oracle, 200, seed=5)
    rng = np.random.default_rng(77)
    blobs = []
    for _ in range(6000):
        m = T.mutate(rng, base[int(rng.integers(len(base)))])
        if rng.random() < 0.3:
            m = T.mutate(rng, m)
        blobs.append(m)
    exp = _blob_expectations(oracle, blobs)
    bits, st, ids = stl.tx_blob_verify_batch(blobs, tx_ids=True)
    _check_blob_results(bits, st, ids, exp)
    assert exp["built"].sum() > 1000


def test_tx_blob_prepare_device(stl, oracle, torch_cuda):
    """Device-resident prepare + verify == host entry point; msg / sig / pk as
    the blob holds them; deferred rows get the always-reject signature."""
    torch = torch_cuda
    from tests import txblob as T
    from tests.oracle_bind import pack_blobs
    blobs = [b for _, b, _ in T.special_cases(oracle)] + T.valid_corpus(oracle, 300, seed=8, memos=1)
    buf, offs, lens = pack_blobs(blobs)
    d_buf = torch.from_numpy(buf).cuda()
    d_off = torch.from_numpy(offs.astype(np.int64)).cuda()
    d_len = torch.from_numpy(lens.astype(np.int32)).cuda()
    out = stl.tx_blob_prepare_device(d_buf, d_off, d_len)
    words = stl.verify_batch_device(out["sig"], out["msg"], out["pk"])
    torch.cuda.synchronize()
    n = len(blobs)
    got = stl.words_to_bool(words, n)
    bits, st, ids = stl.tx_blob_verify_batch(blobs, tx_ids=True)
    assert np.array_equal(got, bits)
    assert np.array_equal(out["status"].cpu().numpy(), st)
    assert np.array_equal(out["tx_id"].cpu().numpy(), ids)
    sig = out["sig"].cpu().numpy()
    pk = out["pk"].cpu().numpy()
    for i, b in enumerate(blobs):
        if st[i] == 0:
            ok, info, signing, full = oracle.tx_blob(b)
            assert bytes(sig[i]) == bytes(info.sig) and bytes(pk[i]) == bytes(info.pk[:32])
            assert bytes(out["msg"][i].cpu().numpy()) == hashlib.sha512(signing).digest()[:32]
        else:
            assert not sig[i, :32].any() and (sig[i, 32:] == 255).all() and not pk[i].any()


def test_tx_blob_config5_sizes(stl, oracle):
    """Ledger-replay shaped blobs (tests/datasets.py blob_ledger_plan: log-
    uniform 100 B - 4 KB, 2 % invalid -- payload / R / S bits flipped after
    signing, Flags and Sequence swapped, 33-byte keys) in one batch of 20,000
    (SURVEY config-5 ledger size): every row's bit, status and transaction id
    against the re-serialising oracle and the device pass's host build
    (not only bits.all())."""
    from tests import datasets as D
    bp, blobs = D.blob_ledger_cpu(oracle, 20000, frac=0.02)
    exp = _blob_expectations(oracle, blobs)
    assert np.array_equal(exp["status"], D.blob_expected_status(bp))
    for policy in (0, stl.DEDUP_KEYS):
        bits, st, ids = stl.tx_blob_verify_batch(blobs, policy=policy, tx_ids=True)
        _check_blob_results(bits, st, ids, exp)
    assert (st == 1).sum() == (bp["kind"] == 3).sum() and (st == 2).sum() == (bp["kind"] == 4).sum()
    assert bits.sum() == len(blobs) - bp["bad"].size


def test_batcher_verdicts(stl, oracle, golden):
    """The request aggregator (f2): single requests from 4 threads, batched by
    size and delay, give the same verdicts as the batch calls -- golden
    signatures (every Appendix-B class) and serialized transactions (special
    cases: accept / reject / defer)."""
    import threading
    from tests import txblob as T
    sig, msg, pk = _golden_arrays(golden)
    exp = golden["expected_sodium_1_0_18"].astype(bool)
    cases = T.special_cases(oracle)
    blobs = [b for _, b, _ in cases]
    bits, st = stl.tx_blob_verify_batch(blobs)
    with stl.Batcher(max_batch=256, max_delay_us=300) as b:
        hs, ht = [None] * len(sig), [None] * len(blobs)

        def worker(k):
            for i in range(k, len(sig), 4):
                hs[i] = b.submit(sig[i], msg[i], pk[i])
            for i in range(k, len(blobs), 4):
                ht[i] = b.submit_tx(blobs[i])

        ts = [threading.Thread(target=worker, args=(k,)) for k in range(4)]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        b.flush()
        got = np.array([h.result(timeout=30) for h in hs])
        assert np.array_equal(got == stl.VERDICT_ACCEPT, exp)
        assert set(np.unique(got)) <= {stl.VERDICT_ACCEPT, stl.VERDICT_REJECT}
        gt = np.array([h.result(timeout=30) for h in ht])
        want = np.where(st == 1, stl.VERDICT_DEFER, np.where(bits, stl.VERDICT_ACCEPT, stl.VERDICT_REJECT))
        assert np.array_equal(gt, want)
        s = b.stats()
        assert s["completed"] == len(sig) + len(blobs)


@pytest.mark.parametrize("policy", [0, 1])
def test_shared_key_domain_same_bits(stl, golden, oracle, torch_cuda, policy):
    """Round 6: a device-resident call of several chunks with key dedup builds
    ONE key domain for all of them (STL_TUNE_SHARED_KEYS, default on): its
    first chunk builds the hash slots, decoded keys and wide / shared key
    tables over every row, the others wait for them.  Bits equal the
    per-chunk domains', the 9-entry-only tables' (STL_TUNE_WIDE_MIN_ROWS) and
    the no-dedup path's, at sizes of 2 chunks (100k,
    300k), 4 chunks (1M) and with wide (1,000 signers) and 9-entry (10,000
    signers on 100k rows: < 32 rows per key) tables, 5 % of rows mutated --
    and through the one-call checkSign from preimages."""
    torch = torch_cuda
    rng = np.random.default_rng(0x5EED5)
    for n, signers in ((100_000, 1000), (300_000, 1000), (1 << 20, 1000), (100_000, 10_000)):
        aseed = rng.integers(0, 256, (signers, 32), dtype=np.uint8)
        who = rng.integers(0, signers, n)
        msgs = torch.from_numpy(rng.integers(0, 256, (n, 32), dtype=np.uint8)).cuda()
        pkd, sigd = stl.sign_batch_device(torch.from_numpy(aseed[who]).cuda(), msgs)
        bad = rng.random(n) < 0.05
        col = torch.from_numpy(rng.integers(0, 64, int(bad.sum()))).cuda()
        sigd[torch.from_numpy(np.nonzero(bad)[0]).cuda(), col] ^= 0x10
        got = {}
        # (shared domain, wide-table row minimum): 1 << 20 builds 9-entry tables only
        for shared, wmin in ((1, 0), (0, 0), (1, 1 << 20)):
            old = stl.debug_tuning(stl.TUNE_SHARED_KEYS, shared)
            oldw = stl.debug_tuning(stl.TUNE_WIDE_MIN_ROWS, wmin)
            try:
                w = stl.verify_batch_device(sigd, msgs, pkd, policy=policy | stl.DEDUP_KEYS)
                torch.cuda.synchronize()
                got[(shared, wmin)] = stl.words_to_bool(w, n)
            finally:
                stl.debug_tuning(stl.TUNE_SHARED_KEYS, old)
                stl.debug_tuning(stl.TUNE_WIDE_MIN_ROWS, oldw)
        assert np.array_equal(got[(1, 0)], got[(1, 1 << 20)]), (n, signers)
        got = {k[0]: v for k, v in got.items() if k[1] == 0}
        w = stl.verify_batch_device(sigd, msgs, pkd, policy=policy | stl.NO_AUTO_DEDUP)
        torch.cuda.synchronize()
        plain = stl.words_to_bool(w, n)
        assert np.array_equal(got[1], got[0]), (n, signers)
        assert np.array_equal(got[1], plain), (n, signers)
        assert np.array_equal(plain, ~bad), (n, signers)
        samp = rng.choice(n, 2000, replace=False)
        s_np, m_np, p_np = sigd.cpu().numpy(), msgs.cpu().numpy(), pkd.cpu().numpy()
        assert np.array_equal(got[1][samp], oracle.verify_batch(s_np[samp], m_np[samp], p_np[samp], policy=policy))
    # one-call checkSign over preimages, 2 chunks, forced dedup, shared vs not;
    # 99,968 rows: chunks of 50,048 and 49,920 rows whose verify grids differ
    # (196 vs 195 workgroups' worth) while they share one key domain;
    # 90,000 rows: a 65,536-row one-lane chunk and a lane-pair remainder,
    # which decodes its own R (only the first chunk's rows are decoded ahead)
    for n in (150_000, 99_968, 90_000):
        _one_call_shared_keys(stl, torch, rng, n, policy)


def _one_call_shared_keys(stl, torch, rng, n, policy):
    lens = rng.integers(113, 1500, n).astype(np.int32)
    offs = np.zeros(n, np.int64)
    offs[1:] = np.cumsum(lens[:-1])
    pre = rng.integers(0, 256, int(offs[-1] + lens[-1]) + 16, dtype=np.uint8)
    d_pre = torch.from_numpy(pre).cuda()
    d_off = torch.from_numpy(offs).cuda()
    d_len = torch.from_numpy(lens).cuda()
    m = stl.tx_hash_batch_device(d_pre, d_off, d_len)
    aseed = rng.integers(0, 256, (500, 32), dtype=np.uint8)
    pkd, sigd = stl.sign_batch_device(torch.from_numpy(aseed[rng.integers(0, 500, n)]).cuda(), m)
    bad = rng.random(n) < 0.03
    sigd[torch.from_numpy(np.nonzero(bad)[0]).cuda(), 50] ^= 0x04
    outs = []
    # (shared domain, R decoded ahead on its own stream)
    for shared, ahead in ((1, 1), (1, 0), (0, 0)):
        old = stl.debug_tuning(stl.TUNE_SHARED_KEYS, shared)
        olda = stl.debug_tuning(stl.TUNE_R_AHEAD, ahead)
        try:
            w = stl.tx_verify_batch_device(d_pre, d_off, d_len, sigd, pkd, policy=policy | stl.DEDUP_KEYS)
            torch.cuda.synchronize()
            outs.append(stl.words_to_bool(w, n))
        finally:
            stl.debug_tuning(stl.TUNE_SHARED_KEYS, old)
            stl.debug_tuning(stl.TUNE_R_AHEAD, olda)
    assert np.array_equal(outs[0], outs[1]) and np.array_equal(outs[0], outs[2])
    assert np.array_equal(outs[0], ~bad)


@pytest.mark.parametrize("policy", [0, 1, 4])
def test_dedup_keys_same_bits(stl, golden, oracle, torch_cuda, policy):
    """STL_DEDUP_KEYS (each distinct key decoded once per batch) gives the same
    bits as the default path: golden rows (every adversarial key class, keys
    repeated across rows), and a 1,000-signer batch with mutations that
    straddles the 2^20-signature chunk, on the host and device entry points."""
    torch = torch_cuda
    sig, msg, pk = golden["sig"], golden["msg"], golden["pk"]
    key = "expected_stellard_1_0_0_unpinned" if policy & 1 else "expected_sodium_1_0_18"
    # 20,000 rows over the 525 golden keys (>= 32 rows per key): the wide
    # per-key tables (c's digits in radix-256 pairs); 8,000 rows: the 9-entry
    # per-key tables
    # (STL_ONE_LANE: batches this small otherwise run on lane pairs, no dedup)
    for rows in (20000, 8000):
        idx = np.random.default_rng(3).integers(0, sig.shape[0], rows)
        for extra in (stl.ONE_LANE, 0):
            got = stl.verify_batch(sig[idx], msg[idx], pk[idx], policy=policy | stl.DEDUP_KEYS | extra)
            assert np.array_equal(got, golden[key][idx].astype(bool)), (rows, extra)
    # 1,000 signers, (1 << 20) + 4099 rows: two chunks, keys shared across both
    n = (1 << 20) + 4099
    rng = np.random.default_rng(5)
    aseed = rng.integers(0, 256, (1000, 32), dtype=np.uint8)
    who = rng.integers(0, 1000, n)
    seeds = torch.from_numpy(aseed[who]).cuda()
    msgs = torch.from_numpy(rng.integers(0, 256, (n, 32), dtype=np.uint8)).cuda()
    pkd, sigd = stl.sign_batch_device(seeds, msgs)
    s_np, m_np, p_np = sigd.cpu().numpy(), msgs.cpu().numpy(), pkd.cpu().numpy()
    bad = rng.random(n) < 0.05
    s_np[bad, 40] ^= 0x20
    d = [torch.from_numpy(a).cuda() for a in (s_np, m_np, p_np)]
    w0 = stl.verify_batch_device(*d, policy=policy)
    w1 = stl.verify_batch_device(*d, policy=policy | stl.DEDUP_KEYS)
    torch.cuda.synchronize()
    b0, b1 = stl.words_to_bool(w0, n), stl.words_to_bool(w1, n)
    assert np.array_equal(b0, b1)
    assert np.array_equal(b1, ~bad)
    # the device API follows the key sample of the previous call on its
    # stream (w0's call above sampled these 1,000 signers): dedup, same bits
    stl.reset_stats()
    w2 = stl.verify_batch_device(*d, policy=policy)
    torch.cuda.synchronize()
    assert np.array_equal(stl.words_to_bool(w2, n), b1)
    auto = (policy & stl.FULL_LENGTH) == 0  # the cross-check mode keeps the caller's choice
    assert stl.get_stats()["auto_dedup_chunks"] == (1 if auto else 0)
    # the host API chooses dedup by itself for these chunks (1,000 signers:
    # the key sample repeats), and not when told not to -- same bits
    stl.reset_stats()
    assert np.array_equal(stl.verify_batch(s_np, m_np, p_np, policy=policy), b1)
    assert stl.get_stats()["auto_dedup_chunks"] == (-(-n // 65536) if auto else 0)
    stl.reset_stats()
    assert np.array_equal(stl.verify_batch(s_np, m_np, p_np, policy=policy | stl.NO_AUTO_DEDUP), b1)
    assert stl.get_stats()["auto_dedup_chunks"] == 0
    samp = rng.choice(n, 4000, replace=False)
    assert np.array_equal(b1[samp], oracle.verify_batch(s_np[samp], m_np[samp], p_np[samp], policy=policy & 1))
    # more distinct keys in one chunk than shared key tables (2^16): the chunk
    # falls back to per-lane A-tables and still gives the same bits
    n2 = 70000
    seeds2 = torch.from_numpy(rng.integers(0, 256, (n2, 32), dtype=np.uint8)).cuda()
    msgs2 = torch.from_numpy(rng.integers(0, 256, (n2, 32), dtype=np.uint8)).cuda()
    pk2, sig2 = stl.sign_batch_device(seeds2, msgs2)
    s2 = sig2.cpu().numpy()
    bad2 = rng.random(n2) < 0.05
    s2[bad2, 3] ^= 0x01
    d2 = [torch.from_numpy(s2).cuda(), msgs2, pk2]
    stl.verify_batch_device(*d2, policy=policy)  # its sample: distinct keys
    torch.cuda.synchronize()
    stl.reset_stats()
    u0 = stl.words_to_bool(stl.verify_batch_device(*d2, policy=policy), n2)
    torch.cuda.synchronize()
    assert stl.get_stats()["auto_dedup_chunks"] == 0
    u1 = stl.words_to_bool(stl.verify_batch_device(*d2, policy=policy | stl.DEDUP_KEYS), n2)
    torch.cuda.synchronize()
    assert np.array_equal(u0, u1)
    assert np.array_equal(u1, ~bad2)
    stl.reset_stats()  # distinct keys: the host API's sample does not repeat, no dedup
    assert np.array_equal(stl.verify_batch(s2, msgs2.cpu().numpy(), pk2.cpu().numpy(), policy=policy), u1)
    assert stl.get_stats()["auto_dedup_chunks"] == 0
