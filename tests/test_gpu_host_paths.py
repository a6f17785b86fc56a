"""GPU tests of the host-side paths around the kernels, through the C ABI:

* half-size and full-length lanes mixed in one wave (contrived k through
  stl_debug_verify_k_device) -- the fallback kernel ORs its bits into the
  words the main kernel wrote;
* the in-process multi-shard path (shards_per_device > 1: several host
  threads and shards per device) and the RCCL gather path (forced on one
  device), for signatures, preimages and serialized transactions, at ragged n;
* 6 host threads calling the batch entry points at once (stellard's JobQueue
  default, JobQueue.cpp:223-236);
* fault injection: every host, device and batcher entry point returns (or
  delivers) a negative code when a HIP/RCCL call fails -- never a reject --
  and the caller's fallback (the oracle standing in for libsodium) plus the
  next clean call reproduce the exact bitmap (SerializedTransaction.cpp:211-217,
  226-229: the reference maps exceptions to false; here an error is an error);
* one-process-per-GPU RCCL communicator (world size 1 on this box);
* f3: serialized validations (SerializedValidation.cpp:70-73, 96-110) and
  consensus proposals (LedgerProposal.cpp:54-65, 88-91).

Run on an MI355X:  python -u -m pytest tests -m gpu -x -v --timeout 120
"""
import contextlib
import os
import sys
import threading

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

L = 2**252 + 27742317777372353535851937790883648493
N8L = 8 * L


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


@contextlib.contextmanager
def reinit(stl, **cfg):
    """Re-initialise libstl with a configuration, restore the default after."""
    stl.shutdown()
    try:
        stl.init(**cfg)
        yield
    finally:
        stl.debug_fault_after(-1)
        stl.shutdown()
        stl.init()


def _golden_rows(golden, n, seed=0):
    idx = np.random.default_rng(seed).integers(0, golden["sig"].shape[0], n)
    return (golden["sig"][idx], golden["msg"][idx], golden["pk"][idx],
            golden["expected_sodium_1_0_18"][idx].astype(bool))


def _preimage_corpus(oracle, n, seed):
    """Variable-length signing preimages (100 B - 4 KB), signed, ~1/3 mutated."""
    rng = np.random.default_rng(seed)
    pres, sigs, pks = [], [], []
    keys = [oracle.keypair(rng.bytes(32)) for _ in range(8)]
    for i in range(n):
        ln = int(np.exp(rng.uniform(np.log(100), np.log(4096))))
        pre = b"STX\x00" + rng.bytes(ln - 4)
        pk, sk = keys[i % 8]
        h = oracle.sha512(pre)[:32]
        s = bytearray(oracle.sign(h, sk))
        if rng.random() < 0.33:
            s[int(rng.integers(0, 64))] ^= 1 << int(rng.integers(0, 8))
        pres.append(pre)
        sigs.append(bytes(s))
        pks.append(pk)
    sig = np.frombuffer(b"".join(sigs), np.uint8).reshape(n, 64)
    pk = np.frombuffer(b"".join(pks), np.uint8).reshape(n, 32)
    return pres, sig, pk


# ---------------------------------------------------------------- mixed waves
def test_mixed_fallback_lanes_in_one_wave(stl, torch_cuda, oracle):
    """Lanes whose k the lattice reduction cannot halve (full-length fallback
    kernel) next to ordinary lanes in the same 64-lane waves: every bit exact
    (ADVICE r1).  Signatures are valid for their given k by construction
    (S = r + k*a mod L), half of them then broken (S+1)."""
    torch = torch_cuda
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), "golden"))
    import ed25519_py as ed

    from tests import oracle_bind
    from tests.test_halfscalar import _boundary_ks, _fib_ks
    emu = oracle_bind.load_hostemu()

    def lattice_ok(k):
        import ctypes
        c, d, s = ctypes.create_string_buffer(20), ctypes.create_string_buffer(20), ctypes.c_uint32(0)
        return bool(emu.hostemu_lattice(k.to_bytes(32, "little"), c, d, ctypes.byref(s)))

    contrived = [k for k in _boundary_ks() + _fib_ks() if not lattice_ok(k)]
    assert len(contrived) >= 3, "no k takes the full-length path"
    rng = np.random.default_rng(21)
    n = 256
    sig, kk, pk, exp = [], [], [], []
    a = int.from_bytes(rng.bytes(32), "little") % L
    A = ed.encode(ed.mul(a, ed.B))
    for i in range(n):
        k = contrived[i % len(contrived)] if i % 9 == 4 else int.from_bytes(rng.bytes(32), "little") % L
        r = int.from_bytes(rng.bytes(32), "little") % L
        R = ed.encode(ed.mul(r, ed.B))
        S = (r + k * a) % L
        good = (i // 2) % 2 == 0
        if not good:
            S = (S + 1) % L
        sig.append(R + S.to_bytes(32, "little"))
        kk.append(k.to_bytes(32, "little"))
        pk.append(A)
        exp.append(good)
    exp = np.array(exp)
    flagged = np.array([i % 9 == 4 for i in range(n)])
    assert all(flagged[w * 64:(w + 1) * 64].any() and (~flagged[w * 64:(w + 1) * 64]).any() for w in range(4))
    d = [torch.from_numpy(np.frombuffer(b"".join(x), np.uint8).reshape(n, -1).copy()).cuda() for x in (sig, kk, pk)]
    for flags in (0, stl.FULL_LENGTH):
        stl.reset_stats()
        words = stl.debug_verify_k_device(d[0], d[1], d[2], policy=flags)
        torch.cuda.synchronize()
        got = stl.words_to_bool(words, n)
        assert np.array_equal(got, exp), (flags, np.nonzero(got != exp)[0][:10])
        # device counters (stl_get_stats): the accepts, and exactly the
        # contrived lanes through the full-length path (every lane with the flag)
        st = stl.get_stats()
        assert st["accepted"] == int(exp.sum())
        assert st["full_length_lanes"] == (n if flags else int(flagged.sum())), st


# ------------------------------------------------------- multi-shard / RCCL
@pytest.mark.parametrize("mode", ["shards3", "rccl1", "rccl1_bytes"])
def test_host_paths_multi_shard_and_rccl(stl, oracle, golden, mode):
    """rccl1_bytes: the byte-balanced shard path on one device (test hook
    STL_TUNE_BYTE_SHARDS) -- the grouped gather's placement and rank 0's own
    device copy run for the preimage and blob batches."""
    from stellard_amd import _native as N
    cfg = dict(shards_per_device=3) if mode == "shards3" else dict(flags=N.STL_CFG_RCCL_GATHER)
    prev = stl.debug_tuning(stl.TUNE_BYTE_SHARDS, 1 if mode == "rccl1_bytes" else 0)
    try:
        _host_paths(stl, oracle, golden, mode, cfg)
    finally:
        stl.debug_tuning(stl.TUNE_BYTE_SHARDS, prev)


def _host_paths(stl, oracle, golden, mode, cfg):
    from tests import txblob
    blobs = txblob.valid_corpus(oracle, 400, 31)
    rng = np.random.default_rng(32)
    blobs = [b[:-1] + bytes([b[-1] ^ 1]) if rng.random() < 0.3 else b for b in blobs]
    exp_blob, exp_ids = oracle.tx_blob_verify_batch(blobs, tx_ids=True)
    pres, psig, ppk = _preimage_corpus(oracle, 700, 33)
    exp_pre = oracle.tx_verify_batch(pres, psig, ppk)
    with reinit(stl, **cfg):
        for n in (1, 63, 65, 64 * 1024 + 37):
            sig, msg, pk, exp = _golden_rows(golden, n, seed=n)
            got = stl.verify_batch(sig, msg, pk)
            assert np.array_equal(got, exp), (mode, n)
        assert np.array_equal(stl.tx_verify_batch(pres, psig, ppk), exp_pre), mode
        bits, status, ids = stl.tx_blob_verify_batch(blobs, tx_ids=True)
        assert np.array_equal(bits, exp_blob), mode
        ok = status != stl.TX_DEFERRED
        assert ok.sum() > 300
        assert np.array_equal(ids[ok], exp_ids[ok])
        # single drop-in call through the same host path
        s, m, p, e = _golden_rows(golden, 8, seed=3)
        for i in range(8):
            assert stl.verify_signature(m[i].tobytes(), s[i].tobytes(), p[i].tobytes()) == bool(e[i])


def test_six_threads_concurrently(stl, oracle, golden):
    """stellard's JobQueue runs min(ncpu,4)+2 = 6 workers (JobQueue.cpp:223-236)
    that may all verify at once: every thread gets its own exact bitmap."""
    pres, psig, ppk = _preimage_corpus(oracle, 300, 41)
    exp_pre = oracle.tx_verify_batch(pres, psig, ppk)
    results, errors = {}, []

    def worker(t):
        try:
            for rep in range(3):
                n = 1000 + 517 * t + rep
                sig, msg, pk, exp = _golden_rows(golden, n, seed=100 * t + rep)
                got = stl.verify_batch(sig, msg, pk)
                results[(t, rep)] = bool(np.array_equal(got, exp))
                if t % 2:
                    results[(t, rep, "tx")] = bool(np.array_equal(stl.tx_verify_batch(pres, psig, ppk), exp_pre))
        except Exception as e:  # noqa: BLE001 - reported below
            errors.append(repr(e))

    ts = [threading.Thread(target=worker, args=(t,)) for t in range(6)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=100)
    assert not errors, errors
    assert len(results) == 18 + 9 and all(results.values()), results


def test_six_threads_multi_shard(stl, golden):
    with reinit(stl, shards_per_device=2):
        errors = []

        def worker(t):
            sig, msg, pk, exp = _golden_rows(golden, 3000 + t, seed=t)
            if not np.array_equal(stl.verify_batch(sig, msg, pk), exp):
                errors.append(t)

        ts = [threading.Thread(target=worker, args=(t,)) for t in range(6)]
        for t in ts:
            t.start()
        for t in ts:
            t.join(timeout=100)
        assert not errors


# ------------------------------------------------------------ fault injection
def _entry_points(stl, torch, oracle, golden):
    sig, msg, pk, exp = _golden_rows(golden, 700, seed=9)
    pres, psig, ppk = _preimage_corpus(oracle, 200, 10)
    exp_pre = oracle.tx_verify_batch(pres, psig, ppk)
    from tests import txblob
    blobs = txblob.valid_corpus(oracle, 150, 12)
    exp_blob = oracle.tx_blob_verify_batch(blobs)
    d = [torch.from_numpy(np.ascontiguousarray(a)).cuda() for a in (sig, msg, pk)]

    def dev():
        w = stl.verify_batch_device(*d)
        torch.cuda.synchronize()
        return stl.words_to_bool(w, sig.shape[0])

    def detached():
        return np.array([stl.verify_signature(msg[i].tobytes(), sig[i].tobytes(), pk[i].tobytes())
                         for i in range(4)])

    def detached_var():
        pkb, sk = oracle.keypair(bytes(range(32)))
        m = b"variable length message" * 3
        return np.array([stl.crypto_sign_verify_detached(oracle.sign(m, sk), m, pkb) == 0])

    return {
        "verify_batch": (lambda: stl.verify_batch(sig, msg, pk), exp,
                         lambda: oracle.verify_batch(sig, msg, pk)),
        "tx_verify_batch": (lambda: stl.tx_verify_batch(pres, psig, ppk), exp_pre,
                            lambda: oracle.tx_verify_batch(pres, psig, ppk)),
        "tx_blob_verify_batch": (lambda: stl.tx_blob_verify_batch(blobs)[0], exp_blob,
                                 lambda: oracle.tx_blob_verify_batch(blobs)),
        "verify_batch_device": (dev, exp, lambda: oracle.verify_batch(sig, msg, pk)),
        "verify_detached": (detached, exp[:4], lambda: oracle.verify_batch(sig[:4], msg[:4], pk[:4])),
        "verify_detached_var": (detached_var, np.array([True]), lambda: np.array([True])),
    }


@pytest.mark.parametrize("mode", ["default", "rccl1"])
def test_fault_injection_every_entry_point(stl, torch_cuda, oracle, golden, mode):
    from stellard_amd import _native as N
    cfg = {} if mode == "default" else dict(flags=N.STL_CFG_RCCL_GATHER)
    with reinit(stl, **cfg):
        eps = _entry_points(stl, torch_cuda, oracle, golden)
        report = {}
        for name, (call, exp, fallback) in eps.items():
            hits = 0
            for k in range(0, 80):
                stl.debug_fault_after(k)
                try:
                    got = call()
                    failed = None
                except N.StlError as e:
                    failed = e.rc
                stl.debug_fault_after(-1)
                if failed is None:
                    # the countdown outlived the call: a clean, exact result
                    assert np.array_equal(got, exp), (name, k)
                    break
                assert failed < 0 and failed != -1, (name, k, failed)  # an error, never a reject
                hits += 1
                # the caller falls back to its own check (libsodium; the oracle here) ...
                assert np.array_equal(fallback(), exp), name
                # ... and the library is not poisoned: the next clean call is exact
                assert np.array_equal(call(), exp), (name, k)
            else:
                pytest.fail(f"{name}: still failing after 80 injected faults")
            report[name] = hits
        assert all(h >= 1 for h in report.values()), report


def test_stats_count_calls_signatures_and_errors(stl, golden):
    """stl_get_stats (SURVEY.md section 5 metrics): host calls, signatures,
    errors, device accepts."""
    sig, msg, pk, exp = _golden_rows(golden, 5000, seed=8)
    stl.reset_stats()
    got = stl.verify_batch(sig, msg, pk)
    assert np.array_equal(got, exp)
    st = stl.get_stats()
    assert st["batches"] == 1 and st["signatures"] == 5000 and st["errors"] == 0
    assert st["accepted"] == int(exp.sum()) and st["host_ns"] > 0
    stl.debug_fault_after(0)
    from stellard_amd import _native as N
    with pytest.raises(N.StlError):
        stl.verify_batch(sig, msg, pk)
    stl.debug_fault_after(-1)
    st = stl.get_stats()
    assert st["batches"] == 2 and st["errors"] == 1


def test_phase_timing(stl, golden, torch_cuda):
    """stl_set_phase_timing: per-phase event times for every chunk of the
    host and device entry points, the same bits with timing on, and nothing
    timed once it is off again."""
    torch = torch_cuda
    sig, msg, pk, exp = _golden_rows(golden, 3000, seed=9)
    stl.reset_stats()
    assert stl.set_phase_timing(True) is False
    try:
        assert np.array_equal(stl.verify_batch(sig, msg, pk), exp)
        d = [torch.from_numpy(a).cuda() for a in (sig, msg, pk)]
        w = stl.verify_batch_device(*d)
        torch.cuda.synchronize()
        assert np.array_equal(stl.words_to_bool(w, 3000), exp)
        st = stl.get_stats()
        assert st["phase_chunks"] == 2, st
        ph = st["phase_ns"]
        assert all(ph[k] > 0 for k in ("phase1", "main")), ph  # "point" is 0 with the fused phase-1 kernel
        assert ph["main"] > ph["phase1"], ph
    finally:
        stl.set_phase_timing(False)
    stl.verify_batch(sig, msg, pk)
    assert stl.get_stats()["phase_chunks"] == 2
    stl.reset_stats()
    assert stl.get_stats()["phase_chunks"] == 0


def test_fault_injection_batcher_delivers_errors(stl, oracle, golden):
    sig, msg, pk, exp = _golden_rows(golden, 50, seed=4)
    for k in (0, 2, 5):
        with stl.Batcher(max_batch=50, max_delay_us=100_000) as b:
            stl.debug_fault_after(k)
            hs = [b.submit(sig[i].tobytes(), msg[i].tobytes(), pk[i].tobytes()) for i in range(50)]
            b.flush()
            stl.debug_fault_after(-1)
            vs = [h.result(timeout=30) for h in hs]
        # a request of a failed batch gets the negative code (never a reject);
        # the others their exact verdict
        for v, e in zip(vs, exp):
            assert v < 0 or (v == stl.VERDICT_ACCEPT) == bool(e), (k, v, e)
        if k == 0:
            assert any(v < 0 for v in vs)


def test_init_fault_then_recover(stl, golden):
    stl.shutdown()
    try:
        for k in range(0, 6):
            stl.debug_fault_after(k)
            from stellard_amd import _native as N
            try:
                stl.init()
                ok = True
            except N.StlError as e:
                ok = False
                assert e.rc < 0
            stl.debug_fault_after(-1)
            if ok:
                break
            stl.shutdown()
    finally:
        stl.debug_fault_after(-1)
        stl.shutdown()
        stl.init()
    sig, msg, pk, exp = _golden_rows(golden, 300, seed=5)
    assert np.array_equal(stl.verify_batch(sig, msg, pk), exp)


# ------------------------------------------------- one process per GPU (RCCL)
def test_comm_world_one_gather_and_allgather(stl, torch_cuda):
    torch = torch_cuda
    uid = stl.comm_unique_id()
    assert len(uid) == 128
    stl.comm_init_rank(1, 0, uid)
    try:
        w = torch.randint(-2**62, 2**62, (16384,), dtype=torch.int64, device="cuda")
        out = torch.zeros_like(w)
        stl.bitmap_gather_device(w, out, root=0)
        torch.cuda.synchronize()
        assert torch.equal(out, w)
        out2 = torch.zeros_like(w)
        stl.bitmap_gather_device(w, out2, root=-1)
        torch.cuda.synchronize()
        assert torch.equal(out2, w)
        from stellard_amd import _native as N
        with pytest.raises(N.StlError):
            stl.bitmap_gather_device(w, out, root=1)  # no such rank
    finally:
        stl.comm_destroy()


# ------------------------------------------------------ f3: other call sites
def test_validations_vs_oracle(stl, oracle, torch_cuda):
    """SerializedValidation::isValid(getSigningHash()) over serialized
    validations: the device splices "VAL\\0" || blob minus Signature and checks
    SigningPubKey / Signature; bits equal the re-serialising oracle, IDs the
    suppression hash SHA512Half(raw) (PeerImp.cpp:1148-1155)."""
    from tests import oracle_bind, txblob
    rng = np.random.default_rng(51)
    keys = [oracle.keypair(rng.bytes(32)) for _ in range(6)]
    blobs = []
    for i in range(600):
        pk, sk = keys[i % 6]
        fs = txblob.validation_fields(rng, pk, full=bool(i % 2))
        b, _, _ = txblob.signed_validation(fs, sk, oracle.sign)
        r = rng.random()
        if r < 0.15:
            b = bytearray(b)
            b[int(rng.integers(0, len(b)))] ^= 1 << int(rng.integers(0, 8))
            b = bytes(b)
        elif r < 0.2:
            b = b[: int(rng.integers(1, len(b)))]  # truncated
        blobs.append(b)
    # a transaction blob is not a validation (TxnSignature, not Signature) and vice versa
    tx = txblob.valid_corpus(oracle, 4, 52)
    blobs += tx
    exp, exp_ids = oracle.signed_blob_verify_batch(1, blobs, ids=True)
    got, status, ids = stl.signed_blob_verify_batch(blobs, kind=stl.BLOB_VALIDATION, ids=True)
    assert np.array_equal(got, exp)
    assert exp[:600].sum() > 400 and not got[600:].any()
    dec = status != stl.TX_DEFERRED
    assert dec[:600].sum() > 450
    assert np.array_equal(ids[dec], exp_ids[dec])
    # transactions through the transaction kind still verify
    assert stl.signed_blob_verify_batch(tx, kind=stl.BLOB_TRANSACTION)[0].all()
    sodium = oracle_bind.load_sodium_ref()
    if sodium is not None:
        assert np.array_equal(oracle_bind.sodium_signed_blob_verify_batch(sodium, 1, blobs), exp)
    # device-resident prepare: signing hashes equal the Python serializer's
    torch = torch_cuda
    from stellard_amd.verify import _pack
    buf, offs, lens = _pack(blobs[:100])
    o = stl.tx_blob_prepare_device(torch.from_numpy(buf).cuda(), torch.from_numpy(offs.view(np.int64)).cuda(),
                                   torch.from_numpy(lens.view(np.int32)).cuda(), tx_ids=True,
                                   kind=stl.BLOB_VALIDATION)
    words = stl.verify_batch_device(o["sig"], o["msg"], o["pk"])
    torch.cuda.synchronize()
    assert np.array_equal(stl.words_to_bool(words, 100), exp[:100])


def test_proposals_vs_oracle(stl, oracle):
    """LedgerProposal::checkSign (LedgerProposal.cpp:88-91) over the 76-byte
    "PRP\\0" preimage of getSigningHash (:54-65), through stl_tx_verify_batch."""
    rng = np.random.default_rng(61)
    keys = [oracle.keypair(rng.bytes(32)) for _ in range(5)]
    pres, sigs, pks = [], [], []
    for i in range(500):
        pk, sk = keys[i % 5]
        pre = stl.proposal_preimage(int(rng.integers(0, 2**32)), int(rng.integers(0, 2**32)), rng.bytes(32),
                                    rng.bytes(32))
        assert len(pre) == 76
        s = bytearray(oracle.sign(oracle.sha512(pre)[:32], sk))
        if i % 4 == 3:
            s[int(rng.integers(0, 64))] ^= 0x10
        if i % 50 == 7:
            pre = pre[:8] + bytes([pre[8] ^ 1]) + pre[9:]  # closeTime changed after signing
        pres.append(pre)
        sigs.append(bytes(s))
        pks.append(pk)
    sig = np.frombuffer(b"".join(sigs), np.uint8).reshape(-1, 64)
    pk = np.frombuffer(b"".join(pks), np.uint8).reshape(-1, 32)
    exp = oracle.tx_verify_batch(pres, sig, pk)
    got = stl.tx_verify_batch(pres, sig, pk)
    assert np.array_equal(got, exp)
    assert 300 < exp.sum() < 400


# --------------------------------------------- single call: caller fallback
def test_fallback_verify_answers_device_failures(stl, oracle, golden):
    """stl_config.fallback_verify (ABI 3): with the caller's own check
    registered (stellard: libsodium's crypto_sign_verify_detached; the oracle's
    raw libsodium-1.0.18 predicate here), stl_ed25519_verify_detached returns
    only 0 or -1 -- a failed device call is answered by the fallback composed
    with S < L, never reported as a reject (RippleAddress.cpp:196-199).
    Without a fallback the same failure is an error code below -1."""
    import ctypes

    from stellard_amd import _native as N
    sig, msg, pk, exp = _golden_rows(golden, 40, seed=17)
    calls = []

    def fb(s, m, mlen, p):
        calls.append(mlen)
        return 0 if oracle.verify_raw(ctypes.string_at(s, 64), ctypes.string_at(m, mlen),
                                      ctypes.string_at(p, 32), policy=0) else -1

    fn = stl.VERIFY_FN(fb)
    lib = N.load()
    with reinit(stl, fallback_verify=fn):
        for i in range(40):
            for k in range(0, 10):
                stl.debug_fault_after(k)
                rc = lib.stl_ed25519_verify_detached(sig[i].tobytes(), msg[i].tobytes(), 32, pk[i].tobytes())
                stl.debug_fault_after(-1)
                assert rc in (0, -1), (i, k, rc)
                assert (rc == 0) == bool(exp[i]), (i, k, rc)
        assert len(calls) >= 40 and set(calls) == {32}
    stl.debug_fault_after(0)
    rc = lib.stl_ed25519_verify_detached(sig[0].tobytes(), msg[0].tobytes(), 32, pk[0].tobytes())
    stl.debug_fault_after(-1)
    assert rc < -1


def test_comm_info(stl):
    """stl_comm_info: what RCCL reports for the communicator libstl gathers
    over (ncclCommCount / ncclCommUserRank) -- the bench asserts it equals
    WORLD_SIZE on every rank before timing."""
    from stellard_amd import _native as N
    with pytest.raises(N.StlError) as e:  # the default init builds no in-process communicator
        stl.comm_info()
    assert e.value.rc == N.STL_ERCCL
    stl.comm_init_rank(1, 0, stl.comm_unique_id())
    try:
        assert stl.comm_info() == (1, 0)
    finally:
        stl.comm_destroy()
    with reinit(stl, flags=N.STL_CFG_RCCL_GATHER):
        assert stl.comm_info() == (1, 0)


def test_fallback_registered_after_implicit_init(stl, oracle, golden):
    """a first entry-point call starts libstl implicitly
    (stl_init(NULL)); a later stl_init(cfg) must still register cfg's
    fallback -- not return early -- so verify_detached keeps returning only
    0 / -1 under injected device faults.  A cfg asking for other live settings
    (here the RCCL gather) is refused, not ignored.  A message longer than one
    device row (mlen > 2^32 - 1, valid input to libsodium) goes to the
    fallback too, composed with S < L."""
    import ctypes

    from stellard_amd import _native as N
    sig, msg, pk, exp = _golden_rows(golden, 12, seed=23)
    lib = N.load()
    seen = []

    def fb(s, m, mlen, p):
        seen.append(mlen)
        if mlen > 0xFFFFFFFF:
            return 0  # stands in for libsodium hashing a huge message; never reads m
        return 0 if oracle.verify_raw(ctypes.string_at(s, 64), ctypes.string_at(m, mlen),
                                      ctypes.string_at(p, 32), policy=0) else -1

    fn = stl.VERIFY_FN(fb)
    stl.shutdown()
    try:
        rc = lib.stl_ed25519_verify_detached(sig[0].tobytes(), msg[0].tobytes(), 32, pk[0].tobytes())
        assert rc == (0 if exp[0] else -1)  # implicit init
        stl.init(fallback_verify=fn)  # already running: registers the fallback
        for i in range(12):
            for k in range(0, 6):
                stl.debug_fault_after(k)
                rc = lib.stl_ed25519_verify_detached(sig[i].tobytes(), msg[i].tobytes(), 32, pk[i].tobytes())
                stl.debug_fault_after(-1)
                assert rc in (0, -1) and (rc == 0) == bool(exp[i]), (i, k, rc)
        assert 32 in seen
        with pytest.raises(N.StlError) as e:
            stl.init(flags=N.STL_CFG_RCCL_GATHER, fallback_verify=fn)
        assert e.value.rc == N.STL_EINVAL
        stl.init(fallback_verify=fn)  # the live settings: idempotent
        big = 1 << 33
        good = sig[int(np.argmax(exp))].tobytes()
        rc = lib.stl_ed25519_verify_detached(good, msg[0].tobytes(), big, pk[0].tobytes())
        assert rc == 0 and seen[-1] == big
        s_plus_l = good[:32] + (int.from_bytes(good[32:], "little") + L).to_bytes(32, "little")
        assert lib.stl_ed25519_verify_detached(s_plus_l, msg[0].tobytes(), big, pk[0].tobytes()) == -1
    finally:
        stl.debug_fault_after(-1)
        stl.shutdown()
        stl.init()
    # without a fallback the oversized message is an argument error
    assert lib.stl_ed25519_verify_detached(sig[0].tobytes(), msg[0].tobytes(), 1 << 33, pk[0].tobytes()) == N.STL_EINVAL


def test_bitmap_gatherv_one_rank(stl, torch_cuda):
    """stl_bitmap_gatherv_device on a one-rank communicator (the 1-GPU box):
    the root's slice lands at its word offset by a device copy; counts that
    disagree with the offsets are refused.  The N > 1 send/recv legs run in
    bench.py's config-4 / config-5 legs on a multi-GPU node."""
    torch = torch_cuda
    from stellard_amd import _native as N
    words = torch.arange(1, 1001, dtype=torch.int64, device="cuda") * 0x0101010101
    full = torch.zeros(1000, dtype=torch.int64, device="cuda")
    stl.comm_init_rank(1, 0, stl.comm_unique_id())
    try:
        stl.bitmap_gatherv_device(words, [0, 1000], full, root=0)
        torch.cuda.synchronize()
        assert torch.equal(full, words)
        with pytest.raises(N.StlError) as e:
            stl.bitmap_gatherv_device(words[:999], [0, 1000], full, root=0)
        assert e.value.rc == N.STL_EINVAL
        with pytest.raises(N.StlError) as e:
            stl.bitmap_gatherv_device(words, [0, 1000], full, root=1)
        assert e.value.rc == N.STL_EINVAL
    finally:
        stl.comm_destroy()
    with pytest.raises(N.StlError) as e:  # no communicator
        stl.bitmap_gatherv_device(words, [0, 1000], full, root=0)
    assert e.value.rc == N.STL_ERCCL


@pytest.mark.timeout(300)
def test_multi_device_in_process_rccl_gather(stl, torch_cuda, oracle, golden):
    """stellard's own shape -- one process, every visible
    device (stl_init with all of them and STL_CFG_RCCL_GATHER: ncclCommInitAll,
    ncclGather of equal index shards, grouped send / recv of byte-balanced
    shards).  Index shards against the golden bits, byte shards (variable-length
    preimages) against the oracle, both with and without the gather.  Needs
    two or more GPUs; skips on a one-GPU box (the [rccl1] variants of the tests
    above run the same code with one device)."""
    from stellard_amd import _native as N
    ndev = torch_cuda.cuda.device_count()
    if ndev < 2:
        pytest.skip(f"{ndev} GPU visible: the in-process multi-device gather needs >= 2")
    sig, msg, pk, exp = _golden_rows(golden, 50_000 + 37, seed=99)
    pres, psig, ppk = _preimage_corpus(oracle, 3_001, seed=98)
    pexp = oracle.tx_verify_batch(pres, psig, ppk)
    for flags in (N.STL_CFG_RCCL_GATHER, N.STL_CFG_NO_RCCL):
        with reinit(stl, flags=flags):
            assert N.load().stl_device_count() == ndev
            if flags == N.STL_CFG_RCCL_GATHER:
                assert stl.comm_info()[0] == ndev
            assert np.array_equal(stl.verify_batch(sig, msg, pk), exp), flags
            assert np.array_equal(stl.tx_verify_batch(pres, psig, ppk), pexp), flags
