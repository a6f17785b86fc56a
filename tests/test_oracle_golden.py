"""Pin the CPU oracle (oracle/stl_oracle.c) before trusting it:
  * every committed golden vector (expected bits from libsodium 1.0.18, both
    policies -- 1.0.0 bits come from the independent pure-Python restatement),
  * the RippleAddress_test known answers (RippleAddress.cpp:812-845),
  * live differential runs against the reference call path over libsodium
    (oracle/_ref/libsodium_ref.so) where libsodium exists.
"""
import hashlib

import numpy as np
import pytest

from tests import oracle_bind

ALPHABET = b"gsphnaf39wBUDNEGHJKLM4PQRST7VWXYZ2bcdeCr65jkm8oFqi1tuvAxyz"  # Base58.cpp:43-49
L = 2**252 + 27742317777372353535851937790883648493


def b58check(payload):
    data = payload + hashlib.sha256(hashlib.sha256(payload).digest()).digest()[:4]
    n = int.from_bytes(data, "big")
    s = b""
    while n:
        n, r = divmod(n, 58)
        s = ALPHABET[r:r + 1] + s
    pad = len(data) - len(data.lstrip(b"\0"))
    return (ALPHABET[:1] * pad + s).decode()


@pytest.mark.parametrize("policy,key", [(0, "expected_sodium_1_0_18"), (1, "expected_stellard_1_0_0_unpinned")])
def test_oracle_matches_golden(oracle, golden, policy, key):
    got = oracle.verify_batch(golden["sig"], golden["msg"], golden["pk"], policy=policy)
    assert np.array_equal(got, golden[key].astype(bool))


def test_golden_covers_every_class(golden):
    exp = golden["expected_sodium_1_0_18"]
    names = [str(x) for x in golden["class_names"]]
    counts = {names[c]: int((golden["cls"] == c).sum()) for c in range(len(names))}
    assert all(v > 0 for v in counts.values()), counts
    assert exp.sum() > 1000 and (exp == 0).sum() > 900
    assert str(golden["sodium_version"]) == "1.0.18"


def test_rippleaddress_kat(oracle):
    """RippleAddress_test: "masterpassphrase" -> seed/public keys (RippleAddress.cpp:812-826),
    sign/verify of the zero uint256 (:829-836), S+L rejected by the composite (:838-845)."""
    seed = hashlib.sha512(b"masterpassphrase").digest()[:32]  # StellarPrivateKey::fromPassPhrase
    assert b58check(bytes([33]) + seed) == "s3q5ZGX2ScQK2rJ4JATp7rND6X5npG3De8jMbB7tuvm2HAVHcCN"
    pk, sk = oracle.keypair(seed)
    assert b58check(bytes([67]) + pk) == "pGreoXKYybde1keKZwDCv8m5V1kT6JH37pgnTUVzdMkdygTixG8"
    assert b58check(bytes([122]) + pk) == "nfbbWHgJqzqfH1cfRpMdPRkJ19cxTsdHkBtz1SLJJQfyf9Ax6vd"
    msg = bytes(32)
    sig = oracle.sign(msg, sk)
    assert oracle.verify(sig, msg, pk)
    S = int.from_bytes(sig[32:], "little") + L
    nc = sig[:32] + S.to_bytes(32, "little")
    assert not oracle.verify(nc, msg, pk, policy=0)
    assert not oracle.verify(nc, msg, pk, policy=1)
    # the bare libsodium call on the S+L signature (RippleAddress.cpp:841-844):
    # the reference expects it to VERIFY -- true of the 1.0.0 predicate it pins
    # (Dockerfile:9-10), false of 1.0.18, which rejects S >= L itself
    assert oracle.verify_raw(nc, msg, pk, policy=1)
    assert not oracle.verify_raw(nc, msg, pk, policy=0)
    assert oracle.verify_raw(sig, msg, pk, policy=0) and oracle.verify_raw(sig, msg, pk, policy=1)
    ref = oracle_bind.load_sodium_ref()
    if ref is not None:  # the container's libsodium 1.0.18 itself
        assert ref.ref_crypto_sign_verify_detached(nc, msg, 32, pk) == -1
        assert ref.ref_crypto_sign_verify_detached(sig, msg, 32, pk) == 0
    # the device verify code compiled for the host, in raw mode (core policy bit 1)
    emu = oracle_bind.load_hostemu()
    rows = [np.frombuffer(x, np.uint8).reshape(1, -1) for x in (nc, msg, pk)]
    for pol, want in ((1 | 2, 1), (1, 0), (0 | 2, 0), (0, 0)):
        bm = np.zeros(1, np.uint8)
        emu.hostemu_verify_batch(*[oracle_bind._buf(np.ascontiguousarray(r)) for r in rows], 1,
                                 oracle_bind._buf(bm), pol)
        assert int(bm[0] & 1) == want, (pol, bm)


def test_oracle_sha512(oracle):
    rng = np.random.default_rng(3)
    for ln in (0, 1, 111, 112, 113, 127, 128, 129, 255, 1000, 4096):
        d = rng.bytes(ln)
        assert oracle.sha512(d) == hashlib.sha512(d).digest()


def test_oracle_vs_libsodium_random():
    ref = oracle_bind.load_sodium_ref()
    if ref is None:
        pytest.skip("libsodium not present")
    o = oracle_bind.load_oracle()
    rng = np.random.default_rng(17)
    n = 3000
    seeds = rng.integers(0, 256, (n, 32), np.uint8)
    msgs = rng.integers(0, 256, (n, 32), np.uint8)
    sig = np.zeros((n, 64), np.uint8)
    pk = np.zeros((n, 32), np.uint8)
    for i in range(n):
        p, sk = o.keypair(seeds[i].tobytes())
        pk[i] = np.frombuffer(p, np.uint8)
        sig[i] = np.frombuffer(o.sign(msgs[i].tobytes(), sk), np.uint8)
    flip = rng.random(n) < 0.4
    for i in np.nonzero(flip)[0]:
        which = rng.integers(3)
        if which == 0:
            sig[i, rng.integers(64)] ^= 1 << rng.integers(8)
        elif which == 1:
            msgs[i, rng.integers(32)] ^= 1 << rng.integers(8)
        else:
            pk[i, rng.integers(32)] ^= 1 << rng.integers(8)
    a = o.verify_batch(sig, msgs, pk, threads=8)
    b = oracle_bind.sodium_verify_batch(ref, sig, msgs, pk, threads=8)
    assert np.array_equal(a, b)
    assert a.sum() >= (~flip).sum()


def test_signatures_match_libsodium():
    ref = oracle_bind.load_sodium_ref()
    if ref is None:
        pytest.skip("libsodium not present")
    import ctypes
    o = oracle_bind.load_oracle()
    rng = np.random.default_rng(23)
    for _ in range(50):
        seed = rng.bytes(32)
        msg = rng.bytes(int(rng.integers(0, 200)))
        p1, s1 = o.keypair(seed)
        pk = ctypes.create_string_buffer(32)
        sk = ctypes.create_string_buffer(64)
        ref.ref_seed_keypair(pk, sk, seed)
        assert pk.raw == p1
        sig = ctypes.create_string_buffer(64)
        ref.ref_sign_detached(sig, msg, len(msg), sk)
        assert sig.raw == o.sign(msg, s1)


def test_work_model_op_counts(oracle):
    """bench.py's frozen work model against the oracle's
    own field-operation counts: a verify averages N_M = 1,520 multiplications
    and N_S = 1,525 squarings (ref10 sliding-window double-scalar multiply +
    one decompression + the final inversion), and one decompression
    (ge_frombytes_negate_vartime, the per-kernel split's DECODE_OPS) is 19 M +
    255 S, plus the conditional sqrt(-1) multiplication."""
    import ctypes
    import bench
    lib = oracle.lib
    lib.oracle_op_counts.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    lib.oracle_decode_op_counts.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
    lib.oracle_decode_op_counts.restype = ctypes.c_int
    rng = np.random.default_rng(5)
    m, s = ctypes.c_uint64(0), ctypes.c_uint64(0)
    muls, sqs, dec = [], [], set()
    for _ in range(64):
        pk, sk = oracle.keypair(rng.bytes(32))
        msg = rng.bytes(32)
        assert oracle.verify(oracle.sign(msg, sk), msg, pk)
        lib.oracle_op_counts(ctypes.byref(m), ctypes.byref(s))
        muls.append(m.value)
        sqs.append(s.value)
        assert lib.oracle_decode_op_counts(pk, ctypes.byref(m), ctypes.byref(s)) == 0
        dec.add((m.value, s.value))
    assert abs(np.mean(muls) - 1520) < 0.02 * 1520 and abs(np.mean(sqs) - 1525) < 0.02 * 1525
    assert dec <= {(19, 255), (20, 255)} and (19, 255) in dec
    assert bench.DECODE_OPS == 64 * 19 + 36 * 255
    assert bench.W_PREP + bench.W_MAIN == bench.W_VERIFY == 64 * 1520 + 36 * 1525 + 5520
