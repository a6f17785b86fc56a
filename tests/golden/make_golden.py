#!/usr/bin/env python3
"""Generates tests/golden/ed25519_golden.npz -- the committed golden vectors.

Run here (the build container), never on the GPU box:
    python tests/golden/make_golden.py

Expected bits for the DEFAULT policy come from the container's real libsodium
1.0.18 (/opt/conda/lib/libsodium.so) through ctypes, composed exactly as
stellard composes them (RippleAddress::verifySignature,
src/ripple_data/protocol/RippleAddress.cpp:190-200):
    crypto_sign_verify_detached(sig, hash, 32, pk) == 0  &&  S < L
Expected bits for the 1.0.0 policy (the version the reference pins,
Dockerfile:9-10, not available offline) come from the independent pure-Python
restatement in ed25519_py.py and are marked UNPINNED by libsodium.

Classes follow SURVEY.md Appendix B (B12, malformed lengths, is a host-side
pre-reject and is covered by tests/test_host_protocol.py).
"""
import ctypes
import hashlib
import os
import random
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import ed25519_py as ed  # noqa: E402

OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "ed25519_golden.npz")
SODIUM = "/opt/conda/lib/libsodium.so"

CLASSES = [
    "valid", "B1_msg_bit", "B2_R_bit", "B3_S_bit", "B4_S_plus_L", "B5_S_top_bits",
    "B6_small_order_pk", "B7_small_order_R", "B8_mixed_order_pk", "B9_noncanonical_pk",
    "B10_pk_not_on_curve", "B11_noncanonical_R", "X_kat_rippleaddress", "X_boundary_S",
    "X_negated_pk", "X_random_bytes",
]


def load_sodium():
    lib = ctypes.CDLL(SODIUM)
    assert lib.sodium_init() >= 0
    lib.sodium_version_string.restype = ctypes.c_char_p
    ver = lib.sodium_version_string().decode()
    assert ver == "1.0.18", ver
    return lib, ver


def main():
    sod, ver = load_sodium()
    rng = random.Random(0x5EED0004)

    def rbytes(n):
        return bytes(rng.getrandbits(8) for _ in range(n))

    def keypair(seed):
        pk = ctypes.create_string_buffer(32)
        sk = ctypes.create_string_buffer(64)
        assert sod.crypto_sign_seed_keypair(pk, sk, seed) == 0
        return pk.raw, sk.raw

    def sign(msg, sk):
        sig = ctypes.create_string_buffer(64)
        sod.crypto_sign_detached(sig, None, msg, ctypes.c_ulonglong(len(msg)), sk)
        return sig.raw

    def sodium_accept(sig, msg, pk):
        raw = sod.crypto_sign_verify_detached(sig, msg, ctypes.c_ulonglong(len(msg)), pk) == 0
        return raw and int.from_bytes(sig[32:], "little") < ed.L

    recs = []  # (sig, msg, pk, class)

    def add(sig, msg, pk, cls):
        assert len(sig) == 64 and len(msg) == 32 and len(pk) == 32
        recs.append((sig, msg, pk, CLASSES.index(cls)))

    keys = [keypair(rbytes(32)) for _ in range(64)]

    def honest():
        pk, sk = keys[rng.randrange(len(keys))]
        msg = rbytes(32)
        return sign(msg, sk), msg, pk, sk

    # valid
    for _ in range(1024):
        sig, msg, pk, _ = honest()
        add(sig, msg, pk, "valid")
    # B1-B3 single-bit flips
    for _ in range(128):
        sig, msg, pk, _ = honest()
        m = bytearray(msg); m[rng.randrange(32)] ^= 1 << rng.randrange(8)
        add(sig, bytes(m), pk, "B1_msg_bit")
    for _ in range(128):
        sig, msg, pk, _ = honest()
        s = bytearray(sig); s[rng.randrange(32)] ^= 1 << rng.randrange(8)
        add(bytes(s), msg, pk, "B2_R_bit")
    for _ in range(128):
        sig, msg, pk, _ = honest()
        s = bytearray(sig); s[32 + rng.randrange(31)] ^= 1 << rng.randrange(8)
        if int.from_bytes(s[32:], "little") >= ed.L:
            continue
        add(bytes(s), msg, pk, "B3_S_bit")
    # B4 S+L (non-canonical S: equation still holds)
    for _ in range(96):
        sig, msg, pk, _ = honest()
        S = int.from_bytes(sig[32:], "little") + ed.L
        add(sig[:32] + S.to_bytes(32, "little"), msg, pk, "B4_S_plus_L")
    # B5 S >= 2^253 / top bits set
    for i in range(64):
        sig, msg, pk, _ = honest()
        S = bytearray(sig[32:])
        S[31] |= (0xE0, 0x80, 0x40, 0x20)[i % 4]
        add(sig[:32] + bytes(S), msg, pk, "B5_S_top_bits")
    # B6 small-order pk (8 torsion points x sign bit + non-canonical encodings)
    tors, T8 = ed.torsion_points()
    so_encodings = set()
    for t in tors:
        e = ed.encode(t)
        so_encodings.add(e)
        so_encodings.add(bytes(e[:31]) + bytes([e[31] ^ 0x80]))
    so_encodings.update(ed.SMALL_ORDER_BLOCKLIST)
    so_encodings.add(bytes(ed.SMALL_ORDER_BLOCKLIST[5][:31]) + bytes([0xFF]))  # p with sign bit
    so_encodings.add(bytes(ed.SMALL_ORDER_BLOCKLIST[6][:31]) + bytes([0xFF]))
    so_encodings = sorted(so_encodings)
    for rep in range(6):
        for enc in so_encodings:
            # R = [r]B, S = r: passes the cofactorless equation iff [k]A == O
            r = rng.randrange(1, ed.L)
            R = ed.encode(ed.mul(r, ed.B))
            msg = rbytes(32)
            add(R + r.to_bytes(32, "little"), msg, enc, "B6_small_order_pk")
    # B7 small-order R with S = k*a (so [S]B - [k]A = O)
    for rep in range(4):
        for enc in so_encodings:
            seed = rbytes(32)
            pk, _ = keypair(seed)
            a, _ = ed.secret_scalar(seed)
            msg = rbytes(32)
            k = ed.sha512_int(enc, pk, msg) % ed.L
            S = (k * a) % ed.L
            add(enc + S.to_bytes(32, "little"), msg, pk, "B7_small_order_R")
    # B8 mixed-order pk A' = A + T (T in the 8-torsion): honest-style signature
    # over A'.  Accepted (cofactorless) iff [k]T == O.
    n8 = 0
    while n8 < 192:
        seed = rbytes(32)
        a, prefix = ed.secret_scalar(seed)
        A = ed.mul(a, ed.B)
        T = tors[1 + rng.randrange(7)]
        Ap = ed.encode(ed.add(A, T))
        msg = rbytes(32)
        r = ed.sha512_int(prefix, msg) % ed.L
        R = ed.encode(ed.mul(r, ed.B))
        k = ed.sha512_int(R, Ap, msg) % ed.L
        S = (r + k * a) % ed.L
        add(R + S.to_bytes(32, "little"), msg, Ap, "B8_mixed_order_pk")
        n8 += 1
    # B9 non-canonical pk, y in [p+2, 2^255) that decodes (not small order)
    for y_off in range(2, 19):
        y = ed.P + y_off
        for sbit in (0, 1):
            enc = (y | (sbit << 255)).to_bytes(32, "little")
            sig, msg, _, _ = honest()
            add(sig, msg, enc, "B9_noncanonical_pk")
    # B10 pk not on the curve
    nb10 = 0
    while nb10 < 64:
        enc = rbytes(32)
        if ed.decode(enc) is not None:
            continue
        sig, msg, _, _ = honest()
        add(sig, msg, enc, "B10_pk_not_on_curve")
        nb10 += 1
    # B11 non-canonical / mis-signed R for a valid signature
    for _ in range(48):
        sig, msg, pk, _ = honest()
        R = bytearray(sig[:32]); R[31] ^= 0x80  # encoding of -R'
        add(bytes(R) + sig[32:], msg, pk, "B11_noncanonical_R")
    for enc_hex in ("ee" + "ff" * 30 + "7f", "01" + "00" * 30 + "80", "ee" + "ff" * 30 + "ff"):
        enc = bytes.fromhex(enc_hex)
        for _ in range(4):
            seed = rbytes(32)
            pk, _ = keypair(seed)
            a, _ = ed.secret_scalar(seed)
            msg = rbytes(32)
            k = ed.sha512_int(enc, pk, msg) % ed.L
            add(enc + ((k * a) % ed.L).to_bytes(32, "little"), msg, pk, "B11_noncanonical_R")
    # RippleAddress_test KAT (RippleAddress.cpp:812-845): masterpassphrase key,
    # all-zero uint256 message, and its S+L variant.
    seed = hashlib.sha512(b"masterpassphrase").digest()[:32]
    pk, sk = keypair(seed)
    msg = bytes(32)
    sig = sign(msg, sk)
    add(sig, msg, pk, "X_kat_rippleaddress")
    S = int.from_bytes(sig[32:], "little") + ed.L
    add(sig[:32] + S.to_bytes(32, "little"), msg, pk, "X_kat_rippleaddress")
    # S boundaries: S = L-1, L, L+1, 0, 2^253-1 with a valid R
    for Sv in (0, 1, ed.L - 1, ed.L, ed.L + 1, 2**253 - 1, 2**252):
        sig, msg, pk, _ = honest()
        add(sig[:32] + Sv.to_bytes(32, "little"), msg, pk, "X_boundary_S")
    # negated public key (sign bit flip of a valid key)
    for _ in range(32):
        sig, msg, pk, _ = honest()
        p2 = bytearray(pk); p2[31] ^= 0x80
        add(sig, msg, bytes(p2), "X_negated_pk")
    # random bytes everywhere
    for _ in range(64):
        add(rbytes(64), rbytes(32), rbytes(32), "X_random_bytes")

    n = len(recs)
    sig = np.frombuffer(b"".join(r[0] for r in recs), dtype=np.uint8).reshape(n, 64)
    msg = np.frombuffer(b"".join(r[1] for r in recs), dtype=np.uint8).reshape(n, 32)
    pk = np.frombuffer(b"".join(r[2] for r in recs), dtype=np.uint8).reshape(n, 32)
    cls = np.array([r[3] for r in recs], dtype=np.uint8)
    exp_1018 = np.array([sodium_accept(r[0], r[1], r[2]) for r in recs], dtype=np.uint8)
    exp_100 = np.array([ed.verify(r[0], r[1], r[2], "1.0.0") for r in recs], dtype=np.uint8)
    # cross-check: the independent python restatement agrees with libsodium
    py_1018 = np.array([ed.verify(r[0], r[1], r[2], "1.0.18") for r in recs], dtype=np.uint8)
    mism = int((py_1018 != exp_1018).sum())
    assert mism == 0, f"python restatement disagrees with libsodium on {mism} vectors"
    np.savez_compressed(
        OUT, sig=sig, msg=msg, pk=pk, cls=cls, expected_sodium_1_0_18=exp_1018,
        expected_stellard_1_0_0_unpinned=exp_100,
        class_names=np.array(CLASSES), sodium_version=np.array(ver))
    print(f"wrote {OUT}: {n} vectors")
    for i, c in enumerate(CLASSES):
        m = cls == i
        print(f"  {c:24s} n={int(m.sum()):5d} accept(1.0.18)={int(exp_1018[m].sum()):5d} "
              f"accept(1.0.0)={int(exp_100[m].sum()):5d}")


if __name__ == "__main__":
    main()
