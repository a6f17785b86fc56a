"""Pure-Python Ed25519 group arithmetic used ONLY to construct adversarial
golden inputs (small-order points, mixed-order keys, non-canonical encodings)
and as a second, independent restatement of the accept predicate.

Test infrastructure: never imported by the product package.

Predicates restated (libsodium is not vendored by the reference):
  * libsodium 1.0.18 crypto_sign_verify_detached (called at
    src/ripple_data/protocol/RippleAddress.cpp:196-197)
  * stellard composite verified && S<L (RippleAddress.cpp:190-200, 226-252)
  * the 1.0.0-era predicate the reference pins (Dockerfile:9-10), which is
    UNPINNED here (no libsodium 1.0.0 offline) -- SURVEY.md Appendix A.
"""
import hashlib

P = 2**255 - 19
L = 2**252 + 27742317777372353535851937790883648493
D = (-121665 * pow(121666, P - 2, P)) % P
SQRTM1 = pow(2, (P - 1) // 4, P)


def inv(x):
    return pow(x, P - 2, P)


# extended coordinates (X, Y, Z, T), x = X/Z, y = Y/Z, T = XY/Z
IDENT = (0, 1, 1, 0)


def add(p, q):
    X1, Y1, Z1, T1 = p
    X2, Y2, Z2, T2 = q
    A = (Y1 - X1) * (Y2 - X2) % P
    B = (Y1 + X1) * (Y2 + X2) % P
    C = T1 * 2 * D * T2 % P
    Dd = Z1 * 2 * Z2 % P
    E, F, G, H = B - A, Dd - C, Dd + C, B + A
    return (E * F % P, G * H % P, F * G % P, E * H % P)


def neg(p):
    X, Y, Z, T = p
    return ((-X) % P, Y, Z, (-T) % P)


def mul(k, p):
    r = IDENT
    for bit in bin(k)[2:] if k > 0 else "":
        r = add(r, r)
        if bit == "1":
            r = add(r, p)
    return r


def affine(p):
    X, Y, Z, _ = p
    zi = inv(Z)
    return X * zi % P, Y * zi % P


def encode(p):
    x, y = affine(p)
    return (y | ((x & 1) << 255)).to_bytes(32, "little")


def recover_x(y, sign):
    """Returns x (or None) for the 255-bit y taken mod p, as libsodium's
    ge25519_frombytes does: x = 0 with sign 1 is NOT rejected."""
    y %= P
    u = (y * y - 1) % P
    v = (D * y * y + 1) % P
    x = u * pow(v, 3, P) * pow(u * pow(v, 7, P), (P - 5) // 8, P) % P
    vxx = v * x * x % P
    if vxx != u % P:
        if vxx != (-u) % P:
            return None
        x = x * SQRTM1 % P
    if (x & 1) != sign:
        x = (-x) % P
    return x


def decode(s):
    """Point for a 32-byte encoding (non-canonical y reduced mod p), or None."""
    v = int.from_bytes(s, "little")
    y = v & ((1 << 255) - 1)
    sign = v >> 255
    x = recover_x(y, sign)
    if x is None:
        return None
    y %= P
    return (x, y, 1, x * y % P)


GY = 4 * inv(5) % P
B = (recover_x(GY, 0), GY, 1, recover_x(GY, 0) * GY % P)


def eq(p, q):
    X1, Y1, Z1, _ = p
    X2, Y2, Z2, _ = q
    return (X1 * Z2 - X2 * Z1) % P == 0 and (Y1 * Z2 - Y2 * Z1) % P == 0


def sha512_int(*parts):
    h = hashlib.sha512()
    for p in parts:
        h.update(p)
    return int.from_bytes(h.digest(), "little")


def secret_scalar(seed):
    h = bytearray(hashlib.sha512(seed).digest())
    h[0] &= 248
    h[31] &= 127
    h[31] |= 64
    return int.from_bytes(bytes(h[:32]), "little"), bytes(h[32:])


SMALL_ORDER_BLOCKLIST = [
    bytes(32),
    bytes([1]) + bytes(31),
    bytes.fromhex("26e8958fc2b227b045c3f489f2ef98f0d5dfac05d3c63339b13802886d53fc05"),
    bytes.fromhex("c7176a703d4dd84fba3c0b760d10670f2a2053fa2c39ccc64ec7fd7792ac037a"),
    (P - 1).to_bytes(32, "little"),
    P.to_bytes(32, "little"),
    (P + 1).to_bytes(32, "little"),
]


def has_small_order(s):
    for bl in SMALL_ORDER_BLOCKLIST:
        if s[:31] == bl[:31] and (s[31] & 0x7F) == bl[31]:
            return True
    return False


def is_canonical_point(s):
    return (int.from_bytes(s, "little") & ((1 << 255) - 1)) < P


def verify(sig, msg, pk, policy="1.0.18"):
    """Independent restatement of the composite accept predicate."""
    R, Sb = sig[:32], sig[32:]
    S = int.from_bytes(Sb, "little")
    if policy == "1.0.18":
        if S >= L or has_small_order(R) or not is_canonical_point(pk) or has_small_order(pk):
            return False
    else:
        # 1.0.0: only the top 3 bits of S; the all-zero key is rejected too (as
        # some 1.0.x releases did; unpinned offline, the conservative side)
        if sig[63] & 0xE0 or bytes(pk) == bytes(32):
            return False
    A = decode(pk)
    if A is None:
        return False
    k = sha512_int(R, pk, msg) % L
    Rp = add(mul(S, B), neg(mul(k, A)))
    ok = encode(Rp) == R
    return ok and S < L  # stellard's crypto_sign_check_S_lt_l


def torsion_points():
    """The 8 points of order dividing 8, as extended points."""
    T8 = decode(SMALL_ORDER_BLOCKLIST[2])
    pts = []
    p = IDENT
    for _ in range(8):
        pts.append(p)
        p = add(p, T8)
    return pts, T8
