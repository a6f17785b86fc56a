"""Seeded synthetic datasets of BASELINE.json configs 2-4 (test
infrastructure): the same bytes whoever builds them, because RFC 8032 signing
is deterministic and every adversarial row is a fixed function of its own
honest row -- libsodium here (tests/golden/make_digests.py, which commits
SHA-256 digests of the inputs and of libsodium's expected accept bitmaps) and
the GPU signer on the box (tests/test_gpu_digests.py, which checks libstl's
bitmaps against those digests).

  config 2   1,048,576 valid signatures, seed 0x5EED0002 (= bench.py rank 0)
  config 4   10,000,000 signatures, 2 % of the rows adversarial, split evenly
             over SURVEY.md Appendix-B classes B1-B11 (B12 is a host-side
             pre-reject), chunks of 2,000,000 with seed 0x5EED0004 + offset
  config 3   67,108,864 signatures, same construction, chunks of 4,194,304
             with seed 0x5EED0003 + chunk offset
  config 5   one ledger of 2^20 signed preimages ("STX\0" + random bytes,
             lengths log-uniform in [113, 4096]), 1,000 signers, 2 % of the
             rows made invalid after signing (a bit of the preimage, of R or
             of S), seed 0x5EED0005 (ledger_plan below)

Block digests: besides the whole-config digests, make_digests.py commits a
SHA-256 (first 16 bytes) of the inputs and of the expected bitmap of every
block of BLOCK = 65,536 rows (tests/golden/block_digests.json), so that each
rank of a sharded run can check its own slice -- ranks own whole blocks
(block_shard) -- before rank 0 checks the gathered bitmap's digest.

Row construction (per chunk): rng = default_rng(seed); seeds = 32 random
bytes per row, msgs = 32 random bytes per row; (pk, sig) = RFC 8032 keypair
and signature; rows = rng.choice(n, n * frac, replace=False) get classes
1 + (i mod 11) in that order and params = rng.integers(0, 2^32) each; row i
of class c is then rebuilt from its own honest row by mutate() below (the
device builds the same rows: stl_kernels.hip adversarial_row,
stl_debug_sign_adversarial_device).  Every adversarial row is therefore
distinct (its own key, message and signature).
"""
import hashlib
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))

CONFIGS = {
    "config2": {"n": 1 << 20, "chunk": 1 << 20, "seed": 0x5EED0002, "frac": 0.0},
    "config4": {"n": 10_000_000, "chunk": 2_000_000, "seed": 0x5EED0004, "frac": 0.02},
    "config3": {"n": 1 << 26, "chunk": 1 << 22, "seed": 0x5EED0003, "frac": 0.02},
}

DIGESTS = os.path.join(ROOT, "tests", "golden", "bitmap_digests.json")
BLOCK_DIGESTS = os.path.join(ROOT, "tests", "golden", "block_digests.json")
BLOCK = 1 << 16
CONFIG5 = {"n": 1 << 20, "seed": 0x5EED0005, "signers": 1000, "frac": 0.02, "len_min": 113, "len_max": 4096}

CLASSES = ["valid", "B1_msg_bit", "B2_R_bit", "B3_S_bit", "B4_S_plus_L", "B5_S_top_bits", "B6_small_order_pk",
           "B7_small_order_R", "B8_mixed_order_pk", "B9_noncanonical_pk", "B10_pk_not_on_curve",
           "B11_noncanonical_R"]
NCLASSES = len(CLASSES) - 1


def _ed():
    # the pure-Python restatement is only needed to build rows on the host
    # (make_digests.py, the CPU tests); the bench builds them on the device
    import ed25519_py
    return ed25519_py


def _small_order_encodings():
    """The 14 encodings of points of order dividing 8 (both sign bits, y = p
    and p + 1), sorted -- kSmallOrderEnc on the device."""
    ed = _ed()
    tors, _ = ed.torsion_points()
    so = set()
    for t in tors:
        e = ed.encode(t)
        so.add(e)
        so.add(bytes(e[:31]) + bytes([e[31] ^ 0x80]))
    so.update(ed.SMALL_ORDER_BLOCKLIST)
    so.add(bytes(ed.SMALL_ORDER_BLOCKLIST[5][:31]) + bytes([0xFF]))
    so.add(bytes(ed.SMALL_ORDER_BLOCKLIST[6][:31]) + bytes([0xFF]))
    return sorted(so)


_CONST = {}


def _const(name):
    if not _CONST:
        ed = _ed()
        _CONST["SMALL_ORDER"] = _small_order_encodings()
        _CONST["TORSION"] = [ed.encode(t) for t in ed.torsion_points()[0]]  # i * T8, kTorsionEnc
    return _CONST[name]


NONCANON_R = [bytes.fromhex(h) for h in ("ee" + "ff" * 30 + "7f", "01" + "00" * 30 + "80", "ee" + "ff" * 30 + "ff")]
S_TOP = (0xE0, 0x80, 0x40, 0x20)


def _k_times_a(R, A, M, a):
    ed = _ed()
    return (ed.sha512_int(R, A, M) % ed.L) * a % ed.L


def mutate_row(c, u, seed, A, sig, M, group):
    """Class-c mutation with parameter u of one honest row (bytes) -> (A, sig,
    M).  group: (scalarmult_base(S) -> 32 B, point_add(P, Q) -> 32 B)."""
    ed = _ed()
    SMALL_ORDER, TORSION = _const("SMALL_ORDER"), _const("TORSION")
    R, S = bytearray(sig[:32]), bytearray(sig[32:])
    A, M = bytearray(A), bytearray(M)
    byte, bit = u % 32, 1 << ((u >> 5) & 7)
    if c == 1:
        M[byte] ^= bit
    elif c == 2:
        R[byte] ^= bit
    elif c == 3:
        s = int.from_bytes(S, "little")
        b0 = u % 252
        for i in range(252):
            b = (b0 - i) % 252
            if (s >> b) & 1:
                s &= ~(1 << b)
                break
        S = bytearray(s.to_bytes(32, "little"))
    elif c == 4:
        S = bytearray((int.from_bytes(S, "little") + ed.L).to_bytes(32, "little"))
    elif c == 5:
        S[31] |= S_TOP[u % 4]
    elif c == 6:
        A = bytearray(SMALL_ORDER[u % 14])
        R = bytearray(group[0](bytes(S)))
    elif c in (7, 11):
        if c == 11 and u % 2 == 0:
            R[31] ^= 0x80
        else:
            R = bytearray(SMALL_ORDER[u % 14] if c == 7 else NONCANON_R[(u >> 1) % 3])
            a, _ = ed.secret_scalar(seed)
            S = bytearray(_k_times_a(bytes(R), bytes(A), bytes(M), a).to_bytes(32, "little"))
    elif c == 8:
        A = bytearray(group[1](bytes(A), TORSION[1 + u % 7]))
        a, prefix = ed.secret_scalar(seed)
        r = ed.sha512_int(prefix, bytes(M)) % ed.L  # R is the honest [r]B
        S = bytearray(((r + ed.sha512_int(bytes(R), bytes(A), bytes(M)) % ed.L * a) % ed.L).to_bytes(32, "little"))
    elif c == 9:
        y = ed.P + 2 + u % 17
        A = bytearray((y | (((u >> 8) & 1) << 255)).to_bytes(32, "little"))
    elif c == 10:
        v = int.from_bytes(A, "little")
        sign, y = v >> 255, v & ((1 << 255) - 1)
        for j in range(1, 65):
            if y + j < ed.P and ed.recover_x(y + j, sign) is None:
                A = bytearray(((y + j) | (sign << 255)).to_bytes(32, "little"))
                break
    return bytes(A), bytes(R) + bytes(S), bytes(M)


def python_group():
    """Group operations in pure Python (slow; for small cross-checks)."""
    ed = _ed()
    return (lambda S: ed.encode(ed.mul(int.from_bytes(S, "little"), ed.B)),
            lambda P, Q: ed.encode(ed.add(ed.decode(P), ed.decode(Q))))


def sodium_group(lib):
    """Group operations through libsodium (oracle/_ref/libsodium_ref.so)."""
    import ctypes

    def smul(S):
        out = ctypes.create_string_buffer(32)
        assert lib.ref_scalarmult_base_noclamp(out, S) == 0
        return out.raw

    def padd(P, Q):
        out = ctypes.create_string_buffer(32)
        assert lib.ref_point_add(out, P, Q) == 0
        return out.raw

    return smul, padd


def mutate(seeds, msgs, pk, sig, cls, param, group):
    """Apply the class mutations in place to the rows with cls > 0 (uint8
    arrays as built by chunk())."""
    for i in np.nonzero(cls)[0]:
        A, s, M = mutate_row(int(cls[i]), int(param[i]), bytes(seeds[i]), bytes(pk[i]), bytes(sig[i]),
                             bytes(msgs[i]), group)
        pk[i] = np.frombuffer(A, np.uint8)
        sig[i] = np.frombuffer(s, np.uint8)
        msgs[i] = np.frombuffer(M, np.uint8)


def chunk_plan(seed, n, frac):
    """(seeds, msgs, cls, param) of one chunk: the honest rows' inputs and the
    adversarial class / parameter of every row (0 = honest)."""
    rng = np.random.default_rng(seed)
    seeds = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    msgs = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    cls = np.zeros(n, np.uint8)
    param = np.zeros(n, np.uint32)
    if frac > 0:
        rows = rng.choice(n, int(n * frac), replace=False)
        cls[rows] = 1 + np.arange(rows.size) % NCLASSES
        param[rows] = rng.integers(0, 1 << 32, rows.size, dtype=np.uint64).astype(np.uint32)
    return seeds, msgs, cls, param


def class_counts(cls):
    return {CLASSES[c]: int((cls == c).sum()) for c in range(1, NCLASSES + 1) if (cls == c).any()}


def chunk(seed, n, frac, make):
    """One chunk: (sig, msg, pk, cls).  make(seeds, msgs, cls, param) ->
    (pk, sig, msg) uint8 arrays: the honest rows with the mutations applied."""
    seeds, msgs, cls, param = chunk_plan(seed, n, frac)
    pk, sig, msg = make(seeds, msgs, cls, param)
    return (np.ascontiguousarray(sig, np.uint8), np.ascontiguousarray(msg, np.uint8),
            np.ascontiguousarray(pk, np.uint8), cls)


def chunks(name):
    c = CONFIGS[name]
    for c0 in range(0, c["n"], c["chunk"]):
        yield c0, c["seed"] + (c0 if c["frac"] > 0 else 0), min(c["chunk"], c["n"] - c0), c["frac"]


def row_keys(sig, msg, pk):
    """A 16-byte key per row (first half of SHA-256 of its 128 bytes), for
    counting distinct rows."""
    rows = np.concatenate([sig, msg, pk], axis=1)
    return np.array([hashlib.sha256(r.tobytes()).digest()[:16] for r in rows])


class Digest:
    """Running SHA-256 of the packed accept bitmap (LSB first, chunk after
    chunk -- every chunk is a multiple of 8 rows) and of the input rows."""

    def __init__(self):
        self.bits = hashlib.sha256()
        self.inputs = hashlib.sha256()
        self.rows = 0
        self.accepted = 0

    def add(self, sig, msg, pk, bits):
        assert bits.shape[0] % 8 == 0 or self.rows == 0
        self.inputs.update(np.ascontiguousarray(sig).tobytes())
        self.inputs.update(np.ascontiguousarray(msg).tobytes())
        self.inputs.update(np.ascontiguousarray(pk).tobytes())
        self.bits.update(np.packbits(np.asarray(bits, bool), bitorder="little").tobytes())
        self.rows += bits.shape[0]
        self.accepted += int(np.count_nonzero(bits))

    def result(self):
        return {"rows": self.rows, "accepted": self.accepted, "bitmap_sha256": self.bits.hexdigest(),
                "inputs_sha256": self.inputs.hexdigest()}


# ---------------------------------------------------------------- blocks
def h16(*arrays):
    """First 16 bytes (hex) of SHA-256 over the arrays' bytes, in order."""
    h = hashlib.sha256()
    for a in arrays:
        h.update(np.ascontiguousarray(a).tobytes())
    return h.hexdigest()[:32]


class BlockDigest:
    """Per-BLOCK digests of a row stream fed chunk by chunk (chunks need not
    be block aligned): inputs = h16(sig, msg, pk of the block's rows), bitmap =
    h16(packbits of the block's accept bits, LSB first)."""

    def __init__(self):
        self.inputs, self.bitmap = [], []
        self._rows = []  # pending (sig, msg, pk, bits) pieces of the current block
        self._n = 0

    def add(self, sig, msg, pk, bits):
        i = 0
        n = bits.shape[0]
        while i < n:
            take = min(BLOCK - self._n, n - i)
            self._rows.append((sig[i:i + take], msg[i:i + take], pk[i:i + take], bits[i:i + take]))
            self._n += take
            i += take
            if self._n == BLOCK:
                self._emit()

    def _emit(self):
        if not self._n:
            return
        parts = list(zip(*self._rows))
        sig, msg, pk, bits = (np.concatenate(p) for p in parts)
        self.inputs.append(h16(sig, msg, pk))
        self.bitmap.append(h16(np.packbits(np.asarray(bits, bool), bitorder="little")))
        self._rows, self._n = [], 0

    def result(self):
        self._emit()
        return {"block_rows": BLOCK, "inputs_h16": self.inputs, "bitmap_h16": self.bitmap}


def block_shard(n, rank, world):
    """Rows [lo, hi) of rank `rank` of `world` when ranks own whole BLOCKs,
    as evenly as blocks allow (the last block may be partial): block range
    [rank*B // world, (rank+1)*B // world) of B = ceil(n / BLOCK) blocks."""
    nb = -(-n // BLOCK)
    b0, b1 = rank * nb // world, (rank + 1) * nb // world
    return min(n, b0 * BLOCK), min(n, b1 * BLOCK), b0, b1


def rows_plan(name, lo, hi):
    """The dataset pieces covering rows [lo, hi) of a config:
    yields (row0, seeds, msgs, cls, param) slices of the chunk plans (each
    chunk's plan is built whole -- it is one rng stream -- and cut)."""
    for c0, seed, n, frac in chunks(name):
        a, b = max(lo, c0), min(hi, c0 + n)
        if a >= b:
            continue
        seeds, msgs, cls, param = chunk_plan(seed, n, frac)
        yield a, seeds[a - c0:b - c0], msgs[a - c0:b - c0], cls[a - c0:b - c0], param[a - c0:b - c0]


# ---------------------------------------------------------------- config 5
def ledger_plan(cfg=CONFIG5):
    """One synthetic ledger: signing preimages packed
    back to back ("STX\\0" || random bytes, lengths log-uniform), the signer
    seed of every row, and the rows made invalid after signing with their
    kind (0 = a preimage bit, 1 = an R bit, 2 = an S bit) and parameter."""
    rng = np.random.default_rng(cfg["seed"])
    n = cfg["n"]
    lens = np.exp(rng.uniform(np.log(cfg["len_min"]), np.log(cfg["len_max"]), n)).astype(np.int32)
    offs = np.zeros(n, np.int64)
    offs[1:] = np.cumsum(lens[:-1], dtype=np.int64)
    total = int(offs[-1] + lens[-1])
    pre = rng.integers(0, 256, total + 16, dtype=np.uint8)  # 16 B of tail padding: the hash kernel's loads
    for j, b in enumerate(b"STX\x00"):
        pre[offs + j] = b
    signers = rng.integers(0, 256, (cfg["signers"], 32), dtype=np.uint8)
    who = rng.integers(0, cfg["signers"], n)
    bad = np.sort(rng.choice(n, int(n * cfg["frac"]), replace=False))
    kind = (np.arange(bad.size) % 3).astype(np.uint8)
    param = rng.integers(0, 1 << 32, bad.size, dtype=np.uint64)
    return {"n": n, "pre": pre, "total": total, "offs": offs, "lens": lens, "signers": signers, "who": who,
            "bad": bad, "kind": kind, "param": param}


def ledger_mutations(lp):
    """Where the invalid rows' bits flip: (preimage byte positions, xor bytes)
    and (signature rows, byte columns, xor bytes) -- applied after signing."""
    bad, kind, u = lp["bad"], lp["kind"], lp["param"]
    bit = (np.uint64(1) << ((u >> np.uint64(16)) & np.uint64(7))).astype(np.uint8)
    k0 = kind == 0
    rows0 = bad[k0]
    pos = lp["offs"][rows0] + 4 + (u[k0] % (lp["lens"][rows0] - 4).astype(np.uint64)).astype(np.int64)
    ks = ~k0
    col = (u[ks] % np.uint64(32)).astype(np.int64) + np.where(kind[ks] == 2, 32, 0)
    return (pos, bit[k0]), (bad[ks], col, bit[ks])


def ledger_input_digest(pre, total, lens, sig, pk):
    return h16(pre[:total], lens.astype("<i4"), sig, pk)
