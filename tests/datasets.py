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


# ---------------------------------------------------------------- config 5, serialized blobs
# One ledger of serialized Payment transactions: what a ledger
# close feeds checkSign -- each transaction rebuilt from its SHAMap item's
# bytes (/root/reference/src/ripple_app/consensus/LedgerConsensus.cpp:1947-1958
# -> SerializedTransaction.cpp:65-92, checkSign at :220-230).  Every blob is in
# canonical STObject::add order (SerializeDeclarations.h field codes):
#
#   TransactionType 12 0000 | Flags 22 80000000 | Sequence 24 .. | [DestinationTag 2E ..]
#   | Amount 61 (native 40 00 00 + 5 B, or IOU: head + "USD" currency + issuer)
#   | Fee 68 40..0A | SigningPubKey 73 20 <pk> | TxnSignature 74 40 <R||S>
#   | Account 81 14 <20 B> | Destination 83 14 <20 B>
#   | [Memos F9 { Memo EA { MemoData 7D VL <bytes> } E1 } F1]
#
# lengths log-uniform in [len_min, len_max] reached with the memo (a bare
# Payment is 175-220 B, so rows drawn shorter stay bare), 1,000 signers.  2 %
# of the rows are made invalid, five kinds in turn:
#   0 payload_bit     a Destination bit flipped after signing   -> reject (status OK)
#   1 R_bit / 2 S_bit a signature bit flipped after signing     -> reject (status OK)
#   3 deferred_order  Flags and Sequence swapped after signing: the reference
#                     re-serialises them in order, so its checkSign accepts;
#                     the device cannot prove the form canonical -> DEFERRED
#   4 malformed_pk33  a 33-byte SigningPubKey (signed over its own preimage)
#                     -> checkSign false (RippleAddress.cpp:192-194), MALFORMED
CONFIG5B = {"n": 1 << 20, "seed": 0x5EED0006, "signers": 1000, "frac": 0.02, "len_min": 100, "len_max": 4096,
            "iou": 0.2, "tag": 0.5}
BLOB_KINDS = ("payload_bit", "R_bit", "S_bit", "deferred_order", "malformed_pk33")


def _put(buf, pos, data):
    """buf[pos + j] = data[j] for a constant byte string, every row."""
    for j, b in enumerate(data):
        buf[pos + j] = b


def _put_rows(buf, pos, rows):
    """buf[pos[i] + j] = rows[i, j] (rows: (m, k) uint8), column by column."""
    for j in range(rows.shape[1]):
        buf[pos + j] = rows[:, j]


def account_ids(pks):
    """Synthetic 20-byte account ids of the signers (tests/txblob.py
    account_id: SHA-256(pk)[:20])."""
    return np.frombuffer(b"".join(hashlib.sha256(bytes(p)).digest()[:20] for p in pks), np.uint8).reshape(-1, 20)


def blob_ledger_plan(signer_pks, cfg=CONFIG5B):
    """The unsigned ledger: blob bytes with a zeroed TxnSignature slot, the
    row layout and the invalid rows.  signer_pks(seeds (s,32)) -> (s,32): the
    RFC 8032 public keys of the signer seeds (the device signer on the box,
    libsodium here -- the same bytes)."""
    rng = np.random.default_rng(cfg["seed"])
    n = cfg["n"]
    seeds = rng.integers(0, 256, (cfg["signers"], 32), dtype=np.uint8)
    who = rng.integers(0, cfg["signers"], n)
    target = np.exp(rng.uniform(np.log(cfg["len_min"]), np.log(cfg["len_max"]), n)).astype(np.int64)
    tag = rng.random(n) < cfg["tag"]
    iou = rng.random(n) < cfg["iou"]
    ni = int(iou.sum())
    mant = rng.integers(10 ** 15, 10 ** 16, ni, dtype=np.uint64)
    expo = rng.integers(-96, 81, ni).astype(np.int64)
    bad = np.sort(rng.choice(n, int(n * cfg["frac"]), replace=False))
    kind = (np.arange(bad.size) % len(BLOB_KINDS)).astype(np.uint8)
    param = rng.integers(0, 1 << 32, bad.size, dtype=np.uint64)
    pk_len = np.full(n, 32, np.int64)
    pk_len[bad[kind == 4]] = 33
    p_amt = 13 + 5 * tag.astype(np.int64)
    p_fee = p_amt + np.where(iou, 49, 9)
    p_pk = p_fee + 9
    p_sig = p_pk + 2 + pk_len
    p_acc = p_sig + 66
    p_dst = p_acc + 22
    p_memo = p_dst + 22
    extra = target - p_memo
    mb = np.where(extra >= 7, np.where(extra - 6 <= 192, extra - 6, np.maximum(extra - 7, 193)), 0)
    vlb = np.where(mb == 0, 0, np.where(mb <= 192, 1, 2))
    lens = p_memo + np.where(mb > 0, 5 + vlb + mb, 0)
    offs = np.zeros(n, np.int64)
    offs[1:] = np.cumsum(lens[:-1])
    total = int(offs[-1] + lens[-1])
    buf = rng.integers(0, 256, total + 16, dtype=np.uint8)  # value bytes; 16 B tail: the kernels' loads
    pks = np.ascontiguousarray(signer_pks(seeds), np.uint8)
    o = offs
    _put(buf, o, b"\x12\x00\x00\x22\x80\x00\x00\x00\x24")
    _put(buf, o[tag] + 13, b"\x2e")
    _put(buf, o + p_amt, b"\x61")
    nat = ~iou
    _put(buf, o[nat] + p_amt[nat] + 1, b"\x40\x00\x00")
    head = mant | ((expo + 512 + 256 + 97).astype(np.uint64) << np.uint64(54))
    _put_rows(buf, o[iou] + p_amt[iou] + 1, head.astype(">u8").view(np.uint8).reshape(-1, 8))
    _put(buf, o[iou] + p_amt[iou] + 9, b"\0" * 12 + b"USD" + b"\0" * 5)
    _put(buf, o + p_fee, b"\x68\x40\x00\x00\x00\x00\x00\x00\x0a")
    _put(buf, o + p_pk, b"\x73")
    buf[o + p_pk + 1] = pk_len.astype(np.uint8)
    _put_rows(buf, o + p_pk + 2, pks[who])
    _put(buf, o + p_sig, b"\x74\x40")
    _put_rows(buf, o + p_sig + 2, np.zeros((n, 64), np.uint8))
    _put(buf, o + p_acc, b"\x81\x14")
    _put_rows(buf, o + p_acc + 2, account_ids(pks)[who])
    _put(buf, o + p_dst, b"\x83\x14")
    m = mb > 0
    pm = o[m] + p_memo[m]
    _put(buf, pm, b"\xf9\xea\x7d")
    one, two = vlb[m] == 1, vlb[m] == 2
    buf[pm[one] + 3] = mb[m][one].astype(np.uint8)
    v = mb[m][two] - 193
    buf[pm[two] + 3] = (193 + (v >> 8)).astype(np.uint8)
    buf[pm[two] + 4] = (v & 0xFF).astype(np.uint8)
    end = pm + 3 + vlb[m] + mb[m]
    _put(buf, end, b"\xe1\xf1")
    return {"n": n, "buf": buf, "total": total, "offs": offs, "lens": lens.astype(np.int32), "seeds": seeds,
            "who": who, "pks": pks, "p_sig": p_sig, "p_dst": p_dst, "bad": bad, "kind": kind, "param": param}


def blob_signing_hashes(bp, rows=None):
    """SHA512Half("STX\\0" || blob minus its TxnSignature field) of every row
    (or of `rows`): the signing hash the reference computes for a canonical
    blob (SerializedTransaction::getSigningHash -> STObject::getSigningHash,
    SerializedObject.cpp:444-450, HashPrefix.cpp:30), hashed on the host with
    hashlib -- independent of the device's splice."""
    mv = memoryview(bp["buf"])
    offs, lens, ps = bp["offs"], bp["lens"], bp["p_sig"]
    idx = range(bp["n"]) if rows is None else rows
    out = bytearray()
    for i in idx:
        o, s = int(offs[i]), int(ps[i])
        h = hashlib.sha512(b"STX\x00")
        h.update(mv[o:o + s])
        h.update(mv[o + s + 66:o + int(lens[i])])
        out += h.digest()[:32]
    return np.frombuffer(out, np.uint8).reshape(-1, 32)  # a writable view of the bytearray


def blob_ledger_finish(bp, sig):
    """Write every row's signature into its TxnSignature slot, then make the
    invalid rows (BLOB_KINDS 0-3; kind 4 is in the layout) -- in place."""
    buf, o = bp["buf"], bp["offs"]
    _put_rows(buf, o + bp["p_sig"] + 2, np.ascontiguousarray(sig, np.uint8))
    bad, kind, u = bp["bad"], bp["kind"], bp["param"]
    bit = (np.uint64(1) << ((u >> np.uint64(16)) & np.uint64(7))).astype(np.uint8)
    r = bad
    at = {0: o[r] + bp["p_dst"][r] + 2 + (u % np.uint64(20)).astype(np.int64),
          1: o[r] + bp["p_sig"][r] + 2 + (u % np.uint64(32)).astype(np.int64),
          2: o[r] + bp["p_sig"][r] + 34 + (u % np.uint64(32)).astype(np.int64)}
    for k, pos in at.items():
        sel = kind == k
        buf[pos[sel]] ^= bit[sel]
    sw = o[bad[kind == 3]]
    a = [buf[sw + 3 + j].copy() for j in range(5)]
    for j in range(5):
        buf[sw + 3 + j] = buf[sw + 8 + j]
        buf[sw + 8 + j] = a[j]
    return bp


def blob_ledger_inputs_h16(bp):
    return h16(bp["buf"][:bp["total"]], bp["lens"].astype("<i4"))


def blob_expected_status(bp):
    """Per-row status the device contract gives this ledger by construction:
    OK, DEFERRED (kind 3) or MALFORMED (kind 4).  make_digests.py checks it
    against the reference re-serialiser (oracle/stl_oracle_tx.c) row by row."""
    st = np.zeros(bp["n"], np.uint8)
    st[bp["bad"][bp["kind"] == 3]] = 1
    st[bp["bad"][bp["kind"] == 4]] = 2
    return st


def blob_ledger_cpu(oracle, n, frac=0.05, seed=0x5EED0007):
    """A small blob ledger of the same construction, keys and signatures from
    the CPU oracle (tests: construction and status checks on the host, the
    config-5-size parity test on the GPU).  -> (plan, list of blob bytes)."""
    sks = []

    def pks(seeds):
        out = []
        for s in seeds:
            pk, sk = oracle.keypair(bytes(s))
            out.append(np.frombuffer(pk, np.uint8))
            sks.append(sk)
        return np.array(out)
    bp = blob_ledger_plan(pks, dict(CONFIG5B, n=n, frac=frac, seed=seed))
    msgs = blob_signing_hashes(bp)
    sig = np.array([np.frombuffer(oracle.sign(bytes(msgs[i]), sks[w]), np.uint8) for i, w in enumerate(bp["who"])])
    blob_ledger_finish(bp, sig)
    buf, offs, lens = bp["buf"], bp["offs"], bp["lens"]
    return bp, [bytes(buf[int(o):int(o) + int(ln)]) for o, ln in zip(offs, lens)]


# ---- configs[0]: 100k Payment blobs ----------------------
# bench.py's config-1 leg construction (tools/payments.py: seed 0x5EED0001,
# 1,000 accounts, ~175-220-byte Payment transactions, every account signing in
# turn), plus 2 % invalid rows of the BLOB_KINDS, drawn from a second seeded
# generator so the valid rows are the bench leg's:
#   0 payload_bit     a Destination bit flipped after signing    -> reject
#   1 R_bit / 2 S_bit a signature bit flipped after signing      -> reject
#   3 deferred_order  Flags and Sequence swapped after signing   -> DEFERRED
#                     (the reference re-serialises and accepts)
#   4 malformed_pk33  a 33-byte SigningPubKey, signed over its own preimage
#                     -> checkSign false (RippleAddress.cpp:192-194), MALFORMED
CONFIG1 = {"n": 100_000, "seed": 0x5EED0001, "accounts": 1000, "frac": 0.02, "bad_seed": 0x5EED0B01}


def config1_plan(signer_pks, cfg=CONFIG1):
    """The unsigned configs[0] set: signing preimages ('STX\\0' || fields)
    with the malformed rows' 33-byte keys already in, each row's signer, the
    invalid rows.  signer_pks(seeds (a,32)) -> (a,32) public keys (the device
    signer on the box, libsodium here -- the same bytes)."""
    from tools.payments import payment_preimages
    rng = np.random.default_rng(cfg["seed"])
    nacc, n = cfg["accounts"], cfg["n"]
    seeds = rng.integers(0, 256, (nacc, 32), dtype=np.uint8)
    pks = np.ascontiguousarray(signer_pks(seeds), np.uint8)
    pre = payment_preimages(pks, n, rng)
    who = np.arange(n) % nacc
    r2 = np.random.default_rng(cfg["bad_seed"])
    bad = np.sort(r2.choice(n, int(n * cfg["frac"]), replace=False))
    kind = (np.arange(bad.size) % len(BLOB_KINDS)).astype(np.uint8)
    param = r2.integers(0, 1 << 32, bad.size, dtype=np.uint64)
    for i, u in zip(bad[kind == 4], param[kind == 4]):
        p = pre[i]
        k = p.index(b"\x73\x20" + pks[who[i]].tobytes())
        pre[i] = p[:k] + b"\x73\x21" + p[k + 2:k + 34] + bytes([int(u) & 0xFF]) + p[k + 34:]
    return {"n": n, "pre": pre, "seeds": seeds, "pks": pks, "who": who, "bad": bad, "kind": kind, "param": param}


def config1_signing_hashes(plan):
    """SHA512Half of every signing preimage (hashlib, on the host)."""
    return np.frombuffer(b"".join(hashlib.sha512(p).digest()[:32] for p in plan["pre"]), np.uint8).reshape(-1, 32)


def config1_finish(plan, sig):
    """The serialized blobs: each preimage without 'STX\\0' with TxnSignature
    (0x74 0x40 + 64 B) after SigningPubKey, as STObject::add(s, true) orders
    them; then the post-signing mutations of kinds 0-3.  -> (buf, offs, lens)
    packed with a 16-byte zero tail (the kernels' loads)."""
    blobs = []
    fee = b"\x68\x40\x00\x00\x00\x00\x00\x00\x0a"  # Fee (10 drops), right before SigningPubKey
    for i, p in enumerate(plan["pre"]):
        k = p.index(fee) + 9
        assert p[k] == 0x73, i
        k += 2 + p[k + 1]
        blobs.append(bytearray(p[4:k] + b"\x74\x40" + bytes(sig[i]) + p[k:]))
    for i, kd, u in zip(plan["bad"], plan["kind"], plan["param"]):
        b, u = blobs[i], int(u)
        bit = 1 << ((u >> 16) & 7)
        s = b.index(b"\x74\x40") + 2
        if kd == 0:
            b[len(b) - 20 + u % 20] ^= bit  # Destination, the last field
        elif kd == 1:
            b[s + u % 32] ^= bit
        elif kd == 2:
            b[s + 32 + u % 32] ^= bit
        elif kd == 3:
            b[3:8], b[8:13] = b[8:13], b[3:8]  # Flags (0x22 ..) <-> Sequence (0x24 ..)
    lens = np.array([len(b) for b in blobs], np.int32)
    offs = np.zeros(len(blobs), np.int64)
    offs[1:] = np.cumsum(lens[:-1])
    buf = np.frombuffer(b"".join(bytes(b) for b in blobs) + bytes(16), np.uint8).copy()
    return buf, offs, lens


def config1_inputs_h16(buf, lens):
    return h16(buf[:int(lens.astype(np.int64).sum())], lens.astype("<i4"))


def config1_expected_status(plan):
    st = np.zeros(plan["n"], np.uint8)
    st[plan["bad"][plan["kind"] == 3]] = 1
    st[plan["bad"][plan["kind"] == 4]] = 2
    return st
