"""Synthetic serialized transactions for the blob-path tests (test
infrastructure only).

A from-scratch Python serializer written from the reference's wire rules --
field ids per Serializer::addFieldID (Serializer.cpp:193-220), VL lengths per
encodeVL (Serializer.cpp:496-521), objects sorted by fieldCode with 0xE1 /
0xF1 end markers (SerializedObject.cpp:353-379, 1208-1216), amounts per
STAmount::add (STAmount.cpp:465-488), path sets per STPathSet::add
(SerializedTypes.cpp:636-666) -- independent of oracle/stl_oracle_tx.c (the C
re-serialiser), so the two cross-check each other.  Also the mutations that
take a blob out of canonical form, for the deferral tests.
"""
import hashlib

import numpy as np

# serialized type ids (SerializeDeclarations.h TYPE lines)
UINT16, UINT32, UINT64, HASH128, HASH256, AMOUNT, VL, ACCOUNT = 1, 2, 3, 4, 5, 6, 7, 8
OBJECT, ARRAY, UINT8, HASH160, PATHSET, VECTOR256 = 14, 15, 16, 17, 18, 19

# a few declared fields (type, index)
TransactionType = (UINT16, 2)
Flags, SourceTag, Sequence, DestinationTag = (UINT32, 2), (UINT32, 3), (UINT32, 4), (UINT32, 14)
LastLedgerSequence = (UINT32, 27)
InvoiceID = (HASH256, 17)
AccountTxnID = (HASH256, 9)
Amount, Fee, SendMax = (AMOUNT, 1), (AMOUNT, 8), (AMOUNT, 9)
SigningPubKey, TxnSignature, Signature = (VL, 3), (VL, 4), (VL, 6)
MemoType, MemoData = (VL, 12), (VL, 13)
Account, Destination = (ACCOUNT, 1), (ACCOUNT, 3)
Paths = (PATHSET, 1)
Hashes = (VECTOR256, 2)
Memo = (OBJECT, 10)
TemplateEntry = (OBJECT, 9)
Memos = (ARRAY, 9)
TxnSignatures = (ARRAY, 3)
Template = (ARRAY, 5)
TakerPaysCurrency = (HASH160, 1)
# fields of the other TxFormats templates (TxFormats.cpp:22-111)
TakerPays, TakerGets = (AMOUNT, 4), (AMOUNT, 5)
Expiration, OfferSequence, SetFlag = (UINT32, 10), (UINT32, 25), (UINT32, 33)
QualityIn, InflateSeq, ReferenceFeeUnits = (UINT32, 20), (UINT32, 26), (UINT32, 30)
RegularKey, InflationDest = (ACCOUNT, 8), (ACCOUNT, 9)
Amendment = (HASH256, 19)
# SerializedValidation's template (SerializedValidation.cpp:134-159)
LedgerSequence, CloseTime, SigningTime = (UINT32, 6), (UINT32, 7), (UINT32, 9)
LoadFee, ReserveBase, ReserveIncrement = (UINT32, 24), (UINT32, 31), (UINT32, 32)
BaseFee = (UINT64, 5)
LedgerHash = (HASH256, 1)
Amendments = (VECTOR256, 3)

NON_SIGNING = {TxnSignature, Signature, TxnSignatures}


def field_id(t, n):
    if t < 16:
        return bytes([(t << 4) | n]) if n < 16 else bytes([t << 4, n])
    return bytes([n, t]) if n < 16 else bytes([0, t, n])


def vl_len(n):
    if n <= 192:
        return bytes([n])
    if n <= 12480:
        n -= 193
        return bytes([193 + (n >> 8), n & 0xFF])
    n -= 12481
    return bytes([241 + (n >> 16), (n >> 8) & 0xFF, n & 0xFF])


def code(f):
    return (f[0] << 16) | f[1]


class Field:
    """One field: (type, index) and its encoded value (no header)."""

    def __init__(self, fid, value):
        self.fid = tuple(fid)
        self.value = bytes(value)

    def encode(self):
        return field_id(*self.fid) + self.value


def serialize(fields, sort=True, skip=()):
    fs = sorted(fields, key=lambda f: code(f.fid)) if sort else list(fields)
    return b"".join(f.encode() for f in fs if f.fid not in skip)


# ------------------------------------------------------------- value encoders
def u16(v): return int(v).to_bytes(2, "big")
def u32(v): return int(v).to_bytes(4, "big")
def u64(v): return int(v).to_bytes(8, "big")
def vl(b): return vl_len(len(b)) + bytes(b)


def amount_native(drops, negative=False):
    v = int(drops)
    return (v if negative else v | 0x4000000000000000).to_bytes(8, "big")


def amount_iou(mantissa, offset, currency, issuer, negative=False):
    if mantissa == 0:
        head = 0x8000000000000000
    else:
        head = mantissa | ((offset + 512 + (0 if negative else 256) + 97) << 54)
    return head.to_bytes(8, "big") + bytes(currency) + bytes(issuer)


def pathset(paths):
    """paths: list of lists of (account|None, currency|None, issuer|None)."""
    out = b""
    for i, p in enumerate(paths):
        if i:
            out += b"\xff"
        for acc, cur, iss in p:
            t = (1 if acc else 0) | (0x10 if cur is not None else 0) | (0x20 if iss else 0)
            out += bytes([t]) + (acc or b"") + (cur if cur is not None else b"") + (iss or b"")
    return out + b"\x00"


def obj_value(fields, sort=True):
    return serialize(fields, sort) + b"\xe1"


def array_value(elements, sort=True):
    """elements: list of (fid, [Field])."""
    out = b""
    for fid, inner in elements:
        out += field_id(*fid) + serialize(inner, sort) + b"\xe1"
    return out + b"\xf1"


# ------------------------------------------------------------- transactions
def account_id(pk):
    return hashlib.sha256(bytes(pk)).digest()[:20]


def payment_fields(rng, pk, seq, *, memos=0, paths=False, pad_to=None, extras=False):
    """Payment fields without TxnSignature (SURVEY Appendix C plus optional
    Memos / Paths / SendMax / InvoiceID / tags)."""
    fs = [Field(TransactionType, u16(0)),
          Field(Flags, u32(0x80000000)),
          Field(Sequence, u32(seq)),
          Field(Fee, amount_native(10)),
          Field(SigningPubKey, vl(pk)),
          Field(Account, vl(account_id(pk))),
          Field(Destination, vl(rng.bytes(20)))]
    iou = rng.random() < 0.3
    cur, iss = b"\0" * 12 + b"USD" + b"\0" * 5, rng.bytes(20)
    if iou:
        fs.append(Field(Amount, amount_iou(int(rng.integers(10**15, 10**16)), int(rng.integers(-96, 81)), cur, iss)))
    else:
        fs.append(Field(Amount, amount_native(int(rng.integers(1, 10**11)))))
    if rng.random() < 0.5:
        fs.append(Field(DestinationTag, u32(rng.integers(0, 2**32))))
    if extras:
        if rng.random() < 0.5:
            fs.append(Field(SourceTag, u32(rng.integers(0, 2**32))))
        if rng.random() < 0.5:
            fs.append(Field(LastLedgerSequence, u32(rng.integers(0, 2**32))))
        if rng.random() < 0.4:
            fs.append(Field(InvoiceID, rng.bytes(32)))
        if rng.random() < 0.3:
            fs.append(Field(SendMax, amount_iou(int(rng.integers(10**15, 10**16)), 0, cur, iss)))
    if paths:
        ps = []
        for _ in range(int(rng.integers(1, 4))):
            p = []
            for _ in range(int(rng.integers(1, 4))):
                k = int(rng.integers(0, 3))
                if k == 0:
                    p.append((rng.bytes(20), None, None))
                elif k == 1:
                    p.append((None, cur, iss))
                else:
                    p.append((None, b"\0" * 20, None))  # currency bit over a zero currency (XRP)
            ps.append(p)
        fs.append(Field(Paths, pathset(ps)))
    if memos:
        els = []
        for _ in range(memos):
            inner = [Field(MemoType, vl(rng.bytes(int(rng.integers(1, 20))))),
                     Field(MemoData, vl(rng.bytes(int(rng.integers(0, 200)))))]
            els.append((Memo, inner))
        fs.append(Field(Memos, array_value(els)))
    if pad_to is not None:
        cur_len = len(serialize(fs)) + 66 + 4
        want = int(pad_to) - cur_len - 4
        if want > 0:
            memo = [Field(MemoData, vl(rng.bytes(min(want, 12000))))]
            fs.append(Field(Memos, array_value([(Memo, memo)])))
    return fs


def signing_preimage(fields):
    return b"STX\x00" + serialize(fields, skip=NON_SIGNING)


def sha512_half(data):
    return hashlib.sha512(data).digest()[:32]


def signed_blob(fields, sk, signer):
    """Sort, sign SHA512Half(STX || signing fields), append TxnSignature."""
    h = sha512_half(signing_preimage(fields))
    sig = signer(h, sk)
    return serialize(fields + [Field(TxnSignature, vl(sig))]), h, sig


def tx_id(blob):
    return sha512_half(b"TXN\x00" + bytes(blob))


def validation_fields(rng, pk, *, full=True, extras=True):
    """A SerializedValidation's fields (SerializedValidation.cpp:39-56,
    134-159): Flags (vfFullyCanonicalSig 0x80000000, kFullFlag 0x1),
    LedgerHash, SigningTime, SigningPubKey, optional LedgerSequence /
    CloseTime / LoadFee / Amendments / BaseFee / Reserve*."""
    fs = [Field(Flags, u32(0x80000000 | (1 if full else 0))),
          Field(LedgerHash, rng.bytes(32)),
          Field(SigningTime, u32(int(rng.integers(0, 2**32)))),
          Field(SigningPubKey, vl(pk))]
    if extras:
        if rng.random() < 0.7:
            fs.append(Field(LedgerSequence, u32(int(rng.integers(1, 2**31)))))
        if rng.random() < 0.5:
            fs.append(Field(CloseTime, u32(int(rng.integers(0, 2**32)))))
        if rng.random() < 0.3:
            fs.append(Field(LoadFee, u32(int(rng.integers(256, 2**16)))))
        if rng.random() < 0.2:
            fs.append(Field(Amendments, vl(rng.bytes(32 * int(rng.integers(1, 4))))))
        if rng.random() < 0.2:
            fs.append(Field(BaseFee, int(rng.integers(1, 2**40)).to_bytes(8, "big")))
            fs.append(Field(ReserveBase, u32(int(rng.integers(1, 2**31)))))
            fs.append(Field(ReserveIncrement, u32(int(rng.integers(1, 2**31)))))
    return fs


def validation_preimage(fields):
    """STObject::getSigningHash(SIGN_VALIDATION) preimage: "VAL\0" || fields
    without Signature (SerializedValidation.cpp:70-73, HashPrefix.cpp:31)."""
    return b"VAL\x00" + serialize(fields, skip=NON_SIGNING)


def signed_validation(fields, sk, signer):
    """SerializedValidation::sign (SerializedValidation.cpp:59-68): sign the
    signing hash, set sfSignature; returns (blob, signing hash, signature)."""
    h = sha512_half(validation_preimage(fields))
    sig = signer(h, sk)
    return serialize(fields + [Field(Signature, vl(sig))]), h, sig


# ------------------------------------------------------------- corpora
def keys(oracle, n, seed):
    rng = np.random.default_rng(seed)
    out = []
    for _ in range(n):
        pk, sk = oracle.keypair(rng.bytes(32))
        out.append((pk, sk))
    return out


def valid_corpus(oracle, n, seed, with_preimages=False, **kw):
    """n canonical, correctly signed blobs with a spread of optional fields
    (and their signing preimages from this serializer)."""
    rng = np.random.default_rng(seed)
    ks = keys(oracle, 8, seed ^ 0x5EED)
    blobs, pres = [], []
    for i in range(n):
        pk, sk = ks[i % len(ks)]
        opts = dict(memos=int(rng.integers(0, 3)) if rng.random() < 0.3 else 0,
                    paths=rng.random() < 0.25, extras=True)
        opts.update(kw)
        fs = payment_fields(rng, pk, i + 1, **opts)
        # (no top-level Signature / TxnSignatures: Payment's template has
        # neither, so SerializedTransaction's constructor would throw)
        blob, _, _ = signed_blob(fs, sk, oracle.sign)
        blobs.append(blob)
        pres.append(signing_preimage(fs))
    return (blobs, pres) if with_preimages else blobs


def special_cases(oracle, seed=7):
    """(name, blob, expectation) with expectation in {"ok", "reject",
    "malformed", "defer", "unconstructible"} for the cases the reference's own
    rules single out."""
    rng = np.random.default_rng(seed)
    pk, sk = keys(oracle, 1, seed)[0]
    out = []

    def fs0(**kw):
        return payment_fields(np.random.default_rng(int(rng.integers(2**32))), pk, 5, **kw)

    base = fs0()
    blob, h, sig = signed_blob(base, sk, oracle.sign)
    out.append(("valid", blob, "ok"))
    # signature over something else -> verify rejects
    bad = bytearray(blob)
    i = blob.index(field_id(*TxnSignature) + b"\x40") + 2 + 10
    bad[i] ^= 1
    out.append(("sig_bitflip", bytes(bad), "reject"))
    # B12: pk length, sig length, missing TxnSignature (checkSign false, blob canonical)
    f = [x for x in base if x.fid != SigningPubKey] + [Field(SigningPubKey, vl(pk + b"\0"))]
    out.append(("pk_33", serialize(f + [Field(TxnSignature, vl(sig))]), "malformed"))
    out.append(("sig_63", serialize(base + [Field(TxnSignature, vl(sig[:63]))]), "malformed"))
    out.append(("sig_65", serialize(base + [Field(TxnSignature, vl(sig + b"\0"))]), "malformed"))
    out.append(("sig_missing", serialize(base), "malformed"))
    f = [x for x in base if x.fid != SigningPubKey]  # SOE_REQUIRED: the constructor throws
    out.append(("pk_missing", serialize(f + [Field(TxnSignature, vl(sig))]), "unconstructible"))
    # non-signing fields at the top level (Signature VL, TxnSignatures array):
    # outside Payment's template, so the constructor throws (setType leftover)
    f = base + [Field(Signature, vl(b"xyz"))]
    out.append(("with_Signature", signed_blob(f, sk, oracle.sign)[0], "unconstructible"))
    f = base + [Field(TxnSignatures, array_value([((OBJECT, 2), [Field(SigningPubKey, vl(bytes(33)))])]))]
    out.append(("with_TxnSignatures", signed_blob(f, sk, oracle.sign)[0], "unconstructible"))
    # ---- TxFormats templates (TxFormats.cpp:22-130, setType SerializedObject.cpp:152-207)
    def without(fields, fid):
        return [x for x in fields if x.fid != fid]
    out.append(("payment_no_amount", signed_blob(without(base, Amount), sk, oracle.sign)[0], "unconstructible"))
    out.append(("payment_no_destination", signed_blob(without(base, Destination), sk, oracle.sign)[0],
                "unconstructible"))
    out.append(("payment_no_fee", signed_blob(without(base, Fee), sk, oracle.sign)[0], "unconstructible"))
    out.append(("no_sequence", signed_blob(without(base, Sequence), sk, oracle.sign)[0], "unconstructible"))
    out.append(("no_account", signed_blob(without(base, Account), sk, oracle.sign)[0], "unconstructible"))
    out.append(("no_transaction_type", signed_blob(without(base, TransactionType), sk, oracle.sign)[0],
                "unconstructible"))
    f = base + [Field(TakerPays, amount_native(5))]  # an OfferCreate field in a Payment
    out.append(("payment_foreign_field", signed_blob(f, sk, oracle.sign)[0], "unconstructible"))
    f = base + [Field(Hashes, vl(rng.bytes(64)))]  # declared, in no transaction template
    out.append(("payment_vector256", signed_blob(f, sk, oracle.sign)[0], "unconstructible"))
    for tt in (2, 6, 9, 10, 99, 102, 0xFFFF):  # WalletAdd, NicknameSet, Contract(Remove): no format
        f = without(base, TransactionType) + [Field(TransactionType, u16(tt))]
        out.append((f"type_{tt}_no_format", signed_blob(f, sk, oracle.sign)[0], "unconstructible"))
    common = without(without(without(base, TransactionType), Amount), Destination)
    typed = {
        "offer_create": (7, [Field(TakerPays, amount_native(5)), Field(TakerGets, amount_native(7)),
                             Field(Expiration, u32(9)), Field(OfferSequence, u32(3))]),
        "offer_cancel": (8, [Field(OfferSequence, u32(3))]),
        "account_set": (3, [Field(SetFlag, u32(1)), Field(InflationDest, vl(rng.bytes(20)))]),
        "account_merge": (4, [Field(Destination, vl(rng.bytes(20)))]),
        "trust_set": (20, [Field(QualityIn, u32(1))]),
        "regular_key": (5, [Field(RegularKey, vl(rng.bytes(20)))]),
        "inflation": (1, [Field(InflateSeq, u32(11))]),
        "amendment": (100, [Field(Amendment, rng.bytes(32))]),
        "set_fee": (101, [Field(BaseFee, u64(10)), Field(ReferenceFeeUnits, u32(10)), Field(ReserveBase, u32(20)),
                          Field(ReserveIncrement, u32(5))]),
    }
    for name, (tt, extra) in typed.items():
        f = common + [Field(TransactionType, u16(tt))] + extra
        out.append((name, signed_blob(f, sk, oracle.sign)[0], "ok"))
        if any(True for _ in extra):  # drop the first field: required ones make it unconstructible
            req = name in ("offer_create", "offer_cancel", "account_merge", "inflation", "amendment", "set_fee")
            f = common + [Field(TransactionType, u16(tt))] + extra[1:]
            out.append((name + "_minus_first", signed_blob(f, sk, oracle.sign)[0], "unconstructible" if req else "ok"))
    f = common + [Field(TransactionType, u16(7)), Field(TakerPays, amount_native(5)), Field(TakerGets, amount_native(7)),
                  Field(Amount, amount_native(1))]
    out.append(("offer_with_amount", signed_blob(f, sk, oracle.sign)[0], "unconstructible"))
    # nested objects and arrays (canonical), path sets, vector256 (inside a
    # Memo: inner objects have no template)
    out.append(("memos", signed_blob(fs0(memos=3), sk, oracle.sign)[0], "ok"))
    out.append(("paths", signed_blob(fs0(paths=True), sk, oracle.sign)[0], "ok"))
    f = base + [Field(Memos, array_value([(Memo, [Field(Hashes, vl(rng.bytes(64)))])]))]
    out.append(("vector256", signed_blob(f, sk, oracle.sign)[0], "ok"))
    deep = [Field(MemoData, vl(b"x"))]
    for _ in range(3):  # (ARRAY > element object) x 4: fields at depth 8, the deepest the device takes
        deep = [Field(Template, array_value([(TemplateEntry, deep)]))]
    f = base + [Field(Memos, array_value([(Memo, deep)]))]
    out.append(("depth_ok", signed_blob(f, sk, oracle.sign)[0], "ok"))
    deep = [Field(MemoData, vl(b"x"))]
    for _ in range(4):
        deep = [Field(Template, array_value([(TemplateEntry, deep)]))]
    f = base + [Field(Memos, array_value([(Memo, deep)]))]
    out.append(("depth_too_deep", signed_blob(f, sk, oracle.sign)[0], "defer"))
    # long VL encodings (2- and 3-byte lengths)
    f = base + [Field(Memos, array_value([(Memo, [Field(MemoData, vl(rng.bytes(300)))])]))]
    out.append(("vl_2byte", signed_blob(f, sk, oracle.sign)[0], "ok"))
    f = base + [Field(Memos, array_value([(Memo, [Field(MemoData, vl(rng.bytes(13000)))])]))]
    out.append(("vl_3byte", signed_blob(f, sk, oracle.sign)[0], "ok"))
    # ---- not canonical: the reference re-serialises differently -> defer
    full = sorted(base + [Field(TxnSignature, vl(sig))], key=lambda x: code(x.fid))
    sw = list(full)
    sw[1], sw[2] = sw[2], sw[1]
    out.append(("order_swapped", serialize(sw, sort=False), "defer"))
    dup = full + [Field(Sequence, u32(9))]
    out.append(("duplicate_field", serialize(sorted(dup, key=lambda x: code(x.fid)), sort=False), "unconstructible"))
    out.append(("top_level_end_marker", blob + b"\xe1" + b"junk", "defer"))
    inner = [Field(MemoData, vl(b"a")), Field(MemoType, vl(b"b"))]  # inner order reversed
    f = base + [Field(Memos, array_value([(Memo, inner)], sort=False))]
    out.append(("inner_order", serialize(f + [Field(TxnSignature, vl(oracle.sign(sha512_half(
        b"STX\x00" + serialize(f, skip=NON_SIGNING)), sk)))]), "defer"))
    f = base + [Field(Memos, array_value([(Memo, [Field(Hashes, vl(rng.bytes(40)))])]))]  # partial Vector256 entry
    out.append(("vector256_partial", signed_blob(f, sk, oracle.sign)[0], "defer"))
    f = base + [Field(Paths, b"\x01" + b"\0" * 20 + b"\x00")]  # account bit over a zero account
    out.append(("path_zero_account", signed_blob(f, sk, oracle.sign)[0], "defer"))
    f = base + [Field(Paths, b"\x20" + b"\0" * 20 + b"\x00")]  # issuer bit over a zero issuer
    out.append(("path_zero_issuer", signed_blob(f, sk, oracle.sign)[0], "defer"))
    f = base + [Field(Paths, b"\xff\x01" + rng.bytes(20) + b"\x00")]  # empty first path
    out.append(("path_empty", signed_blob(f, sk, oracle.sign)[0], "unconstructible"))
    f = base + [Field(Paths, b"\x02" + b"\x00")]
    out.append(("path_bad_type", signed_blob(f, sk, oracle.sign)[0], "unconstructible"))
    # undeclared field of a known type: the reference makes one up; the device defers
    f = base + [Field(Memos, array_value([(Memo, [Field((UINT32, 60), u32(1))])]))]
    out.append(("dynamic_field", signed_blob(f, sk, oracle.sign)[0], "defer"))
    f = base + [Field((UINT32, 60), u32(1))]  # at the top level it is a setType leftover
    out.append(("dynamic_field_top", signed_blob(f, sk, oracle.sign)[0], "unconstructible"))
    # array left open at the end of the blob (re-serialisation adds 0xF1)
    f = base + [Field(TxnSignature, vl(sig))]
    out.append(("array_unterminated", serialize(f) + field_id(*Memos) + field_id(*Memo) + b"\xe1", "defer"))
    out.append(("truncated", blob[:-5], "unconstructible"))
    out.append(("too_short", blob[:20], "unconstructible"))
    # non-minimal field header (type 1 written as an uncommon type)
    hdr = bytes([0x02, 0x01]) + blob[1:]
    out.append(("header_uncommon_form", hdr, "unconstructible"))
    return out


def mutate(rng, blob):
    """One random structural mutation (fuzzing)."""
    b = bytearray(blob)
    if not b:
        return bytes(rng.bytes(int(rng.integers(0, 40))))
    k = int(rng.integers(0, 6))
    i = int(rng.integers(0, len(b)))
    if k == 0:
        b[i] ^= 1 << int(rng.integers(0, 8))
    elif k == 1:
        b[i] = int(rng.integers(0, 256))
    elif k == 2:
        del b[i]
    elif k == 3:
        b.insert(i, int(rng.integers(0, 256)))
    elif k == 4:
        j = int(rng.integers(0, len(b)))
        b[i], b[j] = b[j], b[i]
    else:
        b = b[:i]
    return bytes(b)
