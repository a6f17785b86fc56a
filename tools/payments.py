"""Synthetic Payment transactions of BASELINE.json configs 1 and 5 (SURVEY.md
8d, Appendix C): signing preimages "STX\\0" || the Payment fields, and the
whole serialized transactions with their TxnSignature field.  Used by
bench.py's config-1 leg and tools/report_configs.py (benchmark data, not a
product path)."""
import hashlib

import numpy as np


def payment_preimages(pks, n, rng, pad_lens=None):
    """Signing preimages "STX\\0" || Payment fields without TxnSignature
    (Account/Destination are synthetic 20-byte ids).
    pad_lens: optional target preimage lengths (config 5) reached with a
    Memos array holding one MemoData."""
    out = []
    nacc = pks.shape[0]
    seq = np.zeros(nacc, np.int64)
    for i in range(n):
        a = i % nacc
        seq[a] += 1
        f = bytearray(b"STX\x00")
        f += b"\x12\x00\x00"                                   # TransactionType = Payment
        f += b"\x22" + (0x80000000).to_bytes(4, "big")         # Flags
        f += b"\x24" + int(seq[a]).to_bytes(4, "big")          # Sequence
        if rng.random() < 0.5:
            f += b"\x2e" + int(rng.integers(0, 2**32)).to_bytes(4, "big")  # DestinationTag
        if rng.random() < 0.8:
            amt = int(rng.integers(1, 10**11)) | 0x4000000000000000
            f += b"\x61" + amt.to_bytes(8, "big")              # Amount, native
        else:                                                  # Amount, IOU (STAmount.cpp:465-488)
            head = int(rng.integers(10**15, 10**16)) | ((int(rng.integers(-96, 81)) + 512 + 256 + 97) << 54)
            f += b"\x61" + head.to_bytes(8, "big") + b"\0" * 12 + b"USD" + b"\0" * 5 + rng.bytes(20)
        f += b"\x68" + (10 | 0x4000000000000000).to_bytes(8, "big")  # Fee
        f += b"\x73\x20" + pks[a].tobytes()                    # SigningPubKey
        f += b"\x81\x14" + hashlib.sha256(pks[a].tobytes()).digest()[:20]  # Account
        f += b"\x83\x14" + rng.bytes(20)                                   # Destination
        if pad_lens is not None:
            # Memos [ Memo { MemoData } ]: the one array Payment's template
            # allows (TxFormats.cpp:113-130), last in fieldCode order
            want = int(pad_lens[i]) - len(f)
            if want > 200:
                body = rng.bytes(min(want - 7, 12480))
                v = len(body) - 193                            # VL length, 2-byte form
                f += b"\xf9\xea\x7d" + bytes([193 + (v >> 8), v & 0xff]) + body + b"\xe1\xf1"
        out.append(bytes(f))
    return out


def pack(preimages):
    lens = np.array([len(p) for p in preimages], np.uint32)
    offs = np.zeros(len(preimages), np.uint64)
    offs[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
    blob = np.frombuffer(b"".join(preimages), np.uint8).copy()
    return blob, offs, lens


def blobs_from_preimages(pre, sig_np, pk_np):
    """Whole serialized transactions: the preimage without "STX\\0" with the
    TxnSignature field (0x74 0x40 <64 B>) put after SigningPubKey, as
    STObject::add(s, true) orders them."""
    out = []
    for i, p in enumerate(pre):
        k = p.index(b"\x73\x20" + pk_np[i].tobytes()) + 34
        out.append(p[4:k] + b"\x74\x40" + sig_np[i].tobytes() + p[k:])
    return out
