// stl_txblob.h -- signing hash and transaction ID straight from a serialized
// transaction (the wire / rawTransaction blob), for the gfx950 kernels and
// their host build.
//
// Reference path:
//   SerializedTransaction(SerializerIterator&)   SerializedTransaction.cpp:65-92
//     -> STObject::set                            SerializedObject.cpp:266-306
//   getSigningHash = SHA512Half("STX\0" || STObject::add(s, false))
//                                                 SerializedObject.cpp:444-450, 353-379
//   getTransactionID = SHA512Half("TXN\0" || STObject::add(s, true))
//                                                 SerializedTransaction.cpp:167-171
//   checkSign: getFieldVL(sfSigningPubKey), getFieldVL(sfTxnSignature)
//                                                 SerializedTransaction.cpp:192-230
//
// The reference parses the blob into fields and serialises them again, sorted
// by fieldCode, leaving out the non-signing fields (TxnSignature, Signature,
// TxnSignatures: FieldNames.cpp:49-51).  When the blob is already in the form
// that re-serialisation produces ("canonical"), that is the blob itself with
// those top-level fields cut out, so the kernels splice instead of
// re-serialising: one pass over the fields checks canonical form and records
// the cut ranges, and the SHA-512 message stream skips them.  Anything the pass
// cannot prove canonical is DEFERRED to the caller's own checkSign (a deferral
// is never a reject).  What the pass checks, per reference rule:
//   * field headers in the only form addFieldID writes (Serializer.cpp:193-262);
//   * strictly ascending fieldCode in every object (add() sorts through a
//     std::map; setType rejects duplicates, SerializedObject.cpp:152-207);
//   * every field a declared one (SerializeDeclarations.h; undeclared codes the
//     reference would create on the fly are deferred, not judged);
//   * nested objects end with 0xE1, arrays with 0xF1, no 0xE1 at top level
//     (set() stops there and ignores the rest), at most kBlobMaxDepth levels;
//   * VL lengths in range (decodeVLLength, Serializer.cpp:549-575), Vector256 a
//     multiple of 32 bytes (STVector256::construct drops a partial tail),
//     path elements with only the valid type bits, no empty path, and no
//     account/issuer bit over a zero id (STPathElement recomputes the type
//     from the ids, SerializedTypes.h:1179-1187);
//   * length within [txMinSizeBytes, txMaxSizeBytes] (Protocol.h:41-45);
//   * transactions: the top level fits the TxFormats template of its
//     TransactionType (tx_format below; SerializedTransaction.cpp:79-91);
//     validations: no top-level field outside SerializedValidation's template
//     (validation_field below: the reference drops such fields).
// Amounts, integers, hashes and VL payloads re-serialise byte for byte from any
// encoding the reference constructs (STAmount.cpp:465-560), so they need no
// check beyond their size.
// TxnSignatures (ARRAY 3) is in no TxFormats template and not in the
// validation template, so under kFormatTx / kFormatValidation -- every
// product call -- a blob carrying it is DEFERRED; cutting it out of the
// signing stream (cut_open below) only happens with kFormatNone, the bare pass
// of the host tests (tests/test_txblob.py::test_txnsignatures_always_deferred).
#pragma once
#include "stl_sha512.h"

namespace stl {

constexpr uint32_t kPrefixTxSign = 0x53545800u;  // HashPrefix::txSign "STX\0", HashPrefix.cpp:30
constexpr uint32_t kPrefixTxId = 0x54584E00u;    // HashPrefix::transactionID "TXN\0", HashPrefix.cpp:25
constexpr uint32_t kPrefixValidation = 0x56414C00u;  // HashPrefix::validation "VAL\0", HashPrefix.cpp:31
constexpr uint32_t kTxMinBytes = 32;             // Protocol::txMinSizeBytes
constexpr uint32_t kTxMaxBytes = 1024 * 1024;    // Protocol::txMaxSizeBytes
constexpr uint32_t kValMinBytes = 50;            // PeerImp::recvValidation, PeerImp.cpp:1134
constexpr int kBlobMaxDepth = 8;

// per-transaction status (include/stl.h STL_TX_*)
constexpr uint32_t kTxOk = 0;         // signing hash computed, verify decides
constexpr uint32_t kTxDeferred = 1;   // not provably canonical: caller's serial checkSign
constexpr uint32_t kTxMalformed = 2;  // canonical, but SigningPubKey != 32 B or TxnSignature != 64 B
                                      // (RippleAddress.cpp:192-194 throws -> checkSign false)

// field codes, FIELD_CODE(type, index) = type << 16 | index
constexpr uint32_t kCodeSigningPubKey = 0x70003u;  // VL 3
constexpr uint32_t kCodeTxnSignature = 0x70004u;   // VL 4
constexpr uint32_t kCodeSignature = 0x70006u;      // VL 6
constexpr uint32_t kCodeTxnSignatures = 0xF0003u;  // ARRAY 3
constexpr uint32_t kCodeObjectEnd = 0xE0001u;      // STI_OBJECT, 1
constexpr uint32_t kCodeArrayEnd = 0xF0001u;       // STI_ARRAY, 1

// SField::notSigningField (FieldNames.cpp:49-51): left out of every signing
// hash (STObject::add(s, false)), cut out of the blob by the splice.
STL_HD bool non_signing_field(uint32_t code) {
  return code == kCodeTxnSignature || code == kCodeSignature || code == kCodeTxnSignatures;
}

// Which signed object a blob is (include/stl.h STL_BLOB_*): the signing-hash
// prefix, the field that holds the signature, and the ID hash.
struct BlobKind {
  uint32_t sign_prefix;  // getSigningHash prefix
  uint32_t sig_code;     // signature field (SigningPubKey is VL 3 for both)
  uint32_t id_prefix;    // ID = SHA512Half(id_prefix || blob), or of the blob alone
  uint32_t id_prefixed;  // 0: no prefix
  uint32_t min_len;
  uint32_t format;       // top-level template check: kFormatTx or kFormatValidation
};
constexpr uint32_t kFormatNone = 0;        // no check (host tests of the bare pass)
constexpr uint32_t kFormatTx = 1;          // TxFormats template of the TransactionType (tx_format)
constexpr uint32_t kFormatValidation = 2;  // SerializedValidation's template (validation_field)
// SerializedTransaction: checkSign / getTransactionID (SerializedTransaction.cpp:162-171,220-230)
STL_HD BlobKind blob_kind_tx() { return BlobKind{kPrefixTxSign, kCodeTxnSignature, kPrefixTxId, 1u, kTxMinBytes, kFormatTx}; }
// SerializedValidation::isValid (SerializedValidation.cpp:70-73,96-110); ID =
// the suppression hash SHA512Half(raw validation), PeerImp.cpp:1148-1155
STL_HD BlobKind blob_kind_validation() {
  return BlobKind{kPrefixValidation, kCodeSignature, 0u, 0u, kValMinBytes, kFormatValidation};
}

// ---- TxFormats templates (TxFormats.cpp:22-111, addCommonFields :113-130) ----
// SerializedTransaction(SerializerIterator&) throws after set() unless
// TransactionType is present (getFieldU16, SerializedObject.cpp:661-675), names
// a format (findByType) and STObject::setType accepts the top-level fields
// (SerializedObject.cpp:152-207): every SOE_REQUIRED field present, no field
// outside the template (a leftover is discardable only with fieldValue > 256,
// FieldNames.h:178-181, which no wire header can encode), no SOE_DEFAULT field
// at its default (sfPaths: an empty path set, which the path-set walk already
// defers).  Each template field has a bit; the masks below are the templates.
STL_HD int tx_field_bit(uint32_t code) {
  switch (code) {
    case 0x10002u: return 0;   // TransactionType   (common fields)
    case 0x20002u: return 1;   // Flags
    case 0x20003u: return 2;   // SourceTag
    case 0x80001u: return 3;   // Account
    case 0x20004u: return 4;   // Sequence
    case 0x50005u: return 5;   // PreviousTxnID
    case 0x2001Bu: return 6;   // LastLedgerSequence
    case 0x50009u: return 7;   // AccountTxnID
    case 0x60008u: return 8;   // Fee
    case 0x2001Du: return 9;   // OperationLimit
    case 0xF0009u: return 10;  // Memos
    case 0x70003u: return 11;  // SigningPubKey
    case 0x70004u: return 12;  // TxnSignature
    case 0x2000Bu: return 13;  // TransferRate      (AccountSet)
    case 0x20021u: return 14;  // SetFlag
    case 0x20022u: return 15;  // ClearFlag
    case 0x80009u: return 16;  // InflationDest
    case 0x8000Au: return 17;  // SetAuthKey
    case 0x80003u: return 18;  // Destination       (AccountMerge, Payment)
    case 0x2000Eu: return 19;  // DestinationTag
    case 0x60003u: return 20;  // LimitAmount       (TrustSet)
    case 0x20014u: return 21;  // QualityIn
    case 0x20015u: return 22;  // QualityOut
    case 0x60004u: return 23;  // TakerPays         (OfferCreate)
    case 0x60005u: return 24;  // TakerGets
    case 0x2000Au: return 25;  // Expiration
    case 0x20019u: return 26;  // OfferSequence     (OfferCreate, OfferCancel)
    case 0x80008u: return 27;  // RegularKey        (SetRegularKey)
    case 0x60001u: return 28;  // Amount            (Payment)
    case 0x60009u: return 29;  // SendMax
    case 0x120001u: return 30; // Paths (SOE_DEFAULT)
    case 0x50011u: return 31;  // InvoiceID
    case 0x2001Au: return 32;  // InflateSeq        (Inflation)
    case 0x50013u: return 33;  // Amendment         (EnableAmendment)
    case 0x30005u: return 34;  // BaseFee           (SetFee)
    case 0x2001Eu: return 35;  // ReferenceFeeUnits
    case 0x2001Fu: return 36;  // ReserveBase
    case 0x20020u: return 37;  // ReserveIncrement
    default: return -1;
  }
}

// SerializedValidation's template (SerializedValidation.cpp:134-159).  Its
// constructor calls setType and ignores the result (SerializedObject.h:54-58):
// a field outside the template is dropped from the object, so the signing
// hash is not the splice of the blob -- such blobs are deferred.
STL_HD bool validation_field(uint32_t code) {
  switch (code) {
    case 0x20002u:   // Flags
    case 0x50001u:   // LedgerHash
    case 0x20006u:   // LedgerSequence
    case 0x20007u:   // CloseTime
    case 0x20018u:   // LoadFee
    case 0x130003u:  // Amendments
    case 0x30005u:   // BaseFee
    case 0x2001Fu:   // ReserveBase
    case 0x20020u:   // ReserveIncrement
    case 0x20009u:   // SigningTime
    case 0x70003u:   // SigningPubKey
    case 0x70006u:   // Signature
      return true;
    default:
      return false;
  }
}

STL_HD constexpr uint64_t tx_bits(int a, int b) { return ((2ull << b) - 1ull) & ~((1ull << a) - 1ull); }

// allowed / required field bits of TxType `type`; false for a type TxFormats
// does not define (findByType -> "invalid transaction type")
STL_HD bool tx_format(uint32_t type, uint64_t& allowed, uint64_t& required) {
  constexpr uint64_t kCommon = tx_bits(0, 12);
  constexpr uint64_t kCommonReq = (1ull << 0) | (1ull << 3) | (1ull << 4) | (1ull << 8) | (1ull << 11);
  uint64_t a, r;
  switch (type) {
    case 0: a = (1ull << 18) | (1ull << 19) | tx_bits(28, 31); r = (1ull << 18) | (1ull << 28); break;  // Payment
    case 1: a = r = 1ull << 32; break;                                        // Inflation
    case 3: a = tx_bits(13, 17); r = 0; break;                                // AccountSet
    case 4: a = tx_bits(18, 19); r = 1ull << 18; break;                       // AccountMerge
    case 5: a = 1ull << 27; r = 0; break;                                     // SetRegularKey
    case 7: a = tx_bits(23, 26); r = tx_bits(23, 24); break;                  // OfferCreate
    case 8: a = r = 1ull << 26; break;                                        // OfferCancel
    case 20: a = tx_bits(20, 22); r = 0; break;                               // TrustSet
    case 100: a = r = 1ull << 33; break;                                      // EnableAmendment
    case 101: a = r = tx_bits(34, 37); break;                                 // SetFee
    default: return false;
  }
  allowed = kCommon | a;
  required = kCommonReq | r;
  return true;
}

STL_HD uint64_t name_range(int a, int b) { return ((2ull << b) - 1ull) & ~((1ull << a) - 1ull); }

// Declared field indices per serialized type (SerializeDeclarations.h FIELD
// lines; all indices are < 64).
STL_HD uint64_t declared_names(uint32_t type) {
  switch (type) {
    case 1: return name_range(1, 2);                                // UINT16
    case 2: return name_range(2, 34) & ~(1ull << 15);               // UINT32
    case 3: return name_range(1, 8);                                // UINT64
    case 4: return 1ull << 1;                                       // HASH128
    case 5: return name_range(1, 9) | name_range(16, 19);           // HASH256
    case 6: return name_range(1, 9) | name_range(16, 18);           // AMOUNT
    case 7: return name_range(1, 13);                               // VL
    case 8: return name_range(1, 4) | name_range(7, 10);            // ACCOUNT
    case 14: return name_range(2, 10);                              // OBJECT
    case 15: return name_range(2, 9);                               // ARRAY
    case 16: return name_range(1, 3);                               // UINT8
    case 17: return name_range(1, 4);                               // HASH160
    case 18: return 1ull << 1;                                      // PATHSET
    case 19: return name_range(1, 3);                               // VECTOR256
    default: return 0;
  }
}

STL_HD bool field_declared(uint32_t type, uint32_t name) {
  return name < 64 && ((declared_names(type) >> name) & 1ull) != 0;
}

// Fixed payload size of a type, 0 for the variable ones.
STL_HD uint32_t fixed_size(uint32_t type) {
  switch (type) {
    case 16: return 1;
    case 1: return 2;
    case 2: return 4;
    case 3: return 8;
    case 4: return 16;
    case 17: return 20;
    case 5: return 32;
    default: return 0;
  }
}

// Result of the canonical-form pass.  Cut ranges are ascending; unused ones
// are [len, len).
struct TxLayout {
  uint32_t status;
  uint32_t pk_off, pk_len;    // SigningPubKey payload (pk_len 0xffffffff: absent)
  uint32_t sig_off, sig_len;  // signature payload (TxnSignature; Signature for validations)
  uint32_t xs0, xe0, xs1, xe1, xs2, xe2;
};

template <typename Bytes>
STL_HD bool bytes_nonzero(const Bytes& b, uint32_t pos, uint32_t n) {
  uint32_t acc = 0;
  for (uint32_t i = 0; i < n; ++i) acc |= b[pos + i];
  return acc != 0;
}

// The canonical-form pass over one blob (one lane).  Byte reads only, b[i]
// for i < len: a plain pointer, or the device's staged reader (the blob's
// first bytes in LDS, tx_blob_parse_kernel).
template <typename Bytes>
STL_HD void tx_blob_parse(const Bytes& b, uint32_t len, TxLayout& t, uint32_t sig_code = kCodeTxnSignature,
                          uint32_t min_len = kTxMinBytes, uint32_t format = kFormatTx) {
  t.status = kTxDeferred;
  t.pk_off = t.sig_off = 0;
  t.pk_len = t.sig_len = 0xffffffffu;
  t.xs0 = t.xe0 = t.xs1 = t.xe1 = t.xs2 = t.xe2 = len;
  if (len < min_len || len > kTxMaxBytes) return;
  uint32_t last[kBlobMaxDepth + 1];
  last[0] = 0;
  uint32_t arrays = 0;  // bit d: level d is an array
  int depth = 0;
  int ncut = 0;
  bool cut_open = false;  // a cut TxnSignatures array still open
  uint64_t present = 0;   // template bits of the top-level fields
  bool foreign = false;   // a top-level field outside every template
  uint32_t type_pos = 0;  // TransactionType payload
  uint32_t pos = 0;
  for (;;) {
    if (pos == len) {
      if (depth != 0) return;  // unterminated object / array: re-serialisation adds the marker
      break;
    }
    const uint32_t hpos = pos;
    uint32_t type = b[pos++];
    uint32_t name = type & 15u;
    type >>= 4;
    if (type == 0) {
      if (pos >= len) return;
      type = b[pos++];
      if (type < 16) return;
    }
    if (name == 0) {
      if (pos >= len) return;
      name = b[pos++];
      if (name < 16) return;
    }
    const uint32_t code = (type << 16) | name;
    if ((arrays >> depth) & 1u) {
      // inside an array: an element header (STArray::construct) or the end
      if (code == kCodeArrayEnd) {
        --depth;
        if (depth == 0 && cut_open) {
          cut_open = false;
          if (ncut == 1) t.xe0 = pos;
          else if (ncut == 2) t.xe1 = pos;
          else t.xe2 = pos;
        }
        continue;
      }
      if (!field_declared(type, name) || depth == kBlobMaxDepth) return;
      ++depth;
      arrays &= ~(1u << depth);
      last[depth] = 0;
      continue;
    }
    if (code == kCodeObjectEnd) {
      if (depth == 0) return;  // set() stops at a top-level end marker
      --depth;
      continue;
    }
    if (!field_declared(type, name) || code <= last[depth]) return;
    last[depth] = code;
    if (depth == 0 && format == kFormatTx) {
      const int fb = tx_field_bit(code);
      if (fb < 0) foreign = true;
      else present |= 1ull << fb;
      if (code == 0x10002u) type_pos = pos;
    } else if (depth == 0 && format == kFormatValidation && !validation_field(code)) {
      foreign = true;
    }
    const bool cut = depth == 0 && non_signing_field(code);
    if (cut) {
      // strictly ascending codes: each of the three at most once
      if (ncut == 0) t.xs0 = hpos;
      else if (ncut == 1) t.xs1 = hpos;
      else t.xs2 = hpos;
      ++ncut;
    }
    uint32_t size = fixed_size(type);
    if (type == 6) {  // AMOUNT: native 8 bytes, else 8 + currency + issuer
      if (pos >= len) return;
      size = (b[pos] & 0x80u) ? 48u : 8u;
    } else if (type == 7 || type == 8 || type == 19) {  // VL, ACCOUNT, VECTOR256
      if (pos >= len) return;
      const uint32_t b1 = b[pos++];
      if (b1 <= 192) {
        size = b1;
      } else if (b1 <= 240) {
        if (pos + 1 > len) return;
        size = 193u + (b1 - 193u) * 256u + b[pos];
        pos += 1;
      } else if (b1 <= 254) {
        if (pos + 2 > len) return;
        size = 12481u + (b1 - 241u) * 65536u + (uint32_t)b[pos] * 256u + b[pos + 1];
        pos += 2;
      } else {
        return;
      }
      if (type == 19 && (size & 31u) != 0) return;
      if (depth == 0 && code == kCodeSigningPubKey) {
        t.pk_off = pos;
        t.pk_len = size;
      } else if (depth == 0 && code == sig_code) {
        t.sig_off = pos;
        t.sig_len = size;
      }
    } else if (type == 18) {  // PATHSET
      bool empty = true;
      for (;;) {
        if (pos >= len) return;
        const uint32_t e = b[pos++];
        if (e == 0x00u || e == 0xFFu) {
          if (empty) return;
          if (e == 0x00u) break;
          empty = true;
          continue;
        }
        if (e & ~0x31u) return;
        const uint32_t need = 20u * (((e >> 0) & 1u) + ((e >> 4) & 1u) + ((e >> 5) & 1u));
        if (need > len - pos) return;
        if ((e & 0x01u) && !bytes_nonzero(b, pos, 20)) return;
        if ((e & 0x01u)) pos += 20;
        if ((e & 0x10u)) pos += 20;
        if ((e & 0x20u) && !bytes_nonzero(b, pos, 20)) return;
        if ((e & 0x20u)) pos += 20;
        empty = false;
      }
      size = 0;
    } else if (type == 14 || type == 15) {  // OBJECT, ARRAY
      if (depth == kBlobMaxDepth) return;
      ++depth;
      if (type == 15) arrays |= 1u << depth;
      else arrays &= ~(1u << depth);
      last[depth] = 0;
      if (cut) cut_open = true;  // only TxnSignatures (an array) can be open here
      continue;
    }
    if (size > len - pos) return;
    pos += size;
    if (cut) {
      if (ncut == 1) t.xe0 = pos;
      else if (ncut == 2) t.xe1 = pos;
      else t.xe2 = pos;
    }
  }
  if (format == kFormatValidation && foreign) return;
  if (format == kFormatTx) {
    // the constructor's checks after set(): a blob that fails them never
    // becomes a SerializedTransaction, so the device does not judge it
    uint64_t allowed, required;
    if (!(present & 1ull)) return;
    const uint32_t tt = ((uint32_t)b[type_pos] << 8) | b[type_pos + 1];
    if (foreign || !tx_format(tt, allowed, required)) return;
    if ((present & ~allowed) != 0 || (required & ~present) != 0) return;
  }
  t.status = (t.pk_len == 32u && t.sig_len == 64u) ? kTxOk : kTxMalformed;
}

// Message stream prefix(4 bytes) || blob minus up to three cut ranges, as
// little-endian 32-bit words for SHA-512.  Whole aligned dwords are loaded
// wherever they lie inside the blob; a byte funnel (acc) joins the pieces.
struct SpliceStream {
  const uint8_t* b;
  uint32_t len, pos, total;
  uint32_t xs0, xe0, xs1, xe1, xs2, xe2;
  uint64_t acc;
  uint32_t nb;
  bool done;

  STL_HD void init(const uint8_t* blob, uint32_t n, uint32_t prefix, const TxLayout* t) {
    b = blob;
    len = n;
    pos = 0;
    if (t) {
      xs0 = t->xs0; xe0 = t->xe0; xs1 = t->xs1; xe1 = t->xe1; xs2 = t->xs2; xe2 = t->xe2;
    } else {
      xs0 = xe0 = xs1 = xe1 = xs2 = xe2 = n;
    }
    total = 4u + n - (xe0 - xs0) - (xe1 - xs1) - (xe2 - xs2);
    acc = bswap32(prefix);  // prefix bytes in memory order
    nb = 4;
    done = false;
  }
  // plain global (or host) load of the aligned dword at a
  struct Direct {
    STL_HD uint32_t operator()(const uint8_t* a) const { return *reinterpret_cast<const uint32_t*>(a); }
  };
  template <typename Src>
  STL_HD void fetch(const Src& src) {
    while (pos == xs0 && pos < len) {
      pos = xe0;
      xs0 = xs1; xe0 = xe1;
      xs1 = xs2; xe1 = xe2;
      xs2 = xe2 = len;
    }
    if (pos >= len) {
      done = true;
      return;
    }
    const uint32_t lim = xs0 < len ? xs0 : len;
    const uint32_t sh = (uint32_t)((uintptr_t)(b + pos) & 3u);
    uint32_t k = 4u - sh;
    if (k > lim - pos) k = lim - pos;
    uint32_t v;
    if (pos >= sh && pos - sh + 4u <= len) {
      v = src(b + pos - sh) >> (8u * sh);
    } else {  // the blob's first / last partial dword, byte by byte
      v = 0;
      for (uint32_t i = 0; i < k; ++i) v |= (uint32_t)b[pos + i] << (8u * i);
    }
    if (k < 4) v &= (1u << (8u * k)) - 1u;
    acc |= (uint64_t)v << (8u * nb);
    nb += k;
    pos += k;
  }
  template <typename Src>
  STL_HD uint32_t word(const Src& src) {
    while (nb < 4 && !done) fetch(src);
    const uint32_t w = (uint32_t)acc;
    acc >>= 32;
    nb = nb >= 4 ? nb - 4 : 0;
    return w;
  }
  STL_HD uint32_t blocks() const { return (total + 17u + 127u) / 128u; }
  // next 128-byte block (blocks are consumed in order) with FIPS 180-4 padding
  template <typename Src>
  STL_HD void block(uint64_t w[16], uint32_t blk, bool last, const Src& src) {
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      uint32_t m[2];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        uint32_t v = word(src);
        const int64_t keep = (int64_t)total - (int64_t)(128u * blk + 4u * (2 * j + h));
        if (keep < 4) {
          v = keep <= 0 ? 0u : (v & ((1u << (8 * keep)) - 1u));
          if (keep >= 0) v |= 0x80u << (8 * keep);
        }
        m[h] = v;
      }
      w[j] = be64_from_le32(m[0], m[1]);
    }
    if (last) {
      w[14] = 0;
      w[15] = (uint64_t)total * 8u;
    }
  }
  STL_HD void block(uint64_t w[16], uint32_t blk, bool last) { block(w, blk, last, Direct{}); }
  // blob address of the next byte the stream will read (window placement)
  STL_HD const uint8_t* cursor() const { return b + (pos == xs0 && pos < len ? xe0 : pos); }
  STL_HD const uint8_t* end() const { return b + len; }
};

// Block blk of a one-cut signing preimage, prefix || blob[0, xs) ||
// blob[xe, len) -- every STL_TX_OK transaction or validation has exactly one
// cut, its signature field -- as 16 big-endian words with the FIPS 180-4
// padding, assembled word by word: a preimage word at byte P comes from the
// blob at P - 4 (before the cut) or P - 4 + (xe - xs) (after it), one
// unaligned dword each (two aligned dwords and a v_alignbyte), the word that
// straddles the cut from both.  src(q) returns the aligned blob dword at q
// (the kernel's LDS window, global loads outside it); dwords wholly outside
// the blob are never asked for.  Same words as SpliceStream, without its byte
// funnel (tests/test_txblob.py compares the two on random layouts).
template <typename Src>
STL_HD void splice1_words(uint32_t m[32], const uint8_t* b, uint32_t len, uint32_t xs, uint32_t xe,
                          uint32_t prefix_le, uint32_t blk, const Src& src) {
  const uint32_t cut = xe - xs, total = 4u + len - cut, pb = 4u + xs;
  const uintptr_t lo = (uintptr_t)b, hi = lo + len;
  auto dw = [&](uintptr_t q) -> uint32_t {  // aligned dword q, 0 outside the blob
    return (q + 4u <= lo || q >= hi) ? 0u : src(reinterpret_cast<const uint8_t*>(q));
  };
  auto udw = [&](uintptr_t a) -> uint32_t {  // dword at byte address a (any alignment)
    const uintptr_t q = a & ~(uintptr_t)3;
    return align_byte(dw(q + 4u), dw(q), (uint32_t)(a & 3u));
  };
#pragma unroll
  for (int i = 0; i < 32; ++i) {
    {
      const uint32_t P = 128u * blk + 4u * (uint32_t)i;
      uint32_t v;
      if (P == 0) {
        v = prefix_le;
      } else {
        const int32_t k = (int32_t)pb - (int32_t)P;  // bytes of this word before the cut
        v = udw(lo + P - 4u + (k > 0 ? 0u : cut));
        if (k > 0 && k < 4) {
          const uint32_t mk = (1u << (8 * k)) - 1u;
          v = (v & mk) | (udw(lo + P - 4u + cut) & ~mk);
        }
      }
      const int32_t r = (int32_t)total - (int32_t)P;  // preimage bytes from this word on
      const int32_t rc = r < 0 ? 0 : (r > 4 ? 4 : r);
      const uint32_t keep = rc == 4 ? 0xffffffffu : ((1u << (8 * rc)) - 1u);
      const uint32_t pad = (r >= 0 && r < 4) ? (0x80u << (8 * rc)) : 0u;
      m[i] = (v & keep) | pad;
    }
  }
}

// The same block as 16 big-endian words, with the length in the final block.
template <typename Src>
STL_HD void splice1_block(uint64_t w[16], const uint8_t* b, uint32_t len, uint32_t xs, uint32_t xe,
                          uint32_t prefix_le, uint32_t blk, bool last, const Src& src) {
  uint32_t m[32];
  splice1_words(m, b, len, xs, xe, prefix_le, blk, src);
#pragma unroll
  for (int j = 0; j < 16; ++j) w[j] = be64_from_le32(m[2 * j], m[2 * j + 1]);
  if (last) {
    w[14] = 0;
    w[15] = (uint64_t)(4u + len - (xe - xs)) * 8u;
  }
}

// n little-endian words from blob bytes [off, off + 4n) (off unaligned).
STL_HD void blob_words(uint32_t* out, const uint8_t* b, uint32_t off, uint32_t n, uint32_t len) {
  const uint32_t sh = (uint32_t)((uintptr_t)(b + off) & 3u);
  if (off >= sh && (uint64_t)(off - sh) + 4ull * (n + (sh ? 1u : 0u)) <= (uint64_t)len) {
    const uint32_t* q = reinterpret_cast<const uint32_t*>(b + off - sh);
    if (sh == 0) {
      for (uint32_t i = 0; i < n; ++i) out[i] = q[i];
    } else {
      for (uint32_t i = 0; i < n; ++i) out[i] = align_byte(q[i + 1], q[i], sh);
    }
  } else {
    for (uint32_t i = 0; i < n; ++i)
      out[i] = (uint32_t)b[off + 4 * i] | ((uint32_t)b[off + 4 * i + 1] << 8) |
               ((uint32_t)b[off + 4 * i + 2] << 16) | ((uint32_t)b[off + 4 * i + 3] << 24);
  }
}

// SHA512Half of a one-cut preimage through splice1_block (host tests).
STL_HD void splice1_sha512_half(uint32_t out[8], const uint8_t* blob, uint32_t len, uint32_t prefix, uint32_t xs,
                                uint32_t xe) {
  const uint32_t total = 4u + len - (xe - xs), nb = (total + 17u + 127u) / 128u;
  uint64_t st[8], w[16];
  sha512_init(st);
  const uint32_t prefix_le = bswap32(prefix);
  for (uint32_t k = 0; k < nb; ++k) {
    splice1_block(w, blob, len, xs, xe, prefix_le, k, k + 1 == nb,
                  [](const uint8_t* q) { return *reinterpret_cast<const uint32_t*>(q); });
    sha512_compress(st, w);
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    out[2 * j] = bswap32((uint32_t)(st[j] >> 32));
    out[2 * j + 1] = bswap32((uint32_t)st[j]);
  }
}

// Host-side / test convenience: the whole per-blob computation in one call.
STL_HD void splice_sha512_half(uint32_t out[8], const uint8_t* blob, uint32_t len, uint32_t prefix,
                               const TxLayout* t) {
  SpliceStream s;
  s.init(blob, len, prefix, t);
  uint64_t st[8], w[16];
  sha512_init(st);
  const uint32_t nb = s.blocks();
  for (uint32_t k = 0; k < nb; ++k) {
    s.block(w, k, k + 1 == nb);
    sha512_compress(st, w);
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    out[2 * j] = bswap32((uint32_t)(st[j] >> 32));
    out[2 * j + 1] = bswap32((uint32_t)st[j]);
  }
}

}  // namespace stl
