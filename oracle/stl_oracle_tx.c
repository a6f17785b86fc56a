/*
 * stl_oracle_tx.c -- CPU restatement of stellard's transaction
 * deserialisation and re-serialisation, the checker for libstl's
 * serialized-transaction path (stl_tx_blob_*).
 *
 * TEST INFRASTRUCTURE ONLY (see stl_oracle.h): used by tests/ and the
 * reference harness, never by the product.
 *
 * Unlike the device path, which splices the signing preimage out of a blob it
 * has checked to be canonical, this file does what the reference does: parse
 * every field into a value and serialise the values again.
 *   SerializedTransaction(SerializerIterator&)   SerializedTransaction.cpp:65-92
 *   STObject::set / makeDeserializedObject       SerializedObject.cpp:85-136, 266-306
 *   SerializerIterator::getFieldID                Serializer.cpp:226-262, 586-598
 *   SField::getField (declared + dynamic fields)  FieldNames.cpp:76-111
 *   getVL / decodeVLLength / encodeVL             Serializer.cpp:415-575
 *   STAmount::construct / add                     STAmount.cpp:465-560
 *   STVector256::construct                        SerializedTypes.cpp:374-400
 *   STPathSet::construct / add, STPathElement     SerializedTypes.cpp:465-518, 636-666;
 *                                                 SerializedTypes.h:1166-1187
 *   STArray::construct / add                      SerializedObject.cpp:1208-1256
 *   STObject::add (sorted by fieldCode via std::map, first duplicate kept)
 *                                                 SerializedObject.cpp:353-379
 *   signing fields (TxnSignature, TxnSignatures, Signature not signing)
 *                                                 FieldNames.cpp:49-51, FieldNames.h:213-216
 *   getSigningHash / getTransactionID             SerializedObject.cpp:444-450,
 *                                                 SerializedTransaction.cpp:162-171
 *   validations (kind 1): SerializedValidation(SerializerIterator&) and
 *   isValid(getSigningHash()) -- "VAL\0" prefix, SigningPubKey / Signature
 *                                                 SerializedValidation.cpp:22-34,70-73,96-110,
 *                                                 HashPrefix.cpp:31; suppression
 *                                                 id SHA512Half(raw), PeerImp.cpp:1134,1148-1155
 *   transactions: TransactionType present, a TxFormats template for it, and
 *   setType's required / leftover checks   SerializedTransaction.cpp:79-91,
 *                                          TxFormats.cpp:22-130,
 *                                          SerializedObject.cpp:152-207,661-675
 * Duplicate top-level fields are rejected as setType would reject them (the
 * second one is a leftover).
 */
#include <pthread.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include "stl_oracle.h"

/* The batch checker below is built twice: into liboracle.so over the C
 * restatement, and (-DSTL_TX_REF) into _ref/libsodium_ref.so over libsodium's
 * crypto_sign_verify_detached and OpenSSL's SHA-512, as ref_tx_blob_verify_batch. */
#ifdef STL_TX_REF
#include <openssl/sha.h>
int ref_verify_signature(const unsigned char *sig, const unsigned char *hash32, const unsigned char *pk);
#define TX_SHA512(in, n, out) SHA512((in), (n), (out))
#define TX_VERIFY(sig, h, pk, policy) (ref_verify_signature((sig), (h), (pk)) == 1) /* 1 accept */
#define TX_BATCH_NAME ref_tx_blob_verify_batch
#define KIND_BATCH_NAME ref_signed_blob_verify_batch
#else
#define TX_SHA512(in, n, out) oracle_sha512((in), (n), (out))
#define TX_VERIFY(sig, h, pk, policy) (oracle_verify((sig), (h), 32, (pk), (policy)) == 0)
#define TX_BATCH_NAME oracle_tx_blob_verify_batch
#define KIND_BATCH_NAME oracle_signed_blob_verify_batch
#endif

/* ---------------------------------------------------------------- buffers */
typedef struct {
  uint8_t *p;
  size_t n, cap;
} buf_t;

static void buf_put(buf_t *b, const uint8_t *src, size_t n) {
  if (b->n + n > b->cap) {
    size_t c = b->cap ? b->cap : 256;
    while (c < b->n + n) c *= 2;
    b->p = (uint8_t *)realloc(b->p, c);
    b->cap = c;
  }
  memcpy(b->p + b->n, src, n);
  b->n += n;
}
static void buf_u8(buf_t *b, unsigned v) {
  uint8_t c = (uint8_t)v;
  buf_put(b, &c, 1);
}

/* Serializer::addFieldID (Serializer.cpp:193-220) */
static void put_field_id(buf_t *b, int type, int name) {
  if (type < 16) {
    if (name < 16) {
      buf_u8(b, (unsigned)((type << 4) | name));
    } else {
      buf_u8(b, (unsigned)(type << 4));
      buf_u8(b, (unsigned)name);
    }
  } else if (name < 16) {
    buf_u8(b, (unsigned)name);
    buf_u8(b, (unsigned)type);
  } else {
    buf_u8(b, 0);
    buf_u8(b, (unsigned)type);
    buf_u8(b, (unsigned)name);
  }
}

/* Serializer::encodeVL (Serializer.cpp:496-521) */
static void put_vl(buf_t *b, size_t len) {
  if (len <= 192) {
    buf_u8(b, (unsigned)len);
  } else if (len <= 12480) {
    len -= 193;
    buf_u8(b, (unsigned)(193 + (len >> 8)));
    buf_u8(b, (unsigned)(len & 0xff));
  } else {
    len -= 12481;
    buf_u8(b, (unsigned)(241 + (len >> 16)));
    buf_u8(b, (unsigned)((len >> 8) & 0xff));
    buf_u8(b, (unsigned)(len & 0xff));
  }
}

/* ---------------------------------------------------------------- reader */
typedef struct {
  const uint8_t *b;
  size_t len, pos;
  int err;         /* a reference constructor would have thrown */
  int all_declared;
  int max_depth;
} rd_t;

static int rd_empty(const rd_t *r) { return r->pos >= r->len; }
static unsigned rd_u8(rd_t *r) {
  if (r->pos >= r->len) {
    r->err = 1;
    return 0;
  }
  return r->b[r->pos++];
}
static const uint8_t *rd_raw(rd_t *r, size_t n) {
  if (n > r->len - r->pos) {
    r->err = 1;
    return NULL;
  }
  const uint8_t *p = r->b + r->pos;
  r->pos += n;
  return p;
}

/* Serializer::getFieldID (Serializer.cpp:226-262) */
static void rd_field_id(rd_t *r, int *type, int *name) {
  unsigned t = rd_u8(r);
  unsigned nm = t & 15u;
  t >>= 4;
  if (!r->err && t == 0) {
    t = rd_u8(r);
    if (t < 16) r->err = 1;
  }
  if (!r->err && nm == 0) {
    nm = rd_u8(r);
    if (nm < 16) r->err = 1;
  }
  *type = (int)t;
  *name = (int)nm;
}

/* Serializer::getVL (Serializer.cpp:415-454) */
static size_t rd_vl_len(rd_t *r) {
  unsigned b1 = rd_u8(r);
  if (r->err) return 0;
  if (b1 <= 192) return b1;
  if (b1 <= 240) {
    unsigned b2 = rd_u8(r);
    return 193 + (b1 - 193) * 256 + b2;
  }
  if (b1 <= 254) {
    unsigned b2 = rd_u8(r), b3 = rd_u8(r);
    return 12481 + (b1 - 241) * 65536 + b2 * 256 + b3;
  }
  r->err = 1;
  return 0;
}

/* Declared fields (SerializeDeclarations.h). */
static int field_declared(int type, int name) {
  static const struct {
    int type, lo, hi;
  } R[] = {{1, 1, 2},   {2, 2, 14},  {2, 16, 34}, {3, 1, 8},   {4, 1, 1},   {5, 1, 9},  {5, 16, 19},
           {6, 1, 9},   {6, 16, 18}, {7, 1, 13},  {8, 1, 4},   {8, 7, 10},  {14, 2, 10}, {15, 2, 9},
           {16, 1, 3},  {17, 1, 4},  {18, 1, 1},  {19, 1, 3}};
  for (size_t i = 0; i < sizeof R / sizeof R[0]; ++i)
    if (R[i].type == type && name >= R[i].lo && name <= R[i].hi) return 1;
  return 0;
}

/* SField::notSigningField (FieldNames.cpp:49-51): TxnSignature, TxnSignatures,
 * Signature are left out of STObject::add(s, false). */
static int non_signing(uint32_t code) { return code == 0x70004u || code == 0x70006u || code == 0xF0003u; }

static int type_known(int type) { return (type >= 1 && type <= 8) || (type >= 14 && type <= 19); }

/* SField::getField(type, name) (FieldNames.cpp:76-111): declared fields, or a
 * field created on the fly for a known type.  The reference computes
 * field = code % 0xffff = type + name and refuses values above 255. */
static int field_valid(rd_t *r, int type, int name) {
  if (field_declared(type, name)) return 1;
  r->all_declared = 0;
  return type_known(type) && name >= 1 && type + name <= 255;
}

/* --------------------------------------------------------------- objects */
typedef struct {
  uint32_t code;
  int signing;
  buf_t ser; /* field id + value */
} fld_t;

typedef struct {
  fld_t *f;
  size_t n, cap;
} flist_t;

static void flist_free(flist_t *l) {
  for (size_t i = 0; i < l->n; ++i) free(l->f[i].ser.p);
  free(l->f);
  l->f = NULL;
  l->n = l->cap = 0;
}

static int parse_object(rd_t *r, int depth, flist_t *out);

/* STObject::add: fields sorted by fieldCode through std::map::insert (the
 * first of equal codes wins), non-signing fields left out unless asked. */
static void add_sorted(flist_t *l, buf_t *out, int with_signing) {
  /* stable: sort indices by (code, original position) */
  size_t n = l->n;
  size_t *idx = (size_t *)malloc((n ? n : 1) * sizeof(size_t));
  for (size_t i = 0; i < n; ++i) idx[i] = i;
  for (size_t i = 1; i < n; ++i) { /* insertion sort: lists are short */
    size_t v = idx[i], j = i;
    while (j > 0 && l->f[idx[j - 1]].code > l->f[v].code) {
      idx[j] = idx[j - 1];
      --j;
    }
    idx[j] = v;
  }
  uint32_t prev = 0xffffffffu;
  for (size_t i = 0; i < n; ++i) {
    const fld_t *f = &l->f[idx[i]];
    if (f->code == prev) continue;
    prev = f->code;
    if (!with_signing && !f->signing) continue;
    buf_put(out, f->ser.p, f->ser.n);
  }
  free(idx);
}

static int has_duplicates(const flist_t *l) {
  for (size_t i = 0; i < l->n; ++i)
    for (size_t j = i + 1; j < l->n; ++j)
      if (l->f[i].code == l->f[j].code) return 1;
  return 0;
}

static int nonzero(const uint8_t *p, size_t n) {
  for (size_t i = 0; i < n; ++i)
    if (p[i]) return 1;
  return 0;
}

/* makeDeserializedObject + the type's construct(), re-serialised by add(). */
static void parse_value(rd_t *r, int type, int depth, buf_t *o) {
  switch (type) {
    case 16: case 1: case 2: case 3: case 4: case 17: case 5: {
      static const int sz[20] = {0, 2, 4, 8, 16, 32, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 1, 20, 0, 0};
      const uint8_t *p = rd_raw(r, (size_t)sz[type]);
      if (p) buf_put(o, p, (size_t)sz[type]);
      return;
    }
    case 6: { /* STAmount::construct (STAmount.cpp:532-560) then add (:465-488) */
      const uint8_t *p = rd_raw(r, 8);
      if (!p) return;
      uint64_t v = 0;
      for (int i = 0; i < 8; ++i) v = (v << 8) | p[i];
      const uint64_t kNotNative = 0x8000000000000000ull, kPosNative = 0x4000000000000000ull;
      uint64_t outv;
      if ((v & kNotNative) == 0) {
        if (v & kPosNative) {
          outv = (v & ~kPosNative) | kPosNative;
        } else if (v == 0) {
          r->err = 1; /* negative zero is not canonical */
          return;
        } else {
          outv = v;
        }
        uint8_t be[8];
        for (int i = 0; i < 8; ++i) be[i] = (uint8_t)(outv >> (56 - 8 * i));
        buf_put(o, be, 8);
        return;
      }
      const uint8_t *cur = rd_raw(r, 20);
      if (!cur) return;
      if (!nonzero(cur, 20)) {
        r->err = 1; /* invalid non-native currency */
        return;
      }
      const uint8_t *iss = rd_raw(r, 20);
      if (!iss) return;
      int offset = (int)(v >> 54);
      uint64_t value = v & ~(1023ull << 54);
      if (value) {
        const int neg = (offset & 256) == 0;
        offset = (offset & 255) - 97;
        if (value < 1000000000000000ull || value > 9999999999999999ull || offset < -96 || offset > 80) {
          r->err = 1;
          return;
        }
        outv = value | ((uint64_t)(offset + 512 + (neg ? 0 : 256) + 97) << 54);
      } else {
        if (offset != 512) {
          r->err = 1;
          return;
        }
        outv = kNotNative;
      }
      uint8_t be[8];
      for (int i = 0; i < 8; ++i) be[i] = (uint8_t)(outv >> (56 - 8 * i));
      buf_put(o, be, 8);
      buf_put(o, cur, 20);
      buf_put(o, iss, 20);
      return;
    }
    case 7: case 8: { /* STVariableLength / STAccount: getVL, addVL */
      size_t n = rd_vl_len(r);
      const uint8_t *p = r->err ? NULL : rd_raw(r, n);
      if (!p) return;
      put_vl(o, n);
      buf_put(o, p, n);
      return;
    }
    case 19: { /* STVector256::construct keeps whole 32-byte entries */
      size_t n = rd_vl_len(r);
      const uint8_t *p = r->err ? NULL : rd_raw(r, n);
      if (!p) return;
      size_t keep = (n / 32) * 32;
      put_vl(o, keep);
      buf_put(o, p, keep);
      return;
    }
    case 18: { /* STPathSet */
      buf_t paths = {0};
      int path_len = 0, first = 1;
      buf_t cur = {0};
      for (;;) {
        unsigned e = rd_u8(r);
        if (r->err) break;
        if (e == 0x00 || e == 0xFF) {
          if (path_len == 0) {
            r->err = 1; /* empty path */
            break;
          }
          if (!first) buf_u8(&paths, 0xFF);
          buf_put(&paths, cur.p, cur.n);
          cur.n = 0;
          path_len = 0;
          first = 0;
          if (e == 0x00) break;
          continue;
        }
        if (e & ~0x31u) {
          r->err = 1; /* bad path element */
          break;
        }
        const uint8_t *acc = NULL, *ccy = NULL, *iss = NULL;
        static const uint8_t zero20[20] = {0};
        if (e & 0x01) acc = rd_raw(r, 20);
        if (e & 0x10) ccy = rd_raw(r, 20);
        if (e & 0x20) iss = rd_raw(r, 20);
        if (r->err) break;
        if (!acc) acc = zero20;
        if (!ccy) ccy = zero20;
        if (!iss) iss = zero20;
        unsigned t = (nonzero(acc, 20) ? 0x01u : 0) | ((nonzero(ccy, 20) || (e & 0x10)) ? 0x10u : 0) |
                     (nonzero(iss, 20) ? 0x20u : 0);
        buf_u8(&cur, t);
        if (t & 0x01) buf_put(&cur, acc, 20);
        if (t & 0x10) buf_put(&cur, ccy, 20);
        if (t & 0x20) buf_put(&cur, iss, 20);
        ++path_len;
      }
      if (!r->err) {
        buf_put(o, paths.p, paths.n);
        buf_u8(o, 0x00);
      }
      free(paths.p);
      free(cur.p);
      return;
    }
    case 14: { /* STObject::deserialize: set(sit, 1), add() + end marker */
      flist_t inner = {0};
      parse_object(r, depth + 1, &inner);
      if (!r->err) {
        add_sorted(&inner, o, 1);
        put_field_id(o, 14, 1);
      }
      flist_free(&inner);
      return;
    }
    case 15: { /* STArray::construct / add */
      if (depth + 1 > r->max_depth) r->max_depth = depth + 1;
      while (!rd_empty(r) && !r->err) {
        int t, nm;
        rd_field_id(r, &t, &nm);
        if (r->err) break;
        if (t == 15 && nm == 1) break;
        if (!field_valid(r, t, nm)) {
          r->err = 1;
          break;
        }
        flist_t inner = {0};
        parse_object(r, depth + 2, &inner);
        if (!r->err) {
          put_field_id(o, t, nm);
          add_sorted(&inner, o, 1);
          put_field_id(o, 14, 1);
        }
        flist_free(&inner);
      }
      if (!r->err) put_field_id(o, 15, 1);
      return;
    }
    default:
      r->err = 1; /* Unknown object type */
      return;
  }
}

/* STObject::set: returns 1 when it stopped at an object end marker. */
static int parse_object(rd_t *r, int depth, flist_t *out) {
  if (depth > r->max_depth) r->max_depth = depth;
  if (depth > 200) {
    r->err = 1;
    return 0;
  }
  while (!rd_empty(r) && !r->err) {
    int type, name;
    rd_field_id(r, &type, &name);
    if (r->err) return 0;
    if (type == 14 && name == 1) return 1;
    if (!field_valid(r, type, name)) {
      r->err = 1;
      return 0;
    }
    if (out->n == out->cap) {
      out->cap = out->cap ? 2 * out->cap : 16;
      out->f = (fld_t *)realloc(out->f, out->cap * sizeof(fld_t));
    }
    fld_t *f = &out->f[out->n];
    memset(f, 0, sizeof *f);
    f->code = ((uint32_t)type << 16) | (uint32_t)name;
    f->signing = !non_signing(f->code);
    put_field_id(&f->ser, type, name);
    out->n++;
    parse_value(r, type, depth, &out->f[out->n - 1].ser);
  }
  return 0;
}

/* top-level payload of a VL field in a parsed list (first occurrence) */
static long vl_payload(const flist_t *l, uint32_t code, uint8_t *dst, size_t cap) {
  for (size_t i = 0; i < l->n; ++i) {
    if (l->f[i].code != code) continue;
    rd_t r = {l->f[i].ser.p, l->f[i].ser.n, 0, 0, 1, 0};
    int t, nm;
    rd_field_id(&r, &t, &nm);
    size_t n = rd_vl_len(&r);
    if (r.err || n > r.len - r.pos) return -1;
    memcpy(dst, r.b + r.pos, n < cap ? n : cap);
    return (long)n;
  }
  return -1;
}

/* TxFormats (TxFormats.cpp:22-111; addCommonFields :113-130): per TxType the
 * template's fields with their SOElement flags. */
enum { SOE_REQ = 0, SOE_OPT = 1, SOE_DEF = 2 };
typedef struct {
  uint32_t code;
  int flags;
} soe_t;
static const soe_t kCommonFields[] = {
    {0x10002u, SOE_REQ}, /* TransactionType */
    {0x20002u, SOE_OPT}, /* Flags */
    {0x20003u, SOE_OPT}, /* SourceTag */
    {0x80001u, SOE_REQ}, /* Account */
    {0x20004u, SOE_REQ}, /* Sequence */
    {0x50005u, SOE_OPT}, /* PreviousTxnID */
    {0x2001Bu, SOE_OPT}, /* LastLedgerSequence */
    {0x50009u, SOE_OPT}, /* AccountTxnID */
    {0x60008u, SOE_REQ}, /* Fee */
    {0x2001Du, SOE_OPT}, /* OperationLimit */
    {0xF0009u, SOE_OPT}, /* Memos */
    {0x70003u, SOE_REQ}, /* SigningPubKey */
    {0x70004u, SOE_OPT}, /* TxnSignature */
};
typedef struct {
  int type;
  soe_t f[6];
  int n;
} txformat_t;
static const txformat_t kTxFormats[] = {
    {3, {{0x2000Bu, SOE_OPT}, {0x20021u, SOE_OPT}, {0x20022u, SOE_OPT}, {0x80009u, SOE_OPT}, {0x8000Au, SOE_OPT}}, 5},
    {4, {{0x80003u, SOE_REQ}, {0x2000Eu, SOE_OPT}}, 2},                                        /* AccountMerge */
    {20, {{0x60003u, SOE_OPT}, {0x20014u, SOE_OPT}, {0x20015u, SOE_OPT}}, 3},                  /* TrustSet */
    {7, {{0x60004u, SOE_REQ}, {0x60005u, SOE_REQ}, {0x2000Au, SOE_OPT}, {0x20019u, SOE_OPT}}, 4}, /* OfferCreate */
    {8, {{0x20019u, SOE_REQ}}, 1},                                                             /* OfferCancel */
    {5, {{0x80008u, SOE_OPT}}, 1},                                                             /* SetRegularKey */
    {0,
     {{0x80003u, SOE_REQ}, {0x60001u, SOE_REQ}, {0x60009u, SOE_OPT}, {0x120001u, SOE_DEF}, {0x50011u, SOE_OPT},
      {0x2000Eu, SOE_OPT}},
     6},                                                                                       /* Payment */
    {1, {{0x2001Au, SOE_REQ}}, 1},                                                             /* Inflation */
    {100, {{0x50013u, SOE_REQ}}, 1},                                                           /* EnableAmendment */
    {101, {{0x30005u, SOE_REQ}, {0x2001Eu, SOE_REQ}, {0x2001Fu, SOE_REQ}, {0x20020u, SOE_REQ}}, 4}, /* SetFee */
};

/* one template element against the parsed list: SerializedObject.cpp:159-191 */
static int soe_ok(const flist_t *l, const soe_t *e, uint8_t *used) {
  for (size_t i = 0; i < l->n; ++i) {
    if (used[i] || l->f[i].code != e->code) continue;
    used[i] = 1;
    /* SOE_DEFAULT present at its default: only sfPaths is SOE_DEFAULT, and an
     * empty STPathSet cannot be deserialised (parse_value: "empty path") */
    return 1;
  }
  return e->flags != SOE_REQ;
}

/* SerializedTransaction(SerializerIterator&) after set(): getFieldU16
 * (SerializedObject.cpp:661-675), findByType, setType (SerializedObject.cpp:
 * 152-207).  Leftover fields are never discardable: fieldValue is the wire
 * name byte, at most 255 (FieldNames.h:178-181). */
static int tx_template_ok(const flist_t *top) {
  const fld_t *tf = NULL;
  for (size_t i = 0; i < top->n && !tf; ++i)
    if (top->f[i].code == 0x10002u) tf = &top->f[i];
  if (!tf || tf->ser.n != 3) return 0; /* "Field not found" */
  const int type = (tf->ser.p[1] << 8) | tf->ser.p[2];
  const txformat_t *fmt = NULL;
  for (size_t i = 0; i < sizeof kTxFormats / sizeof kTxFormats[0]; ++i)
    if (kTxFormats[i].type == type) fmt = &kTxFormats[i];
  if (!fmt) return 0; /* "invalid transaction type" */
  uint8_t *used = (uint8_t *)calloc(top->n ? top->n : 1, 1);
  int ok = 1;
  for (size_t i = 0; i < sizeof kCommonFields / sizeof kCommonFields[0]; ++i) ok &= soe_ok(top, &kCommonFields[i], used);
  for (int i = 0; i < fmt->n; ++i) ok &= soe_ok(top, &fmt->f[i], used);
  for (size_t i = 0; i < top->n; ++i) ok &= used[i]; /* "invalid leftover" */
  free(used);
  return ok;
}

/* SerializedValidation's template (SerializedValidation.cpp:134-159).  Its
 * constructor, STObject(getFormat(), sit, sfValidation), calls setType and
 * ignores the result (SerializedObject.h:54-58): fields outside the template
 * are dropped from the object (setType keeps only newData), so they are in
 * neither the signing hash nor a re-serialisation; missing ones are simply
 * absent. */
static const uint32_t kValidationFields[] = {0x20002u,  0x50001u, 0x20006u, 0x20007u, 0x20018u, 0x130003u,
                                             0x30005u,  0x2001Fu, 0x20020u, 0x20009u, 0x70003u, 0x70006u};

static void validation_set_type(flist_t *top) {
  size_t k = 0;
  for (size_t i = 0; i < top->n; ++i) {
    int keep = 0;
    for (size_t j = 0; j < sizeof kValidationFields / sizeof kValidationFields[0]; ++j)
      keep |= top->f[i].code == kValidationFields[j];
    if (keep) {
      top->f[k++] = top->f[i];
    } else {
      free(top->f[i].ser.p);
    }
  }
  top->n = k;
}

int oracle_signed_blob(uint32_t kind, const uint8_t *blob, size_t len, uint8_t *signing, uint8_t *full,
                       size_t cap, oracle_txinfo *info) {
  memset(info, 0, sizeof *info);
  info->pk_len = info->sig_len = -1;
  if (kind > 1) return -1;
  /* transactions: SerializedTransaction.cpp:68-74; validations: PeerImp.cpp:1134 */
  if (len < (kind == 0 ? 32u : 50u) || len > 1024 * 1024) return -1;
  rd_t r = {blob, len, 0, 0, 1, 0};
  flist_t top = {0};
  info->stopped_early = parse_object(&r, 0, &top) && r.pos < len ? 1 : 0;
  int rc = 0;
  /* a duplicate is a setType leftover: fatal for a transaction, dropped for a
   * validation (validation_set_type keeps both, add_sorted the first) */
  if (r.err || (kind == 0 && has_duplicates(&top))) rc = -1;
  if (kind == 0 && rc == 0 && !tx_template_ok(&top)) rc = -1;
  if (kind == 1 && rc == 0) validation_set_type(&top);
  info->all_declared = r.all_declared;
  info->max_depth = r.max_depth;
  if (rc == 0) {
    buf_t s = {0}, f = {0};
    const uint8_t pfx_tx[4] = {'S', 'T', 'X', 0}, pfx_val[4] = {'V', 'A', 'L', 0};
    buf_put(&s, kind == 0 ? pfx_tx : pfx_val, 4);
    add_sorted(&top, &s, 0);
    add_sorted(&top, &f, 1);
    if (s.n > cap || f.n > cap) {
      rc = -1;
    } else {
      memcpy(signing, s.p, s.n);
      memcpy(full, f.p, f.n);
      info->signing_len = s.n;
      info->full_len = f.n;
    }
    free(s.p);
    free(f.p);
    info->pk_len = vl_payload(&top, 0x70003u, info->pk, sizeof info->pk);
    /* TxnSignature (checkSign) or Signature (SerializedValidation::isValid) */
    info->sig_len = vl_payload(&top, kind == 0 ? 0x70004u : 0x70006u, info->sig, sizeof info->sig);
  }
  flist_free(&top);
  return rc;
}

int oracle_tx_blob(const uint8_t *blob, size_t len, uint8_t *signing, uint8_t *full, size_t cap,
                   oracle_txinfo *info) {
  return oracle_signed_blob(0, blob, len, signing, full, cap, info);
}

/* ---------------------------------------------------------------- batch */
typedef struct {
  const uint8_t *blobs;
  const uint64_t *off;
  const uint32_t *len;
  size_t lo, hi;
  uint8_t *bits; /* one byte per tx */
  uint8_t *tx_id;
  uint32_t policy;
  uint32_t kind;
} blob_job_t;

static void *blob_worker(void *arg) {
  blob_job_t *j = (blob_job_t *)arg;
  size_t cap = 1 << 16;
  uint8_t *s = (uint8_t *)malloc(cap), *f = (uint8_t *)malloc(cap);
  for (size_t i = j->lo; i < j->hi; ++i) {
    const size_t n = j->len[i];
    if (n + 64 > cap) {
      cap = n + 64;
      s = (uint8_t *)realloc(s, cap);
      f = (uint8_t *)realloc(f, cap);
    }
    oracle_txinfo info;
    uint8_t ok = 0;
    uint8_t h[64];
    if (oracle_signed_blob(j->kind, j->blobs + j->off[i], n, s, f, cap, &info) == 0) {
      if (info.pk_len == 32 && info.sig_len == 64) {
        TX_SHA512(s, info.signing_len, h);
        ok = TX_VERIFY(info.sig, h, info.pk, j->policy) ? 1 : 0;
      }
      if (j->tx_id && j->kind == 0) {
        uint8_t *t = (uint8_t *)malloc(info.full_len + 4);
        t[0] = 'T'; t[1] = 'X'; t[2] = 'N'; t[3] = 0;
        memcpy(t + 4, f, info.full_len);
        TX_SHA512(t, info.full_len + 4, h);
        memcpy(j->tx_id + 32 * i, h, 32);
        free(t);
      } else if (j->tx_id) { /* validation suppression id: the raw bytes */
        TX_SHA512(j->blobs + j->off[i], n, h);
        memcpy(j->tx_id + 32 * i, h, 32);
      }
    } else if (j->tx_id) {
      memset(j->tx_id + 32 * i, 0, 32);
    }
    j->bits[i] = ok;
  }
  free(s);
  free(f);
  return NULL;
}

void KIND_BATCH_NAME(uint32_t kind, const uint8_t *blobs, const uint64_t *offset, const uint32_t *len, size_t n,
                     uint8_t *bitmap, uint8_t *tx_id, uint32_t policy, int threads);

void TX_BATCH_NAME(const uint8_t *blobs, const uint64_t *offset, const uint32_t *len, size_t n,
                                 uint8_t *bitmap, uint8_t *tx_id, uint32_t policy, int threads) {
  KIND_BATCH_NAME(0, blobs, offset, len, n, bitmap, tx_id, policy, threads);
}

void KIND_BATCH_NAME(uint32_t kind, const uint8_t *blobs, const uint64_t *offset, const uint32_t *len, size_t n,
                     uint8_t *bitmap, uint8_t *tx_id, uint32_t policy, int threads) {
  if (threads < 1) threads = (int)sysconf(_SC_NPROCESSORS_ONLN);
  if (threads < 1) threads = 1;
  uint8_t *bits = (uint8_t *)calloc(n ? n : 1, 1);
  pthread_t th[64];
  blob_job_t jobs[64];
  if (threads > 64) threads = 64;
  for (int t = 0; t < threads; ++t) {
    jobs[t].blobs = blobs;
    jobs[t].off = offset;
    jobs[t].len = len;
    jobs[t].lo = n * (size_t)t / (size_t)threads;
    jobs[t].hi = n * (size_t)(t + 1) / (size_t)threads;
    jobs[t].bits = bits;
    jobs[t].tx_id = tx_id;
    jobs[t].policy = policy;
    jobs[t].kind = kind;
    pthread_create(&th[t], NULL, blob_worker, &jobs[t]);
  }
  for (int t = 0; t < threads; ++t) pthread_join(th[t], NULL);
  memset(bitmap, 0, (n + 7) / 8);
  for (size_t i = 0; i < n; ++i)
    if (bits[i]) bitmap[i >> 3] |= (uint8_t)(1u << (i & 7));
  free(bits);
}

/* ---- table accessors (tests/test_sfields.py pins them to the reference's
 * own text, tests/golden/sfields.json) ---- */
int oracle_table_declared(int type, int name) { return field_declared(type, name); }
int oracle_table_non_signing(uint32_t code) { return non_signing(code); }

/* The TxFormats template of TxType `type`: common fields then the type's own,
 * (code, SOE flag 0 required / 1 optional / 2 default); the count, or -1 for a
 * type with no format. */
int oracle_table_tx_format(int type, uint32_t *codes, int *flags, int cap) {
  const txformat_t *fmt = NULL;
  for (size_t i = 0; i < sizeof kTxFormats / sizeof kTxFormats[0]; ++i)
    if (kTxFormats[i].type == type) fmt = &kTxFormats[i];
  if (!fmt) return -1;
  int k = 0;
  for (size_t i = 0; i < sizeof kCommonFields / sizeof kCommonFields[0]; ++i, ++k)
    if (k < cap) codes[k] = kCommonFields[i].code, flags[k] = kCommonFields[i].flags;
  for (int i = 0; i < fmt->n; ++i, ++k)
    if (k < cap) codes[k] = fmt->f[i].code, flags[k] = fmt->f[i].flags;
  return k;
}

/* SerializedValidation's template codes; the count. */
int oracle_table_validation(uint32_t *codes, int cap) {
  const int n = (int)(sizeof kValidationFields / sizeof kValidationFields[0]);
  for (int i = 0; i < n && i < cap; ++i) codes[i] = kValidationFields[i];
  return n;
}
