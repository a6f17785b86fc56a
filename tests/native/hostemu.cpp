// hostemu.cpp -- TEST HARNESS ONLY.  Compiles the device verify code
// (stellard_amd/csrc/stl_verify_core.h, the exact functions the gfx950 kernel
// runs) for the host so its logic and limb-bound discipline can be checked
// against the oracle in the CPU test suite.  Not part of the product library
// (libstl exposes no CPU verify path).
#include <atomic>
#include <cstdint>
#include <cstring>
#include <mutex>
#include <thread>
#include <vector>

static std::atomic<uint64_t> g_bound_viol{0};
static std::atomic<uint64_t> g_bound_checks{0};

#define STL_BOUND_MUL(a, b) hostemu_check_mul((a), (b))
#define STL_BOUND_SUB(a, b) hostemu_check_sub((a), (b))
#define STL_BOUND_SUBK(a, b, K) hostemu_check_subk((a), (b), (K))
namespace stl { struct fe; }
static void hostemu_check_mul(const stl::fe& a, const stl::fe& b);
static void hostemu_check_sub(const stl::fe& a, const stl::fe& b);
static void hostemu_check_subk(const stl::fe& a, const stl::fe& b, int k);

#include "../../stellard_amd/csrc/stl_base_table.h"
#include "../../stellard_amd/csrc/stl_txblob.h"
#include "../../stellard_amd/csrc/stl_verify_core.h"
// HOSTEMU_SANITIZE_SUBSET (tests/native/sanitize_main.cpp): only the product
// verify path and the blob pass are compiled -- the sanitized build of every
// table-layout variant and the signer took over twelve minutes
#ifndef HOSTEMU_SANITIZE_SUBSET
#include "../../stellard_amd/csrc/stl_sign.h"
#endif

static double alpha(const stl::fe& a) {
  uint32_t m = 0;
  for (int i = 0; i < 9; ++i) m = a.v[i] > m ? a.v[i] : m;
  return m / 536870912.0;
}
static void hostemu_check_mul(const stl::fe& a, const stl::fe& b) {
  g_bound_checks++;
  if (alpha(a) * alpha(b) > 7.0) g_bound_viol++;
}
// fe_sub_nc<K>: no limb of b above K*Z1's, and a + K*Z1 within 32 bits
static void hostemu_check_subk(const stl::fe& a, const stl::fe& b, int k) {
  g_bound_checks++;
  bool bad = b.v[0] > (uint64_t)k * 0x1ffffb40u;
  for (int i = 1; i < 9; ++i) bad = bad || b.v[i] > (uint64_t)k * 0x1fffffffu;
  for (int i = 0; i < 9; ++i) bad = bad || (uint64_t)a.v[i] + (uint64_t)k * 0x1fffffffu > 0xffffffffull;
  if (bad) g_bound_viol++;
}
static void hostemu_check_sub(const stl::fe& a, const stl::fe& b) {
  g_bound_checks++;
  if (alpha(a) > 3.9 || alpha(b) > 3.9) g_bound_viol++;
}

static void load8(uint32_t w[8], const uint8_t* p) { std::memcpy(w, p, 32); }

// The wide base tables as the device builds them (wide_entry), built once per
// process on 8 threads.
static const uint32_t* wide_tables() {
  static std::vector<uint32_t> tab;
  static std::once_flag once;
  std::call_once(once, [] {
    tab.resize(stl::kWideTableWords);
    const uint32_t rows = 2 * stl::kWideEntries;
    std::vector<std::thread> th;
    for (uint32_t t = 0; t < 8; ++t)
      th.emplace_back([t, rows] {
        for (uint32_t r = t; r < rows; r += 8) {
          const int which = r >= stl::kWideEntries ? 1 : 0;
          stl::wide_entry(&tab[(size_t)r * stl::kWideRowWords], which, r - (uint32_t)which * stl::kWideEntries,
                          &stl::kBaseNielsHost[0][0][0]);
        }
      });
    for (auto& x : th) x.join();
  });
  return tab.data();
}

extern "C" {

// Bitmap out, LSB-first; returns number of bound violations observed.
// mode 0: the product's path (half-size scalars, full-length fallback);
// mode 1: full-length path only; mode 2: half-size path only (flagged lanes
// reject).  Returns the number of limb-bound violations observed; *fallbacks
// (if non-null) receives the number of lanes the half-size path flagged.
uint64_t hostemu_verify_batch_mode(const uint8_t* sig, const uint8_t* msg, const uint8_t* pk, size_t n,
                                   uint8_t* bitmap, uint32_t policy, int mode, uint64_t* fallbacks) {
  std::vector<uint4> table(2 * 81);
  const stl::TableView t1 = stl::TableView::contiguous(table.data()), t2 = stl::TableView::contiguous(table.data() + 81);
  const uint32_t* btab = &stl::kBaseNielsHost[0][0][0];
  std::memset(bitmap, 0, (n + 7) / 8);
  uint64_t fb = 0;
  for (size_t i = 0; i < n; ++i) {
    uint32_t R[8], S[8], A[8], M[8], h[16], k[8];
    load8(R, sig + 64 * i);
    load8(S, sig + 64 * i + 32);
    load8(A, pk + 32 * i);
    load8(M, msg + 32 * i);
    stl::sha512_hram32(h, R, A, M);
    stl::sc_reduce64(k, h);
    bool ok;
    if (mode == 1) {
      ok = stl::verify_full_with_k(R, S, A, k, policy, t1, btab);
    } else {
      stl::HalfState hs;
      stl::verify_phase1_half(hs, R, S, A, k, policy);
      const bool flagged = (hs.tops & stl::kHalfFallback) != 0;
      fb += flagged;
      if (flagged && mode == 0) ok = stl::verify_full_with_k(R, S, A, k, policy, t1, btab);
      else {
        stl::WideHost wide{wide_tables(), {0, 0}};
        ok = stl::verify_phase2_half(hs, t1, t2, wide);
      }
    }
    if (ok) bitmap[i >> 3] |= (uint8_t)(1u << (i & 7));
  }
  if (fallbacks) *fallbacks = fb;
  return g_bound_viol.load();
}

#ifndef HOSTEMU_SANITIZE_SUBSET
// The product path (mode 0) with the kernels' split table layout
// (TableView::split): heads of entries 1-8 in one array, entry 0's head one
// shared identity line, tails in a separate array at stride `tstride` quads
// (the main kernel's LDS layout [table*9 + entry][lane] has stride 256).
uint64_t hostemu_verify_batch_split(const uint8_t* sig, const uint8_t* msg, const uint8_t* pk, size_t n,
                                    uint8_t* bitmap, uint32_t policy, int tstride) {
  std::vector<uint4> heads(2 * 8 * 8), tails((size_t)18 * tstride), id(9);
  stl::ge_cached idc;
  stl::ge_cached_0(idc);
  stl::TableView::contiguous(id.data()).store(0, idc);  // identity entry: its 8-quad head
  const stl::TableView t1 = stl::TableView::split(heads.data(), tails.data(), id.data(), tstride),
                       t2 = stl::TableView::split(heads.data() + 64, tails.data() + (size_t)9 * tstride, id.data(),
                                                  tstride);
  std::vector<uint4> full(81);
  const stl::TableView tf = stl::TableView::contiguous(full.data());
  const uint32_t* btab = &stl::kBaseNielsHost[0][0][0];
  std::memset(bitmap, 0, (n + 7) / 8);
  for (size_t i = 0; i < n; ++i) {
    uint32_t R[8], S[8], A[8], M[8], h[16], k[8];
    load8(R, sig + 64 * i);
    load8(S, sig + 64 * i + 32);
    load8(A, pk + 32 * i);
    load8(M, msg + 32 * i);
    stl::sha512_hram32(h, R, A, M);
    stl::sc_reduce64(k, h);
    stl::HalfState hs;
    stl::verify_phase1_half(hs, R, S, A, k, policy);
    bool ok;
    if (hs.tops & stl::kHalfFallback) {
      ok = stl::verify_full_with_k(R, S, A, k, policy, tf, btab);
    } else {
      stl::WideHost wide{wide_tables(), {0, 0}};
      ok = stl::verify_phase2_half(hs, t1, t2, wide);
    }
    if (ok) bitmap[i >> 3] |= (uint8_t)(1u << (i & 7));
  }
  return g_bound_viol.load();
}

// The main kernel's default path (verify_main_kernel<JOINT = true>): one
// joint radix-4 table of a*P1 + b*P2 per lane in the split layout (heads of
// entries 1-12, tails at stride `tstride`), verify_phase2_joint.
uint64_t hostemu_verify_batch_joint(const uint8_t* sig, const uint8_t* msg, const uint8_t* pk, size_t n,
                                    uint8_t* bitmap, uint32_t policy, int tstride) {
  std::vector<uint4> heads(2 * 8 * 8), tails((size_t)18 * tstride), id(9);
  stl::ge_cached idc;
  stl::ge_cached_0(idc);
  stl::TableView::contiguous(id.data()).store(0, idc);
  const stl::TableView tj = stl::TableView::split(heads.data(), tails.data(), id.data(), tstride);
  std::vector<uint4> full(81);
  const stl::TableView tf = stl::TableView::contiguous(full.data());
  const uint32_t* btab = &stl::kBaseNielsHost[0][0][0];
  std::memset(bitmap, 0, (n + 7) / 8);
  for (size_t i = 0; i < n; ++i) {
    uint32_t R[8], S[8], A[8], M[8], h[16], k[8];
    load8(R, sig + 64 * i);
    load8(S, sig + 64 * i + 32);
    load8(A, pk + 32 * i);
    load8(M, msg + 32 * i);
    stl::sha512_hram32(h, R, A, M);
    stl::sc_reduce64(k, h);
    stl::HalfState hs;
    stl::verify_phase1_half(hs, R, S, A, k, policy);
    bool ok;
    if (hs.tops & stl::kHalfFallback) {
      ok = stl::verify_full_with_k(R, S, A, k, policy, tf, btab);
    } else {
      stl::WideHost wide{wide_tables(), {0, 0}};
      static_assert(sizeof(stl::HalfState) == 14 * sizeof(uint4), "state");
      uint4 st[14];
      std::memcpy(st, &hs, sizeof(st));
      ok = stl::verify_phase2_joint(st, tj, wide);
    }
    if (ok) bitmap[i >> 3] |= (uint8_t)(1u << (i & 7));
  }
  return g_bound_viol.load();
}

// The small-batch pair path (verify_prep_pair_kernel +
// verify_main_pair_kernel): each signature's two decodings, its two
// chains (verify_phase2_pair_chain, parity 0 and 1, each on its own split
// table with the kernel's LDS tail stride) and the pair's cancellation check.
uint64_t hostemu_verify_batch_pair(const uint8_t* sig, const uint8_t* msg, const uint8_t* pk, size_t n,
                                   uint8_t* bitmap, uint32_t policy) {
  const int tstride = 256;
  std::vector<uint4> heads(2 * 8 * 8), tails((size_t)9 * tstride + 1), id(9);
  stl::ge_cached idc;
  stl::ge_cached_0(idc);
  stl::TableView::contiguous(id.data()).store(0, idc);
  const stl::TableView t0 = stl::TableView::split(heads.data(), tails.data(), id.data(), tstride),
                       t1 = stl::TableView::split(heads.data() + 64, tails.data() + 1, id.data(), tstride);
  std::vector<uint4> full(81);
  const stl::TableView tf = stl::TableView::contiguous(full.data());
  const uint32_t* btab = &stl::kBaseNielsHost[0][0][0];
  std::memset(bitmap, 0, (n + 7) / 8);
  for (size_t i = 0; i < n; ++i) {
    uint32_t R[8], S[8], A[8], M[8], h[16], k[8];
    load8(R, sig + 64 * i);
    load8(S, sig + 64 * i + 32);
    load8(A, pk + 32 * i);
    load8(M, msg + 32 * i);
    stl::sha512_hram32(h, R, A, M);
    stl::sc_reduce64(k, h);
    stl::HalfState hs;
    stl::verify_phase1_scalars(hs, S, k);
    stl::fe ax, ay, qx, qy;  // the pair's two decodings (the point role of verify_prep_pair_kernel)
    const bool okA = stl::phase1_decode_lane(ax, ay, R, A, 0), okR = stl::phase1_decode_lane(qx, qy, R, A, 1);
    stl::finish_phase1_points(hs, ax, ay, qx, qy, stl::phase1_points_ok(R, S, A, policy, okA, okR));
    bool ok;
    if (hs.tops & stl::kHalfFallback) {
      ok = stl::verify_full_with_k(R, S, A, k, policy, tf, btab);
    } else {
      stl::WideHost w0{wide_tables(), {0, 0}}, w1{wide_tables(), {0, 0}};
      stl::ge_p2 a, b;
      stl::verify_phase2_pair_chain(a, hs, 0, t0, w0);
      stl::verify_phase2_pair_chain(b, hs, 1, t1, w1);
      ok = stl::half_state_accepts(hs) && stl::pair_sums_cancel(a, b) && stl::pair_sums_cancel(b, a);
    }
    if (ok) bitmap[i >> 3] |= (uint8_t)(1u << (i & 7));
  }
  return g_bound_viol.load();
}

#endif  // HOSTEMU_SANITIZE_SUBSET

// Words of the identity entry's head as the split tables expect it (the
// device constant kIdentityHead must equal these 32 words).
void hostemu_identity_head(uint32_t out[32]) {
  std::vector<uint4> id(9);
  stl::ge_cached idc;
  stl::ge_cached_0(idc);
  stl::TableView::contiguous(id.data()).store(0, idc);
  std::memcpy(out, id.data(), 32 * 4);
}

uint64_t hostemu_verify_batch(const uint8_t* sig, const uint8_t* msg, const uint8_t* pk, size_t n,
                              uint8_t* bitmap, uint32_t policy) {
  return hostemu_verify_batch_mode(sig, msg, pk, n, bitmap, policy, 0, nullptr);
}

// Lattice reduction of k (32 bytes LE) to (c, d): magnitudes as 20-byte LE
// integers, signs in *signs (bit 0 c < 0, bit 1 d < 0).  Returns 1 if the pair
// fits the half-size budget, 0 if the lane takes the full-length path.
int hostemu_lattice(const uint8_t kb[32], uint8_t c_out[20], uint8_t d_out[20], uint32_t* signs) {
  uint32_t k[8], c[5], d[5];
  load8(k, kb);
  bool cn = false, dn = false;
  const bool ok = stl::lattice_half(c, cn, d, dn, k);
  std::memcpy(c_out, c, 20);
  std::memcpy(d_out, d, 20);
  *signs = (cn ? 1u : 0u) | (dn ? 2u : 0u);
  return ok ? 1 : 0;
}

// SHA512Half over bytes [p, p + len) with the kernel's word-granular reader.
void hostemu_sha512_half(const uint8_t* p, uint32_t len, uint8_t out[32]) {
  uint32_t o[8];
  stl::sha512_half_words(o, p, len);
  std::memcpy(out, o, 32);
}

// One SHA-512 compression as the long-row kernel runs it on a lane pair
// (stl_sha512.h pair_round_front / _back), both lanes emulated in lockstep:
// st[8] (H0..H7) updated by the block w[16] (big-endian 64-bit words).
void hostemu_sha512_pair_compress(uint64_t st[8], const uint64_t w[16], int add64) {
  uint64_t sched[80];
  stl::sha512_schedule(w, [&](int t, stl::W64 v) { sched[t] = stl::u64(v); });
  stl::W64 r[2][4];
  for (int j = 0; j < 4; ++j) {
    r[0][j] = stl::w64(st[4 + j]);  // e-side lane: e, f, g, h
    r[1][j] = stl::w64(st[j]);      // a-side lane: a, b, c, d
  }
  const stl::PairSide ps[2] = {stl::pair_side(false), stl::pair_side(true)};
  for (int t = 0; t < 80; ++t) {
    const stl::W64 kw = stl::w64(sched[t] + stl::sha_k(t));
    stl::W64 T[2], U[2];
    for (int l = 0; l < 2; ++l) {
      if (add64)
        stl::pair_round_front<true>(r[l], kw, ps[l], T[l], U[l]);
      else
        stl::pair_round_front<false>(r[l], kw, ps[l], T[l], U[l]);
    }
    for (int l = 0; l < 2; ++l) stl::pair_round_back(r[l], T[l], U[1 - l]);
  }
  for (int j = 0; j < 4; ++j) {
    st[4 + j] += stl::u64(r[0][j]);
    st[j] += stl::u64(r[1][j]);
  }
}

// The device's serialized-transaction pass (stl_txblob.h) for one blob:
// status, signing hash (splice), transaction ID, and the layout numbers
// (pk_off, pk_len, sig_off, sig_len, xs0, xe0, xs1, xe1, xs2, xe2).
void hostemu_tx_blob(const uint8_t* blob, uint32_t len, uint32_t* status, uint8_t msg[32], uint8_t txid[32],
                     uint32_t layout[10]) {
  stl::TxLayout t;
  stl::tx_blob_parse(blob, len, t);
  *status = t.status;
  uint32_t h[8];
  std::memset(msg, 0, 32);
  std::memset(txid, 0, 32);
  if (t.status == stl::kTxOk) {
    stl::splice_sha512_half(h, blob, len, stl::kPrefixTxSign, &t);
    std::memcpy(msg, h, 32);
  }
  if (t.status != stl::kTxDeferred) {
    stl::splice_sha512_half(h, blob, len, stl::kPrefixTxId, nullptr);
    std::memcpy(txid, h, 32);
  }
  const uint32_t l[10] = {t.pk_off, t.pk_len, t.sig_off, t.sig_len, t.xs0, t.xe0, t.xs1, t.xe1, t.xs2, t.xe2};
  std::memcpy(layout, l, sizeof l);
}

// The same pass for either signed-object kind (0 transaction, 1 validation,
// stl_txblob.h BlobKind): status, signing hash, ID.
void hostemu_signed_blob(uint32_t kind, const uint8_t* blob, uint32_t len, uint32_t* status, uint8_t msg[32],
                         uint8_t id[32]) {
  const stl::BlobKind k = kind == 1 ? stl::blob_kind_validation() : stl::blob_kind_tx();
  stl::TxLayout t;
  stl::tx_blob_parse(blob, len, t, k.sig_code, k.min_len, k.format);
  *status = t.status;
  uint32_t h[8];
  std::memset(msg, 0, 32);
  std::memset(id, 0, 32);
  if (t.status == stl::kTxOk) {
    stl::splice_sha512_half(h, blob, len, k.sign_prefix, &t);
    std::memcpy(msg, h, 32);
  }
  if (t.status != stl::kTxDeferred) {
    if (k.id_prefixed) stl::splice_sha512_half(h, blob, len, k.id_prefix, nullptr);
    else stl::sha512_half_words(h, blob, len);
    std::memcpy(id, h, 32);
  }
}

// block_from_window (the hash kernels' assembly from an LDS window) against
// ByteStream::block for a message at buf+off of length len: every block,
// optionally with the 4-byte prefix form.  Returns the number of differing
// blocks.  buf must have 16 readable bytes around the message.
uint32_t hostemu_window_blocks(const uint8_t* buf, uint32_t off, uint32_t len, uint32_t prefix_le, int with_prefix) {
  stl::ByteStream ref, bs;
  uint32_t bad = 0;
  if (with_prefix) {
    // reference: the prefix and the message concatenated
    std::vector<uint8_t> cat(4 + len + 4);
    std::memcpy(cat.data(), &prefix_le, 4);
    std::memcpy(cat.data() + 4, buf + off, len);
    ref.init(cat.data(), len + 4);
    bs.init(buf + off - 4, len + 4);
    const uint32_t nb = ref.blocks();
    for (uint32_t blk = 0; blk < nb; ++blk) {
      uint64_t a[16], b[16];
      ref.block(a, blk, blk + 1 == nb);
      const uintptr_t addr = (uintptr_t)(bs.q + 32 * blk), base = addr & ~(uintptr_t)15;
      uint32_t win[36];
      std::memcpy(win, (const void*)base, sizeof win);
      stl::block_from_window(b, win, (uint32_t)(addr & 15u) >> 2, bs.mis, (int32_t)bs.len - (int32_t)(128 * blk),
                             blk + 1 == nb, bs.len, blk == 0, true, prefix_le);
      bad += std::memcmp(a, b, sizeof a) != 0;
    }
    return bad;
  }
  ref.init(buf + off, len);
  const uint32_t nb = ref.blocks();
  for (uint32_t blk = 0; blk < nb; ++blk) {
    uint64_t a[16], b[16];
    ref.block(a, blk, blk + 1 == nb);
    const uintptr_t addr = (uintptr_t)(ref.q + 32 * blk), base = addr & ~(uintptr_t)15;
    uint32_t win[36];
    std::memcpy(win, (const void*)base, sizeof win);
    stl::block_from_window(b, win, (uint32_t)(addr & 15u) >> 2, ref.mis, (int32_t)len - (int32_t)(128 * blk),
                           blk + 1 == nb, len, false, false, 0u);
    bad += std::memcmp(a, b, sizeof a) != 0;
  }
  return bad;
}

// Row j of wide table `which` (28 words) as the device init kernel writes it.
void hostemu_wide_row(int which, uint32_t j, uint32_t out[28]) {
  std::memcpy(out, wide_tables() + ((size_t)which * stl::kWideEntries + j) * stl::kWideRowWords, 28 * 4);
}

// blob_words as the kernel uses it to gather pk / sig (unaligned source)
void hostemu_blob_words(const uint8_t* blob, uint32_t off, uint32_t n, uint32_t len, uint32_t* out) {
  stl::blob_words(out, blob, off, n, len);
}

// e = d * S mod L with signed d (20-byte magnitude, sign), S 32 bytes.
void hostemu_sc_mul_signed(const uint8_t d_in[20], int d_neg, const uint8_t S_in[32], uint8_t out[32]) {
  uint32_t d[5], S[8], o[8];
  std::memcpy(d, d_in, 20);
  load8(S, S_in);
  stl::sc_mul_signed(o, d, d_neg != 0, S);
  std::memcpy(out, o, 32);
}

uint64_t hostemu_bound_checks(void) { return g_bound_checks.load(); }

void hostemu_sha512_hram32(const uint8_t* R, const uint8_t* A, const uint8_t* M, uint8_t out[64]) {
  uint32_t r[8], a[8], m[8], h[16];
  load8(r, R); load8(a, A); load8(m, M);
  stl::sha512_hram32(h, r, a, m);
  std::memcpy(out, h, 64);
}

void hostemu_sc_reduce64(const uint8_t in[64], uint8_t out[32]) {
  uint32_t x[16], o[8];
  std::memcpy(x, in, 64);
  stl::sc_reduce64(o, x);
  std::memcpy(out, o, 32);
}

void hostemu_fe_mul_bytes(const uint8_t a[32], const uint8_t b[32], uint8_t out[32]) {
  uint32_t wa[8], wb[8], wo[8];
  load8(wa, a); load8(wb, b);
  stl::fe fa, fb, fo;
  stl::fe_frombytes(fa, wa);
  stl::fe_frombytes(fb, wb);
  stl::fe_mul(fo, fa, fb);
  stl::fe_tobytes(wo, fo);
  std::memcpy(out, wo, 32);
}

// The wide per-key table j*(-A), j = 0..136, as the two-stage device build
// makes it (key_table_wide_base_kernel: wide_base_index entries by
// small_multiple_cached; key_table_wide_pair_kernel: wide_pair_entry), each
// entry as affine (x, y) bytes; out_direct the same from double-and-add of
// every j (the one-stage build it replaced).  Returns 0 if A does not decode.
static void cached_affine_bytes(uint8_t out[64], const stl::ge_cached& c) {
  stl::fe x2, y2, z2, zi, x, y;
  stl::fe_sub(x2, c.YpX, c.YmX);
  stl::fe_add(y2, c.YpX, c.YmX);
  stl::fe_carry(y2);
  stl::fe_add(z2, c.Z, c.Z);
  stl::fe_carry(z2);
  stl::fe_invert(zi, z2);
  stl::fe_mul(x, x2, zi);
  stl::fe_mul(y, y2, zi);
  uint32_t wx[8], wy[8];
  stl::fe_tobytes(wx, x);
  stl::fe_tobytes(wy, y);
  std::memcpy(out, wx, 32);
  std::memcpy(out + 32, wy, 32);
}

int hostemu_wide_key_table(const uint8_t A_in[32], uint8_t* out_two_stage, uint8_t* out_direct) {
  uint32_t A[8];
  load8(A, A_in);
  stl::ge_p3 negA;
  if (!stl::ge_frombytes_negate_vartime(negA, A)) return 0;
  std::vector<uint4> tab((size_t)stl::kWideKeyEntries * 9);
  const stl::TableView tv = stl::TableView::contiguous(tab.data());
  for (int i = 0; i < stl::kWideBaseEntries; ++i) {
    stl::ge_cached c;
    const int j = stl::wide_base_index(i);
    stl::small_multiple_cached(c, negA.X, negA.Y, j);
    tv.store(j, c);
  }
  for (int j = 17; j < stl::kWideKeyEntries; ++j) {
    if ((j & 15) == 0) continue;
    stl::ge_cached hi, lo, c;
    tv.load(j & ~15, hi);
    tv.load(j & 15, lo);
    stl::wide_pair_entry(c, hi, lo);
    tv.store(j, c);
  }
  for (int j = 0; j < stl::kWideKeyEntries; ++j) {
    stl::ge_cached c, d;
    tv.load(j, c);
    cached_affine_bytes(out_two_stage + 64 * j, c);
    stl::small_multiple_cached(d, negA.X, negA.Y, j);
    cached_affine_bytes(out_direct + 64 * j, d);
  }
  return 1;
}

void hostemu_fe_invert_bytes(const uint8_t a[32], uint8_t out[32]) {
  uint32_t wa[8], wo[8];
  load8(wa, a);
  stl::fe fa, fo;
  stl::fe_frombytes(fa, wa);
  stl::fe_invert(fo, fa);
  stl::fe_tobytes(wo, fo);
  std::memcpy(out, wo, 32);
}

#ifndef HOSTEMU_SANITIZE_SUBSET
// stl_sign.h on the host: the honest rows and the adversarial rows the GPU's
// sign kernel builds (stl_debug_sign_adversarial_device), on 8 threads.
void hostemu_sign_adversarial(const uint8_t* seed, const uint8_t* msg, const uint8_t* cls, const uint32_t* param,
                              size_t n, uint8_t* pk, uint8_t* sig, uint8_t* msg_out) {
  std::vector<std::thread> th;
  for (size_t t = 0; t < 8; ++t)
    th.emplace_back([=] {
      std::vector<uint4> table(81);
      const stl::TableView tv = stl::TableView::contiguous(table.data());
      const uint32_t* btab = &stl::kBaseNielsHost[0][0][0];
      for (size_t i = t; i < n; i += 8) {
        uint32_t sd[8], M[8], A[8], R[8], S[8], a[8], r[8];
        load8(sd, seed + 32 * i);
        load8(M, msg + 32 * i);
        stl::sign_row(A, R, S, a, r, sd, M, tv, btab);
        if (cls && cls[i]) stl::adversarial_row(cls[i], param[i], A, R, S, M, a, r, tv, btab);
        std::memcpy(pk + 32 * i, A, 32);
        std::memcpy(sig + 64 * i, R, 32);
        std::memcpy(sig + 64 * i + 32, S, 32);
        std::memcpy(msg_out + 32 * i, M, 32);
      }
    });
  for (auto& x : th) x.join();
}
#endif  // HOSTEMU_SANITIZE_SUBSET
}

// ---- the device pass's field tables (tests/test_sfields.py pins them to the
// reference's own text, tests/golden/sfields.json) ----
extern "C" {
int hostemu_tx_field_bit(uint32_t code) { return stl::tx_field_bit(code); }
int hostemu_tx_format(uint32_t type, uint64_t* allowed, uint64_t* required) {
  return stl::tx_format(type, *allowed, *required) ? 1 : 0;
}
uint64_t hostemu_declared_names(uint32_t type) { return stl::declared_names(type); }
int hostemu_validation_field(uint32_t code) { return stl::validation_field(code) ? 1 : 0; }
int hostemu_non_signing_field(uint32_t code) { return stl::non_signing_field(code) ? 1 : 0; }

// SpliceStream and splice1_block over the same one-cut layout (the two
// preimage assemblies of tx_blob_kernel): SHA512Half of each
void hostemu_splice_pair(const uint8_t* blob, uint32_t len, uint32_t prefix, uint32_t xs, uint32_t xe,
                         uint8_t out_stream[32], uint8_t out_words[32]) {
  stl::TxLayout t;
  t.xs0 = xs; t.xe0 = xe;
  t.xs1 = t.xe1 = t.xs2 = t.xe2 = len;
  uint32_t a[8], b[8];
  stl::splice_sha512_half(a, blob, len, prefix, &t);
  stl::splice1_sha512_half(b, blob, len, prefix, xs, xe);
  std::memcpy(out_stream, a, 32);
  std::memcpy(out_words, b, 32);
}

// tx_blob_kernel's phase 0 on the host: blocks before the cut's block read
// the blob 4 bytes early, the cut's block is tx_blob_parse_kernel's spliced
// block (splice1_words), later blocks read past the cut -- each through a
// 144-byte window of 16-byte granules (zero outside [lo, end)), as
// wave_window_fill and block_from_window take it.
void hostemu_splice_kernel(const uint8_t* blob, uint32_t len, uint32_t prefix, uint32_t xs, uint32_t xe,
                           uint8_t out[32]) {
  const uint32_t cut = xe - xs, total = 4u + len - cut, nb = (total + 17u + 127u) / 128u, sblk = (4u + xs) >> 7;
  const uint32_t prefix_le = stl::bswap32(prefix);
  uint32_t side[32];
  stl::splice1_words(side, blob, len, xs, xe, prefix_le, sblk,
                     [](const uint8_t* q) { return *reinterpret_cast<const uint32_t*>(q); });
  uint64_t st[8], w[16];
  stl::sha512_init(st);
  for (uint32_t blk = 0; blk < nb; ++blk) {
    const bool spliced = blk == sblk;
    uintptr_t src = (uintptr_t)blob + 128u * blk - 4u + (blk > sblk ? cut : 0u);
    uintptr_t lo = (uintptr_t)blob, end = lo + len;
    if (spliced) {
      src = (uintptr_t)side;
      lo = src;
      end = src + 128u;
    }
    const uintptr_t base = src & ~(uintptr_t)15;
    uint32_t win[36];
    for (uint32_t c = 0; c < 9; ++c) {
      const uintptr_t a = base + 16u * c;
      for (int k = 0; k < 4; ++k)
        win[4 * c + k] = (a < end && a + 16u > lo) ? reinterpret_cast<const uint32_t*>(a)[k] : 0u;
    }
    stl::block_from_window(w, win, (uint32_t)(src & 15u) >> 2, (uint32_t)(src & 3u),
                           (int32_t)total - (int32_t)(128u * blk), blk + 1 == nb, total, blk == 0 && !spliced, true,
                           prefix_le);
    stl::sha512_compress(st, w);
  }
  uint32_t h[8];
  for (int j = 0; j < 4; ++j) {
    h[2 * j] = stl::bswap32((uint32_t)(st[j] >> 32));
    h[2 * j + 1] = stl::bswap32((uint32_t)st[j]);
  }
  std::memcpy(out, h, 32);
}
}
