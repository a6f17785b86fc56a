// stl_sha512.h -- SHA-512 (FIPS 180-4) for the gfx950 kernels.
//
// Two users on the hot path:
//   * k = SHA-512(R || A || M) inside crypto_sign_verify_detached
//     (libsodium, called at RippleAddress.cpp:196-197): one 128-byte block for
//     the 32-byte stellard message (96 bytes of input).
//   * SHA512Half(preimage) = the transaction signing hash
//     (Serializer.cpp:354-360 via STObject::getSigningHash,
//     SerializedObject.cpp:444-450): 1..33 blocks for 100 B .. 4 KB preimages.
// 64-bit words on 32-bit ALUs: the compiler lowers rotates to v_alignbit_b32
// pairs and adds to v_add_co/v_addc pairs; xor3 / ch / maj are one
// v_bitop3_b32 per half.
#pragma once
#include "stl_fe25519.h"

namespace stl {

STL_HD uint64_t sha_ror(uint64_t x, int n) { return (x >> n) | (x << (64 - n)); }

STL_HD uint64_t sha_k(int i) {
  // stored as a switch-free constant table; indexed with compile-time i after unrolling
  const uint64_t K[80] = {
      0x428a2f98d728ae22ULL, 0x7137449123ef65cdULL, 0xb5c0fbcfec4d3b2fULL, 0xe9b5dba58189dbbcULL,
      0x3956c25bf348b538ULL, 0x59f111f1b605d019ULL, 0x923f82a4af194f9bULL, 0xab1c5ed5da6d8118ULL,
      0xd807aa98a3030242ULL, 0x12835b0145706fbeULL, 0x243185be4ee4b28cULL, 0x550c7dc3d5ffb4e2ULL,
      0x72be5d74f27b896fULL, 0x80deb1fe3b1696b1ULL, 0x9bdc06a725c71235ULL, 0xc19bf174cf692694ULL,
      0xe49b69c19ef14ad2ULL, 0xefbe4786384f25e3ULL, 0x0fc19dc68b8cd5b5ULL, 0x240ca1cc77ac9c65ULL,
      0x2de92c6f592b0275ULL, 0x4a7484aa6ea6e483ULL, 0x5cb0a9dcbd41fbd4ULL, 0x76f988da831153b5ULL,
      0x983e5152ee66dfabULL, 0xa831c66d2db43210ULL, 0xb00327c898fb213fULL, 0xbf597fc7beef0ee4ULL,
      0xc6e00bf33da88fc2ULL, 0xd5a79147930aa725ULL, 0x06ca6351e003826fULL, 0x142929670a0e6e70ULL,
      0x27b70a8546d22ffcULL, 0x2e1b21385c26c926ULL, 0x4d2c6dfc5ac42aedULL, 0x53380d139d95b3dfULL,
      0x650a73548baf63deULL, 0x766a0abb3c77b2a8ULL, 0x81c2c92e47edaee6ULL, 0x92722c851482353bULL,
      0xa2bfe8a14cf10364ULL, 0xa81a664bbc423001ULL, 0xc24b8b70d0f89791ULL, 0xc76c51a30654be30ULL,
      0xd192e819d6ef5218ULL, 0xd69906245565a910ULL, 0xf40e35855771202aULL, 0x106aa07032bbd1b8ULL,
      0x19a4c116b8d2d0c8ULL, 0x1e376c085141ab53ULL, 0x2748774cdf8eeb99ULL, 0x34b0bcb5e19b48a8ULL,
      0x391c0cb3c5c95a63ULL, 0x4ed8aa4ae3418acbULL, 0x5b9cca4f7763e373ULL, 0x682e6ff3d6b2b8a3ULL,
      0x748f82ee5defb2fcULL, 0x78a5636f43172f60ULL, 0x84c87814a1f0ab72ULL, 0x8cc702081a6439ecULL,
      0x90befffa23631e28ULL, 0xa4506cebde82bde9ULL, 0xbef9a3f7b2c67915ULL, 0xc67178f2e372532bULL,
      0xca273eceea26619cULL, 0xd186b8c721c0c207ULL, 0xeada7dd6cde0eb1eULL, 0xf57d4f7fee6ed178ULL,
      0x06f067aa72176fbaULL, 0x0a637dc5a2c898a6ULL, 0x113f9804bef90daeULL, 0x1b710b35131c471bULL,
      0x28db77f523047d84ULL, 0x32caab7b40c72493ULL, 0x3c9ebe0a15c9bebcULL, 0x431d67c49c100d4cULL,
      0x4cc5d4becb3e42b6ULL, 0x597f299cfc657e2aULL, 0x5fcb6fab3ad6faecULL, 0x6c44198c4a475817ULL};
  return K[i];
}

STL_HD void sha512_init(uint64_t st[8]) {
  st[0] = 0x6a09e667f3bcc908ULL; st[1] = 0xbb67ae8584caa73bULL;
  st[2] = 0x3c6ef372fe94f82bULL; st[3] = 0xa54ff53a5f1d36f1ULL;
  st[4] = 0x510e527fade682d1ULL; st[5] = 0x9b05688c2b3e6c1fULL;
  st[6] = 0x1f83d9abfb41bd6bULL; st[7] = 0x5be0cd19137e2179ULL;
}

// ---- 64-bit words as 32-bit halves ----
// gfx950 runs 64-bit shifts and adds (v_lshrrev_b64, v_lshl_add_u64) at a
// fraction of the 32-bit rate; a rotate is two v_alignbit_b32, an add is
// v_add_co_u32 + v_addc_co_u32, and three-way xors fuse into v_xor3_b32.
struct W64 {
  uint32_t lo, hi;
};

STL_HD W64 w64(uint64_t v) { return W64{(uint32_t)v, (uint32_t)(v >> 32)}; }
STL_HD uint64_t u64(W64 v) { return ((uint64_t)v.hi << 32) | v.lo; }

STL_HD uint32_t abit(uint32_t hi, uint32_t lo, uint32_t n) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_alignbit(hi, lo, n);
#else
  return (uint32_t)((((uint64_t)hi << 32) | lo) >> (n & 31));
#endif
}

template <int N>
STL_HD W64 rotr(W64 x) {
  static_assert(N > 0 && N < 64 && N != 32, "rotate");
  if (N < 32) return W64{abit(x.hi, x.lo, N), abit(x.lo, x.hi, N)};
  return W64{abit(x.lo, x.hi, N - 32), abit(x.hi, x.lo, N - 32)};
}

template <int N>
STL_HD W64 shr(W64 x) {
  static_assert(N > 0 && N < 32, "shift");
  return W64{abit(x.hi, x.lo, N), x.hi >> N};
}

// Any three-input bitwise function as one v_bitop3_b32 (gfx950): IMM is its
// truth table, bit (a << 2 | b << 1 | c) = f(a, b, c).  The compiler does not
// fuse a three-way xor by itself here (two v_xor_b32 per half), which made
// the xors the largest instruction group of a compression.
template <uint32_t IMM>
STL_HD uint32_t bitop3(uint32_t a, uint32_t b, uint32_t c) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_bitop3_b32(a, b, c, IMM);
#else
  uint32_t r = 0;
  for (uint32_t i = 0; i < 8; ++i)
    if ((IMM >> i) & 1u) r |= ((i & 4u) ? a : ~a) & ((i & 2u) ? b : ~b) & ((i & 1u) ? c : ~c);
  return r;
#endif
}

STL_HD W64 xor3(W64 a, W64 b, W64 c) {
  return W64{bitop3<0x96u>(a.lo, b.lo, c.lo), bitop3<0x96u>(a.hi, b.hi, c.hi)};
}

STL_HD W64 add(W64 a, W64 b) {
  unsigned c;
  const uint32_t lo = __builtin_addc(a.lo, b.lo, 0u, &c);
  const uint32_t hi = __builtin_addc(a.hi, b.hi, c, &c);
  return W64{lo, hi};
}

// (e & f) ^ (~e & g) = e ? f : g, one bitop3 per half
STL_HD W64 ch(W64 e, W64 f, W64 g) { return W64{bitop3<0xCAu>(e.lo, f.lo, g.lo), bitop3<0xCAu>(e.hi, f.hi, g.hi)}; }
// majority, one bitop3 per half
STL_HD W64 maj(W64 a, W64 b, W64 c) { return W64{bitop3<0xE8u>(a.lo, b.lo, c.lo), bitop3<0xE8u>(a.hi, b.hi, c.hi)}; }

// Round constant, pinned per round as a scalar pair (see the loop below).
STL_HD W64 sha_kw(int i) {
  W64 k = w64(sha_k(i));
#if defined(__HIP_DEVICE_COMPILE__)
  asm volatile("" : "+s"(k.lo), "+s"(k.hi));
#endif
  return k;
}

// One compression; w[16] = the block as big-endian 64-bit words (clobbered).
STL_HD void sha512_compress(uint64_t st[8], uint64_t w64in[16]) {
  W64 w[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) w[j] = w64(w64in[j]);
  W64 a = w64(st[0]), b = w64(st[1]), c = w64(st[2]), d = w64(st[3]);
  W64 e = w64(st[4]), f = w64(st[5]), g = w64(st[6]), h = w64(st[7]);
#pragma clang loop unroll(full)
  for (int i = 0; i < 80; ++i) {
#if defined(__HIP_DEVICE_COMPILE__)
    // Pin round i's message-schedule inputs behind round i-1's state, so the
    // compiler cannot compute all 64 expansions up front (that keeps 80 words
    // = 160 VGPRs live and caps occupancy at 2 waves per SIMD).
    if (i >= 16) {
      asm volatile("" : "+v"(a.lo), "+v"(e.lo), "+v"(w[(i - 15) & 15].lo), "+v"(w[(i - 15) & 15].hi),
                   "+v"(w[(i - 2) & 15].lo), "+v"(w[(i - 2) & 15].hi));
    }
#endif
    W64 wi;
    if (i < 16) {
      wi = w[i];
    } else {
      const W64 w15 = w[(i - 15) & 15], w2 = w[(i - 2) & 15];
      const W64 s0 = xor3(rotr<1>(w15), rotr<8>(w15), shr<7>(w15));
      const W64 s1 = xor3(rotr<19>(w2), rotr<61>(w2), shr<6>(w2));
      wi = add(add(w[i & 15], s0), add(w[(i - 7) & 15], s1));
      w[i & 15] = wi;
    }
    const W64 S1 = xor3(rotr<14>(e), rotr<18>(e), rotr<41>(e));
    const W64 t1 = add(add(h, S1), add(add(ch(e, f, g), sha_kw(i)), wi));
    const W64 S0 = xor3(rotr<28>(a), rotr<34>(a), rotr<39>(a));
    const W64 t2 = add(S0, maj(a, b, c));
    h = g; g = f; f = e; e = add(d, t1); d = c; c = b; b = a; a = add(t1, t2);
  }
  st[0] = u64(add(w64(st[0]), a)); st[1] = u64(add(w64(st[1]), b));
  st[2] = u64(add(w64(st[2]), c)); st[3] = u64(add(w64(st[3]), d));
  st[4] = u64(add(w64(st[4]), e)); st[5] = u64(add(w64(st[5]), f));
  st[6] = u64(add(w64(st[6]), g)); st[7] = u64(add(w64(st[7]), h));
}

// ---- compression over a precomputed message schedule ----
// The latency path of a small batch (the longest preimage of a ledger: up to
// 33 dependent compressions) hashes one long message per wave: the lanes
// expand the schedules of up to kLongBatch blocks side by side (one lane per
// block), and the rounds then read W[t] from LDS -- a third of a
// compression's instructions leave its dependent chain.

// W[16..79] of one block from w[0..15], each word handed to put(t, W[t]) as it
// is made (a 16-word ring in registers).
template <typename Put>
STL_HD void sha512_schedule(const uint64_t win[16], Put put) {
  W64 w[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    w[j] = w64(win[j]);
    put(j, w[j]);
  }
#pragma unroll
  for (int i = 16; i < 80; ++i) {
    const W64 w15 = w[(i - 15) & 15], w2 = w[(i - 2) & 15];
    const W64 s0 = xor3(rotr<1>(w15), rotr<8>(w15), shr<7>(w15));
    const W64 s1 = xor3(rotr<19>(w2), rotr<61>(w2), shr<6>(w2));
    w[i & 15] = add(add(w[i & 15], s0), add(w[(i - 7) & 15], s1));
    put(i, w[i & 15]);
  }
}

// 64-bit add as one 64-bit VALU op (v_lshl_add_u64 on gfx950): no carry
// through an SGPR, so no hazard nop -- the lone-wave latency path's add
STL_HD W64 add64(W64 a, W64 b) { return w64(u64(a) + u64(b)); }

// ---- the rounds on a lane pair (one long row: the latency path) ----
// A round's two halves are one instruction stream with per-lane operands.
// The e-side lane keeps (e, f, g, h) and makes T1 = h + S1(e) + Ch(e, f, g)
// + K + W; the a-side lane keeps (a, b, c, d) and makes T2 = S0(a) +
// Maj(a, b, c).  S1 and S0 are three rotations and a xor3 each, with
// per-lane amounts (one of S0's is >= 32 where S1's is not: that lane
// rotates its word with the halves swapped); Maj(a, b, c) = (~(a ^ b)) ? b
// : c, so both lanes run Ch(x, y, z) = x ? y : z with x = e or ~(a ^ b)
// (one bitop3 per half on a lane mask).  Then each lane adds the value its
// partner sends -- d to the e-side (e' = d + T1), T1 to the a-side (a' = T1
// + T2) -- and shifts its four words.  ≈28 instructions per round for the
// pair against ≈40 for the whole round on one lane.
struct PairSide {
  uint32_t s1, s2, s3;  // alignbit amounts of the three rotations
  uint32_t am;          // ~0 on the a-side, 0 on the e-side
  bool a_side;
};

STL_HD PairSide pair_side(bool a_side) {
  // S1: rotr 14, 18, 41 (the last as 32 + 9); S0: rotr 28, 34 (32 + 2, on the
  // swapped word), 39 (32 + 7)
  return a_side ? PairSide{28u, 2u, 7u, ~0u, true} : PairSide{14u, 18u, 9u, 0u, false};
}

// front half: T (T1 on the e-side, T2 on the a-side) and U, the word the
// partner lane needs (the e-side sends T1, the a-side sends d)
template <bool ADD64 = true>
STL_HD void pair_round_front(const W64 r[4], W64 kw, const PairSide& ps, W64& T, W64& U) {
  auto ad = [](W64 a, W64 b) { return ADD64 ? add64(a, b) : add(a, b); };
  const W64 x = r[0];
  const W64 xs = ps.a_side ? W64{x.hi, x.lo} : x;
  const W64 r1{abit(x.hi, x.lo, ps.s1), abit(x.lo, x.hi, ps.s1)};
  const W64 r2{abit(xs.hi, xs.lo, ps.s2), abit(xs.lo, xs.hi, ps.s2)};
  const W64 r3{abit(x.lo, x.hi, ps.s3), abit(x.hi, x.lo, ps.s3)};
  const W64 S = xor3(r1, r2, r3);
  // x' = x ^ (am & ~y): e on the e-side, ~(a ^ b) on the a-side
  const W64 xp{bitop3<0xD2u>(x.lo, r[1].lo, ps.am), bitop3<0xD2u>(x.hi, r[1].hi, ps.am)};
  const W64 C = ch(xp, r[1], r[2]);
  W64 P = ad(r[3], kw);  // h + K + W, the e-side's only
  P.lo &= ~ps.am;
  P.hi &= ~ps.am;
  T = ad(ad(S, C), P);
  U = ps.a_side ? r[3] : T;
}

// back half: the partner's word added, the four words shifted
template <bool ADD64 = true>
STL_HD void pair_round_back(W64 r[4], W64 T, W64 Up) {
  r[3] = r[2];
  r[2] = r[1];
  r[1] = r[0];
  r[0] = ADD64 ? add64(T, Up) : add(T, Up);
}

STL_HD uint32_t bswap32(uint32_t x) {
  return (x >> 24) | ((x >> 8) & 0xff00u) | ((x << 8) & 0xff0000u) | (x << 24);
}

// Two little-endian memory words (bytes 8j..8j+7) -> big-endian 64-bit word.
STL_HD uint64_t be64_from_le32(uint32_t lo_word, uint32_t hi_word) {
  return ((uint64_t)bswap32(lo_word) << 32) | bswap32(hi_word);
}

// k-hash for a 32-byte message: SHA-512(R || A || M), 96 bytes, one block.
// Inputs are 8 little-endian 32-bit words each (memory order); the 64-byte
// digest is returned as 16 little-endian 32-bit words (memory order).
STL_HD void sha512_hram32(uint32_t out[16], const uint32_t R[8], const uint32_t A[8], const uint32_t M[8]) {
  uint64_t st[8], w[16];
  sha512_init(st);
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    w[j] = be64_from_le32(R[2 * j], R[2 * j + 1]);
    w[4 + j] = be64_from_le32(A[2 * j], A[2 * j + 1]);
    w[8 + j] = be64_from_le32(M[2 * j], M[2 * j + 1]);
  }
  w[12] = 0x8000000000000000ULL;
  w[13] = 0;
  w[14] = 0;
  w[15] = 96 * 8;
  sha512_compress(st, w);
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    out[2 * j] = bswap32((uint32_t)(st[j] >> 32));
    out[2 * j + 1] = bswap32((uint32_t)st[j]);
  }
}

// Byte-granular streaming SHA-512 over an arbitrary byte string in (global)
// memory, preceded by an optional 64-byte prefix held in registers (R || A for
// variable-length Ed25519 messages, or the 4-byte "STX\0" hash prefix).
// Reads every byte through a 64-bit big-endian assembler; used for the
// variable-length paths (tx preimages up to ~4 KB, generic verify_detached).
STL_HD uint8_t sha_byte_at(const uint8_t* prefix, uint32_t plen, const uint8_t* msg, uint64_t mlen, uint64_t pos) {
  if (pos < plen) return prefix[pos];
  pos -= plen;
  if (pos < mlen) return msg[pos];
  return 0;
}

STL_HD void sha512_prefixed(uint64_t st[8], const uint8_t* prefix, uint32_t plen, const uint8_t* msg, uint64_t mlen) {
  sha512_init(st);
  const uint64_t total = plen + mlen;
  const uint64_t nblocks = (total + 17 + 127) / 128;
  for (uint64_t blk = 0; blk < nblocks; ++blk) {
    uint64_t w[16];
    for (int j = 0; j < 16; ++j) {
      uint64_t v = 0;
      for (int b = 0; b < 8; ++b) {
        const uint64_t pos = blk * 128 + 8 * j + b;
        uint8_t byte;
        if (pos < total) byte = sha_byte_at(prefix, plen, msg, mlen, pos);
        else if (pos == total) byte = 0x80;
        else byte = 0;
        v = (v << 8) | byte;
      }
      w[j] = v;
    }
    if (blk == nblocks - 1) w[15] = total * 8;  // lengths < 2^61 bytes: high word stays 0
    sha512_compress(st, w);
  }
}

// ---- word-granular streaming SHA-512 over a byte string at any alignment ----
// The transaction path (SHA512Half of the signing preimage, config 5: 100 B to
// 4 KB) reads each 128-byte block as 33 aligned dwords and shifts them into
// message order with v_alignbyte_b32 (one load per 4 bytes instead of one per
// byte).  The 3 bytes of the last aligned dword past the message are never
// read: that dword is assembled from byte loads.

STL_HD uint32_t align_byte(uint32_t hi, uint32_t lo, uint32_t shift) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_alignbyte(hi, lo, shift);
#else
  return (uint32_t)((((uint64_t)hi << 32) | lo) >> (8 * (shift & 3)));
#endif
}

// Message view: bytes [p, p + len).  q = p rounded down to 4, mis = p & 3,
// nw = aligned dwords holding message bytes.
struct ByteStream {
  const uint8_t* p;
  const uint32_t* q;
  uint32_t mis, len, nw;
  STL_HD void init(const uint8_t* ptr, uint32_t n) {
    p = ptr;
    mis = (uint32_t)((uintptr_t)ptr & 3u);
    q = reinterpret_cast<const uint32_t*>(ptr - mis);
    len = n;
    nw = (mis + n + 3) >> 2;
  }
  // aligned dword idx of q[] (0 past the message; the last one byte by byte)
  STL_HD uint32_t dword(uint32_t idx) const {
    if (idx + 1 < nw || (idx + 1 == nw && ((mis + len) & 3u) == 0)) return q[idx];
    if (idx + 1 != nw) return 0u;
    const uint32_t valid = (mis + len) & 3u;  // bytes of the last dword inside the message
    const uint8_t* b = reinterpret_cast<const uint8_t*>(q + idx);
    uint32_t v = 0;
    for (uint32_t t = 0; t < valid; ++t) v |= (uint32_t)b[t] << (8 * t);
    return v;
  }
  // aligned dword idx through a source that may serve it from a cache (the
  // kernels' LDS window); Src(addr_of_dword, idx) falls back to dword(idx)
  struct Direct {
    const ByteStream* s;
    STL_HD uint32_t operator()(uint32_t idx) const { return s->dword(idx); }
  };
  // block blk as 16 big-endian words with the FIPS 180-4 padding applied
  // (0x80 after the message, zeros, 128-bit length in the final block)
  template <typename Src>
  STL_HD void block(uint64_t w[16], uint32_t blk, bool last, const Src& src) const {
    uint32_t prev = src(32 * blk);
#pragma unroll
    for (int j = 0; j < 32; j += 2) {
      uint32_t m[2];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const uint32_t next = src(32 * blk + j + h + 1);
        uint32_t v = align_byte(next, prev, mis);
        prev = next;
        const int64_t keep = (int64_t)len - (int64_t)(128 * blk + 4 * (j + h));
        if (keep < 4) {
          v = keep <= 0 ? 0u : (v & ((1u << (8 * keep)) - 1u));
          if (keep >= 0) v |= 0x80u << (8 * keep);
        }
        m[h] = v;
      }
      w[j >> 1] = be64_from_le32(m[0], m[1]);
    }
    if (last) {
      w[14] = 0;
      w[15] = (uint64_t)len * 8;
    }
  }
  STL_HD void block(uint64_t w[16], uint32_t blk, bool last) const { block(w, blk, last, Direct{this}); }
  STL_HD uint32_t blocks() const { return (len + 17 + 127) / 128; }
};

// Block assembly from a 36-word window: win[d4 .. d4+32] are the aligned
// dwords 32*blk .. 32*blk+32 of a ByteStream (the kernels fill the window by
// wave-cooperative 16-byte loads; d4 = that dword's offset in its 16-byte
// granule).  rem = message bytes left at the block start (may be <= 0 in a
// padding-only block).  With `prefix`, the message is a 4-byte prefix
// followed by the stream's bytes shifted by 4: the caller built the stream 4
// bytes before the data, and word 0 of block 0 is replaced by the prefix.
STL_HD void block_from_window(uint64_t w[16], const uint32_t* win, uint32_t d4, uint32_t mis, int32_t rem,
                              bool last, uint32_t total, bool first, bool has_prefix, uint32_t prefix_le) {
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    uint32_t m[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int i = 2 * j + h;
      uint32_t v = align_byte(win[d4 + i + 1], win[d4 + i], mis);
      if (i == 0 && has_prefix && first) v = prefix_le;
      const int32_t k = rem - 4 * i;  // message bytes from this word on
      const int32_t kc = k < 0 ? 0 : (k > 4 ? 4 : k);
      const uint32_t keep = kc == 4 ? 0xffffffffu : ((1u << (8 * kc)) - 1u);
      const uint32_t pad = (k >= 0 && k < 4) ? (0x80u << (8 * kc)) : 0u;
      m[h] = (v & keep) | pad;
    }
    w[j] = be64_from_le32(m[0], m[1]);
  }
  if (last) {
    w[14] = 0;
    w[15] = (uint64_t)total * 8u;
  }
}

// SHA512Half(bytes) -> 8 little-endian words (the first 32 digest bytes)
STL_HD void sha512_half_words(uint32_t out[8], const uint8_t* p, uint32_t len) {
  ByteStream bs;
  bs.init(p, len);
  uint64_t st[8], w[16];
  sha512_init(st);
  const uint32_t nb = bs.blocks();
  for (uint32_t b = 0; b < nb; ++b) {
    bs.block(w, b, b + 1 == nb);
    sha512_compress(st, w);
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    out[2 * j] = bswap32((uint32_t)(st[j] >> 32));
    out[2 * j + 1] = bswap32((uint32_t)st[j]);
  }
}

STL_HD void sha512_digest_le32(uint32_t out[16], const uint64_t st[8]) {
  for (int j = 0; j < 8; ++j) {
    out[2 * j] = bswap32((uint32_t)(st[j] >> 32));
    out[2 * j + 1] = bswap32((uint32_t)st[j]);
  }
}

}  // namespace stl
