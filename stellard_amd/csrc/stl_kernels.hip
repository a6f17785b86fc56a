// stl_kernels.hip -- gfx950 kernels of libstl.
//
//   verify_scalar_kernel  phase 1a of one Ed25519 verification per lane
//                         (RippleAddress::verifySignature over the 32-byte
//                         signing hash, RippleAddress.cpp:190-200): k,
//                         half-size scalars (c, d), e, digits.
//   verify_point_kernel   phase 1b: pre-checks, decompression of A and R.
//   verify_main_kernel    phase 2, the hot loop: [e]B + [c](-A) + [d](-Q) == O,
//                         accept bits assembled per wave with a 64-bit ballot.
//   verify_fallback_kernel  full-length check for the rare flagged lanes.
//   hram_var_kernel       k for arbitrary-length messages.
//   tx_hash_kernel        SHA512Half(signing preimage) per transaction
//                         (Serializer.cpp:354-360 / SerializedObject.cpp:444-450).
//   tx_blob_kernel        from serialized transactions: canonical-form pass,
//                         signing hash by splice, transaction ID, verify inputs
//                         (stl_txblob.h).
//   sign_kernel           RFC 8032 keypair + signature (synthetic data only).
//
// Launch geometry: 256-thread workgroups (4 waves); phases 2 and 3 use a grid
// sized by the host to the resident capacity and grid-stride over
// 256-signature tiles, so the per-lane table workspace is bounded by the
// resident lanes.
#include "stl_base_table.h"
#include "stl_kernels.h"
#include "stl_sign.h"
#include "stl_txblob.h"
#include "stl_verify_core.h"

// Occupancy target of the verify kernel (waves per SIMD); register budget =
// 512 / waves.  Tuned on MI355X ("occupancy").
#ifndef STL_VERIFY_WAVES_PER_SIMD
#define STL_VERIFY_WAVES_PER_SIMD 2
#endif
#ifndef STL_PRE_WAVES_PER_SIMD
#define STL_PRE_WAVES_PER_SIMD 4
#endif
// Scalar half of phase 1 (SHA-512 of k, lattice reduction): serial
// dependency chains with few live registers, so occupancy hides latency.
#ifndef STL_SCALAR_WAVES_PER_SIMD
#define STL_SCALAR_WAVES_PER_SIMD 4
#endif
// Hash kernels: waves per SIMD (SHA-512 rounds are a serial chain per lane,
// so occupancy hides the VALU and memory latency).
#ifndef STL_HASH_WAVES_PER_SIMD
#define STL_HASH_WAVES_PER_SIMD 4
#endif

namespace stl {

__device__ __forceinline__ void ld8(uint32_t w[8], const uint8_t* p) {
  const uint4* q = reinterpret_cast<const uint4*>(p);
  const uint4 a = q[0], b = q[1];
  w[0] = a.x; w[1] = a.y; w[2] = a.z; w[3] = a.w;
  w[4] = b.x; w[5] = b.y; w[6] = b.z; w[7] = b.w;
}

__device__ __forceinline__ void st8(uint8_t* p, const uint32_t w[8]) {
  uint4* q = reinterpret_cast<uint4*>(p);
  q[0] = make_uint4(w[0], w[1], w[2], w[3]);
  q[1] = make_uint4(w[4], w[5], w[6], w[7]);
}

// Copy `tables` affine base tables (14 KiB each) into LDS once per workgroup.
__device__ __forceinline__ void stage_base_table(uint32_t* sB, int tables) {
  const uint4* g = reinterpret_cast<const uint4*>(&kBaseNiels[0][0][0]);
  uint4* d = reinterpret_cast<uint4*>(sB);
  for (uint32_t i = threadIdx.x; i < (uint32_t)(tables * kBaseTableWords / 4); i += kBlock) d[i] = g[i];
  __syncthreads();
}

// Per-lane workspace: two 9-entry cached tables per resident lane, split
// (TableView::split): the 128-B heads of entries 1-8, 2 x 8 x 8 quads per
// lane, in whole aligned lines from the start of the area, then the 16-B
// tails, 2 x 9 quads per lane (the main kernel keeps its tails in LDS).  Entry
// 0 is the identity; its head is kIdentityHead, shared by every lane.
// Not const: a const __device__ array lives in the constant address space,
// and TableView::head's select between it and the global workspace then
// becomes a generic pointer (flat loads); as a global array the table reads
// are global loads (measured neutral, round 4).
__device__ __attribute__((aligned(128))) uint4 kIdentityHead[8] = {
    {1u, 0u, 0u, 0u}, {0u, 0u, 0u, 0u}, {0u, 1u, 0u, 0u}, {0u, 0u, 0u, 0u},
    {0u, 0u, 1u, 0u}, {0u, 0u, 0u, 0u}, {0u, 0u, 0u, 0u}, {0u, 0u, 0u, 0u}};  // YpX = YmX = Z = 1, T2d = 0
__device__ __forceinline__ void lane_tables(uint4* ws, TableView& t1, TableView& t2) {
  const size_t lanes = (size_t)gridDim.x * kBlock;
  const size_t gl = (size_t)blockIdx.x * kBlock + threadIdx.x;
  uint4* head = ws + gl * kHeadQuads;
  uint4* tails = ws + lanes * kHeadQuads + gl * (2 * 9);
  t1 = TableView::split(head, tails, kIdentityHead);
  t2 = TableView::split(head + kHeadQuads / 2, tails + 9, kIdentityHead);
}
static_assert(kSlotQuads >= kHeadQuads + 2 * 9, "per-lane slot = heads + tails");

// Phase-1 state (HalfState) is written once and read once (non-temporal
// loads / stores measured +0.9 %, DESIGN_EXPERIMENTS.md).
typedef unsigned int stl_u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void st_state(uint4* p, uint4 v) {
  *p = v;
}
__device__ __forceinline__ uint4 ld_state(const uint4* p) {
  return *p;
}

template <int NQ, typename T>
__device__ __forceinline__ void ld_state_words(T& out, const uint4* q) {
  static_assert(sizeof(T) == NQ * 16, "size");
  uint32_t* w = reinterpret_cast<uint32_t*>(&out);
#pragma unroll
  for (int i = 0; i < NQ; ++i) {
    const uint4 v = ld_state(q + i);
    w[4 * i] = v.x; w[4 * i + 1] = v.y; w[4 * i + 2] = v.z; w[4 * i + 3] = v.w;
  }
}

template <int NQ, typename T>
__device__ __forceinline__ void ld_words(T& out, const uint4* q) {
  static_assert(sizeof(T) == NQ * 16, "size");
  uint32_t* w = reinterpret_cast<uint32_t*>(&out);
#pragma unroll
  for (int i = 0; i < NQ; ++i) {
    const uint4 v = q[i];
    w[4 * i] = v.x; w[4 * i + 1] = v.y; w[4 * i + 2] = v.z; w[4 * i + 3] = v.w;
  }
}

template <int NQ, typename T>
__device__ __forceinline__ void st_words(uint4* q, const T& in) {
  static_assert(sizeof(T) == NQ * 16, "size");
  const uint32_t* w = reinterpret_cast<const uint32_t*>(&in);
#pragma unroll
  for (int i = 0; i < NQ; ++i) q[i] = make_uint4(w[4 * i], w[4 * i + 1], w[4 * i + 2], w[4 * i + 3]);
}

__device__ __forceinline__ void load_k(uint32_t k[8], const uint32_t R[8], const uint32_t A[8],
                                       const uint8_t* msg_or_k, size_t j, bool pre_k) {
  uint32_t M[8];
  ld8(M, msg_or_k + 32 * j);
  if (pre_k) {
#pragma unroll
    for (int i = 0; i < 8; ++i) k[i] = M[i];
  } else {
    uint32_t h[16];
    sha512_hram32(h, R, A, M);
    sc_reduce64(k, h);
  }
}

// Phase 1a: one signature per lane -- k = SHA-512(R||A||M) mod L (or k
// given, PRE_K), lattice reduction of k to half-size (c, d), e = d*S mod L,
// digits.  Writes quads 0-4 of the lane's HalfState.  Signatures [base,
// base+cnt).
template <bool PRE_K>
__global__ __launch_bounds__(kBlock, STL_SCALAR_WAVES_PER_SIMD) void verify_scalar_kernel(
    const uint8_t* __restrict__ sig, const uint8_t* __restrict__ msg_or_k, const uint8_t* __restrict__ pk,
    uint32_t base, uint32_t cnt, uint4* __restrict__ pre) {
  const uint32_t t = blockIdx.x * kBlock + threadIdx.x;
  if (t >= cnt) return;  // no wave-level collective in this kernel
  const size_t j = (size_t)base + t;
  uint32_t R[8], S[8], A[8], k[8];
  ld8(R, sig + 64 * j);
  ld8(S, sig + 64 * j + 32);
  ld8(A, pk + 32 * j);
  load_k(k, R, A, msg_or_k, j, PRE_K);
  HalfState h;
  verify_phase1_scalars(h, S, k);
  const uint32_t* w = reinterpret_cast<const uint32_t*>(&h);
  uint4* q = pre + (size_t)t * 14;
#pragma unroll
  for (int i = 0; i < kHalfScalarQuads; ++i) st_state(q + i, make_uint4(w[4 * i], w[4 * i + 1], w[4 * i + 2], w[4 * i + 3]));
}

// Phase 1b: pre-checks, decompression of A and R, signed P1 / P2, final
// flags (quad 2 rewritten, quads 5-13 written); one ballot word of "needs
// the full-length path" flags per wave.
__global__ __launch_bounds__(kBlock, STL_PRE_WAVES_PER_SIMD) void verify_point_kernel(
    const uint8_t* __restrict__ sig, const uint8_t* __restrict__ pk, uint32_t base, uint32_t cnt, uint32_t policy,
    uint4* __restrict__ pre, uint64_t* __restrict__ fb_words) {
  const uint32_t t = blockIdx.x * kBlock + threadIdx.x;
  const bool live = t < cnt;
  const uint32_t tt = live ? t : cnt - 1;
  const size_t j = (size_t)base + tt;
  uint32_t R[8], S[8], A[8];
  ld8(R, sig + 64 * j);
  ld8(S, sig + 64 * j + 32);
  ld8(A, pk + 32 * j);
  uint4* q = pre + (size_t)tt * 14;
  HalfState h;
  uint32_t* w = reinterpret_cast<uint32_t*>(&h);
  const uint4 q2 = q[kHalfTopsWord / 4];
  w[8] = q2.x; w[9] = q2.y; w[10] = q2.z; w[11] = q2.w;
  static_assert(kHalfTopsWord == 10, "tops is word 2 of quad 2");
  verify_phase1_points(h, R, S, A, core_policy(policy));
  if ((policy & kModeFullLength) && (h.tops & kHalfOk)) h.tops |= kHalfFallback;
  if (live) {
    st_state(q + kHalfTopsWord / 4, make_uint4(w[8], w[9], w[10], w[11]));
#pragma unroll
    for (int i = kHalfScalarQuads; i < 14; ++i) st_state(q + i, make_uint4(w[4 * i], w[4 * i + 1], w[4 * i + 2], w[4 * i + 3]));
  }
  const uint64_t fb = __ballot(live && (h.tops & kHalfFallback) != 0);
  if ((threadIdx.x & 63u) == 0 && t < cnt) fb_words[t >> 6] = fb;
}

// Phase 1 in one launch (the default for chunks that run one lane per
// signature without key dedup): the scalar half, then the point half, in the
// same lane.  The two halves' state never leaves the registers between them,
// and the chunk pays one kernel boundary instead of two -- the scalar
// kernel alone ends in a ragged last round (3.2 rounds of 5 workgroups per
// CU for 2^20 signatures).
template <bool PRE_K>
__global__ __launch_bounds__(kBlock, STL_PRE_WAVES_PER_SIMD) void verify_prep_kernel(
    const uint8_t* __restrict__ sig, const uint8_t* __restrict__ msg_or_k, const uint8_t* __restrict__ pk,
    uint32_t base, uint32_t cnt, uint32_t policy, uint4* __restrict__ pre, uint64_t* __restrict__ fb_words) {
  const uint32_t t = blockIdx.x * kBlock + threadIdx.x;
  const bool live = t < cnt;
  const uint32_t tt = live ? t : cnt - 1;
  const size_t j = (size_t)base + tt;
  uint32_t R[8], S[8], A[8], k[8];
  ld8(R, sig + 64 * j);
  ld8(S, sig + 64 * j + 32);
  ld8(A, pk + 32 * j);
  load_k(k, R, A, msg_or_k, j, PRE_K);
  HalfState h;
  verify_phase1_scalars(h, S, k);
  // the scalar half's digits leave the registers before the square-root
  // chains (only `tops` stays live); quad 2 is rewritten with the final flags.
  // Same-box A/B: -0.3 % per launch against storing all 14 quads at the end
  // (profiles/r03/c).
  uint4* q = pre + (size_t)tt * 14;
  {
    const uint32_t* w = reinterpret_cast<const uint32_t*>(&h);
    if (live) {
#pragma unroll
      for (int i = 0; i < kHalfScalarQuads; ++i)
        st_state(q + i, make_uint4(w[4 * i], w[4 * i + 1], w[4 * i + 2], w[4 * i + 3]));
    }
  }
  verify_phase1_points(h, R, S, A, core_policy(policy));
  if ((policy & kModeFullLength) && (h.tops & kHalfOk)) h.tops |= kHalfFallback;
  if (live) {
    const uint32_t* w = reinterpret_cast<const uint32_t*>(&h);
    st_state(q + kHalfTopsWord / 4, make_uint4(w[8], w[9], w[10], w[11]));
#pragma unroll
    for (int i = kHalfScalarQuads; i < 14; ++i)
      st_state(q + i, make_uint4(w[4 * i], w[4 * i + 1], w[4 * i + 2], w[4 * i + 3]));
  }
  const uint64_t fb = __ballot(live && (h.tops & kHalfFallback) != 0);
  if ((threadIdx.x & 63u) == 0 && t < cnt) fb_words[t >> 6] = fb;
}

// The value of the other lane of this lane's pair (lane ^ 1): one DPP move,
// quad_perm [1,0,3,2] (dpp_ctrl 0xB1), a register-to-register swap inside the
// VALU -- __shfl_xor lowers to ds_bpermute_b32, an LDS round trip per value.
__device__ __forceinline__ uint32_t pair_swap(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, false);
}


// Phase 1 of the lane-pair path (chunks that run verify_main_pair_kernel) as
// ONE launch whose workgroups take one of two roles, so the scalar half
// (SHA-512, lattice: a latency-bound chain) and the two square-root chains run
// side by side on different CUs instead of one launch after the other -- a
// small batch leaves most of the chip idle, so the phase costs the longer of
// the two chains, not their sum:
//   blocks [0, nbs)         scalar role, one lane per signature: quads 0-3
//                           and words 16-18 of the HalfState (digits, tops
//                           with the c / d signs and the fit flag);
//   blocks [nbs, gridDim)   point role, two lanes per signature (lane 2j
//                           decodes A, 2j+1 decodes R, one DPP swap): lane 0
//                           stores -A and -Q raw in quads 5-13 and word 19 =
//                           pre-checks && both decodings (kPairPointOk).
// The two roles write disjoint words; verify_main_pair_kernel combines them
// (finish_phase1_points, as the split kernels do) and writes the fallback
// words.
constexpr uint32_t kPairPointOk = 1u;
template <bool PRE_K>
__global__ __launch_bounds__(kBlock, 2) void verify_prep_pair_kernel(
    const uint8_t* __restrict__ sig, const uint8_t* __restrict__ msg_or_k, const uint8_t* __restrict__ pk,
    uint32_t base, uint32_t cnt, uint32_t policy, uint4* __restrict__ pre, uint32_t nbs) {
  if (blockIdx.x < nbs) {  // scalar role (workgroup-uniform)
    const uint32_t t = blockIdx.x * kBlock + threadIdx.x;
    if (t >= cnt) return;  // no wave-level collective in this role
    const size_t j = (size_t)base + t;
    uint32_t R[8], S[8], A[8], k[8];
    ld8(R, sig + 64 * j);
    ld8(S, sig + 64 * j + 32);
    ld8(A, pk + 32 * j);
    load_k(k, R, A, msg_or_k, j, PRE_K);
    HalfState h;
    verify_phase1_scalars(h, S, k);
    const uint32_t* w = reinterpret_cast<const uint32_t*>(&h);
    uint4* q = pre + (size_t)t * 14;
#pragma unroll
    for (int i = 0; i < 4; ++i) st_state(q + i, make_uint4(w[4 * i], w[4 * i + 1], w[4 * i + 2], w[4 * i + 3]));
    uint32_t* q4 = reinterpret_cast<uint32_t*>(q + 4);  // words 16-18; word 19 is the point role's
    q4[0] = w[16];
    q4[1] = w[17];
    q4[2] = w[18];
    return;
  }
  const uint32_t g = (blockIdx.x - nbs) * kBlock + threadIdx.x;  // point role
  const uint32_t t = g >> 1;
  const int par = (int)(g & 1u);
  const bool live = t < cnt;
  const uint32_t tt = live ? t : cnt - 1;
  const size_t j = (size_t)base + tt;
  uint32_t R[8], A[8];
  ld8(R, sig + 64 * j);
  ld8(A, pk + 32 * j);
  fe mx, my, ox, oy;
  const bool mok = phase1_decode_lane(mx, my, R, A, par);
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    ox.v[i] = pair_swap(mx.v[i]);
    oy.v[i] = pair_swap(my.v[i]);
  }
  const bool ook = pair_swap((uint32_t)mok) != 0;
  if (live && par == 0) {  // lane 0 holds A's decoding in m, R's in o
    uint32_t S[8];
    ld8(S, sig + 64 * j + 32);
    const uint32_t pol = core_policy(policy);
    const bool ok = phase1_points_ok(R, S, A, pol, mok, ook);
    HalfState h;
    h.P1x = mx;
    h.P1y = my;
    h.P2x = ox;
    h.P2y = oy;
    h.pad = ok ? kPairPointOk : 0u;
    const uint32_t* w = reinterpret_cast<const uint32_t*>(&h);
    uint4* q = pre + (size_t)t * 14;
    reinterpret_cast<uint32_t*>(q + 4)[3] = w[19];
#pragma unroll
    for (int i = kHalfScalarQuads; i < 14; ++i) st_state(q + i, make_uint4(w[4 * i], w[4 * i + 1], w[4 * i + 2], w[4 * i + 3]));
  }
}

// After verify_prep_pair_kernel, for chunks whose point decodings run on lane
// pairs but whose main kernel runs one lane per signature (between a quarter
// and a half of the resident lanes): the two roles' words -> the finished
// HalfState the one-lane main kernel reads, and the fallback words, one lane
// per signature.
__global__ __launch_bounds__(kBlock) void verify_finish_pair_kernel(uint32_t cnt, uint32_t policy,
                                                                    uint4* __restrict__ pre,
                                                                    uint64_t* __restrict__ fb_words) {
  const uint32_t t = blockIdx.x * kBlock + threadIdx.x;
  const bool live = t < cnt;
  uint4* q = pre + (size_t)(live ? t : cnt - 1) * 14;
  HalfState h;
  ld_state_words<14>(h, q);
  const fe nAx = h.P1x, nAy = h.P1y, nQx = h.P2x, nQy = h.P2y;
  finish_phase1_points(h, nAx, nAy, nQx, nQy, (h.pad & kPairPointOk) != 0);
  if ((policy & kModeFullLength) && (h.tops & kHalfOk)) h.tops |= kHalfFallback;
  if (live) {
    const uint32_t* w = reinterpret_cast<const uint32_t*>(&h);
    st_state(q + kHalfTopsWord / 4, make_uint4(w[8], w[9], w[10], w[11]));
#pragma unroll
    for (int i = kHalfScalarQuads; i < 14; ++i) st_state(q + i, make_uint4(w[4 * i], w[4 * i + 1], w[4 * i + 2], w[4 * i + 3]));
  }
  const uint64_t fb = __ballot(live && (h.tops & kHalfFallback) != 0);
  if ((threadIdx.x & 63u) == 0 && t < cnt) fb_words[t >> 6] = fb;
}

// ---- per-batch key dedup (STL_DEDUP_KEYS) ----
// stellard's signers repeat (configs 1 and 5: 1,000 accounts for 100k
// transactions), so the batch decodes each distinct key once:
//   key_insert_kernel   open addressing on a table of 2*chunk slots: the first
//                       lane to claim a key's slot owns it, later lanes with
//                       the same 32 bytes point at the owner; owners get
//                       compact ids (one atomic per wave).  At most
//                       kKeyProbes probes: a lane that finds no slot (a
//                       crowded or adversarial table) owns its own key, so the
//                       work per lane stays bounded;
//   key_decode_kernel   one lane per distinct key: the square-root chain of -A,
//                       and the key's 9-entry table;
//   key_table_wide_base_kernel / key_table_wide_pair_kernel  few keys, many
//                       signatures each (kWideKeys, kWideKeyRepeat): j*(-A)
//                       for j = 0..136, the table of c's radix-256 digit
//                       pairs -- 24 entries by double-and-add, the others one
//                       addition of two of them;
//   verify_point_kernel_keyed  the point half with only R decoded.
constexpr uint32_t kKeyEmpty = 0xffffffffu;
constexpr int kKeyProbes = 32;

__device__ __forceinline__ uint32_t key_hash(const uint32_t A[8]) {
  uint32_t h = A[0] * 0x9E3779B1u;
  h ^= A[1] * 0x85EBCA6Bu;
  h = (h << 13) | (h >> 19);
  h ^= A[2] * 0xC2B2AE35u;
  h ^= A[5] * 0x27D4EB2Fu;
  h ^= h >> 16;
  return h * 0x7FEB352Du;
}

// Key-repeat sample of the device-resident API's automatic dedup choice
// (stl_api.cpp, StreamCtx::auto_flag): one workgroup puts up to kSampleKeys
// evenly spaced keys of [0, n) into an LDS table of 64-bit fingerprints and
// writes 1 to *flag (host-mapped memory, read by the next call on the stream)
// when at least a quarter of them repeat an earlier sampled key.  The choice
// only selects a path: the accept bits are the same either way.
constexpr uint32_t kSampleKeys = 2048, kSampleSlots = 4096, kSampleBlock = 1024;
__global__ __launch_bounds__(kSampleBlock) void key_sample_kernel(const uint8_t* __restrict__ pk, uint32_t n,
                                                                  uint32_t* __restrict__ flag) {
  __shared__ unsigned long long tab[kSampleSlots];
  __shared__ uint32_t dups;
  for (uint32_t i = threadIdx.x; i < kSampleSlots; i += kSampleBlock) tab[i] = 0;
  if (threadIdx.x == 0) dups = 0;
  __syncthreads();
  const uint32_t s = n < kSampleKeys ? n : kSampleKeys;
  for (uint32_t k = threadIdx.x; k < s; k += kSampleBlock) {
    uint32_t A[8];
    ld8(A, pk + 32 * ((uint64_t)k * n / s));
    const unsigned long long a = ((unsigned long long)A[1] << 32) | A[0];
    const unsigned long long c = ((unsigned long long)A[7] << 32) | A[6];
    const unsigned long long f = (a ^ (c * 0x9E3779B97F4A7C15ull)) | 1ull;  // 0 marks an empty slot
    uint32_t h = (uint32_t)((f * 0xD6E8FEB86659FD93ull) >> 52) & (kSampleSlots - 1);
    for (uint32_t probe = 0; probe < kSampleSlots; ++probe) {
      const unsigned long long old = atomicCAS(&tab[h], 0ull, f);
      if (old == 0ull) break;
      if (old == f) {
        atomicAdd(&dups, 1u);
        break;
      }
      h = (h + 1u) & (kSampleSlots - 1);
    }
  }
  __syncthreads();
  if (threadIdx.x < 64) {  // one wave writes the (uniform) verdict with a vector store
    const uint32_t v = 4u * dups >= s ? 1u : 0u;
    if (threadIdx.x == 0) *flag = v;
  }
}

hipError_t launch_key_sample(const uint8_t* pk, uint32_t n, uint32_t* flag, hipStream_t stream) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(key_sample_kernel, dim3(1), dim3(kSampleBlock), 0, stream, pk, n, flag);
  return hipGetLastError();
}

// Shader-clock stamps (stl_debug_clock_stamp; bench.py's clock_ghz, VERDICT
// r5 #5): lane 0 of each one-wave workgroup writes the free-running shader
// cycle counter (s_memtime), the 100 MHz constant-rate counter
// (s_memrealtime), and the XCC_ID / HW_ID registers naming the XCD, shader
// engine and CU it ran on.  Two stamps around a timed region give the average
// shader clock over it as d(memtime) / d(memrealtime) x 100 MHz, taken per
// XCD (each XCD keeps its own cycle counter).  Vector stores only.
__global__ __launch_bounds__(64) void clock_stamp_kernel(unsigned long long* __restrict__ out) {
  if (threadIdx.x != 0) return;
  const unsigned long long rt = __builtin_amdgcn_s_memrealtime();
  const unsigned long long t = __builtin_amdgcn_s_memtime();
  uint32_t xcc, hw;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
  unsigned long long* o = out + 4 * (size_t)blockIdx.x;
  o[0] = t;
  o[1] = rt;
  o[2] = xcc;
  o[3] = hw;
}

hipError_t launch_clock_stamp(unsigned long long* out, uint32_t nwg, hipStream_t stream) {
  if (nwg == 0) return hipSuccess;
  hipLaunchKernelGGL(clock_stamp_kernel, dim3(nwg), dim3(64), 0, stream, out);
  return hipGetLastError();
}

// The key-dedup chain (insert, decode, wide tables) is a few latency-bound
// waves (one lane per distinct key) that gate every chunk of a call, while
// the chunks' own phase-1 kernels fill the same SIMDs: its waves raise their
// issue priority (s_setprio, wave-level arbitration only) so their dependent
// chains do not queue behind the co-resident waves.
#ifndef STL_CHAIN_PRIO
#define STL_CHAIN_PRIO 3
#endif
__device__ __forceinline__ void chain_priority() {
  if (STL_CHAIN_PRIO > 0) __builtin_amdgcn_s_setprio(STL_CHAIN_PRIO);
}

__global__ __launch_bounds__(kBlock) void key_insert_kernel(const uint8_t* __restrict__ pk, uint32_t base,
                                                            uint32_t cnt, uint32_t* __restrict__ slots, uint32_t mask,
                                                            uint32_t* __restrict__ rep, uint32_t* __restrict__ uid_of,
                                                            uint32_t* __restrict__ counter,
                                                            uint32_t* __restrict__ owners) {
  chain_priority();
  const uint32_t t = blockIdx.x * kBlock + threadIdx.x;
  const uint32_t lane = threadIdx.x & 63u;
  const bool live = t < cnt;
  uint32_t r = t;
  if (live) {
    uint32_t A[8];
    ld8(A, pk + 32 * ((size_t)base + t));
    uint32_t h = key_hash(A) & mask;
    for (int probe = 0; probe < kKeyProbes; ++probe) {
      const uint32_t old = atomicCAS(&slots[h], kKeyEmpty, t);
      if (old == kKeyEmpty) break;  // claimed: this lane owns the key (r == t)
      uint32_t B[8];
      ld8(B, pk + 32 * ((size_t)base + old));
      bool eq = true;
#pragma unroll
      for (int i = 0; i < 8; ++i) eq = eq && A[i] == B[i];
      if (eq) {
        r = old;
        break;
      }
      h = (h + 1u) & mask;
    }
    rep[t] = r;
  }
  // compact ids for the owners: one atomic per wave (no loop: the broadcast
  // base only offsets each owner lane's own id)
  const bool owner = live && r == t;
  const uint64_t m = __ballot(owner);
  if (m == 0) return;
  const int leader = __ffsll((unsigned long long)m) - 1;
  uint32_t b0 = 0;
  if ((int)lane == leader) b0 = atomicAdd(counter, (uint32_t)__popcll(m));
  b0 = __shfl(b0, leader);
  if (owner) {
    const uint32_t u = b0 + (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
    uid_of[t] = u;
    owners[u] = t;
  }
}

// the chunk's keys get the wide tables (wave-uniform: one chunk per launch)
__device__ __forceinline__ bool wide_keys(uint32_t nu, uint32_t cnt) {
  return nu <= kWideKeys && (uint64_t)nu * kWideKeyRepeat <= cnt;
}

__global__ __launch_bounds__(kBlock, 4) void key_decode_kernel(const uint8_t* __restrict__ pk, uint32_t base,
                                                               const uint32_t* __restrict__ counter,
                                                               const uint32_t* __restrict__ owners,
                                                               uint4* __restrict__ keytab,
                                                               uint4* __restrict__ keytabs, uint32_t cnt) {
  chain_priority();
  const uint32_t u = blockIdx.x * kBlock + threadIdx.x;
  const uint32_t nu = *counter;
  if (u >= nu) return;  // no wave-level collective in this kernel
  uint32_t A[8];
  ld8(A, pk + 32 * ((size_t)base + owners[u]));
  ge_p3 negA;
  const bool ok = ge_frombytes_negate_vartime(negA, A);
  uint32_t w[20];
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    w[i] = negA.X.v[i];
    w[9 + i] = negA.Y.v[i];
  }
  w[18] = ok ? 1u : 0u;
  w[19] = 0;
  uint4* q = keytab + (size_t)u * 5;
#pragma unroll
  for (int i = 0; i < 5; ++i) q[i] = make_uint4(w[4 * i], w[4 * i + 1], w[4 * i + 2], w[4 * i + 3]);
  if (nu <= kKeyTables && !wide_keys(nu, cnt)) {  // the shared A-table: j*(-A), j = 0..8, as a lane would build it
    ge_p3 P;
    affine_to_p3(P, negA.X, negA.Y);
    build_cached_table(TableView::contiguous(keytabs + (size_t)u * kTableQuadsPerKey), P);
  }
}

// The chunk's wide key tables j*(-A), j = 0..136, in two stages
// (stl_verify_core.h wide_base_index / wide_pair_entry), each a no-op unless
// the chunk is in wide mode.  Stage 1: one lane per (key u, i < 24) builds
// entry wide_base_index(i) by double-and-add from the decoded key.
__device__ __forceinline__ void wide_key_point(fe& x, fe& y, const uint4* __restrict__ keytab, uint32_t u) {
  const uint4* kq = keytab + (size_t)u * 5;
  uint32_t kw[20];
#pragma unroll
  for (int i = 0; i < 5; ++i) {
    const uint4 v = kq[i];
    kw[4 * i] = v.x; kw[4 * i + 1] = v.y; kw[4 * i + 2] = v.z; kw[4 * i + 3] = v.w;
  }
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    x.v[i] = kw[i];
    y.v[i] = kw[9 + i];
  }
}

__global__ __launch_bounds__(kBlock) void key_table_wide_base_kernel(const uint32_t* __restrict__ counter,
                                                                     uint32_t cnt, const uint4* __restrict__ keytab,
                                                                     uint4* __restrict__ widetabs) {
  chain_priority();
  const uint32_t nu = *counter;
  if (!wide_keys(nu, cnt)) return;
  const uint32_t g = blockIdx.x * kBlock + threadIdx.x;
  const uint32_t u = g / (uint32_t)kWideBaseEntries, i = g % (uint32_t)kWideBaseEntries;
  if (u >= nu) return;  // no wave-level collective in this kernel
  fe x, y;
  wide_key_point(x, y, keytab, u);
  const int j = wide_base_index((int)i);
  ge_cached c;
  small_multiple_cached(c, x, y, j);
  TableView::contiguous(widetabs + (size_t)u * (kWideKeyEntries * 9)).store(j, c);
}

// Stage 2: one lane per (key u, entry j = 16b + a, b >= 1, a = 1..15):
// entry 16b + entry a.
__global__ __launch_bounds__(kBlock) void key_table_wide_pair_kernel(const uint32_t* __restrict__ counter,
                                                                     uint32_t cnt, uint4* __restrict__ widetabs) {
  chain_priority();
  const uint32_t nu = *counter;
  if (!wide_keys(nu, cnt)) return;
  const uint32_t g = blockIdx.x * kBlock + threadIdx.x;
  const uint32_t u = g / (uint32_t)kWideKeyEntries, j = g % (uint32_t)kWideKeyEntries;
  if (u >= nu || j < 16 || (j & 15u) == 0) return;  // no wave-level collective in this kernel
  const TableView tv = TableView::contiguous(widetabs + (size_t)u * (kWideKeyEntries * 9));
  ge_cached hi, lo, c;
  tv.load((int)(j & ~15u), hi);
  tv.load((int)(j & 15u), lo);
  wide_pair_entry(c, hi, lo);
  tv.store((int)j, c);
}

// The keyed point half split in two (round 6), so that R's square-root chain
// runs while the key domain is still being built instead of after it:
//   verify_point_r_kernel      rows [0, n) of a call, one lane each: the
//                              pre-checks, stellard's S < L, R canonical and
//                              R's decoding -Q, into rdec[i] (5 quads: -Q x, y,
//                              word 18 = all of them passed);
//   verify_finish_keyed_kernel a chunk's rows once rdec and the key domain are
//                              ready: -A from the key table, then exactly the
//                              state verify_point_kernel_keyed writes.
// verify_phase1_points_keyed is the same computation in one lane.
__global__ __launch_bounds__(kBlock, 4) void verify_point_r_kernel(const uint8_t* __restrict__ sig,
                                                                   const uint8_t* __restrict__ pk, uint32_t n,
                                                                   uint32_t policy, uint4* __restrict__ rdec) {
  const uint32_t t = blockIdx.x * kBlock + threadIdx.x;
  if (t >= n) return;  // no wave-level collective in this kernel
  uint32_t R[8], S[8], A[8];
  ld8(R, sig + 64 * (size_t)t);
  ld8(S, sig + 64 * (size_t)t + 32);
  ld8(A, pk + 32 * (size_t)t);
  const uint32_t pol = core_policy(policy);
  bool ok = verify_prechecks(R, S, A, pol);
  ok = ok && composite_s_ok(S, pol) && r_is_canonical(R);
  ge_p3 negQ;
  const bool okR = ge_frombytes_negate_vartime(negQ, R);
  uint32_t w[20];
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    w[i] = negQ.X.v[i];
    w[9 + i] = negQ.Y.v[i];
  }
  w[18] = ok && okR ? 1u : 0u;
  w[19] = 0;
  uint4* q = rdec + (size_t)t * 5;
#pragma unroll
  for (int i = 0; i < 5; ++i) q[i] = make_uint4(w[4 * i], w[4 * i + 1], w[4 * i + 2], w[4 * i + 3]);
}

__global__ __launch_bounds__(kBlock, 4) void verify_finish_keyed_kernel(
    uint32_t cnt, uint32_t policy, uint4* __restrict__ pre, uint64_t* __restrict__ fb_words,
    const uint32_t* __restrict__ rep, const uint32_t* __restrict__ uid_of, const uint4* __restrict__ keytab,
    const uint32_t* __restrict__ counter, uint32_t kcnt, const uint4* __restrict__ rdec) {
  const uint32_t t = blockIdx.x * kBlock + threadIdx.x;
  const bool live = t < cnt;
  const uint32_t tt = live ? t : cnt - 1;
  const uint32_t uid = uid_of[rep[tt]];
  uint32_t kw[20], rw[20];
#pragma unroll
  for (int i = 0; i < 5; ++i) {
    const uint4 v = keytab[(size_t)uid * 5 + i];
    kw[4 * i] = v.x; kw[4 * i + 1] = v.y; kw[4 * i + 2] = v.z; kw[4 * i + 3] = v.w;
    const uint4 r = rdec[(size_t)tt * 5 + i];
    rw[4 * i] = r.x; rw[4 * i + 1] = r.y; rw[4 * i + 2] = r.z; rw[4 * i + 3] = r.w;
  }
  fe nAx, nAy, nQx, nQy;
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    nAx.v[i] = kw[i];
    nAy.v[i] = kw[9 + i];
    nQx.v[i] = rw[i];
    nQy.v[i] = rw[9 + i];
  }
  uint4* q = pre + (size_t)tt * 14;
  HalfState h;
  uint32_t* w = reinterpret_cast<uint32_t*>(&h);
  const uint4 q2 = q[kHalfTopsWord / 4], q4 = q[4];
  w[8] = q2.x; w[9] = q2.y; w[10] = q2.z; w[11] = q2.w;
  w[16] = q4.x; w[17] = q4.y; w[18] = q4.z;
  const uint32_t c_neg = h.tops & kHalfCNeg;
  finish_phase1_points(h, nAx, nAy, nQx, nQy, rw[18] != 0 && kw[18] != 0);
  if ((policy & kModeFullLength) && (h.tops & kHalfOk)) h.tops |= kHalfFallback;
  h.pad = uid;
  const uint32_t nu = *counter;
  if (nu <= kKeyTables) h.tops |= kHalfKeyed | c_neg;  // the main kernel reads the key's table
  if (wide_keys(nu, kcnt)) h.tops |= kHalfKeyedWide;
  if (live) {
    q[4] = make_uint4(w[16], w[17], w[18], w[19]);
    st_state(q + kHalfTopsWord / 4, make_uint4(w[8], w[9], w[10], w[11]));
#pragma unroll
    for (int i = kHalfScalarQuads; i < 14; ++i) st_state(q + i, make_uint4(w[4 * i], w[4 * i + 1], w[4 * i + 2], w[4 * i + 3]));
  }
  const uint64_t fb = __ballot(live && (h.tops & kHalfFallback) != 0);
  if ((threadIdx.x & 63u) == 0 && t < cnt) fb_words[t >> 6] = fb;
}

hipError_t launch_point_r(const uint8_t* sig, const uint8_t* pk, uint32_t n, uint32_t policy, uint4* rdec,
                          hipStream_t stream) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(verify_point_r_kernel, dim3((n + kBlock - 1) / kBlock), dim3(kBlock), 0, stream, sig, pk, n,
                     policy, rdec);
  return hipGetLastError();
}

// Phase 1b with the keys already decoded: only R's square-root chain, so the
// kernel runs at more waves per SIMD than the paired one.
__global__ __launch_bounds__(kBlock, 4) void verify_point_kernel_keyed(
    const uint8_t* __restrict__ sig, const uint8_t* __restrict__ pk, uint32_t base, uint32_t cnt, uint32_t policy,
    uint4* __restrict__ pre, uint64_t* __restrict__ fb_words, const uint32_t* __restrict__ rep,
    const uint32_t* __restrict__ uid_of, const uint4* __restrict__ keytab, const uint32_t* __restrict__ counter,
    uint32_t kcnt) {
  const uint32_t t = blockIdx.x * kBlock + threadIdx.x;
  const bool live = t < cnt;
  const uint32_t tt = live ? t : cnt - 1;
  const size_t j = (size_t)base + tt;
  uint32_t R[8], S[8], A[8];
  ld8(R, sig + 64 * j);
  ld8(S, sig + 64 * j + 32);
  ld8(A, pk + 32 * j);
  const uint32_t uid = uid_of[rep[tt]];
  const uint4* kq = keytab + (size_t)uid * 5;
  uint32_t kw[20];
#pragma unroll
  for (int i = 0; i < 5; ++i) {
    const uint4 v = kq[i];
    kw[4 * i] = v.x; kw[4 * i + 1] = v.y; kw[4 * i + 2] = v.z; kw[4 * i + 3] = v.w;
  }
  fe nAx, nAy;
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    nAx.v[i] = kw[i];
    nAy.v[i] = kw[9 + i];
  }
  uint4* q = pre + (size_t)tt * 14;
  HalfState h;
  uint32_t* w = reinterpret_cast<uint32_t*>(&h);
  const uint4 q2 = q[kHalfTopsWord / 4], q4 = q[4];
  w[8] = q2.x; w[9] = q2.y; w[10] = q2.z; w[11] = q2.w;
  w[16] = q4.x; w[17] = q4.y; w[18] = q4.z;
  const uint32_t c_neg = h.tops & kHalfCNeg;
  verify_phase1_points_keyed(h, R, S, A, core_policy(policy), nAx, nAy, kw[18] != 0);
  if ((policy & kModeFullLength) && (h.tops & kHalfOk)) h.tops |= kHalfFallback;
  h.pad = uid;
  const uint32_t nu = *counter;
  if (nu <= kKeyTables) h.tops |= kHalfKeyed | c_neg;  // the main kernel reads the key's table
  if (wide_keys(nu, kcnt)) h.tops |= kHalfKeyedWide;  // kcnt: the key domain's rows (key_table_wide_base_kernel's choice)
  if (live) {
    q[4] = make_uint4(w[16], w[17], w[18], w[19]);
    st_state(q + kHalfTopsWord / 4, make_uint4(w[8], w[9], w[10], w[11]));
#pragma unroll
    for (int i = kHalfScalarQuads; i < 14; ++i) st_state(q + i, make_uint4(w[4 * i], w[4 * i + 1], w[4 * i + 2], w[4 * i + 3]));
  }
  const uint64_t fb = __ballot(live && (h.tops & kHalfFallback) != 0);
  if ((threadIdx.x & 63u) == 0 && t < cnt) fb_words[t >> 6] = fb;
}

// Wide-table rows in HBM: 7 quads (3 x 9 canonical limbs + a pad word).
constexpr int kWideQuads = 7;

__device__ __forceinline__ void wide_row_to_niels(ge_niels& n, const uint32_t* row) {
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    n.ypx.v[i] = row[i];
    n.ymx.v[i] = row[9 + i];
    n.xy2d.v[i] = row[18 + i];
  }
}

// Wide rows read straight into VGPRs at the madd (the per-lane table tails
// take the LDS; staging the rows in LDS by global_load_lds measured slower,
// DESIGN_EXPERIMENTS.md).
struct WideGlobal {
  const uint4* gtab;
  int d[2];
  __device__ void prefetch(int d0, int d1) {
    d[0] = d0;
    d[1] = d1;
  }
  // the signed row of wide table `which` as a Niels point
  __device__ void niels(ge_niels& n, int which) const {
    const uint32_t a = (uint32_t)(d[which] < 0 ? -d[which] : d[which]);
    const uint4* src = gtab + ((size_t)which * kWideEntries + a) * kWideQuads;
    uint32_t row[4 * kWideQuads];
#pragma unroll
    for (int c = 0; c < kWideQuads; ++c) {
      const uint4 v = src[c];
      row[4 * c] = v.x; row[4 * c + 1] = v.y; row[4 * c + 2] = v.z; row[4 * c + 3] = v.w;
    }
    wide_row_to_niels(n, row);
    ge_niels_cneg(n, d[which] < 0);
  }
  __device__ void madd(ge_p1p1& t, const ge_p3& acc, int which) const {
    const uint32_t a = (uint32_t)(d[which] < 0 ? -d[which] : d[which]);
    const uint4* src = gtab + ((size_t)which * kWideEntries + a) * kWideQuads;
    uint32_t row[4 * kWideQuads];
#pragma unroll
    for (int c = 0; c < kWideQuads; ++c) {
      const uint4 v = src[c];
      row[4 * c] = v.x; row[4 * c + 1] = v.y; row[4 * c + 2] = v.z; row[4 * c + 3] = v.w;
    }
    ge_niels n;
    wide_row_to_niels(n, row);
    ge_niels_cneg(n, d[which] < 0);
    ge_madd(t, acc, n);
  }
};

// Phase 2: [e]B + [c](-A) + [d](-Q) == O over [base, base+cnt); one ballot
// word per wave.  The grid is the resident capacity (the per-lane table
// workspace is bounded by the resident lanes).  Work unit = 64 signatures
// (one wave, one bitmap word): with `queue` each wave pulls its next unit from
// that counter (zeroed by the launcher), so waves that finish early take more
// and the kernel's last round is not fixed in advance; without it the units
// are dealt out statically (grid stride).  Every wave leaves after one pull
// past the end.
// JOINT (chunks without key dedup): one joint radix-4 table of a*P1 + b*P2
// per lane (verify_phase2_joint); otherwise two radix-16 tables, the A-table
// possibly the key's shared one (verify_phase2_half).
template <bool JOINT>
__global__ __launch_bounds__(kBlock, STL_VERIFY_WAVES_PER_SIMD) void verify_main_kernel(
    const uint4* __restrict__ pre, uint32_t base, uint32_t cnt, uint64_t* __restrict__ bitmap,
    uint4* __restrict__ ws, const uint4* __restrict__ wide, unsigned long long* __restrict__ ctr,
    const uint4* __restrict__ keytabs, const uint4* __restrict__ widetabs, uint32_t* __restrict__ queue) {
  TableView tab1, tab2;
  lane_tables(ws, tab1, tab2);
  // The tables' 16-B tails live in LDS, [table*9 + entry][lane] (conflict-
  // free; 72 KiB per workgroup, two workgroups per CU): a lookup reads one
  // aligned HBM line (its head) and one LDS quad.  LDS then has no room for
  // the wide-row stage, so wide rows are read into VGPRs at their madd.
  // Same-box A/B: main kernel -4.1 %.
  __shared__ uint4 tails[18][kBlock];
  tab1.tail = &tails[0][threadIdx.x];
  tab2.tail = &tails[9][threadIdx.x];
  tab1.tstride = tab2.tstride = kBlock;
  const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63u;
  WideGlobal wl{wide, {0, 0}};
  const uint32_t units = (cnt + 63) >> 6;
  const uint32_t stride = gridDim.x * (kBlock / 64);
  uint32_t unit = blockIdx.x * (kBlock / 64) + wave;
  for (;;) {
    if (queue) {  // wave-uniform: one atomic per wave and unit
      // The claimed unit is broadcast with readfirstlane, so it lives in an
      // SGPR and the exit test below is a scalar compare (s_cmp + s_cbranch_scc
      // in the ISA): the loop is uniform control flow whose back-edge always
      // passes through the claim.  A VGPR broadcast (__shfl) would make the
      // exit test a VGPR compare that the structuriser may split into nested
      // exec-masked loops, one of them not re-running the claim (DESIGN.md
      // section 4, "Work queues": the round-5 long-row hang).
      uint32_t u = 0;
      if (lane == 0) u = atomicAdd(queue, 1u);
      unit = (uint32_t)__builtin_amdgcn_readfirstlane((int)u);
    }
    if (unit >= units) break;
    const uint32_t wbase = unit * 64;
    const uint32_t t = wbase + lane;
    const bool live = t < cnt;
    const uint4* st = pre + (size_t)(live ? t : cnt - 1) * 14;
    bool ok;
    if (JOINT) {
      ok = verify_phase2_joint(st, tab1, wl) && live;
    } else {
      HalfState h;
      ld_state_words<14>(h, st);
      ok = verify_phase2_half(h, tab1, tab2, wl, keytabs, widetabs) && live;
    }
    const uint64_t word = __ballot(ok);
    if (lane == 0) {
      bitmap[(base + wbase) >> 6] = word;
      if (ctr) atomicAdd(&ctr[0], (unsigned long long)__popcll(word));  // accepted (stl_get_stats)
    }
    if (!queue) unit += stride;
  }
}

// Phase 2 for small batches (2 x cnt lanes fit in one round of resident
// lanes, no key dedup): lanes 2j and 2j+1 run signature j's two half chains
// (verify_phase2_pair_chain) on one table each, swap their sums across the
// pair, and both test that they cancel.  A wave decides 32 signatures: the
// even bits of its ballot are one 32-bit half of a bitmap word (the other
// half is the next wave's, in the same tile).
__global__ __launch_bounds__(kBlock, STL_VERIFY_WAVES_PER_SIMD) void verify_main_pair_kernel(
    const uint4* __restrict__ pre, uint32_t base, uint32_t cnt, uint32_t policy, uint64_t* __restrict__ bitmap,
    uint64_t* __restrict__ fb_words, uint4* __restrict__ ws, const uint4* __restrict__ wide,
    unsigned long long* __restrict__ ctr) {
  TableView tab, unused;
  lane_tables(ws, tab, unused);
  __shared__ uint4 tails[9][kBlock];
  tab.tail = &tails[0][threadIdx.x];
  tab.tstride = kBlock;
  const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63u;
  const int par = (int)(lane & 1u);
  WideGlobal wl{wide, {0, 0}};
  const uint32_t words = (cnt + 63) >> 6;
  for (uint32_t tile = blockIdx.x * kBlock; tile < 2 * cnt; tile += gridDim.x * kBlock) {
    const uint32_t t = (tile + threadIdx.x) >> 1;  // signature of this lane pair
    const bool live = t < cnt;
    HalfState h;
    ld_state_words<14>(h, pre + (size_t)(live ? t : cnt - 1) * 14);
    {  // the two roles of verify_prep_pair_kernel -> P1 = sign(c) A, P2 = sign(d) Q, final flags
      const fe nAx = h.P1x, nAy = h.P1y, nQx = h.P2x, nQy = h.P2y;
      finish_phase1_points(h, nAx, nAy, nQx, nQy, (h.pad & kPairPointOk) != 0);
      if ((policy & kModeFullLength) && (h.tops & kHalfOk)) h.tops |= kHalfFallback;
    }
    const uint64_t fball = __ballot(live && (h.tops & kHalfFallback) != 0);
    ge_p2 mine, other;
    verify_phase2_pair_chain(mine, h, par, tab, wl);
#pragma unroll
    for (int i = 0; i < 9; ++i) {
      other.X.v[i] = pair_swap(mine.X.v[i]);
      other.Y.v[i] = pair_swap(mine.Y.v[i]);
      other.Z.v[i] = pair_swap(mine.Z.v[i]);
    }
    const bool ok = live && half_state_accepts(h) && pair_sums_cancel(mine, other);
    const uint64_t ball = __ballot(ok);
    uint32_t half = 0;  // the even lanes' bits, compressed
#pragma unroll
    for (int b = 0; b < 32; ++b) half |= (uint32_t)((ball >> (2 * b)) & 1u) << b;
    const uint32_t wsig = (tile + wave * 64) >> 1;  // first signature of this wave, a multiple of 32
    uint32_t fhalf = 0;  // fallback flags of the even lanes, for verify_fallback_kernel
#pragma unroll
    for (int b = 0; b < 32; ++b) fhalf |= (uint32_t)((fball >> (2 * b)) & 1u) << b;
    if (lane == 0 && (wsig >> 6) < words) {
      reinterpret_cast<uint32_t*>(fb_words)[wsig >> 5] = fhalf;
      reinterpret_cast<uint32_t*>(bitmap)[(base + wsig) >> 5] = half;
      if (ctr) atomicAdd(&ctr[0], (unsigned long long)__popc(half));  // accepted (stl_get_stats)
    }
  }
}

// ---- lane groups per chain: the smallest batches (verify_main_group_kernel) ----
// A chunk this small leaves most SIMDs idle, so its time is one lane's
// dependent chain, which a lone wave issues at about one mad64 per 5.8 cycles.
// Here the four products of each group formula (the squarings of a doubling,
// the products of an addition or of a conversion) are spread over a group of
// G lanes -- G = 4 (a quad: one product per lane, four DPP quad broadcasts)
// or G = 2 (a duo: two interleaved products per lane, one DPP pair swap) --
// and every lane then holds the whole point again.  Role bits b0 = lane & 1,
// b1 = lane & 2.
struct GroupRole {
  bool b0, b1;
};

template <int S>
__device__ __forceinline__ uint32_t quad_bcast(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, S | (S << 2) | (S << 4) | (S << 6), 0xF, 0xF, false);
}

__device__ __forceinline__ void fe_sel2(fe& o, const fe& a0, const fe& a1, bool b) {
#pragma unroll
  for (int i = 0; i < 9; ++i) o.v[i] = b ? a1.v[i] : a0.v[i];
}

// o = [a0, a1, a2, a3][role]
__device__ __forceinline__ void fe_sel4(fe& o, const fe& a0, const fe& a1, const fe& a2, const fe& a3, GroupRole r) {
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    const uint32_t lo = r.b0 ? a1.v[i] : a0.v[i];
    const uint32_t hi = r.b0 ? a3.v[i] : a2.v[i];
    o.v[i] = r.b1 ? hi : lo;
  }
}

__device__ __forceinline__ void quad_gather(fe out[4], const fe& p) {
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    out[0].v[i] = quad_bcast<0>(p.v[i]);
    out[1].v[i] = quad_bcast<1>(p.v[i]);
    out[2].v[i] = quad_bcast<2>(p.v[i]);
    out[3].v[i] = quad_bcast<3>(p.v[i]);
  }
}

// duo: this lane's products p0, p1 are products 2*b0 and 2*b0 + 1
__device__ __forceinline__ void duo_gather(fe out[4], const fe& p0, const fe& p1, bool b0) {
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    const uint32_t q0 = pair_swap(p0.v[i]), q1 = pair_swap(p1.v[i]);
    out[0].v[i] = b0 ? q0 : p0.v[i];
    out[1].v[i] = b0 ? q1 : p1.v[i];
    out[2].v[i] = b0 ? p0.v[i] : q0;
    out[3].v[i] = b0 ? p1.v[i] : q1;
  }
}

// out[j] = a_j * b_j on every lane of the group (same bounds as fe_mul)
template <int G>
__device__ __forceinline__ void group_mul4(fe out[4], const fe& a0, const fe& b0, const fe& a1, const fe& b1,
                                           const fe& a2, const fe& b2, const fe& a3, const fe& b3, GroupRole r) {
  if (G == 4) {
    fe a, b, p;
    fe_sel4(a, a0, a1, a2, a3, r);
    fe_sel4(b, b0, b1, b2, b3, r);
    fe_mul(p, a, b);
    quad_gather(out, p);
  } else {
    fe x0, y0, x1, y1, p0, p1;
    fe_sel2(x0, a0, a2, r.b0);
    fe_sel2(y0, b0, b2, r.b0);
    fe_sel2(x1, a1, a3, r.b0);
    fe_sel2(y1, b1, b3, r.b0);
    fe_mul2(p0, x0, y0, p1, x1, y1);
    duo_gather(out, p0, p1, r.b0);
  }
}

template <int G>
__device__ __forceinline__ void group_sq4(fe out[4], const fe& a0, const fe& a1, const fe& a2, const fe& a3,
                                          GroupRole r) {
  if (G == 4) {
    fe a, p;
    fe_sel4(a, a0, a1, a2, a3, r);
    fe_sq(p, a);
    quad_gather(out, p);
  } else {
    fe x0, x1, p0, p1;
    fe_sel2(x0, a0, a2, r.b0);
    fe_sel2(x1, a1, a3, r.b0);
    fe_sq2(p0, x0, p1, x1);
    duo_gather(out, p0, p1, r.b0);
  }
}

// ge_p2_dbl (non-lazy X): the four squarings spread over the group
template <int G>
__device__ __forceinline__ void group_p2_dbl(ge_p1p1& r, const ge_p2& p, GroupRole q) {
  fe XpY, S[4];
  fe_add(XpY, p.X, p.Y);     // [2]
  group_sq4<G>(S, p.X, p.Y, p.Z, XpY, q);  // XX, YY, Z^2, A
  fe ZZ2;
  fe_add(ZZ2, S[2], S[2]);   // [2]
  fe_add(r.Y, S[1], S[0]);   // [2]
  fe_sub_nc<2>(r.Z, S[1], S[0]);  // [3]
  fe_sub(r.X, S[3], r.Y);    // [1]
  fe_sub(r.T, ZZ2, r.Z);     // [1]
}

// ge_p1p1_to_p3 (the p2 conversion is its first three products)
template <int G>
__device__ __forceinline__ void group_to_p3(ge_p3& r, const ge_p1p1& t, GroupRole q) {
  fe O[4];
  group_mul4<G>(O, t.X, t.T, t.Y, t.Z, t.Z, t.T, t.X, t.Y, q);
  r.X = O[0];
  r.Y = O[1];
  r.Z = O[2];
  r.T = O[3];
}

template <int G>
__device__ __forceinline__ void group_to_p2(ge_p2& r, const ge_p1p1& t, GroupRole q) {
  ge_p3 p;
  group_to_p3<G>(p, t, q);
  r.X = p.X;
  r.Y = p.Y;
  r.Z = p.Z;
}

// ge_add_cached
template <int G>
__device__ __forceinline__ void group_add_cached(ge_p1p1& r, const ge_p3& p, const ge_cached& c, GroupRole q) {
  fe t, t2, O[4];
  fe_sub_nc<2>(t, p.Y, p.X);  // [3]
  fe_add(t2, p.Y, p.X);       // [2]
  group_mul4<G>(O, t, c.YmX, t2, c.YpX, c.T2d, p.T, p.Z, c.Z, q);
  fe D;
  fe_add(D, O[3], O[3]);      // [2]
  fe_sub_nc<2>(r.X, O[1], O[0]);  // [3]
  fe_add(r.Y, O[1], O[0]);    // [2]
  fe_add(r.Z, D, O[2]);       // [3]
  fe_sub(r.T, D, O[2]);       // [1]
}

// ge_madd (the fourth product is not used)
template <int G>
__device__ __forceinline__ void group_madd(ge_p1p1& r, const ge_p3& p, const ge_niels& n, GroupRole q) {
  fe t, t2, O[4];
  fe_sub_nc<2>(t, p.Y, p.X);  // [3]
  fe_add(t2, p.Y, p.X);       // [2]
  group_mul4<G>(O, t, n.ymx, t2, n.ypx, n.xy2d, p.T, p.Z, p.Z, q);
  fe D;
  fe_add(D, p.Z, p.Z);        // [2]
  fe_sub_nc<2>(r.X, O[1], O[0]);  // [3]
  fe_add(r.Y, O[1], O[0]);    // [2]
  fe_add(r.Z, D, O[2]);       // [3]
  fe_sub(r.T, D, O[2]);       // [1]
}

// build_cached_table on a group: entries 2..8 from group doublings / madds
// (same points; the doubling of the affine P with Z = 1 is ge_affine_dbl's
// arithmetic), the cached conversions on every lane, the stores by `store`.
template <int G>
__device__ void group_build_table(const TableView& tab, const ge_p3& P, GroupRole q, bool store) {
  ge_cached c1, c;
  ge_cached_0(c);
  if (store) tab.store(0, c);
  ge_p3_to_cached(c1, P);
  if (store) tab.store(1, c1);
  ge_niels n1;
  n1.ypx = c1.YpX;
  n1.ymx = c1.YmX;
  n1.xy2d = c1.T2d;
  ge_p1p1 t;
  ge_p3 p3;
  {
    ge_p2 P2;
    P2.X = P.X;
    P2.Y = P.Y;
    P2.Z = P.Z;
    group_p2_dbl<G>(t, P2, q);
  }
  group_to_p3<G>(p3, t, q);
  ge_p3_to_cached(c, p3);
  if (store) tab.store(2, c);
#pragma unroll 1
  for (int e = 3; e <= 8; ++e) {
    group_madd<G>(t, p3, n1, q);
    group_to_p3<G>(p3, t, q);
    ge_p3_to_cached(c, p3);
    if (store) tab.store(e, c);
  }
}

// verify_phase2_pair_chain on a group: the same digits, table and wide-row
// schedule, every group formula spread over the G lanes.  One table per
// group (built by the group, stored by its role-0 lane).
template <int G>
__device__ void group_chain(ge_p2& out, const HalfState& p, int par, const TableView& tab, const WideGlobal& wide0,
                            GroupRole q, bool store) {
  WideGlobal wide = wide0;
  {
    ge_p3 P;
    affine_to_p3(P, par ? p.P2x : p.P1x, par ? p.P2y : p.P1y);
    group_build_table<G>(tab, P, q, store);
  }
  __syncthreads();  // role 0's stores before the group's loads (LDS tails, global heads)
  const int npos = half_positions((int)(p.tops & 0xffu));
  uint32_t dg[5], ed[4];
#pragma unroll
  for (int i = 0; i < 5; ++i) dg[i] = par ? p.ddig[i] : p.cdig[i];
#pragma unroll
  for (int i = 0; i < 4; ++i) ed[i] = par ? p.edig[4 + i] : p.edig[i];
  ge_p3 acc;
  ge_p2 acc2;
  ge_p1p1 t;
  ge_p3_0(acc);
  ge_p2_0(acc2);
  uint32_t w = 0, we = 0;
#pragma unroll 1
  for (int i = kHalfDigits - 1; i >= 0; --i) {
    if ((i & 7) == 7) {
      w = dg[4];
#pragma unroll
      for (int m = 4; m > 0; --m) dg[m] = dg[m - 1];
    }
    if ((i & 7) == 4 && i < 32) {
      we = ed[3];
#pragma unroll
      for (int m = 3; m > 0; --m) ed[m] = ed[m - 1];
    }
    const int d = (int32_t)w >> 28;
    w <<= 4;
    const bool bpos = (i & 3) == 0 && i < 32;  // wave-uniform
    int de = 0;
    if (bpos) de = (i & 4) ? (int32_t)we >> 16 : (int32_t)(we << 16) >> 16;
    if (i >= npos) continue;  // wave-uniform
    ge_cached c;
    tab.load(d < 0 ? -d : d, c);
    if (bpos) wide.prefetch(par ? 0 : de, par ? de : 0);
    if (i != npos - 1) {
#pragma unroll 1
      for (int r = 0; r < 3; ++r) {
        group_p2_dbl<G>(t, acc2, q);
        group_to_p2<G>(acc2, t, q);
      }
      group_p2_dbl<G>(t, acc2, q);
      group_to_p3<G>(acc, t, q);
    }
    ge_cached_cneg(c, d < 0);
    group_add_cached<G>(t, acc, c, q);
    if (!bpos) {
      group_to_p2<G>(acc2, t, q);
    } else {
      group_to_p3<G>(acc, t, q);
      ge_niels n;
      wide.niels(n, par);
      group_madd<G>(t, acc, n, q);
      group_to_p2<G>(acc2, t, q);
    }
  }
  out = acc2;
}

// Phase 2 for the smallest chunks (one group wave per SIMD at most:
// quad_max / duo_max in launch_verify): signature j on lanes 2Gj..2Gj+2G-1,
// the first G lanes the [e_lo]B + [c]P1 chain and the next G the
// [e_hi]2^128 B + [d]P2 chain (verify_phase2_pair_chain's split); the
// chains' sums are exchanged (lane ^ G) and tested to cancel.  A wave decides
// 64 / 2G signatures: a bitmap byte (G = 4) or half-word (G = 2).  Same
// phase-1 input as the pair kernel.
template <int G>
__global__ __launch_bounds__(kBlock, STL_VERIFY_WAVES_PER_SIMD) void verify_main_group_kernel(
    const uint4* __restrict__ pre, uint32_t base, uint32_t cnt, uint32_t policy, uint64_t* __restrict__ bitmap,
    uint64_t* __restrict__ fb_words, uint4* __restrict__ ws, const uint4* __restrict__ wide,
    unsigned long long* __restrict__ ctr) {
  static_assert(G == 2 || G == 4, "group size");
  constexpr uint32_t kLanes = 2 * G;          // lanes per signature
  constexpr uint32_t kSigsPerWave = 64 / kLanes;
  // one table per group: heads in the per-lane slots (slot = global lane / G),
  // tails in LDS
  __shared__ uint4 tails[9][kBlock / G];
  const size_t gl = (size_t)blockIdx.x * kBlock + threadIdx.x;
  TableView tab = TableView::split(ws + (gl / G) * kHeadQuads, &tails[0][threadIdx.x / G], kIdentityHead,
                                   kBlock / G);
  const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63u;
  const GroupRole q{(lane & 1u) != 0, (lane & 2u) != 0};
  const bool role0 = (lane & (G - 1)) == 0;
  const int par = (int)((lane / G) & 1u);
  const WideGlobal wl{wide, {0, 0}};
  const uint32_t words = (cnt + 63) >> 6;
  // every bit of every bitmap word the chunk owns is written (the fallback
  // kernel ORs into whole words)
  for (uint32_t tile = blockIdx.x * kBlock; tile < kLanes * 64u * words; tile += gridDim.x * kBlock) {
    const uint32_t t = (tile + threadIdx.x) / kLanes;  // signature of this lane's group pair
    const bool live = t < cnt;
    HalfState h;
    ld_state_words<14>(h, pre + (size_t)(live ? t : cnt - 1) * 14);
    {
      const fe nAx = h.P1x, nAy = h.P1y, nQx = h.P2x, nQy = h.P2y;
      finish_phase1_points(h, nAx, nAy, nQx, nQy, (h.pad & kPairPointOk) != 0);
      if ((policy & kModeFullLength) && (h.tops & kHalfOk)) h.tops |= kHalfFallback;
    }
    const uint64_t fball = __ballot(live && (h.tops & kHalfFallback) != 0);
    ge_p2 mine, other;
    group_chain<G>(mine, h, par, tab, wl, q, role0);
#pragma unroll
    for (int i = 0; i < 9; ++i) {
      other.X.v[i] = (uint32_t)__shfl_xor((int)mine.X.v[i], G);
      other.Y.v[i] = (uint32_t)__shfl_xor((int)mine.Y.v[i], G);
      other.Z.v[i] = (uint32_t)__shfl_xor((int)mine.Z.v[i], G);
    }
    const bool ok = live && half_state_accepts(h) && pair_sums_cancel(mine, other);
    const uint64_t ball = __ballot(ok);
    uint32_t bits = 0, fbits = 0;  // the first lane of each signature's lanes
#pragma unroll
    for (uint32_t b = 0; b < kSigsPerWave; ++b) {
      bits |= (uint32_t)((ball >> (kLanes * b)) & 1u) << b;
      fbits |= (uint32_t)((fball >> (kLanes * b)) & 1u) << b;
    }
    const uint32_t wsig = (tile + wave * 64) / kLanes;  // first signature of this wave
    if (lane == 0 && (wsig >> 6) < words) {
      if (G == 4) {
        reinterpret_cast<uint8_t*>(fb_words)[wsig >> 3] = (uint8_t)fbits;
        reinterpret_cast<uint8_t*>(bitmap)[(base + wsig) >> 3] = (uint8_t)bits;
      } else {
        reinterpret_cast<uint16_t*>(fb_words)[wsig >> 4] = (uint16_t)fbits;
        reinterpret_cast<uint16_t*>(bitmap)[(base + wsig) >> 4] = (uint16_t)bits;
      }
      if (ctr) atomicAdd(&ctr[0], (unsigned long long)__popc(bits));  // accepted (stl_get_stats)
    }
    __syncthreads();  // the next tile's table stores after every group's last loads
  }
}

// Full-length path for the lanes phase 1 flagged (rare: the lattice
// reduction did not fit 2^131).  Waves with no flagged lane skip their tile;
// flagged lanes OR their exact bit into the word phase 2 wrote.
template <bool PRE_K>
__global__ __launch_bounds__(kBlock, 2) void verify_fallback_kernel(
    const uint8_t* __restrict__ sig, const uint8_t* __restrict__ msg_or_k, const uint8_t* __restrict__ pk,
    uint32_t base, uint32_t cnt, uint32_t policy, const uint64_t* __restrict__ fb_words,
    uint64_t* __restrict__ bitmap, uint4* __restrict__ ws, unsigned long long* __restrict__ ctr) {
  // A workgroup none of whose tiles has a flagged lane (almost all of them)
  // ends before staging the base table.
  int any = 0;
  for (uint32_t tile = blockIdx.x * kBlock; tile < cnt; tile += gridDim.x * kBlock) {
    const uint32_t wbase = tile + (threadIdx.x >> 6) * 64;
    if ((threadIdx.x & 63u) == 0 && wbase < cnt && fb_words[wbase >> 6] != 0) any = 1;
  }
  if (!__syncthreads_or(any)) return;  // workgroup-uniform
  __shared__ uint32_t sB[kBaseTableWords];
  stage_base_table(sB, 1);
  TableView tab, unused;
  lane_tables(ws, tab, unused);
  const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63u;
  for (uint32_t tile = blockIdx.x * kBlock; tile < cnt; tile += gridDim.x * kBlock) {
    const uint32_t wbase = tile + wave * 64;
    if (wbase >= cnt) continue;
    const uint64_t fb = fb_words[wbase >> 6];
    if (fb == 0) continue;  // wave-uniform
    bool ok = false;
    if ((fb >> lane) & 1u) {
      const size_t j = (size_t)base + wbase + lane;
      uint32_t R[8], S[8], A[8], k[8];
      ld8(R, sig + 64 * j);
      ld8(S, sig + 64 * j + 32);
      ld8(A, pk + 32 * j);
      load_k(k, R, A, msg_or_k, j, PRE_K);
      ok = verify_full_with_k(R, S, A, k, core_policy(policy), tab, sB);
    }
    const uint64_t word = __ballot(ok);
    if (lane == 0) {
      bitmap[(base + wbase) >> 6] |= word;
      if (ctr) {  // full-length lanes and their accepts (stl_get_stats)
        atomicAdd(&ctr[1], (unsigned long long)__popcll(fb));
        atomicAdd(&ctr[0], (unsigned long long)__popcll(word));
      }
    }
  }
}

// k_i = SHA-512(R_i || A_i || m_i) mod L for arbitrary-length messages.
__global__ void hram_var_kernel(const uint8_t* __restrict__ sig, const uint8_t* __restrict__ pk,
                                const uint8_t* __restrict__ m, const uint64_t* __restrict__ moff,
                                const uint64_t* __restrict__ mlen, uint32_t n, uint8_t* __restrict__ k_out) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint8_t prefix[64];
  for (int b = 0; b < 32; ++b) {
    prefix[b] = sig[64 * (size_t)i + b];
    prefix[32 + b] = pk[32 * (size_t)i + b];
  }
  uint64_t st[8];
  sha512_prefixed(st, prefix, 64, m + moff[i], mlen[i]);
  uint32_t h[16], k[8];
  sha512_digest_le32(h, st);
  sc_reduce64(k, h);
  st8(k_out + 32 * (size_t)i, k);
}

// ---- wave-cooperative message windows for the hash kernels ----
// Each lane hashes its own message, so a lane-private dword load touches 64
// different cache lines per instruction and the blocks are re-read from L2
// once per dword.  Instead, every iteration the wave fills, for each lane, a
// 144-byte window at a 16-byte aligned address of that lane's choosing:
// consecutive lanes load consecutive 16-byte chunks of one lane's window (so
// one load instruction covers ~9 lines), through LDS, and each lane then reads
// its 128-byte block from its own window.  Chunks wholly past the message end
// are not loaded; the 16-byte granules holding the first and last message
// bytes are read whole.
constexpr uint32_t kWinChunks = 9;  // 144 bytes: a 128-byte block at any alignment
constexpr uint32_t kWinBytes = 16 * kWinChunks;

__device__ __forceinline__ uint64_t shfl_u64(uint64_t v, uint32_t src) {
  const uint32_t lo = (uint32_t)__shfl((int)(uint32_t)v, (int)src);
  const uint32_t hi = (uint32_t)__shfl((int)(uint32_t)(v >> 32), (int)src);
  return ((uint64_t)hi << 32) | lo;
}

// win: this wave's 64 * kWinChunks uint4; base == 0 marks an idle lane.
// Only granules that hold bytes of [lo, end) are loaded.
__device__ __forceinline__ void wave_window_fill(uint4* win, uintptr_t base, uintptr_t lo, uintptr_t end,
                                                 uint32_t lane) {
#pragma unroll
  for (uint32_t k = 0; k < kWinChunks; ++k) {
    const uint32_t g = k * 64u + lane;
    const uint32_t src = g / kWinChunks;
    const uint32_t c = g - src * kWinChunks;
    const uintptr_t b = (uintptr_t)shfl_u64(base, src), e = (uintptr_t)shfl_u64(end, src);
    const uintptr_t l = (uintptr_t)shfl_u64(lo, src);
    const uintptr_t a = b + 16u * c;
    uint4 v = make_uint4(0u, 0u, 0u, 0u);
    if (b != 0 && a < e && a + 16u > l) v = *reinterpret_cast<const uint4*>(a);
    win[g] = v;  // = window of lane src, chunk c
  }
  __builtin_amdgcn_wave_barrier();
  asm volatile("" ::: "memory");
}

// Dword source over a lane's window, global loads outside it.
struct WinSrc {
  const uint32_t* w;  // this lane's kWinBytes / 4 words in LDS
  uintptr_t base;
  const uint32_t* q;  // ByteStream: aligned start of the message
  __device__ uint32_t at(uintptr_t a) const {
    const uintptr_t off = a - base;
    return off < kWinBytes ? w[off >> 2] : *reinterpret_cast<const uint32_t*>(a);
  }
  __device__ uint32_t operator()(uint32_t idx) const { return at((uintptr_t)(q + idx)); }
  __device__ uint32_t operator()(const uint8_t* a) const { return at((uintptr_t)a); }
};

// ---- longest-first order for the hash work queues ----
// A 1M-transaction batch is only ~4 messages per resident lane, so a lane that
// draws a 4 KB message (33 blocks) near the end of the queue sets the tail.
// A counting sort by SHA-512 block count (64 buckets, longest first) makes the
// queue hand out long messages first; the last draws are all short.
constexpr uint32_t kOrderBuckets = 64;

__device__ __forceinline__ uint32_t order_bucket(uint32_t bytes) {
  const uint32_t nb = (bytes + 17u + 127u) >> 7;
  return (kOrderBuckets - 1u) - (nb < kOrderBuckets - 1u ? nb : kOrderBuckets - 1u);
}

__global__ __launch_bounds__(kBlock) void order_count_kernel(const uint32_t* __restrict__ len, uint32_t n,
                                                             uint32_t extra, uint32_t* __restrict__ hist) {
  __shared__ uint32_t h[kOrderBuckets];
  if (threadIdx.x < kOrderBuckets) h[threadIdx.x] = 0;
  __syncthreads();
  for (uint32_t i = blockIdx.x * kBlock + threadIdx.x; i < n; i += gridDim.x * kBlock)
    atomicAdd(&h[order_bucket(len[i] + extra)], 1u);
  __syncthreads();
  if (threadIdx.x < kOrderBuckets && h[threadIdx.x]) atomicAdd(&hist[threadIdx.x], h[threadIdx.x]);
}

// Rows hashed one per wave (tx_hash_kernel's long mode): at most this many,
// the longest of the batch, and only rows of more than long_min blocks --
// one long wave per SIMD of a 256-CU chip: two per SIMD run each block
// ≈1.45x slower (8,000-row ledgers' hash 0.44 ms at 2,048 rows, profiles/r05/g).
constexpr uint32_t kLongMaxRows = 1024;
constexpr uint32_t kLongBatch = (64u * kWinBytes) / (80u * 8u);  // block schedules in a wave's window area

// exclusive scan of the 64 bucket counts into bucket cursors (one wave); with
// long_min > 0 also the number K of rows at the front of the order that the
// hash kernel takes wave-wise -- min(kLongMaxRows, rows of more than
// long_min blocks) -- in header[2], and header[0], the per-lane queue's
// counter, starts after them
__global__ __launch_bounds__(64) void order_scan_kernel(const uint32_t* __restrict__ hist, uint32_t* __restrict__ cursor,
                                                        uint32_t* __restrict__ header, uint32_t long_min) {
  const uint32_t t = threadIdx.x;
  uint32_t v = hist[t];
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t u = (uint32_t)__shfl_up((int)v, d);
    if (t >= (uint32_t)d) v += u;
  }
  cursor[t] = v - hist[t];
  // bucket t holds rows of 63 - t blocks (bucket 0: 63 or more), longest first
  if (long_min > 0 && long_min < kOrderBuckets - 1u && t == kOrderBuckets - 2u - long_min) {
    const uint32_t k = v < kLongMaxRows ? v : kLongMaxRows;
    header[0] = k;
    header[2] = k;
  }
}

__global__ __launch_bounds__(kBlock) void order_scatter_kernel(const uint32_t* __restrict__ len, uint32_t n,
                                                               uint32_t extra, uint32_t* __restrict__ cursor,
                                                               uint32_t* __restrict__ order) {
  __shared__ uint32_t h[kOrderBuckets], base[kOrderBuckets];
  for (uint32_t tile = blockIdx.x * kBlock; tile < n; tile += gridDim.x * kBlock) {
    if (threadIdx.x < kOrderBuckets) h[threadIdx.x] = 0;
    __syncthreads();
    const uint32_t i = tile + threadIdx.x;
    uint32_t b = 0, pos = 0;
    if (i < n) {
      b = order_bucket(len[i] + extra);
      pos = atomicAdd(&h[b], 1u);
    }
    __syncthreads();
    if (threadIdx.x < kOrderBuckets && h[threadIdx.x]) base[threadIdx.x] = atomicAdd(&cursor[threadIdx.x], h[threadIdx.x]);
    __syncthreads();
    if (i < n) order[base[b] + pos] = i;
    __syncthreads();
  }
}

// The long row's 80 rounds on lane pairs (stl_sha512.h pair_round_front /
// _back) and the feed-forward: this lane's four state words s4, the
// partner's word by one DPP swap, W[t] + K[t] = get(t) read kAhead rounds
// ahead of its use (a ring in registers, each read pinned behind round
// t - kAhead's state, so the compiler neither hoists all 80 reads nor leaves
// a read's latency inside the chain).  Round 6: 36 instructions per round
// against 41 for the whole round on every lane (the previous form), a
// 4-KB row's hash 12 % faster (DESIGN_EXPERIMENTS.md).
template <typename Get>
__device__ __forceinline__ void sha512_rounds_pair(W64 s4[4], const PairSide& ps, const Get& get) {
  constexpr int kAhead = 8;
  W64 r[4] = {s4[0], s4[1], s4[2], s4[3]};
  W64 ring[kAhead];
#pragma unroll
  for (int i = 0; i < kAhead; ++i) ring[i] = get(i);
#pragma clang loop unroll(full)
  for (int i = 0; i < 80; ++i) {
    const W64 kw = ring[i % kAhead];
    if (i + kAhead < 80) {
      asm volatile("" : "+v"(r[0].lo)::"memory");
      ring[i % kAhead] = get(i + kAhead);
    }
    W64 T, U;
    pair_round_front<true>(r, kw, ps, T, U);
    pair_round_back<true>(r, T, W64{pair_swap(U.lo), pair_swap(U.hi)});
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) s4[j] = add64(s4[j], r[j]);
}

// tx_hash_kernel's long mode (small batches: the longest row sets the
// call's latency): the first K = counter[2] rows of the order, one per wave.
// Lanes 0..kLongBatch-1 each load one block of the row (a 144-byte window of
// 16-byte loads, as wave_window_fill takes them) and expand its schedule into
// the wave's window area; the wave then runs the rounds block after block
// on lane pairs (sha512_rounds_pair) reading W[t] from LDS (a broadcast
// read), so the schedule leaves the dependent chain.
__device__ __forceinline__ void hash_long_rows(const uint8_t* __restrict__ pre, const uint64_t* __restrict__ off,
                                               const uint32_t* __restrict__ len, uint8_t* __restrict__ msg,
                                               uint32_t* __restrict__ counter, const uint32_t* __restrict__ order,
                                               uint4* win, uint32_t lane) {
  uint2* wsch = reinterpret_cast<uint2*>(win);
  // rows r = wave, wave + waves, ... < K: a static deal (the rows are the
  // longest of the batch, about equal), every index a scalar, so the row loop
  // is uniform control flow (s_cmp / s_cbranch_scc on K, r in the ISA).  A
  // dynamic deal -- lane 0 claiming the row with an atomic, __shfl broadcasting
  // it -- hung in round 5: the index was a VGPR, and in the ISA of a rebuilt
  // form of it the claim sits in an outer loop's header while the broadcast,
  // the exit test and the body form a nested exec-masked loop that iterates
  // without re-claiming ("Work queues").
  const uint32_t K = __builtin_amdgcn_readfirstlane(counter[2]);
  const uint32_t waves = gridDim.x * (kBlock / 64u);
  const uint32_t first = __builtin_amdgcn_readfirstlane(blockIdx.x * (kBlock / 64u) + (threadIdx.x >> 6));
  for (uint32_t r = first; r < K; r += waves) {
    const uint32_t row = order[r];
    const uint8_t* p = pre + off[row];
    const uint32_t L = len[row];
    const uint32_t mis = (uint32_t)((uintptr_t)p & 3u);
    const uintptr_t q = (uintptr_t)p - mis;  // aligned dword 0 of the message
    const uintptr_t lo = (uintptr_t)p, end = lo + L;
    const uint32_t nbl = (L + 17u + 127u) >> 7;
    uint64_t st[8];
    sha512_init(st);
    // lane pairs: the odd lanes keep H0..H3 (a..d), the even lanes H4..H7
    const PairSide ps = pair_side((lane & 1u) != 0);
    W64 s4[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) s4[j] = w64(st[(ps.a_side ? 0 : 4) + j]);
    for (uint32_t b0 = 0; b0 < nbl; b0 += kLongBatch) {
      const uint32_t cnt = nbl - b0 < kLongBatch ? nbl - b0 : kLongBatch;
      if (lane < cnt) {
        const uint32_t blk = b0 + lane;
        const uintptr_t blk_addr = q + 128u * blk;
        const uintptr_t wbase = blk_addr & ~(uintptr_t)15;
        uint32_t wr[4 * kWinChunks];
#pragma unroll
        for (uint32_t c = 0; c < kWinChunks; ++c) {
          const uintptr_t a = wbase + 16u * c;
          uint4 v = make_uint4(0u, 0u, 0u, 0u);
          if (a < end && a + 16u > lo) v = *reinterpret_cast<const uint4*>(a);
          wr[4 * c] = v.x; wr[4 * c + 1] = v.y; wr[4 * c + 2] = v.z; wr[4 * c + 3] = v.w;
        }
        uint64_t w[16];
        block_from_window(w, wr, (uint32_t)(blk_addr & 15u) >> 2, mis, (int32_t)L - (int32_t)(128u * blk),
                          blk + 1 == nbl, L, false, false, 0u);
        uint2* dst = wsch + 80u * lane;
        // W[t] + K[t]: the round constant added here, in parallel over the
        // lanes, instead of on the wave's chain of rounds
        sha512_schedule(w, [&](int t, W64 v) {
          const W64 kw = add64(v, w64(sha_k(t)));
          dst[t] = make_uint2(kw.lo, kw.hi);
        });
      }
      __builtin_amdgcn_wave_barrier();
      asm volatile("" ::: "memory");
      for (uint32_t j = 0; j < cnt; ++j) {
        const uint2* src = wsch + 80u * j;
        auto get = [&](int t) {
          const uint2 v = src[t];
          return W64{v.x, v.y};
        };
        sha512_rounds_pair(s4, ps, get);
      }
      __builtin_amdgcn_wave_barrier();
      asm volatile("" ::: "memory");
    }
    if (lane == 1u) {  // an a-side lane: H0..H3, the signing hash
      uint32_t h[8];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        h[2 * j] = bswap32(s4[j].hi);
        h[2 * j + 1] = bswap32(s4[j].lo);
      }
      st8(msg + 32 * (size_t)row, h);
    }
  }
}

// msg_i = SHA512Half(preimage_i) (Serializer.cpp:354-360 via
// STObject::getSigningHash, SerializedObject.cpp:444-450).  Lanes pull
// preimages from a global counter and advance one 128-byte block per
// iteration, refilling as they finish: waves stay full whatever the length
// mix (config 5: 100 B - 4 KB, log-uniform), with no sort pass.
__global__ __launch_bounds__(kBlock, STL_HASH_WAVES_PER_SIMD) void tx_hash_kernel(const uint8_t* __restrict__ pre,
                                                         const uint64_t* __restrict__ off,
                                                         const uint32_t* __restrict__ len, uint32_t n,
                                                         uint8_t* __restrict__ msg, uint32_t* __restrict__ counter,
                                                         const uint32_t* __restrict__ order) {
  __shared__ uint4 win_all[kBlock / 64][64 * kWinChunks];
  const uint32_t lane = threadIdx.x & 63u;
  uint4* win = win_all[threadIdx.x >> 6];
  // Long mode (small batches): the first K rows of the order, one per wave
  if (counter[2] != 0) hash_long_rows(pre, off, len, msg, counter, order, win, lane);
  ByteStream bs;
  bs.init(pre, 0);
  uint64_t st[8];
  sha512_init(st);
  uint32_t mi = 0, blk = 0, nb = 0;
  bool active = false, exhausted = false;
  for (;;) {
    // Work queue, per lane: the leader claims one row for every idle lane and
    // __shfl hands the base to all of them (a VGPR, by design: each lane then
    // takes its own row, so the rows ARE divergent).  The loop's exit is the
    // ballot `__any(active)` below -- a scalar of the whole wave -- so no lane
    // can stay in the loop on a stale claim, and a lane that found the queue
    // empty simply idles until the wave leaves.
    const uint64_t need = __ballot(!active);
    if (need != 0 && !exhausted) {  // wave-uniform
      const int leader = __ffsll((unsigned long long)need) - 1;
      uint32_t base = 0;
      if ((int)lane == leader) base = atomicAdd(counter, (uint32_t)__popcll(need));
      base = __shfl(base, leader);
      exhausted = base + (uint32_t)__popcll(need) >= n;
      if (!active) {
        mi = base + (uint32_t)__popcll(need & ((1ull << lane) - 1ull));
        if (mi < n) {
          mi = order[mi];
          bs.init(pre + off[mi], len[mi]);
          nb = bs.blocks();
          blk = 0;
          sha512_init(st);
          active = true;
        }
      }
    }
    if (!__any(active)) break;
    const uintptr_t blk_addr = (uintptr_t)(bs.q + 32 * blk);
    const uintptr_t wbase = active ? (blk_addr & ~(uintptr_t)15) : 0;
    wave_window_fill(win, wbase, (uintptr_t)bs.p, (uintptr_t)(bs.p + bs.len), lane);
    if (active) {
      uint64_t w[16];
      block_from_window(w, reinterpret_cast<const uint32_t*>(win) + lane * (kWinBytes / 4),
                        (uint32_t)(blk_addr & 15u) >> 2, bs.mis, (int32_t)bs.len - (int32_t)(128 * blk),
                        blk + 1 == nb, bs.len, false, false, 0u);
      sha512_compress(st, w);
      if (++blk == nb) {
        uint32_t h[8];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          h[2 * j] = bswap32((uint32_t)(st[j] >> 32));
          h[2 * j + 1] = bswap32((uint32_t)st[j]);
        }
        st8(msg + 32 * (size_t)mi, h);
        active = false;
      }
    }
  }
}

// The canonical-form pass of every blob (stl_txblob.h tx_blob_parse), one
// lane per row, ahead of the hashing (the blob ledger ran 10 %
// behind preimages).  A lane-per-row walk over global memory makes every load
// instruction touch 64 cache lines, one per row, so the wave first stages the
// first kParseStage bytes of its 64 rows in LDS with 16-byte loads dealt
// across the lanes (12 instructions, about a dozen lines each); the walk, the
// signature and key and the spliced block then read LDS (a Payment's fields
// up to its memos lie inside; the rest are global loads).  Writes each row's
// status and layout {status, xs, xe, 0} -- an STL_TX_OK row has exactly one
// cut, its signature field (every other non-signing field is outside both
// templates), so a row with more is deferred (never taken) -- the verify
// inputs (signature and key; the always-reject signature, a zero key and
// message for a deferred or malformed row; a zero id for a deferred one) and,
// for an STL_TX_OK row, the SHA-512 block of its signing preimage that holds
// the cut (splice1_words): the hash kernel reads every block as a plain
// window.
#ifndef STL_PARSE_STAGE
#define STL_PARSE_STAGE 192
#endif
constexpr uint32_t kParseStage = STL_PARSE_STAGE;
constexpr uint32_t kParseChunks = kParseStage / 16u;
constexpr uint32_t kParseStride = kParseStage / 4u + 1u;  // dwords per row, odd: no bank conflicts
static_assert(kParseChunks * 16u == kParseStage && kParseChunks <= 64u, "stage: whole 16-byte chunks");

struct StagedBytes {  // b[i] of a blob whose first bytes are staged in LDS
  const uint8_t* g;
  const uint8_t* s;  // LDS copy of the aligned 16-byte granules from g - off
  uint32_t off;
  __device__ uint8_t operator[](uint32_t i) const {
    const uint32_t j = i + off;
    return j < kParseStage ? s[j] : g[i];
  }
};

struct StagedDwords {  // aligned blob dwords: LDS inside the stage, global outside
  const uint32_t* s;
  uintptr_t base;
  __device__ uint32_t operator()(const uint8_t* q) const {
    const uintptr_t o = (uintptr_t)q - base;
    return o < kParseStage ? s[o >> 2] : *reinterpret_cast<const uint32_t*>(q);
  }
};

// n little-endian words from blob bytes [pos, pos + 4n): LDS when inside the
// stage (sh = the blob's offset in its first granule), else blob_words
__device__ __forceinline__ void staged_words(uint32_t* out, const uint32_t* s, uint32_t sh, const uint8_t* b,
                                             uint32_t pos, uint32_t n, uint32_t len) {
  const uint32_t j = sh + pos;
  if (j + 4u * n + 4u <= kParseStage) {
    const uint32_t q = j >> 2, r = j & 3u;
    for (uint32_t i = 0; i < n; ++i) out[i] = align_byte(s[q + i + 1], s[q + i], r);
  } else {
    blob_words(out, b, pos, n, len);
  }
}

__global__ __launch_bounds__(kBlock, 3) void tx_blob_parse_kernel(const uint8_t* __restrict__ blobs,
                                                               const uint64_t* __restrict__ off,
                                                               const uint32_t* __restrict__ len, uint32_t n,
                                                               uint8_t* __restrict__ msg, uint8_t* __restrict__ sig,
                                                               uint8_t* __restrict__ pk, uint8_t* __restrict__ txid,
                                                               uint8_t* __restrict__ status, uint4* __restrict__ layout,
                                                               uint4* __restrict__ side, BlobKind kind) {
  __shared__ uint32_t stage_all[kBlock * kParseStride];
  const uint32_t lane = threadIdx.x & 63u;
  uint32_t* wstage = stage_all + (threadIdx.x & ~63u) * kParseStride;  // the wave's 64 rows
  uint32_t* stage = stage_all + threadIdx.x * kParseStride;           // this lane's row
  const uint32_t sign_le = bswap32(kind.sign_prefix);
  // tiles of kBlock rows: every lane of a wave takes part in every staging
  for (uint32_t tile = blockIdx.x * kBlock; tile < n; tile += gridDim.x * kBlock) {
    const uint32_t mi = tile + threadIdx.x;
    const bool valid = mi < n;
    const uint8_t* b = blobs;
    uint32_t L = 0;
    if (valid) {
      b = blobs + off[mi];
      L = len[mi];
    }
    const uintptr_t lo = (uintptr_t)b, end = lo + L, base = lo & ~(uintptr_t)15;
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");
#pragma unroll
    for (uint32_t k = 0; k < kParseChunks; ++k) {
      const uint32_t g = k * 64u + lane, r = g / kParseChunks, c = g - r * kParseChunks;
      const uintptr_t rb = (uintptr_t)shfl_u64(base, r), re = (uintptr_t)shfl_u64(end, r);
      const uintptr_t a = rb + 16u * c;
      uint4 v = make_uint4(0u, 0u, 0u, 0u);
      if (a < re) v = *reinterpret_cast<const uint4*>(a);
      uint32_t* d = wstage + r * kParseStride + 4u * c;
      d[0] = v.x;
      d[1] = v.y;
      d[2] = v.z;
      d[3] = v.w;
    }
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");
    if (!valid) continue;
    const uint32_t sh = (uint32_t)(lo - base);
    const StagedBytes sb{b, reinterpret_cast<const uint8_t*>(stage), sh};
    TxLayout t;
    tx_blob_parse(sb, L, t, kind.sig_code, kind.min_len, kind.format);
    if (t.status == kTxOk && t.xs1 != L) t.status = kTxDeferred;
    status[mi] = (uint8_t)t.status;
    layout[2 * (size_t)mi] = make_uint4(t.status, t.xs0, t.xe0, 0u);
    uint4* sq = reinterpret_cast<uint4*>(sig + 64 * (size_t)mi);
    if (t.status == kTxOk) {
      uint32_t sgw[16], pkw[8];
      staged_words(sgw, stage, sh, b, t.sig_off, 16, L);
      staged_words(pkw, stage, sh, b, t.pk_off, 8, L);
      sq[0] = make_uint4(sgw[0], sgw[1], sgw[2], sgw[3]);
      sq[1] = make_uint4(sgw[4], sgw[5], sgw[6], sgw[7]);
      sq[2] = make_uint4(sgw[8], sgw[9], sgw[10], sgw[11]);
      sq[3] = make_uint4(sgw[12], sgw[13], sgw[14], sgw[15]);
      st8(pk + 32 * (size_t)mi, pkw);
      // the preimage block holding the cut (preimage byte 4 + xs0)
      uint32_t m[32];
      splice1_words(m, b, L, t.xs0, t.xe0, sign_le, (4u + t.xs0) >> 7, StagedDwords{stage, base});
      uint4* dq = side + 8 * (size_t)mi;
#pragma unroll
      for (int j = 0; j < 8; ++j) dq[j] = make_uint4(m[4 * j], m[4 * j + 1], m[4 * j + 2], m[4 * j + 3]);
    } else {
      const uint4 z = make_uint4(0u, 0u, 0u, 0u), f = make_uint4(~0u, ~0u, ~0u, ~0u);
      sq[0] = z; sq[1] = z; sq[2] = f; sq[3] = f;
      uint4* pq = reinterpret_cast<uint4*>(pk + 32 * (size_t)mi);
      pq[0] = z; pq[1] = z;
      uint4* mq = reinterpret_cast<uint4*>(msg + 32 * (size_t)mi);
      mq[0] = z; mq[1] = z;
      if (t.status == kTxDeferred && txid != nullptr) {
        uint4* tq = reinterpret_cast<uint4*>(txid + 32 * (size_t)mi);
        tq[0] = z; tq[1] = z;
      }
    }
  }
}

// Serialized transactions -> verify inputs.  Same work queue as
// tx_hash_kernel; a lane runs the canonical-form pass when it takes a blob,
// then one SHA-512 block per iteration: first the signing hash
// ("STX\0" || blob minus the cut fields), then, if requested, the transaction
// ID ("TXN\0" || blob).  A lane whose blob is deferred or malformed writes a
// signature the verify kernels always reject (S = 2^256 - 1) and a zero key.
__global__ __launch_bounds__(kBlock, STL_HASH_WAVES_PER_SIMD) void tx_blob_kernel(const uint8_t* __restrict__ blobs,
                                                         const uint64_t* __restrict__ off,
                                                         const uint32_t* __restrict__ len, uint32_t n,
                                                         uint8_t* __restrict__ msg, uint8_t* __restrict__ sig,
                                                         uint8_t* __restrict__ pk, uint8_t* __restrict__ txid,
                                                         uint8_t* __restrict__ status, uint32_t* __restrict__ counter,
                                                         const uint32_t* __restrict__ order,
                                                         const uint4* __restrict__ layout,
                                                         const uint4* __restrict__ side, BlobKind kind) {
  __shared__ uint4 win_all[kBlock / 64][64 * kWinChunks];
  const uint32_t lane = threadIdx.x & 63u;
  uint4* win = win_all[threadIdx.x >> 6];
  // phase 0: sign prefix || blob[0, cxs) || blob[cxe, len) -- an STL_TX_OK row
  // has exactly one cut, its signature field: blocks before block sb read the
  // blob 4 bytes early (word 0 -> sign prefix), block sb is the parse
  // kernel's spliced block, blocks after it read the blob past the cut;
  // phase 1: [the 4 bytes before the blob, word 0 -> id prefix] || blob
  ByteStream bs;
  bs.init(blobs, 0);
  uint32_t cxs = 0, cut = 0, sblk = 0, total = 0;
  const uint32_t sign_le = bswap32(kind.sign_prefix);
  const uint32_t txn_le = bswap32(kind.id_prefix);
  const bool id_pfx = kind.id_prefixed != 0;
  const uint32_t pfx_bytes = id_pfx ? 4u : 0u;
  uint64_t st[8];
  sha512_init(st);
  uint32_t mi = 0, blk = 0, nb = 0, phase = 0;
  const uint8_t* b = blobs;
  const uint8_t* bend = blobs;
  bool active = false, exhausted = false;
  for (;;) {
    // the per-lane work queue of tx_hash_kernel (each lane its own row, the
    // loop left on the wave-wide ballot below)
    const uint64_t need = __ballot(!active);
    if (need != 0 && !exhausted) {  // wave-uniform
      const int leader = __ffsll((unsigned long long)need) - 1;
      uint32_t base = 0;
      if ((int)lane == leader) base = atomicAdd(counter, (uint32_t)__popcll(need));
      base = __shfl(base, leader);
      exhausted = base + (uint32_t)__popcll(need) >= n;
      if (!active) {
        mi = base + (uint32_t)__popcll(need & ((1ull << lane) - 1ull));
        if (mi < n) {
          mi = order[mi];
          b = blobs + off[mi];
          const uint32_t L = len[mi];
          bend = b + L;
          // the row's layout from tx_blob_parse_kernel (status, sig, pk, the
          // reject inputs and a deferred row's zero id are written there)
          const uint4 la = layout[2 * (size_t)mi];
          const uint32_t row_status = la.x;
          if (row_status == kTxOk) {
            cxs = la.y;
            cut = la.z - la.y;
            sblk = (4u + cxs) >> 7;
            total = 4u + L - cut;
            nb = (total + 17u + 127u) >> 7;
            phase = 0;
          } else {
            bs.init(b - pfx_bytes, L + pfx_bytes);
            nb = bs.blocks();
            phase = 1;
          }
          if (row_status == kTxDeferred || (phase == 1 && txid == nullptr)) {
            // nothing to hash (the parse kernel wrote everything)
          } else {
            blk = 0;
            sha512_init(st);
            active = true;
          }
        }
      }
    }
    if (!__any(active)) break;
    const uint32_t p0 = 128u * blk;
    const bool spliced = phase == 0 && blk == sblk;
    // window source: the block's first message byte (phase 0: of the blob,
    // 4 bytes early, past the cut after block sblk; the spliced block's slot)
    uintptr_t wsrc = (uintptr_t)(bs.q + 32 * blk), wlo = (uintptr_t)b, wend = (uintptr_t)bend;
    uint32_t mis = bs.mis, tot = bs.len;
    if (phase == 0) {
      wsrc = (uintptr_t)b + p0 - 4u + (blk > sblk ? cut : 0u);
      tot = total;
      if (spliced) {
        wsrc = (uintptr_t)(side + 8 * (size_t)mi);
        wlo = wsrc;
        wend = wsrc + 128u;
      }
      mis = (uint32_t)(wsrc & 3u);
    }
    const uintptr_t wbase = active ? (wsrc & ~(uintptr_t)15) : 0;
    wave_window_fill(win, wbase, wlo, wend, lane);
    if (active) {
      const uint32_t* lw = reinterpret_cast<const uint32_t*>(win) + lane * (kWinBytes / 4);
      uint64_t w[16];
      block_from_window(w, lw, (uint32_t)(wsrc & 15u) >> 2, mis, (int32_t)tot - (int32_t)p0, blk + 1 == nb, tot,
                        blk == 0 && !spliced, phase == 1 ? id_pfx : true, phase == 1 ? txn_le : sign_le);
      sha512_compress(st, w);
      if (++blk == nb) {
        uint32_t h[8];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          h[2 * j] = bswap32((uint32_t)(st[j] >> 32));
          h[2 * j + 1] = bswap32((uint32_t)st[j]);
        }
        if (phase == 0) {
          st8(msg + 32 * (size_t)mi, h);
          if (txid != nullptr) {
            bs.init(b - pfx_bytes, len[mi] + pfx_bytes);
            nb = bs.blocks();
            blk = 0;
            sha512_init(st);
            phase = 1;
          } else {
            active = false;
          }
        } else {
          st8(txid + 32 * (size_t)mi, h);
          active = false;
        }
      }
    }
  }
}

// RFC 8032 keypair + signature per row (stl_sign.h); with `cls` (test data
// only) rows whose class is not 0 are then mutated by adversarial_row and
// msg_out gets the (possibly mutated) message.
template <bool ADV>
__global__ __launch_bounds__(kBlock, 2) void sign_kernel(const uint8_t* __restrict__ seed,
                                                      const uint8_t* __restrict__ msg, uint32_t n,
                                                      uint8_t* __restrict__ pk_out, uint8_t* __restrict__ sig_out,
                                                      uint4* __restrict__ ws, const uint8_t* __restrict__ cls,
                                                      const uint32_t* __restrict__ param,
                                                      uint8_t* __restrict__ msg_out) {
  __shared__ uint32_t sB[kBaseTableWords];
  stage_base_table(sB, 1);
  TableView tv, unused;
  lane_tables(ws, tv, unused);
  for (uint32_t base = blockIdx.x * kBlock; base < n; base += gridDim.x * kBlock) {
    const uint32_t i = base + threadIdx.x;
    const bool live = i < n;
    const size_t j = live ? i : (n - 1);
    uint32_t sd[8], M[8], A[8], R[8], S[8], a[8], r[8];
    ld8(sd, seed + 32 * j);
    ld8(M, msg + 32 * j);
    sign_row(A, R, S, a, r, sd, M, tv, sB);
    if (ADV) {
      const uint32_t c = cls[j];
      if (c != 0) adversarial_row(c, param[j], A, R, S, M, a, r, tv, sB);
    }
    if (live) {
      st8(pk_out + 32 * j, A);
      st8(sig_out + 64 * j, R);
      st8(sig_out + 64 * j + 32, S);
      if (ADV) st8(msg_out + 32 * j, M);
    }
  }
}

// ---- host-side launchers (called from stl_api.cpp) ----
const void* kernel_verify_msg32() { return reinterpret_cast<const void*>(&verify_main_kernel<false>); }

// Wide base tables: one thread per row (stl_verify_core.h wide_entry).
__global__ __launch_bounds__(kBlock) void wide_table_kernel(uint32_t* __restrict__ out) {
  const uint32_t r = blockIdx.x * kBlock + threadIdx.x;
  if (r >= 2 * kWideEntries) return;
  const int which = r >= kWideEntries ? 1 : 0;
  uint32_t row[28];
  wide_entry(row, which, r - (uint32_t)which * kWideEntries, &kBaseNiels[0][0][0]);
  const uint32_t* src = row;
  uint4* q = reinterpret_cast<uint4*>(out) + (size_t)r * kWideQuads;
#pragma unroll
  for (int c = 0; c < kWideQuads; ++c) q[c] = make_uint4(src[4 * c], src[4 * c + 1], src[4 * c + 2], src[4 * c + 3]);
}

hipError_t launch_wide_table(uint4* out, hipStream_t stream) {
  hipLaunchKernelGGL(wide_table_kernel, dim3((2 * kWideEntries + kBlock - 1) / kBlock), dim3(kBlock), 0, stream,
                     reinterpret_cast<uint32_t*>(out));
  return hipGetLastError();
}

// Small chunks: two lanes per signature in the point decodings and the main
// kernel (verify_prep_pair_kernel, verify_main_pair_kernel); the bits are the
// same.  It also takes precedence over key dedup: a chunk this small is
// latency-bound, and measured 0.46-0.52 ms on pairs against 0.68-0.75 ms
// deduplicated (1,000 signers).
static bool pair_chunk(uint32_t cnt, uint32_t policy, const VerifyExec& x) {
  return (policy & kModeOneLane) == 0 && cnt <= x.pair_max && 2ull * cnt <= (uint64_t)x.grid * kBlock;
}

// The point decodings' pairs split the two square roots without duplicating
// work, so they pay up to twice that size (two pair waves per SIMD; no
// workspace), ahead of the one-lane main kernel (verify_finish_pair_kernel in
// between).
static bool pair_point_chunk(uint32_t cnt, uint32_t policy, const VerifyExec& x) {
  const bool dedup = (policy & kModeDedupKeys) != 0;
  return pair_chunk(cnt, policy, x) ||
         (!x.concurrent && (policy & kModeOneLane) == 0 && !dedup && cnt <= 2ull * x.pair_max);
}

bool verify_pair_points(uint32_t n, uint32_t policy, const VerifyExec& x) {
  return n > 0 && n <= kPreChunk && pair_point_chunk(n, policy, x);
}

// The point role of verify_prep_pair_kernel alone (nbs = 0: every block is a
// point block) for rows [0, n), into the phase-1 state of x.ws[0] -- where
// launch_verify's single chunk reads it.
hipError_t launch_verify_points(const uint8_t* sig, const uint8_t* pk, uint32_t n, uint32_t policy,
                                const VerifyExec& x, hipStream_t stream) {
  if (!verify_pair_points(n, policy, x)) return hipErrorInvalidValue;
  uint4* pre = x.ws[0] + (size_t)x.grid * (kWsBytesPerBlock / 16);
  const dim3 gp((2 * n + kBlock - 1) / kBlock);
  hipLaunchKernelGGL(verify_prep_pair_kernel<false>, gp, dim3(kBlock), 0, stream, sig, nullptr, pk, 0u, n, policy,
                     pre, 0u);
  return hipGetLastError();
}

// The key-dedup area of a verify workspace (after verify_ws_bytes(grid)):
// hash slots, per-row representative, per-owner id and owner row, the
// distinct-key counter, the decoded keys and the shared / wide key tables.
struct KeyDomain {
  uint32_t *kslots, *rep, *uid_of, *owners, *counter;
  uint4 *keytab, *keytabs, *widetabs;
};
static KeyDomain key_domain(uint4* ws, uint32_t grid) {
  KeyDomain k;
  uint32_t* dd = reinterpret_cast<uint32_t*>(reinterpret_cast<uint8_t*>(ws) + verify_ws_bytes(grid));
  k.kslots = dd;
  k.rep = k.kslots + kDedupSlots;
  k.uid_of = k.rep + kPreChunk;
  k.owners = k.uid_of + kPreChunk;
  k.counter = k.owners + kPreChunk;
  k.keytab = reinterpret_cast<uint4*>(k.counter + 64);
  k.keytabs = k.keytab + (size_t)kPreChunk * 5;
  k.widetabs = k.keytabs + (size_t)kKeyTables * kTableQuadsPerKey;
  return k;
}

// The dedup chain over rows [base, base+cnt) (cnt <= kPreChunk): hash slots,
// owners, decoded keys, shared or wide key tables -- rep[i] for row base+i.
// wcnt: the row count the wide-table choice sees (wide_keys): cnt, or 0 to
// build the 9-entry tables only (VerifyExec::wide_min).
static hipError_t launch_key_domain(const uint8_t* pk, uint32_t base, uint32_t cnt, uint32_t wcnt,
                                    const KeyDomain& kd, hipStream_t stream) {
  const dim3 g1((cnt + kBlock - 1) / kBlock);
  uint32_t nslots = 64;
  while (nslots < 2 * cnt) nslots <<= 1;  // <= kDedupSlots
  hipError_t e = hipMemsetAsync(kd.kslots, 0xff, (size_t)nslots * 4, stream);
  if (e != hipSuccess) return e;
  e = hipMemsetAsync(kd.counter, 0, 4, stream);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(key_insert_kernel, g1, dim3(kBlock), 0, stream, pk, base, cnt, kd.kslots, nslots - 1, kd.rep,
                     kd.uid_of, kd.counter, kd.owners);
  hipLaunchKernelGGL(key_decode_kernel, g1, dim3(kBlock), 0, stream, pk, base, kd.counter, kd.owners, kd.keytab,
                     kd.keytabs, wcnt);
  const uint32_t wmax = wcnt / kWideKeyRepeat < kWideKeys ? wcnt / kWideKeyRepeat : kWideKeys;  // keys that can be wide
  if (wmax > 0) {
    hipLaunchKernelGGL(key_table_wide_base_kernel, dim3((wmax * (uint32_t)kWideBaseEntries + kBlock - 1) / kBlock),
                       dim3(kBlock), 0, stream, kd.counter, wcnt, kd.keytab, kd.widetabs);
    hipLaunchKernelGGL(key_table_wide_pair_kernel, dim3((wmax * (uint32_t)kWideKeyEntries + kBlock - 1) / kBlock),
                       dim3(kBlock), 0, stream, kd.counter, wcnt, kd.widetabs);
  }
  return hipGetLastError();
}

static uint32_t wide_count(uint32_t cnt, uint32_t wide_min) { return cnt >= wide_min ? cnt : 0u; }

hipError_t launch_key_domain_ws(const uint8_t* pk, uint32_t n, uint4* ws, uint32_t grid, uint32_t wide_min,
                                hipStream_t stream) {
  if (n == 0 || n > kPreChunk) return hipErrorInvalidValue;
  return launch_key_domain(pk, 0, n, wide_count(n, wide_min), key_domain(ws, grid), stream);
}

// One chunk (<= kPreChunk signatures at [base, base+cnt)) on one stream and
// workspace: phase 1, main, fallback.  `qctr` is the chunk's zeroed counter
// of the main kernel's unit queue.
static hipError_t verify_chunk(const uint8_t* sig, const uint8_t* msg_or_k, const uint8_t* pk, uint32_t base,
                               uint32_t cnt, uint64_t* bitmap, uint32_t policy, bool pre_k, const VerifyExec& x,
                               hipStream_t stream, uint4* ws, uint32_t* qctr, const PhaseClock* clock) {
  const uint32_t grid = x.grid, pair_max = x.pair_max;
  const uint4* wide = x.wide;
  unsigned long long* counters = x.counters;
  auto mark = [&](int i) {
    if (clock) clock->mark(clock->ctx, stream, i);
  };
  // ws = [per-lane slots: grid x kWsBytesPerBlock][HalfState x kPreChunk][fallback words][queue counters]
  //      [dedup (kModeDedupKeys): slots, rep, uid_of, owners, counter, decoded keys]
  uint4* slots = ws;
  uint4* pre = ws + (size_t)grid * (kWsBytesPerBlock / 16);
  uint64_t* fb = reinterpret_cast<uint64_t*>(pre + (size_t)kPreChunk * 14);
  const bool dedup = (policy & kModeDedupKeys) != 0;
  // a launch-wide key domain (KeyDomain: one key table for every chunk of
  // the launch, in x.key_ws) or this chunk's own, in its workspace
  // at the workspace's own offset: chunks of one call may differ in grid
  // (verify_grid_for), the domain they share may not
  const KeyDomain kd = key_domain(x.key_ws ? x.key_ws : ws, x.ws_grid ? x.ws_grid : grid);
  uint32_t* kslots = kd.kslots;
  uint32_t* rep = x.key_ws ? kd.rep + x.key_base + base : kd.rep;
  uint32_t* uid_of = kd.uid_of;
  uint32_t* owners = kd.owners;
  uint32_t* counter = kd.counter;
  uint4* keytab = kd.keytab;
  uint4* keytabs = kd.keytabs;
  uint4* widetabs = kd.widetabs;
  // rows of the key domain as the wide-table choice sees them
  const uint32_t kcnt = wide_count(x.key_ws ? x.key_n : cnt, x.wide_min);
  {
    const dim3 g1((cnt + kBlock - 1) / kBlock);
    const uint32_t units = (cnt + 63) / 64;
    const uint32_t wgs = (units + kBlock / 64 - 1) / (kBlock / 64);
    const dim3 g2(wgs < grid ? wgs : grid);
    const bool pair = pair_chunk(cnt, policy, x);
    const bool pair_point = pair_point_chunk(cnt, policy, x);
    const dim3 gp((2 * cnt + kBlock - 1) / kBlock);
    const bool fused = x.fused_prep != 0 && !pair_point && !dedup;
    mark(0);
    // pair_point implies !dedup or pair (pair chunks ignore STL_DEDUP_KEYS)
    if (pair_point) {
      // both halves of phase 1 in one launch, side by side (verify_prep_pair_kernel);
      // the main pair kernel finishes the state itself, the one-lane main
      // kernel gets it from verify_finish_pair_kernel.  With points_done the
      // point role already ran (launch_verify_points): scalar blocks only.
      const uint32_t nbs = (cnt + kBlock - 1) / kBlock;
      const uint32_t nblk = nbs + (x.points_done ? 0u : gp.x);
      if (pre_k)
        hipLaunchKernelGGL(verify_prep_pair_kernel<true>, dim3(nblk), dim3(kBlock), 0, stream, sig, msg_or_k, pk,
                           base, cnt, policy, pre, nbs);
      else
        hipLaunchKernelGGL(verify_prep_pair_kernel<false>, dim3(nblk), dim3(kBlock), 0, stream, sig, msg_or_k,
                           pk, base, cnt, policy, pre, nbs);
    } else if (fused && pre_k)
      hipLaunchKernelGGL(verify_prep_kernel<true>, g1, dim3(kBlock), 0, stream, sig, msg_or_k, pk, base, cnt, policy,
                         pre, fb);
    else if (fused)
      hipLaunchKernelGGL(verify_prep_kernel<false>, g1, dim3(kBlock), 0, stream, sig, msg_or_k, pk, base, cnt, policy,
                         pre, fb);
    else if (pre_k)
      hipLaunchKernelGGL(verify_scalar_kernel<true>, g1, dim3(kBlock), 0, stream, sig, msg_or_k, pk, base, cnt, pre);
    else
      hipLaunchKernelGGL(verify_scalar_kernel<false>, g1, dim3(kBlock), 0, stream, sig, msg_or_k, pk, base, cnt, pre);
    mark(1);
    if (pair_point) {
      if (!pair)
        hipLaunchKernelGGL(verify_finish_pair_kernel, g1, dim3(kBlock), 0, stream, cnt, policy, pre, fb);
    } else if (fused) {
      // phase 1 done
    } else if (dedup) {
      if (!x.key_ws) {
        hipError_t e = launch_key_domain(pk, base, cnt, kcnt, kd, stream);
        if (e != hipSuccess) return e;
      } else if (x.key_build) {
        // the launch-wide domain, built once on this (the first) stream
        // after this chunk's scalar kernel, over every row of the launch
        hipError_t e = x.key_after ? hipStreamWaitEvent(stream, x.key_after, 0) : hipSuccess;
        if (e == hipSuccess) e = launch_key_domain(pk, 0, x.key_n, kcnt, kd, stream);
        if (e == hipSuccess) e = hipEventRecord(x.key_ready, stream);
        if (e != hipSuccess) return e;
      } else {
        hipError_t e = hipStreamWaitEvent(stream, x.key_ready, 0);
        if (e != hipSuccess) return e;
      }
      if (x.key_ws && x.rdec) {  // R decoded ahead (VerifyExec::rdec)
        hipError_t e = hipStreamWaitEvent(stream, x.r_ready, 0);
        if (e != hipSuccess) return e;
        hipLaunchKernelGGL(verify_finish_keyed_kernel, g1, dim3(kBlock), 0, stream, cnt, policy, pre, fb, rep, uid_of,
                           keytab, counter, kcnt, x.rdec + (size_t)(x.key_base + base) * 5);
      } else {
        hipLaunchKernelGGL(verify_point_kernel_keyed, g1, dim3(kBlock), 0, stream, sig, pk, base, cnt, policy, pre,
                           fb, rep, uid_of, keytab, counter, kcnt);
      }
    } else {
      hipLaunchKernelGGL(verify_point_kernel, g1, dim3(kBlock), 0, stream, sig, pk, base, cnt, policy, pre, fb);
    }
    mark(2);
    // lane groups: G lanes per chain, 2G per signature, one table per group:
    // G * words / 2 workgroups, whose slots (one per G lanes) fit the
    // workspace when words <= 2 * grid
    const uint32_t words = (cnt + 63) / 64;
    const bool fits = pair && words <= 2 * grid;
    if (fits && cnt <= x.quad_max)
      hipLaunchKernelGGL(verify_main_group_kernel<4>, dim3(2 * words), dim3(kBlock), 0, stream, pre, base, cnt, policy,
                         bitmap, fb, slots, wide, counters);
    else if (fits && cnt <= x.duo_max)
      hipLaunchKernelGGL(verify_main_group_kernel<2>, dim3(words), dim3(kBlock), 0, stream, pre, base, cnt, policy,
                         bitmap, fb, slots, wide, counters);
    else if (pair)
      hipLaunchKernelGGL(verify_main_pair_kernel, gp, dim3(kBlock), 0, stream, pre, base, cnt, policy, bitmap, fb,
                         slots, wide, counters);
    else if (!dedup)
      hipLaunchKernelGGL(verify_main_kernel<true>, g2, dim3(kBlock), 0, stream, pre, base, cnt, bitmap, slots, wide,
                         counters, nullptr, nullptr, qctr);
    else
      hipLaunchKernelGGL(verify_main_kernel<false>, g2, dim3(kBlock), 0, stream, pre, base, cnt, bitmap, slots, wide,
                         counters, dedup ? keytabs : nullptr, dedup ? widetabs : nullptr, qctr);
    mark(3);
    if (pre_k)
      hipLaunchKernelGGL(verify_fallback_kernel<true>, g2, dim3(kBlock), 0, stream, sig, msg_or_k, pk, base, cnt,
                         policy, fb, bitmap, slots, counters);
    else
      hipLaunchKernelGGL(verify_fallback_kernel<false>, g2, dim3(kBlock), 0, stream, sig, msg_or_k, pk, base, cnt,
                         policy, fb, bitmap, slots, counters);
    mark(4);
  }
  return hipGetLastError();
}

// queue counters of workspace ws (after the fallback words)
static uint32_t* queue_counters(uint4* ws, uint32_t grid) {
  uint4* pre = ws + (size_t)grid * (kWsBytesPerBlock / 16);
  return reinterpret_cast<uint32_t*>(reinterpret_cast<uint64_t*>(pre + (size_t)kPreChunk * 14) + kPreChunk / 64);
}

hipError_t launch_verify(const uint8_t* sig, const uint8_t* msg_or_k, const uint8_t* pk, uint32_t n,
                         uint64_t* bitmap, uint32_t policy, bool pre_k, const VerifyExec& x) {
  if (n == 0) return hipSuccess;
  // chunks over concurrent streams only where each stream gets whole chunks
  // larger than the lane-pair size, and never under the phase clock
  uint32_t S = x.nstreams < kMaxVerifyStreams ? x.nstreams : kMaxVerifyStreams;
  const uint32_t sub = x.sub;
  if (S > 1 && (x.clock != nullptr || sub > kPreChunk || (sub & 63u) != 0 || n <= sub ||
                ((uint64_t)n + sub - 1) / sub > (uint64_t)kMainQueueWords))
    S = 1;
  const uint32_t csize = S > 1 ? sub : kPreChunk;
  // an optional smaller first chunk (VerifyExec::first): its phase 1 is the
  // launch's one phase 1 that no main kernel overlaps
  const uint32_t first = S > 1 && x.first && (x.first & 63u) == 0 && x.first < csize && x.first < n ? x.first : 0u;
  const uint64_t nchunks = first ? 1 + ((uint64_t)(n - first) + csize - 1) / csize : ((uint64_t)n + csize - 1) / csize;
  if (S > (uint32_t)nchunks) S = (uint32_t)nchunks;
  // points_done covers exactly one lane-pair chunk (launch_verify_points)
  if (x.points_done && (nchunks != 1 || !verify_pair_points(n, policy, x))) return hipErrorInvalidValue;
  hipError_t e;
  if (S > 1) {
    if ((e = hipEventRecord(x.fork, x.streams[0])) != hipSuccess) return e;
    for (uint32_t j = 1; j < S; ++j)
      if ((e = hipStreamWaitEvent(x.streams[j], x.fork, 0)) != hipSuccess) return e;
  }
  // zero each stream's counters, one per chunk it runs (a lone lane-pair or
  // lane-group chunk uses none: one dependent memset less on the latency path)
  if (x.main_queue && !(nchunks == 1 && pair_chunk(n, policy, x))) {
    for (uint32_t j = 0; j < S; ++j) {
      const uint64_t cj = (nchunks - j + S - 1) / S;
      e = hipMemsetAsync(queue_counters(x.ws[j], x.grid), 0, cj * 4, x.streams[j]);
      if (e != hipSuccess) return e;
    }
  }
  // one key domain for every chunk of the launch (see VerifyExec::key_ready):
  // built by chunk 0 on streams[0] right after its scalar kernel
  VerifyExec xk = x;
  const bool shared_keys = (policy & kModeDedupKeys) && nchunks > 1 && n <= kPreChunk && x.key_ready &&
                           !x.key_ws && csize > x.pair_max &&  // chunk 0 runs the one-lane path that builds it
                           (first == 0 || first > x.pair_max);
  if (shared_keys) {
    xk.key_ws = x.ws[0];
    xk.key_base = 0;
    xk.key_n = n;
    if (x.key_stream) {  // beside the chunks' scalar kernels, on its own stream
      e = S > 1 ? hipStreamWaitEvent(x.key_stream, x.fork, 0) : hipSuccess;
      if (e == hipSuccess)
        e = launch_key_domain(pk, 0, n, wide_count(n, x.wide_min),
                              key_domain(x.ws[0], x.ws_grid ? x.ws_grid : x.grid), x.key_stream);
      if (e == hipSuccess) e = hipEventRecord(x.key_ready, x.key_stream);
      if (e != hipSuccess) return e;
    }
  }
  for (uint64_t c = 0; c < nchunks; ++c) {  // 64-bit: n may reach 2^32 - 64
    const uint32_t j = (uint32_t)(c % S);
    const uint32_t base = first ? (c == 0 ? 0u : (uint32_t)(first + (c - 1) * csize)) : (uint32_t)(c * csize);
    const uint32_t cap = first && c == 0 ? first : csize;
    const uint32_t cnt = n - base < cap ? n - base : cap;
    uint32_t* q = x.main_queue ? queue_counters(x.ws[j], x.grid) + c / S : nullptr;
    if (shared_keys) xk.key_build = c == 0 && !x.key_stream;
    e = verify_chunk(sig, msg_or_k, pk, base, cnt, bitmap, policy, pre_k, xk, x.streams[j], x.ws[j], q,
                     S > 1 ? nullptr : x.clock);
    if (e != hipSuccess) return e;
  }
  if (S > 1) {
    for (uint32_t j = 1; j < S; ++j) {
      if ((e = hipEventRecord(x.join[j], x.streams[j])) != hipSuccess) return e;
      if ((e = hipStreamWaitEvent(x.streams[0], x.join[j], 0)) != hipSuccess) return e;
    }
  }
  return hipGetLastError();
}

hipError_t launch_hram_var(const uint8_t* sig, const uint8_t* pk, const uint8_t* m, const uint64_t* moff,
                           const uint64_t* mlen, uint32_t n, uint8_t* k_out, hipStream_t stream) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(hram_var_kernel, dim3((n + 63) / 64), dim3(64), 0, stream, sig, pk, m, moff, mlen, n, k_out);
  return hipGetLastError();
}

// queue workspace: [0] counter, [64..127] bucket counts, [128..191] cursors,
// [256..) the order (n words)
static hipError_t launch_order(const uint32_t* len, uint32_t n, uint32_t extra, uint32_t* qws, hipStream_t stream,
                               uint32_t long_min = 0) {
  hipError_t e = hipMemsetAsync(qws, 0, kQueueHeaderBytes, stream);
  if (e != hipSuccess) return e;
  uint32_t* hist = qws + 64;
  uint32_t* cursor = qws + 128;
  uint32_t* order = qws + kQueueHeaderBytes / 4;
  const uint32_t tiles = (n + kBlock - 1) / kBlock;
  const uint32_t grid = tiles < 1024u ? tiles : 1024u;
  hipLaunchKernelGGL(order_count_kernel, dim3(grid), dim3(kBlock), 0, stream, len, n, extra, hist);
  hipLaunchKernelGGL(order_scan_kernel, dim3(1), dim3(64), 0, stream, hist, cursor, qws, long_min);
  hipLaunchKernelGGL(order_scatter_kernel, dim3(grid), dim3(kBlock), 0, stream, len, n, extra, cursor, order);
  return hipGetLastError();
}

hipError_t launch_tx_hash(const uint8_t* pre, const uint64_t* off, const uint32_t* len, uint32_t n, uint8_t* msg,
                          uint32_t* qws, uint32_t grid, hipStream_t stream, uint32_t long_min) {
  if (n == 0) return hipSuccess;
  hipError_t e = launch_order(len, n, 0u, qws, stream, long_min);
  if (e != hipSuccess) return e;
  uint32_t blocks = (n + kBlock - 1) / kBlock;
  if (blocks > grid) blocks = grid;
  // long mode: waves 0..K-1 take the long rows first, so the grid gets
  // kLongMaxRows waves on top of the per-lane queue's, which start on it at
  // once (those the long rows do not need skip to the queue)
  if (long_min) blocks += kLongMaxRows / (kBlock / 64u);
  hipLaunchKernelGGL(tx_hash_kernel, dim3(blocks), dim3(kBlock), 0, stream, pre, off, len, n, msg, qws,
                     qws + kQueueHeaderBytes / 4);
  return hipGetLastError();
}

// The blob pass in two halves (the one-call checkSign enqueues both rows'
// parse kernels, then the key work that needs only their keys, then the
// hashing): launch_tx_blob_parse writes status, layout, signature and key of
// every row (and records `parsed`), launch_tx_blob_hash orders the rows and
// hashes them.
hipError_t launch_tx_blob_parse(const uint8_t* blobs, const uint64_t* off, const uint32_t* len, uint32_t n,
                                uint8_t* msg, uint8_t* sig, uint8_t* pk, uint8_t* txid, uint8_t* status,
                                uint32_t* qws, uint32_t grid, hipStream_t stream, uint32_t kind_id,
                                hipEvent_t parsed) {
  if (n == 0) return hipSuccess;
  const BlobKind kind = kind_id == 1u ? blob_kind_validation() : blob_kind_tx();
  uint4* layout = reinterpret_cast<uint4*>(reinterpret_cast<uint8_t*>(qws) + blob_layout_offset(n));
  uint4* side = reinterpret_cast<uint4*>(reinterpret_cast<uint8_t*>(qws) + blob_side_offset(n));
  const uint32_t blocks = (n + kBlock - 1) / kBlock;
  // parse: one lane per row, two rounds of the chip's resident workgroups
  const uint32_t pgrid = 2u * grid;
  hipLaunchKernelGGL(tx_blob_parse_kernel, dim3(blocks < pgrid ? blocks : pgrid), dim3(kBlock), 0, stream, blobs, off,
                     len, n, msg, sig, pk, txid, status, layout, side, kind);
  hipError_t e = hipGetLastError();
  if (e == hipSuccess && parsed) e = hipEventRecord(parsed, stream);
  return e;
}

hipError_t launch_tx_blob_hash(const uint8_t* blobs, const uint64_t* off, const uint32_t* len, uint32_t n,
                               uint8_t* msg, uint8_t* sig, uint8_t* pk, uint8_t* txid, uint8_t* status,
                               uint32_t* qws, uint32_t grid, hipStream_t stream, uint32_t kind_id) {
  if (n == 0) return hipSuccess;
  const BlobKind kind = kind_id == 1u ? blob_kind_validation() : blob_kind_tx();
  uint4* layout = reinterpret_cast<uint4*>(reinterpret_cast<uint8_t*>(qws) + blob_layout_offset(n));
  uint4* side = reinterpret_cast<uint4*>(reinterpret_cast<uint8_t*>(qws) + blob_side_offset(n));
  const uint32_t blocks = (n + kBlock - 1) / kBlock;
  hipError_t e = launch_order(len, n, kind.id_prefixed ? 4u : 0u, qws, stream);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(tx_blob_kernel, dim3(blocks < grid ? blocks : grid), dim3(kBlock), 0, stream, blobs, off, len,
                     n, msg, sig, pk, txid, status, qws, qws + kQueueHeaderBytes / 4, layout, side, kind);
  return hipGetLastError();
}

hipError_t launch_tx_blob(const uint8_t* blobs, const uint64_t* off, const uint32_t* len, uint32_t n, uint8_t* msg,
                          uint8_t* sig, uint8_t* pk, uint8_t* txid, uint8_t* status, uint32_t* qws, uint32_t grid,
                          hipStream_t stream, uint32_t kind_id, hipEvent_t parsed) {
  hipError_t e = launch_tx_blob_parse(blobs, off, len, n, msg, sig, pk, txid, status, qws, grid, stream, kind_id,
                                      parsed);
  if (e != hipSuccess) return e;
  return launch_tx_blob_hash(blobs, off, len, n, msg, sig, pk, txid, status, qws, grid, stream, kind_id);
}

hipError_t launch_sign(const uint8_t* seed, const uint8_t* msg, uint32_t n, uint8_t* pk, uint8_t* sig, uint4* ws,
                       uint32_t grid, hipStream_t stream, const uint8_t* cls, const uint32_t* param,
                       uint8_t* msg_out) {
  if (n == 0) return hipSuccess;
  if (cls)
    hipLaunchKernelGGL(sign_kernel<true>, dim3(grid), dim3(kBlock), 0, stream, seed, msg, n, pk, sig, ws, cls, param,
                       msg_out);
  else
    hipLaunchKernelGGL(sign_kernel<false>, dim3(grid), dim3(kBlock), 0, stream, seed, msg, n, pk, sig, ws, nullptr,
                       nullptr, nullptr);
  return hipGetLastError();
}

}  // namespace stl
