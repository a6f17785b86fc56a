// stl_kernels.hip -- gfx950 kernels of libstl.
//
//   verify_msg32_kernel   the hot path: one Ed25519 verification per lane
//                         (RippleAddress::verifySignature over the 32-byte
//                         signing hash, RippleAddress.cpp:190-200), accept
//                         bits assembled per wave with a 64-bit ballot.
//   verify_prek_kernel    same with k = H(R||A||M) mod L precomputed (used by
//                         the generic verify_detached path for mlen != 32).
//   hram_var_kernel       k for arbitrary-length messages.
//   tx_hash_kernel        SHA512Half(signing preimage) per transaction
//                         (Serializer.cpp:354-360 / SerializedObject.cpp:444-450).
//   sign_kernel           RFC 8032 keypair + signature (synthetic data only).
//
// Launch geometry: 256-thread workgroups (4 waves), grid sized by the host to
// the resident capacity and grid-striding over 256-signature tiles, so the
// per-lane [k](-A) table workspace is bounded by the resident lanes.
#include "stl_base_table.h"
#include "stl_kernels.h"
#include "stl_verify_core.h"

// Occupancy target of the verify kernel (waves per SIMD); register budget =
// 512 / waves.  Tuned on MI355X ("occupancy").
#ifndef STL_VERIFY_WAVES_PER_SIMD
#define STL_VERIFY_WAVES_PER_SIMD 3
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

// Copy the 128-entry affine base table (14 KiB) into LDS once per workgroup.
__device__ __forceinline__ void stage_base_table(uint32_t* sB) {
  const uint32_t* g = &kBaseNiels[0][0];
  for (uint32_t i = threadIdx.x; i < (uint32_t)(kBaseTableEntries * kBaseNielsWords); i += kBlock) sB[i] = g[i];
  __syncthreads();
}

__device__ __forceinline__ TableView lane_table(uint4* ws) {
  const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
  // per-lane contiguous entries: one lookup touches 2-3 whole 128-B lines of
  // its own lane instead of 16 B of nine lines shared by lanes with other digits
  return TableView{ws + (((size_t)blockIdx.x * (kBlock / 64) + wave) * 64 + lane) * kTableQuads, 1};
}

__device__ __forceinline__ void ld_pre(PreState& p, const uint4* q) {
  uint32_t w[28];
#pragma unroll
  for (int i = 0; i < 7; ++i) {
    const uint4 v = q[i];
    w[4 * i] = v.x; w[4 * i + 1] = v.y; w[4 * i + 2] = v.z; w[4 * i + 3] = v.w;
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) p.k[i] = w[i];
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    p.negAx.v[i] = w[8 + i];
    p.negAy.v[i] = w[17 + i];
  }
  p.ok = w[26];
  p.pad = 0;
}

__device__ __forceinline__ void st_pre(uint4* q, const PreState& p) {
  uint32_t w[28];
#pragma unroll
  for (int i = 0; i < 8; ++i) w[i] = p.k[i];
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    w[8 + i] = p.negAx.v[i];
    w[17 + i] = p.negAy.v[i];
  }
  w[26] = p.ok;
  w[27] = 0;
#pragma unroll
  for (int i = 0; i < 7; ++i) q[i] = make_uint4(w[4 * i], w[4 * i + 1], w[4 * i + 2], w[4 * i + 3]);
}

// Phase 1: one signature per lane -- pre-checks, k = SHA-512(R||A||M) mod L
// (or k given, PRE_K), decompression of A.  Signatures [base, base+cnt).
template <bool PRE_K>
__global__ __launch_bounds__(kBlock) void verify_pre_kernel(const uint8_t* __restrict__ sig,
                                                            const uint8_t* __restrict__ msg_or_k,
                                                            const uint8_t* __restrict__ pk, uint32_t base,
                                                            uint32_t cnt, uint32_t policy, uint4* __restrict__ pre) {
  const uint32_t t = blockIdx.x * kBlock + threadIdx.x;
  if (t >= cnt) return;
  const size_t j = (size_t)base + t;
  uint32_t R[8], S[8], A[8], M[8], k[8];
  ld8(R, sig + 64 * j);
  ld8(S, sig + 64 * j + 32);
  ld8(A, pk + 32 * j);
  ld8(M, msg_or_k + 32 * j);
  if (PRE_K) {
#pragma unroll
    for (int i = 0; i < 8; ++i) k[i] = M[i];
  } else {
    uint32_t h[16];
    sha512_hram32(h, R, A, M);
    sc_reduce64(k, h);
  }
  PreState p;
  verify_phase1(p, R, S, A, k, policy);
  st_pre(pre + (size_t)t * 7, p);
}

// Phase 2: the Straus loop, encode and compare; grid-strides over 256-signature
// tiles of [base, base+cnt) so the per-lane table workspace is bounded by the
// resident lanes; one ballot word per wave.
__global__ __launch_bounds__(kBlock, STL_VERIFY_WAVES_PER_SIMD) void verify_main_kernel(
    const uint8_t* __restrict__ sig, const uint4* __restrict__ pre, uint32_t base, uint32_t cnt,
    uint64_t* __restrict__ bitmap, uint4* __restrict__ ws) {
  __shared__ uint32_t sB[kBaseTableEntries * kBaseNielsWords];
  stage_base_table(sB);
  const TableView tv = lane_table(ws);
  const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63u;
  for (uint32_t tile = blockIdx.x * kBlock; tile < cnt; tile += gridDim.x * kBlock) {
    const uint32_t t = tile + threadIdx.x;
    const bool live = t < cnt;
    const uint32_t tt = live ? t : (cnt - 1);  // tail lanes re-read a valid element
    const size_t j = (size_t)base + tt;
    PreState p;
    ld_pre(p, pre + (size_t)tt * 7);
    uint32_t R[8], S[8];
    ld8(R, sig + 64 * j);
    ld8(S, sig + 64 * j + 32);
    bool ok = verify_phase2(p, R, S, tv, sB);
    ok = ok && live;
    const uint64_t word = __ballot(ok);
    const uint32_t wbase = tile + wave * 64;
    if (lane == 0 && wbase < cnt) bitmap[(base + wbase) >> 6] = word;
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

// msg_i = SHA512Half(preimage_i)
__global__ void tx_hash_kernel(const uint8_t* __restrict__ pre, const uint64_t* __restrict__ off,
                               const uint32_t* __restrict__ len, uint32_t n, uint8_t* __restrict__ msg) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint64_t st[8];
  sha512_prefixed(st, nullptr, 0, pre + off[i], len[i]);
  uint32_t h[16];
  sha512_digest_le32(h, st);
  st8(msg + 32 * (size_t)i, h);
}

// SHA-512 of a short word-aligned input (nwords even, nwords*4 <= 108 bytes).
__device__ __forceinline__ void sha512_short(uint32_t out[16], const uint32_t* in, int nwords) {
  uint64_t st[8], w[16];
  sha512_init(st);
#pragma unroll
  for (int j = 0; j < 16; ++j) w[j] = 0;
  for (int j = 0; j < nwords / 2; ++j) w[j] = be64_from_le32(in[2 * j], in[2 * j + 1]);
  w[nwords / 2] = 0x8000000000000000ULL;
  w[15] = (uint64_t)nwords * 32;
  sha512_compress(st, w);
  sha512_digest_le32(out, st);
}

__global__ __launch_bounds__(kBlock, 2) void sign_kernel(const uint8_t* __restrict__ seed,
                                                      const uint8_t* __restrict__ msg, uint32_t n,
                                                      uint8_t* __restrict__ pk_out, uint8_t* __restrict__ sig_out,
                                                      uint4* __restrict__ ws) {
  __shared__ uint32_t sB[kBaseTableEntries * kBaseNielsWords];
  stage_base_table(sB);
  const TableView tv = lane_table(ws);
  for (uint32_t base = blockIdx.x * kBlock; base < n; base += gridDim.x * kBlock) {
    const uint32_t i = base + threadIdx.x;
    const bool live = i < n;
    const size_t j = live ? i : (n - 1);
    uint32_t sd[8], M[8], h[16];
    ld8(sd, seed + 32 * j);
    ld8(M, msg + 32 * j);
    sha512_short(h, sd, 8);
    uint32_t a[8], pre[16];
#pragma unroll
    for (int q = 0; q < 8; ++q) a[q] = h[q];
    a[0] &= 0xfffffff8u;            // clamp: h[0] &= 248
    a[7] = (a[7] & 0x7fffffffu) | 0x40000000u;  // h[31] &= 127; h[31] |= 64
    uint32_t x[16], a_red[8], zero[8];
#pragma unroll
    for (int q = 0; q < 16; ++q) x[q] = q < 8 ? a[q] : 0u;
    sc_reduce64(a_red, x);
#pragma unroll
    for (int q = 0; q < 8; ++q) zero[q] = 0;
    ge_p3 id;
    ge_p3_0(id);
    ge_p2 P;
    uint32_t A[8];
    double_scalarmult(P, id, zero, a_red, tv, sB);  // A = [a]B
    ge_tobytes(A, P);
    // r = SHA-512(h[32..63] || M) mod L
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      pre[q] = h[8 + q];
      pre[8 + q] = M[q];
    }
    uint32_t rh[16], r[8], R[8];
    sha512_short(rh, pre, 16);
    sc_reduce64(r, rh);
    double_scalarmult(P, id, zero, r, tv, sB);      // R = [r]B
    ge_tobytes(R, P);
    uint32_t kh[16], k[8], S[8];
    sha512_hram32(kh, R, A, M);
    sc_reduce64(k, kh);
    sc_muladd(S, k, a, r);                                   // S = r + k a mod L
    if (live) {
      st8(pk_out + 32 * j, A);
      st8(sig_out + 64 * j, R);
      st8(sig_out + 64 * j + 32, S);
    }
  }
}

// ---- host-side launchers (called from stl_api.cpp) ----
const void* kernel_verify_msg32() { return reinterpret_cast<const void*>(&verify_main_kernel); }

hipError_t launch_verify(const uint8_t* sig, const uint8_t* msg_or_k, const uint8_t* pk, uint32_t n,
                         uint64_t* bitmap, uint32_t policy, uint4* ws, uint32_t grid, bool pre_k,
                         hipStream_t stream) {
  if (n == 0) return hipSuccess;
  // ws = [per-lane tables: grid x kWsBytesPerBlock][PreState x kPreChunk]
  uint4* tables = ws;
  uint4* pre = ws + (size_t)grid * (kWsBytesPerBlock / 16);
  for (uint32_t base = 0; base < n; base += kPreChunk) {
    const uint32_t cnt = n - base < kPreChunk ? n - base : kPreChunk;
    const dim3 g1((cnt + kBlock - 1) / kBlock);
    if (pre_k)
      hipLaunchKernelGGL(verify_pre_kernel<true>, g1, dim3(kBlock), 0, stream, sig, msg_or_k, pk, base, cnt, policy,
                         pre);
    else
      hipLaunchKernelGGL(verify_pre_kernel<false>, g1, dim3(kBlock), 0, stream, sig, msg_or_k, pk, base, cnt,
                         policy, pre);
    const uint32_t tiles = (cnt + kBlock - 1) / kBlock;
    hipLaunchKernelGGL(verify_main_kernel, dim3(tiles < grid ? tiles : grid), dim3(kBlock), 0, stream, sig, pre,
                       base, cnt, bitmap, tables);
  }
  return hipGetLastError();
}

hipError_t launch_hram_var(const uint8_t* sig, const uint8_t* pk, const uint8_t* m, const uint64_t* moff,
                           const uint64_t* mlen, uint32_t n, uint8_t* k_out, hipStream_t stream) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(hram_var_kernel, dim3((n + 63) / 64), dim3(64), 0, stream, sig, pk, m, moff, mlen, n, k_out);
  return hipGetLastError();
}

hipError_t launch_tx_hash(const uint8_t* pre, const uint64_t* off, const uint32_t* len, uint32_t n, uint8_t* msg,
                          hipStream_t stream) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(tx_hash_kernel, dim3((n + 255) / 256), dim3(256), 0, stream, pre, off, len, n, msg);
  return hipGetLastError();
}

hipError_t launch_sign(const uint8_t* seed, const uint8_t* msg, uint32_t n, uint8_t* pk, uint8_t* sig, uint4* ws,
                       uint32_t grid, hipStream_t stream) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(sign_kernel, dim3(grid), dim3(kBlock), 0, stream, seed, msg, n, pk, sig, ws);
  return hipGetLastError();
}

}  // namespace stl
