// stl_kernels.h -- launch interface between stl_api.cpp (host) and
// stl_kernels.hip (gfx950 device code).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace stl {

constexpr uint32_t kBlock = 256;          // threads per workgroup (4 waves)
// per-lane slot: two split tables (stl_kernels.hip lane_tables): 2 x 8 heads
// of 8 quads (entry 0, the identity, shares one line) + 2 x 9 tail quads
constexpr uint32_t kHeadQuads = 2 * 8 * 8;
constexpr uint32_t kSlotQuads = kHeadQuads + 2 * 9;
// workspace bytes per resident workgroup: 256 lanes x 146 x 16 B = 584 KiB
constexpr size_t kWsBytesPerBlock = (size_t)kBlock * kSlotQuads * 16;
// verify phase-1 state (HalfState, 224 B) is produced and consumed in chunks
// of kPreChunk signatures (a multiple of 64, so chunks start on bitmap words),
// plus one fallback-flag word per 64 signatures
constexpr uint32_t kPreChunk = 1u << 20;
// work counters of the main kernel's unit queue, one per chunk a launch_verify
// call runs on a workspace (chunks >= 2^16 signatures, n < 2^32)
constexpr uint32_t kMainQueueWords = 1u << 16;
constexpr size_t kPreBytes = (size_t)kPreChunk * 224 + (size_t)kPreChunk / 8 + (size_t)kMainQueueWords * 4;
// Per-batch key dedup (STL_DEDUP_KEYS), per kPreChunk signatures: an open-
// addressing table of 2 * kPreChunk slots, representative / unique-id /
// owner arrays, a counter, and the decoded keys (-A affine + ok, 5 x uint4).
constexpr size_t kDedupSlots = 2 * (size_t)kPreChunk;
// shared per-key A-tables (9 cached entries, 1,296 B) for up to kKeyTables
// distinct keys per chunk; above that the chunk builds per-lane tables
constexpr uint32_t kKeyTables = 1u << 16;
// wide shared A-tables (137 cached entries, 19,728 B) when a chunk has at most
// kWideKeys distinct keys and at least kWideKeyRepeat signatures per key
constexpr uint32_t kWideKeys = 4096;
constexpr uint32_t kWideKeyRepeat = 32;
constexpr size_t kDedupBytes = kDedupSlots * 4 + 3 * (size_t)kPreChunk * 4 + 256 + (size_t)kPreChunk * 80 +
                               (size_t)kKeyTables * 81 * 16 + (size_t)kWideKeys * 137 * 9 * 16;
// verify workspace for a grid of `grid` resident workgroups
inline size_t verify_ws_bytes(uint32_t grid, bool dedup = false) {
  return kWsBytesPerBlock * grid + kPreBytes + (dedup ? kDedupBytes : 0);
}

// Kernel mode word: bit 0 = policy (STL_POLICY_*), bit 8 = full-length path
// for every lane (STL_FULL_LENGTH), bit 9 = per-batch key dedup (STL_DEDUP_KEYS),
// bit 10 = never two lanes per signature (STL_ONE_LANE).
constexpr uint32_t kModeFullLength = 0x100u;
constexpr uint32_t kModeDedupKeys = 0x200u;
constexpr uint32_t kModeOneLane = 0x400u;
// bit 11 = the raw predicate without stellard's S < L (STL_DEBUG_RAW_PREDICATE, test-only)
constexpr uint32_t kModeRaw = 0x800u;
inline uint32_t kernel_mode(uint32_t flags) {
  return (flags & 0x1u) | ((flags & 0x4u) ? kModeFullLength : 0u) | ((flags & 0x8u) ? kModeDedupKeys : 0u) |
         ((flags & 0x10u) ? kModeOneLane : 0u) | ((flags & 0x80000000u) ? kModeRaw : 0u);
}
// the policy argument of the verify core (stl_verify_core.h): bit 0 the
// libsodium policy, bit 1 (kPolicyRaw) the raw predicate
__host__ __device__ inline uint32_t core_policy(uint32_t mode) { return (mode & 1u) | ((mode & kModeRaw) ? 2u : 0u); }

const void* kernel_verify_msg32();
// counters (nullable): device u64 [0] accept bits written, [1] lanes checked by
// the full-length fallback path (stl_get_stats)
// pair_max: chunks of at most this many signatures (and 2x as many workspace
// lanes in `grid`) run two lanes per signature (verify_main_pair_kernel);
// the caller passes a quarter of the device's resident lanes, i.e. at most one
// pair wave per SIMD -- above that the duplicated doublings cost more than the
// shorter chains save.
// Optional phase clock (stl_set_phase_timing): launch_verify calls
// mark(ctx, stream, i) before a chunk's first kernel (i = 0) and after each
// phase -- 1 scalar (the whole of phase 1 when it runs as one kernel), 2 point
// (+ the key-dedup kernels), 3 main, 4 fallback.
struct PhaseClock {
  void (*mark)(void* ctx, hipStream_t stream, int i);
  void* ctx;
};
// How launch_verify runs a batch.  The batch is cut into chunks (at most
// kPreChunk signatures, the phase-1 state a workspace holds); each chunk is
// phase 1, main, fallback on one stream.  With nstreams > 1 (and no phase
// clock, whose per-kernel durations need kernels that do not overlap) chunk i
// of `sub` signatures runs on streams[i % nstreams] with workspace
// ws[i % nstreams]: the streams fork from streams[0] (the caller's) through
// `fork` and join it through `join`, so one chunk's phase-1 kernels and the
// next chunks' kernels fill the ragged last rounds of each other's launches.
constexpr uint32_t kMaxVerifyStreams = 4;
struct VerifyExec {
  uint32_t grid = 1;                    // resident workgroups = per-lane workspace slots per ws
  uint32_t ws_grid = 0;                 // the grid the workspaces were sized for (verify_ws_bytes): the key
                                        // domain sits after it, wherever a launch's own grid ends (0: grid)
  uint32_t pair_max = 0;                // chunks up to this size run two lanes per signature
  const uint4* wide = nullptr;          // wide base tables
  unsigned long long* counters = nullptr;
  const PhaseClock* clock = nullptr;
  int fused_prep = 1;                   // 0: scalar and point kernels; 1: phase 1 in one kernel
  bool main_queue = true;               // main kernel pulls 64-signature units from a counter
  bool concurrent = false;              // other chunks share the chip (host API, two streams): no
                                        // two-role phase 1 above pair_max (it trades work for latency)
  uint32_t nstreams = 1;
  uint32_t sub = kPreChunk;             // chunk size when nstreams > 1 (multiple of 64, >= 2^16)
  uint32_t first = 0;                   // nstreams > 1: a first chunk of this many rows (multiple of 64,
                                        // < sub), then chunks of `sub`; 0: all of `sub`
  hipStream_t streams[kMaxVerifyStreams] = {};
  uint4* ws[kMaxVerifyStreams] = {};    // verify_ws_bytes(grid, dedup) each
  hipEvent_t fork = nullptr;
  hipEvent_t join[kMaxVerifyStreams] = {};
  uint32_t quad_max = 0;                // lane-pair chunks up to this size run their main kernel on
                                        // eight lanes per signature (verify_main_group_kernel<4>),
  uint32_t duo_max = 0;                 // up to this size on four (verify_main_group_kernel<2>); 0: never
  bool points_done = false;             // one lane-pair chunk whose point role already ran
                                        // (launch_verify_points, ordered before this launch)
  // Key dedup over a whole batch (kModeDedupKeys): one key domain -- hash
  // slots, owners, decoded keys, key tables -- for every chunk, instead of one
  // per chunk (round 6: a chunk of config 1's 100k rows rebuilt the same 1,000
  // keys' tables on the critical path).  launch_verify sets it up by itself
  // for a launch of several chunks when key_ready is given; a caller that
  // runs the chunks as separate launches (the one-call checkSign) sets
  // key_ws to the workspace holding the domain, key_n to its rows, key_base to
  // this launch's first row in it, and key_build on the launch that builds it
  // (its first chunk's stream records key_ready; the others wait for it).
  hipEvent_t key_ready = nullptr;
  hipEvent_t key_after = nullptr;       // the builder's stream waits for it first (keys of other rows
                                        // still being produced, e.g. by the blob pass on another stream)
  uint4* key_ws = nullptr;
  uint32_t key_base = 0, key_n = 0;
  bool key_build = false;
  // launch_verify's own shared domain: built on this otherwise idle stream
  // (forked from streams[0]) beside the chunks' scalar kernels, every chunk
  // waiting for key_ready; nullptr: built by chunk 0 after its scalar kernel
  hipStream_t key_stream = nullptr;
  // rows below which a key domain builds no wide (137-entry) key tables --
  // the 9-entry ones instead -- so a short call does not wait for the wide
  // build (STL_TUNE_WIDE_MIN_ROWS)
  uint32_t wide_min = 0;
  // With key_ws: R decoded ahead for every row of the key domain
  // (launch_point_r, 5 quads per row, recording r_ready): the chunks run the
  // short verify_finish_keyed_kernel instead of the keyed point kernel
  const uint4* rdec = nullptr;
  hipEvent_t r_ready = nullptr;
};
// The pre-checks and R's decoding of rows [0, n) into rdec (5 quads per row),
// for VerifyExec::rdec.
hipError_t launch_point_r(const uint8_t* sig, const uint8_t* pk, uint32_t n, uint32_t policy, uint4* rdec,
                          hipStream_t stream);
// The dedup chain over rows [0, n) of pk into the key domain of workspace ws
// (grid: its resident workgroups) on `stream` -- what a chunk with
// kModeDedupKeys builds for itself, for a caller that runs it beside other
// work and hands the domain to the chunks through VerifyExec::key_ws.
hipError_t launch_key_domain_ws(const uint8_t* pk, uint32_t n, uint4* ws, uint32_t grid, uint32_t wide_min,
                                hipStream_t stream);
// Whether launch_verify of n <= kPreChunk signatures (one chunk) runs its
// phase 1 as the two-role lane-pair kernel -- then its point role (the two
// square-root chains; needs only the signatures and keys) may be launched
// ahead by launch_verify_points, e.g. while the messages are still being
// hashed, and launch_verify with points_done runs only the scalar role.
bool verify_pair_points(uint32_t n, uint32_t policy, const VerifyExec& x);
hipError_t launch_verify_points(const uint8_t* sig, const uint8_t* pk, uint32_t n, uint32_t policy,
                                const VerifyExec& x, hipStream_t stream);
hipError_t launch_verify(const uint8_t* sig, const uint8_t* msg_or_k, const uint8_t* pk, uint32_t n,
                         uint64_t* bitmap, uint32_t policy, bool pre_k, const VerifyExec& x);
hipError_t launch_hram_var(const uint8_t* sig, const uint8_t* pk, const uint8_t* m, const uint64_t* moff,
                           const uint64_t* mlen, uint32_t n, uint8_t* k_out, hipStream_t stream);
// counter: one device word of scratch (reset by the launcher); grid: upper
// bound on workgroups (the kernel pulls work from the counter)
// Hash-kernel queue workspace: a header (work counter, bucket counts and
// cursors of the longest-first order) and the order itself.
constexpr size_t kQueueHeaderBytes = 1024;
inline size_t hash_queue_bytes(size_t n) { return kQueueHeaderBytes + 4 * n; }
// The blob path's queue also holds each row's layout from the parse kernel
// (32 B: status and the cut ranges), 16-byte aligned after the order, and
// each row's spliced block (128 B: the SHA-512 block of the signing preimage
// that holds the cut, assembled by the parse kernel).
inline size_t blob_layout_offset(size_t n) { return (hash_queue_bytes(n) + 15) / 16 * 16; }
inline size_t blob_side_offset(size_t n) { return blob_layout_offset(n) + 32 * n; }
inline size_t blob_queue_bytes(size_t n) { return blob_side_offset(n) + 128 * n; }
// long_min > 0: up to 1,024 of the longest rows of more than long_min SHA-512
// blocks are hashed one per wave (the latency path of small batches)
hipError_t launch_tx_hash(const uint8_t* pre, const uint64_t* off, const uint32_t* len, uint32_t n, uint8_t* msg,
                          uint32_t* qws, uint32_t grid, hipStream_t stream, uint32_t long_min = 0);
// qws: blob_queue_bytes(n)
// parsed (nullable): recorded after the parse kernel (the rows' signatures and
// keys are out; the hashing follows)
hipError_t launch_tx_blob(const uint8_t* blobs, const uint64_t* off, const uint32_t* len, uint32_t n, uint8_t* msg,
                          uint8_t* sig, uint8_t* pk, uint8_t* txid, uint8_t* status, uint32_t* qws, uint32_t grid,
                          hipStream_t stream, uint32_t kind = 0u /* STL_BLOB_* */, hipEvent_t parsed = nullptr);
// its two halves: the parse kernel (+ `parsed`), then the ordering and hashing
hipError_t launch_tx_blob_parse(const uint8_t* blobs, const uint64_t* off, const uint32_t* len, uint32_t n,
                                uint8_t* msg, uint8_t* sig, uint8_t* pk, uint8_t* txid, uint8_t* status,
                                uint32_t* qws, uint32_t grid, hipStream_t stream, uint32_t kind, hipEvent_t parsed);
hipError_t launch_tx_blob_hash(const uint8_t* blobs, const uint64_t* off, const uint32_t* len, uint32_t n,
                               uint8_t* msg, uint8_t* sig, uint8_t* pk, uint8_t* txid, uint8_t* status,
                               uint32_t* qws, uint32_t grid, hipStream_t stream, uint32_t kind);
// Wide base tables (stl_verify_core.h): 2 * 32769 rows of 28 words.
constexpr size_t kWideTableBytes = 2ull * 32769 * 28 * 4;
// Key-repeat sample of [0, n): *flag = 1 when a quarter of up to 2,048 sampled
// keys repeat (device-resident automatic dedup; flag may be host-mapped).
hipError_t launch_key_sample(const uint8_t* pk, uint32_t n, uint32_t* flag, hipStream_t stream);
hipError_t launch_wide_table(uint4* out, hipStream_t stream);
// nwg one-wave workgroups, each {memtime, memrealtime, XCC_ID, HW_ID} (4 u64)
hipError_t launch_clock_stamp(unsigned long long* out, uint32_t nwg, hipStream_t stream);
// cls / param (nullable, test data only): per-row adversarial class and its
// parameter (stl_kernels.hip adversarial_row); msg_out receives the messages.
hipError_t launch_sign(const uint8_t* seed, const uint8_t* msg, uint32_t n, uint8_t* pk, uint8_t* sig, uint4* ws,
                       uint32_t grid, hipStream_t stream, const uint8_t* cls = nullptr,
                       const uint32_t* param = nullptr, uint8_t* msg_out = nullptr);

}  // namespace stl
