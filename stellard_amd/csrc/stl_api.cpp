// stl_api.cpp -- host side of libstl: the extern "C" boundary declared in
// include/stl.h.  Owns devices, streams, workspaces, staging buffers and RCCL
// communicators; has no CPU verification path (a device failure returns < 0
// and the caller -- stellard -- falls back to libsodium, as SURVEY.md
// section 8b requires).
//
// Threading: stellard calls verify concurrently from JobQueue workers
// (JobQueue.cpp:217-243).  Every device has a mutex that serialises the host
// batch entry points on that device; a batch that gathers over RCCL holds
// every device's mutex for its whole run.  The device-resident entry points
// key their workspace by (device, stream) so concurrent streams never share
// one.
//
// Multi-GPU: a host batch is split into contiguous 64-aligned
// shards (by index, or by preimage bytes for variable-length rows), one host
// thread per shard.  With two or more devices each device keeps its slice of
// the accept bitmap in HBM and RCCL gathers the slices into device 0 over
// xGMI (ncclGather for equal slices, grouped send/recv for byte-balanced
// ones), then one copy brings the bitmap to the host.  One process per GPU
// uses stl_comm_* + stl_bitmap_gather_device instead.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <array>
#include <atomic>
#include <chrono>
#include <cstddef>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

#include "../../include/stl.h"
#include "stl_kernels.h"

namespace {

// ---- fault injection (stl_debug_fault_after) --------------------------------
// A countdown over the HIP / RCCL calls libstl checks; the call at which it
// reaches zero is not executed and reports failure.  One shot.
std::atomic<long long> g_fault_after{-1};

bool fault_now() {
  long long v = g_fault_after.load(std::memory_order_relaxed);
  while (v >= 0) {
    if (g_fault_after.compare_exchange_weak(v, v - 1, std::memory_order_relaxed)) return v == 0;
  }
  return false;
}

#define STL_TRY(expr)                        \
  do {                                       \
    if (fault_now()) return STL_EHIP;        \
    hipError_t e_ = (expr);                  \
    if (e_ != hipSuccess) return STL_EHIP;   \
  } while (0)

#define STL_RCCL_TRY(expr)                   \
  do {                                       \
    if (fault_now()) return STL_ERCCL;       \
    ncclResult_t r_ = (expr);                \
    if (r_ != ncclSuccess) return STL_ERCCL; \
  } while (0)

#define STL_RC(expr)        \
  do {                      \
    int rc_ = (expr);       \
    if (rc_) return rc_;    \
  } while (0)

// ---- RCCL, loaded on first use (libstl does not need it on one device) ----
struct Rccl {
  std::once_flag once;
  bool ok = false;
  decltype(&ncclGetUniqueId) GetUniqueId = nullptr;
  decltype(&ncclCommInitRank) CommInitRank = nullptr;
  decltype(&ncclCommInitAll) CommInitAll = nullptr;
  decltype(&ncclCommDestroy) CommDestroy = nullptr;
  decltype(&ncclGather) Gather = nullptr;
  decltype(&ncclAllGather) AllGather = nullptr;
  decltype(&ncclSend) Send = nullptr;
  decltype(&ncclRecv) Recv = nullptr;
  decltype(&ncclGroupStart) GroupStart = nullptr;
  decltype(&ncclGroupEnd) GroupEnd = nullptr;
  decltype(&ncclCommCount) CommCount = nullptr;
  decltype(&ncclCommUserRank) CommUserRank = nullptr;
  // nonblocking bring-up with a deadline; optional symbols
  decltype(&ncclCommInitRankConfig) CommInitRankConfig = nullptr;
  decltype(&ncclCommGetAsyncError) CommGetAsyncError = nullptr;
  decltype(&ncclCommAbort) CommAbort = nullptr;
  bool nonblocking() const { return CommInitRankConfig && CommGetAsyncError && CommAbort; }

  template <typename F>
  static bool sym(void* h, const char* name, F& f) {
    f = reinterpret_cast<F>(dlsym(h, name));
    return f != nullptr;
  }
  bool load() {
    std::call_once(once, [this] {
      // an already loaded librccl (e.g. PyTorch's) is reused by soname
      void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
      if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
      if (!h) return;
      ok = sym(h, "ncclGetUniqueId", GetUniqueId) && sym(h, "ncclCommInitRank", CommInitRank) &&
           sym(h, "ncclCommInitAll", CommInitAll) && sym(h, "ncclCommDestroy", CommDestroy) &&
           sym(h, "ncclGather", Gather) && sym(h, "ncclAllGather", AllGather) && sym(h, "ncclSend", Send) &&
           sym(h, "ncclRecv", Recv) && sym(h, "ncclGroupStart", GroupStart) && sym(h, "ncclGroupEnd", GroupEnd) &&
           sym(h, "ncclCommCount", CommCount) && sym(h, "ncclCommUserRank", CommUserRank);
      (void)(sym(h, "ncclCommInitRankConfig", CommInitRankConfig) &&
             sym(h, "ncclCommGetAsyncError", CommGetAsyncError) && sym(h, "ncclCommAbort", CommAbort));
    });
    return ok;
  }
};
Rccl g_rccl;

// Deadline of the one-process-per-GPU communicator's RCCL operations: the
// bring-up (a rank that never joins would block ncclCommInitRank forever) and
// stl_comm_sync's wait on a gather.  STL_RCCL_TIMEOUT_S at stl_init, or
// STL_TUNE_RCCL_TIMEOUT_MS.
std::atomic<int> g_rccl_timeout_ms{120000};

// Settles a nonblocking communicator's call that returned r: ncclInProgress
// is polled (ncclCommGetAsyncError) until it completes or the deadline
// passes.  STL_OK, or STL_ERCCL on an error or a timeout (the caller aborts).
int rccl_settle(ncclComm_t comm, ncclResult_t r) {
  if (r == ncclSuccess) return STL_OK;
  if (r != ncclInProgress || !comm || !g_rccl.CommGetAsyncError) return STL_ERCCL;
  const auto end = std::chrono::steady_clock::now() + std::chrono::milliseconds(g_rccl_timeout_ms.load());
  ncclResult_t st = ncclInProgress;
  while (g_rccl.CommGetAsyncError(comm, &st) == ncclSuccess && st == ncclInProgress) {
    if (std::chrono::steady_clock::now() > end) return STL_ERCCL;
    std::this_thread::sleep_for(std::chrono::microseconds(200));
  }
  return st == ncclSuccess ? STL_OK : STL_ERCCL;
}

struct DevBuf {
  void* p = nullptr;
  size_t cap = 0;
  int ensure(size_t bytes) {
    if (bytes <= cap) return STL_OK;
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
    if (fault_now() || hipMalloc(&p, bytes) != hipSuccess) {
      p = nullptr;
      return STL_ENOMEM;
    }
    cap = bytes;
    return STL_OK;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
  }
};

// Phase timing (stl_set_phase_timing): launch_verify marks the phase
// boundaries of each chunk; each mark records a pooled HIP event on the launch
// stream.  stl_get_stats sums the completed chunks' phase durations.  Timing
// calls bypass the fault-injection countdown and never fail a launch: a chunk
// whose events could not be recorded is dropped from the sums.
struct PhaseTimer {
  std::mutex mu;
  std::vector<hipEvent_t> pool;
  std::vector<std::array<hipEvent_t, 5>> done;
  uint64_t ns[4] = {0, 0, 0, 0};
  uint64_t chunks = 0;
  hipEvent_t take() {
    std::lock_guard<std::mutex> lk(mu);
    if (!pool.empty()) {
      hipEvent_t e = pool.back();
      pool.pop_back();
      return e;
    }
    hipEvent_t e = nullptr;
    if (hipEventCreate(&e) != hipSuccess) e = nullptr;
    return e;
  }
  void give(hipEvent_t e) {
    if (!e) return;
    std::lock_guard<std::mutex> lk(mu);
    pool.push_back(e);
  }
  // completed chunks -> sums.  A chunk another thread enqueued after the
  // caller's synchronisation is left in `done` until its last event has
  // completed (hipEventQuery), so it is neither dropped nor recycled early.
  void collect() {
    std::lock_guard<std::mutex> lk(mu);
    std::vector<std::array<hipEvent_t, 5>> pending;
    for (auto& c : done) {
      if (hipEventQuery(c[4]) == hipErrorNotReady) {
        pending.push_back(c);
        continue;
      }
      uint64_t t[4];
      bool ok = true;
      for (int i = 0; i < 4 && ok; ++i) {
        float ms = 0.f;
        ok = hipEventElapsedTime(&ms, c[i], c[i + 1]) == hipSuccess;
        t[i] = (uint64_t)((double)ms * 1e6);
      }
      if (ok) {
        for (int i = 0; i < 4; ++i) ns[i] += t[i];
        ++chunks;
      }
      for (hipEvent_t e : c) pool.push_back(e);
    }
    done.swap(pending);
  }
  void reset() {
    collect();
    std::lock_guard<std::mutex> lk(mu);
    for (auto& v : ns) v = 0;
    chunks = 0;
  }
  void release() {
    std::lock_guard<std::mutex> lk(mu);
    for (auto& c : done)
      for (hipEvent_t e : c) pool.push_back(e);
    done.clear();
    for (hipEvent_t e : pool) (void)hipEventDestroy(e);
    pool.clear();
  }
};

std::atomic<bool> g_phase_timing{false};

// one chunk being marked by this thread (marks of a chunk come from one thread)
thread_local std::array<hipEvent_t, 5> t_marks;
thread_local bool t_marks_ok = false;

void phase_mark(void* ctx, hipStream_t s, int i) {
  auto* t = static_cast<PhaseTimer*>(ctx);
  if (i == 0) {
    // events left by a chunk whose launches stopped between its marks (their
    // timer may be gone after stl_shutdown): destroy them
    for (hipEvent_t& m : t_marks) {
      if (m) (void)hipEventDestroy(m);
      m = nullptr;
    }
    t_marks_ok = true;
  }
  hipEvent_t e = t->take();
  if (!e || hipEventRecord(e, s) != hipSuccess) {
    t->give(e);
    t_marks[i] = nullptr;
    t_marks_ok = false;
  } else {
    t_marks[i] = e;
  }
  if (i == 4) {
    if (t_marks_ok) {
      std::lock_guard<std::mutex> lk(t->mu);
      t->done.push_back(t_marks);
    } else {
      for (hipEvent_t m : t_marks) t->give(m);
    }
    t_marks.fill(nullptr);
    t_marks_ok = false;
  }
}

// Execution tuning (stl_debug_tuning): how a verify launch is cut into kernels
// and streams.  Every setting gives the same accept bits (tests run them all).
std::atomic<int> g_tune_fused{1};     // phase 1 as one kernel
std::atomic<int> g_tune_queue{1};     // main kernel pulls units from a counter
std::atomic<int> g_tune_streams{2};   // concurrent streams per device-resident call (A/B: DESIGN.md section 8)
std::atomic<int> g_tune_sub_log2{0};  // log2 signatures per stream chunk; 0 = by batch size (chunk_for)
std::atomic<int> g_tune_byte_shards{0};  // test hook: byte-balanced shards even for one shard
std::atomic<int> g_tune_quad{3};      // smallest chunks' main kernel on lane groups: bit 0 quads, bit 1 duos
std::atomic<int> g_tune_long_hash{8}; // small batches: rows of more than this many blocks hashed one per wave (0 off)
std::atomic<int> g_tune_shared_keys{1}; // key dedup over several chunks: one key domain per call (0: one per chunk)
std::atomic<int> g_tune_wide_min{0};    // key domains of fewer rows build no wide key tables (the 9-entry ones)
std::atomic<int> g_tune_r_ahead{1};     // one-call checkSign with a shared key domain: R decoded ahead on its own stream
std::atomic<int> g_tune_first_chunk{0}; // device-resident verify: rows of a smaller first chunk (0: equal chunks)

// Rows per step of verify time: the device-resident verify runs a chunk's
// 64-signature units on its resident waves, two per SIMD, so its time rises in
// steps of one wave per SIMD (65,536 rows on 256 CUs): a
// shard one row past a multiple pays a whole extra step on its slowest SIMDs.
// Set at stl_init from the first device; 65,536 (MI355X) before that.
std::atomic<uint64_t> g_shard_quantum{65536};

// Chunk size of a device-resident call of n signatures over several streams
// (DESIGN.md section 4): round(n / 2^18) chunks, at least two, of equal size
// (a multiple of 64, above the lane-pair size), so a mid-size batch still has
// two chunks whose phase 1 and main kernels overlap and no small remainder
// chunk runs alone at the end; 1M signatures: four chunks of 2^18 (the
// measured best).  STL_TUNE_CHUNK_LOG2 15..20 fixes the size instead.
uint32_t pair_max_lanes(uint32_t grid);
uint32_t chunk_for(uint32_t grid, size_t n) {
  const int t = g_tune_sub_log2.load();
  if (t) return 1u << t;
  // up to two lane-pair chunks' worth: one chunk (its phase 1 runs as the
  // two-role launch), measured 0.63 against 0.89 ms split at 65,536; up to
  // three: 2 * pair_max and a lane-pair remainder (98,304: 1.01 vs 1.05 ms)
  const size_t pm = pair_max_lanes(grid);
  if (n <= 2 * pm) return (uint32_t)std::min<size_t>(std::max<size_t>(n, 64), stl::kPreChunk);
  if (n <= 3 * pm) return (uint32_t)(2 * pm);
  const size_t nc = std::max<size_t>(2, (n + ((size_t)1 << 17)) >> 18);
  size_t sub = ((n + nc - 1) / nc + 63) / 64 * 64;
  sub = std::max<size_t>(sub, pair_max_lanes(grid) + 64);
  return (uint32_t)std::min<size_t>(sub, stl::kPreChunk);
}

// The verify workspace of one stream: every launch that runs kernels on a
// stream uses that stream's workspace, in stream order -- the caller's streams
// (device-resident API) and the library's own pool streams alike, so a pool
// stream shared by several callers and both APIs needs only one.  `mu` is
// held while a launch is planned and enqueued (the workspace may grow), and
// every buffer below is only grown or read under it (the hash
// queue of a shared pool stream was grown outside it).  Caller streams'
// contexts are capped per device (kMaxCallerStreams, least recently used
// evicted) and stl_release_stream drops one: a context lives on in a
// shared_ptr until its last user returns, then hands its buffers to the
// device's spare list (CtxSpares) instead of freeing them.  Every use of a
// caller context ends by recording `done` on its stream (stream_ctx's use
// token), so a spare's buffers are free once `done` has completed: the next
// caller context adopts them and makes its stream wait for that event on the
// device -- no host wait, no hipFree (which would synchronise the whole
// device: VERDICT r5 #4).
struct StreamCtx;
struct CtxSpares {
  std::mutex mu;
  std::vector<std::unique_ptr<StreamCtx>> list;  // oldest first
};
std::atomic<int>& max_caller_streams();
struct StreamCtx {
  std::mutex mu;
  int ordinal = -1;        // device of the buffers below
  bool pool = false;       // a library pool stream's context (never evicted)
  uint64_t last_use = 0;   // LRU tick (Device::ws_mu)
  // caller contexts: completes after the last work enqueued with this
  // context's buffers (recorded on the caller's stream after every use)
  hipEvent_t done = nullptr;
  std::weak_ptr<CtxSpares> spares;  // where the buffers go when the context dies
  DevBuf ws;
  // work counter + longest-first order of the device-resident hash kernels
  // (stl::hash_queue_bytes(n)) of the launches on this stream
  DevBuf queue;
  // fork / join events of launches whose chunks this (caller) stream spreads
  // over pool streams
  hipEvent_t fork = nullptr;
  hipEvent_t join[stl::kMaxVerifyStreams] = {};
  // a launch's shared key domain is built (stl::VerifyExec::key_ready); the
  // one-call blob path's two parse kernels are done (the keys are out)
  hipEvent_t keys = nullptr;
  hipEvent_t parsed[2] = {};
  // R decoded ahead for the one-call checkSign's shared key domain
  // (stl::VerifyExec::rdec: 80 B per row) and its ready event
  DevBuf rdec;
  hipEvent_t rready = nullptr;
  // device-resident automatic dedup: host-mapped word the key sample kernel
  // writes after each call on this stream (1 = its keys repeated); the next
  // call reads it without waiting (feedback, so a stale value only picks the
  // other path -- the bits are the same)
  uint32_t* auto_flag = nullptr;
  uint32_t* auto_flag_dev = nullptr;
  // the device-resident checkSign calls' verify inputs (signing hashes, and
  // from blobs the signatures and keys), 32 or 128 B per row
  DevBuf scratch;
  void release() {
    if (auto_flag) (void)hipHostFree(auto_flag);
    auto_flag = auto_flag_dev = nullptr;
    scratch.release();
    ws.release();
    queue.release();
    for (hipEvent_t& e : join) {
      if (e) (void)hipEventDestroy(e);
      e = nullptr;
    }
    if (fork) (void)hipEventDestroy(fork);
    fork = nullptr;
    if (keys) (void)hipEventDestroy(keys);
    keys = nullptr;
    for (hipEvent_t& e : parsed) {
      if (e) (void)hipEventDestroy(e);
      e = nullptr;
    }
    rdec.release();
    if (rready) (void)hipEventDestroy(rready);
    rready = nullptr;
    if (done) (void)hipEventDestroy(done);
    done = nullptr;
  }
  bool holds_memory() const {
    return auto_flag || scratch.p || ws.p || queue.p || fork || keys || parsed[0] || parsed[1] || rdec.p || rready ||
           done;
  }
  // moves every buffer and event of `o` into this (empty) context
  void adopt(StreamCtx& o) {
    std::swap(ws, o.ws);
    std::swap(queue, o.queue);
    std::swap(scratch, o.scratch);
    std::swap(fork, o.fork);
    std::swap(keys, o.keys);
    std::swap(parsed[0], o.parsed[0]);
    std::swap(parsed[1], o.parsed[1]);
    std::swap(rdec, o.rdec);
    std::swap(rready, o.rready);
    for (uint32_t j = 0; j < stl::kMaxVerifyStreams; ++j) std::swap(join[j], o.join[j]);
    std::swap(auto_flag, o.auto_flag);
    std::swap(auto_flag_dev, o.auto_flag_dev);
    std::swap(done, o.done);
  }
  ~StreamCtx() {
    if (!holds_memory() || ordinal < 0) return;
    // an evicted or released caller context: its buffers go to the device's
    // spares, to be adopted behind `done` (see above), while the list holds
    // fewer than the caller-stream cap
    if (done) {
      if (std::shared_ptr<CtxSpares> sp = spares.lock()) {
        auto z = std::make_unique<StreamCtx>();
        z->ordinal = ordinal;
        z->adopt(*this);
        std::unique_ptr<StreamCtx> over;
        {
          std::lock_guard<std::mutex> lk(sp->mu);
          sp->list.push_back(std::move(z));
          if (sp->list.size() > (size_t)max_caller_streams().load()) {
            over = std::move(sp->list.front());
            sp->list.erase(sp->list.begin());
          }
        }
        return;  // `over` (a spare beyond the cap: no spares link) is freed below
      }
    }
    // no spare list (library shut down, or no `done` event): the buffers'
    // kernels (and the key sample's write to auto_flag) may still be in
    // flight on a stream the caller may have destroyed since, so wait for the
    // whole device before freeing
    int prev = -1;
    (void)hipGetDevice(&prev);
    if (hipSetDevice(ordinal) == hipSuccess) (void)hipDeviceSynchronize();
    release();
    if (prev >= 0) (void)hipSetDevice(prev);
  }
};

// A spare whose last work has completed if there is one, else the oldest
// (its adopter's stream waits for it on the device); nullptr if none.
std::unique_ptr<StreamCtx> take_spare(CtxSpares& sp) {
  std::lock_guard<std::mutex> lk(sp.mu);
  if (sp.list.empty()) return nullptr;
  size_t pick = 0;
  for (size_t i = 0; i < sp.list.size(); ++i)
    if (sp.list[i]->done && hipEventQuery(sp.list[i]->done) == hipSuccess) {
      pick = i;
      break;
    }
  std::unique_ptr<StreamCtx> z = std::move(sp.list[pick]);
  sp.list.erase(sp.list.begin() + (long)pick);
  return z;
}

// Streams ("stream pool"): HIP maps the streams of a
// process onto GPU_MAX_HW_QUEUES (4 on the pool) hardware queues in creation
// order, and two streams on one queue run one after another.  So libstl makes
// exactly three streams per device, in stl_init, in a fixed order -- two
// kernel streams and one copy stream -- and both APIs share them: the host
// batch API runs even / odd chunks on `stream` / `stream2` and copies on
// `copy`; a device-resident call runs its chunks on the caller's stream plus
// `stream2` (then `stream`).  Made before the caller's later streams, they
// keep their own queues whatever the caller creates afterwards.
struct Device {
  int ordinal = 0;
  int cus = 0;
  uint32_t grid = 0;  // resident workgroups for the verify kernel
  hipStream_t stream = nullptr;   // kernel stream 0: host batch API even chunks and results
  hipStream_t stream2 = nullptr;  // kernel stream 1: host API odd chunks; a device call's second stream
  hipStream_t copy = nullptr;     // host-to-device copies (overlap the previous chunk's kernels)
  // a device call's fourth stream (STL_TUNE_STREAMS 4 only; made on use under
  // ws_mu, read without a lock by drain / run_verify -- ADVICE r4)
  std::atomic<hipStream_t> stream3{nullptr};
  ncclComm_t comm = nullptr;      // in-process communicator (rank = device index)
  std::mutex mu;
  DevBuf sig, msg, pk, bitmap, pre, off, len, ctr, ctr2, txid, status, wide, gather;
  DevBuf counters;  // device u64 counters of stl_get_stats: [0] accepted, [1] full-length lanes
  // workspace of every stream used: the pool streams' for good, at most
  // kMaxCallerStreams caller streams' (LRU)
  std::map<hipStream_t, std::shared_ptr<StreamCtx>> stream_ws;
  // buffers of evicted / released caller contexts, adopted by the next ones
  std::shared_ptr<CtxSpares> spares = std::make_shared<CtxSpares>();
  uint64_t ws_tick = 0;
  std::mutex ws_mu;
  void* stage = nullptr;  // pinned host staging of small host batches (run_small), under mu
  size_t stage_cap = 0;
  PhaseTimer timer;
  stl::PhaseClock clock{phase_mark, &timer};
};

// the device's phase clock when timing is on, else none
const stl::PhaseClock* phase_clock(Device& d) { return g_phase_timing.load() ? &d.clock : nullptr; }

std::mutex g_mu;
std::vector<std::unique_ptr<Device>> g_devs;
bool g_init = false;
int g_shards_per_device = 1;
bool g_comm_gather = false;  // host batches gather their bitmap over RCCL
// the caller's own check for stl_ed25519_verify_detached's device failures
std::atomic<stl_verify_fn> g_fallback_verify{nullptr};

// one process per GPU (stl_comm_*)
std::mutex g_pcomm_mu;
ncclComm_t g_pcomm = nullptr;
int g_pcomm_ranks = 0;
// the last gather's start: recorded on its stream just before the collective
// is enqueued, so stl_comm_sync's deadline covers the gather only, not the
// verify work queued ahead of it on that stream
hipEvent_t g_gather_start = nullptr;
hipStream_t g_gather_stream = nullptr;

// Aborts the communicator (its kernels end, so the streams drain) and forgets
// it: a failed or stalled collective leaves it unusable.  Holds g_pcomm_mu.
void pcomm_abort_locked() {
  if (g_pcomm && g_rccl.ok) (void)(g_rccl.CommAbort ? g_rccl.CommAbort(g_pcomm) : g_rccl.CommDestroy(g_pcomm));
  g_pcomm = nullptr;
  g_pcomm_ranks = 0;
}

// Marks the start of a gather on stream s (holds g_pcomm_mu); a timing
// helper, so it never fails the gather.
void mark_gather_start(hipStream_t s) {
  if (!g_gather_start && hipEventCreateWithFlags(&g_gather_start, hipEventDisableTiming) != hipSuccess) {
    g_gather_start = nullptr;
    g_gather_stream = nullptr;
    return;
  }
  g_gather_stream = hipEventRecord(g_gather_start, s) == hipSuccess ? s : nullptr;
}

unsigned long long* dev_counters(Device& d) { return static_cast<unsigned long long*>(d.counters.p); }

// ---- host-side statistics (stl_get_stats) and tracing (STL_TRACE=1) ----
std::atomic<uint64_t> g_st_batches{0}, g_st_sigs{0}, g_st_errors{0}, g_st_host_ns{0}, g_st_gather_ns{0},
    g_st_auto_dedup{0};
bool g_trace = false;

uint64_t now_ns() {
  return (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(
             std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

// Counts one host entry-point call: signatures, wall time, errors; with
// STL_TRACE=1 one JSON line per call on stderr (host spans; the kernels are
// rocprofv3's).
struct CallSpan {
  const char* name;
  size_t n;
  uint64_t t0 = now_ns();
  int finish(int rc, uint64_t gather_ns = 0) {
    const uint64_t dt = now_ns() - t0;
    g_st_batches++;
    g_st_sigs += n;
    g_st_host_ns += dt;
    g_st_gather_ns += gather_ns;
    if (rc < 0) g_st_errors++;
    if (g_trace)
      std::fprintf(stderr, "{\"stl_trace\": \"%s\", \"n\": %zu, \"rc\": %d, \"ms\": %.3f, \"gather_ms\": %.3f}\n", name, n,
                   rc, dt * 1e-6, gather_ns * 1e-6);
    return rc;
  }
};

// Restores the calling thread's current HIP device on scope exit: the host
// entry points switch devices internally, and a library call must not leave
// the caller (stellard, or a PyTorch user of the device API) on another one.
struct DeviceGuard {
  int prev = -1;
  DeviceGuard() {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
  }
  ~DeviceGuard() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
};

int current_device_index() {
  int ord = -1;
  if (hipGetDevice(&ord) != hipSuccess) return -1;
  for (size_t i = 0; i < g_devs.size(); ++i)
    if (g_devs[i]->ordinal == ord) return (int)i;
  return -1;
}

int setup_device(Device& d) {
  STL_TRY(hipSetDevice(d.ordinal));
  hipDeviceProp_t prop;
  STL_TRY(hipGetDeviceProperties(&prop, d.ordinal));
  if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0) return STL_ENODEV;
  d.cus = prop.multiProcessorCount;
  int per_cu = 0;
  STL_TRY(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, stl::kernel_verify_msg32(), stl::kBlock, 0));
  if (per_cu < 1) per_cu = 1;
  d.grid = (uint32_t)(d.cus * per_cu);
  g_shard_quantum.store((uint64_t)d.grid * stl::kBlock / 2);  // one verify wave per SIMD
  // the stream pool, in this order (see Device)
  STL_TRY(hipStreamCreateWithFlags(&d.stream, hipStreamNonBlocking));
  STL_TRY(hipStreamCreateWithFlags(&d.stream2, hipStreamNonBlocking));
  STL_TRY(hipStreamCreateWithFlags(&d.copy, hipStreamNonBlocking));
  STL_RC(d.counters.ensure(64));
  STL_TRY(hipMemsetAsync(d.counters.p, 0, 64, d.stream));
  // wide base tables for [e]B (7.3 MB), built once on the device
  STL_RC(d.wide.ensure(stl::kWideTableBytes));
  STL_TRY(stl::launch_wide_table(static_cast<uint4*>(d.wide.p), d.stream));
  STL_TRY(hipStreamSynchronize(d.stream));
  return STL_OK;
}

void release_device(Device& d) {
  (void)hipSetDevice(d.ordinal);
  const hipStream_t s3 = d.stream3.load();
  for (hipStream_t s : {d.stream, d.stream2, s3, d.copy})
    if (s) (void)hipStreamSynchronize(s);
  (void)hipDeviceSynchronize();  // caller streams' work on the workspaces freed below
  if (d.comm && g_rccl.ok) (void)g_rccl.CommDestroy(d.comm);
  d.comm = nullptr;
  for (DevBuf* b : {&d.sig, &d.msg, &d.pk, &d.bitmap, &d.pre, &d.off, &d.len, &d.ctr, &d.ctr2, &d.txid, &d.status,
                    &d.wide, &d.gather, &d.counters})
    b->release();
  {
    std::lock_guard<std::mutex> lk(d.ws_mu);
    for (auto& kv : d.stream_ws) {
      std::lock_guard<std::mutex> cl(kv.second->mu);
      kv.second->release();
    }
    d.stream_ws.clear();
    // the spares (the device is idle); a context a caller still holds now
    // finds no spare list and frees its own buffers
    if (std::shared_ptr<CtxSpares> sp = std::move(d.spares)) {
      std::lock_guard<std::mutex> sl(sp->mu);
      for (auto& z : sp->list) z->release();
      sp->list.clear();
    }
  }
  if (d.stage) (void)hipHostFree(d.stage);
  d.stage = nullptr;
  d.stage_cap = 0;
  d.timer.release();
  for (hipStream_t s : {d.stream, d.stream2, s3, d.copy})
    if (s) (void)hipStreamDestroy(s);
  d.stream = d.stream2 = d.copy = nullptr;
  d.stream3.store(nullptr);
}

int ensure_init() {
  {
    std::lock_guard<std::mutex> lk(g_mu);
    if (g_init) return STL_OK;
  }
  return stl_init(nullptr);
}

// Caller streams whose contexts a device keeps: each holds a
// verify workspace (stl::verify_ws_bytes: ~0.44 GB, ~0.7 GB with key dedup),
// so a caller cycling through many streams must not grow device memory
// without bound.  STL_MAX_STREAM_WORKSPACES overrides (1..64) at stl_init.
// Default 8: stellard's JobQueue auto-tunes to min(CPUs, 4) + 2 = up to 6
// workers (JobQueue.cpp:217-243), so one stream per worker stays resident
// with room to spare -- 8 contexts hold <= 5.6 GB of the 288 GB.
constexpr int kDefaultCallerStreams = 8;
std::atomic<int> g_max_caller_streams{kDefaultCallerStreams};
std::atomic<int>& max_caller_streams() { return g_max_caller_streams; }

bool is_pool_stream(const Device& d, hipStream_t s) {
  return s && (s == d.stream || s == d.stream2 || s == d.copy || s == d.stream3.load());
}

// One use of a caller stream's context: when the caller's last copy of the
// pointer stream_ctx returned goes (after its kernels are enqueued and its
// locks released), `done` is recorded on the stream, so it completes after
// every kernel that used the context's buffers.
struct CtxUse {
  std::shared_ptr<StreamCtx> c;
  hipStream_t s = nullptr;
  ~CtxUse() {
    if (!c || c->pool || !c->done) return;
    std::lock_guard<std::mutex> lk(c->mu);
    (void)hipEventRecord(c->done, s);
  }
};

// The context of stream s on device d (created on first use).  Creating a
// caller stream's context beyond the cap evicts the least recently used
// caller context; the evicted one hands its buffers to d.spares outside
// ws_mu, once its last user has let go, and a new caller context adopts a
// spare's buffers with its stream waiting for the spare's `done` event.
std::shared_ptr<StreamCtx> stream_ctx(Device& d, hipStream_t s) {
  std::vector<std::shared_ptr<StreamCtx>> evicted;
  std::shared_ptr<StreamCtx> out;
  {
    std::lock_guard<std::mutex> lk(d.ws_mu);
    auto& slot = d.stream_ws[s];
    if (!slot) {
      slot = std::make_shared<StreamCtx>();
      slot->ordinal = d.ordinal;
      slot->pool = is_pool_stream(d, s);
      if (!slot->pool) {
        // the least recently used caller contexts beyond the cap (the cap
        // may have been lowered since they were made)
        std::vector<std::pair<uint64_t, hipStream_t>> callers;
        for (auto& kv : d.stream_ws)
          if (!kv.second->pool && kv.first != s) callers.emplace_back(kv.second->last_use, kv.first);
        std::sort(callers.begin(), callers.end());
        const size_t keep = (size_t)std::max(0, g_max_caller_streams.load() - 1);  // plus s
        for (size_t i = 0; i + keep < callers.size(); ++i) {
          auto it = d.stream_ws.find(callers[i].second);
          evicted.push_back(std::move(it->second));
          d.stream_ws.erase(it);
        }
      }
      if (!slot->pool && d.spares) {
        slot->spares = d.spares;
        // buffers for the new context: an evicted context no call holds any
        // more (out of the map, so no new holder can appear), else a spare
        StreamCtx* src = nullptr;
        for (auto& e : evicted)
          if (!src && e.use_count() == 1 && e->done) src = e.get();
        std::unique_ptr<StreamCtx> z;
        if (!src && (z = take_spare(*d.spares))) src = z.get();
        if (src) {
          slot->adopt(*src);
          // its last kernels may still run on its (old) stream: order this
          // stream's work behind them on the device
          if (slot->done && hipStreamWaitEvent(s, slot->done, 0) != hipSuccess) (void)hipEventSynchronize(slot->done);
        }
        if (!slot->done && hipEventCreateWithFlags(&slot->done, hipEventDisableTiming) != hipSuccess)
          slot->done = nullptr;  // then this context frees its buffers after a device sync
      }
    }
    out = d.stream_ws[s];
    out->last_use = ++d.ws_tick;
  }
  if (out->pool) return out;  // evicted contexts are released here, without ws_mu
  auto use = std::make_shared<CtxUse>();
  use->c = out;
  use->s = s;
  return std::shared_ptr<StreamCtx>(use, use->c.get());
}

// Caller contexts currently kept on device d (tests: the cap holds).
int caller_contexts(Device& d) {
  std::lock_guard<std::mutex> lk(d.ws_mu);
  int k = 0;
  for (auto& kv : d.stream_ws) k += kv.second->pool ? 0 : 1;
  return k;
}

// Per-lane workspace slots (workgroups) for launch_verify: room for two lanes
// per signature when the batch is small enough to run that way.
uint32_t verify_grid_for(const Device& d, size_t n) {
  const size_t tiles = (n + stl::kBlock - 1) / stl::kBlock;
  return (uint32_t)std::max<size_t>(1, std::min<size_t>(2 * tiles, d.grid));
}

// Largest chunk launch_verify runs on two lanes per signature: one pair wave
// per SIMD at most (a quarter of the resident lanes).
uint32_t pair_max_lanes(uint32_t grid) { return grid * stl::kBlock / 4; }
uint32_t pair_max(const Device& d) { return pair_max_lanes(d.grid); }
// Largest chunks whose main kernel runs on eight (quad_max) or four (duo_max)
// lanes per signature: one such wave per SIMD at most (a second one per SIMD
// measured slower than lane pairs; STL_TUNE_QUAD bits 0 / 1 turn them on).
uint32_t quad_max(const Device& d) { return (g_tune_quad.load() & 1) ? d.grid * stl::kBlock / 16 : 0u; }
uint32_t duo_max(const Device& d) { return (g_tune_quad.load() & 2) ? d.grid * stl::kBlock / 8 : 0u; }

unsigned long long* dev_counters(Device& d);
const stl::PhaseClock* phase_clock(Device& d);

// A pool kernel stream that a call running on streams[0..S) does not use:
// the shared key domain is built there, beside the chunks' scalar kernels
// (stl::VerifyExec::key_stream); nullptr when every one is taken.
hipStream_t key_stream_for(const Device& d, const hipStream_t* used, uint32_t S) {
  for (hipStream_t c : {d.stream, d.stream2}) {
    bool taken = c == nullptr;
    for (uint32_t j = 0; j < S; ++j) taken = taken || used[j] == c;
    if (!taken) return c;
  }
  return nullptr;
}

// Plans and enqueues one launch_verify of n signatures on stream s: with
// `streams` > 1 (device-resident API only: the host batch API already overlaps
// its copies with the previous chunk's kernels) chunks also go to the pool
// streams stream2, stream, stream3 (the caller's own stream excluded), forked
// from and joined to s by s's events.  Every stream involved contributes its
// workspace; their mutexes are held (in address order) until the launch is
// enqueued.  On an error the pool streams used are drained before returning
// (nothing may still run on the caller's buffers outside the caller's stream).
int run_verify(Device& d, hipStream_t s, const uint8_t* sig, const uint8_t* msg_or_k, const uint8_t* pk, size_t n,
               uint64_t* words, uint32_t mode, bool pre_k, int streams, bool concurrent = false) {
  const bool dedup = (mode & stl::kModeDedupKeys) != 0;
  stl::VerifyExec x;
  x.grid = verify_grid_for(d, n);
  x.ws_grid = d.grid;  // every workspace is verify_ws_bytes(d.grid, ...)
  x.pair_max = pair_max(d);
  x.quad_max = quad_max(d);
  x.duo_max = duo_max(d);
  x.wide = static_cast<const uint4*>(d.wide.p);
  x.counters = dev_counters(d);
  x.clock = phase_clock(d);
  x.fused_prep = g_tune_fused.load();
  x.main_queue = g_tune_queue.load() != 0;
  x.concurrent = concurrent;
  x.sub = chunk_for(d.grid, n);
  x.first = (uint32_t)g_tune_first_chunk.load();
  uint32_t S = (uint32_t)std::max(1, std::min<int>(streams, (int)stl::kMaxVerifyStreams));
  if (x.clock || n <= x.sub || x.sub <= x.pair_max) S = 1;
  S = (uint32_t)std::min<size_t>(S, (n + x.sub - 1) / x.sub);
  hipStream_t pool[stl::kMaxVerifyStreams] = {s};
  uint32_t np = 1;
  if (S > 1) {
    if (S > 3 && !d.stream3.load()) {
      std::lock_guard<std::mutex> lk(d.ws_mu);
      if (!d.stream3.load()) {
        hipStream_t s3 = nullptr;
        STL_TRY(hipStreamCreateWithFlags(&s3, hipStreamNonBlocking));
        d.stream3.store(s3);
      }
    }
    for (hipStream_t p : {d.stream2, d.stream, d.stream3.load()})
      if (np < S && p && p != s) pool[np++] = p;
  }
  S = np;
  x.nstreams = S;
  std::shared_ptr<StreamCtx> hold[stl::kMaxVerifyStreams];
  StreamCtx* ctx[stl::kMaxVerifyStreams];
  for (uint32_t j = 0; j < S; ++j) {
    hold[j] = stream_ctx(d, pool[j]);
    ctx[j] = hold[j].get();
  }
  StreamCtx* order[stl::kMaxVerifyStreams];
  std::copy(ctx, ctx + S, order);
  std::sort(order, order + S);
  std::vector<std::unique_lock<std::mutex>> locks;
  for (uint32_t j = 0; j < S; ++j) locks.emplace_back(order[j]->mu);
  StreamCtx& c = *ctx[0];
  for (uint32_t j = 0; j < S; ++j) {
    STL_RC(ctx[j]->ws.ensure(stl::verify_ws_bytes(d.grid, dedup)));
    x.ws[j] = static_cast<uint4*>(ctx[j]->ws.p);
    x.streams[j] = pool[j];
    if (j > 0) {
      if (!c.join[j]) STL_TRY(hipEventCreateWithFlags(&c.join[j], hipEventDisableTiming));
      x.join[j] = c.join[j];
    }
  }
  if (S > 1 && !c.fork) STL_TRY(hipEventCreateWithFlags(&c.fork, hipEventDisableTiming));
  x.fork = c.fork;
  x.wide_min = (uint32_t)g_tune_wide_min.load();
  if (S > 1 && dedup && g_tune_shared_keys.load()) {  // the chunks share one key domain in the caller's workspace
    if (!c.keys) STL_TRY(hipEventCreateWithFlags(&c.keys, hipEventDisableTiming));
    x.key_ready = c.keys;
    x.key_stream = key_stream_for(d, pool, S);  // built beside the scalar kernels when a pool stream is idle
  }
  if (fault_now() || stl::launch_verify(sig, msg_or_k, pk, (uint32_t)n, words, mode, pre_k, x) != hipSuccess) {
    for (uint32_t j = 1; j < S; ++j) (void)hipStreamSynchronize(pool[j]);
    if (x.key_stream) (void)hipStreamSynchronize(x.key_stream);
    return STL_EHIP;
  }
  return STL_OK;
}

// Hash work queue of stream context c for n rows (counter + longest-first
// order, stl::hash_queue_bytes(n)).  Caller holds c.mu until the hash kernel
// using it is enqueued (a concurrent grow would free it first -- ADVICE r4).
int ctx_queue(StreamCtx& c, size_t n, uint32_t** qws, bool blob = false) {
  STL_RC(c.queue.ensure(blob ? stl::blob_queue_bytes(n) : stl::hash_queue_bytes(n)));
  *qws = static_cast<uint32_t*>(c.queue.p);
  return STL_OK;
}

// tx-hash grid: 8 workgroups per CU (the kernel pulls preimages from a counter)
uint32_t hash_grid(const Device& d) { return (uint32_t)d.cus * 8u; }

// The hash kernel's long mode for a call of n preimages (DESIGN.md section 4,
// small batches): on for calls of at most two lane-pair chunks -- latency-
// bound, the chip mostly idle, the longest row's chain the hash's length --
// off for throughput batches, where a wave per row would waste 63 lanes.
uint32_t hash_long_min(const Device& d, size_t n) {
  return n <= 2 * (size_t)pair_max(d) ? (uint32_t)g_tune_long_hash.load() : 0u;
}

uint32_t grid_for(const Device& d, size_t n) {
  const size_t tiles = (n + stl::kBlock - 1) / stl::kBlock;
  return (uint32_t)std::max<size_t>(1, std::min<size_t>(tiles, d.grid));
}

// Contiguous 64-aligned shard of [0, n) for shard r of g (stl_shard_range).
void shard(size_t n, int r, int g, size_t* lo, size_t* hi) {
  const size_t words = (n + 63) / 64;
  const size_t per = (words + g - 1) / g;
  *lo = std::min(n, (size_t)r * per * 64);
  *hi = std::min(n, (size_t)(r + 1) * per * 64);
}


// Byte-balanced 64-aligned shard boundaries: bound[r] = the 64-aligned row at
// or after the first row whose byte prefix sum reaches r/g of the total --
// then moved to the nearest multiple of g_shard_quantum rows when that moves
// its byte prefix by at most 2.5 % of one rank's share (config
// 5's 2^20-row ledger over 8 ranks byte-balances to 130,304-131,584 rows, and
// the ranks past 131,072 paid a sliver of a second round: max / mean rank time
// 1.03-1.11; equal rows cost a rank at most ~0.6 % of its bytes, i.e. of the
// fifth of its time that is hashing).  tests/test_multigpu_host.py holds the
// Python mirror to it.
void shard_bytes_bounds(const uint32_t* len, size_t n, int g, std::vector<size_t>& bound) {
  bound.assign(g + 1, n);
  bound[0] = 0;
  uint64_t total = 0;
  for (size_t i = 0; i < n; ++i) total += len[i];
  const uint64_t q = g_shard_quantum.load();
  uint64_t acc = 0;
  size_t i = 0;
  for (int r = 1; r < g; ++r) {
    const uint64_t target = (uint64_t)((__uint128_t)total * (unsigned)r / (unsigned)g);
    while (i < n && acc < target) acc += len[i++];
    size_t b = std::min(n, (i + 63) / 64 * 64);
    if (q >= 64 && q % 64 == 0 && n > q) {
      // the byte prefix at row b (acc is the prefix at row i <= b)
      auto prefix = [&](size_t row) {
        uint64_t p = acc;
        if (row >= i)
          for (size_t k = i; k < row; ++k) p += len[k];
        else
          for (size_t k = row; k < i; ++k) p -= len[k];
        return p;
      };
      const size_t down = b / q * q, up = down + q;
      const size_t c = (b - down <= up - b || up > n) ? down : up;
      const uint64_t pc = prefix(c);
      const uint64_t dev = pc > target ? pc - target : target - pc;
      if (c > 0 && c < n && (__uint128_t)dev * (unsigned)g * 40u <= (__uint128_t)total) b = c;
    }
    bound[r] = std::max(bound[r - 1], b);
  }
}

// ---- host batch API ---------------------------------------------------------
// A shard is processed in chunks of kPipeChunk signatures (a multiple of 64,
// so every chunk starts on a bitmap word).  Chunk c's inputs are copied on
// d.copy while chunk c-1's kernels run on d.stream; an event orders each
// chunk's kernels after its copy.  Device buffers hold the whole shard, so no
// buffer is reused while a kernel may still read it.  Variable-length bytes
// (preimages, blobs) are copied up to a watermark: chunk c copies
// [watermark, max end of its rows), rebased on the shard's lowest offset, so
// any offset order is correct.
#ifndef STL_PIPE_CHUNK_LOG2
#define STL_PIPE_CHUNK_LOG2 16  // 64K: two chunks' kernels share the chip (two streams); A/B in DESIGN.md section 8
#endif
constexpr size_t kPipeChunk = (size_t)1 << STL_PIPE_CHUNK_LOG2;

enum class Mode { kSig, kPre, kBlob };

struct Batch {
  Mode mode;
  const uint8_t *sig, *msg32, *pk, *bytes;  // bytes: preimages or blobs
  const uint64_t* off;
  const uint32_t* len;
  uint8_t *bitmap, *status, *txid;
  uint32_t policy, kind;
  bool auto_dedup;  // choose STL_DEDUP_KEYS per chunk from a key sample (keys_repeat)
};

// The signing key of host row i, for the automatic dedup choice only: the
// pk array, or in a serialized object the 32 bytes after the first
// SigningPubKey header (0x73, VL length 0x20) -- a wrong guess only picks the
// slower path, never other bits.
const uint8_t* row_key(const Batch& b, size_t i) {
  if (b.mode != Mode::kBlob) return b.pk + 32 * i;
  const uint8_t* p = b.bytes + b.off[i];
  const size_t len = b.len[i], lim = len < 34 ? 0 : std::min<size_t>(len - 34, 256);
  for (size_t j = 0; j + 1 <= lim; ++j)
    if (p[j] == 0x73 && p[j + 1] == 0x20) return p + j + 2;
  return nullptr;
}

// Host-side estimate of key repetition over rows [lo, hi) (a
// ledger's signers repeat -- 1,000 accounts for 100k transactions): up to
// 1,024 evenly spaced keys, 64-bit fingerprints in an open-addressing table;
// true when at least a fifth of the sampled keys repeat an earlier one (e.g.
// up to about 2,000 signers per 64K rows), where decoding each key once pays
// (key dedup).  About 40 us per 64K-row chunk from cold
// host memory, overlapped with the previous chunks' kernels.
bool keys_repeat(const Batch& b, size_t lo, size_t hi) {
  constexpr size_t kSample = 1024, kSlots = 2048;
  const size_t n = hi - lo;
  if (n < 4 * 64) return false;
  const size_t s = std::min(n, kSample);
  uint64_t table[kSlots] = {};
  size_t dups = 0;
  for (size_t k = 0; k < s; ++k) {
    const uint8_t* key = row_key(b, lo + k * n / s);
    if (!key) continue;
    uint64_t a, c;
    std::memcpy(&a, key, 8);
    std::memcpy(&c, key + 24, 8);
    uint64_t f = (a ^ (c * 0x9E3779B97F4A7C15ull)) | 1u;  // 0 marks an empty slot
    size_t h = (size_t)((f * 0xD6E8FEB86659FD93ull) >> 52) & (kSlots - 1);
    while (table[h] && table[h] != f) h = (h + 1) & (kSlots - 1);
    if (table[h] == f) ++dups;
    table[h] = f;
  }
  return 5 * dups >= s;
}

// The kernel mode of host rows [lo, hi): the batch's, plus key dedup when the
// automatic choice is on and their keys repeat (counted in stl_stats).
uint32_t chunk_policy(const Batch& b, size_t lo, size_t hi) {
  if (!b.auto_dedup || !keys_repeat(b, lo, hi)) return b.policy;
  g_st_auto_dedup++;
  return b.policy | stl::kModeDedupKeys;
}

// Host-side state of one shard; lives until the batch has synchronised (the
// staging vectors are sources of asynchronous copies).
struct Shard {
  Device* d = nullptr;
  size_t lo = 0, hi = 0;
  std::vector<uint64_t> roff, row_end;
  std::vector<hipEvent_t> ev;
  int rc = STL_OK;
  ~Shard() {
    for (hipEvent_t e : ev) (void)hipEventDestroy(e);
  }
  // Make stream `to` wait for everything issued on `from` so far.
  int join(hipStream_t from, hipStream_t to) {
    hipEvent_t e;
    STL_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    ev.push_back(e);
    STL_TRY(hipEventRecord(e, from));
    STL_TRY(hipStreamWaitEvent(to, e, 0));
    return STL_OK;
  }
};

// Rebased offsets of rows [lo, hi) and the byte range they span.
void rebase(const uint64_t* off, const uint32_t* len, size_t lo, size_t hi, std::vector<uint64_t>& roff,
            std::vector<uint64_t>& row_end, uint64_t* base_out, uint64_t* bytes_out) {
  const size_t n = hi - lo;
  uint64_t base = off[lo], end = 0;
  for (size_t i = lo; i < hi; ++i) base = std::min(base, off[i]);
  roff.resize(n);
  row_end.resize(n);
  for (size_t i = 0; i < n; ++i) {
    roff[i] = off[lo + i] - base;
    row_end[i] = roff[i] + len[lo + i];
    end = std::max(end, row_end[i]);
  }
  *base_out = base;
  *bytes_out = end;
}

// Copy the bytes rows [c0, c1) need that are not on the device yet.
int copy_rows(Shard& s, uint8_t* dst, const uint8_t* src, size_t c0, size_t c1, uint64_t* watermark) {
  uint64_t need = *watermark;
  for (size_t i = c0; i < c1; ++i) need = std::max(need, s.row_end[i]);
  if (need > *watermark)
    STL_TRY(hipMemcpyAsync(dst + *watermark, src + *watermark, need - *watermark, hipMemcpyHostToDevice, s.d->copy));
  *watermark = need;
  return STL_OK;
}

// Enqueue shard [lo, hi) of the batch on its device: copies, kernels, and the
// device-to-host copies of status / ids.  The accept bitmap stays in
// d.bitmap (words [0, ceil(n/64))).  Caller holds d.mu and synchronises.
int enqueue_shard(const Batch& b, Shard& s, size_t words_alloc) {
  Device& d = *s.d;
  const size_t lo = s.lo, n = s.hi - s.lo;
  STL_TRY(hipSetDevice(d.ordinal));
  STL_RC(d.bitmap.ensure(std::max<size_t>(words_alloc, 1) * 8));
  if (n == 0) return STL_OK;
  STL_RC(d.sig.ensure(n * 64));
  STL_RC(d.msg.ensure(n * 32));
  STL_RC(d.pk.ensure(n * 32));
  uint64_t base = 0, bytes = 0, mark = 0;
  uint8_t* dsig = static_cast<uint8_t*>(d.sig.p);
  uint8_t* dmsg = static_cast<uint8_t*>(d.msg.p);
  uint8_t* dpk = static_cast<uint8_t*>(d.pk.p);
  uint8_t* dpre = nullptr;
  uint64_t* doff = nullptr;
  uint32_t* dlen = nullptr;
  if (b.mode != Mode::kSig) {
    rebase(b.off, b.len, lo, s.hi, s.roff, s.row_end, &base, &bytes);
    STL_RC(d.pre.ensure(bytes + 16));
    STL_RC(d.off.ensure(n * 8));
    STL_RC(d.len.ensure(n * 4));
    const size_t qn = std::min(n, kPipeChunk);
    const size_t qbytes = b.mode == Mode::kBlob ? stl::blob_queue_bytes(qn) : stl::hash_queue_bytes(qn);
    STL_RC(d.ctr.ensure(qbytes));
    if (b.mode == Mode::kBlob) {
      STL_RC(d.status.ensure(n));
      if (b.txid) STL_RC(d.txid.ensure(n * 32));
    }
    dpre = static_cast<uint8_t*>(d.pre.p);
    doff = static_cast<uint64_t*>(d.off.p);
    dlen = static_cast<uint32_t*>(d.len.p);
    STL_TRY(hipMemcpyAsync(doff, s.roff.data(), n * 8, hipMemcpyHostToDevice, d.copy));
    STL_TRY(hipMemcpyAsync(dlen, b.len + lo, n * 4, hipMemcpyHostToDevice, d.copy));
  }
  uint8_t* dtxid = (b.mode == Mode::kBlob && b.txid) ? static_cast<uint8_t*>(d.txid.p) : nullptr;
  uint8_t* dstatus = b.mode == Mode::kBlob ? static_cast<uint8_t*>(d.status.p) : nullptr;
  // Odd chunks' kernels go to d.stream2 (own verify workspace and hash work
  // counter), so a chunk's phase 1 runs beside the previous chunk's main
  // kernel, as the device-resident API's sub-chunks do.
  // One stream while the phase clock is on: its per-kernel times must not
  // overlap.
  const bool two = g_tune_streams.load() > 1 && n > kPipeChunk && !phase_clock(d);
  // automatic key dedup: each chunk's policy from a sample of its keys, taken
  // just before the chunk is enqueued (so the sampling overlaps the earlier
  // chunks' kernels); the dedup-sized workspaces are taken before the first
  // chunk, so no workspace grows while earlier chunks still run on it
  if (b.auto_dedup && n > kPipeChunk / 2)
    for (hipStream_t ks : {d.stream, d.stream2}) {
      const std::shared_ptr<StreamCtx> c = stream_ctx(d, ks);
      std::lock_guard<std::mutex> lk(c->mu);
      STL_RC(c->ws.ensure(stl::verify_ws_bytes(d.grid, true)));
    }
  if (two && b.mode != Mode::kSig) {
    const size_t qn = std::min(n, kPipeChunk);
    STL_RC(d.ctr2.ensure(b.mode == Mode::kBlob ? stl::blob_queue_bytes(qn) : stl::hash_queue_bytes(qn)));
  }
  for (size_t c0 = 0; c0 < n; c0 += kPipeChunk) {
    const size_t c1 = std::min(n, c0 + kPipeChunk), cn = c1 - c0;
    const bool odd = two && ((c0 / kPipeChunk) & 1);
    hipStream_t ks = odd ? d.stream2 : d.stream;
    uint32_t* kctr = static_cast<uint32_t*>((odd ? d.ctr2 : d.ctr).p);
    if (b.mode != Mode::kBlob) {
      STL_TRY(hipMemcpyAsync(dsig + 64 * c0, b.sig + 64 * (lo + c0), cn * 64, hipMemcpyHostToDevice, d.copy));
      STL_TRY(hipMemcpyAsync(dpk + 32 * c0, b.pk + 32 * (lo + c0), cn * 32, hipMemcpyHostToDevice, d.copy));
    }
    if (b.mode == Mode::kSig)
      STL_TRY(hipMemcpyAsync(dmsg + 32 * c0, b.msg32 + 32 * (lo + c0), cn * 32, hipMemcpyHostToDevice, d.copy));
    else
      STL_RC(copy_rows(s, dpre, b.bytes + base, c0, c1, &mark));
    STL_RC(s.join(d.copy, ks));
    if (b.mode == Mode::kPre)
      STL_TRY(stl::launch_tx_hash(dpre, doff + c0, dlen + c0, (uint32_t)cn, dmsg + 32 * c0, kctr, hash_grid(d), ks,
                                  hash_long_min(d, n)));
    else if (b.mode == Mode::kBlob)
      STL_TRY(stl::launch_tx_blob(dpre, doff + c0, dlen + c0, (uint32_t)cn, dmsg + 32 * c0, dsig + 64 * c0,
                                  dpk + 32 * c0, dtxid ? dtxid + 32 * c0 : nullptr, dstatus + c0, kctr,
                                  hash_grid(d), ks, b.kind));
    STL_RC(run_verify(d, ks, dsig + 64 * c0, dmsg + 32 * c0, dpk + 32 * c0, cn,
                      static_cast<uint64_t*>(d.bitmap.p) + c0 / 64, chunk_policy(b, lo + c0, lo + c1), false, 1,
                      two));
  }
  if (two) STL_RC(s.join(d.stream2, d.stream));  // results are read on d.stream
  if (dstatus && b.status) STL_TRY(hipMemcpyAsync(b.status + lo, dstatus, n, hipMemcpyDeviceToHost, d.stream));
  if (dtxid) STL_TRY(hipMemcpyAsync(b.txid + 32 * lo, dtxid, n * 32, hipMemcpyDeviceToHost, d.stream));
  return STL_OK;
}

// Wait for everything a shard enqueued, whatever happened (an error return
// must not leave copies that read or write the caller's buffers in flight).
int drain(Device& d) {
  (void)hipSetDevice(d.ordinal);
  const hipError_t a = hipStreamSynchronize(d.copy);
  const hipError_t b = hipStreamSynchronize(d.stream);
  const hipError_t c = hipStreamSynchronize(d.stream2);
  const hipStream_t s3 = d.stream3.load();
  const hipError_t e = s3 ? hipStreamSynchronize(s3) : hipSuccess;
  return (a == hipSuccess && b == hipSuccess && c == hipSuccess && e == hipSuccess) ? STL_OK : STL_EHIP;
}

// Per-device copy: the shard's bitmap words to the host bitmap bytes
// [lo/8, ceil(hi/8)).  lo is a multiple of 64, so the slice is byte aligned.
int finish_direct(const Batch& b, Shard& s, std::vector<uint8_t>& host_words) {
  const size_t n = s.hi - s.lo;
  if (n == 0) return STL_OK;
  host_words.resize((n + 63) / 64 * 8);
  STL_TRY(hipMemcpyAsync(host_words.data(), s.d->bitmap.p, host_words.size(), hipMemcpyDeviceToHost, s.d->stream));
  STL_TRY(hipStreamSynchronize(s.d->stream));
  std::memcpy(b.bitmap + s.lo / 8, host_words.data(), (n + 7) / 8);
  return STL_OK;
}

int run_shard_direct(const Batch& b, Shard& s) {
  std::lock_guard<std::mutex> lk(s.d->mu);
  int rc = enqueue_shard(b, s, (s.hi - s.lo + 63) / 64);
  std::vector<uint8_t> host_words;
  if (rc == STL_OK) rc = finish_direct(b, s, host_words);
  const int drc = drain(*s.d);
  return rc ? rc : drc;
}

// RCCL gather of every shard's words into device 0, then one copy to the host.
// Shards are one per device in device order; `equal` = index shards (every
// shard `per` words, ncclGather), else grouped send/recv at each shard's word
// offset.
int gather_to_host(const Batch& b, std::vector<Shard>& sh, size_t n, size_t per, bool equal) {
  const int g = (int)sh.size();
  Device& root = *sh[0].d;
  const size_t words = (n + 63) / 64;
  STL_TRY(hipSetDevice(root.ordinal));
  STL_RC(root.gather.ensure(std::max(words, per * (size_t)g) * 8));
  uint64_t* rbuf = static_cast<uint64_t*>(root.gather.p);
  // (an injected fault stops here, before the group: a group that some ranks
  // join and others do not would never complete)
  STL_RCCL_TRY(g_rccl.GroupStart());
  // every communicator's ops are posted even after a failed enqueue (the first
  // error is kept): a group that some ranks join and others do not could hang
  // in GroupEnd instead of returning
  int rc = STL_OK;
  for (int r = 0; r < g; ++r) {
    Device& d = *sh[r].d;
    const uint64_t* sbuf = static_cast<const uint64_t*>(d.bitmap.p);
    if (equal) {
      if (g_rccl.Gather(sbuf, rbuf, per, ncclUint64, 0, d.comm, d.stream) != ncclSuccess) rc = STL_ERCCL;
    } else {
      const size_t w = (sh[r].hi - sh[r].lo + 63) / 64;
      if (w == 0 || r == 0) continue;  // rank 0's own slice: a device copy below
      const bool sent = g_rccl.Send(sbuf, w, ncclUint64, 0, d.comm, d.stream) == ncclSuccess;
      const bool recv = g_rccl.Recv(rbuf + sh[r].lo / 64, w, ncclUint64, r, root.comm, root.stream) == ncclSuccess;
      if (!sent || !recv) rc = STL_ERCCL;
    }
  }
  if (g_rccl.GroupEnd() != ncclSuccess && rc == STL_OK) rc = STL_ERCCL;
  if (rc) return rc;
  STL_TRY(hipSetDevice(root.ordinal));
  if (!equal && sh[0].hi > sh[0].lo)
    STL_TRY(hipMemcpyAsync(rbuf, root.bitmap.p, (sh[0].hi - sh[0].lo + 63) / 64 * 8, hipMemcpyDeviceToDevice,
                           root.stream));
  std::vector<uint8_t> host_words(words * 8);
  STL_TRY(hipMemcpyAsync(host_words.data(), rbuf, words * 8, hipMemcpyDeviceToHost, root.stream));
  STL_TRY(hipStreamSynchronize(root.stream));
  std::memcpy(b.bitmap, host_words.data(), (n + 7) / 8);
  return STL_OK;
}

int check_flags(uint32_t flags) {
  return (flags & ~(STL_POLICY_MASK | STL_REQUIRE_S_LT_L | STL_FULL_LENGTH | STL_DEDUP_KEYS | STL_ONE_LANE |
                    STL_NO_AUTO_DEDUP | STL_DEBUG_RAW_PREDICATE))
             ? STL_EINVAL
             : STL_OK;
}

// Host batches choose key dedup per chunk unless the caller decided
// (STL_DEDUP_KEYS on, STL_NO_AUTO_DEDUP off) or the chunk runs on lane pairs.
bool auto_dedup(uint32_t flags) {
  return (flags & (STL_DEDUP_KEYS | STL_NO_AUTO_DEDUP | STL_FULL_LENGTH)) == 0;
}

// Small signature batches on one device (single calls of
// stl_ed25519_verify_detached, the request aggregator's batches): the rows
// are staged in pinned host memory and sent by ONE copy on the kernel stream
// -- no copy stream, no events, one synchronisation -- since at this size the
// call is latency, not bandwidth.
constexpr size_t kSmallBatch = 4096;

int run_small(const Batch& b, size_t n) {
  Device& d = *g_devs[0];
  std::lock_guard<std::mutex> lk(d.mu);
  STL_TRY(hipSetDevice(d.ordinal));
  const size_t bytes = n * 128, words = (n + 63) / 64;
  if (d.stage_cap < bytes + words * 8) {
    if (d.stage) (void)hipHostFree(d.stage);
    d.stage = nullptr;
    d.stage_cap = 0;
    const size_t cap = kSmallBatch * 128 + kSmallBatch / 8;
    if (fault_now() || hipHostMalloc(&d.stage, cap, hipHostMallocDefault) != hipSuccess) {
      d.stage = nullptr;
      return STL_ENOMEM;
    }
    d.stage_cap = cap;
  }
  STL_RC(d.sig.ensure(bytes));
  STL_RC(d.bitmap.ensure(words * 8));
  uint8_t* st = static_cast<uint8_t*>(d.stage);
  std::memcpy(st, b.sig, n * 64);
  std::memcpy(st + 64 * n, b.msg32, n * 32);
  std::memcpy(st + 96 * n, b.pk, n * 32);
  uint8_t* dev = static_cast<uint8_t*>(d.sig.p);
  auto go = [&]() -> int {
    STL_TRY(hipMemcpyAsync(dev, st, bytes, hipMemcpyHostToDevice, d.stream));
    STL_RC(run_verify(d, d.stream, dev, dev + 64 * n, dev + 96 * n, n, static_cast<uint64_t*>(d.bitmap.p),
                      chunk_policy(b, 0, n), false, 1));
    STL_TRY(hipMemcpyAsync(st + bytes, d.bitmap.p, words * 8, hipMemcpyDeviceToHost, d.stream));
    STL_TRY(hipStreamSynchronize(d.stream));
    return STL_OK;
  };
  const int rc = go();
  if (rc) {  // nothing may still read the staging buffer
    (void)hipStreamSynchronize(d.stream);
    return rc;
  }
  std::memcpy(b.bitmap, st + bytes, (n + 7) / 8);
  return STL_OK;
}

int run_batch(const Batch& b, size_t n, uint64_t* gather_ns) {
  if (n == 0) return STL_OK;
  STL_RC(ensure_init());
  DeviceGuard guard;  // the last shard and the gather run on this thread
  const int g = (int)g_devs.size();
  if (g == 0) return STL_ENODEV;
  if (b.mode == Mode::kSig && n <= kSmallBatch && g == 1 && g_shards_per_device == 1 && !g_comm_gather)
    return run_small(b, n);
  // one kernel launch handles up to 2^32-64 signatures per shard
  const size_t kMaxShard = (size_t)1 << 31;
  int gg = g * g_shards_per_device;
  while ((n + gg - 1) / gg > kMaxShard) gg += g;
  std::vector<size_t> bound;
  const bool by_bytes = b.mode != Mode::kSig && (gg > 1 || g_tune_byte_shards.load() != 0);
  if (by_bytes) shard_bytes_bounds(b.len, n, gg, bound);
  std::vector<Shard> sh(gg);
  for (int r = 0; r < gg; ++r) {
    sh[r].d = g_devs[r % g].get();
    if (by_bytes) {
      sh[r].lo = bound[r];
      sh[r].hi = bound[r + 1];
    } else {
      shard(n, r, gg, &sh[r].lo, &sh[r].hi);
    }
  }
  if (g_comm_gather && gg == g) {
    // RCCL path: every device's mutex for the whole batch (device order)
    std::vector<std::unique_lock<std::mutex>> locks;
    for (auto& d : g_devs) locks.emplace_back(d->mu);
    size_t per = 1;
    for (auto& s : sh) per = std::max(per, (s.hi - s.lo + 63) / 64);
    std::vector<std::thread> th;
    for (int r = 0; r < gg; ++r) {
      if (r + 1 == gg) sh[r].rc = enqueue_shard(b, sh[r], per);
      else th.emplace_back([&, r] { sh[r].rc = enqueue_shard(b, sh[r], per); });
    }
    for (auto& t : th) t.join();
    int rc = STL_OK;
    for (auto& s : sh) rc = rc ? rc : s.rc;
    if (rc == STL_OK) {
      const uint64_t g0 = now_ns();
      rc = gather_to_host(b, sh, n, per, !by_bytes);
      *gather_ns = now_ns() - g0;
    }
    for (auto& d : g_devs) {
      const int drc = drain(*d);
      rc = rc ? rc : drc;
    }
    return rc;
  }
  std::vector<std::thread> th;
  for (int r = 0; r < gg; ++r) {
    if (r + 1 == gg) sh[r].rc = run_shard_direct(b, sh[r]);
    else th.emplace_back([&, r] { sh[r].rc = run_shard_direct(b, sh[r]); });
  }
  for (auto& t : th) t.join();
  for (auto& s : sh)
    if (s.rc) return s.rc;
  return STL_OK;
}

int env_int(const char* name, int dflt) {
  const char* v = std::getenv(name);
  return (v && *v) ? std::atoi(v) : dflt;
}

}  // namespace

extern "C" {

int stl_init(const stl_config* cfg) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (!g_init) {
    const char* fa = std::getenv("STL_FAULT_AFTER");
    if (fa && *fa) g_fault_after.store(std::atoll(fa));
    g_trace = env_int("STL_TRACE", 0) != 0;
    if (env_int("STL_PHASE_TIMING", 0) != 0) g_phase_timing.store(true);
    // execution tuning from the environment (same ranges as stl_debug_tuning;
    // profiling runs use STL_STREAMS=1 so that kernels do not overlap)
    const int s = env_int("STL_STREAMS", 0), c = env_int("STL_CHUNK_LOG2", 0);
    if (s >= 1 && s <= (int)stl::kMaxVerifyStreams) g_tune_streams.store(s);
    const int to = env_int("STL_RCCL_TIMEOUT_S", 0);
    if (to > 0 && to <= 3600) g_rccl_timeout_ms.store(to * 1000);
    const int ws = env_int("STL_MAX_STREAM_WORKSPACES", 0);
    if (ws >= 1 && ws <= 64) g_max_caller_streams.store(ws);
    if (c >= 15 && c <= 20) g_tune_sub_log2.store(c);
  }
  int first = 0, want = -1, spd = 1;
  uint32_t cflags = 0;
  if (cfg) {  // argument checks first: they need no device
    const uint32_t abi1 = 4 * sizeof(uint32_t), abi2 = offsetof(stl_config, fallback_verify);
    const uint32_t sz = cfg->struct_size;
    if (sz != sizeof(stl_config) && sz != abi1 && sz != abi2) return STL_EINVAL;
    first = cfg->first_device;
    if (cfg->device_count > 0) want = cfg->device_count;
    cflags = cfg->flags;
    if ((cflags & ~(STL_CFG_RCCL_GATHER | STL_CFG_NO_RCCL)) ||
        (cflags & (STL_CFG_RCCL_GATHER | STL_CFG_NO_RCCL)) == (STL_CFG_RCCL_GATHER | STL_CFG_NO_RCCL) ||
        first < 0)
      return STL_EINVAL;
    if (sz >= abi2) {
      if (cfg->reserved != 0) return STL_EINVAL;
      if (cfg->shards_per_device > 0) spd = cfg->shards_per_device;
    }
    // registered before any device is probed (a host without a usable device
    // still answers single calls through it), and also when the library is
    // already running -- e.g. started implicitly by a first entry-point call
    // (ensure_init -> stl_init(NULL)) -- so that stl_ed25519_verify_detached
    // keeps its 0 / -1 contract
    if (sz == sizeof(stl_config)) g_fallback_verify.store(cfg->fallback_verify);
  }
  int count = 0;
  if (hipGetDeviceCount(&count) != hipSuccess || count <= 0) return g_init ? STL_OK : STL_ENODEV;
  if (want < 0) want = count;
  if (std::getenv("STL_DEVICES")) want = std::max(1, env_int("STL_DEVICES", want));
  spd = std::max(1, std::min(64, env_int("STL_SHARDS_PER_DEVICE", spd)));
  const int env_rccl = env_int("STL_RCCL", -1);
  if (env_rccl == 1) cflags = (cflags & ~STL_CFG_NO_RCCL) | STL_CFG_RCCL_GATHER;
  if (env_rccl == 0) cflags = (cflags & ~STL_CFG_RCCL_GATHER) | STL_CFG_NO_RCCL;
  if (first < 0 || first >= count) return STL_EINVAL;
  want = std::min(want, count - first);
  // The in-process RCCL gather is opt-in (STL_CFG_RCCL_GATHER / STL_RCCL=1):
  // every device copies its own slice to the host unless asked, until a
  // multi-GPU run has shown the gathered bitmaps equal.
  const bool gather = !(cflags & STL_CFG_NO_RCCL) && spd == 1 && (cflags & STL_CFG_RCCL_GATHER);
  if (g_init) {
    // idempotent for NULL or the live settings; a cfg asking for another
    // device set, gather mode or shard count is refused rather than silently
    // ignored (stl_shutdown first)
    if (!cfg) return STL_OK;
    const bool same = !g_devs.empty() && g_devs[0]->ordinal == first && (int)g_devs.size() == want &&
                      gather == g_comm_gather && spd == g_shards_per_device;
    return same ? STL_OK : STL_EINVAL;
  }
  int prev = 0;
  (void)hipGetDevice(&prev);
  auto fail = [&](int rc) {
    for (auto& d : g_devs) release_device(*d);
    g_devs.clear();
    (void)hipSetDevice(prev);
    return rc;
  };
  for (int i = 0; i < want; ++i) {
    std::unique_ptr<Device> d(new Device());
    d->ordinal = first + i;
    g_devs.push_back(std::move(d));
    const int rc = setup_device(*g_devs.back());
    if (rc) return fail(rc);
  }
  if (gather) {
    if (!g_rccl.load() || fault_now()) return fail(STL_ERCCL);
    std::vector<ncclComm_t> comms(want);
    std::vector<int> ords(want);
    for (int i = 0; i < want; ++i) ords[i] = g_devs[i]->ordinal;
    if (g_rccl.CommInitAll(comms.data(), want, ords.data()) != ncclSuccess) return fail(STL_ERCCL);
    for (int i = 0; i < want; ++i) g_devs[i]->comm = comms[i];
  }
  (void)hipSetDevice(prev);
  g_shards_per_device = spd;
  g_comm_gather = gather;
  g_init = true;
  return STL_OK;
}

void stl_shutdown(void) {
  stl_comm_destroy();
  DeviceGuard guard;
  std::lock_guard<std::mutex> lk(g_mu);
  for (auto& d : g_devs) {
    std::lock_guard<std::mutex> dl(d->mu);
    release_device(*d);
  }
  g_devs.clear();
  g_comm_gather = false;
  g_shards_per_device = 1;
  g_init = false;
}

int stl_device_count(void) {
  std::lock_guard<std::mutex> lk(g_mu);
  return (int)g_devs.size();
}

const char* stl_version(void) { return "stl 0.2.0 (gfx950, abi 2)"; }

const char* stl_strerror(int rc) {
  switch (rc) {
    case STL_OK: return "ok";
    case STL_EINVAL: return "invalid argument";
    case STL_ENODEV: return "no gfx950 device";
    case STL_ENOMEM: return "out of memory";
    case STL_EHIP: return "HIP runtime error";
    case STL_ERCCL: return "RCCL error";
    default: return "unknown error";
  }
}

void stl_debug_fault_after(long long calls) { g_fault_after.store(calls < 0 ? -1 : calls); }

int stl_debug_tuning(int key, int value) {
  if (value == -1) {  // query
    switch (key) {
      case STL_TUNE_FUSED_PREP: return g_tune_fused.load();
      case STL_TUNE_MAIN_QUEUE: return g_tune_queue.load();
      case STL_TUNE_STREAMS: return g_tune_streams.load();
      case STL_TUNE_CHUNK_LOG2: return g_tune_sub_log2.load();
      case STL_TUNE_BYTE_SHARDS: return g_tune_byte_shards.load();
      case STL_TUNE_QUAD: return g_tune_quad.load();
      case STL_TUNE_STREAM_WORKSPACES: return g_max_caller_streams.load();
      case STL_TUNE_RCCL_TIMEOUT_MS: return g_rccl_timeout_ms.load();
      case STL_TUNE_LONG_HASH: return g_tune_long_hash.load();
      default: return STL_EINVAL;
    }
  }
  switch (key) {
    case STL_TUNE_FUSED_PREP:
      if (value < 0 || value > 1) return STL_EINVAL;
      return g_tune_fused.exchange(value);
    case STL_TUNE_MAIN_QUEUE:
      if (value != 0 && value != 1) return STL_EINVAL;
      return g_tune_queue.exchange(value);
    case STL_TUNE_STREAMS:
      if (value < 1 || value > (int)stl::kMaxVerifyStreams) return STL_EINVAL;
      return g_tune_streams.exchange(value);
    case STL_TUNE_CHUNK_LOG2:
      if (value != 0 && (value < 15 || value > 20)) return STL_EINVAL;
      return g_tune_sub_log2.exchange(value);
    case STL_TUNE_BYTE_SHARDS:
      if (value != 0 && value != 1) return STL_EINVAL;
      return g_tune_byte_shards.exchange(value);
    case STL_TUNE_QUAD:
      if (value < 0 || value > 3) return STL_EINVAL;
      return g_tune_quad.exchange(value);
    case STL_TUNE_STREAM_WORKSPACES:  // applies as caller contexts are next created
      if (value < 1 || value > 64) return STL_EINVAL;
      return g_max_caller_streams.exchange(value);
    case STL_TUNE_RCCL_TIMEOUT_MS:
      if (value < 1 || value > 3600000) return STL_EINVAL;
      return g_rccl_timeout_ms.exchange(value);
    case STL_TUNE_LONG_HASH:
      if (value < 0 || value > 62) return STL_EINVAL;
      return g_tune_long_hash.exchange(value);
    case STL_TUNE_SHARED_KEYS:
      if (value != 0 && value != 1) return STL_EINVAL;
      return g_tune_shared_keys.exchange(value);
    case STL_TUNE_FIRST_CHUNK:
      if (value < 0 || value % 64 != 0 || value > (1 << 20)) return STL_EINVAL;
      return g_tune_first_chunk.exchange(value);
    case STL_TUNE_R_AHEAD:
      if (value != 0 && value != 1) return STL_EINVAL;
      return g_tune_r_ahead.exchange(value);
    case STL_TUNE_WIDE_MIN_ROWS:
      if (value < 0 || value > (int)stl::kPreChunk) return STL_EINVAL;
      return g_tune_wide_min.exchange(value);
    default:
      return STL_EINVAL;
  }
}

int stl_release_stream(void* stream) {
  const hipStream_t s = static_cast<hipStream_t>(stream);
  std::shared_ptr<StreamCtx> gone;
  {
    std::lock_guard<std::mutex> lk(g_mu);
    if (!g_init) return STL_OK;
    const int di = current_device_index();
    if (di < 0) return STL_ENODEV;
    Device& d = *g_devs[di];
    if (is_pool_stream(d, s)) return STL_EINVAL;
    std::lock_guard<std::mutex> wl(d.ws_mu);
    auto it = d.stream_ws.find(s);
    if (it == d.stream_ws.end()) return STL_OK;
    gone = std::move(it->second);
    d.stream_ws.erase(it);
  }
  return STL_OK;  // `gone` synchronises the device and frees here, once no call holds it
}

int stl_debug_stream_contexts(void) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (!g_init) return 0;
  const int di = current_device_index();
  return di < 0 ? STL_ENODEV : caller_contexts(*g_devs[di]);
}

int stl_get_stats(stl_stats* out) {
  if (!out || (out->struct_size != sizeof(stl_stats) && out->struct_size != offsetof(stl_stats, auto_dedup_chunks)))
    return STL_EINVAL;
  if (out->struct_size == sizeof(stl_stats)) out->auto_dedup_chunks = g_st_auto_dedup.load();
  out->batches = g_st_batches.load();
  out->signatures = g_st_sigs.load();
  out->errors = g_st_errors.load();
  out->host_ns = g_st_host_ns.load();
  out->gather_ns = g_st_gather_ns.load();
  out->accepted = 0;
  out->full_length_lanes = 0;
  for (auto& v : out->phase_ns) v = 0;
  out->phase_chunks = 0;
  DeviceGuard guard;
  std::lock_guard<std::mutex> lk(g_mu);
  for (auto& d : g_devs) {  // device counters: waits for the work queued before the call
    if (!d->counters.p) continue;
    unsigned long long c[2] = {0, 0};
    if (hipSetDevice(d->ordinal) != hipSuccess || hipDeviceSynchronize() != hipSuccess ||
        hipMemcpy(c, d->counters.p, sizeof c, hipMemcpyDeviceToHost) != hipSuccess)
      return STL_EHIP;
    out->accepted += c[0];
    out->full_length_lanes += c[1];
    d->timer.collect();
    std::lock_guard<std::mutex> tl(d->timer.mu);
    for (int i = 0; i < 4; ++i) out->phase_ns[i] += d->timer.ns[i];
    out->phase_chunks += d->timer.chunks;
  }
  return STL_OK;
}

void stl_reset_stats(void) {
  g_st_batches = 0;
  g_st_sigs = 0;
  g_st_errors = 0;
  g_st_host_ns = 0;
  g_st_gather_ns = 0;
  g_st_auto_dedup = 0;
  DeviceGuard guard;
  std::lock_guard<std::mutex> lk(g_mu);
  for (auto& d : g_devs)
    if (d->counters.p && hipSetDevice(d->ordinal) == hipSuccess) {
      (void)hipMemset(d->counters.p, 0, 64);
      (void)hipDeviceSynchronize();  // queued chunks complete before their events are read and dropped
      d->timer.reset();
    }
}

int stl_set_phase_timing(int on) { return g_phase_timing.exchange(on != 0) ? 1 : 0; }

void stl_shard_range(size_t n, int r, int g, size_t* lo, size_t* hi) {
  if (!lo || !hi) return;
  if (g < 1 || r < 0 || r >= g) {
    *lo = *hi = n;
    return;
  }
  shard(n, r, g, lo, hi);
}

void stl_shard_range_bytes(const uint32_t* len, size_t n, int r, int g, size_t* lo, size_t* hi) {
  if (!lo || !hi) return;
  if (g < 1 || r < 0 || r >= g || (n && !len)) {
    *lo = *hi = n;
    return;
  }
  std::vector<size_t> bound;
  shard_bytes_bounds(len, n, g, bound);
  *lo = bound[r];
  *hi = bound[r + 1];
}

int stl_ed25519_verify_batch(const uint8_t* sig, const uint8_t* msg, const uint8_t* pk, size_t n,
                             uint8_t* accept_bitmap, uint32_t flags) {
  if (n == 0) return STL_OK;
  if (!sig || !msg || !pk || !accept_bitmap) return STL_EINVAL;
  STL_RC(check_flags(flags));
  const Batch b{Mode::kSig, sig, msg, pk, nullptr, nullptr, nullptr, accept_bitmap, nullptr, nullptr,
                stl::kernel_mode(flags), 0u, auto_dedup(flags)};
  CallSpan span{"stl_ed25519_verify_batch", n};
  uint64_t g = 0;
  const int rc = run_batch(b, n, &g);
  return span.finish(rc, g);
}

int stl_tx_verify_batch(const uint8_t* preimages, const uint64_t* offset, const uint32_t* len, const uint8_t* sig,
                        const uint8_t* pk, size_t n, uint8_t* accept_bitmap, uint32_t flags) {
  if (n == 0) return STL_OK;
  if (!preimages || !offset || !len || !sig || !pk || !accept_bitmap) return STL_EINVAL;
  STL_RC(check_flags(flags));
  const Batch b{Mode::kPre, sig, nullptr, pk, preimages, offset, len, accept_bitmap, nullptr, nullptr,
                stl::kernel_mode(flags), 0u, auto_dedup(flags)};
  CallSpan span{"stl_tx_verify_batch", n};
  uint64_t g = 0;
  const int rc = run_batch(b, n, &g);
  return span.finish(rc, g);
}

int stl_signed_blob_verify_batch(uint32_t kind, const uint8_t* blobs, const uint64_t* offset, const uint32_t* len,
                                 size_t n, uint8_t* accept_bitmap, uint8_t* status, uint8_t* id, uint32_t flags) {
  if (kind != STL_BLOB_TRANSACTION && kind != STL_BLOB_VALIDATION) return STL_EINVAL;
  if (n == 0) return STL_OK;
  if (!blobs || !offset || !len || !accept_bitmap) return STL_EINVAL;
  STL_RC(check_flags(flags));
  const Batch b{Mode::kBlob, nullptr, nullptr, nullptr, blobs, offset, len, accept_bitmap, status, id,
                stl::kernel_mode(flags), kind, auto_dedup(flags)};
  CallSpan span{kind == STL_BLOB_VALIDATION ? "stl_signed_blob_verify_batch(validation)" : "stl_tx_blob_verify_batch",
                n};
  uint64_t g = 0;
  const int rc = run_batch(b, n, &g);
  return span.finish(rc, g);
}

int stl_tx_blob_verify_batch(const uint8_t* blobs, const uint64_t* offset, const uint32_t* len, size_t n,
                             uint8_t* accept_bitmap, uint8_t* status, uint8_t* tx_id, uint32_t flags) {
  return stl_signed_blob_verify_batch(STL_BLOB_TRANSACTION, blobs, offset, len, n, accept_bitmap, status, tx_id,
                                      flags);
}

namespace {
int verify_detached_device(const uint8_t* sig, const uint8_t* m, unsigned long long mlen, const uint8_t* pk);
bool s_lt_l(const uint8_t* S);
}  // namespace

int stl_ed25519_verify_detached(const uint8_t* sig, const uint8_t* m, unsigned long long mlen, const uint8_t* pk) {
  if (!sig || !pk || (mlen && !m)) return STL_EINVAL;
  const stl_verify_fn fb = g_fallback_verify.load();
  // a message longer than one device row (2^32 - 1 bytes) is valid input to
  // libsodium: with a fallback registered it answers that case too
  const int rc = mlen > 0xffffffffull ? STL_EINVAL : verify_detached_device(sig, m, mlen, pk);
  if (rc >= -1 || fb == nullptr) return rc;
  // a device failure is never a reject: the caller's own check answers,
  // composed as RippleAddress::verifySignature composes it (RippleAddress.cpp:196-199)
  return (fb(sig, m, mlen, pk) == 0 && s_lt_l(sig + 32)) ? 0 : -1;
}

namespace {
// crypto_sign_check_S_lt_l (RippleAddress.cpp:226-245): little-endian S < L
bool s_lt_l(const uint8_t* S) {
  static const uint8_t L[32] = {0xed, 0xd3, 0xf5, 0x5c, 0x1a, 0x63, 0x12, 0x58, 0xd6, 0x9c, 0xf7,
                                0xa2, 0xde, 0xf9, 0xde, 0x14, 0x00, 0x00, 0x00, 0x00, 0x00, 0x00,
                                0x00, 0x00, 0x00, 0x00, 0x00, 0x00, 0x00, 0x00, 0x00, 0x10};
  for (int i = 31; i >= 0; --i)
    if (S[i] != L[i]) return S[i] < L[i];
  return false;
}

int verify_detached_device(const uint8_t* sig, const uint8_t* m, unsigned long long mlen, const uint8_t* pk) {
  if (mlen == 32) {
    uint8_t bit = 0;
    const int rc = stl_ed25519_verify_batch(sig, m, pk, 1, &bit, STL_POLICY_SODIUM_1_0_18);
    if (rc) return rc;
    return (bit & 1) ? 0 : -1;
  }
  if (mlen > 0xffffffffull) return STL_EINVAL;
  // arbitrary-length message: k = H(R||A||m) mod L on the device, then verify
  STL_RC(ensure_init());
  DeviceGuard guard;
  Device& d = *g_devs[0];
  std::lock_guard<std::mutex> lk(d.mu);
  STL_TRY(hipSetDevice(d.ordinal));
  STL_RC(d.sig.ensure(64));
  STL_RC(d.pk.ensure(32));
  STL_RC(d.msg.ensure(32));
  STL_RC(d.bitmap.ensure(8));
  STL_RC(d.pre.ensure(mlen ? mlen : 1));
  STL_RC(d.off.ensure(16));
  hipStream_t s = d.stream;
  const uint64_t hostmeta[2] = {0, mlen};
  uint64_t word = 0;
  auto enqueue = [&]() -> int {
    STL_TRY(hipMemcpyAsync(d.sig.p, sig, 64, hipMemcpyHostToDevice, s));
    STL_TRY(hipMemcpyAsync(d.pk.p, pk, 32, hipMemcpyHostToDevice, s));
    if (mlen) STL_TRY(hipMemcpyAsync(d.pre.p, m, mlen, hipMemcpyHostToDevice, s));
    STL_TRY(hipMemcpyAsync(d.off.p, hostmeta, 16, hipMemcpyHostToDevice, s));
    uint64_t* meta = static_cast<uint64_t*>(d.off.p);
    STL_TRY(stl::launch_hram_var(static_cast<uint8_t*>(d.sig.p), static_cast<uint8_t*>(d.pk.p),
                                 static_cast<uint8_t*>(d.pre.p), meta, meta + 1, 1, static_cast<uint8_t*>(d.msg.p), s));
    STL_RC(run_verify(d, s, static_cast<uint8_t*>(d.sig.p), static_cast<uint8_t*>(d.msg.p),
                      static_cast<uint8_t*>(d.pk.p), 1, static_cast<uint64_t*>(d.bitmap.p), STL_POLICY_SODIUM_1_0_18,
                      true, 1));
    STL_TRY(hipMemcpyAsync(&word, d.bitmap.p, 8, hipMemcpyDeviceToHost, s));
    STL_TRY(hipStreamSynchronize(s));
    return STL_OK;
  };
  const int rc = enqueue();
  const int drc = drain(d);
  if (rc || drc) return rc ? rc : drc;
  return (word & 1) ? 0 : -1;
}
}  // namespace

namespace {
int device_for_call(Device** out) {
  STL_RC(ensure_init());
  const int di = current_device_index();
  if (di < 0) return STL_ENODEV;
  *out = g_devs[di].get();
  return STL_OK;
}
}  // namespace

namespace {
// The device-resident calls' automatic dedup: the keys are in
// HBM, so instead of reading them on the host each call ends with a
// one-workgroup sample kernel on the caller's stream whose verdict the NEXT
// call on that stream uses -- no synchronisation, a few microseconds of GPU
// time.  A stream's first call, or a call issued before the previous call's
// sample has run, uses the last verdict seen (initially: no dedup).
// c: the caller stream's context, kept alive by the caller until the sample
// kernel writing *flag_dev is enqueued.
int auto_dedup_device(StreamCtx& c, uint32_t flags, uint32_t* mode, uint32_t** flag_dev) {
  *flag_dev = nullptr;
  if (!auto_dedup(flags)) return STL_OK;
  std::lock_guard<std::mutex> lk(c.mu);
  if (!c.auto_flag) {
    void* p = nullptr;
    STL_TRY(hipHostMalloc(&p, 64, hipHostMallocMapped | hipHostMallocCoherent));
    c.auto_flag = static_cast<uint32_t*>(p);
    *c.auto_flag = 0;
    void* dp = nullptr;
    if (hipHostGetDevicePointer(&dp, p, 0) != hipSuccess) {
      (void)hipHostFree(p);
      c.auto_flag = nullptr;
      return STL_EHIP;
    }
    c.auto_flag_dev = static_cast<uint32_t*>(dp);
  }
  if (__atomic_load_n(c.auto_flag, __ATOMIC_ACQUIRE) == 1u) {
    *mode |= stl::kModeDedupKeys;
    g_st_auto_dedup++;
  }
  *flag_dev = c.auto_flag_dev;
  return STL_OK;
}
}  // namespace

namespace {
// Device-resident checkSign (SURVEY 8a rows a5-a6 over rows already in HBM):
// SHA512Half of every signing preimage -- or the serialized-object pass of
// tx_blob_kernel -- then the verify, in the verify's chunks (chunk_for) dealt
// to the caller's stream and pool stream 1.  The first chunk is hashed alone
// on the caller's stream while pool stream 1 hashes all the other rows in one
// launch (one balanced longest-first queue: per-chunk hash launches of
// variable-length rows end in a ragged tail); chunk 0's verify then overlaps
// that hashing, and the later chunks wait for it.  Blob rows get their
// signature and key from the pass (deferred / malformed rows a signature that
// always rejects); status / id as stl_tx_blob_prepare_device writes them.
int checksign_device(Device& d, hipStream_t s, bool blob, uint32_t kind, const uint8_t* bytes, const uint64_t* off,
                     const uint32_t* len, const uint8_t* sig_in, const uint8_t* pk_in, size_t n, uint64_t* words,
                     uint8_t* status, uint8_t* id, uint32_t flags) {
  const stl::PhaseClock* clock = phase_clock(d);
  // chunks and streams as a device-resident verify call
  size_t sub = chunk_for(d.grid, n);
  uint32_t S = (uint32_t)std::max(1, std::min(g_tune_streams.load(), 2));
  if (clock || n <= sub) {
    S = 1;
    sub = std::min<size_t>(n, stl::kPreChunk);
  }
  hipStream_t ks[2] = {s, s == d.stream2 ? d.stream : d.stream2};
  const std::shared_ptr<StreamCtx> hold[2] = {stream_ctx(d, ks[0]),
                                              S > 1 ? stream_ctx(d, ks[1]) : std::shared_ptr<StreamCtx>()};
  StreamCtx* kc[2] = {hold[0].get(), hold[1].get()};
  StreamCtx& c = *kc[0];
  uint32_t mode = stl::kernel_mode(flags);
  uint32_t* flag_dev = nullptr;
  STL_RC(auto_dedup_device(c, flags, &mode, &flag_dev));
  const bool dedup = (mode & stl::kModeDedupKeys) != 0;
  // One chunk whose phase 1 runs as the two-role lane-pair kernel (small
  // batches; not blobs, whose signatures and keys come out of the pass): its
  // point role -- the two square-root chains, which need no message -- and
  // the key sample run on the other pool stream while the preimages hash.
  auto exec_for = [&](uint32_t cnt, uint32_t j) {
    stl::VerifyExec x;
    x.grid = verify_grid_for(d, cnt);
    x.ws_grid = d.grid;  // every workspace is verify_ws_bytes(d.grid, ...)
    x.pair_max = pair_max(d);
    x.quad_max = quad_max(d);
    x.duo_max = duo_max(d);
    x.wide = static_cast<const uint4*>(d.wide.p);
    x.counters = dev_counters(d);
    x.clock = S > 1 ? nullptr : clock;
    x.fused_prep = g_tune_fused.load();
    x.main_queue = g_tune_queue.load() != 0;
    x.concurrent = S > 1;
    x.nstreams = 1;
    x.streams[0] = ks[j];
    x.ws[0] = static_cast<uint4*>(kc[j]->ws.p);
    return x;
  };
  const bool ahead = S == 1 && !blob && !clock && n <= stl::kPreChunk &&
                     stl::verify_pair_points((uint32_t)n, mode, exec_for((uint32_t)n, 0));
  std::vector<std::unique_lock<std::mutex>> locks;
  if (S > 1 && kc[1] < kc[0]) locks.emplace_back(kc[1]->mu);
  locks.emplace_back(c.mu);
  if (S > 1 && kc[1] > kc[0]) locks.emplace_back(kc[1]->mu);
  // the hash queues under the locks held through the launches below: pool
  // stream 1's context is shared by every caller stream
  uint32_t* q[2] = {nullptr, nullptr};
  STL_RC(ctx_queue(*kc[0], S > 1 ? sub : n, &q[0], blob));
  if (S > 1) STL_RC(ctx_queue(*kc[1], n - sub, &q[1], blob));
  const size_t row = blob ? 128 : 32;
  STL_RC(c.scratch.ensure(std::max<size_t>(n, 1) * row));
  uint8_t* msg = static_cast<uint8_t*>(c.scratch.p);
  uint8_t* sig = blob ? msg + 32 * n : const_cast<uint8_t*>(sig_in);
  uint8_t* pk = blob ? msg + 96 * n : const_cast<uint8_t*>(pk_in);
  uint8_t* st = status;
  for (uint32_t j = 0; j < S; ++j) STL_RC(kc[j]->ws.ensure(stl::verify_ws_bytes(d.grid, dedup)));
  // dedup over several chunks: one key domain for the call (VerifyExec::key_ws),
  // built on an idle pool stream (cs) as soon as the keys are known -- at
  // once for preimages, after both parse kernels for blobs -- beside the
  // hashing and the scalar kernels; with no idle stream, by chunk 0 after its
  // scalar kernel
  const bool shared_keys = dedup && S > 1 && n <= stl::kPreChunk && sub > pair_max(d) && g_tune_shared_keys.load();
  hipStream_t cs = shared_keys ? key_stream_for(d, ks, S) : nullptr;
  if (shared_keys && !c.keys) STL_TRY(hipEventCreateWithFlags(&c.keys, hipEventDisableTiming));
  if (cs && blob)
    for (hipEvent_t& e : c.parsed)
      if (!e) STL_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  // ... and R's decoding of every row on a fourth stream (the copy stream,
  // idle in a device-resident call), beside the key domain: the chunks then
  // finish their phase 1 without a square-root chain (VerifyExec::rdec)
  hipStream_t cr = cs && g_tune_r_ahead.load() && d.copy != cs && d.copy != ks[0] && d.copy != ks[1] ? d.copy
                                                                                                      : nullptr;
  if (cr) {
    STL_RC(c.rdec.ensure(n * 80));
    if (!c.rready) STL_TRY(hipEventCreateWithFlags(&c.rready, hipEventDisableTiming));
  }
  if (S > 1 || ahead) {
    if (!c.fork) STL_TRY(hipEventCreateWithFlags(&c.fork, hipEventDisableTiming));
    if (!c.join[1]) STL_TRY(hipEventCreateWithFlags(&c.join[1], hipEventDisableTiming));
    if (!c.join[2]) STL_TRY(hipEventCreateWithFlags(&c.join[2], hipEventDisableTiming));
    STL_TRY(hipEventRecord(c.fork, s));
    STL_TRY(hipStreamWaitEvent(ks[1], c.fork, 0));
  }
  auto fail = [&](int rc) {
    if (S > 1 || ahead) (void)hipStreamSynchronize(ks[1]);
    if (cs) (void)hipStreamSynchronize(cs);
    if (cr) (void)hipStreamSynchronize(cr);
    return rc;
  };
  if (ahead) {
    int rc = STL_OK;
    if (fault_now() || stl::launch_verify_points(sig, pk, (uint32_t)n, mode, exec_for((uint32_t)n, 0), ks[1]) !=
                           hipSuccess)
      rc = STL_EHIP;
    if (!rc && flag_dev && stl::launch_key_sample(pk, (uint32_t)n, flag_dev, ks[1]) != hipSuccess) rc = STL_EHIP;
    if (!rc && hipEventRecord(c.join[2], ks[1]) != hipSuccess) rc = STL_EHIP;
    if (rc) return fail(rc);
  }
  // rows [b0, b0 + cnt) hashed (or passed) on stream js with queue qw
  // blob rows' pass in two halves when the key work runs beside it: both
  // streams' parse kernels first (the keys and signatures are out), then the
  // key domain and R's decoding are enqueued, then the hashing -- so the
  // host's enqueue order follows the device's critical path
  const bool split_pass = blob && cs && S > 1;
  auto parse = [&](size_t b0, size_t cnt, hipStream_t js, uint32_t* qw) -> int {
    if (fault_now()) return STL_EHIP;
    const hipError_t e = stl::launch_tx_blob_parse(bytes, off + b0, len + b0, (uint32_t)cnt, msg + 32 * b0,
                                                   sig + 64 * b0, pk + 32 * b0, id ? id + 32 * b0 : nullptr, st + b0,
                                                   qw, hash_grid(d), js, kind, c.parsed[js == ks[0] ? 0 : 1]);
    return e == hipSuccess ? STL_OK : STL_EHIP;
  };
  // rows [b0, b0 + cnt) hashed (or passed) on stream js with queue qw
  auto hash = [&](size_t b0, size_t cnt, hipStream_t js, uint32_t* qw) -> int {
    hipError_t e;
    if (split_pass) {
      e = stl::launch_tx_blob_hash(bytes, off + b0, len + b0, (uint32_t)cnt, msg + 32 * b0, sig + 64 * b0,
                                   pk + 32 * b0, id ? id + 32 * b0 : nullptr, st + b0, qw, hash_grid(d), js, kind);
      return e == hipSuccess ? STL_OK : STL_EHIP;
    }
    if (fault_now()) return STL_EHIP;
    if (blob)
      e = stl::launch_tx_blob(bytes, off + b0, len + b0, (uint32_t)cnt, msg + 32 * b0, sig + 64 * b0, pk + 32 * b0,
                              id ? id + 32 * b0 : nullptr, st + b0, qw, hash_grid(d), js, kind,
                              cs ? c.parsed[js == ks[0] ? 0 : 1] : nullptr);
    else
      e = stl::launch_tx_hash(bytes, off + b0, len + b0, (uint32_t)cnt, msg + 32 * b0, qw, hash_grid(d), js,
                              hash_long_min(d, n));
    return e == hipSuccess ? STL_OK : STL_EHIP;
  };
  auto hash_all = [&]() -> int {
    if (S == 1) {
      int rc = hash(0, n, s, q[0]);
      if (!rc && ahead && hipStreamWaitEvent(s, c.join[2], 0) != hipSuccess) rc = STL_EHIP;
      return rc;
    }
    int rc = hash(0, sub, ks[0], q[0]);
    if (!rc) rc = hash(sub, n - sub, ks[1], q[1]);
    if (!rc && hipEventRecord(c.join[2], ks[1]) != hipSuccess) rc = STL_EHIP;
    return rc;
  };
  if (split_pass) {
    int rc = parse(0, sub, ks[0], q[0]);
    if (!rc) rc = parse(sub, n - sub, ks[1], q[1]);
    if (rc) return fail(rc);
  } else if (int rc = hash_all()) {
    return fail(rc);
  }
  if (cs) {  // the call's key domain on its own stream, in the caller's workspace
    hipError_t e = hipSuccess;
    if (blob) {
      e = hipStreamWaitEvent(cs, c.parsed[0], 0);
      if (e == hipSuccess) e = hipStreamWaitEvent(cs, c.parsed[1], 0);
    } else {
      e = hipStreamWaitEvent(cs, c.fork, 0);
    }
    if (e == hipSuccess && fault_now()) e = hipErrorUnknown;
    if (e == hipSuccess)
      e = stl::launch_key_domain_ws(pk, (uint32_t)n, static_cast<uint4*>(kc[0]->ws.p), d.grid,
                                    (uint32_t)g_tune_wide_min.load(), cs);
    if (e == hipSuccess) e = hipEventRecord(c.keys, cs);
    if (e != hipSuccess) return fail(STL_EHIP);
  }
  if (cr) {  // R's decoding of every row, as soon as the signatures are known
    hipError_t e = hipSuccess;
    if (blob) {
      e = hipStreamWaitEvent(cr, c.parsed[0], 0);
      if (e == hipSuccess) e = hipStreamWaitEvent(cr, c.parsed[1], 0);
    } else {
      e = hipStreamWaitEvent(cr, c.fork, 0);
    }
    if (e == hipSuccess && fault_now()) e = hipErrorUnknown;
    // a last chunk on lane pairs decodes R in its own pair kernel: only the
    // one-lane chunks' rows are decoded ahead
    const size_t last = n - (n - 1) / sub * sub;
    const bool last_pairs = n > sub && !(mode & stl::kModeOneLane) && last <= pair_max(d);
    const size_t r_rows = last_pairs ? n - last : n;
    if (e == hipSuccess)
      e = stl::launch_point_r(sig, pk, (uint32_t)r_rows, mode, static_cast<uint4*>(c.rdec.p), cr);
    if (e == hipSuccess) e = hipEventRecord(c.rready, cr);
    if (e != hipSuccess) return fail(STL_EHIP);
  }
  if (split_pass)
    if (int rc = hash_all()) return fail(rc);
  size_t k = 0;
  for (size_t b0 = 0; b0 < n; b0 += sub, ++k) {
    const uint32_t j = (uint32_t)(k % S);
    const uint32_t cnt = (uint32_t)std::min(sub, n - b0);
    hipStream_t js = ks[j];
    // the caller's stream verifies chunk 0 during the other rows' hashing,
    // then waits for it
    if (S > 1 && k == 2 && hipStreamWaitEvent(ks[0], c.join[2], 0) != hipSuccess) return fail(STL_EHIP);
    stl::VerifyExec x = exec_for(cnt, j);
    x.points_done = ahead;
    if (shared_keys) {
      // one key domain for the whole call, in the caller's workspace: built by
      // chunk 0 on the caller's stream after its scalar kernel -- for blobs
      // once the other rows' keys are out of the pass on pool stream 1
      x.key_ws = static_cast<uint4*>(kc[0]->ws.p);
      x.key_n = (uint32_t)n;
      x.key_base = (uint32_t)b0;
      x.key_build = k == 0 && !cs;
      x.key_ready = c.keys;
      x.key_after = blob && !cs ? c.join[2] : nullptr;
      if (cr) {
        x.rdec = static_cast<const uint4*>(c.rdec.p);
        x.r_ready = c.rready;
      }
    }
    x.wide_min = (uint32_t)g_tune_wide_min.load();
    if (fault_now() || stl::launch_verify(sig + 64 * b0, msg + 32 * b0, pk + 32 * b0, cnt, words + b0 / 64, mode,
                                          false, x) != hipSuccess)
      return fail(STL_EHIP);
  }
  if (S > 1) {
    if (hipEventRecord(c.join[1], ks[1]) != hipSuccess || hipStreamWaitEvent(s, c.join[1], 0) != hipSuccess)
      return fail(STL_EHIP);
  }
  if (flag_dev && !ahead) STL_TRY(stl::launch_key_sample(pk, (uint32_t)n, flag_dev, s));
  return STL_OK;
}
}  // namespace

int stl_tx_verify_batch_device(const uint8_t* d_preimages, const uint64_t* d_offset, const uint32_t* d_len,
                               const uint8_t* d_sig, const uint8_t* d_pk, size_t n, uint64_t* d_bitmap_words,
                               uint32_t flags, void* stream) {
  if (n == 0) return STL_OK;
  if (!d_preimages || !d_offset || !d_len || !d_sig || !d_pk || !d_bitmap_words) return STL_EINVAL;
  STL_RC(check_flags(flags));
  if (n > 0xffffffc0ull) return STL_EINVAL;
  Device* d = nullptr;
  STL_RC(device_for_call(&d));
  return checksign_device(*d, static_cast<hipStream_t>(stream), false, 0u, d_preimages, d_offset, d_len, d_sig, d_pk,
                          n, d_bitmap_words, nullptr, nullptr, flags);
}

int stl_signed_blob_verify_batch_device(uint32_t kind, const uint8_t* d_blobs, const uint64_t* d_offset,
                                        const uint32_t* d_len, size_t n, uint64_t* d_bitmap_words, uint8_t* d_status,
                                        uint8_t* d_id, uint32_t flags, void* stream) {
  if (kind != STL_BLOB_TRANSACTION && kind != STL_BLOB_VALIDATION) return STL_EINVAL;
  if (n == 0) return STL_OK;
  if (!d_blobs || !d_offset || !d_len || !d_bitmap_words || !d_status) return STL_EINVAL;
  STL_RC(check_flags(flags));
  if (n > 0xffffffc0ull) return STL_EINVAL;
  Device* d = nullptr;
  STL_RC(device_for_call(&d));
  return checksign_device(*d, static_cast<hipStream_t>(stream), true, kind, d_blobs, d_offset, d_len, nullptr,
                          nullptr, n, d_bitmap_words, d_status, d_id, flags);
}

int stl_ed25519_verify_batch_device(const uint8_t* d_sig, const uint8_t* d_msg, const uint8_t* d_pk, size_t n,
                                    uint64_t* d_bitmap_words, uint32_t flags, void* stream) {
  if (n == 0) return STL_OK;
  if (!d_sig || !d_msg || !d_pk || !d_bitmap_words) return STL_EINVAL;
  STL_RC(check_flags(flags));
  if (n > 0xffffffc0ull) return STL_EINVAL;
  Device* d = nullptr;
  STL_RC(device_for_call(&d));
  hipStream_t s = static_cast<hipStream_t>(stream);
  const std::shared_ptr<StreamCtx> c = stream_ctx(*d, s);  // alive until the sample kernel is enqueued
  uint32_t mode = stl::kernel_mode(flags);
  uint32_t* flag_dev = nullptr;
  STL_RC(auto_dedup_device(*c, flags, &mode, &flag_dev));
  STL_RC(run_verify(*d, s, d_sig, d_msg, d_pk, n, d_bitmap_words, mode, false, g_tune_streams.load()));
  if (flag_dev) STL_TRY(stl::launch_key_sample(d_pk, (uint32_t)n, flag_dev, s));
  return STL_OK;
}

int stl_debug_clock_stamp(uint64_t* d_out, uint32_t nwg, void* stream) {
  if (!d_out || nwg > 65536) return STL_EINVAL;
  Device* d = nullptr;
  STL_RC(device_for_call(&d));
  STL_TRY(stl::launch_clock_stamp(reinterpret_cast<unsigned long long*>(d_out), nwg,
                                  static_cast<hipStream_t>(stream)));
  return STL_OK;
}

int stl_debug_verify_k_device(const uint8_t* d_sig, const uint8_t* d_k, const uint8_t* d_pk, size_t n,
                              uint64_t* d_bitmap_words, uint32_t flags, void* stream) {
  if (n == 0) return STL_OK;
  if (!d_sig || !d_k || !d_pk || !d_bitmap_words) return STL_EINVAL;
  STL_RC(check_flags(flags));
  if (n > 0xffffffc0ull) return STL_EINVAL;
  Device* d = nullptr;
  STL_RC(device_for_call(&d));
  hipStream_t s = static_cast<hipStream_t>(stream);
  return run_verify(*d, s, d_sig, d_k, d_pk, n, d_bitmap_words, stl::kernel_mode(flags), true,
                    g_tune_streams.load());
}

int stl_tx_hash_batch_device(const uint8_t* d_preimages, const uint64_t* d_offset, const uint32_t* d_len, size_t n,
                             uint8_t* d_msg, void* stream) {
  if (n == 0) return STL_OK;
  if (!d_preimages || !d_offset || !d_len || !d_msg || n > 0xffffffc0ull) return STL_EINVAL;
  Device* d = nullptr;
  STL_RC(device_for_call(&d));
  hipStream_t s = static_cast<hipStream_t>(stream);
  const std::shared_ptr<StreamCtx> c = stream_ctx(*d, s);
  std::lock_guard<std::mutex> lk(c->mu);
  uint32_t* ctr = nullptr;
  STL_RC(ctx_queue(*c, n, &ctr));
  STL_TRY(stl::launch_tx_hash(d_preimages, d_offset, d_len, (uint32_t)n, d_msg, ctr, hash_grid(*d), s,
                              hash_long_min(*d, n)));
  return STL_OK;
}

int stl_signed_blob_prepare_device(uint32_t kind, const uint8_t* d_blobs, const uint64_t* d_offset,
                                   const uint32_t* d_len, size_t n, uint8_t* d_msg, uint8_t* d_sig, uint8_t* d_pk,
                                   uint8_t* d_id, uint8_t* d_status, void* stream) {
  if (kind != STL_BLOB_TRANSACTION && kind != STL_BLOB_VALIDATION) return STL_EINVAL;
  if (n == 0) return STL_OK;
  if (!d_blobs || !d_offset || !d_len || !d_msg || !d_sig || !d_pk || !d_status || n > 0xffffffc0ull)
    return STL_EINVAL;
  Device* d = nullptr;
  STL_RC(device_for_call(&d));
  hipStream_t s = static_cast<hipStream_t>(stream);
  const std::shared_ptr<StreamCtx> c = stream_ctx(*d, s);
  std::lock_guard<std::mutex> lk(c->mu);
  uint32_t* ctr = nullptr;
  STL_RC(ctx_queue(*c, n, &ctr, true));
  STL_TRY(stl::launch_tx_blob(d_blobs, d_offset, d_len, (uint32_t)n, d_msg, d_sig, d_pk, d_id, d_status, ctr,
                              hash_grid(*d), s, kind));
  return STL_OK;
}

int stl_tx_blob_prepare_device(const uint8_t* d_blobs, const uint64_t* d_offset, const uint32_t* d_len, size_t n,
                               uint8_t* d_msg, uint8_t* d_sig, uint8_t* d_pk, uint8_t* d_tx_id, uint8_t* d_status,
                               void* stream) {
  return stl_signed_blob_prepare_device(STL_BLOB_TRANSACTION, d_blobs, d_offset, d_len, n, d_msg, d_sig, d_pk,
                                        d_tx_id, d_status, stream);
}

int stl_ed25519_sign_batch_device(const uint8_t* d_seed, const uint8_t* d_msg, size_t n, uint8_t* d_pk,
                                  uint8_t* d_sig, void* stream) {
  if (n == 0) return STL_OK;
  if (!d_seed || !d_msg || !d_pk || !d_sig || n > 0xffffffc0ull) return STL_EINVAL;
  Device* d = nullptr;
  STL_RC(device_for_call(&d));
  hipStream_t s = static_cast<hipStream_t>(stream);
  const std::shared_ptr<StreamCtx> c = stream_ctx(*d, s);
  std::lock_guard<std::mutex> lk(c->mu);
  STL_RC(c->ws.ensure(stl::verify_ws_bytes(d->grid)));
  STL_TRY(stl::launch_sign(d_seed, d_msg, (uint32_t)n, d_pk, d_sig, static_cast<uint4*>(c->ws.p), grid_for(*d, n), s));
  return STL_OK;
}

int stl_debug_sign_adversarial_device(const uint8_t* d_seed, const uint8_t* d_msg, const uint8_t* d_cls,
                                      const uint32_t* d_param, size_t n, uint8_t* d_pk, uint8_t* d_sig,
                                      uint8_t* d_msg_out, void* stream) {
  if (n == 0) return STL_OK;
  if (!d_seed || !d_msg || !d_cls || !d_param || !d_pk || !d_sig || !d_msg_out || n > 0xffffffc0ull)
    return STL_EINVAL;
  Device* d = nullptr;
  STL_RC(device_for_call(&d));
  hipStream_t s = static_cast<hipStream_t>(stream);
  const std::shared_ptr<StreamCtx> c = stream_ctx(*d, s);
  std::lock_guard<std::mutex> lk(c->mu);
  STL_RC(c->ws.ensure(stl::verify_ws_bytes(d->grid)));
  STL_TRY(stl::launch_sign(d_seed, d_msg, (uint32_t)n, d_pk, d_sig, static_cast<uint4*>(c->ws.p), grid_for(*d, n), s,
                           d_cls, d_param, d_msg_out));
  return STL_OK;
}

// ---- one process per GPU ----------------------------------------------------

int stl_comm_unique_id(uint8_t id[128]) {
  if (!id) return STL_EINVAL;
  static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId is 128 bytes");
  if (!g_rccl.load()) return STL_ERCCL;
  ncclUniqueId u;
  STL_RCCL_TRY(g_rccl.GetUniqueId(&u));
  std::memcpy(id, &u, sizeof u);
  return STL_OK;
}

int stl_comm_init_rank(int nranks, int rank, const uint8_t id[128]) {
  if (!id || nranks < 1 || rank < 0 || rank >= nranks) return STL_EINVAL;
  Device* d = nullptr;
  STL_RC(device_for_call(&d));
  if (!g_rccl.load()) return STL_ERCCL;
  std::lock_guard<std::mutex> lk(g_pcomm_mu);
  if (g_pcomm) return STL_EINVAL;  // one communicator per process; stl_comm_destroy first
  ncclUniqueId u;
  std::memcpy(&u, id, sizeof u);
  ncclComm_t c = nullptr;
  if (g_rccl.nonblocking()) {
    // nonblocking bring-up polled against the deadline: a rank that never
    // joins costs STL_ERCCL after STL_RCCL_TIMEOUT_S, not a hung process
    ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
    cfg.blocking = 0;
    if (fault_now()) return STL_ERCCL;
    const ncclResult_t r = g_rccl.CommInitRankConfig(&c, nranks, u, rank, &cfg);
    const int rc = c ? rccl_settle(c, r) : STL_ERCCL;
    if (rc) {
      if (c) (void)g_rccl.CommAbort(c);
      return rc;
    }
  } else {
    STL_RCCL_TRY(g_rccl.CommInitRank(&c, nranks, u, rank));
  }
  g_pcomm = c;
  g_pcomm_ranks = nranks;
  return STL_OK;
}

void stl_comm_destroy(void) {
  std::lock_guard<std::mutex> lk(g_pcomm_mu);
  if (g_pcomm && g_rccl.ok) (void)g_rccl.CommDestroy(g_pcomm);
  g_pcomm = nullptr;
  g_pcomm_ranks = 0;
}

void stl_comm_abort(void) {
  std::lock_guard<std::mutex> lk(g_pcomm_mu);
  pcomm_abort_locked();
}

int stl_comm_sync(void* stream, int timeout_ms) {
  const hipStream_t s = static_cast<hipStream_t>(stream);
  const int ms = timeout_ms > 0 ? timeout_ms : g_rccl_timeout_ms.load();
  if (fault_now()) {  // fault injection: handled as a failed collective
    std::lock_guard<std::mutex> lk(g_pcomm_mu);
    pcomm_abort_locked();
    return STL_ERCCL;
  }
  // The work queued on s ahead of the last gather (the verify kernels) is not
  // the collective's: wait for the gather's start event first (bounded only
  // by the larger of 10x the deadline and the library's RCCL deadline; a
  // lapse there is a device error and the communicator stays), then give the
  // gather itself the deadline.
  hipEvent_t start = nullptr;
  {
    std::lock_guard<std::mutex> lk(g_pcomm_mu);
    if (g_gather_stream == s) start = g_gather_start;
  }
  if (start) {
    const long long cap_ms = std::max<long long>(10ll * ms, g_rccl_timeout_ms.load());
    const auto cap = std::chrono::steady_clock::now() + std::chrono::milliseconds(cap_ms);
    hipError_t q;
    while ((q = hipEventQuery(start)) == hipErrorNotReady) {
      if (std::chrono::steady_clock::now() > cap) return STL_EHIP;
      std::this_thread::sleep_for(std::chrono::microseconds(50));
    }
    if (q != hipSuccess) return STL_EHIP;
  }
  const auto end = std::chrono::steady_clock::now() + std::chrono::milliseconds(ms);
  for (;;) {
    const hipError_t q = hipStreamQuery(s);
    if (q == hipSuccess) return STL_OK;
    if (q != hipErrorNotReady) return STL_EHIP;
    {
      std::lock_guard<std::mutex> lk(g_pcomm_mu);
      ncclResult_t st = ncclSuccess;
      const bool failed = g_pcomm && g_rccl.CommGetAsyncError &&
                          (g_rccl.CommGetAsyncError(g_pcomm, &st) != ncclSuccess ||
                           (st != ncclSuccess && st != ncclInProgress));
      if (failed || std::chrono::steady_clock::now() > end) {
        // a stalled or failed collective: abort the communicator, which ends
        // its kernels, so the stream drains and the caller can fall back
        pcomm_abort_locked();
        return STL_ERCCL;
      }
    }
    std::this_thread::sleep_for(std::chrono::microseconds(50));
  }
}

int stl_comm_info(int* nranks, int* rank) {
  if (!nranks || !rank) return STL_EINVAL;
  {
    std::lock_guard<std::mutex> lk(g_pcomm_mu);
    if (g_pcomm) {
      STL_RCCL_TRY(g_rccl.CommCount(g_pcomm, nranks));
      STL_RCCL_TRY(g_rccl.CommUserRank(g_pcomm, rank));
      return STL_OK;
    }
  }
  std::lock_guard<std::mutex> lk(g_mu);
  if (!g_comm_gather || g_devs.empty()) return STL_ERCCL;
  int di = current_device_index();
  if (di < 0) di = 0;
  STL_RCCL_TRY(g_rccl.CommCount(g_devs[di]->comm, nranks));
  STL_RCCL_TRY(g_rccl.CommUserRank(g_devs[di]->comm, rank));
  return STL_OK;
}

int stl_bitmap_gather_device(const uint64_t* d_words, size_t words_per_rank, uint64_t* d_all_words, int root,
                             void* stream) {
  std::lock_guard<std::mutex> lk(g_pcomm_mu);
  if (!g_pcomm) return STL_ERCCL;
  if (!d_words || words_per_rank == 0 || root >= g_pcomm_ranks) return STL_EINVAL;
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (root < 0 && !d_all_words) return STL_EINVAL;
  if (fault_now()) return STL_ERCCL;
  mark_gather_start(s);
  ncclResult_t r;
  if (root < 0)
    r = g_rccl.AllGather(d_words, d_all_words, words_per_rank, ncclUint64, g_pcomm, s);
  else
    r = g_rccl.Gather(d_words, d_all_words, words_per_rank, ncclUint64, root, g_pcomm, s);
  // a nonblocking communicator may answer ncclInProgress; one that fails or
  // times out here is unusable: aborted and forgotten
  const int rc = rccl_settle(g_pcomm, r);
  if (rc) pcomm_abort_locked();
  return rc;
}

int stl_bitmap_gatherv_device(const uint64_t* d_words, size_t nwords, uint64_t* d_all_words,
                              const uint64_t* word_offsets, int root, void* stream) {
  std::lock_guard<std::mutex> lk(g_pcomm_mu);
  if (!g_pcomm) return STL_ERCCL;
  if (!word_offsets || root < 0 || root >= g_pcomm_ranks) return STL_EINVAL;
  int me = 0;
  STL_RCCL_TRY(g_rccl.CommUserRank(g_pcomm, &me));
  const int g = g_pcomm_ranks;
  for (int r = 0; r < g; ++r)
    if (word_offsets[r + 1] < word_offsets[r]) return STL_EINVAL;
  if (word_offsets[me + 1] - word_offsets[me] != nwords || (nwords && !d_words)) return STL_EINVAL;
  if (me == root && !d_all_words) return STL_EINVAL;
  hipStream_t s = static_cast<hipStream_t>(stream);
  // the root's own slice: a device copy; every other non-empty slice: one
  // send / recv pair at its word offset, all in one group
  if (me == root && nwords)
    STL_TRY(hipMemcpyAsync(d_all_words + word_offsets[me], d_words, nwords * 8, hipMemcpyDeviceToDevice, s));
  mark_gather_start(s);
  STL_RCCL_TRY(g_rccl.GroupStart());
  int rc = STL_OK;
  if (me != root) {
    if (nwords && g_rccl.Send(d_words, nwords, ncclUint64, root, g_pcomm, s) != ncclSuccess) rc = STL_ERCCL;
  } else {
    for (int r = 0; r < g; ++r) {
      const size_t w = word_offsets[r + 1] - word_offsets[r];
      if (r == root || w == 0) continue;
      if (g_rccl.Recv(d_all_words + word_offsets[r], w, ncclUint64, r, g_pcomm, s) != ncclSuccess) rc = STL_ERCCL;
    }
  }
  const int erc = rccl_settle(g_pcomm, g_rccl.GroupEnd());
  if (erc) pcomm_abort_locked();  // failed or timed out: the communicator is unusable
  return rc ? rc : erc;
}

}  // extern "C"
