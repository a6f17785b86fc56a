// stl_api.cpp -- host side of libstl: the extern "C" boundary declared in
// include/stl.h.  Owns devices, streams, workspaces and staging buffers; has
// no CPU verification path (a device failure returns < 0 and the caller --
// stellard -- falls back to libsodium, as SURVEY.md section 8b requires).
//
// Threading: stellard calls verify concurrently from JobQueue workers
// (JobQueue.cpp:217-243).  Every device has a mutex that serialises the host
// batch entry points on that device; the device-resident entry points key
// their workspace by (device, stream) so concurrent streams never share one.
#include <hip/hip_runtime.h>

#include <algorithm>
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

#define STL_TRY(expr)                        \
  do {                                       \
    hipError_t e_ = (expr);                  \
    if (e_ != hipSuccess) return STL_EHIP;   \
  } while (0)

struct DevBuf {
  void* p = nullptr;
  size_t cap = 0;
  int ensure(size_t bytes) {
    if (bytes <= cap) return STL_OK;
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
    if (hipMalloc(&p, bytes) != hipSuccess) return STL_ENOMEM;
    cap = bytes;
    return STL_OK;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
  }
};

struct Device {
  int ordinal = 0;
  int cus = 0;
  uint32_t grid = 0;  // resident workgroups for the verify kernel
  hipStream_t stream = nullptr;  // kernels of the host batch API
  hipStream_t copy = nullptr;    // its host-to-device copies (overlap the previous chunk's kernels)
  std::mutex mu;
  DevBuf ws, sig, msg, pk, bitmap, pre, off, len, ctr, txid, status, wide;
  std::map<hipStream_t, std::unique_ptr<DevBuf>> stream_ws;   // device-resident API
  std::map<hipStream_t, std::unique_ptr<DevBuf>> stream_ctr;  // tx-hash work counter
  std::mutex ws_mu;
};

std::mutex g_mu;
std::vector<std::unique_ptr<Device>> g_devs;
bool g_init = false;

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
  STL_TRY(hipStreamCreateWithFlags(&d.stream, hipStreamNonBlocking));
  STL_TRY(hipStreamCreateWithFlags(&d.copy, hipStreamNonBlocking));
  // wide base tables for [e]B (7.3 MB), built once on the device
  int rc = d.wide.ensure(stl::kWideTableBytes);
  if (rc) return rc;
  STL_TRY(stl::launch_wide_table(static_cast<uint4*>(d.wide.p), d.stream));
  STL_TRY(hipStreamSynchronize(d.stream));
  return STL_OK;
}

int ensure_init() {
  if (g_init) return STL_OK;
  return stl_init(nullptr);
}

// Workspace for (device, stream) pairs used by the device-resident API.
int stream_workspace(Device& d, hipStream_t s, uint4** ws) {
  std::lock_guard<std::mutex> lk(d.ws_mu);
  auto& slot = d.stream_ws[s];
  if (!slot) slot.reset(new DevBuf());
  int rc = slot->ensure(stl::verify_ws_bytes(d.grid));
  if (rc) return rc;
  *ws = static_cast<uint4*>(slot->p);
  return STL_OK;
}

// Work-queue workspace for (device, stream) of the device-resident hash
// kernels (counter + longest-first order, stl::hash_queue_bytes(n)).
int stream_queue(Device& d, hipStream_t s, size_t n, uint32_t** qws) {
  std::lock_guard<std::mutex> lk(d.ws_mu);
  auto& slot = d.stream_ctr[s];
  if (!slot) slot.reset(new DevBuf());
  int rc = slot->ensure(stl::hash_queue_bytes(n));
  if (rc) return rc;
  *qws = static_cast<uint32_t*>(slot->p);
  return STL_OK;
}

// tx-hash grid: 8 workgroups per CU (the kernel pulls preimages from a counter)
uint32_t hash_grid(const Device& d) { return (uint32_t)d.cus * 8u; }

uint32_t grid_for(const Device& d, size_t n) {
  const size_t tiles = (n + stl::kBlock - 1) / stl::kBlock;
  return (uint32_t)std::max<size_t>(1, std::min<size_t>(tiles, d.grid));
}

// Contiguous 64-aligned shard of [0, n) for device r of g.
void shard(size_t n, int r, int g, size_t* lo, size_t* hi) {
  const size_t words = (n + 63) / 64;
  const size_t per = (words + g - 1) / g;
  *lo = std::min(n, (size_t)r * per * 64);
  *hi = std::min(n, (size_t)(r + 1) * per * 64);
}

// ---- host batch API: chunked copy/compute pipeline ----
// A shard is processed in chunks of kPipeChunk signatures (a multiple of 64,
// so every chunk starts on a bitmap word).  Chunk c's inputs are copied on
// d.copy while chunk c-1's kernels run on d.stream; an event orders each
// chunk's kernels after its copy.  Device buffers hold the whole shard, so no
// buffer is reused while a kernel may still read it.  Variable-length bytes
// (preimages, blobs) are copied up to a watermark: chunk c copies
// [watermark, max end of its rows), which is the whole contiguous range when
// offsets ascend and stays correct for any order (rows below the watermark
// were copied by an earlier chunk).
constexpr size_t kPipeChunk = (size_t)1 << 18;

struct Pipeline {
  Device& d;
  std::vector<hipEvent_t> ev;
  explicit Pipeline(Device& dev) : d(dev) {}
  ~Pipeline() {
    for (hipEvent_t e : ev) (void)hipEventDestroy(e);
  }
  // Make d.stream wait for everything issued on d.copy so far.
  int join_copy() {
    hipEvent_t e;
    STL_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    ev.push_back(e);
    STL_TRY(hipEventRecord(e, d.copy));
    STL_TRY(hipStreamWaitEvent(d.stream, e, 0));
    return STL_OK;
  }
};

// Rebased offsets of rows [lo, hi) and the byte range they span.
int rebase(const uint64_t* off, const uint32_t* len, size_t lo, size_t hi, std::vector<uint64_t>& roff,
           std::vector<uint64_t>& row_end, uint64_t* base_out, uint64_t* bytes_out) {
  const size_t n = hi - lo;
  const uint64_t base = off[lo];
  uint64_t end = base;
  roff.resize(n);
  row_end.resize(n);
  for (size_t i = 0; i < n; ++i) {
    if (off[lo + i] < base) return STL_EINVAL;
    roff[i] = off[lo + i] - base;
    row_end[i] = roff[i] + len[lo + i];
    end = std::max<uint64_t>(end, off[lo + i] + len[lo + i]);
  }
  *base_out = base;
  *bytes_out = end - base;
  return STL_OK;
}

// Copy the bytes rows [c0, c1) need that are not on the device yet.
int copy_rows(Pipeline& pl, uint8_t* dst, const uint8_t* src, const std::vector<uint64_t>& row_end, size_t c0,
              size_t c1, uint64_t* watermark) {
  uint64_t need = *watermark;
  for (size_t i = c0; i < c1; ++i) need = std::max(need, row_end[i]);
  if (need > *watermark)
    STL_TRY(hipMemcpyAsync(dst + *watermark, src + *watermark, need - *watermark, hipMemcpyHostToDevice, pl.d.copy));
  *watermark = need;
  return STL_OK;
}

// Verify one shard [lo, hi) on device d, synchronously; writes the host bitmap
// bytes [lo/8, ceil(hi/8)).  msg32 == nullptr means tx mode (preimages).
int run_shard(Device& d, const uint8_t* sig, const uint8_t* msg32, const uint8_t* pk, const uint8_t* pre,
              const uint64_t* off, const uint32_t* len, size_t lo, size_t hi, uint8_t* bitmap, uint32_t policy) {
  const size_t n = hi - lo;
  if (n == 0) return STL_OK;
  std::lock_guard<std::mutex> lk(d.mu);
  STL_TRY(hipSetDevice(d.ordinal));
  int rc;
  const size_t words = (n + 63) / 64;
  if ((rc = d.ws.ensure(stl::verify_ws_bytes(d.grid))) || (rc = d.sig.ensure(n * 64)) ||
      (rc = d.msg.ensure(n * 32)) || (rc = d.pk.ensure(n * 32)) || (rc = d.bitmap.ensure(words * 8)))
    return rc;
  std::vector<uint64_t> roff, row_end;
  uint64_t base = 0, bytes = 0, mark = 0;
  if (!msg32) {
    if ((rc = rebase(off, len, lo, hi, roff, row_end, &base, &bytes))) return rc;
    if ((rc = d.pre.ensure(bytes + 4)) || (rc = d.off.ensure(n * 8)) || (rc = d.len.ensure(n * 4)) ||
        (rc = d.ctr.ensure(stl::hash_queue_bytes(std::min(n, kPipeChunk)))))
      return rc;
    STL_TRY(hipMemcpyAsync(d.off.p, roff.data(), n * 8, hipMemcpyHostToDevice, d.copy));
    STL_TRY(hipMemcpyAsync(d.len.p, len + lo, n * 4, hipMemcpyHostToDevice, d.copy));
  }
  Pipeline pl(d);
  uint8_t* dsig = static_cast<uint8_t*>(d.sig.p);
  uint8_t* dmsg = static_cast<uint8_t*>(d.msg.p);
  uint8_t* dpk = static_cast<uint8_t*>(d.pk.p);
  for (size_t c0 = 0; c0 < n; c0 += kPipeChunk) {
    const size_t c1 = std::min(n, c0 + kPipeChunk), cn = c1 - c0;
    STL_TRY(hipMemcpyAsync(dsig + 64 * c0, sig + 64 * (lo + c0), cn * 64, hipMemcpyHostToDevice, d.copy));
    STL_TRY(hipMemcpyAsync(dpk + 32 * c0, pk + 32 * (lo + c0), cn * 32, hipMemcpyHostToDevice, d.copy));
    if (msg32) {
      STL_TRY(hipMemcpyAsync(dmsg + 32 * c0, msg32 + 32 * (lo + c0), cn * 32, hipMemcpyHostToDevice, d.copy));
    } else if ((rc = copy_rows(pl, static_cast<uint8_t*>(d.pre.p), pre + base, row_end, c0, c1, &mark))) {
      return rc;
    }
    if ((rc = pl.join_copy())) return rc;
    if (!msg32)
      STL_TRY(stl::launch_tx_hash(static_cast<uint8_t*>(d.pre.p), static_cast<uint64_t*>(d.off.p) + c0,
                                  static_cast<uint32_t*>(d.len.p) + c0, (uint32_t)cn, dmsg + 32 * c0,
                                  static_cast<uint32_t*>(d.ctr.p), hash_grid(d), d.stream));
    STL_TRY(stl::launch_verify(dsig + 64 * c0, dmsg + 32 * c0, dpk + 32 * c0, (uint32_t)cn,
                               static_cast<uint64_t*>(d.bitmap.p) + c0 / 64, policy, static_cast<uint4*>(d.ws.p),
                               grid_for(d, cn), false, static_cast<const uint4*>(d.wide.p), d.stream));
  }
  std::vector<uint8_t> host_words(words * 8);
  STL_TRY(hipMemcpyAsync(host_words.data(), d.bitmap.p, words * 8, hipMemcpyDeviceToHost, d.stream));
  STL_TRY(hipStreamSynchronize(d.stream));
  // lo is a multiple of 64, so the shard starts on a byte boundary
  std::memcpy(bitmap + lo / 8, host_words.data(), (n + 7) / 8);
  return STL_OK;
}

// Serialized-transaction shard [lo, hi) on device d: canonical pass, hashes,
// verify; writes the host bitmap bytes and, when asked, status and tx ids.
int run_blob_shard(Device& d, const uint8_t* blobs, const uint64_t* off, const uint32_t* len, size_t lo, size_t hi,
                   uint8_t* bitmap, uint8_t* status, uint8_t* txid, uint32_t policy) {
  const size_t n = hi - lo;
  if (n == 0) return STL_OK;
  std::lock_guard<std::mutex> lk(d.mu);
  STL_TRY(hipSetDevice(d.ordinal));
  int rc;
  const size_t words = (n + 63) / 64;
  std::vector<uint64_t> roff, row_end;
  uint64_t base = 0, bytes = 0, mark = 0;
  if ((rc = rebase(off, len, lo, hi, roff, row_end, &base, &bytes))) return rc;
  if ((rc = d.ws.ensure(stl::verify_ws_bytes(d.grid))) || (rc = d.sig.ensure(n * 64)) ||
      (rc = d.msg.ensure(n * 32)) || (rc = d.pk.ensure(n * 32)) || (rc = d.bitmap.ensure(words * 8)) ||
      (rc = d.pre.ensure(bytes + 4)) || (rc = d.off.ensure(n * 8)) || (rc = d.len.ensure(n * 4)) ||
      (rc = d.ctr.ensure(stl::hash_queue_bytes(std::min(n, kPipeChunk)))) || (rc = d.status.ensure(n)) ||
      (txid && (rc = d.txid.ensure(n * 32))))
    return rc;
  Pipeline pl(d);
  STL_TRY(hipMemcpyAsync(d.off.p, roff.data(), n * 8, hipMemcpyHostToDevice, d.copy));
  STL_TRY(hipMemcpyAsync(d.len.p, len + lo, n * 4, hipMemcpyHostToDevice, d.copy));
  uint8_t* dsig = static_cast<uint8_t*>(d.sig.p);
  uint8_t* dmsg = static_cast<uint8_t*>(d.msg.p);
  uint8_t* dpk = static_cast<uint8_t*>(d.pk.p);
  uint8_t* dtxid = txid ? static_cast<uint8_t*>(d.txid.p) : nullptr;
  for (size_t c0 = 0; c0 < n; c0 += kPipeChunk) {
    const size_t c1 = std::min(n, c0 + kPipeChunk), cn = c1 - c0;
    if ((rc = copy_rows(pl, static_cast<uint8_t*>(d.pre.p), blobs + base, row_end, c0, c1, &mark))) return rc;
    if ((rc = pl.join_copy())) return rc;
    STL_TRY(stl::launch_tx_blob(static_cast<uint8_t*>(d.pre.p), static_cast<uint64_t*>(d.off.p) + c0,
                                static_cast<uint32_t*>(d.len.p) + c0, (uint32_t)cn, dmsg + 32 * c0, dsig + 64 * c0,
                                dpk + 32 * c0, dtxid ? dtxid + 32 * c0 : nullptr,
                                static_cast<uint8_t*>(d.status.p) + c0, static_cast<uint32_t*>(d.ctr.p),
                                hash_grid(d), d.stream));
    STL_TRY(stl::launch_verify(dsig + 64 * c0, dmsg + 32 * c0, dpk + 32 * c0, (uint32_t)cn,
                               static_cast<uint64_t*>(d.bitmap.p) + c0 / 64, policy, static_cast<uint4*>(d.ws.p),
                               grid_for(d, cn), false, static_cast<const uint4*>(d.wide.p), d.stream));
  }
  std::vector<uint8_t> host_words(words * 8);
  STL_TRY(hipMemcpyAsync(host_words.data(), d.bitmap.p, words * 8, hipMemcpyDeviceToHost, d.stream));
  if (status) STL_TRY(hipMemcpyAsync(status + lo, d.status.p, n, hipMemcpyDeviceToHost, d.stream));
  if (txid) STL_TRY(hipMemcpyAsync(txid + 32 * lo, d.txid.p, n * 32, hipMemcpyDeviceToHost, d.stream));
  STL_TRY(hipStreamSynchronize(d.stream));
  std::memcpy(bitmap + lo / 8, host_words.data(), (n + 7) / 8);
  return STL_OK;
}

int run_batch(const uint8_t* sig, const uint8_t* msg32, const uint8_t* pk, const uint8_t* pre, const uint64_t* off,
              const uint32_t* len, size_t n, uint8_t* bitmap, uint32_t flags) {
  if (n == 0) return STL_OK;
  if (!sig || !pk || !bitmap || (!msg32 && (!pre || !off || !len))) return STL_EINVAL;
  if (flags & ~(STL_POLICY_MASK | STL_REQUIRE_S_LT_L | STL_FULL_LENGTH)) return STL_EINVAL;
  int rc = ensure_init();
  if (rc) return rc;
  const uint32_t policy = stl::kernel_mode(flags);
  const int g = (int)g_devs.size();
  if (g == 0) return STL_ENODEV;
  // one kernel launch handles up to 2^32-64 signatures per shard
  const size_t kMaxShard = (size_t)1 << 31;
  int gg = (int)std::max<size_t>((size_t)g, (n + kMaxShard - 1) / kMaxShard);
  std::vector<int> rcs(gg, STL_OK);
  std::vector<std::thread> th;
  for (int r = 0; r < gg; ++r) {
    size_t lo, hi;
    shard(n, r, gg, &lo, &hi);
    Device& d = *g_devs[r % g];
    if (gg == 1) {
      rcs[r] = run_shard(d, sig, msg32, pk, pre, off, len, lo, hi, bitmap, policy);
    } else {
      th.emplace_back([&, r, lo, hi]() { rcs[r] = run_shard(*g_devs[r % g], sig, msg32, pk, pre, off, len, lo, hi, bitmap, policy); });
    }
  }
  for (auto& t : th) t.join();
  for (int r : rcs)
    if (r) return r;
  return STL_OK;
}

}  // namespace

extern "C" {

int stl_init(const stl_config* cfg) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (g_init) return STL_OK;
  int count = 0;
  if (hipGetDeviceCount(&count) != hipSuccess || count <= 0) return STL_ENODEV;
  int first = 0, want = count;
  if (cfg) {
    if (cfg->struct_size != sizeof(stl_config)) return STL_EINVAL;
    first = cfg->first_device;
    if (cfg->device_count > 0) want = cfg->device_count;
  }
  if (const char* env = std::getenv("STL_DEVICES")) want = std::max(1, std::atoi(env));
  if (first < 0 || first >= count) return STL_EINVAL;
  want = std::min(want, count - first);
  int prev = 0;
  (void)hipGetDevice(&prev);
  for (int i = 0; i < want; ++i) {
    std::unique_ptr<Device> d(new Device());
    d->ordinal = first + i;
    int rc = setup_device(*d);
    if (rc) {
      (void)hipSetDevice(prev);
      g_devs.clear();
      return rc;
    }
    g_devs.push_back(std::move(d));
  }
  (void)hipSetDevice(prev);
  g_init = true;
  return STL_OK;
}

void stl_shutdown(void) {
  std::lock_guard<std::mutex> lk(g_mu);
  for (auto& d : g_devs) {
    std::lock_guard<std::mutex> dl(d->mu);
    (void)hipSetDevice(d->ordinal);
    (void)hipStreamSynchronize(d->stream);
    for (DevBuf* b : {&d->ws, &d->sig, &d->msg, &d->pk, &d->bitmap, &d->pre, &d->off, &d->len, &d->ctr, &d->txid,
                      &d->status, &d->wide})
      b->release();
    for (auto& kv : d->stream_ws) kv.second->release();
    for (auto& kv : d->stream_ctr) kv.second->release();
    (void)hipStreamSynchronize(d->copy);
    (void)hipStreamDestroy(d->stream);
    (void)hipStreamDestroy(d->copy);
  }
  g_devs.clear();
  g_init = false;
}

int stl_device_count(void) {
  std::lock_guard<std::mutex> lk(g_mu);
  return (int)g_devs.size();
}

const char* stl_version(void) { return "stl 0.1.0 (gfx950, abi 1)"; }

const char* stl_strerror(int rc) {
  switch (rc) {
    case STL_OK: return "ok";
    case STL_EINVAL: return "invalid argument";
    case STL_ENODEV: return "no gfx950 device";
    case STL_ENOMEM: return "out of memory";
    case STL_EHIP: return "HIP runtime error";
    default: return "unknown error";
  }
}

int stl_ed25519_verify_batch(const uint8_t* sig, const uint8_t* msg, const uint8_t* pk, size_t n,
                             uint8_t* accept_bitmap, uint32_t flags) {
  if (n && !msg) return STL_EINVAL;
  return run_batch(sig, msg, pk, nullptr, nullptr, nullptr, n, accept_bitmap, flags);
}

int stl_tx_verify_batch(const uint8_t* preimages, const uint64_t* offset, const uint32_t* len, const uint8_t* sig,
                        const uint8_t* pk, size_t n, uint8_t* accept_bitmap, uint32_t flags) {
  return run_batch(sig, nullptr, pk, preimages, offset, len, n, accept_bitmap, flags);
}

int stl_tx_blob_verify_batch(const uint8_t* blobs, const uint64_t* offset, const uint32_t* len, size_t n,
                             uint8_t* accept_bitmap, uint8_t* status, uint8_t* tx_id, uint32_t flags) {
  if (n == 0) return STL_OK;
  if (!blobs || !offset || !len || !accept_bitmap) return STL_EINVAL;
  if (flags & ~(STL_POLICY_MASK | STL_REQUIRE_S_LT_L | STL_FULL_LENGTH)) return STL_EINVAL;
  int rc = ensure_init();
  if (rc) return rc;
  const uint32_t policy = stl::kernel_mode(flags);
  const int g = (int)g_devs.size();
  if (g == 0) return STL_ENODEV;
  const size_t kMaxShard = (size_t)1 << 31;
  const int gg = (int)std::max<size_t>((size_t)g, (n + kMaxShard - 1) / kMaxShard);
  std::vector<int> rcs(gg, STL_OK);
  std::vector<std::thread> th;
  for (int r = 0; r < gg; ++r) {
    size_t lo, hi;
    shard(n, r, gg, &lo, &hi);
    if (gg == 1) {
      rcs[r] = run_blob_shard(*g_devs[0], blobs, offset, len, lo, hi, accept_bitmap, status, tx_id, policy);
    } else {
      th.emplace_back([&, r, lo, hi]() {
        rcs[r] = run_blob_shard(*g_devs[r % g], blobs, offset, len, lo, hi, accept_bitmap, status, tx_id, policy);
      });
    }
  }
  for (auto& t : th) t.join();
  for (int r : rcs)
    if (r) return r;
  return STL_OK;
}

int stl_ed25519_verify_detached(const uint8_t* sig, const uint8_t* m, unsigned long long mlen, const uint8_t* pk) {
  if (!sig || !pk || (mlen && !m)) return STL_EINVAL;
  if (mlen == 32) {
    uint8_t bit = 0;
    int rc = stl_ed25519_verify_batch(sig, m, pk, 1, &bit, STL_POLICY_SODIUM_1_0_18);
    if (rc) return rc;
    return (bit & 1) ? 0 : -1;
  }
  // arbitrary-length message: k = H(R||A||m) mod L on the device, then verify
  int rc = ensure_init();
  if (rc) return rc;
  Device& d = *g_devs[0];
  std::lock_guard<std::mutex> lk(d.mu);
  STL_TRY(hipSetDevice(d.ordinal));
  if ((rc = d.ws.ensure(stl::verify_ws_bytes(d.grid))) || (rc = d.sig.ensure(64)) || (rc = d.pk.ensure(32)) ||
      (rc = d.msg.ensure(32)) || (rc = d.bitmap.ensure(8)) || (rc = d.pre.ensure(mlen ? mlen : 1)) ||
      (rc = d.off.ensure(16)))
    return rc;
  hipStream_t s = d.stream;
  const uint64_t hostmeta[2] = {0, mlen};
  STL_TRY(hipMemcpyAsync(d.sig.p, sig, 64, hipMemcpyHostToDevice, s));
  STL_TRY(hipMemcpyAsync(d.pk.p, pk, 32, hipMemcpyHostToDevice, s));
  if (mlen) STL_TRY(hipMemcpyAsync(d.pre.p, m, mlen, hipMemcpyHostToDevice, s));
  STL_TRY(hipMemcpyAsync(d.off.p, hostmeta, 16, hipMemcpyHostToDevice, s));
  uint64_t* meta = static_cast<uint64_t*>(d.off.p);
  STL_TRY(stl::launch_hram_var(static_cast<uint8_t*>(d.sig.p), static_cast<uint8_t*>(d.pk.p),
                               static_cast<uint8_t*>(d.pre.p), meta, meta + 1, 1, static_cast<uint8_t*>(d.msg.p), s));
  STL_TRY(stl::launch_verify(static_cast<uint8_t*>(d.sig.p), static_cast<uint8_t*>(d.msg.p),
                             static_cast<uint8_t*>(d.pk.p), 1, static_cast<uint64_t*>(d.bitmap.p),
                             STL_POLICY_SODIUM_1_0_18, static_cast<uint4*>(d.ws.p), 1, true,
                             static_cast<const uint4*>(d.wide.p), s));
  uint64_t word = 0;
  STL_TRY(hipMemcpyAsync(&word, d.bitmap.p, 8, hipMemcpyDeviceToHost, s));
  STL_TRY(hipStreamSynchronize(s));
  return (word & 1) ? 0 : -1;
}

int stl_ed25519_verify_batch_device(const uint8_t* d_sig, const uint8_t* d_msg, const uint8_t* d_pk, size_t n,
                                    uint64_t* d_bitmap_words, uint32_t flags, void* stream) {
  if (n == 0) return STL_OK;
  if (!d_sig || !d_msg || !d_pk || !d_bitmap_words) return STL_EINVAL;
  if (flags & ~(STL_POLICY_MASK | STL_REQUIRE_S_LT_L | STL_FULL_LENGTH)) return STL_EINVAL;
  if (n > 0xffffffc0ull) return STL_EINVAL;
  int rc = ensure_init();
  if (rc) return rc;
  const int di = current_device_index();
  if (di < 0) return STL_ENODEV;
  Device& d = *g_devs[di];
  hipStream_t s = static_cast<hipStream_t>(stream);
  uint4* ws = nullptr;
  if ((rc = stream_workspace(d, s, &ws))) return rc;
  STL_TRY(stl::launch_verify(d_sig, d_msg, d_pk, (uint32_t)n, d_bitmap_words, stl::kernel_mode(flags), ws,
                             grid_for(d, n), false, static_cast<const uint4*>(d.wide.p), s));
  return STL_OK;
}

int stl_tx_hash_batch_device(const uint8_t* d_preimages, const uint64_t* d_offset, const uint32_t* d_len, size_t n,
                             uint8_t* d_msg, void* stream) {
  if (n == 0) return STL_OK;
  if (!d_preimages || !d_offset || !d_len || !d_msg || n > 0xffffffc0ull) return STL_EINVAL;
  int rc = ensure_init();
  if (rc) return rc;
  const int di = current_device_index();
  if (di < 0) return STL_ENODEV;
  Device& d = *g_devs[di];
  hipStream_t s = static_cast<hipStream_t>(stream);
  uint32_t* ctr = nullptr;
  if ((rc = stream_queue(d, s, n, &ctr))) return rc;
  STL_TRY(stl::launch_tx_hash(d_preimages, d_offset, d_len, (uint32_t)n, d_msg, ctr, hash_grid(d), s));
  return STL_OK;
}

int stl_tx_blob_prepare_device(const uint8_t* d_blobs, const uint64_t* d_offset, const uint32_t* d_len, size_t n,
                               uint8_t* d_msg, uint8_t* d_sig, uint8_t* d_pk, uint8_t* d_tx_id, uint8_t* d_status,
                               void* stream) {
  if (n == 0) return STL_OK;
  if (!d_blobs || !d_offset || !d_len || !d_msg || !d_sig || !d_pk || !d_status || n > 0xffffffc0ull)
    return STL_EINVAL;
  int rc = ensure_init();
  if (rc) return rc;
  const int di = current_device_index();
  if (di < 0) return STL_ENODEV;
  Device& d = *g_devs[di];
  hipStream_t s = static_cast<hipStream_t>(stream);
  uint32_t* ctr = nullptr;
  if ((rc = stream_queue(d, s, n, &ctr))) return rc;
  STL_TRY(stl::launch_tx_blob(d_blobs, d_offset, d_len, (uint32_t)n, d_msg, d_sig, d_pk, d_tx_id, d_status, ctr,
                              hash_grid(d), s));
  return STL_OK;
}

int stl_ed25519_sign_batch_device(const uint8_t* d_seed, const uint8_t* d_msg, size_t n, uint8_t* d_pk,
                                  uint8_t* d_sig, void* stream) {
  if (n == 0) return STL_OK;
  if (!d_seed || !d_msg || !d_pk || !d_sig || n > 0xffffffc0ull) return STL_EINVAL;
  int rc = ensure_init();
  if (rc) return rc;
  const int di = current_device_index();
  if (di < 0) return STL_ENODEV;
  Device& d = *g_devs[di];
  hipStream_t s = static_cast<hipStream_t>(stream);
  uint4* ws = nullptr;
  if ((rc = stream_workspace(d, s, &ws))) return rc;
  STL_TRY(stl::launch_sign(d_seed, d_msg, (uint32_t)n, d_pk, d_sig, ws, grid_for(d, n), s));
  return STL_OK;
}

}  // extern "C"
