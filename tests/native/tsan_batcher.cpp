// ThreadSanitizer driver for the request aggregator (stl_batcher.cpp), built
// with g++ -fsanitize=thread by tests/test_sanitizers.py.  The batch entry
// points it calls are stubbed here: mode "enodev" returns STL_ENODEV (the path
// a GPU-less host takes), mode "bits" returns a deterministic bitmap (accept
// iff sig[0] is even; serialized transactions deferred iff blob[0] == 0xFF), so
// the test can check that every request completes exactly once with its own
// verdict while 6 submitter threads (stellard's JobQueue default,
// JobQueue.cpp:223-236), a flusher and the worker race.
#include <atomic>
#include <cstdio>
#include <cstring>
#include <thread>
#include <vector>

#include "../../include/stl.h"

static int g_mode = 0;  // 0 enodev, 1 bits
static std::atomic<long> g_calls{0};

extern "C" int stl_ed25519_verify_batch(const uint8_t* sig, const uint8_t*, const uint8_t*, size_t n, uint8_t* bm,
                                        uint32_t) {
  g_calls++;
  if (g_mode == 0) return STL_ENODEV;
  std::memset(bm, 0, (n + 7) / 8);
  for (size_t i = 0; i < n; ++i)
    if ((sig[64 * i] & 1) == 0) bm[i >> 3] |= (uint8_t)(1u << (i & 7));
  return STL_OK;
}

extern "C" int stl_tx_blob_verify_batch(const uint8_t* blobs, const uint64_t* off, const uint32_t* len, size_t n,
                                        uint8_t* bm, uint8_t* status, uint8_t*, uint32_t) {
  g_calls++;
  if (g_mode == 0) return STL_ENODEV;
  std::memset(bm, 0, (n + 7) / 8);
  for (size_t i = 0; i < n; ++i) {
    const uint8_t b0 = len[i] ? blobs[off[i]] : 0;
    status[i] = b0 == 0xFF ? STL_TX_DEFERRED : STL_TX_OK;
    if (b0 != 0xFF && (b0 & 1) == 0) bm[i >> 3] |= (uint8_t)(1u << (i & 7));
  }
  return STL_OK;
}

#include "../../stellard_amd/csrc/stl_batcher.cpp"

struct Slot {
  std::atomic<int> count{0};
  std::atomic<int> verdict{-99};
  int expect = 0;
};

static void done(void* ctx, int v) {
  Slot* s = static_cast<Slot*>(ctx);
  s->verdict.store(v);
  s->count.fetch_add(1);
}

int main(int argc, char** argv) {
  g_mode = (argc > 1 && std::strcmp(argv[1], "bits") == 0) ? 1 : 0;
  const int kThreads = 6, kPer = 1500;
  std::vector<Slot> slots(kThreads * kPer);
  stl_batcher* b = stl_batcher_create(97, 300, 0);
  if (!b) return 2;
  std::vector<std::thread> th;
  for (int t = 0; t < kThreads; ++t) {
    th.emplace_back([&, t] {
      for (int i = 0; i < kPer; ++i) {
        Slot& s = slots[t * kPer + i];
        uint8_t sig[64] = {0}, msg[32] = {0}, pk[32] = {0};
        const uint8_t v = (uint8_t)(t * 31 + i);
        if (i % 4 == 3) {
          uint8_t blob[150];
          std::memset(blob, v, sizeof blob);
          s.expect = g_mode == 0 ? STL_ENODEV
                                 : (v == 0xFF ? STL_VERDICT_DEFER : ((v & 1) ? STL_VERDICT_REJECT : STL_VERDICT_ACCEPT));
          if (stl_batcher_submit_tx(b, blob, sizeof blob, done, &s) != STL_OK) std::abort();
        } else {
          sig[0] = v;
          s.expect = g_mode == 0 ? STL_ENODEV : ((v & 1) ? STL_VERDICT_REJECT : STL_VERDICT_ACCEPT);
          if (stl_batcher_submit(b, sig, msg, pk, done, &s) != STL_OK) std::abort();
        }
        if (i % 500 == 499) stl_batcher_flush(b);
      }
    });
  }
  std::thread flusher([&] {
    for (int k = 0; k < 20; ++k) {
      stl_batcher_flush(b);
      std::this_thread::yield();
    }
  });
  for (auto& x : th) x.join();
  flusher.join();
  stl_batcher_flush(b);
  uint64_t sub = 0, comp = 0, batches = 0;
  stl_batcher_stats(b, &sub, &comp, &batches);
  stl_batcher_destroy(b);
  int bad = 0;
  for (auto& s : slots)
    if (s.count.load() != 1 || s.verdict.load() != s.expect) ++bad;
  std::printf("mode=%s submitted=%llu completed=%llu batches=%llu device_calls=%ld bad=%d\n", g_mode ? "bits" : "enodev",
              (unsigned long long)sub, (unsigned long long)comp, (unsigned long long)batches, g_calls.load(), bad);
  return bad == 0 && sub == slots.size() && comp == slots.size() ? 0 : 1;
}
