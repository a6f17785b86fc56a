// stl_batcher.cpp -- request aggregator over the batch entry points
// (where batches form in stellard).
//
// stellard checks signatures one transaction at a time from JobQueue workers
// (jtTRANSACTION jobs: PeerImp.cpp:64-73 -> NetworkOPs::processTransaction,
// NetworkOPs.cpp:298-320) and leaves a hook for batching unused
// (TxQueue::addEntryForSigCheck, TxQueue.h:32-33, TxQueue.cpp:32-46).  The
// aggregator is that hook's engine: any thread submits one request with a
// completion callback; one worker thread per aggregator collects requests and
// runs a device batch when max_batch are pending or the oldest has waited
// max_delay_us, then calls every request's callback with its verdict.
//
// Verdicts: STL_VERDICT_ACCEPT / STL_VERDICT_REJECT, STL_VERDICT_DEFER for a
// serialized transaction the device did not decide (its status
// STL_TX_DEFERRED), or a negative STL_E* code when the device batch failed --
// the caller then runs its own check (never a reject).  A batch starts when
// max_batch requests of one kind are pending or the OLDEST pending request has
// waited max_delay_us (each request keeps its arrival time, so leftovers from
// a full batch are not delayed again).  Callbacks run on the worker thread and
// must not call stl_batcher_flush / stl_batcher_destroy on their aggregator.
#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <cstring>
#include <deque>
#include <mutex>
#include <thread>
#include <vector>

#include "../../include/stl.h"

namespace {

using Clock = std::chrono::steady_clock;

struct SigReq {
  uint8_t sig[64], msg[32], pk[32];
  stl_verdict_fn fn;
  void* ctx;
  Clock::time_point arrival;
};

struct TxReq {
  std::vector<uint8_t> blob;
  stl_verdict_fn fn;
  void* ctx;
  Clock::time_point arrival;
};

}  // namespace

struct stl_batcher {
  uint32_t max_batch = 4096;
  std::chrono::microseconds max_delay{1000};
  uint32_t flags = 0;
  std::mutex mu;
  std::condition_variable cv_work, cv_done;
  std::deque<SigReq> sigs;
  std::deque<TxReq> txs;
  uint64_t submitted = 0, completed = 0, batches = 0;
  uint64_t flush_target = 0;  // flush() callers wait for completed >= this
  bool stop = false;
  std::thread worker;

  size_t pending() const { return sigs.size() + txs.size(); }
  bool flushing() const { return completed < flush_target; }
  // arrival of the oldest pending request (each queue is in arrival order)
  Clock::time_point oldest() const {
    if (sigs.empty()) return txs.front().arrival;
    if (txs.empty()) return sigs.front().arrival;
    return std::min(sigs.front().arrival, txs.front().arrival);
  }

  void run() {
    std::unique_lock<std::mutex> lk(mu);
    for (;;) {
      if (pending() == 0) {
        if (stop) return;
        cv_work.wait(lk, [&] { return stop || pending() > 0; });
        continue;
      }
      const bool full = sigs.size() >= max_batch || txs.size() >= max_batch;
      if (!full && !flushing() && !stop) {
        // deadline of the oldest pending request: requests left over from a
        // previous round keep their own arrival time
        const auto deadline = oldest() + max_delay;
        if (Clock::now() < deadline) {
          cv_work.wait_until(lk, deadline);
          continue;
        }
      }
      // take at most max_batch of each kind, oldest first; the rest stays
      const size_t ns = std::min<size_t>(sigs.size(), max_batch), nt = std::min<size_t>(txs.size(), max_batch);
      std::vector<SigReq> s(sigs.begin(), sigs.begin() + ns);
      std::vector<TxReq> t(std::make_move_iterator(txs.begin()), std::make_move_iterator(txs.begin() + nt));
      sigs.erase(sigs.begin(), sigs.begin() + ns);
      txs.erase(txs.begin(), txs.begin() + nt);
      lk.unlock();
      run_sigs(s);
      run_txs(t);
      lk.lock();
      completed += s.size() + t.size();
      batches += (s.empty() ? 0 : 1) + (t.empty() ? 0 : 1);
      cv_done.notify_all();
    }
  }

  void run_sigs(std::vector<SigReq>& s) {
    if (s.empty()) return;
    const size_t n = s.size();
    std::vector<uint8_t> sig(n * 64), msg(n * 32), pk(n * 32), bits((n + 7) / 8);
    for (size_t i = 0; i < n; ++i) {
      std::memcpy(&sig[64 * i], s[i].sig, 64);
      std::memcpy(&msg[32 * i], s[i].msg, 32);
      std::memcpy(&pk[32 * i], s[i].pk, 32);
    }
    const int rc = stl_ed25519_verify_batch(sig.data(), msg.data(), pk.data(), n, bits.data(), flags);
    for (size_t i = 0; i < n; ++i) {
      const int v = rc != STL_OK ? rc : ((bits[i >> 3] >> (i & 7)) & 1 ? STL_VERDICT_ACCEPT : STL_VERDICT_REJECT);
      s[i].fn(s[i].ctx, v);
    }
  }

  void run_txs(std::vector<TxReq>& t) {
    if (t.empty()) return;
    const size_t n = t.size();
    std::vector<uint64_t> off(n);
    std::vector<uint32_t> len(n);
    size_t total = 0;
    for (size_t i = 0; i < n; ++i) {
      off[i] = total;
      len[i] = (uint32_t)t[i].blob.size();
      total += t[i].blob.size();
    }
    std::vector<uint8_t> buf(total + 16), bits((n + 7) / 8), status(n);
    for (size_t i = 0; i < n; ++i)
      if (!t[i].blob.empty()) std::memcpy(&buf[off[i]], t[i].blob.data(), t[i].blob.size());
    const int rc =
        stl_tx_blob_verify_batch(buf.data(), off.data(), len.data(), n, bits.data(), status.data(), nullptr, flags);
    for (size_t i = 0; i < n; ++i) {
      int v;
      if (rc != STL_OK) v = rc;
      else if (status[i] == STL_TX_DEFERRED) v = STL_VERDICT_DEFER;
      else v = ((bits[i >> 3] >> (i & 7)) & 1) ? STL_VERDICT_ACCEPT : STL_VERDICT_REJECT;
      t[i].fn(t[i].ctx, v);
    }
  }

  void note_arrival() {
    ++submitted;
    if (pending() == 1 || sigs.size() >= max_batch || txs.size() >= max_batch) cv_work.notify_one();
  }
};

extern "C" {

stl_batcher* stl_batcher_create(uint32_t max_batch, uint32_t max_delay_us, uint32_t flags) {
  if (max_batch == 0 || (flags & ~(STL_POLICY_MASK | STL_REQUIRE_S_LT_L | STL_FULL_LENGTH | STL_DEDUP_KEYS | STL_ONE_LANE))) return nullptr;
  stl_batcher* b = new (std::nothrow) stl_batcher();
  if (!b) return nullptr;
  b->max_batch = max_batch;
  b->max_delay = std::chrono::microseconds(max_delay_us);
  b->flags = flags;
  b->worker = std::thread([b] { b->run(); });
  return b;
}

int stl_batcher_submit(stl_batcher* b, const uint8_t* sig, const uint8_t* msg32, const uint8_t* pk,
                       stl_verdict_fn fn, void* ctx) {
  if (!b || !sig || !msg32 || !pk || !fn) return STL_EINVAL;
  SigReq r;
  std::memcpy(r.sig, sig, 64);
  std::memcpy(r.msg, msg32, 32);
  std::memcpy(r.pk, pk, 32);
  r.fn = fn;
  r.ctx = ctx;
  r.arrival = Clock::now();
  std::lock_guard<std::mutex> lk(b->mu);
  if (b->stop) return STL_EINVAL;
  b->sigs.push_back(r);
  b->note_arrival();
  return STL_OK;
}

int stl_batcher_submit_tx(stl_batcher* b, const uint8_t* blob, size_t len, stl_verdict_fn fn, void* ctx) {
  if (!b || (len && !blob) || !fn || len > 0xffffffffu) return STL_EINVAL;
  TxReq r;
  r.blob.assign(blob, blob + len);
  r.fn = fn;
  r.ctx = ctx;
  r.arrival = Clock::now();
  std::lock_guard<std::mutex> lk(b->mu);
  if (b->stop) return STL_EINVAL;
  b->txs.push_back(std::move(r));
  b->note_arrival();
  return STL_OK;
}

void stl_batcher_flush(stl_batcher* b) {
  if (!b) return;
  std::unique_lock<std::mutex> lk(b->mu);
  const uint64_t target = b->submitted;
  b->flush_target = std::max(b->flush_target, target);  // cleared by itself once completed >= target
  b->cv_work.notify_one();
  b->cv_done.wait(lk, [&] { return b->completed >= target; });
}

void stl_batcher_stats(stl_batcher* b, uint64_t* submitted, uint64_t* completed, uint64_t* batches) {
  if (!b) return;
  std::lock_guard<std::mutex> lk(b->mu);
  if (submitted) *submitted = b->submitted;
  if (completed) *completed = b->completed;
  if (batches) *batches = b->batches;
}

void stl_batcher_destroy(stl_batcher* b) {
  if (!b) return;
  {
    std::lock_guard<std::mutex> lk(b->mu);
    b->stop = true;
    b->cv_work.notify_one();
  }
  b->worker.join();
  delete b;
}

}  // extern "C"
