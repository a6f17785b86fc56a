// ledger_close.cpp -- libstl from C++ the way stellard would call it
// (INTEGRATION.md sections 2, 4 and 4b), compiled against include/stl.h and
// linked with libstl.so only -- no Python, no HIP headers.
//
//   1. stl_init in place of / next to sodium_init (ripple_app.cpp:129-132);
//   2. the ledger-close pre-verify: one stl_tx_verify_batch over the signing
//      preimages of the whole set, setGood() for accepts only
//      (LedgerConsensus.cpp:1947-1968, 2101-2106; SerializedTransaction.h:124-127);
//   3. six JobQueue-style workers (JobQueue.cpp:223-236) handing single
//      signatures to the aggregator (stl_batcher_submit) and waiting for
//      their verdicts;
//   4. the error contract: rc < 0 means "run your own check", never a reject.
//
// Input file (written by tests/test_examples.py): u32 n, then n records of
// u32 len | preimage[len] | hash[32] | sig[64] | pk[32] (hash = the signing
// hash SHA512Half(preimage), which stellard has at hand per transaction).
// Output: one line per phase and the accept bitmap (one '0'/'1' per
// transaction) for the test to compare.
//
//   g++ -std=c++17 -O2 -I include examples/ledger_close.cpp -L stellard_amd -lstl
//       -Wl,-rpath,$PWD/stellard_amd -Wl,-rpath,/opt/rocm/lib -L/opt/rocm/lib -lamdhip64 -pthread
#include <atomic>
#include <condition_variable>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <thread>
#include <vector>

#include "stl.h"

namespace {

struct Tx {  // the parts of a SerializedTransaction the check uses
  std::vector<uint8_t> preimage;  // "STX\0" || signing fields (getSigningHash input)
  uint8_t hash[32], sig[64], pk[32];
  bool sig_good = false;  // mSigGood (SerializedTransaction.h:116-131)
  bool serial = false;    // left to the unchanged serial checkSign
};

bool read_set(const char* path, std::vector<Tx>& txs) {
  FILE* f = std::fopen(path, "rb");
  if (!f) return false;
  uint32_t n = 0;
  bool ok = std::fread(&n, 4, 1, f) == 1;
  for (uint32_t i = 0; ok && i < n; ++i) {
    Tx t;
    uint32_t len = 0;
    ok = std::fread(&len, 4, 1, f) == 1;
    t.preimage.resize(len);
    ok = ok && std::fread(t.preimage.data(), 1, len, f) == len && std::fread(t.hash, 1, 32, f) == 32 &&
         std::fread(t.sig, 1, 64, f) == 64 && std::fread(t.pk, 1, 32, f) == 32;
    txs.push_back(std::move(t));
  }
  std::fclose(f);
  return ok;
}

struct Waiter {  // a JobQueue worker waiting for its verdict
  std::mutex mu;
  std::condition_variable cv;
  int verdict = 0;
  bool done = false;
};

void on_verdict(void* ctx, int v) {
  Waiter* w = static_cast<Waiter*>(ctx);
  std::lock_guard<std::mutex> lk(w->mu);
  w->verdict = v;
  w->done = true;
  w->cv.notify_one();
}

}  // namespace

int main(int argc, char** argv) {
  if (argc < 2) return 2;
  std::vector<Tx> txs;
  if (!read_set(argv[1], txs)) return 3;
  const size_t n = txs.size();

  // 1. process init
  // stellard passes libsodium's crypto_sign_verify_detached as fallback_verify;
  // this example does not link libsodium, so single calls report device errors
  stl_config cfg = {sizeof(stl_config), /*device_count*/ 0, /*first_device*/ 0, /*flags*/ 0,
                    /*shards_per_device*/ 1, 0, /*fallback_verify*/ nullptr};
  const int init_rc = stl_init(&cfg);
  std::printf("stl_init %d (%s) devices %d %s\n", init_rc, stl_strerror(init_rc), stl_device_count(), stl_version());

  // 2. ledger-close pre-verify: one batch, accepts only
  std::vector<uint8_t> pre, sig(64 * n), pk(32 * n), bits((n + 7) / 8);
  std::vector<uint64_t> off(n);
  std::vector<uint32_t> len(n);
  for (size_t i = 0; i < n; ++i) {
    off[i] = pre.size();
    len[i] = (uint32_t)txs[i].preimage.size();
    pre.insert(pre.end(), txs[i].preimage.begin(), txs[i].preimage.end());
    std::memcpy(&sig[64 * i], txs[i].sig, 64);
    std::memcpy(&pk[32 * i], txs[i].pk, 32);
  }
  // a ledger's signers repeat: decode each distinct key once (STL_DEDUP_KEYS)
  const int rc = stl_tx_verify_batch(pre.data(), off.data(), len.data(), sig.data(), pk.data(), n, bits.data(),
                                     STL_POLICY_SODIUM_1_0_18 | STL_DEDUP_KEYS);
  size_t good = 0;
  for (size_t i = 0; i < n; ++i) {
    if (rc == STL_OK && ((bits[i >> 3] >> (i & 7)) & 1)) {
      txs[i].sig_good = true;  // setGood(): preCheck's checkSign becomes a cache hit
      ++good;
    } else {
      txs[i].serial = true;  // reject or device error: the serial path decides, as before
    }
  }
  std::printf("batch rc %d accepted %zu of %zu, %zu left to the serial checkSign\n", rc, good, n, n - good);

  // 3. six JobQueue workers verifying single signatures (verifySignature(hash,
  //    sig)) through the aggregator, each waiting for its verdict; every
  //    verdict must equal the batch's bit for the same transaction
  std::atomic<long> agree{0}, errors{0}, asked{0};
  if (rc == STL_OK) {
    stl_batcher* b = stl_batcher_create(1024, 500, STL_POLICY_SODIUM_1_0_18);
    std::vector<std::thread> workers;
    const size_t m = n < 600 ? n : 600;
    for (int w = 0; w < 6; ++w) {
      workers.emplace_back([&, w] {
        for (size_t i = w; i < m; i += 6) {
          Waiter wt;
          if (stl_batcher_submit(b, txs[i].sig, txs[i].hash, txs[i].pk, on_verdict, &wt) != STL_OK) {
            errors++;
            continue;
          }
          std::unique_lock<std::mutex> lk(wt.mu);
          wt.cv.wait(lk, [&] { return wt.done; });
          asked++;
          if (wt.verdict < 0) errors++;  // device error: libsodium would run here
          else if ((wt.verdict == STL_VERDICT_ACCEPT) == txs[i].sig_good) agree++;
        }
      });
    }
    for (auto& t : workers) t.join();
    stl_batcher_destroy(b);
  }
  std::printf("batcher asked %ld agree %ld errors %ld\n", asked.load(), agree.load(), errors.load());

  // 4. the bitmap for the test
  std::printf("bitmap ");
  for (size_t i = 0; i < n; ++i) std::putchar(txs[i].sig_good ? '1' : '0');
  std::printf("\n");
  stl_shutdown();
  return rc == STL_OK || rc == STL_ENODEV ? 0 : 1;
}
