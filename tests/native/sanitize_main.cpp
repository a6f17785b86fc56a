// sanitize_main.cpp -- TEST HARNESS ONLY.  An executable that runs the host
// build of the device verify code (hostemu.cpp: the functions the gfx950
// kernels run) and the C oracle (oracle/stl_oracle*.c) over vector files,
// built with AddressSanitizer + UndefinedBehaviorSanitizer by
// tests/test_sanitizers.py (the reference CI only ran
// under MALLOC_CHECK_=3, .travis.yml:45-49).
//
//   sanitize_main VECTORS BLOBS
//   VECTORS: records sig(64) msg(32) pk(32) expected_1_0_18(1) expected_1_0_0(1)
//   BLOBS:   records len(u32 LE) bytes(len)
// Exit status = number of disagreements (0 = the device code, the oracle and
// the expected bits agree everywhere); any sanitizer report aborts.
#include <cstdio>
#include <cstdlib>
#include <vector>

#define HOSTEMU_SANITIZE_SUBSET  // the verify path and the blob pass only
#include "hostemu.cpp"

extern "C" {
#include "../../oracle/stl_oracle.h"
}

static std::vector<uint8_t> slurp(const char* path) {
  std::vector<uint8_t> v;
  FILE* f = std::fopen(path, "rb");
  if (!f) return v;
  uint8_t buf[1 << 16];
  size_t k;
  while ((k = std::fread(buf, 1, sizeof buf, f)) > 0) v.insert(v.end(), buf, buf + k);
  std::fclose(f);
  return v;
}

int main(int argc, char** argv) {
  if (argc < 3) return 100;
  const std::vector<uint8_t> vec = slurp(argv[1]), blobs = slurp(argv[2]);
  const size_t rec = 64 + 32 + 32 + 2, n = vec.size() / rec;
  if (n == 0 || vec.size() % rec) return 101;
  std::vector<uint8_t> sig(n * 64), msg(n * 32), pk(n * 32);
  for (size_t i = 0; i < n; ++i) {
    std::memcpy(&sig[64 * i], &vec[rec * i], 64);
    std::memcpy(&msg[32 * i], &vec[rec * i + 64], 32);
    std::memcpy(&pk[32 * i], &vec[rec * i + 96], 32);
  }
  long bad = 0;
  for (uint32_t policy = 0; policy < 2; ++policy) {
    for (int mode = 0; mode < 2; ++mode) {  // 0: half-size + fallback (the kernels), 1: full length
      std::vector<uint8_t> bm((n + 7) / 8);
      const uint64_t viol = hostemu_verify_batch_mode(sig.data(), msg.data(), pk.data(), n, bm.data(), policy, mode,
                                                      nullptr);
      if (viol) {
        std::printf("limb-bound violations: %llu\n", (unsigned long long)viol);
        ++bad;
      }
      for (size_t i = 0; i < n; ++i) {
        const int got = (bm[i >> 3] >> (i & 7)) & 1;
        const int exp = vec[rec * i + 128 + policy];
        const int orc = oracle_verify(&sig[64 * i], &msg[32 * i], 32, &pk[32 * i], policy) == 0;
        if (got != exp || orc != exp) {
          if (bad < 20) std::printf("vector %zu policy %u mode %d: device %d oracle %d expected %d\n", i, policy, mode,
                                    got, orc, exp);
          ++bad;
        }
      }
    }
  }
  // serialized transactions: the device's canonical-form pass + splice vs the
  // oracle's re-serialisation
  size_t pos = 0, nb = 0;
  long compared = 0;
  std::vector<uint8_t> sg(1 << 21), fl(1 << 21);
  while (pos + 4 <= blobs.size()) {
    uint32_t len;
    std::memcpy(&len, &blobs[pos], 4);
    pos += 4;
    if (pos + len > blobs.size()) return 102;
    std::vector<uint8_t> b(blobs.begin() + pos, blobs.begin() + pos + len);
    b.resize(len + 4, 0);  // the kernels' tail padding
    pos += len;
    ++nb;
    for (uint32_t kind = 0; kind < 2; ++kind) {
      uint32_t st;
      uint8_t m[32], id[32];
      hostemu_signed_blob(kind, b.data(), len, &st, m, id);
      oracle_txinfo info;
      const int rc = oracle_signed_blob(kind, b.data(), len, sg.data(), fl.data(), sg.size(), &info);
      // compared where the device decided and the reference can construct the
      // object (template checks, e.g. a transaction's TransactionType, are the
      // caller's: stl.h)
      if (st == stl::kTxDeferred || rc != 0) continue;
      uint8_t h[64];
      ++compared;
      oracle_sha512(sg.data(), info.signing_len, h);
      if ((st == stl::kTxOk && std::memcmp(h, m, 32) != 0) ||
          (st == stl::kTxOk) != (info.pk_len == 32 && info.sig_len == 64)) {
        if (bad < 40) std::printf("blob %zu kind %u: device status %u, oracle rc %d\n", nb, kind, st, rc);
        ++bad;
      }
    }
  }
  std::printf("vectors %zu blobs %zu compared %ld disagreements %ld\n", n, nb, compared, bad);
  return bad > 250 ? 250 : (int)bad;
}
