// tools/lattice_sim.cpp -- wave-level cost model of lattice_half's Lehmer loops (host build): per
// Build and run on the host:  hipcc -O2 -std=c++17 -o /tmp/lattice_sim tools/lattice_sim.cpp && /tmp/lattice_sim
// wave of 64 random k < L, rounds = max over lanes, inner iterations per
// round = max over the lanes still active.  Policy cap C: at most C inner
// steps per round.
#include <cstdio>
#include <cstdint>
#include <random>
#include <vector>
#include <algorithm>
#include "../stellard_amd/csrc/stl_lattice.h"
using namespace stl;

// instrumented copy of lat_lehmer_round: returns the inner iterations run
// by this lane (certified steps + the failing check), cap limits them
static int round_count(uint32_t rl[8], uint32_t rs[8], uint32_t tl[5], uint32_t ts[5], bool& tl_neg, bool& ok, int cap) {
  double x, y, thr;
  lat_lead(x, y, thr, rl, rs);
  double m00 = 1.0, m01 = 0.0, m10 = 0.0, m11 = 1.0;
  bool go = true, odd = false;
  int iters = 0;
  for (int it = 0; it < cap; ++it) {
    ++iters;
    double q = floor(x / y);
    double r = fma(-q, y, x);
    if (r < 0.0) { q -= 1.0; r += y; } else if (r >= y) { q += 1.0; r -= y; }
    const double M1 = fmax(m11, m01), M2 = fmax(m10, m00);
    const double n00 = fma(m00, q, m01), n10 = fma(m10, q, m11);
    const double M2n = fmax(n00, n10);
    const bool step = y > 0.0 && r >= 0.0 && r < y && r >= fma(q, M2, M1) && y - r >= fma(q + 1.0, M2, M1) &&
                      M2n < 4294967296.0;
    if (!step) break;
    m01 = m00; m00 = n00; m11 = m10; m10 = n10; x = y; y = r; odd = !odd;
    if (r - M2n < thr) break;
  }
  if (m10 != 0.0) {
    const uint32_t u00 = (uint32_t)m00, u01 = (uint32_t)m01, u10 = (uint32_t)m10, u11 = (uint32_t)m11;
    uint32_t X[8], Y[8], TX[5], TY[5];
    bool bad = false;
    lat_comb(X, u11, rl, u01, rs, odd, bad);
    lat_comb(Y, u10, rl, u00, rs, !odd, bad);
    lat_madd2(TX, u11, tl, u01, ts, bad);
    lat_madd2(TY, u10, tl, u00, ts, bad);
    bad = bad || lat_ge(Y, X);
    ok = ok && !bad;
    for (int i = 0; i < 8; ++i) { rl[i] = X[i]; rs[i] = Y[i]; }
    for (int i = 0; i < 5; ++i) { tl[i] = TX[i]; ts[i] = TY[i]; }
    tl_neg = tl_neg != odd;
  } else {
    lat_step(rl, rs, tl, ts, ok);
    for (int i = 0; i < 8; ++i) std::swap(rl[i], rs[i]);
    for (int i = 0; i < 5; ++i) std::swap(tl[i], ts[i]);
    tl_neg = !tl_neg;
  }
  return iters;
}

static std::vector<int> lane(const uint32_t k[8], int cap) {
  uint32_t rl[8], rs[8], tl[5], ts[5];
  for (int i = 0; i < 8; ++i) { rl[i] = lat_N(i); rs[i] = k[i]; }
  for (int i = 0; i < 5; ++i) { tl[i] = 0; ts[i] = i == 0; }
  bool ok = true, tl_neg = true;
  std::vector<int> out;
  for (int round = 0; round < 128 && ok && lat_ge128(rs); ++round) out.push_back(round_count(rl, rs, tl, ts, tl_neg, ok, cap));
  return out;
}

int main() {
  std::mt19937_64 g(1);
  const int W = 2000;
  for (int cap : {64, 19, 18, 17, 16, 15}) {
    double wave_inner = 0, wave_rounds = 0, lane_inner = 0, lane_rounds = 0;
    for (int w = 0; w < W; ++w) {
      std::vector<std::vector<int>> L;
      for (int l = 0; l < 64; ++l) {
        uint32_t k[8];
        for (int i = 0; i < 8; ++i) k[i] = (uint32_t)g();
        k[7] &= 0x0fffffffu;  // < 2^252 ~ L
        L.push_back(lane(k, cap));
      }
      size_t R = 0;
      for (auto& v : L) { R = std::max(R, v.size()); lane_rounds += v.size(); for (int x : v) lane_inner += x; }
      wave_rounds += R;
      for (size_t r = 0; r < R; ++r) {
        int m = 0;
        for (auto& v : L) if (r < v.size()) m = std::max(m, v[r]);
        wave_inner += m;
      }
    }
    printf("cap %2d: wave inner %.1f rounds %.2f | lane avg inner %.1f rounds %.2f | inner waste %.0f%%\n", cap,
           wave_inner / W, wave_rounds / W, lane_inner / (W * 64.0), lane_rounds / (W * 64.0),
           100.0 * (1 - lane_inner / (W * 64.0) / (wave_inner / W)));
  }
}
