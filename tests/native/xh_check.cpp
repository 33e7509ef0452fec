// Host-side check of the round-edge message words (csrc/sgn_internal.h xh_*): every 8-byte word
// of a granule carries the round's tag, so a granule whose halves come from different writes
// (a torn 16-byte store, the previous message of the same round parity, a zeroed inbox) is
// never accepted, and an accepted granule gives back the value written.
#include <cstdio>
#include <random>

#include "sgn_internal.h"

int main() {
  std::mt19937_64 rng(7);
  long bad = 0, n = 0;
  auto fail = [&](const char* what, uint64_t v, uint64_t t) {
    if (bad++ < 10) printf("%s: v=%llx tag=%llu\n", what, (unsigned long long)v, (unsigned long long)t);
  };
  const uint64_t vs[] = {0, 1, 0xFFFFFFFFull, 0x100000000ull, ~0ull, sgn::INVALID, sgn::EMU_MAX};
  for (int i = 0; i < 200000; i++) {
    const uint64_t v = i < 7 ? vs[i] : rng() >> (rng() % 64);
    const uint64_t t = 1 + (rng() % 5000000);  // global round number + 1 (never 0)
    const uint64_t w = i < 7 ? vs[(i + 3) % 7] : rng();
    n++;
    const uint64_t lo = sgn::xh_lo(v, t), hi = sgn::xh_hi(v, t);
    if (!sgn::xh_ok(lo, hi, t) || sgn::xh_val(lo, hi) != v) fail("round trip", v, t);
    // the same parity buffer two rounds ago, and a zeroed inbox: never taken for this round
    const uint64_t plo = sgn::xh_lo(w, t - 2 + (t < 2 ? 4 : 0)), phi = sgn::xh_hi(w, t - 2 + (t < 2 ? 4 : 0));
    if (sgn::xh_ok(lo, phi, t) || sgn::xh_ok(plo, hi, t) || sgn::xh_ok(plo, phi, t)) fail("stale half", v, t);
    if (sgn::xh_ok(0, 0, t) || sgn::xh_ok(lo, 0, t) || sgn::xh_ok(0, hi, t)) fail("zeroed half", v, t);
  }
  printf("%ld checks, %ld bad\n", n, bad);
  return bad != 0;
}
