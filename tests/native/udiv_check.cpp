// Host-side check of sgn::UDiv64 (csrc/sgn_internal.h) against the u64 division operator.
#include <cstdio>
#include <random>

#include "sgn_internal.h"

int main() {
  std::mt19937_64 rng(12345);
  const uint64_t fixed_d[] = {1, 2, 3, 5, 7, 10, 1000, 1000000, 999999, 1000001, 6000000,
                              (1ULL << 32) + 1, 0xFFFFFFFFFFFFFFFFULL, 0x8000000000000001ULL,
                              12345678901ULL};
  const uint64_t fixed_x[] = {0, 1, 2, 999999, 1000000, 0xFFFFFFFFFFFFFFFFULL,
                              0xFFFFFFFFFFFFFFFEULL, 0x8000000000000000ULL, 946684800000000000ULL};
  long bad = 0, n = 0;
  auto check = [&](uint64_t d, uint64_t x) {
    sgn::UDiv64 u;
    u.init(d);
    n++;
    if (u.div(x) != x / d) {
      if (bad++ < 10) printf("mismatch d=%llu x=%llu\n", (unsigned long long)d, (unsigned long long)x);
    }
  };
  for (uint64_t d : fixed_d)
    for (uint64_t x : fixed_x) check(d, x);
  for (int i = 0; i < 200000; i++) {
    const int bits = 1 + (int)(rng() % 64);
    uint64_t d = rng() >> (64 - bits);
    if (d == 0) d = 1;
    check(d, rng());
    check(d, rng() >> (rng() % 64));
  }
  printf("%ld checks, %ld bad\n", n, bad);
  return bad != 0;
}
