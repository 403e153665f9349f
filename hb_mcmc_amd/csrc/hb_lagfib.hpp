// hb_lagfib.hpp -- jump-ahead for glibc's rand() (random_r TYPE_3), host code.
//
// glibc's TYPE_3 generator is the additive lagged-Fibonacci recurrence
// r[k] = r[k-31] + r[k-3] (mod 2^32), rand() = r[k] >> 1.  It is linear over
// Z/2^32, so the state after J more outputs follows from the current window of
// 31 values by the polynomial x^J mod (x^31 - x^28 - 1): with
// x^J = sum_i c_i x^i, r[n + J] = sum_i c_i r[n + i].  The tempering-swap draws
// of one PT-MCMC iteration (ptmcmc, mcmc_wrapper2.c:768-817: two rand() per
// attempt, W attempts, always) therefore start at a known offset, and the
// schedule of any future iteration can be drawn independently of the others
// (hb_dsampler.hip's producer threads) -- bit for bit the sequence the
// reference's process-global rand() would give.
#pragma once
#include <stdint.h>
#include <string.h>

namespace hblf {

constexpr int kLag = 31;

// a <- a * b mod (x^31 - x^28 - 1), coefficients mod 2^32
inline void poly_mulmod(uint32_t* a, const uint32_t* b) {
  uint32_t t[2 * kLag - 1] = {0};
  for (int i = 0; i < kLag; ++i) {
    if (a[i] == 0) continue;
    for (int j = 0; j < kLag; ++j) t[i + j] += a[i] * b[j];
  }
  for (int m = 2 * kLag - 2; m >= kLag; --m) {  // x^m = x^(m-3) + x^(m-31)
    t[m - 3] += t[m];
    t[m - kLag] += t[m];
  }
  memcpy(a, t, sizeof(uint32_t) * kLag);
}

// c <- x^J mod (x^31 - x^28 - 1)
inline void poly_xpow(unsigned long long J, uint32_t* c) {
  uint32_t base[kLag] = {0}, acc[kLag] = {0};
  acc[0] = 1;
  base[1] = 1;  // x
  while (J) {
    if (J & 1ull) poly_mulmod(acc, base);
    J >>= 1;
    if (J) {
      uint32_t sq[kLag];
      memcpy(sq, base, sizeof sq);
      poly_mulmod(base, sq);
    }
  }
  memcpy(c, acc, sizeof acc);
}

// window w[0..30] = r[n .. n+30] -> r[n+J .. n+J+30], given c = x^J mod P
inline void window_jump(uint32_t* w, const uint32_t* cJ) {
  uint32_t c[kLag], out[kLag];
  memcpy(c, cJ, sizeof c);
  for (int i = 0; i < kLag; ++i) {
    uint32_t v = 0;
    for (int j = 0; j < kLag; ++j) v += c[j] * w[j];
    out[i] = v;
    // c <- x * c mod P: shift up; the x^31 coefficient folds into x^28 and x^0
    const uint32_t top = c[kLag - 1];
    for (int j = kLag - 1; j > 0; --j) c[j] = c[j - 1];
    c[0] = top;
    c[28] += top;
  }
  memcpy(w, out, sizeof out);
}

// sequential generator over a window (the continuation of glibc's stream)
struct Stream {
  uint32_t r[34];
  unsigned k;  // next index (mod 34 ring)
  explicit Stream(const uint32_t* w) {
    for (int i = 0; i < kLag; ++i) r[i] = w[i];
    k = kLag;
  }
  uint32_t next() {  // r[k] = r[k-31] + r[k-3]
    const uint32_t v = r[(k + 34 - 31) % 34] + r[(k + 34 - 3) % 34];
    r[k % 34] = v;
    ++k;
    return v;
  }
  int rand() { return (int)(next() >> 1); }
};

}  // namespace hblf
