// hb_glibc_check.cpp -- host build of hb_glibc_math.hpp next to the system
// libm, for tests/test_glibc_math.py (test infrastructure: lib/libhbglibc_check.so).
//   fn 0: exp(x)   1: log(x)   2: pow(x, y)
#include <math.h>

#include "hb_glibc_math.hpp"

extern "C" {

// port values
void hbg_eval(int fn, const double* x, const double* y, long n, double* out) {
  for (long i = 0; i < n; ++i)
    out[i] = fn == 0 ? hbglibc::exp(x[i]) : fn == 1 ? hbglibc::log(x[i]) : hbglibc::pow(x[i], y[i]);
}

// libm values
void hbg_libm(int fn, const double* x, const double* y, long n, double* out) {
  for (long i = 0; i < n; ++i) out[i] = fn == 0 ? ::exp(x[i]) : fn == 1 ? ::log(x[i]) : ::pow(x[i], y[i]);
}

// number of arguments where the port and libm differ in any bit (NaN == NaN)
long hbg_check(int fn, const double* x, const double* y, long n, long* first_bad) {
  long bad = 0;
  *first_bad = -1;
  for (long i = 0; i < n; ++i) {
    const double a = fn == 0 ? hbglibc::exp(x[i]) : fn == 1 ? hbglibc::log(x[i]) : hbglibc::pow(x[i], y[i]);
    const double b = fn == 0 ? ::exp(x[i]) : fn == 1 ? ::log(x[i]) : ::pow(x[i], y[i]);
    const bool same = (a != a && b != b) || hbglibc::asuint64(a) == hbglibc::asuint64(b);
    if (!same) {
      if (*first_bad < 0) *first_bad = i;
      ++bad;
    }
  }
  return bad;
}
}

// ---- walls (hb_walls.hpp): fast-forwarded folds vs the plain loop ----
#include "hb_walls.hpp"

extern "C" {
void hbw_eval(int plain, const double* v, const double* lo, const double* hi, const double* fl, const double* fh,
              long n, double* out) {
  for (long i = 0; i < n; ++i)
    out[i] = plain ? hbwall::apply_wall_plain(v[i], lo[i], hi[i], fl[i], fh[i])
                   : hbwall::apply_wall(v[i], lo[i], hi[i], fl[i], fh[i]);
}
}
