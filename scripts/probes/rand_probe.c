/* rand_probe.c -- which part of the GPU stack calls glibc rand()/srand()?
 * The executable's definitions interpose the shared libraries' calls; each
 * call prints a short backtrace.  Diagnostic for the drop-in path (DESIGN.md
 * section 5, "glibc rand() for swaps"). */
#define _GNU_SOURCE
#include <dlfcn.h>
#include <execinfo.h>
#include <stdio.h>
#include <stdlib.h>

#include "../../include/hbmi.h"

static int armed = 0, shown = 0;
static void trace(const char *what) {
  if (!armed) return;
  if (shown++ > 1) { fprintf(stderr, "== %s\n", what); return; }
  void *bt[48];
  int n = backtrace(bt, 48);
  fprintf(stderr, "== %s called\n", what);
  backtrace_symbols_fd(bt, n, 2);
}
int rand(void) {
  trace("rand");
  static int (*real)(void);
  if (!real) real = (int (*)(void))dlsym(RTLD_NEXT, "rand");
  return real();
}
void srand(unsigned s) {
  trace("srand");
  static void (*real)(unsigned);
  if (!real) real = (void (*)(unsigned))dlsym(RTLD_NEXT, "srand");
  real(s);
}
long random(void) {
  trace("random");
  static long (*real)(void);
  if (!real) real = (long (*)(void))dlsym(RTLD_NEXT, "random");
  return real();
}
void srandom(unsigned s) {
  trace("srandom");
  static void (*real)(unsigned);
  if (!real) real = (void (*)(unsigned))dlsym(RTLD_NEXT, "srandom");
  real(s);
}

int main(void) {
  double t[64], f[64], s[64], p[21] = {0.3, 0.1, 0.3157, 0.4, 1.2, 0.5, 0.3, 0, 0, 0.16, 0.34, 0.16, 0.34,
                                        1, 1, 0, 0, 0, 0, 0.1, 1.0};
  for (int i = 0; i < 64; ++i) { t[i] = 0.05 * i; f[i] = 1.0; s[i] = 1e-3; }
  double mag[5] = {1000, 1, 1, 1, 1}, err[4] = {1e15, 1e15, 1e15, 1e15};
  fprintf(stderr, "-- hb_device_available (one-time runtime init, not traced): %d\n", hb_device_available());
  armed = 1;
  fprintf(stderr, "-- first loglikelihood\n");
  double v = loglikelihood(t, f, s, 64, p, mag, err);
  fprintf(stderr, "-- second loglikelihood\n");
  v += loglikelihood(t, f, s, 64, p, mag, err);
  fprintf(stderr, "-- done %g\n", v);
  armed = 0;
  return 0;
}
