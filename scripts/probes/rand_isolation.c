/* rand_isolation.c -- the caller's glibc rand() sequence must not notice
 * libhbmi: srand(77), 5 draws, then the drop-in entry points (first call =
 * HIP runtime + code-object load) from the main thread and 4 pthreads, then
 * 35 more draws, compared with an undisturbed srand(77) sequence.
 * Exit 0 = identical.  Run by tests/test_capi.py (gpu). */
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>

#include "../../include/hbmi.h"

#define N 96
static double P[21] = {0.3, 0.1, 0.3157, 0.4, 1.2, 0.5, 0.3, 0, 0, 0.16, 0.34, 0.16, 0.34,
                       1, 1, 0, 0, 0, 0, 0.1, 1.0};

static void *work(void *arg) {
  const int k = (int)(long)arg;
  double t[N], f[N], s[N], m[N];
  double mag[5] = {1000, 1, 1, 1, 1}, err[4] = {1e15, 1e15, 1e15, 1e15};
  for (int i = 0; i < N; ++i) { t[i] = 0.031 * i + k; f[i] = 1.0 + 1e-4 * k; s[i] = 1e-3; }
  double v = loglikelihood(t, f, s, N, P, mag, err);
  calc_light_curve(t, N, P, m);
  return (void *)(long)(v == v && m[0] == m[0]);
}

int main(void) {
  int expected[40], bad = 0;
  srand(77);
  for (int i = 0; i < 40; ++i) expected[i] = rand();
  srand(77);
  for (int i = 0; i < 5; ++i) bad |= rand() != expected[i];
  work((void *)0);
  double a[N];
  for (int i = 0; i < N; ++i) a[i] = (double)((i * 37) % N);
  quickSort(a, 0, N - 1);
  for (int i = 0; i < N; ++i) a[i] = (double)((i * 53) % N);
  (void)partition(a, 0, N - 1);
  remove_median(a, 0, N);
  (void)_getT(0.2);
  (void)eclipse_area(1.0, 0.5, 0.7);
  pthread_t th[4];
  for (long k = 0; k < 4; ++k) pthread_create(&th[k], NULL, work, (void *)(k + 1));
  for (int k = 0; k < 4; ++k) pthread_join(th[k], NULL);
  for (int i = 5; i < 40; ++i) {
    const int r = rand();
    if (r != expected[i]) { bad = 1; fprintf(stderr, "draw %d: %d != %d\n", i, r, expected[i]); }
  }
  printf(bad ? "MISMATCH\n" : "rand sequence preserved\n");
  return bad;
}
