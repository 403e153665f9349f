// rcp_probe.hip -- accuracy of the v_rcp_f64 seed and of fast_rcp/fast_div
// with 0/1/2 Newton refinements, on denominators in [0.005, 2] (the Kepler
// and orbit denominators 1 - e cos E).  Diagnostic for hb_math.hpp.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>

__global__ void k(const double* x, const double* n, double* out, int m) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= m) return;
  const double d = x[i];
  double y0 = __builtin_amdgcn_rcp(d);
  double y1 = fma(fma(-d, y0, 1.0), y0, y0);
  double y2 = fma(fma(-d, y1, 1.0), y1, y1);
  const double a = n[i];
  double q0 = a * y0; q0 = fma(fma(-d, q0, a), y0, q0);
  double q1 = a * y1; q1 = fma(fma(-d, q1, a), y1, q1);
  double q2 = a * y2; q2 = fma(fma(-d, q2, a), y2, q2);
  out[6 * i + 0] = y0; out[6 * i + 1] = y1; out[6 * i + 2] = y2;
  out[6 * i + 3] = q0; out[6 * i + 4] = q1; out[6 * i + 5] = q2;
}

int main() {
  const int m = 1 << 22;
  double *x = (double*)malloc(8 * m), *n = (double*)malloc(8 * m), *o = (double*)malloc(48 * (size_t)m);
  unsigned long long s = 88172645463325252ull;
  for (int i = 0; i < m; ++i) {
    s ^= s << 13; s ^= s >> 7; s ^= s << 17;
    x[i] = 0.005 + 1.995 * ((s >> 11) * (1.0 / 9007199254740992.0));
    s ^= s << 13; s ^= s >> 7; s ^= s << 17;
    n[i] = -1.0 + 2.0 * ((s >> 11) * (1.0 / 9007199254740992.0));
  }
  double *dx, *dn, *dout;
  hipMalloc(&dx, 8 * m); hipMalloc(&dn, 8 * m); hipMalloc(&dout, 48 * (size_t)m);
  hipMemcpy(dx, x, 8 * m, hipMemcpyHostToDevice);
  hipMemcpy(dn, n, 8 * m, hipMemcpyHostToDevice);
  k<<<m / 256, 256>>>(dx, dn, dout, m);
  hipMemcpy(o, dout, 48 * (size_t)m, hipMemcpyDeviceToHost);
  double worst[6] = {0};
  long exact[6] = {0};
  for (int i = 0; i < m; ++i) {
    const double r = 1.0 / x[i], q = n[i] / x[i];
    for (int j = 0; j < 6; ++j) {
      const double want = j < 3 ? r : q;
      const double got = o[6 * i + j];
      const double ulp = nextafter(fabs(want), INFINITY) - fabs(want);
      const double e = fabs(got - want) / ulp;
      if (e > worst[j]) worst[j] = e;
      exact[j] += got == want;
    }
  }
  const char* names[6] = {"rcp seed", "rcp +1 NR", "rcp +2 NR", "div(seed)", "div(+1 NR)", "div(+2 NR)"};
  for (int j = 0; j < 6; ++j)
    printf("%-12s max err %.3g ulp, correctly rounded %.4f%%\n", names[j], worst[j], 100.0 * exact[j] / m);
  return 0;
}
