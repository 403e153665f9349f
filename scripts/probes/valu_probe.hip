// valu_probe.hip -- experiment only (not shipped): fp64 VALU latency and
// per-SIMD throughput on gfx950, to size the ILP x waves the eval kernel
// needs.  Each wave runs CH independent chains of R dependent v_fma_f64
// (asm volatile, so the compiler keeps them); the kernel time over the
// number of fma issued per SIMD gives cycles per fma per SIMD.
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/valu_probe scripts/probes/valu_probe.hip
#include <hip/hip_runtime.h>
#include <stdio.h>

#define CHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

template <int CH, int OP>
__global__ __launch_bounds__(64) void probe(double* out, double a, double b, int reps, long long* clk) {
  double x[CH];
#pragma unroll
  for (int c = 0; c < CH; ++c) x[c] = threadIdx.x * 1e-3 + c;
  const long long t0 = clock64();
  for (int r = 0; r < reps; ++r) {
#pragma unroll
    for (int u = 0; u < 16; ++u) {
#pragma unroll
      for (int c = 0; c < CH; ++c) {
        if (OP == 0) asm volatile("v_fma_f64 %0, %1, %2, %0" : "+v"(x[c]) : "v"(a), "v"(b));
        else if (OP == 1) asm volatile("v_mul_f64 %0, %1, %0" : "+v"(x[c]) : "v"(a));
        else if (OP == 2) {  // 32-bit VALU on the low word
          int lo = __double2loint(x[c]);
          asm volatile("v_add_u32 %0, %0, %1" : "+v"(lo) : "v"(reps));
          x[c] = __hiloint2double(__double2hiint(x[c]), lo);
        } else if (OP == 3) asm volatile("v_rcp_f64 %0, %0" : "+v"(x[c]));
      }
    }
  }
  const long long t1 = clock64();
  double s = 0;
#pragma unroll
  for (int c = 0; c < CH; ++c) s += x[c];
  out[blockIdx.x * 64 + threadIdx.x] = s;
  if (threadIdx.x == 0) clk[blockIdx.x] = t1 - t0;
}

template <int CH, int OP>
static int run(const char* name, int waves_per_simd, double* d_out, long long* d_clk) {
  const int nblk = 1024 * waves_per_simd;  // 256 CU x 4 SIMD
  const int reps = 256;
  hipEvent_t e0, e1;
  CHK(hipEventCreate(&e0));
  CHK(hipEventCreate(&e1));
  hipLaunchKernelGGL((probe<CH, OP>), dim3(nblk), dim3(64), 0, 0, d_out, 1.0000001, 1e-9, reps, d_clk);
  CHK(hipDeviceSynchronize());
  CHK(hipEventRecord(e0));
  hipLaunchKernelGGL((probe<CH, OP>), dim3(nblk), dim3(64), 0, 0, d_out, 1.0000001, 1e-9, reps, d_clk);
  CHK(hipEventRecord(e1));
  CHK(hipEventSynchronize(e1));
  float ms = 0;
  CHK(hipEventElapsedTime(&ms, e0, e1));
  long long h[1];
  CHK(hipMemcpy(h, d_clk, sizeof(long long), hipMemcpyDeviceToHost));
  const double ops_per_wave = (double)reps * 16 * CH;
  // cycles at 2.4 GHz per op per SIMD (all waves of a SIMD share its VALU)
  const double cyc_simd = ms * 1e-3 * 2.4e9 / (ops_per_wave * waves_per_simd);
  printf("%-8s CH=%d waves/SIMD=%d: %.3f ms, %.2f cyc/op/SIMD, wave0 clock64 %.2f cyc/op (dependent chain = %.2f)\n", name,
         CH, waves_per_simd, ms, cyc_simd, (double)h[0] / ops_per_wave, (double)h[0] / (reps * 16.0));
  return 0;
}

int main() {
  double* d_out;
  long long* d_clk;
  CHK(hipMalloc(&d_out, 8 * 1024 * 64 * sizeof(double)));
  CHK(hipMalloc(&d_clk, 8 * 1024 * sizeof(long long)));
  for (int w : {1, 2, 4, 8}) {
    run<1, 0>("fma_f64", w, d_out, d_clk);
    run<2, 0>("fma_f64", w, d_out, d_clk);
    run<4, 0>("fma_f64", w, d_out, d_clk);
    run<8, 0>("fma_f64", w, d_out, d_clk);
  }
  for (int w : {1, 4}) {
    run<1, 1>("mul_f64", w, d_out, d_clk);
    run<8, 1>("mul_f64", w, d_out, d_clk);
    run<1, 2>("add_u32", w, d_out, d_clk);
    run<8, 2>("add_u32", w, d_out, d_clk);
    run<1, 3>("rcp_f64", w, d_out, d_clk);
    run<8, 3>("rcp_f64", w, d_out, d_clk);
  }
  return 0;
}
