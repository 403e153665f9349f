// launch_probe.hip -- experiment only (not shipped): the per-launch cost of
// back-to-back kernels on one stream at the C2 geometry (256 workgroups x
// 1024 threads, 160 KB of dynamic LDS each), with and without dirty global
// memory left behind by the waves (the eval kernel's deferred cadence queue
// writes ~16 MB per launch that it reads back itself), and at the one-wave
// geometry (4096 x 64 threads).  Each variant: 20 warm-up launches, then 2000
// launches between two events; prints microseconds per launch.
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/launch_probe scripts/probes/launch_probe.hip
#include <hip/hip_runtime.h>
#include <stdio.h>

#define CHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

typedef double d2v __attribute__((ext_vector_type(2)));

// MODE 0: exit at once; 1: every wave writes `per_wave` bytes (16 B per lane
// per store) to its own region and reads them back (plain stores); 2: the
// same with nontemporal stores
template <int MODE>
__global__ void probe(d2v* buf, int per_wave, double* sink) {
  extern __shared__ unsigned char lds[];
  if (MODE == 0) return;
  const int lane = threadIdx.x & 63;
  const long wave = (long)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  d2v* q = buf + wave * (per_wave / 16);
  const int n = per_wave / 16;
  for (int i = lane; i < n; i += 64) {
    const d2v v = {(double)i, (double)wave};
    if (MODE == 1) q[i] = v;
    else __builtin_nontemporal_store(v, q + i);
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  double s = 0.0;
  for (int i = lane; i < n; i += 64) s += q[i].x;
  if (s == -1.0) sink[0] = s;  // never: keeps the reads
  (void)lds;
}

template <int MODE>
static int run(const char* name, int grid, int block, size_t lds, d2v* buf, int per_wave, double* sink) {
  auto k = probe<MODE>;
  CHK(hipFuncSetAttribute(reinterpret_cast<const void*>(k), hipFuncAttributeMaxDynamicSharedMemorySize, 163840));
  hipEvent_t a, b;
  CHK(hipEventCreate(&a));
  CHK(hipEventCreate(&b));
  for (int i = 0; i < 20; ++i) hipLaunchKernelGGL(k, dim3(grid), dim3(block), lds, 0, buf, per_wave, sink);
  CHK(hipEventRecord(a, 0));
  const int reps = 2000;
  for (int i = 0; i < reps; ++i) hipLaunchKernelGGL(k, dim3(grid), dim3(block), lds, 0, buf, per_wave, sink);
  CHK(hipEventRecord(b, 0));
  CHK(hipEventSynchronize(b));
  float ms = 0.f;
  CHK(hipEventElapsedTime(&ms, a, b));
  printf("%-44s grid %5d x %4d lds %6zu  per-wave %6d B  %8.3f us/launch\n", name, grid, block, lds, per_wave,
         ms * 1e3 / reps);
  return 0;
}

int main() {
  d2v* buf = nullptr;
  double* sink = nullptr;
  CHK(hipMalloc(&buf, (size_t)4096 * 16384));
  CHK(hipMalloc(&sink, 64));
  int rc = 0;
  rc |= run<0>("empty, C2 fused geometry", 256, 1024, 155648, buf, 0, sink);
  rc |= run<1>("queue 3.8 KB/wave, C2 fused geometry", 256, 1024, 155648, buf, 3840, sink);
  rc |= run<1>("queue 16 KB/wave, C2 fused geometry", 256, 1024, 155648, buf, 16384, sink);
  rc |= run<2>("queue 3.8 KB/wave nontemporal, C2 fused", 256, 1024, 155648, buf, 3840, sink);
  rc |= run<0>("empty, one-wave geometry", 4096, 64, 9216, buf, 0, sink);
  rc |= run<1>("queue 3.8 KB/wave, one-wave geometry", 4096, 64, 9216, buf, 3840, sink);
  rc |= run<0>("empty, 1 x 64", 1, 64, 0, buf, 0, sink);
  return rc;
}
