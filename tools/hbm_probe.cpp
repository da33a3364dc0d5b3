// Achievable-bandwidth probe for the read/write mixes of the UPOLS kernels
// (DESIGN.md §2 roofline): copy 1:1, expand 1:2 (K1: 8 B in, 16 B out per
// sample) and reduce 2:1 (K3: 16 B in, 8 B out), 16-B accesses per lane,
// grid-stride, 1 GiB of traffic per launch.  Prints GB/s per mix.
//   hipcc --offload-arch=gfx950 -O3 tools/hbm_probe.cpp -o tools/hbm_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e = (x);                                                    \
    if (e != hipSuccess) {                                                 \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));          \
      std::exit(1);                                                        \
    }                                                                      \
  } while (0)

// out[RO*i + r] = in[RI*i + s] mixing: each lane moves RI loads and RO stores of 16 B
template <int RI, int RO>
__global__ __launch_bounds__(256) void k_mix(const double2* __restrict__ in, double2* __restrict__ out, long n) {
  const long stride = (long)gridDim.x * 256;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += stride) {
    double2 acc = make_double2(0.0, 0.0);
#pragma unroll
    for (int s = 0; s < RI; ++s) {
      const double2 v = in[(long)s * n + i];
      acc.x += v.x;
      acc.y += v.y;
    }
#pragma unroll
    for (int r = 0; r < RO; ++r) out[(long)r * n + i] = make_double2(acc.x + r, acc.y);
  }
}

template <int RI, int RO>
void run(const char* name, double2* a, double2* b, long units, int grid) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int w = 0; w < 3; ++w) hipLaunchKernelGGL((k_mix<RI, RO>), dim3(grid), dim3(256), 0, 0, a, b, units);
  CK(hipEventRecord(e0));
  const int reps = 10;
  for (int w = 0; w < reps; ++w) hipLaunchKernelGGL((k_mix<RI, RO>), dim3(grid), dim3(256), 0, 0, a, b, units);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, e0, e1));
  const double bytes = (double)units * 16.0 * (RI + RO);
  std::printf("%-24s grid %6d  %8.1f us  %7.1f GB/s\n", name, grid, ms * 1e3 / reps, bytes / (ms * 1e-3 / reps) / 1e9);
}

int main() {
  const long units = (1L << 30) / 16 / 3;  // ~1 GiB of traffic for the 1:2 / 2:1 mixes
  double2 *a, *b;
  CK(hipMalloc(&a, units * 16 * 2));
  CK(hipMalloc(&b, units * 16 * 2));
  CK(hipMemset(a, 0, units * 16 * 2));
  for (int grid : {2048, 8192, 32768}) {
    run<1, 1>("copy 1:1", a, b, units, grid);
    run<1, 2>("expand 1:2 (K1-like)", a, b, units, grid);
    run<2, 1>("reduce 2:1 (K3-like)", a, b, units, grid);
    run<1, 0>("read only", a, b, units, grid);
    run<0, 1>("write only", a, b, units, grid);
  }
  return 0;
}
