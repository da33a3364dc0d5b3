// Does the Infinity Cache (MALL, 256 MiB) absorb the UPOLS intermediates?
// Memory-only stand-ins for the three engine kernels run chunk by chunk over
// 2^25 samples (the stereo bench step):
//   kx: in (8 B/sample, HBM, fresh) -> X (16 B/sample, a reused chunk buffer)
//   km: X -> Z (16 B/sample each, reused chunk buffers)
//   kz: Z -> out (8 B/sample, HBM, fresh)
// With whole-step chunks X and Z are 537 MB each (HBM round trips); with small
// chunks they are rewritten while still resident in the MALL.  Prints the
// time per step and the HBM-equivalent rate (80 B/sample).
//   hipcc --offload-arch=gfx950 -O3 tools/chain_probe.hip -o tools/chain_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                     \
  do {                                                            \
    hipError_t e = (x);                                           \
    if (e != hipSuccess) {                                        \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e)); \
      std::exit(1);                                               \
    }                                                             \
  } while (0)

// each thread moves 16 B units: out has RO units per input unit
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

int main() {
  const long S = 1L << 25;  // samples per step
  double2 *in, *out, *X, *Z;
  CK(hipMalloc(&in, S * 8));
  CK(hipMalloc(&out, S * 8));
  CK(hipMalloc(&X, S * 16));
  CK(hipMalloc(&Z, S * 16));
  CK(hipMemset(in, 0, S * 8));
  CK(hipMemset(X, 0, S * 16));
  CK(hipMemset(Z, 0, S * 16));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int grid = 8192;
  for (long c : {S, S / 2, S / 4, S / 8, S / 16, S / 32, S / 64}) {
    const long units = c / 2;  // 16-B units of input per chunk
    auto step = [&]() {
      for (long o = 0; o < S; o += c) {
        // kx: 1 unit in -> 2 units out; km: 2 -> 2 (as two 1 -> 1 passes of 2 units); kz: 2 -> 1
        hipLaunchKernelGGL((k_mix<1, 2>), dim3(grid), dim3(256), 0, 0, in + o / 2, X, units);
        hipLaunchKernelGGL((k_mix<1, 1>), dim3(grid), dim3(256), 0, 0, X, Z, 2 * units);
        hipLaunchKernelGGL((k_mix<2, 1>), dim3(grid), dim3(256), 0, 0, Z, out + o / 2, units);
      }
    };
    for (int w = 0; w < 3; ++w) step();
    CK(hipDeviceSynchronize());
    const int reps = 10;
    CK(hipEventRecord(e0));
    for (int w = 0; w < reps; ++w) step();
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    const double us = ms * 1e3 / reps;
    std::printf("chunk %9ld samples (X = Z = %6.1f MB): %8.1f us per step, %6.2f TB/s at 80 B/sample\n", c,
                c * 16 / 1e6, us, 80.0 * S / (us * 1e-6) / 1e12);
  }
  return 0;
}
