// Microbenchmark: cycles per sample of the DF-II-T biquad recurrence
// (section.go:47-53, no FMA) in one wave, for K independent sections
// interleaved in the instruction stream (ILP), inputs in registers.
#include <hip/hip_runtime.h>
#include <cstdio>

template <int K>
__global__ void biq(double* out, const double* coef, int iters, long long* cyc) {
#pragma clang fp contract(off)
  double q[6];
  for (int i = 0; i < 6; ++i) q[i] = coef[i];
  double d0[K], d1[K], v[K];
  for (int k = 0; k < K; ++k) { d0[k] = 0; d1[k] = 0; v[k] = threadIdx.x * 1e-3 + k; }
  long long t0 = clock64();
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int s = 0; s < 8; ++s) {
#pragma unroll
      for (int k = 0; k < K; ++k) {
        const double x = v[k] * q[0];
        const double y = q[1] * x + d0[k];
        d0[k] = q[2] * x - q[4] * y + d1[k];
        d1[k] = q[3] * x - q[5] * y;
        v[k] = y * 0.5 + 1e-3;
      }
    }
  }
  long long t1 = clock64();
  double s = 0;
  for (int k = 0; k < K; ++k) s += v[k] + d0[k] + d1[k];
  out[threadIdx.x] = s;
  if (threadIdx.x == 0) *cyc = t1 - t0;
}

template <int K>
void run() {
  double *d, *c;
  long long* cy;
  hipMalloc(&d, 64 * 8);
  hipMalloc(&c, 6 * 8);
  hipMalloc(&cy, 8);
  double h[6] = {1.0, 0.2, 0.3, 0.1, -0.5, 0.25};
  hipMemcpy(c, h, 48, hipMemcpyHostToDevice);
  const int iters = 20000;
  hipLaunchKernelGGL(biq<K>, dim3(1), dim3(64), 0, 0, d, c, iters, cy);
  hipDeviceSynchronize();
  hipLaunchKernelGGL(biq<K>, dim3(1), dim3(64), 0, 0, d, c, iters, cy);
  long long v;
  hipMemcpy(&v, cy, 8, hipMemcpyDeviceToHost);
  printf("sections interleaved K=%d: %.1f cycles per sample per section-step, %.1f per sample for all K\n", K,
         (double)v / iters / 8 / K, (double)v / iters / 8);
}

int main() {
  run<1>();
  run<2>();
  run<4>();
  run<5>();
  run<8>();
  return 0;
}
