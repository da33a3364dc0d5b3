// Microbenchmark: cycles per sample of the compressor envelope follower
// (core.go:274-286: attack/release one-pole with a branch on src > env) in
// one wave, written as the staged detector writes it.
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void envf(double* out, const double* in, int iters, double att, double rel, long long* cyc) {
#pragma clang fp contract(off)
  double x[8];
  for (int d = 0; d < 8; ++d) x[d] = in[d * 64 + threadIdx.x];
  double env = 0.0, acc = 0.0;
  long long t0 = clock64();
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int d = 0; d < 8; ++d) {
      const double src = fabs(x[d]);
      const double ne = src > env ? env + (src - env) * att : src + (env - src) * rel;
      env = ne;
      acc += ne;
    }
  }
  long long t1 = clock64();
  out[threadIdx.x] = acc + env;
  if (threadIdx.x == 0) *cyc = t1 - t0;
}

int main() {
  double *d, *in;
  long long* cy;
  if (hipMalloc(&d, 64 * 8) || hipMalloc(&in, 512 * 8) || hipMalloc(&cy, 8)) return 1;
  double h[512];
  for (int i = 0; i < 512; ++i) h[i] = ((i * 7919) % 1000) / 1000.0 - 0.5;
  if (hipMemcpy(in, h, sizeof(h), hipMemcpyHostToDevice)) return 1;
  const int iters = 20000;
  for (int r = 0; r < 2; ++r) hipLaunchKernelGGL(envf, dim3(1), dim3(64), 0, 0, d, in, iters, 0.002, 0.9998, cy);
  long long v;
  if (hipMemcpy(&v, cy, 8, hipMemcpyDeviceToHost)) return 1;
  printf("envelope follower: %.1f cycles per sample (one wave)\n", (double)v / iters / 8);
  return 0;
}
