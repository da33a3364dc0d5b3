// Microbenchmark: dependent-issue latency and issue rate of FP64 VALU ops
// for one wave (and for k interleaved independent chains) on gfx950.
#include <hip/hip_runtime.h>
#include <cstdio>

template <int K>
__global__ void chain(double* out, double a, double b, int iters, long long* cyc) {
#pragma clang fp contract(off)
  double x[K];
  for (int k = 0; k < K; ++k) x[k] = threadIdx.x * 1e-3 + k;
  long long t0 = clock64();
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int k = 0; k < K; ++k) x[k] = x[k] * a + b;  // mul then add (no fma): 2 dependent ops
  }
  long long t1 = clock64();
  double s = 0;
  for (int k = 0; k < K; ++k) s += x[k];
  out[threadIdx.x] = s;
  if (threadIdx.x == 0) *cyc = t1 - t0;
}

template <int K>
__global__ void chain_fma(double* out, double a, double b, int iters, long long* cyc) {
  double x[K];
  for (int k = 0; k < K; ++k) x[k] = threadIdx.x * 1e-3 + k;
  long long t0 = clock64();
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int k = 0; k < K; ++k) x[k] = fma(x[k], a, b);
  }
  long long t1 = clock64();
  double s = 0;
  for (int k = 0; k < K; ++k) s += x[k];
  out[threadIdx.x] = s;
  if (threadIdx.x == 0) *cyc = t1 - t0;
}

template <int K>
__global__ void chain_f32(float* out, float a, float b, int iters, long long* cyc) {
  float x[K];
  for (int k = 0; k < K; ++k) x[k] = threadIdx.x * 1e-3f + k;
  long long t0 = clock64();
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int k = 0; k < K; ++k) x[k] = fmaf(x[k], a, b);
  }
  long long t1 = clock64();
  float s = 0;
  for (int k = 0; k < K; ++k) s += x[k];
  out[threadIdx.x] = s;
  if (threadIdx.x == 0) *cyc = t1 - t0;
}

template <class F>
void run(const char* name, F f, int ops_per_iter) {
  double* d;
  long long* c;
  hipMalloc(&d, 64 * sizeof(double));
  hipMalloc(&c, sizeof(long long));
  const int iters = 100000;
  f(d, iters, c);  // warm
  hipDeviceSynchronize();
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipEventRecord(e0);
  f(d, iters, c);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  long long cy;
  hipMemcpy(&cy, c, sizeof(cy), hipMemcpyDeviceToHost);
  printf("%-28s clock64/op %.2f   ns/op %.3f  (wall %.3f ms)\n", name, (double)cy / iters / ops_per_iter,
         ms * 1e6 / iters / ops_per_iter, ms);
  hipFree(d);
  hipFree(c);
}

int main() {
#define R(K)                                                                                                  \
  run("mul+add f64 chains=" #K, [](double* d, int it, long long* c) {                                        \
    hipLaunchKernelGGL(chain<K>, dim3(1), dim3(64), 0, 0, d, 1.0000001, 1e-9, it, c); }, 2 * K);              \
  run("fma f64 chains=" #K, [](double* d, int it, long long* c) {                                            \
    hipLaunchKernelGGL(chain_fma<K>, dim3(1), dim3(64), 0, 0, d, 1.0000001, 1e-9, it, c); }, K);              \
  run("fma f32 chains=" #K, [](double* d, int it, long long* c) {                                            \
    hipLaunchKernelGGL(chain_f32<K>, dim3(1), dim3(64), 0, 0, (float*)d, 1.0000001f, 1e-9f, it, c); }, K);
  R(1) R(2) R(4) R(8)
  return 0;
}
