// Microbenchmark: cycles per sample of the serial recurrences of config 5's
// compressor detector and Freeverb comb, one wave, in the forms a kernel can
// write them:
//  env/ref    env' = src > env ? env + (src-env)*a : src + (env-src)*r  (core.go:351-355)
//  env/abs    env' = fma(c2, |src-env|, fma(1-c1, env, c1*src)),
//             c1 = (a + b)/2, c2 = (a - b)/2, b = 1 - r  (the same map, other rounding)
//  comb/ref   fs' = flush(out*d2 + fs*d1), flush: |v| < 1e-23 -> 0   (reverb.go:101-117)
//  comb/int   the same with the flush as integer ops on the bit pattern (bit-exact)
//   hipcc --offload-arch=gfx950 -O3 tools/chain_latency.hip -o tools/chain_latency
#include <hip/hip_runtime.h>

#include <cstdio>

template <int V>
__global__ void k_env(double* out, const double* in, int iters, double a, double r, long long* cyc) {
#pragma clang fp contract(off)
  double x[8];
  for (int d = 0; d < 8; ++d) x[d] = in[d * 64 + threadIdx.x];
  const double b = 1.0 - r, c1 = 0.5 * (a + b), c2 = 0.5 * (a - b), k1 = 1.0 - c1;
  double env = 0.0, acc = 0.0;
  const long long t0 = clock64();
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int d = 0; d < 8; ++d) {
      const double src = fabs(x[d]);
      double ne;
      if constexpr (V == 0) {
        ne = src > env ? env + (src - env) * a : src + (env - src) * r;
      } else {
        ne = __builtin_fma(c2, fabs(src - env), __builtin_fma(k1, env, c1 * src));
      }
      env = ne;
      acc += ne;
    }
  }
  const long long t1 = clock64();
  out[threadIdx.x] = acc + env;
  if (threadIdx.x == 0) *cyc = t1 - t0;
}

// env/d: the same map carried as dd = src_t - env_{t-1}:
//   dd' = fma(-c2, |dd|, fma(k1, dd, src_{t+1} - src_t)), env_t = src_{t+1} - dd'
// (V = 0: the differences formed in the loop; V = 1: precomputed outside it)
// env/2s: two samples per step on the convex map (attack faster than release):
//   env'' = max(A1 env + B1, A2 env + B2, A3 env + B3), the three composed lines'
//   slopes constant, their intercepts from the two inputs (off the chain)
template <int V>
__global__ void k_envd(double* out, const double* in, int iters, double a, double r, long long* cyc) {
#pragma clang fp contract(off)
  double x[9];
  for (int d = 0; d < 9; ++d) x[d] = fabs(in[d * 64 + threadIdx.x]);
  const double b = 1.0 - r, c1 = 0.5 * (a + b), c2 = 0.5 * (a - b), k1 = 1.0 - c1;
  double ds[8];
  for (int d = 0; d < 8; ++d) ds[d] = x[d + 1] - x[d];
  double dd = x[0], acc = 0.0;
  const long long t0 = clock64();
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int d = 0; d < 8; ++d) {
      const double dl = V == 0 ? x[d + 1] - x[d] : ds[d];
      dd = __builtin_fma(-c2, fabs(dd), __builtin_fma(k1, dd, dl));
      acc += x[d + 1] - dd;
    }
  }
  const long long t1 = clock64();
  out[threadIdx.x] = acc + dd;
  if (threadIdx.x == 0) *cyc = t1 - t0;
}

__global__ void k_env2s(double* out, const double* in, int iters, double a, double r, long long* cyc) {
#pragma clang fp contract(off)
  double x[8];
  for (int d = 0; d < 8; ++d) x[d] = fabs(in[d * 64 + threadIdx.x]);
  // one sample: L_a(e) = (1-a) e + a s, L_r(e) = r e + (1-r) s; convex when 1-a <= r
  const double sa = 1.0 - a, sr = r;
  double B1[4], B2[4], B3[4];
  for (int p = 0; p < 4; ++p) {
    const double s1 = x[2 * p], s2 = x[2 * p + 1];
    B1[p] = sa * (a * s1) + a * s2;                                  // La2 o La1
    B2[p] = fmax(sa * ((1 - r) * s1) + a * s2, sr * (a * s1) + (1 - r) * s2);  // La2 o Lr1, Lr2 o La1 (same slope)
    B3[p] = sr * ((1 - r) * s1) + (1 - r) * s2;                      // Lr2 o Lr1
  }
  const double A1 = sa * sa, A2 = sa * sr, A3 = sr * sr;
  double env = 0.0, acc = 0.0;
  const long long t0 = clock64();
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      const double e1 = fmax(__builtin_fma(sa, env, a * x[2 * p]), __builtin_fma(sr, env, (1 - r) * x[2 * p]));
      env = fmax(fmax(__builtin_fma(A1, env, B1[p]), __builtin_fma(A2, env, B2[p])), __builtin_fma(A3, env, B3[p]));
      acc += e1 + env;
    }
  }
  const long long t1 = clock64();
  out[threadIdx.x] = acc + env;
  if (threadIdx.x == 0) *cyc = t1 - t0;
}

__device__ __forceinline__ double flush_int(double v) {
  // |v| < 1e-23 -> +0 (v itself otherwise), from the bit pattern: the
  // magnitude bits compare like the magnitudes (non-negative, non-NaN)
  const long long bits = __double_as_longlong(v);
  const long long mag = bits & 0x7fffffffffffffffLL;
  const long long thr = __double_as_longlong(1e-23);
  const long long keep = (thr - 1 - mag) >> 63;  // all ones when mag >= thr
  return __longlong_as_double(bits & keep);
}

template <int V>
__global__ void k_comb(double* out, const double* in, int iters, double d1, double d2, long long* cyc) {
#pragma clang fp contract(off)
  double x[8];
  for (int d = 0; d < 8; ++d) x[d] = in[d * 64 + threadIdx.x];
  double fs = 0.0, acc = 0.0;
  const long long t0 = clock64();
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int d = 0; d < 8; ++d) {
      const double o = x[d];
      double v = o * d2 + fs * d1;
      if constexpr (V == 0)
        v = fabs(v) < 1e-23 ? 0.0 : v;
      else
        v = flush_int(v);
      fs = v;
      acc += v;
    }
  }
  const long long t1 = clock64();
  out[threadIdx.x] = acc + fs;
  if (threadIdx.x == 0) *cyc = t1 - t0;
}

// the shader clock against the constant wall clock (s_memrealtime, 100 MHz) over one
// wave's dependent FP64 chain: the engine clock a lightly loaded chip runs at
__global__ void k_clock(double* out, int iters, long long* cyc) {
  double v = out[threadIdx.x];
  const long long c0 = clock64(), w0 = wall_clock64();
  for (int i = 0; i < iters; ++i) v = __builtin_fma(v, 0.999999, 1e-9);
  const long long c1 = clock64(), w1 = wall_clock64();
  out[threadIdx.x] = v;
  if (threadIdx.x == 0) {
    cyc[0] = c1 - c0;
    cyc[1] = w1 - w0;
  }
}

int main() {
  double *d, *in;
  long long* cy;
  if (hipMalloc(&d, 64 * 8) || hipMalloc(&in, 512 * 8) || hipMalloc(&cy, 8)) return 1;
  double h[512];
  for (int i = 0; i < 512; ++i) h[i] = ((i * 7919) % 1000) / 1000.0 - 0.5;
  if (hipMemcpy(in, h, sizeof(h), hipMemcpyHostToDevice)) return 1;
  const int iters = 20000;
  long long v;
  auto report = [&](const char* name) {
    if (hipMemcpy(&v, cy, 8, hipMemcpyDeviceToHost)) return;
    printf("%-10s %.1f cycles per sample (one wave)\n", name, (double)v / iters / 8);
  };
  for (int r = 0; r < 2; ++r) hipLaunchKernelGGL(k_env<0>, dim3(1), dim3(64), 0, 0, d, in, iters, 0.002, 0.9998, cy);
  report("env/ref");
  for (int r = 0; r < 2; ++r) hipLaunchKernelGGL(k_env<1>, dim3(1), dim3(64), 0, 0, d, in, iters, 0.002, 0.9998, cy);
  report("env/abs");
  for (int r = 0; r < 2; ++r) hipLaunchKernelGGL(k_envd<0>, dim3(1), dim3(64), 0, 0, d, in, iters, 0.002, 0.9998, cy);
  report("env/d");
  for (int r = 0; r < 2; ++r) hipLaunchKernelGGL(k_envd<1>, dim3(1), dim3(64), 0, 0, d, in, iters, 0.002, 0.9998, cy);
  report("env/d-pre");
  for (int r = 0; r < 2; ++r) hipLaunchKernelGGL(k_env2s, dim3(1), dim3(64), 0, 0, d, in, iters, 0.002, 0.9998, cy);
  report("env/2s");
  {
    long long* cy2;
    if (hipMalloc(&cy2, 16)) return 1;
    int wrate = 0;
    (void)hipDeviceGetAttribute(&wrate, hipDeviceAttributeWallClockRate, 0);  // kHz
    for (int grid : {1, 8, 256, 2048}) {
      for (int r = 0; r < 2; ++r) hipLaunchKernelGGL(k_clock, dim3(grid), dim3(64), 0, 0, d, 2000000, cy2);
      long long h2[2];
      if (hipMemcpy(h2, cy2, 16, hipMemcpyDeviceToHost)) return 1;
      printf("clock    %4d waves: %lld shader cycles in %lld wall ticks (%d kHz) = %.0f MHz\n", grid, h2[0], h2[1], wrate,
             (double)h2[0] / ((double)h2[1] / (wrate * 1e3)) / 1e6);
    }
  }
  for (int r = 0; r < 2; ++r) hipLaunchKernelGGL(k_comb<0>, dim3(1), dim3(64), 0, 0, d, in, iters, 0.45, 0.55, cy);
  report("comb/ref");
  for (int r = 0; r < 2; ++r) hipLaunchKernelGGL(k_comb<1>, dim3(1), dim3(64), 0, 0, d, in, iters, 0.45, 0.55, cy);
  report("comb/int");
  return 0;
}
