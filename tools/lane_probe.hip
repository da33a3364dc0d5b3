// Probe: shader clocks per step of K_lanes' step (fx_eq_lanes.hip) in one
// wave, inputs in LDS, and of variants with parts removed, to locate the
// step's cost.  Also the shader clock rate (clock64 ticks over event time).
// hipcc --offload-arch=gfx950 -O3 tools/lane_probe.hip -o /tmp/lane_probe
#include <hip/hip_runtime.h>

#include <cstdio>

__device__ __forceinline__ double row_shr1(double src, double old) {
  const long long s = __double_as_longlong(src), o = __double_as_longlong(old);
  const int lo = __builtin_amdgcn_update_dpp((int)o, (int)s, 0x111, 0xf, 0xf, false);
  const int hi = __builtin_amdgcn_update_dpp((int)(o >> 32), (int)(s >> 32), 0x111, 0xf, 0xf, false);
  return __longlong_as_double(((long long)hi << 32) | (long long)(unsigned)lo);
}

#define SB __builtin_amdgcn_sched_barrier(0)
constexpr int B = 64;

// V: 0 full (pipelined, dpp, LDS write), 1 no LDS write, 2 no dpp (v = yy + x),
// 3 unpipelined order (as the scheduler likes), 4 chain only (no dpp, no LDS,
// no input products beyond the chain's), 5 pipelined, no sched barriers
typedef __attribute__((address_space(3))) void lds_void_t;
__device__ __forceinline__ void dma4(const void* g, unsigned lds) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dword %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(g), "s"(lds)
               : "memory");
}

template <int V>
__global__ __launch_bounds__(64) void probe(double* out, const double* coef, int iters, long long* cyc,
                                            const double* src) {
#pragma clang fp contract(off)
  __shared__ double xl[B * 4];
  __shared__ double dl[4][B * 4];
  __shared__ double yl[B * 64];
  const int lane = threadIdx.x;
  for (int i = lane; i < B * 4; i += 64) xl[i] = 1e-3 * i;
  __syncthreads();
  double q[6];
  for (int i = 0; i < 6; ++i) q[i] = coef[i] * (1.0 + 1e-3 * (lane & 15));
  double d0 = 0, d1 = 0, y = 0;
  const double g0 = coef[0];
  const int r = lane >> 4;
  long long tacc[2] = {0, 0};
  long long t0 = clock64();
  for (int it = 0; it < iters; ++it) {
    const long long tb0 = clock64();
    if constexpr (V == 6 || V == 8 || V == 10) {
      if constexpr (V != 10) asm volatile("s_waitcnt vmcnt(28)" ::: "memory");
      const unsigned base = (unsigned)(uintptr_t)(lds_void_t*)&dl[it & 3][0];
#pragma unroll
      for (int h = 0; h < 8; ++h)
        dma4(reinterpret_cast<const char*>(src + ((int64_t)it * 64 + 8 * h + ((lane & 15) >> 1)) + (blockIdx.x * 4 + r) * 300000) + 4 * (lane & 1),
             base + h * 256);
    }
    double xv[B];
#pragma unroll
    for (int i = 0; i < B; ++i) xv[i] = xl[(i >> 3) * 32 + r * 8 + (i & 7)];
    if constexpr (V >= 9) {
      const double w = xv[0] + xv[B - 1];  // the block's input has landed
      asm volatile("" ::"v"(w));
      tacc[0] += clock64() - tb0;
    }
    auto input = [&](double yp, int i) {
      if constexpr (V == 2 || V == 4) return yp * 0.5 + xv[i];
      else return row_shr1(yp, xv[i] * g0);
    };
    if constexpr (V >= 12) {
      double yb[B];
#pragma unroll
      for (int i = 0; i < B; ++i) {
        const double v = input(y, i);
        const double yy = q[1] * v + d0;
        const double n0 = q[2] * v - q[4] * yy + d1;
        const double n1 = q[3] * v - q[5] * yy;
        d0 = n0;
        d1 = n1;
        y = yy;
        yb[i] = yy;
      }
      constexpr int NW = V == 12 ? 0 : V == 13 ? 8 : V == 14 ? 16 : 32;
      if constexpr (V == 16) {
#pragma unroll
        for (int i = 0; i < 32; ++i) *reinterpret_cast<double2*>(&yl[(2 * i) * 64 + 2 * lane]) = make_double2(yb[2 * i], yb[2 * i + 1]);
      } else if ((lane & 15) == 4) {
#pragma unroll
        for (int i = 0; i < NW; ++i) *reinterpret_cast<double2*>(&yl[r * 80 + 2 * i]) = make_double2(yb[2 * i], yb[2 * i + 1]);
      }
    } else if constexpr (V == 3 || (V >= 6 && V <= 11)) {
#pragma unroll
      for (int i = 0; i < B; ++i) {
        const double v = input(y, i);
        const double yy = q[1] * v + d0;
        const double n0 = q[2] * v - q[4] * yy + d1;
        const double n1 = q[3] * v - q[5] * yy;
        d0 = n0;
        d1 = n1;
        y = yy;
        yl[i * 64 + lane] = yy;
      }
      const long long te0 = clock64();
      if constexpr (V == 9) {  // the four outputs read first (one LDS wait), then stored
        double v4[4];
#pragma unroll
        for (int h = 0; h < 4; ++h) v4[h] = yl[(16 * h + (lane & 15)) * 64 + 16 * r + 4];
#pragma unroll
        for (int h = 0; h < 4; ++h) {
          double* p = out + 64 * 1024 + ((int64_t)(blockIdx.x * 4 + r) * 300000 + (int64_t)it * 64 + 16 * h + (lane & 15));
          asm volatile("global_store_dwordx2 %0, %1, off" ::"v"(p), "v"(v4[h]) : "memory");
        }
      }
      if constexpr (V >= 9) tacc[1] += clock64() - te0;
      if constexpr (V == 7 || V == 8) {
#pragma unroll
        for (int h = 0; h < 4; ++h) {
          const double v = yl[(16 * h + (lane & 15)) * 64 + 16 * r + 4];
          double* p = out + 64 * 1024 + ((int64_t)(blockIdx.x * 4 + r) * 300000 + (int64_t)it * 64 + 16 * h + (lane & 15));
          asm volatile("global_store_dwordx2 %0, %1, off" ::"v"(p), "v"(v) : "memory");
        }
      }
    } else {
      double v = input(y, 0);
      double t1 = q[1] * v, t2 = q[2] * v, t3 = q[3] * v;
#pragma unroll
      for (int i = 0; i < B; ++i) {
        const double yy = t1 + d0;
        if (V != 5) SB;
        const double t4 = q[4] * yy;
        if (V != 5) SB;
        double vn = 0.0;
        if (i + 1 < B) vn = input(yy, i + 1);
        if (V != 5) SB;
        const double t5 = q[5] * yy;
        if (V != 5) SB;
        const double e = t2 - t4;
        if (V != 5) SB;
        double t1n = 0.0, t2n = 0.0, t3n = 0.0;
        if (i + 1 < B) {
          t1n = q[1] * vn;
          t2n = q[2] * vn;
          t3n = q[3] * vn;
        }
        if (V != 5) SB;
        const double n0 = e + d1;
        if (V != 5) SB;
        const double n1 = t3 - t5;
        if (V != 5) SB;
        y = yy;
        if (V != 1 && V != 4) yl[i * 64 + lane] = yy;
        d0 = n0;
        d1 = n1;
        t1 = t1n;
        t2 = t2n;
        t3 = t3n;
        if (V != 5) SB;
      }
    }
  }
  long long t1c = clock64();
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  double s = y + d0 + d1;
  for (int i = 0; i < B; ++i) s += yl[i * 64 + lane];
  out[blockIdx.x * 64 + lane] = s;
  if (lane == 0 && blockIdx.x == 0) {
    *cyc = t1c - t0;
    cyc[1] = tacc[0];
    cyc[2] = tacc[1];
  }
}

template <int V>
void run(const char* name, int blocks) {
  double *d, *c, *src;
  long long* cy;
  hipMalloc(&d, (size_t)blocks * 4 * 300000 * 8 + 64 * 1024 * 8);
  hipMalloc(&src, (size_t)blocks * 4 * 300000 * 8);
  hipMemset(src, 0, (size_t)blocks * 4 * 300000 * 8);
  hipMalloc(&c, 6 * 8);
  hipMalloc(&cy, 24);
  hipMemset(cy, 0, 24);
  double h[6] = {1.0, 0.2, 0.3, 0.1, -0.5, 0.25};
  hipMemcpy(c, h, 48, hipMemcpyHostToDevice);
  const int iters = 4000;  // 256000 steps: rows of 300000 samples per channel
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipLaunchKernelGGL(probe<V>, dim3(blocks), dim3(64), 0, 0, d, c, iters, cy, src);
  hipDeviceSynchronize();
  hipEventRecord(e0, 0);
  hipLaunchKernelGGL(probe<V>, dim3(blocks), dim3(64), 0, 0, d, c, iters, cy, src);
  hipEventRecord(e1, 0);
  hipEventSynchronize(e1);
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  long long v, vv[3];
  hipMemcpy(vv, cy, 24, hipMemcpyDeviceToHost);
  v = vv[0];
  const double steps = (double)iters * B;
  printf("%-34s blocks %5d: %6.1f clocks/step (clock64), %6.2f ns/step (events) -> %.2f GHz\n", name, blocks,
         (double)v / steps, ms * 1e6 / steps, (double)v / (ms * 1e6));
  if (vv[1] || vv[2]) printf("    per block: start (DMA issue .. input read) %.0f clocks, end (outputs) %.0f clocks\n",
                             (double)vv[1] / iters, (double)vv[2] / iters);
  hipFree(d);
  hipFree(src);
  hipFree(c);
  hipFree(cy);
}

int main() {
  for (int blocks : {64}) {
    run<4>("chain only", blocks);
    run<3>("unpipelined order", blocks);
    run<12>("V3, outputs in registers, no writes", blocks);
    run<13>("  + 8 masked b128 writes per block", blocks);
    run<14>("  + 16 masked b128 writes per block", blocks);
    run<15>("  + 32 masked b128 writes per block", blocks);
    run<16>("  + 32 unmasked b128 writes per block", blocks);
  }
  return 0;
}
