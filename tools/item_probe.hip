// Memory-pattern probe for the per-item FFT kernels (K1/K3):
// a 512-thread workgroup moves one "item" -- RB bytes read from a row of a
// strided array and WB bytes written to a contiguous output block -- with the
// kernels' access shapes (16 B per lane per instruction, a wave covering
// 1 KiB), no arithmetic.  A dummy LDS allocation pins the occupancy of the
// real kernels (70 KiB: two workgroups per CU).  Variants: items per launch,
// input row stride, output block stride, non-temporal loads/stores, the
// store chunk order rotated per item, and a grid-stride (persistent) form.
//   hipcc --offload-arch=gfx950 -O3 tools/item_probe.hip -o tools/item_probe
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

typedef double d2v __attribute__((ext_vector_type(2)));

struct Args {
  const double2* in;
  double2* out;
  long in_row;    // input row stride (double2)
  long out_row;   // output block stride (double2)
  int items;
  int persist;    // 1: grid-stride over items
  int rot;        // 1: rotate the store chunk order by item
};

template <int NL, int NS, bool NTL, bool NTS, int LDSB>
__global__ __launch_bounds__(512) void k_item(Args a) {
  __shared__ double2 pin[LDSB > 0 ? LDSB / 16 : 1];
  const int tid = threadIdx.x;
  for (int it = blockIdx.x; it < a.items; it += a.persist ? gridDim.x : a.items) {
    const double2* r = a.in + (long)it * a.in_row;
    double2 v[NL];
#pragma unroll
    for (int s = 0; s < NL; ++s) {
      const double2* p = r + tid + 512 * s;
      if (NTL) {
        const d2v t = __builtin_nontemporal_load(reinterpret_cast<const d2v*>(p));
        v[s] = make_double2(t.x, t.y);
      } else {
        v[s] = *p;
      }
    }
    double2 acc[NS];
#pragma unroll
    for (int s = 0; s < NS; ++s) acc[s] = make_double2(0, 0);
#pragma unroll
    for (int s = 0; s < NL; ++s) {
      acc[s % NS].x += v[s].x;
      acc[s % NS].y += v[s].y;
    }
    if (LDSB > 0 && acc[0].x == 1.2345e300) pin[tid] = acc[0];  // never: keeps the allocation
    double2* o = a.out + (long)it * a.out_row;
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      const int c = a.rot ? ((s + it) & (NS - 1)) : s;
      double2* p = o + tid + 512 * c;
      if (NTS)
        __builtin_nontemporal_store(d2v{acc[s].x, acc[s].y}, reinterpret_cast<d2v*>(p));
      else
        *p = acc[s];
    }
  }
}

template <int NL, int NS, bool NTL, bool NTS, int LDSB>
void run(const char* name, Args a, int grid) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int w = 0; w < 3; ++w) hipLaunchKernelGGL((k_item<NL, NS, NTL, NTS, LDSB>), dim3(grid), dim3(512), 0, 0, a);
  CK(hipGetLastError());
  const int reps = 10;
  float tot = 0;
  for (int w = 0; w < reps; ++w) {
    CK(hipEventRecord(e0));
    hipLaunchKernelGGL((k_item<NL, NS, NTL, NTS, LDSB>), dim3(grid), dim3(512), 0, 0, a);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    tot += ms;
  }
  const double us = tot * 1e3 / reps;
  const double bytes = (double)a.items * 16.0 * 512 * (NL + NS);
  std::printf("%-44s items %5d grid %5d  %7.1f us  %7.1f GB/s\n", name, a.items, grid, us, bytes / (us * 1e-6) / 1e9);
}

int main() {
  const long rows = 4200;
  double2 *in, *out;
  const long in_row_max = 8200 + 4096;
  CK(hipMalloc(&in, rows * in_row_max * 16));
  CK(hipMalloc(&out, rows * 8192L * 16));
  CK(hipMemset(in, 0, rows * in_row_max * 16));
  CK(hipMemset(out, 0, rows * 8192L * 16));
  Args a{in, out, 8200, 4096, 4128, 0, 0};
  // K3 shape: 128 KiB in (16 loads), 64 KiB out (8 stores)
  run<16, 8, false, false, 70656>("K3 shape, MS=M+8", a, a.items);
  a.items = 4096;
  run<16, 8, false, false, 70656>("K3 shape, 4096 items", a, a.items);
  a.items = 4128;
  run<16, 8, true, false, 70656>("K3 shape, nt loads", a, a.items);
  run<16, 8, false, true, 70656>("K3 shape, nt stores", a, a.items);
  run<16, 8, true, true, 70656>("K3 shape, nt both", a, a.items);
  a.rot = 1;
  run<16, 8, false, false, 70656>("K3 shape, rotated store order", a, a.items);
  a.rot = 0;
  a.in_row = 8192;
  run<16, 8, false, false, 70656>("K3 shape, in row stride 8192", a, a.items);
  a.in_row = 8192 + 256;
  run<16, 8, false, false, 70656>("K3 shape, in row stride 8448", a, a.items);
  a.in_row = 8200;
  a.out_row = 4096 + 64;
  run<16, 8, false, false, 70656>("K3 shape, out stride 4160", a, a.items);
  a.out_row = 4096;
  a.persist = 1;
  run<16, 8, false, false, 70656>("K3 shape, persistent 512", a, 512);
  run<16, 8, false, false, 0>("K3 shape, persistent 1024 no LDS", a, 1024);
  a.persist = 0;
  run<16, 8, false, false, 0>("K3 shape, no LDS (occupancy by VGPR)", a, a.items);
  run<16, 8, false, false, 50000>("K3 shape, 3 WG/CU", a, a.items);
  // K1 shape: 64 KiB in (8 loads), 128 KiB out (16 stores)
  a.in_row = 4096;
  a.out_row = 8200;
  a.items = 4096;
  run<8, 16, false, false, 70656>("K1 shape", a, a.items);
  run<8, 16, false, true, 70656>("K1 shape, nt stores", a, a.items);
  run<8, 16, true, false, 70656>("K1 shape, nt loads", a, a.items);
  run<8, 16, false, false, 50000>("K1 shape, 3 WG/CU", a, a.items);
  return 0;
}
