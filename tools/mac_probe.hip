// Memory-pattern probe for K2 (k_fdl_mac_lds): waves stream
// rows of a [rows][8200] complex128 array (the block-spectrum ring) and write
// one 1-KiB run per row to a second array (the Z rows), no arithmetic.  One
// wave = one bin group of one run: 12 waves per CU, R rows per wave, rows
// 131,200 B apart.  Read shapes per row and wave:
//   0: two 512-B runs (bins 32bx.. and their mirrors, K2 today)
//   1: one 1-KiB run
//   2: workgroups of 4 waves (bin groups 4g..4g+3 of one run) with a barrier
//      per row, so a workgroup reads two 2-KiB runs per row together
//   3: shape 0 without the stores (read side alone)
//   4: shape 0 with Z stored transposed ([bin group][row]: contiguous per wave)
//   hipcc --offload-arch=gfx950 -O3 tools/mac_probe.hip -o tools/mac_probe
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

constexpr int M = 8192, MS = 8200, NX = 128;  // 128 bin groups of 32 pairs

struct Args {
  const double2* X;
  double2* Z;
  int runs, R, ch;
};

// rows are loaded D ahead into registers (a ring of 8)
template <int SHAPE, int WPG>
__global__ __launch_bounds__(64 * WPG) void k_probe(Args a) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int wid = blockIdx.x * WPG + w;  // run fastest within (channel, bin group)
  const int ry = (WPG == 1) ? wid % a.runs : (blockIdx.x % a.runs);
  const int bx = (WPG == 1) ? (wid / a.runs) % NX : ((blockIdx.x / a.runs) % (NX / WPG)) * WPG + w;
  const int c = (WPG == 1) ? wid / (a.runs * NX) : blockIdx.x / (a.runs * (NX / WPG));
  const long rows_per_ch = (long)a.runs * a.R + 16;
  const double2* Xc = a.X + (long)c * rows_per_ch * MS;
  double2* Zc = a.Z + (long)c * rows_per_ch * MS;
  int off;
  if (SHAPE == 1)
    off = 64 * bx + lane;
  else
    off = lane < 32 ? 32 * bx + lane : (M - 32 * bx - 32) + (lane - 32);
  const long r0 = (long)ry * a.R;
  double2 ring[8];
#pragma unroll
  for (int d = 0; d < 8; ++d) ring[d] = Xc[(r0 + d) * MS + off];
  double2 acc = make_double2(0, 0);
  for (int r = 0; r < a.R; r += 8) {
#pragma unroll
    for (int d = 0; d < 8; ++d) {
      const double2 v = ring[d];
      ring[d] = Xc[(r0 + r + d + 8) * MS + off];
      acc.x += v.x;
      acc.y += v.y;
      if (SHAPE == 4)  // transposed Z: [bin group][row], each wave a contiguous stream
        Zc[((long)bx * rows_per_ch + r0 + r + d) * 64 + lane] = acc;
      else if (SHAPE != 3)
        Zc[(r0 + r + d) * MS + 64 * bx + lane] = acc;
      if (SHAPE == 2) __syncthreads();
    }
  }
  if (SHAPE == 3 && acc.x == 1.2345e300) Zc[lane] = acc;
}

template <int SHAPE, int WPG>
void run(const char* name, Args a) {
  const int waves = a.ch * NX * a.runs;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int w = 0; w < 2; ++w) hipLaunchKernelGGL((k_probe<SHAPE, WPG>), dim3(waves / WPG), dim3(64 * WPG), 0, 0, a);
  CK(hipGetLastError());
  float tot = 0;
  const int reps = 5;
  for (int w = 0; w < reps; ++w) {
    CK(hipEventRecord(e0));
    hipLaunchKernelGGL((k_probe<SHAPE, WPG>), dim3(waves / WPG), dim3(64 * WPG), 0, 0, a);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    tot += ms;
  }
  const double us = tot * 1e3 / reps;
  const double rb = (double)waves * (a.R + 8) * 1024, wb = SHAPE == 3 ? 0 : (double)waves * a.R * 1024;
  std::printf("%-52s %7.1f us  %7.1f GB/s (reads %.0f MB, writes %.0f MB)\n", name, us, (rb + wb) / (us * 1e-6) / 1e9,
              rb / 1e6, wb / 1e6);
}

int main() {
  Args a{nullptr, nullptr, 12, 176, 2};
  const long rows = (long)a.ch * (a.runs * a.R + 16);
  double2 *X, *Z;
  CK(hipMalloc(&X, rows * MS * 16));
  CK(hipMalloc(&Z, rows * MS * 16));
  CK(hipMemset(X, 0, rows * MS * 16));
  a.X = X;
  a.Z = Z;
  run<0, 1>("shape 0: 2 x 512 B per wave-row (K2 today)", a);
  run<1, 1>("shape 1: 1 KiB per wave-row", a);
  run<2, 4>("shape 2: 4-wave lockstep, 2 x 2 KiB per WG-row", a);
  run<3, 1>("shape 3: shape 0 reads only", a);
  run<4, 1>("shape 4: shape 0 with transposed Z writes", a);
  run<0, 1>("shape 0 again", a);
  return 0;
}
