// Memory-only stand-ins of BigFft's global Stockham passes (bigfft.hip):
// a workgroup of F x R elements reads F consecutive butterflies j of radix R
// (element r of butterfly j at j + r N/R: runs of F complex128 values) and
// writes them to (j / Ns) Ns R + (j mod Ns) + r Ns (runs of min(F, Ns) for
// Ns > 1, of R for Ns = 1), no arithmetic.  Prints the rate for each
// (R, F, Ns) shape at N = 2^24: the ceiling a pass of that shape can reach,
// i.e. how much of a pass's time the run length alone explains.
//   hipcc --offload-arch=gfx950 -O3 tools/stride_probe.hip -o tools/stride_probe
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

// E elements per workgroup (F * R), BLOCK threads, E / BLOCK per thread.
template <int R, int F, int BLOCK>
__global__ __launch_bounds__(BLOCK) void k_pass(const double2* __restrict__ in, double2* __restrict__ out, long N,
                                                long Ns) {
  constexpr int V = F * R / BLOCK;
  const long nb = N / R;
  const long j0 = (long)blockIdx.x * F;
  double2 v[V];
#pragma unroll
  for (int i = 0; i < V; ++i) {
    const int idx = i * BLOCK + threadIdx.x;
    const int jj = idx % F, r = idx / F;
    v[i] = in[j0 + jj + (long)r * nb];
  }
  // the same element back out at its Stockham destination, in the store
  // order bigfft.hip uses (rr fastest when Ns = 1, jj fastest otherwise)
#pragma unroll
  for (int i = 0; i < V; ++i) {
    const int idx = i * BLOCK + threadIdx.x;
    int jj, rr;
    if (Ns == 1) {
      rr = idx % R;
      jj = idx / R;
    } else {
      jj = idx % F;
      rr = idx / F;
    }
    const long jo = j0 + jj;
    const long o = (jo & ~(Ns - 1)) * R + (jo & (Ns - 1)) + (long)rr * Ns;
    // value of (jj, rr): the load above holds element (jj', r') at slot i;
    // a memory-only probe may store any value, so store v[i]
    out[o] = v[i];
  }
}

template <int R, int F, int BLOCK>
void run(const double2* in, double2* out, long N, long Ns, hipEvent_t e0, hipEvent_t e1) {
  const dim3 grid((unsigned)(N / R / F));
  for (int w = 0; w < 3; ++w) hipLaunchKernelGGL((k_pass<R, F, BLOCK>), grid, dim3(BLOCK), 0, 0, in, out, N, Ns);
  CK(hipDeviceSynchronize());
  const int reps = 10;
  CK(hipEventRecord(e0));
  for (int r = 0; r < reps; ++r) hipLaunchKernelGGL((k_pass<R, F, BLOCK>), grid, dim3(BLOCK), 0, 0, in, out, N, Ns);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, e0, e1));
  const double us = ms * 1e3 / reps;
  std::printf("R %5d F %3d (run %5d B) block %4d Ns %8ld: %7.1f us  %5.2f TB/s\n", R, F, F * 16, BLOCK, Ns, us,
              2.0 * N * 16 / (us * 1e-6) / 1e12);
}

int main() {
  const long N = 1L << 24;
  double2 *in, *out;
  CK(hipMalloc(&in, N * 16));
  CK(hipMalloc(&out, N * 16));
  CK(hipMemset(in, 0, N * 16));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  // Ns must stay <= N / R (the last pass of a plan has Ns = N / R)
  const bool two_pass = std::getenv("PROBE_TWO_PASS") != nullptr;
  if (!two_pass) {
    for (long Ns : {1L, 256L, 65536L}) {
      run<256, 16, 256>(in, out, N, Ns, e0, e1);  // today's radix-256 pass
      run<256, 16, 512>(in, out, N, Ns, e0, e1);
      run<256, 32, 512>(in, out, N, Ns, e0, e1);
      run<128, 32, 256>(in, out, N, Ns, e0, e1);
      run<128, 64, 512>(in, out, N, Ns, e0, e1);
      run<64, 64, 256>(in, out, N, Ns, e0, e1);
      run<64, 128, 512>(in, out, N, Ns, e0, e1);
      run<512, 8, 256>(in, out, N, Ns, e0, e1);
    }
  } else {
    // a two-pass 4096 x 4096 plan: both passes read runs of F values
    for (long Ns : {1L, 4096L}) {
      run<4096, 1, 256>(in, out, N, Ns, e0, e1);
      run<4096, 2, 512>(in, out, N, Ns, e0, e1);
      run<4096, 4, 1024>(in, out, N, Ns, e0, e1);
      run<4096, 8, 1024>(in, out, N, Ns, e0, e1);
    }
    for (long Ns : {1L, 8192L}) {
      run<2048, 4, 512>(in, out, N, Ns, e0, e1);
      run<2048, 8, 1024>(in, out, N, Ns, e0, e1);
    }
  }
  return 0;
}
