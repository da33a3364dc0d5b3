// Register-blocked sliding dot product shared by the time-domain FIR-shaped
// kernels (conv.Direct in conv_kernels.hip, fir.Filter in dsp_kernels.hip).
//
// A lane owns R consecutive outputs.  Term u of output r is
//   acc[r] = acc[r] + hs[HSTEP * u] * wt[u + r]          (u = 0, 1, ..., cnt-1)
// with a rounded product and a rounded add (no contraction), so every output
// is summed in exactly the reference's term order.  hs is wave-uniform (scalar
// loads); wt is the lane's window in LDS.  Between terms u and u+1 the window
// slides by one element, so a block of R terms needs 2R-1 window values of
// which R-1 carry over from the previous block: one aligned R-wide LDS read
// feeds R*R products.  That moves the bound from LDS bandwidth (one 8-byte
// read per product, 16 products/clk/CU) to the FP64 VALU (32 mul+add
// products/clk/CU).
//
// Alignment contract: (wt - lds_base) + R - 1 is a multiple of R for the
// R-wide reads, i.e. the caller stores its window one element past an
// R-aligned base and gives lane t the window base + 1 + t*R; the LDS array
// extends 2R elements past the last window value (chunk prefetch over-read).
#pragma once

#include <hip/hip_runtime.h>

namespace adsp {

template <int R>
struct LdsVec;
template <>
struct LdsVec<1> {
  typedef double T;
};
template <>
struct LdsVec<2> {
  typedef double T __attribute__((ext_vector_type(2)));
};
template <>
struct LdsVec<4> {
  typedef double T __attribute__((ext_vector_type(4)));
};

// Scalar-base pointer for a wave-uniform address (loads become s_load).
template <class T>
__device__ __forceinline__ T* bd_uniform(T* p) {
  const uint64_t v = reinterpret_cast<uint64_t>(p);
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
  return reinterpret_cast<T*>(((uint64_t)hi << 32) | lo);
}

// Window chunk q = wt[qR - 1 .. qR + R - 2] (one aligned R-wide read); block
// k (terms kR .. kR + R - 1) uses chunks k and k+1: term kR + j of output r
// is wt[kR + j + r] = chunk k[j + r + 1] for j + r < R - 1, else chunk
// k+1[j + r - R + 1].
template <int R>
__device__ __forceinline__ void bd_block(const double (&c0)[R], const double (&c1)[R], const double (&hv)[R],
                                         double (&acc)[R]) {
#pragma clang fp contract(off)
#pragma unroll
  for (int j = 0; j < R; ++j) {
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const int x = j + r + 1;
      const double w = x < R ? c0[x] : c1[x - R];
      const double p = hv[j] * w;
      acc[r] = acc[r] + p;
    }
  }
}

template <int R>
__device__ __forceinline__ void bd_chunk(const double* wt, int q, double (&c)[R]) {
  typedef typename LdsVec<R>::T V;
  const V v = *(const V*)(wt + q * R - 1);
#pragma unroll
  for (int x = 0; x < R; ++x) c[x] = ((const double*)&v)[x];
}

// The taps are read-only for the whole kernel, so they are read through the
// constant address space: with a wave-uniform base the loads become
// s_load_dwordx8/x16 into SGPRs (the v_mul's scalar operand) instead of
// per-lane vector loads of one address.
typedef const __attribute__((address_space(4))) double bd_const_double;

// taps of blocks k .. k+NB-1: hv[b][j] = hs[HSTEP * ((k + b) R + j)], one
// scalar load run from a wave-uniform base
template <int R, int HSTEP, int NB>
__device__ __forceinline__ void bd_taps(const double* hs, int k, double (&hv)[NB][R]) {
  if (HSTEP > 0) {
    bd_const_double* p = (bd_const_double*)bd_uniform(hs + k * R);
#pragma unroll
    for (int b = 0; b < NB; ++b)
#pragma unroll
      for (int j = 0; j < R; ++j) hv[b][j] = p[b * R + j];
  } else {
    bd_const_double* p = (bd_const_double*)bd_uniform(hs - (k + NB) * R + 1);  // lowest address of the run
#pragma unroll
    for (int b = 0; b < NB; ++b)
#pragma unroll
      for (int j = 0; j < R; ++j) hv[b][j] = p[NB * R - 1 - (b * R + j)];
  }
}

template <int R, int HSTEP>
__device__ __forceinline__ void blocked_dot(const double* __restrict__ hs, const double* wt, int cnt, double (&acc)[R]) {
#pragma clang fp contract(off)
  const int nb = R > 1 ? cnt / R : 0;  // full blocks
  int k = 0;
  if (nb > 0) {
    // ring of three chunks, three blocks per iteration: no register moves,
    // and each iteration's taps arrive with one scalar load run.  Chunk
    // reads run up to R past the window (the caller pads its LDS array).
    double c0[R], c1[R], c2[R];
    bd_chunk<R>(wt, 0, c0);
    bd_chunk<R>(wt, 1, c1);
    for (; k + 3 <= nb; k += 3) {
      double hv[3][R];
      bd_taps<R, HSTEP, 3>(hs, k, hv);
      bd_chunk<R>(wt, k + 2, c2);
      bd_block<R>(c0, c1, hv[0], acc);
      bd_chunk<R>(wt, k + 3, c0);
      bd_block<R>(c1, c2, hv[1], acc);
      bd_chunk<R>(wt, k + 4, c1);
      bd_block<R>(c2, c0, hv[2], acc);
    }
    for (; k < nb; ++k) {  // c0 = chunk k, c1 = chunk k+1
      double hv[1][R];
      bd_taps<R, HSTEP, 1>(hs, k, hv);
      bd_block<R>(c0, c1, hv[0], acc);
#pragma unroll
      for (int x = 0; x < R; ++x) c0[x] = c1[x];
      bd_chunk<R>(wt, k + 2, c1);
    }
  }
  for (int u = k * R; u < cnt; ++u) {
    const double h = hs[HSTEP * u];
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const double p = h * wt[u + r];
      acc[r] = acc[r] + p;
    }
  }
}

}  // namespace adsp
