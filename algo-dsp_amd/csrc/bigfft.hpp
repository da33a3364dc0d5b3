// Power-of-two complex FFTs of any size on the device (spectral row 8(f)3:
// CorrelateFFT / Deconvolve / InverseFilter, dsp/conv/correlate.go:111-172,
// deconvolve.go:72-394).  These call algo-fft's NewPlan64(n).Forward/Inverse
// on one whole zero-padded signal, so the size is nextPow2 of the signal
// (up to 2^27 here), far past one workgroup's LDS.
//
// Global Stockham decomposition N = R_0 R_1 ... R_{P-1}: pass p treats the
// array as N/R_p butterflies j of radix R_p on elements j + r N/R_p,
// pre-twiddled by W_{Ns R}^{(j mod Ns) r} (Ns = R_0 .. R_{p-1}), and writes
// them to (j/Ns) Ns R + (j mod Ns) + r Ns, so the result is in natural order
// after the last pass (no bit reversal, no transpose pass).  Each radix-R
// butterfly is an LDS-resident FftPlan<R, 16> transform; a workgroup carries
// F = 4096/R of them (F consecutive j), staged through LDS in both directions
// so every global access moves runs of F (or R) contiguous complex128 values.
// R <= 512 for multi-pass plans keeps F >= 8 (128-byte runs).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <vector>

namespace adsp {

struct FftPassArgs {
  const double2* in;    // complex input (nullptr when xr is used)
  const double* xr;     // real input (first pass only), zero past n_real
  int64_t n_real;
  int64_t in_batch;     // batch stride (elements) of the input
  double2* out;         // complex output
  double* out_real;     // real-part output (last pass only), scaled by `scale`
  int64_t out_batch;
  double scale;
  int64_t N;            // transform size
  int64_t Ns;           // product of the previous radices
  const double2* twR;   // W_R^e, e < R (the pass's LDS transform)
  const double2* tw_lo; // W_N^e, e < 2^S          (pre-twiddles W_N^e = lo[e & (2^S-1)] * hi[e >> S])
  const double2* tw_hi; // W_N^(e 2^S), e < N/2^S
  int S;
  // Fused edges (CorrelateFFT): per-batch real inputs (first pass, zero past
  // nr[b]: no staging buffer), and the last pass's real output scattered to
  // the caller's lag order (o < n_front -> out_real[front_off + o],
  // o >= back_from -> out_real[o - back_from], the rest dropped).
  const double* xb[2];
  int64_t nr[2];
  int pack2;    // first forward pass: one complex input xb[0] + i xb[1] (both real signals in one transform)
  // pack2 correlation: {max|a|, max|b|} as IEEE bit patterns (k_absmax2).  The
  // first pass multiplies b by 2^e (e = exponent(max|a|) - exponent(max|b|)) so
  // both halves of a + i b have the same scale, and the last pass multiplies
  // the outputs by 2^-e (both exact).  null: no scaling.
  const unsigned long long* amax;
  // split correlation (k_corr_split0 / k_fft_pass_pf PACKIN): per-workgroup
  // max-abs partials of the first pass, [2][amax_parts] (a, then b); the
  // second pass reduces them and stores the totals at amax[0..1] for the last
  // inverse pass.
  unsigned long long* amax_part;
  int amax_parts;
  // half: the inverse of the Hermitian A conj(B) as an N/2-point transform
  // (this plan is N/2 = NF/2): its first pass forms z[k] = E[k] + i O[k] from
  // X[k] and X[k + NF/2] (E = (X[k] + X[k+NF/2])/2, O = (X[k] - X[k+NF/2]) W_NF^-k / 2,
  // X from the forward spectrum's mirror pairs), its last pass writes Re z[m]
  // and Im z[m] as the real outputs 2m and 2m + 1.
  const double2* spec2;     // half: B's own spectrum (A in `in`); null: A, B from Z = FFT(a + i b)
  int op;                   // half: the pointwise step (SpecOp) applied to A, B
  double eps;
  unsigned long long* bad;  // kSpecNaive: first bin with |B| < 1e-15 (atomicMin)
  int half;   // first pass: form z from the spectrum
  int pairs;  // last pass: write Re z[m], Im z[m] as real outputs 2m, 2m + 1
  int64_t NF;
  const double2* ftw_lo;  // W_NF tables of the full-size plan
  const double2* ftw_hi;
  int fS;
  int remap;
  int64_t n_front, front_off, back_from;
};

// Device-resident plan and twiddle tables of one size.
class BigFft {
 public:
  explicit BigFft(int64_t N);
  ~BigFft();
  BigFft(const BigFft&) = delete;
  BigFft& operator=(const BigFft&) = delete;

  int64_t size() const { return N_; }
  // Forward (inverse: conj twiddles, then *scale on output) transform of
  // `batch` arrays.  Input: complex `in` or real `xr` (n_real valid values,
  // zero padded); output: complex `out` or its real part `out_real`.
  // scratch: N*batch complex; in/out may alias each other and scratch must not.
  void run(bool forward, const double2* in, const double* xr, int64_t n_real, int64_t in_batch, double2* out,
           double* out_real, int64_t out_batch, double scale, int batch, double2* scratch, hipStream_t s) const;
  // CorrelateFFT with its edges fused (FftPassArgs): one forward transform of
  // a + i b (n and m real samples, zero padded, read straight from the
  // caller's arrays) into spec [N]; then the inverse of the Hermitian
  // A conj(B) on the half plan (N/2 points), written in lag order to out
  // (n + m - 1 values, correlate.go:165-171).  Both plans need passes (N >= 32).
  // amax: kAbsmaxWords words of device scratch, zeroed once (FftPassArgs::amax):
  // without it, b's spectrum taken out of FFT(a + i b) would carry rounding
  // error of order eps |A|, which for |a| >> |b| is far above eps |B|.
  void correlate_half(const BigFft& half, const double* a, int64_t n, const double* b, int64_t m, double2* spec,
                      double* out, double2* scratch, unsigned long long* amax, hipStream_t s) const;
  // The same structure for any SpecOp: Z = FFT(x + i h) (x: n, h: m real
  // samples; h may be null), the inverse of op(X, H) at half length, real
  // outputs o < n_front to out[front_off + o] and o >= back_from to
  // out[o - back_from].  Deconvolve and InverseFilter (deconvolve.go:104-394).
  // pack: one transform of x + i h (the correlation; h's spectrum is then
  // only as exact as x's magnitude allows, which a division cannot afford,
  // so Deconvolve transforms x and h separately: pack = false, spec [2][N]).
  void spectral_half(const BigFft& half, int op, double eps, unsigned long long* bad, bool pack, const double* x,
                     int64_t n, const double* h, int64_t m, int64_t n_front, int64_t front_off, int64_t back_from,
                     double2* spec, double* out, double2* scratch, hipStream_t s,
                     const unsigned long long* amax = nullptr) const;

 private:
  int64_t N_;
  int S_ = 0;
  std::vector<int> radix_;
  std::vector<double2*> twR_;  // per pass
  double2* tw_lo_ = nullptr;
  double2* tw_hi_ = nullptr;
  bool corr_split(const BigFft& half) const;
  const double2* run_passes(bool forward, FftPassArgs a, const double2* in, const double* xr, int64_t in_batch,
                            double2* out, double* out_real, int64_t out_batch, int batch, double2* scratch,
                            hipStream_t s, int p_begin = 0, int p_end = -1) const;
};

// Pointwise spectral operations (contraction off: Go complex128 arithmetic).
// corr:    a[k] = a[k] * conj(b[k])                          (correlate.go:150-156)
// naive:   a[k] = a[k] / b[k]; first k with |b[k]| < 1e-15 -> *bad (atomicMin) (deconvolve.go:146-154)
// reg:     a[k] = a[k] * conj(b[k]) / (|b[k]|^2 + eps)       (deconvolve.go:208-213, 298-303)
// invfilt: a[k] = conj(a[k]) / (|a[k]|^2 + eps)              (deconvolve.go:384-389)
enum SpecOp { kSpecCorr = 0, kSpecNaive = 1, kSpecReg = 2, kSpecInvFilt = 3 };
// Words of device scratch correlate_half's `amax` needs (zeroed once at
// allocation: the max-abs kernel leaves its counter at zero after each call).
constexpr int kAbsmaxMaxGroups = 8192;  // partials per signal, at most (k_absmax2 workgroups; k_corr_split0's N / 256 / F)
constexpr int kAbsmaxWords = 8 + 2 * kAbsmaxMaxGroups;
void launch_spec_op(int op, double2* a, const double2* b, int64_t n, double eps, unsigned long long* bad,
                    hipStream_t s);

}  // namespace adsp
