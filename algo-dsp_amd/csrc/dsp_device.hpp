// Device helpers shared by the per-sample processor kernels
// (dsp_kernels.hip, fx_staged.hip).
#pragma once

#include <hip/hip_runtime.h>

#include "dsp_kernels.hpp"

namespace adsp {

// Go math.Log2 (frexp split + Log(frac)*(1/Ln2) + exp), core.go via compressor_math.go:8-20.
// One envelope-follower step of dynamicsCore.detectorLevel (core.go:351-355):
//   src > env: env + (src - env) * attack      else: src + (env - src) * release
// Both branches are env + k (src - env) with k = attack or b = 1 - release, so
// the step is env + c1 (src - env) + c2 |src - env|, written as
//   fma(c2, |src - env|, fma(1 - c1, env, c1 src))
// with c1 = (attack + b)/2, c2 = (attack - b)/2 (CompParams::env_*).  The map
// is the reference's; the rounding is not (a few ulps on the envelope, which
// the gain's log2 / exp2 already make a tolerance).  The
// reference's form is a compare, a select and three dependent operations on
// the envelope, 109 clocks per sample for one wave on gfx950; this one has no
// compare or select (|.| is a source modifier) and two dependent FMAs: 24.5
// clocks (tools/chain_latency.hip).  The detector is config 5's longest
// recurrence, so its chain is the engine's floor.
__device__ __forceinline__ double env_step(const CompParams& p, double env, double src) {
  return __builtin_fma(p.env_c2, fabs(src - env), __builtin_fma(p.env_k1, env, p.env_c1 * src));
}

__device__ __forceinline__ double go_log2(double x) {
#pragma clang fp contract(off)
  int e;
  const double frac = frexp(x, &e);
  if (frac == 0.5) return (double)(e - 1);
  return log(frac) * 1.4426950408889634074 + (double)e;
}

// calculateDownwardExpansionGain (expander.go:358-411), Expander and Gate.
__device__ __forceinline__ double expansion_gain(const CompParams& p, double level) {
#pragma clang fp contract(off)
  if (level <= 0.0) return p.range_lin;
  const double undershoot = p.threshold_log2 - go_log2(level);
  double eff;
  if (!p.knee_on) {
    if (undershoot <= 0.0) return 1.0;
    eff = undershoot;
  } else {
    if (undershoot < -p.half_knee) return 1.0;
    if (undershoot > p.half_knee) {
      eff = undershoot;
    } else {
      const double s = undershoot + p.half_knee;
      eff = s * s * 0.5 * p.inv_knee_width_log2;
    }
  }
  const double g = exp2(-eff * p.ratio_m1);
  return g < p.range_lin ? p.range_lin : g;
}

// dynamicsCore.GainForLevel (core.go:288-329).  2^y via exp2 (Go:
// math.Pow(2, y); both within an ulp).  Expander/Gate modes dispatch to
// the downward-expansion gain.
__device__ __forceinline__ double gain_for_level(const CompParams& p, double level) {
#pragma clang fp contract(off)
  if (p.mode) return expansion_gain(p, level);
  if (level <= 0.0) return 1.0;
  const double overshoot = go_log2(level) - p.threshold_log2;
  if (!p.knee_on) {
    if (overshoot <= 0.0) return 1.0;
    return exp2(-overshoot * p.cf);
  }
  double eff;
  if (overshoot < -p.half_knee) return 1.0;
  if (overshoot > p.half_knee) {
    eff = overshoot;
  } else {
    const double s = overshoot + p.half_knee;
    eff = s * s * 0.5 * p.inv_knee_width_log2;
  }
  return exp2(-eff * p.cf);
}

}  // namespace adsp
