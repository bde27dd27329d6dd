// numpy's complex magnitude on the device (gfx950), shared by the |c| reductions
// (reduce.hip), the refine (refine.hip) and the packet detectors (analysis.hip).
#pragma once
#include <hip/hip_runtime.h>

namespace vsig {

// numpy's complex abs (np.abs on complex128 / complex64, numpy 2.x SIMD loop
// loops_unary_complex, oracle/npdot.c np_cabs): L * sqrt(fma(r, r, 1)),
// r = S / L with L / S the larger / smaller of |re|, |im| (r = 0 where L == 0
// or S == inf) -- not hypot, which differs from it in about a third of the
// inputs.  Correctly rounded div / sqrt / mul / fma: numpy's value to the bit
// (fp32 ones through double: 53 >= 2*24 + 2, no double-rounding error).
__device__ __forceinline__ double np_cabs(double re, double im) {
  double a = fabs(re), b = fabs(im);
  if (isinf(a) || isinf(b)) return __builtin_inf();
  const double L = a > b ? a : b, S = b < a ? b : a;
  const double r = L == 0.0 ? 0.0 : __ddiv_rn(S, L);
  return __dmul_rn(L, __dsqrt_rn(fma(r, r, 1.0)));
}
__device__ __forceinline__ float np_cabs(float re, float im) {
  const float a = fabsf(re), b = fabsf(im);
  if (isinf(a) || isinf(b)) return __builtin_inff();
  const float L = a > b ? a : b, S = b < a ? b : a;
  const float r = L == 0.f ? 0.f : (float)((double)S / (double)L);
  const float q = (float)sqrt((double)fmaf(r, r, 1.f));
  return (float)((double)L * (double)q);
}

}  // namespace vsig
