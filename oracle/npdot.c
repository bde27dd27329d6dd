/* numpy's complex128 np.correlate / np.dot and np.abs, operation for operation
 * -- TEST INFRASTRUCTURE ONLY (the checker of refine.hip's numpy-order pass;
 * never linked into the product).
 *
 * The reference's find_correlation_peak (utils.py:1321-1325) takes
 * np.argmax(np.abs(np.correlate(signal2, signal1))) over complex128 operands
 * (cross_correlate_signals, utils.py:1279-1285).  Where |c| has exact ties in
 * exact arithmetic (a tone against itself), which index wins is decided by the
 * rounding of numpy's own evaluation order, so parity needs that order:
 *
 *  np.correlate(a, v) (numpy 2.2.6 multiarray PyArray_Correlate2 ->
 *  _pyarray_correlate): v is conjugated into a new contiguous array, the longer
 *  operand becomes the first (output reversed if swapped), and each output is
 *  CDOUBLE_dot over the overlap in increasing index order -> cblas_zdotu_sub
 *  (one chunk below 2^30) -> OpenBLAS 0.3.29 zdotu_k.  The SkylakeX / Haswell /
 *  Zen kernel (read from the disassembly of numpy.libs/libscipy_openblas64_
 *  zdotu_k_SKYLAKEX, zdot_compute, zdot_kernel_8):
 *    - n8 = n & -8 complex in blocks of 8: four ymm accumulators A0..A3 take
 *      fma(x, y) over complex pairs (2r, 2r+1) of the block (lanes xr*yr,
 *      xi*yi per complex), four more A4..A7 fma(x, swap(y)) (xr*yi, xi*yr);
 *    - A0 = (A0 + A1) + (A2 + A3), A4 likewise, then low + high 128-bit halves:
 *      d0 = sum xr*yr, d1 = sum xi*yi, d2 = sum xr*yi, d3 = sum xi*yr;
 *    - scalar tail k = n8 .. n-1: d_j = fma(., ., d_j) in the same roles;
 *    - re = d0 - d1, im = d2 + d3, re = fma(im, 0, re);
 *    - n > 10000: split over the OpenBLAS threads (widths ceil(rest / threads
 *      left)), the partial results added in thread order onto 0.
 *  numpy adds the result onto a zero sum (CDOUBLE_dot).
 *
 *  np.abs on complex128 (numpy 2.x loops_unary_complex SIMD path, any
 *  contiguous array): larger = max(|re|, |im|), smaller = min, r = smaller /
 *  larger (0 where larger == 0 or smaller == inf), |c| = sqrt(fma(r, r, 1)) *
 *  larger.
 *
 * Checked against numpy itself in tests/test_npdot_cpu.py (bit-exact over
 * random operands of every length class, np.correlate in all modes and both
 * operand orders, np.abs, and the reference's tone goldens).
 * Build: gcc -O2 -ffp-contract=off -mfma -shared -fPIC (oracle/Makefile).
 */
#include <math.h>

static void zdot_compute(long n, const double* x, const double* y, double* re, double* im) {
  double d0 = 0.0, d1 = 0.0, d2 = 0.0, d3 = 0.0;
  const long n8 = n & ~7L;
  if (n8) {
    double A[8][4] = {{0}};
    for (long i = 0; i < n8; i += 8) {
      for (int r = 0; r < 4; ++r) {
        const double* xp = x + 2 * (i + 2 * r);
        const double* yp = y + 2 * (i + 2 * r);
        const double ys[4] = {yp[1], yp[0], yp[3], yp[2]};
        for (int j = 0; j < 4; ++j) {
          A[r][j] = fma(xp[j], yp[j], A[r][j]);
          A[4 + r][j] = fma(xp[j], ys[j], A[4 + r][j]);
        }
      }
    }
    double s[4], t[4];
    for (int j = 0; j < 4; ++j) {
      s[j] = (A[0][j] + A[1][j]) + (A[2][j] + A[3][j]);
      t[j] = (A[4][j] + A[5][j]) + (A[6][j] + A[7][j]);
    }
    d0 = s[0] + s[2];
    d1 = s[1] + s[3];
    d2 = t[0] + t[2];
    d3 = t[1] + t[3];
  }
  for (long k = n8; k < n; ++k) {
    const double xr = x[2 * k], xi = x[2 * k + 1], yr = y[2 * k], yi = y[2 * k + 1];
    d0 = fma(xr, yr, d0);
    d1 = fma(xi, yi, d1);
    d2 = fma(xr, yi, d2);
    d3 = fma(yr, xi, d3);
  }
  double r = d0 - d1;
  const double m = d2 + d3;
  r = fma(m, 0.0, r);
  *re = r;
  *im = m;
}

/* OpenBLAS zdotu_k (x86_64 zdot.c): threads only above 10000 complex. */
void np_zdotu(long n, const double* x, const double* y, long nthreads, double* out) {
  double re = 0.0, im = 0.0;
  if (n <= 10000 || nthreads <= 1) {
    zdot_compute(n, x, y, &re, &im);
  } else {
    long rest = n, off = 0;
    for (long t = 0; t < nthreads && rest > 0; ++t) {
      long w = (rest + (nthreads - t) - 1) / (nthreads - t);
      if (w > rest) w = rest;
      double pr, pi;
      zdot_compute(w, x + 2 * off, y + 2 * off, &pr, &pi);
      re = re + pr;
      im = im + pi;
      off += w;
      rest -= w;
    }
  }
  out[0] = 0.0 + re;
  out[1] = 0.0 + im;
}

/* np.correlate(a, v, mode) for complex128 a (na), v (nv); mode 0 valid, 1 same,
 * 2 full; out holds the mode's length.  vc: scratch of nv complex. */
void np_correlate(const double* a, long na, const double* v, long nv, int mode, long nthreads,
                  double* vc, double* out) {
  for (long k = 0; k < nv; ++k) { vc[2 * k] = v[2 * k]; vc[2 * k + 1] = -v[2 * k + 1]; }
  const double *p1 = a, *p2 = vc;
  long n1 = na, n2 = nv;
  int inv = 0;
  if (n1 < n2) { p1 = vc; p2 = a; n1 = nv; n2 = na; inv = 1; }
  long length = n1, n = n2, nl, nr;
  if (mode == 0) { length = length - n + 1; nl = nr = 0; }
  else if (mode == 1) { nl = n / 2; nr = n - nl - 1; }
  else { nl = nr = n - 1; length = length + n - 1; }
  const double* ip1 = p1;
  const double* ip2 = p2 + 2 * nl;
  n = n - nl;
  long o = 0;
  for (long i = 0; i < nl; ++i) {
    np_zdotu(n, ip1, ip2, nthreads, out + 2 * o++);
    n++;
    ip2 -= 2;
  }
  for (long i = 0; i < n1 - n2 + 1; ++i) {
    np_zdotu(n, ip1, ip2, nthreads, out + 2 * o++);
    ip1 += 2;
  }
  for (long i = 0; i < nr; ++i) {
    n--;
    np_zdotu(n, ip1, ip2, nthreads, out + 2 * o++);
    ip1 += 2;
  }
  if (inv)
    for (long i = 0, j = length - 1; i < j; ++i, --j) {
      const double r = out[2 * i], m = out[2 * i + 1];
      out[2 * i] = out[2 * j]; out[2 * i + 1] = out[2 * j + 1];
      out[2 * j] = r; out[2 * j + 1] = m;
    }
}

void np_cabs(const double* c, long n, double* out) {
  for (long i = 0; i < n; ++i) {
    double re = fabs(c[2 * i]), im = fabs(c[2 * i + 1]);
    if (re == INFINITY) im = INFINITY;
    if (im == INFINITY) re = INFINITY;
    if (isnan(re)) im = NAN;
    if (isnan(im)) re = NAN;
    const double larger = re > im ? re : im;
    const double smaller = im < re ? im : re;
    const int ok = !(larger == 0.0 || smaller == INFINITY);
    const double r = ok ? smaller / larger : 0.0;
    out[i] = sqrt(fma(r, r, 1.0)) * larger;
  }
}
