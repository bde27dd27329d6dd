/* The chain through libvsig.so's C ABI from plain C (no Python, no HIP
 * headers): what a non-Python caller of the reference's utils.py functions
 * would link against.  Host buffers in, host buffers out.
 *
 *   x      = 3 tones + LCG noise + a QPSK preamble planted at K0
 *   y      = FIR(x)                  vsig_fir_c64      (np.convolve(x, h)[:n])
 *   Sxx    = spectrogram(y)          vsig_psd_c64      (utils.py:281-291, Hann 1024)
 *   peak   = correlate(y, tmpl)      vsig_correlate_c64 + fused find_correlation_peak
 *
 * Build (see tests/test_host_cpu.py::test_c_example_compiles):
 *   gcc -std=c99 -O2 -Iinclude examples/chain_c.c -Lvector_amd -lvsig \
 *       -Wl,-rpath,'$ORIGIN/../vector_amd' -lm -o examples/chain_c
 * Run on an MI355X: ./examples/chain_c   (exit status 0 = the preamble was found at K0)
 */
#define _USE_MATH_DEFINES
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include "vsig.h"

#define N (1 << 20)
#define NTAPS 63
#define L 512
#define NFFT 1024
#define K0 300001
#ifndef M_PI
#define M_PI 3.14159265358979323846
#endif

static uint64_t lcg = 20250718u;
static float urand(void) {                       /* uniform in (-1, 1) */
  lcg = lcg * 6364136223846793005ull + 1442695040888963407ull;
  return (float)((double)(lcg >> 11) / 9007199254740992.0 * 2.0 - 1.0);
}

#define CHECK(call)                                                              \
  do {                                                                           \
    int rc_ = (call);                                                            \
    if (rc_ != VSIG_OK) {                                                        \
      fprintf(stderr, "%s: %s (%s)\n", #call, vsig_errstr(rc_),                  \
              ctx ? vsig_last_error(ctx) : "");                                  \
      return 1;                                                                  \
    }                                                                            \
  } while (0)

int main(void) {
  vsig_ctx* ctx = NULL;
  float* x = malloc(sizeof(float) * 2 * N);
  float* y = malloc(sizeof(float) * 2 * N);
  float* pre = malloc(sizeof(float) * 2 * L);
  float* tmpl = malloc(sizeof(float) * 2 * L);
  float* taps = malloc(sizeof(float) * NTAPS);
  float* win = malloc(sizeof(float) * NFFT);
  const int64_t nframes = N / NFFT;
  float* sxx = malloc(sizeof(float) * (size_t)nframes * NFFT);
  if (!x || !y || !pre || !tmpl || !taps || !win || !sxx) return 2;

  /* windowed-sinc lowpass (cutoff 0.25 of Nyquist), Hann window for the PSD */
  for (int k = 0; k < NTAPS; ++k) {
    const double m = k - (NTAPS - 1) / 2.0, fc = 0.125;
    const double s = m == 0.0 ? 2 * fc : sin(2 * M_PI * fc * m) / (M_PI * m);
    taps[k] = (float)(s * (0.54 - 0.46 * cos(2 * M_PI * k / (NTAPS - 1))));
  }
  double wsum = 0.0;
  for (int i = 0; i < NFFT; ++i) {
    win[i] = (float)(0.5 - 0.5 * cos(2 * M_PI * i / NFFT));   /* periodic, get_window('hann') */
    wsum += win[i];
  }
  /* capture: tones + noise, preamble planted at K0 */
  for (int64_t i = 0; i < N; ++i) {
    const double p1 = 2 * M_PI * 0.05 * (double)i, p2 = 2 * M_PI * 0.11 * (double)i;
    x[2 * i] = (float)(cos(p1) + 0.5 * cos(p2)) + 0.7f * urand();
    x[2 * i + 1] = (float)(sin(p1) + 0.5 * sin(p2)) + 0.7f * urand();
  }
  for (int k = 0; k < L; ++k) {
    pre[2 * k] = (urand() > 0 ? 1.f : -1.f) * 0.70710678f;
    pre[2 * k + 1] = (urand() > 0 ? 1.f : -1.f) * 0.70710678f;
    x[2 * (K0 + k)] += 4.f * pre[2 * k];
    x[2 * (K0 + k) + 1] += 4.f * pre[2 * k + 1];
  }

  CHECK(vsig_init(0, &ctx));
  /* the template is the preamble as it leaves the filter (causal part) */
  CHECK(vsig_fir_c64(ctx, pre, L, taps, NTAPS, 1, tmpl, L));
  CHECK(vsig_fir_c64(ctx, x, N, taps, NTAPS, 1, y, N));
  CHECK(vsig_psd_c64(ctx, y, N, win, NFFT, NFFT, NFFT, (float)(1.0 / (wsum * wsum)), 0, sxx,
                     nframes));
  vsig_peak_t pk;
  CHECK(vsig_correlate_c64(ctx, y, N, tmpl, L, VSIG_MODE_VALID, NULL, &pk));
  vsig_free(ctx);

  double e0 = 0.0;
  for (int k = 0; k < NFFT; ++k) e0 += sxx[k];
  const int64_t nout = N - L + 1;
  const double mean = pk.sum_abs / nout, var = pk.sum_abs2 / nout - mean * mean;
  printf("filter+spectrum+sync over %d samples: frame-0 power %.4f, peak |c| %.2f at %lld "
         "(planted %d), confidence %.3f\n",
         N, e0, pk.peak, (long long)pk.index, K0, fmin(1.0, (pk.peak - mean) / sqrt(var) / 10.0));
  free(x); free(y); free(pre); free(tmpl); free(taps); free(win); free(sxx);
  return pk.index == K0 && isfinite(e0) ? 0 : 1;
}
