/* vsig — MI355X-native vector-signal DSP hot path, C ABI (libvsig.so).
 *
 * The reference (ramiyako/vector) is a pure-Python module whose DSP lives in
 * utils.py and calls numpy/scipy directly; it has no FFI.  Each entry point
 * below replaces one numpy/scipy call the reference makes on its hot path, and
 * is what a ctypes / cffi binding in place of that call would bind
 * (INTEGRATION.md shows the binding):
 *
 *   vsig_psd_*        scipy.signal.spectrogram(..., return_onesided=False,
 *                     detrend=False, scaling='spectrum')      utils.py:281-291
 *                     (+ fftshift of Sxx, utils.py:351, when shift = 1)
 *   vsig_fir_*        np.convolve(x, taps, 'full')[:len(x)] then x[::decim]
 *                     (reference idioms utils.py:802,816 and utils.py:194)
 *   vsig_correlate_*  np.correlate(signal2, signal1, mode) in
 *                     cross_correlate_signals                  utils.py:1284-1285
 *   vsig_xcorr_*      the same, streaming form with a fixed template, fused
 *                     with find_correlation_peak               utils.py:1321-1334
 *   vsig_peak_*       find_correlation_peak's |c| argmax / mean / std
 *                                                               utils.py:1321-1334
 *
 * Conventions
 *   - complex data is interleaved float32 pairs (numpy complex64 layout);
 *     complex128 only where stated.
 *   - "_dev" functions take device pointers and enqueue on the context's
 *     stream (vsig_set_stream); they do not synchronise.  Host-pointer
 *     functions copy in, compute and copy out synchronously.
 *   - the caller allocates every output; the library never frees caller
 *     memory.  Output sizes follow the formulas in the comments.
 *   - every function returns VSIG_OK (0) or a negative status; nothing throws
 *     across the ABI.  vsig_last_error(ctx) gives a message.
 *   - one context per host thread.
 */
#ifndef VSIG_H
#define VSIG_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define VSIG_OK 0
#define VSIG_E_INVALID -1     /* bad argument (size, mode, null pointer ...) */
#define VSIG_E_HIP -2         /* HIP runtime error */
#define VSIG_E_NOMEM -3       /* device allocation failed */
#define VSIG_E_UNSUPPORTED -4 /* size outside what the kernels implement */
#define VSIG_E_NODEVICE -5    /* no HIP device */
#define VSIG_E_REFINE -6      /* the exact-argmax refine faulted (watchdog, status 3):
                                 the peak record must not be used */

#define VSIG_MODE_VALID 0
#define VSIG_MODE_FULL 1
#define VSIG_MODE_SAME 2

#define VSIG_DTYPE_C128 0
#define VSIG_DTYPE_C64 1
#define VSIG_DTYPE_F64 2
#define VSIG_DTYPE_F32 3

typedef struct vsig_ctx vsig_ctx;
typedef struct vsig_fir vsig_fir;
typedef struct vsig_xcorr vsig_xcorr;

/* Result of a |c| peak reduction (find_correlation_peak, utils.py:1321-1334).
 * index: first maximum of |c|; peak: |c[index]|; sums over every element.
 * From the fused correlators (a peak record without a stored c) the sums are
 * fp32 per-thread sums of the fp32 |c|, combined in double: relative error
 * ~1e-7, so the single-pass variance var = sum_abs2/n - (sum_abs/n)^2 carries
 * ~1e-7 x (sum_abs2/n) / var.  find_correlation_peak's confidence formed from
 * them is within 1e-5 of numpy's while var >= 0.05 sum_abs2/n (noise-like
 * |c|: 0.21); below that (a flat |c|: a tone, a tone under weak noise) use
 * vsig_correlate_stats_dev for numpy's own mean / std -- the Python front end
 * (correlate_peak) does exactly that (tests/test_gpu_refine.py, tone under
 * noise at 0-60 dB).  An index of -1 means the record is invalid (a refine
 * fault, VSIG_E_REFINE / vsig_refine_status 3). */
typedef struct vsig_peak_t {
  double peak;
  int64_t index;
  double sum_abs;
  double sum_abs2;
} vsig_peak_t;

int vsig_version(void);
const char* vsig_errstr(int status);

/* ---- context ------------------------------------------------------------- */
int vsig_init(int device, vsig_ctx** out);
void vsig_free(vsig_ctx* ctx);
const char* vsig_last_error(const vsig_ctx* ctx);
/* hip_stream: the hipStream_t to enqueue on; NULL is the default (null)
 * stream.  A new context starts on a private non-blocking stream. */
int vsig_set_stream(vsig_ctx* ctx, void* hip_stream);
/* The hipStream_t the context enqueues on. */
void* vsig_get_stream(vsig_ctx* ctx);
/* Copy bytes between device or host buffers, ordered on the context's stream. */
int vsig_copy_dev(vsig_ctx* ctx, void* dst, const void* src, int64_t bytes);
int vsig_synchronize(vsig_ctx* ctx);
/* Options of the correlators' exact-argmax refine pass (refine.hip):
 *   "refine"          1 (default): after every correlation, the outputs whose
 *                     fp32 |c| lies within the band below the fp32 maximum are
 *                     recomputed by direct sums in double precision, and the
 *                     ones that can be the maximum once more in numpy's own
 *                     operation order (OpenBLAS zdotu + numpy's complex abs),
 *                     in the operands' own precision; the record's peak /
 *                     index are replaced by numpy's -- np.argmax over
 *                     np.abs(np.correlate) in complex128, to the bit;
 *                     0: the fp32 FFT result only -- for the fused correlators
 *                     (M >= 16384) the peak is then |c| with the low 6 mantissa
 *                     bits of |c|^2 replaced by the output's rank in its thread
 *                     (up to 3.8e-6 relative low; near-ties within 2^-17
 *                     decided by that rank, not by the lowest index);
 *   "blas_threads"    OpenBLAS threads of the numpy being matched (default 1;
 *                     the Python front end sets numpy's own): its zdotu splits
 *                     sums of more than 10000 terms into that many chunks;
 *   "refine_eps_ppm"  the band, relative to max |c| (default 1000 = 1e-3; the
 *                     fp32 correlation error is ~1e-8 of |p| |s_segment|);
 *   "refine_cap"      0 (default): no limit -- every candidate output is
 *                     evaluated in numpy's order however many there are (a
 *                     flat |c|, e.g. a tone, puts every full-overlap output in
 *                     the band; those run in refine.hip's dense form, about
 *                     1 ms per 2^20 outputs x 4096 terms); > 0 (>= 4096): an
 *                     explicit limit on candidate outputs -- beyond it the
 *                     record is left as the fp32 pass produced it and
 *                     vsig_refine_status reports status 1;
 *   "refine_watchdog_us" bound on the one-launch refine's two waits (default
 *                     2000000; a test hook: tiny values force a fire, status 3);
 *   "refine_async"    0 (default): the refine runs on the context stream after
 *                     its correlator; 1: the refine of vsig_xcorr_exec_dev runs
 *                     on the context's own refine stream (vsig_refine_stream),
 *                     behind an event after the correlator, so the caller's next
 *                     kernels (e.g. the next chunk's filter) overlap it.  The
 *                     peak record is then complete only on the refine stream:
 *                     read it after vsig_refine_join (the context stream waits
 *                     for the last refine) or order its consumers on
 *                     vsig_refine_stream; the caller must not overwrite the
 *                     correlated stream before that.  The library itself joins
 *                     before it reuses the refine's scratch (any later
 *                     correlation, peak, statistics or staging call), and
 *                     vsig_refine_status / vsig_synchronize wait for it. */
int vsig_set_option(vsig_ctx* ctx, const char* key, int value);
int vsig_get_option(const vsig_ctx* ctx, const char* key, int* value);
/* The hipStream_t the "refine_async" refine runs on (the context stream when
 * the option is off), and the join: the context stream waits for the last
 * refine (an event; no host synchronisation). */
void* vsig_refine_stream(vsig_ctx* ctx);
int vsig_refine_join(vsig_ctx* ctx);
/* Outcome of the context's last refine pass (synchronises the stream):
 * status 0 refined, 1 skipped (more candidate outputs than a refine_cap set
 * > 0), 2 no pass ran (refine off, or no correlation yet), 3 the one-launch
 * refine's watchdog fired in some pass since the last call (a block waited
 * longer than the "refine_watchdog_us" option, default 2 s, for the published
 * keys: a device fault, never seen in operation).  Status 3 is an error: the
 * record's index is poisoned (-1) and its values must not be used; this call
 * reports it once and clears the refine's counters so the context's next
 * correlation starts clean (vsig_chain_result returns VSIG_E_REFINE instead);
 * candidates =
 * candidate items (thread columns of the M = 16384 / 32768 correlators, waves
 * of the M = 4096 / 8192 ones, 64-output chunks of a stored array). */
int vsig_refine_status(vsig_ctx* ctx, int32_t* status, int64_t* candidates);
/* Hash of the kernel / ABI sources this library was built from (the Python
 * loader compares it with the sources next to it and refuses a stale build). */
const char* vsig_build_id(void);
/* Per-kernel timing with HIP events on the context stream (for bench.py):
 * enable, run, then read the mean duration in ms of each kernel family. */
int vsig_timing_enable(vsig_ctx* ctx, int on);
int vsig_timing_read(vsig_ctx* ctx, const char* kernel, double* total_ms, int64_t* launches);
int vsig_timing_reset(vsig_ctx* ctx);
/* Per-stage effective clock (a diagnostic, for bench.py's untimed clock steps):
 * while enabled (enable zeroes the sums), the FIR, PSD, correlator and PFB
 * kernels sample the shader clock and the 100 MHz real-time counter at the
 * start and end of every 64th block (wave 0); read returns the mean clock in
 * GHz of a kernel family over those blocks' lifetimes (0 if none ran) and the
 * real-time ticks it averaged over. */
int vsig_clock_enable(vsig_ctx* ctx, int on);
int vsig_clock_read(vsig_ctx* ctx, const char* kernel, double* ghz, int64_t* ticks);

/* ---- spectrum: Sxx[f, k] = |sum_{i<nperseg} w[i] x[f*hop + i] e^{-2 pi j k i / nfft}|^2 * scale
 * nfft: any length >= nperseg up to 2^27 (powers of two in [64, 2^28]: in-LDS plans, above
 *   16384 a four-step FFT per frame; other lengths: Bluestein per frame, bigfft.hip);
 * nframes = (n - nperseg) / hop + 1;
 * sxx is frame-major float32 [nframes][nfft] (Sxx of scipy is its transpose);
 * shift = 1 stores bin k at (k + nfft/2) % nfft (np.fft.fftshift).
 * _dev only: stride reads sample i at x[i*stride] (n counts strided samples),
 * which folds create_spectrogram's sig[::factor] (utils.py:194) into the load. */
int vsig_psd_c64_dev(vsig_ctx* ctx, const void* x, int64_t n, int64_t stride, const float* win,
                     int32_t nperseg, int64_t hop, int32_t nfft, float scale, int32_t shift,
                     float* sxx, int64_t nframes);
int vsig_psd_c64(vsig_ctx* ctx, const void* x, int64_t n, const float* win, int32_t nperseg,
                 int64_t hop, int32_t nfft, float scale, int32_t shift, float* sxx,
                 int64_t nframes);

/* ---- FIR: y[g] = sum_{m<ntaps} h[m] x[g*decim - m] (x = 0 outside [0, n)),
 * g in [0, ceil(n/decim)).  Taps complex64 on the host (real taps: imag = 0);
 * any ntaps >= 1 (np.convolve's contract, utils.py:802,816): up to 8192 one
 * overlap-save pass, beyond that 8192-tap parts run undecimated and summed with
 * their delays (a scratch of n samples). */
int vsig_fir_create(vsig_ctx* ctx, const void* taps, int32_t ntaps, int32_t decim, vsig_fir** out);
void vsig_fir_free(vsig_fir* fir);
/* Overlap-save block size M chosen for the taps (0 for a null handle). */
int vsig_fir_block(const vsig_fir* fir);
int vsig_fir_exec_dev(vsig_fir* fir, const void* x, int64_t n, void* y, int64_t ny);
/* Time-chunk form: x points at nhist history samples (the previous chunk's
 * last samples, the left halo) followed by the n samples to filter; y gets the
 * ceil(n/decim) outputs of those n samples, exactly as if the whole stream
 * had been filtered at once. */
int vsig_fir_exec_hist_dev(vsig_fir* fir, const void* x, int64_t nhist, int64_t n, void* y,
                           int64_t ny);
/* The same with the NCO mixer of apply_frequency_shift (utils.py:120-127)
 * fused into the FIR's loads: filters x[i] * exp(2j*pi*freq_shift*t_i),
 * t_i = (i0 + i) / sample_rate, i0 = global sample index of x[0] (the first
 * history sample), i.e. vsig_mix_c64_dev then vsig_fir_exec_hist_dev in one
 * pass.  freq_shift == 0: plain filter.  Needs the default FIR variant and
 * the 1024-point block (ntaps <= 256); else VSIG_E_UNSUPPORTED (mix first). */
int vsig_fir_exec_mix_dev(vsig_fir* fir, const void* x, int64_t nhist, int64_t n, void* y,
                          int64_t ny, double freq_shift, double sample_rate, int64_t i0);
int vsig_fir_c64(vsig_ctx* ctx, const void* x, int64_t n, const float* taps, int32_t ntaps,
                 int32_t decim, void* y, int64_t ny);
/* ---- streaming correlation with a fixed template p of L samples (any L >= 1;
 * L > 8192 runs as one pass per 8192-sample chunk, accumulated in c):
 * c[o] = sum_{k<L} s[o - off + k] conj(p[k]), mode VALID (off = 0, nout = n-L+1)
 * or FULL (off = L-1, nout = n+L-1).  c may be NULL (peak only).  peak_dev: a
 * device vsig_peak (may be NULL); peak = max |c|, sums over all nout outputs;
 * the peak / index are refined (see "refine" above). */
int vsig_xcorr_create(vsig_ctx* ctx, const void* tmpl, int64_t L, vsig_xcorr** out);
void vsig_xcorr_free(vsig_xcorr* xc);
int vsig_xcorr_exec_dev(vsig_xcorr* xc, const void* s, int64_t n, int32_t mode, void* c,
                        vsig_peak_t* peak_dev);

/* ---- general correlation, np.correlate(a, v, mode) semantics for any length
 * order (cross_correlate_signals, utils.py:1279-1285): output length full
 * na+nv-1, valid |na-nv|+1, same max(na, nv).  The FFT pass runs in complex64;
 * dtype VSIG_DTYPE_C128 takes complex128 operands (converted for the FFT pass,
 * kept for the refine pass), out_dtype VSIG_DTYPE_C128 writes c as complex128
 * with the refined outputs patched in (exact near the peak, fp32 accuracy
 * elsewhere).  The shorter operand up to 8192 samples runs as one streaming
 * pass; longer ones as a sum over 8192-sample chunks of it (one pass per
 * chunk, accumulated in c -- a device scratch c when c is NULL).  All pointers
 * device (dev) or host.  The _c64 forms are dtype = out_dtype = C64. */
int vsig_correlate_dev(vsig_ctx* ctx, int32_t dtype, const void* a, int64_t na, const void* v,
                       int64_t nv, int32_t mode, int32_t out_dtype, void* c, vsig_peak_t* peak_dev);
int vsig_correlate(vsig_ctx* ctx, int32_t dtype, const void* a, int64_t na, const void* v,
                   int64_t nv, int32_t mode, int32_t out_dtype, void* c, vsig_peak_t* peak);
int vsig_correlate_c64_dev(vsig_ctx* ctx, const void* a, int64_t na, const void* v, int64_t nv,
                           int32_t mode, void* c, vsig_peak_t* peak_dev);
int vsig_correlate_c64(vsig_ctx* ctx, const void* a, int64_t na, const void* v, int64_t nv,
                       int32_t mode, void* c, vsig_peak_t* peak);

/* ---- transforms of any length (bigfft.hip: four-step FFT on the in-LDS engine
 * for powers of two above 16384, Bluestein / chirp-z for every other length,
 * up to 2^27 points; complex64 arithmetic).
 * vsig_dft_dev: batch frames of n contiguous samples, y[f][k] = sum_j x[f][j]
 *   e^{-+2 pi i jk/n} (inverse: + and 1/n, numpy.fft's convention).
 * vsig_resample_dev: scipy.signal.resample(x, num) as resample_signal calls it
 *   (utils.py:107-118): spectrum of x, its bins copied / the Nyquist bin split
 *   or folded into num bins, inverse transform, * num / n; y complex64[num]
 *   (real_input: imaginary part 0, scipy's rfft path).
 * vsig_filter_channel_dev: split_channels.filter_channel (vector_analyzer/
 *   split_channels.py:15-44) as written, CENTER_FREQ 5230 MHz: brick-wall mask
 *   on fftfreq(n, 1/sr) * sr + CENTER_FREQ, the negative half replaced by the
 *   conjugate mirror of the masked non-negative half, inverse FFT, real part
 *   (y float64[n]).  Odd n > 1: VSIG_E_INVALID (numpy's shape mismatch). */
int vsig_dft_dev(vsig_ctx* ctx, int32_t dtype, const void* x, int64_t n, int64_t batch,
                 int32_t inverse, int32_t out_dtype, void* y);
int vsig_resample_dev(vsig_ctx* ctx, int32_t dtype, const void* x, int64_t n, int64_t num,
                      int32_t real_input, void* y);
int vsig_filter_channel_dev(vsig_ctx* ctx, int32_t dtype, const void* x, int64_t n,
                            double center_freq, double sample_rate, double bandwidth, double* y);

/* ---- |c| reduction in double precision over an array of dtype VSIG_DTYPE_*:
 * index of the first max of |c|, the max, sum |c|, sum |c|^2. */
int vsig_peak_dev(vsig_ctx* ctx, int32_t dtype, const void* a, int64_t n, vsig_peak_t* peak_dev);
int vsig_peak(vsig_ctx* ctx, int32_t dtype, const void* a, int64_t n, vsig_peak_t* peak);
/* find_correlation_peak's mean_corr / std_corr (utils.py:1329-1330) exactly as
 * numpy forms them: np.mean(np.abs(a)) and np.std(np.abs(a)) in float64, by
 * numpy's pairwise summation over 8192-element buffers (two passes).
 * stats_dev: device double[2] = {mean, std}.  dtype VSIG_DTYPE_C128 or
 * VSIG_DTYPE_F64 (cross_correlate_signals' output is complex128). */
int vsig_abs_stats_dev(vsig_ctx* ctx, int32_t dtype, const void* a, int64_t n, double* stats_dev);
/* The same statistics of |np.correlate(a, v, mode)| without the correlation
 * array: every output evaluated in numpy's operation order (the refine pass's
 * dense form; O(nout x min(na, nv)) fp64 FMAs, about 1 ms per 2^20 outputs x
 * 4096 terms) -- the exact confidence for a flat |c|, where the fused
 * correlators' fp32 sums cannot resolve numpy's rounding-noise std. */
int vsig_correlate_stats_dev(vsig_ctx* ctx, int32_t dtype, const void* a, int64_t na, const void* v,
                             int64_t nv, int32_t mode, double* stats_dev);

/* ---- stream ops either side of the chain.
 * vsig_mix_c64_dev: y[i] = x[i] * exp(j w (i0 + i) / sr) — apply_frequency_shift
 *   (utils.py:120-127) with w = 2*pi*freq_shift as numpy forms it.
 * vsig_scale_c64_dev: y = x * s (transplant_packet_in_vector power scale,
 *   utils.py:1481-1496).
 * vsig_wv_quantize_dev: SMU-WV int16 I/Q interleave of mat2wv
 *   (vector_analyzer/mat_to_wv_converter.py:28-50); norm > 0 divides by norm
 *   first (bNormalize, norm = max |x|); out holds 2n int16.
 * vsig_planar_to_c64_dev: MAT v5 real / imaginary planes of storage type
 *   mi_type (miINT8 1 .. miDOUBLE 9, miINT64 12, miUINT64 13; im may be NULL)
 *   -> complex64 (load_packet, utils.py:48-86).
 * vsig_c64_to_planar_dev: complex64 -> float32 planes (save_vector,
 *   utils.py:659-670). */
int vsig_mix_c64_dev(vsig_ctx* ctx, const void* x, int64_t n, double w, double sr, int64_t i0,
                     void* y);
int vsig_scale_c64_dev(vsig_ctx* ctx, const void* x, int64_t n, float s, void* y);
int vsig_wv_quantize_dev(vsig_ctx* ctx, const void* x, int64_t n, float norm, int16_t* out);
int vsig_planar_to_c64_dev(vsig_ctx* ctx, int32_t mi_type, const void* re, const void* im,
                           int64_t n, void* y);
int vsig_c64_to_planar_dev(vsig_ctx* ctx, const void* x, int64_t n, float* re, float* im);

/* ---- polyphase channelizer (BASELINE config 4; no reference counterpart,
 * nearest analogue vector_analyzer/split_channels.py:15-44):
 * y[m*nchan + k] = sum_p z_m[p] e^{-2 pi j k p / nchan},
 * z_m[p] = sum_q h[q*nchan + p] x[(m + q)*nchan + p];
 * nchan in {64, 128, 256}, ntaps = {4, 8, 16} * nchan,
 * nframes = (n - ntaps) / nchan + 1; y frame-major (nframes x nchan). */
int vsig_pfb_c64_dev(vsig_ctx* ctx, const void* x, int64_t n, const float* h, int32_t ntaps,
                     int32_t nchan, void* y, int64_t nframes);

/* ---- analysis (normalize_spectrogram utils.py:356-404, find_packet_start /
 * detect_packet_bounds utils.py:784-825).  All operate on |a|.
 * vsig_select_dev: k-th smallest |a| for up to 4 0-based ranks (host output;
 *   np.percentile / np.median are interpolations of these).
 * vsig_threshold_dev: count / first / last index of |a| >= thr and max |a|.
 * vsig_boxcar_energy_dev: sm = np.convolve(np.abs(x)**2, ones(w)/w, 'same')
 *   in double (x of any VSIG_DTYPE; sm: max(n, w) doubles on the device).
 * vsig_db_dev: out = 10 log10(|a| + floor), F32 -> float32 math and output,
 *   F64 -> double (numpy's promotion in normalize_spectrogram).
 * vsig_abs_c64_dev / vsig_abs_c128_dev: out = |a| + 0j as complex64 / complex128
 *   (a of any VSIG_DTYPE; np.abs as numpy forms it). */
int vsig_select_dev(vsig_ctx* ctx, int32_t dtype, const void* a, int64_t n, const int64_t* ranks,
                    int32_t nranks, double* values);
int vsig_threshold_dev(vsig_ctx* ctx, int32_t dtype, const void* a, int64_t n, double thr,
                       int64_t* count, int64_t* first, int64_t* last, double* maxval);
int vsig_boxcar_energy_dev(vsig_ctx* ctx, int32_t dtype, const void* x, int64_t n, int64_t w,
                           double* sm);
int vsig_db_dev(vsig_ctx* ctx, int32_t dtype, const void* a, int64_t n, double floor_, void* out);
int vsig_abs_c64_dev(vsig_ctx* ctx, int32_t dtype, const void* a, int64_t n, void* out);
int vsig_abs_c128_dev(vsig_ctx* ctx, int32_t dtype, const void* a, int64_t n, void* out);

/* ---- time-chunk shard of the streaming chain (chain.hip; the C form of
 * vector_amd/shard.py StreamChain; reference precedent: the
 * overlapped chunking of heavy_packet_optimizer.py:114-152).  Rank r of world
 * owns input samples [r n, (r+1) n) of one capture; per step: left halo
 * (hist = ntaps-1 input samples rounded up to a multiple of 16, so that the
 * FIR's segments start on 128-byte lines: the last hist samples of rank r-1;
 * world > 1 needs n >= hist) -> FIR + decimate -> right halo (L-1
 * filtered samples from rank r+1) -> PSD (nfft, hop nfft) -> valid
 * correlation with the template + exact peak -> all-gather of the 32-byte
 * peak records.  Results equal one chain over the whole capture.
 * n must be a multiple of nfft * decim; taps / tmpl complex64 host arrays;
 * window float32[nfft] host; psd_scale = 1 / sum(window)^2 for 'spectrum'
 * scaling; tmpl = NULL: no sync stage. */
typedef struct vsig_chain_config {
  int64_t n_local;
  const void* taps;
  int32_t ntaps;
  int32_t decim;
  int32_t nfft;
  const float* window;
  float psd_scale;
  const void* tmpl;
  int64_t L;
} vsig_chain_config;

/* How ranks exchange: sendrecv sends send_bytes of device memory to rank dst
 * and receives recv_bytes into recv from rank src (dst / src < 0: none),
 * ordered on hip_stream; allgather gathers `bytes` from every rank into recv
 * (world * bytes, rank order).  Return 0 on success. */
typedef struct vsig_transport {
  void* user;
  int (*sendrecv)(void* user, const void* send, int64_t send_bytes, int32_t dst, void* recv,
                  int64_t recv_bytes, int32_t src, void* hip_stream);
  int (*allgather)(void* user, const void* send, void* recv, int64_t bytes, void* hip_stream);
} vsig_transport;

typedef struct vsig_chain vsig_chain;
/* tr may be NULL for world = 1.  The chain enqueues on ctx's stream. */
int vsig_chain_create(vsig_ctx* ctx, const vsig_chain_config* cfg, int32_t rank, int32_t world,
                      const vsig_transport* tr, vsig_chain** out);
void vsig_chain_free(vsig_chain* chain);
const char* vsig_chain_last_error(const vsig_chain* chain);
/* Device complex64[n_local]: this rank's input chunk (fill before a step). */
void* vsig_chain_input(vsig_chain* chain);
int vsig_chain_step(vsig_chain* chain);
/* The global peak of the last step (index in the whole filtered, decimated
 * capture; sums over all nout outputs); synchronises. */
int vsig_chain_result(vsig_chain* chain, vsig_peak_t* peak, int64_t* nout);
/* This rank's filtered stream (complex64[n]) and spectra (frame-major float32
 * [nframes][nfft]) on the device. */
const void* vsig_chain_filtered(const vsig_chain* chain, int64_t* n);
const float* vsig_chain_spectra(const vsig_chain* chain, int64_t* nframes);

/* RCCL over xGMI as the transport (librccl resolved at run time: an RCCL
 * already in the process -- e.g. torch's -- is shared; VSIG_RCCL_LIB names
 * another).  comm is an ncclComm_t; vsig_rccl_comm_init makes one per rank
 * from a unique id that rank 0 creates and the launcher distributes. */
int vsig_rccl_available(void);
int vsig_rccl_unique_id(char id[128]);
int vsig_rccl_comm_init(int32_t world, int32_t rank, const char id[128], int32_t device, void** comm);
int vsig_rccl_comm_destroy(void* comm);
int vsig_rccl_transport(void* comm, vsig_transport* out);

/* In-process loopback transport: ranks as host threads of one process (one
 * context each), halos copied device to device -- several ranks on one GPU
 * for tests, or ranks on the GPUs of one process. */
typedef struct vsig_loopback vsig_loopback;
int vsig_loopback_create(int32_t world, vsig_loopback** out);
void vsig_loopback_free(vsig_loopback* lb);
int vsig_loopback_transport(vsig_loopback* lb, int32_t rank, vsig_transport* out);

#ifdef __cplusplus
}
#endif
#endif /* VSIG_H */
