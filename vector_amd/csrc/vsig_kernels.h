// Internal interface between the C-ABI layer (vsig_api.hip) and the kernels.
#pragma once
#include <hip/hip_runtime.h>

namespace vsig {

// XCD-aware block order.  The dispatcher hands block b to XCD b % 8 and each
// XCD has its own L2, so with the identity mapping the overlap two
// neighbouring overlap-save segments share is fetched from HBM by two
// different L2s.  Remapping gives every XCD one contiguous run of segments
// (a bijection on [0, nb)), so the overlap of b and its successor (dispatched
// at about the same time to the same XCD) hits in L2.
__device__ __forceinline__ long long xcd_remap(long long b, long long nb) {
  const long long q = nb >> 3, r = nb & 7;
  const long long x = b & 7, i = b >> 3;
  return x * q + (x < r ? x : r) + i;
}

// Per-stage effective clock (vsig_clock_*, a diagnostic the bench runs in
// untimed steps after its timed loop).  When a launch gets a sink, wave 0 of
// every 64th block reads the shader clock (s_memtime) and the 100 MHz
// real-time counter (s_memrealtime) at its start and at its end and adds both
// differences into sink[0] / sink[1] by vector atomics; the clock over the
// sampled blocks' lifetimes is then sink[0] / sink[1] x 100 MHz.  With no sink
// (the default) nothing is read and nothing is written.
struct ClockStamp {
  unsigned long long t0 = 0, r0 = 0;
  bool on;
  __device__ __forceinline__ ClockStamp(unsigned long long* sink, unsigned long long blk)
      : on(sink != nullptr && (blk & 63) == 0) {
    if (on) {
      t0 = __builtin_amdgcn_s_memtime();
      r0 = __builtin_amdgcn_s_memrealtime();
      // lgkmcnt(0) alone: the counters' returns are retired here, so the
      // compiler's waits for the kernel's LDS reads stay counted (an SMEM read
      // left pending on one path makes every later LDS wait a full drain)
      __builtin_amdgcn_s_waitcnt(0xC07F);
    }
  }
  __device__ __forceinline__ void done(unsigned long long* sink) const {
    if (on && threadIdx.x < 2) {
      const unsigned long long t1 = __builtin_amdgcn_s_memtime();
      const unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
      atomicAdd(sink + threadIdx.x, threadIdx.x == 0 ? t1 - t0 : r1 - r0);
    }
  }
};
// The sink of the launch being issued on this host thread (set by the C-ABI
// layer's per-stage timer when the clock option is on, else null); the launch
// functions pass it to the kernels that take one.
extern thread_local unsigned long long* g_clock_sink;

enum { VSIG_C128 = 0, VSIG_C64 = 1, VSIG_F64 = 2, VSIG_F32 = 3 };

// NCO mixer of apply_frequency_shift (utils.py:120-127): x[gi] * exp(j theta),
// theta = w * (gi / sr) with w = (2 pi) f, formed in double exactly as numpy
// forms it (t = np.arange(n) / sample_rate; (2j*pi*f) * t), reduced modulo 2 pi
// in double (Cody-Waite), rotation in fp32.  Used by mix_c64 and fused into the
// FIR's segment loads (fir.hip).
struct MixArgs {
  double w, sr;
  long long i0;      // global sample index of x[0]
  double wsr;        // w / sr (the fused loads' phase slope)
  // exp(j wsr d_e) for the fused loads' element offsets d_e = 64 e (the
  // 1024-point one-wave plan, 16 elements per lane), formed in double on the
  // host and rounded once to fp32: a lane rotates by exp(j theta(g + t)) once
  // and then by these, so the double-precision phase runs once per segment
  // and lane instead of once per sample.
  float rot[32];     // (cos, sin) interleaved
};
__device__ __forceinline__ float2 mix_at(float2 v, long long gi, double w, double sr) {
  constexpr double kTwoPiHi = 6.28318530717958623200e+00;
  constexpr double kTwoPiLo = 2.44929359829470635445e-16;
  constexpr double kInvTwoPi = 1.59154943091895345608e-01;
  const double t = __ddiv_rn((double)gi, sr);          // np.arange(n) / sample_rate
  const double th = __dmul_rn(w, t);                   // imaginary part of (2j*pi*f) * t
  const double k = rint(th * kInvTwoPi);
  const double r = fma(-k, kTwoPiLo, fma(-k, kTwoPiHi, th));
  float s, c;
  sincosf((float)r, &s, &c);
  return make_float2(v.x * c - v.y * s, v.x * s + v.y * c);
}

// The fused loads' form: exp(j theta), theta = (w / sr) * gi, one double
// multiply instead of numpy's division then multiply (|difference| <= ~2 ulp
// of theta, e.g. 2e-7 rad at |theta| = 1e9 rad; the standalone mixer keeps
// numpy's order).
// exp(2 pi j rev) for a phase given in revolutions (double): reduced in double
// to a quarter turn q and |g| <= 1/8 turn, then fp32 Taylor polynomials to
// degree 9 / 10 on |2 pi g| <= pi/4 (truncation < 2e-9); no ocml sincosf, whose
// large-argument path keeps a private array in scratch.
__device__ __forceinline__ float2 cis_rev(double rev) {
  const double f = rev - rint(rev);                    // [-1/2, 1/2] turn
  const double q = rint(4.0 * f);                      // quarter turns, -2..2
  const float x = (float)(f - 0.25 * q) * 6.283185307179586f;   // |x| <= pi/4
  const float x2 = x * x;
  const float sn = x * fmaf(x2, fmaf(x2, fmaf(x2, fmaf(x2, 2.7557319e-6f, -1.9841270e-4f),
                                              8.3333333e-3f), -1.6666667e-1f), 1.0f);
  const float cs = fmaf(x2, fmaf(x2, fmaf(x2, fmaf(x2, fmaf(x2, -2.7557319e-7f, 2.4801587e-5f),
                                                    -1.3888889e-3f), 4.1666667e-2f), -0.5f), 1.0f);
  const int qi = ((int)q) & 3;                         // rotate by q quarter turns
  const float c = qi == 0 ? cs : qi == 1 ? -sn : qi == 2 ? -cs : sn;
  const float s = qi == 0 ? sn : qi == 1 ? cs : qi == 2 ? -sn : -cs;
  return make_float2(c, s);
}
__device__ __forceinline__ float2 mix_rot_fast(long long gi, double wsr) {
  constexpr double kInvTwoPi = 1.59154943091895345608e-01;
  return cis_rev((wsr * kInvTwoPi) * (double)gi);
}

// One block's |c| reduction partial (also the layout of the final result).
struct PeakPartial {
  double max2;       // max |c|^2 (kernels on |c|^2) or max |c| (peak_reduce / finalized)
  long long idx;     // index of the first maximum
  double sum_abs;    // sum |c|
  double sum_abs2;   // sum |c|^2
};

// Radices of the plan for N points (N = -1024: the one-wave FIR plan; -512 /
// -256: the decimating FIR's inverse plans).
hipError_t plan_info(int N, int* radices, int* npasses);
// Two-level twiddle table geometry: W_N^m = A[m >> shift] * B[m & (2^shift - 1)],
// A has `hi` entries, B has 2^shift.
hipError_t tw2_info(int N, int* shift, int* hi);

// Spectrum: nfft >= 4096 two frames per block (anchors, fft_pair), smaller
// plans several frames per block (LDS twiddles, split exchange; tw = the
// two-level table, see psd_plan_threads).
hipError_t launch_psd(int N, const float2* x, long long stride, const float* win, int nperseg,
                      long long hop, float scale, float* out, long long nframes, int shift,
                      const float2* tw, hipStream_t st);
// Threads per frame of the spectrum plan for N points (0: no plan): >= 256
// reads the per-pass twiddle table, below the two-level one.
int psd_plan_threads(int N);
hipError_t launch_spectrum_prep(int N, const float2* u, int len, float gain, float2* S,
                                const float2* tw, hipStream_t st);
// Decimating FIR in the frequency domain (M = 1024, D = 2 / 4; see fir.hip).
// mix != nullptr: the mixer above applied to every loaded sample (fused).
hipError_t launch_fir_dec(int decim, const float2* x, long long n, long long g0, const float2* Hs,
                          int lo2, long long hop, float2* y, const float2* tw, const float2* twd,
                          hipStream_t st, const MixArgs* mix = nullptr);
// D = 4 at M = 1024 in polyphase form (fir.hip fir_poly_kernel): G = the
// 4 x 256 component filters from Hs (launch_fir_poly_gtable), tw = Plan256's
// table, twd = Plan256d's.
hipError_t launch_fir_poly_gtable(const float2* Hs, float2* G, hipStream_t st);
hipError_t launch_fir_poly(const float2* x, long long n, long long g0, const float2* G, int lo2,
                           long long hop, float2* y, const float2* tw, const float2* twd,
                           hipStream_t st, const MixArgs* mix = nullptr);
// Overlap-save FIR, M in {1024, 4096, 8192, 16384} (mix: M = 1024 only).
hipError_t launch_fir_os(int M, const float2* x, long long n, long long g0, const float2* Hs,
                         int ntaps, long long hop, int decim, float2* y, const float2* tw,
                         hipStream_t st, const MixArgs* mix = nullptr);
// Correlator, M in {4096, 8192, 16384} (16384: half-frame kernel, tw = the
// 8192-point table, wt = W_M^t for t < 512).
hipError_t launch_xcorr_os(int M, const float2* s, long long n, const float2* Ps, long long off,
                           long long nout, long long hop, float2* c, int store_mode,
                           PeakPartial* partials, const float2* tw, const float2* wt,
                           hipStream_t st, unsigned* lkeys = nullptr);
// Rows per thread column if the correlator for M can write lane keys
// (lkeys[b TF + m(t)]: thread t's max |c|^2 key, the refine's column
// candidates), else 0.
int xcorr_lane_keys(int M);
// Outputs of wave w of block b of the correlator for M (the refine pass's
// items): ob + wstep w + l + 64 (q % rsub) + stride (q / rsub), l < 64, q < Q.
hipError_t xcorr_geom(int M, int* waves, int* Q, int* stride, int* plan, int* wstep, int* rsub);
#ifdef VSIG_TUNING
// Tuning micro-benchmarks: iters FFTs per frame, frames blocks (key: plan key).
hipError_t launch_fft_bench(int key, float2* io, int frames, int iters, const float2* tw, int twl,
                            hipStream_t st);
hipError_t launch_copy_probe(const float2* x, long long n, float2* y, int variant, int grid,
                             hipStream_t st);
#endif
hipError_t launch_peak_reduce(int dtype, const void* a, long long n, PeakPartial* partials,
                              int nparts, hipStream_t st);
constexpr int kFinalizeTmp = 1024;   // first-level partials of a two-level finalize
// zeroed PeakPartial-sized slots after the kFinalizeTmp records: the
// finalize's counter (first 8 B) and refine_fused's counters (128 B)
constexpr int kCounterRecs = 4;
hipError_t launch_partial_finalize(const PeakPartial* parts, long long nparts, int sqrt_max,
                                   PeakPartial* out, PeakPartial* tmp, hipStream_t st);

// refine.hip: exact re-rank of the |c| peak (see the file's header).
struct RefineArgs {
  const void* a; long long na;      // np.correlate(a, v) operands (device),
  const void* v; long long nv;      //   complex128 if c128 else complex64
  int c128;
  long long nout, F;                // final outputs; o <-> full index F + o
  int rev;                          // kernel raw index -> final nout - 1 - raw
  int from_array;                   // candidates from a stored c64 array c64[nout]
  const float2* c64;
  const PeakPartial* parts;         // or from the fused correlator's wave partials
  long long nparts, hop;
  int waves, Q, stride;             // wave w of block b: ob + wstep w + l + 64 (q % rsub)
  int wstep, rsub;                  //   + stride (q / rsub), l < 64, q < Q (xcorr_geom)
  double eps;                       // fp32 candidate band (relative)
  int blas_threads;                 // OpenBLAS threads of the numpy matched (sums > 10000)
  int cols;                         // > 0: thread-column items from lane keys (Q = 1;
  const unsigned* lkeys;            //   cols rows each), lkeys: 64 per wave partial
  int finalize;                     // finalize the partials here (+ select, one launch):
  PeakPartial* tmp;                 //   kFinalizeTmp first-level records,
  unsigned long long* done;         //   kCounterRecs records' worth of counters,
                                    //   zero between launches
  long long cap;                    // opt-in limit on candidate outputs (0: none)
  void* scratch;                    // refine_scratch_bytes(*this)
  PeakPartial* rec;                 // finalized record (max |c|), updated in place
  void* out128;                     // optional complex128 c to patch (final space)
  unsigned long long wd_ticks;      // fused launch's watchdog, 100 MHz ticks (0: 2 s)
};
size_t refine_scratch_bytes(const RefineArgs& r);
hipError_t launch_refine(const RefineArgs& r, hipStream_t st);
// numpy's |c| of every output o in [lo, hi] into vals[o - lo] (operands and
// geometry of r; scratch: refine_values_scratch_bytes()); r.rec (optional)
// receives numpy's argmax over the range.
size_t refine_values_scratch_bytes();
hipError_t launch_refine_values(const RefineArgs& r, long long lo, long long hi, double* vals,
                                hipStream_t st);
// reduce.hip: numpy's np.mean(np.abs(a)) and np.std(np.abs(a)) (float64
// pairwise sums over 8192-element buffers, two passes) of an array of dtype
// VSIG_C128 or VSIG_F64 into out[0], out[1] (device); scratch:
// np_stats_scratch_bytes(n).
size_t np_stats_scratch_bytes(long long n);
hipError_t launch_np_stats(int dtype, const void* a, long long n, double* out, void* scratch,
                           hipStream_t st);
hipError_t launch_convert_c(int to128, const void* x, long long n, void* y, hipStream_t st);

// bigfft.hip: four-step FFT of M = N1 N2 > 16384 points, Bluestein for any
// length (see the file's header).
struct BigIn {                 // operand n of frame f
  const void* src;
  int kind;                    // 0 complex64, 1 complex128, 2 zeros
  long long fstride, estride, nvalid;
  const float2* chirp;         // optional * chirp[n]
  const float* win;            // optional * win[n]
  int conj;                    // conj(x) first (inverse DFT)
  float scale;
};
struct BigOut {                // natural-order result n of frame f
  void* dst;
  int kind;                    // 0 complex64, 1 complex128, 2 float64 real part, 3 complex64 real part,
                               // 4 float32 |X|^2 * scale (PSD), at (n + nout/2) % nout if shift
  long long fstride, nout;
  const float2* chirp;         // optional * chirp[n], then conj
  int conj;
  float scale;
  int shift = 0;
};
void bigfft_split(long long M, int* N1, int* N2);
hipError_t launch_bf_chirp(long long N, long long M, float2* c, float2* b, hipStream_t st);
hipError_t launch_bf_col(int N1, int N2, long long batch, const BigIn& in, float2* tmp,
                         const float2* tw1, const float2* t2, int S, int hiA, hipStream_t st);
hipError_t launch_bf_icol(int N1, int N2, long long batch, float2* tmp, const BigOut& out,
                          const float2* tw1, const float2* t2, int S, int hiA, hipStream_t st);
hipError_t launch_bf_row(int mode, int N1, int N2, long long batch, float2* tmp, const float2* Bk,
                         const float2* tw2, float scale, float* psd, int shift, hipStream_t st);
hipError_t launch_bf_small(int mode, int M, long long batch, const BigIn& in, const BigOut& out,
                           const float2* Bk, const float2* tw, hipStream_t st);
hipError_t launch_resample_spectrum(const float2* X, long long Nx, long long num, float2* Y,
                                    hipStream_t st);
hipError_t launch_channel_mask(const float2* X, long long n, double sr, double center, double lo,
                               double hi, float2* F, hipStream_t st);
// kept bins [ka, kb] (kb < ka: none) of the channel filter by direct double sums;
// part: 256 * (kb - ka + 1) scratch, X: kb - ka + 1
hipError_t launch_channel_direct(int c128, const void* x, long long n, long long ka, long long kb,
                                 double2* part, double2* X, double* y, hipStream_t st);

// pfb.hip: C in {64, 128, 256}, PT in {4, 8, 16}; y frame-major (M x C)
hipError_t launch_pfb(int C, int PT, const float2* x, long long n, const float* h, long long M,
                      float2* y, const float2* tw, hipStream_t st);

// stream_ops.hip
hipError_t launch_mix_c64(const float2* x, long long n, double w, double sr, long long i0, float2* y,
                          hipStream_t st);
hipError_t launch_scale_c64(const float2* x, long long n, float s, float2* y, hipStream_t st);
hipError_t launch_fir_part_accum(const float2* z, long long nz, long long off, int D, long long ny,
                                 int first, float2* y, hipStream_t st);
hipError_t launch_wv_quantize(const float2* x, long long n, float norm, short* out, hipStream_t st);
hipError_t launch_planar_to_c64(int mi_type, const void* re, const void* im, long long n, float2* y,
                                hipStream_t st);
hipError_t launch_c64_to_planar(const float2* x, long long n, float* re, float* im, hipStream_t st);

// analysis.hip
hipError_t launch_radix_hist(int dtype, const void* a, long long n, const unsigned long long* prefix,
                             const unsigned long long* mask, int nq, int shift,
                             unsigned long long* hist, hipStream_t st);
struct ThreshPartialH { long long count, first, last; double max; };   // = ThreshPartial
hipError_t launch_thresh_reduce(int dtype, const void* a, long long n, double thr, void* parts,
                                int nparts, hipStream_t st);
long long energy_scan_tiles(long long n);
hipError_t launch_energy_prefix(int dtype, const void* x, long long n, double* sums, double* P,
                                hipStream_t st);
hipError_t launch_boxcar_same(const double* P, long long n, long long w, double* sm, hipStream_t st);
hipError_t launch_db_transform(int dtype, const void* a, long long n, double floor_, void* out,
                               hipStream_t st);
hipError_t launch_abs_c64(int dtype, const void* a, long long n, float2* out, hipStream_t st);
hipError_t launch_abs_c128(int dtype, const void* a, long long n, double2* out, hipStream_t st);

}  // namespace vsig
