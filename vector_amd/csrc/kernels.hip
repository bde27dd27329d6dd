// HIP kernels of the vector-signal DSP hot path (gfx950 / CDNA4).
//
//   psd_kernel       windowed block FFT -> |X|^2 * scale   (spectrum / create_spectrogram)
//   fir_os_kernel    overlap-save FIR, decimation folded into the store (filter)
//   xcorr_os_kernel  overlap-save cross-correlation + fused |c|^2 argmax / sums (correlate)
//   peak_reduce      double-precision |c| argmax / mean / std over an array (find_correlation_peak)
//   partial_finalize deterministic reduction of per-block partials
//   spectrum_prep    FFT of a zero-padded short vector (filter taps / correlation template)
//
// All FFT work goes through fft_engine.hpp.  No MFMA: there is no dense
// contraction on this path; every kernel is HBM- or VALU-bound.
#include "fft_engine.hpp"
#include "vsig_kernels.h"

namespace vsig {

// Occupancy request (min waves per SIMD) of a kernel variant: the split
// exchange (variant 4) exists to fit two 16k / four 8k frames per CU, which
// needs <= 128 VGPRs, so ask the register allocator for 4 waves/SIMD there.
template <class P, int PERSIST>
constexpr int min_waves() {
#ifdef VSIG_EXP_SPLIT_W4
  return PERSIST == 4 ? 4 : 1;
#else
  return (PERSIST == 4 && P::E <= 16) ? 4 : 1;
#endif
}

// Overlap-save kernels run one frame per block: TF threads (one wave for the
// 1024 / 2048-point plans, whose barriers then cost nothing).
template <class P>
constexpr int os_threads() { return P::TF; }

// ---------------------------------------------------------------------------
// Persistent-kernel skeleton shared by the streaming kernels: a block walks
// units u = blockIdx.x, + gridDim.x, ...; the next unit's samples are loaded
// into registers at the top of each iteration, so their HBM latency hides
// behind the current unit's FFTs (the only global loads in flight are stream
// loads: twiddles, window and filter spectra live in registers).
// ---------------------------------------------------------------------------

// spectrum: frames = (n - nperseg) / hop + 1; FPB frames per unit
// (scipy.signal.spectrogram, scipy/signal/_spectral_py.py:2158-2205, as called
// at utils.py:281-291).
template <class P>
__device__ __forceinline__ void psd_load(float2* v, const float2* __restrict__ x, long long stride,
                                         int nperseg, long long hop, long long frame,
                                         long long nframes, int t) {
  const bool active = frame < nframes;
  const float2* xf = x + (active ? frame * hop * stride : 0);
#pragma unroll
  for (int e = 0; e < P::E; ++e) {
    const int i = in_index<P>(t, e);
    v[e] = (active && i < nperseg) ? xf[(long long)i * stride] : make_float2(0.f, 0.f);
  }
}

template <class P, int PERSIST>
__global__ __launch_bounds__(block_threads<P>(), (min_waves<P, PERSIST>())) void psd_kernel(
    const float2* __restrict__ x, long long stride, const float* __restrict__ win, int nperseg,
    long long hop, float scale, float* __restrict__ out, long long nframes, int shift,
    const float2* __restrict__ tw) {
  constexpr int BT = block_threads<P>();
  constexpr int FPB = BT / P::TF;
  __shared__ float2 lds[FPB * (PERSIST == 4 ? (P::LDS + 1) / 2 : P::LDS) +
                       ((PERSIST == 3 || PERSIST == 4) ? tw2_size<P>() : 0)];
  const int fl = threadIdx.x / P::TF;
  const int t = threadIdx.x % P::TF;
  const long long units = (nframes + FPB - 1) / FPB;
  long long u = blockIdx.x;
  if (u >= units) return;
  if constexpr (PERSIST == 4) {      // one unit per block, LDS twiddles, split exchange
    constexpr int FL = (P::LDS + 1) / 2;
    float2* t2 = lds + FPB * FL;
    load_tw2<P>(t2, tw, threadIdx.x, BT);
    float2 v[P::E];
    psd_load<P>(v, x, stride, nperseg, hop, u * FPB + fl, nframes, t);
#pragma unroll
    for (int e = 0; e < P::E; ++e) {
      const int i = in_index<P>(t, e);
      const float w = i < nperseg ? win[i] : 0.f;
      v[e] = make_float2(v[e].x * w, v[e].y * w);
    }
    fft_frame_split<P>(v, reinterpret_cast<float*>(lds + fl * FL), t2, t);
    const long long frame = u * FPB + fl;
    if (frame < nframes) {
      float* of = out + frame * P::N;
#pragma unroll
      for (int e = 0; e < P::E; ++e) {
        const int i = out_index<P>(t, e);
        const int o = shift ? ((i + P::N / 2) & (P::N - 1)) : i;
        of[o] = (v[e].x * v[e].x + v[e].y * v[e].y) * scale;
      }
    }
    return;
  }
  if constexpr (PERSIST == 3) {      // one unit per block, two-level LDS twiddles
    float2* t2 = lds + FPB * P::LDS;
    load_tw2<P>(t2, tw, threadIdx.x, BT);
    float2 v[P::E];
    psd_load<P>(v, x, stride, nperseg, hop, u * FPB + fl, nframes, t);
#pragma unroll
    for (int e = 0; e < P::E; ++e) {
      const int i = in_index<P>(t, e);
      const float w = i < nperseg ? win[i] : 0.f;
      v[e] = make_float2(v[e].x * w, v[e].y * w);
    }
    fft_frame_t2<P>(v, lds + fl * P::LDS, t2, t);
    const long long frame = u * FPB + fl;
    if (frame < nframes) {
      float* of = out + frame * P::N;
#pragma unroll
      for (int e = 0; e < P::E; ++e) {
        const int i = out_index<P>(t, e);
        const int o = shift ? ((i + P::N / 2) & (P::N - 1)) : i;
        of[o] = (v[e].x * v[e].x + v[e].y * v[e].y) * scale;
      }
    }
    return;
  }

  if constexpr (!PERSIST) {          // one unit per block, table twiddles
    float2 v[P::E];
    psd_load<P>(v, x, stride, nperseg, hop, u * FPB + fl, nframes, t);
#pragma unroll
    for (int e = 0; e < P::E; ++e) {
      const int i = in_index<P>(t, e);
      const float w = i < nperseg ? win[i] : 0.f;
      v[e] = make_float2(v[e].x * w, v[e].y * w);
    }
    fft_frame<P>(v, lds + fl * P::LDS, tw, t);
    const long long frame = u * FPB + fl;
    if (frame < nframes) {
      float* of = out + frame * P::N;
#pragma unroll
      for (int e = 0; e < P::E; ++e) {
        const int i = out_index<P>(t, e);
        const int o = shift ? ((i + P::N / 2) & (P::N - 1)) : i;
        of[o] = (v[e].x * v[e].x + v[e].y * v[e].y) * scale;
      }
    }
    return;
  } else if constexpr (PERSIST == 2) {   // persistent, table twiddles, late prefetch
    float2 v[P::E];
    psd_load<P>(v, x, stride, nperseg, hop, u * FPB + fl, nframes, t);
    for (; u < units; u += gridDim.x) {
#pragma unroll
      for (int e = 0; e < P::E; ++e) {
        const int i = in_index<P>(t, e);
        const float w = i < nperseg ? win[i] : 0.f;
        v[e] = make_float2(v[e].x * w, v[e].y * w);
      }
      float2 nv[P::E];
      const long long nu = u + gridDim.x;
      fft_frame_hook<P>(v, lds + fl * P::LDS, tw, t, [&] {
        if (nu < units) psd_load<P>(nv, x, stride, nperseg, hop, nu * FPB + fl, nframes, t);
      });
      const long long frame = u * FPB + fl;
      if (frame < nframes) {
        float* of = out + frame * P::N;
#pragma unroll
        for (int e = 0; e < P::E; ++e) {
          const int i = out_index<P>(t, e);
          const int o = shift ? ((i + P::N / 2) & (P::N - 1)) : i;
          of[o] = (v[e].x * v[e].x + v[e].y * v[e].y) * scale;
        }
      }
#pragma unroll
      for (int e = 0; e < P::E; ++e) v[e] = nv[e];
    }
    return;
  }
  float2 wa[nanch_total<P>()];
  load_anchors<P>(wa, tw, t);
  float wr[P::E];
#pragma unroll
  for (int e = 0; e < P::E; ++e) {
    const int i = in_index<P>(t, e);
    wr[e] = i < nperseg ? win[i] : 0.f;
  }
  float2 v[P::E];
  psd_load<P>(v, x, stride, nperseg, hop, u * FPB + fl, nframes, t);
  for (; u < units; u += gridDim.x) {
    float2 nv[P::E];
    const long long nu = u + gridDim.x;
    if (nu < units) psd_load<P>(nv, x, stride, nperseg, hop, nu * FPB + fl, nframes, t);
#pragma unroll
    for (int e = 0; e < P::E; ++e) v[e] = make_float2(v[e].x * wr[e], v[e].y * wr[e]);
    fft_frame_anch<P>(v, lds + fl * P::LDS, wa, t);
    const long long frame = u * FPB + fl;
    if (frame < nframes) {
      float* of = out + frame * P::N;
#pragma unroll
      for (int e = 0; e < P::E; ++e) {
        const int i = out_index<P>(t, e);
        const int o = shift ? ((i + P::N / 2) & (P::N - 1)) : i;
        of[o] = (v[e].x * v[e].x + v[e].y * v[e].y) * scale;
      }
    }
#pragma unroll
    for (int e = 0; e < P::E; ++e) v[e] = nv[e];
  }
}

// ---------------------------------------------------------------------------
// spectrum_prep: S = FFT_M(zero-padded u) * gain, one frame of M points.
// conj_in conjugates u first.  Used for the FIR response (H / M) and the
// correlation template spectrum (P / M).
// ---------------------------------------------------------------------------
template <class P>
__global__ __launch_bounds__(block_threads<P>()) void spectrum_prep(
    const float2* __restrict__ u, int len, float gain, float2* __restrict__ S,
    const float2* __restrict__ tw) {
  constexpr int BT = block_threads<P>();
  __shared__ float2 lds[(BT / P::TF) * P::LDS];
  const int fl = threadIdx.x / P::TF;
  const int t = threadIdx.x % P::TF;
  float2 v[P::E];
#pragma unroll
  for (int e = 0; e < P::E; ++e) {
    const int i = in_index<P>(t, e);
    v[e] = (fl == 0 && i < len) ? u[i] : make_float2(0.f, 0.f);
  }
  fft_frame<P>(v, lds + fl * P::LDS, tw, t);
  if (fl != 0) return;
#pragma unroll
  for (int e = 0; e < P::E; ++e) {
    const int i = out_index<P>(t, e);
    S[i] = make_float2(v[e].x * gain, v[e].y * gain);
  }
}

// LDS (in float2) of a one-frame block: data (halved by the split exchange)
// plus the two-level twiddle table for variants 3 and 4.
template <class P, int PERSIST>
constexpr int os_lds() {
  return (PERSIST == 4 ? (P::LDS + 1) / 2 : P::LDS) +
         ((PERSIST == 3 || PERSIST == 4) ? tw2_size<P>() : 0);
}

// Pass-0 operands of an overlap-save segment x[s0 .. s0 + N) with zero fill
// outside [0, n).  The block-uniform base keeps the address in SGPRs; interior
// segments (the common case) skip the per-element bounds test.
template <class P>
__device__ __forceinline__ void load_segment(float2* v, const float2* __restrict__ x,
                                             long long s0, long long n, int t) {
  const float2* base = x + s0;
  if (s0 >= 0 && s0 + P::N <= n) {
#pragma unroll
    for (int e = 0; e < P::E; ++e) v[e] = base[(unsigned)in_index<P>(t, e)];
  } else {
#pragma unroll
    for (int e = 0; e < P::E; ++e) {
      const int i = in_index<P>(t, e);
      const long long xi = s0 + i;
      v[e] = (xi >= 0 && xi < n) ? base[i] : make_float2(0.f, 0.f);
    }
  }
}

// Store the valid outputs of FIR block b (conj undoes the inverse-by-conj
// trick): block-local 32-bit offsets from a per-block base; hop is a multiple
// of decim, so the decimation phase is the local index's.
template <class P>
__device__ __forceinline__ void fir_store(const float2* v, float2* __restrict__ y, long long b,
                                          long long hop, int lo, long long nloc, int decim, int t) {
  const long long gb = b * hop;
  const long long rem = nloc - gb;
  const int lim = rem < hop ? (int)rem : (int)hop;
  if (decim == 1) {
    float2* yb = y + gb;
#pragma unroll
    for (int e = 0; e < P::E; ++e) {
      const int i = out_index<P>(t, e) - lo;
      if (i >= 0 && i < lim) yb[(unsigned)i] = cconj(v[e]);
    }
  } else {
    // i / decim by a multiply-high with m = floor(2^32 / decim) + 1: exact for
    // i, decim < 2^16 (hop <= 16384), no per-element integer division
    float2* yb = y + gb / decim;
    const unsigned mg = 0xffffffffu / (unsigned)decim + 1u;
#pragma unroll
    for (int e = 0; e < P::E; ++e) {
      const int i = out_index<P>(t, e) - lo;
      const unsigned q = __umulhi((unsigned)i, mg);
      if (i >= 0 && i < lim && (unsigned)i == q * (unsigned)decim) yb[q] = cconj(v[e]);
    }
  }
}

// ---------------------------------------------------------------------------
// FIR, overlap-save.  Block b produces outputs g in [b*hop, b*hop + hop) of
//   y[g] = sum_{m < ntaps} h[m] x[g0 + g - m]   (x = 0 outside [0, n))
// i.e. np.convolve(x, h, 'full')[g0:n]; only g % decim == 0 is stored, at
// g/decim.  The first g0 samples are history (a time-chunk's left halo).
// The segment x[b*hop - (ntaps-1) .. + M) is FFT'd, multiplied by Hs = FFT(h)/M
// and inverse-transformed (conj trick), all in LDS / registers.
// ---------------------------------------------------------------------------
template <class P, int PERSIST>
__global__ __launch_bounds__(os_threads<P>(), (min_waves<P, PERSIST>())) void fir_os_kernel(
    const float2* __restrict__ x, long long n, long long g0, const float2* __restrict__ Hs,
    int ntaps, long long hop, int decim, float2* __restrict__ y, long long nblocks,
    const float2* __restrict__ tw) {
  static_assert(P::R[0] == P::RL, "overlap-save needs a palindromic plan");
  constexpr int BT = os_threads<P>();
  static_assert(BT == P::TF, "one frame per block");
  __shared__ float2 lds[os_lds<P, PERSIST>()];
  const int t = threadIdx.x;
  long long b = PERSIST == 0 || PERSIST >= 3 ? xcd_remap(blockIdx.x, gridDim.x) : blockIdx.x;
  if (b >= nblocks) return;  // uniform per block

  const int lo = ntaps - 1;
  const long long nloc = n - g0;
  if constexpr (PERSIST == 4) {      // one unit per block, LDS twiddles, split exchange
    float2* t2 = lds + (P::LDS + 1) / 2;
    float* ldf = reinterpret_cast<float*>(lds);
    load_tw2<P>(t2, tw, t, BT);
    float2 v[P::E];
    load_segment<P>(v, x, g0 + b * hop - lo, n, t);
    fft_frame_split<P>(v, ldf, t2, t);
#pragma unroll
    for (int e = 0; e < P::E; ++e) v[e] = cconj(cmul(v[e], Hs[out_index<P>(t, e)]));
    fft_frame_split<P>(v, ldf, t2, t);
    fir_store<P>(v, y, b, hop, lo, nloc, decim, t);
    return;
  }
  if constexpr (PERSIST == 3) {      // one unit per block, two-level LDS twiddles
    float2* t2 = lds + P::LDS;
    load_tw2<P>(t2, tw, t, BT);
    float2 v[P::E];
    load_segment<P>(v, x, g0 + b * hop - lo, n, t);
    fft_frame_t2<P>(v, lds, t2, t);
#pragma unroll
    for (int e = 0; e < P::E; ++e) v[e] = cconj(cmul(v[e], Hs[out_index<P>(t, e)]));
    fft_frame_t2<P>(v, lds, t2, t);
    fir_store<P>(v, y, b, hop, lo, nloc, decim, t);
    return;
  }
  if constexpr (!PERSIST) {          // one unit per block, table twiddles
    float2 v[P::E];
    load_segment<P>(v, x, g0 + b * hop - lo, n, t);
    fft_frame<P>(v, lds, tw, t);
#pragma unroll
    for (int e = 0; e < P::E; ++e) v[e] = cconj(cmul(v[e], Hs[out_index<P>(t, e)]));
    fft_frame<P>(v, lds, tw, t);
    fir_store<P>(v, y, b, hop, lo, nloc, decim, t);
    return;
  } else if constexpr (PERSIST == 2) {   // persistent, table twiddles, late prefetch
    float2 v[P::E];
    load_segment<P>(v, x, g0 + b * hop - lo, n, t);
    for (; b < nblocks; b += gridDim.x) {
      fft_frame<P>(v, lds, tw, t);
#pragma unroll
      for (int e = 0; e < P::E; ++e) v[e] = cconj(cmul(v[e], Hs[out_index<P>(t, e)]));
      float2 nv[P::E];
      const long long nb = b + gridDim.x;
      fft_frame_hook<P>(v, lds, tw, t, [&] {
        if (nb < nblocks) load_segment<P>(nv, x, g0 + nb * hop - lo, n, t);
      });
      fir_store<P>(v, y, b, hop, lo, nloc, decim, t);
#pragma unroll
      for (int e = 0; e < P::E; ++e) v[e] = nv[e];
    }
    return;
  }
  float2 wa[nanch_total<P>()];
  load_anchors<P>(wa, tw, t);
  float2 v[P::E];
  load_segment<P>(v, x, g0 + b * hop - lo, n, t);
  for (; b < nblocks; b += gridDim.x) {
    fft_frame_anch<P>(v, lds, wa, t);
#pragma unroll
    for (int e = 0; e < P::E; ++e) v[e] = cconj(cmul(v[e], Hs[out_index<P>(t, e)]));
    // Prefetch after the (L2-resident) filter-spectrum loads: vmcnt retires in
    // issue order, so the next segment then lands behind the inverse FFT.
    float2 nv[P::E];
    const long long nb = b + gridDim.x;
    if (nb < nblocks) load_segment<P>(nv, x, g0 + nb * hop - lo, n, t);
    fft_frame_anch<P>(v, lds, wa, t);
    fir_store<P>(v, y, b, hop, lo, nloc, decim, t);
#pragma unroll
    for (int e = 0; e < P::E; ++e) v[e] = nv[e];
  }
}

// ---------------------------------------------------------------------------
// Block partial of a |c| reduction: max |c|^2 (lowest index on ties),
// sum |c|, sum |c|^2.
// ---------------------------------------------------------------------------
__device__ __forceinline__ void better(float& m, long long& i, float m2, long long i2) {
  if (m2 > m || (m2 == m && i2 < i)) { m = m2; i = i2; }
}
__device__ __forceinline__ void betterd(double& m, long long& i, double m2, long long i2) {
  if (m2 > m || (m2 == m && i2 < i)) { m = m2; i = i2; }
}

template <int BT>
__device__ __forceinline__ void block_partial(double m, long long mi, double s1, double s2,
                                              PeakPartial* out) {
  // wave reduce (64 lanes)
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    const double om = __shfl_xor(m, off);
    const long long oi = __shfl_xor(mi, off);
    betterd(m, mi, om, oi);
    s1 += __shfl_xor(s1, off);
    s2 += __shfl_xor(s2, off);
  }
  constexpr int NW = BT / 64;
  __shared__ double sm[NW], ss1[NW], ss2[NW];
  __shared__ long long si[NW];
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  if (l == 0) { sm[w] = m; si[w] = mi; ss1[w] = s1; ss2[w] = s2; }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int q = 1; q < NW; ++q) { betterd(m, mi, sm[q], si[q]); s1 += ss1[q]; s2 += ss2[q]; }
    out->max2 = m; out->idx = mi; out->sum_abs = s1; out->sum_abs2 = s2;
  }
}

// Partials of the correlators: float |c|^2 / int block-local index / float
// sums, wave-reduced with DPP (VALU-rate lane moves instead of a chain of
// ds_bpermute round trips and a block barrier — a block's tail is exposed at
// one block per CU), one partial per wave.  rev: ties go to the larger index.
template <int CTRL, int RM>
__device__ __forceinline__ float dpp_f(float x) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), CTRL, RM, 0xf, false));
}
template <int CTRL, int RM>
__device__ __forceinline__ int dpp_i(int x) {
  return __builtin_amdgcn_update_dpp(0, x, CTRL, RM, 0xf, false);
}
template <int CTRL, int RM>
__device__ __forceinline__ void peak_dpp_step(float& m, int& mi, float& s1, float& s2, bool rev) {
  const float om = dpp_f<CTRL, RM>(m);
  const int oi = dpp_i<CTRL, RM>(mi);
  const bool take = (om > m) | ((om == m) & (rev ? oi > mi : oi < mi));
  m = take ? om : m;
  mi = take ? oi : mi;
  s1 += dpp_f<CTRL, RM>(s1);
  s2 += dpp_f<CTRL, RM>(s2);
}

// One partial per wave (no block barrier at the block's tail): lane 63 holds
// the wave's result after the DPP steps and writes it.
__device__ __forceinline__ void wave_partial_f(float m, int mi, float s1, float s2, bool rev,
                                               long long ob, long long nout, PeakPartial* out) {
  // rocPRIM-style wave64 reduction: quad xor 1, 2; row_ror 4, 8; row_bcast 15, 31
  // -> lane 63 holds the wave's result (rows not feeding it hold garbage).
  peak_dpp_step<0xb1, 0xf>(m, mi, s1, s2, rev);
  peak_dpp_step<0x4e, 0xf>(m, mi, s1, s2, rev);
  peak_dpp_step<0x124, 0xf>(m, mi, s1, s2, rev);
  peak_dpp_step<0x128, 0xf>(m, mi, s1, s2, rev);
  peak_dpp_step<0x142, 0xa>(m, mi, s1, s2, rev);
  peak_dpp_step<0x143, 0xc>(m, mi, s1, s2, rev);
  if ((threadIdx.x & 63) == 63) {
    long long gi = ob + mi;
    if (rev) gi = nout - 1 - gi;
    PeakPartial r;
    r.max2 = (double)m;
    r.idx = gi;
    r.sum_abs = (double)s1;
    r.sum_abs2 = (double)s2;
    *out = r;
  }
}

// ---------------------------------------------------------------------------
// Cross-correlation, overlap-save:  c[o] = sum_{k<L} s[o - off + k] * conj(p[k]),
// o in [0, nout).  off = 0 -> np.correlate 'valid'; off = L-1 -> 'full'.
// Block b: outputs [b*hop, b*hop + hop), hop <= M - L + 1.
// Epilogue: optional store of c (store_mode 1) or of conj(c) at nout-1-o
// (store_mode 2, the swapped argument order of np.correlate), and the block's
// |c| partial; store_mode bit 4 reports the argmax in the reversed index
// space (first maximum of the reversed output).
// ---------------------------------------------------------------------------
// Epilogue of one correlation block: |c|^2, block argmax / sums, optional store.
template <class P>
__device__ __forceinline__ void xcorr_epilogue(const float2* v, long long b, long long hop,
                                               long long nout, float2* __restrict__ c,
                                               int store_mode, PeakPartial* partials, int t) {
  constexpr int BT = os_threads<P>();
  const long long ob = b * hop;                         // block's first output
  const long long rem = nout - ob;
  const int lim = rem < hop ? (int)rem : (int)hop;
  const bool rev = store_mode & 4;
  const int smode = store_mode & 3;
  // optional store: one uniform branch outside the element loops
  if (smode == 1) {
#pragma unroll
    for (int e = 0; e < P::E; ++e) {
      const int i = out_index<P>(t, e);
      if (i < lim) (c + ob)[(unsigned)i] = cconj(v[e]);
    }
  } else if (smode == 2) {
#pragma unroll
    for (int e = 0; e < P::E; ++e) {
      const int i = out_index<P>(t, e);
      if (i < lim) (c + (nout - 1 - ob))[-i] = v[e];
    }
  }
  if (!partials) return;
  // branch-free peak / sums.  A thread's output indices rise with e, so a
  // strict '>' keeps the first maximum; in the reversed index space (rev)
  // '>=' keeps the last raw index, i.e. the first reversed one.
  float m = -1.f, s1 = 0.f, s2 = 0.f;
  int mi = 0;
#pragma unroll
  for (int e = 0; e < P::E; ++e) {
    const int i = out_index<P>(t, e);
    const bool ok = i < lim;
    const float a2r = v[e].x * v[e].x + v[e].y * v[e].y;
    const float a2 = ok ? a2r : -1.f;
    const bool take = (a2 > m) | (rev & (a2 == m) & ok);
    m = take ? a2 : m;
    mi = take ? i : mi;
    s1 += ok ? __builtin_amdgcn_sqrtf(a2r) : 0.f;   // v_sqrt_f32 (1 ulp), not the IEEE expansion
    s2 += ok ? a2r : 0.f;
  }
  wave_partial_f(m, mi, s1, s2, rev, ob, nout, partials + b * (BT / 64) + (t >> 6));
}

template <class P, int PERSIST>
__global__ __launch_bounds__(os_threads<P>(), (min_waves<P, PERSIST>())) void xcorr_os_kernel(
    const float2* __restrict__ s, long long n, const float2* __restrict__ Ps, long long off,
    long long nout, long long hop, float2* __restrict__ c, int store_mode,
    PeakPartial* __restrict__ partials, long long nblocks, const float2* __restrict__ tw) {
  static_assert(P::R[0] == P::RL, "overlap-save needs a palindromic plan");
  constexpr int BT = os_threads<P>();
  static_assert(BT == P::TF, "one frame per block");
  __shared__ float2 lds[os_lds<P, PERSIST>()];
  const int t = threadIdx.x;
  long long b = PERSIST == 0 || PERSIST >= 3 ? xcd_remap(blockIdx.x, gridDim.x) : blockIdx.x;
  if (b >= nblocks) return;

  if constexpr (PERSIST == 4) {      // one unit per block, LDS twiddles, split exchange
    float2* t2 = lds + (P::LDS + 1) / 2;
    float* ldf = reinterpret_cast<float*>(lds);
    load_tw2<P>(t2, tw, t, BT);
    float2 v[P::E];
    load_segment<P>(v, s, b * hop - off, n, t);
    fft_frame_split<P>(v, ldf, t2, t);
#pragma unroll
    for (int e = 0; e < P::E; ++e) v[e] = cmul(cconj(v[e]), Ps[out_index<P>(t, e)]);
    fft_frame_split<P>(v, ldf, t2, t);
    xcorr_epilogue<P>(v, b, hop, nout, c, store_mode, partials, t);
    return;
  }
  if constexpr (PERSIST == 3) {      // one unit per block, two-level LDS twiddles
    float2* t2 = lds + P::LDS;
    load_tw2<P>(t2, tw, t, BT);
    float2 v[P::E];
#ifdef VSIG_EXP_NO_LOAD      // timing experiments only (results are wrong)
#pragma unroll
    for (int e = 0; e < P::E; ++e) v[e] = make_float2((float)(t + e), (float)(b & 7));
#else
    load_segment<P>(v, s, b * hop - off, n, t);
#endif
    fft_frame_t2<P>(v, lds, t2, t);
#ifdef VSIG_EXP_NO_PS
#pragma unroll
    for (int e = 0; e < P::E; ++e) v[e] = cmul(cconj(v[e]), make_float2(0.5f, 0.25f));
#else
#pragma unroll
    for (int e = 0; e < P::E; ++e) v[e] = cmul(cconj(v[e]), Ps[out_index<P>(t, e)]);
#endif
    fft_frame_t2<P>(v, lds, t2, t);
#ifdef VSIG_EXP_NO_EPI
    float acc = 0.f;
#pragma unroll
    for (int e = 0; e < P::E; ++e) acc += v[e].x + v[e].y;
    if (acc == 12345.f) partials[b].sum_abs = acc;
#else
    xcorr_epilogue<P>(v, b, hop, nout, c, store_mode, partials, t);
#endif
    return;
  }
  if constexpr (!PERSIST) {          // one unit per block, table twiddles
    float2 v[P::E];
    load_segment<P>(v, s, b * hop - off, n, t);
    fft_frame<P>(v, lds, tw, t);
#pragma unroll
    for (int e = 0; e < P::E; ++e) v[e] = cmul(cconj(v[e]), Ps[out_index<P>(t, e)]);
    fft_frame<P>(v, lds, tw, t);
    xcorr_epilogue<P>(v, b, hop, nout, c, store_mode, partials, t);
    return;
  } else if constexpr (PERSIST == 2) {   // persistent, table twiddles, late prefetch
    float2 v[P::E];
    load_segment<P>(v, s, b * hop - off, n, t);
    for (; b < nblocks; b += gridDim.x) {
      fft_frame<P>(v, lds, tw, t);
#pragma unroll
      for (int e = 0; e < P::E; ++e) v[e] = cmul(cconj(v[e]), Ps[out_index<P>(t, e)]);
      float2 nv[P::E];
      const long long nb = b + gridDim.x;
      fft_frame_hook<P>(v, lds, tw, t, [&] {
        if (nb < nblocks) load_segment<P>(nv, s, nb * hop - off, n, t);
      });
      xcorr_epilogue<P>(v, b, hop, nout, c, store_mode, partials, t);
#pragma unroll
      for (int e = 0; e < P::E; ++e) v[e] = nv[e];
    }
    return;
  }
  float2 wa[nanch_total<P>()];
  load_anchors<P>(wa, tw, t);
  float2 v[P::E];
  load_segment<P>(v, s, b * hop - off, n, t);
  for (; b < nblocks; b += gridDim.x) {
    fft_frame_anch<P>(v, lds, wa, t);
#pragma unroll
    for (int e = 0; e < P::E; ++e) v[e] = cmul(cconj(v[e]), Ps[out_index<P>(t, e)]);
    float2 nv[P::E];   // prefetch behind the template-spectrum loads (see fir_os_kernel)
    const long long nb = b + gridDim.x;
    if (nb < nblocks) load_segment<P>(nv, s, nb * hop - off, n, t);
    fft_frame_anch<P>(v, lds, wa, t);
    xcorr_epilogue<P>(v, b, hop, nout, c, store_mode, partials, t);
#pragma unroll
    for (int e = 0; e < P::E; ++e) v[e] = nv[e];
  }
}

// ---------------------------------------------------------------------------
// Partitioned cross-correlation (uniformly partitioned overlap-save): the
// template is cut into two halves of Lp = M/2 samples; hop j's outputs are
//   c[j*Lp + i] = IFFT( X_j conj(P0) + X_{j+1} conj(P1) )[i],   i < Lp,
// X_j = FFT_M(s[j*Lp - off ...]).  A block walks a contiguous run of hops,
// carrying X_{j+1} in registers into hop j+1, so each hop costs one forward and
// one inverse M-point FFT: M = L-point FFTs (4 blocks / CU at L = 4096) instead
// of the 4L-point FFTs plain overlap-save needs for the same efficiency.
// ---------------------------------------------------------------------------
template <class P, int TWL>
__global__ __launch_bounds__(os_threads<P>(), 3) void xcorr_part_kernel(
    const float2* __restrict__ s, long long n, const float2* __restrict__ P0,
    const float2* __restrict__ P1, long long off, long long nout, int Lp, long long nhops,
    long long hpb, float2* __restrict__ c, int store_mode, PeakPartial* __restrict__ partials,
    const float2* __restrict__ tw) {
  static_assert(P::R[0] == P::RL, "overlap-save needs a palindromic plan");
  constexpr int BT = os_threads<P>();
  __shared__ float2 lds[P::LDS + (TWL ? tw2_size<P>() : 0)];
  const int t = threadIdx.x;
  const long long j0 = (long long)blockIdx.x * hpb;
  const long long j1 = j0 + hpb < nhops ? j0 + hpb : nhops;
  if (j0 >= j1) return;
  float2* t2 = lds + P::LDS;
  if constexpr (TWL) load_tw2<P>(t2, tw, t, BT);
  auto fft = [&](float2* v, int tt) {
    if constexpr (TWL) fft_frame_t2<P>(v, lds, t2, tt);
    else fft_frame<P>(v, lds, tw, tt);
  };
  float2 xn[P::E];                      // X_{j+1} of the previous hop
  load_segment<P>(xn, s, j0 * Lp - off, n, t);
  fft(xn, t);
  for (long long j = j0; j < j1; ++j) {
    // An opaque copy of the thread index: keeps the (loop-invariant) LDS and
    // twiddle address arithmetic of the three FFTs inside the loop instead of
    // hoisted into hundreds of live VGPRs.
    const int tt = t + opaque_zero();
    float2 v[P::E];
#pragma unroll
    for (int e = 0; e < P::E; ++e) v[e] = cmul(cconj(xn[e]), P0[out_index<P>(tt, e)]);
    load_segment<P>(xn, s, (j + 1) * Lp - off, n, tt);
    fft(xn, tt);
#pragma unroll
    for (int e = 0; e < P::E; ++e) {
      const float2 a = cmul(cconj(xn[e]), P1[out_index<P>(tt, e)]);
      v[e] = cadd(v[e], a);
    }
    fft(v, tt);
    xcorr_epilogue<P>(v, j, Lp, nout, c, store_mode, partials, tt);
  }
}

// ---------------------------------------------------------------------------
// Engine micro-benchmark (tuning only): `iters` back-to-back FFTs of one frame
// per block with no HBM traffic in the loop — the compute/LDS ceiling of a plan.
// ---------------------------------------------------------------------------
template <class P, int TWL>
__global__ __launch_bounds__(os_threads<P>()) void fft_bench_kernel(float2* __restrict__ io,
                                                                    int iters,
                                                                    const float2* __restrict__ tw) {
  __shared__ float2 lds[P::LDS + (TWL ? tw2_size<P>() : 0)];
  const int t = threadIdx.x;
  float2* t2 = lds + P::LDS;
  if constexpr (TWL) load_tw2<P>(t2, tw, t, os_threads<P>());
  float2 v[P::E];
  float2* f = io + (long long)blockIdx.x * P::N;
#pragma unroll
  for (int e = 0; e < P::E; ++e) v[e] = f[in_index<P>(t, e)];
  for (int it = 0; it < iters; ++it) {
    const int tt = t + opaque_zero();
    if constexpr (TWL) fft_frame_t2<P>(v, lds, t2, tt);
    else fft_frame<P>(v, lds, tw, tt);
#pragma unroll
    for (int e = 0; e < P::E; ++e) v[e] = make_float2(v[e].x * 1e-4f, v[e].y * 1e-4f);
  }
#pragma unroll
  for (int e = 0; e < P::E; ++e) f[out_index<P>(t, e)] = v[e];
}

hipError_t launch_fft_bench(int key, float2* io, int frames, int iters, const float2* tw, int twl,
                            hipStream_t st) {
#define VSIG_FB(PL)                                                                          \
  {                                                                                          \
    auto k = twl ? fft_bench_kernel<PL, 1> : fft_bench_kernel<PL, 0>;                         \
    hipLaunchKernelGGL(k, dim3(frames), dim3(os_threads<PL>()), 0, st, io, iters, tw);        \
  }
  switch (key) {
    case -1024: VSIG_FB(Plan1024s) break;
    case -2048: VSIG_FB(Plan2048s) break;
    case 4096: VSIG_FB(Plan4096) break;
    case 8192: VSIG_FB(Plan8192) break;
    case 16384: VSIG_FB(Plan16384) break;
    case -16384: VSIG_FB(Plan16384w) break;
    default: return hipErrorInvalidValue;
  }
#undef VSIG_FB
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// |c| reduction over an array in double precision (find_correlation_peak,
// utils.py:1321-1334): |c| = hypot(re, im) like np.abs, first max wins.
// T = double2 (complex128), float2 (complex64), double, float.
// ---------------------------------------------------------------------------
template <class T> __device__ __forceinline__ double absval(const T* p, long long i);
template <> __device__ __forceinline__ double absval<double2>(const double2* p, long long i) {
  const double2 v = p[i]; return hypot(v.x, v.y);
}
template <> __device__ __forceinline__ double absval<float2>(const float2* p, long long i) {
  const float2 v = p[i]; return (double)hypotf(v.x, v.y);
}
template <> __device__ __forceinline__ double absval<double>(const double* p, long long i) { return fabs(p[i]); }
template <> __device__ __forceinline__ double absval<float>(const float* p, long long i) { return (double)fabsf(p[i]); }

template <class T>
__global__ __launch_bounds__(256) void peak_reduce(const T* __restrict__ a, long long n,
                                                   PeakPartial* __restrict__ partials) {
  double m = -1.0, s1 = 0.0, s2 = 0.0;
  long long mi = 0x7fffffffffffffffLL;
  const long long stride = (long long)gridDim.x * 256;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += stride) {
    const double v = absval<T>(a, i);
    betterd(m, mi, v, i);
    s1 += v;
    s2 += v * v;
  }
  block_partial<256>(m, mi, s1, s2, partials + blockIdx.x);
}

// Fixed-order reduction of nparts partials into out[0]; sqrt_max converts a
// max |c|^2 into max |c|.
__global__ __launch_bounds__(1024) void partial_finalize(const PeakPartial* __restrict__ parts,
                                                         long long nparts, int sqrt_max,
                                                         PeakPartial* __restrict__ out) {
  double m = -1.0, s1 = 0.0, s2 = 0.0;
  long long mi = 0x7fffffffffffffffLL;
  for (long long i = threadIdx.x; i < nparts; i += 1024) {
    const PeakPartial p = parts[i];
    betterd(m, mi, p.max2, p.idx);
    s1 += p.sum_abs;
    s2 += p.sum_abs2;
  }
  __shared__ PeakPartial tmp[1];
  block_partial<1024>(m, mi, s1, s2, tmp);
  __syncthreads();
  if (threadIdx.x == 0) {
    PeakPartial r = tmp[0];
    if (sqrt_max) r.max2 = sqrt(r.max2);
    *out = r;
  }
}

// First level of a large reduction: block k reduces the fixed chunk
// [k*chunk, (k+1)*chunk) into tmp[k] (fixed order -> reproducible).
__global__ __launch_bounds__(256) void partial_chunks(const PeakPartial* __restrict__ parts,
                                                      long long nparts, long long chunk,
                                                      PeakPartial* __restrict__ tmp) {
  const long long lo = (long long)blockIdx.x * chunk;
  const long long hi = lo + chunk < nparts ? lo + chunk : nparts;
  double m = -1.0, s1 = 0.0, s2 = 0.0;
  long long mi = 0x7fffffffffffffffLL;
  for (long long i = lo + threadIdx.x; i < hi; i += 256) {
    const PeakPartial p = parts[i];
    betterd(m, mi, p.max2, p.idx);
    s1 += p.sum_abs;
    s2 += p.sum_abs2;
  }
  block_partial<256>(m, mi, s1, s2, tmp + blockIdx.x);
}

// ---------------------------------------------------------------------------
// Host-side launchers (called from vsig_api.hip), dispatching N to plans.
// ---------------------------------------------------------------------------
// Resident blocks of a persistent kernel: CUs x blocks per CU (occupancy API).
template <class K>
long long persistent_grid(K kernel, int block, long long units) {
  static thread_local int cus = 0;
  if (!cus) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (cus <= 0) cus = 256;
  }
  int per = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, kernel, block, 0) != hipSuccess || per < 1)
    per = 1;
  const long long g = (long long)cus * per;
  return units < g ? units : g;
}

#define VSIG_PLAN_SWITCH(N, ...)                          \
  switch (N) {                                             \
    case 64: { using PL = Plan64; __VA_ARGS__; } break;           \
    case 128: { using PL = Plan128; __VA_ARGS__; } break;         \
    case 256: { using PL = Plan256; __VA_ARGS__; } break;         \
    case 512: { using PL = Plan512; __VA_ARGS__; } break;         \
    case 1024: { using PL = Plan1024; __VA_ARGS__; } break;       \
    case 2048: { using PL = Plan2048; __VA_ARGS__; } break;       \
    case 4096: { using PL = Plan4096; __VA_ARGS__; } break;       \
    case 8192: { using PL = Plan8192; __VA_ARGS__; } break;       \
    case 16384: { using PL = Plan16384; __VA_ARGS__; } break;     \
    default: return hipErrorInvalidValue;                  \
  }

template <class PL, int PERSIST>
void launch_psd_t(const float2* x, long long stride, const float* win, int nperseg, long long hop,
                  float scale, float* out, long long nframes, int shift, const float2* tw,
                  hipStream_t st) {
  constexpr int BT = block_threads<PL>();
  constexpr int FPB = BT / PL::TF;
  const long long units = (nframes + FPB - 1) / FPB;
  const long long grid =
      (PERSIST == 1 || PERSIST == 2) ? persistent_grid(psd_kernel<PL, PERSIST>, BT, units) : units;
  hipLaunchKernelGGL((psd_kernel<PL, PERSIST>), dim3((unsigned)grid), dim3(BT), 0, st, x, stride,
                     win, nperseg, hop, scale, out, nframes, shift, tw);
}

hipError_t launch_psd(int N, const float2* x, long long stride, const float* win, int nperseg,
                      long long hop, float scale, float* out, long long nframes, int shift,
                      const float2* tw, int variant, hipStream_t st) {
  if (nframes <= 0) return hipSuccess;
  VSIG_PLAN_SWITCH(N, {
    if (variant & 16) launch_psd_t<PL, 4>(x, stride, win, nperseg, hop, scale, out, nframes, shift, tw, st);
    else if (variant & 8) launch_psd_t<PL, 3>(x, stride, win, nperseg, hop, scale, out, nframes, shift, tw, st);
    else if (variant & 4) launch_psd_t<PL, 2>(x, stride, win, nperseg, hop, scale, out, nframes, shift, tw, st);
    else if (variant & 1) launch_psd_t<PL, 1>(x, stride, win, nperseg, hop, scale, out, nframes, shift, tw, st);
    else launch_psd_t<PL, 0>(x, stride, win, nperseg, hop, scale, out, nframes, shift, tw, st);
  });
  return hipGetLastError();
}

hipError_t launch_spectrum_prep(int N, const float2* u, int len, float gain, float2* S,
                                const float2* tw, hipStream_t st) {
  VSIG_PLAN_SWITCH(N, {
    hipLaunchKernelGGL(spectrum_prep<PL>, dim3(1), dim3(block_threads<PL>()), 0, st, u, len,
                       gain, S, tw);
  });
  return hipGetLastError();
}

// Only plans with one frame per block can run the overlap-save kernels.
// variant bit 0: persistent (prefetch + register anchors); bit 1: the E = 32 /
// 512-thread plan for M = 16384 instead of E = 16 / 1024 threads.
#define VSIG_OS_SWITCH(N, V, ...)                                          \
  switch (N) {                                                              \
    case 1024: { using PL = Plan1024s; __VA_ARGS__; } break;                \
    case 2048: { using PL = Plan2048s; __VA_ARGS__; } break;                \
    case 4096: { using PL = Plan4096; __VA_ARGS__; } break;                        \
    case 8192: { using PL = Plan8192; __VA_ARGS__; } break;                        \
    case 16384:                                                             \
      if ((V) & 2) { using PL = Plan16384w; __VA_ARGS__; }                         \
      else { using PL = Plan16384; __VA_ARGS__; }                                  \
      break;                                                                \
    default: return hipErrorInvalidValue;                                   \
  }

template <class PL, int PERSIST>
void launch_fir_t(const float2* x, long long n, long long g0, const float2* Hs, int ntaps,
                  long long hop, int decim, float2* y, long long nblocks, const float2* tw,
                  hipStream_t st) {
  const long long grid =
      (PERSIST == 1 || PERSIST == 2)
          ? persistent_grid(fir_os_kernel<PL, PERSIST>, os_threads<PL>(), nblocks) : nblocks;
  hipLaunchKernelGGL((fir_os_kernel<PL, PERSIST>), dim3((unsigned)grid), dim3(os_threads<PL>()),
                     0, st, x, n, g0, Hs, ntaps, hop, decim, y, nblocks, tw);
}

hipError_t launch_fir_os(int M, const float2* x, long long n, long long g0, const float2* Hs,
                         int ntaps, long long hop, int decim, float2* y, const float2* tw,
                         int variant, hipStream_t st) {
  if (n - g0 <= 0) return hipSuccess;
  const long long nblocks = (n - g0 + hop - 1) / hop;
  VSIG_OS_SWITCH(M, variant, {
    if (variant & 16) launch_fir_t<PL, 4>(x, n, g0, Hs, ntaps, hop, decim, y, nblocks, tw, st);
    else if (variant & 8) launch_fir_t<PL, 3>(x, n, g0, Hs, ntaps, hop, decim, y, nblocks, tw, st);
    else if (variant & 4) launch_fir_t<PL, 2>(x, n, g0, Hs, ntaps, hop, decim, y, nblocks, tw, st);
    else if (variant & 1) launch_fir_t<PL, 1>(x, n, g0, Hs, ntaps, hop, decim, y, nblocks, tw, st);
    else launch_fir_t<PL, 0>(x, n, g0, Hs, ntaps, hop, decim, y, nblocks, tw, st);
  });
  return hipGetLastError();
}

template <class PL, int PERSIST>
void launch_xcorr_t(const float2* s, long long n, const float2* Ps, long long off, long long nout,
                    long long hop, float2* c, int store_mode, PeakPartial* partials,
                    long long nblocks, const float2* tw, hipStream_t st) {
  const long long grid =
      (PERSIST == 1 || PERSIST == 2)
          ? persistent_grid(xcorr_os_kernel<PL, PERSIST>, os_threads<PL>(), nblocks) : nblocks;
  hipLaunchKernelGGL((xcorr_os_kernel<PL, PERSIST>), dim3((unsigned)grid),
                     dim3(os_threads<PL>()), 0, st, s, n, Ps, off, nout, hop, c, store_mode,
                     partials, nblocks, tw);
}

hipError_t launch_xcorr_os(int M, const float2* s, long long n, const float2* Ps, long long off,
                           long long nout, long long hop, float2* c, int store_mode,
                           PeakPartial* partials, const float2* tw, int variant, hipStream_t st) {
  if (nout <= 0) return hipSuccess;
  const long long nblocks = (nout + hop - 1) / hop;
  VSIG_OS_SWITCH(M, variant, {
    if (variant & 16) launch_xcorr_t<PL, 4>(s, n, Ps, off, nout, hop, c, store_mode, partials, nblocks, tw, st);
    else if (variant & 8) launch_xcorr_t<PL, 3>(s, n, Ps, off, nout, hop, c, store_mode, partials, nblocks, tw, st);
    else if (variant & 4) launch_xcorr_t<PL, 2>(s, n, Ps, off, nout, hop, c, store_mode, partials, nblocks, tw, st);
    else if (variant & 1) launch_xcorr_t<PL, 1>(s, n, Ps, off, nout, hop, c, store_mode, partials, nblocks, tw, st);
    else launch_xcorr_t<PL, 0>(s, n, Ps, off, nout, hop, c, store_mode, partials, nblocks, tw, st);
  });
  return hipGetLastError();
}

hipError_t launch_xcorr_part(int M, const float2* s, long long n, const float2* P0,
                             const float2* P1, long long off, long long nout, float2* c,
                             int store_mode, PeakPartial* partials, const float2* tw, int twl,
                             hipStream_t st) {
  if (nout <= 0) return hipSuccess;
  const int Lp = M / 2;
  const long long nhops = (nout + Lp - 1) / Lp;
  VSIG_OS_SWITCH(M, 0, {
    auto k = twl ? xcorr_part_kernel<PL, 1> : xcorr_part_kernel<PL, 0>;
    const long long g = persistent_grid(k, os_threads<PL>(), nhops);
    const long long hpb = (nhops + g - 1) / g;
    const long long grid = (nhops + hpb - 1) / hpb;
    hipLaunchKernelGGL(k, dim3((unsigned)grid), dim3(os_threads<PL>()), 0, st, s, n, P0, P1,
                       off, nout, Lp, nhops, hpb, c, store_mode, partials, tw);
  });
  return hipGetLastError();
}

hipError_t launch_peak_reduce(int dtype, const void* a, long long n, PeakPartial* partials,
                              int nparts, hipStream_t st) {
  switch (dtype) {
    case VSIG_C128: hipLaunchKernelGGL(peak_reduce<double2>, dim3(nparts), dim3(256), 0, st, (const double2*)a, n, partials); break;
    case VSIG_C64: hipLaunchKernelGGL(peak_reduce<float2>, dim3(nparts), dim3(256), 0, st, (const float2*)a, n, partials); break;
    case VSIG_F64: hipLaunchKernelGGL(peak_reduce<double>, dim3(nparts), dim3(256), 0, st, (const double*)a, n, partials); break;
    case VSIG_F32: hipLaunchKernelGGL(peak_reduce<float>, dim3(nparts), dim3(256), 0, st, (const float*)a, n, partials); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

hipError_t launch_partial_finalize(const PeakPartial* parts, long long nparts, int sqrt_max,
                                   PeakPartial* out, PeakPartial* tmp, hipStream_t st) {
  if (nparts > 8192 && tmp) {       // two levels: chunks in parallel, then one block
    long long g1 = (nparts + 2047) / 2048;
    if (g1 > kFinalizeTmp) g1 = kFinalizeTmp;
    const long long chunk = (nparts + g1 - 1) / g1;
    g1 = (nparts + chunk - 1) / chunk;
    hipLaunchKernelGGL(partial_chunks, dim3((unsigned)g1), dim3(256), 0, st, parts, nparts, chunk, tmp);
    hipLaunchKernelGGL(partial_finalize, dim3(1), dim3(1024), 0, st, tmp, g1, sqrt_max, out);
  } else {
    hipLaunchKernelGGL(partial_finalize, dim3(1), dim3(1024), 0, st, parts, nparts, sqrt_max, out);
  }
  return hipGetLastError();
}

int os_waves(int M, int variant) {
  switch (M) {
    case 1024: return os_threads<Plan1024s>() / 64;
    case 2048: return os_threads<Plan2048s>() / 64;
    case 4096: return os_threads<Plan4096>() / 64;
    case 8192: return os_threads<Plan8192>() / 64;
    case 16384: return (variant & 2) ? os_threads<Plan16384w>() / 64 : os_threads<Plan16384>() / 64;
    default: return 0;
  }
}

}  // namespace vsig

namespace vsig {
hipError_t tw2_info(int N, int* shift, int* hi) {
  if (N == -16384) { *shift = tw2_shift<Plan16384w>(); *hi = tw2_hi<Plan16384w>(); return hipSuccess; }
  if (N == -1024) { *shift = tw2_shift<Plan1024s>(); *hi = tw2_hi<Plan1024s>(); return hipSuccess; }
  if (N == -2048) { *shift = tw2_shift<Plan2048s>(); *hi = tw2_hi<Plan2048s>(); return hipSuccess; }
  VSIG_PLAN_SWITCH(N, { *shift = tw2_shift<PL>(); *hi = tw2_hi<PL>(); });
  return hipSuccess;
}

hipError_t plan_info(int N, int* radices, int* npasses) {
  if (N == -16384) {   // the E = 32 plan of 16384 points (variant bit 1)
    *npasses = Plan16384w::NP;
    for (int q = 0; q < Plan16384w::NP; ++q) radices[q] = Plan16384w::R[q];
    return hipSuccess;
  }
  if (N == -1024 || N == -2048) {   // one-wave overlap-save plans
    const int np = N == -1024 ? Plan1024s::NP : Plan2048s::NP;
    *npasses = np;
    for (int q = 0; q < np; ++q) radices[q] = N == -1024 ? Plan1024s::R[q] : Plan2048s::R[q];
    return hipSuccess;
  }
  VSIG_PLAN_SWITCH(N, {
    *npasses = PL::NP;
    for (int q = 0; q < PL::NP; ++q) radices[q] = PL::R[q];
  });
  return hipSuccess;
}
}  // namespace vsig
