// Fused FIR -> PSD kernel (gfx950): one launch filters a chunk (overlap-save,
// M = 1024, one wave per segment pair) and computes the Hann/any-window
// spectrogram of the filtered stream (nfft = nperseg = hop = 8192, two frames
// per block through fft_pair), so the filtered stream is written to HBM once
// (filter()'s output) and re-read by the PSD from this XCD's L2 / the Infinity
// Cache instead of HBM: 20 instead of 28 HBM bytes per input sample.
//
// Semantics = vsig_fir_exec_hist_dev (np.convolve(x, h, 'full')[g0:n], the
// first g0 samples of x history) followed by vsig_psd_c64_dev on its output
// (scipy.signal.spectrogram, return_onesided=False, scaling='spectrum', as
// called at utils.py:281-291), frame f = y[f*8192 .. +8192).
#include "os_common.hpp"

namespace vsig {

// Block u owns outputs [u*2N, u*2N + 2N) of the chunk (N = PSD frame) and the
// two PSD frames over them.
//   FIR phase: the 2N outputs are cut into SEG = 2 * NW * ROUNDS segments of
//   `sh` outputs (the last one shorter); wave w filters segment pairs
//   p = r*NW + w, r < ROUNDS, each through its own slice of the block's LDS
//   (overlap-save with the one-wave 1024-point plan, register anchors); the
//   outputs are stored to y (plain stores: they are read back below).
//   PSD phase: after every wave's stores have completed (vmcnt(0) + barrier),
//   the block loads its two frames back (L2 hits), windows them and runs one
//   fft_pair over the whole LDS buffer; |X|^2 * scale -> sxx (non-temporal).
template <class PF, class PS, int ROUNDS, bool NT_Y, bool PREF>
__global__ __launch_bounds__(PS::TF, 2) void fir_psd_kernel(
    const float2* __restrict__ x, long long n, long long g0, const float2* __restrict__ Hs,
    int ntaps, int sh, float2* __restrict__ y, const float* __restrict__ win, float scale,
    int shift, float* __restrict__ sxx, long long nframes, long long nblocks,
    const float2* __restrict__ twf, const float2* __restrict__ tws) {
  constexpr int NW = PS::TF / 64;
  constexpr int OUT = 2 * PS::N;
  static_assert(PF::TF == 64 && PF::R[0] == PF::RL, "one-wave palindromic FIR plan");
  static_assert(NW * PF::LDS <= PS::LDS, "FIR slices must fit the PSD buffer");
  __shared__ float2 lds[PS::LDS];
  const int wv = threadIdx.x >> 6, l = threadIdx.x & 63;
  const long long u = xcd_remap(blockIdx.x, gridDim.x);
  if (u >= nblocks) return;                           // uniform per block
  const long long nloc = n - g0;
  const long long o0 = u * OUT;
  const int lo = ntaps - 1;
  float2* wl = lds + wv * PF::LDS;
  {
    float2 wa[nanch_total<PF>()];
    load_anchors<PF>(wa, twf, l);
    // segment pair of round r: outputs from o0 + j0*sh, j0 = 2 (r NW + wv)
    auto seg0 = [&](int r) { return o0 + (long long)(2 * (r * NW + wv)) * sh; };
    float2 a[PF::E], d[PF::E];
    load_segment<PF>(a, x, g0 + seg0(0) - lo, n, l);
    load_segment<PF>(d, x, g0 + seg0(0) + sh - lo, n, l);
#pragma unroll 1
    for (int r = 0; r < ROUNDS; ++r) {
      const int j0 = 2 * (r * NW + wv);
      const long long s0 = seg0(r);
      launder_anchors<PF>(wa);
      fft_pair<PF>(a, d, wl, TwAnchors{wa}, l);
#pragma unroll
      for (int e = 0; e < PF::E; ++e) {
        const float2 h = Hs[out_index<PF>(l, e)];
        a[e] = cconj(cmul(a[e], h));
        d[e] = cconj(cmul(d[e], h));
      }
      // next round's segments: issued behind the (L2-resident) filter-spectrum
      // loads, so they land while the inverse transforms run
      float2 na[PF::E], nd[PF::E];
      if (PREF && r + 1 < ROUNDS) {
        const long long s1 = seg0(r + 1);
        load_segment<PF>(na, x, g0 + s1 - lo, n, l);
        load_segment<PF>(nd, x, g0 + s1 + sh - lo, n, l);
      }
      launder_anchors<PF>(wa);
      fft_pair<PF>(a, d, wl, TwAnchors{wa}, l);
      // valid circular outputs i in [lo, lo + cnt) of each segment
#pragma unroll
      for (int f = 0; f < 2; ++f) {
        const int j = j0 + f;
        const long long sb = s0 + (long long)f * sh;
        const long long blk_rem = (long long)OUT - (long long)j * sh;
        const long long loc_rem = nloc - sb;
        long long cnt = blk_rem < sh ? blk_rem : sh;
        cnt = loc_rem < cnt ? loc_rem : cnt;
        const int c = cnt > 0 ? (int)cnt : 0;
        float2* yb = y + sb;
        const float2* v = f ? d : a;
#pragma unroll
        for (int e = 0; e < PF::E; ++e) {
          const int i = out_index<PF>(l, e) - lo;
          if (i >= 0 && i < c) st_stream<NT_Y>(yb + i, cconj(v[e]));
        }
      }
      if (r + 1 < ROUNDS) {
        if (PREF) {
#pragma unroll
          for (int e = 0; e < PF::E; ++e) { a[e] = na[e]; d[e] = nd[e]; }
        } else {
          const long long s1 = seg0(r + 1);
          load_segment<PF>(a, x, g0 + s1 - lo, n, l);
          load_segment<PF>(d, x, g0 + s1 + sh - lo, n, l);
        }
      }
    }
  }
  // every wave's filtered samples are in L2 before any wave reads them back
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  const int t = threadIdx.x;
  float2 wa[nanch_total<PS>()];
  load_anchors<PS>(wa, tws, t);
  float2 v[2][PS::E];
#pragma unroll
  for (int f = 0; f < 2; ++f) {
    const long long frame = 2 * u + f;
    const bool active = frame < nframes;
    const float2* yf = y + (active ? frame * PS::N : 0);
#pragma unroll
    for (int e = 0; e < PS::E; ++e) {
      const int i = in_index<PS>(t, e);
      const float2 s = active ? yf[i] : make_float2(0.f, 0.f);
      const float w = win[i];
      v[f][e] = make_float2(s.x * w, s.y * w);
    }
  }
  launder_anchors<PS>(wa);
  fft_pair<PS>(v[0], v[1], lds, TwAnchors{wa}, t);
#pragma unroll
  for (int f = 0; f < 2; ++f) {
    const long long frame = 2 * u + f;
    if (frame < nframes) {
      float* of = sxx + frame * PS::N;
#pragma unroll
      for (int e = 0; e < PS::E; ++e) {
        const int i = out_index<PS>(t, e);
        const int o = shift ? ((i + PS::N / 2) & (PS::N - 1)) : i;
        __builtin_nontemporal_store((v[f][e].x * v[f][e].x + v[f][e].y * v[f][e].y) * scale, of + o);
      }
    }
  }
}

// Segment length of the fused kernel for nfft = 8192: 24 segments of 683
// outputs per 16384-output block (3 rounds of one pair per wave); needs
// ntaps - 1 + 683 <= 1024.
int fir_psd_seg_hop(int nfft) { return nfft == 8192 ? 683 : 0; }

hipError_t launch_fir_psd(int nfft, const float2* x, long long n, long long g0, const float2* Hs,
                          int ntaps, float2* y, const float* win, float scale, int shift,
                          float* sxx, long long nframes, const float2* twf, const float2* tws,
                          int variant, hipStream_t st) {
  const long long nloc = n - g0;
  if (nloc <= 0) return hipSuccess;
  if (nfft != 8192) return hipErrorInvalidValue;
  using PS = Plan8192;
  constexpr int ROUNDS = 3;
  const int sh = fir_psd_seg_hop(nfft);
  static_assert(2 * (PS::TF / 64) * ROUNDS * 683 >= 2 * PS::N, "segments must cover the block");
  if (ntaps - 1 + sh > Plan1024s::N) return hipErrorInvalidValue;
  const long long nblocks = (nloc + 2 * PS::N - 1) / (2 * PS::N);
  if ((nframes + 1) / 2 > nblocks) return hipErrorInvalidValue;
  const dim3 g((unsigned)nblocks), b(PS::TF);
  // variant bit 0: non-temporal y stores; bit 1: block barriers in the FIR
  // phase (instead of wave barriers); bit 2: next-round prefetch (spills)
#define VSIG_FP(NT, PF_, PREF)                                                                  \
  hipLaunchKernelGGL((fir_psd_kernel<PF_, PS, ROUNDS, NT, PREF>), g, b, 0, st, x, n, g0, Hs,    \
                     ntaps, sh, y, win, scale, shift, sxx, nframes, nblocks, twf, tws)
  using PW = WaveSync<Plan1024s>;
  switch (variant & 7) {
    case 0: VSIG_FP(false, PW, false); break;
    case 1: VSIG_FP(true, PW, false); break;
    case 2: VSIG_FP(false, Plan1024s, false); break;
    case 4: VSIG_FP(false, PW, true); break;
    case 6: VSIG_FP(false, Plan1024s, true); break;
    default: return hipErrorInvalidValue;
  }
#undef VSIG_FP
  return hipGetLastError();
}

}  // namespace vsig
