// Overlap-save FIR kernel (gfx950), decimation folded into the store (filter).
#include "os_common.hpp"

namespace vsig {

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
      if (i >= 0 && i < lim) st_stream(yb + (unsigned)i, cconj(v[e]));
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
      if (i >= 0 && i < lim && (unsigned)i == q * (unsigned)decim) st_stream(yb + q, cconj(v[e]));
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
template <class P, int PERSIST, bool MIX = false>
__global__ __launch_bounds__(os_threads<P>(), (min_waves<P, PERSIST>())) void fir_os_kernel(
    const float2* __restrict__ x, long long n, long long g0, const float2* __restrict__ Hs,
    int ntaps, long long hop, int decim, float2* __restrict__ y, long long nblocks,
    const float2* __restrict__ tw, MixArgs mix) {
  static_assert(!MIX || PERSIST == 6, "the fused mixer is built for the pair kernel");
  static_assert(P::R[0] == P::RL, "overlap-save needs a palindromic plan");
  constexpr int BT = os_threads<P>();
  static_assert(BT == P::TF, "one frame per block");
  __shared__ float2 lds[os_lds<P, PERSIST>()];
  const int t = threadIdx.x;
  long long b = PERSIST == 0 || PERSIST >= 3 ? xcd_remap(stage_bid<1>(), gridDim.x) : blockIdx.x;
  if (b >= nblocks) return;  // uniform per block

  const int lo = ntaps - 1;
  const long long nloc = n - g0;
  if constexpr (PERSIST == 5) {      // one unit per block, register twiddle anchors
    float2 wa[nanch_total<P>()];
    load_anchors<P>(wa, tw, t);
    float2 v[P::E];
    load_segment<P>(v, x, g0 + b * hop - lo, n, t);
    fft_frame_anch<P>(v, lds, wa, t);
#pragma unroll
    for (int e = 0; e < P::E; ++e) v[e] = cconj(cmul(v[e], Hs[out_index<P>(t, e)]));
    fft_frame_anch<P>(v, lds, wa, t);
    fir_store<P>(v, y, b, hop, lo, nloc, decim, t);
    return;
  }
  if constexpr (PERSIST == 6 || PERSIST == 7) {   // two consecutive units per block (fft_pair):
    // 6: register twiddle anchors; 7: exact per-thread twiddles in registers (TwRegs)
    constexpr bool RT = PERSIST == 7;
    float2 wa[RT ? rtw_total<P>() : nanch_total<P>()];
    if constexpr (RT) load_rtw<P>(wa, tw, t);
    else load_anchors<P>(wa, tw, t);
    const long long b0 = 2 * b, b1 = 2 * b + 1;
    float2 a[P::E], d[P::E];
    if constexpr (MIX) {
      load_segment_mix<P>(a, x, g0 + b0 * hop - lo, n, t, mix);
      load_segment_mix<P>(d, x, g0 + b1 * hop - lo, n, t, mix);
    } else {
      load_segment<P>(a, x, g0 + b0 * hop - lo, n, t);
      load_segment<P>(d, x, g0 + b1 * hop - lo, n, t);
    }
    auto fft2 = [&]() {
      if constexpr (RT) fft_pair<P>(a, d, lds, TwRegs{wa}, t);
      else { launder_anchors<P>(wa); fft_pair<P>(a, d, lds, TwAnchors{wa}, t); }
    };
    fft2();
#pragma unroll
    for (int e = 0; e < P::E; ++e) {
      const float2 h = Hs[out_index<P>(t, e)];
      a[e] = cconj(cmul(a[e], h));
      d[e] = cconj(cmul(d[e], h));
    }
    fft2();
    fir_store<P>(a, y, b0, hop, lo, nloc, decim, t);
    fir_store<P>(d, y, b1, hop, lo, nloc, decim, t);
    return;
  }
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
// Decimating FIR (variant bit 8), decimation in the frequency domain: after
// FFT_M(segment) x H/M, only every D-th output of the block is wanted, and
//   y[D n] = sum_{k' < M/D} Yd[k'] W_{M/D}^{-n k'},  Yd[k'] = sum_{m < D} Y[k' + m M/D],
// so the inverse transform shrinks to M/D points (PD) after an in-register
// fold (thread t holds Y[t + 64 r] and Yd[t + 64 r'] with r = r' + m E/D).
// The segment starts lo2 = ceil((ntaps-1)/D)*D samples before the block's
// first output so kept outputs sit at circular indices D n, n >= lo2/D; hop
// is a multiple of D.  Two segments per wave (fft_pair), anchors for the
// M-point transforms, exact register twiddles for the small ones.
// ---------------------------------------------------------------------------
template <class P, class PD, bool MIX = false>
__global__ __launch_bounds__(P::TF) void fir_dec_kernel(
    const float2* __restrict__ x, long long n, long long g0, const float2* __restrict__ Hs, int lo2,
    long long hop, float2* __restrict__ y, long long nblocks, const float2* __restrict__ tw,
    const float2* __restrict__ twd, MixArgs mix) {
  constexpr int D = P::N / PD::N;
  static_assert(P::TF == PD::TF && P::E == D * PD::E && P::RL == P::E && PD::R[0] == PD::E,
                "fold needs thread t to hold bins t + TF r of both plans");
  __shared__ float2 lds[P::LDS];
  const int t = threadIdx.x;
  const long long b = xcd_remap(blockIdx.x, gridDim.x);
  if (2 * b >= nblocks) return;
  const long long nloc = n - g0;
  float2 wa[nanch_total<P>()];
  load_anchors<P>(wa, tw, t);
  float2 wr[rtw_total<PD>()];
  load_rtw<PD>(wr, twd, t);
  float2 a[P::E], d[P::E];
  if constexpr (MIX) {
    load_segment_mix<P>(a, x, g0 + (2 * b) * hop - lo2, n, t, mix);
    load_segment_mix<P>(d, x, g0 + (2 * b + 1) * hop - lo2, n, t, mix);
  } else {
    load_segment<P>(a, x, g0 + (2 * b) * hop - lo2, n, t);
    load_segment<P>(d, x, g0 + (2 * b + 1) * hop - lo2, n, t);
  }
  launder_anchors<P>(wa);
  fft_pair<P>(a, d, lds, TwAnchors{wa}, t);
  float2 ua[PD::E], ud[PD::E];
#pragma unroll
  for (int r = 0; r < PD::E; ++r) {
    float2 sa = make_float2(0.f, 0.f), sd = make_float2(0.f, 0.f);
#pragma unroll
    for (int m = 0; m < D; ++m) {
      const int e = r + m * PD::E;
      const float2 h = Hs[out_index<P>(t, e)];
      sa = cadd(sa, cmul(a[e], h));
      sd = cadd(sd, cmul(d[e], h));
    }
    ua[r] = cconj(sa);
    ud[r] = cconj(sd);
  }
  fft_pair<PD>(ua, ud, lds, TwRegs{wr}, t);
  const int n0 = lo2 / D, n1 = (lo2 + (int)hop) / D;
#pragma unroll
  for (int f = 0; f < 2; ++f) {
    const long long bb = 2 * b + f;
    const long long gb = bb * hop - lo2;          // chunk output of circular index 0
    float2* yb = y + bb * (hop / D) - n0;
    const float2* u = f ? ud : ua;
#pragma unroll
    for (int e = 0; e < PD::E; ++e) {
      const int i = out_index<PD>(t, e);
      if (i >= n0 && i < n1 && gb + (long long)i * D < nloc) st_stream(yb + i, cconj(u[e]));
    }
  }
}

hipError_t launch_fir_dec(int decim, const float2* x, long long n, long long g0, const float2* Hs,
                          int lo2, long long hop, float2* y, const float2* tw, const float2* twd,
                          hipStream_t st, const MixArgs* mix) {
  if (n - g0 <= 0) return hipSuccess;
  const long long nblocks = (n - g0 + hop - 1) / hop;
  const dim3 g((unsigned)((nblocks + 1) / 2)), blk(Plan1024s::TF);
  const MixArgs m = mix ? *mix : MixArgs{};
#define VSIG_FD(PD)                                                                              \
  do {                                                                                           \
    if (mix)                                                                                     \
      hipLaunchKernelGGL((fir_dec_kernel<Plan1024s, PD, true>), g, blk, 0, st, x, n, g0, Hs, lo2, \
                         hop, y, nblocks, tw, twd, m);                                           \
    else                                                                                         \
      hipLaunchKernelGGL((fir_dec_kernel<Plan1024s, PD, false>), g, blk, 0, st, x, n, g0, Hs,    \
                         lo2, hop, y, nblocks, tw, twd, m);                                      \
  } while (0)
  if (decim == 4) VSIG_FD(Plan256d);
  else if (decim == 2) VSIG_FD(Plan512d);
  else return hipErrorInvalidValue;
#undef VSIG_FD
  return hipGetLastError();
}

template <class PL, int PERSIST, bool MIX = false>
void launch_fir_t(const float2* x, long long n, long long g0, const float2* Hs, int ntaps,
                  long long hop, int decim, float2* y, long long nblocks, const float2* tw,
                  hipStream_t st, MixArgs mix = MixArgs{}) {
  const long long grid =
      (PERSIST == 1 || PERSIST == 2)
          ? persistent_grid(fir_os_kernel<PL, PERSIST>, os_threads<PL>(), nblocks)
          : (PERSIST == 6 || PERSIST == 7) ? (nblocks + 1) / 2 : nblocks;
  hipLaunchKernelGGL((fir_os_kernel<PL, PERSIST, MIX>), dim3((unsigned)grid), dim3(os_threads<PL>()),
                     0, st, x, n, g0, Hs, ntaps, hop, decim, y, nblocks, tw, mix);
}

hipError_t launch_fir_os(int M, const float2* x, long long n, long long g0, const float2* Hs,
                         int ntaps, long long hop, int decim, float2* y, const float2* tw,
                         int variant, hipStream_t st, const MixArgs* mix) {
  if (n - g0 <= 0) return hipSuccess;
  const long long nblocks = (n - g0 + hop - 1) / hop;
  if (mix) {   // fused mixer: the default one-wave pair kernel (M = 1024) only
    if ((variant & (8 | 16 | 128)) || !(variant & 64) || M != 1024) return hipErrorInvalidValue;
    launch_fir_t<Plan1024s, 6, true>(x, n, g0, Hs, ntaps, hop, decim, y, nblocks, tw, st, *mix);
    return hipGetLastError();
  }
  VSIG_OS_SWITCH(M, variant, {
    // (bits 3/4 first: they select the two-level twiddle table the API built)
    if (variant & 16) launch_fir_t<PL, 4>(x, n, g0, Hs, ntaps, hop, decim, y, nblocks, tw, st);
    else if (variant & 8) launch_fir_t<PL, 3>(x, n, g0, Hs, ntaps, hop, decim, y, nblocks, tw, st);
    else if (variant & 128) launch_fir_t<PL, 7>(x, n, g0, Hs, ntaps, hop, decim, y, nblocks, tw, st);
    else if (variant & 64) launch_fir_t<PL, 6>(x, n, g0, Hs, ntaps, hop, decim, y, nblocks, tw, st);
    else if (variant & 32) launch_fir_t<PL, 5>(x, n, g0, Hs, ntaps, hop, decim, y, nblocks, tw, st);
    else if (variant & 4) launch_fir_t<PL, 2>(x, n, g0, Hs, ntaps, hop, decim, y, nblocks, tw, st);
    else if (variant & 1) launch_fir_t<PL, 1>(x, n, g0, Hs, ntaps, hop, decim, y, nblocks, tw, st);
    else launch_fir_t<PL, 0>(x, n, g0, Hs, ntaps, hop, decim, y, nblocks, tw, st);
  });
  return hipGetLastError();
}

}  // namespace vsig
