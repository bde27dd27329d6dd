// Cross-correlation kernels (gfx950): overlap-save correlation with the fused
// |c|^2 argmax / sums epilogue (correlate, find_correlation_peak), its
// half-frame (two blocks per CU) and partitioned-template forms.
#include "os_common.hpp"

namespace vsig {

// ---------------------------------------------------------------------------
// Cross-correlation, overlap-save:  c[o] = sum_{k<L} s[o - off + k] * conj(p[k]),
// o in [0, nout).  off = 0 -> np.correlate 'valid'; off = L-1 -> 'full'.
// Block b: outputs [b*hop, b*hop + hop), hop <= M - L + 1.
// Epilogue: optional store of c (store_mode 1) or of conj(c) at nout-1-o
// (store_mode 2, the swapped argument order of np.correlate), and the block's
// |c| partial; store_mode bit 4 reports the argmax in the reversed index
// space (first maximum of the reversed output); bit 8 adds to c instead of
// storing (templates longer than 8192 run as a sum of template chunks).
__device__ __forceinline__ void put_c(float2* p, float2 v, bool accum) {
  *p = accum ? cadd(*p, v) : v;
}
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
  const bool accum = store_mode & 8;
  const int smode = store_mode & 3;
  // optional store: one uniform branch outside the element loops
  if (smode == 1) {
#pragma unroll
    for (int e = 0; e < P::E; ++e) {
      const int i = out_index<P>(t, e);
      if (i < lim) put_c(c + ob + (unsigned)i, cconj(v[e]), accum);
    }
  } else if (smode == 2) {
#pragma unroll
    for (int e = 0; e < P::E; ++e) {
      const int i = out_index<P>(t, e);
      if (i < lim) put_c(c + (nout - 1 - ob) - i, v[e], accum);
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
// Half-frame correlator (variant bit 6): the same overlap-save correlation with
// M = 2 * P::N points, but the M-point transforms are split by one radix-2
// step held in registers, so LDS only ever holds one P::N-point half:
//   forward (DIF):  a[j] = x[j] + x[j+H],  d[j] = (x[j] - x[j+H]) W_M^j,
//                   X[2k] = FFT_H(a)[k],   X[2k+1] = FFT_H(d)[k]       (H = M/2)
//   inverse (DIT):  r[n] = E[n] + W_M^n O[n],  r[n+H] = E[n] - W_M^n O[n],
//                   E / O = FFT_H of the even / odd bins of conj(X) Ps.
// Every thread keeps the whole frame in VGPRs (2 * P::E values), the LDS
// exchange buffer is 69 KB at M = 16384, so two blocks share a CU and one
// block's loads / barriers / LDS exchanges overlap the other's butterflies
// (the one-block-per-CU M = 16384 kernel exposes all of them).
// With P palindromic, in_index == out_index = t + (e / R0) TF + (e % R0) N / R0,
// so W_M^j = W_M^t * W_64^K(e): one per-thread twiddle (table wt) and a
// compile-time 64th root per element.
// ---------------------------------------------------------------------------
template <class P, int M>
constexpr int half_root(int e) {
  return ((e / P::R[0]) * P::TF + (e % P::R[0]) * (P::N / P::R[0])) / (M / 64);
}

template <class P>
__device__ __forceinline__ void load_halves(float2* a, float2* d, const float2* __restrict__ x,
                                            long long s0, long long n, int t) {
  constexpr int H = P::N;
  const float2* base = x + s0;
  if (s0 >= 0 && s0 + 2 * H <= n) {
#pragma unroll
    for (int e = 0; e < P::E; ++e) {
      const unsigned i = (unsigned)in_index<P>(t, e);
      a[e] = base[i];
      d[e] = base[i + H];
    }
  } else {
#pragma unroll
    for (int e = 0; e < P::E; ++e) {
      const int i = in_index<P>(t, e);
      const long long x0 = s0 + i, x1 = x0 + H;
      a[e] = (x0 >= 0 && x0 < n) ? base[i] : make_float2(0.f, 0.f);
      d[e] = (x1 >= 0 && x1 < n) ? base[i + H] : make_float2(0.f, 0.f);
    }
  }
}

// Epilogue of a half-frame block: a holds outputs i = out_index(t, e), d holds
// i + H; a thread's indices rise through a then d (first-maximum rule as in
// xcorr_epilogue).
template <class P>
__device__ __forceinline__ void xcorr_half_epilogue(const float2* a, const float2* d, long long b,
                                                    long long hop, long long nout,
                                                    float2* __restrict__ c, int store_mode,
                                                    PeakPartial* partials, int t) {
  constexpr int H = P::N;
  const long long ob = b * hop;
  const long long rem = nout - ob;
  const int lim = rem < hop ? (int)rem : (int)hop;
  const bool rev = store_mode & 4;
  const bool accum = store_mode & 8;
  const int smode = store_mode & 3;
  if (smode == 1) {
#pragma unroll
    for (int e = 0; e < P::E; ++e) {
      const int i = out_index<P>(t, e);
      if (i < lim) put_c(c + ob + (unsigned)i, cconj(a[e]), accum);
      if (i + H < lim) put_c(c + ob + (unsigned)(i + H), cconj(d[e]), accum);
    }
  } else if (smode == 2) {
#pragma unroll
    for (int e = 0; e < P::E; ++e) {
      const int i = out_index<P>(t, e);
      if (i < lim) put_c(c + (nout - 1 - ob) - i, a[e], accum);
      if (i + H < lim) put_c(c + (nout - 1 - ob) - (i + H), d[e], accum);
    }
  }
  if (!partials) return;
  float m = -1.f, s1 = 0.f, s2 = 0.f;
  int mi = 0;
  auto acc = [&](float2 v, int i) {
    const bool ok = i < lim;
    const float a2r = v.x * v.x + v.y * v.y;
    const float a2 = ok ? a2r : -1.f;
    const bool take = (a2 > m) | (rev & (a2 == m) & ok);
    m = take ? a2 : m;
    mi = take ? i : mi;
    s1 += ok ? __builtin_amdgcn_sqrtf(a2r) : 0.f;
    s2 += ok ? a2r : 0.f;
  };
  if (!rev && lim > H) {
    // every index of the a half is valid (< H < lim): no masks, strict '>'
#pragma unroll
    for (int e = 0; e < P::E; ++e) {
      const float a2 = a[e].x * a[e].x + a[e].y * a[e].y;
      const bool take = a2 > m;
      m = take ? a2 : m;
      mi = take ? out_index<P>(t, e) : mi;
      s1 += __builtin_amdgcn_sqrtf(a2);
      s2 += a2;
    }
  } else {
#pragma unroll
    for (int e = 0; e < P::E; ++e) acc(a[e], out_index<P>(t, e));
  }
#pragma unroll
  for (int e = 0; e < P::E; ++e) acc(d[e], out_index<P>(t, e) + H);
  wave_partial_f(m, mi, s1, s2, rev, ob, nout, partials + b * (P::TF / 64) + (t >> 6));
}

// TW: twiddle source of the passes: 0 the global per-pass table, 1 the
// two-level LDS table, 2 per-thread register anchors (no loads inside the
// transforms; see TwAnchors in fft_engine.hpp).  PAIR: the two halves go
// through fft_pair (LDS stores of one half overlap the other's butterflies)
// instead of two back-to-back fft_frame calls.
template <class P, int TW, int PAIR>
__global__ __launch_bounds__(P::TF, 2) void xcorr_half_kernel(
    const float2* __restrict__ s, long long n, const float4* __restrict__ Ps2, long long off,
    long long nout, long long hop, float2* __restrict__ c, int store_mode,
    PeakPartial* __restrict__ partials, long long nblocks, const float2* __restrict__ tw,
    const float2* __restrict__ wt) {
  static_assert(P::R[0] == P::RL, "overlap-save needs a palindromic plan");
  constexpr int M = 2 * P::N;
  static_assert(P::TF % (M / 64) == 0 && (P::N / P::R[0]) % (M / 64) == 0,
                "per-element split twiddles must be 64th roots of unity");
  __shared__ float2 lds[P::LDS + (TW == 1 ? tw2_size<P>() : 0)];
  const int t = threadIdx.x;
  const long long b = xcd_remap(stage_bid<4>(), gridDim.x);
  if (b >= nblocks) return;
  float2* t2 = lds + P::LDS;
  if constexpr (TW == 1) load_tw2<P>(t2, tw, t, P::TF);
  float2 wa[TW == 2 ? nanch_total<P>() : 1];
  if constexpr (TW == 2) load_anchors<P>(wa, tw, t);
  auto fft = [&](float2* v) {
    if constexpr (TW == 1) fft_frame_t2<P>(v, lds, t2 + opaque_zero(), t);
    else if constexpr (TW == 2) fft_frame_anch<P>(v, lds, wa, t);
    else fft_frame<P>(v, lds, tw, t);
  };
  auto fft2 = [&](float2* x, float2* y) {
    if constexpr (PAIR) {
      if constexpr (TW == 1) fft_pair<P>(x, y, lds, TwLds{t2 + opaque_zero()}, t);
      else if constexpr (TW == 2) { launder_anchors<P>(wa); fft_pair<P>(x, y, lds, TwAnchors{wa}, t); }
      else fft_pair<P>(x, y, lds, TwTable{tw + opaque_zero()}, t);
    } else {
      fft(x);
      fft(y);
    }
  };
  float2 a[P::E], d[P::E];
#ifdef VSIG_EXP_NO_LOAD      // timing experiments only (results are wrong)
#pragma unroll
  for (int e = 0; e < P::E; ++e) { a[e] = make_float2((float)(t + e), (float)(b & 7)); d[e] = make_float2((float)e, 1.f); }
#else
  load_halves<P>(a, d, s, b * hop - off, n, t);
#endif
  const float2 w = wt[t];
  static_for<0, P::E>([&](auto ei) {
    constexpr int e = decltype(ei)::value;
    const float2 x0 = a[e], x1 = d[e];
    a[e] = cadd(x0, x1);
    d[e] = twc<half_root<P, M>(e), 64>(cmul(csub(x0, x1), w));
  });
  fft2(a, d);
#pragma unroll
  for (int e = 0; e < P::E; ++e) {
#ifdef VSIG_EXP_NO_PS
    const float4 p = make_float4(0.5f, 0.25f, 0.125f, 0.5f);
#else
    const float4 p = Ps2[out_index<P>(t, e)];
#endif
    a[e] = cmul(cconj(a[e]), make_float2(p.x, p.y));
    d[e] = cmul(cconj(d[e]), make_float2(p.z, p.w));
  }
  fft2(a, d);
  static_for<0, P::E>([&](auto ei) {
    constexpr int e = decltype(ei)::value;
    const float2 o = twc<half_root<P, M>(e), 64>(cmul(d[e], w));
    const float2 ev = a[e];
    a[e] = cadd(ev, o);
    d[e] = csub(ev, o);
  });
#ifdef VSIG_EXP_NO_EPI
  float acc = 0.f;
#pragma unroll
  for (int e = 0; e < P::E; ++e) acc += a[e].x + a[e].y + d[e].x + d[e].y;
  if (acc == 12345.f) partials[b].sum_abs = acc;
#else
  xcorr_half_epilogue<P>(a, d, b, hop, nout, c, store_mode, partials, t);
#endif
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
__global__ __launch_bounds__(os_threads<P>(), 2) void xcorr_part_kernel(
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
                           PeakPartial* partials, const float2* tw, const float2* wt, int variant,
                           hipStream_t st) {
  if (nout <= 0) return hipSuccess;
  const long long nblocks = (nout + hop - 1) / hop;
  if ((variant & 64) && M == 16384) {   // half-frame kernel, two blocks per CU
    auto k = (variant & 128)
                 ? ((variant & 8)   ? xcorr_half_kernel<Plan8192, 1, 1>
                    : (variant & 1) ? xcorr_half_kernel<Plan8192, 2, 1>
                                    : xcorr_half_kernel<Plan8192, 0, 1>)
                 : ((variant & 8)   ? xcorr_half_kernel<Plan8192, 1, 0>
                    : (variant & 1) ? xcorr_half_kernel<Plan8192, 2, 0>
                                    : xcorr_half_kernel<Plan8192, 0, 0>);
    hipLaunchKernelGGL(k, dim3((unsigned)nblocks), dim3(Plan8192::TF), 0, st, s, n,
                       reinterpret_cast<const float4*>(Ps), off, nout, hop, c, store_mode,
                       partials, nblocks, tw, wt);
    return hipGetLastError();
  }
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

int os_waves(int M, int variant) {
  switch (M) {
    case 1024: return os_threads<Plan1024s>() / 64;
    case 2048: return os_threads<Plan2048s>() / 64;
    case 4096: return os_threads<Plan4096>() / 64;
    case 8192: return os_threads<Plan8192>() / 64;
    case 16384:
      if (variant & 64) return Plan8192::TF / 64;
      return (variant & 2) ? os_threads<Plan16384w>() / 64 : os_threads<Plan16384>() / 64;
    default: return 0;
  }
}

}  // namespace vsig
