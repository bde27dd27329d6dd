// Cross-correlation kernels (gfx950): overlap-save correlation with the fused
// |c|^2 argmax / sums epilogue (correlate, find_correlation_peak).
//   M = 16384 (templates of 2049 .. 8192 samples): xcorr_half_kernel, two
//     8192-point halves through LDS, two blocks per CU;
//   M = 32768 (8193 .. 16384): the same with 16384-point halves;
//   M = 4096 / 8192 (templates up to 1024 / 2048): xcorr_os_kernel, one frame
//     per block, persistent with the next segment prefetched.
// Both use register twiddle anchors (no global loads inside a transform).
#include "os_common.hpp"

namespace vsig {

// ---------------------------------------------------------------------------
// c[o] = sum_{k<L} s[o - off + k] * conj(p[k]), o in [0, nout).  off = 0 ->
// np.correlate 'valid'; off = L-1 -> 'full'.  Block b: outputs
// [b*hop, b*hop + hop), hop <= M - L + 1.
// store_mode: bits 0-1: 1 store c, 2 store conj(c) at nout-1-o (np.correlate's
// swapped argument order); bit 2 (4): argmax in the reversed index space;
// bit 3 (8): add to c instead of storing (templates longer than 8192 run as a
// sum of template chunks).
// Partials: one per wave.  Wave w of block b covers the outputs
//   b*hop + 64 w + l + TF q,   l < 64, q < Q   (Q = E, or 2 E for the half
// kernel), which refine.hip uses to revisit a wave's outputs (xcorr_geom).
// ---------------------------------------------------------------------------
__device__ __forceinline__ void put_c(float2* p, float2 v, bool accum) {
  *p = accum ? cadd(*p, v) : v;
}

template <class P>
__device__ __forceinline__ void xcorr_epilogue(const float2* v, long long b, long long hop,
                                               long long nout, float2* __restrict__ c,
                                               int store_mode, PeakPartial* partials, int t) {
  const long long ob = b * hop;                         // block's first output
  const long long rem = nout - ob;
  const int lim = rem < hop ? (int)rem : (int)hop;
  const bool rev = store_mode & 4;
  const bool accum = store_mode & 8;
  const int smode = store_mode & 3;
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
  wave_partial_f(m, mi, s1, s2, rev, ob, nout, partials + b * (P::TF / 64) + (t >> 6));
}

// Persistent: a block walks blocks b, b + grid, ...; the next segment is
// loaded behind the (L2-resident) template-spectrum loads, so it lands while
// the inverse FFT runs (vmcnt retires in issue order).
template <class P>
__global__ __launch_bounds__(P::TF) void xcorr_os_kernel(
    const float2* __restrict__ s, long long n, const float2* __restrict__ Ps, long long off,
    long long nout, long long hop, float2* __restrict__ c, int store_mode,
    PeakPartial* __restrict__ partials, long long nblocks, const float2* __restrict__ tw) {
  static_assert(P::R[0] == P::RL, "overlap-save needs a palindromic plan");
  __shared__ __attribute__((aligned(16))) float2 lds[lds_size<P>()];
  const int t = threadIdx.x;
  long long b = blockIdx.x;
  if (b >= nblocks) return;
  float2 wa[nanch_total<P>()];
  load_anchors<P>(wa, tw, t);
  float2 v[P::E];
  load_segment<P>(v, s, b * hop - off, n, t);
  for (; b < nblocks; b += gridDim.x) {
    fft_frame_anch<P>(v, lds, wa, t);
#pragma unroll
    for (int e = 0; e < P::E; ++e) v[e] = cmul(cconj(v[e]), Ps[out_index<P>(t, e)]);
    float2 nv[P::E];
    const long long nb = b + gridDim.x;
    if (nb < nblocks) load_segment<P>(nv, s, nb * hop - off, n, t);
    fft_frame_anch<P>(v, lds, wa, t);
    xcorr_epilogue<P>(v, b, hop, nout, c, store_mode, partials, t);
#pragma unroll
    for (int e = 0; e < P::E; ++e) v[e] = nv[e];
  }
}

// ---------------------------------------------------------------------------
// Half-frame correlator: the same overlap-save correlation with M = 2 * P::N
// points, the M-point transforms split by one radix-2 step held in registers,
// so LDS only ever holds one P::N-point half:
//   forward (DIF):  a[j] = x[j] + x[j+H],  d[j] = (x[j] - x[j+H]) W_M^j,
//                   X[2k] = FFT_H(a)[k],   X[2k+1] = FFT_H(d)[k]       (H = M/2)
//   inverse (DIT):  r[n] = E[n] + W_M^n O[n],  r[n+H] = E[n] - W_M^n O[n],
//                   E / O = FFT_H of the even / odd bins of conj(X) Ps.
// Every thread keeps the whole frame in VGPRs (2 * P::E values); the LDS
// exchange buffer is 69 KB at M = 16384, so two blocks share a CU and one
// block's loads / barriers / LDS exchanges overlap the other's butterflies.
// The two halves go through fft_pair (LDS stores of one half overlap the
// other's butterflies), twiddles from register anchors.
// With P palindromic, in_index == out_index, and W_M^j = W_M^base * W_64^K(e)
// (half_root): one per-thread twiddle from the table wt and a compile-time
// 64th root per element.
// ---------------------------------------------------------------------------
// The M = 32768 correlator (templates of 8193 .. 16384 samples in one pass):
// 16384-point halves, 512 threads x 32 values, 3 passes, one block per CU.
// Measured on templates of 4096: 1.89 ms per 2^28 samples against 1.42 ms for
// the M = 16384 kernel (round 2, r02_v6 A/B), and again on round 6's kernels
// 2.65-2.68 against 2.24-2.25 ms at config 5 (profiles/r06_xcorr_plan_ab.txt:
// one 512-thread block per CU has no second block to run while its waves meet
// at the exchange barriers), so shorter templates keep M = 16384.
using PlanX32k = Plan16384w;
// The 32 / 8 / 32 identity-map plan (Plan8192c, fft_engine.hpp); round 6:
// 2.24-2.25 ms at config 5 against 2.27-2.28 for round 5's 16 / 32 / 16 sigma
// map (profiles/r06_xcorr_plan_ab.txt).  Measured against the sigma map
// (rounds 2-3): the interleaved map (16-byte loads, two split twiddles per
// thread) 2.67 vs 2.58 ms at config 5 (profiles/r02_v19_ab.txt); the
// 512-thread, 16-value plan (4 waves per SIMD, a third exchange per half)
// 2.67 vs 2.48 ms (r03_v11), +11 % in round 5.
using PlanX16k = Plan8192c;
constexpr int kPlanKey16k = -8192;      // its twiddle table (plan_info)

// in_index(t, e) = base(t) + off(e): the split twiddle
// W_M^in_index = W_M^base * W_64^half_root(e).
template <class P, int M>
constexpr int half_root(int e) {
  return ((e / P::R[0]) * P::TF + (e % P::R[0]) * (P::N / P::R[0])) / (M / 64);
}

template <class P>
__device__ __forceinline__ void load_halves(float2* a, float2* d, const float2* __restrict__ x,
                                            long long s0, long long n, int t) {
  constexpr int H = P::N;
  const float2* base = x + s0;
  if (s0 >= 0 && s0 + 2 * H <= n) {     // one voffset per thread, the rest in soffset
    const auto rs = make_rsrc(base, 2u * H * (unsigned)sizeof(float2));
    const unsigned v0 = (unsigned)in_index<P>(t, 0) * (unsigned)sizeof(float2);
    static_for<0, P::E>([&](auto ei) {
      constexpr int e = decltype(ei)::value;
      a[e] = buf_load2(rs, v0, in_off<P>(e) * (int)sizeof(float2));
      d[e] = buf_load2(rs, v0, (in_off<P>(e) + H) * (int)sizeof(float2));
    });
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

// A thread's outputs out_index(t, e) = m(t) + c_e (+ H for the second half)
// are evenly spaced: c_e = kStep * rank(e), rank a permutation of [0, E), and
// H = kStep * E, so rank and index convert by one multiply (plain / sigma
// maps; the interleaved map's c_e = b + (N/R) r are not).
template <class P>
struct KeyedRank {
  static constexpr int c(int e) { return (e / P::RL) * P::TF + (e % P::RL) * (P::N / P::RL); }
  static constexpr int rank(int e) {
    int r = 0;
    for (int q = 0; q < P::E; ++q) r += c(q) < c(e);
    return r;
  }
  static constexpr int kStep = P::TF < P::N / P::RL ? P::TF : P::N / P::RL;
  static constexpr bool check() {
    if (mapl_of<P>::value == kMapIlv || 2 * P::E > 64 || P::N != kStep * P::E) return false;
    for (int e = 0; e < P::E; ++e)
      if (c(e) != kStep * rank(e)) return false;
    return true;
  }
  static constexpr bool ok = check();
};

// Epilogue of a half-frame block: a holds outputs i = out_index(t, e), d holds
// i + H; a thread's indices rise through a then d (first-maximum rule as in
// xcorr_epilogue).
// DV >= 0: the launch's interior blocks (lim == hop) keep exactly the d ranks
// below DV (hop - H = DV kStep), a compile-time split: straight-line code with
// no per-element branch or mask for them (the runtime split's uniform branches
// cost ~6 % of the kernel, profiles/r03_v19_*); other blocks, and DV < 0,
// take the runtime split.
template <class P, int DV = -1>
__device__ __forceinline__ void xcorr_half_epilogue(const float2* a, const float2* d, long long b,
                                                    long long hop, long long nout,
                                                    float2* __restrict__ c, int store_mode,
                                                    PeakPartial* partials, unsigned* lkeys, int t) {
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
  if constexpr (KeyedRank<P>::ok) {
    // Per-thread argmax by key: the bits of |c|^2 (>= 0, so they order as the
    // floats) with the low 6 mantissa bits replaced by the output's rank in
    // the thread (rev: reversed), one v_and_or + one max per output instead of
    // a compare and two selects.  Ties among values equal to 2^-17 relative go
    // to the lowest index (rev: the highest) -- numpy's first-max rule in the
    // (reversed) output space; the partial's max is that truncated |c|^2
    // (<= 2^-17 low).  The refine band (1e-3) and its exact fp64 re-rank are
    // unaffected; with refine off the peak is the fp32 result within 8e-6.
    using KR = KeyedRank<P>;
    // rev as a compile-time flag (the uniform branch below): each key is then
    // one v_and_or with the rank (^ 63) as an inline constant
    auto keyed = [&](auto revc) {
    constexpr bool kRev = decltype(revc)::value;
    constexpr unsigned rx = kRev ? 0u : 63u;
    unsigned key = 0u;
    bool any = false;
    float s1 = 0.f, s2 = 0.f;
    auto acc = [&](float2 v, int i, int rank, auto masked) {
      const float a2 = v.x * v.x + v.y * v.y;
      const unsigned k = (__float_as_uint(a2) & ~63u) | ((unsigned)rank ^ rx);
      if constexpr (decltype(masked)::value) {
        const bool ok = i < lim;
        key = ok ? (k > key ? k : key) : key;
        any |= ok;
        s1 += ok ? __builtin_amdgcn_sqrtf(a2) : 0.f;
        s2 += ok ? a2 : 0.f;
      } else {
        key = k > key ? k : key;
        any = true;
        s1 += __builtin_amdgcn_sqrtf(a2);
        s2 += a2;
      }
    };
    if (DV >= 0 && lim == hop) {       // interior block, compile-time split
      static_for<0, P::E>([&](auto ei) {
        constexpr int e = decltype(ei)::value;
        acc(a[e], 0, KR::rank(e), IC<0>{});
        if constexpr (KR::rank(e) < DV) acc(d[e], 0, KR::rank(e) + P::E, IC<0>{});
      });
    } else {
    if (lim > H) {                     // every index of the a half is valid
      static_for<0, P::E>([&](auto ei) {
        constexpr int e = decltype(ei)::value;
        acc(a[e], 0, KR::rank(e), IC<0>{});
      });
    } else {
      static_for<0, P::E>([&](auto ei) {
        constexpr int e = decltype(ei)::value;
        acc(a[e], out_index<P>(t, e), KR::rank(e), IC<1>{});
      });
    }
    // the second half's outputs i + H, i = m(t) + kStep rank(e), m(t) < kStep:
    // an element is valid on every lane when kStep (rank + 1) <= lim - H and
    // on none when kStep rank >= lim - H -- wave-uniform branches, so only the
    // one straddling element of a block needs the per-lane mask (an interior
    // block at L = 4096: the 16 lower ranks whole, the upper 16 skipped)
    const int cut = lim - H;
    static_for<0, P::E>([&](auto ei) {
      constexpr int e = decltype(ei)::value;
      constexpr int c0 = KR::kStep * KR::rank(e);
      if constexpr (KR::kStep == P::TF) {      // m(t) < TF = kStep
        if (c0 + KR::kStep <= cut) acc(d[e], 0, KR::rank(e) + P::E, IC<0>{});
        else if (c0 < cut) acc(d[e], out_index<P>(t, e) + H, KR::rank(e) + P::E, IC<1>{});
      } else {
        acc(d[e], out_index<P>(t, e) + H, KR::rank(e) + P::E, IC<1>{});
      }
    });
    }
    // lane keys (refine candidates per thread column, see xcorr_lane_keys)
    if (lkeys) lkeys[b * P::TF + tmapl<P>(t)] = key;
    const int rank = (int)((key & 63u) ^ rx);
    const int mi = tmapl<P>(t) + KR::kStep * rank;
    const float m = any ? __uint_as_float(key & ~63u) : -1.f;
    wave_partial_f(m, mi, s1, s2, kRev, ob, nout, partials + b * (P::TF / 64) + (t >> 6));
    };
    if (rev) keyed(IC<1>{});
    else keyed(IC<0>{});
    return;
  }
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

// waves per SIMD: 16-value plans (Plan8192w) two 512-thread blocks per CU =
// 4; 32-value plans two 256-thread blocks (2) or one 512-thread block (1)
template <class P>
constexpr int xcorr_waves_per_eu() { return P::E <= 16 ? 4 : P::TF >= 512 ? 1 : 2; }

// The segment prefetch distance: one 4-byte load per 128-byte line of the
// segment kSegPfDist blocks ahead -- about the block that takes this slot of
// the XCD next (xcd_remap hands each XCD a contiguous run, two blocks per CU x
// 32 CUs in flight) -- so that its loads find the lines in L2 instead of HBM.
// Issued just before the epilogue and consumed only at the end of the block,
// so nothing waits for it.  Earlier issue loses: right after the segment loads
// the 63-deep vmcnt makes the split step wait for the prefetch too (+14 %);
// after the spectrum product the lines live long enough in the 4 MB L2 to be
// evicted again (+45 % L2 fills).  Distances 32 / 96 / 128 / 192 / 256 are
// slower or equal.  profiles/r03_v22_xcorr_segpf_ab.txt: -5 % correlator
// time, +2.5 % reads.  Re-measured on round 6's 32 / 8 / 32 plan
// (profiles/r06_xcorr_plan_ab.txt): 64 still best; 96 / 128 +1.7 / +2 %,
// 48 +5 %, a prefetch of the block's own segment (no look-ahead) +6.7 %.
constexpr int kSegPfDist = 64;

template <class P, int DV = -1>
__global__ __launch_bounds__(P::TF, xcorr_waves_per_eu<P>()) void xcorr_half_kernel(
    const float2* __restrict__ s, long long n, const float4* __restrict__ Ps2, long long off,
    long long nout, long long hop, float2* __restrict__ c, int store_mode,
    PeakPartial* __restrict__ partials, long long nblocks, const float2* __restrict__ tw,
    const float2* __restrict__ wt, unsigned* __restrict__ lkeys, unsigned long long* clk) {
  static_assert(P::R[0] == P::RL, "overlap-save needs a palindromic plan");
  static_assert(map0_of<P>::value != kMapIlv, "one split twiddle per thread");
  constexpr int M = 2 * P::N;
  static_assert(P::TF % (M / 64) == 0 && (P::N / P::R[0]) % (M / 64) == 0,
                "per-element split twiddles must be 64th roots of unity");
  __shared__ __attribute__((aligned(16))) float2 lds[lds_size<P>()];
  const int t = threadIdx.x;
  const ClockStamp cs(clk, blockIdx.x);
  float2 wa[nanch_total<P>()];
  load_anchors<P>(wa, tw, t);
  // the radix-8 middle pass (one k per thread) from 7 exact twiddles in VGPRs
  // instead of 6 generated powers per transform (TwAnchorsX): -0.5 % at
  // config 5, profiles/r06_conj_std_ab.txt
  float2 wx[twx_total<P>()];
  load_twx<P>(wx, tw, t);
  const long long b = xcd_remap(blockIdx.x, gridDim.x);
  if (b >= nblocks) return;
  auto fft2 = [&](float2* x, float2* y) {
    launder_anchors<P>(wa);
    fft_pair<P>(x, y, lds, TwAnchorsX{wa, wx}, t);
  };
  // W_M^base: base = in_index(t, 0), loaded ahead of the segment and the
  // prefetch below (loads complete in issue order)
  const float2 w = wt[in_index<P>(t, 0)];
  float2 a[P::E], d[P::E];
  load_halves<P>(a, d, s, b * hop - off, n, t);
  constexpr int kPfLines = 2 * P::N * 8 / 128 / P::TF;          // 128-byte lines per thread
  float pfv[kPfLines];
#pragma unroll
  for (int k = 0; k < kPfLines; ++k) pfv[k] = 0.f;
  static_for<0, P::E>([&](auto ei) {
    constexpr int e = decltype(ei)::value;
    const float2 x0 = a[e], x1 = d[e];
    a[e] = cadd(x0, x1);
    d[e] = twc<half_root<P, M>(e), 64>(cmul(csub(x0, x1), w));
  });
  fft2(a, d);
  {
    const auto rp = make_rsrc(Ps2, (unsigned)P::N * (unsigned)sizeof(float4));
    const unsigned v0 = (unsigned)out_index<P>(t, 0) * (unsigned)sizeof(float4);
    static_for<0, P::E>([&](auto ei) {
      constexpr int e = decltype(ei)::value;
      const float4 p = buf_load4(rp, v0, out_off<P>(e) * (int)sizeof(float4));
      // (conj folded into the product's neg modifiers: fewer instructions,
      // but +4 % at config 5 in both its forms, profiles/r06_conj_std_ab.txt)
      a[e] = cmul(cconj(a[e]), make_float2(p.x, p.y));
      d[e] = cmul(cconj(d[e]), make_float2(p.z, p.w));
    });
  }
  fft2(a, d);
  static_for<0, P::E>([&](auto ei) {
    constexpr int e = decltype(ei)::value;
    const float2 o = twc<half_root<P, M>(e), 64>(cmul(d[e], w));
    const float2 ev = a[e];
    a[e] = cadd(ev, o);
    d[e] = csub(ev, o);
  });
  {                                          // the segment prefetch (kSegPfDist)
    const long long bn = b + kSegPfDist;
    const long long s0 = bn * hop - off;
    if (bn < nblocks && s0 >= 0 && s0 + 2 * P::N <= n) {
      const float* q = reinterpret_cast<const float*>(s + s0);
#pragma unroll
      for (int k = 0; k < kPfLines; ++k) pfv[k] = q[(t + k * P::TF) * 32];
    }
  }
  xcorr_half_epilogue<P, DV>(a, d, b, hop, nout, c, store_mode, partials, lkeys, t);
#pragma unroll
  for (int k = 0; k < kPfLines; ++k)   // the prefetch loads stay; their values are never used
    asm volatile("" ::"v"(pfv[k]));
  cs.done(clk);
}

hipError_t launch_xcorr_os(int M, const float2* s, long long n, const float2* Ps, long long off,
                           long long nout, long long hop, float2* c, int store_mode,
                           PeakPartial* partials, const float2* tw, const float2* wt,
                           hipStream_t st, unsigned* lkeys) {
  if (nout <= 0) return hipSuccess;
  if (lkeys && !xcorr_lane_keys(M)) return hipErrorInvalidValue;
  const long long nblocks = (nout + hop - 1) / hop;
  if (M == 16384) {
    // interior blocks keep the second half's ranks below (hop - H) / kStep: the
    // common split (hop = 12288: L = 4096, 4097) has its compile-time epilogue
    using KR = KeyedRank<PlanX16k>;
    constexpr int kDv = PlanX16k::E / 2;
    const long long cut = hop - PlanX16k::N;
    const bool dv = KR::ok && KR::kStep == PlanX16k::TF && cut == (long long)kDv * KR::kStep;
    if (dv) {
      hipLaunchKernelGGL((xcorr_half_kernel<PlanX16k, kDv>), dim3((unsigned)nblocks),
                         dim3(PlanX16k::TF), 0, st, s, n, reinterpret_cast<const float4*>(Ps), off, nout,
                         hop, c, store_mode, partials, nblocks, tw, wt, lkeys, g_clock_sink);
      return hipGetLastError();
    }
    hipLaunchKernelGGL(xcorr_half_kernel<PlanX16k>, dim3((unsigned)nblocks), dim3(PlanX16k::TF), 0,
                       st, s, n, reinterpret_cast<const float4*>(Ps), off, nout, hop, c, store_mode,
                       partials, nblocks, tw, wt, lkeys, g_clock_sink);
    return hipGetLastError();
  }
  if (M == 32768) {     // 16384-point halves, one block per CU
    hipLaunchKernelGGL(xcorr_half_kernel<PlanX32k>, dim3((unsigned)nblocks), dim3(PlanX32k::TF), 0,
                       st, s, n, reinterpret_cast<const float4*>(Ps), off, nout, hop, c, store_mode,
                       partials, nblocks, tw, wt, lkeys, g_clock_sink);
    return hipGetLastError();
  }
  auto run = [&](auto plan) {
    using PL = decltype(plan);
    auto k = xcorr_os_kernel<PL>;
    const long long grid = persistent_grid(k, PL::TF, nblocks);
    hipLaunchKernelGGL(k, dim3((unsigned)grid), dim3(PL::TF), 0, st, s, n, Ps, off, nout, hop, c,
                       store_mode, partials, nblocks, tw);
  };
  if (M == 4096) run(Plan4096{});
  else if (M == 8192) run(Plan8192{});
  else return hipErrorInvalidValue;
  return hipGetLastError();
}

// Rows per thread column when the correlator for M writes lane keys (the
// keyed epilogue: thread t of block b stores its max key at b TF + m(t),
// m(t) = its last-pass butterfly base, which is column m(t) mod 64 of wave
// m(t) / 64 in xcorr_geom's terms), else 0.
// The column's outputs m(t) + kStep R (R < 2E) are xcorr_geom's rows q = R
// when kStep is the row stride TF.
template <class P>
constexpr int lane_key_rows() {
  return KeyedRank<P>::ok && KeyedRank<P>::kStep == P::TF && 2 * P::E <= 64 ? 2 * P::E : 0;
}
int xcorr_lane_keys(int M) {
  if (M == 16384) return lane_key_rows<PlanX16k>();
  if (M == 32768) return lane_key_rows<PlanX32k>();
  return 0;
}

// Wave geometry of the correlator's partials (see the header comment):
// waves per block, rows Q and their stride; twiddle plan size.
hipError_t xcorr_geom(int M, int* waves, int* Q, int* stride, int* plan, int* wstep, int* rsub) {
  *wstep = 64;
  *rsub = 1;
  if (M == 32768) { *waves = PlanX32k::TF / 64; *Q = 2 * PlanX32k::E; *stride = PlanX32k::TF; *plan = -16384; }
  else if (M == 16384) {
    *waves = PlanX16k::TF / 64; *Q = 2 * PlanX16k::E; *stride = PlanX16k::TF; *plan = kPlanKey16k;
  }
  else if (M == 8192) { *waves = Plan8192::TF / 64; *Q = Plan8192::E; *stride = Plan8192::TF; *plan = 8192; }
  else if (M == 4096) { *waves = Plan4096::TF / 64; *Q = Plan4096::E; *stride = Plan4096::TF; *plan = 4096; }
  else return hipErrorInvalidValue;
  return hipSuccess;
}

}  // namespace vsig
