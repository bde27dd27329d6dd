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
      if (i >= 0 && i < lim) st_stream(yb + (unsigned)i, conj1(v[e]));
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
      if (i >= 0 && i < lim && (unsigned)i == q * (unsigned)decim) st_stream(yb + q, conj1(v[e]));
    }
  }
}

// The same for decim = 1 with the pair lane map (out_index(t, e) = m(t) + 64 e)
// by 16-byte stores: the inverse of load_segment_x4's swap gives lane l the
// outputs 2l + 128 i and 2l + 1 + 128 i.  Needs lo even and y + b hop 16-byte
// aligned (launch-time choice); an odd tail (lim odd) stores its last single.
template <class P>
__device__ __forceinline__ void fir_store_x4(const float2* v, float2* __restrict__ y, long long b,
                                             long long hop, int lo, long long nloc, int t) {
  static_assert(mapl_of<P>::value == kMapPair && P::TF == 64 && P::E == 16 && P::RL == 16,
                "result layout m(t) + 64 e");
  typedef float f4 __attribute__((ext_vector_type(4)));
  const long long gb = b * hop;
  const long long rem = nloc - gb;
  const int lim = rem < hop ? (int)rem : (int)hop;
  float2* yb = y + gb;
#pragma unroll
  for (int i = 0; i < P::E / 2; ++i) {
    const float2 p = conj1(v[2 * i]), q = conj1(v[2 * i + 1]);
    const auto rx = __builtin_amdgcn_permlane32_swap(__float_as_uint(p.x), __float_as_uint(q.x), false, false);
    const auto ry = __builtin_amdgcn_permlane32_swap(__float_as_uint(p.y), __float_as_uint(q.y), false, false);
    const int io = 2 * t + 128 * i - lo;               // even: lo is
    const f4 w = {__uint_as_float(rx[0]), __uint_as_float(ry[0]), __uint_as_float(rx[1]),
                  __uint_as_float(ry[1])};
    if (io >= 0 && io + 1 < lim) {
      __builtin_nontemporal_store(w, reinterpret_cast<f4*>(yb + io));
    } else if (io >= 0 && io < lim) {
      st_stream(yb + io, make_float2(w.x, w.y));
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
// Two consecutive blocks per workgroup (fft_pair: the LDS stores of one
// segment overlap the other's butterflies), twiddles from register anchors.
// MIX: the NCO mixer applied to every loaded sample (vsig_fir_exec_mix_dev).
// lo: the segment's offset before its block's first output (>= ntaps - 1, and
// lo + hop <= M): outputs are the circular indices [lo, lo + hop).
template <class P, bool MIX = false, bool X4 = false, bool XS = false>
__global__ __launch_bounds__(P::TF) void fir_os_kernel(
    const float2* __restrict__ x, long long n, long long g0, const float2* __restrict__ Hs,
    int lo, long long hop, int decim, float2* __restrict__ y, long long nblocks,
    const float2* __restrict__ tw, MixArgs mix, unsigned long long* clk) {
  static_assert(P::R[0] == P::RL, "overlap-save needs a palindromic plan");
  __shared__ float2 lds[lds_size<P>()];
  const int t = threadIdx.x;
  const ClockStamp cs(clk, blockIdx.x);
  const long long b = xcd_remap(blockIdx.x, gridDim.x);
  if (2 * b >= nblocks) return;  // uniform per block
  const long long nloc = n - g0;
  float2 wa[nanch_total<P>()];
  load_anchors<P>(wa, tw, t);
  const long long b0 = 2 * b, b1 = 2 * b + 1;
  float2 a[P::E], d[P::E];
  if constexpr (MIX) {
    load_segment_mix<P>(a, x, g0 + b0 * hop - lo, n, t, mix);
    load_segment_mix<P>(d, x, g0 + b1 * hop - lo, n, t, mix);
  } else if constexpr (X4) {
    load_pair_x4<P>(a, d, x, g0 + b0 * hop - lo, hop, n, t);
  } else {
    load_segment<P>(a, x, g0 + b0 * hop - lo, n, t);
    load_segment<P>(d, x, g0 + b1 * hop - lo, n, t);
  }
  launder_anchors<P>(wa);
  fft_pair<P>(a, d, lds, TwAnchors{wa}, t);
#pragma unroll
  for (int e = 0; e < P::E; ++e) {
    const float2 h = Hs[out_index<P>(t, e)];
    a[e] = cmul_conj(a[e], h);
    d[e] = cmul_conj(d[e], h);
  }
  launder_anchors<P>(wa);
  fft_pair<P>(a, d, lds, TwAnchors{wa}, t);
  if constexpr (XS) {
    fir_store_x4<P>(a, y, b0, hop, lo, nloc, t);
    fir_store_x4<P>(d, y, b1, hop, lo, nloc, t);
  } else {
    fir_store<P>(a, y, b0, hop, lo, nloc, decim, t);
    fir_store<P>(d, y, b1, hop, lo, nloc, decim, t);
  }
  cs.done(clk);
}

// ---------------------------------------------------------------------------
// Decimating FIR (D = 2 / 4 at M = 1024), decimation in the frequency domain: after
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
  static_assert(lds_need<PD>() <= lds_size<P>(), "exchange buffer");
  __shared__ float2 lds[lds_size<P>()];
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

// ---------------------------------------------------------------------------
// D = 4, polyphase form.  The 1024-point segment transform of fir_dec_kernel
// followed by x H and the fold by 4 equals, per decimated bin j < 256,
//   Yd[j] = sum_k U_k[j] G_k[j],   U_k = FFT_256(x[k + 4 m]),
//   G_k[j] = W_1024^{k j} sum_s W_4^{k s} Hs[j + 256 s]        (fir_poly_gtable)
// so the segment needs only the two radix-16 passes of Plan1024q (thread t
// ends with U_{t/16}[(t%16) + 16 r], r < 16): one LDS exchange and one
// twiddled pass fewer.  The sum over k = t/16 runs across the lanes t, t^16,
// t^32, t^48 as a reduce-scatter with v_permlane32_swap / v_permlane16_swap
// (no LDS): afterwards lane t holds Yd[tq + 64 i], i < 4, with tq = t with
// bits 4 and 5 exchanged -- Plan256d's operand layout for thread tq, which
// runs the inverse transform and the stores under that index.
// ---------------------------------------------------------------------------
// a + b across lane pairs (l, l ^ 32): lanes < 32 return a(l) + a(l + 32),
// lanes >= 32 return b(l - 32) + b(l).
__device__ __forceinline__ float2 swap32_add(float2 a, float2 b) {
  const auto rx = __builtin_amdgcn_permlane32_swap(__float_as_uint(a.x), __float_as_uint(b.x), false, false);
  const auto ry = __builtin_amdgcn_permlane32_swap(__float_as_uint(a.y), __float_as_uint(b.y), false, false);
  return cadd(make_float2(__uint_as_float(rx[0]), __uint_as_float(ry[0])),
              make_float2(__uint_as_float(rx[1]), __uint_as_float(ry[1])));
}
// the same across (l, l ^ 16), conjugated (the inverse transform's operand):
// lanes with bit 4 clear return conj(a(l) + a(l + 16)), the others
// conj(b(l - 16) + b(l)).
__device__ __forceinline__ float2 swap16_add_conj(float2 a, float2 b) {
  const auto rx = __builtin_amdgcn_permlane16_swap(__float_as_uint(a.x), __float_as_uint(b.x), false, false);
  const auto ry = __builtin_amdgcn_permlane16_swap(__float_as_uint(a.y), __float_as_uint(b.y), false, false);
  return cadd_conj(make_float2(__uint_as_float(rx[0]), __uint_as_float(ry[0])),
                   make_float2(__uint_as_float(rx[1]), __uint_as_float(ry[1])));
}

// A memory-only knock-out of this kernel (both transform pairs skipped,
// outputs wrong; round 2): 3.85-3.94 ms at config 5 against 4.32-4.37 ms
// for the kernel then (profiles/r02_v12_ab.txt), i.e. the loads / stores of
// this access pattern alone run at 5.5 TB/s and the transforms add ~0.45 ms.

// STD: the chain's geometry (255 taps: lo2 = 256, hop = 768), for which every
// thread's stored outputs are known at compile time -- circular indices
// i = tq + 64 e, kept for n0 = 64 <= i < n1 = 256, i.e. e = 1..3 on every lane
// -- so a pair whose outputs all lie inside the chunk stores with no
// per-element compare or exec-mask branch (the last pair keeps the tests).
constexpr int kStdLo2 = 256, kStdHop = 768;

template <bool MIX = false, bool X4 = false, bool STD = false>
__global__ __launch_bounds__(64) void fir_poly_kernel(
    const float2* __restrict__ x, long long n, long long g0, const float2* __restrict__ G, int lo2,
    long long hop, float2* __restrict__ y, long long nblocks, const float2* __restrict__ tw,
    const float2* __restrict__ twd, MixArgs mix, unsigned long long* clk) {
  using P = Plan1024q;
  using PD = Plan256d;
  constexpr int D = 4;
  static_assert(P::TF == 64 && P::E == 16 && P::NP == 2 && P::R[1] == 16 && PD::E == 4,
                "lane layout of the reduce-scatter");
  static_assert(lds_need<PD>() <= lds_size<P>(), "exchange buffer");
  __shared__ float2 lds[lds_size<P>()];
  const int t0 = threadIdx.x;
  const ClockStamp cs(clk, blockIdx.x);
  const long long nloc = n - g0;
  const int tq0 = (t0 & 15) | ((t0 & 16) << 1) | ((t0 & 32) >> 1);
  float2 wa[nanch_total<P>()];
  load_anchors<P>(wa, tw, t0);
  float2 wr[rtw_total<PD>()];
  load_rtw<PD>(wr, twd, tq0);
  const long long b = xcd_remap(blockIdx.x, gridDim.x);
  if (2 * b >= nblocks) return;
  const int t = t0, tq = tq0;
  float2 a[P::E], d[P::E];
  if constexpr (MIX) {
    load_segment_mix<P>(a, x, g0 + (2 * b) * hop - lo2, n, t, mix);
    load_segment_mix<P>(d, x, g0 + (2 * b + 1) * hop - lo2, n, t, mix);
  } else if constexpr (X4) {
    load_pair_x4<P>(a, d, x, g0 + (2 * b) * hop - lo2, hop, n, t);
  } else {
    load_segment<P>(a, x, g0 + (2 * b) * hop - lo2, n, t);
    load_segment<P>(d, x, g0 + (2 * b + 1) * hop - lo2, n, t);
  }
  launder_anchors<P>(wa);
  fft_pair<P>(a, d, lds, TwAnchors{wa}, t);
  // lane-major G (fir_poly_gtable): load r gives lane t its G(t, 2r), G(t, 2r + 1)
  const float4* G4 = reinterpret_cast<const float4*>(G) + t;
  float2 ua[PD::E], ud[PD::E];
#pragma unroll
  for (int i = 0; i < PD::E; ++i) {
    float2 pa[4], pd[4];
    const float4 g01 = G4[64 * (2 * i)], g23 = G4[64 * (2 * i + 1)];
    const float2 gq[4] = {make_float2(g01.x, g01.y), make_float2(g01.z, g01.w),
                          make_float2(g23.x, g23.y), make_float2(g23.z, g23.w)};
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float2 g = gq[q];
      pa[q] = cmul(a[4 * i + q], g);
      pd[q] = cmul(d[4 * i + q], g);
    }
    const float2 sa0 = swap32_add(pa[0], pa[1]), sa1 = swap32_add(pa[2], pa[3]);
    const float2 sd0 = swap32_add(pd[0], pd[1]), sd1 = swap32_add(pd[2], pd[3]);
    ua[i] = swap16_add_conj(sa0, sa1);
    ud[i] = swap16_add_conj(sd0, sd1);
  }
  fft_pair<PD>(ua, ud, lds, TwRegs{wr}, tq);
  if constexpr (STD) {
    static_assert(out_off<PD>(1) == 64 && PD::E == 4 && kStdLo2 / D == 64 &&
                  (kStdLo2 + kStdHop) / D == 256, "e = 1..3 kept on every lane");
    // both segments' last output (index 255) inside the chunk: uniform
    if ((2 * b + 1) * kStdHop - kStdLo2 + 255LL * D < nloc) {
#pragma unroll
      for (int f = 0; f < 2; ++f) {
        float2* yb = y + (2 * b + f) * (kStdHop / D) - kStdLo2 / D + tq;
        const float2* u = f ? ud : ua;
#pragma unroll
        for (int e = 1; e < PD::E; ++e) st_stream(yb + 64 * e, conj1(u[e]));
      }
      cs.done(clk);
      return;
    }
  }
  const int n0 = lo2 / D, n1 = (lo2 + (int)hop) / D;
#pragma unroll
  for (int f = 0; f < 2; ++f) {
    const long long bb = 2 * b + f;
    const long long gb = bb * hop - lo2;          // chunk output of circular index 0
    float2* yb = y + bb * (hop / D) - n0;
    const float2* u = f ? ud : ua;
#pragma unroll
    for (int e = 0; e < PD::E; ++e) {
      const int i = out_index<PD>(tq, e);
      if (i >= n0 && i < n1 && gb + (long long)i * D < nloc) st_stream(yb + i, conj1(u[e]));
    }
  }
  cs.done(clk);
}

// G_k[j] (see fir_poly_kernel) from Hs = FFT_1024(h) / 1024, in double.
__global__ void fir_poly_gtable(const float2* __restrict__ Hs, float2* __restrict__ G) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= 1024) return;
  const int k = i >> 8, j = i & 255;
  double re = 0.0, im = 0.0;
  for (int s = 0; s < 4; ++s) {
    double sn, cs;
    sincospi(-2.0 * (double)(k * (j + 256 * s)) / 1024.0, &sn, &cs);
    const float2 h = Hs[j + 256 * s];
    re += (double)h.x * cs - (double)h.y * sn;
    im += (double)h.x * sn + (double)h.y * cs;
  }
  // lane-major: lane t = 16 k + (j & 15) uses G(t, m), m = j >> 4, from its
  // float4 m >> 1 (fir_poly_kernel)
  const int t = (k << 4) | (j & 15), m = j >> 4;
  G[((m >> 1) * 64 + t) * 2 + (m & 1)] = make_float2((float)re, (float)im);
}

hipError_t launch_fir_poly_gtable(const float2* Hs, float2* G, hipStream_t st) {
  hipLaunchKernelGGL(fir_poly_gtable, dim3(4), dim3(256), 0, st, Hs, G);
  return hipGetLastError();
}

// Every segment start x + off + k hop (k >= 0) 16-byte aligned: the 16-byte
// segment loads (load_segment_x4) apply.
static bool x4_aligned(const float2* x, long long off, long long hop) {
  return (hop % 2) == 0 && ((reinterpret_cast<uintptr_t>(x) + 8 * (uintptr_t)off) & 15) == 0;
}

hipError_t launch_fir_poly(const float2* x, long long n, long long g0, const float2* G, int lo2,
                           long long hop, float2* y, const float2* tw, const float2* twd,
                           hipStream_t st, const MixArgs* mix) {
  if (n - g0 <= 0) return hipSuccess;
  const long long nblocks = (n - g0 + hop - 1) / hop;
  const dim3 g((unsigned)((nblocks + 1) / 2)), blk(64);
  const MixArgs m = mix ? *mix : MixArgs{};
  if (mix)
    hipLaunchKernelGGL(fir_poly_kernel<true>, g, blk, 0, st, x, n, g0, G, lo2, hop, y, nblocks, tw, twd, m,
                       g_clock_sink);
  else if (x4_aligned(x, g0 - lo2, hop) && lo2 == kStdLo2 && hop == kStdHop)
    hipLaunchKernelGGL((fir_poly_kernel<false, true, true>), g, blk, 0, st, x, n, g0, G, lo2, hop, y,
                       nblocks, tw, twd, m, g_clock_sink);
  else if (x4_aligned(x, g0 - lo2, hop))
    hipLaunchKernelGGL((fir_poly_kernel<false, true>), g, blk, 0, st, x, n, g0, G, lo2, hop, y, nblocks, tw,
                       twd, m, g_clock_sink);
  else
    hipLaunchKernelGGL(fir_poly_kernel<false>, g, blk, 0, st, x, n, g0, G, lo2, hop, y, nblocks, tw, twd, m,
                       g_clock_sink);
  return hipGetLastError();
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

hipError_t launch_fir_os(int M, const float2* x, long long n, long long g0, const float2* Hs,
                         int ntaps, long long hop, int decim, float2* y, const float2* tw,
                         hipStream_t st, const MixArgs* mix) {
  if (n - g0 <= 0) return hipSuccess;
  const long long nblocks = (n - g0 + hop - 1) / hop;
  const dim3 grid((unsigned)((nblocks + 1) / 2));
  const MixArgs m = mix ? *mix : MixArgs{};
  auto run = [&](auto plan) {
    using PL = decltype(plan);
    if constexpr (PL::TF == 64) {
      if (mix) {
        hipLaunchKernelGGL((fir_os_kernel<PL, true>), grid, dim3(PL::TF), 0, st, x, n, g0, Hs, ntaps - 1,
                           hop, decim, y, nblocks, tw, m, g_clock_sink);
        return;
      }
    }
    if constexpr (map0_of<PL>::value == kMapPair) {
      // the pair map's 16-byte stores write 128-output runs at circular
      // indices 128 i: with lo a multiple of 16 every run covers whole 128-byte
      // lines of y (one store instruction per line, none split between two) --
      // the segment then starts a few samples earlier (lo >= ntaps - 1 and
      // lo + hop <= M still hold).  Config 2 (255 taps, lo 254 -> 256): FIR
      // 0.822 -> 0.789 ms (profiles/r05_fir_align_ab.txt); the loads' own
      // alignment (the chain's 16-multiple history) measured neutral at D = 1.
      int lo = ntaps - 1;
      const int lo16 = (lo + 15) & ~15;
      if (decim == 1 && lo16 + hop <= PL::N && x4_aligned(x, g0 - lo16, hop)) lo = lo16;
      const bool xs = decim == 1 && lo % 2 == 0 && x4_aligned(y, 0, hop);
      if (x4_aligned(x, g0 - lo, hop)) {
        if (xs)
          hipLaunchKernelGGL((fir_os_kernel<PL, false, true, true>), grid, dim3(PL::TF), 0, st, x, n, g0,
                             Hs, lo, hop, decim, y, nblocks, tw, m, g_clock_sink);
        else
          hipLaunchKernelGGL((fir_os_kernel<PL, false, true>), grid, dim3(PL::TF), 0, st, x, n, g0, Hs,
                             lo, hop, decim, y, nblocks, tw, m, g_clock_sink);
        return;
      }
    }
    hipLaunchKernelGGL((fir_os_kernel<PL, false>), grid, dim3(PL::TF), 0, st, x, n, g0, Hs, ntaps - 1,
                       hop, decim, y, nblocks, tw, m, g_clock_sink);
  };
  switch (M) {
    case 1024: run(Plan1024x{}); break;
    case 4096: if (mix) return hipErrorInvalidValue; run(Plan4096{}); break;
    case 8192: if (mix) return hipErrorInvalidValue; run(Plan8192{}); break;
    case 16384: if (mix) return hipErrorInvalidValue; run(Plan16384{}); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

}  // namespace vsig
