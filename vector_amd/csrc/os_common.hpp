// Shared pieces of the overlap-save / streaming kernels (gfx950): launch
// geometry, segment loads, DPP wave reductions of |c| partials, plan switches.
// Included by psd.hip, fir.hip, xcorr.hip, reduce.hip (one translation unit
// each, compiled in parallel; every kernel is launched from its own TU).
#pragma once
#include "fft_engine.hpp"
#include "vsig_kernels.h"
#include "npabs.hpp"

namespace vsig {

// Streaming accesses (input read once, output written once) with a
// non-temporal hint where it measured faster on the chain: the PSD's frame
// loads and the FIR's output stores (so the filtered stream does not sit in
// L2 / the Infinity Cache as dirty lines while the PSD and the correlator
// read it), and the FIR pairs' rows no other pair reads (load_pair_x4); the
// rows neighbouring pairs share stay plain (their second read is an L2 hit).
template <bool NT = false>
__device__ __forceinline__ float2 ld_stream(const float2* p) {
  if constexpr (NT) return fromv(__builtin_nontemporal_load(reinterpret_cast<const f2v*>(p)));
  else return *p;
}
template <bool NT = true>
__device__ __forceinline__ void st_stream(float2* p, float2 v) {
  if constexpr (NT) __builtin_nontemporal_store(tov(v), reinterpret_cast<f2v*>(p));
  else *p = v;
}

// Pass-0 operands of an overlap-save segment x[s0 .. s0 + N) with zero fill
// outside [0, n).  The block-uniform base keeps the address in SGPRs; interior
// segments (the common case) skip the per-element bounds test.
// Raw buffer loads with a wave-uniform descriptor: the per-lane part of the
// address is one 32-bit voffset shared by all of a thread's loads, the
// per-element constants go to soffset (SGPRs), so a burst of loads costs no
// 64-bit address arithmetic (v_add_co / v_addc pairs and their wait states).
// The descriptor inputs pass readfirstlane so the compiler sees them uniform.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* p, unsigned bytes) {
  const unsigned long long a = reinterpret_cast<unsigned long long>(p);
  const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)a);
  const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(a >> 32));
  void* q = reinterpret_cast<void*>(((unsigned long long)hi << 32) | lo);
  return __builtin_amdgcn_make_buffer_rsrc(q, (short)0, (int)__builtin_amdgcn_readfirstlane(bytes),
                                           0x00020000);
}
__device__ __forceinline__ float2 buf_load2(__amdgpu_buffer_rsrc_t r, unsigned voff, int soff) {
  return __builtin_bit_cast(float2, __builtin_amdgcn_raw_buffer_load_b64(r, (int)voff, soff, 0));
}
__device__ __forceinline__ float4 buf_load4(__amdgpu_buffer_rsrc_t r, unsigned voff, int soff) {
  return __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(r, (int)voff, soff, 0));
}

template <class P, bool NT = false>
__device__ __forceinline__ void load_segment(float2* v, const float2* __restrict__ x,
                                             long long s0, long long n, int t) {
  const float2* base = x + s0;
  if (s0 >= 0 && s0 + P::N <= n) {
#pragma unroll
    for (int e = 0; e < P::E; ++e) v[e] = ld_stream<NT>(base + (unsigned)in_index<P>(t, e));
  } else {
#pragma unroll
    for (int e = 0; e < P::E; ++e) {
      const int i = in_index<P>(t, e);
      const long long xi = s0 + i;
      v[e] = (xi >= 0 && xi < n) ? ld_stream<NT>(base + i) : make_float2(0.f, 0.f);
    }
  }
}

// load_segment for one-wave plans whose first pass has the pair map (operand
// e of thread t = x[s0 + m(t) + 64 e], m(l) = 2l for l < 32, 2(l-32) + 1
// above) by 16-byte loads: load i gives lane l the samples 2l + 128 i and
// 2l + 1 + 128 i; one v_permlane32_swap of the odd samples of lanes < 32 with
// the even samples of lanes >= 32 leaves lane l with x[m(l) + 128 i] and
// x[m(l) + 64 + 128 i], i.e. operands 2 i and 2 i + 1 -- half the load
// instructions of load_segment (the FIR's load / store pattern measured 8 %
// faster this way with its transforms knocked out).  x + s0 must be 16-byte
// aligned (a launch-time property: the callers' segment starts are all even
// offsets from one base); segments not inside [0, n) take load_segment.
template <class P>
__device__ __forceinline__ void load_segment_x4(float2* v, const float2* __restrict__ x,
                                                long long s0, long long n, int t) {
  static_assert(map0_of<P>::value == kMapPair && P::TF == 64 && P::E == 16 && P::R[0] == 16,
                "operand layout m(t) + 64 e");
  if (s0 >= 0 && s0 + P::N <= n) {
    typedef float f4 __attribute__((ext_vector_type(4)));
    const f4* b4 = reinterpret_cast<const f4*>(x + s0);
#pragma unroll
    for (int i = 0; i < P::E / 2; ++i) {
      const f4 u = b4[t + 64 * i];
      const auto rx = __builtin_amdgcn_permlane32_swap(__float_as_uint(u.x), __float_as_uint(u.z), false, false);
      const auto ry = __builtin_amdgcn_permlane32_swap(__float_as_uint(u.y), __float_as_uint(u.w), false, false);
      v[2 * i] = make_float2(__uint_as_float(rx[0]), __uint_as_float(ry[0]));
      v[2 * i + 1] = make_float2(__uint_as_float(rx[1]), __uint_as_float(ry[1]));
    }
  } else {
    load_segment<P>(v, x, s0, n, t);
  }
}

// The two segments of a one-wave FIR pair (s0 and s0 + hop) by 16-byte loads.
// At hop = 3N/4 the second segment's first quarter is the first one's last
// quarter in the same lanes (load i of the second = load i + 6 of the first),
// so its rows 0..3 are copied instead of loaded: 14 loads per pair, not 16.
template <class P>
__device__ __forceinline__ void load_pair_x4(float2* a, float2* d, const float2* __restrict__ x,
                                             long long s0, long long hop, long long n, int t) {
  static_assert(map0_of<P>::value == kMapPair && P::TF == 64 && P::E == 16 && P::R[0] == 16,
                "operand layout m(t) + 64 e");
  constexpr int kQ = 3 * P::N / 4;
  if (hop == kQ && s0 >= 0 && s0 + kQ + P::N <= n) {      // uniform
    typedef float f4 __attribute__((ext_vector_type(4)));
    const f4* b4 = reinterpret_cast<const f4*>(x + s0);
    f4 u[P::E / 2 + 6];
    // rows 0, 1 and 12, 13 are also read by the neighbouring pairs (their 256
    // overlap samples, from L2); the rows only this pair reads are loaded
    // non-temporal.  With the segment starts on 128-byte lines (the chain's
    // 16-multiple halo) this took the D = 4 FIR 3.67 -> 3.57 ms at config 5
    // (profiles/r05_fir_nt_ab.txt; all rows non-temporal, or all but 12 / 13:
    // slower than plain; D = 1 neutral).  Before the alignment fix the same
    // split measured neutral (r04_ab_neutral.txt item 1).
#pragma unroll
    for (int i = 0; i < P::E / 2 + 6; ++i) {                      // float4 rows 0..13
      if (i >= 2 && i < 12) u[i] = __builtin_nontemporal_load(b4 + t + 64 * i);
      else u[i] = b4[t + 64 * i];
    }
    auto unpack = [&](float2* v, int e, const f4& w) {
      const auto rx = __builtin_amdgcn_permlane32_swap(__float_as_uint(w.x), __float_as_uint(w.z), false, false);
      const auto ry = __builtin_amdgcn_permlane32_swap(__float_as_uint(w.y), __float_as_uint(w.w), false, false);
      v[e] = make_float2(__uint_as_float(rx[0]), __uint_as_float(ry[0]));
      v[e + 1] = make_float2(__uint_as_float(rx[1]), __uint_as_float(ry[1]));
    };
#pragma unroll
    for (int i = 0; i < P::E / 2; ++i) unpack(a, 2 * i, u[i]);
#pragma unroll
    for (int e = 0; e < 4; ++e) d[e] = a[12 + e];
#pragma unroll
    for (int i = 2; i < P::E / 2; ++i) unpack(d, 2 * i, u[6 + i]);
    return;
  }
  load_segment_x4<P>(a, x, s0, n, t);
  load_segment_x4<P>(d, x, s0 + hop, n, t);
}

// load_segment with the NCO mixer applied to each sample (global index
// mix.i0 + s0 + i; the zero fill stays zero): one double-precision phase per
// lane (sample g + t), then the per-element offsets' rotations
// (offsets 64 e, mix.rot) in fp32 -- about 2e-7 relative per sample.
template <class P>
__device__ __forceinline__ void load_segment_mix(float2* v, const float2* __restrict__ x,
                                                 long long s0, long long n, int t, const MixArgs& mix) {
  static_assert(P::TF == 64 && P::E == 16 && P::R[0] == 16,
                "the rotation table assumes in_index(t, e) = m(t) + 64 e");
  load_segment<P>(v, x, s0, n, t);
  const float2 r0 = mix_rot_fast(mix.i0 + s0 + in_index<P>(t, 0), mix.wsr);
#pragma unroll
  for (int e = 0; e < P::E; ++e) {
    const float2 r = cmul(r0, make_float2(mix.rot[2 * e], mix.rot[2 * e + 1]));
    v[e] = cmul(v[e], r);
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

}  // namespace vsig
