// In-LDS Stockham FFT engine for CDNA4 (gfx950), complex fp32.
//
// One "frame" of N points is transformed by TF = N / E threads, each holding E
// complex values in VGPRs.  A pass of radix R does E / R register butterflies
// per thread; passes exchange data through LDS (padded one float2 per 16 to
// keep the stride-R scatter writes of the early passes bank-conflict free).
// The first pass reads its operands straight from the caller's registers (the
// kernel loads them from HBM with the window / zero-fill fused), the last pass
// leaves the natural-order spectrum in registers for a fused epilogue
// (|X|^2 store, filter multiply, correlation peak reduction ...).
//
// Index convention (Stockham autosort, natural order in and out):
//   pass p, radix R, Ns = R_0 * ... * R_{p-1}, butterfly j (0 <= j < N/R):
//     in : a[j + r*N/R]            r = 0..R-1
//     tw : a_r *= exp(-2*pi*i * r*(j mod Ns) / (Ns*R))        (p > 0)
//     out: b[(j/Ns)*Ns*R + (j mod Ns) + r*Ns] = DFT_R(a)_r
//   thread t of a frame owns butterflies j = t + b*TF, b = 0..E/R-1, and keeps
//   them in v[b*R + r].  Before pass 0, v[b*R0 + r] must hold x[j + r*N/R0];
//   after the last pass v[b*RL + r] holds X[j + r*N/RL].
//
// Twiddles come from a per-plan table in global memory (L2 resident, built on
// the host in double precision): for pass p >= 1 the block
//   tw[off_p + (r-1)*Ns + k] = exp(-2*pi*i * r*k / (Ns*R)),  k < Ns, 1 <= r < R,
// so the lanes of a wave (consecutive k) read consecutive addresses.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

namespace vsig {

// Complex arithmetic.  CDNA3/4 execute packed fp32 (v_pk_add/mul/fma_f32) at
// the scalar rate, so a complex value in an (even-aligned) VGPR pair costs one
// instruction per add and two per multiply when the operand swizzles go into
// the VOP3P op_sel / neg modifiers — which the compiler does not do on its own
// for swizzled operands, hence the inline asm below.
typedef float f2v __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f2v tov(float2 a) { return (f2v){a.x, a.y}; }
__device__ __forceinline__ float2 fromv(f2v a) { return make_float2(a.x, a.y); }

__device__ __forceinline__ float2 cadd(float2 a, float2 b) { return fromv(tov(a) + tov(b)); }
__device__ __forceinline__ float2 csub(float2 a, float2 b) { return fromv(tov(a) - tov(b)); }
// a * b = b.x * (a.x, a.y) + b.y * (-a.y, a.x)
__device__ __forceinline__ float2 cmul(float2 a, float2 b) {
  const f2v av = tov(a), bv = tov(b);
  const f2v t = av * bv.xx;
  f2v r;
  asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[1,1,0] op_sel_hi:[0,1,1] neg_lo:[1,0,0]"
      : "=v"(r) : "v"(av), "v"(bv), "v"(t));
  return fromv(r);
}
// cmul(a, b) given t = a * b.xx (so that the two halves can be scheduled apart)
__device__ __forceinline__ float2 cmul_fin(float2 a, float2 b, f2v t) {
  f2v r;
  asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[1,1,0] op_sel_hi:[0,1,1] neg_lo:[1,0,0]"
      : "=v"(r) : "v"(tov(a)), "v"(tov(b)), "v"(t));
  return fromv(r);
}
// a + (-i) b = (a.x + b.y, a.y - b.x)   and   a - (-i) b = (a.x - b.y, a.y + b.x)
__device__ __forceinline__ float2 cadd_mi(float2 a, float2 b) {
  f2v r;
  asm("v_pk_add_f32 %0, %1, %2 op_sel:[0,1] op_sel_hi:[1,0] neg_hi:[0,1]"
      : "=v"(r) : "v"(tov(a)), "v"(tov(b)));
  return fromv(r);
}
__device__ __forceinline__ float2 csub_mi(float2 a, float2 b) {
  f2v r;
  asm("v_pk_add_f32 %0, %1, %2 op_sel:[0,1] op_sel_hi:[1,0] neg_lo:[0,1]"
      : "=v"(r) : "v"(tov(a)), "v"(tov(b)));
  return fromv(r);
}
// a + h * u with a compile-time scalar h (SGPR pair (h, h))
__device__ __forceinline__ float2 cfma_s(float2 u, float h, float2 a) {
  f2v r;
  const f2v hh = (f2v){h, h};
  asm("v_pk_fma_f32 %0, %1, %2, %3" : "=v"(r) : "v"(tov(u)), "s"(hh), "v"(tov(a)));
  return fromv(r);
}
// b * (c - i s) for compile-time c, s: c * (b.x, b.y) + s * (b.y, -b.x)
__device__ __forceinline__ float2 cmul_cs(float2 b, float c, float s_) {
  const f2v bv = tov(b);
  const f2v ss = (f2v){s_, s_};
  const f2v t = bv * (f2v){c, c};       // plain product: the compiler schedules it
  f2v r;
  asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[1,0,0] op_sel_hi:[0,1,1] neg_hi:[1,0,0]"
      : "=v"(r) : "v"(bv), "s"(ss), "v"(t));
  return fromv(r);
}
__device__ __forceinline__ float2 cconj(float2 a) { return make_float2(a.x, -a.y); }
// The conjugates of the overlap-save kernels (inverse transform by conj) with
// the sign in the VOP3P neg modifiers -- the compiler's own form of a lone
// conj negates both halves and moves one back (two instructions and a wait
// state), and it does not fold one into a neighbouring asm product:
// conj(v) as (v.x + 0, -v.y + 0)
__device__ __forceinline__ float2 conj1(float2 v) {
  f2v r;
  asm("v_pk_add_f32 %0, %1, 0 neg_hi:[1,0]" : "=v"(r) : "v"(tov(v)));
  return fromv(r);
}
// conj(a * b): cmul with the high half's sum negated (neg_hi on its product
// and its addend)
__device__ __forceinline__ float2 cmul_conj(float2 a, float2 b) {
  const f2v av = tov(a), bv = tov(b);
  const f2v t = av * bv.xx;
  f2v r;
  asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[1,1,0] op_sel_hi:[0,1,1] neg_lo:[1,0,0] neg_hi:[1,0,1]"
      : "=v"(r) : "v"(av), "v"(bv), "v"(t));
  return fromv(r);
}
// conj(a + b)
__device__ __forceinline__ float2 cadd_conj(float2 a, float2 b) {
  f2v r;
  asm("v_pk_add_f32 %0, %1, %2 neg_hi:[1,1]" : "=v"(r) : "v"(tov(a)), "v"(tov(b)));
  return fromv(r);
}
// (The correlator's spectrum product conj(X) P keeps cmul(cconj(a), b): with
// the conj folded into neg modifiers -- two asm ops, or cmul's own shape with
// one -- it measured 1.3-4 % slower at config 5 (206 -> 249-253 VGPRs),
// profiles/r06_conj_std_ab.txt.)

// cos / sin of 2*pi*k/64, k = 0..31 (enough for every in-register radix <= 64).
constexpr float kCos64[32] = {
    1.000000000e+00f, 9.951847267e-01f, 9.807852804e-01f, 9.569403357e-01f,
    9.238795325e-01f, 8.819212643e-01f, 8.314696123e-01f, 7.730104534e-01f,
    7.071067812e-01f, 6.343932842e-01f, 5.555702330e-01f, 4.713967368e-01f,
    3.826834324e-01f, 2.902846773e-01f, 1.950903220e-01f, 9.801714033e-02f,
    0.0f,             -9.801714033e-02f, -1.950903220e-01f, -2.902846773e-01f,
    -3.826834324e-01f, -4.713967368e-01f, -5.555702330e-01f, -6.343932842e-01f,
    -7.071067812e-01f, -7.730104534e-01f, -8.314696123e-01f, -8.819212643e-01f,
    -9.238795325e-01f, -9.569403357e-01f, -9.807852804e-01f, -9.951847267e-01f};
constexpr float kSin64[32] = {
    0.0f,             9.801714033e-02f, 1.950903220e-01f, 2.902846773e-01f,
    3.826834324e-01f, 4.713967368e-01f, 5.555702330e-01f, 6.343932842e-01f,
    7.071067812e-01f, 7.730104534e-01f, 8.314696123e-01f, 8.819212643e-01f,
    9.238795325e-01f, 9.569403357e-01f, 9.807852804e-01f, 9.951847267e-01f,
    1.000000000e+00f, 9.951847267e-01f, 9.807852804e-01f, 9.569403357e-01f,
    9.238795325e-01f, 8.819212643e-01f, 8.314696123e-01f, 7.730104534e-01f,
    7.071067812e-01f, 6.343932842e-01f, 5.555702330e-01f, 4.713967368e-01f,
    3.826834324e-01f, 2.902846773e-01f, 1.950903220e-01f, 9.801714033e-02f};

// Compile-time loop: f(IC<B>{}) ... f(IC<E - 1>{}).
template <int I> struct IC { static constexpr int value = I; };
template <int B, int E, class F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (B < E) { f(IC<B>{}); static_for<B + 1, E>(f); }
}

// b * exp(-2*pi*i*K/M) with compile-time K, M (M <= 64).  Trivial factors
// (1, -i, and the 45-degree family) are special-cased so they cost no multiply.
template <int K, int M>
__device__ __forceinline__ float2 twc(float2 b) {
  static_assert(M <= 64 && K < M, "in-register twiddle out of range");
  if constexpr (K == 0) {
    return b;
  } else if constexpr (4 * K == M) {            // * (-i)
    return make_float2(b.y, -b.x);
  } else if constexpr (8 * K == M) {            // * (1 - i)/sqrt2
    constexpr float h = 7.071067812e-01f;
    return make_float2(h * (b.x + b.y), h * (b.y - b.x));
  } else if constexpr (8 * K == 3 * M) {        // * (-1 - i)/sqrt2
    constexpr float h = 7.071067812e-01f;
    return make_float2(h * (b.y - b.x), -h * (b.x + b.y));
  } else {
    constexpr int idx = K * (64 / M);
    return cmul_cs(b, kCos64[idx], kSin64[idx]);
  }
}

// One radix-2 Stockham step inside registers: Ns = 2^P.  The step runs in
// two phases over all its butterflies J -- (A) each twiddled operand's
// ratio form u, (C) the sums -- so that a packed op and its consumer are never
// adjacent: gfx950 needs one wait state between a packed fp32 op and a
// dependent one, and hipcc pads every inline-asm boundary with one, while
// independent work in between costs nothing.
// General twiddles w = c - i s take the ratio (Linzer-Feig) form: with
// rot(b) = (b.y, -b.x), w b = c (b + (s/c) rot(b)) when |c| >= |s|, else
// s ((c/s) b + rot(b)) -- u is one packed fma with the swizzle and the sign in
// op_sel / neg_hi, and x0 +- w b two packed fmas with the scalar (c or s):
// 3 packed ops per butterfly instead of 4 (a product in two halves, then an
// add and a sub).  The ratio is at most 1, so the rounding is the product's.
template <int K, int M>
struct RatioTw {
  static constexpr int idx = K * (64 / M);
  static constexpr float c = kCos64[idx], s = kSin64[idx];
  static constexpr bool cbig = (c < 0 ? -c : c) >= (s < 0 ? -s : s);
  static constexpr float ratio = cbig ? (float)((double)s / (double)c) : (float)((double)c / (double)s);
  static constexpr float scale = cbig ? c : s;
};
template <int K, int M>
__device__ __forceinline__ float2 ratio_u(float2 b) {
  using T = RatioTw<K, M>;
  const f2v bv = tov(b), rr = (f2v){T::ratio, T::ratio};
  f2v r;
  if constexpr (T::cbig)      // b + ratio * (b.y, -b.x)
    asm("v_pk_fma_f32 %0, %1, %2, %1 op_sel:[1,0,0] op_sel_hi:[0,1,1] neg_hi:[1,0,0]"
        : "=v"(r) : "v"(bv), "s"(rr));
  else                        // ratio * b + (b.y, -b.x)
    asm("v_pk_fma_f32 %0, %1, %2, %1 op_sel:[0,0,1] op_sel_hi:[1,1,0] neg_hi:[0,0,1]"
        : "=v"(r) : "v"(bv), "s"(rr));
  return fromv(r);
}
// a - h * u with a compile-time scalar h (the same SGPR pair as cfma_s, negated
// by the neg modifiers)
__device__ __forceinline__ float2 cfms_s(float2 u, float h, float2 a) {
  f2v r;
  const f2v hh = (f2v){h, h};
  asm("v_pk_fma_f32 %0, %1, %2, %3 neg_lo:[0,1,0] neg_hi:[0,1,0]"
      : "=v"(r) : "v"(tov(u)), "s"(hh), "v"(tov(a)));
  return fromv(r);
}

template <int R, int P>
struct Radix2Phased {
  static constexpr int Ns = 1 << P, M = 2 * Ns;
  template <int J> static constexpr int kk() { return J & (Ns - 1); }
  template <int J> static constexpr bool general() {
    constexpr int k = kk<J>();
    return k != 0 && 4 * k != M && 8 * k != M && 8 * k != 3 * M;
  }
  __device__ __forceinline__ static void run(const float2* a, float2* t) {
    float2 u[R / 2];
    // (A) general twiddles: the ratio form; 45-degree family: (b.x +- b.y, ...)
    static_for<0, R / 2>([&](auto ji) {
      constexpr int J = decltype(ji)::value;
      constexpr int k = kk<J>();
      const float2 b = a[J + R / 2];
      if constexpr (general<J>()) {
        u[J] = ratio_u<k, M>(b);
      } else if constexpr (8 * k == M) {
        u[J] = cadd_mi(b, b);
      } else if constexpr (8 * k == 3 * M) {
        u[J] = csub_mi(b, b);
      }
    });
    // (C) the butterflies' sums
    static_for<0, R / 2>([&](auto ji) {
      constexpr int J = decltype(ji)::value;
      constexpr int k = kk<J>();
      constexpr int o = ((J >> P) << (P + 1)) + k;
      const float2 x0 = a[J];
      const float2 b = a[J + R / 2];
      if constexpr (k == 0) {
        t[o] = cadd(x0, b);
        t[o + Ns] = csub(x0, b);
      } else if constexpr (4 * k == M) {           // (-i) b folded into the adds
        t[o] = cadd_mi(x0, b);
        t[o + Ns] = csub_mi(x0, b);
      } else if constexpr (8 * k == M) {           // h (b.x + b.y, b.y - b.x)
        constexpr float h = 7.071067812e-01f;
        t[o] = cfma_s(u[J], h, x0);
        t[o + Ns] = cfms_s(u[J], h, x0);
      } else if constexpr (8 * k == 3 * M) {       // -h (b.x - b.y, b.x + b.y)
        constexpr float h = 7.071067812e-01f;
        t[o] = cfms_s(u[J], h, x0);
        t[o + Ns] = cfma_s(u[J], h, x0);
      } else {
        constexpr float sc = RatioTw<k, M>::scale;
        t[o] = cfma_s(u[J], sc, x0);
        t[o + Ns] = cfms_s(u[J], sc, x0);
      }
    });
  }
};

template <int R, int P>
struct DftPasses {
  __device__ __forceinline__ static void run(float2* v) {
    float2 t[R];
    Radix2Phased<R, P>::run(v, t);
#pragma unroll
    for (int i = 0; i < R; ++i) v[i] = t[i];
    if constexpr ((2 << P) < R) DftPasses<R, P + 1>::run(v);
  }
};

// In-place natural-order DFT of R = 2^k values held in registers.
template <int R>
__device__ __forceinline__ void dft_reg(float2* v) {
  static_assert((R & (R - 1)) == 0 && R >= 2 && R <= 64, "radix must be a power of two in [2, 64]");
  DftPasses<R, 0>::run(v);
}

// ---------------------------------------------------------------------------
// Plans
// ---------------------------------------------------------------------------
template <int N_, int E_, int... Rs>
struct Plan {
  static constexpr int N = N_;
  static constexpr int E = E_;
  static constexpr int TF = N_ / E_;               // threads per frame
  static constexpr int NP = sizeof...(Rs);         // number of passes
  static constexpr int R[NP] = {Rs...};
  static constexpr int LDS = N_ + N_ / 16;         // padded float2 per frame

  static constexpr int ns(int p) { int s = 1; for (int q = 0; q < p; ++q) s *= R[q]; return s; }
  static constexpr int twoff(int p) { int o = 0; for (int q = 1; q < p; ++q) o += (R[q] - 1) * ns(q); return o; }
  static constexpr int twsize() { return twoff(NP); }
  static constexpr int RL = R[NP - 1];
  static constexpr bool valid() {
    int prod = 1;
    for (int q = 0; q < NP; ++q) { if (E_ % R[q]) return false; prod *= R[q]; }
    return prod == N_;
  }
};

__device__ __forceinline__ int lpad(int i) { return i + (i >> 4); }

// Per-plan LDS exchange geometry.  Default: 1 float2 of padding per 16, every
// pass's butterfly j = t + b TF.  A plan may pad 1 per 2^PADSH instead and
// give its first pass (MAP0) and its last pass (MAPL) a lane map m(t): the
// pass then runs butterfly j = m(t) + b TF (the passes in between keep
// j = t; a pass's thread map changes only who computes which butterfly, the
// LDS image between passes is the same).  Maps:
//   kMapId    m(t) = t;
//   kMapSigma m(t) = (t & ~31) | ((t & 15) << 1) | ((t >> 4) & 1)
//             (lanes 0-15 take the even j of their 32-lane half, lanes 16-31
//             the odd);
//   kMapPair  m(t) = ((t & 31) << 1) | (t >> 5)   (TF = 64: lane l < 32 takes
//             j = 2l, lane l + 32 takes j = 2l + 1) -- the layout a 16-byte
//             load (samples 2l, 2l + 1) reaches after one v_permlane32_swap
//             (load_segment_x4);
//   kMapIlv   butterflies j = B t + b (B = E / R per thread: adjacent j), so a
//             first pass with two butterflies per thread reads its operands
//             x[2t + b + (N/R) r] as one 16-byte load per r and a last pass
//             leaves adjacent bins 2t, 2t + 1 in one thread (8-byte |X|^2
//             pairs) -- no lane exchange at all.
// Why padding 1 per 32 with sigma or pair maps (Plan8192x, the FIR plans): the
// first pass's stride-R scatter stores (R j + r, ds_write_b64: 16-lane groups,
// banks mod 32 dwords) need the padding to differ across the group's j, and
// the later passes' reads (t + (N/R) m, ds_read_b64: 32-lane groups, banks mod
// 64 dwords) need it equal across a 32-lane run.  1 per 16 serves the stores
// but puts lanes 0 and 31 of every read group on one bank (one extra cycle
// per ds_read_b64); 1 per 32 serves the reads, and both maps give each store
// group 16 j of one parity, whose padding j / 2 is again distinct.  The
// operand / result layouts follow the maps (in_index: MAP0, out_index: MAPL).
constexpr int kMapId = 0, kMapSigma = 1, kMapPair = 2, kMapIlv = 3;
template <class P, class = void>
struct padsh_of { static constexpr int value = 4; };
template <class P>
struct padsh_of<P, decltype(void(P::PADSH))> { static constexpr int value = P::PADSH; };
template <class P, class = void>
struct map0_of { static constexpr int value = kMapId; };
template <class P>
struct map0_of<P, decltype(void(P::MAP0))> { static constexpr int value = P::MAP0; };
template <class P, class = void>
struct mapl_of { static constexpr int value = kMapId; };
template <class P>
struct mapl_of<P, decltype(void(P::MAPL))> { static constexpr int value = P::MAPL; };

template <class P, class = void>
struct padun_of { static constexpr int value = 0; };
template <class P>
struct padun_of<P, decltype(void(P::PADUN))> { static constexpr int value = P::PADUN; };
// padding before index i: 2^PADUN float2 per 2^PADSH (PADUN = 1 keeps even
// indices 16-byte aligned: adjacent pairs become one ds_read/write_b128).
// Exchange X (1 <= X < NP: pass X-1's stores, pass X's loads) may pad its own
// way (xpad, specialised per plan; X = 0: the plan's default) -- the stores
// and loads of one exchange agree, and the LDS image of one exchange is never
// read under another's padding.
template <class P, int X>
struct xpad {
  static constexpr int S = padsh_of<P>::value;
  static constexpr int U = padun_of<P>::value;
};
template <class P, int X = 0>
__host__ __device__ constexpr int padc(int i) {
  return (i >> xpad<P, X>::S) << xpad<P, X>::U;
}
template <class P, int X = 0>
__device__ __forceinline__ int lpadp(int i) { return i + padc<P, X>(i); }
// float2 an exchange buffer of plan P needs (the widest exchange), and the
// size kernels declare: P::LDS (the default padding) or more under xpad
template <class P, int X = 1>
constexpr int lds_need() {
  if constexpr (X >= P::NP) return 0;
  else {
    constexpr int need = P::N + padc<P, X>(P::N - 1);
    constexpr int rest = lds_need<P, X + 1>();
    return need > rest ? need : rest;
  }
}
template <class P>
constexpr int lds_size() { return lds_need<P>() > P::LDS ? lds_need<P>() : P::LDS; }
template <int MAP>
__device__ __forceinline__ int lane_map(int t) {
  if constexpr (MAP == kMapSigma) return (t & ~31) | ((t & 15) << 1) | ((t >> 4) & 1);
  else if constexpr (MAP == kMapPair) return ((t & 31) << 1) | (t >> 5);
  else return t;
}
template <class P>
__device__ __forceinline__ int tmap0(int t) { return lane_map<map0_of<P>::value>(t); }
template <class P>
__device__ __forceinline__ int tmapl(int t) { return lane_map<mapl_of<P>::value>(t); }
template <class P, int p>
constexpr int pass_map() {
  return p == P::NP - 1 ? mapl_of<P>::value : p == 0 ? map0_of<P>::value : kMapId;
}
// thread t's butterfly index base in pass p (maps other than kMapIlv)
template <class P, int p>
__device__ __forceinline__ int tpass(int t) {
  static_assert(pass_map<P, p>() != kMapIlv, "kMapIlv: use bfly");
  return lane_map<pass_map<P, p>()>(t);
}
// butterfly b of thread t in pass p
template <class P, int p>
__device__ __forceinline__ int bfly(int t, int b) {
  if constexpr (pass_map<P, p>() == kMapIlv) return (P::E / P::R[p]) * t + b;
  else return lane_map<pass_map<P, p>()>(t) + b * P::TF;
}

// A plan with its exchange geometry set (see above).
template <class P, int M0, int ML, int S = 5, int U = 0>
struct Lanes : P {
  static_assert((M0 != kMapPair && ML != kMapPair) || P::TF == 64,
                "the pair map is for one-wave frames (not a permutation of t >= 64)");
  static_assert((M0 != kMapIlv || P::E / P::R[0] == 2) && (ML != kMapIlv || P::E / P::RL == 2),
                "the interleaved map pairs two butterflies per thread");
  static_assert(P::TF % 64 == 0 && (P::N / P::R[0]) % 32 == 0, "maps permute 32-lane runs");
  static constexpr int PADSH = S;
  static constexpr int PADUN = U;
  static constexpr int MAP0 = M0;
  static constexpr int MAPL = ML;
  static constexpr int LDS = P::N + ((P::N >> S) << U);
};
template <class P>
using Swz = Lanes<P, kMapSigma, kMapSigma, 5>;

// A plan whose frame is owned by one wave and whose LDS slice is private to
// that wave: the engine's exchanges then need only a wave barrier (LDS
// requests of one wave complete in issue order), so the waves of a
// multi-wave block run their transforms decoupled (fir_psd_kernel).
template <class P>
struct WaveSync : P {
  static_assert(P::TF <= 64, "wave-private frames only");
  static constexpr bool WAVE_SYNC = true;
};
// The first passes of an N-point plan only (product of the radices L divides
// N): the engine stops with the L-point transforms of the N / L polyphase
// components x[k + (N/L) m] in registers, thread t holding butterfly j's
// outputs b[(j/Ns)*Ns*R + (j mod Ns) + r*Ns] of the last pass -- i.e.
// component k = j / Ns, bins (j mod Ns) + r*Ns (Stockham after L points).
// The decimating FIR replaces the N-point transform's remaining passes, the
// filter multiply and the fold by one multiply-sum over the components.
template <class P>
struct Partial : P {
  static constexpr bool valid() {
    int prod = 1;
    for (int q = 0; q < P::NP; ++q) { if (P::E % P::R[q]) return false; prod *= P::R[q]; }
    return P::N % prod == 0;
  }
};

template <class P, class = void>
struct wave_sync_of { static constexpr bool value = false; };
template <class P>
struct wave_sync_of<P, decltype(void(P::WAVE_SYNC))> { static constexpr bool value = P::WAVE_SYNC; };

template <class P>
__device__ __forceinline__ void plan_sync() {
  if constexpr (wave_sync_of<P>::value) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  } else {
    __syncthreads();
  }
}

// 0, but unknown to the optimiser (blocks CSE / LICM across FFT calls).
__device__ __forceinline__ int opaque_zero() {
  int z = 0;
  asm volatile("" : "+s"(z));
  return z;
}

// Twiddle sources for passes p >= 1.
//  TwTable  : the global per-plan table (one load per element and pass).
//  TwAnchors: per-thread register anchors w^a, a in {1, 8, 16, 24} (< R), read
//             once per persistent block from the table; w^r is rebuilt per
//             frame as anchor * w^(r mod 8) (a chain of at most 7 multiplies,
//             |error| <~ 10 ulp).  Keeps every global load out of the FFT, so a
//             prefetch of the next unit stays in flight across it (vmcnt is
//             retired in issue order).
struct TwTable { const float2* tw; };
struct TwAnchors { const float2* wa; };
//  TwAnchorsX: anchors, except that a pass whose butterflies all share one k
//             (one anchor set) and whose radix is at most 8 takes its R - 1
//             exact twiddles from wx (load_twx: a few VGPRs, no generated
//             powers; the correlator's radix-8 middle pass).
struct TwAnchorsX { const float2* wa; const float2* wx; };
//  TwLds    : a two-level table in LDS, W_N^m = A[m >> S] * B[m & (2^S - 1)]
//             (S = ceil(log2 N / 2); <= 256 entries, 2 KB), filled once per
//             block from global memory: LDS latency instead of an L2 round
//             trip per pass, one extra complex multiply per twiddle.
struct TwLds { const float2* t2; };
//  TwRegs   : every twiddle the thread applies, exact (from the table), held in
//             VGPRs for the life of the block: no loads and no generating
//             multiplies inside the transforms.  Thread t's butterflies in pass
//             p are j = t + b*TF, so when TF is a multiple of Ns they share one
//             k = j mod Ns and one set of R-1 twiddles; small plans (the FIR's
//             1024 points: 3 + 15 values) fit.
struct TwRegs { const float2* w; };

constexpr int ilog2c(int n) { int l = 0; while ((1 << l) < n) ++l; return l; }
template <class P> constexpr int tw2_shift() { return (ilog2c(P::N) + 1) / 2; }
template <class P> constexpr int tw2_hi() { return P::N >> tw2_shift<P>(); }
template <class P> constexpr int tw2_size() { return tw2_hi<P>() + (1 << tw2_shift<P>()); }

// Copy the global two-level table (A then B, built on the host) into LDS.
template <class P>
__device__ __forceinline__ void load_tw2(float2* t2, const float2* __restrict__ g, int tid, int nthreads) {
  for (int i = tid; i < tw2_size<P>(); i += nthreads) t2[i] = g[i];
}

template <class P>
constexpr int rtw_nb(int p) { return (P::TF % P::ns(p) == 0) ? 1 : P::E / P::R[p]; }
template <class P>
constexpr int rtw_off(int p) {
  int o = 0;
  for (int q = 1; q < p; ++q) o += rtw_nb<P>(q) * (P::R[q] - 1);
  return o;
}
template <class P>
constexpr int rtw_total() { return rtw_off<P>(P::NP) > 0 ? rtw_off<P>(P::NP) : 1; }

// Load thread t's exact twiddles (TwRegs) from the per-pass table.
template <class P>
__device__ __forceinline__ void load_rtw(float2* w, const float2* __restrict__ tw, int t) {
  static_for<1, P::NP>([&](auto pi) {
    constexpr int p = decltype(pi)::value;
    constexpr int R = P::R[p], Ns = P::ns(p), NB = rtw_nb<P>(p);
    static_for<0, NB>([&](auto bi) {
      constexpr int b = decltype(bi)::value;
      const int k = bfly<P, p>(t, b) & (Ns - 1);
#pragma unroll
      for (int r = 1; r < R; ++r) w[rtw_off<P>(p) + b * (R - 1) + r - 1] = tw[P::twoff(p) + (r - 1) * Ns + k];
    });
  });
}

template <class P>
constexpr int nanch(int p) { return 1 + (P::R[p] - 1) / 8; }
template <class P>
constexpr int anch_nb(int p);
// passes TwAnchorsX serves from exact register twiddles, and their offsets
template <class P>
constexpr bool twx_pass(int p) { return p >= 1 && p < P::NP && P::R[p] <= 8 && anch_nb<P>(p) == 1; }
template <class P>
constexpr int twx_off(int p) {
  int o = 0;
  for (int q = 1; q < p; ++q) o += twx_pass<P>(q) ? P::R[q] - 1 : 0;
  return o;
}
template <class P>
constexpr int twx_total() { return twx_off<P>(P::NP) > 0 ? twx_off<P>(P::NP) : 1; }
// anchor sets per thread in pass p: one per butterfly, or a single one when
// every butterfly j = m(t) + b TF of the thread has the same k = j mod Ns
// (TF a multiple of Ns, maps other than kMapIlv)
template <class P>
constexpr int anch_nb(int p) {
  return (P::TF % P::ns(p) == 0 && !(p == 0 && map0_of<P>::value == kMapIlv) &&
          !(p == P::NP - 1 && mapl_of<P>::value == kMapIlv))
             ? 1 : P::E / P::R[p];
}
template <class P>
constexpr int anch_off(int p) {
  int o = 0;
  for (int q = 1; q < p; ++q) o += anch_nb<P>(q) * nanch<P>(q);
  return o;
}
template <class P>
constexpr int nanch_total() { return anch_off<P>(P::NP) > 0 ? anch_off<P>(P::NP) : 1; }

// Load this thread's exact twiddles of the twx_pass passes (TwAnchorsX).
template <class P>
__device__ __forceinline__ void load_twx(float2* wx, const float2* __restrict__ tw, int t) {
  static_for<1, P::NP>([&](auto pi) {
    constexpr int p = decltype(pi)::value;
    if constexpr (twx_pass<P>(p)) {
      constexpr int R = P::R[p], Ns = P::ns(p);
      const int k = bfly<P, p>(t, 0) & (Ns - 1);
#pragma unroll
      for (int r = 1; r < R; ++r) wx[twx_off<P>(p) + r - 1] = tw[P::twoff(p) + (r - 1) * Ns + k];
    }
  });
}

// Load this thread's anchors (thread t of its frame).
template <class P>
__device__ __forceinline__ void load_anchors(float2* wa, const float2* __restrict__ tw, int t) {
  static_for<1, P::NP>([&](auto pi) {
    constexpr int p = decltype(pi)::value;
    constexpr int Ns = P::ns(p), B = anch_nb<P>(p), NA = nanch<P>(p);
    static_for<0, B>([&](auto bi) {
      constexpr int b = decltype(bi)::value;
      const int k = bfly<P, p>(t, b) & (Ns - 1);
      static_for<0, NA>([&](auto ai) {
        constexpr int a = decltype(ai)::value;
        constexpr int r = a == 0 ? 1 : 8 * a;
        wa[anch_off<P>(p) + b * NA + a] = tw[P::twoff(p) + (r - 1) * Ns + k];
      });
    });
  });
}

// stage p: twiddle (p > 0) + register DFT for each of this thread's butterflies.
// hook() runs in the last pass after all of its twiddle loads have been issued
// and consumed, before the DFTs: a persistent kernel issues its next-unit
// prefetch there, so no later load in the unit has to wait behind it.
struct NoHook { __device__ __forceinline__ void operator()() const {} };

template <class P, int p, class TW>
__device__ __forceinline__ void fft_twiddle(float2* v, TW tws, int t, int b) {
  constexpr int R = P::R[p];
  constexpr int Ns = P::ns(p);
  if constexpr (std::is_same<TW, TwTable>::value) {
    const unsigned j = (unsigned)bfly<P, p>(t, b);
    const unsigned k = j & (Ns - 1);
    const float2* twp = tws.tw + P::twoff(p);
#pragma unroll
    for (int r = 1; r < R; ++r) v[b * R + r] = cmul(v[b * R + r], twp[k + (unsigned)((r - 1) * Ns)]);
  } else if constexpr (std::is_same<TW, TwRegs>::value) {
    constexpr int NB = rtw_nb<P>(p);
    const float2* wp = tws.w + rtw_off<P>(p) + (NB == 1 ? 0 : b) * (R - 1);
#pragma unroll
    for (int r = 1; r < R; ++r) v[b * R + r] = cmul(v[b * R + r], wp[r - 1]);
  } else if constexpr (std::is_same<TW, TwAnchorsX>::value && twx_pass<P>(p)) {
    const float2* wp = tws.wx + twx_off<P>(p);
#pragma unroll
    for (int r = 1; r < R; ++r) v[b * R + r] = cmul(v[b * R + r], wp[r - 1]);
  } else if constexpr (std::is_same<TW, TwLds>::value) {
    constexpr int S = tw2_shift<P>();
    constexpr int stride = P::N / (Ns * R);       // W_{Ns R}^{rk} = W_N^{rk stride}
    const int j = bfly<P, p>(t, b);
    const int k = j & (Ns - 1);
    const float2* A = tws.t2;
    const float2* Bt = tws.t2 + tw2_hi<P>();
#pragma unroll
    for (int r = 1; r < R; ++r) {
      const int m = k * (r * stride);
      const float2 w = cmul(A[m >> S], Bt[m & ((1 << S) - 1)]);
      v[b * R + r] = cmul(v[b * R + r], w);
    }
  } else {
    static_assert(std::is_same<TW, TwAnchors>::value || std::is_same<TW, TwAnchorsX>::value,
                  "twiddle source");
    constexpr int NA = nanch<P>(p);
    const float2* wa = tws.wa + anch_off<P>(p) + (anch_nb<P>(p) == 1 ? 0 : b) * NA;
    const float2 w1 = wa[0];
    float2 cur = w1;
    // software-pipelined by one power: the next power's product and this
    // element's product alternate, so no packed op is followed by its
    // dependent (one wait state each otherwise, see Radix2Phased)
    static_for<1, R>([&](auto ri) {
      constexpr int r = decltype(ri)::value;
      constexpr bool adv = r + 1 < R && (r + 1) % 8 != 0;
      f2v tc;
      if constexpr (adv) tc = tov(cur) * tov(w1).xx;
      const f2v tv = tov(v[b * R + r]) * tov(cur).xx;
      float2 nxt = cur;
      if constexpr (adv) nxt = cmul_fin(cur, w1, tc);
      else if constexpr (r + 1 < R) nxt = wa[(r + 1) / 8];
      v[b * R + r] = cmul_fin(v[b * R + r], cur, tv);
      cur = nxt;
    });
  }
}

template <class P, int p, class TW, class H = NoHook>
__device__ __forceinline__ void fft_stage(float2* v, TW tws, int t, H hook = H{}) {
  constexpr int R = P::R[p];
  constexpr int B = P::E / R;
  if constexpr (p == P::NP - 1 && !std::is_same<H, NoHook>::value) {
    if constexpr (p > 0) {
#pragma unroll
      for (int b = 0; b < B; ++b) fft_twiddle<P, p>(v, tws, t, b);
    }
    __builtin_amdgcn_sched_barrier(0);
    hook();
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int b = 0; b < B; ++b) dft_reg<R>(v + b * R);
  } else {
#pragma unroll
    for (int b = 0; b < B; ++b) {
      if constexpr (p > 0) fft_twiddle<P, p>(v, tws, t, b);
      dft_reg<R>(v + b * R);
    }
  }
}

// lpad(base + c) for a compile-time c: multiples of 2^S become an immediate
// offset from lpad(base) (lpad(b + 16m) = lpad(b) + 17m at S = 4), so a pass
// needs one LDS base address per butterfly instead of one per element.
template <class P, int C, int X = 0>
__device__ __forceinline__ int lpad_off(int base, int base_pad) {
  constexpr int S = xpad<P, X>::S;
  if constexpr (C % (1 << S) == 0) return base_pad + C + padc<P, X>(C);
  else return lpadp<P, X>(base + C);
}

// Padded LDS index of butterfly j's output 0 in pass p, such that output r
// sits at store_base + C + pad(C), C = r Ns (pad(i) = padc: (i >> S) << U):
// the destination base + C, base = hi + lo with hi = (j / Ns) Ns R, lo = j
// mod Ns, pads as
//   Ns >= 2^S : lpad(base) + C + pad(C)               (C a multiple of 2^S);
//   Ns <  2^S : base + pad(hi) + C + pad(C)           (lo + C never carries
//               past bit S into hi's multiple of 2^S, or stays below Ns R <=
//               2^S) -- one address per butterfly, immediate offsets per r.
template <class P, int p>
__device__ __forceinline__ int store_base(int j) {
  constexpr int R = P::R[p];
  constexpr int Ns = P::ns(p);
  constexpr int X = p + 1;                       // the exchange pass p stores into
  constexpr int S = xpad<P, X>::S;
  const int hi = (j / Ns) * Ns * R;
  const int base = hi + (j & (Ns - 1));
  if constexpr (Ns >= (1 << S)) return lpadp<P, X>(base);
  else return base + padc<P, X>(hi);
}

template <class P, int p>
__device__ __forceinline__ void fft_store(const float2* v, float2* lds, int t) {
  constexpr int R = P::R[p];
  constexpr int Ns = P::ns(p);
  constexpr int B = P::E / R;
  static_for<0, B>([&](auto bi) {
    constexpr int b = decltype(bi)::value;
    const int j = bfly<P, p>(t, b);
    const int bp = store_base<P, p>(j);
    static_for<0, R>([&](auto ri) {
      constexpr int r = decltype(ri)::value;
      constexpr int C = r * Ns;
      lds[bp + C + padc<P, p + 1>(C)] = v[b * R + r];
    });
  });
}

template <class P, int p>
__device__ __forceinline__ void fft_load(float2* v, const float2* lds, int t) {
  constexpr int R = P::R[p];
  constexpr int B = P::E / R;
  if constexpr (pass_map<P, p>() == kMapIlv) {
    // butterflies 2t, 2t + 1 share one padded base (never split by a pad:
    // S >= 1); with U = 1 the base is even, so each r is one 16-byte read
    static_assert(B == 2 && (P::N / R) % (1 << xpad<P, p>::S) == 0, "interleaved pairs");
    const int jb = bfly<P, p>(t, 0);
    const int jp = lpadp<P, p>(jb);
    static_for<0, B>([&](auto bi) {
      constexpr int b = decltype(bi)::value;
      static_for<0, R>([&](auto ri) {
        constexpr int r = decltype(ri)::value;
        v[b * R + r] = lds[jp + b + r * (P::N / R) + padc<P, p>(r * (P::N / R))];
      });
    });
  } else {
    const int tl = tpass<P, p>(t);
    const int tp = lpadp<P, p>(tl);
    static_for<0, B>([&](auto bi) {
      constexpr int b = decltype(bi)::value;
      static_for<0, R>([&](auto ri) {
        constexpr int r = decltype(ri)::value;
        v[b * R + r] = lds[lpad_off<P, b * P::TF + r * (P::N / R), p>(tl, tp)];
      });
    });
  }
}

// Split exchange: real and imaginary parts go through an LDS buffer of N
// floats in two rounds (4 barriers instead of 2), halving the LDS a frame
// needs so two 16384-point blocks fit on one CU.
template <class P, int p, int C>
__device__ __forceinline__ void fft_store_c(const float2* v, float* lds, int t) {
  constexpr int R = P::R[p];
  constexpr int Ns = P::ns(p);
  constexpr int B = P::E / R;
  static_for<0, B>([&](auto bi) {
    constexpr int b = decltype(bi)::value;
    const int j = bfly<P, p>(t, b);
    const int bp = store_base<P, p>(j);
    static_for<0, R>([&](auto ri) {
      constexpr int r = decltype(ri)::value;
      constexpr int O = r * Ns;
      lds[bp + O + padc<P, p + 1>(O)] = C == 0 ? v[b * R + r].x : v[b * R + r].y;
    });
  });
}

template <class P, int p, int C>
__device__ __forceinline__ void fft_load_c(float2* v, const float* lds, int t) {
  constexpr int R = P::R[p];
  constexpr int B = P::E / R;
  static_assert(pass_map<P, p>() != kMapIlv, "split exchange: plain maps only");
  const int tl = tpass<P, p>(t);
  const int tp = lpadp<P, p>(tl);
  static_for<0, B>([&](auto bi) {
    constexpr int b = decltype(bi)::value;
    static_for<0, R>([&](auto ri) {
      constexpr int r = decltype(ri)::value;
      const float f = lds[lpad_off<P, b * P::TF + r * (P::N / R), p>(tl, tp)];
      if constexpr (C == 0) v[b * R + r].x = f; else v[b * R + r].y = f;
    });
  });
}

template <class P, int p, class TW>
__device__ __forceinline__ void fft_tail_split(float2* v, float* lds, TW tws, int t) {
  if constexpr (p < P::NP) {
    plan_sync<P>();
    fft_store_c<P, p - 1, 0>(v, lds, t);
    plan_sync<P>();
    fft_load_c<P, p, 0>(v, lds, t);
    plan_sync<P>();
    fft_store_c<P, p - 1, 1>(v, lds, t);
    plan_sync<P>();
    fft_load_c<P, p, 1>(v, lds, t);
    fft_stage<P, p>(v, tws, t);
    fft_tail_split<P, p + 1>(v, lds, tws, t);
  }
}

// Two-level LDS twiddles + split exchange (LDS: P::LDS floats + the table).
template <class P>
__device__ __forceinline__ void fft_frame_split(float2* v, float* lds, const float2* t2, int t) {
  static_assert(P::valid(), "invalid FFT plan");
  fft_stage<P, 0>(v, TwLds{t2}, t);
  fft_tail_split<P, 1>(v, lds, TwLds{t2}, t);
}

template <class P, int p, class TW, class H = NoHook>
__device__ __forceinline__ void fft_tail(float2* v, float2* lds, TW tws, int t, H hook = H{}) {
  if constexpr (p < P::NP) {
    plan_sync<P>();               // previous readers of lds are done
    fft_store<P, p - 1>(v, lds, t);
    plan_sync<P>();
    fft_load<P, p>(v, lds, t);
    fft_stage<P, p>(v, tws, t, hook);
    fft_tail<P, p + 1>(v, lds, tws, t, hook);
  }
}

// Full forward FFT of one frame.  v holds the pass-0 operands on entry and the
// natural-order spectrum (index j + r*N/RL) on exit.  Contains block barriers:
// every thread of the block must call it.
template <class P>
__device__ __forceinline__ void fft_frame(float2* v, float2* lds, const float2* tw, int t) {
  static_assert(P::valid(), "invalid FFT plan");
  // Launder the table offset: a kernel running two FFTs (overlap-save) would
  // otherwise have its twiddle loads CSE'd across them and keep every twiddle
  // of the first FFT live in VGPRs until the second.  (An opaque zero offset,
  // not the pointer itself, so the loads stay global_load, not flat_load.)
  tw += opaque_zero();
  fft_stage<P, 0>(v, TwTable{tw}, t);
  fft_tail<P, 1>(v, lds, TwTable{tw}, t);
}

// Opaque to the optimiser: stops LICM from hoisting the per-frame twiddle
// powers (loop-invariant functions of the anchors) out of a persistent loop,
// which would pin every twiddle of the plan in VGPRs.
template <class P>
__device__ __forceinline__ void launder_anchors(float2* wa) {
#pragma unroll
  for (int i = 0; i < nanch_total<P>(); ++i) asm volatile("" : "+v"(wa[i].x), "+v"(wa[i].y));
}

// Two-level LDS twiddles (see TwLds); t2 must be filled before the call.
template <class P>
__device__ __forceinline__ void fft_frame_t2(float2* v, float2* lds, const float2* t2, int t) {
  static_assert(P::valid(), "invalid FFT plan");
  fft_stage<P, 0>(v, TwLds{t2}, t);
  fft_tail<P, 1>(v, lds, TwLds{t2}, t);
}

// Table twiddles + a hook in the last pass (see fft_stage).
template <class P, class H>
__device__ __forceinline__ void fft_frame_hook(float2* v, float2* lds, const float2* tw, int t,
                                               H hook) {
  static_assert(P::valid(), "invalid FFT plan");
  tw += opaque_zero();
  fft_stage<P, 0>(v, TwTable{tw}, t, hook);
  fft_tail<P, 1>(v, lds, TwTable{tw}, t, hook);
}

// The same with register-resident twiddle anchors (see TwAnchors).
template <class P>
__device__ __forceinline__ void fft_frame_anch(float2* v, float2* lds, float2* wa, int t) {
  static_assert(P::valid(), "invalid FFT plan");
  launder_anchors<P>(wa);
  fft_stage<P, 0>(v, TwAnchors{wa}, t);
  fft_tail<P, 1>(v, lds, TwAnchors{wa}, t);
}

// Two independent frames a, d through one LDS buffer, interleaved so that every
// LDS store of one frame is followed by register work of the other (the store
// drains while the butterflies issue; the barrier's lgkmcnt(0) then finds it
// done; left to the scheduler: pinning that order with sched_barrier / register
// fences measured slower).  Same barrier count as two back-to-back fft_frame calls:
//   stage0(a) store(a) stage0(d) | B load(a) B store(d) stage1(a) | B load(d) B
//   store(a) stage1(d) | ... | B load(d) stageL(d)
// Begins with a barrier (the buffer's previous readers are done).
template <class P, int p, class TW>
__device__ __forceinline__ void fft_pair_tail(float2* a, float2* d, float2* lds, TW tws, int t) {
  // entry: LDS holds a's pass p-1 output; d finished stage p-1 in registers
  plan_sync<P>();
  fft_load<P, p>(a, lds, t);
  plan_sync<P>();
  fft_store<P, p - 1>(d, lds, t);
  fft_stage<P, p>(a, tws, t);
  plan_sync<P>();
  fft_load<P, p>(d, lds, t);
  if constexpr (p + 1 < P::NP) {
    plan_sync<P>();
    fft_store<P, p>(a, lds, t);
    fft_stage<P, p>(d, tws, t);
    fft_pair_tail<P, p + 1>(a, d, lds, tws, t);
  } else {
    fft_stage<P, p>(d, tws, t);
  }
}

// hook() runs after a's first stage is stored, before d's first stage: a
// caller finishing d's operands there (e.g. a spectrum multiply whose loads
// were issued before the call) overlaps that work's latency with a's stage.
template <class P, class TW, class H = NoHook>
__device__ __forceinline__ void fft_pair(float2* a, float2* d, float2* lds, TW tws, int t,
                                         H hook = H{}) {
  static_assert(P::valid() && P::NP >= 2, "invalid FFT plan");
  plan_sync<P>();
  fft_stage<P, 0>(a, tws, t);
  fft_store<P, 0>(a, lds, t);
  hook();
  fft_stage<P, 0>(d, tws, t);
  fft_pair_tail<P, 1>(a, d, lds, tws, t);
}

// Index helpers for the operand / result layout.
template <class P>
__device__ __forceinline__ int in_index(int t, int e) {          // pass-0 operand e of thread t
  constexpr int R = P::R[0];
  return bfly<P, 0>(t, e / R) + (e % R) * (P::N / R);
}
template <class P>
__device__ __forceinline__ int out_index(int t, int e) {         // result e of thread t
  constexpr int R = P::RL;
  return bfly<P, P::NP - 1>(t, e / R) + (e % R) * (P::N / R);
}
// in_index(t, e) - in_index(t, 0) and out_index(t, e) - out_index(t, 0): the
// same for every thread under the lane maps other than kMapIlv (one per-lane
// base address plus compile-time offsets per element)
template <class P>
constexpr int in_off(int e) {
  static_assert(map0_of<P>::value != kMapIlv, "per-lane constant offsets");
  return (e / P::R[0]) * P::TF + (e % P::R[0]) * (P::N / P::R[0]);
}
template <class P>
constexpr int out_off(int e) {
  static_assert(mapl_of<P>::value != kMapIlv, "per-lane constant offsets");
  return (e / P::RL) * P::TF + (e % P::RL) * (P::N / P::RL);
}

// ---------------------------------------------------------------------------
// The plans instantiated by the library (N -> elements/thread, radices).
// Plans used by the overlap-save kernels are palindromic in their first/last
// radix so the forward FFT's result layout is the inverse FFT's operand layout.
// ---------------------------------------------------------------------------
using Plan64 = Plan<64, 8, 8, 8>;
using Plan128 = Plan<128, 16, 8, 16>;
using Plan256 = Plan<256, 16, 16, 16>;
using Plan512 = Plan<512, 16, 8, 8, 8>;
using Plan1024 = Plan<1024, 32, 32, 32>;
using Plan2048 = Plan<2048, 32, 8, 32, 8>;
using Plan4096 = Plan<4096, 16, 16, 16, 16>;
using Plan8192 = Plan<8192, 32, 16, 32, 16>;
using Plan16384 = Plan<16384, 16, 16, 4, 16, 16>;
// Overlap-save alternatives: 512-thread 16k plan; one-wave 1k / 2k plans.
using Plan16384w = Plan<16384, 32, 32, 16, 32>;
using Plan1024s = Plan<1024, 16, 16, 4, 16>;
using Plan2048s = Plan<2048, 32, 8, 32, 8>;
// Inverse transforms of the decimating FIR (fold of a Plan1024s spectrum by
// D = 2 / 4, same 64 threads): thread t holds bins t + 64 r of both.
using Plan512d = Plan<512, 8, 8, 8, 8>;
using Plan256d = Plan<256, 4, 4, 4, 4, 4>;
// Plan256d's second exchange (pass 1 stores at (j / 4) 16 + j % 4 + 4 r) puts
// 16 lanes on 4 bank pairs under 1 pad per 16 (4-way, 96 extra LDS cycles per
// FIR wave, = SQ_LDS_BANK_CONFLICT / wave of the D = 4 FIR); 4 pads per 16
// spread them over all 32 banks.  Exchanges 1 and 3 are conflict-free as they
// are (tools/ldssim.py models every exchange of fir_poly_kernel / fir_dec_kernel).
template <>
struct xpad<Plan256d, 2> {
  static constexpr int S = 4;
  static constexpr int U = 2;
};
// Polyphase front of the D = 4 decimating FIR: the two radix-16 passes of a
// 1024-point transform = the 256-point spectra of its 4 polyphase components
// (pass-1 twiddles = Plan256's table).
using Plan1024q = Lanes<Partial<Plan<1024, 16, 16, 16>>, kMapPair, kMapId>;
// The D = 1 FIR's one-wave overlap-save plan with the pair map in its first and
// last pass (16-byte segment loads, conflict-free exchanges).
using Plan1024x = Lanes<Plan1024s, kMapPair, kMapPair>;
// Its second exchange (pass 1 stores, pass 2 pair-map loads pair(t) + 64 r)
// puts lanes t and t + 16 of a 16-lane load group on one bank under 1 pad per
// 32 (2-way: 256 extra LDS cycles per D = 1 FIR wave, = the c2 PMC's
// SQ_LDS_BANK_CONFLICT / wave); 1 pad per 16 there is conflict-free for both
// sides (tools/ldssim.py).
template <>
struct xpad<Plan1024x, 2> {
  static constexpr int S = 4;
  static constexpr int U = 0;
};
// The correlator's / PSD's 8192-point plan with conflict-free exchanges (Swz).
using Plan8192x = Swz<Plan8192>;
// The correlator's 8192-point halves: radices 32 / 8 / 32.  Against 16 / 32 /
// 16 the middle pass's four radix-8 butterflies per thread share one k (TF a
// multiple of Ns = 32), so its twiddles come from one anchor (6 generated
// powers per transform instead of 27) and the last pass's 31 from four
// (27 instead of 2 x 13); the register DFTs cost the same.  The identity map
// keeps the radix-32 first pass's stores conflict-free (16-lane groups write
// 33 j + r: distinct banks for 16 consecutive j; the sigma map's even j would
// meet 2-way) and its segment loads 512-byte runs per wave.
using Plan8192c = Lanes<Plan<8192, 32, 32, 8, 32>, kMapId, kMapId, 5>;
// The PSD's 8192-point plan with interleaved first / last passes (16-byte
// frame loads, 8-byte |X|^2 stores, conflict-free exchanges).
using Plan8192i = Lanes<Plan8192, kMapIlv, kMapIlv, 5, 1>;
// Its second exchange's 16-byte pair reads (2t + 512 r: ds_read_b128 lane groups
// of 16) meet 2-way on banks under 2 pads per 32; 2 pads per 64 spreads them
// (tools/ldssim.py: 64 extra LDS cycles per wave and frame -> 0).
template <>
struct xpad<Plan8192i, 2> {
  static constexpr int S = 6;
  static constexpr int U = 1;
};

template <class P>
constexpr int block_threads() { return P::TF > 256 ? P::TF : 256; }

}  // namespace vsig
