// Spectrum kernels (gfx950): psd_kernel (windowed block FFT -> |X|^2 * scale,
// spectrum / create_spectrogram), spectrum_prep (FFT of a zero-padded short
// vector: filter taps / correlation template), the FFT engine micro-benchmark,
// plan geometry queries.  No MFMA: no dense contraction on this path.
#include "os_common.hpp"

namespace vsig {

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
    v[e] = (active && i < nperseg) ? ld_stream<true>(xf + (long long)i * stride) : make_float2(0.f, 0.f);
  }
}

// Plans of >= 256 threads per frame (nfft >= 4096): two frames per block
// through fft_pair (the LDS stores of one frame overlap the other's
// butterflies), twiddles from register anchors.  (The conflict-free Plan8192x
// exchange that the correlator uses measured slower here -- 1.43 vs 1.17 ms at
// config 5: at 254 VGPRs the sigma map's extra registers spill.)
template <class P>
__global__ __launch_bounds__(P::TF) void psd_pair_kernel(
    const float2* __restrict__ x, long long stride, const float* __restrict__ win, int nperseg,
    long long hop, float scale, float* __restrict__ out, long long nframes, int shift,
    const float2* __restrict__ tw, bool x4, unsigned long long* clk) {
  static_assert(P::TF >= 256, "one frame per block");
  __shared__ __attribute__((aligned(16))) float2 lds[lds_size<P>()];
  const int t = threadIdx.x;
  const ClockStamp cs(clk, blockIdx.x);
  const long long u = blockIdx.x;
  float2 wa[nanch_total<P>()];
  load_anchors<P>(wa, tw, t);
  float2 v[2][P::E];
  constexpr bool ILV = map0_of<P>::value == kMapIlv && mapl_of<P>::value == kMapIlv;
  // interleaved plans (Plan8192i): thread t's operands are x[2t + b + (N/R0) r],
  // b < 2 -- one 16-byte load per r -- when the frames are contiguous, full
  // and 16-byte aligned (uniform per launch: stride 1, nperseg = N, even hop,
  // aligned x; the caller's flag x4)
  if constexpr (ILV) {
    static_assert(P::E == 2 * P::R[0] && P::E == 2 * P::RL, "two butterflies per thread");
    if (x4) {
      typedef float f4 __attribute__((ext_vector_type(4)));
      constexpr int R0 = P::R[0], S0 = P::N / R0;
#pragma unroll
      for (int f = 0; f < 2; ++f) {
        const long long frame = u * 2 + f;
        const bool active = frame < nframes;
        const float2* xf = x + (active ? frame * hop : 0);
#pragma unroll
        for (int r = 0; r < R0; ++r) {
          const int i = 2 * t + S0 * r;
          const f4 q = active ? __builtin_nontemporal_load(reinterpret_cast<const f4*>(xf + i))
                              : f4{0.f, 0.f, 0.f, 0.f};
          const f2v w2 = *reinterpret_cast<const f2v*>(win + i);   // packed: window broadcast
          v[f][r] = fromv((f2v){q.x, q.y} * w2.xx);
          v[f][R0 + r] = fromv((f2v){q.z, q.w} * w2.yy);
        }
      }
    }
  }
  if (!ILV || !x4) {
#pragma unroll
    for (int f = 0; f < 2; ++f) {
      psd_load<P>(v[f], x, stride, nperseg, hop, u * 2 + f, nframes, t);
#pragma unroll
      for (int e = 0; e < P::E; ++e) {
        const int i = in_index<P>(t, e);
        const float w = i < nperseg ? win[i] : 0.f;
        v[f][e] = make_float2(v[f][e].x * w, v[f][e].y * w);
      }
    }
  }
  launder_anchors<P>(wa);
  fft_pair<P>(v[0], v[1], lds, TwAnchors{wa}, t);
#pragma unroll
  for (int f = 0; f < 2; ++f) {
    const long long frame = u * 2 + f;
    if (frame < nframes) {
      float* of = out + frame * P::N;
      if constexpr (ILV) {
        // bins 2t + RLs r and the next one: one 8-byte store each (fftshift by
        // N/2 keeps the pair adjacent)
        typedef float f2 __attribute__((ext_vector_type(2)));
        constexpr int RL = P::RL, SL = P::N / RL;
#pragma unroll
        for (int r = 0; r < RL; ++r) {
          const int i = 2 * t + SL * r;
          const int o = shift ? ((i + P::N / 2) & (P::N - 1)) : i;
          const float2 a0 = v[f][r], a1 = v[f][RL + r];
          const f2 pw = {(a0.x * a0.x + a0.y * a0.y) * scale, (a1.x * a1.x + a1.y * a1.y) * scale};
          __builtin_nontemporal_store(pw, reinterpret_cast<f2*>(of + o));
        }
      } else {
#pragma unroll
        for (int e = 0; e < P::E; ++e) {
          const int i = out_index<P>(t, e);
          const int o = shift ? ((i + P::N / 2) & (P::N - 1)) : i;
          __builtin_nontemporal_store((v[f][e].x * v[f][e].x + v[f][e].y * v[f][e].y) * scale, of + o);
        }
      }
    }
  }
  cs.done(clk);
}

// Smaller plans (several frames per 256-thread block): two-level twiddle
// table in LDS and the real / imaginary parts exchanged in two rounds, so
// four blocks fit a CU.
template <class P>
__global__ __launch_bounds__(block_threads<P>(), (P::E <= 16 ? 4 : 1)) void psd_split_kernel(
    const float2* __restrict__ x, long long stride, const float* __restrict__ win, int nperseg,
    long long hop, float scale, float* __restrict__ out, long long nframes, int shift,
    const float2* __restrict__ tw) {
  constexpr int BT = block_threads<P>();
  constexpr int FPB = BT / P::TF;
  constexpr int FL = (lds_size<P>() + 1) / 2;
  __shared__ float2 lds[FPB * FL + tw2_size<P>()];
  const int fl = threadIdx.x / P::TF;
  const int t = threadIdx.x % P::TF;
  const long long u = blockIdx.x;
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
      __builtin_nontemporal_store((v[e].x * v[e].x + v[e].y * v[e].y) * scale, of + o);
    }
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
  __shared__ float2 lds[(BT / P::TF) * lds_size<P>()];
  const int fl = threadIdx.x / P::TF;
  const int t = threadIdx.x % P::TF;
  float2 v[P::E];
#pragma unroll
  for (int e = 0; e < P::E; ++e) {
    const int i = in_index<P>(t, e);
    v[e] = (fl == 0 && i < len) ? u[i] : make_float2(0.f, 0.f);
  }
  fft_frame<P>(v, lds + fl * lds_size<P>(), tw, t);
  if (fl != 0) return;
#pragma unroll
  for (int e = 0; e < P::E; ++e) {
    const int i = out_index<P>(t, e);
    S[i] = make_float2(v[e].x * gain, v[e].y * gain);
  }
}

#ifdef VSIG_TUNING
// ---------------------------------------------------------------------------
// Engine micro-benchmark (tuning only): `iters` back-to-back FFTs of one frame
// per block with no HBM traffic in the loop — the compute/LDS ceiling of a plan.
// ---------------------------------------------------------------------------
template <class P, int TWL>
__global__ __launch_bounds__(P::TF) void fft_bench_kernel(float2* __restrict__ io,
                                                                    int iters,
                                                                    const float2* __restrict__ tw) {
  __shared__ float2 lds[lds_size<P>() + (TWL ? tw2_size<P>() : 0)];
  const int t = threadIdx.x;
  float2* t2 = lds + lds_size<P>();
  if constexpr (TWL) load_tw2<P>(t2, tw, t, P::TF);
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

// The correlator's engine configuration: register twiddle anchors, two blocks
// per CU; PAIR = 1: two frames per block through fft_pair (the half-frame
// correlator's inner loop without its loads, multiply and epilogue).
template <class P, int PAIR>
__global__ __launch_bounds__(P::TF, 2) void fft_bench_anch_kernel(float2* __restrict__ io, int iters,
                                                                  const float2* __restrict__ tw) {
  __shared__ __attribute__((aligned(16))) float2 lds[lds_size<P>()];
  const int t = threadIdx.x;
  float2 wa[nanch_total<P>()];
  load_anchors<P>(wa, tw, t);
  float2 a[P::E], d[P::E];
  float2* f = io + (long long)blockIdx.x * P::N * (PAIR ? 2 : 1);
#pragma unroll
  for (int e = 0; e < P::E; ++e) {
    a[e] = f[in_index<P>(t, e)];
    d[e] = PAIR ? f[P::N + in_index<P>(t, e)] : make_float2(0.f, 0.f);
  }
  for (int it = 0; it < iters; ++it) {
    if constexpr (PAIR) {
      launder_anchors<P>(wa);
      fft_pair<P>(a, d, lds, TwAnchors{wa}, t);
    } else {
      fft_frame_anch<P>(a, lds, wa, t);
    }
#pragma unroll
    for (int e = 0; e < P::E; ++e) {
      a[e] = make_float2(a[e].x * 1e-4f, a[e].y * 1e-4f);
      if (PAIR) d[e] = make_float2(d[e].x * 1e-4f, d[e].y * 1e-4f);
    }
  }
#pragma unroll
  for (int e = 0; e < P::E; ++e) {
    f[out_index<P>(t, e)] = a[e];
    if (PAIR) f[P::N + out_index<P>(t, e)] = d[e];
  }
}

hipError_t launch_fft_bench(int key, float2* io, int frames, int iters, const float2* tw, int twl,
                            hipStream_t st) {
  if (twl >= 2) {          // anchors (2) / anchors + pair (3), 8192-point plan only
    if (key != 8192) return hipErrorInvalidValue;
    if (twl == 3)
      hipLaunchKernelGGL((fft_bench_anch_kernel<Plan8192, 1>), dim3(frames / 2), dim3(Plan8192::TF), 0,
                         st, io, iters, tw);
    else
      hipLaunchKernelGGL((fft_bench_anch_kernel<Plan8192, 0>), dim3(frames), dim3(Plan8192::TF), 0,
                         st, io, iters, tw);
    return hipGetLastError();
  }
#define VSIG_FB(PL)                                                                          \
  {                                                                                          \
    auto k = twl ? fft_bench_kernel<PL, 1> : fft_bench_kernel<PL, 0>;                         \
    hipLaunchKernelGGL(k, dim3(frames), dim3(PL::TF), 0, st, io, iters, tw);        \
  }
  switch (key) {
    case -1024: VSIG_FB(Plan1024s) break;
    case 4096: VSIG_FB(Plan4096) break;
    case 8192: VSIG_FB(Plan8192) break;
    case 16384: VSIG_FB(Plan16384) break;
    default: return hipErrorInvalidValue;
  }
#undef VSIG_FB
  return hipGetLastError();
}

#endif  // VSIG_TUNING

hipError_t launch_psd(int N, const float2* x, long long stride, const float* win, int nperseg,
                      long long hop, float scale, float* out, long long nframes, int shift,
                      const float2* tw, hipStream_t st) {
  if (nframes <= 0) return hipSuccess;
  if (N == 8192) {      // interleaved first / last pass: 16-byte loads, 8-byte stores
    const bool x4 = stride == 1 && nperseg == N && hop % 2 == 0 &&
                    (reinterpret_cast<uintptr_t>(x) & 15) == 0 && (reinterpret_cast<uintptr_t>(win) & 7) == 0;
    hipLaunchKernelGGL(psd_pair_kernel<Plan8192i>, dim3((unsigned)((nframes + 1) / 2)), dim3(Plan8192i::TF),
                       0, st, x, stride, win, nperseg, hop, scale, out, nframes, shift, tw, x4,
                       g_clock_sink);
    return hipGetLastError();
  }
  VSIG_PLAN_SWITCH(N, {
    if constexpr (PL::TF >= 256) {
      hipLaunchKernelGGL(psd_pair_kernel<PL>, dim3((unsigned)((nframes + 1) / 2)), dim3(PL::TF), 0,
                         st, x, stride, win, nperseg, hop, scale, out, nframes, shift, tw, false,
                         g_clock_sink);
    } else {
      constexpr int FPB = block_threads<PL>() / PL::TF;
      hipLaunchKernelGGL(psd_split_kernel<PL>, dim3((unsigned)((nframes + FPB - 1) / FPB)),
                         dim3(block_threads<PL>()), 0, st, x, stride, win, nperseg, hop, scale, out,
                         nframes, shift, tw);
    }
  });
  return hipGetLastError();
}

int psd_plan_threads(int N) {
  auto f = [](int n, int* tf) -> hipError_t {
    VSIG_PLAN_SWITCH(n, { *tf = PL::TF; });
    return hipSuccess;
  };
  int tf = 0;
  return f(N, &tf) == hipSuccess ? tf : 0;
}

hipError_t launch_spectrum_prep(int N, const float2* u, int len, float gain, float2* S,
                                const float2* tw, hipStream_t st) {
  VSIG_PLAN_SWITCH(N, {
    hipLaunchKernelGGL(spectrum_prep<PL>, dim3(1), dim3(block_threads<PL>()), 0, st, u, len,
                       gain, S, tw);
  });
  return hipGetLastError();
}

hipError_t tw2_info(int N, int* shift, int* hi) {
  if (N == -1024) { *shift = tw2_shift<Plan1024s>(); *hi = tw2_hi<Plan1024s>(); return hipSuccess; }
  VSIG_PLAN_SWITCH(N, { *shift = tw2_shift<PL>(); *hi = tw2_hi<PL>(); });
  return hipSuccess;
}

hipError_t plan_info(int N, int* radices, int* npasses) {
  if (N == -512 || N == -256) {     // decimating-FIR inverse plans
    const int np = N == -512 ? Plan512d::NP : Plan256d::NP;
    *npasses = np;
    for (int q = 0; q < np; ++q) radices[q] = N == -512 ? Plan512d::R[q] : Plan256d::R[q];
    return hipSuccess;
  }
  if (N == -1024) {                 // the one-wave overlap-save plan
    *npasses = Plan1024s::NP;
    for (int q = 0; q < Plan1024s::NP; ++q) radices[q] = Plan1024s::R[q];
    return hipSuccess;
  }
  if (N == -8192) {                 // the correlator halves' 8192-point plan
    *npasses = Plan8192c::NP;
    for (int q = 0; q < Plan8192c::NP; ++q) radices[q] = Plan8192c::R[q];
    return hipSuccess;
  }
  if (N == -16384) {                // the 512-thread plan (M = 32768 correlator halves)
    *npasses = Plan16384w::NP;
    for (int q = 0; q < Plan16384w::NP; ++q) radices[q] = Plan16384w::R[q];
    return hipSuccess;
  }
  VSIG_PLAN_SWITCH(N, {
    *npasses = PL::NP;
    for (int q = 0; q < PL::NP; ++q) radices[q] = PL::R[q];
  });
  return hipSuccess;
}

}  // namespace vsig
