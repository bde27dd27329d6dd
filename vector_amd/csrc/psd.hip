// Spectrum kernels (gfx950): psd_kernel (windowed block FFT -> |X|^2 * scale,
// spectrum / create_spectrogram), spectrum_prep (FFT of a zero-padded short
// vector: filter taps / correlation template), the FFT engine micro-benchmark,
// plan geometry queries.  No MFMA: no dense contraction on this path.
#include "os_common.hpp"

namespace vsig {

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
    v[e] = (active && i < nperseg) ? ld_stream<true>(xf + (long long)i * stride) : make_float2(0.f, 0.f);
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
  long long u = PERSIST == 6 ? stage_bid<2>() : blockIdx.x;
  if (u >= units) return;
  if constexpr (PERSIST == 5 || PERSIST == 6) {   // register twiddle anchors; 6: two frames (fft_pair)
    if constexpr (FPB != 1) return;                // launch_psd only picks these for TF >= 256
    constexpr int NF = PERSIST == 6 ? 2 : 1;
    float2 wa[nanch_total<P>()];
    load_anchors<P>(wa, tw, t);
    float2 v[NF][P::E];
#pragma unroll
    for (int f = 0; f < NF; ++f) {
      psd_load<P>(v[f], x, stride, nperseg, hop, u * NF + f, nframes, t);
#pragma unroll
      for (int e = 0; e < P::E; ++e) {
        const int i = in_index<P>(t, e);
        const float w = i < nperseg ? win[i] : 0.f;
        v[f][e] = make_float2(v[f][e].x * w, v[f][e].y * w);
      }
    }
    launder_anchors<P>(wa);
    if constexpr (NF == 2) fft_pair<P>(v[0], v[1], lds, TwAnchors{wa}, t);
    else fft_frame_anch<P>(v[0], lds, wa, t);
#pragma unroll
    for (int f = 0; f < NF; ++f) {
      const long long frame = u * NF + f;
      if (frame < nframes) {
        float* of = out + frame * P::N;
#pragma unroll
        for (int e = 0; e < P::E; ++e) {
          const int i = out_index<P>(t, e);
          const int o = shift ? ((i + P::N / 2) & (P::N - 1)) : i;
          __builtin_nontemporal_store((v[f][e].x * v[f][e].x + v[f][e].y * v[f][e].y) * scale, of + o);
        }
      }
    }
    return;
  }
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
        __builtin_nontemporal_store((v[e].x * v[e].x + v[e].y * v[e].y) * scale, of + o);
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
        __builtin_nontemporal_store((v[e].x * v[e].x + v[e].y * v[e].y) * scale, of + o);
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
        __builtin_nontemporal_store((v[e].x * v[e].x + v[e].y * v[e].y) * scale, of + o);
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
          __builtin_nontemporal_store((v[e].x * v[e].x + v[e].y * v[e].y) * scale, of + o);
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
        __builtin_nontemporal_store((v[e].x * v[e].x + v[e].y * v[e].y) * scale, of + o);
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

// The correlator's engine configuration: register twiddle anchors, two blocks
// per CU; PAIR = 1: two frames per block through fft_pair (the half-frame
// correlator's inner loop without its loads, multiply and epilogue).
template <class P, int PAIR>
__global__ __launch_bounds__(P::TF, 2) void fft_bench_anch_kernel(float2* __restrict__ io, int iters,
                                                                  const float2* __restrict__ tw) {
  __shared__ float2 lds[P::LDS];
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

// Grid cap of the persistent variants (0: every resident slot).  A cap of one
// block per CU leaves the other slot to a concurrently launched correlator.
static int g_psd_grid_cap = 0;
void set_psd_grid_cap(int cap) { g_psd_grid_cap = cap; }

template <class PL, int PERSIST>
void launch_psd_t(const float2* x, long long stride, const float* win, int nperseg, long long hop,
                  float scale, float* out, long long nframes, int shift, const float2* tw,
                  hipStream_t st) {
  constexpr int BT = block_threads<PL>();
  constexpr int FPB = BT / PL::TF;
  const long long units = (nframes + FPB - 1) / FPB;
  long long grid =
      (PERSIST == 1 || PERSIST == 2) ? persistent_grid(psd_kernel<PL, PERSIST>, BT, units)
      : PERSIST == 6 ? (units + 1) / 2 : units;
  if ((PERSIST == 1 || PERSIST == 2) && g_psd_grid_cap > 0 && grid > g_psd_grid_cap)
    grid = g_psd_grid_cap;
  hipLaunchKernelGGL((psd_kernel<PL, PERSIST>), dim3((unsigned)grid), dim3(BT), 0, st, x, stride,
                     win, nperseg, hop, scale, out, nframes, shift, tw);
}

hipError_t launch_psd(int N, const float2* x, long long stride, const float* win, int nperseg,
                      long long hop, float scale, float* out, long long nframes, int shift,
                      const float2* tw, int variant, hipStream_t st) {
  if (nframes <= 0) return hipSuccess;
  VSIG_PLAN_SWITCH(N, {
    // bits 5/6 (anchors, frame pairs) need one frame per block (TF >= 256);
    // smaller plans take the split-exchange kernel instead.
    const bool big = PL::TF >= 256;
    if ((variant & 64) && big) launch_psd_t<PL, 6>(x, stride, win, nperseg, hop, scale, out, nframes, shift, tw, st);
    else if ((variant & 32) && big) launch_psd_t<PL, 5>(x, stride, win, nperseg, hop, scale, out, nframes, shift, tw, st);
    else if (variant & (16 | 32 | 64)) launch_psd_t<PL, 4>(x, stride, win, nperseg, hop, scale, out, nframes, shift, tw, st);
    else if (variant & 8) launch_psd_t<PL, 3>(x, stride, win, nperseg, hop, scale, out, nframes, shift, tw, st);
    else if (variant & 4) launch_psd_t<PL, 2>(x, stride, win, nperseg, hop, scale, out, nframes, shift, tw, st);
    else if (variant & 1) launch_psd_t<PL, 1>(x, stride, win, nperseg, hop, scale, out, nframes, shift, tw, st);
    else launch_psd_t<PL, 0>(x, stride, win, nperseg, hop, scale, out, nframes, shift, tw, st);
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
  if (N == -512 || N == -256) {     // decimating-FIR inverse plans
    const int np = N == -512 ? Plan512d::NP : Plan256d::NP;
    *npasses = np;
    for (int q = 0; q < np; ++q) radices[q] = N == -512 ? Plan512d::R[q] : Plan256d::R[q];
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
