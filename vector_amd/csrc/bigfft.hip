// Transforms longer than one LDS frame, and of any length (gfx950).
//
// Four-step FFT of M = N1 * N2 points (powers of two, N1 <= 16384,
// 512 <= N2 <= 16384, so M <= 2^28) on the in-LDS engine (fft_engine.hpp):
//   column pass : for each n2, X1[k1, n2] = FFT_N1 over n1 of x[n1 N2 + n2],
//                 times W_M^(n2 k1)        (strided loads / stores, F adjacent
//                 columns per block so a wave's lanes read F-sample runs);
//   row pass    : X[k1 + N1 k2] = FFT_N2 over n2 of X1[k1, n2] (contiguous rows);
// the spectrum stays in that permuted order (element k1 N2 + k2 holds
// X[k1 + N1 k2]) because every consumer here is element-wise: the PSD of long
// frames stores |X|^2 at its natural index, and Bluestein's convolution
// multiplies by a kernel spectrum kept in the same order and runs the inverse
// passes back (row inverse, conj twiddles, inverse column pass) to natural
// order.  Inverse transforms by conj: IFFT(v) = conj(FFT(conj(v))).
//
// Bluestein (chirp-z) for any length N: with c[n] = exp(-i pi n^2 / N),
//   X[k] = c[k] sum_n (x[n] c[n]) conj(c[k - n]),
// a linear convolution done circularly in M >= 2N - 1 points:
//   a = x c (zero-padded), B = FFT_M(b) / M with b[m] = conj(c[m]) for
//   |m| < N (wrapped), X = c * IFFT_M(FFT_M(a) B).
// M <= 16384: one block per frame does all of it in LDS (bf_small_kernel);
// larger: column pass (load x c) -> row pass (FFT, * B, IFFT, same block) ->
// inverse column pass (store c X).  The chirps are formed in double on the
// device from n^2 mod 2N (exact integers).
//
// Used by resample_signal (utils.py:107-118: scipy.signal.resample = FFT of
// any length, spectrum copy, inverse FFT of any length), the channel filter
// (vector_analyzer/split_channels.py:15-44: full-length FFT / IFFT) and the
// spectrogram for nfft > 16384 (utils.py:281-291 with a long window).
#include "os_common.hpp"

namespace vsig {

// ---------------------------------------------------------------------------
// element access functors (kernel arguments, by value)
// ---------------------------------------------------------------------------
struct BfIn {                 // operand n of frame f of a forward pass
  const void* src;
  int kind;                   // 0 complex64, 1 complex128 (converted), 2 none (zeros)
  long long fstride, estride; // frame f at f * fstride, element n at n * estride
  long long nvalid;           // n >= nvalid -> 0
  const float2* chirp;        // optional * chirp[n]
  const float* win;           // optional * win[n]
  int conj;                   // conj(x) first (inverse DFT)
  float scale;
  __device__ __forceinline__ float2 operator()(long long f, long long n) const {
    if (n >= nvalid || kind == 2) return make_float2(0.f, 0.f);
    const long long i = f * fstride + n * estride;
    float2 v;
    if (kind == 1) {
      const double2 d = static_cast<const double2*>(src)[i];
      v = make_float2((float)d.x, (float)d.y);
    } else {
      v = static_cast<const float2*>(src)[i];
    }
    if (conj) v = cconj(v);                  // inverse DFT: conj(x), then the chirp
    if (chirp) v = cmul(v, chirp[n]);
    if (win) { const float w = win[n]; v = make_float2(v.x * w, v.y * w); }
    return make_float2(v.x * scale, v.y * scale);
  }
};

struct BfOut {                // natural-order result n of frame f
  void* dst;
  int kind;                   // 0 complex64, 1 complex128, 2 float64 real part, 3 complex64 real part,
                              // 4 float32 |X|^2 * scale (PSD frames, optionally fftshift-ed)
  long long fstride;
  long long nout;             // store n < nout
  const float2* chirp;        // optional * chirp[n] (after conj)
  int conj;
  float scale;
  int shift;
  __device__ __forceinline__ void operator()(long long f, long long n, float2 v) const {
    if (n >= nout) return;
    if (chirp) v = cmul(v, chirp[n]);        // c[k] S[k], then conj (inverse DFT)
    if (conj) v = cconj(v);
    if (kind == 4) {                         // np.fft.fftshift: bin n at (n + nout // 2) % nout
      long long o = n;
      if (shift) { o = n + nout / 2; if (o >= nout) o -= nout; }
      static_cast<float*>(dst)[f * fstride + o] = (v.x * v.x + v.y * v.y) * scale;
      return;
    }
    v = make_float2(v.x * scale, v.y * scale);
    const long long i = f * fstride + n;
    switch (kind) {
      case 0: static_cast<float2*>(dst)[i] = v; break;
      case 1: static_cast<double2*>(dst)[i] = make_double2((double)v.x, (double)v.y); break;
      case 2: static_cast<double*>(dst)[i] = (double)v.x; break;
      default: static_cast<float2*>(dst)[i] = make_float2(v.x, 0.f); break;
    }
  }
};

// W_M^m from the two-level table: A[m >> S] * B[m & (2^S - 1)]
__device__ __forceinline__ float2 tw_big(const float2* __restrict__ t2, int S, int hiA,
                                         unsigned long long m) {
  return cmul(t2[m >> S], t2[hiA + (m & ((1ull << S) - 1))]);
}

template <class P>
constexpr int col_frames() {
  // adjacent columns per block: <= 1024 threads, LDS <= 140 KB
  constexpr int byT = 1024 / P::TF;
  constexpr int byL = 17920 / lds_size<P>();
  constexpr int f = byT < byL ? byT : byL;
  return f >= 64 ? 64 : f >= 32 ? 32 : f >= 16 ? 16 : f >= 8 ? 8 : f >= 4 ? 4 : f >= 2 ? 2 : 1;
}

// Column pass.  INV = 0: x (BfIn) -> FFT_N1 -> * W_M^(n2 k1) -> tmp[f][k1 N2 + n2].
// INV = 1: tmp[f][k1 N2 + n2] * conj(W_M^(n2 k1)) -> IFFT_N1 (conj trick) ->
// out(f, n1 N2 + n2) (BfOut).
template <class P, int INV>
__global__ __launch_bounds__(col_frames<P>() * P::TF) void bf_col_kernel(
    BfIn in, BfOut out, float2* __restrict__ tmp, int N2, long long M,
    const float2* __restrict__ tw, const float2* __restrict__ t2, int S, int hiA) {
  constexpr int F = col_frames<P>();
  __shared__ float2 lds[F * lds_size<P>()];
  const int tid = threadIdx.x;
  const int fl = tid % F, t = tid / F;
  const long long cols = N2 / F;                     // column groups per frame
  const long long f = blockIdx.x / cols;
  const int n2 = (int)(blockIdx.x % cols) * F + fl;
  float2* lf = lds + fl * lds_size<P>();
  float2* tf = tmp + f * M;
  float2 v[P::E];
#pragma unroll
  for (int e = 0; e < P::E; ++e) {
    const int k = in_index<P>(t, e);                  // n1 (fwd) or k1 (inv)
    if constexpr (INV) {
      const float2 w = tw_big(t2, S, hiA, (unsigned long long)n2 * (unsigned long long)k);
      v[e] = cconj(cmul(tf[(long long)k * N2 + n2], cconj(w)));
    } else {
      v[e] = in(f, (long long)k * N2 + n2);
    }
  }
  fft_frame<P>(v, lf, tw, t);
#pragma unroll
  for (int e = 0; e < P::E; ++e) {
    const int k = out_index<P>(t, e);                 // k1 (fwd) or n1 (inv)
    if constexpr (INV) {
      out(f, (long long)k * N2 + n2, cconj(v[e]));
    } else {
      const float2 w = tw_big(t2, S, hiA, (unsigned long long)n2 * (unsigned long long)k);
      tf[(long long)k * N2 + n2] = cmul(v[e], w);
    }
  }
}

template <class P>
constexpr int row_frames() {
  constexpr int byT = 1024 / P::TF;
  constexpr int byL = 17920 / lds_size<P>();
  constexpr int f = byT < byL ? byT : byL;
  return f >= 8 ? 8 : f >= 4 ? 4 : f >= 2 ? 2 : 1;
}

// Row pass over tmp[f][k1 N2 + n2] (rows k1, contiguous).
// MODE 0 (Bluestein): FFT_N2, * Bk[k1 N2 + k2], IFFT_N2 (conj trick), back to tmp.
// MODE 1 (kernel spectrum): FFT_N2 * scale back to tmp (permuted order).
// MODE 2 (PSD): |X|^2 * scale into psd[f][shift(k)], k = k1 + N1 k2 (float32).
// MODE 3: X * scale at its natural index into ((float2*) psd)[f][k].
template <class P, int MODE>
__global__ __launch_bounds__(row_frames<P>() * P::TF) void bf_row_kernel(
    float2* __restrict__ tmp, int N1, long long M, const float2* __restrict__ Bk,
    const float2* __restrict__ tw, float scale, float* __restrict__ psd, int shift) {
  static_assert(P::R[0] == P::RL, "in-register convolution needs a palindromic plan");
  constexpr int F = row_frames<P>();
  constexpr int N2 = P::N;
  __shared__ float2 lds[F * lds_size<P>()];
  const int fl = threadIdx.x / P::TF, t = threadIdx.x % P::TF;
  const long long rows = N1 / F;
  const long long f = blockIdx.x / rows;
  const long long k1 = (blockIdx.x % rows) * F + fl;
  float2* row = tmp + f * M + k1 * N2;
  float2* lf = lds + fl * lds_size<P>();
  float2 v[P::E];
#pragma unroll
  for (int e = 0; e < P::E; ++e) v[e] = row[in_index<P>(t, e)];
  fft_frame<P>(v, lf, tw, t);
  if constexpr (MODE == 0) {
    const float2* bk = Bk + k1 * N2;
#pragma unroll
    for (int e = 0; e < P::E; ++e) v[e] = cconj(cmul(v[e], bk[out_index<P>(t, e)]));
    fft_frame<P>(v, lf, tw + opaque_zero(), t);
#pragma unroll
    for (int e = 0; e < P::E; ++e) row[out_index<P>(t, e)] = cconj(v[e]);
  } else if constexpr (MODE == 1) {
#pragma unroll
    for (int e = 0; e < P::E; ++e) row[out_index<P>(t, e)] = make_float2(v[e].x * scale, v[e].y * scale);
  } else if constexpr (MODE == 2) {
    float* of = psd + f * M;
#pragma unroll
    for (int e = 0; e < P::E; ++e) {
      const long long k = k1 + (long long)N1 * out_index<P>(t, e);
      const long long o = shift ? ((k + M / 2) & (M - 1)) : k;
      of[o] = (v[e].x * v[e].x + v[e].y * v[e].y) * scale;
    }
  } else {
    float2* of = reinterpret_cast<float2*>(psd) + f * M;
#pragma unroll
    for (int e = 0; e < P::E; ++e)
      of[k1 + (long long)N1 * out_index<P>(t, e)] = make_float2(v[e].x * scale, v[e].y * scale);
  }
}

// One frame of M <= 16384 points per block, all in LDS.
// MODE 0 (Bluestein): in -> FFT_M -> * Bk -> IFFT_M (conj trick) -> out.
// MODE 1: in -> FFT_M -> out (natural order; the kernel spectrum B).
template <class P, int MODE>
__global__ __launch_bounds__(P::TF) void bf_small_kernel(BfIn in, BfOut out,
                                                         const float2* __restrict__ Bk,
                                                         const float2* __restrict__ tw) {
  static_assert(P::R[0] == P::RL, "in-register convolution needs a palindromic plan");
  __shared__ float2 lds[lds_size<P>()];
  const int t = threadIdx.x;
  const long long f = blockIdx.x;
  float2 v[P::E];
#pragma unroll
  for (int e = 0; e < P::E; ++e) v[e] = in(f, in_index<P>(t, e));
  fft_frame<P>(v, lds, tw, t);
  if constexpr (MODE == 0) {
#pragma unroll
    for (int e = 0; e < P::E; ++e) v[e] = cconj(cmul(v[e], Bk[out_index<P>(t, e)]));
    fft_frame<P>(v, lds, tw + opaque_zero(), t);
#pragma unroll
    for (int e = 0; e < P::E; ++e) out(f, out_index<P>(t, e), cconj(v[e]));
  } else {
#pragma unroll
    for (int e = 0; e < P::E; ++e) out(f, out_index<P>(t, e), v[e]);
  }
}

// chirp c[n] = exp(-i pi (n^2 mod 2N) / N) and the Bluestein kernel
// b[m] = conj(c[min(m, M - m)]) for m < N or m > M - N, else 0 (double math).
__global__ __launch_bounds__(256) void bf_chirp_kernel(long long N, long long M, float2* __restrict__ c,
                                                       float2* __restrict__ b) {
  const long long stride = (long long)gridDim.x * 256;
  const unsigned long long twoN = 2ull * (unsigned long long)N;
  for (long long m = (long long)blockIdx.x * 256 + threadIdx.x; m < M; m += stride) {
    const long long d = m < M - m ? m : M - m;        // circular distance
    float2 cv = make_float2(0.f, 0.f);
    const bool in_b = d < N;
    double s = 0.0, co = 1.0;
    if (in_b) {
      const unsigned long long r = ((unsigned long long)d * (unsigned long long)d) % twoN;
      sincospi((double)r / (double)N, &s, &co);
      cv = make_float2((float)co, (float)-s);          // c[d]
    }
    b[m] = cconj(cv);
    if (m < N) c[m] = cv;
  }
}

// ---------------------------------------------------------------------------
// glue: resample's spectrum copy, the channel filter's mask + mirror
// ---------------------------------------------------------------------------
// scipy.signal.resample (scipy 1.15.3 _signaltools.py): Y[num] from X[Nx]:
// N = min(num, Nx), nyq = N//2 + 1, Y[:nyq] = X[:nyq], Y[nyq-N:] = X[nyq-N:]
// (N > 2), even N: downsampling Y[-N/2] += X[-N/2]; upsampling Y[N/2] *= 1/2,
// Y[num-N/2] = Y[N/2].
__global__ __launch_bounds__(256) void resample_spectrum_kernel(const float2* __restrict__ X,
                                                                long long Nx, long long num,
                                                                float2* __restrict__ Y) {
  const long long N = num < Nx ? num : Nx;
  const long long nyq = N / 2 + 1;
  const long long nneg = N > 2 ? N - nyq : 0;            // copied negative bins
  const long long stride = (long long)gridDim.x * 256;
  for (long long j = (long long)blockIdx.x * 256 + threadIdx.x; j < num; j += stride) {
    float2 v = make_float2(0.f, 0.f);
    if (j < nyq && j < N) v = X[j];
    else if (j >= num - nneg) v = X[Nx - (num - j)];
    if ((N & 1) == 0 && N > 0) {
      if (num < Nx && j == num - N / 2) v = cadd(v, X[Nx - N / 2]);
      if (Nx < num && (j == N / 2 || j == num - N / 2)) {
        const float2 h = X[N / 2];
        v = make_float2(0.5f * h.x, 0.5f * h.y);
      }
    }
    Y[j] = v;
  }
}

// split_channels.filter_channel's spectrum edit for even n (the mirror needs
// equal halves): f_k = fftfreq(n, 1/sr)[k] * sr + CENTER formed in double as
// numpy forms it, F[k] = X[k] if cf - bw/2 <= f_k <= cf + bw/2 for the
// non-negative bins k < n/2, and the negative bins the conjugate mirror
// F[k] = conj(F[n - 1 - k]) of the masked non-negative half.
#pragma clang fp contract(off)
__device__ __forceinline__ bool channel_keep(long long k, long long n, double sr, double center,
                                             double lo, double hi) {
  const long long ks = k < (n - 1) / 2 + 1 ? k : k - n;  // numpy's fftfreq integers
  const double d = 1.0 / sr;
  const double val = 1.0 / ((double)n * d);
  const double f = (double)ks * val * sr + center;
  return f >= lo && f <= hi;
}
__global__ __launch_bounds__(256) void channel_mask_kernel(const float2* __restrict__ X, long long n,
                                                           double sr, double center, double lo,
                                                           double hi, float2* __restrict__ F) {
  const long long stride = (long long)gridDim.x * 256;
  const long long h = n / 2;
  for (long long k = (long long)blockIdx.x * 256 + threadIdx.x; k < n; k += stride) {
    if (n == 1) {                                        // no negative bins to mirror
      F[0] = channel_keep(0, 1, sr, center, lo, hi) ? X[0] : make_float2(0.f, 0.f);
      continue;
    }
    const long long src = k < h ? k : n - 1 - k;
    const float2 v = channel_keep(src, n, sr, center, lo, hi) ? X[src] : make_float2(0.f, 0.f);
    F[k] = k < h ? v : cconj(v);
  }
}

// Few kept bins (the common case: at 56 MHz the reference's axis keeps only
// bin 0): the kept spectrum and the synthesis exactly, by direct sums in
// double precision -- the reference's own numpy FFT / IFFT are double for
// complex128 input, and an output of |X0| / n can sit far below the input's
// scale, out of reach of a float32 transform.
//   X[k] = sum_m x[m] e^{-2 pi i k m / n}                 k in [ka, kb]
//   y[m] = Re sum_k (X[k] e^{2 pi i k m / n} + conj X[k] e^{2 pi i (n-1-k) m / n}) / n
// (the mirror lands on bin n-1-k: split_channels.py:37-38's flip of the
// fftshift-ed halves).  Phases from exact integer reductions (k m mod n).
template <class T>
__global__ __launch_bounds__(256) void channel_bins_kernel(const T* __restrict__ x, long long n,
                                                           long long ka, long long chunk,
                                                           double2* __restrict__ part) {
  const long long k = ka + blockIdx.y;
  const long long m0 = (long long)blockIdx.x * chunk;
  const long long m1 = m0 + chunk < n ? m0 + chunk : n;
  double re = 0.0, im = 0.0;
  for (long long m = m0 + threadIdx.x; m < m1; m += 256) {
    const long long r = (long long)(((unsigned long long)k * (unsigned long long)m) % (unsigned long long)n);
    double s, c;
    sincospi(-2.0 * (double)r / (double)n, &s, &c);
    double xr, xi;
    if constexpr (sizeof(T) == sizeof(double2)) { xr = ((const double2*)x)[m].x; xi = ((const double2*)x)[m].y; }
    else { xr = ((const float2*)x)[m].x; xi = ((const float2*)x)[m].y; }
    re += xr * c - xi * s;
    im += xr * s + xi * c;
  }
  __shared__ double sr[256], si[256];
  sr[threadIdx.x] = re;
  si[threadIdx.x] = im;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) { sr[threadIdx.x] += sr[threadIdx.x + w]; si[threadIdx.x] += si[threadIdx.x + w]; }
    __syncthreads();
  }
  if (threadIdx.x == 0) part[blockIdx.y * gridDim.x + blockIdx.x] = make_double2(sr[0], si[0]);
}

__global__ __launch_bounds__(256) void channel_reduce_kernel(const double2* __restrict__ part,
                                                             int nchunks, int nk,
                                                             double2* __restrict__ X) {
  const int k = blockIdx.x * 256 + threadIdx.x;
  if (k >= nk) return;
  double re = 0.0, im = 0.0;
  for (int c = 0; c < nchunks; ++c) { re += part[k * nchunks + c].x; im += part[k * nchunks + c].y; }
  X[k] = make_double2(re, im);
}

__global__ __launch_bounds__(256) void channel_synth_kernel(const double2* __restrict__ X, long long ka,
                                                            int nk, long long n, double* __restrict__ y) {
  const long long stride = (long long)gridDim.x * 256;
  for (long long m = (long long)blockIdx.x * 256 + threadIdx.x; m < n; m += stride) {
    double acc = 0.0;
    for (int j = 0; j < nk; ++j) {
      const long long k = ka + j;
      const double2 v = X[j];
      if (n == 1) { acc += v.x; continue; }          // a single bin: nothing to mirror
      const unsigned long long un = (unsigned long long)n, um = (unsigned long long)m;
      const long long r1 = (long long)(((unsigned long long)k * um) % un);
      const long long r2 = (long long)(((unsigned long long)(n - 1 - k) * um) % un);
      double s1, c1, s2, c2;
      sincospi(2.0 * (double)r1 / (double)n, &s1, &c1);
      sincospi(2.0 * (double)r2 / (double)n, &s2, &c2);
      acc += v.x * c1 - v.y * s1;          // Re(X e^{i a})
      acc += v.x * c2 + v.y * s2;          // Re(conj(X) e^{i b})
    }
    y[m] = acc / (double)n;
  }
}
#pragma clang fp contract(on)

// ---------------------------------------------------------------------------
// launchers
// ---------------------------------------------------------------------------
template <class F>
static hipError_t plan_dispatch(int N, F&& f) {
  switch (N) {
    case 256: f(Plan256{}); break;
    case 512: f(Plan512{}); break;
    case 1024: f(Plan1024{}); break;
    case 2048: f(Plan2048{}); break;
    case 4096: f(Plan4096{}); break;
    case 8192: f(Plan8192{}); break;
    case 16384: f(Plan16384{}); break;
    default: return hipErrorInvalidValue;
  }
  return hipSuccess;
}
template <class F>
static hipError_t col_dispatch(int N, F&& f) {
  switch (N) {
    case 64: f(Plan64{}); break;
    case 128: f(Plan128{}); break;
    default: return plan_dispatch(N, f);
  }
  return hipSuccess;
}

hipError_t launch_resample_spectrum(const float2* X, long long Nx, long long num, float2* Y,
                                    hipStream_t st) {
  long long g = (num + 255) / 256;
  if (g > 8192) g = 8192;
  hipLaunchKernelGGL(resample_spectrum_kernel, dim3((unsigned)g), dim3(256), 0, st, X, Nx, num, Y);
  return hipGetLastError();
}

hipError_t launch_channel_mask(const float2* X, long long n, double sr, double center, double lo,
                               double hi, float2* F, hipStream_t st) {
  long long g = (n + 255) / 256;
  if (g > 8192) g = 8192;
  hipLaunchKernelGGL(channel_mask_kernel, dim3((unsigned)g), dim3(256), 0, st, X, n, sr, center, lo,
                     hi, F);
  return hipGetLastError();
}

hipError_t launch_channel_direct(int c128, const void* x, long long n, long long ka, long long kb,
                                 double2* part, double2* X, double* y, hipStream_t st) {
  const int nk = (int)(kb - ka + 1);
  if (nk > 0) {
    long long chunk = 1 << 16;
    int nchunks = (int)((n + chunk - 1) / chunk);
    if (nchunks > 256) { nchunks = 256; chunk = (n + 255) / 256; }
    const dim3 g((unsigned)nchunks, (unsigned)nk);
    if (c128)
      hipLaunchKernelGGL(channel_bins_kernel<double2>, g, dim3(256), 0, st, (const double2*)x, n, ka, chunk, part);
    else
      hipLaunchKernelGGL(channel_bins_kernel<float2>, g, dim3(256), 0, st, (const float2*)x, n, ka, chunk, part);
    hipLaunchKernelGGL(channel_reduce_kernel, dim3((unsigned)((nk + 255) / 256)), dim3(256), 0, st, part,
                       nchunks, nk, X);
  }
  long long g = (n + 255) / 256;
  if (g > 8192) g = 8192;
  hipLaunchKernelGGL(channel_synth_kernel, dim3((unsigned)g), dim3(256), 0, st, X, ka, nk > 0 ? nk : 0, n, y);
  return hipGetLastError();
}

void bigfft_split(long long M, int* N1, int* N2) {
  if (M <= 16384) { *N1 = 1; *N2 = (int)M; return; }
  long long n2 = M / 64;
  if (n2 > 16384) n2 = 16384;
  if (n2 < 512) n2 = 512;
  *N2 = (int)n2;
  *N1 = (int)(M / n2);
}

hipError_t launch_bf_chirp(long long N, long long M, float2* c, float2* b, hipStream_t st) {
  long long g = (M + 255) / 256;
  if (g > 16384) g = 16384;
  hipLaunchKernelGGL(bf_chirp_kernel, dim3((unsigned)g), dim3(256), 0, st, N, M, c, b);
  return hipGetLastError();
}

// Forward column pass (x -> tmp, twiddled).
hipError_t launch_bf_col(int N1, int N2, long long batch, const BigIn& in, float2* tmp,
                         const float2* tw1, const float2* t2, int S, int hiA, hipStream_t st) {
  const long long M = (long long)N1 * N2;
  BfIn bi{in.src, in.kind, in.fstride, in.estride, in.nvalid, in.chirp, in.win, in.conj, in.scale};
  BfOut bo{};
  hipError_t e = col_dispatch(N1, [&](auto plan) {
    using PL = decltype(plan);
    constexpr int F = col_frames<PL>();
    const long long grid = batch * (N2 / F);
    hipLaunchKernelGGL((bf_col_kernel<PL, 0>), dim3((unsigned)grid), dim3(F * PL::TF), 0, st, bi,
                       bo, tmp, N2, M, tw1, t2, S, hiA);
  });
  return e != hipSuccess ? e : hipGetLastError();
}

// Inverse column pass (tmp -> out, natural order).
hipError_t launch_bf_icol(int N1, int N2, long long batch, float2* tmp, const BigOut& out,
                          const float2* tw1, const float2* t2, int S, int hiA, hipStream_t st) {
  const long long M = (long long)N1 * N2;
  BfIn bi{};
  BfOut bo{out.dst, out.kind, out.fstride, out.nout, out.chirp, out.conj, out.scale, out.shift};
  hipError_t e = col_dispatch(N1, [&](auto plan) {
    using PL = decltype(plan);
    constexpr int F = col_frames<PL>();
    const long long grid = batch * (N2 / F);
    hipLaunchKernelGGL((bf_col_kernel<PL, 1>), dim3((unsigned)grid), dim3(F * PL::TF), 0, st, bi,
                       bo, tmp, N2, M, tw1, t2, S, hiA);
  });
  return e != hipSuccess ? e : hipGetLastError();
}

hipError_t launch_bf_row(int mode, int N1, int N2, long long batch, float2* tmp, const float2* Bk,
                         const float2* tw2, float scale, float* psd, int shift, hipStream_t st) {
  const long long M = (long long)N1 * N2;
  hipError_t e = plan_dispatch(N2, [&](auto plan) {
    using PL = decltype(plan);
    constexpr int F = row_frames<PL>();
    const long long grid = batch * (N1 / F);
    const dim3 g((unsigned)grid), b(F * PL::TF);
    if (mode == 0) hipLaunchKernelGGL((bf_row_kernel<PL, 0>), g, b, 0, st, tmp, N1, M, Bk, tw2, scale, psd, shift);
    else if (mode == 1) hipLaunchKernelGGL((bf_row_kernel<PL, 1>), g, b, 0, st, tmp, N1, M, Bk, tw2, scale, psd, shift);
    else if (mode == 2) hipLaunchKernelGGL((bf_row_kernel<PL, 2>), g, b, 0, st, tmp, N1, M, Bk, tw2, scale, psd, shift);
    else hipLaunchKernelGGL((bf_row_kernel<PL, 3>), g, b, 0, st, tmp, N1, M, Bk, tw2, scale, psd, shift);
  });
  return e != hipSuccess ? e : hipGetLastError();
}

hipError_t launch_bf_small(int mode, int M, long long batch, const BigIn& in, const BigOut& out,
                           const float2* Bk, const float2* tw, hipStream_t st) {
  BfIn bi{in.src, in.kind, in.fstride, in.estride, in.nvalid, in.chirp, in.win, in.conj, in.scale};
  BfOut bo{out.dst, out.kind, out.fstride, out.nout, out.chirp, out.conj, out.scale, out.shift};
  hipError_t e = plan_dispatch(M, [&](auto plan) {
    using PL = decltype(plan);
    if (mode == 0)
      hipLaunchKernelGGL((bf_small_kernel<PL, 0>), dim3((unsigned)batch), dim3(PL::TF), 0, st, bi, bo, Bk, tw);
    else
      hipLaunchKernelGGL((bf_small_kernel<PL, 1>), dim3((unsigned)batch), dim3(PL::TF), 0, st, bi, bo, Bk, tw);
  });
  return e != hipSuccess ? e : hipGetLastError();
}

}  // namespace vsig
