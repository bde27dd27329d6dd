// Data-parallel analysis kernels behind the reference's detection / display
// helpers:
//
//   radix_hist      one pass of an MSB-first radix select (order statistics ->
//                   np.percentile / np.median), 8-bit digits of order-preserving
//                   keys of float32 / float64 data
//   thresh_reduce   count / first / last index with value >= threshold, max
//                   (np.where(sm >= thr)[0][0 / -1], np.max)
//   energy_scan     inclusive prefix sums of |x|^2 in double (3 kernels)
//   boxcar_same     np.convolve(e, ones(w)/w, 'same') from the prefix sums
//   db_transform    10*log10(|S| + floor) in double (normalize_spectrogram)
//   abs_c64         |x| as a complex64 stream with zero imaginary part (the
//                   template branch of find_packet_start correlates magnitudes)
//
// All are HBM-bound streaming kernels (grid-stride, 16-B loads where the type
// allows); order statistics cost ceil(bits/8) histogram passes.
#include <hip/hip_runtime.h>

#include "vsig_kernels.h"
#include "npabs.hpp"

namespace vsig {

// ---------------------------------------------------------------- keys
// Order-preserving unsigned key of a float (IEEE total order for non-NaN).
__device__ __forceinline__ unsigned int fkey(float f) {
  const unsigned int u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ unsigned long long dkey(double d) {
  const unsigned long long u = (unsigned long long)__double_as_longlong(d);
  return (u & 0x8000000000000000ull) ? ~u : (u | 0x8000000000000000ull);
}

template <class T> struct Key;
template <> struct Key<float> {
  using U = unsigned int;
  static constexpr int BITS = 32;
  __device__ static U of(float f) { return fkey(f); }
};
template <> struct Key<double> {
  using U = unsigned long long;
  static constexpr int BITS = 64;
  __device__ static U of(double d) { return dkey(d); }
};

// ---------------------------------------------------------------- radix select
// For each target q: count, per 8-bit digit at `shift`, the elements whose key
// matches prefix[q] on the bits above `shift` (mask[q]).  hist: nq x 256.
// Keys are of |a| (np.abs is applied first by every caller in the reference).
template <class T>
__global__ __launch_bounds__(256) void radix_hist(const T* __restrict__ a, long long n,
                                                  const unsigned long long* __restrict__ prefix,
                                                  const unsigned long long* __restrict__ mask,
                                                  int nq, int shift,
                                                  unsigned long long* __restrict__ hist) {
  using U = typename Key<T>::U;
  __shared__ unsigned int h[4][256];
  for (int i = threadIdx.x; i < 4 * 256; i += 256) (&h[0][0])[i] = 0;
  __syncthreads();
  U pf[4], mk[4];
  for (int q = 0; q < 4; ++q) {
    pf[q] = q < nq ? (U)prefix[q] : 0;
    mk[q] = q < nq ? (U)mask[q] : 0;
  }
  const long long stride = (long long)gridDim.x * 256;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += stride) {
    const U k = Key<T>::of(fabs(a[i]));
    const unsigned int d = (unsigned int)((k >> shift) & 0xff);
    for (int q = 0; q < nq; ++q)
      if ((k & mk[q]) == pf[q]) atomicAdd(&h[q][d], 1u);
  }
  __syncthreads();
  for (int i = threadIdx.x; i < nq * 256; i += 256) {
    const unsigned int c = (&h[0][0])[i];
    if (c) atomicAdd(&hist[i], (unsigned long long)c);
  }
}

// ---------------------------------------------------------------- thresholds
// out: {count(|a| >= thr), first index or n, last index or -1} and max |a|
// (as double) — one partial per block, finalised on the host.
struct ThreshPartial {
  long long count, first, last;
  double max;
};

template <class T>
__global__ __launch_bounds__(256) void thresh_reduce(const T* __restrict__ a, long long n, double thr,
                                                     ThreshPartial* __restrict__ parts) {
  long long cnt = 0, first = n, last = -1;
  double mx = -1.0 / 0.0;
  const long long stride = (long long)gridDim.x * 256;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += stride) {
    const double v = fabs((double)a[i]);
    if (v >= thr) {
      ++cnt;
      if (i < first) first = i;
      if (i > last) last = i;
    }
    mx = v > mx ? v : mx;
  }
  for (int off = 32; off > 0; off >>= 1) {
    cnt += __shfl_xor(cnt, off);
    const long long f2 = __shfl_xor(first, off), l2 = __shfl_xor(last, off);
    const double m2 = __shfl_xor(mx, off);
    first = f2 < first ? f2 : first;
    last = l2 > last ? l2 : last;
    mx = m2 > mx ? m2 : mx;
  }
  __shared__ ThreshPartial w[4];
  if ((threadIdx.x & 63) == 0) w[threadIdx.x >> 6] = ThreshPartial{cnt, first, last, mx};
  __syncthreads();
  if (threadIdx.x == 0) {
    ThreshPartial r = w[0];
    for (int q = 1; q < 4; ++q) {
      r.count += w[q].count;
      r.first = w[q].first < r.first ? w[q].first : r.first;
      r.last = w[q].last > r.last ? w[q].last : r.last;
      r.max = w[q].max > r.max ? w[q].max : r.max;
    }
    parts[blockIdx.x] = r;
  }
}

// ---------------------------------------------------------------- energy scan
// Inclusive prefix sums P[i] = sum_{j<=i} |x[j]|^2 in double, in tiles of
// 256 x 16 elements: tile sums -> scan of tile sums (one block) -> tile prefix.
constexpr int SCAN_T = 256, SCAN_E = 16, SCAN_TILE = SCAN_T * SCAN_E;

// |x|^2 exactly as numpy forms np.abs(x) ** 2 (squared in the abs's dtype).
__device__ __forceinline__ double energy_of(const float2* x, long long i) {
  const float2 v = x[i];
  const float h = np_cabs(v.x, v.y);
  return (double)__fmul_rn(h, h);
}
__device__ __forceinline__ double energy_of(const double2* x, long long i) {
  const double2 v = x[i];
  const double h = np_cabs(v.x, v.y);
  return __dmul_rn(h, h);
}
__device__ __forceinline__ double energy_of(const float* x, long long i) {
  return (double)__fmul_rn(x[i], x[i]);
}
__device__ __forceinline__ double energy_of(const double* x, long long i) {
  return __dmul_rn(x[i], x[i]);
}

template <int BT>
__device__ __forceinline__ double block_scan_excl(double v, double* total) {
  // inclusive wave scan, then block
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  double s = v;
  for (int off = 1; off < 64; off <<= 1) {
    const double o = __shfl_up(s, off);
    if (lane >= off) s += o;
  }
  __shared__ double ws[BT / 64];
  if (lane == 63) ws[w] = s;
  __syncthreads();
  double base = 0.0, tot = 0.0;
  for (int q = 0; q < BT / 64; ++q) {
    if (q < w) base += ws[q];
    tot += ws[q];
  }
  __syncthreads();
  *total = tot;
  return base + s - v;
}

template <class T>
__global__ __launch_bounds__(SCAN_T) void energy_tile_sums(const T* __restrict__ x, long long n,
                                                           double* __restrict__ sums) {
  const long long base = (long long)blockIdx.x * SCAN_TILE + threadIdx.x * SCAN_E;
  double acc = 0.0;
#pragma unroll
  for (int e = 0; e < SCAN_E; ++e)
    if (base + e < n) acc += energy_of(x, base + e);
  double tot;
  block_scan_excl<SCAN_T>(acc, &tot);
  if (threadIdx.x == 0) sums[blockIdx.x] = tot;
}

__global__ __launch_bounds__(1024) void scan_sums(double* __restrict__ sums, long long nt) {
  // exclusive scan in place, one block, sequential chunks of 1024
  double carry = 0.0;
  for (long long c0 = 0; c0 < nt; c0 += 1024) {
    const long long i = c0 + threadIdx.x;
    const double v = i < nt ? sums[i] : 0.0;
    double tot;
    const double ex = block_scan_excl<1024>(v, &tot);
    if (i < nt) sums[i] = carry + ex;
    carry += tot;
    __syncthreads();
  }
}

template <class T>
__global__ __launch_bounds__(SCAN_T) void energy_prefix(const T* __restrict__ x, long long n,
                                                        const double* __restrict__ sums,
                                                        double* __restrict__ P) {
  const long long base = (long long)blockIdx.x * SCAN_TILE + threadIdx.x * SCAN_E;
  double loc[SCAN_E];
  double acc = 0.0;
#pragma unroll
  for (int e = 0; e < SCAN_E; ++e) {
    acc += (base + e < n) ? energy_of(x, base + e) : 0.0;
    loc[e] = acc;
  }
  double tot;
  const double ex = block_scan_excl<SCAN_T>(acc, &tot) + sums[blockIdx.x];
#pragma unroll
  for (int e = 0; e < SCAN_E; ++e)
    if (base + e < n) P[base + e] = ex + loc[e];
}

// np.convolve(e, ones(w)/w, 'same') from the inclusive prefix sums P of e:
// output length nout = max(n, w), centre offset c = (min(n, w) - 1) / 2,
// sm[i] = (1/w) * sum_{k = i+c-w+1 .. i+c} e[k]  (e = 0 outside [0, n)).
__global__ __launch_bounds__(256) void boxcar_same(const double* __restrict__ P, long long n, long long w,
                                                   long long nout, long long c,
                                                   double* __restrict__ sm) {
  const long long stride = (long long)gridDim.x * 256;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < nout; i += stride) {
    long long hi = i + c;              // inclusive upper index
    const long long lo = i + c - w;    // exclusive lower index (always < n)
    if (hi > n - 1) hi = n - 1;
    const double ph = hi >= 0 ? P[hi] : 0.0;
    const double pl = lo >= 0 ? P[lo] : 0.0;
    sm[i] = (ph - pl) / (double)w;
  }
}

// ---------------------------------------------------------------- dB / abs
// normalize_spectrogram's 10 * np.log10(|S| + floor) in the dtype numpy
// evaluates it in (float32 S with a float32 floor stays float32).  The
// float32 log10 is correctly rounded here; numpy's SIMD log10f is within a
// few ulp of that, so dB maps agree to a few ulp (not bit-exact).
__global__ __launch_bounds__(256) void db_transform_f64(const double* __restrict__ a, long long n,
                                                        double floor_, double* __restrict__ out) {
  const long long stride = (long long)gridDim.x * 256;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += stride)
    out[i] = 10.0 * log10(__dadd_rn(fabs(a[i]), floor_));
}
__global__ __launch_bounds__(256) void db_transform_f32(const float* __restrict__ a, long long n,
                                                        float floor_, float* __restrict__ out) {
  const long long stride = (long long)gridDim.x * 256;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += stride)
    out[i] = __fmul_rn(10.f, (float)log10((double)__fadd_rn(fabsf(a[i]), floor_)));
}

// |a| + 0j (np.abs as numpy computes it: complex -> np_cabs, real -> fabs),
// written as complex64 (O = float2) or complex128 (O = double2).
template <class T> __device__ __forceinline__ double absd(const T& v) { return np_cabs(v.x, v.y); }
template <> __device__ __forceinline__ double absd<double>(const double& v) { return fabs(v); }
template <> __device__ __forceinline__ double absd<float>(const float& v) { return (double)fabsf(v); }
template <class O> __device__ __forceinline__ O mk_re(double r);
template <> __device__ __forceinline__ float2 mk_re<float2>(double r) { return make_float2((float)r, 0.f); }
template <> __device__ __forceinline__ double2 mk_re<double2>(double r) { return make_double2(r, 0.0); }

template <class T, class O>
__global__ __launch_bounds__(256) void abs_to_c(const T* __restrict__ a, long long n,
                                                O* __restrict__ out) {
  const long long stride = (long long)gridDim.x * 256;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += stride)
    out[i] = mk_re<O>(absd<T>(a[i]));
}

// ---------------------------------------------------------------- launchers
static int grid_for(long long n) {
  long long g = (n + 255) / 256;
  if (g > 4096) g = 4096;
  return g < 1 ? 1 : (int)g;
}

hipError_t launch_radix_hist(int dtype, const void* a, long long n, const unsigned long long* prefix,
                             const unsigned long long* mask, int nq, int shift,
                             unsigned long long* hist, hipStream_t st) {
  const int g = grid_for(n) > 2048 ? 2048 : grid_for(n);
  if (dtype == VSIG_F32)
    hipLaunchKernelGGL(radix_hist<float>, dim3(g), dim3(256), 0, st, (const float*)a, n, prefix,
                       mask, nq, shift, hist);
  else if (dtype == VSIG_F64)
    hipLaunchKernelGGL(radix_hist<double>, dim3(g), dim3(256), 0, st, (const double*)a, n, prefix,
                       mask, nq, shift, hist);
  else
    return hipErrorInvalidValue;
  return hipGetLastError();
}

hipError_t launch_thresh_reduce(int dtype, const void* a, long long n, double thr, void* parts,
                                int nparts, hipStream_t st) {
  if (dtype == VSIG_F32)
    hipLaunchKernelGGL(thresh_reduce<float>, dim3(nparts), dim3(256), 0, st, (const float*)a, n,
                       thr, (ThreshPartial*)parts);
  else if (dtype == VSIG_F64)
    hipLaunchKernelGGL(thresh_reduce<double>, dim3(nparts), dim3(256), 0, st, (const double*)a, n,
                       thr, (ThreshPartial*)parts);
  else
    return hipErrorInvalidValue;
  return hipGetLastError();
}

long long energy_scan_tiles(long long n) { return (n + SCAN_TILE - 1) / SCAN_TILE; }

template <class T>
static void energy_prefix_t(const void* x, long long n, double* sums, double* P, hipStream_t st) {
  const long long nt = energy_scan_tiles(n);
  hipLaunchKernelGGL(energy_tile_sums<T>, dim3((unsigned)nt), dim3(SCAN_T), 0, st, (const T*)x, n, sums);
  hipLaunchKernelGGL(scan_sums, dim3(1), dim3(1024), 0, st, sums, nt);
  hipLaunchKernelGGL(energy_prefix<T>, dim3((unsigned)nt), dim3(SCAN_T), 0, st, (const T*)x, n, sums, P);
}

hipError_t launch_energy_prefix(int dtype, const void* x, long long n, double* sums, double* P,
                                hipStream_t st) {
  switch (dtype) {
    case VSIG_C128: energy_prefix_t<double2>(x, n, sums, P, st); break;
    case VSIG_C64: energy_prefix_t<float2>(x, n, sums, P, st); break;
    case VSIG_F64: energy_prefix_t<double>(x, n, sums, P, st); break;
    case VSIG_F32: energy_prefix_t<float>(x, n, sums, P, st); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

hipError_t launch_boxcar_same(const double* P, long long n, long long w, double* sm, hipStream_t st) {
  const long long nout = n > w ? n : w;
  const long long c = ((n < w ? n : w) - 1) / 2;
  hipLaunchKernelGGL(boxcar_same, dim3(grid_for(nout)), dim3(256), 0, st, P, n, w, nout, c, sm);
  return hipGetLastError();
}

hipError_t launch_db_transform(int dtype, const void* a, long long n, double floor_, void* out,
                               hipStream_t st) {
  if (dtype == VSIG_F32)
    hipLaunchKernelGGL(db_transform_f32, dim3(grid_for(n)), dim3(256), 0, st, (const float*)a, n,
                       (float)floor_, (float*)out);
  else if (dtype == VSIG_F64)
    hipLaunchKernelGGL(db_transform_f64, dim3(grid_for(n)), dim3(256), 0, st, (const double*)a, n,
                       floor_, (double*)out);
  else
    return hipErrorInvalidValue;
  return hipGetLastError();
}

template <class O>
static hipError_t launch_abs_t(int dtype, const void* a, long long n, O* out, hipStream_t st) {
  const int g = grid_for(n);
  switch (dtype) {
    case VSIG_C128: hipLaunchKernelGGL((abs_to_c<double2, O>), dim3(g), dim3(256), 0, st, (const double2*)a, n, out); break;
    case VSIG_C64: hipLaunchKernelGGL((abs_to_c<float2, O>), dim3(g), dim3(256), 0, st, (const float2*)a, n, out); break;
    case VSIG_F64: hipLaunchKernelGGL((abs_to_c<double, O>), dim3(g), dim3(256), 0, st, (const double*)a, n, out); break;
    case VSIG_F32: hipLaunchKernelGGL((abs_to_c<float, O>), dim3(g), dim3(256), 0, st, (const float*)a, n, out); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}
hipError_t launch_abs_c64(int dtype, const void* a, long long n, float2* out, hipStream_t st) {
  return launch_abs_t<float2>(dtype, a, n, out, st);
}
hipError_t launch_abs_c128(int dtype, const void* a, long long n, double2* out, hipStream_t st) {
  return launch_abs_t<double2>(dtype, a, n, out, st);
}

}  // namespace vsig
