// |c| reductions (gfx950): peak_reduce over an array (find_correlation_peak on a
// stored correlation) and the deterministic finalize of per-block partials.
#include "os_common.hpp"

namespace vsig {

// ---------------------------------------------------------------------------
// |c| reduction over an array in double precision (find_correlation_peak,
// utils.py:1321-1334): |c| = numpy's own complex abs (np_cabs, in the array's
// precision), first max wins.
// T = double2 (complex128), float2 (complex64), double, float.
// ---------------------------------------------------------------------------
template <class T> __device__ __forceinline__ double absval(const T* p, long long i);
template <> __device__ __forceinline__ double absval<double2>(const double2* p, long long i) {
  const double2 v = p[i]; return np_cabs(v.x, v.y);
}
template <> __device__ __forceinline__ double absval<float2>(const float2* p, long long i) {
  const float2 v = p[i]; return (double)np_cabs(v.x, v.y);
}
template <> __device__ __forceinline__ double absval<double>(const double* p, long long i) { return fabs(p[i]); }
template <> __device__ __forceinline__ double absval<float>(const float* p, long long i) { return (double)fabsf(p[i]); }

template <class T>
__global__ __launch_bounds__(256) void peak_reduce(const T* __restrict__ a, long long n,
                                                   PeakPartial* __restrict__ partials) {
  double m = -1.0, s1 = 0.0, s2 = 0.0;
  long long mi = 0x7fffffffffffffffLL;
  const long long stride = (long long)gridDim.x * 256;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += stride) {
    const double v = absval<T>(a, i);
    betterd(m, mi, v, i);
    s1 += v;
    s2 += v * v;
  }
  block_partial<256>(m, mi, s1, s2, partials + blockIdx.x);
}

// Fixed-order reduction of nparts partials into out[0]; sqrt_max converts a
// max |c|^2 into max |c|.
__global__ __launch_bounds__(1024) void partial_finalize(const PeakPartial* __restrict__ parts,
                                                         long long nparts, int sqrt_max,
                                                         PeakPartial* __restrict__ out) {
  double m = -1.0, s1 = 0.0, s2 = 0.0;
  long long mi = 0x7fffffffffffffffLL;
  for (long long i = threadIdx.x; i < nparts; i += 1024) {
    const PeakPartial p = parts[i];
    betterd(m, mi, p.max2, p.idx);
    s1 += p.sum_abs;
    s2 += p.sum_abs2;
  }
  __shared__ PeakPartial tmp[1];
  block_partial<1024>(m, mi, s1, s2, tmp);
  __syncthreads();
  if (threadIdx.x == 0) {
    PeakPartial r = tmp[0];
    if (sqrt_max) r.max2 = sqrt(r.max2);
    *out = r;
  }
}

// First level of a large reduction: block k reduces the fixed chunk
// [k*chunk, (k+1)*chunk) into tmp[k] (fixed order -> reproducible).
__global__ __launch_bounds__(256) void partial_chunks(const PeakPartial* __restrict__ parts,
                                                      long long nparts, long long chunk,
                                                      PeakPartial* __restrict__ tmp) {
  const long long lo = (long long)blockIdx.x * chunk;
  const long long hi = lo + chunk < nparts ? lo + chunk : nparts;
  double m = -1.0, s1 = 0.0, s2 = 0.0;
  long long mi = 0x7fffffffffffffffLL;
  for (long long i = lo + threadIdx.x; i < hi; i += 256) {
    const PeakPartial p = parts[i];
    betterd(m, mi, p.max2, p.idx);
    s1 += p.sum_abs;
    s2 += p.sum_abs2;
  }
  block_partial<256>(m, mi, s1, s2, tmp + blockIdx.x);
}

hipError_t launch_peak_reduce(int dtype, const void* a, long long n, PeakPartial* partials,
                              int nparts, hipStream_t st) {
  switch (dtype) {
    case VSIG_C128: hipLaunchKernelGGL(peak_reduce<double2>, dim3(nparts), dim3(256), 0, st, (const double2*)a, n, partials); break;
    case VSIG_C64: hipLaunchKernelGGL(peak_reduce<float2>, dim3(nparts), dim3(256), 0, st, (const float2*)a, n, partials); break;
    case VSIG_F64: hipLaunchKernelGGL(peak_reduce<double>, dim3(nparts), dim3(256), 0, st, (const double*)a, n, partials); break;
    case VSIG_F32: hipLaunchKernelGGL(peak_reduce<float>, dim3(nparts), dim3(256), 0, st, (const float*)a, n, partials); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

hipError_t launch_partial_finalize(const PeakPartial* parts, long long nparts, int sqrt_max,
                                   PeakPartial* out, PeakPartial* tmp, hipStream_t st) {
  if (nparts > 8192 && tmp) {       // two levels: chunks in parallel, then one block
    long long g1 = (nparts + 2047) / 2048;
    if (g1 > kFinalizeTmp) g1 = kFinalizeTmp;
    const long long chunk = (nparts + g1 - 1) / g1;
    g1 = (nparts + chunk - 1) / chunk;
    hipLaunchKernelGGL(partial_chunks, dim3((unsigned)g1), dim3(256), 0, st, parts, nparts, chunk, tmp);
    hipLaunchKernelGGL(partial_finalize, dim3(1), dim3(1024), 0, st, tmp, g1, sqrt_max, out);
  } else {
    hipLaunchKernelGGL(partial_finalize, dim3(1), dim3(1024), 0, st, parts, nparts, sqrt_max, out);
  }
  return hipGetLastError();
}

}  // namespace vsig
