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

// ---------------------------------------------------------------------------
// numpy's float64 statistics of |a| (find_correlation_peak's mean_corr /
// std_corr, utils.py:1329-1330, over np.abs(correlation)):
//   sum  = np.add.reduce over a contiguous array: numpy's reduction walks the
//          array in buffers of 8192 elements, r = 0; r += pairwise(buffer),
//          pairwise = numpy's pairwise_sum (umath loops_utils.h.src: blocks of
//          <= 128 summed with 8 accumulators and a fixed tree, larger ranges
//          split at n / 2 rounded down to a multiple of 8; fewer than 8
//          elements summed from -0.0);
//   mean = sum / n;  std = sqrt(sum((|a| - mean) * (|a| - mean)) / n)
//          (np.std's _var: x = arr - arrmean, x = x * x, the same sum).
// Pinned against numpy by tests/test_npdot_cpu.py (oracle/npdot.c np_stats).
// One wave per buffer: lane-parallel leaves (each stored at its offset / 32:
// leaves hold >= 57 elements, so at most one starts in any 32-element
// window), then lane 0 combines them in the pairwise tree's order; one block
// adds the buffer sums in order.
// ---------------------------------------------------------------------------
#pragma clang fp contract(off)

constexpr int kNpBuf = 8192;

template <class T>
__device__ __forceinline__ double np_elem(const T* __restrict__ a, long long i, int sq, double mean) {
  double x = absval<T>(a, i);
  if (sq) {
    x = x - mean;
    x = x * x;
  }
  return x;
}

template <class T>
__device__ double np_leaf(const T* __restrict__ a, long long off, int n, int sq, double mean) {
  if (n < 8) {
    double res = -0.0;
    for (int i = 0; i < n; ++i) res += np_elem<T>(a, off + i, sq, mean);
    return res;
  }
  double r[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = np_elem<T>(a, off + j, sq, mean);
  int i = 8;
  for (; i < n - (n % 8); i += 8) {
#pragma unroll
    for (int j = 0; j < 8; ++j) r[j] += np_elem<T>(a, off + i + j, sq, mean);
  }
  double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
  for (; i < n; ++i) res += np_elem<T>(a, off + i, sq, mean);
  return res;
}

template <class T>
__global__ __launch_bounds__(256) void np_buf_sums(const T* __restrict__ a, long long n,
                                                   const double* __restrict__ meanp, int sq,
                                                   double* __restrict__ bsum) {
  __shared__ double leaf[4][kNpBuf / 32];
  __shared__ int soff[4][24], sn[4][24], sst[4][24];
  __shared__ double sleft[4][24];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const long long b = (long long)blockIdx.x * 4 + wv;
  const long long nb = (n + kNpBuf - 1) / kNpBuf;
  if (b >= nb) return;                             // whole waves; no block barrier below
  const double mean = sq ? *meanp : 0.0;
  const long long off = b * kNpBuf;
  const int len = (int)(n - off < kNpBuf ? n - off : kNpBuf);
  for (int k = lane; k < kNpBuf / 32; k += 64) {
    const int wlo = 32 * k;
    if (wlo >= len) break;
    const int pos = wlo + 31 < len - 1 ? wlo + 31 : len - 1;
    int no = 0, nn = len;
    while (nn > 128) {                             // the leaf holding pos
      int h = nn / 2;
      h -= h % 8;
      if (pos < no + h) nn = h;
      else { no += h; nn -= h; }
    }
    if (no >= wlo) leaf[wv][no >> 5] = np_leaf<T>(a, off + no, nn, sq, mean);
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
  if (lane != 0) return;
  // post-order walk of the pairwise tree of [0, len)
  int top = 0;
  soff[wv][0] = 0;
  sn[wv][0] = len;
  sst[wv][0] = 0;
  double ret = 0.0;
  for (;;) {
    const int o = soff[wv][top], m = sn[wv][top];
    int h = m / 2;
    h -= h % 8;
    if (m <= 128) {
      ret = leaf[wv][o >> 5];
    } else if (sst[wv][top] == 0) {
      sst[wv][top] = 1;
      ++top;
      soff[wv][top] = o;
      sn[wv][top] = h;
      sst[wv][top] = 0;
      continue;
    } else if (sst[wv][top] == 1) {
      sleft[wv][top] = ret;
      sst[wv][top] = 2;
      ++top;
      soff[wv][top] = o + h;
      sn[wv][top] = m - h;
      sst[wv][top] = 0;
      continue;
    } else {
      ret = sleft[wv][top] + ret;
    }
    if (top == 0) break;
    --top;
  }
  bsum[b] = ret;
}

// r = 0; r += bsum[k] in order; out[0] = r / n (mean) or out[1] = sqrt(r / n).
__global__ __launch_bounds__(256) void np_finish(const double* __restrict__ bsum, long long nb,
                                                 long long n, int sq, double* __restrict__ out) {
  __shared__ double t[256];
  const int tid = threadIdx.x;
  double r = 0.0;
  for (long long b0 = 0; b0 < nb; b0 += 256) {
    __syncthreads();
    if (b0 + tid < nb) t[tid] = bsum[b0 + tid];
    __syncthreads();
    if (tid == 0) {
      const int m = nb - b0 < 256 ? (int)(nb - b0) : 256;
      for (int k = 0; k < m; ++k) r += t[k];
    }
  }
  if (tid == 0) {
    const double q = r / (double)n;
    if (sq) out[1] = sqrt(q);
    else out[0] = q;
  }
}

size_t np_stats_scratch_bytes(long long n) {
  return (size_t)((n + kNpBuf - 1) / kNpBuf) * sizeof(double) + 64;
}

hipError_t launch_np_stats(int dtype, const void* a, long long n, double* out, void* scratch,
                           hipStream_t st) {
  if (n < 1 || !out || !scratch) return hipErrorInvalidValue;
  const long long nb = (n + kNpBuf - 1) / kNpBuf;
  const unsigned grid = (unsigned)((nb + 3) / 4);
  double* bsum = static_cast<double*>(scratch);
  for (int sq = 0; sq < 2; ++sq) {
    switch (dtype) {
      case VSIG_C128:
        hipLaunchKernelGGL(np_buf_sums<double2>, dim3(grid), dim3(256), 0, st,
                           static_cast<const double2*>(a), n, out, sq, bsum);
        break;
      case VSIG_F64:
        hipLaunchKernelGGL(np_buf_sums<double>, dim3(grid), dim3(256), 0, st,
                           static_cast<const double*>(a), n, out, sq, bsum);
        break;
      default:
        return hipErrorInvalidValue;
    }
    hipLaunchKernelGGL(np_finish, dim3(1), dim3(256), 0, st, bsum, nb, n, sq, out);
  }
  return hipGetLastError();
}

}  // namespace vsig
