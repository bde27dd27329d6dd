// Exact-argmax refinement of the correlators' |c| peak (gfx950).
//
// The correlators compute c in fp32 by overlap-save FFTs; their |c| argmax is
// exact whenever the maximum stands clear of the fp32 error (planted
// preambles), but numpy's argmax (find_correlation_peak, utils.py:1321-1325,
// over np.correlate's complex128 direct sums, cross_correlate_signals
// utils.py:1279-1285) separates near-ties at the 1e-13 level: the reference's
// own tone data (data/packet_*.mat against data/fixed_test_vector.mat) have
// top-2 gaps of 1e-13 .. 7e-12 in |c|^2, 1e5 x below the fp32 error.  This
// pass re-ranks, in double precision and in the caller's operand precision
// (complex64 or complex128), every output whose fp32 |c| lies within a band
// eps of the fp32 maximum:
//   select  : candidate items -- for the fused correlator, fused with the
//             finalize of its wave partials into one launch (the last block
//             to finish reduces, then selects): the thread columns whose lane
//             key is in the band (64 outputs m(t) + TF q of one thread, where
//             the kernel writes lane keys), else the waves whose partial max
//             is (a wave covers ob + wstep w + l + 64 (q % rsub) + stride
//             (q / rsub), see xcorr.hip); for a stored c64 array, its
//             64-output chunks holding one;
//   numpy   : every output of every item evaluated in numpy's own operation
//             order -- np.correlate's complex128 dot is OpenBLAS zdotu (8 fma
//             accumulators per component over complex k mod 8, a fixed add
//             tree, a scalar fma tail, re = d0 - d1, im = d2 + d3; above 10000
//             terms split over T = blas_threads chunks added in order), |c| by
//             numpy's complex abs (larger * sqrt(fma(r, r, 1)), r = smaller /
//             larger) -- so every value is numpy's to the bit (oracle/npdot.c
//             restates it on the CPU, tests/test_npdot_cpu.py pins it against
//             numpy).  np.argmax's rule then applies as is: the max |c| and the
//             lowest output index attaining it, by the last block, which
//             replaces the peak record's max / index (sums untouched).  The
//             operand windows go through LDS (the whole block loads a tile,
//             the 8 lanes of zdot's slots consume it), so the sequential fma
//             chains do not wait on a memory round trip per step;
//   patch   : optionally the refined values into a complex128 c.
// All sizes on the device (no host synchronisation); more than `cap` items
// leaves the record as the fp32 pass produced it and sets status = 1.
// Cross-block hand-offs (last block to finish) use one agent-scope fence per
// block and agent-scope atomic loads of what other blocks wrote.
#include "os_common.hpp"

namespace vsig {

#pragma clang fp contract(off)

template <class T> __device__ __forceinline__ double2 ld2(const T* p, long long i);
template <> __device__ __forceinline__ double2 ld2<float2>(const float2* p, long long i) {
  const float2 v = p[i];
  return make_double2((double)v.x, (double)v.y);
}
template <> __device__ __forceinline__ double2 ld2<double2>(const double2* p, long long i) {
  return p[i];
}

// Overlap of output i (index into the 'full' correlation) with a: taps
// k in [k0, k1), a index i - (nv - 1) + k.
__device__ __forceinline__ void tap_range(long long i, long long na, long long nv, long long& k0,
                                          long long& k1) {
  const long long lo = (nv - 1) - i;             // a index >= 0
  const long long hi = na + (nv - 1) - i;        // a index < na
  k0 = lo > 0 ? lo : 0;
  k1 = hi < nv ? hi : nv;
}

// Shared scratch header (zeroed before select: by the fused finalize, or a memset).
struct RefineKeys {
  unsigned long long count;    // candidate items appended by select
  unsigned long long unused1;
  unsigned long long max2;     // bits of numpy's max |c| (>= 0: integer order)
  unsigned long long unused3;
  unsigned long long status;   // 1: more than cap items (record left unrefined)
  unsigned long long done;     // numpy-pass blocks finished (the last one finishes)
};
static_assert(sizeof(RefineKeys) <= 64, "the items follow the keys at +64 B");

__device__ __forceinline__ double band_threshold(const PeakPartial* rec, double eps) {
  const double t = rec->max2 * (1.0 - eps);     // finalized record: max |c|
  return t > 0.0 ? t : 0.0;
}

__global__ __launch_bounds__(256) void refine_select_array(
    const float2* __restrict__ c, long long nout, const PeakPartial* __restrict__ rec, double eps,
    long long cap, long long* __restrict__ items, RefineKeys* __restrict__ keys) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  const double t = band_threshold(rec, eps);
  const bool hit = i < nout && (double)hypotf(c[i].x, c[i].y) >= t;
  // one candidate per 64-output chunk: the chunk's lowest hitting lane appends
  const unsigned long long m = __ballot(hit);
  if (hit && (threadIdx.x & 63) == (unsigned)__builtin_ctzll(m)) {
    const unsigned long long j = atomicAdd(&keys->count, 1ull);
    if ((long long)j < cap) items[j] = i >> 6;
    else atomicOr(&keys->status, 1ull);
  }
}

// Finalize + select in one launch (the fused correlator's partials): block k
// reduces partial chunk k into tmp[k] (fixed order); the last block to finish
// reduces tmp into the record (max |c|), resets the refine keys and selects
// the candidates: chunks whose max is in the band, their wave partials in the
// band, and -- with lane keys -- the thread columns of those waves in the
// band (items p * 64 + l), else the waves (items p).  One launch where there
// were four (a keys memset, partial_chunks, partial_finalize, a select).
struct FinalizeSelect {
  const PeakPartial* parts; long long nparts, chunk;
  PeakPartial* tmp;                 // gridDim.x first-level records
  unsigned long long* done;         // zero between launches (reset here)
  PeakPartial* rec;                 // finalized record (max |c|)
  double eps; long long cap;
  long long* items; RefineKeys* keys;
  const unsigned* lkeys;            // optional lane keys (64 per wave partial)
};

// A record another block of this launch wrote (possibly on another XCD).
__device__ __forceinline__ PeakPartial ld_agent(const PeakPartial* p) {
  PeakPartial r;
  r.max2 = __hip_atomic_load(&p->max2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  r.idx = __hip_atomic_load(&p->idx, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  r.sum_abs = __hip_atomic_load(&p->sum_abs, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  r.sum_abs2 = __hip_atomic_load(&p->sum_abs2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return r;
}

__global__ __launch_bounds__(256) void refine_finalize_select(FinalizeSelect f) {
  const int tid = threadIdx.x;
  __shared__ int slast, ncl;
  __shared__ int clist[kFinalizeTmp];
  __shared__ double cmax[kFinalizeTmp];
  __shared__ unsigned long long scount;
  __shared__ double sthr;
  {
    const long long lo = (long long)blockIdx.x * f.chunk;
    const long long hi = lo + f.chunk < f.nparts ? lo + f.chunk : f.nparts;
    double m = -1.0, s1 = 0.0, s2 = 0.0;
    long long mi = 0x7fffffffffffffffLL;
#pragma unroll 8
    for (long long i = lo + tid; i < hi; i += 256) {
      const PeakPartial p = f.parts[i];
      betterd(m, mi, p.max2, p.idx);
      s1 += p.sum_abs;
      s2 += p.sum_abs2;
    }
    block_partial<256>(m, mi, s1, s2, f.tmp + blockIdx.x);   // thread 0 writes
  }
#if VSIG_REFINE_KO == 5                            // tuning: the first level alone
  return;
#endif
  if (tid == 0) {      // one release per block (an agent-scope fence writes L2 back)
    __threadfence();
    slast = atomicAdd(f.done, 1ull) == (unsigned long long)gridDim.x - 1;
    if (slast) __threadfence();
  }
  __syncthreads();
  if (!slast) return;
  const int g1 = (int)gridDim.x;
  {
    double m = -1.0, s1 = 0.0, s2 = 0.0;
    long long mi = 0x7fffffffffffffffLL;
    for (int k = tid; k < g1; k += 256) {
      const PeakPartial p = ld_agent(f.tmp + k);
      cmax[k] = p.max2;
      betterd(m, mi, p.max2, p.idx);
      s1 += p.sum_abs;
      s2 += p.sum_abs2;
    }
    __shared__ PeakPartial r[1];
    block_partial<256>(m, mi, s1, s2, r);
    __syncthreads();
    if (tid == 0) {
      PeakPartial o = r[0];
      o.max2 = sqrt(o.max2);
      *f.rec = o;
      const double t = o.max2 * (1.0 - f.eps);
      sthr = t > 0.0 ? t * t : 0.0;                // partials hold fp32 |c|^2
      *f.done = 0;
      ncl = 0;
      scount = 0;
    }
    __syncthreads();
  }
  const double t2 = sthr;
#if VSIG_REFINE_KO == 4                            // tuning: no candidate select
  if (tid == 0) *f.keys = RefineKeys{};
  return;
#endif
  for (int k = tid; k < g1; k += 256)
    if (cmax[k] >= t2) clist[atomicAdd(&ncl, 1)] = k;
  __syncthreads();
  // the in-band chunks' partials, a wave per 64; a wave takes each hit's 64
  // lane keys with one coalesced load and appends the in-band columns
  const int lane = tid & 63;
  const int nc = ncl;
  for (int c = 0; c < nc; ++c) {
    const long long lo = (long long)clist[c] * f.chunk;
    const long long hi = lo + f.chunk < f.nparts ? lo + f.chunk : f.nparts;
    constexpr int kPre = 8;                       // partial maxima loaded ahead
    for (long long pb0 = lo + (tid - lane); pb0 < hi; pb0 += 256LL * kPre) {   // uniform per wave
      double pm[kPre];
#pragma unroll
      for (int q = 0; q < kPre; ++q) {
        const long long p = pb0 + 256LL * q + lane;
        pm[q] = p < hi ? f.parts[p].max2 : -1.0;
      }
#pragma unroll 1
      for (int q = 0; q < kPre; ++q) {
      const long long pb = pb0 + 256LL * q;
      unsigned long long hits = __ballot(pm[q] >= t2);
      // past the cap the refine is skipped anyway (status 1): stop appending
      // (a flat |c| puts every partial in the band)
      if (*(volatile unsigned long long*)&scount > (unsigned long long)f.cap) hits = 0;
      while (hits) {
        const int src = __builtin_ctzll(hits);
        hits &= hits - 1;
        const long long hp = pb + src;
        bool take;
        long long item;
        if (f.lkeys) {
          take = (double)__uint_as_float(f.lkeys[hp * 64 + lane] & ~63u) >= t2;
          item = hp * 64 + lane;
        } else {
          take = lane == src;
          item = hp;
        }
        const unsigned long long km = __ballot(take);
        unsigned long long j0 = 0;
        if (lane == 0) j0 = atomicAdd(&scount, (unsigned long long)__popcll(km));
        j0 = __shfl(j0, 0);
        const unsigned long long j = j0 + __popcll(km & ((1ull << lane) - 1));
        if (take && (long long)j < f.cap) f.items[j] = item;
      }
      }
    }
    __syncthreads();
    if (scount > (unsigned long long)f.cap) break;   // uniform
  }
  __syncthreads();
  if (tid == 0) {
    RefineKeys z{};
    z.count = scount;
    z.status = (long long)scount > f.cap ? 1ull : 0ull;
    *f.keys = z;
  }
}

struct RefineGeom {
  long long nout;       // outputs (final space)
  long long F;          // final output o is full-correlation index F + o
  long long na, nv;     // np.correlate(a, v) operand lengths
  int rev;              // raw (kernel) index -> final: nout - 1 - raw
  int from_array;       // items are 64-output chunks of a stored array
  long long hop;        // partial items: outputs per block, waves per block,
  int waves, Q, stride; //   rows per item and their stride,
  int wstep, rsub;      //   wave base step, 64-output rows per stride step
  int cols;             // > 0: items are thread columns (wave p, column l) =
                        //   p * 64 + l, cols rows each (xcorr_lane_keys)
  int nthr;             // OpenBLAS threads of the numpy being matched (zdotu
                        //   splits sums over 10000 terms into nthr chunks)
};

__device__ __forceinline__ long long item_output(const RefineGeom& g, long long item, int q, int l) {
  long long raw;
  if (g.from_array) {
    raw = item * 64 + l;
    return raw < g.nout ? raw : -1;
  }
  const long long b = item / g.waves;
  const int w = (int)(item - b * g.waves);
  const long long ob = b * g.hop;
  const long long rem = g.nout - ob;
  const long long lim = rem < g.hop ? rem : g.hop;
  const long long r = (long long)g.wstep * w + l + 64LL * (q % g.rsub) + (long long)g.stride * (q / g.rsub);
  if (r >= lim) return -1;
  raw = ob + r;
  return g.rev ? g.nout - 1 - raw : raw;
}

// Output po (< 64) of unit qu of an item: a wave item's unit qu is its row q
// (64 outputs l); a column item has one unit, its rows q = po.
__device__ __forceinline__ long long unit_output(const RefineGeom& g, long long item, int qu, int po) {
  if (g.cols) return po < g.cols ? item_output(g, item >> 6, po, (int)(item & 63)) : -1;
  return item_output(g, item, qu, po);
}

// One zdot_compute over chunk [c0, c0 + w) of output i's overlap (x = a +
// ax, y = conj(v)), in numpy's order.  Tiles of kTile complex are staged by
// the whole block into LDS as planar doubles (xr, xi, yr, -yi); lane
// 8 comp + s (< 32) of wave 0 runs one of zdot_kernel_8's fma chains: slot s
// (complex k = s mod 8 of the block part n8 = w & -8) of component comp (xr yr,
// xi yi, xr yi, xi yr) -- one dependent fma per step, its operands two LDS
// reads.  The add tree combines the slots as the kernel does ((s, s^2), then
// (s, s^4), then the two 128-bit halves: s, s^1); lane 0 gathers the four
// sums and runs the scalar tail.  Result in lane 0.
#ifndef VSIG_REFINE_KO
#define VSIG_REFINE_KO 0
#endif
constexpr int kNpThreads = 256;
constexpr int kTile = 2048;                    // 4 x 16 KB of LDS
constexpr long long kBlasThreadMin = 10000;   // zdotu_k: threads only above this n

template <class T>
__device__ __forceinline__ void np_zdot_chunk(const T* __restrict__ a, const T* __restrict__ v,
                                              long long ax, long long c0, long long w,
                                              double* lds, double& re, double& im) {
  const int tid = threadIdx.x, s = tid & 7, comp = (tid >> 3) & 3;
  double* xr = lds;
  double* xi = lds + kTile;
  double* yr = lds + 2 * kTile;
  double* yn = lds + 3 * kTile;
  const double* X = (comp == 0 || comp == 2) ? xr : xi;
  const double* Y = (comp == 0 || comp == 3) ? yr : yn;
  const long long n8 = w & ~7LL;
  double acc = 0.0;
  // tile t + 1's loads are in flight (registers) while the chains run over
  // tile t (LDS)
  constexpr int kPer = kTile / kNpThreads;
  T xs[kPer], ys[kPer];
  auto fetch = [&](long long tb) {
    const int tl = n8 - tb < kTile ? (int)(n8 - tb) : kTile;
#pragma unroll
    for (int q = 0; q < kPer; ++q) {
      const int j = tid + q * kNpThreads;
      const bool in = j < tl;
      xs[q] = in ? a[ax + c0 + tb + j] : T{};
      ys[q] = in ? v[c0 + tb + j] : T{};
    }
  };
#if VSIG_REFINE_KO == 2                            // tuning: no staging loads
  if (n8 > 0) return;
#endif
  if (n8 > 0) fetch(0);
  for (long long tb = 0; tb < n8; tb += kTile) {  // uniform
    const int tl = n8 - tb < kTile ? (int)(n8 - tb) : kTile;
    __syncthreads();                              // the previous tile is consumed
#pragma unroll
    for (int q = 0; q < kPer; ++q) {
      const int j = tid + q * kNpThreads;
      xr[j] = (double)xs[q].x;
      xi[j] = (double)xs[q].y;
      yr[j] = (double)ys[q].x;
      yn[j] = -(double)ys[q].y;
    }
    __syncthreads();
    if (tb + kTile < n8) fetch(tb + kTile);
#if VSIG_REFINE_KO != 1                            // tuning: no fma chains
    if (tid < 32) {
#pragma unroll 16
      for (int k = s; k < tl; k += 8) acc = fma(X[k], Y[k], acc);
    }
#endif
  }
  if (tid < 32) {                                 // lanes 0..31 of wave 0
    acc = acc + __shfl_xor(acc, 2, 8);
    acc = acc + __shfl_xor(acc, 4, 8);
    acc = acc + __shfl_xor(acc, 1, 8);            // lane 8 comp: d_comp
    double d0 = acc;
    const double d1 = __shfl(acc, 8), d2s = __shfl(acc, 16), d3s = __shfl(acc, 24);
    if (tid == 0) {
      double d1t = d1, d2 = d2s, d3 = d3s;
      for (long long t = n8; t < w; ++t) {
        const double2 x = ld2<T>(a, ax + c0 + t), y = ld2<T>(v, c0 + t);
        const double yi = -y.y;
        d0 = fma(x.x, y.x, d0);
        d1t = fma(x.y, yi, d1t);
        d2 = fma(x.x, yi, d2);
        d3 = fma(y.x, x.y, d3);
      }
      double r = d0 - d1t;
      const double m = d2 + d3;
      r = fma(m, 0.0, r);
      re = r;
      im = m;
    }
  }
}

// Every candidate output (entry e = u * 64 + po of unit u of an item), one
// per block iteration: numpy's complex128 value and |c|, the max |c| by a
// 64-bit atomic max; the last block to finish takes the lowest output index
// attaining it (np.argmax's first-max rule) and writes the record.
template <class T>
__global__ __launch_bounds__(kNpThreads) void refine_numpy(const T* __restrict__ a, const T* __restrict__ v,
                                                         RefineGeom g, const long long* __restrict__ items,
                                                         long long cap, RefineKeys* __restrict__ keys,
                                                         double* __restrict__ vals,
                                                         long long* __restrict__ oidx,
                                                         double2* __restrict__ cv,
                                                         PeakPartial* __restrict__ rec) {
  const long long cnt = (long long)keys->count;
  if (keys->status || cnt == 0) return;            // uniform: no block counts itself
#if VSIG_REFINE_KO == 3 || VSIG_REFINE_KO == 5     // tuning: the launch alone
  return;
#endif
  const long long n = (cnt < cap ? cnt : cap) * g.Q * 64;
  // blocks past the entry count take no part (the last-block hand-off counts
  // only the nact blocks that have entries)
  const long long nact = n < (long long)gridDim.x ? n : (long long)gridDim.x;
  if ((long long)blockIdx.x >= nact) return;
  const int tid = threadIdx.x;
  __shared__ double tiles[4 * kTile];
  __shared__ int slast;
  __shared__ long long smin;
  for (long long e = blockIdx.x; e < n; e += gridDim.x) {   // uniform per block
    const long long u = e >> 6;
    const int po = (int)(e & 63);
    const long long o = unit_output(g, items[u / g.Q], (int)(u % g.Q), po);
    if (o < 0) {
      if (tid == 0) { vals[e] = -1.0; oidx[e] = -1; }
      continue;
    }
    const long long i = g.F + o;
    long long k0, k1;
    tap_range(i, g.na, g.nv, k0, k1);
    const long long nt = k1 - k0;
    const long long ax = i - (g.nv - 1);
    const int nch = (nt <= kBlasThreadMin || g.nthr <= 1) ? 1 : g.nthr;
    double re = 0.0, im = 0.0;
    long long rest = nt, c0 = k0;
    for (int t = 0; t < nch && rest > 0; ++t) {    // OpenBLAS threads' chunks, in order
      long long wd = (rest + (nch - t) - 1) / (nch - t);
      if (wd > rest) wd = rest;
      double pr = 0.0, pi = 0.0;
      np_zdot_chunk<T>(a, v, ax, c0, wd, tiles, pr, pi);
      re = re + pr;
      im = im + pi;
      c0 += wd;
      rest -= wd;
    }
    if (tid == 0) {
      re = 0.0 + re;                               // numpy's CDOUBLE_dot sum
      im = 0.0 + im;
      const double av = np_cabs(re, im);
      vals[e] = av;
      oidx[e] = o;
      cv[e] = make_double2(re, im);
      atomicMax(&keys->max2, (unsigned long long)__double_as_longlong(av));
    }
  }
  // the last block to finish: argmin over the entries, then the record (one
  // release per block: thread 0 made every store of this block)
  __syncthreads();
  if (tid == 0) {
    __threadfence();
    slast = atomicAdd(&keys->done, 1ull) == (unsigned long long)nact - 1;
    if (slast) __threadfence();
    smin = 0x7fffffffffffffffLL;
  }
  __syncthreads();
  if (!slast) return;
  const double m2 = __longlong_as_double(
      (long long)__hip_atomic_load(&keys->max2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
  long long mi = 0x7fffffffffffffffLL;
  for (long long q = tid; q < n; q += kNpThreads) {
    const double ve = __hip_atomic_load(&vals[q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (ve == m2 && ve >= 0.0) {
      const long long o = __hip_atomic_load(&oidx[q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      mi = o < mi ? o : mi;
    }
  }
  for (int off = 32; off > 0; off >>= 1) {
    const long long om = __shfl_xor(mi, off);
    mi = om < mi ? om : mi;
  }
  if ((tid & 63) == 0) atomicMin(&smin, mi);
  __syncthreads();
  if (tid == 0 && smin != 0x7fffffffffffffffLL) {
    rec->max2 = m2;                                // numpy's |c| at its argmax
    rec->idx = smin;
  }
}

// Refined values into a complex128 output (stage-2 values where computed,
// else the plain fp64 stage-1 sums; both beat the fp32 array they replace).
__global__ __launch_bounds__(256) void refine_patch(long long cap, int Q,
                                                    const RefineKeys* __restrict__ keys,
                                                    const long long* __restrict__ oidx,
                                                    const double2* __restrict__ cv,
                                                    double2* __restrict__ out) {
  const long long cnt = (long long)keys->count;
  if (keys->status || cnt == 0) return;
  const long long n = (cnt < cap ? cnt : cap) * Q * 64;
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < n; e += stride) {
    const long long o = oidx[e];
    if (o >= 0) out[o] = cv[e];
  }
}

size_t refine_scratch_bytes(long long cap_items, int Q) {
  const long long n = cap_items * Q * 64;
  return sizeof(RefineKeys) + 64 + (size_t)n * (8 + 8 + 16);
}

hipError_t launch_refine(const RefineArgs& r, hipStream_t st) {
  if (r.cap_items < 1 || (r.cols && (r.from_array || r.cols > 64))) return hipErrorInvalidValue;
  char* base = static_cast<char*>(r.scratch);
  RefineKeys* keys = reinterpret_cast<RefineKeys*>(base);
  const long long n = r.cap_items * r.Q * 64;
  long long* items = reinterpret_cast<long long*>(base + 64);
  double* vals = reinterpret_cast<double*>(items + r.cap_items);
  long long* oidx = reinterpret_cast<long long*>(vals + n);
  double2* cv = reinterpret_cast<double2*>(oidx + n);
  RefineGeom g{r.nout, r.F, r.na, r.nv, r.rev, r.from_array, r.hop, r.waves, r.Q, r.stride,
               r.wstep, r.rsub, r.cols, r.blas_threads > 1 ? r.blas_threads : 1};
  PeakPartial* rec = r.rec;
  if (r.finalize) {              // the partials' finalize + select in one launch
    if (r.from_array || !r.tmp || !r.done) return hipErrorInvalidValue;
#ifndef VSIG_FIN_CHUNK
#define VSIG_FIN_CHUNK 1024
#endif
    long long g1 = (r.nparts + VSIG_FIN_CHUNK - 1) / VSIG_FIN_CHUNK;
    if (g1 < 1) g1 = 1;
    if (g1 > kFinalizeTmp) g1 = kFinalizeTmp;
    long long chunk = (r.nparts + g1 - 1) / g1;
    if (chunk < 1) chunk = 1;
    g1 = (r.nparts + chunk - 1) / chunk;
    if (g1 < 1) g1 = 1;
    const FinalizeSelect f{r.parts, r.nparts, chunk, r.tmp, r.done, rec, r.eps, r.cap_items,
                           items, keys, r.lkeys};
    hipLaunchKernelGGL(refine_finalize_select, dim3((unsigned)g1), dim3(256), 0, st, f);
  } else {
    if (r.cols || r.lkeys) return hipErrorInvalidValue;
    hipError_t e = hipMemsetAsync(keys, 0, sizeof(RefineKeys), st);
    if (e != hipSuccess) return e;
    // a stored c64 array (the correlator's partials are finalized and
    // selected by refine_finalize_select above)
    if (!r.from_array) return hipErrorInvalidValue;
    const long long grid = (r.nout + 255) / 256;
    hipLaunchKernelGGL(refine_select_array, dim3((unsigned)grid), dim3(256), 0, st, r.c64, r.nout,
                       rec, r.eps, r.cap_items, items, keys);
  }
  // one output per block iteration (grid-stride over the device-side count),
  // capped so that the usual 64 candidate outputs get a block each
#ifndef VSIG_REFINE_GRID
#define VSIG_REFINE_GRID 256
#endif
  const long long gl = n < VSIG_REFINE_GRID ? n : VSIG_REFINE_GRID;
  const unsigned gn = (unsigned)(gl > 0 ? gl : 1);
  auto stages = [&](auto tag) {
    using T = decltype(tag);
    hipLaunchKernelGGL(refine_numpy<T>, dim3(gn), dim3(kNpThreads), 0, st, static_cast<const T*>(r.a),
                       static_cast<const T*>(r.v), g, items, r.cap_items, keys, vals, oidx, cv, rec);
  };
  if (r.c128) stages(double2{});
  else stages(float2{});
  const unsigned g2 = gn;
  if (r.out128)
    hipLaunchKernelGGL(refine_patch, dim3(g2), dim3(256), 0, st, r.cap_items, r.Q, keys, oidx, cv,
                       static_cast<double2*>(r.out128));
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// complex128 <-> complex64 conversions for the complex128 correlation path
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void c128_to_c64(const double2* __restrict__ x, long long n,
                                                   float2* __restrict__ y) {
  const long long stride = (long long)gridDim.x * 256;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += stride)
    y[i] = make_float2((float)x[i].x, (float)x[i].y);
}
__global__ __launch_bounds__(256) void c64_to_c128(const float2* __restrict__ x, long long n,
                                                   double2* __restrict__ y) {
  const long long stride = (long long)gridDim.x * 256;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += stride)
    y[i] = make_double2((double)x[i].x, (double)x[i].y);
}

hipError_t launch_convert_c(int to128, const void* x, long long n, void* y, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  long long grid = (n + 255) / 256;
  if (grid > 8192) grid = 8192;
  if (to128)
    hipLaunchKernelGGL(c64_to_c128, dim3((unsigned)grid), dim3(256), 0, st,
                       static_cast<const float2*>(x), n, static_cast<double2*>(y));
  else
    hipLaunchKernelGGL(c128_to_c64, dim3((unsigned)grid), dim3(256), 0, st,
                       static_cast<const double2*>(x), n, static_cast<float2*>(y));
  return hipGetLastError();
}

}  // namespace vsig
