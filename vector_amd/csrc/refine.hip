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
//   stage 1 : every output of every item by a plain fp64 direct sum
//             c[o] = sum_k a[i - (nv-1) + k] conj(v[k]), i = F + o, with the
//             sum S of the products' component magnitudes; that bounds how far
//             both this sum and numpy's own (below) lie from the exact value:
//             |c| +- E, E = (n/8 + n/64 + T + 300) 2^-52 S + 2^-49 |c|; the
//             largest lower end (|c| - E) by a 64-bit atomic max;
//   stage 2 : the outputs whose upper end reaches that lower end, evaluated in
//             numpy's own operation order -- np.correlate's complex128 dot is
//             OpenBLAS zdotu (8 fma accumulators per component over complex
//             k mod 8, a fixed add tree, a scalar fma tail, re = d0 - d1,
//             im = d2 + d3; above 10000 terms split over T = blas_threads
//             chunks added in order), |c| by numpy's complex abs (larger *
//             sqrt(fma(r, r, 1)), r = smaller / larger) -- so every value is
//             numpy's to the bit (oracle/npdot.c restates it on the CPU and
//             tests/test_npdot_cpu.py pins it against numpy).  np.argmax's
//             rule then applies as is: the max |c| and the lowest output index
//             attaining it, by the last stage-2 block, which replaces the peak
//             record's max / index (sums untouched);
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
  unsigned long long max1;     // bits of the stage-1 max |c|^2 (>= 0: integer order)
  unsigned long long max2;     // bits of the stage-2 max |c|^2
  unsigned long long negidx;   // INT64_MAX - lowest output index attaining max2
  unsigned long long status;   // 1: more than cap items (record left unrefined)
  unsigned long long done;     // stage-2 blocks finished (the last one finishes)
  unsigned long long nsurv;    // stage-2 survivors (listed in items while <= cap)
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
    for (long long i = lo + tid; i < hi; i += 256) {
      const PeakPartial p = f.parts[i];
      betterd(m, mi, p.max2, p.idx);
      s1 += p.sum_abs;
      s2 += p.sum_abs2;
    }
    block_partial<256>(m, mi, s1, s2, f.tmp + blockIdx.x);   // thread 0 writes
  }
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
    for (long long pb = lo + (tid - lane); pb < hi; pb += 256) {   // uniform per wave
      const long long p = pb + lane;
      unsigned long long hits = __ballot(p < hi && f.parts[p].max2 >= t2);
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

// Stage 1: 64 / OUTS blocks per unit of 64 outputs (a wave item's row q, or
// a column item), OUTS outputs each: thread (w, l) of a 16-wave block sums
// output OUTS sub + (l mod OUTS) over tap chunk (64 / OUTS) w + l / OUTS of
// kS1Waves 64 / OUTS (independent partial sums, loads unrolled 8-deep), the
// chunk sums combined in LDS in chunk order.  OUTS = 16 for wave items (64
// chunks: 8 load batches for 4096 taps), 4 for the 64x fewer column items
// (256 chunks, 2 batches).  vals / idx / cv are indexed by u * 64 + o, u =
// item slot * Q + q, o the output's place in the unit.
template <class T>
__device__ __forceinline__ void direct_sum(const T* __restrict__ a, const T* __restrict__ v,
                                           long long abase, long long k0, long long k1,
                                           double& re, double& im, double& sa) {
  long long k = k0;
  double r0 = 0, r1 = 0, i0 = 0, i1 = 0, s0 = 0, s1 = 0;
  for (; k + 8 <= k1; k += 8) {
    double2 x[8], y[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) { x[j] = ld2<T>(a, abase + k + j); y[j] = ld2<T>(v, k + j); }
#pragma unroll
    for (int j = 0; j < 8; j += 2) {
      r0 = fma(x[j].x, y[j].x, r0); r0 = fma(x[j].y, y[j].y, r0);
      i0 = fma(x[j].y, y[j].x, i0); i0 = fma(-x[j].x, y[j].y, i0);
      s0 = fma(fabs(x[j].x) + fabs(x[j].y), fabs(y[j].x) + fabs(y[j].y), s0);
      r1 = fma(x[j + 1].x, y[j + 1].x, r1); r1 = fma(x[j + 1].y, y[j + 1].y, r1);
      i1 = fma(x[j + 1].y, y[j + 1].x, i1); i1 = fma(-x[j + 1].x, y[j + 1].y, i1);
      s1 = fma(fabs(x[j + 1].x) + fabs(x[j + 1].y), fabs(y[j + 1].x) + fabs(y[j + 1].y), s1);
    }
  }
  for (; k < k1; ++k) {
    const double2 x = ld2<T>(a, abase + k), y = ld2<T>(v, k);
    r0 = fma(x.x, y.x, r0); r0 = fma(x.y, y.y, r0);
    i0 = fma(x.y, y.x, i0); i0 = fma(-x.x, y.y, i0);
    s0 = fma(fabs(x.x) + fabs(x.y), fabs(y.x) + fabs(y.y), s0);
  }
  re = r0 + r1;
  im = i0 + i1;
  sa = s0 + s1;
}

// Half-width of the interval around a stage-1 |c| that holds both the exact
// |c| and numpy's (see the header): n overlap terms, S the sum of the
// products' component magnitudes (>= 1 ulp-scale error sources of both sums).
__device__ __forceinline__ double np_band(long long n, int nthr, double S, double c1) {
  const double m = (double)(n / 8 + n / 64 + nthr + 300);
  return m * 0x1p-52 * S + 0x1p-49 * c1;
}

constexpr int kS1Waves = 16;

template <class T, int OUTS>
__global__ __launch_bounds__(kS1Waves * 64) void refine_stage1(const T* __restrict__ a, const T* __restrict__ v,
                                                     RefineGeom g, const long long* __restrict__ items,
                                                     long long cap, RefineKeys* __restrict__ keys,
                                                     double* __restrict__ vals,
                                                     long long* __restrict__ oidx,
                                                     double2* __restrict__ cv) {
  constexpr int kChunks = kS1Waves * 64 / OUTS;     // tap chunks per output
  constexpr int kSplit = 64 / OUTS;                 // blocks per unit
  const long long cnt = (long long)keys->count;
  if (keys->status || cnt == 0) return;
  const long long nunits = (cnt < cap ? cnt : cap) * g.Q;
  const int l = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int ol = l & (OUTS - 1);                    // output within the block
  const int ch = w * (64 / OUTS) + (l / OUTS);      // tap chunk
  __shared__ double pr[kChunks][OUTS], pi[kChunks][OUTS], pa[kChunks][OUTS];
  for (long long ub = blockIdx.x; ub < nunits * kSplit; ub += gridDim.x) {   // uniform per block
    const long long u = ub / kSplit;
    const int sub = (int)(ub - u * kSplit);
    const long long item = items[u / g.Q];
    const int q = (int)(u % g.Q);
    const int po = sub * OUTS + ol;                 // output's place in the unit (0..63)
    const long long o = unit_output(g, item, q, po);
    double re = 0.0, im = 0.0, sa = 0.0;
    long long k0 = 0, k1 = 0;
    if (o >= 0) {
      const long long i = g.F + o;
      tap_range(i, g.na, g.nv, k0, k1);
      const long long span = (k1 - k0 + kChunks - 1) / kChunks;      // this chunk's share
      const long long q0 = k0 + ch * span;
      const long long q1 = q0 + span < k1 ? q0 + span : k1;
      if (q0 < q1) direct_sum<T>(a, v, i - (g.nv - 1), q0, q1, re, im, sa);
    }
    pr[ch][ol] = re;
    pi[ch][ol] = im;
    pa[ch][ol] = sa;
    __syncthreads();
    if (threadIdx.x < OUTS) {                       // lanes 0..OUTS-1 of wave 0 (chunk 0): output ol
      re = 0.0;
      im = 0.0;
      sa = 0.0;
#pragma unroll 8
      for (int c = 0; c < kChunks; ++c) { re += pr[c][ol]; im += pi[c][ol]; sa += pa[c][ol]; }
      // vals: the upper end of the output's interval, max1: the largest lower end
      double up = -1.0, lo = -1.0;
      if (o >= 0) {
        const double c1 = sqrt(re * re + im * im);
        const double E = np_band(k1 - k0, g.nthr, sa, c1);
        up = c1 + E;
        lo = c1 - E > 0.0 ? c1 - E : 0.0;
      }
      const long long e = u * 64 + po;
      vals[e] = up;
      oidx[e] = o;
      cv[e] = make_double2(re, im);
      double wm = lo;
#pragma unroll
      for (int off = OUTS / 2; off > 0; off >>= 1) {
        const double o2 = __shfl_xor(wm, off);
        wm = o2 > wm ? o2 : wm;
      }
      if (ol == 0 && wm >= 0.0) atomicMax(&keys->max1, (unsigned long long)__double_as_longlong(wm));
    }
    __syncthreads();
  }
}

// Stage 2: numpy's value of every output whose interval reaches the largest
// lower end (see the header), then np.argmax.  One 8-lane group per output
// (a wave takes up to 8 outputs): lane s of the group runs OpenBLAS zdot
// kernel slot s -- the four fma chains over complex k = s mod 8 of the block
// part n8 = n & -8 of a chunk -- the add tree combines the slots exactly as
// zdot_kernel_8 does ((s, s^2), then (s, s^4), then the two 128-bit halves:
// s, s^1), and slot 0 runs the scalar tail.  Chunks (OpenBLAS threads, only
// above 10000 terms) run one after another in the group and are added in
// order onto zero, as zdotu_k does.  Every step is an IEEE double fma / add /
// sub / div / sqrt, so the values are numpy's bit for bit.
constexpr int kS2Threads = 1024;
constexpr long long kBlasThreadMin = 10000;   // zdotu_k: threads only above this n

template <class T>
__device__ __forceinline__ double2 ldc(const T* p, long long i) { return ld2<T>(p, i); }

// One zdot_compute over chunk [c0, c0 + w) of the overlap (x = a + ax, y =
// conj(v)); the result in slot 0 (lane s == 0) of the group.
template <class T>
__device__ __forceinline__ void np_zdot_chunk(const T* __restrict__ a, const T* __restrict__ v,
                                              long long ax, long long c0, long long w, int s,
                                              double& re, double& im) {
  const long long n8 = w & ~7LL;
  double P = 0.0, Q = 0.0, R = 0.0, U = 0.0;     // xr yr, xi yi, xr yi, xi yr
  long long k = s;
  for (; k + 56 < n8; k += 64) {                  // 8 rows in flight
    double2 x[8], y[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      x[j] = ldc<T>(a, ax + c0 + k + 8 * j);
      y[j] = ldc<T>(v, c0 + k + 8 * j);
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const double yi = -y[j].y;
      P = fma(x[j].x, y[j].x, P);
      Q = fma(x[j].y, yi, Q);
      R = fma(x[j].x, yi, R);
      U = fma(x[j].y, y[j].x, U);
    }
  }
  for (; k < n8; k += 8) {
    const double2 x = ldc<T>(a, ax + c0 + k), y = ldc<T>(v, c0 + k);
    const double yi = -y.y;
    P = fma(x.x, y.x, P);
    Q = fma(x.y, yi, Q);
    R = fma(x.x, yi, R);
    U = fma(x.y, y.x, U);
  }
  // (A0 + A1) + (A2 + A3) per ymm lane, then low + high halves
  P = P + __shfl_xor(P, 2, 8);  Q = Q + __shfl_xor(Q, 2, 8);
  R = R + __shfl_xor(R, 2, 8);  U = U + __shfl_xor(U, 2, 8);
  P = P + __shfl_xor(P, 4, 8);  Q = Q + __shfl_xor(Q, 4, 8);
  R = R + __shfl_xor(R, 4, 8);  U = U + __shfl_xor(U, 4, 8);
  double d0 = P + __shfl_xor(P, 1, 8), d1 = Q + __shfl_xor(Q, 1, 8);
  double d2 = R + __shfl_xor(R, 1, 8), d3 = U + __shfl_xor(U, 1, 8);
  if (s == 0) {
    for (long long t = n8; t < w; ++t) {
      const double2 x = ldc<T>(a, ax + c0 + t), y = ldc<T>(v, c0 + t);
      const double yi = -y.y;
      d0 = fma(x.x, y.x, d0);
      d1 = fma(x.y, yi, d1);
      d2 = fma(x.x, yi, d2);
      d3 = fma(y.x, x.y, d3);
    }
  }
  double r = d0 - d1;
  const double m = d2 + d3;
  r = fma(m, 0.0, r);
  re = r;
  im = m;
}

template <class T>
__global__ __launch_bounds__(kS2Threads) void refine_stage2(const T* __restrict__ a, const T* __restrict__ v,
                                                            RefineGeom g, long long cap,
                                                            RefineKeys* __restrict__ keys,
                                                            double* __restrict__ vals,
                                                            const long long* __restrict__ oidx,
                                                            double2* __restrict__ cv,
                                                            PeakPartial* __restrict__ rec,
                                                            long long* __restrict__ items) {
  constexpr int NW = kS2Threads / 64;
  const long long cnt = (long long)keys->count;
  if (keys->status || cnt == 0) return;            // uniform: no block counts itself
  const long long n = (cnt < cap ? cnt : cap) * g.Q * 64;
  const double lo1 = __longlong_as_double((long long)keys->max1);
  const int tid = threadIdx.x, l = tid & 63, w = tid >> 6;
  const int grp = l >> 3, s = l & 7;
  __shared__ unsigned long long smask;
  __shared__ int slast;
  __shared__ long long smin;
  for (long long base = (long long)blockIdx.x * 64; base < n; base += (long long)gridDim.x * 64) {
    if (w == 0) {                                  // 64 entries per block step
      const long long e = base + l;
      const double v1 = e < n ? vals[e] : -1.0;
      const bool surv = v1 >= 0.0 && v1 >= lo1;
      if (e < n && v1 >= 0.0 && !surv) vals[e] = -1.0;
      const unsigned long long m = __ballot(surv);
      if (l == 0) smask = m;
      // the survivor list for the finish (items are free after stage 1)
      unsigned long long j0 = 0;
      if (l == 0 && m) j0 = atomicAdd(&keys->nsurv, (unsigned long long)__popcll(m));
      j0 = __shfl(j0, 0);
      const unsigned long long j = j0 + __popcll(m & ((1ull << l) - 1));
      if (surv && (long long)j < cap) items[j] = e;
    }
    __syncthreads();
    // survivors in mask order, in batches of 8: batch b -> wave b % NW, its
    // r-th survivor -> group r (the groups of a wave run side by side)
    const unsigned long long mask = smask;
    const int nsv = __popcll(mask);
    for (int b = w; b * 8 < nsv; b += NW) {        // uniform per wave
      const int r = b * 8 + grp;
      if (r >= nsv) continue;                      // uniform per group
      unsigned long long mm = mask;
      for (int q = 0; q < r; ++q) mm &= mm - 1;
      const int src = __builtin_ctzll(mm);
      const long long es = base + src;
      const long long i = g.F + oidx[es];
      long long k0, k1;
      tap_range(i, g.na, g.nv, k0, k1);
      const long long nt = k1 - k0;
      const long long ax = i - (g.nv - 1);
      const int nch = (nt <= kBlasThreadMin || g.nthr <= 1) ? 1 : g.nthr;
      double re = 0.0, im = 0.0;
      long long rest = nt, c0 = k0;
      for (int t = 0; t < nch && rest > 0; ++t) {
        long long wd = (rest + (nch - t) - 1) / (nch - t);
        if (wd > rest) wd = rest;
        double pr, pi;
        np_zdot_chunk<T>(a, v, ax, c0, wd, s, pr, pi);
        re = re + pr;
        im = im + pi;
        c0 += wd;
        rest -= wd;
      }
      if (s == 0) {
        re = 0.0 + re;                             // numpy's CDOUBLE_dot sum
        im = 0.0 + im;
        const double av = np_cabs(re, im);
        vals[es] = av;
        cv[es] = make_double2(re, im);
        atomicMax(&keys->max2, (unsigned long long)__double_as_longlong(av));
      }
    }
    __syncthreads();
  }
  // the last block to finish: argmin over the entries, then the record (one
  // release per block: the block's stores are complete at the barrier above)
  __syncthreads();
  if (tid == 0) {
    __threadfence();
    slast = atomicAdd(&keys->done, 1ull) == (unsigned long long)gridDim.x - 1;
    if (slast) __threadfence();
    smin = 0x7fffffffffffffffLL;
  }
  __syncthreads();
  if (!slast) return;
  const double m2 = __longlong_as_double(
      (long long)__hip_atomic_load(&keys->max2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
  long long mi = 0x7fffffffffffffffLL;
  const long long ns = (long long)__hip_atomic_load(&keys->nsurv, __ATOMIC_RELAXED,
                                                    __HIP_MEMORY_SCOPE_AGENT);
  const bool listed = ns <= cap;                   // else every entry
  const long long ne = listed ? ns : n;
  for (long long q = tid; q < ne; q += kS2Threads) {
    const long long e = listed ? __hip_atomic_load(&items[q], __ATOMIC_RELAXED,
                                                   __HIP_MEMORY_SCOPE_AGENT) : q;
    const double ve = __hip_atomic_load(&vals[e], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (ve == m2 && ve >= 0.0) {
      const long long o = oidx[e];
      mi = o < mi ? o : mi;
    }
  }
  for (int off = 32; off > 0; off >>= 1) {
    const long long om = __shfl_xor(mi, off);
    mi = om < mi ? om : mi;
  }
  if (l == 0) atomicMin(&smin, mi);
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
    long long g1 = (r.nparts + 2047) / 2048;
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
  // stage grids (grid-stride over the device-side candidate count): stage 1
  // 64 / OUTS blocks per unit, stage 2 one block per 64 entries, capped so
  // that the usual few candidates do not pay for thousands of idle blocks
  const int split = r.cols ? 16 : 4;
  long long units = r.cap_items * r.Q * split;
#ifndef VSIG_REFINE_G1
#define VSIG_REFINE_G1 256
#define VSIG_REFINE_G2 64
#endif
  if (units > VSIG_REFINE_G1) units = VSIG_REFINE_G1;   // one block per CU
  const unsigned g1 = (unsigned)units;
  long long g2l = n / 64;
  if (g2l > VSIG_REFINE_G2) g2l = VSIG_REFINE_G2;
  const unsigned g2 = (unsigned)g2l;
  auto stages = [&](auto tag) {
    using T = decltype(tag);
    const T* a = static_cast<const T*>(r.a);
    const T* v = static_cast<const T*>(r.v);
    if (r.cols)
      hipLaunchKernelGGL((refine_stage1<T, 4>), dim3(g1), dim3(kS1Waves * 64), 0, st, a, v, g, items,
                         r.cap_items, keys, vals, oidx, cv);
    else
      hipLaunchKernelGGL((refine_stage1<T, 16>), dim3(g1), dim3(kS1Waves * 64), 0, st, a, v, g, items,
                         r.cap_items, keys, vals, oidx, cv);
    hipLaunchKernelGGL(refine_stage2<T>, dim3(g2), dim3(kS2Threads), 0, st, a, v, g, r.cap_items,
                       keys, vals, oidx, cv, rec, items);
  };
  if (r.c128) stages(double2{});
  else stages(float2{});
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
