// Exact-argmax refinement of the correlators' |c| peak (gfx950).
//
// The correlators compute c in fp32 by overlap-save FFTs; their |c| argmax is
// exact whenever the maximum stands clear of the fp32 error (planted
// preambles), but numpy's argmax (find_correlation_peak, utils.py:1321-1325,
// over np.correlate's complex128 direct sums, cross_correlate_signals
// utils.py:1279-1285) separates near-ties at the 1e-13 level: the reference's
// own tone data (data/packet_*.mat against data/fixed_test_vector.mat) have
// top-2 gaps of 1e-13 .. 7e-12 in |c|^2, 1e5 x below the fp32 error, and a
// tone against itself ties in exact arithmetic at every full-overlap lag.
// This pass re-ranks every output whose fp32 |c| lies within a band eps of the
// fp32 maximum, in numpy's own operation order and the caller's operand
// precision (complex64 or complex128):
//   select  : candidate items -- for the fused correlator, in the same launch
//             as the finalize of its wave partials (the last block to finish
//             reduces, then selects) and the numpy pass (refine_fused: one
//             launch for the whole refine): the thread columns whose lane
//             key is in the band (the outputs m(t) + TF q of one thread, where
//             the kernel writes lane keys), else the waves whose partial max
//             is (a wave covers ob + wstep w + l + 64 (q % rsub) + stride
//             (q / rsub), see xcorr.hip); for a stored c64 array, its
//             64-output chunks holding one.  Every item is kept (the scratch
//             holds all of them) together with the span [lo, hi] of final
//             outputs the items cover;
//   numpy   : every candidate output evaluated in numpy's own operation order
//             -- np.correlate's complex128 dot is OpenBLAS zdotu (8 fma
//             accumulators per component over complex k mod 8, a fixed add
//             tree, a scalar fma tail, re = d0 - d1, im = d2 + d3; above 10000
//             terms split over T = blas_threads chunks added in order), |c| by
//             numpy's complex abs (larger * sqrt(fma(r, r, 1)), r = smaller /
//             larger) -- so every value is numpy's to the bit (oracle/npdot.c
//             restates it on the CPU, tests/test_npdot_cpu.py pins it against
//             numpy).  np.argmax's rule then applies as is: the max |c| and the
//             lowest output index attaining it replace the peak record's max /
//             index (sums untouched).  Two forms, chosen on the device:
//               sparse (<= kSparseMax candidate outputs, or a span much wider
//                 than the candidates): one output per block iteration, its
//                 operand windows staged through LDS by the whole block, the 32
//                 fma chains of zdot's slots on 32 lanes (latency form: the
//                 usual handful of outputs around a planted peak);
//               dense (flat |c|: a tone, a periodic vector of tone packets --
//                 up to every output): every output of the span, 64
//                 consecutive full-overlap outputs per wave; lane (c, s) runs
//                 zdot slot s of the 8 outputs c + 8 r, 32 independent fma
//                 chains, with the sliding operand held as an 8-element
//                 register window (one new element per step serves all 8
//                 outputs) -- throughput form, fp64-FMA bound.  The few
//                 partial-overlap outputs of the span take the sparse form.
//             No cap: the pass always finishes with numpy's answer; the
//             "refine_cap" option is an explicit opt-in limit (status 1);
//   patch   : optionally numpy's complex128 value of every evaluated output
//             into a complex128 c.
// The same dense kernel evaluates numpy's |c| of every output of a range into
// an array (launch_refine_values: the exact confidence statistics of
// find_correlation_peak on a flat |c|, see reduce.hip np_stats).
// All sizes on the device (no host synchronisation).  Cross-block hand-offs
// (last block to finish, and refine_fused's published keys) write with
// agent-scope atomic stores completed before the counter / flag, and read
// with agent-scope atomic loads: no L2 write-back fences (stores_done).
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
__device__ __forceinline__ double2 to_d2(float2 v) { return make_double2((double)v.x, (double)v.y); }
__device__ __forceinline__ double2 to_d2(double2 v) { return v; }

template <class U>
__device__ __forceinline__ void st_agent(U* p, U v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
template <class U>
__device__ __forceinline__ U ld_agent(const U* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// The cross-block hand-offs: what a block hands over is written with
// agent-scope atomic stores (coherent across the XCDs' L2s) and completed
// (s_waitcnt: the stores acknowledged) before the counter's atomic or the
// flag; readers use agent-scope atomic loads.  No L2 write-back fence
// (buffer_wbl2 costs microseconds behind the correlator's dirty lines).
__device__ __forceinline__ void stores_done() { __builtin_amdgcn_s_waitcnt(0); }

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
  unsigned long long lo_inv;   // ~(lowest final output an item covers)  (atomic max)
  unsigned long long hi_p1;    // highest final output an item covers + 1 (atomic max)
  unsigned long long status;   // 1: more candidate outputs than the opt-in cap
  unsigned long long done;     // numpy-pass blocks finished (the last one reduces)
  unsigned long long fault;    // sticky: a refine_fused watchdog fired.  Nothing on
                               // the device clears it (the finalize resets status,
                               // not this); vsig_refine_status reports status 3 and
                               // clears it with the launch's counters.
  unsigned long long pad[2];
};
static_assert(sizeof(RefineKeys) == 64, "the items follow the keys at +64 B");

struct RefineSlot { double m; long long i; };   // one per numpy-pass block

constexpr int kNpThreads = 256;
constexpr int kNpGrid = 512;                   // 2 blocks per CU (64 KB of LDS each)
constexpr int kNpFast = 64;                    // refine_fused: ticketed numpy blocks
constexpr int kTile = 2048;                    // 4 x 16 KB of LDS
constexpr int kTilePad = 8;                    // doubles: 64 B = 16 LDS banks
constexpr long long kBlasThreadMin = 10000;    // zdotu_k: threads only above this n
constexpr long long kSparseMax = 4096;         // candidate outputs of the sparse form

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
  long long per_item;   // candidate outputs per item
  long long cap;        // opt-in limit on candidate outputs (0: none)
};

__device__ __forceinline__ long long row_offset(const RefineGeom& g, int w, int q, int l) {
  return (long long)g.wstep * w + l + 64LL * (q % g.rsub) + (long long)g.stride * (q / g.rsub);
}

// Final output of row q, lane l of wave partial p (-1: past the block's outputs).
__device__ __forceinline__ long long item_output(const RefineGeom& g, long long p, int q, int l) {
  const long long b = p / g.waves;
  const int w = (int)(p - b * g.waves);
  const long long ob = b * g.hop;
  const long long rem = g.nout - ob;
  const long long lim = rem < g.hop ? rem : g.hop;
  const long long r = row_offset(g, w, q, l);
  if (r >= lim) return -1;
  const long long raw = ob + r;
  return g.rev ? g.nout - 1 - raw : raw;
}

// Candidate output e (item e / per_item = it, its output e % per_item), -1:
// none; item0: items[it0] already loaded.
__device__ __forceinline__ long long entry_output(const RefineGeom& g, const long long* items,
                                                  long long e, long long it0 = -1,
                                                  long long item0 = 0) {
  const long long it = e / g.per_item;
  const int sub = (int)(e - it * g.per_item);
  const long long item = it == it0 ? item0 : ld_agent(items + it);
  if (g.from_array) {
    const long long raw = item * 64 + sub;
    return raw < g.nout ? raw : -1;
  }
  if (g.cols) return item_output(g, item >> 6, sub, (int)(item & 63));
  return item_output(g, item, sub >> 6, sub & 63);
}

// Final outputs [lo, hi] an item covers (rows are increasing in q and the
// valid ones a prefix); false: none.
__device__ __forceinline__ bool item_span(const RefineGeom& g, long long item, long long& lo,
                                          long long& hi) {
  long long rlo, rhi;
  if (g.from_array) {
    rlo = item * 64;
    if (rlo >= g.nout) return false;
    rhi = rlo + 63 < g.nout - 1 ? rlo + 63 : g.nout - 1;
    lo = rlo;
    hi = rhi;
    return true;
  }
  const long long p = g.cols ? item >> 6 : item;
  const int l = g.cols ? (int)(item & 63) : 0;
  const long long b = p / g.waves;
  const int w = (int)(p - b * g.waves);
  const long long ob = b * g.hop;
  const long long rem = g.nout - ob;
  const long long lim = rem < g.hop ? rem : g.hop;
  if (row_offset(g, w, 0, l) >= lim) return false;
  int qh = (g.cols ? g.cols : g.Q) - 1;
  while (row_offset(g, w, qh, l) >= lim) --qh;
  rlo = ob + row_offset(g, w, 0, l);
  long long top = row_offset(g, w, qh, l) + (g.cols ? 0 : 63);
  if (top >= lim) top = lim - 1;
  rhi = ob + top;
  if (g.rev) {
    lo = g.nout - 1 - rhi;
    hi = g.nout - 1 - rlo;
  } else {
    lo = rlo;
    hi = rhi;
  }
  return true;
}

__device__ __forceinline__ double band_threshold(const PeakPartial* rec, double eps) {
  const double t = rec->max2 * (1.0 - eps);     // finalized record: max |c|
  return t > 0.0 ? t : 0.0;
}

__global__ __launch_bounds__(256) void refine_select_array(
    const float2* __restrict__ c, long long nout, const PeakPartial* __restrict__ rec, double eps,
    long long* __restrict__ items, RefineKeys* __restrict__ keys) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  const double t = band_threshold(rec, eps);
  const bool hit = i < nout && (double)hypotf(c[i].x, c[i].y) >= t;
  // one candidate per 64-output chunk: the chunk's lowest hitting lane appends
  const unsigned long long m = __ballot(hit);
  if (hit && (threadIdx.x & 63) == (unsigned)__builtin_ctzll(m)) {
    const long long ch = i >> 6;
    const unsigned long long j = atomicAdd(&keys->count, 1ull);
    items[j] = ch;
    const long long hi = ch * 64 + 63 < nout - 1 ? ch * 64 + 63 : nout - 1;
    atomicMax(&keys->lo_inv, ~(unsigned long long)(ch * 64));
    atomicMax(&keys->hi_p1, (unsigned long long)(hi + 1));
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
  double eps;
  long long* items; long long maxitems; RefineKeys* keys;
  const unsigned* lkeys;            // optional lane keys (64 per wave partial)
  RefineGeom g;                     // item -> output spans
  unsigned long long wd_ticks;      // refine_fused's watchdog (s_memrealtime, 100 MHz)
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

__device__ __forceinline__ void st_agent(PeakPartial* o, const PeakPartial& r) {
  __hip_atomic_store(&o->max2, r.max2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store(&o->idx, r.idx, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store(&o->sum_abs, r.sum_abs, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store(&o->sum_abs2, r.sum_abs2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// A watchdog fire leaves the record unusable: index -1 (no output has it), so
// a caller that reads the record without vsig_refine_status still cannot take
// it for a peak (the sharded chain's gathered rows, StreamChain.global_peak).
__device__ __forceinline__ void poison_record(PeakPartial* rec) {
  __hip_atomic_store(&rec->idx, -1LL, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void watchdog_fired(const FinalizeSelect& f) {
  st_agent(&f.keys->fault, 1ull);
  stores_done();
  poison_record(f.rec);
}

#ifndef VSIG_REFINE_TRACE
#define VSIG_REFINE_TRACE 0  // A/B: phase timestamps (printf by the last block)
#endif
#if VSIG_REFINE_TRACE
__device__ unsigned long long g_rt_first[2] = {~0ull, ~0ull};
__shared__ unsigned long long g_rtz[8];       // np_zdot_chunk / phase-A sub-steps (thread 0)
#define RT(x) const unsigned long long x = wall_clock64()
#else
#define RT(x)
#endif

// Block vb of g1 (first-level chunk vb); true for the block that finished
// last, after it has reduced, selected and written the keys.
__device__ __forceinline__ bool finalize_select_block(const FinalizeSelect& f, int vb, int g1) {
  const int tid = threadIdx.x;
  RT(rt0);
#if VSIG_REFINE_TRACE
  if (tid == 0) atomicMin(&g_rt_first[0], rt0);
#endif
  __shared__ int slast, ncl;
  __shared__ int clist[kFinalizeTmp];
  __shared__ double cmax[kFinalizeTmp];
  __shared__ unsigned long long scount, slo, shi;
  __shared__ double sthr;
  {
    const long long lo = (long long)vb * f.chunk;
    const long long hi = lo + f.chunk < f.nparts ? lo + f.chunk : f.nparts;
    double m = -1.0, s1 = 0.0, s2 = 0.0;
    long long mi = 0x7fffffffffffffffLL;
    constexpr int kL = 4;                       // loads in flight per thread
    for (long long i0 = lo + tid; i0 < hi; i0 += 256 * kL) {   // a thread's partials in order
      PeakPartial p[kL];
#pragma unroll
      for (int q = 0; q < kL; ++q) {
        const long long i = i0 + 256LL * q;
        if (i < hi) p[q] = f.parts[i];
      }
#pragma unroll
      for (int q = 0; q < kL; ++q) {
        if (i0 + 256LL * q < hi) {
          betterd(m, mi, p[q].max2, p[q].idx);
          s1 += p[q].sum_abs;
          s2 += p[q].sum_abs2;
        }
      }
    }
#if VSIG_REFINE_TRACE
    if (tid == 0) g_rtz[5] = wall_clock64();
    {   // the same loads again (lines and translations now warm): latency of a warm round trip
      double z = 0.0;
      for (long long i0 = lo + tid; i0 < hi; i0 += 256 * kL) {
        double p[kL];
#pragma unroll
        for (int q = 0; q < kL; ++q) {
          const long long i = i0 + 256LL * q;
          p[q] = i < hi ? *reinterpret_cast<const volatile double*>(&f.parts[i].sum_abs) : 0.0;
        }
#pragma unroll
        for (int q = 0; q < kL; ++q) z += p[q];
      }
      if (tid == 0) g_rtz[6] = wall_clock64() + 0 * (unsigned long long)__double_as_longlong(z);
    }
#endif
    __shared__ PeakPartial r0[1];
    block_partial<256>(m, mi, s1, s2, r0);
    __syncthreads();
    if (tid == 0) st_agent(f.tmp + vb, r0[0]);
  }
  RT(rt1);
  if (tid == 0) {
    stores_done();
    slast = atomicAdd(f.done, 1ull) == (unsigned long long)g1 - 1;
  }
  __syncthreads();
  if (!slast) return false;
  RT(rt2);
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
      st_agent(f.rec, o);
      stores_done();
      if (ld_agent(&f.keys->fault)) poison_record(f.rec);   // a watchdog fired first
      const double t = o.max2 * (1.0 - f.eps);
      sthr = t > 0.0 ? t * t : 0.0;                // partials hold fp32 |c|^2
      st_agent(f.done, 0ull);
      ncl = 0;
      scount = 0;
      slo = ~0ull;
      shi = 0;
    }
    __syncthreads();
  }
  RT(rt3);
  const double t2 = sthr;
  for (int k = tid; k < g1; k += 256)
    if (cmax[k] >= t2) clist[atomicAdd(&ncl, 1)] = k;
  __syncthreads();
  RT(rt4);
  // the in-band chunks' partials, a wave per 64; a wave takes each hit's 64
  // lane keys with one coalesced load and appends the in-band columns
  const int lane = tid & 63;
  const int nc = ncl;
  unsigned long long mylo = ~0ull, myhi = 0;
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
          if (take) {
            st_agent(f.items + j, item);
            long long ilo, ihi;
            if (item_span(f.g, item, ilo, ihi)) {
              mylo = (unsigned long long)ilo < mylo ? (unsigned long long)ilo : mylo;
              myhi = (unsigned long long)ihi + 1 > myhi ? (unsigned long long)ihi + 1 : myhi;
            }
          }
        }
      }
    }
  }
  if (myhi) {
    atomicMin(&slo, mylo);
    atomicMax(&shi, myhi);
  }
  __syncthreads();                                // the totals in LDS
  RT(rt5);
  if (tid == 0) {
    st_agent(&f.keys->count, scount);
    st_agent(&f.keys->lo_inv, ~slo);
    st_agent(&f.keys->hi_p1, shi);
    st_agent(&f.keys->status, 0ull);
    st_agent(&f.keys->done, 0ull);
  }
  stores_done();                                  // this thread's items (thread 0: the keys)
  __syncthreads();                                // ... all complete before the caller's flag
  if (tid == 0) {
#if VSIG_REFINE_TRACE
    const unsigned long long tf = g_rt_first[0];
    g_rt_first[0] = ~0ull;
    printf("RT fin g1=%d nc=%d items=%llu per_item=%lld | first->t0 %.2f loads %.2f (again %.2f) hand %.2f "
           "lvl2 %.2f clist %.2f select %.2f total %.2f us\n",
           g1, nc, scount, f.g.per_item, (rt0 - tf) * 0.01, (g_rtz[5] - rt0) * 0.01,
           ((long long)g_rtz[6] - (long long)g_rtz[5]) * 0.01, (rt2 - rt1) * 0.01,
           (rt3 - rt2) * 0.01, (rt4 - rt3) * 0.01, (rt5 - rt4) * 0.01, (rt5 - tf) * 0.01);
#endif
  }
  return true;
}

// One zdot_compute over chunk [c0, c0 + w) of output i's overlap (x = a +
// ax, y = conj(v)), in numpy's order.  Tiles of kTile complex are staged by
// the whole block into LDS as planar doubles (xr, xi, yr, -yi); lane
// 8 comp + s (< 32) of wave 0 runs one of zdot_kernel_8's fma chains: slot s
// (complex k = s mod 8 of the block part n8 = w & -8) of component comp (xr yr,
// xi yi, xr yi, xi yr) -- one dependent fma per step (one wave instruction
// for all 32 chains), its operands read a batch of kB steps ahead.  Measured
// (tools/probes/fma_lat.hip): 15 clocks per dependent fp64 fma, ~25 per step
// of this loop; four chains per lane (8 lanes) run at ~50.  The add tree
// combines the slots as the kernel does ((s, s^2), then (s, s^4), then the two
// 128-bit halves: s, s^1); lane 0 gathers the four sums and runs the scalar
// tail.  Result in lane 0.
template <class T>
__device__ __forceinline__ void np_zdot_chunk(const T* __restrict__ a, const T* __restrict__ v,
                                              long long ax, long long c0, long long w,
                                              double* lds, double& re, double& im) {
  const int tid = threadIdx.x, s = tid & 7, comp = (tid >> 3) & 3;
  // xi and yn start 16 banks (64 B) off xr's / yr's bank alignment: a step's
  // read serves components 0 / 2 from xr and 1 / 3 from xi (and 0 / 3 from
  // yr, 1 / 2 from yn) in one instruction, which would otherwise meet on the
  // same banks (2-way conflicts: 46 instead of ~25 clocks per step)
  double* xr = lds;
  double* xi = lds + kTile + kTilePad;
  double* yr = lds + 2 * kTile + 2 * kTilePad;
  double* yn = lds + 3 * kTile + 3 * kTilePad;
  const double* X = (comp == 0 || comp == 2) ? xr : xi;
  const double* Y = (comp == 0 || comp == 3) ? yr : yn;
  const long long n8 = w & ~7LL;
  double acc = 0.0;
  // tile t + 1's loads are in flight (registers) while the chains run over
  // tile t (LDS)
  constexpr int kPer = kTile / kNpThreads;
  T xg[kPer], yg[kPer];
  auto fetch = [&](long long tb) {
    const int tl = n8 - tb < kTile ? (int)(n8 - tb) : kTile;
#pragma unroll
    for (int q = 0; q < kPer; ++q) {
      const int j = tid + q * kNpThreads;
      const bool in = j < tl;
      xg[q] = in ? a[ax + c0 + tb + j] : T{};
      yg[q] = in ? v[c0 + tb + j] : T{};
    }
  };
#if VSIG_REFINE_TRACE
  if (tid == 0) g_rtz[0] = wall_clock64();
#endif
  if (n8 > 0) fetch(0);
  for (long long tb = 0; tb < n8; tb += kTile) {  // uniform
    const int tl = n8 - tb < kTile ? (int)(n8 - tb) : kTile;
    __syncthreads();                              // the previous tile is consumed
#pragma unroll
    for (int q = 0; q < kPer; ++q) {
      const int j = tid + q * kNpThreads;
      xr[j] = (double)xg[q].x;
      xi[j] = (double)xg[q].y;
      yr[j] = (double)yg[q].x;
      yn[j] = -(double)yg[q].y;
    }
    __syncthreads();
#if VSIG_REFINE_TRACE
    if (tid == 0 && tb == 0) { g_rtz[1] = wall_clock64(); g_rtz[6] = clock64(); }
#endif
    if (tb + kTile < n8) fetch(tb + kTile);
    if (tid < 32) {
      // two register batches of kB steps in turn: batch B's reads are in
      // flight while batch A's fmas run and vice versa (no register copies
      // between the reads and the fmas)
      constexpr int kB = 8;
      const double* Xs = X + s;
      const double* Ys = Y + s;
      const int nst = tl >> 3;                    // steps of this tile (tl % 8 == 0)
      const int nfull = nst & ~(2 * kB - 1);
      double xa[kB], ya[kB], xb[kB], yb[kB];
      auto rd = [&](double* xv, double* yv, int j) {
#pragma unroll
        for (int i = 0; i < kB; ++i) {
          xv[i] = Xs[8 * (j + i)];
          yv[i] = Ys[8 * (j + i)];
        }
      };
      auto run = [&](const double* xv, const double* yv) {
#pragma unroll
        for (int i = 0; i < kB; ++i) acc = fma(xv[i], yv[i], acc);
      };
      if (nfull > 0) rd(xa, ya, 0);
      for (int j = 0; j < nfull; j += 2 * kB) {  // uniform
        // (scheduling barriers keep each batch's reads ahead of the other
        // batch's fmas: left alone the compiler sinks them to their use)
        rd(xb, yb, j + kB);
        __builtin_amdgcn_sched_barrier(0);
        run(xa, ya);
        __builtin_amdgcn_sched_barrier(0);
        rd(xa, ya, j + 2 * kB < nfull ? j + 2 * kB : j);   // the last pass re-reads
        __builtin_amdgcn_sched_barrier(0);
        run(xb, yb);
        __builtin_amdgcn_sched_barrier(0);
      }
      for (int j = nfull; j < nst; ++j) acc = fma(Xs[8 * j], Ys[8 * j], acc);
    }
#if VSIG_REFINE_TRACE
    if (tid == 0) g_rtz[tb == 0 ? 2 : 3] = wall_clock64() + 0 * (unsigned long long)__double_as_longlong(acc);
    if (tid == 0 && tb == 0) g_rtz[7] = clock64() + 0 * (unsigned long long)__double_as_longlong(acc);
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
#if VSIG_REFINE_TRACE
      g_rtz[4] = wall_clock64() + 0 * (unsigned long long)__double_as_longlong(r);
#endif
    }
  }
}

// OpenBLAS's split of an nt-term zdot over its threads (zdotu_k: only above
// 10000 terms): chunk t of nch.
__device__ __forceinline__ int blas_chunks(long long nt, int nthr) {
  return (nt <= kBlasThreadMin || nthr <= 1) ? 1 : nthr;
}

// numpy's complex128 c[o] by the whole block (result in thread 0).
template <class T>
__device__ __forceinline__ void eval_single(const T* __restrict__ a, const T* __restrict__ v,
                                            const RefineGeom& g, long long o, double* tiles,
                                            double& re, double& im) {
  const long long i = g.F + o;
  long long k0, k1;
  tap_range(i, g.na, g.nv, k0, k1);
  const long long nt = k1 - k0;
  const long long ax = i - (g.nv - 1);
  const int nch = blas_chunks(nt, g.nthr);
  re = 0.0;
  im = 0.0;
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
  re = 0.0 + re;                                   // numpy's CDOUBLE_dot sum
  im = 0.0 + im;
}

// numpy's complex128 c[o] for the 64 consecutive full-overlap outputs
// ob + c + 8 r (lane = 8 c + s, r < 8) of one wave; lane (c, s) returns output
// ob + c + 8 s.  Term t of output o is x = a[xa(o) + t], y = conj(v[yv(o) + t]),
// t < wf = min(na, nv); D = +1 (na >= nv): xa = o + F - (nv - 1), yv = 0 (a
// slides); D = -1: xa = 0, yv = (nv - 1) - (o + F) (v slides, backwards).
// Slot s of zdot's 8-way split covers t = c0 + s + 8 j of each chunk; for the
// lane's outputs r the sliding operand at step j is element m = j + D r of
// the lane's sequence S[B + 8 m], so the 8 outputs share one register window
// of 8 elements that advances by one element per step (loaded a block of 8
// steps ahead); the fixed operand's element c0 + s + 8 j is shared by all
// outputs of the block and staged through LDS (tiles of 4096 elements, the
// block's 4 waves step through the same tiles).
template <class T, int D>
__device__ __forceinline__ void eval_group(const T* __restrict__ a, const T* __restrict__ v,
                                           const RefineGeom& g, long long ob, long long wf,
                                           double* tiles, double& re_out, double& im_out) {
  const int lane = threadIdx.x & 63, c = lane >> 3, s = lane & 7;
  const T* S = D > 0 ? a : v;
  const T* X = D > 0 ? v : a;
  const long long ns = D > 0 ? g.na : g.nv;
  const long long sb = D > 0 ? ob + g.F - (g.nv - 1) : (g.nv - 1) - (ob + g.F);
  double2* xs = reinterpret_cast<double2*>(tiles);
  constexpr long long kXT = 2 * kTile;             // fixed-operand elements per LDS tile
  const int nch = blas_chunks(wf, g.nthr);
  double re = 0.0, im = 0.0;
  long long rest = wf, c0 = 0;
  for (int t = 0; t < nch && rest > 0; ++t) {    // uniform
    long long wd = (rest + (nch - t) - 1) / (nch - t);
    if (wd > rest) wd = rest;
    const long long n8 = wd & ~7LL;
    const long long B = (D > 0 ? sb + c : sb - c) + s + c0;
    // indices clamped into the operand (lanes of outputs past the range and
    // loads past the last step read a valid element they do not use)
    auto sl = [&](long long m) {
      long long i = B + 8 * m;
      i = i < 0 ? 0 : i;
      return S[i < ns ? i : ns - 1];
    };
    double acc[8][4];
#pragma unroll
    for (int r = 0; r < 8; ++r)
#pragma unroll
      for (int k = 0; k < 4; ++k) acc[r][k] = 0.0;
    double2 ring[8];
    T P[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int m = D > 0 ? k : k - 7;             // window at step 0
      ring[m & 7] = to_d2(sl(m));
      P[k] = sl(D > 0 ? k + 8 : k + 1);            // inserted after step k
    }
    for (long long tb = 0; tb < n8; tb += kXT) {   // uniform across the block
      const long long tl = n8 - tb < kXT ? n8 - tb : kXT;
      __syncthreads();                             // the previous tile is consumed
      for (int i = threadIdx.x; i < tl; i += kNpThreads) xs[i] = to_d2(X[c0 + tb + i]);
      __syncthreads();
      const long long j0 = tb >> 3, j1 = (tb + tl) >> 3;   // this tile's steps
      for (long long J0 = j0; J0 < j1; J0 += 8) {   // uniform
        T Pn[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) Pn[k] = sl(D > 0 ? J0 + 16 + k : J0 + 9 + k);
#pragma unroll
        for (int jj = 0; jj < 8; ++jj) {
          if (J0 + jj < j1) {                        // uniform
            const double2 f = xs[(J0 + jj - j0) * 8 + s];
#pragma unroll
            for (int r = 0; r < 8; ++r) {
              const double2 e = ring[(D > 0 ? jj + r : jj - r) & 7];
              const double2 x = D > 0 ? e : f;
              const double2 y = D > 0 ? f : e;
              const double yn = -y.y;
              acc[r][0] = fma(x.x, y.x, acc[r][0]);
              acc[r][1] = fma(x.y, yn, acc[r][1]);
              acc[r][2] = fma(x.x, yn, acc[r][2]);
              acc[r][3] = fma(x.y, y.x, acc[r][3]);
            }
          }
          ring[(D > 0 ? jj : jj + 1) & 7] = to_d2(P[jj]);
        }
#pragma unroll
        for (int k = 0; k < 8; ++k) P[k] = Pn[k];
      }
    }
    // zdot's add tree over the 8 slots (lanes 8 c + s, s < 8), then lane s
    // keeps output r = s
    double d0 = 0.0, d1 = 0.0, d2 = 0.0, d3 = 0.0;
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      double q[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        double u = acc[r][k];
        u = u + __shfl_xor(u, 2, 8);
        u = u + __shfl_xor(u, 4, 8);
        u = u + __shfl_xor(u, 1, 8);
        q[k] = u;
      }
      if (r == s) { d0 = q[0]; d1 = q[1]; d2 = q[2]; d3 = q[3]; }
    }
    const long long o = ob + c + 8 * s;
    const long long xo = D > 0 ? o + g.F - (g.nv - 1) : 0;
    const long long yo = D > 0 ? 0 : (g.nv - 1) - (o + g.F);
    for (long long tt = n8; tt < wd; ++tt) {        // scalar tail (uniform trip count)
      long long ia = xo + c0 + tt, iv = yo + c0 + tt;
      ia = ia < 0 ? 0 : (ia < g.na ? ia : g.na - 1);
      iv = iv < 0 ? 0 : (iv < g.nv ? iv : g.nv - 1);
      const double2 x = ld2<T>(a, ia), y = ld2<T>(v, iv);
      const double yi = -y.y;
      d0 = fma(x.x, y.x, d0);
      d1 = fma(x.y, yi, d1);
      d2 = fma(x.x, yi, d2);
      d3 = fma(y.x, x.y, d3);
    }
    double rr = d0 - d1;
    const double mm = d2 + d3;
    rr = fma(mm, 0.0, rr);
    re = re + rr;
    im = im + mm;
    c0 += wd;
    rest -= wd;
  }
  re_out = 0.0 + re;
  im_out = 0.0 + im;
}

// The numpy pass of virtual block vb of nb.  Candidate mode (vals ==
// nullptr): the select's cnt items spanning outputs [~lo_inv, hi_p1 - 1];
// values mode: every output of [vlo, vhi], |c| into vals[o - vlo].  Every
// evaluated output updates the block's (max |c|, lowest index); the last block
// to finish writes numpy's argmax into rec.  nact: blocks that take part (the
// others return at once); true for the block that finished last.
template <class T>
__device__ __forceinline__ bool numpy_pass(
    const T* __restrict__ a, const T* __restrict__ v, const RefineGeom& g,
    const long long* __restrict__ items, RefineKeys* __restrict__ keys, RefineSlot* __restrict__ slots,
    double2* __restrict__ cv, double* __restrict__ vals, long long vlo, long long vhi,
    PeakPartial* __restrict__ rec, unsigned long long cnt, unsigned long long lo_inv,
    unsigned long long hi_p1, long long vb, long long nb, long long& nact, long long it0 = -1,
    long long item0 = 0) {
  const int tid = threadIdx.x;
  __shared__ double tiles[4 * kTile + 4 * kTilePad];
  __shared__ int slast;
  __shared__ double wm[kNpThreads / 64];
  __shared__ long long wi[kNpThreads / 64];
  RT(t0);
#if VSIG_REFINE_TRACE
  if (tid == 0) atomicMin(&g_rt_first[1], t0);
#endif
  nact = 0;
  long long lo, hi, n;
  bool dense;
  if (vals) {
    lo = vlo;
    hi = vhi;
    n = hi - lo + 1;
    dense = true;
  } else {
    if (cnt == 0) return false;                    // uniform: no block counts itself
    n = (long long)cnt * g.per_item;
    if (g.cap > 0 && n > g.cap) {                  // opt-in limit: record left fp32
      if (vb == 0 && tid == 0) st_agent(&keys->status, 1ull);
      return false;
    }
    lo = (long long)~lo_inv;
    hi = (long long)hi_p1 - 1;
    dense = n > kSparseMax && hi - lo + 1 <= 8 * n;
  }
  // full-overlap (interior) outputs of the span
  const long long wf = g.na < g.nv ? g.na : g.nv;
  const long long i1 = (g.na < g.nv ? g.nv : g.na) - 1;
  long long ilo = wf - 1 - g.F, ihi = i1 - g.F;
  ilo = ilo > lo ? ilo : lo;
  ihi = ihi < hi ? ihi : hi;
  const long long nin = (dense && ihi >= ilo) ? ihi - ilo + 1 : 0;
  const long long ngroups = (nin + 255) / 256;
  const long long nleft = dense ? (nin ? ilo - lo : hi - lo + 1) : 0;
  const long long nright = (dense && nin) ? hi - ihi : 0;
  const long long ntask = dense ? ngroups + nleft + nright : n;
  // blocks past the task count take no part (the last-block hand-off counts
  // only the nact blocks that have work)
  const long long nbe = nb;
  nact = ntask < nbe ? ntask : nbe;
  if (vb >= nact) return false;
  const long long vbi = vb;
  RT(t1);
  double bm = -1.0;
  long long bi = 0x7fffffffffffffffLL;
  auto record = [&](long long o, double re, double im) {
    const double av = np_cabs(re, im);
    betterd(bm, bi, av, o);
    if (cv) cv[o] = make_double2(re, im);
    if (vals) vals[o - lo] = av;
  };
  for (long long t = vbi; t < ntask; t += nbe) {   // uniform per block
    if (dense && t < ngroups) {
      const long long ob = ilo + 256 * t + 64 * (tid >> 6);
      double re, im;
      if (g.na >= g.nv) eval_group<T, 1>(a, v, g, ob, wf, tiles, re, im);
      else eval_group<T, -1>(a, v, g, ob, wf, tiles, re, im);
      const long long o = ob + ((tid & 63) >> 3) + 8 * (tid & 7);
      if (o <= ihi) record(o, re, im);
    } else {
      long long o;
      if (dense) {
        const long long e = t - ngroups;
        o = e < nleft ? lo + e : ihi + 1 + (e - nleft);
      } else {
        o = entry_output(g, items, t, it0, item0);
        if (o < 0) continue;
      }
      double re, im;
      eval_single<T>(a, v, g, o, tiles, re, im);
      if (tid == 0) record(o, re, im);
    }
  }
  RT(t2);
  // the block's (max, lowest index), then the last block to finish reduces
  // the nact block slots (one release per block)
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    const double om = __shfl_xor(bm, off);
    const long long oi = __shfl_xor(bi, off);
    betterd(bm, bi, om, oi);
  }
  if ((tid & 63) == 0) {
    wm[tid >> 6] = bm;
    wi[tid >> 6] = bi;
  }
  __syncthreads();
  if (tid == 0) {
    for (int q = 1; q < kNpThreads / 64; ++q) betterd(bm, bi, wm[q], wi[q]);
    st_agent(&slots[vbi].m, bm);
    st_agent(&slots[vbi].i, bi);
    stores_done();
    slast = atomicAdd(&keys->done, 1ull) == (unsigned long long)nact - 1;
  }
  __syncthreads();
  if (!slast) return false;
  RT(t3);
  bm = -1.0;
  bi = 0x7fffffffffffffffLL;
  for (long long q = tid; q < nact; q += kNpThreads) {
    const double m = __hip_atomic_load(&slots[q].m, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const long long i = __hip_atomic_load(&slots[q].i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    betterd(bm, bi, m, i);
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    const double om = __shfl_xor(bm, off);
    const long long oi = __shfl_xor(bi, off);
    betterd(bm, bi, om, oi);
  }
  __syncthreads();
  if ((tid & 63) == 0) {
    wm[tid >> 6] = bm;
    wi[tid >> 6] = bi;
  }
  __syncthreads();
  if (tid == 0) {
    for (int q = 1; q < kNpThreads / 64; ++q) betterd(bm, bi, wm[q], wi[q]);
    if (rec && bm >= 0.0) {
      st_agent(&rec->max2, bm);                    // numpy's |c| at its argmax
      st_agent(&rec->idx, bi);
    }
    st_agent(&keys->done, 0ull);
#if VSIG_REFINE_TRACE
    const unsigned long long tf = g_rt_first[1], t4 = wall_clock64();
    g_rt_first[1] = ~0ull;
    printf("RT np n=%lld dense=%d ntask=%lld nact=%lld | first->t0 %.2f setup %.2f eval %.2f "
           "[pre %.2f fetch0 %.2f chain0 %.2f (%.0f clk/step, %.2f GHz) chain1 %.2f tail %.2f] hand %.2f final %.2f total %.2f us\n",
           n, (int)dense, ntask, nact, (t0 - tf) * 0.01, (t1 - t0) * 0.01, (t2 - t1) * 0.01,
           ((long long)g_rtz[0] - (long long)t1) * 0.01, ((long long)g_rtz[1] - (long long)g_rtz[0]) * 0.01,
           ((long long)g_rtz[2] - (long long)g_rtz[1]) * 0.01,
           (double)((long long)g_rtz[7] - (long long)g_rtz[6]) / 256.0,
           (double)((long long)g_rtz[7] - (long long)g_rtz[6]) / ((double)((long long)g_rtz[2] - (long long)g_rtz[1]) * 10.0),
           ((long long)g_rtz[3] - (long long)g_rtz[2]) * 0.01,
           ((long long)g_rtz[4] - (long long)g_rtz[3]) * 0.01,
           (t3 - t2) * 0.01, (t4 - t3) * 0.01, (t4 - tf) * 0.01);
#endif
  }
  return true;
}

// The numpy pass as a launch of its own: values mode, and candidates selected
// from a stored c64 array (refine_select_array).
template <class T>
__global__ __launch_bounds__(kNpThreads, 2) void refine_numpy(
    const T* __restrict__ a, const T* __restrict__ v, RefineGeom g, const long long* __restrict__ items,
    RefineKeys* __restrict__ keys, RefineSlot* __restrict__ slots, double2* __restrict__ cv,
    double* __restrict__ vals, long long vlo, long long vhi, PeakPartial* __restrict__ rec) {
  unsigned long long cnt = 0, lo_inv = 0, hi_p1 = 0;
  if (!vals) {
    cnt = keys->count;
    lo_inv = keys->lo_inv;
    hi_p1 = keys->hi_p1;
  }
  long long nact;
  (void)numpy_pass<T>(a, v, g, items, keys, slots, cv, vals, vlo, vhi, rec, cnt, lo_inv, hi_p1,
                      blockIdx.x, gridDim.x, nact);
}

// The fused correlator's whole refine in one launch: g1 finalize / select
// blocks, then kNpGrid numpy blocks.  The first g1 + kNpFast blocks (by
// index) take tickets in the order they start; tickets < g1 run
// finalize_select_block and exit (the last one publishes the keys with a
// flag), tickets >= g1 are the numpy blocks a sparse pass uses; the blocks
// after them (dense-pass helpers) keep their index.  Every numpy block waits
// for the flag: a ticketed one only for blocks that started before it and
// never wait, whatever the residency; a helper relies on the dispatcher
// starting workgroups in index order (every ticketed block is then running or
// done when a helper starts), as CDNA's does.  The four counters (zero
// between launches) are reset by the last numpy block once every numpy block
// has read the keys.
// Watchdog on refine_fused's two waits (s_memrealtime, 100 MHz): the waits
// end by the argument above, so this bound only turns a fault -- or a
// dispatcher that broke index order -- into status 3 (a sticky fault word and
// a poisoned record, see RefineKeys::fault) instead of a hung GPU.  Default
// 2 s; the context option "refine_watchdog_us" sets it (tests force fires).
constexpr unsigned long long kWatchdogTicks = 200000000ull;   // 2 s

struct FusedCounters {
  unsigned long long done_a;   // FinalizeSelect::done (first-level blocks finished)
  unsigned long long ticket;   // blocks started
  unsigned long long seen;     // numpy blocks that have read the keys
  unsigned long long pad0[5];
  unsigned long long flag;     // 1: keys and items published (own 64-byte line: polled)
  unsigned long long pad1[7];
};
static_assert(sizeof(FusedCounters) == kCounterRecs * sizeof(PeakPartial), "counter slots");

template <class T>
__global__ __launch_bounds__(kNpThreads, 2) void refine_fused(
    FinalizeSelect f, int g1, const T* __restrict__ a, const T* __restrict__ v,
    RefineSlot* __restrict__ slots, double2* __restrict__ cv) {
  FusedCounters* fc = reinterpret_cast<FusedCounters*>(f.done);
  const int tid = threadIdx.x;
  __shared__ long long stk, sitem0;
  __shared__ unsigned long long skeys[3];
  // tickets for the first g1 + kNpFast blocks only (the finalize roles and
  // the numpy blocks a sparse pass uses); the rest are helpers of a dense
  // pass that keep their block index (one atomic per block on one address
  // costs ~15 ns of serialisation: 683 tickets at config 5 were ~7 us of the
  // finalize's start)
  const int nticket = g1 + kNpFast;
  if (tid == 0) stk = (int)blockIdx.x < nticket ? (long long)atomicAdd(&fc->ticket, 1ull)
                                                 : (long long)blockIdx.x;
  __syncthreads();
  const long long tk = stk;
  if (tk < g1) {
    // keys + items completed before (stores_done in finalize_select_block); the
    // flag goes up by an atomic add, so every hand-off signal of this file is
    // one global_atomic_add behind a drained vmcnt (tools/isa_handoffs.py)
    if (finalize_select_block(f, (int)tk, g1) && tid == 0)
      atomicAdd(&fc->flag, 1ull);
    return;
  }
  const long long vb = tk - g1;
  // the item of this block's first task in the sparse form, read with the keys
  const long long it0 = vb / f.g.per_item;
  if (tid == 0) {
    // the kNpFast ticketed numpy blocks poll every ~1300 clocks (the usual
    // handful of candidates), the helpers every ~8000 (they matter only for
    // a dense pass); one 64-byte line holds the flag alone
    const unsigned long long w0 = wall_clock64();
    bool timed_out = false;
    while (__hip_atomic_load(&fc->flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0) {
      if (wall_clock64() - w0 > f.wd_ticks) {
        timed_out = true;
        break;
      }
      if (vb < kNpFast) __builtin_amdgcn_s_sleep(20);
      else __builtin_amdgcn_s_sleep(127);
    }
    if (timed_out) watchdog_fired(f);
    skeys[0] = timed_out ? 0 : ld_agent(&f.keys->count);
    skeys[1] = ld_agent(&f.keys->lo_inv);
    skeys[2] = ld_agent(&f.keys->hi_p1);
    sitem0 = it0 < f.maxitems ? ld_agent(f.items + it0) : 0;
    stores_done();                                 // a fault word before the count
    atomicAdd(&fc->seen, 1ull);
  }
  __syncthreads();
  long long nact;
  const bool last = numpy_pass<T>(a, v, f.g, f.items, f.keys, slots, cv, nullptr, 0, 0, f.rec,
                                  skeys[0], skeys[1], skeys[2], vb, kNpGrid, nact,
                                  (unsigned long long)it0 < skeys[0] ? it0 : -1, sitem0);
  if (tid == 0 && (last || (nact == 0 && vb == 0))) {
    const unsigned long long w0 = wall_clock64();
    while (__hip_atomic_load(&fc->seen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < (unsigned long long)kNpGrid) {
      if (wall_clock64() - w0 > f.wd_ticks) {
        watchdog_fired(f);
        break;
      }
      __builtin_amdgcn_s_sleep(20);
    }
    // every numpy block has read the keys (or the wait above fired): a fire of
    // any of them is in the fault word by now; the record must not survive it
    // (the reducing block may have written numpy's answer without it)
    if (ld_agent(&f.keys->fault)) poison_record(f.rec);
    __hip_atomic_store(&fc->seen, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(&fc->flag, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(&fc->ticket, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

static RefineGeom make_geom(const RefineArgs& r) {
  RefineGeom g{r.nout, r.F, r.na, r.nv, r.rev, r.from_array, r.hop, r.waves, r.Q, r.stride,
               r.wstep, r.rsub, r.cols, r.blas_threads > 1 ? r.blas_threads : 1, 0, r.cap};
  g.per_item = r.from_array ? 64 : r.cols ? r.cols : (long long)r.Q * 64;
  return g;
}

static long long max_items(const RefineArgs& r) {
  if (r.from_array) return (r.nout + 63) / 64;
  return r.cols ? r.nparts * 64 : r.nparts;
}

size_t refine_scratch_bytes(const RefineArgs& r) {
  return sizeof(RefineKeys) + (size_t)max_items(r) * 8 + kNpGrid * sizeof(RefineSlot);
}

static hipError_t launch_numpy(const RefineArgs& r, const RefineGeom& g, const long long* items,
                               RefineKeys* keys, RefineSlot* slots, double* vals, long long vlo,
                               long long vhi, hipStream_t st) {
  auto go = [&](auto tag) {
    using T = decltype(tag);
    hipLaunchKernelGGL(refine_numpy<T>, dim3(kNpGrid), dim3(kNpThreads), 0, st,
                       static_cast<const T*>(r.a), static_cast<const T*>(r.v), g, items, keys,
                       slots, static_cast<double2*>(r.out128), vals, vlo, vhi, r.rec);
  };
  if (r.c128) go(double2{});
  else go(float2{});
  return hipGetLastError();
}

hipError_t launch_refine(const RefineArgs& r, hipStream_t st) {
  if (r.cols && (r.from_array || r.cols > 64)) return hipErrorInvalidValue;
  char* base = static_cast<char*>(r.scratch);
  RefineKeys* keys = reinterpret_cast<RefineKeys*>(base);
  long long* items = reinterpret_cast<long long*>(base + sizeof(RefineKeys));
  RefineSlot* slots = reinterpret_cast<RefineSlot*>(items + max_items(r));
  const RefineGeom g = make_geom(r);
  if (r.finalize) {              // the partials' finalize + select + numpy pass in one launch
    if (r.from_array || !r.tmp || !r.done) return hipErrorInvalidValue;
    constexpr long long kFinChunk = 1024;   // wave partials per first-level block
    long long g1 = (r.nparts + kFinChunk - 1) / kFinChunk;
    if (g1 < 1) g1 = 1;
    if (g1 > kFinalizeTmp) g1 = kFinalizeTmp;
    long long chunk = (r.nparts + g1 - 1) / g1;
    if (chunk < 1) chunk = 1;
    g1 = (r.nparts + chunk - 1) / chunk;
    if (g1 < 1) g1 = 1;
    const FinalizeSelect f{r.parts, r.nparts, chunk, r.tmp, r.done, r.rec, r.eps, items,
                           max_items(r), keys, r.lkeys, g,
                           r.wd_ticks ? r.wd_ticks : kWatchdogTicks};
    const dim3 grid((unsigned)(g1 + kNpGrid));
    if (r.c128)
      hipLaunchKernelGGL(refine_fused<double2>, grid, dim3(kNpThreads), 0, st, f, (int)g1,
                         static_cast<const double2*>(r.a), static_cast<const double2*>(r.v), slots,
                         static_cast<double2*>(r.out128));
    else
      hipLaunchKernelGGL(refine_fused<float2>, grid, dim3(kNpThreads), 0, st, f, (int)g1,
                         static_cast<const float2*>(r.a), static_cast<const float2*>(r.v), slots,
                         static_cast<double2*>(r.out128));
    return hipGetLastError();
  }
  // a stored c64 array: keys memset (up to the sticky fault word, which only
  // vsig_refine_status clears), select, numpy pass
  if (r.cols || r.lkeys || !r.from_array) return hipErrorInvalidValue;
  hipError_t e = hipMemsetAsync(keys, 0, offsetof(RefineKeys, fault), st);
  if (e != hipSuccess) return e;
  const long long grid = (r.nout + 255) / 256;
  hipLaunchKernelGGL(refine_select_array, dim3((unsigned)grid), dim3(256), 0, st, r.c64, r.nout,
                     r.rec, r.eps, items, keys);
  return launch_numpy(r, g, items, keys, slots, nullptr, 0, 0, st);
}

size_t refine_values_scratch_bytes() { return sizeof(RefineKeys) + kNpGrid * sizeof(RefineSlot); }

hipError_t launch_refine_values(const RefineArgs& r, long long lo, long long hi, double* vals,
                                hipStream_t st) {
  if (!vals || lo < 0 || hi < lo || hi >= r.nout) return hipErrorInvalidValue;
  RefineKeys* keys = static_cast<RefineKeys*>(r.scratch);
  RefineSlot* slots = reinterpret_cast<RefineSlot*>(keys + 1);
  hipError_t e = hipMemsetAsync(keys, 0, sizeof(RefineKeys), st);
  if (e != hipSuccess) return e;
  RefineArgs q = r;
  q.from_array = 1;                                // geometry unused in values mode
  return launch_numpy(q, make_geom(q), nullptr, keys, slots, vals, lo, hi, st);
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
