// Critically sampled polyphase filter-bank analysis channelizer (BASELINE
// config 4; no reference counterpart — the nearest analogue is the FFT
// brick-wall split vector_analyzer/split_channels.py:15-44; definition in
// oracle/ref.py pfb_channelize):
//
//   z_m[p]  = sum_{q<PT} h[q*C + p] * x[m*C + q*C + p]        (windowed pre-sum)
//   Y[m, k] = sum_{p<C} z_m[p] * exp(-2j*pi*k*p/C)             (C-point FFT)
//
// One block = 256 threads = G = 256/C groups of C lanes; lane p of a group
// owns branch p and walks the group's frames in order, keeping the PT input
// rows of the current frame in a register ring (one coalesced row load per
// frame: every input sample is read from HBM once).  Every E frames of every
// group (256*E/C frames, 256*E points) the pre-sums go through LDS into the
// in-LDS Stockham engine (fft_engine.hpp, TF = C/E threads per frame) and the
// spectra are written frame-major: y[m*C + k] (the (C, M) result is the
// transposed view, as spectrum() returns Sxx).
//
// HBM: 8 B in + 8 B out per input sample (critically sampled).
#include <hip/hip_runtime.h>

#include "fft_engine.hpp"
#include "vsig_kernels.h"

namespace vsig {

constexpr int cgcd(int a, int b) { return b == 0 ? a : cgcd(b, a % b); }

// a + hp.x * u (HI = 0) or a + hp.y * u (HI = 1), both halves of u: one
// v_pk_fma_f32 with the tap broadcast by op_sel / op_sel_hi
template <int HI>
__device__ __forceinline__ f2v tap_fma(f2v hp, f2v u, f2v a) {
  return __builtin_elementwise_fma(HI ? hp.yy : hp.xx, u, a);
}

// VAR bit 0: spectra leave through LDS so every store is a full C-point row
// (512 B per wave instruction for C = 64) instead of TF-point runs.
// VAR bit 1: the next batch's E input rows are loaded before this batch's FFT
// and stores, so their HBM latency overlaps the compute (more bytes in flight
// per CU for the same occupancy).
// VAR bit 2: cap registers for 4 waves / SIMD (4 blocks per CU).
//
// Measured against (round 6, profiles/r06_pfb_ab.txt): each group's wave
// transforming its own 8 frames (wave barriers only, LDS padding 1 per 8,
// frames 72 float2 apart) 1.596-1.599 ms against 1.537-1.543 for this
// block-wide layout with its five barriers per batch.

template <class PL, int PT, int VAR>
__global__ __launch_bounds__(256, (VAR & 4) ? 4 : 1) void pfb_kernel(const float2* __restrict__ x, long long n,
                                                  const float* __restrict__ h, long long M,
                                                  long long fpg, float2* __restrict__ y,
                                                  const float2* __restrict__ tw,
                                                  unsigned long long* clk) {
  const ClockStamp cs(clk, blockIdx.x);
  constexpr int C = PL::N, E = PL::E, TF = PL::TF, G = 256 / C;
  constexpr int U = PT / cgcd(E, PT);          // batches per ring period
  static_assert(G * E * TF == 256, "one FFT thread per (frame, t) of a batch");
  // frame slots of a batch: FB = G E frames, each in an LDS slice of S float2
  // (odd: see the FFT role below)
  constexpr int FB = G * E, S = PL::LDS | 1;
  __shared__ float2 lds[FB * S];
  const int tid = threadIdx.x, p = tid % C, g = tid / C;
  // the FFT's twiddle table (56 .. 240 entries) copied into LDS once: no
  // global loads inside a batch -- a table load there waits, by vmcnt's issue
  // order, for the next batch's row prefetch as well -- and no VGPRs (exact
  // register twiddles push the 4-wave C = 64 kernel into spills); the 16 lanes
  // of an access group read one entry (broadcast)
  __shared__ float2 twl[PL::twsize()];
  for (int i = tid; i < PL::twsize(); i += 256) twl[i] = tw[i];
  // taps in pairs (h[2j C + p], h[(2j + 1) C + p]): one packed FMA per tap
  // with the pair's low / high half broadcast through op_sel
  static_assert(PT % 2 == 0, "tap pairs");
  f2v hq2[PT / 2];
#pragma unroll
  for (int j = 0; j < PT / 2; ++j) hq2[j] = (f2v){h[2 * j * C + p], h[(2 * j + 1) * C + p]};
  const long long blk = xcd_remap(blockIdx.x, gridDim.x);   // contiguous runs per XCD
  const long long gid = blk * G + g;                          // this lane's group
  const long long m0 = gid * fpg;
  // rows by offset r from the group's first frame: x[(m0 + r) C + p], bounds-
  // checked (zero past n) only in the walks that reach the end of the stream
  const float2* xg = x + m0 * C + p;
  const bool inside = (m0 + fpg + PT - 1) * C <= n;          // wave-uniform
  auto row = [&](long long r, auto chkc) -> float2 {
    if constexpr (decltype(chkc)::value) {
      const long long i = (m0 + r) * C + p;
      return i < n ? x[i] : make_float2(0.f, 0.f);
    } else {
      return xg[(int)r * C];
    }
  };
  // rows only this group reads (walk steps below fpg - PT + 1, either
  // direction) load non-temporal: they need no L2 residency (round 6 A/B, with
  // the non-temporal spectrum stores: 1.537-1.540 -> 1.460-1.463 ms, of which
  // the stores 1.469-1.470, profiles/r06_pfb_ab.txt)
  auto row_nt = [&](long long r) -> float2 {
    const f2v q = __builtin_nontemporal_load(reinterpret_cast<const f2v*>(xg + (int)r * C));
    return fromv(q);
  };
  constexpr bool PF = (VAR & 2) != 0;
  // FFT role of this thread: frame slot ff of the batch, thread t of the frame,
  // frames across the lanes (ff = tid mod FB): the 16 lanes of an LDS access
  // group then hold 16 frames at one intra-frame index, at addresses S apart,
  // and an odd S puts them on 16 distinct banks for every exchange of the
  // engine (with ff = tid / TF two frames' threads met 2-4 way)
  const int ff = tid % FB, t = tid / FB;
  float2* fl = lds + ff * S;
  // Odd groups walk their frames backwards: the PT - 1 rows two neighbouring
  // groups share are then read by both near the same time (both walks start,
  // or both end, there), so the second read is an L2 hit instead of a
  // re-fetch from HBM one whole walk later.  Walk step f is frame mf(f); its
  // new row is the frame's last row (forward) or first row (backward); ring
  // slot of row mf(f) + q: (f + q) % PT forward, (f + PT - 1 - q) % PT backward.
  // Where two groups of a block END at their shared rows (even group g
  // forward, g + 1 backward) the walks meet those rows in opposite orders, up
  // to PT - 2 steps apart -- long enough for L2 to lose many of them (round 6
  // PMC: 1.18 x algorithmic reads).  With XCH (PT = 2 E, two batches per ring
  // period, the whole block inside the stream) the pair shares them through
  // LDS instead: in the second-to-last batch each group also stores its new
  // rows 1 .. E-1 to its slot of xb, and in the last batch each takes its new
  // rows 1 .. E-1 from the partner's slot (row E - i of it: the partner met
  // them in the opposite order) -- 14 of the 15 shared rows read from HBM once.
  // The last batch issues no prefetch (its rows lie past the walk).
  constexpr bool XCH_OK = PF && PT == 2 * E && U == 2 && G % 2 == 0;
  __shared__ float2 xb[XCH_OK ? G * (E - 1) * C : 1];
  auto walk = [&](auto bwdc, auto chkc, auto xchc) {
    constexpr bool BWD = decltype(bwdc)::value;
    constexpr bool X = XCH_OK && decltype(xchc)::value;
    auto rf = [&](long long f) { return BWD ? fpg - 1 - f : f; };     // frame offset
    auto mf = [&](long long f) { return m0 + rf(f); };
    auto newrow = [&](long long f) { return BWD ? rf(f) : rf(f) + PT - 1; };
    float2 ring[PT];
#pragma unroll
    for (int q = 1; q < PT; ++q)                      // rows of frame mf(0) but its new one
      ring[BWD ? PT - 1 - q : q - 1] = row(rf(0) + (BWD ? q : q - 1), chkc);
    float2 nxt[PF ? E : 1];
    if constexpr (PF) {
#pragma unroll
      for (int i = 0; i < E; ++i) nxt[i] = row(newrow(i), chkc);
    }
    for (long long b = 0; b < fpg; b += (long long)E * U) {
      const bool last = b + (long long)E * U >= fpg;           // uniform
      static_for<0, U>([&](auto ui) {
        constexpr int u = decltype(ui)::value;
        static_for<0, E>([&](auto ii) {
          constexpr int i = decltype(ii)::value;
          constexpr int k = u * E + i;                        // walk step mod ring period
          if constexpr (X && u == U - 1 && i >= 1) {
            if (last) ring[(k + PT - 1) % PT] = xb[((g ^ 1) * (E - 1) + (E - i) - 1) * C + p];
            else ring[(k + PT - 1) % PT] = nxt[i];
          } else if constexpr (PF) {
            ring[(k + PT - 1) % PT] = nxt[i];
          } else {
            ring[(k + PT - 1) % PT] = row(newrow(b + k), chkc);
          }
          f2v z[2] = {(f2v){0.f, 0.f}, (f2v){0.f, 0.f}};   // even / odd taps: no
          static_for<0, PT>([&](auto qi) {                    // back-to-back dependence
            constexpr int q = decltype(qi)::value;
            constexpr int slot = BWD ? (k + PT - 1 - q) % PT : (k + q) % PT;
            z[q & 1] = tap_fma<q & 1>(hq2[q / 2], tov(ring[slot]), z[q & 1]);
          });
          lds[(g * E + i) * S + lpad(p)] = fromv(z[0] + z[1]);
        });
        if constexpr (X && u == 0) {
          if (last) {
#pragma unroll
            for (int i = 1; i < E; ++i) xb[(g * (E - 1) + i - 1) * C + p] = nxt[i];
          }
        }
        if constexpr (PF) {
          if (!(last && u == U - 1)) {                        // next batch
            if (X && u == 0 && last) {                        // only its row 0 from HBM
              nxt[0] = row(newrow(b + (u + 1) * E), chkc);
            } else if (!decltype(chkc)::value &&
                       b + (u + 2) * E <= fpg - PT + 1) {   // rows no other group reads
#pragma unroll
              for (int i = 0; i < E; ++i) nxt[i] = row_nt(newrow(b + (u + 1) * E + i));
            } else {
#pragma unroll
              for (int i = 0; i < E; ++i) nxt[i] = row(newrow(b + (u + 1) * E + i), chkc);
            }
          }
        }
        __syncthreads();
        float2 v[E];
        fft_load<PL, 0>(v, fl, t);
        fft_stage<PL, 0>(v, TwTable{twl}, t);
        fft_tail<PL, 1>(v, fl, TwTable{twl}, t);
        static_assert(VAR & 1, "the walk directions need the LDS-staged stores");
        __syncthreads();                                      // last FFT pass read lds
#pragma unroll
        for (int e = 0; e < E; ++e) fl[lpad(out_index<PL>(t, e))] = v[e];
        __syncthreads();
#pragma unroll
        for (int i = 0; i < E; ++i) {
          const long long m = mf(b + u * E + i);
          // spectra leave non-temporal: written once, never re-read here
          if (m < M)
            __builtin_nontemporal_store(tov(lds[(g * E + i) * S + lpad(p)]),
                                        reinterpret_cast<f2v*>(y + m * C + p));
        }
        __syncthreads();                                      // lds reused by the next batch
      });
    }
  };
  // the exchange needs both groups of every pair on the unchecked path: the
  // whole block inside the stream (block-uniform); other blocks check bounds
  const bool inside_blk = (((blk + 1) * G) * fpg + PT - 1) * C <= n;
  const bool fast = XCH_OK ? inside_blk : inside;
  if (gid & 1) {
    if (fast) walk(IC<1>{}, IC<0>{}, IC<1>{});
    else walk(IC<1>{}, IC<1>{}, IC<0>{});
  } else {
    if (fast) walk(IC<0>{}, IC<0>{}, IC<1>{});
    else walk(IC<0>{}, IC<1>{}, IC<0>{});
  }
  cs.done(clk);
}

// Shipped configuration: LDS-staged stores + next-batch prefetch (VAR 3;
// C = 64: registers capped for 4 waves / SIMD, VAR 7: 128 VGPRs, no scratch),
// 64 frames per group (128 / 256 / 512 measured slower, profiles/r02_v13_pfb_ab.txt;
// again in round 6 with the row exchange: 128 +9 %, 32 +0.1..1 %; VAR 3 +1 %;
// with the non-temporal policy 128 +11 %, 32 +3 %, profiles/r06_pfb_ab.txt).
constexpr int kPfbVar64 = 7;
constexpr long long kPfbFramesPerGroup = 64;
template <class PL, int PT>
static void launch_pfb_t(const float2* x, long long n, const float* h, long long M, float2* y,
                         const float2* tw, hipStream_t st) {
  constexpr int G = 256 / PL::N, E = PL::E;
  constexpr int step = E * (PT / cgcd(E, PT));
  // frames per group: a multiple of the unrolled step, so the (PT-1)-row ring
  // prologue stays a small fraction of the group's reads
  constexpr long long want = kPfbFramesPerGroup;
  const long long fpg = ((want + step - 1) / step) * step;
  const long long groups = (M + fpg - 1) / fpg;
  const long long blocks = (groups + G - 1) / G;
  hipLaunchKernelGGL((pfb_kernel<PL, PT, PL::N == 64 ? kPfbVar64 : 3>), dim3((unsigned)blocks), dim3(256), 0, st, x, n, h, M,
                     fpg, y, tw, g_clock_sink);
}

hipError_t launch_pfb(int C, int PT, const float2* x, long long n, const float* h, long long M,
                      float2* y, const float2* tw, hipStream_t st) {
#define VSIG_PFB_CASE(CC, PL)                                                        \
  if (C == CC) {                                                                     \
    switch (PT) {                                                                    \
      case 4: launch_pfb_t<PL, 4>(x, n, h, M, y, tw, st); break;                     \
      case 8: launch_pfb_t<PL, 8>(x, n, h, M, y, tw, st); break;                     \
      case 16: launch_pfb_t<PL, 16>(x, n, h, M, y, tw, st); break;                   \
      default: return hipErrorInvalidValue;                                          \
    }                                                                                \
    return hipGetLastError();                                                        \
  }
  VSIG_PFB_CASE(64, Plan64)
  VSIG_PFB_CASE(128, Plan128)
  VSIG_PFB_CASE(256, Plan256)
#undef VSIG_PFB_CASE
  return hipErrorInvalidValue;
}

}  // namespace vsig
