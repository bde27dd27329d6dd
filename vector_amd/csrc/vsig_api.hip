// C-ABI layer of libvsig.so (declared in include/vsig.h): contexts, plans
// (twiddle tables, filter / template spectra), launch geometry, host staging.
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <string>
#include <vector>

#include "../../include/vsig.h"
#include "vsig_kernels.h"

using vsig::PeakPartial;

struct TimingRec {
  std::vector<std::pair<hipEvent_t, hipEvent_t>> ev;
};

constexpr size_t kRefineKeysBytes = 64;   // refine.hip RefineKeys (the scratch header)
constexpr int kClockSlots = 32;            // per-stage clock sinks (vsig_clock_*)

namespace vsig {
thread_local unsigned long long* g_clock_sink = nullptr;
}

struct vsig_ctx {
  int device = 0;
  hipStream_t own = nullptr;
  hipStream_t stream = nullptr;
  std::map<int, float2*> tw;             // FFT size -> device twiddle table
  PeakPartial* partials = nullptr;       // per-block partials
  long long npartials = 0;
  PeakPartial* result = nullptr;         // scratch device result
  void* stage[3] = {nullptr, nullptr, nullptr};  // host-API device staging
  size_t stage_bytes[3] = {0, 0, 0};
  void* conv[3] = {nullptr, nullptr, nullptr};   // complex128 path: c64 operands / output
  size_t conv_bytes[3] = {0, 0, 0};
  void* rscratch = nullptr;              // refine.hip scratch (keys first)
  size_t rscratch_bytes = 0;
  void* lkeys = nullptr;                 // correlator lane keys (refine column candidates)
  size_t lkeys_bytes = 0;
  void* vscratch = nullptr;              // numpy-order |c| of every output (exact stats)
  size_t vscratch_bytes = 0;
  void* sscratch = nullptr;              // np_stats buffer sums
  size_t sscratch_bytes = 0;
  int refine = 1;                        // exact re-rank of the correlators' peak
  int refine_eps_ppm = 1000;             // fp32 candidate band (relative, ppm of max |c|)
  long long refine_cap = 0;              // opt-in limit on candidate outputs (0: none)
  long long refine_wd_us = 2000000;      // refine_fused watchdog (option "refine_watchdog_us")
  int blas_threads = 1;                  // numpy's OpenBLAS threads (its zdotu splits > 10000 terms)
  bool refine_ran = false;
  struct Chirp { long long M; float2* c; float2* B; };
  std::map<long long, Chirp> chirps;     // Bluestein plans by length (bigfft.hip)
  void* bigtmp = nullptr;                // four-step scratch
  size_t bigtmp_bytes = 0;
  void* spec[2] = {nullptr, nullptr};    // resample / channel spectra
  size_t spec_bytes[2] = {0, 0};
  std::string err;
  bool timing = false;
  std::map<std::string, TimingRec> timers;
  // "refine_async": the xcorr handle's refine on its own stream behind ev_corr,
  // ev_ref recorded after it; joined (the context stream waits on ev_ref) before
  // any reuse of its scratch -- see join_refine
  int refine_async = 0;
  hipStream_t rstream = nullptr;
  hipEvent_t ev_corr = nullptr, ev_ref = nullptr;
  bool refine_pending = false;           // an async refine was enqueued
  bool refine_joined = false;            // ... and joined on refine_joined_on
  hipStream_t refine_joined_on = nullptr;
  bool clock = false;                    // per-stage clock sinks on (vsig_clock_enable)
  unsigned long long* clkbuf = nullptr;  // kClockSlots x {shader ticks, 100 MHz ticks}
  std::map<std::string, int> clkslot;
};

struct vsig_fir {
  vsig_ctx* ctx;
  int ntaps, decim, M;
  long long hop;
  float2* Hs;
  float2* G = nullptr;   // D = 4 polyphase component filters (M = 1024)
  // more than kFirPartTaps taps: undecimated parts of kFirPartTaps taps each,
  // summed with their delays (fir_part_accum); z: one part's output
  std::vector<vsig_fir*> parts;
  float2* z = nullptr;
  size_t zbytes = 0;
};
constexpr int kFirPartTaps = 8192;

// A correlation template: L <= 8192 one spectrum of M points; longer
// templates a spectrum per 8192-sample chunk (M = 16384), applied as a sum of
// passes accumulated in c (a scratch kept with the handle when the caller
// passes none).  tmpl: the template on the device (refine pass).
struct vsig_xcorr {
  vsig_ctx* ctx;
  long long L;
  int M;
  std::vector<float2*> Ps;
  float2* tmpl = nullptr;
  void* cbuf = nullptr;
  size_t cbuf_bytes = 0;
};

namespace {

int fail(vsig_ctx* c, int code, const std::string& msg) {
  if (c) c->err = msg;
  return code;
}

// The context stream waits for the last asynchronous refine (once per stream
// after each refine): called before anything reuses the refine's scratch or
// operands -- every scratch / partials / staging allocation and use below goes
// through ensure_buf / ensure_partials / ensure_stage -- and by vsig_refine_join.
void join_refine(vsig_ctx* c) {
  if (!c->refine_pending) return;
  if (c->refine_joined && c->refine_joined_on == c->stream) return;
  (void)hipStreamWaitEvent(c->stream, c->ev_ref, 0);
  c->refine_joined = true;
  c->refine_joined_on = c->stream;
}

#define HIPCHK(ctx, expr)                                                              \
  do {                                                                                 \
    hipError_t e_ = (expr);                                                            \
    if (e_ != hipSuccess)                                                              \
      return fail(ctx, e_ == hipErrorOutOfMemory ? VSIG_E_NOMEM : VSIG_E_HIP,          \
                  std::string(#expr) + ": " + hipGetErrorString(e_));                 \
  } while (0)

// Twiddle table of the plan for N (see fft_engine.hpp):
// tw[off_p + (r-1)*Ns + k] = exp(-2 pi i r k / (Ns R)), passes p >= 1.
int get_twiddles(vsig_ctx* c, int N, const float2** out) {
  auto it = c->tw.find(N);
  if (it != c->tw.end()) { *out = it->second; return VSIG_OK; }
  int R[16], np = 0;
  if (vsig::plan_info(N, R, &np) != hipSuccess)
    return fail(c, VSIG_E_UNSUPPORTED, "FFT size " + std::to_string(N) + " not supported");
  // (N < 0 keys an alternative plan of |N| points)
  std::vector<float2> h;
  int Ns = R[0];
  for (int p = 1; p < np; ++p) {
    for (int r = 1; r < R[p]; ++r)
      for (int k = 0; k < Ns; ++k) {
        const double a = -2.0 * M_PI * (double)r * (double)k / ((double)Ns * R[p]);
        h.push_back(make_float2((float)std::cos(a), (float)std::sin(a)));
      }
    Ns *= R[p];
  }
  if (h.empty()) h.push_back(make_float2(1.f, 0.f));
  float2* d = nullptr;
  HIPCHK(c, hipMalloc(&d, h.size() * sizeof(float2)));
  HIPCHK(c, hipMemcpy(d, h.data(), h.size() * sizeof(float2), hipMemcpyHostToDevice));
  c->tw[N] = d;
  *out = d;
  return VSIG_OK;
}

// Two-level table for plan key N (cached under key N + 2^20).
int get_tw2(vsig_ctx* c, int N, const float2** out) {
  const int key = N + (1 << 20);
  auto it = c->tw.find(key);
  if (it != c->tw.end()) { *out = it->second; return VSIG_OK; }
  int S = 0, hi = 0;
  if (vsig::tw2_info(N, &S, &hi) != hipSuccess)
    return fail(c, VSIG_E_UNSUPPORTED, "FFT size " + std::to_string(N) + " not supported");
  const int n = N < 0 ? -N : N;
  std::vector<float2> h;
  for (int i = 0; i < hi; ++i) {
    const double a = -2.0 * M_PI * (double)i * (double)(1 << S) / (double)n;
    h.push_back(make_float2((float)std::cos(a), (float)std::sin(a)));
  }
  for (int i = 0; i < (1 << S); ++i) {
    const double a = -2.0 * M_PI * (double)i / (double)n;
    h.push_back(make_float2((float)std::cos(a), (float)std::sin(a)));
  }
  float2* d = nullptr;
  HIPCHK(c, hipMalloc(&d, h.size() * sizeof(float2)));
  HIPCHK(c, hipMemcpy(d, h.data(), h.size() * sizeof(float2), hipMemcpyHostToDevice));
  c->tw[key] = d;
  *out = d;
  return VSIG_OK;
}

// W_M^t for t < T (the per-thread twiddle of the half-frame correlator),
// cached under key M + 2^21.
int get_half_tw(vsig_ctx* c, int M, int T, const float2** out) {
  const int key = M + (1 << 21);
  auto it = c->tw.find(key);
  if (it != c->tw.end()) { *out = it->second; return VSIG_OK; }
  std::vector<float2> h;
  for (int t = 0; t < T; ++t) {
    const double a = -2.0 * M_PI * (double)t / (double)M;
    h.push_back(make_float2((float)std::cos(a), (float)std::sin(a)));
  }
  float2* d = nullptr;
  HIPCHK(c, hipMalloc(&d, h.size() * sizeof(float2)));
  HIPCHK(c, hipMemcpy(d, h.data(), h.size() * sizeof(float2), hipMemcpyHostToDevice));
  c->tw[key] = d;
  *out = d;
  return VSIG_OK;
}

int ensure_partials(vsig_ctx* c, long long n) {
  join_refine(c);
  if (n <= c->npartials) return VSIG_OK;
  if (c->partials) (void)hipFree(c->partials);
  c->partials = nullptr;
  c->npartials = 0;
  long long cap = n < 4096 ? 4096 : n + n / 4;
  // + the first-level buffer of a two-level finalize, right after the partials,
  // and the fused finalize's block counter (zero between launches)
  HIPCHK(c, hipMalloc(&c->partials, (cap + vsig::kFinalizeTmp + vsig::kCounterRecs) * sizeof(PeakPartial)));
  HIPCHK(c, hipMemset(c->partials + cap + vsig::kFinalizeTmp, 0, vsig::kCounterRecs * sizeof(PeakPartial)));
  c->npartials = cap;
  return VSIG_OK;
}

int ensure_stage(vsig_ctx* c, int i, size_t bytes) {
  join_refine(c);
  if (bytes <= c->stage_bytes[i]) return VSIG_OK;
  if (c->stage[i]) (void)hipFree(c->stage[i]);
  c->stage[i] = nullptr;
  c->stage_bytes[i] = 0;
  HIPCHK(c, hipMalloc(&c->stage[i], bytes));
  c->stage_bytes[i] = bytes;
  return VSIG_OK;
}

// Event pair around one kernel launch (only when timing is on); with the
// clock option on, the stage's clock sink for the launches in its scope.
struct Timed {
  vsig_ctx* c;
  hipEvent_t b = nullptr, e = nullptr;
  const char* name;
  unsigned long long* prev_sink;
  hipStream_t st;
  Timed(vsig_ctx* c_, const char* n, hipStream_t s = nullptr)
      : c(c_), name(n), prev_sink(vsig::g_clock_sink), st(s ? s : c_->stream) {
    if (c->clock && c->clkbuf) {
      auto it = c->clkslot.find(name);
      int slot = -1;
      if (it != c->clkslot.end()) slot = it->second;
      else if ((int)c->clkslot.size() < kClockSlots) slot = c->clkslot[name] = (int)c->clkslot.size();
      if (slot >= 0) vsig::g_clock_sink = c->clkbuf + 2 * slot;
    }
    if (!c->timing) return;
    if (hipEventCreate(&b) != hipSuccess || hipEventCreate(&e) != hipSuccess) { b = e = nullptr; return; }
    (void)hipEventRecord(b, st);
  }
  ~Timed() {
    vsig::g_clock_sink = prev_sink;
    if (!b) return;
    (void)hipEventRecord(e, st);
    c->timers[name].ev.emplace_back(b, e);
  }
};

bool pow2_in(long long v, long long lo, long long hi) {
  return v >= lo && v <= hi && (v & (v - 1)) == 0;
}

// Overlap-save block sizes (measured best on MI355X for the chain's sizes).
int os_size_fir(int ntaps) {
  if (ntaps <= 256) return 1024;      // one-wave blocks; hop >= 769 (measured best at 255 taps)
  if (ntaps <= 512) return 4096;
  if (ntaps <= 2048) return 8192;
  if (ntaps <= 8192) return 16384;
  return 0;
}
// templates of 8193 .. 16384 samples use M = 32768 (measured slower than
// M = 16384 for shorter ones, xcorr.hip PlanX32k)
int os_size_xcorr(long long L) {
  if (L <= 1024) return 4096;
  if (L <= 2048) return 8192;
  if (L <= 8192) return 16384;
  if (L <= 16384) return 32768;
  return 0;
}

int ensure_buf(vsig_ctx* c, void** buf, size_t* have, size_t bytes) {
  join_refine(c);
  if (bytes <= *have) return VSIG_OK;
  if (*buf) (void)hipFree(*buf);
  *buf = nullptr;
  *have = 0;
  HIPCHK(c, hipMalloc(buf, bytes));
  *have = bytes;
  return VSIG_OK;
}

// FFT_M(zero-padded u[0..len)) / M into a new device buffer (natural order;
// M > 16384 by the four-step passes of bigfft.hip).
int big_plan_fwd(vsig_ctx* c, long long M, const float2* u, long long len, float2* S);
int make_spectrum(vsig_ctx* c, const float2* u_dev, int len, int M, float2** out) {
  float2* S = nullptr;
  HIPCHK(c, hipMalloc(&S, (size_t)M * sizeof(float2)));
  if (M > 16384) {
    const int rc = big_plan_fwd(c, M, u_dev, len, S);
    if (rc) { (void)hipFree(S); return rc; }
    *out = S;
    return VSIG_OK;
  }
  const float2* tw;
  int rc = get_twiddles(c, M, &tw);
  if (rc) { (void)hipFree(S); return rc; }
  hipError_t e = vsig::launch_spectrum_prep(M, u_dev, len, 1.0f / (float)M, S, tw, c->stream);
  if (e != hipSuccess) { (void)hipFree(S); return fail(c, VSIG_E_HIP, hipGetErrorString(e)); }
  *out = S;
  return VSIG_OK;
}

int finalize_peak(vsig_ctx* c, long long nparts, int sqrt_max, vsig_peak_t* peak_dev) {
  PeakPartial* dst = peak_dev ? reinterpret_cast<PeakPartial*>(peak_dev) : c->result;
  HIPCHK(c, vsig::launch_partial_finalize(c->partials, nparts, sqrt_max, dst,
                                          c->partials + c->npartials, c->stream));
  return VSIG_OK;
}

// Operands of the refine pass: np.correlate(a, v) in the final output
// space (o <-> full index F + o), complex128 or complex64 on the device.
struct RefineOperands {
  const void* a; long long na;
  const void* v; long long nv;
  int c128;
  long long F;
};

// Re-rank the peak record rec (finalized, max |c|) over the outputs within the
// fp32 band; src: the correlator's wave partials (geometry of an M-point
// launch with raw->final reversal rev) or, if c64 != null, a stored c64 array.
// fused: the correlator's partials are not finalized yet -- the refine's first
// launch finalizes them into rec and selects (thread columns when lkeys).
int run_refine(vsig_ctx* c, const RefineOperands& op, long long nout, int M, long long hop,
               long long nparts, int rev, const float2* c64, PeakPartial* rec, void* out128,
               bool fused = false, const unsigned* lkeys = nullptr, bool async = false) {
  c->refine_ran = false;
  if (!c->refine) return fused ? fail(c, VSIG_E_INVALID, "refine: fused finalize with refine off")
                             : VSIG_OK;
  vsig::RefineArgs r{};
  r.a = op.a; r.na = op.na; r.v = op.v; r.nv = op.nv; r.c128 = op.c128;
  r.nout = nout; r.F = op.F; r.rev = rev;
  if (c64) {
    r.from_array = 1; r.c64 = c64; r.Q = 1; r.stride = 0; r.waves = 1; r.hop = 64;
    r.wstep = 64; r.rsub = 1;
  } else {
    int waves, Q, stride, plan, wstep, rsub;
    if (vsig::xcorr_geom(M, &waves, &Q, &stride, &plan, &wstep, &rsub) != hipSuccess)
      return fail(c, VSIG_E_INVALID, "refine: no correlator geometry for M");
    r.parts = c->partials; r.nparts = nparts; r.hop = hop;
    r.waves = waves; r.Q = Q; r.stride = stride; r.wstep = wstep; r.rsub = rsub;
    if (fused) {
      r.finalize = 1;
      r.tmp = c->partials + c->npartials;
      r.done = reinterpret_cast<unsigned long long*>(r.tmp + vsig::kFinalizeTmp);
    }
    if (lkeys) {                 // items = thread columns of Q rows, one unit each
      r.cols = Q; r.lkeys = lkeys; r.Q = 1;
    }
  }
  r.eps = c->refine_eps_ppm * 1e-6;
  r.blas_threads = c->blas_threads;
  r.cap = c->refine_cap;
  r.wd_ticks = (unsigned long long)c->refine_wd_us * 100ull;   // s_memrealtime: 100 MHz
  const size_t need = vsig::refine_scratch_bytes(r);
  const bool fresh = need > c->rscratch_bytes;
  // a watchdog fire of an earlier pass whose status nobody read (device-tensor
  // callers) lives in the old scratch's sticky fault word: carry it into the
  // new one, so vsig_refine_status still reports 3 ("fired in some pass since
  // the last call"), and clear the fused launch's counters as that report
  // does (a fire can leave them inconsistent)
  unsigned long long pending_fault = 0;
  if (fresh && c->rscratch) {
    unsigned long long keys[6];      // refine.hip RefineKeys: ..., fault
    HIPCHK(c, hipMemcpyAsync(keys, c->rscratch, sizeof(keys), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    pending_fault = keys[5];
  }
  int rc = ensure_buf(c, &c->rscratch, &c->rscratch_bytes, need);
  if (rc) return rc;
  // a new scratch starts with zero keys (the sticky fault word is read by
  // vsig_refine_status; the finalize resets only the per-launch words)
  if (fresh) HIPCHK(c, hipMemsetAsync(c->rscratch, 0, kRefineKeysBytes, c->stream));
  if (pending_fault) {
    HIPCHK(c, hipMemcpyAsync(static_cast<unsigned long long*>(c->rscratch) + 5, &pending_fault,
                             sizeof(pending_fault), hipMemcpyHostToDevice, c->stream));
    if (c->partials)
      HIPCHK(c, hipMemsetAsync(c->partials + c->npartials + vsig::kFinalizeTmp, 0,
                               vsig::kCounterRecs * sizeof(PeakPartial), c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));     // pending_fault is a host local
  }
  r.scratch = c->rscratch;
  r.rec = rec;
  r.out128 = out128;
  if (async && c->refine_async) {
    // on the refine stream behind the correlator; ev_ref marks its end
    HIPCHK(c, hipEventRecord(c->ev_corr, c->stream));
    HIPCHK(c, hipStreamWaitEvent(c->rstream, c->ev_corr, 0));
    {
      Timed t(c, "refine", c->rstream);
      HIPCHK(c, vsig::launch_refine(r, c->rstream));
    }
    HIPCHK(c, hipEventRecord(c->ev_ref, c->rstream));
    c->refine_pending = true;
    c->refine_joined = false;
    c->refine_ran = true;
    return VSIG_OK;
  }
  Timed t(c, "refine");
  HIPCHK(c, vsig::launch_refine(r, c->stream));
  c->refine_ran = true;
  return VSIG_OK;
}

// W_M^m for the four-step twiddles (bigfft.hip): two-level table
// A[i] = W_M^(i 2^S), B[j] = W_M^j, S = ceil(log2 M / 2), built in double.
int get_tw_big(vsig_ctx* c, long long M, const float2** out, int* S, int* hiA) {
  int lg = 0;
  while ((1LL << lg) < M) ++lg;
  *S = (lg + 1) / 2;
  *hiA = (int)(M >> *S);
  const int key = (1 << 22) + lg;
  auto it = c->tw.find(key);
  if (it != c->tw.end()) { *out = it->second; return VSIG_OK; }
  std::vector<float2> h;
  for (long long i = 0; i < *hiA; ++i) {
    const double a = -2.0 * M_PI * (double)(i << *S) / (double)M;
    h.push_back(make_float2((float)std::cos(a), (float)std::sin(a)));
  }
  for (long long j = 0; j < (1LL << *S); ++j) {
    const double a = -2.0 * M_PI * (double)j / (double)M;
    h.push_back(make_float2((float)std::cos(a), (float)std::sin(a)));
  }
  float2* d = nullptr;
  HIPCHK(c, hipMalloc(&d, h.size() * sizeof(float2)));
  HIPCHK(c, hipMemcpy(d, h.data(), h.size() * sizeof(float2), hipMemcpyHostToDevice));
  c->tw[key] = d;
  *out = d;
  return VSIG_OK;
}

constexpr long long kBigMax = 1LL << 28;    // largest four-step transform

// split_channels.py's frequency axis, as numpy forms it: fftfreq(n, 1/sr)[k]
// * sr + CENTER_FREQ (k >= 0 here, or -1), no contraction into FMAs.
#pragma clang fp contract(off)
double channel_freq(long long k, long long n, double sr, double center) {
  const double d = 1.0 / sr;
  const double val = 1.0 / ((double)n * d);
  const double f = (double)k * val;
  const double g = f * sr;
  return g + center;
}
#pragma clang fp contract(on)

// Twiddles of a (four-step) transform of M points.
struct BigPlan {
  long long M;
  int N1, N2, S, hiA;
  const float2 *tw1, *tw2, *t2;
};
int big_plan(vsig_ctx* c, long long M, BigPlan* p) {
  p->M = M;
  vsig::bigfft_split(M, &p->N1, &p->N2);
  int rc;
  p->tw1 = p->t2 = nullptr;
  p->S = p->hiA = 0;
  if ((rc = get_twiddles(c, p->N2, &p->tw2))) return rc;
  if (p->N1 > 1) {
    if ((rc = get_twiddles(c, p->N1, &p->tw1))) return rc;
    if ((rc = get_tw_big(c, M, &p->t2, &p->S, &p->hiA))) return rc;
  }
  return VSIG_OK;
}

// S = FFT_M(zero-padded u[0..len)) / M in natural order (four-step, M > 16384).
int big_plan_fwd(vsig_ctx* c, long long M, const float2* u, long long len, float2* S) {
  BigPlan bp;
  int rc = big_plan(c, M, &bp);
  if (rc) return rc;
  if ((rc = ensure_buf(c, &c->bigtmp, &c->bigtmp_bytes, (size_t)M * sizeof(float2)))) return rc;
  vsig::BigIn in{u, 0, 0, 1, len, nullptr, nullptr, 0, 1.0f / (float)M};
  HIPCHK(c, vsig::launch_bf_col(bp.N1, bp.N2, 1, in, (float2*)c->bigtmp, bp.tw1, bp.t2, bp.S, bp.hiA,
                                c->stream));
  HIPCHK(c, vsig::launch_bf_row(3, bp.N1, bp.N2, 1, (float2*)c->bigtmp, nullptr, bp.tw2, 1.0f,
                                reinterpret_cast<float*>(S), 0, c->stream));
  return VSIG_OK;
}

// Bluestein plan for length N: chirp c[N] and B = FFT_M(b) / M (permuted order
// for the four-step sizes), M = the power of two >= max(256, 2N - 1).
int chirp_plan(vsig_ctx* c, long long N, vsig_ctx::Chirp** out) {
  auto it = c->chirps.find(N);
  if (it != c->chirps.end()) { *out = &it->second; return VSIG_OK; }
  long long M = 256;
  while (M < 2 * N - 1) M *= 2;
  if (M > kBigMax) return fail(c, VSIG_E_UNSUPPORTED, "transform length above 2^27");
  BigPlan bp;
  int rc = big_plan(c, M, &bp);
  if (rc) return rc;
  float2 *cv = nullptr, *B = nullptr, *b = nullptr;
  auto cleanup = [&]() { if (cv) (void)hipFree(cv); if (B) (void)hipFree(B); if (b) (void)hipFree(b); };
  if (hipMalloc(&cv, N * sizeof(float2)) != hipSuccess || hipMalloc(&B, M * sizeof(float2)) != hipSuccess ||
      hipMalloc(&b, M * sizeof(float2)) != hipSuccess) {
    cleanup();
    return fail(c, VSIG_E_NOMEM, "Bluestein plan allocation");
  }
  hipError_t e = vsig::launch_bf_chirp(N, M, cv, b, c->stream);
  vsig::BigIn in{b, 0, 0, 1, M, nullptr, nullptr, 0, 1.0f / (float)M};
  if (e == hipSuccess) {
    if (bp.N1 == 1) {
      vsig::BigOut o{B, 0, 0, M, nullptr, 0, 1.0f};
      e = vsig::launch_bf_small(1, (int)M, 1, in, o, nullptr, bp.tw2, c->stream);
    } else {
      e = vsig::launch_bf_col(bp.N1, bp.N2, 1, in, B, bp.tw1, bp.t2, bp.S, bp.hiA, c->stream);
      if (e == hipSuccess)
        e = vsig::launch_bf_row(1, bp.N1, bp.N2, 1, B, nullptr, bp.tw2, 1.0f, nullptr, 0, c->stream);
    }
  }
  if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
  (void)hipFree(b);
  b = nullptr;
  if (e != hipSuccess) { cleanup(); return fail(c, VSIG_E_HIP, hipGetErrorString(e)); }
  auto& ch = c->chirps[N];
  ch = vsig_ctx::Chirp{M, cv, B};
  *out = &ch;
  return VSIG_OK;
}

// DFT of any length N (batch frames): X[k] = sum_n x[n] W_N^(nk), or the
// inverse (conj) form; in / out describe the operands (their chirp / conj
// fields are set here), out.scale includes any 1/N.
int dft_any(vsig_ctx* c, long long N, long long batch, vsig::BigIn in, vsig::BigOut out, bool inverse) {
  vsig_ctx::Chirp* ch;
  int rc = chirp_plan(c, N, &ch);
  if (rc) return rc;
  BigPlan bp;
  if ((rc = big_plan(c, ch->M, &bp))) return rc;
  in.chirp = ch->c;
  in.conj = inverse ? 1 : 0;
  in.nvalid = in.nvalid < N ? in.nvalid : N;
  out.chirp = ch->c;
  out.conj = inverse ? 1 : 0;
  if (bp.N1 == 1) {
    HIPCHK(c, vsig::launch_bf_small(0, (int)ch->M, batch, in, out, ch->B, bp.tw2, c->stream));
    return VSIG_OK;
  }
  if ((rc = ensure_buf(c, &c->bigtmp, &c->bigtmp_bytes, (size_t)(batch * ch->M) * sizeof(float2)))) return rc;
  float2* tmp = static_cast<float2*>(c->bigtmp);
  HIPCHK(c, vsig::launch_bf_col(bp.N1, bp.N2, batch, in, tmp, bp.tw1, bp.t2, bp.S, bp.hiA, c->stream));
  HIPCHK(c, vsig::launch_bf_row(0, bp.N1, bp.N2, batch, tmp, ch->B, bp.tw2, 1.0f, nullptr, 0, c->stream));
  HIPCHK(c, vsig::launch_bf_icol(bp.N1, bp.N2, batch, tmp, out, bp.tw1, bp.t2, bp.S, bp.hiA, c->stream));
  return VSIG_OK;
}

}  // namespace

extern "C" {

#ifndef VSIG_SRC_HASH
#define VSIG_SRC_HASH "unknown"
#endif
int vsig_version(void) { return 2; }
const char* vsig_build_id(void) { return VSIG_SRC_HASH; }

const char* vsig_errstr(int s) {
  switch (s) {
    case VSIG_OK: return "ok";
    case VSIG_E_INVALID: return "invalid argument";
    case VSIG_E_HIP: return "HIP runtime error";
    case VSIG_E_NOMEM: return "device out of memory";
    case VSIG_E_UNSUPPORTED: return "unsupported size";
    case VSIG_E_NODEVICE: return "no HIP device";
    case VSIG_E_REFINE: return "exact-argmax refine faulted (watchdog); peak record invalid";
    default: return "unknown status";
  }
}

int vsig_init(int device, vsig_ctx** out) {
  if (!out) return VSIG_E_INVALID;
  *out = nullptr;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return VSIG_E_NODEVICE;
  if (device < 0 || device >= ndev) return VSIG_E_INVALID;
  if (hipSetDevice(device) != hipSuccess) return VSIG_E_HIP;
  vsig_ctx* c = new vsig_ctx();
  c->device = device;
  if (hipStreamCreateWithFlags(&c->own, hipStreamNonBlocking) != hipSuccess) { delete c; return VSIG_E_HIP; }
  c->stream = c->own;
  if (hipMalloc(&c->result, sizeof(PeakPartial)) != hipSuccess) { vsig_free(c); return VSIG_E_NOMEM; }
  *out = c;
  return VSIG_OK;
}

int vsig_timing_reset(vsig_ctx* c) {
  if (!c) return VSIG_E_INVALID;
  for (auto& kv : c->timers)
    for (auto& p : kv.second.ev) { (void)hipEventDestroy(p.first); (void)hipEventDestroy(p.second); }
  c->timers.clear();
  return VSIG_OK;
}

void vsig_free(vsig_ctx* c) {
  if (!c) return;
  (void)hipSetDevice(c->device);
  (void)hipDeviceSynchronize();
  vsig_timing_reset(c);
  for (auto& kv : c->tw) (void)hipFree(kv.second);
  if (c->partials) (void)hipFree(c->partials);
  if (c->result) (void)hipFree(c->result);
  for (int i = 0; i < 3; ++i) if (c->stage[i]) (void)hipFree(c->stage[i]);
  for (int i = 0; i < 3; ++i) if (c->conv[i]) (void)hipFree(c->conv[i]);
  if (c->rscratch) (void)hipFree(c->rscratch);
  if (c->lkeys) (void)hipFree(c->lkeys);
  if (c->vscratch) (void)hipFree(c->vscratch);
  if (c->sscratch) (void)hipFree(c->sscratch);
  for (auto& kv : c->chirps) { (void)hipFree(kv.second.c); (void)hipFree(kv.second.B); }
  if (c->bigtmp) (void)hipFree(c->bigtmp);
  for (int i = 0; i < 2; ++i) if (c->spec[i]) (void)hipFree(c->spec[i]);
  if (c->clkbuf) (void)hipFree(c->clkbuf);
  if (c->rstream) (void)hipStreamDestroy(c->rstream);
  if (c->ev_corr) (void)hipEventDestroy(c->ev_corr);
  if (c->ev_ref) (void)hipEventDestroy(c->ev_ref);
  if (c->own) (void)hipStreamDestroy(c->own);
  delete c;
}

const char* vsig_last_error(const vsig_ctx* c) { return c ? c->err.c_str() : "null context"; }

void* vsig_get_stream(vsig_ctx* c) { return c ? (void*)c->stream : nullptr; }

int vsig_set_stream(vsig_ctx* c, void* s) {
  if (!c) return VSIG_E_INVALID;
  c->stream = (hipStream_t)s;  // NULL is the device's default (null) stream
  return VSIG_OK;
}

int vsig_set_option(vsig_ctx* c, const char* key, int value) {
  if (!c || !key) return VSIG_E_INVALID;
  const std::string k(key);
  if (k == "refine") {
    c->refine = value != 0;
  } else if (k == "refine_eps_ppm") {
    if (value < 1 || value > 500000) return fail(c, VSIG_E_INVALID, "refine_eps_ppm must be in [1, 500000]");
    c->refine_eps_ppm = value;
  } else if (k == "refine_cap") {
    if (value != 0 && value < 4096) return fail(c, VSIG_E_INVALID, "refine_cap must be 0 or >= 4096");
    c->refine_cap = value;
  } else if (k == "refine_watchdog_us") {
    if (value < 1) return fail(c, VSIG_E_INVALID, "refine_watchdog_us must be >= 1");
    c->refine_wd_us = value;
  } else if (k == "blas_threads") {
    if (value < 1 || value > 1024) return fail(c, VSIG_E_INVALID, "blas_threads must be in [1, 1024]");
    c->blas_threads = value;
  } else if (k == "refine_async") {
    if (value && !c->rstream) {
      // the highest stream priority: the refine's few blocks are dispatched
      // ahead of the next step's FIR blocks queued beside them (at the default
      // priority they waited for CU slots behind the FIR and spun for ~3 ms)
      int lo = 0, hi = 0;
      if (hipDeviceGetStreamPriorityRange(&lo, &hi) != hipSuccess) lo = hi = 0;
      HIPCHK(c, hipStreamCreateWithPriority(&c->rstream, hipStreamNonBlocking, hi));
      HIPCHK(c, hipEventCreateWithFlags(&c->ev_corr, hipEventDisableTiming));
      HIPCHK(c, hipEventCreateWithFlags(&c->ev_ref, hipEventDisableTiming));
    }
    if (!value) join_refine(c);
    c->refine_async = value != 0;
  } else {
    return fail(c, VSIG_E_INVALID, "unknown option " + k);
  }
  return VSIG_OK;
}

int vsig_get_option(const vsig_ctx* c, const char* key, int* value) {
  if (!c || !key || !value) return VSIG_E_INVALID;
  const std::string k(key);
  if (k == "refine") *value = c->refine;
  else if (k == "refine_eps_ppm") *value = c->refine_eps_ppm;
  else if (k == "refine_cap") *value = (int)c->refine_cap;
  else if (k == "refine_watchdog_us") *value = (int)c->refine_wd_us;
  else if (k == "blas_threads") *value = c->blas_threads;
  else if (k == "refine_async") *value = c->refine_async;
  else return VSIG_E_INVALID;
  return VSIG_OK;
}

void* vsig_refine_stream(vsig_ctx* c) {
  if (!c) return nullptr;
  return (void*)(c->refine_async && c->rstream ? c->rstream : c->stream);
}

int vsig_refine_join(vsig_ctx* c) {
  if (!c) return VSIG_E_INVALID;
  join_refine(c);
  return VSIG_OK;
}

int vsig_refine_status(vsig_ctx* c, int32_t* status, int64_t* candidates) {
  if (!c || !status || !candidates) return VSIG_E_INVALID;
  *status = 2;
  *candidates = 0;
  join_refine(c);
  if (!c->refine_ran || !c->rscratch) return VSIG_OK;
  // refine.hip RefineKeys: count, lo_inv, hi_p1, status, done, fault
  unsigned long long keys[6];
  HIPCHK(c, hipMemcpyAsync(keys, c->rscratch, sizeof(keys), hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  *candidates = (int64_t)keys[0];
  if (keys[5]) {
    // a watchdog fired in some refine since the last report: status 3 once,
    // then the fused launch's counters and the keys (fault word included) are
    // cleared -- a fire can leave them inconsistent, and the next launch must
    // start from zero -- and the record is not to be trusted until then
    *status = 3;
    HIPCHK(c, hipMemsetAsync(c->rscratch, 0, kRefineKeysBytes, c->stream));
    if (c->partials)
      HIPCHK(c, hipMemsetAsync(c->partials + c->npartials + vsig::kFinalizeTmp, 0,
                               vsig::kCounterRecs * sizeof(PeakPartial), c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    c->refine_ran = false;
    return VSIG_OK;
  }
  *status = keys[3] ? 1 : 0;
  return VSIG_OK;
}

#ifdef VSIG_TUNING
int vsig_fft_bench(vsig_ctx* c, int key, void* io, int frames, int iters, int twl) {
  if (!c || !io || frames < 1 || iters < 1) return fail(c, VSIG_E_INVALID, "bad arguments");
  const float2* tw;
  int rc = twl == 1 ? get_tw2(c, key, &tw) : get_twiddles(c, key, &tw);
  if (rc) return rc;
  Timed t(c, "fft_bench");
  HIPCHK(c, vsig::launch_fft_bench(key, (float2*)io, frames, iters, tw, twl, c->stream));
  return VSIG_OK;
}

int vsig_copy_bench(vsig_ctx* c, const void* x, int64_t n, void* y, int variant, int grid) {
  if (!c || !x || !y || n < 0) return fail(c, VSIG_E_INVALID, "bad arguments");
  Timed t(c, "copy_bench");
  HIPCHK(c, vsig::launch_copy_probe((const float2*)x, n, (float2*)y, variant, grid, c->stream));
  return VSIG_OK;
}
#endif

int vsig_copy_dev(vsig_ctx* c, void* dst, const void* src, int64_t bytes) {
  if (!c || !dst || !src || bytes < 0) return fail(c, VSIG_E_INVALID, "bad copy");
  if (bytes) HIPCHK(c, hipMemcpyAsync(dst, src, (size_t)bytes, hipMemcpyDefault, c->stream));
  return VSIG_OK;
}

int vsig_synchronize(vsig_ctx* c) {
  if (!c) return VSIG_E_INVALID;
  join_refine(c);
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return VSIG_OK;
}

int vsig_clock_enable(vsig_ctx* c, int on) {
  if (!c) return VSIG_E_INVALID;
  if (on) {
    if (!c->clkbuf) HIPCHK(c, hipMalloc(&c->clkbuf, 2 * kClockSlots * sizeof(unsigned long long)));
    HIPCHK(c, hipMemsetAsync(c->clkbuf, 0, 2 * kClockSlots * sizeof(unsigned long long), c->stream));
  }
  c->clock = on != 0;
  return VSIG_OK;
}

int vsig_clock_read(vsig_ctx* c, const char* kernel, double* ghz, int64_t* ticks) {
  if (!c || !kernel || !ghz) return VSIG_E_INVALID;
  *ghz = 0.0;
  if (ticks) *ticks = 0;
  auto it = c->clkslot.find(kernel);
  if (!c->clkbuf || it == c->clkslot.end()) return VSIG_OK;
  unsigned long long h[2] = {0, 0};
  HIPCHK(c, hipStreamSynchronize(c->stream));
  HIPCHK(c, hipMemcpy(h, c->clkbuf + 2 * it->second, sizeof(h), hipMemcpyDeviceToHost));
  if (h[1]) *ghz = (double)h[0] / (double)h[1] * 0.1;      // s_memrealtime runs at 100 MHz
  if (ticks) *ticks = (int64_t)h[1];
  return VSIG_OK;
}

int vsig_timing_enable(vsig_ctx* c, int on) {
  if (!c) return VSIG_E_INVALID;
  c->timing = on != 0;
  return VSIG_OK;
}

int vsig_timing_read(vsig_ctx* c, const char* kernel, double* total_ms, int64_t* launches) {
  if (!c || !kernel || !total_ms || !launches) return VSIG_E_INVALID;
  *total_ms = 0.0;
  *launches = 0;
  auto it = c->timers.find(kernel);
  if (it == c->timers.end()) return VSIG_OK;
  for (auto& p : it->second.ev) {
    HIPCHK(c, hipEventSynchronize(p.second));
    float ms = 0.f;
    HIPCHK(c, hipEventElapsedTime(&ms, p.first, p.second));
    *total_ms += ms;
    *launches += 1;
  }
  return VSIG_OK;
}

// ---------------------------------------------------------------- spectrum
int vsig_psd_c64_dev(vsig_ctx* c, const void* x, int64_t n, int64_t stride, const float* win,
                     int32_t nperseg, int64_t hop, int32_t nfft, float scale, int32_t shift,
                     float* sxx, int64_t nframes) {
  if (!c || !x || !win || !sxx) return fail(c, VSIG_E_INVALID, "null pointer");
  if (stride < 1) return fail(c, VSIG_E_INVALID, "stride must be >= 1");
  if (nperseg < 1 || nperseg > nfft || hop < 1 || n < nperseg)
    return fail(c, VSIG_E_INVALID, "need 1 <= nperseg <= nfft, hop >= 1, n >= nperseg");
  if (nframes != (n - nperseg) / hop + 1) return fail(c, VSIG_E_INVALID, "nframes mismatch");
  if (!pow2_in(nfft, 64, kBigMax)) {
    // any other length: Bluestein per frame (bigfft.hip), |X|^2 stored by the
    // transform's output stage; frames in batches of <= 256 MB of scratch
    if (2LL * nfft - 1 > kBigMax) return fail(c, VSIG_E_UNSUPPORTED, "nfft above 2^27");
    vsig_ctx::Chirp* ch;
    int rc = chirp_plan(c, nfft, &ch);
    if (rc) return rc;
    long long fb = ch->M <= 16384 ? nframes : (256LL << 20) / (ch->M * 8);
    if (fb < 1) fb = 1;
    Timed t(c, "psd");
    for (long long f0 = 0; f0 < nframes; f0 += fb) {
      const long long nb = nframes - f0 < fb ? nframes - f0 : fb;
      vsig::BigIn in{(const float2*)x + f0 * hop * stride, 0, hop * stride, stride, nperseg, nullptr,
                     win, 0, 1.0f};
      vsig::BigOut out{sxx + f0 * (long long)nfft, 4, nfft, nfft, nullptr, 0, scale, shift ? 1 : 0};
      if ((rc = dft_any(c, nfft, nb, in, out, false))) return rc;
    }
    return VSIG_OK;
  }
  if (nfft > 16384) {          // long frames: four-step FFT per frame (bigfft.hip)
    BigPlan bp;
    int rc = big_plan(c, nfft, &bp);
    if (rc) return rc;
    long long fb = (256LL << 20) / ((long long)nfft * 8);   // frames per 256 MB of scratch
    if (fb < 1) fb = 1;
    if (fb > nframes) fb = nframes;
    if ((rc = ensure_buf(c, &c->bigtmp, &c->bigtmp_bytes, (size_t)(fb * nfft) * sizeof(float2)))) return rc;
    Timed t(c, "psd");
    for (long long f0 = 0; f0 < nframes; f0 += fb) {
      const long long nb = nframes - f0 < fb ? nframes - f0 : fb;
      vsig::BigIn in{(const float2*)x + f0 * hop * stride, 0, hop * stride, stride, nperseg, nullptr,
                     win, 0, 1.0f};
      HIPCHK(c, vsig::launch_bf_col(bp.N1, bp.N2, nb, in, (float2*)c->bigtmp, bp.tw1, bp.t2, bp.S,
                                    bp.hiA, c->stream));
      HIPCHK(c, vsig::launch_bf_row(2, bp.N1, bp.N2, nb, (float2*)c->bigtmp, nullptr, bp.tw2, scale,
                                    sxx + f0 * nfft, shift, c->stream));
    }
    return VSIG_OK;
  }
  const float2* tw;
  // pair kernel (>= 256 threads per frame): per-pass table; smaller plans: two-level table
  const bool pair = vsig::psd_plan_threads(nfft) >= 256;
  int rc = pair ? get_twiddles(c, nfft, &tw) : get_tw2(c, nfft, &tw);
  if (rc) return rc;
  Timed t(c, "psd");
  HIPCHK(c, vsig::launch_psd(nfft, (const float2*)x, stride, win, nperseg, hop, scale, sxx, nframes,
                             shift, tw, c->stream));
  return VSIG_OK;
}

int vsig_psd_c64(vsig_ctx* c, const void* x, int64_t n, const float* win, int32_t nperseg,
                 int64_t hop, int32_t nfft, float scale, int32_t shift, float* sxx,
                 int64_t nframes) {
  if (!c || !x || !win || !sxx) return fail(c, VSIG_E_INVALID, "null pointer");
  if (n < nperseg || nperseg < 1 || hop < 1) return fail(c, VSIG_E_INVALID, "bad sizes");
  const size_t bx = (size_t)n * 8, bw = (size_t)nperseg * 4, bo = (size_t)nframes * nfft * 4;
  int rc;
  if ((rc = ensure_stage(c, 0, bx)) || (rc = ensure_stage(c, 1, bw)) || (rc = ensure_stage(c, 2, bo)))
    return rc;
  HIPCHK(c, hipMemcpyAsync(c->stage[0], x, bx, hipMemcpyHostToDevice, c->stream));
  HIPCHK(c, hipMemcpyAsync(c->stage[1], win, bw, hipMemcpyHostToDevice, c->stream));
  rc = vsig_psd_c64_dev(c, c->stage[0], n, 1, (const float*)c->stage[1], nperseg, hop, nfft, scale,
                        shift, (float*)c->stage[2], nframes);
  if (rc) return rc;
  HIPCHK(c, hipMemcpyAsync(sxx, c->stage[2], bo, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return VSIG_OK;
}

// ---------------------------------------------------------------- FIR
int vsig_fir_create(vsig_ctx* c, const void* taps, int32_t ntaps, int32_t decim, vsig_fir** out) {
  if (!c || !taps || !out) return fail(c, VSIG_E_INVALID, "null pointer");
  *out = nullptr;
  if (ntaps < 1 || decim < 1) return fail(c, VSIG_E_INVALID, "ntaps and decim must be >= 1");
  if (ntaps > kFirPartTaps) {        // np.convolve has no length limit: parts
    auto* f = new vsig_fir{c, ntaps, decim, 0, 0, nullptr};
    for (int j = 0; j * kFirPartTaps < ntaps; ++j) {
      const int nt = ntaps - j * kFirPartTaps < kFirPartTaps ? ntaps - j * kFirPartTaps : kFirPartTaps;
      vsig_fir* p = nullptr;
      const int rc = vsig_fir_create(c, static_cast<const float2*>(taps) + (size_t)j * kFirPartTaps, nt, 1, &p);
      if (rc) { vsig_fir_free(f); return rc; }
      f->parts.push_back(p);
    }
    f->M = f->parts[0]->M;
    *out = f;
    return VSIG_OK;
  }
  const int M = os_size_fir(ntaps);
  if (!M) return fail(c, VSIG_E_UNSUPPORTED, "no block size for ntaps");
  long long hop = ((long long)M - (ntaps - 1)) / decim * decim;
  if (hop < 1) return fail(c, VSIG_E_UNSUPPORTED, "decim too large for the block size");
  // 1024-point pairs at hop 768 (ntaps 225..257): the second segment's first
  // quarter comes from the first one's registers (load_pair_x4), 14 loads per
  // pair instead of 16 for <= 4 % more segments (0.84 -> 0.80 ms at config 2,
  // profiles/r03_pl1_ab.txt)
  if (M == 1024 && decim == 1 && hop > 768 && hop < 800) hop = 768;
  float2* hd = nullptr;
  HIPCHK(c, hipMalloc(&hd, (size_t)ntaps * sizeof(float2)));
  hipError_t e = hipMemcpyAsync(hd, taps, (size_t)ntaps * sizeof(float2), hipMemcpyHostToDevice, c->stream);
  if (e != hipSuccess) { (void)hipFree(hd); return fail(c, VSIG_E_HIP, hipGetErrorString(e)); }
  float2* Hs = nullptr;
  int rc = make_spectrum(c, hd, ntaps, M, &Hs);
  float2* G = nullptr;
  if (!rc && M == 1024 && decim == 4) {
    hipError_t ge = hipMalloc(&G, 1024 * sizeof(float2));
    if (ge == hipSuccess) ge = vsig::launch_fir_poly_gtable(Hs, G, c->stream);
    if (ge != hipSuccess) rc = fail(c, VSIG_E_HIP, hipGetErrorString(ge));
  }
  (void)hipStreamSynchronize(c->stream);
  (void)hipFree(hd);
  if (rc) {
    (void)hipFree(Hs);
    (void)hipFree(G);
    return rc;
  }
  *out = new vsig_fir{c, ntaps, decim, M, hop, Hs, G};
  return VSIG_OK;
}

void vsig_fir_free(vsig_fir* f) {
  if (!f) return;
  (void)hipStreamSynchronize(f->ctx->stream);
  for (vsig_fir* p : f->parts) vsig_fir_free(p);
  (void)hipFree(f->z);
  (void)hipFree(f->Hs);
  (void)hipFree(f->G);
  delete f;
}

static int fir_exec(vsig_fir* f, const void* x, int64_t nhist, int64_t n, void* y, int64_t ny,
                    const vsig::MixArgs* mix) {
  if (!f) return VSIG_E_INVALID;
  vsig_ctx* c = f->ctx;
  if (!x || !y) return fail(c, VSIG_E_INVALID, "null pointer");
  if (n < 1 || nhist < 0) return fail(c, VSIG_E_INVALID, "need n >= 1 and nhist >= 0");
  if (ny != (n + f->decim - 1) / f->decim) return fail(c, VSIG_E_INVALID, "ny != ceil(n/decim)");
  const float2* tw;
  int rc;
  if (!f->parts.empty()) {
    if (mix) return fail(c, VSIG_E_UNSUPPORTED, "fused mixer needs ntaps <= 256 (mix first)");
    const long long nz = nhist + n;
    if ((rc = ensure_buf(c, reinterpret_cast<void**>(&f->z), &f->zbytes, (size_t)nz * sizeof(float2))))
      return rc;
    for (size_t j = 0; j < f->parts.size(); ++j) {
      if ((rc = fir_exec(f->parts[j], x, 0, nz, f->z, nz, nullptr))) return rc;
      Timed t(c, "fir");
      HIPCHK(c, vsig::launch_fir_part_accum(f->z, nz, nhist - (long long)j * kFirPartTaps, f->decim, ny,
                                            j == 0, (float2*)y, c->stream));
    }
    return VSIG_OK;
  }
  if (f->M == 1024 && (f->decim == 2 || f->decim == 4)) {
    // decimation in the frequency domain: M/D-point inverse transforms
    const float2* twd;
    const int D = f->decim;
    int lo2 = (f->ntaps - 1 + D - 1) / D * D;
    // a multiple of 16 when the block allows (as fir_os_kernel's lo): the
    // decimated output runs (64 per store instruction) then start on 128-byte
    // lines, and so do the segments of a 16-multiple history (the chain's)
    if (((lo2 + 15) & ~15) + 768 <= f->M) lo2 = (lo2 + 15) & ~15;
    const long long hop = (long long)(f->M - lo2) / D * D;
    if (hop < D) return fail(c, VSIG_E_UNSUPPORTED, "decim too large for the block size");
    if (f->G) {      // D = 4: polyphase form (fir_poly_kernel)
      if ((rc = get_twiddles(c, 256, &tw)) || (rc = get_twiddles(c, -256, &twd))) return rc;
      Timed t(c, "fir");
      HIPCHK(c, vsig::launch_fir_poly((const float2*)x, nhist + n, nhist, f->G, lo2, hop, (float2*)y, tw,
                                      twd, c->stream, mix));
      return VSIG_OK;
    }
    if ((rc = get_twiddles(c, -1024, &tw)) || (rc = get_twiddles(c, -1024 / f->decim, &twd))) return rc;
    Timed t(c, "fir");
    HIPCHK(c, vsig::launch_fir_dec(D, (const float2*)x, nhist + n, nhist, f->Hs, lo2, hop, (float2*)y,
                                   tw, twd, c->stream, mix));
    return VSIG_OK;
  }
  if (mix && f->M != 1024)
    return fail(c, VSIG_E_UNSUPPORTED, "fused mixer needs the 1024-point block (ntaps <= 256)");
  rc = get_twiddles(c, f->M == 1024 ? -1024 : f->M, &tw);
  if (rc) return rc;
  Timed t(c, "fir");
  HIPCHK(c, vsig::launch_fir_os(f->M, (const float2*)x, nhist + n, nhist, f->Hs, f->ntaps, f->hop,
                                f->decim, (float2*)y, tw, c->stream, mix));
  return VSIG_OK;
}

int vsig_fir_block(const vsig_fir* f) { return f ? f->M : 0; }

int vsig_fir_exec_hist_dev(vsig_fir* f, const void* x, int64_t nhist, int64_t n, void* y,
                           int64_t ny) {
  return fir_exec(f, x, nhist, n, y, ny, nullptr);
}

int vsig_fir_exec_mix_dev(vsig_fir* f, const void* x, int64_t nhist, int64_t n, void* y, int64_t ny,
                          double freq_shift, double sample_rate, int64_t i0) {
  if (!f) return VSIG_E_INVALID;
  if (freq_shift == 0.0) return fir_exec(f, x, nhist, n, y, ny, nullptr);   // utils.py:122-123
  if (!(sample_rate != 0.0)) return fail(f->ctx, VSIG_E_INVALID, "sample_rate must be non-zero");
  const double w = (2.0 * M_PI) * freq_shift;
  vsig::MixArgs m{};
  m.w = w;
  m.sr = sample_rate;
  m.i0 = (long long)i0;
  m.wsr = w / sample_rate;
  for (int e = 0; e < 16; ++e) {       // exp(j wsr 64 e), reduced mod 2 pi in double
    const double a = std::remainder(m.wsr * 64.0 * e, 2.0 * M_PI);
    m.rot[2 * e] = (float)std::cos(a);
    m.rot[2 * e + 1] = (float)std::sin(a);
  }
  return fir_exec(f, x, nhist, n, y, ny, &m);
}

int vsig_fir_exec_dev(vsig_fir* f, const void* x, int64_t n, void* y, int64_t ny) {
  return vsig_fir_exec_hist_dev(f, x, 0, n, y, ny);
}

int vsig_fir_c64(vsig_ctx* c, const void* x, int64_t n, const float* taps, int32_t ntaps,
                 int32_t decim, void* y, int64_t ny) {
  if (!c || !x || !taps || !y) return fail(c, VSIG_E_INVALID, "null pointer");
  if (ntaps < 1) return fail(c, VSIG_E_INVALID, "ntaps must be >= 1");
  std::vector<float2> tc(ntaps);
  for (int i = 0; i < ntaps; ++i) tc[i] = make_float2(taps[i], 0.f);
  vsig_fir* f = nullptr;
  int rc = vsig_fir_create(c, tc.data(), ntaps, decim, &f);
  if (rc) return rc;
  const size_t bx = (size_t)n * 8, by = (size_t)ny * 8;
  if ((rc = ensure_stage(c, 0, bx)) || (rc = ensure_stage(c, 1, by))) { vsig_fir_free(f); return rc; }
  hipError_t e = hipMemcpyAsync(c->stage[0], x, bx, hipMemcpyHostToDevice, c->stream);
  if (e == hipSuccess) {
    rc = vsig_fir_exec_dev(f, c->stage[0], n, c->stage[1], ny);
    if (!rc) e = hipMemcpyAsync(y, c->stage[1], by, hipMemcpyDeviceToHost, c->stream);
  }
  if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
  vsig_fir_free(f);
  if (rc) return rc;
  if (e != hipSuccess) return fail(c, VSIG_E_HIP, hipGetErrorString(e));
  return VSIG_OK;
}

// ---------------------------------------------------------------- correlation
// Template spectra from a device c64 template of L samples: L <= 8192 one
// M-point spectrum; longer templates one M = 16384 spectrum per 8192-sample
// chunk (sum of passes, see xcorr_run).
static int xcorr_build(vsig_ctx* c, const float2* td, long long L, vsig_xcorr* x) {
  constexpr long long B = 8192;
  x->ctx = c;
  x->L = L;
  x->M = os_size_xcorr(L) ? os_size_xcorr(L) : 16384;
  const long long Bc = x->M == 32768 ? 16384 : B;    // one pass up to 16384 at M = 32768
  for (long long p = 0; p * Bc < L || p == 0; ++p) {
    const long long Lp = L <= Bc ? L : ((L - p * Bc) < B ? (L - p * Bc) : B);
    float2* P = nullptr;
    const int rc = make_spectrum(c, td + p * B, (int)Lp, x->M, &P);
    if (rc) return rc;
    x->Ps.push_back(P);
    if (L <= Bc) break;
  }
  return VSIG_OK;
}

static void xcorr_release(vsig_xcorr* x) {
  (void)hipStreamSynchronize(x->ctx->stream);
  for (float2* P : x->Ps) (void)hipFree(P);
  x->Ps.clear();
  if (x->tmpl) (void)hipFree(x->tmpl);
  if (x->cbuf) (void)hipFree(x->cbuf);
  x->tmpl = nullptr;
  x->cbuf = nullptr;
}

// The correlation c[o] = sum_k s[o - off + k] conj(p[k]) of the handle's
// template over the c64 stream s, o < nout, stored per store_mode bits 0-2
// into cout (c64, may be null), the peak record into rec, then refined with
// op (see run_refine; out128: complex128 c to patch).  Templates longer than
// 8192: the chunks' passes accumulate in c (store bit 8; a scratch kept with
// the handle when cout is null), then one fp64 peak reduction over c and the
// refine from the stored array.
static int xcorr_run(vsig_xcorr* x, const float2* s, long long n, long long off, long long nout,
                     int store_mode, float2* cout, vsig_peak_t* peak_dev,
                     const RefineOperands* op, void* out128, bool async = false) {
  vsig_ctx* c = x->ctx;
  PeakPartial* rec = peak_dev ? reinterpret_cast<PeakPartial*>(peak_dev) : c->result;
  if (x->Ps.size() == 1 && x->L <= (x->M == 32768 ? 16384 : 8192)) {
    // outputs per block: M - L + 1, rounded down to even at M = 16384 (every
    // segment start then has one parity: the correlator's 16-byte loads)
    long long hop = (long long)x->M - x->L + 1;
    if (x->M == 16384 && hop > 1) hop &= ~1LL;
    const long long nblocks = (nout + hop - 1) / hop;
    int waves, Q, stride, plan, wstep, rsub;
    if (vsig::xcorr_geom(x->M, &waves, &Q, &stride, &plan, &wstep, &rsub) != hipSuccess)
      return fail(c, VSIG_E_UNSUPPORTED, "correlator block size");
    const long long nparts = nblocks * waves;   // one partial per wave
    int rc = ensure_partials(c, nparts);
    if (rc) return rc;
    // with the refine on, the partials' finalize and the candidate select run
    // as the refine's first launch, on thread columns where the kernel writes
    // lane keys (64x fewer outputs re-ranked than whole waves)
    const bool fused = op && c->refine && !(store_mode & 8);
    unsigned* lk = nullptr;
    if (fused && Q <= 64 && vsig::xcorr_lane_keys(x->M) == Q) {
      if ((rc = ensure_buf(c, &c->lkeys, &c->lkeys_bytes, (size_t)nparts * 64 * sizeof(unsigned))))
        return rc;
      lk = static_cast<unsigned*>(c->lkeys);
    }
    const float2* tw;
    const float2* wt = nullptr;
    if ((rc = get_twiddles(c, plan, &tw))) return rc;
    if (x->M >= 16384 && (rc = get_half_tw(c, x->M, x->M == 16384 ? 512 : 1024, &wt))) return rc;
    {
      Timed t(c, "xcorr");
      HIPCHK(c, vsig::launch_xcorr_os(x->M, s, n, x->Ps[0], off, nout, hop, cout, store_mode,
                                      c->partials, tw, wt, c->stream, lk));
    }
    if (!fused) {
      if ((rc = finalize_peak(c, nparts, 1, peak_dev))) return rc;
      if (!op) return VSIG_OK;
    }
    if (out128 && cout) HIPCHK(c, vsig::launch_convert_c(1, cout, nout, out128, c->stream));
    return run_refine(c, *op, nout, x->M, hop, nparts, (store_mode & 4) ? 1 : 0, nullptr, rec, out128,
                      fused, lk, async && peak_dev != nullptr);
  }
  constexpr long long B = 8192;
  constexpr int M = 16384;
  float2* cbuf = cout;
  int rc;
  if (!cbuf) {
    if ((rc = ensure_buf(c, &x->cbuf, &x->cbuf_bytes, (size_t)nout * sizeof(float2)))) return rc;
    cbuf = static_cast<float2*>(x->cbuf);
  }
  const float2 *tw, *wt;
  int waves, Q, stride, plan, wstep, rsub;
  if (vsig::xcorr_geom(M, &waves, &Q, &stride, &plan, &wstep, &rsub) != hipSuccess)
    return fail(c, VSIG_E_UNSUPPORTED, "correlator block size");
  if ((rc = get_twiddles(c, plan, &tw)) || (rc = get_half_tw(c, M, 512, &wt))) return rc;
  {
    Timed t(c, "xcorr");            // the whole chunked correlation + its peak pass
    for (size_t p = 0; p < x->Ps.size(); ++p) {
      const long long Lp = (x->L - (long long)p * B) < B ? (x->L - (long long)p * B) : B;
      const int mode = (store_mode & 4 ? 2 | 4 : 1) | (p ? 8 : 0);
      HIPCHK(c, vsig::launch_xcorr_os(M, s, n, x->Ps[p], off - (long long)p * B, nout,
                                      (long long)M - Lp + 1, cbuf, mode, nullptr, tw, wt,
                                      c->stream));
    }
    if ((rc = vsig_peak_dev(c, VSIG_DTYPE_C64, cbuf, nout, peak_dev))) return rc;
  }
  if (!op) return VSIG_OK;
  if (out128 && cout) HIPCHK(c, vsig::launch_convert_c(1, cout, nout, out128, c->stream));
  return run_refine(c, *op, nout, M, 0, 0, 0, cbuf, rec, out128);
}

int vsig_xcorr_create(vsig_ctx* c, const void* tmpl, int64_t L, vsig_xcorr** out) {
  if (!c || !tmpl || !out) return fail(c, VSIG_E_INVALID, "null pointer");
  *out = nullptr;
  if (L < 1) return fail(c, VSIG_E_INVALID, "template length must be >= 1");
  vsig_xcorr* x = new vsig_xcorr();
  x->ctx = c;
  hipError_t e = hipMalloc(&x->tmpl, (size_t)L * sizeof(float2));
  if (e == hipSuccess)
    e = hipMemcpyAsync(x->tmpl, tmpl, (size_t)L * sizeof(float2), hipMemcpyHostToDevice, c->stream);
  if (e != hipSuccess) {
    xcorr_release(x);
    delete x;
    return fail(c, e == hipErrorOutOfMemory ? VSIG_E_NOMEM : VSIG_E_HIP, hipGetErrorString(e));
  }
  const int rc = xcorr_build(c, x->tmpl, L, x);
  (void)hipStreamSynchronize(c->stream);
  if (rc) {
    xcorr_release(x);
    delete x;
    return rc;
  }
  *out = x;
  return VSIG_OK;
}

void vsig_xcorr_free(vsig_xcorr* x) {
  if (!x) return;
  xcorr_release(x);
  delete x;
}

int vsig_xcorr_exec_dev(vsig_xcorr* x, const void* s, int64_t n, int32_t mode, void* cout,
                        vsig_peak_t* peak_dev) {
  if (!x) return VSIG_E_INVALID;
  vsig_ctx* c = x->ctx;
  if (!s) return fail(c, VSIG_E_INVALID, "null pointer");
  long long off, nout;
  if (mode == VSIG_MODE_VALID) { off = 0; nout = n - x->L + 1; }
  else if (mode == VSIG_MODE_FULL) { off = x->L - 1; nout = n + x->L - 1; }
  else return fail(c, VSIG_E_INVALID, "streaming correlation supports VALID and FULL");
  if (nout < 1) return fail(c, VSIG_E_INVALID, "stream shorter than the template");
  // np.correlate(s, p): output o is full index (L - 1 - off) + o
  const RefineOperands op{s, n, x->tmpl, x->L, 0, (x->L - 1) - off};
  return xcorr_run(x, (const float2*)s, n, off, nout, cout ? 1 : 0, (float2*)cout, peak_dev, &op,
                   nullptr, true);
}

// np.correlate(a, v, mode): the shorter operand is the template; with
// nv > na the correlation of v by a is computed and stored conj() reversed.
static int correlate_impl(vsig_ctx* c, int in128, const void* a, long long na, const void* v,
                          long long nv, int32_t mode, int out128, void* cout,
                          vsig_peak_t* peak_dev) {
  if (!c || !a || !v) return fail(c, VSIG_E_INVALID, "null pointer");
  if (na < 1 || nv < 1) return fail(c, VSIG_E_INVALID, "empty input");  // numeric.py:865-868
  const long long nmin = na < nv ? na : nv, nmax = na < nv ? nv : na;
  long long F, nout;  // start index into the 'full' correlation, output length
  if (mode == VSIG_MODE_FULL) { F = 0; nout = na + nv - 1; }
  else if (mode == VSIG_MODE_VALID) { F = nmin - 1; nout = nmax - nmin + 1; }
  else if (mode == VSIG_MODE_SAME) { F = na >= nv ? nmin - 1 - nmin / 2 : nmin / 2; nout = nmax; }
  else return fail(c, VSIG_E_INVALID, "mode must be VALID, FULL or SAME");
  int rc;
  // complex64 operands of the FFT pass (complex128 callers: converted copies)
  const float2 *a64 = (const float2*)a, *v64 = (const float2*)v;
  if (in128) {
    if ((rc = ensure_buf(c, &c->conv[0], &c->conv_bytes[0], (size_t)na * 8)) ||
        (rc = ensure_buf(c, &c->conv[1], &c->conv_bytes[1], (size_t)nv * 8)))
      return rc;
    HIPCHK(c, vsig::launch_convert_c(0, a, na, c->conv[0], c->stream));
    HIPCHK(c, vsig::launch_convert_c(0, v, nv, c->conv[1], c->stream));
    a64 = (const float2*)c->conv[0];
    v64 = (const float2*)c->conv[1];
  }
  float2* c64 = (float2*)cout;
  if (out128 && cout) {
    if ((rc = ensure_buf(c, &c->conv[2], &c->conv_bytes[2], (size_t)nout * 8))) return rc;
    c64 = (float2*)c->conv[2];
  }
  const bool swap = nv > na;  // template must be the shorter operand
  const float2* tmpl = swap ? a64 : v64;
  const float2* strm = swap ? v64 : a64;
  // c[o] = full[F + o]; full[i] = sum_k a[i-(nv-1)+k] conj(v[k]).
  // Not swapped: kernel offset off = (L-1) - F.  Swapped: compute the
  // correlation of v by a and store conj() reversed, off' = F + nout - nv.
  const long long off = swap ? F + nout - nv : (nmin - 1) - F;
  vsig_xcorr x;
  x.ctx = c;
  rc = xcorr_build(c, tmpl, nmin, &x);
  if (!rc) {
    const RefineOperands op{a, na, v, nv, in128, F};
    const int store = (cout ? (swap ? 2 : 1) : 0) | (swap ? 4 : 0);
    rc = xcorr_run(&x, strm, nmax, off, nout, store, c64, peak_dev, &op, out128 ? cout : nullptr);
  }
  xcorr_release(&x);     // synchronises before freeing the template spectra
  return rc;
}

int vsig_correlate_dev(vsig_ctx* c, int32_t dtype, const void* a, int64_t na, const void* v,
                       int64_t nv, int32_t mode, int32_t out_dtype, void* cout,
                       vsig_peak_t* peak_dev) {
  if ((dtype != VSIG_DTYPE_C64 && dtype != VSIG_DTYPE_C128) ||
      (out_dtype != VSIG_DTYPE_C64 && out_dtype != VSIG_DTYPE_C128))
    return fail(c, VSIG_E_INVALID, "dtype must be VSIG_DTYPE_C64 or VSIG_DTYPE_C128");
  return correlate_impl(c, dtype == VSIG_DTYPE_C128, a, na, v, nv, mode,
                        out_dtype == VSIG_DTYPE_C128, cout, peak_dev);
}

int vsig_correlate_c64_dev(vsig_ctx* c, const void* a, int64_t na, const void* v, int64_t nv,
                           int32_t mode, void* cout, vsig_peak_t* peak_dev) {
  return correlate_impl(c, 0, a, na, v, nv, mode, 0, cout, peak_dev);
}

int vsig_correlate(vsig_ctx* c, int32_t dtype, const void* a, int64_t na, const void* v,
                   int64_t nv, int32_t mode, int32_t out_dtype, void* cout, vsig_peak_t* peak) {
  if (!c || !a || !v) return fail(c, VSIG_E_INVALID, "null pointer");
  if (na < 1 || nv < 1) return fail(c, VSIG_E_INVALID, "empty input");
  if ((dtype != VSIG_DTYPE_C64 && dtype != VSIG_DTYPE_C128) ||
      (out_dtype != VSIG_DTYPE_C64 && out_dtype != VSIG_DTYPE_C128))
    return fail(c, VSIG_E_INVALID, "dtype must be VSIG_DTYPE_C64 or VSIG_DTYPE_C128");
  const size_t es = dtype == VSIG_DTYPE_C128 ? 16 : 8, eo = out_dtype == VSIG_DTYPE_C128 ? 16 : 8;
  const long long nmin = na < nv ? na : nv, nmax = na < nv ? nv : na;
  const long long nout = mode == VSIG_MODE_FULL ? na + nv - 1
                       : mode == VSIG_MODE_VALID ? nmax - nmin + 1 : nmax;
  int rc;
  if ((rc = ensure_stage(c, 0, (size_t)na * es)) || (rc = ensure_stage(c, 1, (size_t)nv * es)) ||
      (cout && (rc = ensure_stage(c, 2, (size_t)nout * eo))))
    return rc;
  HIPCHK(c, hipMemcpyAsync(c->stage[0], a, (size_t)na * es, hipMemcpyHostToDevice, c->stream));
  HIPCHK(c, hipMemcpyAsync(c->stage[1], v, (size_t)nv * es, hipMemcpyHostToDevice, c->stream));
  rc = vsig_correlate_dev(c, dtype, c->stage[0], na, c->stage[1], nv, mode, out_dtype,
                          cout ? c->stage[2] : nullptr, nullptr);
  if (rc) return rc;
  if (cout) HIPCHK(c, hipMemcpyAsync(cout, c->stage[2], (size_t)nout * eo, hipMemcpyDeviceToHost, c->stream));
  if (peak) HIPCHK(c, hipMemcpyAsync(peak, c->result, sizeof(vsig_peak_t), hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return VSIG_OK;
}

int vsig_correlate_c64(vsig_ctx* c, const void* a, int64_t na, const void* v, int64_t nv,
                       int32_t mode, void* cout, vsig_peak_t* peak) {
  return vsig_correlate(c, VSIG_DTYPE_C64, a, na, v, nv, mode, VSIG_DTYPE_C64, cout, peak);
}

// ---------------------------------------------------------------- any-length transforms
int vsig_dft_dev(vsig_ctx* c, int32_t dtype, const void* x, int64_t n, int64_t batch, int32_t inverse,
                 int32_t out_dtype, void* y) {
  if (!c || !x || !y) return fail(c, VSIG_E_INVALID, "null pointer");
  if (n < 1 || batch < 1) return fail(c, VSIG_E_INVALID, "need n >= 1 and batch >= 1");
  if ((dtype != VSIG_DTYPE_C64 && dtype != VSIG_DTYPE_C128) ||
      (out_dtype != VSIG_DTYPE_C64 && out_dtype != VSIG_DTYPE_C128))
    return fail(c, VSIG_E_INVALID, "dtype must be VSIG_DTYPE_C64 or VSIG_DTYPE_C128");
  vsig::BigIn in{x, dtype == VSIG_DTYPE_C128 ? 1 : 0, n, 1, n, nullptr, nullptr, 0, 1.0f};
  vsig::BigOut out{y, out_dtype == VSIG_DTYPE_C128 ? 1 : 0, n, n, nullptr, 0,
                   inverse ? (float)(1.0 / (double)n) : 1.0f};
  Timed t(c, "dft");
  return dft_any(c, n, batch, in, out, inverse != 0);
}

int vsig_resample_dev(vsig_ctx* c, int32_t dtype, const void* x, int64_t n, int64_t num,
                      int32_t real_input, void* y) {
  if (!c || !x || !y) return fail(c, VSIG_E_INVALID, "null pointer");
  if (n < 1 || num < 1) return fail(c, VSIG_E_INVALID, "need n >= 1 and num >= 1");
  if (dtype != VSIG_DTYPE_C64 && dtype != VSIG_DTYPE_C128)
    return fail(c, VSIG_E_INVALID, "dtype must be VSIG_DTYPE_C64 or VSIG_DTYPE_C128");
  int rc;
  if ((rc = ensure_buf(c, &c->spec[0], &c->spec_bytes[0], (size_t)n * 8)) ||
      (rc = ensure_buf(c, &c->spec[1], &c->spec_bytes[1], (size_t)num * 8)))
    return rc;
  float2* X = (float2*)c->spec[0];
  float2* Y = (float2*)c->spec[1];
  Timed t(c, "resample");
  vsig::BigIn in{x, dtype == VSIG_DTYPE_C128 ? 1 : 0, n, 1, n, nullptr, nullptr, 0, 1.0f};
  vsig::BigOut ox{X, 0, n, n, nullptr, 0, 1.0f};
  if ((rc = dft_any(c, n, 1, in, ox, false))) return rc;
  HIPCHK(c, vsig::launch_resample_spectrum(X, n, num, Y, c->stream));
  // y = ifft(Y) * num / n  ->  the inverse DFT's 1/num and num/n leave 1/n
  vsig::BigIn iy{Y, 0, num, 1, num, nullptr, nullptr, 0, 1.0f};
  vsig::BigOut oy{y, real_input ? 3 : 0, num, num, nullptr, 0, (float)(1.0 / (double)n)};
  return dft_any(c, num, 1, iy, oy, true);
}

int vsig_filter_channel_dev(vsig_ctx* c, int32_t dtype, const void* x, int64_t n,
                            double center_freq, double sample_rate, double bandwidth,
                            double* y) {
  if (!c || !x || !y) return fail(c, VSIG_E_INVALID, "null pointer");
  if (n < 1) return fail(c, VSIG_E_INVALID, "empty input");
  if (n > 1 && (n & 1))
    return fail(c, VSIG_E_INVALID, "odd length: the conjugate mirror's halves differ (numpy "
                                   "raises on the shape mismatch)");
  if (dtype != VSIG_DTYPE_C64 && dtype != VSIG_DTYPE_C128)
    return fail(c, VSIG_E_INVALID, "dtype must be VSIG_DTYPE_C64 or VSIG_DTYPE_C128");
  const double center = 5230e6;                  // split_channels.py:7 CENTER_FREQ
  const double lo = center_freq - bandwidth / 2, hi = center_freq + bandwidth / 2;
  if (n > 1) {   // the mirror's halves are the natural ones unless f(-1) rounds onto CENTER
    if (!(channel_freq(-1, n, sample_rate, center) < center))
      return fail(c, VSIG_E_UNSUPPORTED, "frequency spacing below the rounding of CENTER_FREQ");
  }
  // kept non-negative bins: f(k) rises with k, so the mask is one range [ka, kb]
  const long long h = n == 1 ? 1 : n / 2;
  auto keep = [&](long long k) { const double f = channel_freq(k, n, sample_rate, center); return f >= lo && f <= hi; };
  auto first_at_least = [&](double bound) {      // smallest k in [0, h] with f(k) >= bound
    long long a = 0, b = h;
    while (a < b) { const long long m = (a + b) / 2; if (channel_freq(m, n, sample_rate, center) >= bound) b = m; else a = m + 1; }
    return a;
  };
  long long ka = first_at_least(lo), kb = ka - 1;
  if (ka < h && keep(ka)) {
    long long a = ka, b = h - 1;                 // largest kept k
    while (a < b) { const long long m = (a + b + 1) / 2; if (keep(m)) a = m; else b = m - 1; }
    kb = a;
  }
  const long long nk = kb >= ka ? kb - ka + 1 : 0;
  int rc;
  if (nk * n <= (1LL << 32)) {                   // direct double-precision path
    if ((rc = ensure_buf(c, &c->spec[0], &c->spec_bytes[0], (size_t)(nk > 0 ? nk : 1) * 256 * 16)) ||
        (rc = ensure_buf(c, &c->spec[1], &c->spec_bytes[1], (size_t)(nk > 0 ? nk : 1) * 16)))
      return rc;
    Timed t(c, "channel");
    HIPCHK(c, vsig::launch_channel_direct(dtype == VSIG_DTYPE_C128, x, n, ka, kb, (double2*)c->spec[0],
                                          (double2*)c->spec[1], y, c->stream));
    return VSIG_OK;
  }
  if ((rc = ensure_buf(c, &c->spec[0], &c->spec_bytes[0], (size_t)n * 8)) ||
      (rc = ensure_buf(c, &c->spec[1], &c->spec_bytes[1], (size_t)n * 8)))
    return rc;
  float2* X = (float2*)c->spec[0];
  float2* F = (float2*)c->spec[1];
  Timed t(c, "channel");
  vsig::BigIn in{x, dtype == VSIG_DTYPE_C128 ? 1 : 0, n, 1, n, nullptr, nullptr, 0, 1.0f};
  vsig::BigOut ox{X, 0, n, n, nullptr, 0, 1.0f};
  if ((rc = dft_any(c, n, 1, in, ox, false))) return rc;
  HIPCHK(c, vsig::launch_channel_mask(X, n, sample_rate, center, center_freq - bandwidth / 2,
                                      center_freq + bandwidth / 2, F, c->stream));
  vsig::BigIn iF{F, 0, n, 1, n, nullptr, nullptr, 0, 1.0f};
  vsig::BigOut oy{y, 2, n, n, nullptr, 0, (float)(1.0 / (double)n)};
  return dft_any(c, n, 1, iF, oy, true);
}

// ---------------------------------------------------------------- peak
int vsig_peak_dev(vsig_ctx* c, int32_t dtype, const void* a, int64_t n, vsig_peak_t* peak_dev) {
  if (!c || !a) return fail(c, VSIG_E_INVALID, "null pointer");
  if (n < 1) return fail(c, VSIG_E_INVALID, "empty input");  // np.argmax of empty raises
  if (dtype < VSIG_DTYPE_C128 || dtype > VSIG_DTYPE_F32) return fail(c, VSIG_E_INVALID, "dtype");
  long long nparts = (n + 255) / 256;
  if (nparts > 2048) nparts = 2048;
  int rc = ensure_partials(c, nparts);
  if (rc) return rc;
  {
    Timed t(c, "peak");
    HIPCHK(c, vsig::launch_peak_reduce(dtype, a, n, c->partials, (int)nparts, c->stream));
  }
  return finalize_peak(c, nparts, 0, peak_dev);
}

int vsig_peak(vsig_ctx* c, int32_t dtype, const void* a, int64_t n, vsig_peak_t* peak) {
  if (!c || !a || !peak) return fail(c, VSIG_E_INVALID, "null pointer");
  if (n < 1) return fail(c, VSIG_E_INVALID, "empty input");
  const size_t es = dtype == VSIG_DTYPE_C128 ? 16 : (dtype == VSIG_DTYPE_F32 ? 4 : 8);
  int rc = ensure_stage(c, 0, (size_t)n * es);
  if (rc) return rc;
  HIPCHK(c, hipMemcpyAsync(c->stage[0], a, (size_t)n * es, hipMemcpyHostToDevice, c->stream));
  rc = vsig_peak_dev(c, dtype, c->stage[0], n, nullptr);
  if (rc) return rc;
  HIPCHK(c, hipMemcpyAsync(peak, c->result, sizeof(vsig_peak_t), hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return VSIG_OK;
}

// numpy's np.mean / np.std of |a| (find_correlation_peak's mean_corr /
// std_corr, utils.py:1329-1330) in numpy's own summation order.
int vsig_abs_stats_dev(vsig_ctx* c, int32_t dtype, const void* a, int64_t n, double* stats_dev) {
  if (!c || !a || !stats_dev) return fail(c, VSIG_E_INVALID, "null pointer");
  if (n < 1) return fail(c, VSIG_E_INVALID, "empty input");
  if (dtype != VSIG_DTYPE_C128 && dtype != VSIG_DTYPE_F64)
    return fail(c, VSIG_E_UNSUPPORTED, "abs stats: dtype must be VSIG_DTYPE_C128 or VSIG_DTYPE_F64");
  int rc = ensure_buf(c, &c->sscratch, &c->sscratch_bytes, vsig::np_stats_scratch_bytes(n));
  if (rc) return rc;
  Timed t(c, "stats");
  HIPCHK(c, vsig::launch_np_stats(dtype, a, n, stats_dev, c->sscratch, c->stream));
  return VSIG_OK;
}

// np.correlate(a, v, mode)'s |c| for every output in numpy's operation order
// (refine.hip, values mode), then its mean / std as above.
int vsig_correlate_stats_dev(vsig_ctx* c, int32_t dtype, const void* a, int64_t na, const void* v,
                             int64_t nv, int32_t mode, double* stats_dev) {
  if (!c || !a || !v || !stats_dev) return fail(c, VSIG_E_INVALID, "null pointer");
  if (na < 1 || nv < 1) return fail(c, VSIG_E_INVALID, "empty input");
  if (dtype != VSIG_DTYPE_C64 && dtype != VSIG_DTYPE_C128)
    return fail(c, VSIG_E_INVALID, "dtype must be VSIG_DTYPE_C64 or VSIG_DTYPE_C128");
  const long long nmin = na < nv ? na : nv, nmax = na < nv ? nv : na;
  long long F, nout;
  if (mode == VSIG_MODE_FULL) { F = 0; nout = na + nv - 1; }
  else if (mode == VSIG_MODE_VALID) { F = nmin - 1; nout = nmax - nmin + 1; }
  else if (mode == VSIG_MODE_SAME) { F = na >= nv ? nmin - 1 - nmin / 2 : nmin / 2; nout = nmax; }
  else return fail(c, VSIG_E_INVALID, "mode must be VALID, FULL or SAME");
  const size_t vb = ((size_t)nout * 8 + 255) & ~(size_t)255;
  const size_t kb = (vsig::refine_values_scratch_bytes() + 255) & ~(size_t)255;
  int rc = ensure_buf(c, &c->vscratch, &c->vscratch_bytes, vb + kb);
  if (rc) return rc;
  if ((rc = ensure_buf(c, &c->sscratch, &c->sscratch_bytes, vsig::np_stats_scratch_bytes(nout))))
    return rc;
  double* vals = static_cast<double*>(c->vscratch);
  vsig::RefineArgs r{};
  r.a = a; r.na = na; r.v = v; r.nv = nv; r.c128 = dtype == VSIG_DTYPE_C128;
  r.nout = nout; r.F = F; r.waves = 1; r.Q = 1; r.rsub = 1;
  r.blas_threads = c->blas_threads;
  r.scratch = static_cast<char*>(c->vscratch) + vb;
  Timed t(c, "stats");
  HIPCHK(c, vsig::launch_refine_values(r, 0, nout - 1, vals, c->stream));
  HIPCHK(c, vsig::launch_np_stats(VSIG_DTYPE_F64, vals, nout, stats_dev, c->sscratch, c->stream));
  return VSIG_OK;
}

// ---------------------------------------------------------------- stream ops
int vsig_mix_c64_dev(vsig_ctx* c, const void* x, int64_t n, double w, double sr, int64_t i0,
                     void* y) {
  if (!c || !x || !y) return fail(c, VSIG_E_INVALID, "null pointer");
  if (n < 0 || !(sr != 0.0)) return fail(c, VSIG_E_INVALID, "need n >= 0 and sample_rate != 0");
  if (n == 0) return VSIG_OK;
  HIPCHK(c, vsig::launch_mix_c64((const float2*)x, n, w, sr, i0, (float2*)y, c->stream));
  return VSIG_OK;
}

int vsig_scale_c64_dev(vsig_ctx* c, const void* x, int64_t n, float s, void* y) {
  if (!c || !x || !y) return fail(c, VSIG_E_INVALID, "null pointer");
  if (n < 0) return fail(c, VSIG_E_INVALID, "n < 0");
  if (n == 0) return VSIG_OK;
  HIPCHK(c, vsig::launch_scale_c64((const float2*)x, n, s, (float2*)y, c->stream));
  return VSIG_OK;
}

int vsig_wv_quantize_dev(vsig_ctx* c, const void* x, int64_t n, float norm, int16_t* out) {
  if (!c || !x || !out) return fail(c, VSIG_E_INVALID, "null pointer");
  if (n < 0) return fail(c, VSIG_E_INVALID, "n < 0");
  if (n == 0) return VSIG_OK;
  HIPCHK(c, vsig::launch_wv_quantize((const float2*)x, n, norm, (short*)out, c->stream));
  return VSIG_OK;
}

int vsig_planar_to_c64_dev(vsig_ctx* c, int32_t mi_type, const void* re, const void* im, int64_t n,
                           void* y) {
  if (!c || !re || !y) return fail(c, VSIG_E_INVALID, "null pointer");
  if (n < 0) return fail(c, VSIG_E_INVALID, "n < 0");
  if (n == 0) return VSIG_OK;
  const hipError_t e = vsig::launch_planar_to_c64(mi_type, re, im, n, (float2*)y, c->stream);
  if (e == hipErrorInvalidValue) return fail(c, VSIG_E_UNSUPPORTED, "MAT storage type");
  HIPCHK(c, e);
  return VSIG_OK;
}

int vsig_c64_to_planar_dev(vsig_ctx* c, const void* x, int64_t n, float* re, float* im) {
  if (!c || !x || !re || !im) return fail(c, VSIG_E_INVALID, "null pointer");
  if (n < 0) return fail(c, VSIG_E_INVALID, "n < 0");
  if (n == 0) return VSIG_OK;
  HIPCHK(c, vsig::launch_c64_to_planar((const float2*)x, n, re, im, c->stream));
  return VSIG_OK;
}

// ---------------------------------------------------------------- PFB
int vsig_pfb_c64_dev(vsig_ctx* c, const void* x, int64_t n, const float* h, int32_t ntaps,
                     int32_t nchan, void* y, int64_t nframes) {
  if (!c || !x || !h || !y) return fail(c, VSIG_E_INVALID, "null pointer");
  if (nchan != 64 && nchan != 128 && nchan != 256)
    return fail(c, VSIG_E_UNSUPPORTED, "nchan must be 64, 128 or 256");
  const int pt = ntaps / nchan;
  if (ntaps % nchan || (pt != 4 && pt != 8 && pt != 16))
    return fail(c, VSIG_E_UNSUPPORTED, "ntaps must be 4, 8 or 16 times nchan");
  if (n < ntaps) return fail(c, VSIG_E_INVALID, "signal shorter than the prototype filter");
  if (nframes != (n - ntaps) / nchan + 1) return fail(c, VSIG_E_INVALID, "nframes mismatch");
  const float2* tw;
  int rc = get_twiddles(c, nchan, &tw);
  if (rc) return rc;
  Timed t(c, "pfb");
  HIPCHK(c, vsig::launch_pfb(nchan, pt, (const float2*)x, n, h, nframes, (float2*)y, tw, c->stream));
  return VSIG_OK;
}

// ---------------------------------------------------------------- analysis
// k-th smallest of |a| (0-based ranks) by MSB-first 8-bit radix select:
// ceil(bits/8) histogram passes over the data, all ranks at once.
int vsig_select_dev(vsig_ctx* c, int32_t dtype, const void* a, int64_t n, const int64_t* ranks,
                    int32_t nranks, double* values) {
  if (!c || !a || !ranks || !values) return fail(c, VSIG_E_INVALID, "null pointer");
  if (dtype != VSIG_DTYPE_F32 && dtype != VSIG_DTYPE_F64) return fail(c, VSIG_E_INVALID, "dtype");
  if (nranks < 1 || nranks > 4 || n < 1) return fail(c, VSIG_E_INVALID, "1..4 ranks, n >= 1");
  for (int q = 0; q < nranks; ++q)
    if (ranks[q] < 0 || ranks[q] >= n) return fail(c, VSIG_E_INVALID, "rank out of range");
  const int bits = dtype == VSIG_DTYPE_F32 ? 32 : 64;
  unsigned long long pf[4] = {0, 0, 0, 0}, mk[4] = {0, 0, 0, 0};
  long long k[4];
  for (int q = 0; q < nranks; ++q) k[q] = ranks[q];
  int rc = ensure_stage(c, 2, 4096 * 8 + 64);
  if (rc) return rc;
  unsigned long long* dhist = (unsigned long long*)c->stage[2];
  unsigned long long* dpf = dhist + 4 * 256;
  unsigned long long* dmk = dpf + 4;
  std::vector<unsigned long long> h(4 * 256);
  for (int shift = bits - 8; shift >= 0; shift -= 8) {
    HIPCHK(c, hipMemsetAsync(dhist, 0, 4 * 256 * 8, c->stream));
    HIPCHK(c, hipMemcpyAsync(dpf, pf, sizeof(pf), hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, hipMemcpyAsync(dmk, mk, sizeof(mk), hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, vsig::launch_radix_hist(dtype, a, n, dpf, dmk, nranks, shift, dhist, c->stream));
    HIPCHK(c, hipMemcpyAsync(h.data(), dhist, 4 * 256 * 8, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    for (int q = 0; q < nranks; ++q) {
      long long acc = 0;
      int d = 0;
      for (; d < 255; ++d) {
        const long long cnt = (long long)h[q * 256 + d];
        if (k[q] < acc + cnt) break;
        acc += cnt;
      }
      k[q] -= acc;
      pf[q] |= (unsigned long long)d << shift;
      mk[q] |= 0xffull << shift;
    }
  }
  for (int q = 0; q < nranks; ++q) {
    // invert the order-preserving key (|a| >= 0: sign bit set, no flip)
    if (bits == 32) {
      const unsigned int u = (unsigned int)pf[q] & 0x7fffffffu;
      float f;
      memcpy(&f, &u, 4);
      values[q] = (double)f;
    } else {
      const unsigned long long u = pf[q] & 0x7fffffffffffffffull;
      double d;
      memcpy(&d, &u, 8);
      values[q] = d;
    }
  }
  return VSIG_OK;
}

int vsig_threshold_dev(vsig_ctx* c, int32_t dtype, const void* a, int64_t n, double thr,
                       int64_t* count, int64_t* first, int64_t* last, double* maxval) {
  if (!c || !a || !count || !first || !last || !maxval) return fail(c, VSIG_E_INVALID, "null pointer");
  if (dtype != VSIG_DTYPE_F32 && dtype != VSIG_DTYPE_F64) return fail(c, VSIG_E_INVALID, "dtype");
  if (n < 1) return fail(c, VSIG_E_INVALID, "empty input");
  long long nparts = (n + 255) / 256;
  if (nparts > 2048) nparts = 2048;
  int rc = ensure_stage(c, 2, (size_t)nparts * sizeof(vsig::ThreshPartialH));
  if (rc) return rc;
  HIPCHK(c, vsig::launch_thresh_reduce(dtype, a, n, thr, c->stage[2], (int)nparts, c->stream));
  std::vector<vsig::ThreshPartialH> h(nparts);
  HIPCHK(c, hipMemcpyAsync(h.data(), c->stage[2], nparts * sizeof(vsig::ThreshPartialH),
                           hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  long long cnt = 0, f = n, l = -1;
  double mx = -INFINITY;
  for (auto& p : h) {
    cnt += p.count;
    f = p.first < f ? p.first : f;
    l = p.last > l ? p.last : l;
    mx = p.max > mx ? p.max : mx;
  }
  *count = cnt;
  *first = f;
  *last = l;
  *maxval = mx;
  return VSIG_OK;
}

int vsig_boxcar_energy_dev(vsig_ctx* c, int32_t dtype, const void* x, int64_t n, int64_t w,
                           double* sm) {
  if (!c || !x || !sm) return fail(c, VSIG_E_INVALID, "null pointer");
  if (dtype < VSIG_DTYPE_C128 || dtype > VSIG_DTYPE_F32) return fail(c, VSIG_E_INVALID, "dtype");
  if (n < 1 || w < 1) return fail(c, VSIG_E_INVALID, "need n >= 1, w >= 1");
  const long long nt = vsig::energy_scan_tiles(n);
  int rc;
  if ((rc = ensure_stage(c, 1, (size_t)nt * 8)) || (rc = ensure_stage(c, 2, (size_t)n * 8))) return rc;
  double* P = (double*)c->stage[2];
  HIPCHK(c, vsig::launch_energy_prefix(dtype, x, n, (double*)c->stage[1], P, c->stream));
  HIPCHK(c, vsig::launch_boxcar_same(P, n, w, sm, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));   // stage buffers are reused by the next call
  return VSIG_OK;
}

int vsig_db_dev(vsig_ctx* c, int32_t dtype, const void* a, int64_t n, double floor_, void* out) {
  if (!c || !a || !out) return fail(c, VSIG_E_INVALID, "null pointer");
  if (n < 1) return fail(c, VSIG_E_INVALID, "empty input");
  HIPCHK(c, vsig::launch_db_transform(dtype, a, n, floor_, out, c->stream));
  return VSIG_OK;
}

int vsig_abs_c64_dev(vsig_ctx* c, int32_t dtype, const void* a, int64_t n, void* out) {
  if (!c || !a || !out) return fail(c, VSIG_E_INVALID, "null pointer");
  if (n < 1) return fail(c, VSIG_E_INVALID, "empty input");
  HIPCHK(c, vsig::launch_abs_c64(dtype, a, n, (float2*)out, c->stream));
  return VSIG_OK;
}

int vsig_abs_c128_dev(vsig_ctx* c, int32_t dtype, const void* a, int64_t n, void* out) {
  if (!c || !a || !out) return fail(c, VSIG_E_INVALID, "null pointer");
  if (n < 1) return fail(c, VSIG_E_INVALID, "empty input");
  HIPCHK(c, vsig::launch_abs_c128(dtype, a, n, (double2*)out, c->stream));
  return VSIG_OK;
}

}  // extern "C"
