// Native time-chunk shard of the streaming chain (C ABI: vsig_chain_*), the
// C form of vector_amd/shard.py's StreamChain for callers without Python:
//
//   rank r of P owns X[r n, (r+1) n) of one capture;
//   1. left halo  : X[r n - (ntaps-1), r n) from rank r-1 (rank 0: zeros),
//                   exchanged on a side stream while the FIR filters every
//                   output that needs only the rank's own samples;
//   2. FIR + D    : y = filter(X)[r n / D, (r+1) n / D) (vsig_fir);
//   3. right halo : y[(r+1) n / D, + L-1) from rank r+1, on the side stream
//                   while the PSD runs;
//   4. PSD        : frames of nfft, hop nfft, never straddling a chunk;
//   5. sync       : valid correlation of [y | halo] with the template, fused
//                   |c| peak + exact refine (vsig_xcorr);
//   6. peak rows  : all-gather of the ranks' 32-byte peak records; the global
//                   peak is the largest, lowest global index on ties.
// Only the halos (KB) and the peak records cross the transport.  Reference
// precedent: heavy_packet_optimizer.py:114-152's overlapped chunking (its
// merge duplicated the overlap, :195-222; not reproduced).
//
// Transports (vsig_transport): RCCL over xGMI (librccl resolved at run time,
// so libvsig.so carries no link dependency on it) and an in-process loopback
// (ranks on host threads of one process) that the tests use to run several
// ranks on one GPU.
#include <dlfcn.h>

#include <condition_variable>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/vsig.h"
#include "vsig_kernels.h"

struct vsig_chain {
  vsig_ctx* ctx = nullptr;
  int rank = 0, world = 1;
  vsig_transport tr{};
  long long n = 0, ny = 0, L = 0, hist = 0;
  int decim = 1, nfft = 0;
  float scale = 1.f;
  vsig_fir* fir = nullptr;
  vsig_xcorr* xc = nullptr;
  float2* x_ext = nullptr;           // [left halo | chunk]
  float2* y_ext = nullptr;           // [chunk output | right halo]
  float* sxx = nullptr;              // frame-major spectra
  float* win = nullptr;
  vsig_peak_t* rec = nullptr;        // this rank's record
  vsig_peak_t* rows = nullptr;       // world records (all-gather)
  hipStream_t side = nullptr;        // halo exchanges
  hipEvent_t ev_in = nullptr, ev_halo = nullptr, ev_fir = nullptr, ev_rhalo = nullptr;
  std::string err;
};

namespace {

int chain_fail(vsig_chain* ch, int code, const std::string& m) {
  if (ch) ch->err = m;
  return code;
}

#define CHK(ch, expr)                                                                    \
  do {                                                                                   \
    hipError_t e_ = (expr);                                                              \
    if (e_ != hipSuccess) return chain_fail(ch, VSIG_E_HIP, std::string(#expr) + ": " + hipGetErrorString(e_)); \
  } while (0)

hipStream_t ctx_stream(vsig_ctx* c) { return (hipStream_t)vsig_get_stream(c); }

}  // namespace

extern "C" {

void vsig_chain_free(vsig_chain* ch) {
  if (!ch) return;
  (void)hipDeviceSynchronize();
  if (ch->fir) vsig_fir_free(ch->fir);
  if (ch->xc) vsig_xcorr_free(ch->xc);
  for (void* p : {(void*)ch->x_ext, (void*)ch->y_ext, (void*)ch->sxx, (void*)ch->win, (void*)ch->rec,
                  (void*)ch->rows})
    if (p) (void)hipFree(p);
  for (hipEvent_t e : {ch->ev_in, ch->ev_halo, ch->ev_fir, ch->ev_rhalo})
    if (e) (void)hipEventDestroy(e);
  if (ch->side) (void)hipStreamDestroy(ch->side);
  delete ch;
}

int vsig_chain_create(vsig_ctx* ctx, const vsig_chain_config* cfg, int32_t rank, int32_t world,
                      const vsig_transport* tr, vsig_chain** out) {
  if (!ctx || !cfg || !out || !cfg->taps || !cfg->window) return VSIG_E_INVALID;
  *out = nullptr;
  if (world < 1 || rank < 0 || rank >= world) return VSIG_E_INVALID;
  if (world > 1 && (!tr || !tr->sendrecv || !tr->allgather)) return VSIG_E_INVALID;
  const long long n = cfg->n_local, D = cfg->decim, nfft = cfg->nfft;
  if (n < 1 || D < 1 || nfft < 1 || cfg->ntaps < 1) return VSIG_E_INVALID;
  if (n % (nfft * D)) return VSIG_E_INVALID;              // frames never straddle chunks
  vsig_chain* ch = new vsig_chain();
  ch->ctx = ctx;
  ch->rank = rank;
  ch->world = world;
  if (tr) ch->tr = *tr;
  ch->n = n;
  ch->decim = (int)D;
  ch->nfft = (int)nfft;
  ch->ny = n / D;
  ch->hist = (cfg->ntaps - 1 + 15) / 16 * 16;   // 128-byte-aligned segment starts (shard.py)
  ch->L = cfg->tmpl ? cfg->L : 0;
  ch->scale = cfg->psd_scale;
  if (world > 1 && (n < ch->hist || (ch->L && ch->ny < ch->L - 1))) {
    vsig_chain_free(ch);
    return VSIG_E_INVALID;                                 // halos longer than a chunk
  }
  int rc = vsig_fir_create(ctx, cfg->taps, cfg->ntaps, cfg->decim, &ch->fir);
  if (!rc && ch->L) rc = vsig_xcorr_create(ctx, cfg->tmpl, ch->L, &ch->xc);
  if (rc) { vsig_chain_free(ch); return rc; }
  const long long yl = ch->ny + (ch->L ? ch->L - 1 : 0);
  hipError_t e = hipMalloc(&ch->x_ext, (size_t)(ch->hist + n) * 8);
  if (e == hipSuccess) e = hipMalloc(&ch->y_ext, (size_t)yl * 8);
  if (e == hipSuccess) e = hipMalloc(&ch->sxx, (size_t)ch->ny * 4);
  if (e == hipSuccess) e = hipMalloc(&ch->win, (size_t)nfft * 4);
  if (e == hipSuccess) e = hipMalloc(&ch->rec, sizeof(vsig_peak_t));
  if (e == hipSuccess) e = hipMalloc(&ch->rows, sizeof(vsig_peak_t) * world);
  if (e == hipSuccess) e = hipMemset(ch->x_ext, 0, (size_t)(ch->hist + n) * 8);
  if (e == hipSuccess) e = hipMemset(ch->y_ext, 0, (size_t)yl * 8);
  if (e == hipSuccess) e = hipMemcpy(ch->win, cfg->window, (size_t)nfft * 4, hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipStreamCreateWithFlags(&ch->side, hipStreamNonBlocking);
  for (hipEvent_t* ev : {&ch->ev_in, &ch->ev_halo, &ch->ev_fir, &ch->ev_rhalo})
    if (e == hipSuccess) e = hipEventCreateWithFlags(ev, hipEventDisableTiming);
  if (e != hipSuccess) {
    vsig_chain_free(ch);
    return e == hipErrorOutOfMemory ? VSIG_E_NOMEM : VSIG_E_HIP;
  }
  *out = ch;
  return VSIG_OK;
}

const char* vsig_chain_last_error(const vsig_chain* ch) { return ch ? ch->err.c_str() : "null chain"; }

void* vsig_chain_input(vsig_chain* ch) { return ch ? (void*)(ch->x_ext + ch->hist) : nullptr; }

const void* vsig_chain_filtered(const vsig_chain* ch, int64_t* n) {
  if (!ch) return nullptr;
  if (n) *n = ch->ny;
  return ch->y_ext;
}

const float* vsig_chain_spectra(const vsig_chain* ch, int64_t* nframes) {
  if (!ch) return nullptr;
  if (nframes) *nframes = ch->ny / ch->nfft;
  return ch->sxx;
}

int vsig_chain_step(vsig_chain* ch) {
  if (!ch) return VSIG_E_INVALID;
  vsig_ctx* c = ch->ctx;
  hipStream_t st = ctx_stream(c);
  const int r = ch->rank, w = ch->world;
  const long long n = ch->n, D = ch->decim, h = ch->hist, ny = ch->ny;
  int rc;
  // 1-2. left halo on the side stream, the FIR's bulk meanwhile
  const bool lh = w > 1 && h > 0;
  if (lh) {
    CHK(ch, hipEventRecord(ch->ev_in, st));              // the caller's input is in place
    CHK(ch, hipStreamWaitEvent(ch->side, ch->ev_in, 0));
    rc = ch->tr.sendrecv(ch->tr.user, r < w - 1 ? (const void*)(ch->x_ext + n) : nullptr,
                         r < w - 1 ? h * 8 : 0, r < w - 1 ? r + 1 : -1,
                         r > 0 ? (void*)ch->x_ext : nullptr, r > 0 ? h * 8 : 0, r > 0 ? r - 1 : -1,
                         ch->side);
    if (rc) return chain_fail(ch, VSIG_E_HIP, "transport: left-halo exchange failed");
    CHK(ch, hipEventRecord(ch->ev_halo, ch->side));
  }
  const long long s = lh ? ((h + D - 1) / D) * D : 0;    // first output needing only own samples
  auto fir = [&](long long a, long long b) {             // chunk samples [a, b) -> y[a/D, b/D)
    return vsig_fir_exec_hist_dev(ch->fir, ch->x_ext + a, h, b - a, ch->y_ext + a / D,
                                  (b - a + D - 1) / D);
  };
  if (s < n && (rc = fir(s, n))) return rc;
  if (lh) CHK(ch, hipStreamWaitEvent(st, ch->ev_halo, 0));
  if (s > 0 && (rc = fir(0, s < n ? s : n))) return rc;
  // 3. right halo of the filtered stream while the PSD runs
  const long long L = ch->L;
  const bool rh = w > 1 && L > 1;
  if (rh) {
    CHK(ch, hipEventRecord(ch->ev_fir, st));
    CHK(ch, hipStreamWaitEvent(ch->side, ch->ev_fir, 0));
    rc = ch->tr.sendrecv(ch->tr.user, r > 0 ? (const void*)ch->y_ext : nullptr,
                         r > 0 ? (L - 1) * 8 : 0, r > 0 ? r - 1 : -1,
                         r < w - 1 ? (void*)(ch->y_ext + ny) : nullptr,
                         r < w - 1 ? (L - 1) * 8 : 0, r < w - 1 ? r + 1 : -1, ch->side);
    if (rc) return chain_fail(ch, VSIG_E_HIP, "transport: right-halo exchange failed");
    CHK(ch, hipEventRecord(ch->ev_rhalo, ch->side));
  }
  // 4. PSD
  const long long nframes = ny / ch->nfft;
  if (nframes > 0 &&
      (rc = vsig_psd_c64_dev(c, ch->y_ext, ny, 1, ch->win, ch->nfft, ch->nfft, ch->nfft, ch->scale, 0,
                             ch->sxx, nframes)))
    return rc;
  if (!L) return VSIG_OK;
  // 5. sync correlation over [y | right halo]
  if (rh) CHK(ch, hipStreamWaitEvent(st, ch->ev_rhalo, 0));
  const long long halo = r < w - 1 ? L - 1 : 0;
  if ((rc = vsig_xcorr_exec_dev(ch->xc, ch->y_ext, ny + halo, VSIG_MODE_VALID, nullptr, ch->rec)))
    return rc;
  // 6. peak records of every rank (through the transport whenever one is given)
  if (ch->tr.allgather) {
    if (ch->tr.allgather(ch->tr.user, ch->rec, ch->rows, sizeof(vsig_peak_t), st))
      return chain_fail(ch, VSIG_E_HIP, "transport: peak all-gather failed");
  } else {
    CHK(ch, hipMemcpyAsync(ch->rows, ch->rec, sizeof(vsig_peak_t), hipMemcpyDeviceToDevice, st));
  }
  return VSIG_OK;
}

int vsig_chain_result(vsig_chain* ch, vsig_peak_t* peak, int64_t* nout) {
  if (!ch || !peak) return VSIG_E_INVALID;
  if (!ch->L) return chain_fail(ch, VSIG_E_INVALID, "chain without a sync template");
  std::vector<vsig_peak_t> rows(ch->world);
  hipStream_t st = ctx_stream(ch->ctx);
  CHK(ch, hipMemcpyAsync(rows.data(), ch->rows, sizeof(vsig_peak_t) * ch->world,
                         hipMemcpyDeviceToHost, st));
  CHK(ch, hipStreamSynchronize(st));
  // the exact-argmax contract: a refine fault on this rank (sticky since the
  // last check) or on any other (its gathered row's poisoned index) is an error
  int32_t rst = 0;
  int64_t rcand = 0;
  int rc = vsig_refine_status(ch->ctx, &rst, &rcand);
  if (rc) return chain_fail(ch, rc, "refine status");
  if (rst == 3) return chain_fail(ch, VSIG_E_REFINE, "exact-argmax refine faulted on this rank");
  for (int q = 0; q < ch->world; ++q)
    if (rows[q].index < 0)
      return chain_fail(ch, VSIG_E_REFINE, "exact-argmax refine faulted on rank " + std::to_string(q));
  vsig_peak_t best{-1.0, 0, 0.0, 0.0};
  bool have = false;
  double s1 = 0.0, s2 = 0.0;
  for (int q = 0; q < ch->world; ++q) {
    const int64_t gi = (int64_t)q * ch->ny + rows[q].index;
    if (!have || rows[q].peak > best.peak || (rows[q].peak == best.peak && gi < best.index)) {
      best.peak = rows[q].peak;
      best.index = gi;
      have = true;
    }
    s1 += rows[q].sum_abs;
    s2 += rows[q].sum_abs2;
  }
  best.sum_abs = s1;
  best.sum_abs2 = s2;
  *peak = best;
  if (nout) *nout = (int64_t)ch->world * ch->ny - ch->L + 1;
  return VSIG_OK;
}

}  // extern "C"

// ---------------------------------------------------------------------------
// RCCL transport (librccl resolved at run time)
// ---------------------------------------------------------------------------
namespace {

typedef int nccl_result;
typedef void* nccl_comm;
struct nccl_uid { char internal[128]; };

struct Rccl {
  bool ok = false;
  nccl_result (*GetUniqueId)(nccl_uid*) = nullptr;
  nccl_result (*CommInitRank)(nccl_comm*, int, nccl_uid, int) = nullptr;
  nccl_result (*CommDestroy)(nccl_comm) = nullptr;
  nccl_result (*GroupStart)() = nullptr;
  nccl_result (*GroupEnd)() = nullptr;
  nccl_result (*Send)(const void*, size_t, int, int, nccl_comm, hipStream_t) = nullptr;
  nccl_result (*Recv)(void*, size_t, int, int, nccl_comm, hipStream_t) = nullptr;
  nccl_result (*AllGather)(const void*, void*, size_t, int, nccl_comm, hipStream_t) = nullptr;
};

constexpr int kNcclUint8 = 1;        // ncclUint8 (rccl.h)

Rccl& rccl() {
  static Rccl r;
  static std::once_flag once;
  std::call_once(once, [] {
    void* h = nullptr;
    if (const char* p = getenv("VSIG_RCCL_LIB")) h = dlopen(p, RTLD_NOW);
    // a process that already holds an RCCL (e.g. torch's) shares it
    for (const char* nm : {"librccl.so", "librccl.so.1"})
      if (!h) h = dlopen(nm, RTLD_NOW | RTLD_NOLOAD);
    for (const char* nm : {"librccl.so.1", "/opt/rocm/lib/librccl.so.1"})
      if (!h) h = dlopen(nm, RTLD_NOW);
    if (!h) return;
    auto sym = [&](auto& fp, const char* nm) { fp = reinterpret_cast<std::remove_reference_t<decltype(fp)>>(dlsym(h, nm)); return fp != nullptr; };
    r.ok = sym(r.GetUniqueId, "ncclGetUniqueId") && sym(r.CommInitRank, "ncclCommInitRank") &&
           sym(r.CommDestroy, "ncclCommDestroy") && sym(r.GroupStart, "ncclGroupStart") &&
           sym(r.GroupEnd, "ncclGroupEnd") && sym(r.Send, "ncclSend") && sym(r.Recv, "ncclRecv") &&
           sym(r.AllGather, "ncclAllGather");
  });
  return r;
}

int rccl_sendrecv(void* user, const void* send, int64_t sb, int32_t dst, void* recv, int64_t rb,
                  int32_t src, void* stream) {
  Rccl& r = rccl();
  nccl_comm comm = user;
  hipStream_t st = (hipStream_t)stream;
  if (r.GroupStart()) return -1;
  if (send && dst >= 0 && sb > 0 && r.Send(send, (size_t)sb, kNcclUint8, dst, comm, st)) { r.GroupEnd(); return -1; }
  if (recv && src >= 0 && rb > 0 && r.Recv(recv, (size_t)rb, kNcclUint8, src, comm, st)) { r.GroupEnd(); return -1; }
  return r.GroupEnd() ? -1 : 0;
}

int rccl_allgather(void* user, const void* send, void* recv, int64_t bytes, void* stream) {
  Rccl& r = rccl();
  return r.AllGather(send, recv, (size_t)bytes, kNcclUint8, (nccl_comm)user, (hipStream_t)stream) ? -1 : 0;
}

}  // namespace

extern "C" {

int vsig_rccl_available(void) { return rccl().ok ? 1 : 0; }

int vsig_rccl_unique_id(char id[128]) {
  if (!id) return VSIG_E_INVALID;
  Rccl& r = rccl();
  if (!r.ok) return VSIG_E_UNSUPPORTED;
  nccl_uid u;
  if (r.GetUniqueId(&u)) return VSIG_E_HIP;
  memcpy(id, u.internal, 128);
  return VSIG_OK;
}

int vsig_rccl_comm_init(int32_t world, int32_t rank, const char id[128], int32_t device, void** comm) {
  if (!id || !comm || world < 1 || rank < 0 || rank >= world) return VSIG_E_INVALID;
  Rccl& r = rccl();
  if (!r.ok) return VSIG_E_UNSUPPORTED;
  // the communicator binds to the current device: set it for the call only
  int prev = 0;
  if (hipGetDevice(&prev) != hipSuccess || hipSetDevice(device) != hipSuccess) return VSIG_E_HIP;
  nccl_uid u;
  memcpy(u.internal, id, 128);
  nccl_comm cm = nullptr;
  const int rc = r.CommInitRank(&cm, world, u, rank);
  (void)hipSetDevice(prev);
  if (rc) return VSIG_E_HIP;
  *comm = cm;
  return VSIG_OK;
}

int vsig_rccl_comm_destroy(void* comm) {
  Rccl& r = rccl();
  if (!r.ok || !comm) return VSIG_E_INVALID;
  return r.CommDestroy((nccl_comm)comm) ? VSIG_E_HIP : VSIG_OK;
}

int vsig_rccl_transport(void* comm, vsig_transport* out) {
  if (!comm || !out) return VSIG_E_INVALID;
  if (!rccl().ok) return VSIG_E_UNSUPPORTED;
  out->user = comm;
  out->sendrecv = rccl_sendrecv;
  out->allgather = rccl_allgather;
  return VSIG_OK;
}

}  // extern "C"

// ---------------------------------------------------------------------------
// In-process loopback transport: the ranks are host threads of one process
// (one vsig_ctx / stream each, any devices with peer access).  A send posts
// its buffer and an event recorded after it on the sender's stream; the
// receiver waits for the post, makes its stream wait on the event and copies;
// sendrecv returns once its own post has been copied (blocking, as
// MPI_Sendrecv: the sender's next kernels may overwrite the buffer).
// ---------------------------------------------------------------------------
struct vsig_loopback {
  int world = 0;
  std::mutex mu;
  std::condition_variable cv;
  struct Post { const void* p = nullptr; int64_t bytes = 0; hipEvent_t ev = nullptr; bool full = false; };
  std::vector<Post> box;             // box[src * world + dst]
  std::vector<Post> gather;          // gather[rank] for the current all-gather round
  std::vector<int> done;             // ranks finished copying this round
  long long round = 0;
  int arrived = 0, left = 0;
  std::vector<void*> transports;     // the per-rank handles given out
};

namespace {

struct LoopRank { vsig_loopback* lb; int rank; };

int loop_sendrecv(void* user, const void* send, int64_t sb, int32_t dst, void* recv, int64_t rb,
                  int32_t src, void* stream) {
  LoopRank* lr = static_cast<LoopRank*>(user);
  vsig_loopback* lb = lr->lb;
  hipStream_t st = (hipStream_t)stream;
  const int W = lb->world;
  if (send && dst >= 0) {
    hipEvent_t ev;
    if (hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess) return -1;
    if (hipEventRecord(ev, st) != hipSuccess) return -1;
    std::unique_lock<std::mutex> lk(lb->mu);
    auto& b = lb->box[lr->rank * W + dst];
    lb->cv.wait(lk, [&] { return !b.full; });           // the previous post was consumed
    b = vsig_loopback::Post{send, sb, ev, true};
    lb->cv.notify_all();
  }
  if (recv && src >= 0) {
    vsig_loopback::Post p;
    {
      std::unique_lock<std::mutex> lk(lb->mu);
      auto& b = lb->box[src * W + lr->rank];
      lb->cv.wait(lk, [&] { return b.full; });
      p = b;
    }
    if (p.bytes != rb) return -1;
    if (hipStreamWaitEvent(st, p.ev, 0) != hipSuccess) return -1;
    if (hipMemcpyAsync(recv, p.p, (size_t)rb, hipMemcpyDeviceToDevice, st) != hipSuccess) return -1;
    if (hipStreamSynchronize(st) != hipSuccess) return -1;   // the sender may reuse its buffer
    (void)hipEventDestroy(p.ev);
    std::unique_lock<std::mutex> lk(lb->mu);
    lb->box[src * W + lr->rank].full = false;
    lb->cv.notify_all();
  }
  if (send && dst >= 0) {
    // like MPI_Sendrecv: return once the receiver has copied our buffer (the
    // caller's later kernels may overwrite it)
    std::unique_lock<std::mutex> lk(lb->mu);
    auto& b = lb->box[lr->rank * W + dst];
    lb->cv.wait(lk, [&] { return !b.full; });
  }
  return 0;
}

int loop_allgather(void* user, const void* send, void* recv, int64_t bytes, void* stream) {
  LoopRank* lr = static_cast<LoopRank*>(user);
  vsig_loopback* lb = lr->lb;
  hipStream_t st = (hipStream_t)stream;
  const int W = lb->world;
  hipEvent_t ev;
  if (hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess) return -1;
  if (hipEventRecord(ev, st) != hipSuccess) return -1;
  std::unique_lock<std::mutex> lk(lb->mu);
  lb->cv.wait(lk, [&] { return lb->left == 0; });       // the previous round has drained
  lb->gather[lr->rank] = vsig_loopback::Post{send, bytes, ev, true};
  const long long my_round = lb->round;
  if (++lb->arrived == W) lb->cv.notify_all();
  lb->cv.wait(lk, [&] { return lb->arrived == W || lb->round != my_round; });
  std::vector<vsig_loopback::Post> all = lb->gather;
  lk.unlock();
  int rc = 0;
  for (int q = 0; q < W && !rc; ++q) {
    if (hipStreamWaitEvent(st, all[q].ev, 0) != hipSuccess ||
        hipMemcpyAsync(static_cast<char*>(recv) + q * bytes, all[q].p, (size_t)bytes,
                       hipMemcpyDeviceToDevice, st) != hipSuccess)
      rc = -1;
  }
  if (hipStreamSynchronize(st) != hipSuccess) rc = -1;
  lk.lock();
  if (++lb->left == W) {                                 // last one out resets the round
    for (auto& g : lb->gather) { (void)hipEventDestroy(g.ev); g = vsig_loopback::Post{}; }
    lb->arrived = 0;
    lb->left = 0;
    ++lb->round;
    lb->cv.notify_all();
  } else {
    lb->cv.wait(lk, [&] { return lb->round != my_round; });
  }
  return rc;
}

}  // namespace

extern "C" {

int vsig_loopback_create(int32_t world, vsig_loopback** out) {
  if (world < 1 || !out) return VSIG_E_INVALID;
  vsig_loopback* lb = new vsig_loopback();
  lb->world = world;
  lb->box.resize((size_t)world * world);
  lb->gather.resize(world);
  *out = lb;
  return VSIG_OK;
}

void vsig_loopback_free(vsig_loopback* lb) {
  if (!lb) return;
  for (auto& r : lb->transports) delete static_cast<LoopRank*>(r);
  delete lb;
}

int vsig_loopback_transport(vsig_loopback* lb, int32_t rank, vsig_transport* out) {
  if (!lb || !out || rank < 0 || rank >= lb->world) return VSIG_E_INVALID;
  LoopRank* lr = new LoopRank{lb, rank};
  {
    std::lock_guard<std::mutex> g(lb->mu);
    lb->transports.push_back(lr);
  }
  out->user = lr;
  out->sendrecv = loop_sendrecv;
  out->allgather = loop_allgather;
  return VSIG_OK;
}

}  // extern "C"
