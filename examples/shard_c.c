/* The time-chunk shard of the chain through the C ABI (vsig_chain_*) from
 * plain C: FIR -> decimate 4 -> PSD -> sync correlation, the capture split
 * across ranks that exchange only the FIR / correlation halos and 32-byte peak
 * records (the C form of vector_amd/shard.py).
 *
 *   ./shard_c loopback W            W ranks as threads of this process, all on
 *                                   device 0 (in-process loopback transport)
 *   ./shard_c rccl RANK WORLD FILE [DEVICE]
 *                                   one rank per process and GPU over RCCL:
 *                                   rank 0 writes the RCCL unique id to FILE,
 *                                   the others wait for it (one node); DEVICE
 *                                   (default RANK) puts every rank on one GPU
 *                                   for a one-GPU rehearsal (each rank then
 *                                   needs its own NCCL_HOSTID: RCCL's socket
 *                                   transport, tests/test_gpu_native_chain.py)
 *
 * Every rank synthesises its own chunk of one capture (tones + LCG noise seeded
 * by the global sample index, a QPSK preamble planted at K0) and prints the
 * global peak; exit status 0 = the preamble found at K0 / D on every rank.
 *
 * Build (tests/test_host_cpu.py::test_c_examples_compile):
 *   gcc -std=c99 -O2 -Iinclude examples/shard_c.c -Lvector_amd -lvsig \
 *       -Wl,-rpath,'$ORIGIN/../vector_amd' -lpthread -lm -o examples/shard_c
 */
#define _POSIX_C_SOURCE 200809L
#define _USE_MATH_DEFINES
#include <math.h>
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <unistd.h>

#include "vsig.h"

#define NLOC (1 << 20)          /* input samples per rank */
#define D 4
#define NTAPS 63
#define L 256                   /* template samples (decimated rate) */
#define NFFT 1024
#ifndef M_PI
#define M_PI 3.14159265358979323846
#endif

static float taps[2 * NTAPS];      /* complex64: windowed-sinc lowpass, cutoff 0.2 */
static float tmpl[2 * L];          /* preamble through the filter, every D-th sample */
static float pre[2 * L * D];       /* QPSK preamble at the input rate */
static float win[NFFT];
static int64_t K0;

static float hash01(uint64_t i) {  /* deterministic noise from the global index */
  uint64_t z = i * 0x9E3779B97F4A7C15ull + 0x632BE59BD9B4E019ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  z ^= z >> 31;
  return (float)((double)(z >> 11) / 9007199254740992.0 * 2.0 - 1.0);
}

static void design(int world) {
  double s = 0.0;
  for (int k = 0; k < NTAPS; ++k) {
    const double m = k - (NTAPS - 1) / 2.0;
    const double h = (m == 0 ? 0.4 : sin(0.4 * M_PI * m) / (M_PI * m)) *
                     (0.54 - 0.46 * cos(2 * M_PI * k / (NTAPS - 1)));
    taps[2 * k] = (float)h;
    taps[2 * k + 1] = 0.f;
    s += h;
  }
  for (int k = 0; k < NTAPS; ++k) taps[2 * k] = (float)(taps[2 * k] / s);
  uint64_t st = 4096;
  for (int i = 0; i < L * D; ++i) {
    st = st * 6364136223846793005ull + 1442695040888963407ull;
    pre[2 * i] = (st >> 62) & 1 ? 0.70710677f : -0.70710677f;
    pre[2 * i + 1] = (st >> 61) & 1 ? 0.70710677f : -0.70710677f;
  }
  for (int o = 0; o < L; ++o) {      /* causal filtered preamble at o * D */
    double re = 0, im = 0;
    for (int k = 0; k < NTAPS && k <= o * D; ++k) {
      re += taps[2 * k] * pre[2 * (o * D - k)];
      im += taps[2 * k] * pre[2 * (o * D - k) + 1];
    }
    tmpl[2 * o] = (float)re;
    tmpl[2 * o + 1] = (float)im;
  }
  for (int i = 0; i < NFFT; ++i) win[i] = (float)(0.5 - 0.5 * cos(2 * M_PI * i / NFFT));
  K0 = ((int64_t)world * NLOC / D / 2 + 777) * D;
}

static void fill(float* x, int rank) {   /* this rank's chunk of the capture */
  for (int64_t i = 0; i < NLOC; ++i) {
    const int64_t g = (int64_t)rank * NLOC + i;
    const double ph = 2 * M_PI * fmod(0.05 * (double)g, 1.0);
    x[2 * i] = (float)cos(ph) + 0.5f * hash01(2 * (uint64_t)g);
    x[2 * i + 1] = (float)sin(ph) + 0.5f * hash01(2 * (uint64_t)g + 1);
    if (g >= K0 && g < K0 + L * D) {
      x[2 * i] += 3.f * pre[2 * (g - K0)];
      x[2 * i + 1] += 3.f * pre[2 * (g - K0) + 1];
    }
  }
}

struct rank_args { int rank, world, device; vsig_transport tr; int have_tr; int ok; };

static void* run_rank(void* p) {
  struct rank_args* a = (struct rank_args*)p;
  a->ok = 0;
  vsig_ctx* ctx = NULL;
  vsig_chain* ch = NULL;
  float* x = (float*)malloc((size_t)NLOC * 8);
  if (!x || vsig_init(a->device, &ctx)) { fprintf(stderr, "rank %d: init failed\n", a->rank); return NULL; }
  double ws = 0;
  for (int i = 0; i < NFFT; ++i) ws += win[i];
  vsig_chain_config cfg = {NLOC, taps, NTAPS, D, NFFT, win, (float)(1.0 / (ws * ws)), tmpl, L};
  int rc = vsig_chain_create(ctx, &cfg, a->rank, a->world, a->have_tr ? &a->tr : NULL, &ch);
  if (rc) { fprintf(stderr, "rank %d: chain_create %d %s\n", a->rank, rc, vsig_last_error(ctx)); return NULL; }
  fill(x, a->rank);
  if ((rc = vsig_copy_dev(ctx, vsig_chain_input(ch), x, (int64_t)NLOC * 8)) ||
      (rc = vsig_chain_step(ch))) {
    fprintf(stderr, "rank %d: step %d %s\n", a->rank, rc, vsig_chain_last_error(ch));
    return NULL;
  }
  vsig_peak_t pk;
  int64_t nout = 0;
  if ((rc = vsig_chain_result(ch, &pk, &nout))) { fprintf(stderr, "rank %d: result %d\n", a->rank, rc); return NULL; }
  printf("rank %d/%d: global peak |c| = %.4f at lag %lld (planted %lld), %lld outputs\n", a->rank,
         a->world, pk.peak, (long long)pk.index, (long long)(K0 / D), (long long)nout);
  a->ok = pk.index == K0 / D;
  vsig_chain_free(ch);
  vsig_free(ctx);
  free(x);
  return NULL;
}

int main(int argc, char** argv) {
  if (argc >= 3 && !strcmp(argv[1], "loopback")) {
    const int W = atoi(argv[2]);
    if (W < 1 || W > 16) return 2;
    design(W);
    vsig_loopback* lb = NULL;
    if (vsig_loopback_create(W, &lb)) return 2;
    struct rank_args a[16];
    pthread_t th[16];
    for (int r = 0; r < W; ++r) {
      a[r].rank = r; a[r].world = W; a[r].device = 0; a[r].have_tr = 1;
      if (vsig_loopback_transport(lb, r, &a[r].tr)) return 2;
      pthread_create(&th[r], NULL, run_rank, &a[r]);
    }
    int ok = 1;
    for (int r = 0; r < W; ++r) { pthread_join(th[r], NULL); ok &= a[r].ok; }
    vsig_loopback_free(lb);
    return ok ? 0 : 1;
  }
  if (argc >= 5 && !strcmp(argv[1], "rccl")) {
    const int rank = atoi(argv[2]), world = atoi(argv[3]);
    const char* file = argv[4];
    const int device = argc >= 6 ? atoi(argv[5]) : rank;
    design(world);
    char id[128];
    if (rank == 0) {
      /* IDFILE must be a fresh path per run: ranks > 0 take the first file
       * they find there, so a stale one would make them join an old id */
      remove(file);
      if (vsig_rccl_unique_id(id)) { fprintf(stderr, "no RCCL\n"); return 2; }
      char tmp[4096];
      snprintf(tmp, sizeof tmp, "%s.tmp", file);
      FILE* f = fopen(tmp, "wb");
      if (!f || fwrite(id, 1, 128, f) != 128) return 2;
      fclose(f);
      rename(tmp, file);
    } else {
      FILE* f = NULL;
      for (int t = 0; t < 600 && !(f = fopen(file, "rb")); ++t) {
        struct timespec ts = {0, 100000000};
        nanosleep(&ts, NULL);
      }
      if (!f || fread(id, 1, 128, f) != 128) return 2;
      fclose(f);
    }
    void* comm = NULL;
    if (vsig_rccl_comm_init(world, rank, id, device, &comm)) { fprintf(stderr, "comm init failed\n"); return 2; }
    struct rank_args a = {rank, world, device, {0}, 1, 0};
    if (vsig_rccl_transport(comm, &a.tr)) return 2;
    run_rank(&a);
    vsig_rccl_comm_destroy(comm);
    return a.ok ? 0 : 1;
  }
  fprintf(stderr, "usage: shard_c loopback W | shard_c rccl RANK WORLD IDFILE [DEVICE] (a fresh IDFILE per run)\n");
  return 2;
}
