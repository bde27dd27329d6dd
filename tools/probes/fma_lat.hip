// Latency probe (measurement aid): one wave runs a dependent fp64 fma chain,
// a dependent LDS-load chain and fp64 chains fed from LDS in several loop
// forms; prints cycles per step (s_memtime) and the shader clock against the
// 100 MHz wall clock.
#include <hip/hip_runtime.h>
#include <cstdio>

template <int KB>
__device__ double batched(const double* Xs, const double* Ys, int nst, double acc) {
  const int nfull = nst & ~(KB - 1);
  double xb[KB], yb[KB];
#pragma unroll
  for (int i = 0; i < KB; ++i) { xb[i] = Xs[8 * i]; yb[i] = Ys[8 * i]; }
  for (int j = 0; j < nfull; j += KB) {
    double xn[KB], yn[KB];
    const int jn = j + KB < nfull ? j + KB : j;
#pragma unroll
    for (int i = 0; i < KB; ++i) { xn[i] = Xs[8 * (jn + i)]; yn[i] = Ys[8 * (jn + i)]; }
#pragma unroll
    for (int i = 0; i < KB; ++i) acc = fma(xb[i], yb[i], acc);
#pragma unroll
    for (int i = 0; i < KB; ++i) { xb[i] = xn[i]; yb[i] = yn[i]; }
  }
  return acc;
}

// ring of R batches of 8 in flight
template <int R>
__device__ double ring(const double* Xs, const double* Ys, int nst, double acc) {
  double xb[R][8], yb[R][8];
#pragma unroll
  for (int r = 0; r < R; ++r)
#pragma unroll
    for (int i = 0; i < 8; ++i) { xb[r][i] = Xs[8 * (8 * r + i)]; yb[r][i] = Ys[8 * (8 * r + i)]; }
  for (int j = 0; j < nst; j += 8 * R) {
#pragma unroll
    for (int r = 0; r < R; ++r) {
#pragma unroll
      for (int i = 0; i < 8; ++i) acc = fma(xb[r][i], yb[r][i], acc);
      int jn = j + 8 * R + 8 * r;
      jn = jn < nst ? jn : 0;
#pragma unroll
      for (int i = 0; i < 8; ++i) { xb[r][i] = Xs[8 * (jn + i)]; yb[r][i] = Ys[8 * (jn + i)]; }
    }
  }
  return acc;
}

// lanes 0..7: the four component chains of slot s per lane, batches of KB steps
template <int KB>
__device__ double4 quad(const double2* Xs, const double2* Ys, int nst) {
  double d0 = 0, d1 = 0, d2 = 0, d3 = 0;
  auto step = [&](const double2& x, const double2& y) {
    d0 = fma(x.x, y.x, d0); d1 = fma(x.y, y.y, d1); d2 = fma(x.x, y.y, d2); d3 = fma(x.y, y.x, d3);
  };
  double2 xb[KB], yb[KB];
#pragma unroll
  for (int i = 0; i < KB; ++i) { xb[i] = Xs[8 * i]; yb[i] = Ys[8 * i]; }
  for (int j = 0; j < nst; j += KB) {
    double2 xn[KB], yn[KB];
    const int jn = j + KB < nst ? j + KB : j;
#pragma unroll
    for (int i = 0; i < KB; ++i) { xn[i] = Xs[8 * (jn + i)]; yn[i] = Ys[8 * (jn + i)]; }
#pragma unroll
    for (int i = 0; i < KB; ++i) step(xb[i], yb[i]);
#pragma unroll
    for (int i = 0; i < KB; ++i) { xb[i] = xn[i]; yb[i] = yn[i]; }
  }
  return make_double4(d0, d1, d2, d3);
}

__global__ void probe(double* out, long long* cyc, int n) {
  __shared__ double lds[8192];
  const int t = threadIdx.x;
  for (int i = t; i < 8192; i += blockDim.x) lds[i] = 1.0 + 1e-9 * i;
  __syncthreads();
  double a = out[t], b = 1.0000001, c = 1e-7;
  long long w0 = wall_clock64(), c0 = clock64();
  for (int i = 0; i < n; ++i) {            // dependent fma chain
    a = fma(a, b, c);
    a = fma(a, b, c);
    a = fma(a, b, c);
    a = fma(a, b, c);
  }
  long long c1 = clock64(), w1 = wall_clock64();
  int idx = t & 7;
  long long c2 = clock64();
  for (int i = 0; i < n; ++i) {            // dependent LDS loads
    idx = (int)lds[idx] & 7;
    idx = (int)lds[idx + 8] & 7;
    idx = (int)lds[idx + 16] & 7;
    idx = (int)lds[idx + 24] & 7;
  }
  long long c3 = clock64();
  const double* X = lds + (t & 7);
  const double* Y = lds + 4096 + (t & 7);
  double acc = 0.0;
  long long c4 = clock64();
  if (t < 32) {
#pragma unroll 16
    for (int k = 0; k < 2048; k += 8) acc = fma(X[k], Y[k], acc);
  }
  long long c5 = clock64();
  if (t < 32) acc = batched<8>(X, Y, 256, acc);
  long long c6 = clock64();
  if (t < 32) acc = batched<16>(X, Y, 256, acc);
  long long c7 = clock64();
  if (t < 32) acc = ring<2>(X, Y, 256, acc);
  long long c8 = clock64();
  if (t < 32) acc = ring<4>(X, Y, 256, acc);
  long long c9 = clock64();
  const double2* X2 = reinterpret_cast<const double2*>(lds) + (t & 7);
  const double2* Y2 = reinterpret_cast<const double2*>(lds) + 2048 + (t & 7);
  long long c10 = clock64();
  if (t < 8) { double4 q = quad<4>(X2, Y2, 256); acc += q.x + q.y + q.z + q.w; }
  long long c11 = clock64();
  if (t < 8) { double4 q = quad<8>(X2, Y2, 256); acc += q.x + q.y + q.z + q.w; }
  long long c12 = clock64();
  out[t] = a + idx + acc;
  if (t == 0) {
    cyc[0] = c1 - c0; cyc[1] = w1 - w0; cyc[2] = c3 - c2; cyc[3] = c5 - c4;
    cyc[4] = c6 - c5; cyc[5] = c7 - c6; cyc[6] = c8 - c7; cyc[7] = c9 - c8;
    cyc[8] = c11 - c10; cyc[9] = c12 - c11;
  }
}

int main() {
  double* out; long long* cyc;
  (void)hipMalloc(&out, 64 * 8); (void)hipMemset(out, 0, 64 * 8);
  (void)hipMalloc(&cyc, 10 * 8);
  const int n = 4096;
  for (int rep = 0; rep < 3; ++rep) {
    hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, out, cyc, n);
    long long h[10];
    (void)hipMemcpy(h, cyc, sizeof(h), hipMemcpyDeviceToHost);
    printf("fma chain %.2f cyc/fma (clock %.2f GHz); LDS dep load %.1f cyc; LDS-fed chain cyc/step: "
           "plain %.1f  batch8 %.1f  batch16 %.1f  ring2 %.1f  ring4 %.1f  quad4 %.1f  quad8 %.1f\n",
           h[0] / (4.0 * n), h[0] / (h[1] * 10.0), h[2] / (4.0 * n), h[3] / 256.0, h[4] / 256.0,
           h[5] / 256.0, h[6] / 256.0, h[7] / 256.0, h[8] / 256.0, h[9] / 256.0);
  }
  return 0;
}
