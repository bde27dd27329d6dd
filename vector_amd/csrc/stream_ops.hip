// Streaming element-wise kernels on either side of the chain:
//
//   mix_c64          apply_frequency_shift (utils.py:120-127): x * exp(j*theta),
//                    theta = (2*pi*f) * (i / sr) formed in double exactly as numpy
//                    forms it (once per lane), reduced mod 2*pi in double, sincos
//                    in fp32, lane-to-element steps from a rotation table
//   scale_c64        y = x * s (transplant_packet_in_vector's power scale,
//                    utils.py:1481-1496)
//   wv_quantize      SMU-WV int16 interleave of mat2wv
//                    (vector_analyzer/mat_to_wv_converter.py:28-50)
//   planar_to_c64    MAT v5 real / imaginary planes (any numeric storage type)
//                    -> interleaved complex64 (load_packet, utils.py:48-86)
//   c64_to_planar    complex64 -> float32 planes (save_vector, utils.py:659-670)
//
// All are HBM-bound grid-stride loops (8-16 B per element each way).
#include <hip/hip_runtime.h>

#include <cmath>
#include <type_traits>

#include "vsig_kernels.h"

namespace vsig {

static int ew_grid(long long n) {
  long long g = (n + 255) / 256;
  if (g > 8192) g = 8192;
  return g < 1 ? 1 : (int)g;
}

// ---------------------------------------------------------------- mixer
// One tile of 256 x 16 samples per block, sample base + t + 256 e in lane t:
// the lane forms numpy's phase once (sample base + t, mix_at's exact order),
// then rotates by exp(j w 256 e / sr) (host table in the kernel arguments,
// double -> fp32 once): a double division per lane instead of per sample,
// ~3e-7 relative per sample.
struct MixTile {
  float rot[32];   // (cos, sin) of w * 256 e / sr, e < 16, interleaved
};

__global__ __launch_bounds__(256) void mix_c64(const float2* __restrict__ x, long long n, double w,
                                               double sr, long long i0, float2* __restrict__ y,
                                               MixTile tab) {
  const long long base = (long long)blockIdx.x * 4096 + threadIdx.x;
  const float2 r0 = mix_at(make_float2(1.f, 0.f), i0 + base, w, sr);
  if (base + 15 * 256 < n) {
    float2 v[16];
#pragma unroll
    for (int e = 0; e < 16; ++e) v[e] = x[base + 256 * e];
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const float2 r = make_float2(r0.x * tab.rot[2 * e] - r0.y * tab.rot[2 * e + 1],
                                   r0.x * tab.rot[2 * e + 1] + r0.y * tab.rot[2 * e]);
      const float2 a = v[e];
      y[base + 256 * e] = make_float2(a.x * r.x - a.y * r.y, a.x * r.y + a.y * r.x);
    }
  } else {
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const long long i = base + 256 * e;
      if (i < n) {
        const float2 r = make_float2(r0.x * tab.rot[2 * e] - r0.y * tab.rot[2 * e + 1],
                                     r0.x * tab.rot[2 * e + 1] + r0.y * tab.rot[2 * e]);
        const float2 a = x[i];
        y[i] = make_float2(a.x * r.x - a.y * r.y, a.x * r.y + a.y * r.x);
      }
    }
  }
}

// ---------------------------------------------------------------- scale
__global__ __launch_bounds__(256) void scale_c64(const float2* __restrict__ x, long long n, float s,
                                                 float2* __restrict__ y) {
  const long long stride = (long long)gridDim.x * 256;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += stride) {
    const float2 v = x[i];
    y[i] = make_float2(v.x * s, v.y * s);
  }
}

// ------------------------------------------------ long FIR: delayed partial sums
// A filter of more than 8192 taps runs as parts h_j = h[8192 j, 8192 (j+1)),
// each an undecimated overlap-save FIR z_j = conv(x, h_j) over the whole
// buffer; y[k] (+)= z_j[off + k D] with off = nhist - 8192 j (zero where the
// index is negative: the delay reaches before the buffer).
__global__ __launch_bounds__(256) void fir_part_accum(const float2* __restrict__ z, long long nz,
                                                      long long off, int D, long long ny, int first,
                                                      float2* __restrict__ y) {
  const long long stride = (long long)gridDim.x * 256;
  for (long long k = (long long)blockIdx.x * 256 + threadIdx.x; k < ny; k += stride) {
    const long long i = off + k * D;
    const float2 v = (i >= 0 && i < nz) ? z[i] : make_float2(0.f, 0.f);
    if (first) {
      y[k] = v;
    } else {
      const float2 a = y[k];
      y[k] = make_float2(a.x + v.x, a.y + v.y);
    }
  }
}

// ---------------------------------------------------------------- SMU-WV
// numpy's float32 -> int16 cast on x86: truncate to int32 (out of range and
// NaN -> INT_MIN), keep the low 16 bits.
__device__ __forceinline__ short np_f32_to_i16(float f) {
  int v;
  if (!(f > -2147483648.f && f < 2147483648.f)) v = (int)0x80000000u;
  else v = (int)f;                                     // truncation toward zero
  return (short)(v & 0xffff);
}

// norm > 0: signal / norm first, then * 32767 in float32, as mat2wv does.
// numpy divides a complex64 by a real scalar with Smith's formula, which for
// a zero imaginary divisor is a multiply by the rounded reciprocal 1/norm.
__global__ __launch_bounds__(256) void wv_quantize(const float2* __restrict__ x, long long n, float norm,
                                                   short2* __restrict__ out) {
  const long long stride = (long long)gridDim.x * 256;
  const float rcp = norm > 0.f ? __fdiv_rn(1.f, norm) : 1.f;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += stride) {
    float2 v = x[i];
    if (norm > 0.f) v = make_float2(v.x * rcp, v.y * rcp);
    out[i] = make_short2(np_f32_to_i16(v.x * 32767.f), np_f32_to_i16(v.y * 32767.f));
  }
}

// ---------------------------------------------------------------- MAT planes
template <class T>
__global__ __launch_bounds__(256) void planar_to_c64(const T* __restrict__ re, const T* __restrict__ im,
                                                     long long n, float2* __restrict__ y) {
  const long long stride = (long long)gridDim.x * 256;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += stride)
    y[i] = make_float2((float)re[i], im ? (float)im[i] : 0.f);
}

__global__ __launch_bounds__(256) void c64_to_planar(const float2* __restrict__ x, long long n,
                                                     float* __restrict__ re, float* __restrict__ im) {
  const long long stride = (long long)gridDim.x * 256;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += stride) {
    const float2 v = x[i];
    re[i] = v.x;
    im[i] = v.y;
  }
}

// ---------------------------------------------------------------- launchers
hipError_t launch_mix_c64(const float2* x, long long n, double w, double sr, long long i0, float2* y,
                          hipStream_t st) {
  MixTile tab;
  for (int e = 0; e < 16; ++e) {       // w * 256 e / sr reduced mod 2 pi in double
    const double a = std::remainder(w * (256.0 * e) / sr, 2.0 * M_PI);
    tab.rot[2 * e] = (float)std::cos(a);
    tab.rot[2 * e + 1] = (float)std::sin(a);
  }
  const long long g = (n + 4095) / 4096;
  hipLaunchKernelGGL(mix_c64, dim3((unsigned)g), dim3(256), 0, st, x, n, w, sr, i0, y, tab);
  return hipGetLastError();
}

hipError_t launch_scale_c64(const float2* x, long long n, float s, float2* y, hipStream_t st) {
  hipLaunchKernelGGL(scale_c64, dim3(ew_grid(n)), dim3(256), 0, st, x, n, s, y);
  return hipGetLastError();
}

hipError_t launch_fir_part_accum(const float2* z, long long nz, long long off, int D, long long ny,
                                 int first, float2* y, hipStream_t st) {
  hipLaunchKernelGGL(fir_part_accum, dim3(ew_grid(ny)), dim3(256), 0, st, z, nz, off, D, ny, first, y);
  return hipGetLastError();
}

hipError_t launch_wv_quantize(const float2* x, long long n, float norm, short* out, hipStream_t st) {
  hipLaunchKernelGGL(wv_quantize, dim3(ew_grid(n)), dim3(256), 0, st, x, n, norm, (short2*)out);
  return hipGetLastError();
}

// MAT v5 storage types (miINT8 = 1 ... miDOUBLE = 9)
hipError_t launch_planar_to_c64(int mi_type, const void* re, const void* im, long long n, float2* y,
                                hipStream_t st) {
  const int g = ew_grid(n);
#define VSIG_PLANES(T)                                                                          \
  hipLaunchKernelGGL(planar_to_c64<T>, dim3(g), dim3(256), 0, st, (const T*)re, (const T*)im, n, y); \
  break;
  switch (mi_type) {
    case 1: VSIG_PLANES(signed char)
    case 2: VSIG_PLANES(unsigned char)
    case 3: VSIG_PLANES(short)
    case 4: VSIG_PLANES(unsigned short)
    case 5: VSIG_PLANES(int)
    case 6: VSIG_PLANES(unsigned int)
    case 7: VSIG_PLANES(float)
    case 9: VSIG_PLANES(double)
    case 12: VSIG_PLANES(long long)
    case 13: VSIG_PLANES(unsigned long long)
    default: return hipErrorInvalidValue;
  }
#undef VSIG_PLANES
  return hipGetLastError();
}

hipError_t launch_c64_to_planar(const float2* x, long long n, float* re, float* im, hipStream_t st) {
  hipLaunchKernelGGL(c64_to_planar, dim3(ew_grid(n)), dim3(256), 0, st, x, n, re, im);
  return hipGetLastError();
}

}  // namespace vsig

#ifdef VSIG_TUNING
namespace vsig {

// ---------------------------------------------------------------- copy probe
// HBM ceiling probe for the tuning tools (tools/membw.py): copy n complex64
// with 8-B (float2) or 16-B (float4) lanes, plain or non-temporal stores.
template <int W, bool NT>
__global__ __launch_bounds__(256) void copy_probe(const float2* __restrict__ x, long long n,
                                                  float2* __restrict__ y) {
  const long long stride = (long long)gridDim.x * 256;
  typedef float v4 __attribute__((ext_vector_type(4)));
  typedef float v2 __attribute__((ext_vector_type(2)));
  if constexpr (W == 16) {
    const v4* x4 = reinterpret_cast<const v4*>(x);
    v4* y4 = reinterpret_cast<v4*>(y);
    for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n / 2; i += stride) {
      const v4 v = x4[i];
      if constexpr (NT) __builtin_nontemporal_store(v, y4 + i);
      else y4[i] = v;
    }
  } else {
    const v2* x2 = reinterpret_cast<const v2*>(x);
    v2* y2 = reinterpret_cast<v2*>(y);
    for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += stride) {
      const v2 v = x2[i];
      if constexpr (NT) __builtin_nontemporal_store(v, y2 + i);
      else y2[i] = v;
    }
  }
}

// Unrolled form: each thread moves U consecutive float4 per iteration with all
// U loads issued before the first store (U * 16 B in flight per lane), loads
// and/or stores non-temporal; block-contiguous chunks (no grid stride).
typedef float f4v __attribute__((ext_vector_type(4)));
typedef float f2v __attribute__((ext_vector_type(2)));
template <int U, bool NTL, bool NTS, class V = f4v>
__global__ __launch_bounds__(256) void copy_probe_u(const V* __restrict__ x, long long n4,
                                                    V* __restrict__ y) {
  const long long base = ((long long)blockIdx.x * 256) * U + threadIdx.x;
  V v[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const long long i = base + (long long)u * 256;
    if (i < n4) v[u] = NTL ? __builtin_nontemporal_load(x + i) : x[i];
  }
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const long long i = base + (long long)u * 256;
    if (i < n4) {
      if constexpr (NTS) __builtin_nontemporal_store(v[u], y + i);
      else y[i] = v[u];
    }
  }
}

// Read-mostly form (the D = 4 FIR's 4:1 pattern without its overlap): each
// thread loads U float4 (2U samples), writes one float2 per 4 samples.
template <int U, bool NTL>
__global__ __launch_bounds__(256) void reduce4_probe(const f4v* __restrict__ x, long long n4,
                                                     f2v* __restrict__ y) {
  const long long base = ((long long)blockIdx.x * 256) * U + threadIdx.x;
  f4v v[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const long long i = base + (long long)u * 256;
    v[u] = i < n4 ? (NTL ? __builtin_nontemporal_load(x + i) : x[i]) : f4v{0, 0, 0, 0};
  }
#pragma unroll
  for (int u = 0; u < U; u += 2) {
    const long long i = ((long long)blockIdx.x * 256) * (U / 2) + threadIdx.x + (long long)(u / 2) * 256;
    const f4v s = v[u] + v[u + 1];
    if (i < n4 / 2) y[i] = f2v{s.x + s.z, s.y + s.w};
  }
}

// The same 4:1 pattern with the loads as LDS-DMA (global_load_lds_dwordx4:
// each wave-instruction lands 1 KB in the wave's LDS slice, no VGPR
// destination), read back with ds_read_b128 once the wave's DMAs are done.
// AUX 2: the non-temporal policy.
template <int U, int AUX>
__global__ __launch_bounds__(256) void reduce4_glds_probe(const f4v* __restrict__ x, long long n4,
                                                          f2v* __restrict__ y) {
  __shared__ __attribute__((aligned(16))) f4v slab[4][U][64];
  const int t = threadIdx.x, w = t >> 6, l = t & 63;
  const long long base = ((long long)blockIdx.x * 256) * U + 64LL * U * w;   // the wave's rows
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const long long i = base + 64LL * u + l;
    const f4v* src = x + (i < n4 ? i : n4 - 1);
#if defined(__HIP_DEVICE_COMPILE__)   // a device builtin: the host pass only needs the stub
    __builtin_amdgcn_global_load_lds(src, &slab[w][u][0], 16, 0, AUX);
#else
    (void)src;
#endif
  }
  __builtin_amdgcn_s_waitcnt(0x3f70);   // vmcnt(0): the wave's DMAs have landed (gfx9 encoding)
  f4v v[U];
#pragma unroll
  for (int u = 0; u < U; ++u) v[u] = slab[w][u][l];
#pragma unroll
  for (int u = 0; u < U; u += 2) {
    const long long i = ((long long)blockIdx.x * 256) * (U / 2) + 64LL * (U / 2) * w + 64LL * (u / 2) + l;
    const f4v s = v[u] + v[u + 1];
    if (i < n4 / 2) y[i] = f2v{s.x + s.z, s.y + s.w};
  }
}

// The 4:1 read-mostly pattern with the load width, the unroll and both
// non-temporal policies free (variants 50..): lanes of W bytes (8: float2,
// 16: float4), U loads in flight per lane, one float2 store per 4 samples.
template <int W, int U, bool NTL, bool NTS>
__global__ __launch_bounds__(256) void reduce4w_probe(const float2* __restrict__ x, long long n,
                                                      f2v* __restrict__ y) {
  constexpr int S = W / 8;                        // samples per lane per load
  typedef typename std::conditional<W == 16, f4v, f2v>::type V;
  const V* xv = reinterpret_cast<const V*>(x);
  const long long nv = n / S;
  const long long base = ((long long)blockIdx.x * 256) * U + threadIdx.x;
  V v[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const long long i = base + (long long)u * 256;
    v[u] = i < nv ? (NTL ? __builtin_nontemporal_load(xv + i) : xv[i]) : V{};
  }
  constexpr int G = 4 / S;                        // loads per output
#pragma unroll
  for (int u = 0; u < U; u += G) {
    f2v s = {0.f, 0.f};
#pragma unroll
    for (int q = 0; q < G; ++q) {
      if constexpr (W == 16) s += f2v{v[u + q].x + v[u + q].z, v[u + q].y + v[u + q].w};
      else s += v[u + q];
    }
    const long long i = ((long long)blockIdx.x * 256) * (U / G) + threadIdx.x + (long long)(u / G) * 256;
    if (i < n / 4) {
      if constexpr (NTS) __builtin_nontemporal_store(s, y + i);
      else y[i] = s;
    }
  }
}

hipError_t launch_copy_probe(const float2* x, long long n, float2* y, int variant, int grid,
                             hipStream_t st) {
  if (variant >= 50 && variant < 74) {   // 50 + wi*12 + ui*4 + NTL*2 + NTS; W = 8 (U 4, 8, 16) / 16 (U 2, 4, 8)
    const int k = variant - 50, wi = k / 12, ui = (k % 12) / 4, ntl = (k >> 1) & 1, nts = k & 1;
    const int U = wi == 0 ? (4 << ui) : (2 << ui);
    const long long per = 256LL * U * (wi == 0 ? 1 : 2);
    const dim3 g((unsigned)((n + per - 1) / per)), b(256);
    f2v* y2 = reinterpret_cast<f2v*>(y);
#define VSIG_RW_(WW, UU)                                                                           \
    if (ntl && nts) hipLaunchKernelGGL((reduce4w_probe<WW, UU, true, true>), g, b, 0, st, x, n, y2);   \
    else if (ntl) hipLaunchKernelGGL((reduce4w_probe<WW, UU, true, false>), g, b, 0, st, x, n, y2);    \
    else if (nts) hipLaunchKernelGGL((reduce4w_probe<WW, UU, false, true>), g, b, 0, st, x, n, y2);    \
    else hipLaunchKernelGGL((reduce4w_probe<WW, UU, false, false>), g, b, 0, st, x, n, y2);
    if (wi == 0) {
      if (U == 4) { VSIG_RW_(8, 4) } else if (U == 8) { VSIG_RW_(8, 8) } else { VSIG_RW_(8, 16) }
    } else {
      if (U == 2) { VSIG_RW_(16, 2) } else if (U == 4) { VSIG_RW_(16, 4) } else { VSIG_RW_(16, 8) }
    }
#undef VSIG_RW_
    return hipGetLastError();
  }
  if (variant >= 40) {      // LDS-DMA read-mostly probes: 40 + (U index)*2 + NT, U = 2, 4, 8
    const int ui = (variant - 40) / 2, nt = variant & 1;
    const long long n4 = n / 2;
    const int U = ui == 0 ? 2 : ui == 1 ? 4 : 8;
    const dim3 g((unsigned)((n4 + 256LL * U - 1) / (256LL * U))), b(256);
    const f4v* x4 = reinterpret_cast<const f4v*>(x);
    f2v* y2 = reinterpret_cast<f2v*>(y);
#define VSIG_RG_(UU)                                                                       \
    if (nt) hipLaunchKernelGGL((reduce4_glds_probe<UU, 2>), g, b, 0, st, x4, n4, y2);        \
    else hipLaunchKernelGGL((reduce4_glds_probe<UU, 0>), g, b, 0, st, x4, n4, y2);
    if (U == 2) { VSIG_RG_(2) } else if (U == 4) { VSIG_RG_(4) } else { VSIG_RG_(8) }
#undef VSIG_RG_
    return hipGetLastError();
  }
  if (variant >= 28) {      // read-mostly probes: 28 + (U index)*2 + NTL, U = 2, 4, 8
    const int ui = (variant - 28) / 2, ntl = variant & 1;
    const long long n4 = n / 2;
    const int U = ui == 0 ? 2 : ui == 1 ? 4 : 8;
    const dim3 g((unsigned)((n4 + 256LL * U - 1) / (256LL * U))), b(256);
    const f4v* x4 = reinterpret_cast<const f4v*>(x);
    f2v* y2 = reinterpret_cast<f2v*>(y);
#define VSIG_R4_(UU)                                                                  \
    if (ntl) hipLaunchKernelGGL((reduce4_probe<UU, true>), g, b, 0, st, x4, n4, y2);    \
    else hipLaunchKernelGGL((reduce4_probe<UU, false>), g, b, 0, st, x4, n4, y2);
    if (U == 2) { VSIG_R4_(2) } else if (U == 4) { VSIG_R4_(4) } else { VSIG_R4_(8) }
#undef VSIG_R4_
    return hipGetLastError();
  }
  if (variant >= 16) {      // unrolled 8-B probes: 16 + (U index)*4 + NTL*2 + NTS
    const int ui = (variant - 16) / 4, ntl = (variant >> 1) & 1, nts = variant & 1;
    const int U = ui == 0 ? 4 : ui == 1 ? 8 : 16;
    const dim3 g((unsigned)((n + 256LL * U - 1) / (256LL * U))), b(256);
    const f2v* x2 = reinterpret_cast<const f2v*>(x);
    f2v* y2 = reinterpret_cast<f2v*>(y);
#define VSIG_CP8_(UU)                                                                              \
    if (ntl && nts) hipLaunchKernelGGL((copy_probe_u<UU, true, true, f2v>), g, b, 0, st, x2, n, y2);  \
    else if (ntl) hipLaunchKernelGGL((copy_probe_u<UU, true, false, f2v>), g, b, 0, st, x2, n, y2);   \
    else if (nts) hipLaunchKernelGGL((copy_probe_u<UU, false, true, f2v>), g, b, 0, st, x2, n, y2);   \
    else hipLaunchKernelGGL((copy_probe_u<UU, false, false, f2v>), g, b, 0, st, x2, n, y2);
    if (U == 4) { VSIG_CP8_(4) } else if (U == 8) { VSIG_CP8_(8) } else { VSIG_CP8_(16) }
#undef VSIG_CP8_
    return hipGetLastError();
  }
  if (variant >= 4) {       // unrolled probes: 4 + (U index)*4 + NTL*2 + NTS
    const long long n4 = n / 2;
    const int ui = (variant - 4) / 4, ntl = (variant >> 1) & 1, nts = variant & 1;
    const int U = ui == 0 ? 2 : ui == 1 ? 4 : 8;
    const dim3 g((unsigned)((n4 + 256LL * U - 1) / (256LL * U))), b(256);
    const f4v* x4 = reinterpret_cast<const f4v*>(x);
    f4v* y4 = reinterpret_cast<f4v*>(y);
#define VSIG_CPU_(UU)                                                                   \
    if (ntl && nts) hipLaunchKernelGGL((copy_probe_u<UU, true, true>), g, b, 0, st, x4, n4, y4);  \
    else if (ntl) hipLaunchKernelGGL((copy_probe_u<UU, true, false>), g, b, 0, st, x4, n4, y4);   \
    else if (nts) hipLaunchKernelGGL((copy_probe_u<UU, false, true>), g, b, 0, st, x4, n4, y4);   \
    else hipLaunchKernelGGL((copy_probe_u<UU, false, false>), g, b, 0, st, x4, n4, y4);
    if (U == 2) { VSIG_CPU_(2) } else if (U == 4) { VSIG_CPU_(4) } else { VSIG_CPU_(8) }
#undef VSIG_CPU_
    (void)grid;
    return hipGetLastError();
  }
  const dim3 g(grid > 0 ? grid : 8192), b(256);
  switch (variant) {
    case 0: hipLaunchKernelGGL((copy_probe<8, false>), g, b, 0, st, x, n, y); break;
    case 1: hipLaunchKernelGGL((copy_probe<8, true>), g, b, 0, st, x, n, y); break;
    case 2: hipLaunchKernelGGL((copy_probe<16, false>), g, b, 0, st, x, n, y); break;
    case 3: hipLaunchKernelGGL((copy_probe<16, true>), g, b, 0, st, x, n, y); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}
}  // namespace vsig
#endif  // VSIG_TUNING
