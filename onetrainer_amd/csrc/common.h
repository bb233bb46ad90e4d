// Shared device helpers for the gfx950 (CDNA4) kernels of onetrainer_amd.
// Wave = 64 lanes; bf16 is stored as uint16_t in HBM and converted with the
// hardware RNE conversion (v_cvt_pk_bf16_f32) via __bf16 casts.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define OTAMD_API extern "C" __attribute__((visibility("default")))

// status codes returned by every C-ABI launcher (mapped to RuntimeError in Python)
enum {
  OTAMD_OK = 0,
  OTAMD_EINVAL = 1,     // shape / pointer / alignment contract violated
  OTAMD_ELAUNCH = 2,    // hipGetLastError after launch
  OTAMD_EUNSUPPORTED = 3
};

typedef uint16_t bf16_t;
typedef short short8 __attribute__((ext_vector_type(8)));
typedef short short4v __attribute__((ext_vector_type(4)));
typedef float float4v __attribute__((ext_vector_type(4)));
typedef float float16v __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float bf2f(bf16_t v) {
  return __uint_as_float(((uint32_t)v) << 16);
}
// round-to-nearest-even f32 -> bf16 (hardware cvt on gfx950, NaN-preserving)
__device__ __forceinline__ bf16_t f2bf(float f) {
  __bf16 b = (__bf16)f;
  return __builtin_bit_cast(bf16_t, b);
}
// round to bf16 and back (emulates one torch bf16 op's output rounding)
__device__ __forceinline__ float rbf(float f) { return bf2f(f2bf(f)); }

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}
__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// block-wide sum of one float; `red` must hold >= blockDim/64 floats
__device__ __forceinline__ float block_sum(float v, float* red) {
  v = wave_sum(v);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  __syncthreads();
  if (lane == 0) red[w] = v;
  __syncthreads();
  float t = 0.f;
  for (int i = 0; i < nw; ++i) t += red[i];
  return t;
}

// sigmoid through v_rcp_f32 (1 ulp) instead of an IEEE divide (~10 VALU ops): the GroupNorm(+SiLU)
// backward passes are VALU-bound on this per element
__device__ __forceinline__ float sigmoid_f(float x) { return __builtin_amdgcn_rcpf(1.f + __expf(-x)); }
__device__ __forceinline__ float silu_f(float x) { return x * sigmoid_f(x); }
__device__ __forceinline__ float dsilu_f(float x) {
  const float s = sigmoid_f(x);
  return s * (1.f + x * (1.f - s));
}
// exact (erf) GELU as torch.nn.functional.gelu(approximate='none').  erf(z), z = x / sqrt(2), by Abramowitz & Stegun
// 7.1.26 (|error| <= 1.5e-7, far below the bf16 rounding of every GELU output here): one v_rcp, one v_exp and five
// FMAs, against ~40 VALU ops of the library erff that left the GEGLU kernels VALU-bound at 3.3-3.5 TB/s.  The exp
// term e^{-z^2} = e^{-x^2/2} is also the normal pdf's, so the backward shares it.
struct GeluTerms { float cdf, pdf; };
__device__ __forceinline__ GeluTerms gelu_terms(float x) {
  const float z = fabsf(x) * 0.70710678118654752f;
  const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f, z, 1.f));
  const float poly =
      t * fmaf(t, fmaf(t, fmaf(t, fmaf(t, 1.061405429f, -1.453152027f), 1.421413741f), -0.284496736f), 0.254829592f);
  const float e = __expf(-z * z);
  const float tail = 0.5f * poly * e;   // 0.5 erfc(|z|): Phi(-|x|), taken directly (no 1 - erf cancellation)
  GeluTerms r;
  r.cdf = x < 0.f ? tail : 1.f - tail;
  r.pdf = 0.39894228040143268f * e;
  return r;
}
__device__ __forceinline__ float gelu_f(float x) { return x * gelu_terms(x).cdf; }
__device__ __forceinline__ float dgelu_f(float x) {
  const GeluTerms g = gelu_terms(x);
  return fmaf(x, g.pdf, g.cdf);
}

// 8 bf16 in one 16-byte register tuple
struct __align__(16) bf8 { uint32_t w[4]; };
// make the compiler treat v as freshly produced (no reuse of values derived from it before this point)
__device__ __forceinline__ void opaque(bf8& v) {
  asm volatile("" : "+v"(v.w[0]), "+v"(v.w[1]), "+v"(v.w[2]), "+v"(v.w[3]));
}
__device__ __forceinline__ void unpack8(const bf8& v, float* f) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    f[2 * i] = __uint_as_float(v.w[i] << 16);
    f[2 * i + 1] = __uint_as_float(v.w[i] & 0xffff0000u);
  }
}
__device__ __forceinline__ bf8 pack8(const float* f) {
  bf8 v;
#pragma unroll
  for (int i = 0; i < 4; ++i) v.w[i] = (uint32_t)f2bf(f[2 * i]) | ((uint32_t)f2bf(f[2 * i + 1]) << 16);
  return v;
}

static inline int ceil_div(long a, long b) { return (int)((a + b - 1) / b); }

#define OTAMD_CHECK_LAUNCH()                              \
  do {                                                    \
    if (hipGetLastError() != hipSuccess) return OTAMD_ELAUNCH; \
  } while (0)
