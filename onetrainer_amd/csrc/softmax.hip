// Row softmax forward / backward for the materialized attention path.
//
// The flash kernels (attention.hip) cover head dims <= 128.  Heads wider than that -- SD 1.5's
// 160-wide heads at its 1280-channel level (v1-inference.yaml:29-44: 8 heads at every level)
// and the VAE mid-block's single 512-wide head (AutoencoderKL, reached from
// StableDiffusionXLBaseDataLoader.py:65-100 EncodeVAE) -- run as S = Q K^T (batched MFMA GEMM,
// fp32 out) -> P = softmax(scale S) (this file, bf16 out) -> O = P V (batched GEMM), and the
// backward as dP = dO V^T -> dS = scale P (dP - rowsum(P dP)) (this file) -> dQ, dK, dV GEMMs.
// Both kernels are HBM-bound: fwd reads S twice (4+4 B) and writes P (2 B) per element; bwd
// reads P and dP twice (2+4 per pass) and writes dS (2 B).
//
// One wave per row, 4 rows per 256-thread block; lanes stride the row in float4 chunks.
// Columns [ncols, ncols_pad) are written as exact zeros (keys padded to a multiple of 8 so the
// P / dS rows stay 16-byte aligned GEMM operands).
#include "common.h"

__device__ __forceinline__ void load4(const float* p, int c, int ncols, float (&x)[4]) {
  if (c + 3 < ncols) {
    const float4 v = *reinterpret_cast<const float4*>(p + c);
    x[0] = v.x; x[1] = v.y; x[2] = v.z; x[3] = v.w;
  } else {
#pragma unroll
    for (int j = 0; j < 4; ++j) x[j] = (c + j < ncols) ? p[c + j] : 0.f;
  }
}
__device__ __forceinline__ void load4bf(const bf16_t* p, int c, int ncols, float (&x)[4]) {
  if (c + 3 < ncols) {
    const uint2 v = *reinterpret_cast<const uint2*>(p + c);
    x[0] = __uint_as_float(v.x << 16); x[1] = __uint_as_float(v.x & 0xffff0000u);
    x[2] = __uint_as_float(v.y << 16); x[3] = __uint_as_float(v.y & 0xffff0000u);
  } else {
#pragma unroll
    for (int j = 0; j < 4; ++j) x[j] = (c + j < ncols) ? bf2f(p[c + j]) : 0.f;
  }
}
__device__ __forceinline__ void store4bf(bf16_t* p, int c, const float (&y)[4]) {
  uint2 o;
  o.x = (uint32_t)f2bf(y[0]) | ((uint32_t)f2bf(y[1]) << 16);
  o.y = (uint32_t)f2bf(y[2]) | ((uint32_t)f2bf(y[3]) << 16);
  *reinterpret_cast<uint2*>(p + c) = o;
}

// P[r, c] = exp(scale S[r, c] - m_r) / l_r; lse[r] = m_r + ln l_r (natural log)
__global__ void __launch_bounds__(256) softmax_rows_fwd_kernel(const float* __restrict__ S, long long lds,
                                                               bf16_t* __restrict__ P, long long ldp,
                                                               float* __restrict__ lse, long long rows, int ncols,
                                                               int ncols_pad, float scale) {
  const int lane = threadIdx.x & 63;
  for (long long r = (long long)blockIdx.x * 4 + (threadIdx.x >> 6); r < rows; r += (long long)gridDim.x * 4) {
    const float* s = S + r * lds;
    float m = -INFINITY, l = 0.f;
    for (int c = lane * 4; c < ncols; c += 256) {
      float x[4];
      load4(s, c, ncols, x);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if (c + j >= ncols) continue;
        const float v = x[j] * scale;
        if (v > m) { l = l * __expf(m - v) + 1.f; m = v; }
        else l += __expf(v - m);
      }
    }
    const float M = wave_max(m);
    l = (m == -INFINITY) ? 0.f : l * __expf(m - M);
    const float L = wave_sum(l);
    const float inv = 1.f / L;
    bf16_t* p = P + r * ldp;
    for (int c = lane * 4; c < ncols_pad; c += 256) {
      float x[4], y[4];
      load4(s, c, ncols, x);
#pragma unroll
      for (int j = 0; j < 4; ++j) y[j] = (c + j < ncols) ? __expf(x[j] * scale - M) * inv : 0.f;
      store4bf(p, c, y);
    }
    if (lane == 0 && lse) lse[r] = M + __logf(L);
  }
}

// dS[r, c] = scale * P[r, c] * (dP[r, c] - sum_c' P[r, c'] dP[r, c'])
__global__ void __launch_bounds__(256) softmax_rows_bwd_kernel(const bf16_t* __restrict__ P, long long ldp,
                                                               const float* __restrict__ dP, long long lddp,
                                                               bf16_t* __restrict__ dS, long long ldds, long long rows,
                                                               int ncols, int ncols_pad, float scale) {
  const int lane = threadIdx.x & 63;
  for (long long r = (long long)blockIdx.x * 4 + (threadIdx.x >> 6); r < rows; r += (long long)gridDim.x * 4) {
    const bf16_t* p = P + r * ldp;
    const float* g = dP + r * lddp;
    float dot = 0.f;
    for (int c = lane * 4; c < ncols; c += 256) {
      float x[4], y[4];
      load4bf(p, c, ncols, x);
      load4(g, c, ncols, y);
#pragma unroll
      for (int j = 0; j < 4; ++j) dot = fmaf(x[j], y[j], dot);
    }
    dot = wave_sum(dot);
    bf16_t* d = dS + r * ldds;
    for (int c = lane * 4; c < ncols_pad; c += 256) {
      float x[4], y[4], o[4];
      load4bf(p, c, ncols, x);
      load4(g, c, ncols, y);
#pragma unroll
      for (int j = 0; j < 4; ++j) o[j] = (c + j < ncols) ? scale * x[j] * (y[j] - dot) : 0.f;
      store4bf(d, c, o);
    }
  }
}

static int rows_grid(long long rows) { return (int)std::min<long long>((rows + 3) / 4, 65536); }

OTAMD_API int otamd_softmax_rows_fwd(const float* S, long long lds, bf16_t* P, long long ldp, float* lse,
                                     long long rows, int ncols, int ncols_pad, float scale, hipStream_t stream) {
  if (!S || !P || rows <= 0 || ncols <= 0 || ncols_pad < ncols || ncols_pad % 4 || lds % 4 || ldp % 4 ||
      lds < ncols || ldp < ncols_pad || ((uintptr_t)S & 15) || ((uintptr_t)P & 7))
    return OTAMD_EINVAL;
  softmax_rows_fwd_kernel<<<rows_grid(rows), 256, 0, stream>>>(S, lds, P, ldp, lse, rows, ncols, ncols_pad, scale);
  OTAMD_CHECK_LAUNCH();
  return OTAMD_OK;
}

OTAMD_API int otamd_softmax_rows_bwd(const bf16_t* P, long long ldp, const float* dP, long long lddp, bf16_t* dS,
                                     long long ldds, long long rows, int ncols, int ncols_pad, float scale,
                                     hipStream_t stream) {
  if (!P || !dP || !dS || rows <= 0 || ncols <= 0 || ncols_pad < ncols || ncols_pad % 4 || ldp % 4 || lddp % 4 ||
      ldds % 4 || ldp < ncols || lddp < ncols || ldds < ncols_pad || ((uintptr_t)P & 7) || ((uintptr_t)dP & 15) ||
      ((uintptr_t)dS & 7))
    return OTAMD_EINVAL;
  softmax_rows_bwd_kernel<<<rows_grid(rows), 256, 0, stream>>>(P, ldp, dP, lddp, dS, ldds, rows, ncols, ncols_pad,
                                                               scale);
  OTAMD_CHECK_LAUNCH();
  return OTAMD_OK;
}
