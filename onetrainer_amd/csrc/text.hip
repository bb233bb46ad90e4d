// Text-encoder caching kernels: the CLIP-L / CLIP-bigG text transformers of
// SD 1.5 / SDXL and the T5 encoder of FLUX.1, run forward-only when text states are cached
// (modules/model/StableDiffusionXLModel.py:199-286 encode_text -> model/util/clip_util.py:6-43
// encode_clip, modules/model/util/t5_util.py encode_t5).  The projections, residual adds and layer
// norms reuse the GEMM / LayerNorm engines; this file holds what those lack:
//   * token (+ position) embedding gather,
//   * the MLP activations (quick_gelu for CLIP-L, erf GELU for bigG) and T5's gated tanh-GELU,
//   * T5's RMS LayerNorm (T5LayerNorm: fp32 mean square, no mean subtraction, no bias),
//   * row softmax with CLIP's causal mask and/or T5's additive relative-position bias.
// All are HBM-bound elementwise / row kernels over [tokens, channels] bf16 rows.
#include "common.h"

// out[r, :] = tok[clamp(ids[r])] (+ pos[r % T]); one 16-byte chunk per thread
__global__ void embed_tokens_kernel(const long long* __restrict__ ids, long long n, int T,
                                    const bf16_t* __restrict__ tok, const bf16_t* __restrict__ pos,
                                    bf16_t* __restrict__ out, int D, int vocab) {
  const int D8 = D >> 3;
  const long long total = n * D8;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total; i += (long long)gridDim.x * blockDim.x) {
    const long long r = i / D8;
    const int c8 = (int)(i - r * D8);
    long long id = ids[r];
    id = id < 0 ? 0 : (id >= vocab ? vocab - 1 : id);   // an out-of-range id must not fault the device
    float v[8];
    unpack8(*reinterpret_cast<const bf8*>(tok + id * D + c8 * 8), v);
    if (pos) {
      float p[8];
      unpack8(*reinterpret_cast<const bf8*>(pos + (long long)(r % T) * D + c8 * 8), p);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] += p[j];
    }
    *reinterpret_cast<bf8*>(out + r * D + c8 * 8) = pack8(v);
  }
}

enum { ACT_QUICK_GELU = 0, ACT_GELU_ERF = 1, ACT_GELU_TANH = 2 };

__device__ __forceinline__ float act_f(float x, int kind) {
  if (kind == ACT_QUICK_GELU) return x / (1.f + __expf(-1.702f * x));
  if (kind == ACT_GELU_ERF) return 0.5f * x * (1.f + erff(x * 0.70710678118654752f));
  const float u = 0.7978845608028654f * (x + 0.044715f * x * x * x);
  return 0.5f * x * (1.f + tanhf(u));
}

// y = act(x) over [rows, C] (strided rows, C % 8 == 0); in place allowed
__global__ void act_kernel(const bf16_t* __restrict__ x, long long ldx, bf16_t* __restrict__ y, long long ldy,
                           long long rows, int C, int kind) {
  const int C8 = C >> 3;
  const long long total = rows * C8;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total; i += (long long)gridDim.x * blockDim.x) {
    const long long r = i / C8;
    const int c = (int)(i - r * C8) * 8;
    float v[8];
    unpack8(*reinterpret_cast<const bf8*>(x + r * ldx + c), v);
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = act_f(v[j], kind);
    *reinterpret_cast<bf8*>(y + r * ldy + c) = pack8(v);
  }
}

// out[r, c] = act(h[r, c]) * h[r, F + c]  (T5 DenseGatedActDense: wi_0 | wi_1 fused, gelu_new on wi_0)
__global__ void gated_act_kernel(const bf16_t* __restrict__ h, long long ldh, bf16_t* __restrict__ out, long long ldo,
                                 long long rows, int F, int kind) {
  const int F8 = F >> 3;
  const long long total = rows * F8;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total; i += (long long)gridDim.x * blockDim.x) {
    const long long r = i / F8;
    const int c = (int)(i - r * F8) * 8;
    float a[8], g[8];
    unpack8(*reinterpret_cast<const bf8*>(h + r * ldh + c), a);
    unpack8(*reinterpret_cast<const bf8*>(h + r * ldh + F + c), g);
#pragma unroll
    for (int j = 0; j < 8; ++j) a[j] = act_f(a[j], kind) * g[j];
    *reinterpret_cast<bf8*>(out + r * ldo + c) = pack8(a);
  }
}

// T5LayerNorm: y = bf16(x * rsqrt(mean(x^2) + eps)) * w  (fp32 statistics; the reference casts the
// normalised value to the weight dtype before the scale).  One wave per row.
__global__ void __launch_bounds__(256) rmsnorm_kernel(const bf16_t* __restrict__ x, long long ldx, bf16_t* __restrict__ y,
                                                      long long ldy, long long rows, int C, float eps,
                                                      const bf16_t* __restrict__ w) {
  const int lane = threadIdx.x & 63;
  for (long long r = (long long)blockIdx.x * 4 + (threadIdx.x >> 6); r < rows; r += (long long)gridDim.x * 4) {
    const bf16_t* xr = x + r * ldx;
    float q = 0.f;
    for (int c = lane * 8; c < C; c += 512) {
      float v[8];
      unpack8(*reinterpret_cast<const bf8*>(xr + c), v);
#pragma unroll
      for (int j = 0; j < 8; ++j) q = fmaf(v[j], v[j], q);
    }
    const float rs = rsqrtf(wave_sum(q) / C + eps);
    for (int c = lane * 8; c < C; c += 512) {
      float v[8], g[8];
      unpack8(*reinterpret_cast<const bf8*>(xr + c), v);
      unpack8(*reinterpret_cast<const bf8*>(w + c), g);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = bf2f(f2bf(v[j] * rs)) * g[j];
      *reinterpret_cast<bf8*>(y + r * ldy + c) = pack8(v);
    }
  }
}

// P = softmax(scale S + bias) with an optional causal mask, rows r = (b H + h) Nq + q:
//   causal: column c > q is masked (CLIP's causal attention mask);
//   bias:   bf16 bias[q * bsq + c * bsc + h * bsh] added after scaling (T5 relative position bias).
// Columns [ncols, ncols_pad) are written as zeros (padded keys).
__global__ void __launch_bounds__(256) softmax_masked_kernel(const float* __restrict__ S, long long lds,
                                                             bf16_t* __restrict__ P, long long ldp, long long rows,
                                                             int ncols, int ncols_pad, float scale, int Nq, int H,
                                                             int causal, const bf16_t* __restrict__ bias,
                                                             long long bsq, long long bsc, long long bsh) {
  const int lane = threadIdx.x & 63;
  for (long long r = (long long)blockIdx.x * 4 + (threadIdx.x >> 6); r < rows; r += (long long)gridDim.x * 4) {
    const int q = (int)(r % Nq);
    const int h = (int)((r / Nq) % H);
    const float* s = S + r * lds;
    const int lim = causal ? min(ncols, q + 1) : ncols;
    auto val = [&](int c) {
      float v = s[c] * scale;
      if (bias) v += bf2f(bias[q * bsq + c * bsc + h * bsh]);
      return v;
    };
    float m = -INFINITY;
    for (int c = lane; c < lim; c += 64) m = fmaxf(m, val(c));
    const float M = wave_max(m);
    float l = 0.f;
    for (int c = lane; c < lim; c += 64) l += __expf(val(c) - M);
    const float inv = 1.f / wave_sum(l);
    bf16_t* p = P + r * ldp;
    for (int c = lane; c < ncols_pad; c += 64) p[c] = f2bf(c < lim ? __expf(val(c) - M) * inv : 0.f);
  }
}

static int grid_for(long long work, int per_block) {
  return (int)std::min<long long>((work + per_block - 1) / per_block, 16384);
}

OTAMD_API int otamd_embed_tokens(const long long* ids, long long n, int T, const void* tok, const void* pos, void* out,
                                 int D, int vocab, hipStream_t stream) {
  if (!ids || !tok || !out || n <= 0 || T <= 0 || D <= 0 || D % 8 || vocab <= 0) return OTAMD_EINVAL;
  if (((uintptr_t)tok | (uintptr_t)pos | (uintptr_t)out) & 15) return OTAMD_EINVAL;
  embed_tokens_kernel<<<grid_for(n * (D / 8), 256), 256, 0, stream>>>(ids, n, T, (const bf16_t*)tok,
                                                                       (const bf16_t*)pos, (bf16_t*)out, D, vocab);
  OTAMD_CHECK_LAUNCH();
  return OTAMD_OK;
}

OTAMD_API int otamd_act_fwd(const void* x, long long ldx, void* y, long long ldy, long long rows, int C, int kind,
                            hipStream_t stream) {
  if (!x || !y || rows <= 0 || C <= 0 || C % 8 || ldx % 8 || ldy % 8 || kind < 0 || kind > 2) return OTAMD_EINVAL;
  if (((uintptr_t)x | (uintptr_t)y) & 15) return OTAMD_EINVAL;
  act_kernel<<<grid_for(rows * (C / 8), 256), 256, 0, stream>>>((const bf16_t*)x, ldx, (bf16_t*)y, ldy, rows, C, kind);
  OTAMD_CHECK_LAUNCH();
  return OTAMD_OK;
}

OTAMD_API int otamd_gated_act_fwd(const void* h, long long ldh, void* out, long long ldo, long long rows, int F,
                                  int kind, hipStream_t stream) {
  if (!h || !out || rows <= 0 || F <= 0 || F % 8 || ldh % 8 || ldo % 8 || ldh < 2 * F || kind < 0 || kind > 2)
    return OTAMD_EINVAL;
  if (((uintptr_t)h | (uintptr_t)out) & 15) return OTAMD_EINVAL;
  gated_act_kernel<<<grid_for(rows * (F / 8), 256), 256, 0, stream>>>((const bf16_t*)h, ldh, (bf16_t*)out, ldo, rows,
                                                                       F, kind);
  OTAMD_CHECK_LAUNCH();
  return OTAMD_OK;
}

OTAMD_API int otamd_rmsnorm_fwd(const void* x, long long ldx, void* y, long long ldy, long long rows, int C, float eps,
                                const void* w, hipStream_t stream) {
  if (!x || !y || !w || rows <= 0 || C <= 0 || C % 8 || ldx % 8 || ldy % 8) return OTAMD_EINVAL;
  if (((uintptr_t)x | (uintptr_t)y | (uintptr_t)w) & 15) return OTAMD_EINVAL;
  rmsnorm_kernel<<<grid_for(rows, 4), 256, 0, stream>>>((const bf16_t*)x, ldx, (bf16_t*)y, ldy, rows, C, eps,
                                                        (const bf16_t*)w);
  OTAMD_CHECK_LAUNCH();
  return OTAMD_OK;
}

OTAMD_API int otamd_softmax_masked_fwd(const float* S, long long lds, void* P, long long ldp, long long rows, int ncols,
                                       int ncols_pad, float scale, int Nq, int H, int causal, const void* bias,
                                       long long bsq, long long bsc, long long bsh, hipStream_t stream) {
  if (!S || !P || rows <= 0 || ncols <= 0 || ncols_pad < ncols || lds < ncols || ldp < ncols_pad || Nq <= 0 ||
      H <= 0 || rows % ((long long)Nq * H))
    return OTAMD_EINVAL;
  softmax_masked_kernel<<<grid_for(rows, 4), 256, 0, stream>>>(S, lds, (bf16_t*)P, ldp, rows, ncols, ncols_pad, scale,
                                                               Nq, H, causal, (const bf16_t*)bias, bsq, bsc, bsh);
  OTAMD_CHECK_LAUNCH();
  return OTAMD_OK;
}
