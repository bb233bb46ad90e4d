// FLUX.1 transformer kernels: the ops of diffusers FluxTransformer2DModel that
// are not GEMMs or attention, reached from modules/modelSetup/BaseFluxSetup.py:289-299 (model.transformer(...)).
//
// Activation layout (MI355X-first): token-major, batch-minor rows, r = t * B + b, over the JOINT
// sequence [text tokens (L) ; image tokens (N)].  A stream (text or image rows) is then one contiguous
// row block, so the double blocks' per-stream GEMMs, the single blocks' joint GEMMs and the joint
// attention (token stride B*ld, batch stride ld) all read the same buffers -- the reference's
// torch.cat / split of the two streams costs nothing.  Per-sample modulation vectors are indexed by
// b = r % B.
//
//   adaln_*       AdaLayerNormZero / AdaLayerNormZeroSingle / AdaLayerNormContinuous:
//                 y = LN(x) * (1 + scale[b]) + shift[b], LayerNorm without affine, eps 1e-6
//   gated_*       x + gate[b] * y (the gate_msa / gate_mlp residual adds)
//   qknorm_rope_* RMSNorm over each 128-wide head (norm_q / norm_k / norm_added_q / norm_added_k, eps 1e-6)
//                 fused with the rotary embedding (FluxPosEmbed + apply_rotary_emb, interleaved pairs)
//   gelu_tanh_*   GELU(approximate="tanh") of the feed-forward / proj_mlp
//   flux_pack     FluxModel.pack_latents / unpack_latents (modules/model/FluxModel.py:317-344)
// All HBM-bound; fp32 math, one bf16 rounding per output.
#include "common.h"

#define AD_MAXCH 8   // 8-element chunks per lane: D <= 4096

__device__ __forceinline__ void ld8(const bf16_t* p, float (&f)[8]) { unpack8(*reinterpret_cast<const bf8*>(p), f); }
__device__ __forceinline__ void st8(bf16_t* p, const float (&f)[8]) { *reinterpret_cast<bf8*>(p) = pack8(f); }

// ---------------------------------------------------------------------------------------------
// adaLN forward: rows [0, rows) of x; modulation mod[b * ldm + shift_off / scale_off + c]
__global__ void __launch_bounds__(256) adaln_fwd_kernel(const bf16_t* __restrict__ x, long long ldx,
                                                        bf16_t* __restrict__ y, long long ldy, int rows, int D,
                                                        float eps, const bf16_t* __restrict__ mod, long long ldm,
                                                        int shift_off, int scale_off, int B,
                                                        float* __restrict__ mean_out, float* __restrict__ rstd_out) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const int D8 = D >> 3;
  float f[AD_MAXCH][8];
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < AD_MAXCH; ++k) {
    const int c8 = lane + 64 * k;
    if (c8 < D8) {
      ld8(x + (long long)row * ldx + c8 * 8, f[k]);
#pragma unroll
      for (int j = 0; j < 8; ++j) s += f[k][j];
    }
  }
  const float mean = wave_sum(s) / D;
  float q = 0.f;
#pragma unroll
  for (int k = 0; k < AD_MAXCH; ++k)
    if (lane + 64 * k < D8) {
#pragma unroll
      for (int j = 0; j < 8; ++j) { const float d = f[k][j] - mean; q = fmaf(d, d, q); }
    }
  const float rstd = rsqrtf(wave_sum(q) / D + eps);
  const bf16_t* m = mod + (long long)(row % B) * ldm;
#pragma unroll
  for (int k = 0; k < AD_MAXCH; ++k) {
    const int c8 = lane + 64 * k;
    if (c8 < D8) {
      float sh[8], sc[8], o[8];
      ld8(m + shift_off + c8 * 8, sh);
      ld8(m + scale_off + c8 * 8, sc);
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = fmaf((f[k][j] - mean) * rstd, 1.f + sc[j], sh[j]);
      st8(y + (long long)row * ldy + c8 * 8, o);
    }
  }
  if (lane == 0) { mean_out[row] = mean; rstd_out[row] = rstd; }
}

// adaLN backward, input gradient: g = dy (1 + scale[b]); dx = rstd (g - mean(g) - xhat mean(g xhat))
__global__ void __launch_bounds__(256) adaln_bwd_dx_kernel(const bf16_t* __restrict__ x, long long ldx,
                                                           const bf16_t* __restrict__ dy, long long lddy,
                                                           bf16_t* __restrict__ dx, long long lddx, int rows, int D,
                                                           const bf16_t* __restrict__ mod, long long ldm, int scale_off,
                                                           int B, const float* __restrict__ mean_in,
                                                           const float* __restrict__ rstd_in,
                                                           const bf16_t* __restrict__ res, long long ldres) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const int D8 = D >> 3;
  const float mean = mean_in[row], rstd = rstd_in[row];
  const bf16_t* m = mod + (long long)(row % B) * ldm + scale_off;
  float xh[AD_MAXCH][8], g[AD_MAXCH][8];
  float s1 = 0.f, s2 = 0.f;
#pragma unroll
  for (int k = 0; k < AD_MAXCH; ++k) {
    const int c8 = lane + 64 * k;
    if (c8 < D8) {
      float dv[8], sc[8];
      ld8(x + (long long)row * ldx + c8 * 8, xh[k]);
      ld8(dy + (long long)row * lddy + c8 * 8, dv);
      ld8(m + c8 * 8, sc);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        xh[k][j] = (xh[k][j] - mean) * rstd;
        g[k][j] = dv[j] * (1.f + sc[j]);
        s1 += g[k][j];
        s2 = fmaf(g[k][j], xh[k][j], s2);
      }
    }
  }
  s1 = wave_sum(s1) / D;
  s2 = wave_sum(s2) / D;
#pragma unroll
  for (int k = 0; k < AD_MAXCH; ++k) {
    const int c8 = lane + 64 * k;
    if (c8 < D8) {
      float o[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = rstd * (g[k][j] - s1 - xh[k][j] * s2);
      if (res) {   // + the input's gradient through its residual use (the block's gated add)
        float rv[8];
        ld8(res + (long long)row * ldres + c8 * 8, rv);
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] += rv[j];
      }
      st8(dx + (long long)row * lddx + c8 * 8, o);
    }
  }
}

// Per-sample column reductions over the tokens of one batch element (grid: x = column chunks of
// 8 x 256, y = b, z = token split).  mode 0 (adaLN): part[z][b][0][c] += dy * xhat (dscale),
// part[z][b][1][c] += dy (dshift).  mode 1 (gated add): dy_out = gate[b] * dout, part[z][b][0][c] += dout * y.
template <int MODE>
__global__ void __launch_bounds__(256) mod_partial_kernel(const bf16_t* __restrict__ a, long long lda,
                                                          const bf16_t* __restrict__ bsrc, long long ldb, int T, int D,
                                                          int B, int tchunk, const float* __restrict__ mean_in,
                                                          const float* __restrict__ rstd_in,
                                                          const bf16_t* __restrict__ mod, long long ldm, int gate_off,
                                                          bf16_t* __restrict__ out, long long ldo,
                                                          float* __restrict__ part) {
  const int c8 = blockIdx.x * 256 + threadIdx.x;
  const int b = blockIdx.y, z = blockIdx.z;
  if (c8 * 8 >= D) return;
  const int t0 = z * tchunk, t1 = min(T, t0 + tchunk);
  float acc0[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f}, acc1[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  float gate[8];
  if (MODE == 1) ld8(mod + (long long)b * ldm + gate_off + c8 * 8, gate);
  for (int t = t0; t < t1; ++t) {
    const long long r = (long long)t * B + b;
    float av[8], bv[8];
    ld8(a + r * lda + c8 * 8, av);   // dy (mode 0) / dout (mode 1)
    ld8(bsrc + r * ldb + c8 * 8, bv);   // x (mode 0) / y (mode 1)
    if (MODE == 0) {
      const float mean = mean_in[r], rstd = rstd_in[r];
#pragma unroll
      for (int j = 0; j < 8; ++j) { acc0[j] = fmaf(av[j], (bv[j] - mean) * rstd, acc0[j]); acc1[j] += av[j]; }
    } else {
      float o[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) { acc0[j] = fmaf(av[j], bv[j], acc0[j]); o[j] = gate[j] * av[j]; }
      st8(out + r * ldo + c8 * 8, o);
    }
  }
  const int NP = MODE == 0 ? 2 : 1;
  float* p = part + ((long long)z * B + b) * NP * D + c8 * 8;
  *reinterpret_cast<float4*>(p) = make_float4(acc0[0], acc0[1], acc0[2], acc0[3]);
  *reinterpret_cast<float4*>(p + 4) = make_float4(acc0[4], acc0[5], acc0[6], acc0[7]);
  if (MODE == 0) {
    *reinterpret_cast<float4*>(p + D) = make_float4(acc1[0], acc1[1], acc1[2], acc1[3]);
    *reinterpret_cast<float4*>(p + D + 4) = make_float4(acc1[4], acc1[5], acc1[6], acc1[7]);
  }
}

// sum the token splits: dmod[b * ldm + off[i] + c] = bf16(sum_z part[z][b][i][c]), i < NP
__global__ void __launch_bounds__(256) mod_reduce_kernel(const float* __restrict__ part, int S, int B, int NP, int D,
                                                         bf16_t* __restrict__ dmod, long long ldm, int off0,
                                                         int off1) {
  const long long total = (long long)B * NP * D;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total; i += (long long)gridDim.x * blockDim.x) {
    float s = 0.f;
    for (int z = 0; z < S; ++z) s += part[(long long)z * total + i];
    const int c = (int)(i % D);
    const long long bi = i / D;
    const int which = (int)(bi % NP), b = (int)(bi / NP);
    dmod[(long long)b * ldm + (which ? off1 : off0) + c] = f2bf(s);
  }
}

// gated residual forward: out = x + gate[b] * y
__global__ void __launch_bounds__(256) gated_add_kernel(const bf16_t* __restrict__ x, long long ldx,
                                                        const bf16_t* __restrict__ y, long long ldy,
                                                        bf16_t* __restrict__ out, long long ldo, int rows, int D,
                                                        const bf16_t* __restrict__ mod, long long ldm, int gate_off,
                                                        int B) {
  const int D8 = D >> 3;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < (long long)rows * D8;
       i += (long long)gridDim.x * blockDim.x) {
    const long long r = i / D8;
    const int c = (int)(i - r * D8) * 8;
    float xv[8], yv[8], g[8], o[8];
    ld8(x + r * ldx + c, xv);
    ld8(y + r * ldy + c, yv);
    ld8(mod + (long long)(r % B) * ldm + gate_off + c, g);
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = fmaf(g[j], yv[j], xv[j]);
    st8(out + r * ldo + c, o);
  }
}

// ---------------------------------------------------------------------------------------------
// q/k RMSNorm over 128-wide heads + rotary embedding.  One wave per (row, q|k); a half-wave per
// head (32 lanes x 4 elements = interleaved pairs (4l, 4l+1), (4l+2, 4l+3)).  Rows of text
// tokens (t < L) use the *_ctx weights (norm_added_q / norm_added_k) when given.
struct QKRopeArgs {
  const bf16_t* x; long long ldx; int qoff, koff;     // q at x[r*ldx + qoff + h*128], k at koff
  bf16_t* y; long long ldy; int yqoff, ykoff;         // outputs (fwd: normalized + rotated; bwd: dx)
  const bf16_t* dy; long long lddy; int dyqoff, dykoff;
  const bf16_t* wq; const bf16_t* wk; const bf16_t* wq_ctx; const bf16_t* wk_ctx;
  const float* cs; const float* sn;                   // [T][128] rotary cos / sin (repeat-interleaved)
  float* dw_part;                                     // bwd: [blocks][4][128] (q_img, k_img, q_ctx, k_ctx) or null
  int rows, B, H, L;
  float eps;
  int pad_;
};

__device__ __forceinline__ float half_sum(float v) {
#pragma unroll
  for (int o = 16; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__global__ void __launch_bounds__(256) qknorm_rope_fwd_kernel(QKRopeArgs a) {
  const int lane = threadIdx.x & 63, hl = lane & 31, half = lane >> 5;
  const long long w = blockIdx.x * 4LL + (threadIdx.x >> 6);
  if (w >= 2LL * a.rows) return;
  const long long r = w >> 1;
  const int isk = (int)(w & 1);
  const int t = (int)(r / a.B);
  const bool ctx = t < a.L && a.wq_ctx;
  const bf16_t* wt = isk ? (ctx ? a.wk_ctx : a.wk) : (ctx ? a.wq_ctx : a.wq);
  const bf16_t* xr = a.x + r * a.ldx + (isk ? a.koff : a.qoff);
  bf16_t* yr = a.y + r * a.ldy + (isk ? a.ykoff : a.yqoff);
  const float4 c4 = *reinterpret_cast<const float4*>(a.cs + (long long)t * 128 + 4 * hl);
  const float4 s4 = *reinterpret_cast<const float4*>(a.sn + (long long)t * 128 + 4 * hl);
  const uint2 wv = *reinterpret_cast<const uint2*>(wt + 4 * hl);
  const float w0 = __uint_as_float(wv.x << 16), w1 = __uint_as_float(wv.x & 0xffff0000u);
  const float w2 = __uint_as_float(wv.y << 16), w3 = __uint_as_float(wv.y & 0xffff0000u);
  for (int h = half; h < a.H; h += 2) {
    const uint2 xv = *reinterpret_cast<const uint2*>(xr + h * 128 + 4 * hl);
    const float x0 = __uint_as_float(xv.x << 16), x1 = __uint_as_float(xv.x & 0xffff0000u);
    const float x2 = __uint_as_float(xv.y << 16), x3 = __uint_as_float(xv.y & 0xffff0000u);
    const float ss = half_sum(x0 * x0 + x1 * x1 + x2 * x2 + x3 * x3);
    const float rr = rsqrtf(ss * (1.f / 128.f) + a.eps);
    const float n0 = x0 * rr * w0, n1 = x1 * rr * w1, n2 = x2 * rr * w2, n3 = x3 * rr * w3;
    const float o0 = n0 * c4.x - n1 * s4.x, o1 = n1 * c4.y + n0 * s4.y;
    const float o2 = n2 * c4.z - n3 * s4.z, o3 = n3 * c4.w + n2 * s4.w;
    uint2 ov;
    ov.x = (uint32_t)f2bf(o0) | ((uint32_t)f2bf(o1) << 16);
    ov.y = (uint32_t)f2bf(o2) | ((uint32_t)f2bf(o3) << 16);
    *reinterpret_cast<uint2*>(yr + h * 128 + 4 * hl) = ov;
  }
}

// backward: dn = rope^T(dy); dw += dn * xhat; dx = rr (dn w - xhat mean(dn w xhat))
__global__ void __launch_bounds__(256) qknorm_rope_bwd_kernel(QKRopeArgs a) {
  __shared__ float red[4][4][128];
  const int lane = threadIdx.x & 63, hl = lane & 31, half = lane >> 5, wid = threadIdx.x >> 6;
  float dwa[4][4];   // [weight type][element]
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) dwa[i][j] = 0.f;
  for (long long w = blockIdx.x * 4LL + wid; w < 2LL * a.rows; w += (long long)gridDim.x * 4) {
    const long long r = w >> 1;
    const int isk = (int)(w & 1);
    const int t = (int)(r / a.B);
    const bool ctx = t < a.L && a.wq_ctx;
    const int wtype = isk + (ctx ? 2 : 0);
    const bf16_t* wt = isk ? (ctx ? a.wk_ctx : a.wk) : (ctx ? a.wq_ctx : a.wq);
    const bf16_t* xr = a.x + r * a.ldx + (isk ? a.koff : a.qoff);
    const bf16_t* dyr = a.dy + r * a.lddy + (isk ? a.dykoff : a.dyqoff);
    bf16_t* dxr = a.y + r * a.ldy + (isk ? a.ykoff : a.yqoff);
    const float4 c4 = *reinterpret_cast<const float4*>(a.cs + (long long)t * 128 + 4 * hl);
    const float4 s4 = *reinterpret_cast<const float4*>(a.sn + (long long)t * 128 + 4 * hl);
    const uint2 wv = *reinterpret_cast<const uint2*>(wt + 4 * hl);
    const float wf[4] = {__uint_as_float(wv.x << 16), __uint_as_float(wv.x & 0xffff0000u), __uint_as_float(wv.y << 16),
                         __uint_as_float(wv.y & 0xffff0000u)};
    float dws[4] = {0.f, 0.f, 0.f, 0.f};
    for (int h = half; h < a.H; h += 2) {
      const uint2 xv = *reinterpret_cast<const uint2*>(xr + h * 128 + 4 * hl);
      const uint2 gv = *reinterpret_cast<const uint2*>(dyr + h * 128 + 4 * hl);
      const float xf[4] = {__uint_as_float(xv.x << 16), __uint_as_float(xv.x & 0xffff0000u),
                           __uint_as_float(xv.y << 16), __uint_as_float(xv.y & 0xffff0000u)};
      const float g0 = __uint_as_float(gv.x << 16), g1 = __uint_as_float(gv.x & 0xffff0000u);
      const float g2 = __uint_as_float(gv.y << 16), g3 = __uint_as_float(gv.y & 0xffff0000u);
      const float dn[4] = {g0 * c4.x + g1 * s4.x, g1 * c4.y - g0 * s4.y, g2 * c4.z + g3 * s4.z, g3 * c4.w - g2 * s4.w};
      const float ss = half_sum(xf[0] * xf[0] + xf[1] * xf[1] + xf[2] * xf[2] + xf[3] * xf[3]);
      const float rr = rsqrtf(ss * (1.f / 128.f) + a.eps);
      float xh[4], dxh[4], dot = 0.f;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        xh[j] = xf[j] * rr;
        dxh[j] = dn[j] * wf[j];
        dot = fmaf(dxh[j], xh[j], dot);
        dws[j] = fmaf(dn[j], xh[j], dws[j]);
      }
      dot = half_sum(dot) * (1.f / 128.f);
      uint2 ov;
      ov.x = (uint32_t)f2bf(rr * (dxh[0] - xh[0] * dot)) | ((uint32_t)f2bf(rr * (dxh[1] - xh[1] * dot)) << 16);
      ov.y = (uint32_t)f2bf(rr * (dxh[2] - xh[2] * dot)) | ((uint32_t)f2bf(rr * (dxh[3] - xh[3] * dot)) << 16);
      *reinterpret_cast<uint2*>(dxr + h * 128 + 4 * hl) = ov;
    }
    if (a.dw_part) {
#pragma unroll
      for (int wt2 = 0; wt2 < 4; ++wt2)
        if (wt2 == wtype) {
#pragma unroll
          for (int j = 0; j < 4; ++j) dwa[wt2][j] += dws[j];
        }
    }
  }
  if (!a.dw_part) return;
  // combine the two half-waves (same elements, other heads) and the 4 waves of the block
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) dwa[i][j] += __shfl_xor(dwa[i][j], 32, 64);
  if (half == 0) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) red[wid][i][4 * hl + j] = dwa[i][j];
  }
  __syncthreads();
  for (int e = threadIdx.x; e < 4 * 128; e += 256) {
    const int i = e / 128, c = e % 128;
    a.dw_part[(long long)blockIdx.x * 512 + e] = red[0][i][c] + red[1][i][c] + red[2][i][c] + red[3][i][c];
  }
}

// dw[i][c] = sum_blocks part[blk][i][c] -> out_i[c] (bf16 or fp32, overwrite or accumulate)
__global__ void qk_dw_reduce_kernel(const float* __restrict__ part, int nblk, void* o0, void* o1, void* o2, void* o3,
                                    int f32, int accumulate) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= 512) return;
  float s = 0.f;
  for (int k = 0; k < nblk; ++k) s += part[(long long)k * 512 + e];
  const int i = e / 128, c = e % 128;
  void* o = i == 0 ? o0 : i == 1 ? o1 : i == 2 ? o2 : o3;
  if (!o) return;
  if (f32) {
    float* p = reinterpret_cast<float*>(o) + c;
    *p = accumulate ? *p + s : s;
  } else {
    bf16_t* p = reinterpret_cast<bf16_t*>(o) + c;
    *p = f2bf(accumulate ? bf2f(*p) + s : s);
  }
}

// ---------------------------------------------------------------------------------------------
// GELU(approximate="tanh"): 0.5 x (1 + tanh(sqrt(2/pi) (x + 0.044715 x^3)))
__device__ __forceinline__ float gelu_tanh(float x) {
  const float u = 0.7978845608028654f * fmaf(0.044715f * x, x * x, x);
  return 0.5f * x * (1.f + tanhf(u));
}
__device__ __forceinline__ float dgelu_tanh(float x) {
  const float u = 0.7978845608028654f * fmaf(0.044715f * x, x * x, x);
  const float th = tanhf(u);
  const float du = 0.7978845608028654f * fmaf(3.f * 0.044715f * x, x, 1.f);
  return 0.5f * (1.f + th) + 0.5f * x * (1.f - th * th) * du;
}

__global__ void __launch_bounds__(256) gelu_tanh_fwd_kernel(const bf16_t* __restrict__ x, long long ldx,
                                                            bf16_t* __restrict__ y, long long ldy, int rows, int F) {
  const int F8 = F >> 3;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < (long long)rows * F8;
       i += (long long)gridDim.x * blockDim.x) {
    const long long r = i / F8;
    const int c = (int)(i - r * F8) * 8;
    float v[8];
    ld8(x + r * ldx + c, v);
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = gelu_tanh(v[j]);
    st8(y + r * ldy + c, v);
  }
}

__global__ void __launch_bounds__(256) gelu_tanh_bwd_kernel(const bf16_t* __restrict__ x, long long ldx,
                                                            const bf16_t* __restrict__ dy, long long lddy,
                                                            bf16_t* __restrict__ dx, long long lddx, int rows, int F) {
  const int F8 = F >> 3;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < (long long)rows * F8;
       i += (long long)gridDim.x * blockDim.x) {
    const long long r = i / F8;
    const int c = (int)(i - r * F8) * 8;
    float v[8], g[8];
    ld8(x + r * ldx + c, v);
    ld8(dy + r * lddy + c, g);
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = g[j] * dgelu_tanh(v[j]);
    st8(dx + r * lddx + c, v);
  }
}

// ---------------------------------------------------------------------------------------------
// pack: NHWC latent [B, h, w, C] (row stride ldl >= C) -> packed tokens rows (t * B + b), t = (y/2)(w/2) + x/2,
// channel c * 4 + dy * 2 + dx (pack_latents' permute(0, 2, 4, 1, 3, 5)).  dir = 1: the inverse (unpack).
__global__ void __launch_bounds__(256) flux_pack_kernel(const bf16_t* __restrict__ src, bf16_t* __restrict__ dst,
                                                        int B, int h, int w, int C, int ldl, int dir) {
  const long long total = (long long)B * h * w * C;
  const int hw2 = (h / 2) * (w / 2);
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total; i += (long long)gridDim.x * blockDim.x) {
    const int c = (int)(i % C);
    long long p = i / C;
    const int x = (int)(p % w);
    p /= w;
    const int y = (int)(p % h);
    const int b = (int)(p / h);
    const long long lat = (((long long)b * h + y) * w + x) * ldl + c;
    const long long tok = ((long long)((y >> 1) * (w >> 1) + (x >> 1)) * B + b) * (4LL * C) + c * 4 + (y & 1) * 2 + (x & 1);
    (void)hw2;
    if (dir == 0) dst[tok] = src[lat];
    else dst[lat] = src[tok];
  }
}

// ---------------------------------------------------------------------------------------------
static int gfor(long long n) { return (int)std::max<long long>(1, std::min<long long>((n + 255) / 256, 16384)); }
static bool a16(const void* p) { return ((uintptr_t)p & 15) == 0; }

OTAMD_API int otamd_adaln_fwd(const void* x, long long ldx, void* y, long long ldy, int rows, int D, float eps,
                              const void* mod, long long ldm, int shift_off, int scale_off, int B, float* mean,
                              float* rstd, hipStream_t s) {
  if (!x || !y || !mod || !mean || !rstd || rows <= 0 || B <= 0 || D % 8 || D > 512 * AD_MAXCH || ldx % 8 || ldy % 8 ||
      ldm % 8 || shift_off % 8 || scale_off % 8 || !a16(x) || !a16(y) || !a16(mod))
    return OTAMD_EINVAL;
  adaln_fwd_kernel<<<(rows + 3) / 4, 256, 0, s>>>((const bf16_t*)x, ldx, (bf16_t*)y, ldy, rows, D, eps,
                                                  (const bf16_t*)mod, ldm, shift_off, scale_off, B, mean, rstd);
  OTAMD_CHECK_LAUNCH();
  return OTAMD_OK;
}

// token splits of the per-sample column reductions: >= 64 tokens per thread (the slab the reduce
// pass re-reads stays small), and enough blocks to cover the CUs
static int mod_splits(int T, int D, int B) {
  const int xb = (D / 8 + 255) / 256;
  int S = std::max(1, 512 / std::max(1, xb * B));
  S = std::min(S, std::max(1, (T + 63) / 64));
  return S;
}

// float scratch the adaLN / gated backward reductions need (pass as `part`)
OTAMD_API long long otamd_mod_part_floats(int T, int D, int B) { return 2LL * mod_splits(T, D, B) * B * D; }

// rows = T * B; dmod gets bf16(dscale) at scale_off and bf16(dshift) at shift_off (overwrite); res (nullable):
// dx += res in the same pass
static int adaln_bwd_impl(const void* x, long long ldx, const void* dy, long long lddy, const void* res, long long ldres,
                          void* dx, long long lddx, int rows, int D, const void* mod, long long ldm, int shift_off,
                          int scale_off, int B, const float* mean, const float* rstd, void* dmod, float* part,
                          hipStream_t s) {
  if (!x || !dy || !dx || !mod || !mean || !rstd || rows <= 0 || B <= 0 || rows % B || D % 8 || D > 512 * AD_MAXCH ||
      ldx % 8 || lddy % 8 || lddx % 8 || ldm % 8 || !a16(x) || !a16(dy) || !a16(dx) || (res && (ldres % 8 || !a16(res))))
    return OTAMD_EINVAL;
  adaln_bwd_dx_kernel<<<(rows + 3) / 4, 256, 0, s>>>((const bf16_t*)x, ldx, (const bf16_t*)dy, lddy, (bf16_t*)dx,
                                                     lddx, rows, D, (const bf16_t*)mod, ldm, scale_off, B, mean, rstd,
                                                     (const bf16_t*)res, ldres);
  OTAMD_CHECK_LAUNCH();
  if (dmod) {
    if (!part) return OTAMD_EINVAL;
    const int T = rows / B, S = mod_splits(T, D, B);
    dim3 g((D / 8 + 255) / 256, B, S);
    mod_partial_kernel<0><<<g, 256, 0, s>>>((const bf16_t*)dy, lddy, (const bf16_t*)x, ldx, T, D, B, (T + S - 1) / S,
                                            mean, rstd, nullptr, 0, 0, nullptr, 0, part);
    OTAMD_CHECK_LAUNCH();
    mod_reduce_kernel<<<gfor(2LL * B * D), 256, 0, s>>>(part, S, B, 2, D, (bf16_t*)dmod, ldm, scale_off, shift_off);
    OTAMD_CHECK_LAUNCH();
  }
  return OTAMD_OK;
}

// the modulation gradient alone (the dmod half of otamd_adaln_bwd): dmod[b, shift_off + c] = sum_t dy,
// dmod[b, scale_off + c] = sum_t dy * xhat -- queued on the weight-gradient stream when the modulation branch runs
// there (module/flux.py), while the dx pass stays on the critical stream
OTAMD_API int otamd_adaln_dmod(const void* x, long long ldx, const void* dy, long long lddy, int rows, int D, long long ldm,
                               int shift_off, int scale_off, int B, const float* mean, const float* rstd, void* dmod,
                               float* part, hipStream_t s) {
  if (!x || !dy || !dmod || !part || !mean || !rstd || rows <= 0 || B <= 0 || rows % B || D % 8 || ldx % 8 ||
      lddy % 8 || ldm % 8 || !a16(x) || !a16(dy))
    return OTAMD_EINVAL;
  const int T = rows / B, S = mod_splits(T, D, B);
  dim3 g((D / 8 + 255) / 256, B, S);
  mod_partial_kernel<0><<<g, 256, 0, s>>>((const bf16_t*)dy, lddy, (const bf16_t*)x, ldx, T, D, B, (T + S - 1) / S,
                                          mean, rstd, nullptr, 0, 0, nullptr, 0, part);
  OTAMD_CHECK_LAUNCH();
  mod_reduce_kernel<<<gfor(2LL * B * D), 256, 0, s>>>(part, S, B, 2, D, (bf16_t*)dmod, ldm, scale_off, shift_off);
  OTAMD_CHECK_LAUNCH();
  return OTAMD_OK;
}

OTAMD_API int otamd_adaln_bwd(const void* x, long long ldx, const void* dy, long long lddy, void* dx, long long lddx,
                              int rows, int D, const void* mod, long long ldm, int shift_off, int scale_off, int B,
                              const float* mean, const float* rstd, void* dmod, float* part, hipStream_t s) {
  return adaln_bwd_impl(x, ldx, dy, lddy, nullptr, 0, dx, lddx, rows, D, mod, ldm, shift_off, scale_off, B, mean, rstd,
                        dmod, part, s);
}
OTAMD_API int otamd_adaln_bwd_res(const void* x, long long ldx, const void* dy, long long lddy, const void* res,
                                  long long ldres, void* dx, long long lddx, int rows, int D, const void* mod,
                                  long long ldm, int shift_off, int scale_off, int B, const float* mean,
                                  const float* rstd, void* dmod, float* part, hipStream_t s) {
  if (!res) return OTAMD_EINVAL;
  return adaln_bwd_impl(x, ldx, dy, lddy, res, ldres, dx, lddx, rows, D, mod, ldm, shift_off, scale_off, B, mean, rstd,
                        dmod, part, s);
}

OTAMD_API int otamd_gated_add_fwd(const void* x, long long ldx, const void* y, long long ldy, void* out, long long ldo,
                                  int rows, int D, const void* mod, long long ldm, int gate_off, int B, hipStream_t s) {
  if (!x || !y || !out || !mod || rows <= 0 || B <= 0 || D % 8 || ldx % 8 || ldy % 8 || ldo % 8 || ldm % 8 ||
      gate_off % 8 || !a16(x) || !a16(y) || !a16(out) || !a16(mod))
    return OTAMD_EINVAL;
  gated_add_kernel<<<gfor((long long)rows * D / 8), 256, 0, s>>>((const bf16_t*)x, ldx, (const bf16_t*)y, ldy,
                                                                 (bf16_t*)out, ldo, rows, D, (const bf16_t*)mod, ldm,
                                                                 gate_off, B);
  OTAMD_CHECK_LAUNCH();
  return OTAMD_OK;
}

// dy = gate[b] * dout; dmod[b, gate_off + c] = bf16(sum_t dout * y)
OTAMD_API int otamd_gated_add_bwd(const void* dout, long long lddo, const void* y, long long ldy, void* dy,
                                  long long lddy, int rows, int D, const void* mod, long long ldm, int gate_off, int B,
                                  void* dmod, float* part, hipStream_t s) {
  if (!dout || !y || !dy || !mod || !dmod || !part || rows <= 0 || B <= 0 || rows % B || D % 8 || lddo % 8 ||
      ldy % 8 || lddy % 8 || ldm % 8 || !a16(dout) || !a16(y) || !a16(dy))
    return OTAMD_EINVAL;
  const int T = rows / B, S = mod_splits(T, D, B);
  dim3 g((D / 8 + 255) / 256, B, S);
  mod_partial_kernel<1><<<g, 256, 0, s>>>((const bf16_t*)dout, lddo, (const bf16_t*)y, ldy, T, D, B, (T + S - 1) / S,
                                          nullptr, nullptr, (const bf16_t*)mod, ldm, gate_off, (bf16_t*)dy, lddy, part);
  OTAMD_CHECK_LAUNCH();
  mod_reduce_kernel<<<gfor((long long)B * D), 256, 0, s>>>(part, S, B, 1, D, (bf16_t*)dmod, ldm, gate_off, gate_off);
  OTAMD_CHECK_LAUNCH();
  return OTAMD_OK;
}

OTAMD_API int otamd_qk_rope_args_size(void) { return (int)sizeof(QKRopeArgs); }

static bool qk_ok(const QKRopeArgs& a) {
  if (!a.x || !a.y || !a.wq || !a.wk || !a.cs || !a.sn || a.rows <= 0 || a.B <= 0 || a.H <= 0) return false;
  if (a.ldx % 4 || a.ldy % 4 || a.qoff % 4 || a.koff % 4 || a.yqoff % 4 || a.ykoff % 4) return false;
  if (((uintptr_t)a.x | (uintptr_t)a.y | (uintptr_t)a.cs | (uintptr_t)a.sn) & 15) return false;
  if (!a.wq_ctx != !a.wk_ctx) return false;
  return true;
}

OTAMD_API int otamd_qknorm_rope_fwd(const QKRopeArgs* in, hipStream_t s) {
  if (!in || !qk_ok(*in)) return OTAMD_EINVAL;
  const long long waves = 2LL * in->rows;
  qknorm_rope_fwd_kernel<<<(int)((waves + 3) / 4), 256, 0, s>>>(*in);
  OTAMD_CHECK_LAUNCH();
  return OTAMD_OK;
}

// dw_out*: the four norm weights' grads (q_img, k_img, q_ctx, k_ctx; null = skip); part: >= 512 * 1024 floats
OTAMD_API int otamd_qknorm_rope_bwd(const QKRopeArgs* in, void* dwq, void* dwk, void* dwq_ctx, void* dwk_ctx,
                                    int dw_f32, int dw_acc, float* part, hipStream_t s) {
  if (!in || !qk_ok(*in) || !in->dy || in->lddy % 4 || in->dyqoff % 4 || in->dykoff % 4 || ((uintptr_t)in->dy & 15))
    return OTAMD_EINVAL;
  QKRopeArgs a = *in;
  const bool need_dw = dwq || dwk || dwq_ctx || dwk_ctx;
  if (need_dw && !part) return OTAMD_EINVAL;
  a.dw_part = need_dw ? part : nullptr;
  const long long waves = 2LL * a.rows;
  const int nblk = (int)std::min<long long>((waves + 3) / 4, 1024);
  qknorm_rope_bwd_kernel<<<nblk, 256, 0, s>>>(a);
  OTAMD_CHECK_LAUNCH();
  if (need_dw) {
    qk_dw_reduce_kernel<<<2, 256, 0, s>>>(part, nblk, dwq, dwk, dwq_ctx, dwk_ctx, dw_f32, dw_acc);
    OTAMD_CHECK_LAUNCH();
  }
  return OTAMD_OK;
}

OTAMD_API int otamd_gelu_tanh_fwd(const void* x, long long ldx, void* y, long long ldy, int rows, int F, hipStream_t s) {
  if (!x || !y || rows <= 0 || F % 8 || ldx % 8 || ldy % 8 || !a16(x) || !a16(y)) return OTAMD_EINVAL;
  gelu_tanh_fwd_kernel<<<gfor((long long)rows * F / 8), 256, 0, s>>>((const bf16_t*)x, ldx, (bf16_t*)y, ldy, rows, F);
  OTAMD_CHECK_LAUNCH();
  return OTAMD_OK;
}

OTAMD_API int otamd_gelu_tanh_bwd(const void* x, long long ldx, const void* dy, long long lddy, void* dx,
                                  long long lddx, int rows, int F, hipStream_t s) {
  if (!x || !dy || !dx || rows <= 0 || F % 8 || ldx % 8 || lddy % 8 || lddx % 8 || !a16(x) || !a16(dy) || !a16(dx))
    return OTAMD_EINVAL;
  gelu_tanh_bwd_kernel<<<gfor((long long)rows * F / 8), 256, 0, s>>>((const bf16_t*)x, ldx, (const bf16_t*)dy, lddy,
                                                                     (bf16_t*)dx, lddx, rows, F);
  OTAMD_CHECK_LAUNCH();
  return OTAMD_OK;
}

// dir 0: latent NHWC [B,h,w,C] (row stride ldl) -> packed [(h/2)(w/2) * B, 4C]; dir 1: packed -> latent
OTAMD_API int otamd_flux_pack(const void* src, void* dst, int B, int h, int w, int C, int ldl, int dir, hipStream_t s) {
  if (!src || !dst || B <= 0 || h <= 0 || w <= 0 || C <= 0 || h % 2 || w % 2 || ldl < C || (dir != 0 && dir != 1))
    return OTAMD_EINVAL;
  flux_pack_kernel<<<gfor((long long)B * h * w * C), 256, 0, s>>>((const bf16_t*)src, (bf16_t*)dst, B, h, w, C, ldl, dir);
  OTAMD_CHECK_LAUNCH();
  return OTAMD_OK;
}
