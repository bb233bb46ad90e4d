// GroupNorm (+ fused SiLU) and LayerNorm, forward and backward, on NHWC bf16 activations.
// Replaces the diffusers ResnetBlock2D norm1/norm2 + SiLU, Transformer2DModel.norm and
// BasicTransformerBlock norm1-3 (SURVEY.md §2.3 "GroupNorm(32 groups)+SiLU fwd/bwd" and
// "LayerNorm"); under the reference's autocast(bf16) these run in fp32 and their output is
// rounded to bf16 once by the consuming conv/linear - this file computes in fp32 and rounds
// once on store, which is the same numerics.
//
// GroupNorm works on [N, HW, C] with G groups of Cg = C/G channels (Cg need not be a multiple
// of 8: 320/32 = 10).  Statistics are accumulated per (n, channel) and folded into groups
// afterwards, so every load is a 16-byte chunk of 8 channels.
// HBM-bound: fwd reads x twice (stats, apply) and writes y once; bwd reads x, dy twice and
// writes dx once.
#include "common.h"

__device__ __forceinline__ void store_param_grad(void* p, long long i, float v, int f32, int acc);

// ------------------------------------------------------------------------------------------
// per-(n, c) partial sums of x and x^2, accumulated in double via atomics
// grid: (pixel blocks, N); block 256 threads; thread t owns channel chunk t % C8 and pixels
// p = t / C8 + k * (256 / C8)
__global__ void __launch_bounds__(256) gn_stats_kernel(const bf16_t* __restrict__ x, long long ldx, int HW, int C,
                                                       int pix_per_block, double* __restrict__ sum,
                                                       double* __restrict__ sumsq) {
  extern __shared__ float sred[];   // [2][C]
  const int n = blockIdx.y;
  const int C8 = C >> 3;
  const int lanes_per_pix = C8 <= 256 ? C8 : 256;
  const int pix_stride = 256 / lanes_per_pix;
  const int t = threadIdx.x;
  for (int i = t; i < 2 * C; i += 256) sred[i] = 0.f;
  __syncthreads();
  const int p0 = blockIdx.x * pix_per_block;
  const int p1 = min(HW, p0 + pix_per_block);
  if (t < lanes_per_pix * pix_stride) {
    for (int c8 = t % lanes_per_pix; c8 < C8; c8 += lanes_per_pix) {
      float s[8] = {0}, q[8] = {0};
      for (int p = p0 + t / lanes_per_pix; p < p1; p += pix_stride) {
        bf8 v = *reinterpret_cast<const bf8*>(x + ((long long)n * HW + p) * ldx + c8 * 8);
        float f[8];
        unpack8(v, f);
#pragma unroll
        for (int j = 0; j < 8; ++j) { s[j] += f[j]; q[j] = fmaf(f[j], f[j], q[j]); }
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        atomicAdd(&sred[c8 * 8 + j], s[j]);
        atomicAdd(&sred[C + c8 * 8 + j], q[j]);
      }
    }
  }
  __syncthreads();
  for (int c = t; c < C; c += 256) {
    atomicAdd(&sum[(long long)n * C + c], (double)sred[c]);
    atomicAdd(&sumsq[(long long)n * C + c], (double)sred[C + c]);
  }
}

// fold channel sums into groups; emit per-(n,c) affine a = rstd*gamma, b = beta - mean*a,
// and per-(n,g) mean / rstd for the backward.  grid N, block 256
__global__ void gn_finalize_kernel(const double* __restrict__ sum, const double* __restrict__ sumsq, int HW, int C,
                                   int G, float eps, const bf16_t* __restrict__ gamma, const bf16_t* __restrict__ beta,
                                   float* __restrict__ mean_out, float* __restrict__ rstd_out, float* __restrict__ a_out,
                                   float* __restrict__ b_out) {
  const int n = blockIdx.x;
  const int Cg = C / G;
  for (int g = threadIdx.x; g < G; g += blockDim.x) {
    double s = 0, q = 0;
    for (int c = g * Cg; c < (g + 1) * Cg; ++c) { s += sum[(long long)n * C + c]; q += sumsq[(long long)n * C + c]; }
    const double cnt = (double)HW * Cg;
    const double mean = s / cnt;
    double var = q / cnt - mean * mean;
    if (var < 0) var = 0;
    const float rstd = (float)(1.0 / sqrt(var + (double)eps));
    mean_out[n * G + g] = (float)mean;
    rstd_out[n * G + g] = rstd;
    for (int c = g * Cg; c < (g + 1) * Cg; ++c) {
      const float gm = gamma ? bf2f(gamma[c]) : 1.f;
      const float bt = beta ? bf2f(beta[c]) : 0.f;
      const float a = rstd * gm;
      a_out[n * C + c] = a;
      b_out[n * C + c] = bt - (float)mean * a;
    }
  }
}

// y = [silu](x * a[n,c] + b[n,c]); grid-stride over 16-byte chunks
template <bool SILU>
__global__ void __launch_bounds__(256) gn_apply_kernel(const bf16_t* __restrict__ x, long long ldx, bf16_t* __restrict__ y,
                                                       long long ldy, int N, int HW, int C, const float* __restrict__ a,
                                                       const float* __restrict__ b) {
  const int C8 = C >> 3;
  const long long total = (long long)N * HW * C8;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total; i += (long long)gridDim.x * blockDim.x) {
    const long long pix = i / C8;
    const int c0 = (int)(i - pix * C8) * 8;
    const int n = (int)(pix / HW);
    bf8 v = *reinterpret_cast<const bf8*>(x + pix * ldx + c0);
    float f[8];
    unpack8(v, f);
    const float4 a0 = *reinterpret_cast<const float4*>(a + (long long)n * C + c0);
    const float4 a1 = *reinterpret_cast<const float4*>(a + (long long)n * C + c0 + 4);
    const float4 b0 = *reinterpret_cast<const float4*>(b + (long long)n * C + c0);
    const float4 b1 = *reinterpret_cast<const float4*>(b + (long long)n * C + c0 + 4);
    const float av[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
    const float bv[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float z = fmaf(f[j], av[j], bv[j]);
      f[j] = SILU ? silu_f(z) : z;
    }
    *reinterpret_cast<bf8*>(y + pix * ldy + c0) = pack8(f);
  }
}

// backward pass 1: per-(n,c) S1 = sum dz, S2 = sum dz * xhat   (dz = dy * silu'(z) when SILU)
template <bool SILU>
__global__ void __launch_bounds__(256) gn_bwd_reduce_kernel(const bf16_t* __restrict__ x, long long ldx,
                                                            const bf16_t* __restrict__ dy, long long lddy, int HW, int C,
                                                            int G, int pix_per_block, const float* __restrict__ a,
                                                            const float* __restrict__ b, const float* __restrict__ mean,
                                                            const float* __restrict__ rstd, double* __restrict__ s1,
                                                            double* __restrict__ s2) {
  extern __shared__ float sred[];   // [2][C]
  const int n = blockIdx.y;
  const int C8 = C >> 3;
  const int Cg = C / G;
  const int lanes_per_pix = C8 <= 256 ? C8 : 256;
  const int pix_stride = 256 / lanes_per_pix;
  const int t = threadIdx.x;
  for (int i = t; i < 2 * C; i += 256) sred[i] = 0.f;
  __syncthreads();
  const int p0 = blockIdx.x * pix_per_block;
  const int p1 = min(HW, p0 + pix_per_block);
  if (t < lanes_per_pix * pix_stride) {
    for (int c8 = t % lanes_per_pix; c8 < C8; c8 += lanes_per_pix) {
      const int c0 = c8 * 8;
      float av[8], bv[8], mv[8], rv[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        av[j] = a[(long long)n * C + c0 + j];
        bv[j] = b[(long long)n * C + c0 + j];
        const int g = (c0 + j) / Cg;
        mv[j] = mean[n * G + g];
        rv[j] = rstd[n * G + g];
      }
      float s[8] = {0}, q[8] = {0};
      for (int p = p0 + t / lanes_per_pix; p < p1; p += pix_stride) {
        const long long pix = (long long)n * HW + p;
        bf8 xv = *reinterpret_cast<const bf8*>(x + pix * ldx + c0);
        bf8 gv = *reinterpret_cast<const bf8*>(dy + pix * lddy + c0);
        float xf[8], gf[8];
        unpack8(xv, xf);
        unpack8(gv, gf);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          float dz = gf[j];
          if (SILU) dz *= dsilu_f(fmaf(xf[j], av[j], bv[j]));
          const float xh = (xf[j] - mv[j]) * rv[j];
          s[j] += dz;
          q[j] = fmaf(dz, xh, q[j]);
        }
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        atomicAdd(&sred[c0 + j], s[j]);
        atomicAdd(&sred[C + c0 + j], q[j]);
      }
    }
  }
  __syncthreads();
  for (int c = t; c < C; c += 256) {
    atomicAdd(&s1[(long long)n * C + c], (double)sred[c]);
    atomicAdd(&s2[(long long)n * C + c], (double)sred[C + c]);
  }
}

// per-(n,g) constants c1 = sum_c gamma_c S1 / cnt, c2 = sum_c gamma_c S2 / cnt; also dgamma/dbeta
__global__ void gn_bwd_finalize_kernel(const double* __restrict__ s1, const double* __restrict__ s2, int N, int HW,
                                       int C, int G, const bf16_t* __restrict__ gamma, float* __restrict__ c1,
                                       float* __restrict__ c2, void* __restrict__ dgamma, void* __restrict__ dbeta,
                                       int pf32, int pacc) {
  const int Cg = C / G;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < N * G; i += gridDim.x * blockDim.x) {
    const int n = i / G, g = i - n * G;
    double a = 0, bsum = 0;
    for (int c = g * Cg; c < (g + 1) * Cg; ++c) {
      const double gm = gamma ? bf2f(gamma[c]) : 1.0;
      a += gm * s1[(long long)n * C + c];
      bsum += gm * s2[(long long)n * C + c];
    }
    const double cnt = (double)HW * Cg;
    c1[i] = (float)(a / cnt);
    c2[i] = (float)(bsum / cnt);
  }
  for (int c = blockIdx.x * blockDim.x + threadIdx.x; c < C; c += gridDim.x * blockDim.x) {
    double dg = 0, db = 0;
    for (int n = 0; n < N; ++n) { dg += s2[(long long)n * C + c]; db += s1[(long long)n * C + c]; }
    if (dgamma) store_param_grad(dgamma, c, (float)dg, pf32, pacc);
    if (dbeta) store_param_grad(dbeta, c, (float)db, pf32, pacc);
  }
}

// dx = rstd * (dz*gamma - c1 - xhat*c2)
template <bool SILU>
__global__ void __launch_bounds__(256) gn_bwd_apply_kernel(const bf16_t* __restrict__ x, long long ldx,
                                                           const bf16_t* __restrict__ dy, long long lddy,
                                                           bf16_t* __restrict__ dx, long long lddx, int N, int HW, int C,
                                                           int G, const bf16_t* __restrict__ gamma,
                                                           const float* __restrict__ a, const float* __restrict__ b,
                                                           const float* __restrict__ mean, const float* __restrict__ rstd,
                                                           const float* __restrict__ c1, const float* __restrict__ c2,
                                                           int accumulate) {
  const int C8 = C >> 3;
  const int Cg = C / G;
  const long long total = (long long)N * HW * C8;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total; i += (long long)gridDim.x * blockDim.x) {
    const long long pix = i / C8;
    const int c0 = (int)(i - pix * C8) * 8;
    const int n = (int)(pix / HW);
    bf8 xv = *reinterpret_cast<const bf8*>(x + pix * ldx + c0);
    bf8 gv = *reinterpret_cast<const bf8*>(dy + pix * lddy + c0);
    float xf[8], gf[8], o[8];
    unpack8(xv, xf);
    unpack8(gv, gf);
    float prev[8];
    if (accumulate) { bf8 pv = *reinterpret_cast<const bf8*>(dx + pix * lddx + c0); unpack8(pv, prev); }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int c = c0 + j, g = c / Cg, ng = n * G + g;
      float dz = gf[j];
      if (SILU) dz *= dsilu_f(fmaf(xf[j], a[(long long)n * C + c], b[(long long)n * C + c]));
      const float r = rstd[ng];
      const float xh = (xf[j] - mean[ng]) * r;
      const float gm = gamma ? bf2f(gamma[c]) : 1.f;
      o[j] = r * (dz * gm - c1[ng] - xh * c2[ng]);
      if (accumulate) o[j] += prev[j];
    }
    *reinterpret_cast<bf8*>(dx + pix * lddx + c0) = pack8(o);
  }
}

static int ew_blocks(long long n) {
  long long b = (n + 255) / 256;
  return (int)(b < 1 ? 1 : (b > 8192 ? 8192 : b));
}

// ws: double[4*N*C] scratch.  stats out (fp32): mean[N*G], rstd[N*G], a[N*C], b[N*C]
OTAMD_API int otamd_groupnorm_fwd(const void* x, long long ldx, void* y, long long ldy, int N, int HW, int C, int G,
                                  float eps, const void* gamma, const void* beta, int silu, float* mean, float* rstd,
                                  float* a, float* b, double* ws, hipStream_t stream) {
  if (!x || !y || !mean || !rstd || !a || !b || !ws || N <= 0 || HW <= 0 || C <= 0 || G <= 0) return OTAMD_EINVAL;
  if (C % 8 || C % G || ldx % 8 || ldy % 8 || ((uintptr_t)x & 15) || ((uintptr_t)y & 15) || C > 8192) return OTAMD_EINVAL;
  if (hipMemsetAsync(ws, 0, sizeof(double) * 2 * N * C, stream) != hipSuccess) return OTAMD_ELAUNCH;
  const int ppb = 128;
  dim3 grid((HW + ppb - 1) / ppb, N);
  gn_stats_kernel<<<grid, 256, 2 * C * sizeof(float), stream>>>((const bf16_t*)x, ldx, HW, C, ppb, ws, ws + (long long)N * C);
  OTAMD_CHECK_LAUNCH();
  gn_finalize_kernel<<<N, 64, 0, stream>>>(ws, ws + (long long)N * C, HW, C, G, eps, (const bf16_t*)gamma,
                                           (const bf16_t*)beta, mean, rstd, a, b);
  OTAMD_CHECK_LAUNCH();
  const long long chunks = (long long)N * HW * (C / 8);
  if (silu) gn_apply_kernel<true><<<ew_blocks(chunks), 256, 0, stream>>>((const bf16_t*)x, ldx, (bf16_t*)y, ldy, N, HW, C, a, b);
  else gn_apply_kernel<false><<<ew_blocks(chunks), 256, 0, stream>>>((const bf16_t*)x, ldx, (bf16_t*)y, ldy, N, HW, C, a, b);
  OTAMD_CHECK_LAUNCH();
  return OTAMD_OK;
}

// ws: double[2*N*C] + float scratch c1,c2 [2*N*G] given separately in fws
OTAMD_API int otamd_groupnorm_bwd(const void* x, long long ldx, const void* dy, long long lddy, void* dx,
                                  long long lddx, int N, int HW, int C, int G, const void* gamma, int silu,
                                  const float* mean, const float* rstd, const float* a, const float* b,
                                  void* dgamma, void* dbeta, int param_f32, int param_acc, double* ws, float* fws,
                                  int accumulate, hipStream_t stream) {
  if (!x || !dy || !dx || !mean || !rstd || !a || !b || !ws || !fws || N <= 0 || HW <= 0) return OTAMD_EINVAL;
  if (C % 8 || C % G || ldx % 8 || lddy % 8 || lddx % 8 || C > 8192) return OTAMD_EINVAL;
  if (((uintptr_t)x | (uintptr_t)dy | (uintptr_t)dx) & 15) return OTAMD_EINVAL;
  if (hipMemsetAsync(ws, 0, sizeof(double) * 2 * N * C, stream) != hipSuccess) return OTAMD_ELAUNCH;
  const int ppb = 128;
  dim3 grid((HW + ppb - 1) / ppb, N);
  double* s1 = ws;
  double* s2 = ws + (long long)N * C;
  if (silu)
    gn_bwd_reduce_kernel<true><<<grid, 256, 2 * C * sizeof(float), stream>>>(
        (const bf16_t*)x, ldx, (const bf16_t*)dy, lddy, HW, C, G, ppb, a, b, mean, rstd, s1, s2);
  else
    gn_bwd_reduce_kernel<false><<<grid, 256, 2 * C * sizeof(float), stream>>>(
        (const bf16_t*)x, ldx, (const bf16_t*)dy, lddy, HW, C, G, ppb, a, b, mean, rstd, s1, s2);
  OTAMD_CHECK_LAUNCH();
  float* c1 = fws;
  float* c2 = fws + N * G;
  gn_bwd_finalize_kernel<<<8, 256, 0, stream>>>(s1, s2, N, HW, C, G, (const bf16_t*)gamma, c1, c2, dgamma, dbeta,
                                                param_f32, param_acc);
  OTAMD_CHECK_LAUNCH();
  const long long chunks = (long long)N * HW * (C / 8);
  if (silu)
    gn_bwd_apply_kernel<true><<<ew_blocks(chunks), 256, 0, stream>>>(
        (const bf16_t*)x, ldx, (const bf16_t*)dy, lddy, (bf16_t*)dx, lddx, N, HW, C, G, (const bf16_t*)gamma, a, b,
        mean, rstd, c1, c2, accumulate);
  else
    gn_bwd_apply_kernel<false><<<ew_blocks(chunks), 256, 0, stream>>>(
        (const bf16_t*)x, ldx, (const bf16_t*)dy, lddy, (bf16_t*)dx, lddx, N, HW, C, G, (const bf16_t*)gamma, a, b,
        mean, rstd, c1, c2, accumulate);
  OTAMD_CHECK_LAUNCH();
  return OTAMD_OK;
}

// ------------------------------------------------------------------------------------------
// LayerNorm over the last dim C (C % 8 == 0, C <= 64*8*4 = 2048): one wave per row
#define LN_MAXCH 4
__global__ void __launch_bounds__(256) ln_fwd_kernel(const bf16_t* __restrict__ x, long long ldx, bf16_t* __restrict__ y,
                                                     long long ldy, int rows, int C, float eps,
                                                     const bf16_t* __restrict__ gamma, const bf16_t* __restrict__ beta,
                                                     float* __restrict__ mean_out, float* __restrict__ rstd_out) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const int C8 = C >> 3;
  float f[LN_MAXCH][8];
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < LN_MAXCH; ++k) {
    const int c8 = lane + 64 * k;
    if (c8 < C8) {
      bf8 v = *reinterpret_cast<const bf8*>(x + (long long)row * ldx + c8 * 8);
      unpack8(v, f[k]);
#pragma unroll
      for (int j = 0; j < 8; ++j) s += f[k][j];
    }
  }
  const float mean = wave_sum(s) / C;
  float q = 0.f;
#pragma unroll
  for (int k = 0; k < LN_MAXCH; ++k) {
    if (lane + 64 * k < C8) {
#pragma unroll
      for (int j = 0; j < 8; ++j) { const float d = f[k][j] - mean; q = fmaf(d, d, q); }
    }
  }
  const float rstd = rsqrtf(wave_sum(q) / C + eps);
#pragma unroll
  for (int k = 0; k < LN_MAXCH; ++k) {
    const int c8 = lane + 64 * k;
    if (c8 < C8) {
      float o[8];
      bf8 gv = *reinterpret_cast<const bf8*>(gamma + c8 * 8);
      bf8 bv = *reinterpret_cast<const bf8*>(beta + c8 * 8);
      float gf[8], bf[8];
      unpack8(gv, gf);
      unpack8(bv, bf);
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = (f[k][j] - mean) * rstd * gf[j] + bf[j];
      *reinterpret_cast<bf8*>(y + (long long)row * ldy + c8 * 8) = pack8(o);
    }
  }
  if (lane == 0) { mean_out[row] = mean; rstd_out[row] = rstd; }
}

// dx = rstd * (g - mean(g) - xhat * mean(g*xhat)), g = dy*gamma; partial dgamma/dbeta per block
__global__ void __launch_bounds__(256) ln_bwd_kernel(const bf16_t* __restrict__ x, long long ldx,
                                                     const bf16_t* __restrict__ dy, long long lddy, bf16_t* __restrict__ dx,
                                                     long long lddx, int rows, int C, const bf16_t* __restrict__ gamma,
                                                     const float* __restrict__ mean_in, const float* __restrict__ rstd_in,
                                                     float* __restrict__ part, int accumulate) {
  extern __shared__ float sp[];    // [4 waves][2][C]
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int C8 = C >> 3;
  float dgp[LN_MAXCH][8], dbp[LN_MAXCH][8], gm[LN_MAXCH][8];
#pragma unroll
  for (int k = 0; k < LN_MAXCH; ++k)
#pragma unroll
    for (int j = 0; j < 8; ++j) { dgp[k][j] = 0.f; dbp[k][j] = 0.f; gm[k][j] = 0.f; }
#pragma unroll
  for (int k = 0; k < LN_MAXCH; ++k)
    if (lane + 64 * k < C8) { bf8 gv = *reinterpret_cast<const bf8*>(gamma + (lane + 64 * k) * 8); unpack8(gv, gm[k]); }
  for (int row = blockIdx.x * 4 + w; row < rows; row += gridDim.x * 4) {
    const float mean = mean_in[row], rstd = rstd_in[row];
    float xh[LN_MAXCH][8], g[LN_MAXCH][8], dyv[LN_MAXCH][8];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int k = 0; k < LN_MAXCH; ++k) {
      const int c8 = lane + 64 * k;
      if (c8 < C8) {
        bf8 xv = *reinterpret_cast<const bf8*>(x + (long long)row * ldx + c8 * 8);
        bf8 dv = *reinterpret_cast<const bf8*>(dy + (long long)row * lddy + c8 * 8);
        float xf[8];
        unpack8(xv, xf);
        unpack8(dv, dyv[k]);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          xh[k][j] = (xf[j] - mean) * rstd;
          g[k][j] = dyv[k][j] * gm[k][j];
          s1 += g[k][j];
          s2 = fmaf(g[k][j], xh[k][j], s2);
          dgp[k][j] = fmaf(dyv[k][j], xh[k][j], dgp[k][j]);
          dbp[k][j] += dyv[k][j];
        }
      }
    }
    const float m1 = wave_sum(s1) / C, m2 = wave_sum(s2) / C;
#pragma unroll
    for (int k = 0; k < LN_MAXCH; ++k) {
      const int c8 = lane + 64 * k;
      if (c8 < C8) {
        float o[8];
        float prev[8];
        if (accumulate) { bf8 pv = *reinterpret_cast<const bf8*>(dx + (long long)row * lddx + c8 * 8); unpack8(pv, prev); }
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          o[j] = rstd * (g[k][j] - m1 - xh[k][j] * m2);
          if (accumulate) o[j] += prev[j];
        }
        *reinterpret_cast<bf8*>(dx + (long long)row * lddx + c8 * 8) = pack8(o);
      }
    }
  }
  // block reduce of dgamma/dbeta partials
#pragma unroll
  for (int k = 0; k < LN_MAXCH; ++k) {
    const int c8 = lane + 64 * k;
    if (c8 < C8)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        sp[(w * 2) * C + c8 * 8 + j] = dgp[k][j];
        sp[(w * 2 + 1) * C + c8 * 8 + j] = dbp[k][j];
      }
  }
  __syncthreads();
  for (int c = threadIdx.x; c < C; c += 256) {
    float dg = 0.f, db = 0.f;
    for (int ww = 0; ww < 4; ++ww) { dg += sp[(ww * 2) * C + c]; db += sp[(ww * 2 + 1) * C + c]; }
    part[(long long)blockIdx.x * 2 * C + c] = dg;
    part[(long long)blockIdx.x * 2 * C + C + c] = db;
  }
}

// sum block partials [nb][2][C] -> dgamma[C], dbeta[C] (fp32).  block: 32 columns x 8 partial-lanes
__device__ __forceinline__ void store_param_grad(void* p, long long i, float v, int f32, int acc) {
  if (f32) { float* d = reinterpret_cast<float*>(p) + i; *d = acc ? *d + v : v; }
  else { bf16_t* d = reinterpret_cast<bf16_t*>(p) + i; *d = f2bf(acc ? bf2f(*d) + v : v); }
}

__global__ void __launch_bounds__(256) ln_param_reduce_kernel(const float* __restrict__ part, int nb, int C,
                                                              void* __restrict__ dgamma, void* __restrict__ dbeta,
                                                              int pf32, int pacc) {
  __shared__ float red[8][33];
  const int cl = threadIdx.x & 31, pl = threadIdx.x >> 5;
  const int c = blockIdx.x * 32 + cl;
  float s0 = 0.f, s1 = 0.f;
  if (c < 2 * C) {
    int b = pl;
    for (; b + 8 < nb; b += 16) {
      s0 += part[(long long)b * 2 * C + c];
      s1 += part[(long long)(b + 8) * 2 * C + c];
    }
    for (; b < nb; b += 8) s0 += part[(long long)b * 2 * C + c];
  }
  red[pl][cl] = s0 + s1;
  __syncthreads();
  if (pl == 0 && c < 2 * C) {
    float t = 0.f;
#pragma unroll
    for (int k = 0; k < 8; ++k) t += red[k][cl];
    if (c < C) store_param_grad(dgamma, c, t, pf32, pacc); else store_param_grad(dbeta, c - C, t, pf32, pacc);
  }
}

OTAMD_API int otamd_layernorm_fwd(const void* x, long long ldx, void* y, long long ldy, int rows, int C, float eps,
                                  const void* gamma, const void* beta, float* mean, float* rstd, hipStream_t stream) {
  if (!x || !y || !gamma || !beta || !mean || !rstd || rows < 0 || C % 8 || C > 64 * 8 * LN_MAXCH) return OTAMD_EINVAL;
  if (ldx % 8 || ldy % 8 || (((uintptr_t)x | (uintptr_t)y | (uintptr_t)gamma | (uintptr_t)beta) & 15)) return OTAMD_EINVAL;
  if (rows == 0) return OTAMD_OK;
  ln_fwd_kernel<<<(rows + 3) / 4, 256, 0, stream>>>((const bf16_t*)x, ldx, (bf16_t*)y, ldy, rows, C, eps,
                                                    (const bf16_t*)gamma, (const bf16_t*)beta, mean, rstd);
  OTAMD_CHECK_LAUNCH();
  return OTAMD_OK;
}

// part: float scratch >= 1024 * 2 * C
OTAMD_API int otamd_layernorm_bwd(const void* x, long long ldx, const void* dy, long long lddy, void* dx,
                                  long long lddx, int rows, int C, const void* gamma, const float* mean,
                                  const float* rstd, void* dgamma, void* dbeta, int param_f32, int param_acc,
                                  float* part, int accumulate, hipStream_t stream) {
  // dgamma == dbeta == nullptr: frozen affine (LoRA training), no parameter-gradient reduce
  if (!x || !dy || !dx || !gamma || !mean || !rstd || (!dgamma != !dbeta) || !part) return OTAMD_EINVAL;
  if (rows <= 0 || C % 8 || C > 64 * 8 * LN_MAXCH || ldx % 8 || lddy % 8 || lddx % 8) return OTAMD_EINVAL;
  if (((uintptr_t)x | (uintptr_t)dy | (uintptr_t)dx | (uintptr_t)gamma) & 15) return OTAMD_EINVAL;
  int nb = (rows + 3) / 4;
  if (nb > 512) nb = 512;
  ln_bwd_kernel<<<nb, 256, 8 * C * sizeof(float), stream>>>((const bf16_t*)x, ldx, (const bf16_t*)dy, lddy,
                                                            (bf16_t*)dx, lddx, rows, C, (const bf16_t*)gamma, mean,
                                                            rstd, part, accumulate);
  OTAMD_CHECK_LAUNCH();
  if (!dgamma) return OTAMD_OK;
  ln_param_reduce_kernel<<<(2 * C + 31) / 32, 256, 0, stream>>>(part, nb, C, dgamma, dbeta, param_f32, param_acc);
  OTAMD_CHECK_LAUNCH();
  return OTAMD_OK;
}
