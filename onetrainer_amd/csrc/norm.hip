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

#include <stdlib.h>
#include <mutex>
#include <unordered_map>

__device__ __forceinline__ void store_param_grad(void* p, long long i, float v, int f32, int acc);

// ------------------------------------------------------------------------------------------
// Pixel-loop structure (all four passes): a block of C8 * PPP threads (PPP = max(1, 256 / C8)
// pixels per pass) gives each thread ONE fixed 8-channel chunk, so its per-channel constants
// live in registers and every load is a 16-byte chunk; the thread walks pixels p = p0 + lane_pix,
// p0 + lane_pix + PPP, ... of the block's pixel range, 4 pixels per iteration in flight.
// Reductions write per-block partial slabs (no atomics, deterministic); a finalize kernel folds
// blocks and channels into the (n, group) constants.
static inline int gn_threads(int C8) { return C8 * (C8 >= 256 ? 1 : 256 / C8); }

__device__ __forceinline__ void gn_coef8(const float* __restrict__ p, float (&v)[8]) {
  const float4 u0 = *reinterpret_cast<const float4*>(p), u1 = *reinterpret_cast<const float4*>(p + 4);
  v[0] = u0.x; v[1] = u0.y; v[2] = u0.z; v[3] = u0.w; v[4] = u1.x; v[5] = u1.y; v[6] = u1.z; v[7] = u1.w;
}

// fwd pass 1: part[blk][0|1][c] = sum x, sum x^2 over the block's pixels of image n = blockIdx.y
__global__ void __launch_bounds__(512) gn_stats_kernel(const bf16_t* __restrict__ x, long long ldx, int HW, int C,
                                                       int pix_per_block, float* __restrict__ part) {
  extern __shared__ float sred[];   // [PPP][2][C]
  const int n = blockIdx.y;
  const int C8 = C >> 3;
  const int PPP = blockDim.x / C8;
  const int t = threadIdx.x, c8 = t % C8, lp = t / C8;
  const int p0 = blockIdx.x * pix_per_block, p1 = min(HW, p0 + pix_per_block);
  const bf16_t* xb = x + (long long)n * HW * ldx + c8 * 8;
  float s[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f}, q[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  int p = p0 + lp;
  for (; p + 3 * PPP < p1; p += 4 * PPP) {
    bf8 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = *reinterpret_cast<const bf8*>(xb + (long long)(p + u * PPP) * ldx);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      float f[8];
      unpack8(v[u], f);
#pragma unroll
      for (int j = 0; j < 8; ++j) { s[j] += f[j]; q[j] = fmaf(f[j], f[j], q[j]); }
    }
  }
  for (; p < p1; p += PPP) {
    float f[8];
    unpack8(*reinterpret_cast<const bf8*>(xb + (long long)p * ldx), f);
#pragma unroll
    for (int j = 0; j < 8; ++j) { s[j] += f[j]; q[j] = fmaf(f[j], f[j], q[j]); }
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) { sred[(lp * 2) * C + c8 * 8 + j] = s[j]; sred[(lp * 2 + 1) * C + c8 * 8 + j] = q[j]; }
  __syncthreads();
  float* dst = part + ((long long)n * gridDim.x + blockIdx.x) * 2 * C;
  for (int i = t; i < 2 * C; i += blockDim.x) {
    const int w = i / C, c = i - w * C;
    float acc = 0.f;
    for (int k = 0; k < PPP; ++k) acc += sred[(k * 2 + w) * C + c];
    dst[i] = acc;
  }
}

// sum the per-block partial slabs over blocks in double: out[n][i] = sum_blk part[n][blk][i], i < 2C.
// grid (ceil(2C / 16), N), block 1024 = 16 columns x 64 partial lanes: lane p sums blocks p, p + 64, ... (a few loads
// in flight each), the 64 partials are folded in lane order (deterministic).  (64 columns x 16 lanes ran 16
// dependent iterations per lane over ~40 blocks: 8.4 us per launch in the SDXL step.)
__global__ void __launch_bounds__(1024) gn_colreduce_kernel(const float* __restrict__ part, int nblk, int C2,
                                                            double* __restrict__ out) {
  __shared__ double red[64][17];
  const int cl = threadIdx.x & 15, pl = threadIdx.x >> 4;
  const int n = blockIdx.y, i = blockIdx.x * 16 + cl;
  double s = 0.0;
  if (i < C2) {
    const float* pb = part + (long long)n * nblk * C2 + i;
    for (int blk = pl; blk < nblk; blk += 64) s += pb[(long long)blk * C2];
  }
  red[pl][cl] = s;
  __syncthreads();
  if (pl == 0 && i < C2) {
    double t = 0.0;
    for (int k = 0; k < 64; ++k) t += red[k][cl];
    out[(long long)n * C2 + i] = t;
  }
}

// fold channel sums into groups: mean / rstd per (n, g); a = rstd*gamma, b = beta - mean*a per (n, c).
// sums: [N][2][C] double (sum x, sum x^2).  One wave per (group, image): the group's channel sums split over the
// lanes and folded by a fixed xor butterfly (deterministic); grid (G, N).  The one-block-per-image form walked the
// groups' channels serially (a dependent chain of global loads per group: 8.6 us per launch in the SDXL step).
__global__ void __launch_bounds__(64) gn_finalize_g_kernel(const double* __restrict__ sums, int HW, int C, int G,
                                                           float eps, const bf16_t* __restrict__ gamma,
                                                           const bf16_t* __restrict__ beta, float* __restrict__ mean_out,
                                                           float* __restrict__ rstd_out, float* __restrict__ a_out,
                                                           float* __restrict__ b_out) {
  const int g = blockIdx.x, n = blockIdx.y, lane = threadIdx.x;
  const int Cg = C / G, c0 = g * Cg;
  const double* s = sums + (long long)n * 2 * C;
  double sm = 0, sq = 0;
  for (int c = c0 + lane; c < c0 + Cg; c += 64) { sm += s[c]; sq += s[C + c]; }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) { sm += __shfl_xor(sm, o, 64); sq += __shfl_xor(sq, o, 64); }
  const double cnt = (double)HW * Cg;
  const double mean = sm / cnt;
  double var = sq / cnt - mean * mean;
  if (var < 0) var = 0;
  const float m = (float)mean, r = (float)(1.0 / sqrt(var + (double)eps));
  if (lane == 0) { mean_out[n * G + g] = m; rstd_out[n * G + g] = r; }
  for (int c = c0 + lane; c < c0 + Cg; c += 64) {
    const float gm = gamma ? bf2f(gamma[c]) : 1.f;
    const float bt = beta ? bf2f(beta[c]) : 0.f;
    const float av = r * gm;
    a_out[n * C + c] = av;
    b_out[n * C + c] = bt - m * av;
  }
}

// y = [silu](x * a[n,c] + b[n,c])
template <bool SILU>
__global__ void __launch_bounds__(512) gn_apply_kernel(const bf16_t* __restrict__ x, long long ldx, bf16_t* __restrict__ y,
                                                       long long ldy, int HW, int C, int pix_per_block,
                                                       const float* __restrict__ a, const float* __restrict__ b) {
  const int n = blockIdx.y;
  const int C8 = C >> 3;
  const int PPP = blockDim.x / C8;
  const int t = threadIdx.x, c8 = t % C8, lp = t / C8;
  float av[8], bv[8];
  gn_coef8(a + (long long)n * C + c8 * 8, av);
  gn_coef8(b + (long long)n * C + c8 * 8, bv);
  const int p0 = blockIdx.x * pix_per_block, p1 = min(HW, p0 + pix_per_block);
  const bf16_t* xb = x + (long long)n * HW * ldx + c8 * 8;
  bf16_t* yb = y + (long long)n * HW * ldy + c8 * 8;
  int p = p0 + lp;
  for (; p + 3 * PPP < p1; p += 4 * PPP) {
    bf8 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = *reinterpret_cast<const bf8*>(xb + (long long)(p + u * PPP) * ldx);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      float f[8];
      unpack8(v[u], f);
#pragma unroll
      for (int j = 0; j < 8; ++j) { const float z = fmaf(f[j], av[j], bv[j]); f[j] = SILU ? silu_f(z) : z; }
      *reinterpret_cast<bf8*>(yb + (long long)(p + u * PPP) * ldy) = pack8(f);
    }
  }
  for (; p < p1; p += PPP) {
    float f[8];
    unpack8(*reinterpret_cast<const bf8*>(xb + (long long)p * ldx), f);
#pragma unroll
    for (int j = 0; j < 8; ++j) { const float z = fmaf(f[j], av[j], bv[j]); f[j] = SILU ? silu_f(z) : z; }
    *reinterpret_cast<bf8*>(yb + (long long)p * ldy) = pack8(f);
  }
}

// backward pass 1: part[blk][0|1][c] = sum dz, sum dz * xhat   (dz = dy * silu'(z) when SILU)
template <bool SILU>
__global__ void __launch_bounds__(512) gn_bwd_reduce_kernel(const bf16_t* __restrict__ x, long long ldx,
                                                            const bf16_t* __restrict__ dy, long long lddy, int HW, int C,
                                                            int G, int pix_per_block, const float* __restrict__ a,
                                                            const float* __restrict__ b, const float* __restrict__ mean,
                                                            const float* __restrict__ rstd, float* __restrict__ part) {
  extern __shared__ float sred[];   // [PPP][2][C]
  const int n = blockIdx.y;
  const int C8 = C >> 3;
  const int PPP = blockDim.x / C8;
  const int Cg = C / G;
  const int t = threadIdx.x, c8 = t % C8, lp = t / C8;
  float av[8], bv[8], mv[8], rv[8];
  gn_coef8(a + (long long)n * C + c8 * 8, av);
  gn_coef8(b + (long long)n * C + c8 * 8, bv);
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int g = (c8 * 8 + j) / Cg;
    mv[j] = mean[n * G + g];
    rv[j] = rstd[n * G + g];
  }
  const int p0 = blockIdx.x * pix_per_block, p1 = min(HW, p0 + pix_per_block);
  const bf16_t* xb = x + (long long)n * HW * ldx + c8 * 8;
  const bf16_t* gb = dy + (long long)n * HW * lddy + c8 * 8;
  float s[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f}, q[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  auto body = [&](const bf8& xv, const bf8& gv) {
    float xf[8], gf[8];
    unpack8(xv, xf);
    unpack8(gv, gf);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float dz = gf[j];
      if (SILU) dz *= dsilu_f(fmaf(xf[j], av[j], bv[j]));
      s[j] += dz;
      q[j] = fmaf(dz, (xf[j] - mv[j]) * rv[j], q[j]);
    }
  };
  int p = p0 + lp;
  for (; p + PPP < p1; p += 2 * PPP) {
    const bf8 x0 = *reinterpret_cast<const bf8*>(xb + (long long)p * ldx);
    const bf8 g0 = *reinterpret_cast<const bf8*>(gb + (long long)p * lddy);
    const bf8 x1 = *reinterpret_cast<const bf8*>(xb + (long long)(p + PPP) * ldx);
    const bf8 g1 = *reinterpret_cast<const bf8*>(gb + (long long)(p + PPP) * lddy);
    body(x0, g0);
    body(x1, g1);
  }
  for (; p < p1; p += PPP)
    body(*reinterpret_cast<const bf8*>(xb + (long long)p * ldx), *reinterpret_cast<const bf8*>(gb + (long long)p * lddy));
#pragma unroll
  for (int j = 0; j < 8; ++j) { sred[(lp * 2) * C + c8 * 8 + j] = s[j]; sred[(lp * 2 + 1) * C + c8 * 8 + j] = q[j]; }
  __syncthreads();
  float* dst = part + ((long long)n * gridDim.x + blockIdx.x) * 2 * C;
  for (int i = t; i < 2 * C; i += blockDim.x) {
    const int w = i / C, c = i - w * C;
    float acc = 0.f;
    for (int k = 0; k < PPP; ++k) acc += sred[(k * 2 + w) * C + c];
    dst[i] = acc;
  }
}

// per (n, g) c1 = sum_c gamma S1 / cnt, c2 = sum_c gamma S2 / cnt from the block-summed
// sums [N][2][C] (S1 = sum dz, S2 = sum dz xhat), folded into the apply coefficients
// dx = A dz + B x + Cc with A = rstd gamma, B = -rstd^2 c2, Cc = rstd (mean rstd c2 - c1).
// coef: [3][N][C] fp32.  One wave per (group, image), grid (G, N), as gn_finalize_g_kernel (the serial
// one-block-per-image form took 13.9 us per launch)
__global__ void __launch_bounds__(64) gn_bwd_finalize_g_kernel(const double* __restrict__ sums, int N, int HW, int C,
                                                               int G, const bf16_t* __restrict__ gamma,
                                                               const float* __restrict__ mean,
                                                               const float* __restrict__ rstd, float* __restrict__ coef) {
  const int g = blockIdx.x, n = blockIdx.y, lane = threadIdx.x;
  const int Cg = C / G, c0 = g * Cg;
  const double* s1 = sums + (long long)n * 2 * C;
  const double* s2 = s1 + C;
  double a = 0, q = 0;
  for (int c = c0 + lane; c < c0 + Cg; c += 64) {
    const double gm = gamma ? bf2f(gamma[c]) : 1.0;
    a += gm * s1[c];
    q += gm * s2[c];
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) { a += __shfl_xor(a, o, 64); q += __shfl_xor(q, o, 64); }
  const float c1 = (float)(a / ((double)HW * Cg)), c2 = (float)(q / ((double)HW * Cg));
  const int ng = n * G + g;
  const float r = rstd[ng], m = mean[ng];
  for (int c = c0 + lane; c < c0 + Cg; c += 64) {
    const float gm = gamma ? bf2f(gamma[c]) : 1.f;
    coef[(long long)n * C + c] = r * gm;
    coef[(long long)(N + n) * C + c] = -r * r * c2;
    coef[(long long)(2 * N + n) * C + c] = r * (m * r * c2 - c1);
  }
}

// dgamma[c] = sum_n S2[n][c], dbeta[c] = sum_n S1[n][c]
__global__ void gn_param_grad_kernel(const double* __restrict__ sums, int N, int C, void* __restrict__ dgamma,
                                     void* __restrict__ dbeta, int pf32, int pacc) {
  for (int c = blockIdx.x * blockDim.x + threadIdx.x; c < C; c += gridDim.x * blockDim.x) {
    double dg = 0, db = 0;
    for (int n = 0; n < N; ++n) { db += sums[(long long)n * 2 * C + c]; dg += sums[(long long)n * 2 * C + C + c]; }
    if (dgamma) store_param_grad(dgamma, c, (float)dg, pf32, pacc);
    if (dbeta) store_param_grad(dbeta, c, (float)db, pf32, pacc);
  }
}

// dx = A dz + B x + Cc  (dz = dy * silu'(x a + b) when SILU)
template <bool SILU>
__global__ void __launch_bounds__(512) gn_bwd_apply_kernel(const bf16_t* __restrict__ x, long long ldx,
                                                           const bf16_t* __restrict__ dy, long long lddy,
                                                           bf16_t* __restrict__ dx, long long lddx, int N, int HW, int C,
                                                           int pix_per_block, const float* __restrict__ a,
                                                           const float* __restrict__ b, const float* __restrict__ coef,
                                                           int accumulate, const bf16_t* __restrict__ res = nullptr,
                                                           long long ldres = 0) {
  const int n = blockIdx.y;
  const int C8 = C >> 3;
  const int PPP = blockDim.x / C8;
  const int t = threadIdx.x, c8 = t % C8, lp = t / C8;
  float av[8], bv[8], A[8], Bv[8], Cc[8];
  gn_coef8(coef + (long long)n * C + c8 * 8, A);
  gn_coef8(coef + (long long)(N + n) * C + c8 * 8, Bv);
  gn_coef8(coef + (long long)(2 * N + n) * C + c8 * 8, Cc);
  if (SILU) {
    gn_coef8(a + (long long)n * C + c8 * 8, av);
    gn_coef8(b + (long long)n * C + c8 * 8, bv);
  }
  const int p0 = blockIdx.x * pix_per_block, p1 = min(HW, p0 + pix_per_block);
  const bf16_t* xb = x + (long long)n * HW * ldx + c8 * 8;
  const bf16_t* gb = dy + (long long)n * HW * lddy + c8 * 8;
  bf16_t* ob = dx + (long long)n * HW * lddx + c8 * 8;
  const bf16_t* rb = res ? res + (long long)n * HW * ldres + c8 * 8 : nullptr;
  auto body = [&](int pp, const bf8& xv, const bf8& gv) {
    float xf[8], gf[8], o[8];
    unpack8(xv, xf);
    unpack8(gv, gf);
    float prev[8];
    if (accumulate) unpack8(*reinterpret_cast<const bf8*>(ob + (long long)pp * lddx), prev);
    float rv[8];
    if (res) unpack8(*reinterpret_cast<const bf8*>(rb + (long long)pp * ldres), rv);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float dz = gf[j];
      if (SILU) dz *= dsilu_f(fmaf(xf[j], av[j], bv[j]));
      o[j] = fmaf(A[j], dz, fmaf(Bv[j], xf[j], Cc[j]));
      if (accumulate) o[j] += prev[j];
      if (res) o[j] += rv[j];
    }
    *reinterpret_cast<bf8*>(ob + (long long)pp * lddx) = pack8(o);
  };
  int p = p0 + lp;
  for (; p + PPP < p1; p += 2 * PPP) {
    const bf8 x0 = *reinterpret_cast<const bf8*>(xb + (long long)p * ldx);
    const bf8 g0 = *reinterpret_cast<const bf8*>(gb + (long long)p * lddy);
    const bf8 x1 = *reinterpret_cast<const bf8*>(xb + (long long)(p + PPP) * ldx);
    const bf8 g1 = *reinterpret_cast<const bf8*>(gb + (long long)(p + PPP) * lddy);
    body(p, x0, g0);
    body(p + PPP, x1, g1);
  }
  for (; p < p1; p += PPP)
    body(p, *reinterpret_cast<const bf8*>(xb + (long long)p * ldx), *reinterpret_cast<const bf8*>(gb + (long long)p * lddy));
}

// pixel blocks per image: enough blocks to cover the chip ~4x, >= 4 pixel passes per block
static int gn_pix_per_block(int N, int HW, int C8) {
  const int ppp = C8 >= 256 ? 1 : 256 / C8;
  int nb = std::max(1, (1024 + N - 1) / N);
  int ppb = (HW + nb - 1) / nb;
  ppb = std::max(ppb, 4 * ppp);
  ppb = (ppb + ppp - 1) / ppp * ppp;
  return ppb;
}

// scratch floats otamd_groupnorm_fwd / _bwd need (ws): partial slabs + coefficients + double sums
OTAMD_API long long otamd_groupnorm_ws_floats(int N, int HW, int C) {
  if (N <= 0 || HW <= 0 || C <= 0 || C % 8) return -1;
  const int ppb = gn_pix_per_block(N, HW, C / 8);
  const long long nblk = (HW + ppb - 1) / ppb;
  return (long long)N * nblk * 2 * C + 3LL * N * C + 4LL * N * C + 64;
}

// ws: otamd_groupnorm_ws_floats floats.  stats out (fp32): mean[N*G], rstd[N*G], a[N*C], b[N*C]
OTAMD_API int otamd_groupnorm_fwd(const void* x, long long ldx, void* y, long long ldy, int N, int HW, int C, int G,
                                  float eps, const void* gamma, const void* beta, int silu, float* mean, float* rstd,
                                  float* a, float* b, float* ws, hipStream_t stream) {
  if (!x || !y || !mean || !rstd || !a || !b || !ws || N <= 0 || HW <= 0 || C <= 0 || G <= 0) return OTAMD_EINVAL;
  if (C % 8 || C % G || ldx % 8 || ldy % 8 || ((uintptr_t)x & 15) || ((uintptr_t)y & 15) || C > 8192 ||
      ((uintptr_t)ws & 7))
    return OTAMD_EINVAL;
  const int C8 = C / 8, nt = gn_threads(C8);
  if (nt > 512) return OTAMD_EINVAL;
  const int ppb = gn_pix_per_block(N, HW, C8);
  dim3 grid((HW + ppb - 1) / ppb, N);
  const int ppp = nt / C8;
  gn_stats_kernel<<<grid, nt, ppp * 2 * C * sizeof(float), stream>>>((const bf16_t*)x, ldx, HW, C, ppb, ws);
  OTAMD_CHECK_LAUNCH();
  double* sums = reinterpret_cast<double*>(ws + (long long)N * grid.x * 2 * C + 3LL * N * C + ((3LL * N * C) & 1));
  gn_colreduce_kernel<<<dim3((2 * C + 15) / 16, N), 1024, 0, stream>>>(ws, grid.x, 2 * C, sums);
  OTAMD_CHECK_LAUNCH();
  gn_finalize_g_kernel<<<dim3(G, N), 64, 0, stream>>>(sums, HW, C, G, eps, (const bf16_t*)gamma, (const bf16_t*)beta,
                                                      mean, rstd, a, b);
  OTAMD_CHECK_LAUNCH();
  if (silu) gn_apply_kernel<true><<<grid, nt, 0, stream>>>((const bf16_t*)x, ldx, (bf16_t*)y, ldy, HW, C, ppb, a, b);
  else gn_apply_kernel<false><<<grid, nt, 0, stream>>>((const bf16_t*)x, ldx, (bf16_t*)y, ldy, HW, C, ppb, a, b);
  OTAMD_CHECK_LAUNCH();
  return OTAMD_OK;
}

// res (nullable): dx += res in the apply pass -- the input's gradient through its other (residual /
// shortcut) use, summed here instead of by a separate autograd add
static int groupnorm_bwd_impl(const void* x, long long ldx, const void* dy, long long lddy, void* dx, long long lddx,
                              int N, int HW, int C, int G, const void* gamma, int silu, const float* mean,
                              const float* rstd, const float* a, const float* b, void* dgamma, void* dbeta,
                              int param_f32, int param_acc, float* ws, int accumulate, const void* res,
                              long long ldres, hipStream_t stream) {
  if (!x || !dy || !dx || !mean || !rstd || !a || !b || !ws || N <= 0 || HW <= 0) return OTAMD_EINVAL;
  if (C % 8 || C % G || ldx % 8 || lddy % 8 || lddx % 8 || C > 8192 || ((uintptr_t)ws & 7)) return OTAMD_EINVAL;
  if (((uintptr_t)x | (uintptr_t)dy | (uintptr_t)dx) & 15) return OTAMD_EINVAL;
  if (res && (ldres % 8 || ((uintptr_t)res & 15) || accumulate)) return OTAMD_EINVAL;
  const int C8 = C / 8, nt = gn_threads(C8);
  if (nt > 512) return OTAMD_EINVAL;
  const int ppb = gn_pix_per_block(N, HW, C8);
  dim3 grid((HW + ppb - 1) / ppb, N);
  const int ppp = nt / C8;
  float* part = ws;
  float* coef = ws + (long long)N * grid.x * 2 * C;
  double* sums = reinterpret_cast<double*>(coef + 3LL * N * C + ((3LL * N * C) & 1));
  if (silu)
    gn_bwd_reduce_kernel<true><<<grid, nt, ppp * 2 * C * sizeof(float), stream>>>(
        (const bf16_t*)x, ldx, (const bf16_t*)dy, lddy, HW, C, G, ppb, a, b, mean, rstd, part);
  else
    gn_bwd_reduce_kernel<false><<<grid, nt, ppp * 2 * C * sizeof(float), stream>>>(
        (const bf16_t*)x, ldx, (const bf16_t*)dy, lddy, HW, C, G, ppb, a, b, mean, rstd, part);
  OTAMD_CHECK_LAUNCH();
  gn_colreduce_kernel<<<dim3((2 * C + 15) / 16, N), 1024, 0, stream>>>(part, grid.x, 2 * C, sums);
  OTAMD_CHECK_LAUNCH();
  gn_bwd_finalize_g_kernel<<<dim3(G, N), 64, 0, stream>>>(sums, N, HW, C, G, (const bf16_t*)gamma, mean, rstd, coef);
  OTAMD_CHECK_LAUNCH();
  if (dgamma || dbeta) {
    gn_param_grad_kernel<<<(C + 255) / 256, 256, 0, stream>>>(sums, N, C, dgamma, dbeta, param_f32, param_acc);
    OTAMD_CHECK_LAUNCH();
  }
  if (silu)
    gn_bwd_apply_kernel<true><<<grid, nt, 0, stream>>>((const bf16_t*)x, ldx, (const bf16_t*)dy, lddy, (bf16_t*)dx,
                                                        lddx, N, HW, C, ppb, a, b, coef, accumulate,
                                                        (const bf16_t*)res, ldres);
  else
    gn_bwd_apply_kernel<false><<<grid, nt, 0, stream>>>((const bf16_t*)x, ldx, (const bf16_t*)dy, lddy, (bf16_t*)dx,
                                                         lddx, N, HW, C, ppb, a, b, coef, accumulate,
                                                         (const bf16_t*)res, ldres);
  OTAMD_CHECK_LAUNCH();
  return OTAMD_OK;
}

// ws: otamd_groupnorm_ws_floats floats (8-byte aligned)
OTAMD_API int otamd_groupnorm_bwd(const void* x, long long ldx, const void* dy, long long lddy, void* dx,
                                  long long lddx, int N, int HW, int C, int G, const void* gamma, int silu,
                                  const float* mean, const float* rstd, const float* a, const float* b,
                                  void* dgamma, void* dbeta, int param_f32, int param_acc, float* ws,
                                  int accumulate, hipStream_t stream) {
  return groupnorm_bwd_impl(x, ldx, dy, lddy, dx, lddx, N, HW, C, G, gamma, silu, mean, rstd, a, b, dgamma, dbeta,
                            param_f32, param_acc, ws, accumulate, nullptr, 0, stream);
}

// dx = GroupNorm(+SiLU)-backward(dy) + dres in the apply pass (dres: the gradient of the GroupNorm input through
// its residual / shortcut use: ResnetBlock2D norm1 + shortcut, Transformer2DModel norm + proj_out residual)
OTAMD_API int otamd_groupnorm_bwd_res(const void* x, long long ldx, const void* dy, long long lddy, const void* dres,
                                      long long ldres, void* dx, long long lddx, int N, int HW, int C, int G,
                                      const void* gamma, int silu, const float* mean, const float* rstd, const float* a,
                                      const float* b, void* dgamma, void* dbeta, int param_f32, int param_acc,
                                      float* ws, hipStream_t stream) {
  if (!dres) return OTAMD_EINVAL;
  return groupnorm_bwd_impl(x, ldx, dy, lddy, dx, lddx, N, HW, C, G, gamma, silu, mean, rstd, a, b, dgamma, dbeta,
                            param_f32, param_acc, ws, 0, dres, ldres, stream);
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

// ---- LayerNorm, row-group form.  L = C8 / CPL lanes per row (a power of two <= 64), RPW = 64 / L
// rows per wave; lane li of a row owns the CPL 16-byte chunks c8 = li + L*k.  Several rows per wave
// with CPL loads per lane in flight keep enough bytes moving for HBM (one row per wave with
// 1-2 chunks per lane left LN at 15-30 % of the HBM roofline); reductions are xor-shuffles inside
// the row group.
__device__ __forceinline__ float group_sum(float v, int L) {
  for (int o = L >> 1; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

template <int CPL>
__global__ void __launch_bounds__(256) ln_fwd_rows_kernel(const bf16_t* __restrict__ x, long long ldx,
                                                          bf16_t* __restrict__ y, long long ldy, int rows, int C,
                                                          float eps, const bf16_t* __restrict__ gamma,
                                                          const bf16_t* __restrict__ beta, float* __restrict__ mean_out,
                                                          float* __restrict__ rstd_out, int L) {
  const int lane = threadIdx.x & 63;
  const int li = lane & (L - 1);
  const int RPW = 64 / L;
  const long long row = ((long long)blockIdx.x * 4 + (threadIdx.x >> 6)) * RPW + lane / L;
  const bool ok = row < rows;
  float f[CPL][8];
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < CPL; ++k) {
    if (ok) {
      unpack8(*reinterpret_cast<const bf8*>(x + row * ldx + (li + L * k) * 8), f[k]);
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) f[k][j] = 0.f;
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) s += f[k][j];
  }
  const float mean = group_sum(s, L) / C;
  float q = 0.f;
#pragma unroll
  for (int k = 0; k < CPL; ++k)
#pragma unroll
    for (int j = 0; j < 8; ++j) { const float d = f[k][j] - mean; q = fmaf(d, d, q); }
  const float rstd = rsqrtf(group_sum(q, L) / C + eps);
  if (!ok) return;
#pragma unroll
  for (int k = 0; k < CPL; ++k) {
    const int c8 = li + L * k;
    float gf[8], bf[8], o[8];
    unpack8(*reinterpret_cast<const bf8*>(gamma + c8 * 8), gf);
    unpack8(*reinterpret_cast<const bf8*>(beta + c8 * 8), bf);
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = (f[k][j] - mean) * rstd * gf[j] + bf[j];
    *reinterpret_cast<bf8*>(y + row * ldy + c8 * 8) = pack8(o);
  }
  if (li == 0) { mean_out[row] = mean; rstd_out[row] = rstd; }
}

// dx = rstd (g - mean(g) - xhat mean(g xhat)), g = dy gamma.  Grid-stride over row groups; the
// parameter gradients come from ln_param_part_kernel (per-lane dgamma/dbeta accumulators here cost
// ~16 VGPRs per chunk and pushed CPL=5 rows to one wave per SIMD).
template <int CPL>
__global__ void __launch_bounds__(256) ln_bwd_rows_kernel(const bf16_t* __restrict__ x, long long ldx,
                                                          const bf16_t* __restrict__ dy, long long lddy,
                                                          bf16_t* __restrict__ dx, long long lddx, int rows, int C,
                                                          const bf16_t* __restrict__ gamma,
                                                          const float* __restrict__ mean_in,
                                                          const float* __restrict__ rstd_in, int accumulate, int L,
                                                          const bf16_t* __restrict__ res = nullptr, long long ldres = 0) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int li = lane & (L - 1), RPW = 64 / L;
  const long long row = ((long long)blockIdx.x * 4 + w) * RPW + lane / L;
  if (row >= rows) return;
  const float mean = mean_in[row], rstd = rstd_in[row];
  // every HBM operand of the row is requested up front (x, dy and the residual gradient / previous dx
  // to add): issuing the add-in loads after the row reductions exposed a second full memory latency
  bf8 xr[CPL], dr[CPL], ar[CPL];
  const bf16_t* add = res ? res : (accumulate ? dx : nullptr);
  const long long ldadd = res ? ldres : lddx;
#pragma unroll
  for (int k = 0; k < CPL; ++k) {
    const int c8 = li + L * k;
    xr[k] = *reinterpret_cast<const bf8*>(x + row * ldx + c8 * 8);
    dr[k] = *reinterpret_cast<const bf8*>(dy + row * lddy + c8 * 8);
  }
  if (add) {
#pragma unroll
    for (int k = 0; k < CPL; ++k) ar[k] = *reinterpret_cast<const bf8*>(add + row * ldadd + (li + L * k) * 8);
  }
  float s1 = 0.f, s2 = 0.f;
#pragma unroll
  for (int k = 0; k < CPL; ++k) {
    float xf[8], dv[8], gm[8];
    unpack8(xr[k], xf);
    unpack8(dr[k], dv);
    unpack8(*reinterpret_cast<const bf8*>(gamma + (li + L * k) * 8), gm);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float g = dv[j] * gm[j];
      s1 += g;
      s2 = fmaf(g, (xf[j] - mean) * rstd, s2);
    }
  }
  // partial row groups: rows past the end returned above, so every lane of a live group is live
  const float m1 = group_sum(s1, L) / C, m2 = group_sum(s2, L) / C;
#pragma unroll
  for (int k = 0; k < CPL; ++k) {   // re-unpack below rather than keep the first pass's floats live
    opaque(xr[k]);
    opaque(dr[k]);
    if (add) opaque(ar[k]);
  }
#pragma unroll
  for (int k = 0; k < CPL; ++k) {
    const int c8 = li + L * k;
    float xf[8], dv[8], gm[8], o[8];
    unpack8(xr[k], xf);
    unpack8(dr[k], dv);
    unpack8(*reinterpret_cast<const bf8*>(gamma + c8 * 8), gm);
    float ad[8];
    if (add) unpack8(ar[k], ad);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      o[j] = rstd * (dv[j] * gm[j] - m1 - (xf[j] - mean) * rstd * m2);
      if (add) o[j] += ad[j];
    }
    *reinterpret_cast<bf8*>(dx + row * lddx + c8 * 8) = pack8(o);
  }
}

// dgamma / dbeta partials per row slab: part[slab][0|1][c] = sum_rows dy xhat | dy.  Column-tiled
// (lane = one 16-byte chunk, 64 chunks per block column, 8 waves stride the slab's rows) so every
// load is a coalesced row segment.  grid (ceil(C8 / 64), slabs), block 512
__global__ void __launch_bounds__(512) ln_param_part_kernel(const bf16_t* __restrict__ x, long long ldx,
                                                            const bf16_t* __restrict__ dy, long long lddy, int rows,
                                                            int C, const float* __restrict__ mean_in,
                                                            const float* __restrict__ rstd_in, int rps,
                                                            float* __restrict__ part) {
  __shared__ float red[8][2][8][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int C8 = C >> 3;
  const int c8 = blockIdx.x * 64 + lane;
  const bool ok = c8 < C8;
  const long long r0 = (long long)blockIdx.y * rps;
  const long long r1 = min((long long)rows, r0 + rps);
  float dg[8], db[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) { dg[j] = 0.f; db[j] = 0.f; }
  if (ok) {
    auto body = [&](const bf8& xv, const bf8& dvv, float m, float rs) {
      float xf[8], dv[8];
      unpack8(xv, xf);
      unpack8(dvv, dv);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        dg[j] = fmaf(dv[j], (xf[j] - m) * rs, dg[j]);
        db[j] += dv[j];
      }
    };
    long long r = r0 + w;
    // 4 rows (8 independent 16-byte loads) in flight per lane before any math
    for (; r + 24 < r1; r += 32) {
      bf8 xv[4], dv[4];
      float m[4], rs[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        xv[u] = *reinterpret_cast<const bf8*>(x + (r + 8 * u) * ldx + c8 * 8);
        dv[u] = *reinterpret_cast<const bf8*>(dy + (r + 8 * u) * lddy + c8 * 8);
        m[u] = mean_in[r + 8 * u];
        rs[u] = rstd_in[r + 8 * u];
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) body(xv[u], dv[u], m[u], rs[u]);
    }
    for (; r < r1; r += 8)
      body(*reinterpret_cast<const bf8*>(x + r * ldx + c8 * 8), *reinterpret_cast<const bf8*>(dy + r * lddy + c8 * 8),
           mean_in[r], rstd_in[r]);
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) { red[w][0][j][lane] = dg[j]; red[w][1][j][lane] = db[j]; }
  __syncthreads();
  for (int i = threadIdx.x; i < 2 * 8 * 64; i += 512) {
    const int wh = i >> 9, j = (i >> 6) & 7, l = i & 63;
    const int cc8 = blockIdx.x * 64 + l;
    if (cc8 >= C8) continue;
    float t = 0.f;
#pragma unroll
    for (int ww = 0; ww < 8; ++ww) t += red[ww][wh][j][l];
    part[(long long)blockIdx.y * 2 * C + wh * C + cc8 * 8 + j] = t;
  }
}

// chunks per lane for a row of C8 16-byte chunks: L = C8 / CPL a power of two <= 64 (0: no fit)
static int ln_pick(int C8, int* L) {
  const int cands[] = {5, 4, 3, 6, 2, 8, 1};
  for (int c : cands) {
    if (C8 % c) continue;
    const int l = C8 / c;
    if (l <= 64 && (l & (l - 1)) == 0) { *L = l; return c; }
  }
  return 0;
}

// sum block partials [nb][2][C] -> dgamma, dbeta: 16 columns x 64 partial lanes per block (as gn_colreduce_kernel:
// a few loads in flight per lane, the partials folded in lane order; 64 x 16 ran up to 32 dependent iterations per
// lane over 40 blocks, 5.4 us per launch in the SDXL step)
__device__ __forceinline__ void ln_param_reduce_body(const float* __restrict__ part, int nb, int C,
                                                     void* __restrict__ dgamma, void* __restrict__ dbeta, int pf32,
                                                     int pacc, int bx) {
  __shared__ float red[64][17];
  const int cl = threadIdx.x & 15, pl = threadIdx.x >> 4;
  const int c = bx * 16 + cl;
  float s = 0.f;
  if (c < 2 * C)
    for (int b = pl; b < nb; b += 64) s += part[(long long)b * 2 * C + c];
  red[pl][cl] = s;
  __syncthreads();
  if (pl == 0 && c < 2 * C) {
    float t = 0.f;
    for (int k = 0; k < 64; ++k) t += red[k][cl];
    if (c < C) store_param_grad(dgamma, c, t, pf32, pacc); else store_param_grad(dbeta, c - C, t, pf32, pacc);
  }
}

__global__ void __launch_bounds__(1024) ln_param_reduce2_kernel(const float* __restrict__ part, int nb, int C,
                                                                void* __restrict__ dgamma, void* __restrict__ dbeta,
                                                                int pf32, int pacc) {
  ln_param_reduce_body(part, nb, C, dgamma, dbeta, pf32, pacc, blockIdx.x);
}

// ---- deferred LayerNorm parameter reduces (otamd_layernorm_defer_*) ----------------------------------------------
// dgamma / dbeta only feed the optimizer, so on a deferring stream the parameter-gradient pass writes its per-slab
// partials into a caller-owned arena and the final sums of up to kLnMaxDefer LayerNorms go out in one grouped launch
// (each LayerNorm's columns summed exactly as ln_param_reduce2_kernel sums them: bit-identical).  210 reduce launches
// of ~5 us each per SDXL 1024^2 step otherwise sit on the critical stream.
struct LnDeferDesc {
  const float* part; void* dg; void* db;
  int nb, C, flags;   // flags: 1 fp32 destinations, 2 accumulate
  unsigned block0;
};
constexpr int kLnMaxDefer = 64;
struct LnDeferBatch { int n; unsigned blocks; LnDeferDesc d[kLnMaxDefer]; };

__global__ void __launch_bounds__(1024) ln_param_reduce_grouped_kernel(LnDeferBatch bt) {
  int i = 0;
  while (i + 1 < bt.n && blockIdx.x >= bt.d[i + 1].block0) ++i;
  const LnDeferDesc& d = bt.d[i];
  ln_param_reduce_body(d.part, d.nb, d.C, d.dg, d.db, d.flags & 1, (d.flags >> 1) & 1, blockIdx.x - d.block0);
}

struct LnDeferState {
  char* arena = nullptr;
  long long bytes = 0, used = 0;
  LnDeferBatch batch{};
};
static std::mutex g_ln_defer_mu;
static std::unordered_map<hipStream_t, LnDeferState> g_ln_defer;
static long long g_ln_defer_norms = 0, g_ln_defer_launches = 0;

static void ln_defer_flush_locked(LnDeferState& st, hipStream_t stream) {
  if (st.batch.n > 0) {
    ln_param_reduce_grouped_kernel<<<st.batch.blocks, 1024, 0, stream>>>(st.batch);
    g_ln_defer_norms += st.batch.n;
    ++g_ln_defer_launches;
    st.batch.n = 0;
    st.batch.blocks = 0;
  }
  st.used = 0;
}

// partial slab memory for one LayerNorm's parameter pass on a deferring stream (nullptr: not deferring, or the
// partials do not fit the arena).  A pending reduce into the same dgamma / dbeta is flushed first (two grouped
// reduces of one destination would race).
static float* ln_defer_slot(long long need, const void* dg, const void* db, hipStream_t stream) {
  std::lock_guard<std::mutex> lk(g_ln_defer_mu);
  auto it = g_ln_defer.find(stream);
  if (it == g_ln_defer.end()) return nullptr;
  LnDeferState& st = it->second;
  need = (need + 255) / 256 * 256;
  if (need > st.bytes) return nullptr;
  bool clash = false;
  for (int i = 0; i < st.batch.n && !clash; ++i) clash = st.batch.d[i].dg == dg || st.batch.d[i].db == db;
  if (clash || st.batch.n == kLnMaxDefer || st.used + need > st.bytes) ln_defer_flush_locked(st, stream);
  float* p = reinterpret_cast<float*>(st.arena + st.used);
  st.used += need;
  return p;
}

static void ln_defer_record(const float* part, int nb, int C, void* dg, void* db, int f32, int acc,
                            hipStream_t stream) {
  std::lock_guard<std::mutex> lk(g_ln_defer_mu);
  LnDeferState& st = g_ln_defer[stream];
  LnDeferDesc& d = st.batch.d[st.batch.n++];
  d.part = part; d.dg = dg; d.db = db; d.nb = nb; d.C = C; d.flags = (f32 ? 1 : 0) | (acc ? 2 : 0);
  d.block0 = st.batch.blocks;
  st.batch.blocks += (unsigned)((2 * C + 15) / 16);
}

// start deferring this stream's LayerNorm parameter reduces into `arena` (>= 1 MiB, 256-byte aligned, kept alive by
// the caller until otamd_layernorm_defer_end); reduces pending from an earlier begin are flushed first
OTAMD_API int otamd_layernorm_defer_begin(hipStream_t stream, void* arena, long long bytes) {
  if (!arena || ((uintptr_t)arena & 255) || bytes < (1 << 20)) return OTAMD_EINVAL;
  std::lock_guard<std::mutex> lk(g_ln_defer_mu);
  LnDeferState& st = g_ln_defer[stream];
  ln_defer_flush_locked(st, stream);
  st.arena = (char*)arena;
  st.bytes = bytes;
  st.used = 0;
  OTAMD_CHECK_LAUNCH();
  return OTAMD_OK;
}
// launch the grouped reduce of every pending LayerNorm on this stream (stream-ordered); a no-op when none is pending
OTAMD_API int otamd_layernorm_defer_flush(hipStream_t stream) {
  std::lock_guard<std::mutex> lk(g_ln_defer_mu);
  auto it = g_ln_defer.find(stream);
  if (it != g_ln_defer.end()) ln_defer_flush_locked(it->second, stream);
  OTAMD_CHECK_LAUNCH();
  return OTAMD_OK;
}
// flush and leave defer mode; the pending reduces go out on `launch` (the caller orders it after `stream`'s
// parameter passes: the two-stream step flushes on the weight-gradient stream, whose join ends the backward)
OTAMD_API int otamd_layernorm_defer_end_on(hipStream_t stream, hipStream_t launch) {
  std::lock_guard<std::mutex> lk(g_ln_defer_mu);
  auto it = g_ln_defer.find(stream);
  if (it == g_ln_defer.end()) return OTAMD_OK;
  ln_defer_flush_locked(it->second, launch);
  g_ln_defer.erase(it);
  OTAMD_CHECK_LAUNCH();
  return OTAMD_OK;
}
OTAMD_API int otamd_layernorm_defer_end(hipStream_t stream) { return otamd_layernorm_defer_end_on(stream, stream); }
// out[0] = LayerNorms whose parameter reduce went out deferred, out[1] = grouped launches, out[2] = pending on stream
OTAMD_API int otamd_layernorm_defer_stats(hipStream_t stream, long long* out) {
  if (!out) return OTAMD_EINVAL;
  std::lock_guard<std::mutex> lk(g_ln_defer_mu);
  out[0] = g_ln_defer_norms;
  out[1] = g_ln_defer_launches;
  auto it = g_ln_defer.find(stream);
  out[2] = it == g_ln_defer.end() ? 0 : it->second.batch.n;
  return OTAMD_OK;
}

static int ln_param_grads(const void* x, long long ldx, const void* dy, long long lddy, int rows, int C,
                          const float* mean, const float* rstd, void* dgamma, void* dbeta, int param_f32,
                          int param_acc, float* part, hipStream_t stream);

OTAMD_API int otamd_layernorm_fwd(const void* x, long long ldx, void* y, long long ldy, int rows, int C, float eps,
                                  const void* gamma, const void* beta, float* mean, float* rstd, hipStream_t stream) {
  if (!x || !y || !gamma || !beta || !mean || !rstd || rows < 0 || C % 8 || C > 64 * 8 * LN_MAXCH) return OTAMD_EINVAL;
  if (ldx % 8 || ldy % 8 || (((uintptr_t)x | (uintptr_t)y | (uintptr_t)gamma | (uintptr_t)beta) & 15)) return OTAMD_EINVAL;
  if (rows == 0) return OTAMD_OK;
  int L = 0;
  const int cpl = ln_pick(C / 8, &L);
  if (cpl) {
    const int rpb = 4 * (64 / L);
    const int nb = (rows + rpb - 1) / rpb;
#define LNF(K) ln_fwd_rows_kernel<K><<<nb, 256, 0, stream>>>((const bf16_t*)x, ldx, (bf16_t*)y, ldy, rows, C, eps, \
                                                            (const bf16_t*)gamma, (const bf16_t*)beta, mean, rstd, L)
    switch (cpl) {
      case 1: LNF(1); break;
      case 2: LNF(2); break;
      case 3: LNF(3); break;
      case 4: LNF(4); break;
      case 5: LNF(5); break;
      case 6: LNF(6); break;
      default: LNF(8); break;
    }
#undef LNF
    OTAMD_CHECK_LAUNCH();
    return OTAMD_OK;
  }
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
  int L = 0;
  const int cpl = ln_pick(C / 8, &L);
  if (cpl) {
    const int rpb = 4 * (64 / L);
    const int nbr = (rows + rpb - 1) / rpb;
#define LNB(K) ln_bwd_rows_kernel<K><<<nbr, 256, 0, stream>>>((const bf16_t*)x, ldx, (const bf16_t*)dy, lddy, \
                                                              (bf16_t*)dx, lddx, rows, C, (const bf16_t*)gamma, mean, \
                                                              rstd, accumulate, L)
    switch (cpl) {
      case 1: LNB(1); break;
      case 2: LNB(2); break;
      case 3: LNB(3); break;
      case 4: LNB(4); break;
      case 5: LNB(5); break;
      case 6: LNB(6); break;
      default: LNB(8); break;
    }
#undef LNB
    OTAMD_CHECK_LAUNCH();
    if (!dgamma) return OTAMD_OK;
    return ln_param_grads(x, ldx, dy, lddy, rows, C, mean, rstd, dgamma, dbeta, param_f32, param_acc, part, stream);
  }
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

// dgamma / dbeta only (the dx pass ran with dgamma == nullptr): lets the parameter-gradient reduction
// run on the weight-gradient side stream, off the critical dgrad chain (module/streams.py).
// part: float scratch >= 1024 * 2 * C
OTAMD_API int otamd_layernorm_param_grad(const void* x, long long ldx, const void* dy, long long lddy, int rows,
                                         int C, const float* mean, const float* rstd, void* dgamma, void* dbeta,
                                         int param_f32, int param_acc, float* part, hipStream_t stream) {
  if (!x || !dy || !mean || !rstd || !dgamma || !dbeta || !part) return OTAMD_EINVAL;
  if (rows <= 0 || C % 8 || C > 64 * 8 * LN_MAXCH || ldx % 8 || lddy % 8) return OTAMD_EINVAL;
  if (((uintptr_t)x | (uintptr_t)dy) & 15) return OTAMD_EINVAL;
  return ln_param_grads(x, ldx, dy, lddy, rows, C, mean, rstd, dgamma, dbeta, param_f32, param_acc, part, stream);
}

// dx = LayerNorm-backward(dy) + dres in one pass: the LayerNorm input is also the block's residual
// (BasicTransformerBlock norm1/2/3 + to_out / ff residual), so the two gradient contributions are
// summed here instead of by a separate autograd add.  dgamma / dbeta: otamd_layernorm_param_grad.
OTAMD_API int otamd_layernorm_bwd_res(const void* x, long long ldx, const void* dy, long long lddy, const void* dres,
                                      long long ldres, void* dx, long long lddx, int rows, int C, const void* gamma,
                                      const float* mean, const float* rstd, hipStream_t stream) {
  if (!x || !dy || !dres || !dx || !gamma || !mean || !rstd) return OTAMD_EINVAL;
  if (rows <= 0 || C % 8 || C > 64 * 8 * LN_MAXCH || ldx % 8 || lddy % 8 || lddx % 8 || ldres % 8) return OTAMD_EINVAL;
  if (((uintptr_t)x | (uintptr_t)dy | (uintptr_t)dx | (uintptr_t)dres | (uintptr_t)gamma) & 15) return OTAMD_EINVAL;
  int L = 0;
  const int cpl = ln_pick(C / 8, &L);
  if (!cpl) return OTAMD_EUNSUPPORTED;
  const int rpb = 4 * (64 / L);
  const int nbr = (rows + rpb - 1) / rpb;
#define LNBR(K) ln_bwd_rows_kernel<K><<<nbr, 256, 0, stream>>>((const bf16_t*)x, ldx, (const bf16_t*)dy, lddy, \
                                                               (bf16_t*)dx, lddx, rows, C, (const bf16_t*)gamma, mean, \
                                                               rstd, 0, L, (const bf16_t*)dres, ldres)
  switch (cpl) {
    case 1: LNBR(1); break;
    case 2: LNBR(2); break;
    case 3: LNBR(3); break;
    case 4: LNBR(4); break;
    case 5: LNBR(5); break;
    case 6: LNBR(6); break;
    default: LNBR(8); break;
  }
#undef LNBR
  OTAMD_CHECK_LAUNCH();
  return OTAMD_OK;
}

static int ln_param_grads(const void* x, long long ldx, const void* dy, long long lddy, int rows, int C,
                          const float* mean, const float* rstd, void* dgamma, void* dbeta, int param_f32,
                          int param_acc, float* part, hipStream_t stream) {
  {
    // ~512 blocks of >= 32 rows (4 per wave, one unrolled batch), at most 512 slabs (the part buffer holds
    // 1024 x 2C floats): few slabs keep the second (reduce) pass short -- with 16-row slabs both passes were
    // latency-bound (~11 us + ~8.5 us per LayerNorm at 4096 x 1280)
    // workgroups per parameter pass: 512 (two per CU) measured -0.11 ms per SDXL step against 256 once the slab
    // reduce went out grouped (profiles/r5_ln_param_blocks_ab.txt); OTAMD_LN_PARAM_BLOCKS overrides (A/B)
    static const int target = [] {
      const char* e = getenv("OTAMD_LN_PARAM_BLOCKS");
      const int v = e ? atoi(e) : 0;
      return v > 0 ? v : 512;
    }();
    const int cb = (C / 8 + 63) / 64;
    int slabs = (target + cb - 1) / cb;
    slabs = min(slabs, max(1, rows / 32));
    slabs = min(slabs, 512);
    const int rps = (rows + slabs - 1) / slabs;
    slabs = (rows + rps - 1) / rps;
    float* dpart = ln_defer_slot((long long)slabs * 2 * C * sizeof(float), dgamma, dbeta, stream);
    ln_param_part_kernel<<<dim3(cb, slabs), 512, 0, stream>>>((const bf16_t*)x, ldx, (const bf16_t*)dy, lddy, rows, C,
                                                              mean, rstd, rps, dpart ? dpart : part);
    OTAMD_CHECK_LAUNCH();
    if (dpart) {
      ln_defer_record(dpart, slabs, C, dgamma, dbeta, param_f32, param_acc, stream);
      return OTAMD_OK;
    }
    ln_param_reduce2_kernel<<<(2 * C + 15) / 16, 1024, 0, stream>>>(part, slabs, C, dgamma, dbeta, param_f32, param_acc);
    OTAMD_CHECK_LAUNCH();
    return OTAMD_OK;
  }
}
