// HBM-bound helper kernels of the UNet step (all 16-byte vectorized, grid-stride):
//   GEGLU fwd/bwd (diffusers GEGLU: hidden, gate = proj(x).chunk(2); hidden * gelu(gate)),
//   SiLU fwd/bwd, channel concat (skip connections), nearest-2x upsample backward (2x2 sum),
//   per-group column sums (bias / time-embedding grads), conv weight transposes,
//   sinusoidal timestep embedding (diffusers get_timestep_embedding, flip_sin_to_cos=True,
//   downscale_freq_shift=0), add.
#include "common.h"

static int grid_for(long long n) {
  long long b = (n + 255) / 256;
  return (int)(b < 1 ? 1 : (b > 16384 ? 16384 : b));
}
#define GRID_STRIDE(i, n) for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < (n); i += (long long)gridDim.x * blockDim.x)

// h: [M, 2F] (hidden | gate), out: [M, F]
__global__ void geglu_fwd_kernel(const bf16_t* __restrict__ h, long long ldh, bf16_t* __restrict__ out, long long ldo,
                                 int M, int F) {
  const int F8 = F >> 3;
  GRID_STRIDE(i, (long long)M * F8) {
    const long long m = i / F8;
    const int c = (int)(i - m * F8) * 8;
    float a[8], g[8];
    unpack8(*reinterpret_cast<const bf8*>(h + m * ldh + c), a);
    unpack8(*reinterpret_cast<const bf8*>(h + m * ldh + F + c), g);
#pragma unroll
    for (int j = 0; j < 8; ++j) a[j] = a[j] * gelu_f(g[j]);
    *reinterpret_cast<bf8*>(out + m * ldo + c) = pack8(a);
  }
}
__global__ void geglu_bwd_kernel(const bf16_t* __restrict__ h, long long ldh, const bf16_t* __restrict__ dout,
                                 long long lddo, bf16_t* __restrict__ dh, long long lddh, int M, int F) {
  const int F8 = F >> 3;
  GRID_STRIDE(i, (long long)M * F8) {
    const long long m = i / F8;
    const int c = (int)(i - m * F8) * 8;
    float a[8], g[8], d[8], da[8], dg[8];
    unpack8(*reinterpret_cast<const bf8*>(h + m * ldh + c), a);
    unpack8(*reinterpret_cast<const bf8*>(h + m * ldh + F + c), g);
    unpack8(*reinterpret_cast<const bf8*>(dout + m * lddo + c), d);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const GeluTerms t = gelu_terms(g[j]);
      da[j] = d[j] * g[j] * t.cdf;                      // d * gelu(g)
      dg[j] = d[j] * a[j] * fmaf(g[j], t.pdf, t.cdf);   // d * a * gelu'(g)
    }
    *reinterpret_cast<bf8*>(dh + m * lddh + c) = pack8(da);
    *reinterpret_cast<bf8*>(dh + m * lddh + F + c) = pack8(dg);
  }
}

// elementwise SiLU on a dense bf16 buffer (n % 8 == 0)
__global__ void silu_fwd_kernel(const bf16_t* __restrict__ x, bf16_t* __restrict__ y, long long n8) {
  GRID_STRIDE(i, n8) {
    float f[8];
    unpack8(reinterpret_cast<const bf8*>(x)[i], f);
#pragma unroll
    for (int j = 0; j < 8; ++j) f[j] = silu_f(f[j]);
    reinterpret_cast<bf8*>(y)[i] = pack8(f);
  }
}
__global__ void silu_bwd_kernel(const bf16_t* __restrict__ x, const bf16_t* __restrict__ dy, bf16_t* __restrict__ dx,
                                long long n8) {
  GRID_STRIDE(i, n8) {
    float f[8], g[8];
    unpack8(reinterpret_cast<const bf8*>(x)[i], f);
    unpack8(reinterpret_cast<const bf8*>(dy)[i], g);
#pragma unroll
    for (int j = 0; j < 8; ++j) g[j] = g[j] * dsilu_f(f[j]);
    reinterpret_cast<bf8*>(dx)[i] = pack8(g);
  }
}

// out[p, 0:Ca] = a[p], out[p, Ca:Ca+Cb] = b[p]
__global__ void concat_kernel(const bf16_t* __restrict__ a, long long lda, int Ca, const bf16_t* __restrict__ b,
                              long long ldb, int Cb, bf16_t* __restrict__ out, long long P) {
  const int C8 = (Ca + Cb) >> 3, A8 = Ca >> 3;
  GRID_STRIDE(i, P * C8) {
    const long long p = i / C8;
    const int c8 = (int)(i - p * C8);
    const bf8 v = c8 < A8 ? *reinterpret_cast<const bf8*>(a + p * lda + c8 * 8)
                          : *reinterpret_cast<const bf8*>(b + p * ldb + (c8 - A8) * 8);
    *reinterpret_cast<bf8*>(out + p * (Ca + Cb) + c8 * 8) = v;
  }
}

// dx[n,h,w,c] = sum over the 2x2 block of dup[n,2h+i,2w+j,c]   (+ dx if accumulate)
__global__ void upsample_bwd_kernel(const bf16_t* __restrict__ dup, bf16_t* __restrict__ dx, int N, int H, int W, int C,
                                    int accumulate) {
  const int C8 = C >> 3;
  GRID_STRIDE(i, (long long)N * H * W * C8) {
    const int c8 = (int)(i % C8);
    long long t = i / C8;
    const int w = (int)(t % W);
    t /= W;
    const int h = (int)(t % H), n = (int)(t / H);
    float s[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
    for (int dy = 0; dy < 2; ++dy)
#pragma unroll
      for (int dxx = 0; dxx < 2; ++dxx) {
        float f[8];
        unpack8(*reinterpret_cast<const bf8*>(dup + (((long long)n * 2 * H + 2 * h + dy) * 2 * W + 2 * w + dxx) * C + c8 * 8), f);
#pragma unroll
        for (int j = 0; j < 8; ++j) s[j] += f[j];
      }
    bf16_t* dst = dx + (((long long)n * H + h) * W + w) * C + c8 * 8;
    if (accumulate) {
      float f[8];
      unpack8(*reinterpret_cast<const bf8*>(dst), f);
#pragma unroll
      for (int j = 0; j < 8; ++j) s[j] += f[j];
    }
    *reinterpret_cast<bf8*>(dst) = pack8(s);
  }
}

// column sums per row group, two deterministic passes (no atomics, no memset):
//   pass 1: ws[g][rb][n] = sum of rows [rb*rpb, (rb+1)*rpb) of group g   (block: 32 col-chunks x 8 row-lanes)
//   pass 2: out[g][n] (bf16 or f32, optionally accumulated) = sum_rb ws[g][rb][n]
__global__ void __launch_bounds__(256) colsum_partial_kernel(const bf16_t* __restrict__ x, long long ldx, int M, int N,
                                                             int rows_per_group, int rpb, int RB, float* __restrict__ ws) {
  __shared__ float red[8][256 + 4];
  const int cchunk = threadIdx.x & 31, rl = threadIdx.x >> 5;
  const int col = (blockIdx.x * 32 + cchunk) * 8;
  const int g = blockIdx.z, rb = blockIdx.y;
  const int r0 = g * rows_per_group + rb * rpb;
  const int r1 = min(min(M, (g + 1) * rows_per_group), r0 + rpb);
  float s[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (col < N) {
    // 8 independent 16-byte loads in flight per thread before any add (HBM latency, not the adds,
    // bounds a dependent load chain)
    int m = r0 + rl;
    for (; m + 56 < r1; m += 64) {
      bf8 v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = *reinterpret_cast<const bf8*>(x + (long long)(m + 8 * u) * ldx + col);
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        float f[8];
        unpack8(v[u], f);
#pragma unroll
        for (int j = 0; j < 8; ++j) s[j] += f[j];
      }
    }
    for (; m < r1; m += 8) {
      float f[8];
      unpack8(*reinterpret_cast<const bf8*>(x + (long long)m * ldx + col), f);
#pragma unroll
      for (int j = 0; j < 8; ++j) s[j] += f[j];
    }
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) red[rl][cchunk * 8 + j] = s[j];
  __syncthreads();
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c < N) {
    float t = 0.f;
#pragma unroll
    for (int k = 0; k < 8; ++k) t += red[k][threadIdx.x];
    ws[((long long)g * RB + rb) * N + c] = t;
  }
}
// second pass: block = 64 columns x 16 row-block lanes (float4 loads), grid = (N/64, groups)
__global__ void __launch_bounds__(256) colsum_reduce_kernel(const float* __restrict__ ws, int RB, int N, int groups,
                                                            void* __restrict__ out, int out_f32, int acc) {
  __shared__ float red[16][64 + 4];
  const int cq = threadIdx.x & 15, rl = threadIdx.x >> 4;
  const int g = blockIdx.y;
  const int c = blockIdx.x * 64 + cq * 4;
  float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
  if (c < N) {
    const float* p = ws + (long long)g * RB * N + c;
#pragma unroll 4
    for (int rb = rl; rb < RB; rb += 16) {
      const float4 v = *reinterpret_cast<const float4*>(p + (long long)rb * N);
      s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
    }
  }
  red[rl][cq * 4 + 0] = s.x; red[rl][cq * 4 + 1] = s.y; red[rl][cq * 4 + 2] = s.z; red[rl][cq * 4 + 3] = s.w;
  __syncthreads();
  const int col = blockIdx.x * 64 + threadIdx.x;
  if (threadIdx.x < 64 && col < N) {
    float t = 0.f;
#pragma unroll
    for (int k = 0; k < 16; ++k) t += red[k][threadIdx.x];
    const long long i = (long long)g * N + col;
    if (out_f32) {
      float* d = reinterpret_cast<float*>(out) + i;
      *d = acc ? *d + t : t;
    } else {
      bf16_t* d = reinterpret_cast<bf16_t*>(out) + i;
      *d = f2bf(acc ? bf2f(*d) + t : t);
    }
  }
}

// w [Cout][KH][KW][Cin] -> wt [Cin][KH][KW][Cout]
__global__ void conv_wt_kernel(const bf16_t* __restrict__ w, bf16_t* __restrict__ wt, int Cout, int KK, int Cin) {
  GRID_STRIDE(i, (long long)Cout * KK * Cin) {
    const int ci = (int)(i % Cin);
    long long t = i / Cin;
    const int kk = (int)(t % KK), co = (int)(t / KK);
    wt[((long long)ci * KK + kk) * Cout + co] = w[i];
  }
}

// LoRA bf16 shadow refresh (one launch per step for every adapter): entry e copies a [rows x cols]
// fp32 block at src + e.src (contiguous) to bf16 at dst + e.dst with row stride e.dst_ld, times
// e.scale (alpha / rank for up projections; fused q|k|v ups land on the diagonal of one [3C x 3r]).
// transpose = 1: the [rows][cols] source lands as [cols][rows] (row stride dst_ld): the transposed up / down copies
// the fused LoRA input-gradient GEMM reads in K-mode (gemm2_kernel.h)
struct LoraShadowEntry { long long src, dst; int rows, cols, dst_ld; float scale; int transpose, pad; };
__global__ void __launch_bounds__(256) lora_shadow_kernel(const float* __restrict__ src, bf16_t* __restrict__ dst,
                                                          const LoraShadowEntry* __restrict__ tab) {
  const LoraShadowEntry e = tab[blockIdx.y];
  const long long n = (long long)e.rows * e.cols;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    const long long r = i / e.cols, c = i - r * e.cols;
    dst[e.dst + (e.transpose ? c * e.dst_ld + r : r * e.dst_ld + c)] = f2bf(src[e.src + i] * e.scale);
  }
}

// fp32 -> bf16 / f32 destination, optionally accumulating (grad writes of bias / norm params)
__global__ void cast_f2b_kernel(const float* __restrict__ x, void* __restrict__ y, long long n, int dst_f32, int acc) {
  GRID_STRIDE(i, n) {
    if (dst_f32) {
      float* d = reinterpret_cast<float*>(y);
      d[i] = acc ? d[i] + x[i] : x[i];
    } else {
      bf16_t* d = reinterpret_cast<bf16_t*>(y);
      d[i] = f2bf(acc ? bf2f(d[i]) + x[i] : x[i]);
    }
  }
}

// emb[b, :] = [cos(t*f_i), sin(t*f_i)], f_i = exp(-ln(10000) * i / half)   (flip_sin_to_cos=True, shift 0)
// t is float32 (timesteps cast by .float() in diffusers); out bf16 row stride ldo
__global__ void timestep_embedding_kernel(const float* __restrict__ t, int n, int dim, bf16_t* __restrict__ out,
                                          long long ldo) {
  const int half = dim / 2;
  GRID_STRIDE(i, (long long)n * half) {
    const int b = (int)(i / half), k = (int)(i - (long long)b * half);
    // torch: exponent = -math.log(10000) * arange(half, f32) ; exponent / half ; exp(exponent)
    const float expo = (-9.210340371976184f * (float)k) / (float)half;
    const float f = expf(expo);
    const float a = t[b] * f;
    out[(long long)b * ldo + k] = f2bf(cosf(a));
    out[(long long)b * ldo + half + k] = f2bf(sinf(a));
  }
}

// y = a + b (dense bf16)
__global__ void add_kernel(const bf16_t* __restrict__ a, const bf16_t* __restrict__ b, bf16_t* __restrict__ y, long long n8) {
  GRID_STRIDE(i, n8) {
    float fa[8], fb[8];
    unpack8(reinterpret_cast<const bf8*>(a)[i], fa);
    unpack8(reinterpret_cast<const bf8*>(b)[i], fb);
#pragma unroll
    for (int j = 0; j < 8; ++j) fa[j] += fb[j];
    reinterpret_cast<bf8*>(y)[i] = pack8(fa);
  }
}

static bool al16(const void* p) { return ((uintptr_t)p & 15) == 0; }

OTAMD_API int otamd_geglu_fwd(const void* h, long long ldh, void* out, long long ldo, int M, int F, hipStream_t s) {
  if (!h || !out || M < 0 || F % 8 || ldh % 8 || ldo % 8 || !al16(h) || !al16(out)) return OTAMD_EINVAL;
  if (M == 0) return OTAMD_OK;
  geglu_fwd_kernel<<<grid_for((long long)M * F / 8), 256, 0, s>>>((const bf16_t*)h, ldh, (bf16_t*)out, ldo, M, F);
  OTAMD_CHECK_LAUNCH();
  return OTAMD_OK;
}
OTAMD_API int otamd_geglu_bwd(const void* h, long long ldh, const void* dout, long long lddo, void* dh, long long lddh,
                              int M, int F, hipStream_t s) {
  if (!h || !dout || !dh || M < 0 || F % 8 || ldh % 8 || lddo % 8 || lddh % 8) return OTAMD_EINVAL;
  if (!al16(h) || !al16(dout) || !al16(dh)) return OTAMD_EINVAL;
  if (M == 0) return OTAMD_OK;
  geglu_bwd_kernel<<<grid_for((long long)M * F / 8), 256, 0, s>>>((const bf16_t*)h, ldh, (const bf16_t*)dout, lddo,
                                                                  (bf16_t*)dh, lddh, M, F);
  OTAMD_CHECK_LAUNCH();
  return OTAMD_OK;
}
OTAMD_API int otamd_silu_fwd(const void* x, void* y, long long n, hipStream_t s) {
  if (!x || !y || n % 8 || !al16(x) || !al16(y)) return OTAMD_EINVAL;
  if (n == 0) return OTAMD_OK;
  silu_fwd_kernel<<<grid_for(n / 8), 256, 0, s>>>((const bf16_t*)x, (bf16_t*)y, n / 8);
  OTAMD_CHECK_LAUNCH();
  return OTAMD_OK;
}
OTAMD_API int otamd_silu_bwd(const void* x, const void* dy, void* dx, long long n, hipStream_t s) {
  if (!x || !dy || !dx || n % 8 || !al16(x) || !al16(dy) || !al16(dx)) return OTAMD_EINVAL;
  if (n == 0) return OTAMD_OK;
  silu_bwd_kernel<<<grid_for(n / 8), 256, 0, s>>>((const bf16_t*)x, (const bf16_t*)dy, (bf16_t*)dx, n / 8);
  OTAMD_CHECK_LAUNCH();
  return OTAMD_OK;
}
OTAMD_API int otamd_concat_channels(const void* a, long long lda, int Ca, const void* b, long long ldb, int Cb,
                                    void* out, long long P, hipStream_t s) {
  if (!a || !b || !out || Ca % 8 || Cb % 8 || lda % 8 || ldb % 8 || P < 0) return OTAMD_EINVAL;
  if (!al16(a) || !al16(b) || !al16(out)) return OTAMD_EINVAL;
  if (P == 0) return OTAMD_OK;
  concat_kernel<<<grid_for(P * (Ca + Cb) / 8), 256, 0, s>>>((const bf16_t*)a, lda, Ca, (const bf16_t*)b, ldb, Cb,
                                                            (bf16_t*)out, P);
  OTAMD_CHECK_LAUNCH();
  return OTAMD_OK;
}
OTAMD_API int otamd_upsample2x_bwd(const void* dup, void* dx, int N, int H, int W, int C, int accumulate,
                                   hipStream_t s) {
  if (!dup || !dx || C % 8 || N <= 0 || H <= 0 || W <= 0 || !al16(dup) || !al16(dx)) return OTAMD_EINVAL;
  upsample_bwd_kernel<<<grid_for((long long)N * H * W * C / 8), 256, 0, s>>>((const bf16_t*)dup, (bf16_t*)dx, N, H, W,
                                                                             C, accumulate);
  OTAMD_CHECK_LAUNCH();
  return OTAMD_OK;
}
// out: [groups][N] bf16 (out_f32=0) or f32; ws: >= groups * RB * N floats where RB = colsum_row_blocks(...)
static int colsum_rpb(int rows_per_group, int N, int groups) {
  const int cblocks = (N + 255) / 256;
  int rpb = rows_per_group;
  // ~2048 first-pass blocks (8 per CU) so enough loads are in flight to cover HBM latency; each block
  // still streams >= 128 rows (16 per thread-row: two batches of 8 loads) and RB stays small
  while (rpb > 128 && (long long)cblocks * groups * ((rows_per_group + rpb - 1) / rpb) < 2048) rpb = (rpb + 1) / 2;
  return rpb;
}
OTAMD_API long long otamd_colsum_ws_floats(int M, int N, int rows_per_group) {
  const int groups = (M + rows_per_group - 1) / rows_per_group;
  const int rpb = colsum_rpb(rows_per_group, N, groups);
  return (long long)groups * ((rows_per_group + rpb - 1) / rpb) * N;
}
OTAMD_API int otamd_colsum(const void* x, long long ldx, int M, int N, int rows_per_group, void* out, int out_f32,
                           int accumulate, float* ws, long long ws_floats, hipStream_t s) {
  if (!x || !out || !ws || M <= 0 || N % 8 || ldx % 8 || rows_per_group <= 0 || !al16(x)) return OTAMD_EINVAL;
  const int groups = (M + rows_per_group - 1) / rows_per_group;
  const int rpb = colsum_rpb(rows_per_group, N, groups);
  const int RB = (rows_per_group + rpb - 1) / rpb;
  if (ws_floats < (long long)groups * RB * N) return OTAMD_EINVAL;
  dim3 grid((N + 255) / 256, RB, groups);
  colsum_partial_kernel<<<grid, 256, 0, s>>>((const bf16_t*)x, ldx, M, N, rows_per_group, rpb, RB, ws);
  OTAMD_CHECK_LAUNCH();
  colsum_reduce_kernel<<<dim3((N + 63) / 64, groups), 256, 0, s>>>(ws, RB, N, groups, out, out_f32, accumulate);
  OTAMD_CHECK_LAUNCH();
  return OTAMD_OK;
}
OTAMD_API int otamd_conv_weight_transpose(const void* w, void* wt, int Cout, int KK, int Cin, hipStream_t s) {
  if (!w || !wt || Cout <= 0 || KK <= 0 || Cin <= 0) return OTAMD_EINVAL;
  conv_wt_kernel<<<grid_for((long long)Cout * KK * Cin), 256, 0, s>>>((const bf16_t*)w, (bf16_t*)wt, Cout, KK, Cin);
  OTAMD_CHECK_LAUNCH();
  return OTAMD_OK;
}
OTAMD_API int otamd_lora_shadow(const float* src, void* dst, const void* table, int n_entries, hipStream_t s) {
  if (!src || !dst || !table || n_entries < 0 || n_entries > 65535) return OTAMD_EINVAL;
  if (n_entries == 0) return OTAMD_OK;
  lora_shadow_kernel<<<dim3(16, n_entries), 256, 0, s>>>(src, (bf16_t*)dst, (const LoraShadowEntry*)table);
  OTAMD_CHECK_LAUNCH();
  return OTAMD_OK;
}
OTAMD_API int otamd_lora_shadow_entry_size(void) { return (int)sizeof(LoraShadowEntry); }
OTAMD_API int otamd_cast_f32(const float* x, void* y, long long n, int dst_f32, int accumulate, hipStream_t s) {
  if (!x || !y || n < 0) return OTAMD_EINVAL;
  if (n == 0) return OTAMD_OK;
  cast_f2b_kernel<<<grid_for(n), 256, 0, s>>>(x, y, n, dst_f32, accumulate);
  OTAMD_CHECK_LAUNCH();
  return OTAMD_OK;
}
OTAMD_API int otamd_timestep_embedding(const float* t, int n, int dim, void* out, long long ldo, hipStream_t s) {
  if (!t || !out || n <= 0 || dim % 2) return OTAMD_EINVAL;
  timestep_embedding_kernel<<<grid_for((long long)n * dim / 2), 256, 0, s>>>(t, n, dim, (bf16_t*)out, ldo);
  OTAMD_CHECK_LAUNCH();
  return OTAMD_OK;
}
OTAMD_API int otamd_add(const void* a, const void* b, void* y, long long n, hipStream_t s) {
  if (!a || !b || !y || n % 8 || !al16(a) || !al16(b) || !al16(y)) return OTAMD_EINVAL;
  if (n == 0) return OTAMD_OK;
  add_kernel<<<grid_for(n / 8), 256, 0, s>>>((const bf16_t*)a, (const bf16_t*)b, (bf16_t*)y, n / 8);
  OTAMD_CHECK_LAUNCH();
  return OTAMD_OK;
}

// RCCL footprint emulation on one GPU (trainer/ddp.py, OTAMD_DP_EMULATE): a bucket's ring all-reduce
// over N ranks holds RCCL's channel workgroups on their CUs for its wire time and streams its local HBM bytes.
// `gridDim.x` workgroups (the channels) copy n16 16-byte vectors, src wrapping over src_n16 and dst over dst_n16,
// paced by the 100 MHz real-time counter so that workgroup b finishes its share no earlier than `ticks` after
// it started.  Vector stores only.
__global__ void __launch_bounds__(256) dp_emulate_kernel(const uint4* __restrict__ src, long long src_n16,
                                                         uint4* __restrict__ dst, long long dst_n16, long long n16,
                                                         long long ticks) {
  const long long per = (n16 + gridDim.x - 1) / gridDim.x;
  const long long b0 = (long long)blockIdx.x * per, b1 = min(n16, b0 + per);
  if (b0 >= b1) return;
  constexpr long long CH = 256 * 8;   // vectors per paced step (32 KiB)
  const long long nsteps = (b1 - b0 + CH - 1) / CH;
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  for (long long st = 0; st < nsteps; ++st) {
    const long long base = b0 + st * CH;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const long long i = base + j * 256 + threadIdx.x;
      if (i < b1) dst[i % dst_n16] = src[i % src_n16];
    }
    const unsigned long long due = t0 + (unsigned long long)((st + 1) * ticks / nsteps);
    while (__builtin_amdgcn_s_memrealtime() < due) __builtin_amdgcn_s_sleep(4);
  }
}
OTAMD_API int otamd_dp_emulate(const void* src, long long src_bytes, void* dst, long long dst_bytes, long long bytes,
                               int blocks, long long ns, hipStream_t s) {
  if (!src || !dst || src_bytes < 16 || dst_bytes < 16 || bytes < 0 || blocks <= 0 || blocks > 4096 || ns < 0 ||
      !al16(src) || !al16(dst))
    return OTAMD_EINVAL;
  if (bytes < 16) return OTAMD_OK;
  dp_emulate_kernel<<<blocks, 256, 0, s>>>((const uint4*)src, src_bytes / 16, (uint4*)dst, dst_bytes / 16, bytes / 16,
                                           ns / 10);
  OTAMD_CHECK_LAUNCH();
  return OTAMD_OK;
}

// Image batch -> VAE encoder input: mgds RescaleImageChannels (0..1 -> -1..1, i.e. x * mul + add;
// StableDiffusionXLBaseDataLoader.py:66) fused with the NCHW fp32 -> NHWC bf16 relayout, channels
// zero-padded to cpad (conv_in reads whole 16-byte chunks).  One thread per output pixel.
__global__ void __launch_bounds__(256) image_to_nhwc_kernel(const float* __restrict__ img, int B, int C, int H, int W,
                                                            float mul, float add, bf16_t* __restrict__ out,
                                                            int cpad) {
  const long long npix = (long long)B * H * W;
  const long long hw = (long long)H * W;
  for (long long p = blockIdx.x * (long long)blockDim.x + threadIdx.x; p < npix; p += (long long)gridDim.x * blockDim.x) {
    const long long b = p / hw, r = p - b * hw;
    bf16_t* o = out + p * cpad;
    for (int c0 = 0; c0 < cpad; c0 += 8) {
      float f[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int c = c0 + j;
        f[j] = c < C ? fmaf(img[(b * C + c) * hw + r], mul, add) : 0.f;
      }
      *reinterpret_cast<bf8*>(o + c0) = pack8(f);
    }
  }
}

OTAMD_API int otamd_image_to_nhwc(const float* img, int B, int C, int H, int W, float mul, float add, void* out,
                                  int cpad, hipStream_t s) {
  if (!img || !out || B <= 0 || C <= 0 || H <= 0 || W <= 0 || cpad < C || cpad % 8 || !al16(out)) return OTAMD_EINVAL;
  image_to_nhwc_kernel<<<grid_for((long long)B * H * W), 256, 0, s>>>(img, B, C, H, W, mul, add, (bf16_t*)out, cpad);
  OTAMD_CHECK_LAUNCH();
  return OTAMD_OK;
}
