// Shared GEMM-engine definitions (gemm.hip = 128x128 4-wave kernel, gemm2.hip = 8-wave
// 256-wide LDS-DMA kernels).  GemmArgs is passed by value to the kernels and through the C ABI.
#pragma once
#include "common.h"

// OPM_CONV_WT (v2 only): B of conv dgrad read straight from the stored weight W[Cout][KH][KW][Cin] as
// an MN-mode operand B[k = tap*Cout + co][ci] (row address (co*KK + tap)*ld); gb.SC = Cout, gb.KH/KW.
enum { OPM_K = 0, OPM_MN = 1, OPM_CONV_FWD = 2, OPM_CONV_DGRAD = 3, OPM_CONV_WGRAD = 4, OPM_CONV_WT = 5 };

struct ConvGeom {
  int N;             // batch
  int SH, SW, SC;    // gathered (source) tensor: spatial dims and channel count
  int RH, RW;        // spatial dims decoding a GEMM row index (fwd: output, dgrad: input, wgrad: output)
  int KH, KW, stride, pad;
  int upsample;      // source read through a virtual nearest-2x upsample (fwd / wgrad)
  int pad_;
  long long ld;      // pixel stride of the source, elements
};

struct GemmArgs {
  const bf16_t* A; long long lda; int amode;
  const bf16_t* B; long long ldb; int bmode;
  void* C; long long ldc; int c_f32; int accumulate;
  int M, N, K;
  float alpha;
  const bf16_t* bias;                                          // + bias[n]
  const bf16_t* rowvec; long long ldv; int rows_per_vec;       // + rowvec[(m/rows_per_vec)*ldv + n]
  const bf16_t* residual; long long ldr;                       // + residual[m*ldr + n]
  float* slab;                                                 // split-K partials [splits][M][N]
  int k_per_split;
  ConvGeom ga, gb;
  // optional second K segment (v2 tiles; LoRA fused into its base GEMM): k in [K1, K1+K2) reads
  // A2[m][k-K1] (K-mode) and B2 (K-mode [N][K2] when B is K-mode, MN-mode [K2][N] when B is MN-mode).
  // K == K1 + K2, K1 % 64 == 0.  A2 == nullptr: single segment (K1, K2 ignored).
  const bf16_t* A2; long long lda2;
  const bf16_t* B2; long long ldb2;
  int K1, K2;
  // batched GEMM (K/MN operand modes, one K segment, no split-K): grid.y = batch index z; every
  // operand base moves by (z / bdiv) * s0 + (z % bdiv) * s1 elements -- (image, head) pairs of a
  // [B, N, H*D] activation are bdiv = H, s0 = batch stride, s1 = D.  batch <= 1: unbatched.
  int batch, bdiv;
  long long sa0, sa1, sb0, sb1, sc0, sc1;
  // column sums of the MN-mode A over the K range (wgrad: the bias gradient sum_k dY[k][m]) -- colsum bf16 /
  // f32 [M], overwrite or accumulate; split-K: per-split partials in colsum_slab [splits][M], folded by the
  // split-K reduce.  v2 tiles only; tile-column 0 workgroups accumulate them from the LDS image of A.
  void* colsum; int colsum_f32; int colsum_acc;
  float* colsum_slab;
  // LoRA down-projection fused into the K loop of a forward base GEMM (v2 tiles, gemm2_tiles_e.hip): D = down
  // [P*lora_r][K] (K-mode, the K layout of B), B2 / ldb2 = up [N][P*lora_r] (alpha/rank folded in), T = t [M][ldt]
  // (bf16 out, for the backward), lora_pw = output columns per adapter part (tiles never straddle parts).  K is the
  // base K (no second segment operand A2).  D == nullptr: off.  On a linear dgrad (B = W MN-mode): u = dY (sB) with
  // D = (sB)^T [lora_r][K], B2 = A^T [N][lora_r], T = u, lora_pw = N (the LoRA backward's dX, include/otamd.h).
  const bf16_t* D; long long ldd;
  bf16_t* T; long long ldt;
  int lora_r, lora_pw;
};

__device__ __forceinline__ void gemm_batch_offset(GemmArgs& a) {
  if (a.batch > 1) {
    const int z = blockIdx.y;
    const long long q = z / a.bdiv, r = z - q * a.bdiv;
    a.A += q * a.sa0 + r * a.sa1;
    a.B += q * a.sb0 + r * a.sb1;
    a.C = (char*)a.C + (q * a.sc0 + r * a.sc1) * (a.c_f32 ? 4 : 2);
  }
}


__device__ __forceinline__ void add_bf8(float (&v)[8], const uint4& b) {
  v[0] += __uint_as_float(b.x << 16); v[1] += __uint_as_float(b.x & 0xffff0000u);
  v[2] += __uint_as_float(b.y << 16); v[3] += __uint_as_float(b.y & 0xffff0000u);
  v[4] += __uint_as_float(b.z << 16); v[5] += __uint_as_float(b.z & 0xffff0000u);
  v[6] += __uint_as_float(b.w << 16); v[7] += __uint_as_float(b.w & 0xffff0000u);
}

// true when every epilogue operand allows 16-byte accesses at 8-column granules (kernel-uniform)
__device__ __forceinline__ bool gemm_wide_ok(const GemmArgs& a) {
  const uintptr_t al = (uintptr_t)a.C | (uintptr_t)a.bias | (uintptr_t)a.rowvec | (uintptr_t)a.residual;
  return (al & 15) == 0 && (a.ldc % 8) == 0 && (!a.rowvec || (a.ldv % 8) == 0) && (!a.residual || (a.ldr % 8) == 0);
}

// epilogue for 8 consecutive output columns n..n+7 of row m: same math as gemm_store4, 16-byte
// loads / stores (half the store instructions of the 4-column form; the tail is issue-bound)
__device__ __forceinline__ void gemm_store8(const GemmArgs& args, int m, int n, float (&v)[8], int split,
                                            bool use_slab) {
  if (use_slab) {
    const long long e = ((long long)split * args.M + m) * args.N + n;
    float* dst = args.slab + e;
    reinterpret_cast<float4*>(dst)[0] = make_float4(v[0], v[1], v[2], v[3]);
    reinterpret_cast<float4*>(dst)[1] = make_float4(v[4], v[5], v[6], v[7]);
    return;
  }
#pragma unroll
  for (int t = 0; t < 8; ++t) v[t] *= args.alpha;
  if (args.bias) add_bf8(v, *reinterpret_cast<const uint4*>(args.bias + n));
  if (args.rowvec) add_bf8(v, *reinterpret_cast<const uint4*>(args.rowvec + (long long)(m / args.rows_per_vec) * args.ldv + n));
  if (args.residual) add_bf8(v, *reinterpret_cast<const uint4*>(args.residual + (long long)m * args.ldr + n));
  if (args.c_f32) {
    float4* dst = reinterpret_cast<float4*>(reinterpret_cast<float*>(args.C) + (long long)m * args.ldc + n);
    if (args.accumulate) {
      const float4 o0 = dst[0], o1 = dst[1];
      v[0] += o0.x; v[1] += o0.y; v[2] += o0.z; v[3] += o0.w; v[4] += o1.x; v[5] += o1.y; v[6] += o1.z; v[7] += o1.w;
    }
    dst[0] = make_float4(v[0], v[1], v[2], v[3]);
    dst[1] = make_float4(v[4], v[5], v[6], v[7]);
  } else {
    bf16_t* dst = reinterpret_cast<bf16_t*>(args.C) + (long long)m * args.ldc + n;
    if (args.accumulate) add_bf8(v, *reinterpret_cast<const uint4*>(dst));
    uint4 o;
    o.x = (uint32_t)f2bf(v[0]) | ((uint32_t)f2bf(v[1]) << 16);
    o.y = (uint32_t)f2bf(v[2]) | ((uint32_t)f2bf(v[3]) << 16);
    o.z = (uint32_t)f2bf(v[4]) | ((uint32_t)f2bf(v[5]) << 16);
    o.w = (uint32_t)f2bf(v[6]) | ((uint32_t)f2bf(v[7]) << 16);
    *reinterpret_cast<uint4*>(dst) = o;
  }
}

// epilogue for 4 consecutive output columns n..n+3 of row m (fp32 accumulators in v[])
__device__ __forceinline__ void gemm_store4(const GemmArgs& args, int m, int n, float (&v)[4], int split,
                                            bool use_slab) {
  if (use_slab) {
    const long long e = ((long long)split * args.M + m) * args.N + n;
    *reinterpret_cast<float4*>(args.slab + e) = make_float4(v[0], v[1], v[2], v[3]);
    return;
  }
#pragma unroll
  for (int t = 0; t < 4; ++t) v[t] *= args.alpha;
  if (args.bias) {
    const uint2 b = *reinterpret_cast<const uint2*>(args.bias + n);
    v[0] += __uint_as_float(b.x << 16); v[1] += __uint_as_float(b.x & 0xffff0000u);
    v[2] += __uint_as_float(b.y << 16); v[3] += __uint_as_float(b.y & 0xffff0000u);
  }
  if (args.rowvec) {
    const uint2 b = *reinterpret_cast<const uint2*>(args.rowvec + (long long)(m / args.rows_per_vec) * args.ldv + n);
    v[0] += __uint_as_float(b.x << 16); v[1] += __uint_as_float(b.x & 0xffff0000u);
    v[2] += __uint_as_float(b.y << 16); v[3] += __uint_as_float(b.y & 0xffff0000u);
  }
  if (args.residual) {
    const uint2 b = *reinterpret_cast<const uint2*>(args.residual + (long long)m * args.ldr + n);
    v[0] += __uint_as_float(b.x << 16); v[1] += __uint_as_float(b.x & 0xffff0000u);
    v[2] += __uint_as_float(b.y << 16); v[3] += __uint_as_float(b.y & 0xffff0000u);
  }
  if (args.c_f32) {
    float* dst = reinterpret_cast<float*>(args.C) + (long long)m * args.ldc + n;
    if (args.accumulate) { float4 o = *reinterpret_cast<float4*>(dst); v[0] += o.x; v[1] += o.y; v[2] += o.z; v[3] += o.w; }
    *reinterpret_cast<float4*>(dst) = make_float4(v[0], v[1], v[2], v[3]);
  } else {
    bf16_t* dst = reinterpret_cast<bf16_t*>(args.C) + (long long)m * args.ldc + n;
    if (args.accumulate) {
      const uint2 o = *reinterpret_cast<const uint2*>(dst);
      v[0] += __uint_as_float(o.x << 16); v[1] += __uint_as_float(o.x & 0xffff0000u);
      v[2] += __uint_as_float(o.y << 16); v[3] += __uint_as_float(o.y & 0xffff0000u);
    }
    uint2 o;
    o.x = (uint32_t)f2bf(v[0]) | ((uint32_t)f2bf(v[1]) << 16);
    o.y = (uint32_t)f2bf(v[2]) | ((uint32_t)f2bf(v[3]) << 16);
    *reinterpret_cast<uint2*>(dst) = o;
  }
}

// XCD-aware bijective remap of a linear workgroup id (cdna_hip_programming.md §5 T1)
__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int q = nwg / 8, r = nwg % 8, xcd = bid % 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + bid / 8;
}

// Grouped tile order: consecutive tile ids walk GM tile-rows down, then the next column, so the
// ~32 tiles one XCD runs at a time (consecutive ids after xcd_remap) form an 8x4 block that shares
// 8 A row-panels and 4 B column-panels in that XCD's L2 -- instead of one full column of A.
__device__ __forceinline__ void tile_coords(int wg, int tiles_m, int tiles_n, int& tm, int& tn) {
  constexpr int GM = 8;
  const int per_group = GM * tiles_n;
  const int g = wg / per_group, first = g * GM;
  const int gsz = min(tiles_m - first, GM);
  const int idx = wg - g * per_group;
  tm = first + idx % gsz;
  tn = idx / gsz;
}

// K-mode LDS image: [rows][64 k], 128-byte rows, 16-byte chunk c of row r stored at c ^ (r & 7)
__device__ __forceinline__ int kimg_off(int row, int chunk) { return row * 128 + ((chunk ^ (row & 7)) << 4); }
// MN-mode LDS image: [64 k rows][RB bytes], 32-byte block b of row k stored at b ^ s(k)
__device__ __forceinline__ int mn_swz(int k) { return (k & 3) | (((k >> 3) & 1) << 2); }
// the same for an image of RB-byte rows: a 64-wide tile (128-byte rows) has only 4 blocks per row
// and 160-wide tiles (320-byte rows, 10 blocks): the 80-dword row pitch already spreads rows k..k+3 over
// four 8-bank groups; rows k+8.. alias them, so block bit 0 flips with k bit 3 (stays inside the row)
template <int RB> __device__ __forceinline__ int mn_swz_rb(int k) {
  return RB == 320 ? ((k >> 3) & 1) : (RB >= 256 ? mn_swz(k) : (k & 3));
}

// alpha * sum_s slab[s] (+bias, +rowvec, +residual) (+C if accumulate) for V consecutive columns
// n.. of row m: the split-K combine of splitk_reduce_kernel (splits summed in index order).
__device__ __forceinline__ float4 slab_load(const GemmArgs& args, long long e) {
  return *reinterpret_cast<const float4*>(args.slab + e);
}

template <int V>
__device__ __forceinline__ void splitk_combine(const GemmArgs& args, unsigned m, unsigned n, int splits) {
  const long long MN = (long long)args.M * args.N;
  const long long e = (long long)m * args.N + n;
  float v[V];
  {
    const float4 t = slab_load(args, e);
    v[0] = t.x; v[1] = t.y; v[2] = t.z; v[3] = t.w;
    if constexpr (V == 8) {
      const float4 u = slab_load(args, e + 4);
      v[4] = u.x; v[5] = u.y; v[6] = u.z; v[7] = u.w;
    }
  }
  int z = 1;
  for (; z + 3 < splits; z += 4) {
    float4 t[4][V / 4];
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int h = 0; h < V / 4; ++h) t[q][h] = slab_load(args, (z + q) * MN + e + 4 * h);
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int h = 0; h < V / 4; ++h) {
        v[4 * h] += t[q][h].x; v[4 * h + 1] += t[q][h].y; v[4 * h + 2] += t[q][h].z; v[4 * h + 3] += t[q][h].w;
      }
  }
  for (; z < splits; ++z)
#pragma unroll
    for (int h = 0; h < V / 4; ++h) {
      const float4 t = slab_load(args, z * MN + e + 4 * h);
      v[4 * h] += t.x; v[4 * h + 1] += t.y; v[4 * h + 2] += t.z; v[4 * h + 3] += t.w;
    }
#pragma unroll
  for (int t = 0; t < V; ++t) v[t] *= args.alpha;
  if constexpr (V == 8) {   // 16-byte epilogue operands (one load each instead of 8 two-byte loads)
    if (gemm_wide_ok(args) && !args.c_f32) {
      float w[8];
#pragma unroll
      for (int t = 0; t < 8; ++t) w[t] = v[t];
      if (args.bias) add_bf8(w, *reinterpret_cast<const uint4*>(args.bias + n));
      if (args.rowvec) add_bf8(w, *reinterpret_cast<const uint4*>(args.rowvec + (long long)(m / args.rows_per_vec) * args.ldv + n));
      if (args.residual) add_bf8(w, *reinterpret_cast<const uint4*>(args.residual + (long long)m * args.ldr + n));
      bf16_t* dst = reinterpret_cast<bf16_t*>(args.C) + (long long)m * args.ldc + n;
      if (args.accumulate) add_bf8(w, *reinterpret_cast<const uint4*>(dst));
      *reinterpret_cast<bf8*>(dst) = pack8(w);
      return;
    }
  }
  if (args.bias)
#pragma unroll
    for (int t = 0; t < V; ++t) v[t] += bf2f(args.bias[n + t]);
  if (args.rowvec)
#pragma unroll
    for (int t = 0; t < V; ++t) v[t] += bf2f(args.rowvec[(long long)(m / args.rows_per_vec) * args.ldv + n + t]);
  if (args.residual)
#pragma unroll
    for (int t = 0; t < V; ++t) v[t] += bf2f(args.residual[(long long)m * args.ldr + n + t]);
  if (args.c_f32) {
    float* dst = reinterpret_cast<float*>(args.C) + (long long)m * args.ldc + n;
#pragma unroll
    for (int t = 0; t < V; ++t) dst[t] = args.accumulate ? dst[t] + v[t] : v[t];
  } else {
    bf16_t* dst = reinterpret_cast<bf16_t*>(args.C) + (long long)m * args.ldc + n;
    if constexpr (V == 8) {
      if (args.accumulate) {
        float p[8];
        unpack8(*reinterpret_cast<const bf8*>(dst), p);
#pragma unroll
        for (int t = 0; t < 8; ++t) v[t] += p[t];
      }
      *reinterpret_cast<bf8*>(dst) = pack8(v);
    } else {
#pragma unroll
      for (int t = 0; t < V; ++t) dst[t] = f2bf(args.accumulate ? bf2f(dst[t]) + v[t] : v[t]);
    }
  }
}


