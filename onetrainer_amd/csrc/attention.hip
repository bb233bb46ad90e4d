// Flash attention forward / backward for gfx950 (v_mfma_f32_32x32x16_bf16, fp32 softmax).
// Replaces diffusers Attention + F.scaled_dot_product_attention in every
// BasicTransformerBlock attn1 (self) / attn2 (cross, Lk = 77) (SURVEY.md §2.3 "Self-attention",
// "Cross-attention"; reached from modules/modelSetup/BaseStableDiffusionXLSetup.py:268-273).
//
// Layout: Q [B, Nq, H, D], K/V [B, Nk, H, D] with explicit token / batch strides (the
// to_q/to_k/to_v GEMM outputs are read in place: no head permute).  O likewise; LSE is
// stored per (b, h, q) in the log2 domain.  Head dim Dv <= D (D in {64, 128}), zero padded.
//
// Structure (per wave, 32 rows):
//   forward / dQ : S^T = K Q^T  (keys in registers, query on the lane -> softmax row reduce is
//                  lane-local + one xor-32 shuffle); P^T accumulator registers feed O^T = V^T P^T
//                  directly as the MFMA B operand; V^T comes from ds_read_b64_tr_b16.
//   dK/dV        : S = Q K^T with the key on the lane; P and dS accumulators feed
//                  dV^T = dO^T P and dK^T = Q^T dS directly; dO^T, Q^T by transposed LDS reads.
#include "common.h"

struct AttnArgs {
  const bf16_t* q; const bf16_t* k; const bf16_t* v; bf16_t* o; float* lse;
  const bf16_t* dout; const float* delta; bf16_t* dq; bf16_t* dk; bf16_t* dv; float* dk32; float* dv32;
  long long ldq, ldk, ldv, ldo, lddo, lddq, lddk, lddv;     // token strides (elements)
  long long bsq, bsk, bsv, bso, bsdo, bsdq, bsdk, bsdv;     // batch strides (elements)
  int B, H, Nq, Nk, Dv;
  float scale;
  int qsplit;
  int pad_;
};

#define KT 64   // keys per staged tile (fwd / dQ)
#define QT 32   // queries per staged tile (dK/dV)
static constexpr float LOG2E = 1.4426950408889634f;

typedef __attribute__((address_space(3))) short4v lds_s4;

// row image: [rows][D] bf16, 16-byte chunk c of row r stored at c ^ (r & 7)
template <int D> __device__ __forceinline__ int row_off(int r, int c) { return r * (D * 2) + ((c ^ (r & 7)) << 4); }
// transposed-read image: [rows][D] bf16, 32-byte block b of row r stored at b ^ sw(r)
template <int D> __device__ __forceinline__ int tr_off(int r, int col) {
  const int blk = col >> 4, within = (col & 15) << 1;
  const int sw = (D == 64) ? (((r >> 1) & 1) << 1) : ((r & 3) << 1);
  return r * (D * 2) + ((blk ^ sw) << 5) + within;
}

__device__ __forceinline__ bf16x8 lds_row_frag(const char* img, int D2, int r, int c) {
  return *reinterpret_cast<const bf16x8*>(img + r * D2 + ((c ^ (r & 7)) << 4));
}

// 32x32x16 A operand with the accumulator-operand k order (cdna_hip_programming.md §3):
// element j of lane half h <-> row row0 + 16s + 8(j>>2) + 4h + (j&3); column col0 + (lane & 31)
template <int D>
__device__ __forceinline__ bf16x8 tr_frag(const char* img, int row0, int s, int col0) {
  const int lane = threadIdx.x & 63;
  const int G = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3, h = lane >> 5;
  const int r = row0 + 16 * s + 4 * h + q;
  const int col = col0 + 16 * (G & 1) + 4 * p;
  const short4v lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(img + tr_off<D>(r, col)));
  const short4v hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(img + tr_off<D>(r + 8, col)));
  short8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8, v);
}

__device__ __forceinline__ bf16x8 pack_acc(const float16v& a, int s) {
  bf16x8 r;
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = (__bf16)a[8 * s + j];
  return r;
}

__device__ __forceinline__ float16v mfma32(const bf16x8& a, const bf16x8& b, const float16v& c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ float16v zero16() {
  float16v z;
#pragma unroll
  for (int i = 0; i < 16; ++i) z[i] = 0.f;
  return z;
}
// row (in the 32-row accumulator tile) held by register i of this lane
__device__ __forceinline__ int acc_row(int i, int h) { return (i & 3) + 8 * (i >> 2) + 4 * h; }

// load a [rows x D] tile (token stride ld) into registers: NCH chunks per thread
template <int D, int ROWS>
struct TileLoader {
  static constexpr int CH = D / 8;
  static constexpr int NPER = ROWS * CH / 256;
  bf8 v[NPER];
  __device__ __forceinline__ void load(const bf16_t* base, long long ld, int row0, int nrows, int Dv) {
#pragma unroll
    for (int i = 0; i < NPER; ++i) {
      const int idx = threadIdx.x + 256 * i;
      const int r = idx / CH, c = idx % CH;
      const bool ok = (row0 + r < nrows) && (c * 8 < Dv);
      if (ok) v[i] = *reinterpret_cast<const bf8*>(base + (long long)(row0 + r) * ld + c * 8);
      else { v[i].w[0] = v[i].w[1] = v[i].w[2] = v[i].w[3] = 0; }
    }
  }
  __device__ __forceinline__ void store_row(char* img) const {
#pragma unroll
    for (int i = 0; i < NPER; ++i) {
      const int idx = threadIdx.x + 256 * i;
      const int r = idx / CH, c = idx % CH;
      *reinterpret_cast<bf8*>(img + row_off<D>(r, c)) = v[i];
    }
  }
  __device__ __forceinline__ void store_tr(char* img) const {
#pragma unroll
    for (int i = 0; i < NPER; ++i) {
      const int idx = threadIdx.x + 256 * i;
      const int r = idx / CH, c = idx % CH;
      *reinterpret_cast<bf8*>(img + tr_off<D>(r, c * 8)) = v[i];
    }
  }
};

// B-operand fragments of a 32-row block held in registers: lane (r,h) holds X[row0+r][16s+8h .. +7]
template <int D>
__device__ __forceinline__ void load_row_frags(bf16x8 (&f)[D / 16], const bf16_t* base, long long ld, int row0,
                                               int nrows, int Dv) {
  const int lane = threadIdx.x & 63, r = lane & 31, h = lane >> 5;
#pragma unroll
  for (int s = 0; s < D / 16; ++s) {
    const int d = 16 * s + 8 * h;
    if (row0 + r < nrows && d < Dv) f[s] = *reinterpret_cast<const bf16x8*>(base + (long long)(row0 + r) * ld + d);
    else { for (int j = 0; j < 8; ++j) f[s][j] = (__bf16)0.f; }
  }
}

// ------------------------------------------------------------------------------------------
template <int D>
__global__ void __launch_bounds__(256, 2) attn_fwd_kernel(AttnArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int TILE = KT * D * 2;   // bytes of one [64 x D] image
  const int b = blockIdx.z, hh = blockIdx.y;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, r = lane & 31, h = lane >> 5;
  const int q0 = blockIdx.x * 128 + wave * 32;
  const bf16_t* Q = a.q + b * a.bsq + hh * a.Dv;
  const bf16_t* Kp = a.k + b * a.bsk + hh * a.Dv;
  const bf16_t* Vp = a.v + b * a.bsv + hh * a.Dv;

  bf16x8 qf[D / 16];
  load_row_frags<D>(qf, Q, a.ldq, q0, a.Nq, a.Dv);
  const float c = a.scale * LOG2E;

  float16v O[D / 32];
#pragma unroll
  for (int t = 0; t < D / 32; ++t) O[t] = zero16();
  float m = -INFINITY, l = 0.f;

  TileLoader<D, KT> lk, lv;
  const int ntiles = (a.Nk + KT - 1) / KT;
  lk.load(Kp, a.ldk, 0, a.Nk, a.Dv);
  lv.load(Vp, a.ldv, 0, a.Nk, a.Dv);
  lk.store_row(smem);
  lv.store_tr(smem + TILE);
  __syncthreads();
  for (int t = 0; t < ntiles; ++t) {
    const int cur = t & 1;
    const char* kimg = smem + cur * 2 * TILE;
    const char* vimg = kimg + TILE;
    if (t + 1 < ntiles) { lk.load(Kp, a.ldk, (t + 1) * KT, a.Nk, a.Dv); lv.load(Vp, a.ldv, (t + 1) * KT, a.Nk, a.Dv); }
#pragma unroll
    for (int sub = 0; sub < KT / 32; ++sub) {
      float16v S = zero16();
#pragma unroll
      for (int s = 0; s < D / 16; ++s) S = mfma32(lds_row_frag(kimg, D * 2, sub * 32 + r, 2 * s + h), qf[s], S);
      const int kbase = t * KT + sub * 32;
      float tmax = -INFINITY;
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const float sv = (kbase + acc_row(i, h) < a.Nk) ? S[i] * c : -INFINITY;
        S[i] = sv;
        tmax = fmaxf(tmax, sv);
      }
      tmax = fmaxf(tmax, __shfl_xor(tmax, 32, 64));
      const float mn = fmaxf(m, tmax);
      const float alpha = __builtin_amdgcn_exp2f(m - mn);
      float rs = 0.f;
#pragma unroll
      for (int i = 0; i < 16; ++i) { const float p = __builtin_amdgcn_exp2f(S[i] - mn); S[i] = p; rs += p; }
      rs += __shfl_xor(rs, 32, 64);
      l = l * alpha + rs;
      m = mn;
#pragma unroll
      for (int dt = 0; dt < D / 32; ++dt)
#pragma unroll
        for (int i = 0; i < 16; ++i) O[dt][i] *= alpha;
      const bf16x8 p0 = pack_acc(S, 0), p1 = pack_acc(S, 1);
#pragma unroll
      for (int dt = 0; dt < D / 32; ++dt) {
        O[dt] = mfma32(tr_frag<D>(vimg, sub * 32, 0, dt * 32), p0, O[dt]);
        O[dt] = mfma32(tr_frag<D>(vimg, sub * 32, 1, dt * 32), p1, O[dt]);
      }
    }
    if (t + 1 < ntiles) {
      char* nimg = smem + (cur ^ 1) * 2 * TILE;
      lk.store_row(nimg);
      lv.store_tr(nimg + TILE);
    }
    __syncthreads();
  }
  const int q = q0 + r;
  if (q < a.Nq) {
    const float inv = 1.f / l;
    bf16_t* Op = a.o + b * a.bso + (long long)q * a.ldo + hh * a.Dv;
#pragma unroll
    for (int dt = 0; dt < D / 32; ++dt)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int d = dt * 32 + 8 * g + 4 * h;
        if (d < a.Dv) {
          uint2 w;
          w.x = (uint32_t)f2bf(O[dt][4 * g] * inv) | ((uint32_t)f2bf(O[dt][4 * g + 1] * inv) << 16);
          w.y = (uint32_t)f2bf(O[dt][4 * g + 2] * inv) | ((uint32_t)f2bf(O[dt][4 * g + 3] * inv) << 16);
          *reinterpret_cast<uint2*>(Op + d) = w;
        }
      }
    if (h == 0 && a.lse) a.lse[((long long)b * a.H + hh) * a.Nq + q] = m + __log2f(l);
  }
}

// delta[b,h,q] = sum_d dO * O  (fp32)
__global__ void __launch_bounds__(256) attn_bwd_delta_kernel(AttnArgs a, float* __restrict__ delta) {
  const long long total = (long long)a.B * a.Nq * a.H;
  const int lane = threadIdx.x & 63;
  const int sub = lane & 7;    // 8 lanes per row, 8 elements each (Dv <= 64 per pass)
  for (long long row = (blockIdx.x * (long long)blockDim.x + threadIdx.x) / 8; row < total;
       row += (long long)gridDim.x * blockDim.x / 8) {
    const int hh = (int)(row % a.H);
    const long long bq = row / a.H;
    const int q = (int)(bq % a.Nq), b = (int)(bq / a.Nq);
    const bf16_t* Op = a.o + b * a.bso + (long long)q * a.ldo + hh * a.Dv;
    const bf16_t* Gp = a.dout + b * a.bsdo + (long long)q * a.lddo + hh * a.Dv;
    float s = 0.f;
    for (int d = sub * 8; d < a.Dv; d += 64) {
      bf8 ov = *reinterpret_cast<const bf8*>(Op + d);
      bf8 gv = *reinterpret_cast<const bf8*>(Gp + d);
      float of[8], gf[8];
      unpack8(ov, of);
      unpack8(gv, gf);
#pragma unroll
      for (int j = 0; j < 8; ++j) s = fmaf(of[j], gf[j], s);
    }
    s += __shfl_xor(s, 1, 64);
    s += __shfl_xor(s, 2, 64);
    s += __shfl_xor(s, 4, 64);
    if (sub == 0) delta[((long long)b * a.H + hh) * a.Nq + q] = s;
  }
}

// dQ: per wave 32 queries, iterate over key tiles
template <int D>
__global__ void __launch_bounds__(256, 2) attn_bwd_dq_kernel(AttnArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int TILE = KT * D * 2;
  const int b = blockIdx.z, hh = blockIdx.y;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, r = lane & 31, h = lane >> 5;
  const int q0 = blockIdx.x * 128 + wave * 32;
  const bf16_t* Kp = a.k + b * a.bsk + hh * a.Dv;
  const bf16_t* Vp = a.v + b * a.bsv + hh * a.Dv;
  bf16x8 qf[D / 16], gf[D / 16];
  load_row_frags<D>(qf, a.q + b * a.bsq + hh * a.Dv, a.ldq, q0, a.Nq, a.Dv);
  load_row_frags<D>(gf, a.dout + b * a.bsdo + hh * a.Dv, a.lddo, q0, a.Nq, a.Dv);
  const float c = a.scale * LOG2E;
  const int q = q0 + r;
  const long long srow = ((long long)b * a.H + hh) * a.Nq;
  const float lse2 = q < a.Nq ? a.lse[srow + q] : 0.f;
  const float dlt = q < a.Nq ? a.delta[srow + q] : 0.f;

  float16v dQ[D / 32];
#pragma unroll
  for (int t = 0; t < D / 32; ++t) dQ[t] = zero16();

  TileLoader<D, KT> lk, lv;
  const int ntiles = (a.Nk + KT - 1) / KT;
  lk.load(Kp, a.ldk, 0, a.Nk, a.Dv);
  lv.load(Vp, a.ldv, 0, a.Nk, a.Dv);
  lk.store_row(smem);
  lk.store_tr(smem + TILE);
  lv.store_row(smem + 2 * TILE);
  __syncthreads();
  for (int t = 0; t < ntiles; ++t) {
    const int cur = t & 1;
    const char* krow = smem + cur * 3 * TILE;
    const char* ktr = krow + TILE;
    const char* vrow = krow + 2 * TILE;
    if (t + 1 < ntiles) { lk.load(Kp, a.ldk, (t + 1) * KT, a.Nk, a.Dv); lv.load(Vp, a.ldv, (t + 1) * KT, a.Nk, a.Dv); }
#pragma unroll
    for (int sub = 0; sub < KT / 32; ++sub) {
      float16v S = zero16(), dP = zero16();
#pragma unroll
      for (int s = 0; s < D / 16; ++s) {
        S = mfma32(lds_row_frag(krow, D * 2, sub * 32 + r, 2 * s + h), qf[s], S);
        dP = mfma32(lds_row_frag(vrow, D * 2, sub * 32 + r, 2 * s + h), gf[s], dP);
      }
      const int kbase = t * KT + sub * 32;
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const bool ok = kbase + acc_row(i, h) < a.Nk;
        const float p = ok ? __builtin_amdgcn_exp2f(S[i] * c - lse2) : 0.f;
        S[i] = p * (dP[i] - dlt);   // dS^T
      }
      const bf16x8 s0 = pack_acc(S, 0), s1 = pack_acc(S, 1);
#pragma unroll
      for (int dt = 0; dt < D / 32; ++dt) {
        dQ[dt] = mfma32(tr_frag<D>(ktr, sub * 32, 0, dt * 32), s0, dQ[dt]);
        dQ[dt] = mfma32(tr_frag<D>(ktr, sub * 32, 1, dt * 32), s1, dQ[dt]);
      }
    }
    if (t + 1 < ntiles) {
      char* nimg = smem + (cur ^ 1) * 3 * TILE;
      lk.store_row(nimg);
      lk.store_tr(nimg + TILE);
      lv.store_row(nimg + 2 * TILE);
    }
    __syncthreads();
  }
  if (q < a.Nq) {
    bf16_t* Dp = a.dq + b * a.bsdq + (long long)q * a.lddq + hh * a.Dv;
#pragma unroll
    for (int dt = 0; dt < D / 32; ++dt)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int d = dt * 32 + 8 * g + 4 * h;
        if (d < a.Dv) {
          uint2 w;
          w.x = (uint32_t)f2bf(dQ[dt][4 * g] * a.scale) | ((uint32_t)f2bf(dQ[dt][4 * g + 1] * a.scale) << 16);
          w.y = (uint32_t)f2bf(dQ[dt][4 * g + 2] * a.scale) | ((uint32_t)f2bf(dQ[dt][4 * g + 3] * a.scale) << 16);
          *reinterpret_cast<uint2*>(Dp + d) = w;
        }
      }
  }
}

// dK, dV: per wave 32 keys (block 128 keys), iterate over query tiles of 32 in this split's range
template <int D>
__global__ void __launch_bounds__(256, 2) attn_bwd_dkv_kernel(AttnArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int TILE = QT * D * 2;                 // one [32 x D] image
  constexpr int STAGE = 4 * TILE + 2 * QT * 4;     // q row, q tr, do row, do tr, lse2, delta
  const int bz = blockIdx.z;
  const int b = bz / a.qsplit, split = bz % a.qsplit;
  const int hh = blockIdx.y;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, r = lane & 31, h = lane >> 5;
  const int k0 = blockIdx.x * 128 + wave * 32;
  bf16x8 kf[D / 16], vf[D / 16];
  load_row_frags<D>(kf, a.k + b * a.bsk + hh * a.Dv, a.ldk, k0, a.Nk, a.Dv);
  load_row_frags<D>(vf, a.v + b * a.bsv + hh * a.Dv, a.ldv, k0, a.Nk, a.Dv);
  const float c = a.scale * LOG2E;
  const bf16_t* Qp = a.q + b * a.bsq + hh * a.Dv;
  const bf16_t* Gp = a.dout + b * a.bsdo + hh * a.Dv;
  const long long srow = ((long long)b * a.H + hh) * a.Nq;

  const int per = (((a.Nq + a.qsplit - 1) / a.qsplit) + QT - 1) / QT * QT;
  const int qbeg = split * per;
  const int qend = min(a.Nq, qbeg + per);
  const int ntiles = qend > qbeg ? (qend - qbeg + QT - 1) / QT : 0;

  float16v dK[D / 32], dV[D / 32];
#pragma unroll
  for (int t = 0; t < D / 32; ++t) { dK[t] = zero16(); dV[t] = zero16(); }

  TileLoader<D, QT> lq, lg;
  float ls_v = 0.f, dl_v = 0.f;   // thread t < 32 stages lse2/delta of query t
  auto load_stage = [&](int qt0) {
    lq.load(Qp, a.ldq, qt0, qend, a.Dv);
    lg.load(Gp, a.lddo, qt0, qend, a.Dv);
    if (threadIdx.x < QT) {
      const int qq = qt0 + threadIdx.x;
      ls_v = qq < qend ? a.lse[srow + qq] : INFINITY;
      dl_v = qq < qend ? a.delta[srow + qq] : 0.f;
    }
  };
  auto store_stage = [&](char* st) {
    lq.store_row(st);
    lq.store_tr(st + TILE);
    lg.store_row(st + 2 * TILE);
    lg.store_tr(st + 3 * TILE);
    if (threadIdx.x < QT) {
      reinterpret_cast<float*>(st + 4 * TILE)[threadIdx.x] = ls_v;
      reinterpret_cast<float*>(st + 4 * TILE)[QT + threadIdx.x] = dl_v;
    }
  };
  if (ntiles > 0) {
    load_stage(qbeg);
    store_stage(smem);
    __syncthreads();
  }
  for (int t = 0; t < ntiles; ++t) {
    const int cur = t & 1;
    const char* st = smem + cur * STAGE;
    const char* qrow = st;
    const char* qtr = st + TILE;
    const char* grow = st + 2 * TILE;
    const char* gtr = st + 3 * TILE;
    const float* lsv = reinterpret_cast<const float*>(st + 4 * TILE);
    const float* dlv = lsv + QT;
    if (t + 1 < ntiles) load_stage(qbeg + (t + 1) * QT);
    float16v S = zero16(), dP = zero16();
#pragma unroll
    for (int s = 0; s < D / 16; ++s) {
      S = mfma32(lds_row_frag(qrow, D * 2, r, 2 * s + h), kf[s], S);
      dP = mfma32(lds_row_frag(grow, D * 2, r, 2 * s + h), vf[s], dP);
    }
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int qr = acc_row(i, h);
      const float p = __builtin_amdgcn_exp2f(S[i] * c - lsv[qr]);
      S[i] = p;
      dP[i] = p * (dP[i] - dlv[qr]);
    }
    const bf16x8 p0 = pack_acc(S, 0), p1 = pack_acc(S, 1);
    const bf16x8 s0 = pack_acc(dP, 0), s1 = pack_acc(dP, 1);
#pragma unroll
    for (int dt = 0; dt < D / 32; ++dt) {
      dV[dt] = mfma32(tr_frag<D>(gtr, 0, 0, dt * 32), p0, dV[dt]);
      dV[dt] = mfma32(tr_frag<D>(gtr, 0, 1, dt * 32), p1, dV[dt]);
      dK[dt] = mfma32(tr_frag<D>(qtr, 0, 0, dt * 32), s0, dK[dt]);
      dK[dt] = mfma32(tr_frag<D>(qtr, 0, 1, dt * 32), s1, dK[dt]);
    }
    if (t + 1 < ntiles) store_stage(smem + (cur ^ 1) * STAGE);
    __syncthreads();
  }
  const int key = k0 + r;
  if (key < a.Nk) {
#pragma unroll
    for (int dt = 0; dt < D / 32; ++dt)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int d = dt * 32 + 8 * g + 4 * h;
        if (d >= a.Dv) continue;
        if (a.qsplit > 1) {
          float* kp = a.dk32 + (((long long)b * a.Nk + key) * a.H + hh) * a.Dv + d;
          float* vp = a.dv32 + (((long long)b * a.Nk + key) * a.H + hh) * a.Dv + d;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            atomicAdd(kp + e, dK[dt][4 * g + e] * a.scale);
            atomicAdd(vp + e, dV[dt][4 * g + e]);
          }
        } else {
          bf16_t* kp = a.dk + b * a.bsdk + (long long)key * a.lddk + hh * a.Dv + d;
          bf16_t* vp = a.dv + b * a.bsdv + (long long)key * a.lddv + hh * a.Dv + d;
          uint2 w;
          w.x = (uint32_t)f2bf(dK[dt][4 * g] * a.scale) | ((uint32_t)f2bf(dK[dt][4 * g + 1] * a.scale) << 16);
          w.y = (uint32_t)f2bf(dK[dt][4 * g + 2] * a.scale) | ((uint32_t)f2bf(dK[dt][4 * g + 3] * a.scale) << 16);
          *reinterpret_cast<uint2*>(kp) = w;
          w.x = (uint32_t)f2bf(dV[dt][4 * g]) | ((uint32_t)f2bf(dV[dt][4 * g + 1]) << 16);
          w.y = (uint32_t)f2bf(dV[dt][4 * g + 2]) | ((uint32_t)f2bf(dV[dt][4 * g + 3]) << 16);
          *reinterpret_cast<uint2*>(vp) = w;
        }
      }
  }
}

// fp32 [B, Nk, H, Dv] partials -> bf16 dK / dV with their strides
__global__ void attn_dkv_cast_kernel(AttnArgs a) {
  const long long total = (long long)a.B * a.Nk * a.H * a.Dv;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total; i += (long long)gridDim.x * blockDim.x) {
    const int d = (int)(i % a.Dv);
    long long t = i / a.Dv;
    const int hh = (int)(t % a.H);
    t /= a.H;
    const int key = (int)(t % a.Nk), b = (int)(t / a.Nk);
    a.dk[b * a.bsdk + (long long)key * a.lddk + hh * a.Dv + d] = f2bf(a.dk32[i]);
    a.dv[b * a.bsdv + (long long)key * a.lddv + hh * a.Dv + d] = f2bf(a.dv32[i]);
  }
}

static bool attn_ok(const AttnArgs& a) {
  if (a.B <= 0 || a.H <= 0 || a.Nq <= 0 || a.Nk <= 0 || a.Dv <= 0 || a.Dv % 8 || a.Dv > 128) return false;
  const long long lds[] = {a.ldq, a.ldk, a.ldv, a.bsq, a.bsk, a.bsv};
  for (long long v : lds) if (v % 8) return false;
  if (((uintptr_t)a.q | (uintptr_t)a.k | (uintptr_t)a.v) & 15) return false;
  return true;
}

OTAMD_API int otamd_attn_fwd(const AttnArgs* in, hipStream_t stream) {
  if (!in || !attn_ok(*in) || !in->o || !in->lse) return OTAMD_EINVAL;
  AttnArgs a = *in;
  if (a.ldo % 4 || a.bso % 4) return OTAMD_EINVAL;
  dim3 grid((a.Nq + 127) / 128, a.H, a.B);
  if (a.Dv <= 64) hipLaunchKernelGGL(attn_fwd_kernel<64>, grid, dim3(256), 2 * 2 * KT * 64 * 2, stream, a);
  else hipLaunchKernelGGL(attn_fwd_kernel<128>, grid, dim3(256), 2 * 2 * KT * 128 * 2, stream, a);
  OTAMD_CHECK_LAUNCH();
  return OTAMD_OK;
}

// ws: float[B*H*Nq] for delta + (qsplit>1 ? 2*B*Nk*H*Dv floats) ; lse from the forward
OTAMD_API int otamd_attn_bwd(const AttnArgs* in, float* ws, long long ws_bytes, hipStream_t stream) {
  if (!in || !attn_ok(*in) || !in->o || !in->lse || !in->dout || !in->dq || !in->dk || !in->dv || !ws) return OTAMD_EINVAL;
  AttnArgs a = *in;
  if (a.lddo % 8 || a.bsdo % 8 || a.lddq % 4 || a.lddk % 4 || a.lddv % 4) return OTAMD_EINVAL;
  const long long nrow = (long long)a.B * a.H * a.Nq;
  const long long nkv = (long long)a.B * a.Nk * a.H * a.Dv;
  // parallelism for dK/dV: split the query range when there are few key blocks
  const int kblocks = (a.Nk + 127) / 128;
  int qsplit = 1;
  while (kblocks * a.H * a.B * qsplit < 512 && qsplit < 64 && (a.Nq / (qsplit * 2)) >= 128) qsplit *= 2;
  a.qsplit = qsplit;
  const long long need = nrow * 4 + (qsplit > 1 ? 2 * nkv * 4 : 0);
  if (ws_bytes < need) return OTAMD_EINVAL;
  float* delta = ws;
  a.delta = delta;
  if (qsplit > 1) {
    a.dk32 = ws + ((nrow + 3) / 4) * 4;
    a.dv32 = a.dk32 + nkv;
    if (hipMemsetAsync(a.dk32, 0, 2 * nkv * 4, stream) != hipSuccess) return OTAMD_ELAUNCH;
  }
  {
    long long threads = nrow * 8;
    int blocks = (int)std::min<long long>((threads + 255) / 256, 8192);
    attn_bwd_delta_kernel<<<blocks, 256, 0, stream>>>(a, delta);
    OTAMD_CHECK_LAUNCH();
  }
  dim3 gq((a.Nq + 127) / 128, a.H, a.B);
  dim3 gk(kblocks, a.H, a.B * qsplit);
  if (a.Dv <= 64) {
    hipLaunchKernelGGL(attn_bwd_dq_kernel<64>, gq, dim3(256), 2 * 3 * KT * 64 * 2, stream, a);
    hipLaunchKernelGGL(attn_bwd_dkv_kernel<64>, gk, dim3(256), 2 * (4 * QT * 64 * 2 + 2 * QT * 4), stream, a);
  } else {
    hipLaunchKernelGGL(attn_bwd_dq_kernel<128>, gq, dim3(256), 2 * 3 * KT * 128 * 2, stream, a);
    hipLaunchKernelGGL(attn_bwd_dkv_kernel<128>, gk, dim3(256), 2 * (4 * QT * 128 * 2 + 2 * QT * 4), stream, a);
  }
  OTAMD_CHECK_LAUNCH();
  if (qsplit > 1) {
    int blocks = (int)std::min<long long>((nkv + 255) / 256, 8192);
    attn_dkv_cast_kernel<<<blocks, 256, 0, stream>>>(a);
    OTAMD_CHECK_LAUNCH();
  }
  return OTAMD_OK;
}

OTAMD_API int otamd_attn_args_size(void) { return (int)sizeof(AttnArgs); }
