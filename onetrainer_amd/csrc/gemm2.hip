// bf16 MFMA GEMM engine v2: 8 waves, 256-wide tiles, LDS-DMA staging (gfx950).
//
// Same operand modes / epilogues as gemm.hip (see its header for the op -> mode table), but
// built for the L2->CU bandwidth budget of MI355X: a 128x128 tile needs ~64 B/clk/CU of operand
// traffic at full MFMA rate, more than the XCD L2 delivers; 256x256 halves it.
//   * tiles 256x256 (8 waves as 2x4, 128x64 each), 256x128 or 128x256 (8 waves, 64x64 each);
//   * operands are moved HBM/L2 -> LDS by `buffer_load_dwordx4 ... lds` (LDS-DMA): no VGPR
//     staging, and the buffer descriptor's range check zero-fills every out-of-range lane, which
//     is how conv padding / tile tails become zeros;
//   * LDS images are lane-linear per 1 KiB DMA piece; the XOR swizzles that make ds_read_b128 /
//     ds_read_b64_tr_b16 bank-conflict free are applied on the SOURCE address (rule 21);
//   * two LDS stages, raw s_barrier, counted s_waitcnt vmcnt(N): the next tile's DMA stays in
//     flight across the barrier while the current one is multiplied.
#include "gemm.h"

#include <mutex>
#include <unordered_set>
#include <map>
#include <algorithm>

typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(3))) short4v lds_s4_t;
#define OFF_INVALID 0x80000000u

#define MEMBAR() asm volatile("" ::: "memory")
#define BARRIER()                      \
  do {                                 \
    MEMBAR();                          \
    __builtin_amdgcn_s_barrier();      \
    MEMBAR();                          \
  } while (0)

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  if constexpr (N == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  else if constexpr (N == 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  else if constexpr (N == 6) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
  else if constexpr (N == 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  else if constexpr (N == 12) asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
  else if constexpr (N == 16) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
  else static_assert(N == 0, "unsupported vmcnt");
}

// One 16-byte-per-lane LDS-DMA (1 KiB per wave). Issued as inline asm on purpose: the compiler's
// waitcnt pass cannot prove that a later ds_read of the OTHER LDS stage does not alias an
// in-flight builtin LDS-DMA and would drain vmcnt in front of it, serialising the pipeline.
// Ordering is owned here: every read of a stage follows wait_vmcnt<> + BARRIER on its DMA.
__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t rs, char* lds, unsigned off) {
  const unsigned m0 = (unsigned)(size_t)(lds_void_t*)lds;
  asm volatile("buffer_load_dwordx4 %1, %2, 0 offen lds" ::"{m0}"(m0), "v"(off), "s"(rs) : "memory");
}

template <int MODE> struct IsKMode {
  static constexpr bool v = (MODE == OPM_K || MODE == OPM_CONV_FWD || MODE == OPM_CONV_DGRAD);
};

// Per-lane DMA state of one operand tile (BMN rows/cols x 64 k): BMN/8 pieces of 1 KiB, NW waves
// take NI = BMN/(8 NW) each (piece j = wave + NW i).
template <int MODE, int BMN, int NW>
struct Stage {
  static constexpr bool KM = IsKMode<MODE>::v;
  static constexpr int NI = BMN / (8 * NW);
  static constexpr int RB = BMN * 2;      // MN-mode row bytes
  int a[NI], b[NI], c[NI];                // K: (row elem offset | conv n,y0,x0) ; MN: (k row, col, -)
  int t0, t1, t2;                         // K: logical chunk ; MN-conv: per-piece decode lives in a/b/c
  bool ok[NI];

  __device__ __forceinline__ void prepare(const ConvGeom& g, long long ld, int mn0, int MNsz, int wave, int lane) {
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int j = wave + NW * i;
      if constexpr (KM) {
        const int r = 8 * j + (lane >> 3);
        const int gm = mn0 + r;
        ok[i] = gm < MNsz;
        if constexpr (MODE == OPM_K) {
          a[i] = gm * (int)ld;
        } else {
          const int rr = ok[i] ? gm : 0;
          const int hw = g.RH * g.RW;
          const int n = rr / hw, rem = rr - n * hw;
          const int y = rem / g.RW, x = rem - y * g.RW;
          a[i] = n;
          if constexpr (MODE == OPM_CONV_FWD) { b[i] = y * g.stride - g.pad; c[i] = x * g.stride - g.pad; }
          else { b[i] = y + g.pad; c[i] = x + g.pad; }
        }
      } else {
        const int byte = j * 1024 + lane * 16;
        const int r = byte / RB;
        const int pc = (byte % RB) >> 4;
        const int lb = (pc >> 1) ^ mn_swz(r);
        const int col = mn0 + (lb * 2 + (pc & 1)) * 8;
        a[i] = r;
        ok[i] = col < MNsz;
        if constexpr (MODE == OPM_MN || MODE == OPM_CONV_WT) {
          b[i] = col;
        } else {   // OPM_CONV_WGRAD: col = (tap, ch)
          const int cc = ok[i] ? col : 0;
          const int tap = cc / g.SC;
          c[i] = cc - tap * g.SC;
          b[i] = tap;
        }
      }
    }
    if constexpr (KM) t0 = (lane & 7) ^ ((lane >> 3) & 7);
  }

  __device__ __forceinline__ void issue(__amdgpu_buffer_rsrc_t rs, char* img, const ConvGeom& g, long long ld, int k0,
                                        int Kend, int wave) {
    if constexpr (KM) {
      const int k = k0 + 8 * t0;
      const bool kok = k < Kend;
      int r_ = 0, s_ = 0, ch = 0;
      if constexpr (MODE != OPM_K) {
        const int tap = kok ? k / g.SC : 0;
        ch = k - tap * g.SC;
        r_ = tap / g.KW;
        s_ = tap - r_ * g.KW;
      }
#pragma unroll
      for (int i = 0; i < NI; ++i) {
        unsigned off = OFF_INVALID;
        if constexpr (MODE == OPM_K) {
          if (kok && ok[i]) off = (unsigned)(a[i] + k) * 2u;
        } else {
          bool v = kok && ok[i];
          int sy, sx;
          if constexpr (MODE == OPM_CONV_FWD) {
            const int y = b[i] + r_, x = c[i] + s_;
            if (g.upsample) { v = v && y >= 0 && y < 2 * g.SH && x >= 0 && x < 2 * g.SW; sy = y >> 1; sx = x >> 1; }
            else { v = v && y >= 0 && y < g.SH && x >= 0 && x < g.SW; sy = y; sx = x; }
          } else {
            const int ty = b[i] - r_, tx = c[i] - s_;
            if (g.stride == 1) { sy = ty; sx = tx; }
            else {
              v = v && ty >= 0 && tx >= 0 && (ty % g.stride) == 0 && (tx % g.stride) == 0;
              sy = ty / g.stride; sx = tx / g.stride;
            }
            v = v && sy >= 0 && sy < g.SH && sx >= 0 && sx < g.SW;
          }
          if (v) off = (unsigned)(((a[i] * g.SH + sy) * g.SW + sx) * (int)g.ld + ch) * 2u;
        }
        dma16(rs, img + (wave + NW * i) * 1024, off);
      }
    } else {
#pragma unroll
      for (int i = 0; i < NI; ++i) {
        const int k = k0 + a[i];
        unsigned off = OFF_INVALID;
        if constexpr (MODE == OPM_MN) {
          if (ok[i] && k < Kend) off = (unsigned)(k * (int)ld + b[i]) * 2u;
        } else if constexpr (MODE == OPM_CONV_WT) {   // k = tap*Cout + co -> W row co*KK + tap
          if (ok[i] && k < Kend) {
            const int tap = k / g.SC, co = k - tap * g.SC;
            off = (unsigned)((co * (g.KH * g.KW) + tap) * (int)ld + b[i]) * 2u;
          }
        } else {   // conv wgrad: k = output pixel
          bool v = ok[i] && k < Kend;
          const int kk = v ? k : 0;
          const int hw = g.RH * g.RW;
          const int n = kk / hw, rem = kk - n * hw;
          const int p = rem / g.RW, q = rem - p * g.RW;
          const int tr = b[i] / g.KW, ts = b[i] - (b[i] / g.KW) * g.KW;
          const int y = p * g.stride - g.pad + tr, x = q * g.stride - g.pad + ts;
          int sy, sx;
          if (g.upsample) { v = v && y >= 0 && y < 2 * g.SH && x >= 0 && x < 2 * g.SW; sy = y >> 1; sx = x >> 1; }
          else { v = v && y >= 0 && y < g.SH && x >= 0 && x < g.SW; sy = y; sx = x; }
          if (v) off = (unsigned)(((n * g.SH + sy) * g.SW + sx) * (int)g.ld + c[i]) * 2u;
        }
        dma16(rs, img + (wave + NW * i) * 1024, off);
      }
    }
  }
};

// fragment of a 16x16x32 operand: lane holds X[mnb + (lane&15)][kb + 8*(lane>>4) + j]
__device__ __forceinline__ bf16x8 frag_k2(const char* img, int mnb, int kb) {
  const int lane = threadIdx.x & 63;
  const int row = mnb + (lane & 15);
  return *reinterpret_cast<const bf16x8*>(img + kimg_off(row, (kb >> 3) + (lane >> 4)));
}
template <int RB>
__device__ __forceinline__ int mn_off(int k, int col) {
  return k * RB + ((((col >> 4)) ^ mn_swz(k)) << 5) + ((col & 15) << 1);
}
template <int RB>
__device__ __forceinline__ bf16x8 frag_mn2(const char* img, int mnb, int kb) {
  const int lane = threadIdx.x & 63;
  const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
  const int k0 = kb + 8 * g + q;
  const int col = mnb + 4 * p;
  const short4v lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4_t*)(img + mn_off<RB>(k0, col)));
  const short4v hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4_t*)(img + mn_off<RB>(k0 + 4, col)));
  short8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8, v);
}

// NW = 8: 2 waves/SIMD (<= 256 VGPRs), wave tiles 128x64 / 64x64.  NW = 4: 1 wave/SIMD (512-entry
// unified VGPR/AGPR file), 256x256 as 2x2 wave tiles of 128x128 -- a third less LDS read traffic
// per MFMA (one 16x16x32 fragment read per 4 MFMAs instead of per 2.7).
__device__ __forceinline__ void* sgpr_ptr(const void* p) {
  const unsigned long long v = (unsigned long long)p;
  const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)v), hi = __builtin_amdgcn_readfirstlane((unsigned)(v >> 32));
  return (void*)(((unsigned long long)hi << 32) | lo);
}

template <int AM, int BMODE, int BM, int BN, int NW, bool SEG2>
struct G2 {
  static constexpr int WN = NW == 4 ? 2 : ((BM == 256 && BN == 128) ? 2 : 4);
  static constexpr int WM = NW / WN;
  static constexpr int TM = BM / WM, TN = BN / WN;
  static constexpr int MI = TM / 16, NJ = TN / 16;
  static constexpr int ABYTES = BM * 128, BBYTES = BN * 128;
  static constexpr int STAGE = ABYTES + BBYTES;
  static constexpr int LOADS = Stage<AM, BM, NW>::NI + Stage<BMODE, BN, NW>::NI;
  static constexpr bool AK = IsKMode<AM>::v, BKm = IsKMode<BMODE>::v;
};

// acc += A[m0.., k] B[k, n0..] over the K-tiles [kbeg, kend) of one output tile (2 LDS stages)
template <int AM, int BMODE, int BM, int BN, int NW, bool SEG2>
__device__ __forceinline__ void g2_mainloop(const GemmArgs& args, char* smem, int m0, int n0, int kbeg, int kend,
                                            unsigned a_bytes, unsigned b_bytes, unsigned a2_bytes, unsigned b2_bytes,
                                            float4v (&acc)[G2<AM, BMODE, BM, BN, NW, SEG2>::MI][G2<AM, BMODE, BM, BN, NW, SEG2>::NJ]) {
  using T = G2<AM, BMODE, BM, BN, NW, SEG2>;
  constexpr int WN = T::WN, TM = T::TM, TN = T::TN, MI = T::MI, NJ = T::NJ;
  constexpr int ABYTES = T::ABYTES, STAGE = T::STAGE, LOADS = T::LOADS;
  constexpr bool AK = T::AK, BKm = T::BKm;
  const int nk = (kend - kbeg + 63) / 64;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;

  // (the base pointers are wave-uniform; readfirstlane keeps the descriptors in SGPRs even when the
  // batched kernel's offset copy of args lives in private memory)
  const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc(sgpr_ptr(args.A), (short)0, (int)a_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc(sgpr_ptr(args.B), (short)0, (int)b_bytes, 0x00020000);
  Stage<AM, BM, NW> sa;
  Stage<BMODE, BN, NW> sb;
  sa.prepare(args.ga, args.lda, m0, args.M, wave, lane);
  sb.prepare(args.gb, args.ldb, n0, args.N, wave, lane);
  // second K segment: A2 always K-mode; B2 in the LDS image mode of B
  constexpr int B2M = BKm ? OPM_K : OPM_MN;
  Stage<OPM_K, SEG2 ? BM : 64 * NW / 8, NW> sa2;
  Stage<B2M, SEG2 ? BN : 64 * NW / 8, NW> sb2;
  __amdgpu_buffer_rsrc_t ra2 = ra, rb2 = rb;
  if constexpr (SEG2) {
    ra2 = __builtin_amdgcn_make_buffer_rsrc(sgpr_ptr(args.A2), (short)0, (int)a2_bytes, 0x00020000);
    rb2 = __builtin_amdgcn_make_buffer_rsrc(sgpr_ptr(args.B2), (short)0, (int)b2_bytes, 0x00020000);
    sa2.prepare(args.ga, args.lda2, m0, args.M, wave, lane);
    sb2.prepare(args.gb, args.ldb2, n0, args.N, wave, lane);
  }
  // K tile at k0 (never straddles K1: K1 % 64 == 0) into the stage at img
  auto issue_tile = [&](char* img, int k0) {
    if (!SEG2 || k0 < args.K1) {
      sa.issue(ra, img, args.ga, args.lda, k0, SEG2 ? args.K1 : kend, wave);
      sb.issue(rb, img + ABYTES, args.gb, args.ldb, k0, SEG2 ? args.K1 : kend, wave);
    } else {
      sa2.issue(ra2, img, args.ga, args.lda2, k0 - args.K1, args.K2, wave);
      sb2.issue(rb2, img + ABYTES, args.gb, args.ldb2, k0 - args.K1, args.K2, wave);
    }
  };

  const int wm = wave / WN, wn = wave % WN;
  // fragment loaders (h selects the 32-wide half of the 64-deep K tile)
  auto load_a = [&](bf16x8 (&f)[MI], const char* ia, int h) {
#pragma unroll
    for (int i = 0; i < MI; ++i) f[i] = AK ? frag_k2(ia, wm * TM + i * 16, 32 * h) : frag_mn2<BM * 2>(ia, wm * TM + i * 16, 32 * h);
  };
  auto load_b = [&](bf16x8 (&f)[NJ], const char* ib, int h) {
#pragma unroll
    for (int j = 0; j < NJ; ++j) f[j] = BKm ? frag_k2(ib, wn * TN + j * 16, 32 * h) : frag_mn2<BN * 2>(ib, wn * TN + j * 16, 32 * h);
  };
  auto mfma_block = [&](const bf16x8 (&fa)[MI], const bf16x8 (&fb)[NJ]) {
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[j], fa[i], acc[i][j], 0, 0, 0);
  };
  // interleave the next fragment reads into the current MFMA block: {2 MFMA, reads of 1 fragment} x (MI+NJ)
  // (128x128: 8 MFMAs per half for 6 fragment reads -> {1 MFMA, reads} x 6, then the rest)
  constexpr int NR = MI + NJ;
  constexpr int PER = (MI * NJ) / NR >= 2 ? 2 : 1;
  constexpr int REST = MI * NJ - PER * NR;
  auto interleave = [&]() {
#pragma unroll
    for (int t = 0; t < NR; ++t) {
      __builtin_amdgcn_sched_group_barrier(0x008, PER, 0);
      __builtin_amdgcn_sched_group_barrier(0x100, AK && BKm ? 1 : 2, 0);
    }
    if constexpr (REST > 0) __builtin_amdgcn_sched_group_barrier(0x008, REST, 0);
  };

  // Pipeline, ONE barrier per K-step:
  //   phase A: MFMA(h0 of tile k) || ds_read(h1 of tile k)
  //   wait DMA(tile k+1); barrier  -- RAW for tile k+1, WAR for tile k's stage (all its reads retired)
  //   DMA(tile k+2) -> stage of tile k
  //   phase B: MFMA(h1 of tile k) || ds_read(h0 of tile k+1)
  bf16x8 fa0[MI], fb0[NJ], fa1[MI], fb1[NJ];
  if (nk > 0) {
    issue_tile(smem, kbeg);
    if (nk > 1) {
      issue_tile(smem + STAGE, kbeg + 64);
      wait_vmcnt<LOADS>();
    } else {
      wait_vmcnt<0>();
    }
    BARRIER();
    load_b(fb0, smem + ABYTES, 0);
    load_a(fa0, smem, 0);
  }
  for (int kt = 0; kt < nk; ++kt) {
    const char* ia = smem + (kt & 1) * STAGE;
    const char* ib = ia + ABYTES;
    // phase A
    __builtin_amdgcn_sched_barrier(0);
    load_b(fb1, ib, 1);
    load_a(fa1, ia, 1);
    mfma_block(fa0, fb0);
    interleave();
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    wait_vmcnt<0>();       // tile k+1 (the only DMA in flight) has landed
    BARRIER();
    if (kt + 2 < nk) issue_tile(smem + (kt & 1) * STAGE, kbeg + (kt + 2) * 64);
    // phase B
    __builtin_amdgcn_sched_barrier(0);
    {   // on the last step this reads a stale stage; harmless and keeps the loop branch-free
      const char* na = smem + ((kt + 1) & 1) * STAGE;
      load_b(fb0, na + ABYTES, 0);
      load_a(fa0, na, 0);
      mfma_block(fa1, fb1);
      interleave();
    }
    __builtin_amdgcn_sched_barrier(0);
  }
}

// epilogue of one tile: C (or a split-K slab) <- alpha * acc (+ bias, rowvec, residual, C)
template <int AM, int BMODE, int BM, int BN, int NW, bool SEG2>
__device__ __forceinline__ void g2_store(const GemmArgs& args, int m0, int n0, int split, bool use_slab,
                                         float4v (&acc)[G2<AM, BMODE, BM, BN, NW, SEG2>::MI][G2<AM, BMODE, BM, BN, NW, SEG2>::NJ],
                                         int u_lo = 0, int u_hi = 1 << 30) {
  // (u_lo, u_hi: only the store units (i / 2) * NJ + j in [u_lo, u_hi) -- the cooperative fix-up's slice)
  using T = G2<AM, BMODE, BM, BN, NW, SEG2>;
  constexpr int WN = T::WN, TM = T::TM, TN = T::TN, MI = T::MI, NJ = T::NJ;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const int wm = wave / WN, wn = wave % WN;
  const int g = lane >> 4;
  if (use_slab || gemm_wide_ok(args)) {
    // Row blocks (i, i+1) of one column block exchange lane groups with v_permlane16_swap:
    // afterwards lane group g holds 8 consecutive columns 8(g>>1).. of row block i + (g&1).
#pragma unroll
    for (int i = 0; i < MI; i += 2) {
      const int m = m0 + wm * TM + (i + (g & 1)) * 16 + (lane & 15);
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        float v[8];
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(acc[i][j][t]), __float_as_uint(acc[i + 1][j][t]),
                                                          false, false);
          v[t] = __uint_as_float(r[0]);
          v[4 + t] = __uint_as_float(r[1]);
        }
        const int n = n0 + wn * TN + j * 16 + 8 * (g >> 1);
        if ((i / 2) * NJ + j < u_lo || (i / 2) * NJ + j >= u_hi) continue;
        if (m >= args.M || n >= args.N) continue;
        if (n + 8 <= args.N) {
          gemm_store8(args, m, n, v, split, use_slab);
        } else {
          float v4[4] = {v[0], v[1], v[2], v[3]};
          gemm_store4(args, m, n, v4, split, use_slab);
        }
      }
    }
    return;
  }
#pragma unroll
  for (int i = 0; i < MI; ++i) {
    const int m = m0 + wm * TM + i * 16 + (lane & 15);
    if (m >= args.M) continue;
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int n = n0 + wn * TN + j * 16 + 4 * g;
      if ((i / 2) * NJ + j < u_lo || (i / 2) * NJ + j >= u_hi) continue;
      if (n >= args.N) continue;
      float v[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
      gemm_store4(args, m, n, v, split, use_slab);
    }
  }
}

template <int AM, int BMODE, int BM, int BN, int NW, bool SEG2>
__global__ void __launch_bounds__(NW * 64, (BM == 128 && BN == 128) ? 4 : NW / 4) gemm2_kernel(GemmArgs args, unsigned a_bytes, unsigned b_bytes,
                                                                 unsigned a2_bytes, unsigned b2_bytes) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  using T = G2<AM, BMODE, BM, BN, NW, SEG2>;
  constexpr int MI = T::MI, NJ = T::NJ;
  if constexpr (!SEG2 && AM <= OPM_MN && BMODE <= OPM_MN) gemm_batch_offset(args);

  const int tiles_m = (args.M + BM - 1) / BM, tiles_n = (args.N + BN - 1) / BN;
  const int wg = xcd_remap(blockIdx.x, tiles_m * tiles_n);
  int tm, tn;
  tile_coords(wg, tiles_m, tiles_n, tm, tn);
  const int m0 = tm * BM, n0 = tn * BN;
  const int split = blockIdx.z;
  const int kbeg = split * args.k_per_split;
  const int kend = min(args.K, kbeg + args.k_per_split);

  float4v acc[MI][NJ];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = float4v{0.f, 0.f, 0.f, 0.f};
  g2_mainloop<AM, BMODE, BM, BN, NW, SEG2>(args, smem, m0, n0, kbeg, kend, a_bytes, b_bytes, a2_bytes, b2_bytes, acc);

  const bool use_slab = gridDim.z > 1;
  g2_store<AM, BMODE, BM, BN, NW, SEG2>(args, m0, n0, split, use_slab, acc);
  if (use_slab && args.tile_ctr) {
    // Split-K fix-up: the last workgroup of this output tile to arrive sums every split's slab
    // (index order, the reduce kernel's arithmetic) and writes C, so no reduce launch follows.
    // The partials went out as sc1 stores; s_waitcnt vmcnt(0) has them at the coherence point
    // before this workgroup's arrival is counted, and the last arriver reads them with sc1 loads.
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();   // every wave's partial stored; LDS no longer read by the main loop
    unsigned* flag = reinterpret_cast<unsigned*>(smem);
    if (threadIdx.x == 0) {
      unsigned* ctr = args.tile_ctr + blockIdx.x;
      const unsigned last = atomicAdd(ctr, 1u) == gridDim.z - 1;
      if (last) atomicExch(ctr, 0u);   // zero again for the stream's next split-K launch
      flag[0] = last;
    }
    __syncthreads();
    if (!flag[0]) return;
    const int rows = min(BM, args.M - m0), cols = min(BN, args.N - n0);
    const int splits = gridDim.z;
    if ((args.N % 8) == 0 && (args.ldc % 8) == 0 && ((uintptr_t)args.C & 15) == 0) {
      const int cu = cols / 8;
      for (int u = threadIdx.x; u < rows * cu; u += NW * 64) {
        const int r = u / cu;
        splitk_combine<8, true>(args, (unsigned)(m0 + r), (unsigned)(n0 + 8 * (u - r * cu)), splits);
      }
    } else {
      const int cu = cols / 4;
      for (int u = threadIdx.x; u < rows * cu; u += NW * 64) {
        const int r = u / cu;
        splitk_combine<4, true>(args, (unsigned)(m0 + r), (unsigned)(n0 + 4 * (u - r * cu)), splits);
      }
    }
  }
}

// ---------------------------------------------------------------------------------------------
// Cooperative split-K ("coop", plan tile 5) for GEMMs with fewer output tiles than CUs: P <= CUs
// workgroups, all resident at once (one per CU, 128 KB of LDS each), each computing ONE contiguous
// K-range of ONE 256x256 output tile.  A tile gets floor(P/T) or floor(P/T)+1 workgroups, so every
// CU has the same MFMA work to within one K-step: no wave quantisation, and no reduce launch.
// The workgroups of a tile then combine cooperatively instead of leaving it to one last arriver:
// each stores its fp32 partial to its slab (sc1 stores past the XCD-private L2, every wave drains),
// arrives at the tile's barrier and waits for its peers, then runs the split-K combine
// (splitk_combine, slabs summed in index order: the reduce kernel's bits for the same K-ranges)
// over 1/s of the tile's rows with sc1 loads.  The barrier is a sense-reversing one per tile slot
// (arrival count + generation word, relaxed agent-scope atomics issued by one lane; the waiters
// poll the generation with s_sleep and a bounded spin that reports instead of hanging): the last
// arriver re-zeroes the count before it bumps the generation, so the words need no per-launch value
// and a launch captured into a graph replays correctly.  Peers of a tile are consecutive ids (one
// XCD after xcd_remap) and all of a grid's workgroups fit on the chip at once, so a group waits at
// most for its own members to be dispatched.
struct SkArgs {
  unsigned* count;      // [1024] arrivals per tile slot (zero between launches)
  unsigned* gen;        // [1024] barrier generation per tile slot
  unsigned* err;        // set when a bounded spin gave up (never expected; checked by tests)
  int P, nkt, tiles_m, tiles_n;
};

typedef __attribute__((address_space(1))) unsigned gu32_t;

template <int AM, int BMODE, int BM, int BN, int NW, bool SEG2>
__global__ void __launch_bounds__(NW * 64, NW / 4) gemm2_sk_kernel(GemmArgs args, unsigned a_bytes, unsigned b_bytes,
                                                                   unsigned a2_bytes, unsigned b2_bytes, SkArgs sk) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  using T = G2<AM, BMODE, BM, BN, NW, SEG2>;
  constexpr int MI = T::MI, NJ = T::NJ;
  const int w = xcd_remap(blockIdx.x, sk.P);
  // w -> (tile, rank r of s): the first R tiles have s0 + 1 workgroups, the rest s0
  const int T_ = sk.tiles_m * sk.tiles_n;
  const int s0 = sk.P / T_, R = sk.P - s0 * T_;
  int tile, r, s;
  if (w < R * (s0 + 1)) { tile = w / (s0 + 1); r = w - tile * (s0 + 1); s = s0 + 1; }
  else { const int w2 = w - R * (s0 + 1); tile = R + w2 / s0; r = w2 - (tile - R) * s0; s = s0; }
  const int kt0 = sk.nkt * r / s, kt1 = sk.nkt * (r + 1) / s;
  int tm, tn;
  tile_coords(tile, sk.tiles_m, sk.tiles_n, tm, tn);
  const int m0 = tm * BM, n0 = tn * BN;

  float4v acc[MI][NJ];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = float4v{0.f, 0.f, 0.f, 0.f};
  g2_mainloop<AM, BMODE, BM, BN, NW, SEG2>(args, smem, m0, n0, kt0 * 64, min(args.K, kt1 * 64), a_bytes, b_bytes,
                                           a2_bytes, b2_bytes, acc);
  if (s == 1) {
    g2_store<AM, BMODE, BM, BN, NW, SEG2>(args, m0, n0, 0, false, acc);
    return;
  }
  g2_store<AM, BMODE, BM, BN, NW, SEG2>(args, m0, n0, r, true, acc);   // slab r (sc1: args.tile_ctr is set)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");                       // every storing wave drains
  __syncthreads();
  if (threadIdx.x == 0) {
    gu32_t* cnt = (gu32_t*)(sk.count + tile);
    gu32_t* gen = (gu32_t*)(sk.gen + tile);
    const unsigned g0 = __hip_atomic_load(gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // generation read before this arrival
    const unsigned old = __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (old == (unsigned)s - 1) {
      __hip_atomic_store(cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __hip_atomic_store(gen, g0 + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      unsigned spins = 0;
      while (__hip_atomic_load(gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == g0) {
        __builtin_amdgcn_s_sleep(2);
        if (++spins > (1u << 24)) {   // ~1 s: never expected; report instead of hanging the GPU
          __hip_atomic_store((gu32_t*)sk.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          break;
        }
      }
    }
  }
  __syncthreads();
  // rows [r*rows/s, (r+1)*rows/s) of the tile
  const int rows = min(BM, args.M - m0), cols = min(BN, args.N - n0);
  const int r0 = rows * r / s, r1 = rows * (r + 1) / s;
  if ((args.N % 8) == 0 && (args.ldc % 8) == 0 && ((uintptr_t)args.C & 15) == 0) {
    const int cu = cols / 8;
    for (int u = threadIdx.x; u < (r1 - r0) * cu; u += NW * 64) {
      const int rr = u / cu;
      splitk_combine<8, true>(args, (unsigned)(m0 + r0 + rr), (unsigned)(n0 + 8 * (u - rr * cu)), s);
    }
  } else {
    const int cu = cols / 4;
    for (int u = threadIdx.x; u < (r1 - r0) * cu; u += NW * 64) {
      const int rr = u / cu;
      splitk_combine<4, true>(args, (unsigned)(m0 + r0 + rr), (unsigned)(n0 + 4 * (u - rr * cu)), s);
    }
  }
}

typedef void (*gemm2_fn)(GemmArgs, unsigned, unsigned, unsigned, unsigned);

template <int BM, int BN, int NW>
static gemm2_fn pick2(int am, int bm, bool seg2) {
  if (seg2) {   // LoRA-fused forms: linear fwd, conv fwd, linear dgrad
    if (am == OPM_K && bm == OPM_K) return gemm2_kernel<OPM_K, OPM_K, BM, BN, NW, true>;
    if (am == OPM_CONV_FWD && bm == OPM_K) return gemm2_kernel<OPM_CONV_FWD, OPM_K, BM, BN, NW, true>;
    if (am == OPM_K && bm == OPM_MN) return gemm2_kernel<OPM_K, OPM_MN, BM, BN, NW, true>;
    return nullptr;
  }
#define CASE2(a, b) if (am == a && bm == b) return gemm2_kernel<a, b, BM, BN, NW, false>;
  CASE2(OPM_K, OPM_K)
  CASE2(OPM_K, OPM_MN)
  CASE2(OPM_MN, OPM_MN)
  CASE2(OPM_MN, OPM_K)
  CASE2(OPM_CONV_FWD, OPM_K)
  CASE2(OPM_CONV_DGRAD, OPM_K)
  CASE2(OPM_CONV_DGRAD, OPM_CONV_WT)
  CASE2(OPM_MN, OPM_CONV_WGRAD)
#undef CASE2
  return nullptr;
}

// byte extent an operand's gathers may touch (the DMA descriptor's range)
static long long operand_bytes(int mode, const bf16_t* p, long long ld, int MN, int K, const ConvGeom& g) {
  (void)p;
  if (mode == OPM_K) return ((long long)(MN - 1) * ld + K) * 2;
  if (mode == OPM_MN || mode == OPM_CONV_WT) return ((long long)(K - 1) * ld + MN) * 2;
  return ((long long)g.N * g.SH * g.SW - 1) * g.ld * 2 + (long long)g.SC * 2;
}

// launched by otamd_gemm (gemm.hip) when the v2 tile is selected; returns OTAMD_EUNSUPPORTED
// when the operand extents do not fit the 31-bit DMA offsets (caller falls back to v1)
int gemm2_launch(const GemmArgs& a, int tile, int splits, hipStream_t stream) {
  const long long ab = operand_bytes(a.amode, a.A, a.lda, a.M, a.K, a.ga);
  const long long bb = operand_bytes(a.bmode, a.B, a.ldb, a.N, a.K, a.gb);
  if (ab <= 0 || bb <= 0 || ab >= 0x7fff0000LL || bb >= 0x7fff0000LL) return OTAMD_EUNSUPPORTED;
  gemm2_fn fn = nullptr;
  int BMv = 256, BNv = 256, NWv = 8;
  const bool seg2 = a.A2 != nullptr;
  unsigned a2b = 0, b2b = 0;
  if (seg2) {
    const long long x = ((long long)(a.M - 1) * a.lda2 + a.K2) * 2;
    const long long y = a.bmode == OPM_K ? ((long long)(a.N - 1) * a.ldb2 + a.K2) * 2 : ((long long)(a.K2 - 1) * a.ldb2 + a.N) * 2;
    if (x <= 0 || y <= 0 || x >= 0x7fff0000LL || y >= 0x7fff0000LL) return OTAMD_EUNSUPPORTED;
    a2b = (unsigned)x;
    b2b = (unsigned)y;
  }
  if (tile == 0) fn = pick2<256, 256, 8>(a.amode, a.bmode, seg2);
  else if (tile == 1) { fn = pick2<256, 128, 8>(a.amode, a.bmode, seg2); BNv = 128; }
  else if (tile == 2) { fn = pick2<128, 256, 8>(a.amode, a.bmode, seg2); BMv = 128; }
  else if (tile == 4) { fn = pick2<128, 128, 8>(a.amode, a.bmode, seg2); BMv = 128; BNv = 128; }
  else if (!seg2) { fn = pick2<256, 256, 4>(a.amode, a.bmode, false); NWv = 4; }
  if (!fn) return OTAMD_EUNSUPPORTED;
  const int tiles = ((a.M + BMv - 1) / BMv) * ((a.N + BNv - 1) / BNv);
  const int lds = 2 * (BMv + BNv) * 128;
  {   // the LDS opt-in once per kernel instance (a per-launch driver call costs host time on every GEMM)
    static std::mutex mu;
    static std::unordered_set<const void*> done;
    std::lock_guard<std::mutex> lk(mu);
    if (done.insert((const void*)fn).second)
      hipFuncSetAttribute((const void*)fn, hipFuncAttributeMaxDynamicSharedMemorySize, 2 * (256 + 256) * 128);
  }
  hipLaunchKernelGGL(fn, dim3(tiles, a.batch > 1 ? a.batch : 1, splits), dim3(NWv * 64), lds, stream, a, (unsigned)ab,
                     (unsigned)bb, a2b, b2b);
  OTAMD_CHECK_LAUNCH();
  return OTAMD_OK;
}

// ---- stream-K launcher -------------------------------------------------------------------------
typedef void (*gemm2_sk_fn)(GemmArgs, unsigned, unsigned, unsigned, unsigned, SkArgs);

static gemm2_sk_fn pick_sk(int am, int bm, bool seg2) {
  if (seg2) {
    if (am == OPM_K && bm == OPM_K) return gemm2_sk_kernel<OPM_K, OPM_K, 256, 256, 8, true>;
    if (am == OPM_CONV_FWD && bm == OPM_K) return gemm2_sk_kernel<OPM_CONV_FWD, OPM_K, 256, 256, 8, true>;
    if (am == OPM_K && bm == OPM_MN) return gemm2_sk_kernel<OPM_K, OPM_MN, 256, 256, 8, true>;
    return nullptr;
  }
#define CASESK(a, b) if (am == a && bm == b) return gemm2_sk_kernel<a, b, 256, 256, 8, false>;
  CASESK(OPM_K, OPM_K)
  CASESK(OPM_K, OPM_MN)
  CASESK(OPM_MN, OPM_MN)
  CASESK(OPM_MN, OPM_K)
  CASESK(OPM_CONV_FWD, OPM_K)
  CASESK(OPM_CONV_DGRAD, OPM_K)
  CASESK(OPM_CONV_DGRAD, OPM_CONV_WT)
  CASESK(OPM_MN, OPM_CONV_WGRAD)
#undef CASESK
  return nullptr;
}

// Per (device, stream) coop state: the partial slabs and the tile barriers.  Launches of one stream
// run in order, so one state per stream is never shared by two grids in flight (a graph replays
// its kernels on the capture stream's state; replay it on that stream's order, as step_graph does).
struct SkState { float* slab = nullptr; long long slab_bytes = 0; unsigned* words = nullptr; };
#define SK_SLAB_MAX (1LL << 31)   // sc1 slab offsets are 31-bit
static std::mutex g_sk_mu;
static std::map<std::pair<int, hipStream_t>, SkState> g_sk;
static long long g_sk_slab_max = 256LL << 20;   // largest slab any stream needed so far

// allocate a stream's words and a slab of at least `bytes` (and of the largest slab any stream
// needed so far); the caller holds g_sk_mu and the stream is not capturing
static int sk_alloc(SkState& st, long long bytes, hipStream_t stream) {
  if (!st.words) {
    if (hipMalloc(&st.words, (2 * 1024 + 64) * 4) != hipSuccess) return OTAMD_EUNSUPPORTED;
    if (hipMemsetAsync(st.words, 0, (2 * 1024 + 64) * 4, stream) != hipSuccess) return OTAMD_EUNSUPPORTED;
  }
  g_sk_slab_max = std::max(g_sk_slab_max, bytes);
  if (st.slab_bytes < bytes || st.slab_bytes < g_sk_slab_max) {
    if (st.slab) { (void)hipStreamSynchronize(stream); (void)hipFree(st.slab); st.slab = nullptr; st.slab_bytes = 0; }
    const long long want = std::min<long long>((g_sk_slab_max + (64LL << 20) - 1) / (64LL << 20) * (64LL << 20), SK_SLAB_MAX);
    if (hipMalloc(&st.slab, (size_t)want) != hipSuccess) return OTAMD_EUNSUPPORTED;
    st.slab_bytes = want;
  }
  return OTAMD_OK;
}

int gemm2_cu_count() {
  static int cus[64] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 0;
  if (!cus[dev] && hipDeviceGetAttribute(&cus[dev], hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) cus[dev] = 0;
  return cus[dev];
}


// P = workgroups (0 = one per CU).  OTAMD_EUNSUPPORTED when the form / extents / stream do not
// allow it (or its state would have to be allocated inside a graph capture) -- the caller then takes
// its tile plan.
int gemm2_sk_launch(const GemmArgs& in, int P, hipStream_t stream) {
  GemmArgs a = in;
  if (a.batch > 1) return OTAMD_EUNSUPPORTED;
  const long long ab = operand_bytes(a.amode, a.A, a.lda, a.M, a.K, a.ga);
  const long long bb = operand_bytes(a.bmode, a.B, a.ldb, a.N, a.K, a.gb);
  if (ab <= 0 || bb <= 0 || ab >= 0x7fff0000LL || bb >= 0x7fff0000LL) return OTAMD_EUNSUPPORTED;
  const bool seg2 = a.A2 != nullptr;
  unsigned a2b = 0, b2b = 0;
  if (seg2) {
    const long long x = ((long long)(a.M - 1) * a.lda2 + a.K2) * 2;
    const long long y = a.bmode == OPM_K ? ((long long)(a.N - 1) * a.ldb2 + a.K2) * 2 : ((long long)(a.K2 - 1) * a.ldb2 + a.N) * 2;
    if (x <= 0 || y <= 0 || x >= 0x7fff0000LL || y >= 0x7fff0000LL) return OTAMD_EUNSUPPORTED;
    a2b = (unsigned)x;
    b2b = (unsigned)y;
  }
  gemm2_sk_fn fn = pick_sk(a.amode, a.bmode, seg2);
  if (!fn) return OTAMD_EUNSUPPORTED;
  const int cus = gemm2_cu_count();
  if (cus <= 0) return OTAMD_EUNSUPPORTED;
  const int tm = (a.M + 255) / 256, tn = (a.N + 255) / 256, T = tm * tn, nkt = (a.K + 63) / 64;
  if (T > cus || T > 1024) return OTAMD_EUNSUPPORTED;
  if (P <= 0) P = cus;
  P = std::min(P, std::min(cus, 1024));        // every workgroup resident at once (1 per CU); flag words
  P = std::min(P, T * nkt);                    // every K-range non-empty
  P = std::max(P, T);                          // >= 1 workgroup per tile
  const int smax = (P + T - 1) / T;
  const long long slab = smax > 1 ? (long long)smax * a.M * a.N * 4 : 0;
  if (slab >= SK_SLAB_MAX) return OTAMD_EUNSUPPORTED;
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(stream, &cs) != hipSuccess) return OTAMD_EUNSUPPORTED;
  const bool capturing = cs != hipStreamCaptureStatusNone;
  int dev = 0;
  (void)hipGetDevice(&dev);
  SkArgs sk{};
  {
    std::lock_guard<std::mutex> lk(g_sk_mu);
    SkState& st = g_sk[{dev, stream}];
    if (!st.words || st.slab_bytes < slab) {
      if (capturing) return OTAMD_EUNSUPPORTED;   // no allocation inside a capture: that launch takes the tile plan
      if (sk_alloc(st, slab, stream) != OTAMD_OK) return OTAMD_EUNSUPPORTED;
    }
    a.slab = st.slab;
    a.tile_ctr = st.words;             // non-null: slab stores / loads take the sc1 path
    sk.count = st.words;
    sk.gen = st.words + 1024;
    sk.err = st.words + 2048;
  }
  sk.P = P;
  sk.nkt = nkt;
  sk.tiles_m = tm;
  sk.tiles_n = tn;
  {
    static std::mutex mu;
    static std::unordered_set<const void*> done;
    std::lock_guard<std::mutex> lk(mu);
    if (done.insert((const void*)fn).second)
      hipFuncSetAttribute((const void*)fn, hipFuncAttributeMaxDynamicSharedMemorySize, 2 * (256 + 256) * 128);
  }
  hipLaunchKernelGGL(fn, dim3(P), dim3(512), 2 * (256 + 256) * 128, stream, a, (unsigned)ab, (unsigned)bb, a2b, b2b, sk);
  OTAMD_CHECK_LAUNCH();
  return OTAMD_OK;
}

// Number of stream-K launches whose owner gave up waiting for a partial (bounded spin) since the
// last call; synchronises the device.  Never expected to be non-zero: the tests assert it.
// Give `stream` its coop state now (before a graph capture on it: nothing is allocated inside a
// capture, where a coop GEMM would otherwise fall back to its tile plan and change the bits).
OTAMD_API int otamd_gemm_coop_reserve(hipStream_t stream) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return OTAMD_ELAUNCH;
  std::lock_guard<std::mutex> lk(g_sk_mu);
  return sk_alloc(g_sk[{dev, stream}], 0, stream);
}

OTAMD_API int otamd_gemm_sk_errors(void) {
  if (hipDeviceSynchronize() != hipSuccess) return -1;
  int dev = 0;
  (void)hipGetDevice(&dev);
  std::lock_guard<std::mutex> lk(g_sk_mu);
  int n = 0;
  for (auto& kv : g_sk) {
    if (!kv.second.words || kv.first.first != dev) continue;
    unsigned e = 0;
    if (hipMemcpy(&e, kv.second.words + 2048, 4, hipMemcpyDeviceToHost) != hipSuccess) return -1;
    if (e) {
      ++n;
      (void)hipMemset(kv.second.words + 2048, 0, 4);
    }
  }
  return n;
}
