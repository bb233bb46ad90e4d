// bf16 MFMA GEMM engine v2: 8 waves, 256-wide tiles, LDS-DMA staging (gfx950).
// The kernel template; gemm2_tiles_*.hip instantiate it per tile family (parallel compilation),
// gemm2.hip launches it.
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
#pragma once
#include "gemm.h"

// Timing ablations of the K loop (tools/gemm_ablate.sh builds them as separate libraries; results are garbage):
//   1 = no DMA after the prologue, 2 = no MFMA (fragments kept live), 3 = no fragment reads after the prologue,
//   4 = no barrier in the loop.  0 (default): the real kernel.
#ifndef OTAMD_GEMM_ABL
#define OTAMD_GEMM_ABL 0
#endif

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
  static_assert(N >= 0 && N < 64, "vmcnt range");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
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
  static constexpr int NP = BMN / 8;                  // 1 KiB pieces per stage image
  static constexpr int NI = (NP + NW - 1) / NW;       // pieces per wave (the last may be absent)
  static constexpr bool EVEN = NP % NW == 0;          // 160-wide images: 20 pieces over 8 waves
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
        const int lb = (pc >> 1) ^ mn_swz_rb<RB>(r);
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

  // source byte offset of this wave's piece i of the K tile at k0, any mode: offsets() for one piece; with i a compile-time index the other
  // pieces' arithmetic is dead and dropped
  __device__ __forceinline__ unsigned offset_g(const ConvGeom& g, long long ld, int k0, int Kend, int i) const {
    unsigned tmp[NI];
    offsets(g, ld, k0, Kend, tmp);
    return tmp[i];
  }
  // this wave's piece i of the image at img (piece j = wave + NW i); absent pieces of an uneven image are skipped
  __device__ __forceinline__ void put(__amdgpu_buffer_rsrc_t rs, char* img, int wave, int i, unsigned off) const {
    if (EVEN || wave + NW * i < NP) dma16(rs, img + (wave + NW * i) * 1024, off);
  }
  __device__ __forceinline__ void issue(__amdgpu_buffer_rsrc_t rs, char* img, const ConvGeom& g, long long ld, int k0,
                                        int Kend, int wave) {
    unsigned off[NI];
    offsets(g, ld, k0, Kend, off);
#pragma unroll
    for (int i = 0; i < NI; ++i) put(rs, img, wave, i, off[i]);
  }
  // source byte offsets of this wave's pieces of the K tile at k0 (OFF_INVALID: zero-fill)
  __device__ __forceinline__ void offsets(const ConvGeom& g, long long ld, int k0, int Kend, unsigned (&out)[NI]) const {
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
        out[i] = off;
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
        out[i] = off;
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
  return k * RB + ((((col >> 4)) ^ mn_swz_rb<RB>(k)) << 5) + ((col & 15) << 1);
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
// NS = LDS ring depth (every instance today: 2).  NS = 3 / 4 at one workgroup per CU (the ring filling up to
// 156 KiB, NS - 1 K-steps of DMA in flight) was built and measured in round 3 for the small-M SDXL shapes:
// no faster than two 2-stage workgroups per CU (4096x1280x1280: 23.3 vs 22.8 us for 128x160; 30.8 vs 24.0
// for 128x128), so those shapes are not latency-bound; the instances were dropped, the ring code kept.
// CS: also the column sums of the MN-mode A over this split's K range (GemmArgs.colsum: a weight
// gradient's bias gradient from the dY image already in LDS).  Workgroups of tile column 0 read each
// landed A image once more (16-byte chunks, one 64-row K-step) right after the barrier that publishes it;
// BM = 256 tiles keep the per-thread partials in an LDS region after the ring (their register file is
// full), smaller tiles in 8 VGPRs.  Folded in a fixed order at the end: deterministic.
template <int BM, int RB>
__device__ __forceinline__ int mn_chunk_off(int k, int c) {   // 16-byte chunk c (columns 8c..8c+7) of row k
  return k * RB + ((((c >> 1)) ^ mn_swz_rb<RB>(k)) << 5) + ((c & 1) << 4);
}

// LDR > 0: the LoRA down-projection of a frozen base GEMM computed inside its K loop (forward forms, B = K-mode
// weights).  The tile's output columns lie in one adapter part p = n0 / lora_pw; the part's LDR down rows D[p*LDR ..]
// ride in each stage as a third K-mode image, and every wave accumulates t = A D_p^T for all its rows and LDR / WN of
// the part's columns beside the base MFMAs.  After the loop t is rounded to bf16 (as the separate t = x A^T GEMM
// stores it), staged in LDS, written to T by the part's first tile column (for the adapter weight gradients), and
// multiplied by the up projection U = B2 [N][P*LDR] (alpha/rank folded in) into the same accumulators: the second K
// segment of the SEG2 form, without the t GEMM, its split-K reduce and their two launch boundaries.  The t sums run
// over K in the same 64-deep steps and 16x16x32 MFMAs as a one-split t GEMM, so t, and y, are bit-identical to that
// path.  LD tiles use 2 waves along N (wave tiles (BM / 4) x (BN / 2)), so each wave owns whole t column fragments.
// The same instance with B = MN-mode weights is the LoRA backward's input gradient (one adapter part spanning N,
// lora_pw = N): u = dY (sB) accumulated over the dgrad's K loop from D = (sB)^T [LDR][K], stored to T for the down
// projection's weight gradient, and dX = dY W + u A with B2 = A^T [N][LDR] -- the u GEMM, its split-K reduce and the
// second-segment DMA of the two-launch form (u GEMM + SEG2 dgrad) in one launch, bit-identical to it at one split.
// NPART > 1 (the dgrad form of a fused q|k|v site): the K range is NPART adapter parts of args.K1 rows each, u_p sums
// over part p's rows only (u = dY (sB) with sB block-diagonal); one accumulator set per part, rotated at each part
// boundary so the MFMAs always target set 0, and the second segment runs over all NPART * LDR columns of u.
template <int AM, int BMODE, int BM, int BN, int NW, bool SEG2, int NS = 2, bool CS = false, int LDR = 0, int NPART = 1>
__global__ void __launch_bounds__(NW * 64, (LDR == 0 && NS == 2 && BM == 128 && (BN == 128 || BN == 160)) ? 4 : NW / 4) gemm2_kernel(GemmArgs args, unsigned a_bytes, unsigned b_bytes,
                                                                 unsigned a2_bytes, unsigned b2_bytes) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr bool LD = LDR > 0;
  // BN = 160 (N = 320 / 640 / 1280 in 2 / 4 / 8 tiles, no padding): waves 4 x 2, wave tile (BM/4) x 80
  constexpr int WN = (NW == 4 || LD) ? 2 : ((BM == 256 && BN == 128) || BN == 160 ? 2 : 4);
  constexpr int WM = NW / WN;
  constexpr int TM = BM / WM, TN = BN / WN;
  constexpr int MI = TM / 16, NJ = TN / 16;
  constexpr int ABYTES = BM * 128, BBYTES = BN * 128;
  constexpr int RC = LDR / 16;               // t column fragments of the part
  constexpr int RCW = LD ? RC / WN : 0;      // ... owned by one wave
  constexpr int NBT = MI * RCW;              // 16 x 16 t blocks per wave
  constexpr int TBYTES = LD ? LDR * 128 : 0;
  static_assert(!LD || (!SEG2 && !CS && NS == 2 && NW == 8 && (BMODE == OPM_K || BMODE == OPM_MN) && RC % WN == 0 &&
                        RCW >= 1),
                "LoRA projection fusion: linear / conv forward or linear dgrad, 8 waves, whole t fragments per wave");
  constexpr int STAGE = ABYTES + BBYTES + TBYTES;
  constexpr int NIT = LD ? Stage<OPM_K, LD ? LDR : 8, NW>::NI : 0;
  constexpr int LOADS = Stage<AM, BM, NW>::NI + Stage<BMODE, BN, NW>::NI + NIT;
  // DMA pieces this wave issues per K-step (an image of NP pieces over NW waves: waves < NP % NW take one more)
  constexpr int NPA = Stage<AM, BM, NW>::NP, NPB = Stage<BMODE, BN, NW>::NP;
  static_assert(!SEG2 || NS == 2, "the LoRA second segment keeps the two-stage ring");
  constexpr bool AK = IsKMode<AM>::v, BKm = IsKMode<BMODE>::v;
  // per-wave DMA counts differ when an image does not split evenly: the prologue then drains fully
  constexpr bool EVEN_LOADS = Stage<AM, BM, NW>::EVEN && Stage<BMODE, BN, NW>::EVEN && (!SEG2 || (Stage<OPM_K, BM, NW>::EVEN && Stage<BKm ? OPM_K : OPM_MN, BN, NW>::EVEN)) &&
                              (!LD || Stage<OPM_K, LD ? LDR : 8, NW>::EVEN);
  if constexpr (!SEG2 && AM <= OPM_MN && BMODE <= OPM_MN) gemm_batch_offset(args);

  const int tiles_m = (args.M + BM - 1) / BM, tiles_n = (args.N + BN - 1) / BN;
  const int wg = xcd_remap(blockIdx.x, tiles_m * tiles_n);
  int tm, tn;
  tile_coords(wg, tiles_m, tiles_n, tm, tn);
  const int m0 = tm * BM, n0 = tn * BN;
  const int split = blockIdx.z;
  const int kbeg = split * args.k_per_split;
  const int kend = min(args.K, kbeg + args.k_per_split);
  const int nk = (kend - kbeg + 63) / 64;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;

  const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc((void*)args.A, (short)0, (int)a_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc((void*)args.B, (short)0, (int)b_bytes, 0x00020000);
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
    ra2 = __builtin_amdgcn_make_buffer_rsrc((void*)args.A2, (short)0, (int)a2_bytes, 0x00020000);
    rb2 = __builtin_amdgcn_make_buffer_rsrc((void*)args.B2, (short)0, (int)b2_bytes, 0x00020000);
    sa2.prepare(args.ga, args.lda2, m0, args.M, wave, lane);
    sb2.prepare(args.gb, args.ldb2, n0, args.N, wave, lane);
  }
  // down-projection fusion: the part's LDR rows of D (K-mode, the K layout of B) as a third image per stage
  const int lpart = LD ? n0 / args.lora_pw : 0;
  Stage<OPM_K, LD ? LDR : 8, NW> st;
  __amdgpu_buffer_rsrc_t rd = rb;
  if constexpr (LD) {
    const bf16_t* dp = args.D + (long long)lpart * LDR * args.ldd;
    rd = __builtin_amdgcn_make_buffer_rsrc((void*)dp, (short)0, (int)(((long long)(LDR - 1) * args.ldd + args.K) * 2),
                                           0x00020000);
    st.prepare(args.gb, args.ldd, 0, LDR, wave, lane);
  }
  // K tile at k0 (never straddles K1: K1 % 64 == 0) into the stage at img
  auto issue_tile = [&](char* img, int k0) {
    if (!SEG2 || k0 < args.K1) {
      sa.issue(ra, img, args.ga, args.lda, k0, SEG2 ? args.K1 : kend, wave);
      sb.issue(rb, img + ABYTES, args.gb, args.ldb, k0, SEG2 ? args.K1 : kend, wave);
      if constexpr (LD) st.issue(rd, img + ABYTES + BBYTES, args.gb, args.ldd, k0, kend, wave);
    } else {
      sa2.issue(ra2, img, args.ga, args.lda2, k0 - args.K1, args.K2, wave);
      sb2.issue(rb2, img + ABYTES, args.gb, args.ldb2, k0 - args.K1, args.K2, wave);
    }
  };

  const int wm = wave / WN, wn = wave % WN;
  float4v acc[MI][NJ];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = float4v{0.f, 0.f, 0.f, 0.f};

  // fragment loaders (h selects the 32-wide half of the 64-deep K tile)
  auto load_a = [&](bf16x8 (&f)[MI], const char* ia, int h) {
#pragma unroll
    for (int i = 0; i < MI; ++i) f[i] = AK ? frag_k2(ia, wm * TM + i * 16, 32 * h) : frag_mn2<BM * 2>(ia, wm * TM + i * 16, 32 * h);
  };
  auto load_b = [&](bf16x8 (&f)[NJ], const char* ib, int h) {
#pragma unroll
    for (int j = 0; j < NJ; ++j) f[j] = BKm ? frag_k2(ib, wn * TN + j * 16, 32 * h) : frag_mn2<BN * 2>(ib, wn * TN + j * 16, 32 * h);
  };
  // down-projection fusion: this wave's t blocks (rows i of its row range, its RCW column fragments of the part)
  constexpr int NBT1 = NBT > 0 ? NBT : 1, RCW1 = RCW > 0 ? RCW : 1;
  static_assert(NPART == 1 || (LD && BMODE == OPM_MN), "multi-part u: the fused dgrad form only");
  float4v acc_t[NPART][NBT1];   // [0]: the part of the current K step (earlier parts rotate towards NPART - 1)
#pragma unroll
  for (int q = 0; q < NPART; ++q)
#pragma unroll
    for (int b = 0; b < NBT1; ++b) acc_t[q][b] = float4v{0.f, 0.f, 0.f, 0.f};
  bf16x8 ft0[RCW1], ft1[RCW1];
  auto load_t = [&](bf16x8 (&f)[RCW1], const char* it, int h) {
    if constexpr (LD) {
#pragma unroll
      for (int c = 0; c < RCW; ++c) f[c] = frag_k2(it, (wn * RCW + c) * 16, 32 * h);
    }
  };
  auto mfma_block = [&](const bf16x8 (&fa)[MI], const bf16x8 (&fb)[NJ], const bf16x8 (&ft)[RCW1]) {
    if constexpr (OTAMD_GEMM_ABL == 2) {
#pragma unroll
      for (int i = 0; i < MI; ++i) asm volatile("" ::"v"(fa[i]));
#pragma unroll
      for (int j = 0; j < NJ; ++j) asm volatile("" ::"v"(fb[j]));
      return;
    }
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[j], fa[i], acc[i][j], 0, 0, 0);
    if constexpr (LD) {
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int c = 0; c < RCW; ++c)
          acc_t[0][i * RCW + c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ft[c], fa[i], acc_t[0][i * RCW + c], 0, 0, 0);
    }
  };
  // the next half's fragment reads (h = 0, load_b then load_a order) with this wave's refill DMA pieces of the slot
  // at dst placed one after each read: the inline-asm DMA keeps its place among the DS reads (both touch memory)
  // while interleave()'s groups put the MFMAs between the reads
  constexpr int NIA = Stage<AM, BM, NW>::NI, NIB = Stage<BMODE, BN, NW>::NI;
  // plain K / MN operands only: with a conv gather the per-piece offset arithmetic (integer divisions) inside phase B
  // cost more than the burst (conv fwd / dgrad 10-15 % slower, profiles/r4_gemm_spread_conv_*), and the 128-row
  // colsum tiles (at their 128-VGPR cap) spilled 15 registers
  // The LoRA second segment (SEG2) spreads the refills of its first segment too; the few refills that land in the
  // second segment (K2 <= 64 rows: one K-step) go out as a burst through issue_tile.  Not the 128x160 dgrad form with
  // a second segment: at its 128-VGPR cap the spread pushed it to 20 bytes of scratch per lane.
  constexpr bool SPREAD = NW == 8 && !(CS && BM == 128) && !(SEG2 && BM == 128 && BN == 160 && BMODE == OPM_MN) &&
                          (AM == OPM_K || AM == OPM_MN) &&
                          (BMODE == OPM_K || BMODE == OPM_MN);
  auto load_ab_refill = [&](bf16x8 (&fa)[MI], bf16x8 (&fb)[NJ], bf16x8 (&ft)[RCW1], const char* ia, const char* ib,
                            char* dst, int k0) {
    if constexpr (SPREAD) {
      auto piece = [&](int t) {   // offsets computed at the piece (no per-step offset arrays: the 256-wide tiles sit
                                  // at the 256-VGPR cap)
        const int k1end = SEG2 ? args.K1 : kend;
        if (t < NIA) sa.put(ra, dst, wave, t, sa.offset_g(args.ga, args.lda, k0, k1end, t));
        else if (t < NIA + NIB) sb.put(rb, dst + ABYTES, wave, t - NIA, sb.offset_g(args.gb, args.ldb, k0, k1end, t - NIA));
        else if constexpr (LD) {
          if (t < NIA + NIB + NIT)
            st.put(rd, dst + ABYTES + BBYTES, wave, t - NIA - NIB, st.offset_g(args.gb, args.ldd, k0, kend, t - NIA - NIB));
        }
      };
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        fb[j] = BKm ? frag_k2(ib, wn * TN + j * 16, 0) : frag_mn2<BN * 2>(ib, wn * TN + j * 16, 0);
        piece(j);
      }
#pragma unroll
      for (int i = 0; i < MI; ++i) {
        fa[i] = AK ? frag_k2(ia, wm * TM + i * 16, 0) : frag_mn2<BM * 2>(ia, wm * TM + i * 16, 0);
        piece(NJ + i);
      }
      if constexpr (LD) {
#pragma unroll
        for (int c = 0; c < RCW; ++c) {
          ft[c] = frag_k2(ib + BBYTES, (wn * RCW + c) * 16, 0);
          piece(NJ + MI + c);
        }
      }
#pragma unroll
      for (int t = MI + NJ + RCW; t < NIA + NIB + NIT; ++t) piece(t);
    }
  };
  // interleave the next fragment reads into the current MFMA block: {2 MFMA, reads of 1 fragment} x (MI+NJ)
  // (128x128: 8 MFMAs per half for 6 fragment reads -> {1 MFMA, reads} x 6, then the rest)
  constexpr int NR = MI + NJ + RCW;
  constexpr int NMF = MI * NJ + NBT;
  constexpr int PER = NMF / NR >= 2 ? 2 : 1;
  constexpr int REST = NMF - PER * NR;
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
  // this wave's DMA count per K-step (a wave-uniform value)
  const int my_loads = (NPA / NW + (wave < NPA % NW ? 1 : 0)) + (NPB / NW + (wave < NPB % NW ? 1 : 0));
  // wait until at most `tiles` younger K-steps' DMA of this wave are in flight (tiles <= NS - 1)
  auto wait_tiles = [&](int tiles) {
    if constexpr (NS == 2) {
      (void)tiles;
      wait_vmcnt<0>();
    } else if constexpr (EVEN_LOADS && NPA % NW == 0 && NPB % NW == 0) {
      if (tiles >= 3) wait_vmcnt<3 * LOADS>();
      else if (tiles == 2) wait_vmcnt<2 * LOADS>();
      else if (tiles == 1) wait_vmcnt<LOADS>();
      else wait_vmcnt<0>();
    } else {   // uneven images: this wave's count is LOADS or LOADS - 1 (or less); wait per class
      constexpr int LO = NPA / NW + NPB / NW;
      const int extra = my_loads - LO;   // 0, 1 or 2
      if (tiles <= 0) wait_vmcnt<0>();
      else if (tiles == 1) { if (extra == 0) wait_vmcnt<LO>(); else if (extra == 1) wait_vmcnt<LO + 1>(); else wait_vmcnt<LO + 2>(); }
      else if (tiles == 2) { if (extra == 0) wait_vmcnt<2 * LO>(); else if (extra == 1) wait_vmcnt<2 * LO + 2>(); else wait_vmcnt<2 * LO + 4>(); }
      else { if (extra == 0) wait_vmcnt<3 * LO>(); else if (extra == 1) wait_vmcnt<3 * LO + 3>(); else wait_vmcnt<3 * LO + 6>(); }
    }
  };
  if (nk > 0) {
    if constexpr (NS == 2) {
      issue_tile(smem, kbeg);
      if (nk > 1) {
        issue_tile(smem + STAGE, kbeg + 64);
        if constexpr (EVEN_LOADS) wait_vmcnt<LOADS>();
        else wait_vmcnt<0>();
      } else {
        wait_vmcnt<0>();
      }
    } else {
#pragma unroll
      for (int st = 0; st < NS; ++st)
        if (st < nk) issue_tile(smem + st * STAGE, kbeg + st * 64);
      wait_tiles(min(NS, nk) - 1);   // tile 0 has landed
    }
    BARRIER();
    load_b(fb0, smem + ABYTES, 0);
    load_a(fa0, smem, 0);
    load_t(ft0, smem + ABYTES + BBYTES, 0);
    if constexpr (OTAMD_GEMM_ABL == 3) {
#pragma unroll
      for (int i = 0; i < MI; ++i) fa1[i] = fa0[i];
#pragma unroll
      for (int j = 0; j < NJ; ++j) fb1[j] = fb0[j];
    }
  }
  // ---- column sums of A (CS) ----
  static_assert(!CS || (AM == OPM_MN && !SEG2), "column sums of an MN-mode A, single segment");
  constexpr int CPR = BM / 8;                       // 16-byte chunks per A-image row
  constexpr int RG = NW * 64 / CPR;                 // row groups (threads per chunk column)
  constexpr int NCH = 64 / RG;                      // rows of one K-step per thread
  constexpr bool CS_LDS = BM == 256;
  static_assert(!CS || (RG * CPR == NW * 64 && NCH * RG == 64), "colsum thread map");
  const bool cs_on = CS && tn == 0;                 // workgroup-uniform
  const int cs_c = threadIdx.x % CPR, cs_rg = threadIdx.x / CPR;
  float cs[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) cs[j] = 0.f;
  float* cs_lds = reinterpret_cast<float*>(smem + NS * STAGE) + (cs_rg * BM + cs_c * 8);
  auto colsum_tile = [&](const char* ia) {
    float t[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) t[j] = 0.f;
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
      const bf8 v = *reinterpret_cast<const bf8*>(ia + mn_chunk_off<BM, BM * 2>(cs_rg + RG * i, cs_c));
      float f[8];
      unpack8(v, f);
#pragma unroll
      for (int j = 0; j < 8; ++j) t[j] += f[j];
    }
    if constexpr (CS_LDS) {
      float4* q = reinterpret_cast<float4*>(cs_lds);
      float4 a0 = q[0], a1 = q[1];
      a0.x += t[0]; a0.y += t[1]; a0.z += t[2]; a0.w += t[3];
      a1.x += t[4]; a1.y += t[5]; a1.z += t[6]; a1.w += t[7];
      q[0] = a0;
      q[1] = a1;
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) cs[j] += t[j];
    }
  };
  if constexpr (CS) {
    if (cs_on && nk > 0) {
      if constexpr (CS_LDS) {
        float4* q = reinterpret_cast<float4*>(cs_lds);
        q[0] = make_float4(0.f, 0.f, 0.f, 0.f);
        q[1] = make_float4(0.f, 0.f, 0.f, 0.f);
      }
      colsum_tile(smem);   // tile 0 (published by the prologue barrier)
    }
  }

  int stg = 0;   // ring slot of tile kt (kt % NS)
  // One K-step.  REFILL: tile kt + NS exists and goes into tile kt's slot.  The plain single-segment K / MN-mode
  // kernels (SPREAD) place that refill's DMA pieces one after each of phase B's fragment reads: issued as one burst
  // after the barrier they held the issuing wave for the whole burst (~60-185 cycles per 1-KiB piece,
  // MI355X_MICROARCH.md) with its MFMAs waiting behind it.  The K steps without a refill (the last NS) run a copy
  // of the body with no DMA at all, so no branch splits phase B's scheduling region.
  // refill_tag: 0 = no refill, 1 = refill (spread through phase B where SPREAD, else a burst), 2 = refill as a burst
  auto kstep = [&](int kt, auto refill_tag) {
    constexpr int RM = decltype(refill_tag)::value;
    constexpr bool REFILL = RM != 0 && OTAMD_GEMM_ABL != 1;
    constexpr bool BURST = REFILL && (RM == 2 || !SPREAD);
    constexpr bool SPREAD_NOW = REFILL && RM == 1 && SPREAD;
    const char* ia = smem + stg * STAGE;
    const char* ib = ia + ABYTES;
    const int nstg = stg + 1 == NS ? 0 : stg + 1;
    if constexpr (NPART > 1) {   // tile kt opens a new adapter part (K1 = part rows, a multiple of 64)
      if (kt > 0 && (kbeg + kt * 64) % args.K1 == 0) {
#pragma unroll
        for (int q = NPART - 1; q > 0; --q)
#pragma unroll
          for (int b = 0; b < NBT1; ++b) acc_t[q][b] = acc_t[q - 1][b];
#pragma unroll
        for (int b = 0; b < NBT1; ++b) acc_t[0][b] = float4v{0.f, 0.f, 0.f, 0.f};
      }
    }
    // phase A
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (OTAMD_GEMM_ABL != 3) {
      load_b(fb1, ib, 1);
      load_a(fa1, ia, 1);
      load_t(ft1, ib + BBYTES, 1);
    }
    mfma_block(fa0, fb0, ft0);
    if constexpr (OTAMD_GEMM_ABL != 3) interleave();
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    // tile kt+1 has landed: the tiles after it that may still be in flight are kt+2 .. min(kt+NS-1, nk-1)
    wait_tiles(min(NS - 2, nk - kt - 2));
    if constexpr (OTAMD_GEMM_ABL != 4) BARRIER();
    if constexpr (BURST) {   // refill tile kt's slot
      if (kt + NS < nk) issue_tile(smem + stg * STAGE, kbeg + (kt + NS) * 64);
    }
    if constexpr (CS) {   // tile kt+1: published by this barrier, refilled only after the next one
      __builtin_amdgcn_sched_barrier(0);
      if (cs_on && kt + 1 < nk) colsum_tile(smem + nstg * STAGE);
    }
    // phase B
    __builtin_amdgcn_sched_barrier(0);
    {   // on the last step this reads a stale stage; harmless and keeps the loop branch-free
      const char* na = smem + nstg * STAGE;
      if constexpr (OTAMD_GEMM_ABL != 3) {
        if constexpr (SPREAD_NOW) load_ab_refill(fa0, fb0, ft0, na, na + ABYTES, smem + stg * STAGE, kbeg + (kt + NS) * 64);
        else {
          load_b(fb0, na + ABYTES, 0);
          load_a(fa0, na, 0);
          load_t(ft0, na + ABYTES + BBYTES, 0);
        }
      }
      mfma_block(fa1, fb1, ft1);
      if constexpr (OTAMD_GEMM_ABL != 3) interleave();
    }
    __builtin_amdgcn_sched_barrier(0);
    stg = nstg;
  };
  if constexpr (SPREAD) {
    int kt = 0;
    // SEG2: refills whose K-step lies in the second segment (k0 >= K1; K1 and kbeg are multiples of 64) burst
    const int n_spread = SEG2 ? max(0, min(nk - NS, (args.K1 - kbeg) / 64 - NS)) : nk - NS;
    for (; kt < n_spread; ++kt) kstep(kt, std::integral_constant<int, 1>{});
    if constexpr (SEG2)
      for (; kt < nk - NS; ++kt) kstep(kt, std::integral_constant<int, 2>{});
    for (; kt < nk; ++kt) kstep(kt, std::integral_constant<int, 0>{});
  } else {   // conv gathers / the LoRA second segment: one body, the refill as a burst behind a uniform branch (a
             // peeled copy measured 4-8 % slower on the conv tiles)
    for (int kt = 0; kt < nk; ++kt) kstep(kt, std::integral_constant<int, 1>{});
  }

  if constexpr (LD) {   // the second K segment from the t accumulated above (no split-K: the launcher checks)
    constexpr int LU = NPART * LDR;     // columns of t / u (all parts)
    constexpr int KS2 = (LU + 31) / 32;
    const int g = lane >> 4;
    // up-projection fragments of this wave's output columns (K-mode rows of U, 16 bytes per lane), loaded before the t
    // hand-off so their latency hides behind it
    bf16x8 fu[KS2][NJ];
#pragma unroll
    for (int s2 = 0; s2 < KS2; ++s2)
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const int n = n0 + wn * TN + j * 16 + (lane & 15);
        const int kk = 32 * s2 + 8 * g;
        fu[s2][j] = bf16x8{};
        if (n < args.N && kk < LU)
          fu[s2][j] = *reinterpret_cast<const bf16x8*>(args.B2 + (long long)n * args.ldb2 + lpart * LDR + kk);
      }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    BARRIER();   // every wave is past its last stage read: stage 0 becomes the t image (BM rows x 64 k)
    // t / u image: columns [64 i, 64 i + 64) in stage i's A region (K-mode layout, as a DMA'd A tile)
    static_assert((LU + 63) / 64 <= NS, "t / u columns must fit the ring's A regions");
    const bool t_out = (n0 % args.lora_pw) == 0;   // the part's first tile column stores t for the backward
#pragma unroll
    for (int q = 0; q < NPART; ++q)
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int c = 0; c < RCW; ++c) {
          const float4v v = acc_t[NPART - 1 - q][i * RCW + c];   // part q (the last part is in set 0)
          const int row = wm * TM + i * 16 + (lane & 15);
          const int col = q * LDR + (wn * RCW + c) * 16 + 4 * g;
          uint2 o;
          o.x = (uint32_t)f2bf(v[0]) | ((uint32_t)f2bf(v[1]) << 16);
          o.y = (uint32_t)f2bf(v[2]) | ((uint32_t)f2bf(v[3]) << 16);
          char* timg = smem + (col >> 6) * STAGE;
          *reinterpret_cast<uint2*>(timg + kimg_off(row, (col & 63) >> 3) + (col & 7) * 2) = o;
          const int m = m0 + row;
          if (t_out && m < args.M) *reinterpret_cast<uint2*>(args.T + (long long)m * args.ldt + lpart * LDR + col) = o;
        }
    if constexpr (LU % 32) {   // k in [LU, 32 KS2): zeros (the up fragments there are zero; stale LDS bytes may be NaN)
      constexpr int ZC = (32 - LU % 32) / 8;   // 16-byte chunks per row
      for (int e = threadIdx.x; e < BM * ZC; e += NW * 64) {
        const int row = e / ZC, ch = (LU % 64) / 8 + e % ZC;
        *reinterpret_cast<uint4*>(smem + (LU / 64) * STAGE + kimg_off(row, ch)) = make_uint4(0u, 0u, 0u, 0u);
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    BARRIER();
#pragma unroll
    for (int s2 = 0; s2 < KS2; ++s2) {
      bf16x8 fa2[MI];
#pragma unroll
      for (int i = 0; i < MI; ++i) fa2[i] = frag_k2(smem + (s2 >> 1) * STAGE, wm * TM + i * 16, 32 * (s2 & 1));
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fu[s2][j], fa2[i], acc[i][j], 0, 0, 0);
    }
  }

  const bool use_slab = gridDim.z > 1;
  if constexpr (CS) {
    if (cs_on) {   // fold the row groups in a fixed order; tile column 0 only (workgroup-uniform branch)
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      BARRIER();   // every wave past its last ring read (and, for CS_LDS, its last partial update)
      float* red = reinterpret_cast<float*>(smem + (CS_LDS ? NS * STAGE : 0));
      if constexpr (!CS_LDS) {
        float4* q = reinterpret_cast<float4*>(red + cs_rg * BM + cs_c * 8);
        q[0] = make_float4(cs[0], cs[1], cs[2], cs[3]);
        q[1] = make_float4(cs[4], cs[5], cs[6], cs[7]);
        // the row-group partials are read by other waves: their ds_writes must retire before the barrier (gfx950's
        // back-off barrier does not wait for LDS stores, and the compiler adds no waitcnt in front of a raw s_barrier)
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        BARRIER();
      }
      for (int c = threadIdx.x; c < BM; c += NW * 64) {
        float tot = 0.f;
        for (int r = 0; r < RG; ++r) tot += red[r * BM + c];
        const int m = m0 + c;
        if (m < args.M) {
          if (use_slab) args.colsum_slab[(long long)split * args.M + m] = tot;
          else if (args.colsum_f32) {
            float* d = reinterpret_cast<float*>(args.colsum) + m;
            *d = args.colsum_acc ? *d + tot : tot;
          } else {
            bf16_t* d = reinterpret_cast<bf16_t*>(args.colsum) + m;
            *d = f2bf(args.colsum_acc ? bf2f(*d) + tot : tot);
          }
        }
      }
    }
  }
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
      if (n >= args.N) continue;
      float v[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
      gemm_store4(args, m, n, v, split, use_slab);
    }
  }
}

typedef void (*gemm2_fn)(GemmArgs, unsigned, unsigned, unsigned, unsigned);

template <int BM, int BN, int NW, int NS = 2>
static gemm2_fn pick2(int am, int bm, bool seg2, bool cs = false) {
  if (cs) {   // weight gradients with the bias gradient fused: MN-mode A (dY), linear or conv B
    if constexpr (NW == 8) {
      if (seg2) return nullptr;
      if (am == OPM_MN && bm == OPM_MN) return gemm2_kernel<OPM_MN, OPM_MN, BM, BN, NW, false, NS, true>;
      if (am == OPM_MN && bm == OPM_CONV_WGRAD) return gemm2_kernel<OPM_MN, OPM_CONV_WGRAD, BM, BN, NW, false, NS, true>;
    }
    return nullptr;
  }
  if (seg2) {   // LoRA-fused forms: linear fwd, conv fwd, linear dgrad
    if constexpr (NS != 2) return nullptr;
    if (am == OPM_K && bm == OPM_K) return gemm2_kernel<OPM_K, OPM_K, BM, BN, NW, true>;
    if (am == OPM_CONV_FWD && bm == OPM_K) return gemm2_kernel<OPM_CONV_FWD, OPM_K, BM, BN, NW, true>;
    if (am == OPM_K && bm == OPM_MN) return gemm2_kernel<OPM_K, OPM_MN, BM, BN, NW, true>;
    return nullptr;
  }
#define CASE2(a, b) if (am == a && bm == b) return gemm2_kernel<a, b, BM, BN, NW, false, NS>;
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

