// bf16 MFMA GEMM engine v2, half-K DMA units (gfx950): the same tiles, operand modes and epilogue as
// gemm2_kernel.h, with the operand staging cut into half K-tiles so the DMA stays in flight across barriers.
//
// gemm2_kernel stages whole 64-deep K-tiles in a two-slot ring: the DMA of tile k+2 (issued during tile k's second
// half) must land by the end of tile k+1's first half, so every K-step ends in s_waitcnt vmcnt(0) and the loop's
// memory side (DMA issue and landing, LDS reads, the barrier) is its critical path (profiles/r4_gemm_kloop_ablations:
// the loop without a single MFMA took 64 % of the real loop's time at 4096^3).  Here the unit of staging is a half
// K-tile (k 0..31 or 32..63 of A and B): unit u = 2 k + h sits in LDS slot u % 4, and per K-step
//   phase A(k): MFMA on half 0 of tile k | ds_read half 1 of tile k (unit 2k+1) | DMA unit 2k+4 -> slot of unit 2k
//               wait: unit 2k+2 landed (units 2k+3, 2k+4 stay in flight: vmcnt(2 P)), barrier 1
//   phase B(k): MFMA on half 1 of tile k | ds_read half 0 of tile k+1 (unit 2k+2) | DMA unit 2k+5 -> slot of 2k+1
//               wait: unit 2k+3 landed (units 2k+4, 2k+5 stay in flight: vmcnt(2 P)), barrier 2
// (P = this wave's DMA pieces per unit).  Two units are in flight across every barrier and the wait never drains
// the queue inside the loop (cdna_hip_programming.md §5 "Pipelining across barriers", T3+T4): a unit's DMA has
// 1.5 K-steps to land instead of one.  WAR: a slot is refilled one phase after the barrier that follows its last
// read (every read retired by the lgkmcnt(0) in front of that barrier).  RAW: a unit is read only after its
// issuers' counted wait and the barrier behind it.
//
// LDS: the same bytes per stage as gemm2_kernel.  K-mode operands are stored as two half images [rows][64 B]
// (16-byte chunk c of row r at c ^ (((r >> 3) & 1) << 1): ds_read_b128 fragment reads are bank-conflict free for
// gfx950's four 16-lane groups), MN-mode images keep their [64 k][row bytes] layout, whose halves are the k rows
// 0..31 and 32..63.
#pragma once
#include "gemm2_kernel.h"

template <int BMN> __device__ __forceinline__ int khalf_off(int row, int chunk /* 0..3 within the half */) {
  return row * 64 + ((chunk ^ (((row >> 3) & 1) << 1)) << 4);
}

// Per-lane DMA state of one operand's half image (BMN rows/cols x 32 k): BMN/16 pieces of 1 KiB.
template <int MODE, int BMN, int NW>
struct StageH {
  static constexpr bool KM = IsKMode<MODE>::v;
  static constexpr int NP = BMN / 16;
  static constexpr int NI = (NP + NW - 1) / NW;
  static constexpr bool EVEN = NP % NW == 0;
  static constexpr int RB = BMN * 2;      // MN-mode row bytes
  static constexpr int HALF = BMN * 64;   // bytes of one half image
  int a[NI], b[NI], c[NI];
  int t0;
  bool ok[NI];

  __device__ __forceinline__ void prepare(const ConvGeom& g, long long ld, int mn0, int MNsz, int wave, int lane) {
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int j = wave + NW * i;
      if constexpr (KM) {   // piece j: rows 16 j .. 16 j + 15, lane -> (row lane / 4, chunk slot lane % 4)
        const int r = 16 * j + (lane >> 2);
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
      } else {              // piece j: bytes j KiB .. of the [32 k][RB] half image
        const int byte = j * 1024 + lane * 16;
        const int r = byte / RB;
        const int pc = (byte % RB) >> 4;
        const int lb = (pc >> 1) ^ mn_swz_rb<RB>(r);   // k and k + 32 share the swizzle (bits 0, 1, 3)
        const int col = mn0 + (lb * 2 + (pc & 1)) * 8;
        a[i] = r;
        ok[i] = col < MNsz;
        if constexpr (MODE == OPM_MN || MODE == OPM_CONV_WT) {
          b[i] = col;
        } else {
          const int cc = ok[i] ? col : 0;
          const int tap = cc / g.SC;
          c[i] = cc - tap * g.SC;
          b[i] = tap;
        }
      }
    }
    // the source chunk of this lane's 16 bytes: row bit 3 is lane bit 5 for every piece (rows 16 j + lane / 4)
    if constexpr (KM) t0 = (lane & 3) ^ (((lane >> 5) & 1) << 1);
  }

  // source byte offsets of this wave's pieces of the half tile starting at k0h (OFF_INVALID: zero-fill)
  __device__ __forceinline__ void offsets(const ConvGeom& g, long long ld, int k0h, int Kend, unsigned (&out)[NI]) const {
    if constexpr (KM) {
      const int k = k0h + 8 * t0;
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
        const int k = k0h + a[i];
        unsigned off = OFF_INVALID;
        if constexpr (MODE == OPM_MN) {
          if (ok[i] && k < Kend) off = (unsigned)(k * (int)ld + b[i]) * 2u;
        } else if constexpr (MODE == OPM_CONV_WT) {
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
  __device__ __forceinline__ unsigned offset_g(const ConvGeom& g, long long ld, int k0h, int Kend, int i) const {
    unsigned tmp[NI];
    offsets(g, ld, k0h, Kend, tmp);
    return tmp[i];
  }
  __device__ __forceinline__ void put(__amdgpu_buffer_rsrc_t rs, char* half_img, int wave, int i, unsigned off) const {
    if (EVEN || wave + NW * i < NP) dma16(rs, half_img + (wave + NW * i) * 1024, off);
  }
  __device__ __forceinline__ void issue(__amdgpu_buffer_rsrc_t rs, char* half_img, const ConvGeom& g, long long ld,
                                        int k0h, int Kend, int wave) const {
    unsigned off[NI];
    offsets(g, ld, k0h, Kend, off);
#pragma unroll
    for (int i = 0; i < NI; ++i) put(rs, half_img, wave, i, off[i]);
  }
};

// 16x16x32 fragment of a K-mode half image: lane holds X[mnb + (lane & 15)][8 (lane >> 4) + j] of the half
__device__ __forceinline__ bf16x8 frag_kh(const char* half_img, int mnb) {
  const int lane = threadIdx.x & 63;
  const int row = mnb + (lane & 15);
  return *reinterpret_cast<const bf16x8*>(half_img + khalf_off<0>(row, lane >> 4));
}

// CS: also the column sums of the MN-mode A over this split's K range (GemmArgs.colsum, a weight gradient's bias
// gradient), as gemm2_kernel does them: workgroups of tile column 0 read each half image of A once more in the
// phase that reads its fragments (after the barrier that publishes it, before the phase that refills its slot).
template <int AM, int BMODE, int BM, int BN, bool CS = false>
__global__ void __launch_bounds__(512, (BM == 128 && (BN == 128 || BN == 160)) ? 4 : 2)
gemm2h_kernel(GemmArgs args, unsigned a_bytes, unsigned b_bytes, unsigned, unsigned) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int NW = 8;
  constexpr int WN = ((BM == 256 && BN == 128) || BN == 160) ? 2 : 4;
  constexpr int WM = NW / WN;
  constexpr int TM = BM / WM, TN = BN / WN;
  constexpr int MI = TM / 16, NJ = TN / 16;
  constexpr int AH = BM * 64, BH = BN * 64;           // half-image bytes
  constexpr int STAGE = 2 * (AH + BH);                // one K-tile: A h0 | A h1 | B h0 | B h1
  constexpr bool AK = IsKMode<AM>::v, BKm = IsKMode<BMODE>::v;
  using SA = StageH<AM, BM, NW>;
  using SB = StageH<BMODE, BN, NW>;
  constexpr int NPA = SA::NP, NPB = SB::NP;
  if constexpr (AM <= OPM_MN && BMODE <= OPM_MN) gemm_batch_offset(args);

  const int tiles_m = (args.M + BM - 1) / BM, tiles_n = (args.N + BN - 1) / BN;
  const int wg = xcd_remap(blockIdx.x, tiles_m * tiles_n);
  int tm, tn;
  tile_coords(wg, tiles_m, tiles_n, tm, tn);
  const int m0 = tm * BM, n0 = tn * BN;
  const int split = blockIdx.z;
  const int kbeg = split * args.k_per_split;
  const int kend = min(args.K, kbeg + args.k_per_split);
  const int nk = (kend - kbeg + 63) / 64;
  const int U = 2 * nk;   // half-tile units
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;

  const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc((void*)args.A, (short)0, (int)a_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc((void*)args.B, (short)0, (int)b_bytes, 0x00020000);
  SA sa;
  SB sb;
  sa.prepare(args.ga, args.lda, m0, args.M, wave, lane);
  sb.prepare(args.gb, args.ldb, n0, args.N, wave, lane);
  auto a_img = [&](int u) { return smem + ((u >> 1) & 1) * STAGE + (u & 1) * AH; };
  auto b_img = [&](int u) { return smem + ((u >> 1) & 1) * STAGE + 2 * AH + (u & 1) * BH; };
  auto k0_of = [&](int u) { return kbeg + (u >> 1) * 64 + (u & 1) * 32; };
  auto issue_unit = [&](int u) {
    sa.issue(ra, a_img(u), args.ga, args.lda, k0_of(u), kend, wave);
    sb.issue(rb, b_img(u), args.gb, args.ldb, k0_of(u), kend, wave);
  };

  const int wm = wave / WN, wn = wave % WN;
  float4v acc[MI][NJ];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = float4v{0.f, 0.f, 0.f, 0.f};

  auto frag_a = [&](int u, int i) {
    return AK ? frag_kh(a_img(u), wm * TM + i * 16) : frag_mn2<BM * 2>(a_img(u & ~1), wm * TM + i * 16, 32 * (u & 1));
  };
  auto frag_b = [&](int u, int j) {
    return BKm ? frag_kh(b_img(u), wn * TN + j * 16) : frag_mn2<BN * 2>(b_img(u & ~1), wn * TN + j * 16, 32 * (u & 1));
  };
  auto mfma_block = [&](const bf16x8 (&fa)[MI], const bf16x8 (&fb)[NJ]) {
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[j], fa[i], acc[i][j], 0, 0, 0);
  };
  // plain K / MN operands: the unit's DMA pieces are placed one after each fragment read (the inline-asm DMA keeps
  // its place among the DS reads); conv gathers issue theirs as one burst (per-piece offset math is costly there)
  constexpr bool SPREAD = (AM == OPM_K || AM == OPM_MN) && (BMODE == OPM_K || BMODE == OPM_MN);
  constexpr int NIA = SA::NI, NIB = SB::NI;
  auto read_frags = [&](bf16x8 (&fa)[MI], bf16x8 (&fb)[NJ], int u, int du, auto refill) {
    constexpr bool RF = decltype(refill)::value;
    auto piece = [&](int t) {
      if (t < NIA) sa.put(ra, a_img(du), wave, t, sa.offset_g(args.ga, args.lda, k0_of(du), kend, t));
      else if (t < NIA + NIB) sb.put(rb, b_img(du), wave, t - NIA, sb.offset_g(args.gb, args.ldb, k0_of(du), kend, t - NIA));
    };
    if constexpr (RF && !SPREAD) issue_unit(du);
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      fb[j] = frag_b(u, j);
      if constexpr (RF && SPREAD) piece(j);
    }
#pragma unroll
    for (int i = 0; i < MI; ++i) {
      fa[i] = frag_a(u, i);
      if constexpr (RF && SPREAD) piece(NJ + i);
    }
    if constexpr (RF && SPREAD) {
#pragma unroll
      for (int t = MI + NJ; t < NIA + NIB; ++t) piece(t);
    }
  };
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
  // this wave's DMA pieces per unit: P = PLO + extra (extra 0..2 when an image does not split evenly over the waves)
  constexpr int PLO = NPA / NW + NPB / NW;
  const int extra = (wave < NPA % NW ? 1 : 0) + (wave < NPB % NW ? 1 : 0);
  auto wait_units = [&](int n) {   // at most n units of this wave's DMA still in flight
    if (n <= 0) { wait_vmcnt<0>(); return; }
    if (n == 1) {
      if (extra == 0) wait_vmcnt<PLO>(); else if (extra == 1) wait_vmcnt<PLO + 1>(); else wait_vmcnt<PLO + 2>();
    } else {
      if (extra == 0) wait_vmcnt<2 * PLO>(); else if (extra == 1) wait_vmcnt<2 * PLO + 2>(); else wait_vmcnt<2 * PLO + 4>();
    }
  };

  // ---- column sums of A (CS) over half images: 32 k rows of BM columns ----
  static_assert(!CS || AM == OPM_MN, "column sums of an MN-mode A");
  constexpr int CPR = BM / 8;                       // 16-byte chunks per A-image row
  constexpr int RG = NW * 64 / CPR;                 // row groups (threads per chunk column)
  constexpr int NCH = 32 / RG;                      // rows of one half image per thread
  constexpr bool CS_LDS = BM == 256;
  static_assert(!CS || (RG * CPR == NW * 64 && NCH * RG == 32), "colsum thread map");
  const bool cs_on = CS && tn == 0;                 // workgroup-uniform
  const int cs_c = threadIdx.x % CPR, cs_rg = threadIdx.x / CPR;
  float cs[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) cs[j] = 0.f;
  float* cs_lds = reinterpret_cast<float*>(smem + 2 * STAGE) + (cs_rg * BM + cs_c * 8);
  auto colsum_unit = [&](int u) {
    if constexpr (CS) {
      if (!cs_on) return;
      const char* img = a_img(u & ~1);
      float t[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) t[j] = 0.f;
#pragma unroll
      for (int i = 0; i < NCH; ++i) {
        const bf8 v = *reinterpret_cast<const bf8*>(img + mn_chunk_off<BM, BM * 2>(32 * (u & 1) + cs_rg + RG * i, cs_c));
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
    }
  };

  bf16x8 fa0[MI], fb0[NJ], fa1[MI], fb1[NJ];
  if (nk > 0) {
    for (int u = 0; u < min(4, U); ++u) issue_unit(u);
    wait_units((2 < U) + (3 < U));   // tile 0 (units 0, 1) landed
    BARRIER();
    read_frags(fa0, fb0, 0, 0, std::false_type{});
    if constexpr (CS) {
      if (cs_on && CS_LDS) {
        float4* q = reinterpret_cast<float4*>(cs_lds);
        q[0] = make_float4(0.f, 0.f, 0.f, 0.f);
        q[1] = make_float4(0.f, 0.f, 0.f, 0.f);
      }
      __builtin_amdgcn_sched_barrier(0);
      colsum_unit(0);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    BARRIER();   // every wave's reads of unit 0 retired before unit 4 refills its slot
  }
  auto kstep = [&](int kt, auto refill) {
    // phase A: MFMA half 0 of tile kt | reads of half 1 (unit 2kt+1) | DMA of unit 2kt+4
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (CS) {   // first in the phase: its LDS reads overlap the MFMAs below
      colsum_unit(2 * kt + 1);
      __builtin_amdgcn_sched_barrier(0);
    }
    read_frags(fa1, fb1, 2 * kt + 1, 2 * kt + 4, refill);
    mfma_block(fa0, fb0);
    interleave();
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    wait_units(kt + 1 < nk ? (2 * kt + 3 < U) + (2 * kt + 4 < U) : 0);   // unit 2kt+2 landed
    BARRIER();
    // phase B: MFMA half 1 of tile kt | reads of half 0 of tile kt+1 (unit 2kt+2) | DMA of unit 2kt+5
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (CS) {
      if (kt + 1 < nk) colsum_unit(2 * kt + 2);
      __builtin_amdgcn_sched_barrier(0);
    }
    read_frags(fa0, fb0, 2 * kt + 2, 2 * kt + 5, refill);   // the last step reads a stale slot: harmless
    mfma_block(fa1, fb1);
    interleave();
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    wait_units(kt + 1 < nk ? (2 * kt + 4 < U) + (2 * kt + 5 < U) : 0);   // unit 2kt+3 landed
    BARRIER();
  };
  {
    int kt = 0;
    for (; kt < nk - 2; ++kt) kstep(kt, std::true_type{});
    for (; kt < nk; ++kt) kstep(kt, std::false_type{});
  }

  const bool use_slab = gridDim.z > 1;
  if constexpr (CS) {
    if (cs_on) {   // fold the row groups in a fixed order; tile column 0 only (workgroup-uniform branch)
      float* red = reinterpret_cast<float*>(smem + (CS_LDS ? 2 * STAGE : 0));
      if constexpr (!CS_LDS) {   // the ring is free: every wave is past its last read (the loop's last barrier)
        float4* q = reinterpret_cast<float4*>(red + cs_rg * BM + cs_c * 8);
        q[0] = make_float4(cs[0], cs[1], cs[2], cs[3]);
        q[1] = make_float4(cs[4], cs[5], cs[6], cs[7]);
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      BARRIER();
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
    if (use_slab && args.tile_sem) splitk_fixup<BM, BN>(args, m0, n0, reinterpret_cast<int*>(smem));
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

template <int BM, int BN>
static gemm2_fn pick2h(int am, int bm, bool cs = false) {
  if (cs) {   // weight gradients with the bias gradient fused: MN-mode A (dY), linear or conv B
    if (am == OPM_MN && bm == OPM_MN) return gemm2h_kernel<OPM_MN, OPM_MN, BM, BN, true>;
    if (am == OPM_MN && bm == OPM_CONV_WGRAD) return gemm2h_kernel<OPM_MN, OPM_CONV_WGRAD, BM, BN, true>;
    return nullptr;
  }
#define CASE2H(a, b) if (am == a && bm == b) return gemm2h_kernel<a, b, BM, BN>;
  CASE2H(OPM_K, OPM_K)
  CASE2H(OPM_K, OPM_MN)
  CASE2H(OPM_MN, OPM_MN)
  CASE2H(OPM_MN, OPM_K)
  CASE2H(OPM_CONV_FWD, OPM_K)
  CASE2H(OPM_CONV_DGRAD, OPM_K)
  CASE2H(OPM_CONV_DGRAD, OPM_CONV_WT)
  CASE2H(OPM_MN, OPM_CONV_WGRAD)
#undef CASE2H
  return nullptr;
}
