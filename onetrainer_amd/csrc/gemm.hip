// bf16 MFMA GEMM engine for gfx950 (v_mfma_f32_16x16x32_bf16, fp32 accumulate).
//
// One kernel template covers every GEMM-shaped op of the UNet hot path
// (SURVEY.md §2.3 rows conv3x3 / Linear GEMM; reference call sites
// modules/modelSetup/BaseStableDiffusionXLSetup.py:268-273 -> diffusers UNet):
//   Linear fwd   Y = X W^T          A: OPM_K (X [M,K])     B: OPM_K  (W [N,K])
//   Linear dgrad dX = dY W          A: OPM_K (dY [M,N])    B: OPM_MN (W [N,K] read as [K'=N][N'=K])
//   Linear wgrad dW = dY^T X        A: OPM_MN (dY)         B: OPM_MN (X)         (split-K slabs)
//   conv fwd     implicit GEMM      A: OPM_CONV_FWD gather B: OPM_K (W [Cout][kh][kw][Cin])
//   conv dgrad   transposed gather  A: OPM_CONV_DGRAD      B: OPM_CONV_WT (W read in place, v2 tiles)
//                                                          or OPM_K (W^T [Cin][kh][kw][Cout], any tile)
//   conv wgrad   dW = dY^T im2col   A: OPM_MN (dY)         B: OPM_CONV_WGRAD gather
// Activations are NHWC bf16, so a conv's rows are pixels and a Linear over tokens
// reads the same tensor with no permute.
//
// Operand tiles are staged global -> registers -> LDS "as they lie" (16-byte chunks
// along the contiguous dimension).  K-contiguous tiles are read with ds_read_b128,
// MN-contiguous tiles with ds_read_b64_tr_b16 (hardware transpose), both XOR-swizzled
// to be bank-conflict free.  The MFMA is issued with swapped operands (B-fragment as
// the MFMA A operand) so each lane ends with 4 consecutive output columns.
#include "gemm.h"

#include <stdlib.h>

#include <atomic>
#include <mutex>
#include <unordered_map>
#include <string.h>

#define BM 128
#define BN 128
#define BK 64
#define NTHREADS 256

// --- LDS images ------------------------------------------------------------------------
// (K-mode image and the MN-mode swizzle are in gemm.h; v1 MN images have 256-byte rows)
__device__ __forceinline__ int mnimg_off(int k, int col) {  // col: element index, multiple of 4
  const int blk = col >> 4, within = (col & 15) << 1;
  return k * 256 + ((blk ^ mn_swz(k)) << 5) + within;
}

// --- global gathers ----------------------------------------------------------------------
__device__ __forceinline__ bf8 zero8() { bf8 z; z.w[0] = z.w[1] = z.w[2] = z.w[3] = 0; return z; }
__device__ __forceinline__ bf8 ld8(const bf16_t* p) { return *reinterpret_cast<const bf8*>(p); }

// per-thread cached row decode for K-mode gathers (4 rows per thread)
struct RowCtx { int n[4], y0[4], x0[4]; bool ok[4]; };

template <int MODE>
__device__ __forceinline__ void kmode_prepare(const ConvGeom& g, int mn0, int MNsz, RowCtx& rc) {
  const int tid = threadIdx.x;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int row = mn0 + (tid >> 3) + 32 * i;
    rc.ok[i] = row < MNsz;
    if (MODE == OPM_CONV_FWD || MODE == OPM_CONV_DGRAD) {
      const int rr = rc.ok[i] ? row : 0;
      const int hw = g.RH * g.RW;
      const int n = rr / hw, rem = rr - n * hw;
      const int y = rem / g.RW, x = rem - y * g.RW;
      rc.n[i] = n;
      if (MODE == OPM_CONV_FWD) { rc.y0[i] = y * g.stride - g.pad; rc.x0[i] = x * g.stride - g.pad; }
      else { rc.y0[i] = y + g.pad; rc.x0[i] = x + g.pad; }
    }
  }
}

// load this thread's 4 chunks of a K-mode tile (rows mn0.., k chunk k0 + 8*(tid&7))
template <int MODE>
__device__ __forceinline__ void kmode_load(const bf16_t* __restrict__ X, long long ld, const ConvGeom& g, int mn0,
                                           int k0, int K, const RowCtx& rc, bf8 (&st)[4]) {
  const int tid = threadIdx.x;
  const int k = k0 + 8 * (tid & 7);
  const bool kok = k < K;
  if (MODE == OPM_K) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = mn0 + (tid >> 3) + 32 * i;
      st[i] = (kok && rc.ok[i]) ? ld8(X + (long long)row * ld + k) : zero8();
    }
  } else {
    const int tap = kok ? k / g.SC : 0;
    const int ch = k - tap * g.SC;
    const int r = tap / g.KW, s = tap - r * g.KW;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      bool ok = kok && rc.ok[i];
      int sy, sx;
      if (MODE == OPM_CONV_FWD) {
        const int y = rc.y0[i] + r, x = rc.x0[i] + s;
        if (g.upsample) {
          ok = ok && y >= 0 && y < 2 * g.SH && x >= 0 && x < 2 * g.SW;
          sy = y >> 1; sx = x >> 1;
        } else {
          ok = ok && y >= 0 && y < g.SH && x >= 0 && x < g.SW;
          sy = y; sx = x;
        }
      } else {  // dgrad: source pixel ((h+pad-r)/st, (w+pad-s)/st) when divisible
        const int ty = rc.y0[i] - r, tx = rc.x0[i] - s;
        if (g.stride == 1) { sy = ty; sx = tx; }
        else {
          ok = ok && ty >= 0 && tx >= 0 && (ty % g.stride) == 0 && (tx % g.stride) == 0;
          sy = ty / g.stride; sx = tx / g.stride;
        }
        ok = ok && sy >= 0 && sy < g.SH && sx >= 0 && sx < g.SW;
      }
      st[i] = ok ? ld8(X + ((long long)(rc.n[i] * g.SH + sy) * g.SW + sx) * g.ld + ch) : zero8();
    }
  }
}

__device__ __forceinline__ void kmode_store(char* img, const bf8 (&st)[4]) {
  const int tid = threadIdx.x;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int row = (tid >> 3) + 32 * i;
    *reinterpret_cast<bf8*>(img + kimg_off(row, tid & 7)) = st[i];
  }
}

// MN-mode: this thread's 4 chunks are (k rows tid/16 + 16 i, mn chunk 8*(tid&15))
struct ColCtx { int r, s, ch; bool ok; };

template <int MODE>
__device__ __forceinline__ void mnmode_prepare(const ConvGeom& g, int mn0, int MNsz, ColCtx& cc) {
  const int col = mn0 + 8 * (threadIdx.x & 15);
  cc.ok = col < MNsz;
  if (MODE == OPM_CONV_WGRAD) {
    const int c = cc.ok ? col : 0;
    const int tap = c / g.SC;
    cc.ch = c - tap * g.SC;
    cc.r = tap / g.KW;
    cc.s = tap - cc.r * g.KW;
  }
}

template <int MODE>
__device__ __forceinline__ void mnmode_load(const bf16_t* __restrict__ X, long long ld, const ConvGeom& g, int mn0,
                                            int k0, int K, const ColCtx& cc, bf8 (&st)[4]) {
  const int tid = threadIdx.x;
  const int col = mn0 + 8 * (tid & 15);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int k = k0 + (tid >> 4) + 16 * i;
    bool ok = cc.ok && k < K;
    if (MODE == OPM_MN) {
      st[i] = ok ? ld8(X + (long long)k * ld + col) : zero8();
    } else {  // OPM_CONV_WGRAD: k = output pixel, col = (r, s, ch)
      const int kk = ok ? k : 0;
      const int hw = g.RH * g.RW;
      const int n = kk / hw, rem = kk - n * hw;
      const int p = rem / g.RW, q = rem - p * g.RW;
      const int y = p * g.stride - g.pad + cc.r, x = q * g.stride - g.pad + cc.s;
      int sy, sx;
      if (g.upsample) { ok = ok && y >= 0 && y < 2 * g.SH && x >= 0 && x < 2 * g.SW; sy = y >> 1; sx = x >> 1; }
      else { ok = ok && y >= 0 && y < g.SH && x >= 0 && x < g.SW; sy = y; sx = x; }
      st[i] = ok ? ld8(X + ((long long)(n * g.SH + sy) * g.SW + sx) * g.ld + cc.ch) : zero8();
    }
  }
}

__device__ __forceinline__ void mnmode_store(char* img, const bf8 (&st)[4]) {
  const int tid = threadIdx.x;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int k = (tid >> 4) + 16 * i;
    const int col = 8 * (tid & 15);
    *reinterpret_cast<bf8*>(img + mnimg_off(k, col)) = st[i];   // 16 B stay inside one 32-B block
  }
}

// --- fragment reads --------------------------------------------------------------------------
typedef __attribute__((address_space(3))) short4v lds_short4;

__device__ __forceinline__ bf16x8 frag_k(const char* img, int mnb, int kb) {
  const int lane = threadIdx.x & 63;
  const int row = mnb + (lane & 15);
  const int chunk = (kb >> 3) + (lane >> 4);
  return *reinterpret_cast<const bf16x8*>(img + kimg_off(row, chunk));
}
__device__ __forceinline__ bf16x8 frag_mn(const char* img, int mnb, int kb) {
  const int lane = threadIdx.x & 63;
  const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
  const int k0 = kb + 8 * g + q;
  const int col = mnb + 4 * p;
  const short4v lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_short4*)(img + mnimg_off(k0, col)));
  const short4v hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_short4*)(img + mnimg_off(k0 + 4, col)));
  short8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8, v);
}

template <int MODE> struct IsK { static constexpr bool v = (MODE == OPM_K || MODE == OPM_CONV_FWD || MODE == OPM_CONV_DGRAD); };


template <int AM, int BMODE>
__global__ void __launch_bounds__(NTHREADS, 2) gemm_kernel(GemmArgs args) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  if constexpr (AM <= OPM_MN && BMODE <= OPM_MN) gemm_batch_offset(args);
  const int tiles_m = (args.M + BM - 1) / BM, tiles_n = (args.N + BN - 1) / BN;
  const int nwg = tiles_m * tiles_n;
  const int wg = xcd_remap(blockIdx.x, nwg);
  int tm, tn;
  tile_coords(wg, tiles_m, tiles_n, tm, tn);
  const int m0 = tm * BM, n0 = tn * BN;
  const int split = blockIdx.z;
  const int kbeg = split * args.k_per_split;
  const int kend = min(args.K, kbeg + args.k_per_split);
  const int nk = (kend - kbeg + BK - 1) / BK;


  RowCtx rcA, rcB;
  ColCtx ccA, ccB;
  constexpr bool AK = IsK<AM>::v, BKm = IsK<BMODE>::v;
  if (AK) kmode_prepare<AM>(args.ga, m0, args.M, rcA); else mnmode_prepare<AM>(args.ga, m0, args.M, ccA);
  if (BKm) kmode_prepare<BMODE>(args.gb, n0, args.N, rcB); else mnmode_prepare<BMODE>(args.gb, n0, args.N, ccB);

  bf8 sa[4], sb[4];
  auto load_tiles = [&](int k0) {
    if (AK) kmode_load<AM>(args.A, args.lda, args.ga, m0, k0, kend, rcA, sa);
    else mnmode_load<AM>(args.A, args.lda, args.ga, m0, k0, kend, ccA, sa);
    if (BKm) kmode_load<BMODE>(args.B, args.ldb, args.gb, n0, k0, kend, rcB, sb);
    else mnmode_load<BMODE>(args.B, args.ldb, args.gb, n0, k0, kend, ccB, sb);
  };
  auto store_tiles = [&](int buf) {
    char* imA = smem + buf * 16384;
    char* imB = smem + 32768 + buf * 16384;
    if (AK) kmode_store(imA, sa); else mnmode_store(imA, sa);
    if (BKm) kmode_store(imB, sb); else mnmode_store(imB, sb);
  };

  const int wave = threadIdx.x >> 6;
  const int wm = wave >> 1, wn = wave & 1;   // 2 x 2 waves, 64 x 64 each
  float4v acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = float4v{0.f, 0.f, 0.f, 0.f};

  if (nk > 0) {
    load_tiles(kbeg);
    store_tiles(0);
    __syncthreads();
  }
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) load_tiles(kbeg + (kt + 1) * BK);
    const char* ia = smem + cur * 16384;
    const char* ib = smem + 32768 + cur * 16384;
#pragma unroll
    for (int kk = 0; kk < BK; kk += 32) {
      bf16x8 af[4], bfr[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) af[i] = AK ? frag_k(ia, wm * 64 + i * 16, kk) : frag_mn(ia, wm * 64 + i * 16, kk);
#pragma unroll
      for (int j = 0; j < 4; ++j) bfr[j] = BKm ? frag_k(ib, wn * 64 + j * 16, kk) : frag_mn(ib, wn * 64 + j * 16, kk);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[j], af[i], acc[i][j], 0, 0, 0);
    }
    if (kt + 1 < nk) store_tiles(cur ^ 1);
    __syncthreads();
  }

  // epilogue: lane holds C[m][n..n+3], m = ... + (lane&15), n = ... + 4*(lane>>4)
  const int lane = threadIdx.x & 63;
  const bool use_slab = gridDim.z > 1;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int m = m0 + wm * 64 + i * 16 + (lane & 15);
    if (m >= args.M) continue;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int n = n0 + wn * 64 + j * 16 + 4 * (lane >> 4);
      if (n >= args.N) continue;   // N % 4 == 0 is a launcher precondition
      float v[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
      gemm_store4(args, m, n, v, split, use_slab);
    }
  }
}

// split-K reduction + the same epilogue: C = alpha * sum_s slab[s] (+bias, +rowvec, +residual) (+C if accumulate)
// Sum the split-K fp32 slabs and apply the epilogue.  V consecutive columns per thread (8 when
// N % 8 == 0: one 16-byte bf16 store), every split's loads issued before the adds (the slabs were
// just written and mostly sit in the MALL: latency, not bandwidth, bounds a dependent chain).
template <int V>
__global__ void __launch_bounds__(256) splitk_reduce_kernel(GemmArgs args, int splits) {
  const unsigned NV = (unsigned)args.N / V;
  const unsigned total = (unsigned)args.M * NV;
  for (unsigned i = blockIdx.x * 256u + threadIdx.x; i < total; i += gridDim.x * 256u) {
    const unsigned m = i / NV, n = (i - m * NV) * V;
    splitk_combine<V>(args, m, n, splits);
  }
  if (args.colsum) {   // the fused column sums' per-split partials, summed in split order
    for (unsigned m = blockIdx.x * 256u + threadIdx.x; m < (unsigned)args.M; m += gridDim.x * 256u) {
      float t = args.colsum_slab[m];
      for (int z = 1; z < splits; ++z) t += args.colsum_slab[(long long)z * args.M + m];
      if (args.colsum_f32) {
        float* d = reinterpret_cast<float*>(args.colsum) + m;
        *d = args.colsum_acc ? *d + t : t;
      } else {
        bf16_t* d = reinterpret_cast<bf16_t*>(args.colsum) + m;
        *d = f2bf(args.colsum_acc ? bf2f(*d) + t : t);
      }
    }
  }
}

OTAMD_API long long otamd_gemm_ws_bytes(const GemmArgs* in, int splits);

// ---- deferred split-K reduces (otamd_gemm_defer_*) -------------------------------------------------------------------
// A stream in defer mode puts the fp32 split-K slabs of its eligible GEMMs (no bias / row vector / residual operand,
// not batched) into a caller-owned arena instead of the workspace and records their reduces; one grouped launch
// (splitk_reduce_grouped_kernel) later sums up to kMaxDefer of them, each in split order as splitk_reduce_kernel
// does, so the outputs are bit-identical.  For the weight-gradient stream, where the LoRA adapter gradients (rank
// 16-32 wide, K = tokens: split-K is inherent) issued ~2,300 reduce launches per SDXL LoRA step.
struct SplitkDesc {
  float* slab; void* C; long long ldc;
  int M, N, splits, flags;   // flags: 1 C fp32, 2 accumulate into C, 4 colsum fp32, 8 accumulate into colsum
  float alpha; unsigned block0;
  void* colsum; float* colsum_slab;
};
constexpr int kMaxDefer = 40;
struct SplitkBatch { int n; unsigned blocks; SplitkDesc d[kMaxDefer]; };

__global__ void __launch_bounds__(256) splitk_reduce_grouped_kernel(SplitkBatch bt) {
  int i = 0;
  while (i + 1 < bt.n && blockIdx.x >= bt.d[i + 1].block0) ++i;
  const SplitkDesc& d = bt.d[i];
  const unsigned nb = (i + 1 < bt.n ? bt.d[i + 1].block0 : bt.blocks) - d.block0;
  const unsigned lb = blockIdx.x - d.block0;
  GemmArgs a = {};
  a.slab = d.slab; a.C = d.C; a.ldc = d.ldc; a.M = d.M; a.N = d.N; a.alpha = d.alpha;
  a.c_f32 = d.flags & 1; a.accumulate = (d.flags >> 1) & 1;
  const unsigned NV = (unsigned)d.N / 4;
  const unsigned total = (unsigned)d.M * NV;
  for (unsigned e = lb * 256u + threadIdx.x; e < total; e += nb * 256u) {
    const unsigned m = e / NV, n = (e - m * NV) * 4;
    splitk_combine<4>(a, m, n, d.splits);
  }
  if (d.colsum) {
    for (unsigned m = lb * 256u + threadIdx.x; m < (unsigned)d.M; m += nb * 256u) {
      float t = d.colsum_slab[m];
      for (int z = 1; z < d.splits; ++z) t += d.colsum_slab[(long long)z * d.M + m];
      if (d.flags & 4) {
        float* p = reinterpret_cast<float*>(d.colsum) + m;
        *p = (d.flags & 8) ? *p + t : t;
      } else {
        bf16_t* p = reinterpret_cast<bf16_t*>(d.colsum) + m;
        *p = f2bf((d.flags & 8) ? bf2f(*p) + t : t);
      }
    }
  }
}

struct DeferState {
  char* arena = nullptr;
  long long bytes = 0, used = 0;
  uintptr_t out_lo = 0, out_hi = 0;   // only outputs inside this range are deferred
  SplitkBatch batch{};
  uintptr_t lo[kMaxDefer], hi[kMaxDefer];   // byte ranges each pending reduce writes (C, and the colsum)
  uintptr_t clo[kMaxDefer], chi[kMaxDefer];
};
static std::mutex g_defer_mu;
static std::unordered_map<hipStream_t, DeferState> g_defer;
static long long g_defer_gemms = 0, g_defer_launches = 0;   // otamd_gemm_defer_stats

static int defer_flush_locked(DeferState& st, hipStream_t stream) {
  if (st.batch.n > 0) {
    splitk_reduce_grouped_kernel<<<st.batch.blocks, 256, 0, stream>>>(st.batch);
    g_defer_gemms += st.batch.n;
    ++g_defer_launches;
    st.batch.n = 0;
    st.batch.blocks = 0;
    OTAMD_CHECK_LAUNCH();
  }
  st.used = 0;
  return OTAMD_OK;
}

static void c_range(const GemmArgs& a, uintptr_t& lo, uintptr_t& hi) {
  const int es = a.c_f32 ? 4 : 2;
  lo = (uintptr_t)a.C;
  hi = lo + ((long long)(a.M - 1) * a.ldc + a.N) * es;
}

// a GEMM on a deferring stream: a pending reduce whose output this GEMM reads or writes is flushed first
static int defer_guard(const GemmArgs& a, hipStream_t stream) {
  std::lock_guard<std::mutex> lk(g_defer_mu);
  auto it = g_defer.find(stream);
  if (it == g_defer.end() || it->second.batch.n == 0) return OTAMD_OK;
  DeferState& st = it->second;
  uintptr_t lo, hi;
  c_range(a, lo, hi);
  const uintptr_t cl = (uintptr_t)a.colsum, ch = cl + (a.colsum ? (uintptr_t)a.M * (a.colsum_f32 ? 4 : 2) : 0);
  const uintptr_t in[3][2] = {{(uintptr_t)a.A, (uintptr_t)a.A + 1}, {(uintptr_t)a.B, (uintptr_t)a.B + 1}, {lo, hi}};
  for (int i = 0; i < st.batch.n; ++i) {
    bool hit = (lo < st.hi[i] && st.lo[i] < hi) || (a.colsum && cl < st.chi[i] && st.clo[i] < ch) ||
               (a.colsum && cl < st.hi[i] && st.lo[i] < ch);
    for (int j = 0; j < 2 && !hit; ++j)   // an operand that starts inside a pending output
      hit = (in[j][0] < st.hi[i] && st.lo[i] < in[j][1]) || (in[j][0] < st.chi[i] && st.clo[i] < in[j][1]);
    if (hit) return defer_flush_locked(st, stream);
  }
  return OTAMD_OK;
}

// slab memory for a deferrable split-K GEMM on a deferring stream (nullptr: not deferring / not eligible)
static float* defer_slab(const GemmArgs& a, int splits, hipStream_t stream) {
  if (a.bias || a.rowvec || a.residual || a.batch > 1) return nullptr;
  std::lock_guard<std::mutex> lk(g_defer_mu);
  auto it = g_defer.find(stream);
  if (it == g_defer.end()) return nullptr;
  DeferState& st = it->second;
  uintptr_t lo, hi;
  c_range(a, lo, hi);
  if (lo < st.out_lo || hi > st.out_hi) return nullptr;
  if (a.colsum) {
    const uintptr_t cl = (uintptr_t)a.colsum, ch = cl + (uintptr_t)a.M * (a.colsum_f32 ? 4 : 2);
    if (cl < st.out_lo || ch > st.out_hi) return nullptr;
  }
  const long long need = (otamd_gemm_ws_bytes(&a, splits) + 255) / 256 * 256;
  if (need > st.bytes) return nullptr;
  if (st.batch.n == kMaxDefer || st.used + need > st.bytes) defer_flush_locked(st, stream);
  float* p = reinterpret_cast<float*>(st.arena + st.used);
  st.used += need;
  return p;
}

static void defer_record(const GemmArgs& a, int splits, hipStream_t stream) {
  std::lock_guard<std::mutex> lk(g_defer_mu);
  DeferState& st = g_defer[stream];
  SplitkDesc& d = st.batch.d[st.batch.n];
  d.slab = a.slab; d.C = a.C; d.ldc = a.ldc; d.M = a.M; d.N = a.N; d.splits = splits; d.alpha = a.alpha;
  d.flags = (a.c_f32 ? 1 : 0) | (a.accumulate ? 2 : 0) | (a.colsum_f32 ? 4 : 0) | (a.colsum_acc ? 8 : 0);
  d.colsum = a.colsum; d.colsum_slab = a.colsum_slab;
  d.block0 = st.batch.blocks;
  const long long nv = (long long)a.M * a.N / 4;
  st.batch.blocks += (unsigned)std::min<long long>((std::max<long long>(nv, a.M) + 255) / 256, 2048);
  c_range(a, st.lo[st.batch.n], st.hi[st.batch.n]);
  st.clo[st.batch.n] = (uintptr_t)a.colsum;
  st.chi[st.batch.n] = (uintptr_t)a.colsum + (a.colsum ? (uintptr_t)a.M * (a.colsum_f32 ? 4 : 2) : 0);
  ++st.batch.n;
}

// start deferring this stream's split-K reduces of outputs inside [out, out + out_bytes) into `arena` (>= 1 MiB,
// 256-byte aligned; the caller keeps it alive until otamd_gemm_defer_end); pending reduces of an earlier begin are
// flushed first
OTAMD_API int otamd_gemm_defer_begin(hipStream_t stream, void* arena, long long bytes, const void* out,
                                     long long out_bytes) {
  if (!arena || ((uintptr_t)arena & 255) || bytes < (1 << 20) || !out || out_bytes <= 0) return OTAMD_EINVAL;
  std::lock_guard<std::mutex> lk(g_defer_mu);
  DeferState& st = g_defer[stream];
  defer_flush_locked(st, stream);
  st.arena = (char*)arena;
  st.bytes = bytes;
  st.used = 0;
  st.out_lo = (uintptr_t)out;
  st.out_hi = (uintptr_t)out + (uintptr_t)out_bytes;
  return OTAMD_OK;
}
// launch the grouped reduce of every pending GEMM on this stream (stream-ordered); a no-op when none is pending
OTAMD_API int otamd_gemm_defer_flush(hipStream_t stream) {
  std::lock_guard<std::mutex> lk(g_defer_mu);
  auto it = g_defer.find(stream);
  return it == g_defer.end() ? OTAMD_OK : defer_flush_locked(it->second, stream);
}
// flush and leave defer mode
OTAMD_API int otamd_gemm_defer_end(hipStream_t stream) {
  std::lock_guard<std::mutex> lk(g_defer_mu);
  auto it = g_defer.find(stream);
  if (it == g_defer.end()) return OTAMD_OK;
  const int rc = defer_flush_locked(it->second, stream);
  g_defer.erase(it);
  return rc;
}
// totals since load: out[0] = GEMMs whose reduce was deferred, out[1] = grouped reduce launches
OTAMD_API int otamd_gemm_defer_stats(long long* out) {
  if (!out) return OTAMD_EINVAL;
  std::lock_guard<std::mutex> lk(g_defer_mu);
  out[0] = g_defer_gemms;
  out[1] = g_defer_launches;
  return OTAMD_OK;
}
// reduces pending on this stream
OTAMD_API int otamd_gemm_defer_pending(hipStream_t stream) {
  std::lock_guard<std::mutex> lk(g_defer_mu);
  auto it = g_defer.find(stream);
  return it == g_defer.end() ? 0 : it->second.batch.n;
}

typedef void (*gemm_fn)(GemmArgs);

static gemm_fn pick(int am, int bm) {
#define CASE(a, b) if (am == a && bm == b) return gemm_kernel<a, b>;
  CASE(OPM_K, OPM_K)
  CASE(OPM_K, OPM_MN)
  CASE(OPM_MN, OPM_MN)
  CASE(OPM_MN, OPM_K)
  CASE(OPM_CONV_FWD, OPM_K)
  CASE(OPM_CONV_DGRAD, OPM_K)
  CASE(OPM_MN, OPM_CONV_WGRAD)
#undef CASE
  return nullptr;
}

static bool aligned16(const void* p) { return ((uintptr_t)p & 15) == 0; }

int gemm2_launch(const GemmArgs& a, int tile, int splits, hipStream_t stream);   // gemm2.hip

// Plan = (tile, splits).  tile: -1 = v1 128x128 (4 waves, 2 blocks/CU), 0 = 256x256, 1 = 256x128,
// 2 = 128x256 (8 waves, 1 block/CU, LDS-DMA).  Cost model (seconds): waves of resident tiles x
// (tile MACs / relative tile throughput + fixed prologue/epilogue) + split-K slab reduce traffic.
// Relative throughputs are from tools/gemm_bench.py on MI355X.  OTAMD_GEMM_TILE forces the tile.
struct GemmPlan { int tile, splits; };

static int forced_tile() {
  static int forced = -2;
  if (forced == -2) {
    const char* e = getenv("OTAMD_GEMM_TILE");
    forced = -3;
    if (e) {
      if (!strcmp(e, "v1")) forced = -1;
      else if (!strcmp(e, "256x256")) forced = 0;
      else if (!strcmp(e, "256x128")) forced = 1;
      else if (!strcmp(e, "128x256")) forced = 2;
      else if (!strcmp(e, "256x256w4")) forced = 3;
      else if (!strcmp(e, "128x128w8")) forced = 4;
      else if (!strcmp(e, "128x64")) forced = 5;
      else if (!strcmp(e, "64x128")) forced = 6;
      else if (!strcmp(e, "128x160")) forced = 7;
      else if (!strcmp(e, "256x160")) forced = 8;
    }
  }
  return forced;
}

// candidate tiles of the analytic plan: (tile code, BM, BN, workgroups per CU, relative per-CU
// throughput, fixed prologue/epilogue seconds).  Tile 4 (128x128, 8 waves, 2 workgroups per CU) has
// the smallest epilogue and fills the chip on the 4096-row SDXL level-2 shapes where 256-wide tiles
// leave CUs idle (tools/gemm_tiles.py on MI355X: 4096x1280x1280 30.3 -> 26.2 us, 4096x10240x1280
// 129.5 -> 114.2 us, 4096x5120x1280 69.0 -> 60.0 us).
struct TileCand { int tile, bm, bn, per_cu; double rate, fixed; };
// Tiles 5 (128x64) and 6 (64x128): the skinny LoRA GEMMs (t = x A^T and u = dy B with N = rank,
// the adapter wgrads with M or N = rank), where a 128- or 256-wide tile spends 2-8x the MFMA work
// on zero padding; three workgroups per CU (48 KiB of LDS each).
// Tiles 7 (128x160) and 8 (256x160): N = 320 / 640 / 1280 without padding and 256 tiles for the
// 4096 x 1280 and 16384 x 640 shapes; rates fitted to the tools/gemm_tiles.py sweep of the SDXL step.
static const TileCand kTiles[9] = {{-1, 128, 128, 2, 0.55, 2.5e-6}, {0, 256, 256, 1, 1.0, 2.5e-6},
                                   {1, 256, 128, 1, 0.85, 2.5e-6}, {2, 128, 256, 1, 0.85, 2.5e-6},
                                   {4, 128, 128, 2, 0.85, 0.6e-6}, {5, 128, 64, 3, 0.55, 0.6e-6},
                                   {6, 64, 128, 3, 0.55, 0.6e-6}, {7, 128, 160, 2, 0.9, 4e-6},
                                   {8, 256, 160, 1, 0.9, 2.5e-6}};

static bool no_tile4() {   // OTAMD_GEMM_NO_T4=1: plan without the 128x128 tile (A/B measurements)
  static const bool v = getenv("OTAMD_GEMM_NO_T4") && !strcmp(getenv("OTAMD_GEMM_NO_T4"), "1");
  return v;
}

static GemmPlan plan_gemm(int M, int N, int K, int max_splits, bool v2_only = false) {
  const double cu_flops = 1.1e15 / 256.0;    // effective per-CU rate of the 256x256 tile
  const int ft = forced_tile();
  GemmPlan best = {-1, 1};
  double best_t = 1e300;
  for (const TileCand& c : kTiles) {
    if (ft != -3 && c.tile != ft) continue;
    if (v2_only && c.tile < 0) continue;
    if (c.tile == 4 && ft == -3 && no_tile4()) continue;
    int prev_se = 0;
    for (int s = 1; s <= max_splits; ++s) {   // every split count (3 and 5 often fill the chip best)
      const long long kps = ((long long)(K + s - 1) / s + 63) / 64 * 64;
      if (s > 1 && kps < 256) break;
      const int se = (int)((K + kps - 1) / kps);
      if (se == prev_se) continue;
      prev_se = se;
      // split plans are re-tiled by resolve_tile (otamd_gemm is always called with the planned
      // splits), which keeps the 256-wide tiles: the 128x128 tile is an unsplit-only candidate
      if (se > 1 && c.tile == 4) continue;
      const long long tiles = (long long)((M + c.bm - 1) / c.bm) * ((N + c.bn - 1) / c.bn) * se;
      const long long slots = 256LL * c.per_cu;
      const long long waves = (tiles + slots - 1) / slots;
      const double tile_t = 2.0 * c.bm * c.bn * (double)kps / (cu_flops * c.rate / c.per_cu);
      double tt = waves * (tile_t + c.fixed);
      if (se > 1) tt += ((double)se * M * N * 4.0 + (double)M * N * 2.0) / 4.5e12 + 3e-6;
      if (tt < best_t * 0.98) { best_t = tt; best = {c.tile, se}; }
    }
  }
  return best;
}

// workspace bytes a `splits`-way split-K launch needs: the fp32 C slabs [splits][M][N] and, with fused
// column sums, their partials [splits][M] after them
OTAMD_API long long otamd_gemm_ws_bytes(const GemmArgs* in, int splits) {
  if (!in || splits <= 1) return 0;
  return (long long)splits * in->M * in->N * 4 + (in->colsum ? (long long)splits * in->M * 4 : 0);
}

// C-ABI.  Preconditions (checked, OTAMD_EINVAL otherwise): M,N,K > 0; N % 4 == 0; K-mode
// operands need K % 8 == 0, MN-mode operands MN % 8 == 0; leading dims multiples of 8
// elements; base pointers 16-byte aligned; conv gathers need SC % 8 == 0.
// workspace: >= splits * M * N * 4 bytes when splits > 1.
// workspace bytes otamd_gemm needs for `splits` (0 = automatic plan); *splits_out gets the plan's splits
OTAMD_API long long otamd_gemm_plan(const GemmArgs* in, int splits, int* splits_out) {
  if (!in || in->M <= 0 || in->N <= 0 || in->K <= 0) return -1;
  int s = splits;
  if (in->batch > 1) s = 1;
  if (s <= 0) s = plan_gemm(in->M, in->N, in->K, 32, in->bmode == OPM_CONV_WT || in->A2 != nullptr || in->D != nullptr).splits;
  if (splits_out) *splits_out = s;
  return s > 1 ? otamd_gemm_ws_bytes(in, s) : 0;
}

static int resolve_tile(const GemmArgs& a, int splits, GemmPlan plan, bool v2_only);

// the tile otamd_gemm would launch for these arguments and splits (0 = automatic): -1 = v1 128x128,
// 0 = 256x256, 1 = 256x128, 2 = 128x256 (8 waves), 3 = 256x256 (4 waves), 4 = 128x128 (8 waves),
// 5 = 128x64, 6 = 64x128, 7 = 128x160, 8 = 256x160
OTAMD_API int otamd_gemm_plan_tile(const GemmArgs* in, int splits) {
  if (!in || in->M <= 0 || in->N <= 0 || in->K <= 0) return -9;
  const bool v2_only = in->bmode == OPM_CONV_WT || in->A2 != nullptr || in->D != nullptr;
  GemmPlan plan = plan_gemm(in->M, in->N, in->K, splits > 0 ? splits : 32, v2_only);
  if (splits > 0) plan = plan_gemm(in->M, in->N, in->K, 1, v2_only), plan.splits = splits;
  const long long kps = ((long long)(in->K + plan.splits - 1) / plan.splits + BK - 1) / BK * BK;
  return resolve_tile(*in, (int)((in->K + kps - 1) / kps), plan, v2_only);
}

// explicit splits: pick the best tile for them; OTAMD_GEMM_TILE overrides; conv-weight B needs v2
static int resolve_tile(const GemmArgs& a, int splits, GemmPlan plan, bool v2_only) {
  int tile = plan.tile;
  if (splits > 1 && forced_tile() == -3) {
    tile = -1;
    double bt = 1e300;
    for (const TileCand& c : kTiles) {
      if ((v2_only && c.tile < 0) || c.tile == 4) continue;
      const long long tiles = (long long)((a.M + c.bm - 1) / c.bm) * ((a.N + c.bn - 1) / c.bn) * splits;
      const double cost = (double)((tiles + 256LL * c.per_cu - 1) / (256LL * c.per_cu)) * c.bm * c.bn / c.rate * c.per_cu;
      if (cost < bt * 0.98) { bt = cost; tile = c.tile; }
    }
  } else if (forced_tile() != -3) {
    tile = forced_tile();
  }
  if (v2_only && tile < 0) tile = 0;
  return tile;
}

// force_tile: -9 = planned; otherwise the tile code (-1 v1, 0..3 v2) and splits >= 1 as given
static int gemm_impl(const GemmArgs* in, int splits, int force_tile, void* workspace, long long ws_bytes,
                     hipStream_t stream) {
  if (!in) return OTAMD_EINVAL;
  GemmArgs a = *in;
  if (a.M <= 0 || a.N <= 0 || a.K <= 0 || (a.N % 4) != 0 || splits < 0) return OTAMD_EINVAL;
  const bool v2_only = a.bmode == OPM_CONV_WT || a.A2 != nullptr || a.D != nullptr;
  if (a.D) {   // LoRA projection fused into a base GEMM: forward t = x A^T, or the dgrad's u = dY (sB) (gemm2_tiles_e.hip)
    if (a.A2 || !a.B2 || !a.T || a.lora_r != 32 || a.lora_pw <= 0 || a.N % a.lora_pw || a.batch > 1 || a.colsum)
      return OTAMD_EINVAL;
    if (!((a.amode == OPM_K || a.amode == OPM_CONV_FWD) && a.bmode == OPM_K) && !(a.amode == OPM_K && a.bmode == OPM_MN))
      return OTAMD_EUNSUPPORTED;
    if ((a.ldd % 8) || (a.ldb2 % 8) || (a.ldt % 8) || !aligned16(a.D) || !aligned16(a.B2) || !aligned16(a.T))
      return OTAMD_EINVAL;
    // dgrad form with K1 = rows per adapter part (u over several parts along K): whole 64-row K steps per part
    if (a.K1 && (a.bmode != OPM_MN || a.K1 < 0 || a.K1 % 64 || a.K % a.K1)) return OTAMD_EINVAL;
  }
  if (a.A2) {   // second K segment (LoRA fusion): forms and alignment the v2 kernels support
    if (!a.B2 || a.K1 <= 0 || a.K2 <= 0 || a.K1 % 64 || a.K != a.K1 + a.K2) return OTAMD_EINVAL;
    if (!((a.amode == OPM_K || a.amode == OPM_CONV_FWD) && a.bmode == OPM_K) && !(a.amode == OPM_K && a.bmode == OPM_MN))
      return OTAMD_EUNSUPPORTED;
    if ((a.lda2 % 8) || (a.ldb2 % 8) || (a.K2 % 8) || !aligned16(a.A2) || !aligned16(a.B2)) return OTAMD_EINVAL;
  }
  if (a.batch > 1) {   // batched: plain K/MN operands, one segment, no split-K, no fused epilogue operands
    if (a.bdiv <= 0 || a.batch > 65535 || a.A2 || a.amode > OPM_MN || a.bmode > OPM_MN || a.bias || a.rowvec ||
        a.residual || splits > 1)
      return OTAMD_EINVAL;
    if ((a.sa0 | a.sa1 | a.sb0 | a.sb1) % 8 || (a.sc0 | a.sc1) % 4) return OTAMD_EINVAL;
    splits = 1;
  }
  GemmPlan plan = plan_gemm(a.M, a.N, a.K, splits > 0 ? splits : 32, v2_only);
  if (splits > 0) plan = plan_gemm(a.M, a.N, a.K, 1, v2_only), plan.splits = splits;
  splits = plan.splits;
  if (!a.A || !a.B || !a.C || !aligned16(a.A) || !aligned16(a.B)) return OTAMD_EINVAL;
  gemm_fn fn = pick(a.amode, a.bmode);
  if (!fn && !v2_only) return OTAMD_EUNSUPPORTED;
  const bool ak = (a.amode != OPM_MN), bk = (a.bmode == OPM_K);
  if (ak && (a.K % 8)) return OTAMD_EINVAL;
  if (!ak && (a.M % 8)) return OTAMD_EINVAL;
  if (bk && (a.K % 8)) return OTAMD_EINVAL;
  if (!bk && (a.N % 8)) return OTAMD_EINVAL;
  if ((a.lda % 8) || (a.ldb % 8) || (a.ldc % 4)) return OTAMD_EINVAL;
  if (a.amode >= OPM_CONV_FWD && ((a.ga.SC % 8) || (a.ga.ld % 8))) return OTAMD_EINVAL;
  if (a.bmode >= OPM_CONV_FWD && ((a.gb.SC % 8) || (a.gb.ld % 8))) return OTAMD_EINVAL;
  if (a.rowvec && a.rows_per_vec <= 0) return OTAMD_EINVAL;
  long long kps = ((long long)(a.K + splits - 1) / splits + BK - 1) / BK * BK;
  splits = (int)((a.K + kps - 1) / kps);
  a.k_per_split = (int)kps;
  if (const int rc = defer_guard(a, stream)) return rc;
  bool deferred = false;
  if (splits > 1) {
    // the split-K reduce indexes M * N in 32 bits: refuse before anything is launched
    if ((long long)a.M * a.N >= (1LL << 32)) return OTAMD_EINVAL;
    float* ds = defer_slab(a, splits, stream);
    if (ds) {
      deferred = true;
      a.slab = ds;
    } else {
      if (!workspace || ws_bytes < otamd_gemm_ws_bytes(&a, splits) || !aligned16(workspace)) return OTAMD_EINVAL;
      a.slab = (float*)workspace;
    }
    a.colsum_slab = a.colsum ? a.slab + (long long)splits * a.M * a.N : nullptr;
  } else {
    a.slab = nullptr;
    a.colsum_slab = nullptr;
  }
  if (a.colsum && (a.amode != OPM_MN || a.A2 || a.batch > 1)) return OTAMD_EINVAL;
  int tile = force_tile == -9 ? resolve_tile(a, splits, plan, v2_only) : force_tile;
  if (a.colsum && (tile < 0 || tile == 3)) tile = 0;   // the fused column sums live in the 8-wave v2 kernels
  if (v2_only && tile < 0) return OTAMD_EUNSUPPORTED;
  int rc = OTAMD_EUNSUPPORTED;
  if (a.D && splits != 1) return OTAMD_EUNSUPPORTED;   // t needs the whole K range in one workgroup
  if (tile >= 0) rc = gemm2_launch(a, tile, splits, stream);
  if (rc == OTAMD_ELAUNCH) return rc;
  if (rc != OTAMD_OK) {
    if (!fn || a.A2 || a.colsum || a.D) return rc;   // v1 has no conv-weight B, no second K segment, no column sums
    const int tiles = ((a.M + BM - 1) / BM) * ((a.N + BN - 1) / BN);
    dim3 grid(tiles, a.batch > 1 ? a.batch : 1, splits);
    hipLaunchKernelGGL(fn, grid, dim3(NTHREADS), 65536, stream, a);
    OTAMD_CHECK_LAUNCH();
  }
  if (deferred) {
    defer_record(a, splits, stream);
  } else if (splits > 1) {
    // 8-wide needs 16-byte aligned rows of C (bf16: ldc % 8, fp32 handled element-wise)
    const bool v8 = (a.N % 8) == 0 && (a.ldc % 8) == 0 && ((uintptr_t)a.C & 15) == 0;
    const long long nv = (long long)a.M * a.N / (v8 ? 8 : 4);
    const int blocks = (int)std::min<long long>((nv + 255) / 256, 8192);
    if (v8) splitk_reduce_kernel<8><<<blocks, 256, 0, stream>>>(a, splits);
    else splitk_reduce_kernel<4><<<blocks, 256, 0, stream>>>(a, splits);
    OTAMD_CHECK_LAUNCH();
  }
  return OTAMD_OK;
}

OTAMD_API int otamd_gemm(const GemmArgs* in, int splits, void* workspace, long long ws_bytes, hipStream_t stream) {
  return gemm_impl(in, splits, -9, workspace, ws_bytes, stream);
}

// explicit plan (the autotuner's candidates and its cached choice): tile -1 = v1 128x128, 0 = 256x256,
// 1 = 256x128, 2 = 128x256, 3 = 256x256 (4 waves), 4 = 128x128 (8 waves, 2 workgroups per CU),
// 5 = 128x64, 6 = 64x128 (3 workgroups per CU), 7 = 128x160, 8 = 256x160, 9 / 10 = 5 / 6 on a 4-deep LDS ring;
// splits >= 1 (rounded to whole 64-deep K steps)
OTAMD_API int otamd_gemm_explicit(const GemmArgs* in, int tile, int splits, void* workspace, long long ws_bytes,
                                  hipStream_t stream) {
  if (tile < -1 || tile > 10 || splits < 1) return OTAMD_EINVAL;
  return gemm_impl(in, splits, tile, workspace, ws_bytes, stream);
}

OTAMD_API int otamd_gemm_args_size(void) { return (int)sizeof(GemmArgs); }
OTAMD_API int otamd_conv_geom_size(void) { return (int)sizeof(ConvGeom); }
