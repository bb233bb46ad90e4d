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
//                  lane-local + one permlane32 swap); P^T accumulator registers feed O^T = V^T P^T
//                  directly as the MFMA B operand; V^T comes from ds_read_b64_tr_b16.
//   dK/dV        : S = Q K^T with the key on the lane; P and dS accumulators feed
//                  dV^T = dO^T P and dK^T = Q^T dS directly; dO^T, Q^T by transposed LDS reads.
// Staging: every streamed tile (K/V for fwd and dQ, Q/dO and the {lse, delta} pairs for dK/dV)
// goes HBM/L2 -> LDS by LDS-DMA (buffer_load ... lds) into an NS-deep ring, the swizzles applied
// on the source address; one s_barrier per tile (RAW for tile t, WAR for the stage refilled
// with tile t+NS-1).  That barrier is BARRIER_LDS: gfx950's s_barrier does not wait for a wave's
// outstanding ds_reads, and the compiler sinks the last MFMA of a tile (with the lgkmcnt wait for
// its operand reads) below a raw s_barrier -- another wave's refill DMA then raced the reads it
// had issued (dQ run-to-run differences under LDS contention from co-resident kernels, round 6).
// Out-of-range rows / padded head columns are zero-filled by the descriptor range check or an
// invalid offset.
// Softmax VALU is kept under the MFMA time: single-issue fp32 math (no v_pk_*: they cost more than two
// single ops beside MFMAs), key masking only on the partial last tile, and the forward's O rescale skipped
// when no lane's max grew.
#include "common.h"

#include <algorithm>
#include <cstring>
#include <cstdlib>
#include <mutex>
#include <unordered_set>
#include <utility>
#include <type_traits>

struct AttnArgs {
  const bf16_t* q; const bf16_t* k; const bf16_t* v; bf16_t* o; float* lse;
  const bf16_t* dout; const float* delta; bf16_t* dq; bf16_t* dk; bf16_t* dv; float* dk32; float* dv32;
  long long ldq, ldk, ldv, ldo, lddo, lddq, lddk, lddv;     // token strides (elements)
  long long bsq, bsk, bsv, bso, bsdo, bsdq, bsdk, bsdv;     // batch strides (elements)
  int B, H, Nq, Nk, Dv;
  float scale;
  int qsplit;
  int xcd;   // (the header's reserved pad_; callers pass 0) set by the launchers: XCD-grouped block order
};

#define KT 64   // keys per staged tile (fwd / dQ)
#define RESCALE_T 8.0f   // forward: lazy-max threshold (log2 units)
#define OFF_INVALID 0x80000000u
static constexpr float LOG2E = 1.4426950408889634f;

typedef __attribute__((address_space(3))) short4v lds_s4;
typedef __attribute__((address_space(3))) void lds_void_t;

#define MEMBAR() asm volatile("" ::: "memory")
#define BARRIER()                 \
  do {                            \
    MEMBAR();                     \
    __builtin_amdgcn_s_barrier(); \
    MEMBAR();                     \
  } while (0)

// publishes this wave's ds_write results: s_barrier alone does not wait for them (cdna_hip_programming.md §5)
#define BARRIER_LDS()                                     \
  do {                                                    \
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");    \
    BARRIER();                                            \
  } while (0)

template <int N>
__device__ __forceinline__ void wait_vmcnt() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory"); }

// LDS-DMA, 16 / 4 bytes per lane (1 KiB / 256 B per wave instruction).  Inline asm so the
// compiler's waitcnt pass does not drain vmcnt in front of ds_reads of other stages.
__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t rs, char* lds, unsigned off) {
  const unsigned m0 = (unsigned)(size_t)(lds_void_t*)lds;
  asm volatile("buffer_load_dwordx4 %1, %2, 0 offen lds" ::"{m0}"(m0), "v"(off), "s"(rs) : "memory");
}
__device__ __forceinline__ void dma4(__amdgpu_buffer_rsrc_t rs, char* lds, unsigned off) {
  const unsigned m0 = (unsigned)(size_t)(lds_void_t*)lds;
  asm volatile("buffer_load_dword %1, %2, 0 offen lds" ::"{m0}"(m0), "v"(off), "s"(rs) : "memory");
}
// make the compiler drain its own loads of x here (before any DMA it cannot see is in flight)
template <typename T>
__device__ __forceinline__ void consume(const T& x) { asm volatile("" ::"v"(x)); }

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* base, long long bytes) {
  return __builtin_amdgcn_make_buffer_rsrc((void*)base, (short)0, (int)bytes, 0x00020000);
}

// Workgroup order (cdna_hip_programming.md T1): the hardware deals workgroup i (x fastest) to XCD i % 8, so the
// blocks of one (batch, head) -- which all stream that head's K / V (forward, dQ) or Q / dO (dK/dV) tiles --
// land on all 8 XCDs and each XCD's L2 fetches the same tiles.  With a.xcd set, the grid is renumbered so that
// XCD x runs a contiguous range of (block, head, batch): one (batch, head)'s blocks share one L2 (bijective for
// any count).
__device__ __forceinline__ void block_ids(const AttnArgs& a, int& bx, int& by, int& bz) {
  if (!a.xcd) {
    bx = blockIdx.x, by = blockIdx.y, bz = blockIdx.z;
    return;
  }
  const int nx = gridDim.x, ny = gridDim.y;
  const int total = nx * ny * gridDim.z;
  const int lin = blockIdx.x + nx * (blockIdx.y + ny * blockIdx.z);
  const int x = lin & 7, j = lin >> 3, q = total >> 3, rr = total & 7;
  const int n = (x < rr ? x * (q + 1) : rr * (q + 1) + (x - rr) * q) + j;
  bx = n % nx;
  const int t = n / nx;
  by = t % ny;
  bz = t / ny;
}

// row image: [rows][D] bf16, 16-byte chunk c of row r stored at c ^ (r & 7)
// transposed-read image: [rows][D] bf16, 32-byte block b of row r stored at b ^ sw(r)
template <int D> __device__ __forceinline__ int tr_sw(int r) { return (D == 64) ? (((r >> 1) & 1) << 1) : ((r & 3) << 1); }
template <int D> __device__ __forceinline__ int tr_off(int r, int col) {
  return r * (D * 2) + (((col >> 4) ^ tr_sw<D>(r)) << 5) + ((col & 15) << 1);
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

// Dual-use image (cdna_hip_programming.md T10, "one image for row reads AND transposed reads"): [rows][D] bf16,
// 16-byte chunk ch of row r stored at chunk ch ^ dsw(r).  One copy of a tile serves the ds_read_b128 row reads of a
// 32x32x16 operand (lds_row_frag's pattern) and the ds_read_b64_tr_b16 reads (tr_frag's pattern), both
// conflict-free under the gfx950 bank rule (64 x 4-byte banks; b128 in four 16-lane groups, tr_b16 in two 32-lane
// halves: tools/lds_bank_model.py enumerates every XOR of the row bits and prints the cost of each read).  The
// row-only swizzle above (chunk ^ (r & 7)) is 2-way on the b128 row read; the 32-byte-block one conflicts on it.
// D = 64 (128-byte rows): dsw = {r1, r2, r1 ^ r3}; D = 128 (256-byte rows): dsw = (r & 3) << 2 | (r >> 2) & 3.
template <int D> __device__ __forceinline__ int dsw(int r) {
  if constexpr (D == 64) return ((r >> 1) & 1) | (((r >> 2) & 1) << 1) | ((((r >> 1) ^ (r >> 3)) & 1) << 2);
  else return ((r & 3) << 2) | ((r >> 2) & 3);
}
template <int D> __device__ __forceinline__ int dual_off(int r, int col) {   // col: a multiple of 4 for tr reads
  return r * (D * 2) + (((col >> 3) ^ dsw<D>(r)) << 4) + ((col & 7) << 1);
}
// lane-constant byte offsets of the dual-image reads of a 32-row sub-tile at row 0 (rows 32u.. and the second
// 16-row half add multiples of 16 rows, which leave dsw unchanged): row reads of chunk 2s + h, and the two
// ds_read_b64_tr_b16 halves (e = 0: rows 4h + q, e = 1: rows 8 + 4h + q) of column block dt
template <int D> struct DualOffs {
  int row[D / 16];
  int tr[D / 32][2];
  __device__ __forceinline__ void prepare() {
    const int lane = threadIdx.x & 63, r = lane & 31, h = lane >> 5;
    const int G = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
#pragma unroll
    for (int s = 0; s < D / 16; ++s) row[s] = r * (D * 2) + (((2 * s + h) ^ dsw<D>(r)) << 4);
#pragma unroll
    for (int dt = 0; dt < D / 32; ++dt)
#pragma unroll
      for (int e = 0; e < 2; ++e) tr[dt][e] = dual_off<D>(4 * h + q + 8 * e, dt * 32 + 16 * (G & 1) + 4 * p);
  }
  // row fragment s of the sub-tile whose first row is `row0` (a multiple of 16)
  __device__ __forceinline__ bf16x8 rowf(const char* img, int row0, int s) const {
    return *reinterpret_cast<const bf16x8*>(img + row0 * (D * 2) + row[s]);
  }
  // tr_frag's operand (rows row0 + 16 s ..) of column block dt
  __device__ __forceinline__ bf16x8 trf(const char* img, int row0, int s, int dt) const {
    const char* base = img + (row0 + 16 * s) * (D * 2);
    const short4v lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(base + tr[dt][0]));
    const short4v hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(base + tr[dt][1]));
    short8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    return __builtin_bit_cast(bf16x8, v);
  }
};

// x ~= t0 + t1 + t2 (bf16 each, round-to-nearest at every stage): returns {t0 | t1 << 16, t2}
__device__ __forceinline__ uint2 split3_bf16(float x) {
  const bf16_t t0 = f2bf(x);
  const float r1 = x - bf2f(t0);
  const bf16_t t1 = f2bf(r1);
  const bf16_t t2 = f2bf(r1 - bf2f(t1));
  return make_uint2((uint32_t)t0 | ((uint32_t)t1 << 16), (uint32_t)t2);
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

// value of x in lane l ^ 32 (one permlane32 swap + select)
__device__ __forceinline__ float xor32(float x) {
  const auto s = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return __uint_as_float((threadIdx.x & 32) ? s[0] : s[1]);
}

// 32 rows x 32 columns of fp32 accumulators (one 32x32 MFMA tile; lane (r, h) holds columns
// 8g + 4h .. +3 of row r for g = 0..3) -> bf16 row segments of `row` starting at col0, scaled by
// `mul`.  Column groups are paired with v_permlane32_swap so each lane stores 16 contiguous bytes
// (cdna_hip_programming.md T21): 2 dwordx4 stores per lane instead of 4 dwordx2.  All 64 lanes
// execute the swaps; `ok` (row in range) gates only the stores.  Needs 16-byte aligned rows.
__device__ __forceinline__ void store_tile_bf16(bf16_t* row, int col0, const float16v& x, float mul, int Dv, bool ok) {
  const int h = (threadIdx.x >> 5) & 1;
#pragma unroll
  for (int g = 0; g < 4; g += 2) {
    const uint32_t a0 = (uint32_t)f2bf(x[4 * g] * mul) | ((uint32_t)f2bf(x[4 * g + 1] * mul) << 16);
    const uint32_t a1 = (uint32_t)f2bf(x[4 * g + 2] * mul) | ((uint32_t)f2bf(x[4 * g + 3] * mul) << 16);
    const uint32_t b0 = (uint32_t)f2bf(x[4 * g + 4] * mul) | ((uint32_t)f2bf(x[4 * g + 5] * mul) << 16);
    const uint32_t b1 = (uint32_t)f2bf(x[4 * g + 6] * mul) | ((uint32_t)f2bf(x[4 * g + 7] * mul) << 16);
    const auto s0 = __builtin_amdgcn_permlane32_swap(a0, b0, false, false);
    const auto s1 = __builtin_amdgcn_permlane32_swap(a1, b1, false, false);
    const int c = col0 + 8 * g + 8 * h;
    if (ok && c < Dv) *reinterpret_cast<uint4*>(row + c) = make_uint4(s0[0], s1[0], s0[1], s1[1]);
  }
}

// The tile loop unrolled by the ring depth NS: the ring slot t % NS is a compile-time constant in
// every copy of the body, so every LDS address is a lane base + an immediate offset (no per-tile
// address VALU).  step(t, std::integral_constant<int, t % NS>).
template <typename F, int... I>
__device__ __forceinline__ void stage_steps(int t, F& step, std::integer_sequence<int, I...>) {
  (step(t + I, std::integral_constant<int, I>{}), ...);
}
template <typename F, int... I>
__device__ __forceinline__ void stage_tail(int t, int n, F& step, std::integer_sequence<int, I...>) {
  ((t + I < n ? step(t + I, std::integral_constant<int, I>{}) : void()), ...);
}
template <int NS, bool UNROLL = true, typename F>
__device__ __forceinline__ void stage_loop(int ntiles, F&& step) {
  if constexpr (UNROLL) {
    int t = 0;
    for (; t + NS <= ntiles; t += NS) stage_steps(t, step, std::make_integer_sequence<int, NS>{});
    stage_tail(t, ntiles, step, std::make_integer_sequence<int, NS - 1>{});
  } else {   // (D = 128: the unrolled copies would not fit the register budget)
    for (int t = 0; t < ntiles; ++t) step(t, t % NS);
  }
}
// The same with the last tile apart: step(t, slot, std::bool_constant<last>).  Only the last key tile can hold keys
// past Nk, so the per-score tail mask is compiled into that copy alone (in a shared body the compiler if-converts
// the uniform `tile is partial` branch into 32 compares / selects on every tile).
template <typename F, int... I>
__device__ __forceinline__ void stage_steps_nl(int t, F& step, std::integer_sequence<int, I...>) {
  (step(t + I, std::integral_constant<int, I>{}, std::false_type{}), ...);
}
template <typename F, int... I>
__device__ __forceinline__ void stage_tail_nl(int t, int n, F& step, std::integer_sequence<int, I...>) {
  ((t + I < n ? step(t + I, std::integral_constant<int, I>{}, std::false_type{}) : void()), ...);
}
template <int NS, bool UNROLL = true, typename F>
__device__ __forceinline__ void stage_loop_last(int ntiles, F&& step) {
  if (ntiles <= 0) return;
  const int nmain = ntiles - 1;
  if constexpr (UNROLL) {
    int t = 0;
    for (; t + NS <= nmain; t += NS) stage_steps_nl(t, step, std::make_integer_sequence<int, NS>{});
    stage_tail_nl(t, nmain, step, std::make_integer_sequence<int, NS - 1>{});
    step(nmain, nmain % NS, std::true_type{});   // one copy with a run-time ring slot
  } else {
    for (int t = 0; t < nmain; ++t) step(t, t % NS, std::false_type{});
    step(nmain, nmain % NS, std::true_type{});
  }
}

// DMA geometry of one [ROWS x D] bf16 image, split over 4 waves: piece p (1 KiB) = wave + 4 i; lane l writes
// bytes [16 l, 16 l + 16) of the piece.  MODE: IMG_ROW (chunk ^ (r & 7)), IMG_TR (32-byte block ^ tr_sw), IMG_DUAL
// (chunk ^ dsw: row and transposed reads of one copy).
constexpr int IMG_ROW = 0, IMG_TR = 1, IMG_DUAL = 2;
template <int D, int ROWS, int MODE>
struct DmaImg {
  static constexpr int RB = D * 2;
  static constexpr int NP = ROWS * RB / 1024;
  static constexpr int PW = NP / 4;
  static_assert(PW >= 1 && NP % 4 == 0, "image must split into whole pieces per wave");
  int row[PW], col[PW];
  __device__ __forceinline__ void prepare(int wave, int lane) {
#pragma unroll
    for (int i = 0; i < PW; ++i) {
      const int byte = (wave + 4 * i) * 1024 + lane * 16;
      const int r = byte / RB, pos = (byte % RB) >> 4;
      row[i] = r;
      col[i] = MODE == IMG_TR ? ((((pos >> 1) ^ tr_sw<D>(r)) << 4) + ((pos & 1) << 3))
                              : ((pos ^ (MODE == IMG_DUAL ? dsw<D>(r) : (r & 7))) << 3);
    }
  }
  // rows [row0, row0 + ROWS) of a [nrows x ld] operand whose descriptor starts at (batch, head)
  __device__ __forceinline__ void issue(__amdgpu_buffer_rsrc_t rs, char* img, long long ld, int row0, int nrows,
                                        int Dv, int wave) const {
#pragma unroll
    for (int i = 0; i < PW; ++i) {
      const int rr = row0 + row[i];
      const unsigned off = (rr < nrows && col[i] < Dv) ? (unsigned)(rr * (int)ld + col[i]) * 2u : OFF_INVALID;
      dma16(rs, img + (wave + 4 * i) * 1024, off);
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

// P^T = exp2(S^T c - bias) in place (v_fma_f32 + v_exp_f32); masked keys already -inf.  Single-issue f32
// math throughout the softmax: beside MFMAs a packed v_pk_fma_f32 costs more than the two v_fma_f32 it
// replaces (MI355X_MICROARCH.md, per-instruction constants), and the file is built with -fno-slp-vectorize
// so the compiler does not re-pack it.
__device__ __forceinline__ void exp2_scaled(float16v& S, float c, float bias) {
#pragma unroll
  for (int i = 0; i < 16; ++i) S[i] = __builtin_amdgcn_exp2f(fmaf(S[i], c, -bias));
}
// The D = 128 forward and dK/dV kernels keep the packed form (v_pk_fma_f32 / v_pk_mul_f32): at one wave per
// SIMD (dK/dV) the single-issue form measured slower (Flux bwd 1274 -> 1414 us), while D = 64 gained 3-18 % and
// the D = 128 dQ kernel ~1 % (profiles/r3_attn_scalar_ab.txt).  Same operations and rounding either way.
typedef float f2v __attribute__((ext_vector_type(2)));
__device__ __forceinline__ void exp2_scaled_pk(float16v& S, float c, float bias) {
  const f2v c2 = {c, c}, nb = {-bias, -bias};
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    f2v x = {S[2 * k], S[2 * k + 1]};
    x = x * c2 + nb;
    S[2 * k] = __builtin_amdgcn_exp2f(x.x);
    S[2 * k + 1] = __builtin_amdgcn_exp2f(x.y);
  }
}


// ------------------------------------------------------------------------------------------
// NS = LDS ring depth.  D = 128 runs NS = 2 (64 KiB): two blocks (8 waves) per CU instead of one
// with the 96 KiB 3-deep ring -- the MFMA of one wave overlaps the softmax of the SIMD's other wave.
// D = 64 runs NS = 2 (32 KiB) at <= 128 VGPRs: four blocks, four waves per SIMD.
template <int D, int NS>
__global__ void __launch_bounds__(256, (D == 64 && NS == 2) ? 4 : 2) attn_fwd_kernel(AttnArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int TB = KT * D * 2;      // bytes of one [64 x D] image
  constexpr int STG = 2 * TB;         // K row image + V transposed-read image
  using KImg = DmaImg<D, KT, IMG_DUAL>;   // row reads only; the dual swizzle is conflict-free for them
  using VImg = DmaImg<D, KT, IMG_TR>;
  constexpr int LOADS = KImg::PW + VImg::PW;
  int bx, hh, b;
  block_ids(a, bx, hh, b);
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int r = lane & 31, h = lane >> 5;
  const int q0 = bx * 128 + wave * 32;
  const bf16_t* Q = a.q + b * a.bsq + hh * a.Dv;
  const auto rk = rsrc(a.k + b * a.bsk + hh * a.Dv, ((long long)(a.Nk - 1) * a.ldk + a.Dv) * 2);
  const auto rv = rsrc(a.v + b * a.bsv + hh * a.Dv, ((long long)(a.Nk - 1) * a.ldv + a.Dv) * 2);
  KImg ki;
  VImg vi;
  ki.prepare(wave, lane);
  vi.prepare(wave, lane);
  DualOffs<D> dof;
  dof.prepare();
  const int ntiles = (a.Nk + KT - 1) / KT;

  bf16x8 qf[D / 16];
  load_row_frags<D>(qf, Q, a.ldq, q0, a.Nq, a.Dv);
#pragma unroll
  for (int s = 0; s < NS - 1; ++s)
    if (s < ntiles) {
      ki.issue(rk, smem + s * STG, a.ldk, s * KT, a.Nk, a.Dv, wave);
      vi.issue(rv, smem + s * STG + TB, a.ldv, s * KT, a.Nk, a.Dv, wave);
    }
#pragma unroll
  for (int s = 0; s < D / 16; ++s) consume(qf[s]);
  const float c = a.scale * LOG2E;

  float16v O[D / 32];
#pragma unroll
  for (int t = 0; t < D / 32; ++t) O[t] = zero16();
  float m = -INFINITY, l = 0.f;

  auto step = [&](int t, auto si_tag, auto last_tag) {
    const int SI = si_tag;   // t % NS (a compile-time constant when unrolled)
    constexpr bool LAST = decltype(last_tag)::value;

    if (t + NS - 2 < ntiles) wait_vmcnt<(NS - 2) * LOADS>();
    else wait_vmcnt<0>();
    BARRIER_LDS();   // WAR: this wave's reads of the slot refilled next have retired
    if (t + NS - 1 < ntiles) {
      char* st = smem + ((SI + NS - 1) % NS) * STG;
      ki.issue(rk, st, a.ldk, (t + NS - 1) * KT, a.Nk, a.Dv, wave);
      vi.issue(rv, st + TB, a.ldv, (t + NS - 1) * KT, a.Nk, a.Dv, wave);
    }
    const char* kimg = smem + SI * STG;
    const char* vimg = kimg + TB;
#pragma unroll
    for (int sub = 0; sub < KT / 32; ++sub) {
      if (LAST && t * KT + sub * 32 >= a.Nk) break;   // a wholly masked 32-key half of the last tile (Lk = 77): P = 0
      float16v S = zero16();
#pragma unroll
      for (int s = 0; s < D / 16; ++s) S = mfma32(dof.rowf(kimg, sub * 32, s), qf[s], S);
      const int kbase = t * KT + sub * 32;
      if (LAST && kbase + 32 > a.Nk) {
#pragma unroll
        for (int i = 0; i < 16; ++i)
          if (kbase + acc_row(i, h) >= a.Nk) S[i] = -INFINITY;
      }
      float tmax = S[0];
#pragma unroll
      for (int i = 1; i < 16; ++i) tmax = fmaxf(tmax, S[i]);
      // lazy max (cdna_hip_programming.md T13): m only moves when a score of this lane's half-row exceeds it by more
      // than RESCALE_T (log2 units), so P <= 2^RESCALE_T otherwise; any m >= -inf normalises out of O / l and the
      // LSE (m + log2 l), and O and l always see the same factor.  The full row max (the half-rows' xor32) is needed
      // only on that wave-uniform branch.
      if (__builtin_amdgcn_ballot_w64(tmax * c > m + RESCALE_T) != 0) {
        const float mn = fmaxf(m, fmaxf(tmax, xor32(tmax)) * c);
        const float alpha = __builtin_amdgcn_exp2f(m - mn);
        l *= alpha;
        if constexpr (D == 64) {
#pragma unroll
          for (int dt = 0; dt < D / 32; ++dt)
#pragma unroll
            for (int i = 0; i < 16; ++i) O[dt][i] *= alpha;
        } else {
          const f2v a2 = {alpha, alpha};
#pragma unroll
          for (int dt = 0; dt < D / 32; ++dt)
#pragma unroll
            for (int k = 0; k < 8; ++k) {
              f2v o = {O[dt][2 * k], O[dt][2 * k + 1]};
              o *= a2;
              O[dt][2 * k] = o.x;
              O[dt][2 * k + 1] = o.y;
            }
        }
        m = mn;
      }
      float rs;
      if constexpr (D == 64) {
        exp2_scaled(S, c, m);
        float r0 = S[0], r1 = S[1];   // two independent add chains
#pragma unroll
        for (int k = 1; k < 8; ++k) { r0 += S[2 * k]; r1 += S[2 * k + 1]; }
        rs = r0 + r1;
      } else {
        exp2_scaled_pk(S, c, m);
        f2v rs2 = {S[0], S[1]};
#pragma unroll
        for (int k = 1; k < 8; ++k) rs2 += f2v{S[2 * k], S[2 * k + 1]};
        rs = rs2.x + rs2.y;
      }
      l += rs;   // this lane's half-row (the halves meet once, after the loop)
      const bf16x8 p0 = pack_acc(S, 0), p1 = pack_acc(S, 1);
#pragma unroll
      for (int dt = 0; dt < D / 32; ++dt) {
        O[dt] = mfma32(tr_frag<D>(vimg, sub * 32, 0, dt * 32), p0, O[dt]);
        O[dt] = mfma32(tr_frag<D>(vimg, sub * 32, 1, dt * 32), p1, O[dt]);
      }
    }
  };
  stage_loop_last<NS, (D <= 64)>(ntiles, step);
  l += xor32(l);
  const int q = q0 + r;
  const float inv = 1.f / l;
  bf16_t* Op = a.o + b * a.bso + (long long)min(q, a.Nq - 1) * a.ldo + hh * a.Dv;
#pragma unroll
  for (int dt = 0; dt < D / 32; ++dt) store_tile_bf16(Op, dt * 32, O[dt], inv, a.Dv, q < a.Nq);
  if (q < a.Nq && h == 0 && a.lse) a.lse[((long long)b * a.H + hh) * a.Nq + q] = m + __log2f(l);
}

// dQ: per wave 32 queries, iterate over key tiles (a dual-use K image -- row reads for S, transposed reads for
// dQ -- and a V image per stage)
// NS = LDS ring depth, KTD = keys per tile.  Launched as (otamd_attn_bwd):
//   D = 64:  <64, 3> -- 64-key tiles (two 32-key sub-tiles per barrier) 3 deep (48 KiB: one dual-use K image and
//            one V image per stage); three blocks per CU (__launch_bounds__(256, 3), set by the VGPRs), so the SDXL
//            level-2 grid (8 x 20 heads x 4 = 640 blocks) runs in one round of 768 slots
//   D = 128: <128, 2, 64> -- 64-key tiles 2 deep (64 KiB), two blocks per CU: 1086 us per Flux call
//            (4 x 2381 x 24 heads) against 1104 us for 32-key tiles 3 deep (round 4, same box)
template <int D, int NS, int KTD = KT>
__global__ void __launch_bounds__(256, D == 64 ? 3 : 2) attn_bwd_dq_kernel(AttnArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int TB = KTD * D * 2;
  constexpr int STG = 2 * TB;
  using Img = DmaImg<D, KTD, IMG_DUAL>;
  constexpr int LOADS = 2 * Img::PW;
  int bx, hh, b;
  block_ids(a, bx, hh, b);
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int r = lane & 31, h = lane >> 5;
  const int q0 = bx * 128 + wave * 32;
  const auto rk = rsrc(a.k + b * a.bsk + hh * a.Dv, ((long long)(a.Nk - 1) * a.ldk + a.Dv) * 2);
  const auto rv = rsrc(a.v + b * a.bsv + hh * a.Dv, ((long long)(a.Nk - 1) * a.ldv + a.Dv) * 2);
  Img im;
  im.prepare(wave, lane);
  DualOffs<D> dof;
  dof.prepare();
  const int ntiles = (a.Nk + KTD - 1) / KTD;
  auto issue = [&](int t, char* st) {
    im.issue(rk, st, a.ldk, t * KTD, a.Nk, a.Dv, wave);
    im.issue(rv, st + TB, a.ldv, t * KTD, a.Nk, a.Dv, wave);
  };

  bf16x8 qf[D / 16], gf[D / 16];
  load_row_frags<D>(qf, a.q + b * a.bsq + hh * a.Dv, a.ldq, q0, a.Nq, a.Dv);
  load_row_frags<D>(gf, a.dout + b * a.bsdo + hh * a.Dv, a.lddo, q0, a.Nq, a.Dv);
  const int q = q0 + r;
  const long long srow = ((long long)b * a.H + hh) * a.Nq;
  // delta = sum_d dO * O for this lane's query (the two half-waves split the head dim), published
  // with the forward's lse as the {lse, delta} pair the dK/dV kernel (launched next) streams: this
  // replaces a separate delta pass over O and dO
  float dlt = 0.f, lse2 = 0.f;
  if (q < a.Nq) {
    const bf16_t* Op = a.o + b * a.bso + (long long)q * a.ldo + hh * a.Dv;
    const bf16_t* Gp = a.dout + b * a.bsdo + (long long)q * a.lddo + hh * a.Dv;
    const int d1 = min(a.Dv, (h + 1) * (D / 2));
    for (int d = h * (D / 2); d < d1; d += 8) {
      float of[8], gv[8];
      unpack8(*reinterpret_cast<const bf8*>(Op + d), of);
      unpack8(*reinterpret_cast<const bf8*>(Gp + d), gv);
#pragma unroll
      for (int j = 0; j < 8; ++j) dlt = fmaf(of[j], gv[j], dlt);
    }
    lse2 = a.lse[srow + q];
  }
  dlt += __shfl_xor(dlt, 32, 64);
  // the dK/dV kernel's bias record of this query: -lse / c and -delta, each as three bf16 terms (hi + mid + lo
  // carry ~24 bits), [b0 b1 b2 d0 d1 d2 0 0]: used there as an MFMA A-operand k-step so S' = S - lse/c and
  // dP' = dP - delta come out of the accumulator chains (attn_bwd_dkv_kernel)
  if (h == 0 && q < a.Nq) {
    const float cc = a.scale * LOG2E;
    const uint2 bl = split3_bf16(-lse2 / cc), dl = split3_bf16(-dlt);
    reinterpret_cast<uint4*>(const_cast<float*>(a.delta))[srow + q] =
        make_uint4(bl.x, bl.y | (dl.x << 16), (dl.x >> 16) | (dl.y << 16), 0u);
  }
  consume(dlt);
  consume(lse2);
#pragma unroll
  for (int s = 0; s < NS - 1; ++s)
    if (s < ntiles) issue(s, smem + s * STG);
#pragma unroll
  for (int s = 0; s < D / 16; ++s) { consume(qf[s]); consume(gf[s]); }
  const float c = a.scale * LOG2E;
  float16v ndl;
#pragma unroll
  for (int i = 0; i < 16; ++i) ndl[i] = -dlt;

  float16v dQ[D / 32];
#pragma unroll
  for (int t = 0; t < D / 32; ++t) dQ[t] = zero16();

  auto step = [&](int t, auto si_tag, auto last_tag) {
    const int SI = si_tag;   // t % NS (a compile-time constant when unrolled)
    constexpr bool LAST = decltype(last_tag)::value;

    if (t + NS - 2 < ntiles) wait_vmcnt<(NS - 2) * LOADS>();
    else wait_vmcnt<0>();
    BARRIER_LDS();   // WAR: this wave's reads of the slot refilled next have retired
    if (t + NS - 1 < ntiles) issue(t + NS - 1, smem + ((SI + NS - 1) % NS) * STG);
    const char* kimg = smem + SI * STG;
    const char* vimg = kimg + TB;
#pragma unroll
    for (int sub = 0; sub < KTD / 32; ++sub) {
      if (LAST && t * KTD + sub * 32 >= a.Nk) break;   // a wholly masked 32-key half of the last tile: dS = 0
      // dP^T starts from -delta (this lane's query: a per-lane constant vector built once), so
      // dS^T = P^T dP'^T needs no subtraction per score
      float16v S = zero16(), dP = ndl;
#pragma unroll
      for (int s = 0; s < D / 16; ++s) {
        S = mfma32(dof.rowf(kimg, sub * 32, s), qf[s], S);
        dP = mfma32(dof.rowf(vimg, sub * 32, s), gf[s], dP);
      }
      const int kbase = t * KTD + sub * 32;
      if (LAST && kbase + 32 > a.Nk) {
#pragma unroll
        for (int i = 0; i < 16; ++i)
          if (kbase + acc_row(i, h) >= a.Nk) S[i] = -INFINITY;
      }
      exp2_scaled(S, c, lse2);
#pragma unroll
      for (int i = 0; i < 16; ++i) S[i] *= dP[i];   // dS^T = P^T (dP^T - delta)
      const bf16x8 s0 = pack_acc(S, 0), s1 = pack_acc(S, 1);
#pragma unroll
      for (int dt = 0; dt < D / 32; ++dt) {
        dQ[dt] = mfma32(dof.trf(kimg, sub * 32, 0, dt), s0, dQ[dt]);
        dQ[dt] = mfma32(dof.trf(kimg, sub * 32, 1, dt), s1, dQ[dt]);
      }
    }
  };
  stage_loop_last<NS, (D <= 64)>(ntiles, step);
  bf16_t* Dp = a.dq + b * a.bsdq + (long long)min(q, a.Nq - 1) * a.lddq + hh * a.Dv;
#pragma unroll
  for (int dt = 0; dt < D / 32; ++dt) store_tile_bf16(Dp, dt * 32, dQ[dt], a.scale, a.Dv, q < a.Nq);
}

// dK, dV: per wave 32 keys (block 128 keys), iterate over query tiles of QS (32 or 64) in this split's range.
// Stage: dual-use Q and dO images (row reads for S / dP, transposed reads for dK / dV: one copy each) + the tile's
// QS bias records (written by the dQ kernel: -lse/c and -delta as three bf16 terms each).  The record is one extra
// MFMA k-step of S and of dP (A = the record of the lane's query, B = ones in the matching three k slots), so the
// accumulators come out as S - lse/c and dP - delta: no per-score subtraction and no per-register {lse, delta}
// reads in the softmax.  A 64-query stage runs two 32-query sub-tiles per barrier.
// D = 128: the dK/dV accumulators alone take 128 VGPRs, so the full 512-entry register file is used (one wave
// per SIMD) instead of spilling at 256.
// (A software-pipelined D = 128 variant -- S / dP of tile t+1 on the MFMA pipe during tile t's
// softmax, 4-deep ring -- measured slower: 1487-1510 vs 1349 us for the Flux bwd; not kept.)
// OCC = waves per SIMD.  D = 64 at OCC = 3 (<= 168 VGPRs: the tile loop not unrolled) fits 768 blocks on
// the chip, the SDXL level-2 grid (8 key blocks x 20 heads x 4 = 640) in one round instead of 1.25 at OCC 2.
template <int D, int QS> constexpr int dkv_stage() { return 2 * QS * D * 2 + QS * 16; }
template <int D, int QS> constexpr int dkv_lds() { return 3 * dkv_stage<D, QS>(); }   // the kernel's 3-deep ring

template <int D, int OCC, int QS>
__global__ void __launch_bounds__(256, OCC) attn_bwd_dkv_kernel(AttnArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int TB = QS * D * 2;                 // one [QS x D] image
  constexpr int STG = dkv_stage<D, QS>();        // Q + dO images + QS 16-byte bias records
  constexpr int NS = 3;
  constexpr int RPW = QS / 4;                    // bias records moved per wave
  using Img = DmaImg<D, QS, IMG_DUAL>;
  constexpr int LOADS = 2 * Img::PW + 1;
  int bx, hh, bz;
  block_ids(a, bx, hh, bz);
  const int b = bz / a.qsplit, split = bz % a.qsplit;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int r = lane & 31, h = lane >> 5;
  const int k0 = bx * 128 + wave * 32;
  const long long srow = ((long long)b * a.H + hh) * a.Nq;
  const auto rq = rsrc(a.q + b * a.bsq + hh * a.Dv, ((long long)(a.Nq - 1) * a.ldq + a.Dv) * 2);
  const auto rg = rsrc(a.dout + b * a.bsdo + hh * a.Dv, ((long long)(a.Nq - 1) * a.lddo + a.Dv) * 2);
  const auto rp = rsrc(a.delta + 4 * srow, (long long)a.Nq * 16);
  Img im;
  im.prepare(wave, lane);
  DualOffs<D> dof;
  dof.prepare();

  const int per = (((a.Nq + a.qsplit - 1) / a.qsplit) + QS - 1) / QS * QS;
  const int qbeg = split * per;
  const int qend = min(a.Nq, qbeg + per);
  const int ntiles = qend > qbeg ? (qend - qbeg + QS - 1) / QS : 0;
  auto issue = [&](int t, char* st) {
    const int qt0 = qbeg + t * QS;
    im.issue(rq, st, a.ldq, qt0, qend, a.Dv, wave);
    im.issue(rg, st + TB, a.lddo, qt0, qend, a.Dv, wave);
    if (lane < RPW) {   // QS records of 16 B; wave w moves records RPW w .. RPW w + RPW - 1
      const int qr = qt0 + RPW * wave + lane;
      const unsigned off = qr < qend ? (unsigned)qr * 16u : OFF_INVALID;
      dma16(rp, st + 2 * TB + 16 * RPW * wave, off);
    }
  };

  bf16x8 kf[D / 16], vf[D / 16];
  load_row_frags<D>(kf, a.k + b * a.bsk + hh * a.Dv, a.ldk, k0, a.Nk, a.Dv);
  load_row_frags<D>(vf, a.v + b * a.bsv + hh * a.Dv, a.ldv, k0, a.Nk, a.Dv);
#pragma unroll
  for (int s = 0; s < NS - 1; ++s)
    if (s < ntiles) issue(s, smem + s * STG);
#pragma unroll
  for (int s = 0; s < D / 16; ++s) { consume(kf[s]); consume(vf[s]); }
  const float c = a.scale * LOG2E;

  float16v dK[D / 32], dV[D / 32];
#pragma unroll
  for (int t = 0; t < D / 32; ++t) { dK[t] = zero16(); dV[t] = zero16(); }

  // the bias k-step's B operands: ones in k slots 0..2 (S) / 3..5 (dP) of the lower lane half, zero elsewhere
  bf16x8 ones_s, ones_d;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    ones_s[j] = (__bf16)((h == 0 && j < 3) ? 1.f : 0.f);
    ones_d[j] = (__bf16)((h == 0 && j >= 3 && j < 6) ? 1.f : 0.f);
  }
  // S' = Q K^T - lse/c and dP' = dO V^T - delta of the 32-query sub-tile at row u0 of the stage (key on the lane)
  auto sdp = [&](float16v& S_, float16v& dP_, const char* st, int u0) {
    const bf16x8 rec = *reinterpret_cast<const bf16x8*>(st + 2 * TB + (u0 + r) * 16);   // this lane's query
    S_ = mfma32(rec, ones_s, zero16());
    dP_ = mfma32(rec, ones_d, zero16());
#pragma unroll
    for (int s = 0; s < D / 16; ++s) {
      S_ = mfma32(dof.rowf(st, u0, s), kf[s], S_);
      dP_ = mfma32(dof.rowf(st + TB, u0, s), vf[s], dP_);
    }
  };
  // P = exp2(S' c), dS = P dP', packed as the dV / dK B operands
  auto softmax_pack = [&](float16v& S, float16v& dP, bf16x8 (&pk)[4]) {
    if constexpr (D == 64) {
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const float p = __builtin_amdgcn_exp2f(S[i] * c);
        dP[i] = p * dP[i];
        S[i] = p;
      }
    } else {   // packed (see exp2_scaled_pk)
      const f2v c2 = {c, c};
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        f2v x = {S[2 * k], S[2 * k + 1]};
        x = x * c2;
        const f2v p = {__builtin_amdgcn_exp2f(x.x), __builtin_amdgcn_exp2f(x.y)};
        f2v d = {dP[2 * k], dP[2 * k + 1]};
        d = p * d;
        S[2 * k] = p.x;
        S[2 * k + 1] = p.y;
        dP[2 * k] = d.x;
        dP[2 * k + 1] = d.y;
      }
    }
    pk[0] = pack_acc(S, 0);
    pk[1] = pack_acc(S, 1);
    pk[2] = pack_acc(dP, 0);
    pk[3] = pack_acc(dP, 1);
  };
  // dV^T += dO^T P, dK^T += Q^T dS
  auto dvdk = [&](const char* st, int u0, const bf16x8 (&pk)[4]) {
#pragma unroll
    for (int dt = 0; dt < D / 32; ++dt) {
      dV[dt] = mfma32(dof.trf(st + TB, u0, 0, dt), pk[0], dV[dt]);
      dV[dt] = mfma32(dof.trf(st + TB, u0, 1, dt), pk[1], dV[dt]);
      dK[dt] = mfma32(dof.trf(st, u0, 0, dt), pk[2], dK[dt]);
      dK[dt] = mfma32(dof.trf(st, u0, 1, dt), pk[3], dK[dt]);
    }
  };

  auto step = [&](int t, auto si_tag) {
    const int SI = si_tag;   // t % NS (a compile-time constant when unrolled)
    if (t + NS - 2 < ntiles) wait_vmcnt<(NS - 2) * LOADS>();
    else wait_vmcnt<0>();
    BARRIER_LDS();   // WAR: this wave's reads of the slot refilled next have retired
    if (t + NS - 1 < ntiles) issue(t + NS - 1, smem + ((SI + NS - 1) % NS) * STG);
    const char* st = smem + SI * STG;
#pragma unroll 1
    for (int u = 0; u < QS / 32; ++u) {
      if (u > 0 && qbeg + t * QS + 32 * u >= qend) break;   // a wholly padded sub-tile of the last stage
      float16v S, dP;
      bf16x8 pk[4];
      sdp(S, dP, st, 32 * u);
      softmax_pack(S, dP, pk);
      dvdk(st, 32 * u, pk);
    }
  };
  stage_loop<NS, (D <= 64 && OCC < 3)>(ntiles, step);
  const int key = k0 + r;
  if (key < a.Nk) {
#pragma unroll
    for (int dt = 0; dt < D / 32; ++dt)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int d = dt * 32 + 8 * g + 4 * h;
        if (d >= a.Dv) continue;
        if (a.qsplit > 1) {   // this split's fp32 slab [qsplit][B][Nk][H][Dv]; summed by attn_dkv_cast
          const long long base = ((((long long)split * a.B + b) * a.Nk + key) * a.H + hh) * a.Dv + d;
          *reinterpret_cast<float4*>(a.dk32 + base) =
              make_float4(dK[dt][4 * g] * a.scale, dK[dt][4 * g + 1] * a.scale, dK[dt][4 * g + 2] * a.scale,
                          dK[dt][4 * g + 3] * a.scale);
          *reinterpret_cast<float4*>(a.dv32 + base) =
              make_float4(dV[dt][4 * g], dV[dt][4 * g + 1], dV[dt][4 * g + 2], dV[dt][4 * g + 3]);
        }
      }
  }
  if (a.qsplit == 1) {
    bf16_t* kp = a.dk + b * a.bsdk + (long long)min(key, a.Nk - 1) * a.lddk + hh * a.Dv;
    bf16_t* vp = a.dv + b * a.bsdv + (long long)min(key, a.Nk - 1) * a.lddv + hh * a.Dv;
#pragma unroll
    for (int dt = 0; dt < D / 32; ++dt) {
      store_tile_bf16(kp, dt * 32, dK[dt], a.scale, a.Dv, key < a.Nk);
      store_tile_bf16(vp, dt * 32, dV[dt], 1.f, a.Dv, key < a.Nk);
    }
  }
}

// Cross-attention backward (Nk <= 128 keys, head dim <= 64: SDXL / SD 1.5 attn2 over the 77 text tokens), one
// pass instead of the dQ + dK/dV pair (which recompute S and dP, stream Q / dO twice and need a query split for
// dK/dV parallelism over one key block).  Workgroup = (query chunk, head, batch), 4 waves; wave w owns keys
// 32w .. 32w+31: their K / V row fragments stay in registers and their dK^T / dV^T accumulators sum over the
// chunk's queries.  The chunk is walked in rounds of 64 queries, staged by LDS-DMA (dual-use Q and dO images, the O
// row image).  A round:
//   delta = rowsum(dO o O) of its 64 queries from the O / dO images (4 lanes per query) -> {lse, delta} table;
//   S = Q K^T, dP = dO V^T with the key on the lane (row reads of the dual-use Q / dO images); P = exp2(S c - lse),
//   dS = P (dP - delta) feed
//   dV^T += dO^T P and dK^T += Q^T dS as MFMA B operands; dS^T (bf16) -> an LDS [key][query] image;
//   dQ^T = K^T dS^T: one (32 d x 32 q) tile per wave over the active keys (stored at the next round's start).
// 5 MFMA products per (query, key) tile instead of 7.  dK / dV: bf16 directly with one chunk, else fp32 per-chunk
// slabs [chunk][B][Nk][H][Dv] summed in chunk order by attn_dkv_cast_kernel (deterministic).
constexpr int XQR = 64;   // queries per round
constexpr int XIMG = XQR * 64 * 2;                      // one [64 x 64] bf16 image
constexpr int X_KTR = 0;                                // K transposed-read image, 128 keys (16 KiB)
constexpr int X_QIMG = 16384, X_GIMG = X_QIMG + XIMG;  // dual-use Q / dO images (row AND transposed reads)
constexpr int X_OROW = X_GIMG + XIMG;                   // O row image (delta)
constexpr int X_DST = X_OROW + XIMG;                    // dS^T image [128 keys][64 queries] (16 KiB)
constexpr int X_PAIRS = X_DST + 16384;                  // 64 {lse, delta}
constexpr int X_LDS = X_PAIRS + XQR * 8;                // 56.5 KiB: two workgroups per CU (189 VGPRs)

__device__ __forceinline__ int cross_per(const AttnArgs& a) {
  return ((a.Nq + a.qsplit - 1) / a.qsplit + XQR - 1) / XQR * XQR;
}

__global__ void __launch_bounds__(256, 2) attn_bwd_cross_kernel(AttnArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int D = 64;
  using QImg = DmaImg<D, XQR, IMG_DUAL>;
  using RImg = DmaImg<D, XQR, IMG_ROW>;
  using KImg = DmaImg<D, 128, IMG_TR>;
  int chunk, hh, b;
  block_ids(a, chunk, hh, b);
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int r = lane & 31, h = lane >> 5;
  const int nkt = (a.Nk + 31) / 32;                     // key tiles = active waves
  const int per = cross_per(a);
  const int qbeg = chunk * per, qend = min(a.Nq, qbeg + per);
  const int rounds = qend > qbeg ? (qend - qbeg + XQR - 1) / XQR : 0;
  const long long srow = ((long long)b * a.H + hh) * a.Nq;
  const auto rq = rsrc(a.q + b * a.bsq + hh * a.Dv, ((long long)(a.Nq - 1) * a.ldq + a.Dv) * 2);
  const auto rg = rsrc(a.dout + b * a.bsdo + hh * a.Dv, ((long long)(a.Nq - 1) * a.lddo + a.Dv) * 2);
  const auto ro = rsrc(a.o + b * a.bso + hh * a.Dv, ((long long)(a.Nq - 1) * a.ldo + a.Dv) * 2);
  const auto rk = rsrc(a.k + b * a.bsk + hh * a.Dv, ((long long)(a.Nk - 1) * a.ldk + a.Dv) * 2);
  QImg qi;
  RImg ri;
  KImg kti;
  qi.prepare(wave, lane);
  ri.prepare(wave, lane);
  kti.prepare(wave, lane);
  DualOffs<D> dof;
  dof.prepare();
  auto issue = [&](int q0) {   // rows >= qend (the next chunk's, or past Nq) are zero-filled
    qi.issue(rq, smem + X_QIMG, a.ldq, q0, qend, a.Dv, wave);
    qi.issue(rg, smem + X_GIMG, a.lddo, q0, qend, a.Dv, wave);
    ri.issue(ro, smem + X_OROW, a.ldo, q0, qend, a.Dv, wave);
  };
  const int key0 = wave * 32;
  kti.issue(rk, smem + X_KTR, a.ldk, 0, a.Nk, a.Dv, wave);   // rows >= Nk zero: dQ's padded keys add nothing
  if (rounds > 0) issue(qbeg);
  bf16x8 kf[D / 16], vf[D / 16];
  load_row_frags<D>(kf, a.k + b * a.bsk + hh * a.Dv, a.ldk, key0, a.Nk, a.Dv);
  load_row_frags<D>(vf, a.v + b * a.bsv + hh * a.Dv, a.ldv, key0, a.Nk, a.Dv);
  // delta phase: thread t <-> query t >> 2 of the round, head-dim quarter t & 3
  const int dqi = threadIdx.x >> 2, dpart = threadIdx.x & 3;
  float lse_n = (qbeg + dqi < qend) ? a.lse[srow + qbeg + dqi] : INFINITY;   // padded queries: P = 0
#pragma unroll
  for (int s = 0; s < D / 16; ++s) { consume(kf[s]); consume(vf[s]); }
  consume(lse_n);
  const float c = a.scale * LOG2E;

  float16v dK[D / 32], dV[D / 32], dQ = zero16();
#pragma unroll
  for (int t = 0; t < D / 32; ++t) { dK[t] = zero16(); dV[t] = zero16(); }
  const int qdt = wave & 1, qqt = wave >> 1;   // this wave's dQ tile: d tile, query tile
  auto store_dq = [&](int q0) {
    const int q = q0 + qqt * 32 + r;
    bf16_t* Dp = a.dq + b * a.bsdq + (long long)min(q, a.Nq - 1) * a.lddq + hh * a.Dv;
    store_tile_bf16(Dp, qdt * 32, dQ, a.scale, a.Dv, q < qend);
  };

  for (int rd = 0; rd < rounds; ++rd) {
    const int q0 = qbeg + rd * XQR;
    wait_vmcnt<0>();   // this round's images (and the previous round's dQ stores)
    BARRIER();
    if (rd > 0) store_dq(q0 - XQR);
    {   // delta of the round's queries from the LDS images (zero columns past Dv, zero rows past qend)
      float dl = 0.f;
#pragma unroll
      for (int c2 = 0; c2 < 2; ++c2) {
        const int ch = 2 * dpart + c2;
        const bf8 ov = *reinterpret_cast<const bf8*>(smem + X_OROW + dqi * 128 + ((ch ^ (dqi & 7)) << 4));
        const bf8 gv = *reinterpret_cast<const bf8*>(smem + X_GIMG + dqi * 128 + ((ch ^ dsw<D>(dqi)) << 4));
        float of[8], gf[8];
        unpack8(ov, of);
        unpack8(gv, gf);
#pragma unroll
        for (int j = 0; j < 8; ++j) dl = fmaf(of[j], gf[j], dl);
      }
      dl += __shfl_xor(dl, 1, 64);
      dl += __shfl_xor(dl, 2, 64);
      if (dpart == 0) reinterpret_cast<float2*>(smem + X_PAIRS)[dqi] = make_float2(lse_n, dl);
    }
    BARRIER_LDS();   // the {lse, delta} table
    if (wave < nkt) {
#pragma unroll
      for (int qt = 0; qt < 2; ++qt) {
        float16v S = zero16(), dP = zero16();
#pragma unroll
        for (int s = 0; s < D / 16; ++s) {
          S = mfma32(dof.rowf(smem + X_QIMG, qt * 32, s), kf[s], S);
          dP = mfma32(dof.rowf(smem + X_GIMG, qt * 32, s), vf[s], dP);
        }
        const float4* pv = reinterpret_cast<const float4*>(smem + X_PAIRS) + qt * 16;   // pairs 2j, 2j+1
#pragma unroll
        for (int g = 0; g < 4; ++g) {      // registers 4g..4g+3 <-> queries qt*32 + 8g + 4h + (0..3)
          const int q4 = 8 * g + 4 * h;
          const float4 p01 = pv[q4 >> 1], p23 = pv[(q4 >> 1) + 1];
#pragma unroll
          for (int e = 0; e < 2; ++e) {
            const float4 pp = e ? p23 : p01;
            const int i0 = 4 * g + 2 * e;
            // padded keys (the lane past Nk: zero K / V fragments) get a finite P <= 1 (the clamp, folded into
            // v_exp_f32's output modifier) and their dS^T meets zero K rows in dQ = K^T dS^T; their dK / dV are
            // never stored -- no per-lane select
            const float p0 = __builtin_amdgcn_fmed3f(__builtin_amdgcn_exp2f(fmaf(S[i0], c, -pp.x)), 0.f, 1.f);
            const float p1 = __builtin_amdgcn_fmed3f(__builtin_amdgcn_exp2f(fmaf(S[i0 + 1], c, -pp.z)), 0.f, 1.f);
            dP[i0] = p0 * (dP[i0] - pp.y);
            dP[i0 + 1] = p1 * (dP[i0 + 1] - pp.w);
            S[i0] = p0;
            S[i0 + 1] = p1;
          }
        }
        const bf16x8 p0 = pack_acc(S, 0), p1 = pack_acc(S, 1), d0 = pack_acc(dP, 0), d1 = pack_acc(dP, 1);
#pragma unroll
        for (int dt = 0; dt < D / 32; ++dt) {
          dV[dt] = mfma32(dof.trf(smem + X_GIMG, qt * 32, 0, dt), p0, dV[dt]);
          dV[dt] = mfma32(dof.trf(smem + X_GIMG, qt * 32, 1, dt), p1, dV[dt]);
          dK[dt] = mfma32(dof.trf(smem + X_QIMG, qt * 32, 0, dt), d0, dK[dt]);
          dK[dt] = mfma32(dof.trf(smem + X_QIMG, qt * 32, 1, dt), d1, dK[dt]);
        }
        // dS^T -> the [key][query] transposed-read image: registers 4g..4g+3 are 4 consecutive queries
        const uint4 w0 = __builtin_bit_cast(uint4, d0), w1 = __builtin_bit_cast(uint4, d1);
        char* dst = smem + X_DST;
        const int kr = key0 + r, qc = qt * 32 + 4 * h;
        *reinterpret_cast<uint2*>(dst + tr_off<D>(kr, qc)) = make_uint2(w0.x, w0.y);
        *reinterpret_cast<uint2*>(dst + tr_off<D>(kr, qc + 8)) = make_uint2(w0.z, w0.w);
        *reinterpret_cast<uint2*>(dst + tr_off<D>(kr, qc + 16)) = make_uint2(w1.x, w1.y);
        *reinterpret_cast<uint2*>(dst + tr_off<D>(kr, qc + 24)) = make_uint2(w1.z, w1.w);
      }
    }
    BARRIER_LDS();   // dS^T complete; the Q / dO / O images are free
    if (rd + 1 < rounds) {
      issue(q0 + XQR);
      lse_n = (q0 + XQR + dqi < qend) ? a.lse[srow + q0 + XQR + dqi] : INFINITY;
    }
    dQ = zero16();
    for (int kt = 0; kt < nkt; ++kt) {
#pragma unroll
      for (int s = 0; s < 2; ++s)
        dQ = mfma32(tr_frag<D>(smem + X_KTR, kt * 32, s, qdt * 32), tr_frag<D>(smem + X_DST, kt * 32, s, qqt * 32), dQ);
    }
  }
  if (rounds > 0) store_dq(qbeg + (rounds - 1) * XQR);
  wait_vmcnt<0>();   // no LDS-DMA may outlive the workgroup (rounds == 0: the K image)
  if (wave >= nkt) return;
  const int key = key0 + r;
  if (a.qsplit > 1) {   // this chunk's fp32 slab [qsplit][B][Nk][H][Dv]; summed by attn_dkv_cast
    if (key < a.Nk) {
#pragma unroll
      for (int dt = 0; dt < D / 32; ++dt)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int d = dt * 32 + 8 * g + 4 * h;
          if (d >= a.Dv) continue;
          const long long base = ((((long long)chunk * a.B + b) * a.Nk + key) * a.H + hh) * a.Dv + d;
          *reinterpret_cast<float4*>(a.dk32 + base) =
              make_float4(dK[dt][4 * g] * a.scale, dK[dt][4 * g + 1] * a.scale, dK[dt][4 * g + 2] * a.scale,
                          dK[dt][4 * g + 3] * a.scale);
          *reinterpret_cast<float4*>(a.dv32 + base) =
              make_float4(dV[dt][4 * g], dV[dt][4 * g + 1], dV[dt][4 * g + 2], dV[dt][4 * g + 3]);
        }
    }
  } else {
    bf16_t* kp = a.dk + b * a.bsdk + (long long)min(key, a.Nk - 1) * a.lddk + hh * a.Dv;
    bf16_t* vp = a.dv + b * a.bsdv + (long long)min(key, a.Nk - 1) * a.lddv + hh * a.Dv;
#pragma unroll
    for (int dt = 0; dt < D / 32; ++dt) {
      store_tile_bf16(kp, dt * 32, dK[dt], a.scale, a.Dv, key < a.Nk);
      store_tile_bf16(vp, dt * 32, dV[dt], 1.f, a.Dv, key < a.Nk);
    }
  }
}

// sum the qsplit fp32 slabs [qsplit][B, Nk, H, Dv] -> bf16 dK / dV with their strides (4 elements
// per thread; Dv % 8 == 0).  Deterministic: fixed summation order over the splits.  The split loop is
// unrolled by 4 so each thread has 8 loads in flight (a dependent load per split made the launch latency-bound).
__global__ void attn_dkv_cast_kernel(AttnArgs a) {
  const long long total4 = (long long)a.B * a.Nk * a.H * a.Dv / 4;
  const long long slab = total4 * 4;
  for (long long i4 = blockIdx.x * (long long)blockDim.x + threadIdx.x; i4 < total4; i4 += (long long)gridDim.x * blockDim.x) {
    const long long i = i4 * 4;
    float4 sk = make_float4(0.f, 0.f, 0.f, 0.f), sv = sk;
    int s = 0;
    for (; s + 4 <= a.qsplit; s += 4) {
      float4 k[4], v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        k[u] = *reinterpret_cast<const float4*>(a.dk32 + (s + u) * slab + i);
        v[u] = *reinterpret_cast<const float4*>(a.dv32 + (s + u) * slab + i);
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        sk.x += k[u].x; sk.y += k[u].y; sk.z += k[u].z; sk.w += k[u].w;
        sv.x += v[u].x; sv.y += v[u].y; sv.z += v[u].z; sv.w += v[u].w;
      }
    }
    for (; s < a.qsplit; ++s) {
      const float4 k = *reinterpret_cast<const float4*>(a.dk32 + s * slab + i);
      const float4 v = *reinterpret_cast<const float4*>(a.dv32 + s * slab + i);
      sk.x += k.x; sk.y += k.y; sk.z += k.z; sk.w += k.w;
      sv.x += v.x; sv.y += v.y; sv.z += v.z; sv.w += v.w;
    }
    const int d = (int)(i % a.Dv);
    long long t = i / a.Dv;
    const int hh = (int)(t % a.H);
    t /= a.H;
    const int key = (int)(t % a.Nk), b = (int)(t / a.Nk);
    uint2 wk, wv;
    wk.x = (uint32_t)f2bf(sk.x) | ((uint32_t)f2bf(sk.y) << 16);
    wk.y = (uint32_t)f2bf(sk.z) | ((uint32_t)f2bf(sk.w) << 16);
    wv.x = (uint32_t)f2bf(sv.x) | ((uint32_t)f2bf(sv.y) << 16);
    wv.y = (uint32_t)f2bf(sv.z) | ((uint32_t)f2bf(sv.w) << 16);
    *reinterpret_cast<uint2*>(a.dk + b * a.bsdk + (long long)key * a.lddk + hh * a.Dv + d) = wk;
    *reinterpret_cast<uint2*>(a.dv + b * a.bsdv + (long long)key * a.lddv + hh * a.Dv + d) = wv;
  }
}

static bool getenv_flag(const char* name) {
  const char* v = std::getenv(name);
  return v && v[0] && v[0] != '0';
}

// the per-(batch, head) DMA descriptors address rows with 31-bit byte offsets
static bool fits31(int rows, long long ld) { return ((long long)rows * ld + 128) * 2 < 0x7fff0000LL; }

static bool attn_ok(const AttnArgs& a) {
  if (a.B <= 0 || a.H <= 0 || a.Nq <= 0 || a.Nk <= 0 || a.Dv <= 0 || a.Dv % 8 || a.Dv > 128) return false;
  const long long lds[] = {a.ldq, a.ldk, a.ldv, a.bsq, a.bsk, a.bsv};
  for (long long v : lds) if (v % 8) return false;
  if (((uintptr_t)a.q | (uintptr_t)a.k | (uintptr_t)a.v) & 15) return false;
  if (!fits31(a.Nq, a.ldq) || !fits31(a.Nk, a.ldk) || !fits31(a.Nk, a.ldv)) return false;
  return true;
}

// OTAMD_ATTN_XCD=0: hardware block order (the A/B reference)
static int xcd_order() {
  static const int on = [] {
    const char* v = std::getenv("OTAMD_ATTN_XCD");
    return (v && v[0] == '0') ? 0 : 1;
  }();
  return on;
}

template <typename K>
static void launch(K kern, dim3 grid, int lds, hipStream_t s, AttnArgs a) {
  a.xcd = xcd_order();
  {   // LDS opt-in once per kernel instance (its LDS size is fixed by the template)
    static std::mutex mu;
    static std::unordered_set<const void*> done;
    std::lock_guard<std::mutex> lk(mu);
    if (done.insert((const void*)kern).second)
      (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
  }
  hipLaunchKernelGGL(kern, grid, dim3(256), lds, s, a);
}

// one-pass cross-attention backward (attn_bwd_cross_kernel): short key sets at head dim <= 64
// (OTAMD_ATTN_CROSS_OFF=1: the dQ + dK/dV pair for every shape, the A/B reference)
static bool attn_cross_path(const AttnArgs& a) {
  static const bool off = getenv_flag("OTAMD_ATTN_CROSS_OFF");
  return a.Nk <= 128 && a.Dv <= 64 && !off;
}

// query chunks of the one-pass cross backward: ~2 workgroups per CU over (chunk, head, batch), 64-query rounds,
// at most 16 rounds (1024 queries) per chunk; the kernel recomputes the chunk length from the count (cross_per)
static int cross_chunks(const AttnArgs& a) {
  const int bh = a.B * a.H;
  const int target = std::max(1, (512 + bh - 1) / bh);
  int per = ((a.Nq + target - 1) / target + XQR - 1) / XQR * XQR;
  per = std::min(std::max(per, XQR), 16 * XQR);
  return (a.Nq + per - 1) / per;
}

OTAMD_API int otamd_attn_fwd(const AttnArgs* in, hipStream_t stream) {
  if (!in || !attn_ok(*in) || !in->o || !in->lse) return OTAMD_EINVAL;
  AttnArgs a = *in;
  if (a.ldo % 8 || a.bso % 8 || ((uintptr_t)a.o & 15)) return OTAMD_EINVAL;   // 16-byte row stores
  dim3 grid((a.Nq + 127) / 128, a.H, a.B);
  if (a.Dv <= 64) launch(attn_fwd_kernel<64, 2>, grid, 2 * 2 * KT * 64 * 2, stream, a);   // 4 waves/SIMD: 279 vs 288 us
  else launch(attn_fwd_kernel<128, 2>, grid, 2 * 2 * KT * 128 * 2, stream, a);   // 369 vs 512 us (NS = 3), Flux 2381 tokens
  OTAMD_CHECK_LAUNCH();
  return OTAMD_OK;
}

// dK/dV query split of the dQ + dK/dV pair (cross = false) or the chunk count of the one-pass cross kernel
static int attn_qsplit(const AttnArgs& a, bool cross) {
  if (cross) return cross_chunks(a);
  const int kblocks = (a.Nk + 127) / 128;
  int qsplit = 1;
  while (kblocks * a.H * a.B * qsplit < 512 && qsplit < 64 && (a.Nq / (qsplit * 2)) >= 128) qsplit *= 2;
  return qsplit;
}

static long long attn_ws_bytes(const AttnArgs* in, bool cross) {
  if (!in || in->B <= 0 || in->H <= 0 || in->Nq <= 0 || in->Nk <= 0 || in->Dv <= 0) return -1;
  const long long nrow = (long long)in->B * in->H * in->Nq;
  const long long nkv = (long long)in->B * in->Nk * in->H * in->Dv;
  const int qs = attn_qsplit(*in, cross);
  return nrow * 16 + 256 + (qs > 1 ? 2LL * qs * nkv * 4 : 0);
}

// workspace bytes otamd_attn_bwd needs: 16-byte bias records per query + (split queries) fp32 dK/dV partials
OTAMD_API long long otamd_attn_bwd_ws_bytes(const AttnArgs* in) { return in ? attn_ws_bytes(in, attn_cross_path(*in)) : -1; }

// bytes of the fp32 dK / dV partial slabs alone (0: these arguments need none) -- the caller-owned `slabs` buffer of
// otamd_attn_bwd_ex
OTAMD_API long long otamd_attn_bwd_slab_bytes(const AttnArgs* in) {
  if (!in || in->B <= 0 || in->H <= 0 || in->Nq <= 0 || in->Nk <= 0 || in->Dv <= 0) return -1;
  const int qs = attn_qsplit(*in, attn_cross_path(*in));
  return qs > 1 ? 2LL * qs * ((long long)in->B * in->Nk * in->H * in->Dv) * 4 : 0;
}

static int attn_bwd_impl(const AttnArgs* in, float* ws, long long ws_bytes, float* slabs, long long slab_bytes,
                         hipStream_t stream, hipStream_t cast_stream);

// ws: otamd_attn_bwd_ws_bytes(args) bytes, 16-byte aligned; lse from the forward
OTAMD_API int otamd_attn_bwd(const AttnArgs* in, float* ws, long long ws_bytes, hipStream_t stream) {
  return attn_bwd_impl(in, ws, ws_bytes, nullptr, 0, stream, stream);
}

// As otamd_attn_bwd, with the dK / dV partial slabs in the caller's buffer (otamd_attn_bwd_slab_bytes; ws then needs
// only the bias records: otamd_attn_bwd_ws_bytes minus the slab bytes) and their chunk-order sum (the cast kernel)
// on cast_stream, ordered after the main kernels by an event.  For the one-pass cross-attention backward whose dK /
// dV feed only the K / V projections' weight gradients (module/functional.py CrossAttnFn): the cast leaves the
// critical stream.  The caller keeps slabs, dk and dv alive until cast_stream has consumed them.
OTAMD_API int otamd_attn_bwd_ex(const AttnArgs* in, float* ws, long long ws_bytes, float* slabs, long long slab_bytes,
                                hipStream_t stream, hipStream_t cast_stream) {
  if (!slabs || ((uintptr_t)slabs & 15)) return OTAMD_EINVAL;
  return attn_bwd_impl(in, ws, ws_bytes, slabs, slab_bytes, stream, cast_stream);
}

static int attn_bwd_impl(const AttnArgs* in, float* ws, long long ws_bytes, float* slabs, long long slab_bytes,
                         hipStream_t stream, hipStream_t cast_stream) {
  if (!in || !attn_ok(*in) || !in->o || !in->lse || !in->dout || !in->dq || !in->dk || !in->dv || !ws) return OTAMD_EINVAL;
  AttnArgs a = *in;
  if (a.lddo % 8 || a.bsdo % 8 || a.lddq % 8 || a.lddk % 8 || a.lddv % 8 || a.bsdq % 8 || a.bsdk % 8 || a.bsdv % 8 ||
      (((uintptr_t)ws | (uintptr_t)a.dq | (uintptr_t)a.dk | (uintptr_t)a.dv) & 15))
    return OTAMD_EINVAL;   // 16-byte row stores
  if (((uintptr_t)a.dout & 15) || !fits31(a.Nq, a.lddo)) return OTAMD_EINVAL;
  const bool cross = attn_cross_path(a);
  const long long nrow = (long long)a.B * a.H * a.Nq;
  const long long nkv = (long long)a.B * a.Nk * a.H * a.Dv;
  const int qsplit = attn_qsplit(a, cross);
  a.qsplit = qsplit;
  const long long slab_need = qsplit > 1 ? 2LL * qsplit * nkv * 4 : 0;
  if (slabs) {
    if (ws_bytes < attn_ws_bytes(in, cross) - slab_need || slab_bytes < slab_need) return OTAMD_EINVAL;
  } else if (ws_bytes < attn_ws_bytes(in, cross)) {
    return OTAMD_EINVAL;
  }
  a.delta = ws;   // bias records: written by the dQ kernel, read by dK/dV
  if (qsplit > 1) {   // every slab element is written by exactly one block: no memset
    a.dk32 = slabs ? slabs : ws + ((nrow * 4 + 64) / 64) * 64;
    a.dv32 = a.dk32 + (long long)qsplit * nkv;
  }
  const int kblocks = (a.Nk + 127) / 128;
  dim3 gq((a.Nq + 127) / 128, a.H, a.B);
  dim3 gk(kblocks, a.H, a.B * qsplit);
  if (cross) {
    launch(attn_bwd_cross_kernel, dim3(qsplit, a.H, a.B), X_LDS, stream, a);
  } else if (a.Dv <= 64) {
    launch(attn_bwd_dq_kernel<64, 3>, gq, 3 * 2 * KT * 64 * 2, stream, a);
    launch(attn_bwd_dkv_kernel<64, 3, 64>, gk, dkv_lds<64, 64>(), stream, a);
  } else {
    // 64-key tiles 2 deep: 1086 vs 1104 us for 32-key tiles 3 deep (Flux 4x2381x24, round 4, same box)
    launch(attn_bwd_dq_kernel<128, 2, 64>, gq, 2 * 2 * 64 * 128 * 2, stream, a);
    launch(attn_bwd_dkv_kernel<128, 1, 64>, gk, dkv_lds<128, 64>(), stream, a);
  }
  OTAMD_CHECK_LAUNCH();
  if (qsplit > 1) {
    hipStream_t cs = stream;
    if (slabs && cast_stream != stream) {   // the sum after the slabs' producer, on the other stream
      // one fork event per (thread, device): an event records only on streams of the device it was created on
      thread_local hipEvent_t evs[64] = {};
      int dev = 0;
      if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return OTAMD_ELAUNCH;
      hipEvent_t& ev = evs[dev];
      if (!ev && hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess) return OTAMD_ELAUNCH;
      if (hipEventRecord(ev, stream) != hipSuccess || hipStreamWaitEvent(cast_stream, ev, 0) != hipSuccess)
        return OTAMD_ELAUNCH;
      cs = cast_stream;
    }
    int blocks = (int)std::min<long long>((nkv / 4 + 255) / 256, 8192);
    attn_dkv_cast_kernel<<<blocks, 256, 0, cs>>>(a);
    OTAMD_CHECK_LAUNCH();
  }
  return OTAMD_OK;
}

OTAMD_API int otamd_attn_args_size(void) { return (int)sizeof(AttnArgs); }
