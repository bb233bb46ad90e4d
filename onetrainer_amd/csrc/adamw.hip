// Fused AdamW + bf16 stochastic rounding and global grad-norm clipping over a
// flat parameter store.  Replaces, per parameter tensor, the reference's
//   modules/util/optimizer/adamw_extensions.py:17-150  (step_adamw_parameter)
//   modules/util/bf16_stochastic_rounding.py:5-61     (copy/addcdiv_stochastic_)
//   torch.nn.utils.clip_grad_norm_ called at modules/trainer/GenericTrainer.py:712-713
// with ONE launch over the whole flat buffer (the reference runs ~8 torch ops per
// tensor per step in a Python loop).
//
// Numerics: every torch op of the reference's bf16 path rounds its result to bf16;
// this kernel applies the same roundings in the same order, with the same fused
// multiply-adds torch's CPU kernels use (lerp and addcmul are fma; pinned in
// tests/test_oracle_golden.py).  Compile with -ffp-contract=off so no other
// contraction is introduced.
//
// HBM traffic per bf16 element: read p,g,m,v (8 B) + write p,m,v (6 B) = 14 B.
#include "common.h"

#include <algorithm>
#include <cstdlib>

#define ADAMW_MAX_GROUPS 8

struct AdamwGroup {
  long long begin, end;     // element range [begin, end) of this group in the flat store
  float wd_factor;          // 1 - lr * weight_decay           (p.mul_)
  float one_minus_beta1;    // lerp weight                      (exp_avg.lerp_)
  float beta2;              // exp_avg_sq.mul_(beta2)
  float one_minus_beta2;    // addcmul value
  float bc2_sqrt;           // sqrt(1 - beta2^step)
  float eps;
  float neg_step_size;      // -lr / (1 - beta1^step)
  float pad;
};
struct AdamwGroups {
  AdamwGroup g[ADAMW_MAX_GROUPS];
  int n;
};

// counter-based 32-bit mixer (multiply-xorshift, 3 integer multiplies: the 64-bit splitmix it
// replaces cost ~50 quarter-rate multiplies per 8 elements); the high 16 bits are the SR dither.
// Restated bit-for-bit in oracle/adamw.py (sr_bits).
__device__ __forceinline__ uint32_t sr_bits(uint32_t k, uint64_t idx) {
  uint32_t x = (uint32_t)idx * 0x9E3779B1u + k;
  x ^= (uint32_t)(idx >> 32) * 0x85EBCA77u;
  x ^= x >> 16;
  x *= 0x21F0AAADu;
  x ^= x >> 15;
  x *= 0x735A2D97u;
  x ^= x >> 15;
  return x >> 16;
}

// bias-corrected Adam denominator of one (new) exp_avg_sq value, rounded like the reference's
// torch ops: exp_avg_sq.sqrt() / bias_correction2_sqrt .add_(eps), each result bf16
__device__ __forceinline__ float adam_denom_bf16(float v, const AdamwGroup& G) {
  float d = rbf(sqrtf(v));                             // exp_avg_sq.sqrt()
  d = rbf(d / G.bc2_sqrt);                             //   / bias_correction2_sqrt
  return rbf(d + G.eps);                               //   .add_(eps)
}

// The denominator is a function of the bf16 exp_avg_sq alone (per step: bc2_sqrt and eps are
// step constants), so the LUT kernel tabulates it once per workgroup in LDS for every
// non-negative bf16 bit pattern (32768 entries, 64 KiB) with the very same adam_denom_bf16:
// the per-element sqrt + 2 IEEE-divide chain (~40% of the kernel's VALU work, which made the
// plain kernel VALU- rather than HBM-bound) becomes one ds_read_u16.  Patterns with the sign
// bit set (-0.0, NaN) keep the computed path, so results are bit-identical by construction.
#define ADAMW_LUT_ENTRIES 32768

// one element of the bf16 path (p, g, m, v all bf16 in HBM); lut: LDS denominator table or null
__device__ __forceinline__ void adamw_elem_bf16(float& p, float g, float& m, float& v,
                                                const AdamwGroup& G, float coef, bool clip,
                                                bool sr, uint32_t seed, uint64_t idx,
                                                const unsigned short* lut = nullptr) {
  if (clip) g = rbf(g * coef);                         // torch._foreach_mul_(grads, clip_coef)
  p = rbf(p * G.wd_factor);                            // p.mul_(1 - lr*wd)
  m = rbf(fmaf(G.one_minus_beta1, g - m, m));          // exp_avg.lerp_(grad, 1-beta1)
  v = rbf(v * G.beta2);                                // exp_avg_sq.mul_(beta2)
  v = rbf(fmaf(G.one_minus_beta2 * g, g, v));          //   .addcmul_(grad, grad, 1-beta2)
  float d;
  if (lut) {
    const uint32_t vb = __float_as_uint(v) >> 16;      // v is bf16-exact after rbf
    d = vb < ADAMW_LUT_ENTRIES ? __uint_as_float((uint32_t)lut[vb] << 16) : adam_denom_bf16(v, G);
  } else {
    d = adam_denom_bf16(v, G);
  }
  const float r = p + (G.neg_step_size * m) / d;       // fp32 addcdiv on the fp32 copy
  if (sr) {                                            // copy_stochastic_
    uint32_t u = __float_as_uint(r);
    u = (u + sr_bits(seed, idx)) & 0xFFFF0000u;
    p = __uint_as_float(u);
  } else {
    p = rbf(r);                                        // p.addcdiv_ on bf16 p
  }
}

__device__ __forceinline__ int find_group(const AdamwGroups& G, long long e) {
  int gi = 0;
#pragma unroll
  for (int i = 1; i < ADAMW_MAX_GROUPS; ++i)
    if (i < G.n && e >= G.g[i].begin) gi = i;
  return gi;
}

// flat bf16 store; n multiple of 8 (the store pads every tensor to 8 elements)
__global__ void __launch_bounds__(256) adamw_bf16_kernel(bf16_t* __restrict__ P, const bf16_t* __restrict__ Gr,
                                                         bf16_t* __restrict__ M, bf16_t* __restrict__ V, long long v0,
                                                         long long n8, AdamwGroups groups,
                                                         const float* __restrict__ clip_coef, int sr,
                                                         unsigned long long seed) {
  const bool clip = clip_coef != nullptr;
  const float coef = clip ? clip_coef[0] : 1.f;
  const uint32_t k = (uint32_t)(seed ^ (seed >> 32));
  const long long stride = (long long)gridDim.x * blockDim.x;
  long long i = v0 + blockIdx.x * (long long)blockDim.x + threadIdx.x;
  // software pipeline: the next granule's four loads are in flight while this one is computed
  bf8 pv, gv, mv, vv;
  if (i < n8) {
    pv = reinterpret_cast<const bf8*>(P)[i]; gv = reinterpret_cast<const bf8*>(Gr)[i];
    mv = reinterpret_cast<const bf8*>(M)[i]; vv = reinterpret_cast<const bf8*>(V)[i];
  }
  for (; i < n8; i += stride) {
    const long long in = i + stride;
    bf8 pn, gn, mn, vn;
    if (in < n8) {
      pn = reinterpret_cast<const bf8*>(P)[in]; gn = reinterpret_cast<const bf8*>(Gr)[in];
      mn = reinterpret_cast<const bf8*>(M)[in]; vn = reinterpret_cast<const bf8*>(V)[in];
    }
    const long long e0 = i * 8;
    const int gi = find_group(groups, e0);
    const AdamwGroup& G = groups.g[gi];
    if (e0 < G.end) {  // else: padding tail beyond the last group
      float p[8], g[8], m[8], v[8];
      unpack8(pv, p); unpack8(gv, g); unpack8(mv, m); unpack8(vv, v);
#pragma unroll
      for (int j = 0; j < 8; ++j) adamw_elem_bf16(p[j], g[j], m[j], v[j], G, coef, clip, sr != 0, k, (uint64_t)(e0 + j));
      reinterpret_cast<bf8*>(P)[i] = pack8(p);
      reinterpret_cast<bf8*>(M)[i] = pack8(m);
      reinterpret_cast<bf8*>(V)[i] = pack8(v);
    }
    pv = pn; gv = gn; mv = mn; vv = vn;
  }
}

// LUT variant: every group shares bc2_sqrt and eps (the host checks), 1024-thread workgroups,
// two per CU (64 KiB of LDS each)
// streaming 16-byte accesses; NT: non-temporal (the store is touched once per step, 36 GB for SDXL)
template <bool NT>
__device__ __forceinline__ bf8 ldv(const bf16_t* base, long long i) {
  if constexpr (NT) {
    typedef uint32_t u4 __attribute__((ext_vector_type(4)));
    const u4 x = __builtin_nontemporal_load(reinterpret_cast<const u4*>(base) + i);
    bf8 r; r.w[0] = x.x; r.w[1] = x.y; r.w[2] = x.z; r.w[3] = x.w;
    return r;
  } else {
    return reinterpret_cast<const bf8*>(base)[i];
  }
}
template <bool NT>
__device__ __forceinline__ void stv(bf16_t* base, long long i, bf8 x) {
  if constexpr (NT) {
    typedef uint32_t u4 __attribute__((ext_vector_type(4)));
    u4 y; y.x = x.w[0]; y.y = x.w[1]; y.z = x.w[2]; y.w = x.w[3];
    __builtin_nontemporal_store(y, reinterpret_cast<u4*>(base) + i);
  } else {
    reinterpret_cast<bf8*>(base)[i] = x;
  }
}

template <bool NT>
__global__ void __launch_bounds__(1024) adamw_bf16_lut_kernel(bf16_t* __restrict__ P, const bf16_t* __restrict__ Gr,
                                                              bf16_t* __restrict__ M, bf16_t* __restrict__ V,
                                                              long long v0, long long n8, AdamwGroups groups,
                                                              const float* __restrict__ clip_coef, int sr,
                                                              unsigned long long seed) {
  __shared__ unsigned short lut[ADAMW_LUT_ENTRIES];
  for (int b = threadIdx.x; b < ADAMW_LUT_ENTRIES; b += 1024)
    lut[b] = f2bf(adam_denom_bf16(__uint_as_float((uint32_t)b << 16), groups.g[0]));
  __syncthreads();
  const bool clip = clip_coef != nullptr;
  const float coef = clip ? clip_coef[0] : 1.f;
  const uint32_t k = (uint32_t)(seed ^ (seed >> 32));
  const long long stride = (long long)gridDim.x * blockDim.x;
  long long i = v0 + blockIdx.x * (long long)blockDim.x + threadIdx.x;
  bf8 pv, gv, mv, vv;
  if (i < n8) {
    pv = ldv<NT>(P, i); gv = ldv<NT>(Gr, i);
    mv = ldv<NT>(M, i); vv = ldv<NT>(V, i);
  }
  for (; i < n8; i += stride) {
    const long long in = i + stride;
    bf8 pn, gn, mn, vn;
    if (in < n8) {
      pn = ldv<NT>(P, in); gn = ldv<NT>(Gr, in);
      mn = ldv<NT>(M, in); vn = ldv<NT>(V, in);
    }
    const long long e0 = i * 8;
    const int gi = find_group(groups, e0);
    const AdamwGroup& G = groups.g[gi];
    if (e0 < G.end) {
      float p[8], g[8], m[8], v[8];
      unpack8(pv, p); unpack8(gv, g); unpack8(mv, m); unpack8(vv, v);
#pragma unroll
      for (int j = 0; j < 8; ++j)
        adamw_elem_bf16(p[j], g[j], m[j], v[j], G, coef, clip, sr != 0, k, (uint64_t)(e0 + j), lut);
      stv<NT>(P, i, pack8(p));
      stv<NT>(M, i, pack8(m));
      stv<NT>(V, i, pack8(v));
    }
    pv = pn; gv = gn; mv = mn; vv = vn;
  }
}

// one element of the fp32 path: every torch op of step_adamw_parameter on fp32 tensors rounds to fp32
// (p.mul_, exp_avg.lerp_ (fma), exp_avg_sq.mul_().addcmul_ (fma), sqrt()/bc2_sqrt .add_(eps), p.addcdiv_);
// the clipped gradient is _foreach_mul_(grads, clip_coef) in fp32.  Restated in oracle/adamw.py adamw_step_f32.
__device__ __forceinline__ void adamw_elem_f32(float& p, float g, float& m, float& v, const AdamwGroup& G, float coef,
                                               bool clip) {
  if (clip) g = g * coef;
  p = p * G.wd_factor;
  m = fmaf(G.one_minus_beta1, g - m, m);
  v = v * G.beta2;
  v = fmaf(G.one_minus_beta2 * g, g, v);
  const float d = sqrtf(v) / G.bc2_sqrt + G.eps;
  p = p + (G.neg_step_size * m) / d;
}

// fp32 store (LoRA weights are fp32 by default, TrainConfig.py:959): plain fp32 torch ops
__global__ void __launch_bounds__(256) adamw_f32_kernel(float* __restrict__ P, const float* __restrict__ Gr,
                                                        float* __restrict__ M, float* __restrict__ V, long long n4,
                                                        AdamwGroups groups, const float* __restrict__ clip_coef) {
  const bool clip = clip_coef != nullptr;
  const float coef = clip ? clip_coef[0] : 1.f;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n4; i += (long long)gridDim.x * blockDim.x) {
    const long long e0 = i * 4;
    const int gi = find_group(groups, e0);
    const AdamwGroup& G = groups.g[gi];
    if (e0 >= G.end) continue;
    float4 pv = reinterpret_cast<const float4*>(P)[i];
    float4 gv = reinterpret_cast<const float4*>(Gr)[i];
    float4 mv = reinterpret_cast<const float4*>(M)[i];
    float4 vv = reinterpret_cast<const float4*>(V)[i];
    float* p = &pv.x; float* g = &gv.x; float* m = &mv.x; float* v = &vv.x;
#pragma unroll
    for (int j = 0; j < 4; ++j) adamw_elem_f32(p[j], g[j], m[j], v[j], G, coef, clip);
    reinterpret_cast<float4*>(P)[i] = pv;
    reinterpret_cast<float4*>(M)[i] = mv;
    reinterpret_cast<float4*>(V)[i] = vv;
  }
}

// fp32 master weights of a full fine-tune (the reference's default weight_dtype FLOAT_32, TrainConfig.py:782, with
// a bf16 train_dtype: autocast runs every GEMM on a bf16 cast of the fp32 weight, and its weight gradient is the bf16
// GEMM result cast back to fp32).  The kernels read a bf16 working copy and write bf16 gradients, so per element:
// read g (bf16) and p, m, v (fp32), the fp32 step above, write p, m, v and the working copy rne(p) -- the
// round-to-nearest cast autocast applies at the next forward.  28 B per element.
struct __align__(16) f8 { float4 a, b; };
__global__ void __launch_bounds__(256) adamw_master_kernel(float* __restrict__ P, const bf16_t* __restrict__ Gr,
                                                           float* __restrict__ M, float* __restrict__ V,
                                                           bf16_t* __restrict__ W, long long v0, long long n8,
                                                           AdamwGroups groups, const float* __restrict__ clip_coef) {
  const bool clip = clip_coef != nullptr;
  const float coef = clip ? clip_coef[0] : 1.f;
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long i = v0 + blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n8; i += stride) {
    const long long e0 = i * 8;
    const int gi = find_group(groups, e0);
    const AdamwGroup& G = groups.g[gi];
    if (e0 >= G.end) continue;
    const bf8 gv = reinterpret_cast<const bf8*>(Gr)[i];
    f8 pv = reinterpret_cast<const f8*>(P)[i];
    f8 mv = reinterpret_cast<const f8*>(M)[i];
    f8 vv = reinterpret_cast<const f8*>(V)[i];
    float g[8];
    unpack8(gv, g);
    float* p = &pv.a.x; float* m = &mv.a.x; float* v = &vv.a.x;
#pragma unroll
    for (int j = 0; j < 8; ++j) adamw_elem_f32(p[j], g[j], m[j], v[j], G, coef, clip);
    reinterpret_cast<f8*>(P)[i] = pv;
    reinterpret_cast<f8*>(M)[i] = mv;
    reinterpret_cast<f8*>(V)[i] = vv;
    reinterpret_cast<bf8*>(W)[i] = pack8(p);
  }
}

// ---- global grad norm ---------------------------------------------------------
// chunk table: for each block, (tensor index, element begin, element end) in the flat store
struct NormChunk { long long begin, end; int tensor; int pad; };

template <typename T>
__device__ __forceinline__ float ld_as_f(const T* p, long long i);
template <> __device__ __forceinline__ float ld_as_f<bf16_t>(const bf16_t* p, long long i) { return bf2f(p[i]); }
template <> __device__ __forceinline__ float ld_as_f<float>(const float* p, long long i) { return p[i]; }

// chunk_sq[blockIdx.x] = the chunk's sum of squares (one slot per chunk: no atomics, so the per-tensor sums below
// add the chunks in a fixed order -- a double atomicAdd per chunk made the sum's last bits, and now and then the
// bf16-rounded clip coefficient, depend on the chunks' arrival order)
template <typename T>
__global__ void __launch_bounds__(256) grad_sqnorm_kernel(const T* __restrict__ G, const NormChunk* __restrict__ chunks,
                                                          double* __restrict__ chunk_sq) {
  const NormChunk c = chunks[blockIdx.x];
  double acc = 0.0;
  long long e = c.begin + threadIdx.x * 8;
  if (sizeof(T) == 2) {
    // four 16-byte loads in flight per lane before the adds (one per iteration left the pass at ~2.1 TB/s in the
    // step); the per-load partials are added in the same order as the one-load loop: the same bits
    for (; e + 3 * 256 * 8 < c.end; e += 4 * 256 * 8) {
      bf8 v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) v[u] = *reinterpret_cast<const bf8*>(G + e + u * 256 * 8);
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        float f[8];
        unpack8(v[u], f);
        float s = 0.f;
#pragma unroll
        for (int j = 0; j < 8; ++j) s = fmaf(f[j], f[j], s);
        acc += s;
      }
    }
  }
  // 16-byte vector body (chunk bounds are multiples of 8 elements)
  for (; e < c.end; e += 256 * 8) {
    if (sizeof(T) == 2) {
      bf8 v = *reinterpret_cast<const bf8*>(G + e);
      float f[8];
      unpack8(v, f);
      float s = 0.f;
#pragma unroll
      for (int j = 0; j < 8; ++j) s = fmaf(f[j], f[j], s);
      acc += s;
    } else {
      float s = 0.f;
#pragma unroll
      for (int j = 0; j < 8; ++j) { float f = ld_as_f<T>(G, e + j); s = fmaf(f, f, s); }
      acc += s;
    }
  }
  __shared__ double red[4];
  acc = wave_sum_d(acc);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) chunk_sq[blockIdx.x] = red[0] + red[1] + red[2] + red[3];
}

// tensor_sq[t] = sum of tensor t's chunk slots in chunk order (the chunk table lists each tensor's chunks
// contiguously, in element order); the thread of a tensor's first chunk walks them.  Tensors without chunks keep
// the zero the caller's memset left.
__global__ void tensor_sq_kernel(const NormChunk* __restrict__ chunks, int n_chunks, const double* __restrict__ chunk_sq,
                                 double* __restrict__ tensor_sq) {
  for (int c = blockIdx.x * blockDim.x + threadIdx.x; c < n_chunks; c += gridDim.x * blockDim.x) {
    const int t = chunks[c].tensor;
    if (c > 0 && chunks[c - 1].tensor == t) continue;
    double s = 0.0;
    for (int k = c; k < n_chunks && chunks[k].tensor == t; ++k) s += chunk_sq[k];
    tensor_sq[t] = s;
  }
}

// total_norm / clip coefficient with torch's bf16 result dtypes:
//   per-tensor norm (bf16) -> stack -> vector_norm (bf16) -> max_norm/(norm+1e-6) (bf16) -> clamp(max=1)
// out[0] = clip coefficient (as float of a bf16 / f32 value), out[1] = total norm
__global__ void clip_coef_kernel(const double* __restrict__ tensor_sq, int n_tensors, float max_norm, int bf16_grads,
                                 float* __restrict__ out) {
  __shared__ float red[16];
  float acc = 0.f;
  for (int i = threadIdx.x; i < n_tensors; i += blockDim.x) {
    float nrm = (float)sqrt(tensor_sq[i]);
    if (bf16_grads) nrm = rbf(nrm);
    acc = fmaf(nrm, nrm, acc);
  }
  const float tot_sq = block_sum(acc, red);
  if (threadIdx.x == 0) {
    float total = sqrtf(tot_sq);
    float coef;
    if (bf16_grads) {
      total = rbf(total);
      const float denom = rbf(total + 1e-6f);
      coef = rbf(max_norm / denom);
      coef = fminf(coef, 1.f);
    } else {
      coef = fminf(max_norm / (total + 1e-6f), 1.f);
    }
    out[0] = coef;
    out[1] = total;
  }
}

// ---- C ABI ----------------------------------------------------------------------
// workgroup cap of the update launches: OTAMD_ADAMW_BLOCKS (default: the whole chip).  An update overlapped with
// the next forward on its own stream (util/optimizer/adamw_fused.py) holds only that many CUs' worth of slots.
static long long adamw_max_blocks(long long dflt) {
  static const long long cap = [] {
    const char* e = getenv("OTAMD_ADAMW_BLOCKS");
    return e ? atoll(e) : 0LL;
  }();
  return cap > 0 ? std::min(cap, dflt) : dflt;
}

static int adamw_grid(long long nvec) {
  long long blocks = (nvec + 255) / 256;
  if (blocks > 256 * 16) blocks = 256 * 16;
  if (blocks < 1) blocks = 1;
  return (int)blocks;
}

OTAMD_API int otamd_adamw_bf16_range(void* p, const void* g, void* m, void* v, long long begin, long long end,
                                     const AdamwGroup* groups, int n_groups, const float* clip_coef,
                                     int stochastic_rounding, unsigned long long seed, hipStream_t stream) {
  if (!p || !g || !m || !v || begin < 0 || end < begin || (begin % 8) != 0 || (end % 8) != 0 || n_groups < 1 ||
      n_groups > ADAMW_MAX_GROUPS)
    return OTAMD_EINVAL;
  if (((uintptr_t)p | (uintptr_t)g | (uintptr_t)m | (uintptr_t)v) & 15) return OTAMD_EINVAL;
  if (end == begin) return OTAMD_OK;
  AdamwGroups G = {};
  for (int i = 0; i < n_groups; ++i) G.g[i] = groups[i];
  G.n = n_groups;
  // LUT kernel when the denominator constants are shared (always, for one optimizer step with common
  // betas/eps) and the range is large enough to amortise the per-workgroup table.  OTAMD_ADAMW_LUT=0
  // forces the computed path, =1 the LUT with cached accesses, =2 the LUT with non-temporal accesses
  // (parity tests compare them) -- never the LUT when the groups' constants differ.
  const long long n = end - begin;
  bool shared = true;
  for (int i = 1; i < n_groups; ++i) shared = shared && G.g[i].bc2_sqrt == G.g[0].bc2_sqrt && G.g[i].eps == G.g[0].eps;
  bool lut = shared && n >= (1LL << 22);
  // (measured on MI355X, 2.567 G elements: computed 7.0 ms, LUT 6.27 ms, LUT + non-temporal 6.10 ms)
  int nt = 1;
  if (const char* e = getenv("OTAMD_ADAMW_LUT")) { lut = shared && e[0] != '0'; nt = e[0] != '1'; }
  const long long v0 = begin / 8, v1 = end / 8;
  if (lut) {
    const int blocks = (int)std::max(1LL, std::min<long long>((v1 - v0 + 1023) / 1024, adamw_max_blocks(512)));
    if (nt)
      adamw_bf16_lut_kernel<true><<<blocks, 1024, 0, stream>>>((bf16_t*)p, (const bf16_t*)g, (bf16_t*)m, (bf16_t*)v, v0,
                                                               v1, G, clip_coef, stochastic_rounding, seed);
    else
      adamw_bf16_lut_kernel<false><<<blocks, 1024, 0, stream>>>((bf16_t*)p, (const bf16_t*)g, (bf16_t*)m, (bf16_t*)v,
                                                                v0, v1, G, clip_coef, stochastic_rounding, seed);
  } else {
    adamw_bf16_kernel<<<adamw_grid(v1 - v0), 256, 0, stream>>>((bf16_t*)p, (const bf16_t*)g, (bf16_t*)m, (bf16_t*)v,
                                                               v0, v1, G, clip_coef, stochastic_rounding, seed);
  }
  OTAMD_CHECK_LAUNCH();
  return OTAMD_OK;
}

OTAMD_API int otamd_adamw_bf16(void* p, const void* g, void* m, void* v, long long n, const AdamwGroup* groups,
                               int n_groups, const float* clip_coef, int stochastic_rounding,
                               unsigned long long seed, hipStream_t stream) {
  if (n < 0 || (n % 8) != 0) return OTAMD_EINVAL;
  return otamd_adamw_bf16_range(p, g, m, v, 0, n, groups, n_groups, clip_coef, stochastic_rounding, seed, stream);
}

OTAMD_API int otamd_adamw_f32(void* p, const void* g, void* m, void* v, long long n, const AdamwGroup* groups,
                              int n_groups, const float* clip_coef, hipStream_t stream) {
  if (!p || !g || !m || !v || n < 0 || (n % 4) != 0 || n_groups < 1 || n_groups > ADAMW_MAX_GROUPS) return OTAMD_EINVAL;
  if (((uintptr_t)p | (uintptr_t)g | (uintptr_t)m | (uintptr_t)v) & 15) return OTAMD_EINVAL;
  if (n == 0) return OTAMD_OK;
  AdamwGroups G = {};
  for (int i = 0; i < n_groups; ++i) G.g[i] = groups[i];
  G.n = n_groups;
  adamw_f32_kernel<<<adamw_grid(n / 4), 256, 0, stream>>>((float*)p, (const float*)g, (float*)m, (float*)v, n / 4, G,
                                                          clip_coef);
  OTAMD_CHECK_LAUNCH();
  return OTAMD_OK;
}

// p32 / m32 / v32: fp32 flat buffers; g16: the bf16 gradient store; w16: the bf16 working copy the kernels read;
// [begin, end): element range (multiples of 8)
OTAMD_API int otamd_adamw_master_range(void* p32, const void* g16, void* m32, void* v32, void* w16, long long begin,
                                       long long end, const AdamwGroup* groups, int n_groups, const float* clip_coef,
                                       hipStream_t stream) {
  if (!p32 || !g16 || !m32 || !v32 || !w16 || begin < 0 || end < begin || (begin % 8) != 0 || (end % 8) != 0 ||
      n_groups < 1 || n_groups > ADAMW_MAX_GROUPS)
    return OTAMD_EINVAL;
  if (((uintptr_t)p32 | (uintptr_t)g16 | (uintptr_t)m32 | (uintptr_t)v32 | (uintptr_t)w16) & 15) return OTAMD_EINVAL;
  if (end == begin) return OTAMD_OK;
  AdamwGroups G = {};
  for (int i = 0; i < n_groups; ++i) G.g[i] = groups[i];
  G.n = n_groups;
  const long long v0 = begin / 8, v1 = end / 8;
  const int blocks = (int)std::max(1LL, std::min<long long>((v1 - v0 + 255) / 256, adamw_max_blocks(256 * 16)));
  adamw_master_kernel<<<blocks, 256, 0, stream>>>((float*)p32, (const bf16_t*)g16, (float*)m32, (float*)v32,
                                                  (bf16_t*)w16, v0, v1, G, clip_coef);
  OTAMD_CHECK_LAUNCH();
  return OTAMD_OK;
}

// grads: flat store, grad_dtype 0 = bf16, 1 = f32, 2 = bf16 storage of an fp32-master network's gradients (the
// reference holds them as fp32 tensors: clip_grad_norm_ forms the norms and the coefficient in fp32);
// chunks: device table of n_chunks NormChunk;
OTAMD_API int otamd_grad_clip_finalize(const void* chunks, int n_chunks, const double* chunk_sq, double* tensor_sq,
                                       int n_tensors, float max_norm, int grad_dtype, float* out, hipStream_t stream);

// chunk_sq: device double[n_chunks] scratch; tensor_sq: device double[n_tensors] (zeroed here); out: device
// float[2] = {clip coef, total norm}
OTAMD_API int otamd_grad_clip_coef(const void* grads, int grad_dtype, const void* chunks, int n_chunks, double* chunk_sq,
                                   double* tensor_sq, int n_tensors, float max_norm, float* out, hipStream_t stream) {
  if (!grads || !chunks || !tensor_sq || !out || n_chunks < 0 || n_tensors < 1 || (n_chunks > 0 && !chunk_sq))
    return OTAMD_EINVAL;
  if (grad_dtype < 0 || grad_dtype > 2) return OTAMD_EINVAL;
  if (n_chunks > 0) {
    if (grad_dtype != 1)
      grad_sqnorm_kernel<bf16_t><<<n_chunks, 256, 0, stream>>>((const bf16_t*)grads, (const NormChunk*)chunks, chunk_sq);
    else
      grad_sqnorm_kernel<float><<<n_chunks, 256, 0, stream>>>((const float*)grads, (const NormChunk*)chunks, chunk_sq);
    OTAMD_CHECK_LAUNCH();
  }
  return otamd_grad_clip_finalize(chunks, n_chunks, chunk_sq, tensor_sq, n_tensors, max_norm, grad_dtype, out, stream);
}

// the grad-norm pass split over the backward (util/optimizer/adamw_fused.OverlappedGradNorm): the squared norms of
// chunks [c_begin, c_end) into their slots chunk_sq[c] as soon as those tensors' gradients are final, on the
// weight-gradient stream beside the dgrad chain ...
OTAMD_API int otamd_grad_sqnorm_chunks(const void* grads, int grad_dtype, const void* chunks, int c_begin, int c_end,
                                       double* chunk_sq, hipStream_t stream) {
  if (!grads || !chunks || !chunk_sq || c_begin < 0 || c_end < c_begin || grad_dtype < 0 || grad_dtype > 2)
    return OTAMD_EINVAL;
  if (c_end == c_begin) return OTAMD_OK;
  const NormChunk* c = (const NormChunk*)chunks + c_begin;
  if (grad_dtype != 1)
    grad_sqnorm_kernel<bf16_t><<<c_end - c_begin, 256, 0, stream>>>((const bf16_t*)grads, c, chunk_sq + c_begin);
  else
    grad_sqnorm_kernel<float><<<c_end - c_begin, 256, 0, stream>>>((const float*)grads, c, chunk_sq + c_begin);
  OTAMD_CHECK_LAUNCH();
  return OTAMD_OK;
}

// ... and the clip coefficient: per-tensor sums of the chunk slots in chunk order, then clip_grad_norm_'s torch
// dtypes (as otamd_grad_clip_coef)
OTAMD_API int otamd_grad_clip_finalize(const void* chunks, int n_chunks, const double* chunk_sq, double* tensor_sq,
                                       int n_tensors, float max_norm, int grad_dtype, float* out, hipStream_t stream) {
  if (!chunks || !tensor_sq || !out || n_tensors < 1 || n_chunks < 0 || (n_chunks > 0 && !chunk_sq) || grad_dtype < 0 ||
      grad_dtype > 2)
    return OTAMD_EINVAL;
  if (hipMemsetAsync(tensor_sq, 0, sizeof(double) * n_tensors, stream) != hipSuccess) return OTAMD_ELAUNCH;
  if (n_chunks > 0) {
    tensor_sq_kernel<<<(n_chunks + 255) / 256, 256, 0, stream>>>((const NormChunk*)chunks, n_chunks, chunk_sq, tensor_sq);
    OTAMD_CHECK_LAUNCH();
  }
  clip_coef_kernel<<<1, 1024, 0, stream>>>(tensor_sq, n_tensors, max_norm, grad_dtype == 0, out);
  OTAMD_CHECK_LAUNCH();
  return OTAMD_OK;
}

// scale a flat grad store by the device clip coefficient (used when the optimizer is
// not the fused AdamW, e.g. parity checks of clip_grad_norm_ alone)
__global__ void scale_bf16_kernel(bf16_t* __restrict__ g, long long n8, const float* __restrict__ coef) {
  const float c = coef[0];
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n8; i += (long long)gridDim.x * blockDim.x) {
    bf8 v = reinterpret_cast<bf8*>(g)[i];
    float f[8];
    unpack8(v, f);
#pragma unroll
    for (int j = 0; j < 8; ++j) f[j] = f[j] * c;
    reinterpret_cast<bf8*>(g)[i] = pack8(f);
  }
}
OTAMD_API int otamd_scale_bf16_by_device_scalar(void* g, long long n, const float* coef, hipStream_t stream) {
  if (!g || !coef || (n % 8) != 0 || ((uintptr_t)g & 15)) return OTAMD_EINVAL;
  if (n == 0) return OTAMD_OK;
  scale_bf16_kernel<<<adamw_grid(n / 8), 256, 0, stream>>>((bf16_t*)g, n / 8, coef);
  OTAMD_CHECK_LAUNCH();
  return OTAMD_OK;
}
