/* otamd.h -- C ABI of libotamd.so, the MI355X (gfx950) kernels of onetrainer_amd.
 *
 * Drop-in boundary for the diffusion train step of OneTrainer (modules/trainer/GenericTrainer.py:672-749
 * calling modules/modelSetup/<Family>Setup.predict / calculate_loss, loss.backward(), clip_grad_norm_,
 * optimizer.step()).  The reference is pure Python over diffusers/torch, so every entry point
 * below replaces an op the reference reaches through those libraries; each cites it.
 *
 * Conventions (all launchers):
 *   - plain device pointers, sizes and strides (in ELEMENTS), bf16 passed as void* (uint16 bits);
 *   - `stream` is a hipStream_t (torch.cuda.current_stream().cuda_stream in the Python host);
 *   - no implicit allocation: scratch comes in through explicit workspace pointers;
 *   - return 0 on success, 1 = contract violated (shape / alignment; nothing launched),
 *     2 = launch error, 3 = unsupported configuration.  Python maps non-zero to RuntimeError;
 *   - thread-compatible; no global mutable state besides per-process tile-choice caching.
 * Layouts: activations NHWC (pixels x channels) / token-major [B, N, C]; conv weights
 * [Cout][kh][kw][Cin]; Linear weights [out][in]; attention Q/K/V/O [B, N, H*D] with strides.
 */
#ifndef OTAMD_H
#define OTAMD_H
#include <hip/hip_runtime.h>
#ifdef __cplusplus
extern "C" {
#endif

enum { OTAMD_OK = 0, OTAMD_EINVAL = 1, OTAMD_ELAUNCH = 2, OTAMD_EUNSUPPORTED = 3 };

/* GEMM operand modes */
enum { OPM_K = 0, OPM_MN = 1, OPM_CONV_FWD = 2, OPM_CONV_DGRAD = 3, OPM_CONV_WGRAD = 4 };

typedef struct ConvGeom {
  int N, SH, SW, SC, RH, RW, KH, KW, stride, pad, upsample, pad_;
  long long ld;
} ConvGeom;

/* C[M,N] = alpha * op(A) op(B) (+bias[n]) (+rowvec[m/rows_per_vec][n]) (+residual[m][n]) (+C if accumulate) */
typedef struct GemmArgs {
  const void* A; long long lda; int amode;
  const void* B; long long ldb; int bmode;
  void* C; long long ldc; int c_f32; int accumulate;
  int M, N, K;
  float alpha;
  const void* bias;
  const void* rowvec; long long ldv; int rows_per_vec;
  const void* residual; long long ldr;
  float* slab;
  int k_per_split;
  ConvGeom ga, gb;
  /* optional second K segment [K1, K1+K2): A2 K-mode, B2 K-mode (or MN-mode when B is); LoRA up/down fused
     into the base GEMM (replaces the extra GEMM + add of LoRAModule.forward, modules/module/LoRAModule.py:318-322) */
  const void* A2; long long lda2;
  const void* B2; long long ldb2;
  int K1, K2;
  /* batched GEMM (K/MN modes, one segment, no split-K): grid.y = z < batch; operand bases move by
     (z / bdiv) * s0 + (z % bdiv) * s1 elements ((image, head) pairs of [B, N, H*D] activations) */
  int batch, bdiv;
  long long sa0, sa1, sb0, sb1, sc0, sc1;
  /* optional column sums of an MN-mode A over the K range (the bias gradient of a Linear / conv weight
     gradient dW = dY^T X: colsum[m] = sum_k dY[k][m], replaces the separate dY.sum(0) of autograd):
     bf16 or fp32 [M], overwritten or accumulated; with split-K the partials go to the workspace after the
     GEMM slabs (splits * M floats) and the split-K reduce folds them */
  void* colsum; int colsum_f32; int colsum_acc;
  float* colsum_slab;
  /* optional LoRA down-projection fused into a forward base GEMM (linear or 3x3 conv, B = K-mode weights, split 1,
     tiles 1 / 4 / 7 / 8, lora_r = 32): t = A D^T over the K loop for the adapter part of the tile's columns,
     rounded to bf16, stored to T [M][ldt] by the part's first tile column, and t (B2)^T added as the second K
     segment -- replaces the separate down GEMM x A^T + its split-K reduce before the fused up projection
     (LoRAModule.forward, modules/module/LoRAModule.py:318-322).  D = down [P*lora_r][K], B2 / ldb2 = up [N][P*lora_r],
     lora_pw = output columns per part; K = the base K, A2 = NULL.  D == NULL: off.
     The same fields on a linear input-gradient GEMM (A = dY K-mode, B = W MN-mode): u = dY (sB) for one adapter part
     spanning N (lora_pw = N), D = (sB)^T [lora_r][K], B2 / ldb2 = A^T [N][lora_r], T = u [M][ldt] -- the LoRA
     backward's dX = dY W + u A (LoRAModule.py:318-322 differentiated) without the separate u GEMM and its reduce. */
  const void* D; long long ldd;
  void* T; long long ldt;
  int lora_r, lora_pw;
} GemmArgs;

typedef struct AttnArgs {
  const void *q, *k, *v; void* o; float* lse;
  const void* dout; const float* delta; void *dq, *dk, *dv; float *dk32, *dv32;
  long long ldq, ldk, ldv, ldo, lddo, lddq, lddk, lddv;
  long long bsq, bsk, bsv, bso, bsdo, bsdq, bsdk, bsdv;
  int B, H, Nq, Nk, Dv;
  float scale;
  int qsplit, pad_;
} AttnArgs;

/* FLUX q/k RMSNorm + rotary embedding over 128-wide heads (csrc/flux.hip) */
typedef struct QKRopeArgs {
  const void* x; long long ldx; int qoff, koff;
  void* y; long long ldy; int yqoff, ykoff;
  const void* dy; long long lddy; int dyqoff, dykoff;
  const void *wq, *wk, *wq_ctx, *wk_ctx;
  const float *cs, *sn;
  float* dw_part;
  int rows, B, H, L;
  float eps;
  int pad_;
} QKRopeArgs;

typedef struct AdamwGroup {
  long long begin, end;
  float wd_factor, one_minus_beta1, beta2, one_minus_beta2, bc2_sqrt, eps, neg_step_size, pad;
} AdamwGroup;

typedef struct NormChunk { long long begin, end; int tensor, pad; } NormChunk;

/* replaces: diffusers Linear/Conv2d fwd+bwd inside model.unet(...) (modules/modelSetup/BaseStableDiffusionXLSetup.py:268-273); conv/linear dgrad/wgrad of loss.backward() (modules/trainer/GenericTrainer.py:693-696) */
int otamd_gemm(const GemmArgs* in, int splits, void* workspace, long long ws_bytes, hipStream_t stream);

/* plan query: workspace bytes otamd_gemm needs for `splits` (0 = automatic tile + split-K plan) */
long long otamd_gemm_plan(const GemmArgs* in, int splits, int* splits_out);

/* replaces: (plan override) the same GEMM with an explicit plan -- the autotuner's candidates and its
   cached per-shape choice (kernels.py set_gemm_autotune) and the measured plan table
   (onetrainer_amd/gemm_plans_mi355x.json).  tile: -1 v1 128x128, 0 256x256, 1 256x128, 2 128x256,
   3 256x256/4 waves, 4 128x128/8 waves, 5 128x64, 6 64x128, 7 128x160, 8 256x160, 9 / 10 = 5 / 6 on a
   4-deep LDS ring; splits >= 1;
   workspace >= splits*M*N*4 bytes when splits > 1 */
int otamd_gemm_explicit(const GemmArgs* in, int tile, int splits, void* workspace, long long ws_bytes,
                        hipStream_t stream);

/* replaces: (diagnostic) the tile otamd_gemm launches for these arguments: -1 v1 128x128, 0 256x256, 1 256x128, 2 128x256, 3 256x256/4 waves,
   4 128x128, 5 128x64, 6 64x128, 7 128x160, 8 256x160 */
int otamd_gemm_plan_tile(const GemmArgs* in, int splits);
/* workspace bytes of a `splits`-way split-K launch (fp32 slabs, + the column-sum partials when colsum is set) */
long long otamd_gemm_ws_bytes(const GemmArgs* in, int splits);

/* replaces: ABI check */
int otamd_gemm_args_size(void);

/* replaces: ABI check */
int otamd_conv_geom_size(void);

/* replaces: F.scaled_dot_product_attention in diffusers Attention (attn1/attn2 of every BasicTransformerBlock) */
int otamd_attn_fwd(const AttnArgs* in, hipStream_t stream);

/* replaces: autograd of scaled_dot_product_attention (GenericTrainer.py:693-696) */
int otamd_attn_bwd(const AttnArgs* in, float* ws, long long ws_bytes, hipStream_t stream);

/* workspace bytes otamd_attn_bwd needs for these arguments (16-byte bias records per query + split-query or
   per-chunk dK/dV partials) */
long long otamd_attn_bwd_ws_bytes(const AttnArgs* in);

/* bytes of the fp32 dK / dV partial slabs alone (0: none needed), the caller-owned buffer of otamd_attn_bwd_ex */
long long otamd_attn_bwd_slab_bytes(const AttnArgs* in);

/* replaces: as otamd_attn_bwd (autograd of scaled_dot_product_attention, GenericTrainer.py:693-696), with the dK / dV
   partial slabs in a caller-owned buffer and their chunk-order sum on cast_stream (ordered after `stream` by an
   event): the one-pass cross-attention backward's dK / dV feed only the K / V projections' weight gradients */
int otamd_attn_bwd_ex(const AttnArgs* in, float* ws, long long ws_bytes, float* slabs, long long slab_bytes,
                      hipStream_t stream, hipStream_t cast_stream);

/* replaces: ABI check */
int otamd_attn_args_size(void);

/* replaces: the softmax inside F.scaled_dot_product_attention for heads wider than 128 (SD 1.5 160-wide heads,
   v1-inference.yaml:29-44; VAE mid-block 512-wide head): P = softmax(scale S) row-wise, bf16 P, natural-log lse */
int otamd_softmax_rows_fwd(const float* S, long long lds, void* P, long long ldp, float* lse, long long rows,
                           int ncols, int ncols_pad, float scale, hipStream_t stream);

/* replaces: autograd of that softmax: dS = scale P (dP - rowsum(P dP)) */
int otamd_softmax_rows_bwd(const void* P, long long ldp, const float* dP, long long lddp, void* dS, long long ldds,
                           long long rows, int ncols, int ncols_pad, float scale, hipStream_t stream);

/* replaces: mgds RescaleImageChannels(0..1 -> -1..1) + the NCHW image handed to AutoencoderKL.encode
   (StableDiffusionXLBaseDataLoader.py:66-67): out[b,h,w,c] = img[b,c,h,w] * mul + add, NHWC bf16, c >= C zero */
int otamd_image_to_nhwc(const float* img, int B, int C, int H, int W, float mul, float add, void* out, int cpad,
                        hipStream_t s);

/* ---- FLUX.1 transformer (rows r = t * B + b over [text ; image] tokens; modulation mod[b * ldm + off + c]) ---- */
/* replaces: AdaLayerNormZero / AdaLayerNormZeroSingle / AdaLayerNormContinuous forward (diffusers FluxTransformer2DModel,
   called at modules/modelSetup/BaseFluxSetup.py:289-299): y = LN(x) * (1 + scale[b]) + shift[b], no affine */
int otamd_adaln_fwd(const void* x, long long ldx, void* y, long long ldy, int rows, int D, float eps, const void* mod,
                    long long ldm, int shift_off, int scale_off, int B, float* mean, float* rstd, hipStream_t s);

/* replaces: autograd of that adaLN: dx, and bf16 d(shift), d(scale) written into dmod (part: otamd_mod_part_floats) */
int otamd_adaln_bwd(const void* x, long long ldx, const void* dy, long long lddy, void* dx, long long lddx, int rows,
                    int D, const void* mod, long long ldm, int shift_off, int scale_off, int B, const float* mean,
                    const float* rstd, void* dmod, float* part, hipStream_t s);

/* the same + res (the adaLN input's gradient through its residual use, the block's gated add) in the dx pass,
   instead of autograd's separate add of the two contributions */
int otamd_adaln_bwd_res(const void* x, long long ldx, const void* dy, long long lddy, const void* res, long long ldres,
                        void* dx, long long lddx, int rows, int D, const void* mod, long long ldm, int shift_off,
                        int scale_off, int B, const float* mean, const float* rstd, void* dmod, float* part,
                        hipStream_t s);

/* replaces: the modulation half of that autograd alone (bf16 d(shift), d(scale) into dmod), for a caller that runs it
   beside the dx pass on the weight-gradient stream (the modulation only feeds weight gradients) */
int otamd_adaln_dmod(const void* x, long long ldx, const void* dy, long long lddy, int rows, int D, long long ldm,
                     int shift_off, int scale_off, int B, const float* mean, const float* rstd, void* dmod, float* part,
                     hipStream_t s);

/* scratch floats the adaLN / gated-add backward reductions need */
long long otamd_mod_part_floats(int T, int D, int B);

/* replaces: hidden = hidden + gate_msa.unsqueeze(1) * attn_output (and the gate_mlp / single-block gate adds) */
int otamd_gated_add_fwd(const void* x, long long ldx, const void* y, long long ldy, void* out, long long ldo, int rows,
                        int D, const void* mod, long long ldm, int gate_off, int B, hipStream_t s);

/* replaces: autograd of the gated add: dy = gate * dout, d(gate) into dmod */
int otamd_gated_add_bwd(const void* dout, long long lddo, const void* y, long long ldy, void* dy, long long lddy,
                        int rows, int D, const void* mod, long long ldm, int gate_off, int B, void* dmod, float* part,
                        hipStream_t s);

/* replaces: ABI check */
int otamd_qk_rope_args_size(void);

/* replaces: attn.norm_q / norm_k / norm_added_q / norm_added_k (RMSNorm eps 1e-6) + apply_rotary_emb(FluxPosEmbed) */
int otamd_qknorm_rope_fwd(const QKRopeArgs* in, hipStream_t s);

/* replaces: autograd of that; optional norm-weight grads (part: >= 512 * 1024 floats) */
int otamd_qknorm_rope_bwd(const QKRopeArgs* in, void* dwq, void* dwk, void* dwq_ctx, void* dwk_ctx, int dw_f32,
                          int dw_acc, float* part, hipStream_t s);

/* replaces: GELU(approximate="tanh") of FeedForward(activation_fn="gelu-tanh") and the single blocks' act_mlp */
int otamd_gelu_tanh_fwd(const void* x, long long ldx, void* y, long long ldy, int rows, int F, hipStream_t s);

/* replaces: autograd of GELU(tanh) */
int otamd_gelu_tanh_bwd(const void* x, long long ldx, const void* dy, long long lddy, void* dx, long long lddx,
                        int rows, int F, hipStream_t s);

/* replaces: FluxModel.pack_latents (dir 0) / unpack_latents (dir 1), modules/model/FluxModel.py:317-344 */
int otamd_flux_pack(const void* src, void* dst, int B, int h, int w, int C, int ldl, int dir, hipStream_t s);

/* replaces: ResnetBlock2D norm1/norm2 + SiLU, Transformer2DModel.norm, conv_norm_out (diffusers, via BaseStableDiffusionXLSetup.py:268-273) */
int otamd_groupnorm_fwd(const void* x, long long ldx, void* y, long long ldy, int N, int HW, int C, int G,
                        float eps, const void* gamma, const void* beta, int silu, float* mean, float* rstd, float* a,
                        float* b, float* ws, hipStream_t stream);

/* replaces: autograd of GroupNorm(+SiLU) */
int otamd_groupnorm_bwd(const void* x, long long ldx, const void* dy, long long lddy, void* dx, long long lddx,
                        int N, int HW, int C, int G, const void* gamma, int silu, const float* mean, const float* rstd,
                        const float* a, const float* b, void* dgamma, void* dbeta, int param_f32, int param_acc,
                        float* ws, int accumulate, hipStream_t stream);

/* replaces: autograd of GroupNorm(+SiLU) plus the autograd add of its input's second gradient (the
   ResnetBlock2D shortcut / Transformer2DModel proj_out residual): dx = GroupNorm-backward(dy) + dres */
int otamd_groupnorm_bwd_res(const void* x, long long ldx, const void* dy, long long lddy, const void* dres,
                            long long ldres, void* dx, long long lddx, int N, int HW, int C, int G, const void* gamma,
                            int silu, const float* mean, const float* rstd, const float* a, const float* b,
                            void* dgamma, void* dbeta, int param_f32, int param_acc, float* ws, hipStream_t stream);

/* scratch floats otamd_groupnorm_fwd / _bwd need for these sizes (partial slabs, coefficients, sums) */
long long otamd_groupnorm_ws_floats(int N, int HW, int C);

/* replaces: BasicTransformerBlock norm1/norm2/norm3 */
int otamd_layernorm_fwd(const void* x, long long ldx, void* y, long long ldy, int rows, int C, float eps,
    const void* gamma, const void* beta, float* mean, float* rstd, hipStream_t stream);

/* replaces: autograd of LayerNorm */
int otamd_layernorm_bwd(const void* x, long long ldx, const void* dy, long long lddy, void* dx, long long
    lddx, int rows, int C, const void* gamma, const float* mean, const float* rstd, void* dgamma, void* dbeta,
    int param_f32, int param_acc, float* part, int accumulate, hipStream_t stream);

/* replaces: autograd of LayerNorm + the autograd add of its input's second use as the block residual
   (BasicTransformerBlock: norm1/2/3 input = to_out / ff residual): dx = LN_bwd(dy) + dres */
int otamd_layernorm_bwd_res(const void* x, long long ldx, const void* dy, long long lddy, const void* dres,
    long long ldres, void* dx, long long lddx, int rows, int C, const void* gamma, const float* mean,
    const float* rstd, hipStream_t stream);

/* replaces: the LayerNorm weight / bias gradient half of the same autograd node (dgamma = sum dy xhat,
   dbeta = sum dy), issued separately so it can run on the weight-gradient side stream */
int otamd_layernorm_param_grad(const void* x, long long ldx, const void* dy, long long lddy, int rows, int C,
    const float* mean, const float* rstd, void* dgamma, void* dbeta, int param_f32, int param_acc, float* part,
    hipStream_t stream);

/* Deferred LayerNorm parameter reduces: while a stream is in defer mode, otamd_layernorm_param_grad (and
   otamd_layernorm_bwd with parameter gradients) on it write their per-slab partials into `arena` and leave the final
   dgamma / dbeta sums pending; one grouped launch sums up to 64 of them (bit-identical to the immediate path).  The
   caller flushes before anything reads those gradients (the gradient-norm / DP bucket launches, the end of backward).
   Reference: the gamma / beta gradients of diffusers' BasicTransformerBlock norm1-3 (replaces nothing in the
   reference's own code: torch's fused LayerNorm backward reduces them inside one kernel). */
int otamd_layernorm_defer_begin(hipStream_t stream, void* arena, long long bytes);
int otamd_layernorm_defer_flush(hipStream_t stream);
int otamd_layernorm_defer_end(hipStream_t stream);
/* the same with the pending reduces launched on `launch`, which the caller has ordered after `stream` */
int otamd_layernorm_defer_end_on(hipStream_t stream, hipStream_t launch);
/* out[0] LayerNorms deferred, out[1] grouped launches (totals since load), out[2] pending on `stream` */
int otamd_layernorm_defer_stats(hipStream_t stream, long long* out);

/* replaces: diffusers GEGLU (ff.net.0) hidden * gelu(gate) */
int otamd_geglu_fwd(const void* h, long long ldh, void* out, long long ldo, int M, int F, hipStream_t s);

/* ---- text-encoder caching: CLIP-L / CLIP-bigG / T5 forward ---------------- */
/* replaces: CLIPTextEmbeddings / T5 embed_tokens (transformers, called from model/util/clip_util.py:26-31,
   t5_util.py:17-22): out[r] = tok[ids[r]] (+ pos[r % T]); ids clamped to [0, vocab) */
int otamd_embed_tokens(const long long* ids, long long n, int T, const void* tok, const void* pos, void* out, int D,
                       int vocab, hipStream_t stream);
/* replaces: CLIPMLP activation (quick_gelu CLIP-L = 0, erf gelu bigG = 1) / gelu_new (2); y may alias x */
int otamd_act_fwd(const void* x, long long ldx, void* y, long long ldy, long long rows, int C, int kind,
                  hipStream_t stream);
/* replaces: T5DenseGatedActDense's act(wi_0 x) * wi_1 x over the fused [wi_0 | wi_1] projection */
int otamd_gated_act_fwd(const void* h, long long ldh, void* out, long long ldo, long long rows, int F, int kind,
                        hipStream_t stream);
/* replaces: T5LayerNorm (RMS norm, fp32 statistics, no bias) */
int otamd_rmsnorm_fwd(const void* x, long long ldx, void* y, long long ldy, long long rows, int C, float eps,
                      const void* w, hipStream_t stream);
/* replaces: the softmax of CLIPAttention (causal mask) and T5Attention (scores + relative position bias):
   P[r] = softmax(scale S[r] + bias[q, c, h]) with r = (b H + h) Nq + q; causal masks c > q */
int otamd_softmax_masked_fwd(const float* S, long long lds, void* P, long long ldp, long long rows, int ncols,
                             int ncols_pad, float scale, int Nq, int H, int causal, const void* bias, long long bsq,
                             long long bsc, long long bsh, hipStream_t stream);

/* replaces: autograd of GEGLU */
int otamd_geglu_bwd(const void* h, long long ldh, const void* dout, long long lddo, void* dh, long long lddh,
    int M, int F, hipStream_t s);

/* replaces: nonlinearity(temb) / TimestepEmbedding act */
int otamd_silu_fwd(const void* x, void* y, long long n, hipStream_t s);

/* replaces: autograd of SiLU */
int otamd_silu_bwd(const void* x, const void* dy, void* dx, long long n, hipStream_t s);

/* replaces: torch.cat([hidden, res_hidden], dim=1) in up blocks */
int otamd_concat_channels(const void* a, long long lda, int Ca, const void* b, long long ldb, int Cb, void*
    out, long long P, hipStream_t s);

/* replaces: autograd of F.interpolate(scale_factor=2, nearest) in Upsample2D */
int otamd_upsample2x_bwd(const void* dup, void* dx, int N, int H, int W, int C, int accumulate, hipStream_t
    s);

/* replaces: bias / time_emb_proj gradients (autograd of Linear/Conv2d bias, temb broadcast add) */
int otamd_colsum(const void* x, long long ldx, int M, int N, int rows_per_group, void* out, int out_f32, int
    accumulate, float* ws, long long ws_floats, hipStream_t s);

/* replaces: workspace size query for otamd_colsum */
long long otamd_colsum_ws_floats(int M, int N, int rows_per_group);

/* replaces: weight layout transform for conv dgrad (no reference equivalent; internal) */
int otamd_conv_weight_transpose(const void* w, void* wt, int Cout, int KK, int Cin, hipStream_t s);

/* replaces: fp32 reduction result -> bf16/f32 grad (internal) */
int otamd_cast_f32(const float* x, void* y, long long n, int dst_f32, int accumulate, hipStream_t s);

/* replaces: the per-forward autocast casts of every LoRA down/up weight (LoRAModule.forward under
   autocast, modules/module/LoRAModule.py:318-322) -- one launch refreshes all bf16 shadows.
   table: device array of {long long src, dst; int rows, cols, dst_ld; float scale; int transpose, pad}
   (transpose = 1: the [rows][cols] source lands as [cols][rows] with row stride dst_ld) */
int otamd_lora_shadow(const float* src, void* dst, const void* table, int n_entries, hipStream_t s);

/* replaces: ABI check */
int otamd_lora_shadow_entry_size(void);

/* replaces: diffusers get_timestep_embedding (UNet time_proj / add_time_proj) */
int otamd_timestep_embedding(const float* t, int n, int dim, void* out, long long ldo, hipStream_t s);

/* replaces: residual add where not fused into a GEMM epilogue */
int otamd_add(const void* a, const void* b, void* y, long long n, hipStream_t s);

/* replaces: nothing (engine control): deferred split-K reduces.  Between begin and end, the split-K GEMMs launched on
   `stream` without bias / row-vector / residual operands whose output (and fused column sums) lie inside
   [out, out + out_bytes) -- the flat weight-gradient buffer, which only GEMMs on this stream write and nothing reads
   before a flush -- put their fp32 slabs into `arena` (caller-owned, 256-byte aligned, >= 1 MiB, alive until end)
   and their reduces are launched together, up to 40 per grouped launch, at flush / end, when the arena or the batch
   is full, or before a GEMM on the stream reads or writes a pending output.  Each output is summed in split order
   as by the immediate reduce: bit-identical. */
int otamd_gemm_defer_begin(hipStream_t stream, void* arena, long long bytes, const void* out, long long out_bytes);
int otamd_gemm_defer_flush(hipStream_t stream);
int otamd_gemm_defer_end(hipStream_t stream);
int otamd_gemm_defer_pending(hipStream_t stream);
int otamd_gemm_defer_stats(long long* out);

/* replaces: nothing in the reference (it has no DP): the on-chip footprint of one gradient bucket's RCCL ring
   all-reduce, emulated on one GPU for the step-slowdown measurement of DESIGN.md §6 (trainer/ddp.py
   OTAMD_DP_EMULATE): `blocks` workgroups copy `bytes` from src to dst (each wrapping over its size), paced to take
   at least `ns` nanoseconds */
int otamd_dp_emulate(const void* src, long long src_bytes, void* dst, long long dst_bytes, long long bytes, int blocks,
                     long long ns, hipStream_t s);

/* replaces: ModelSetupNoiseMixin._create_noise (modules/modelSetup/mixin/ModelSetupNoiseMixin.py:18-49) */
int otamd_noise(void* out, int f32, long long n, long long offset, unsigned long long seed, hipStream_t s);
/* replaces: the same with offset_noise_weight / perturbation_noise_weight > 0 (ModelSetupNoiseMixin.py:31-46):
   noise + ow * N[sample, channel] (constant over the pixels), then + pw * N, each op rounded to the output
   dtype in the reference's order.  NHWC tensor, hwc = h * w * C; offset = global element index of out[0]. */
int otamd_noise_ex(void* out, int f32, long long n, long long offset, unsigned long long seed, int C,
    long long hwc, float offset_weight, float perturbation_weight, hipStream_t s);
/* test hook: raw standard-normal draws of Philox stream `stream_id` (1 = noise, 4 = offset, 5 = perturbation) */
int otamd_noise_stream(void* out, int f32, long long n, long long offset, unsigned long long seed, int stream_id,
    hipStream_t s);

/* replaces: ModelSetupNoiseMixin._get_timestep_discrete (ModelSetupNoiseMixin.py:51-155), UNIFORM (dist 0) and
   LOGIT_NORMAL (dist 1) with static shift.  min_t / max_t = int(num_train_timesteps * min/max_noising_strength)
   (:69-70).  draws (nullable): injected per-sample draws instead of Philox -- the U[0,1) sample (UNIFORM) or the
   N(bias, weight+1) sample (LOGIT_NORMAL) of the reference's generator. */
int otamd_timesteps(int* out, int n, long long sample0, unsigned long long seed, int dist, int
    num_train_timesteps, int min_t, int max_t, float shift, float bias, float weight, const float* draws,
    hipStream_t s);

/* replaces: BaseStableDiffusionXLSetup.predict scale + _add_noise_discrete + get_velocity (BaseStableDiffusionXLSetup.py:214-236,277-291; ModelSetupDiffusionMixin.py:15-38) */
int otamd_ddpm_prologue(const void* latent, const void* noise, int lat_f32, const int* timestep, const float*
    acp, const float* sqrt_acp, const float* sqrt_1m, float sf, int B, long long HW, int C, int cpad, void*
    unet_in, void* target, int target_kind, float* scaled_out, hipStream_t s);

/* replaces: BaseFluxSetup.predict scale/shift + ModelSetupFlowMatchingMixin._add_noise_discrete (ModelSetupFlowMatchingMixin.py:14-39) + flow target (BaseFluxSetup.py:307) */
int otamd_flow_prologue(const void* latent, const void* noise, int lat_f32, const int* timestep, float sf,
    float shift_factor, int num_t, int B, long long HW, int C, int cpad, void* model_in, void* target,
    hipStream_t s);

/* replaces: ModelSetupDiffusionLossMixin._diffusion_losses / _flow_matching_losses / __unmasked_losses + .mean()
   (ModelSetupDiffusionLossMixin.py:119-168,233-321; BaseStableDiffusionXLSetup.py:360-373; BaseFluxSetup.py:377-390).
   loss_fn: 0 CONSTANT, 1 MIN_SNR_GAMMA, 2 DEBIASED_ESTIMATION, 3 P2 (sqrt_acp / sqrt_1m tables), 4 SIGMA
   ((t+1)/num_t, flow matching).  B <= 1024. */
int otamd_mse_loss(const void* pred, int cpad, const void* target, int tgt_f32, int B, long long HW, int C,
    float mse_strength, float scale, const float* loss_weight, const int* timestep, const float* sqrt_acp,
    const float* sqrt_1m, int loss_fn, float gamma, int v_pred, int num_t, float ga, float* ws, long long ws_floats,
    float* loss_out, float* coef, float* losses_out, hipStream_t s);

/* replaces: autograd of the MSE loss */
int otamd_mse_grad(const void* pred, int cpad, const void* target, int tgt_f32, int B, long long HW, int C,
    const float* coef, const float* grad_out, void* dpred, hipStream_t s);

/* replaces: AdamW step_adamw_parameter + addcdiv_stochastic_ (modules/util/optimizer/adamw_extensions.py:17-150; modules/util/bf16_stochastic_rounding.py:5-61), patched at modules/util/create.py:509-534 */
int otamd_adamw_bf16(void* p, const void* g, void* m, void* v, long long n, const AdamwGroup* groups, int
    n_groups, const float* clip_coef, int stochastic_rounding, unsigned long long seed, hipStream_t stream);

/* replaces: same, restricted to elements [begin, end) of the flat buffers (multiples of 8; the groups and the
   stochastic-rounding stream keep their global element indices, so chunked launches give the bits of one
   whole-store launch).  Lets the optimizer run in parameter-range chunks on its own stream. */
int otamd_adamw_bf16_range(void* p, const void* g, void* m, void* v, long long begin, long long end, const
    AdamwGroup* groups, int n_groups, const float* clip_coef, int stochastic_rounding, unsigned long long seed,
    hipStream_t stream);

/* replaces: same, fp32 parameters (LoRA weights, TrainConfig.py:959) */
int otamd_adamw_f32(void* p, const void* g, void* m, void* v, long long n, const AdamwGroup* groups, int
    n_groups, const float* clip_coef, hipStream_t stream);

/* replaces: same, fp32 master weights of a full fine-tune (weight_dtype FLOAT_32, TrainConfig.py:782, under a bf16
   autocast, dtype_util.py:28-49): p32 / m32 / v32 fp32, g16 the bf16 gradient store, w16 the bf16 working copy the
   GEMMs read, rewritten as rne(p32) (autocast's cast); elements [begin, end), multiples of 8 */
int otamd_adamw_master_range(void* p32, const void* g16, void* m32, void* v32, void* w16, long long begin,
    long long end, const AdamwGroup* groups, int n_groups, const float* clip_coef, hipStream_t stream);

/* replaces: nn.utils.clip_grad_norm_(parameters, clip_grad_norm) (modules/trainer/GenericTrainer.py:712-713);
   grad_dtype 0 bf16, 1 fp32, 2 bf16 storage of fp32-master gradients (norms and coefficient in fp32); 
   chunk_sq: double[n_chunks] scratch (one slot per chunk, summed per tensor in chunk order: deterministic) */
int otamd_grad_clip_coef(const void* grads, int grad_dtype, const void* chunks, int n_chunks, double* chunk_sq,
    double* tensor_sq, int n_tensors, float max_norm, float* out, hipStream_t stream);

/* replaces: clip_grad_norm_ split over the backward (GenericTrainer.py:712-713): squared norms of the chunks
   [c_begin, c_end) into their slots chunk_sq[c] as soon as their gradients are final (every chunk once per step),
   then the per-tensor sums in chunk order and the coefficient (out[0] coefficient, out[1] total norm) */
int otamd_grad_sqnorm_chunks(const void* grads, int grad_dtype, const void* chunks, int c_begin, int c_end,
                             double* chunk_sq, hipStream_t stream);
int otamd_grad_clip_finalize(const void* chunks, int n_chunks, const double* chunk_sq, double* tensor_sq,
                             int n_tensors, float max_norm, int grad_dtype, float* out, hipStream_t stream);

/* replaces: the grad scaling half of clip_grad_norm_ when not fused into AdamW */
int otamd_scale_bf16_by_device_scalar(void* g, long long n, const float* coef, hipStream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* OTAMD_H */
