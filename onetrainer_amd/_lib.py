"""ctypes binding of the C-ABI library (include/otamd.h).

The product path has no CPU fallback: if libotamd.so is missing or does not load,
every op raises.  Structs below mirror the C layouts; `check_layouts()` compares
their sizes with the library's own sizeof() exports.
"""
from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

LIB_PATH = Path(__file__).resolve().parent / "_lib" / "libotamd.so"

OTAMD_OK, OTAMD_EINVAL, OTAMD_ELAUNCH, OTAMD_EUNSUPPORTED = 0, 1, 2, 3
_ERR = {1: "invalid arguments (shape/alignment contract)", 2: "kernel launch failed", 3: "unsupported configuration"}


class ConvGeom(C.Structure):
    _fields_ = [("N", C.c_int), ("SH", C.c_int), ("SW", C.c_int), ("SC", C.c_int), ("RH", C.c_int),
                ("RW", C.c_int), ("KH", C.c_int), ("KW", C.c_int), ("stride", C.c_int), ("pad", C.c_int),
                ("upsample", C.c_int), ("pad_", C.c_int), ("ld", C.c_longlong)]


class GemmArgs(C.Structure):
    _fields_ = [("A", C.c_void_p), ("lda", C.c_longlong), ("amode", C.c_int),
                ("B", C.c_void_p), ("ldb", C.c_longlong), ("bmode", C.c_int),
                ("C", C.c_void_p), ("ldc", C.c_longlong), ("c_f32", C.c_int), ("accumulate", C.c_int),
                ("M", C.c_int), ("N", C.c_int), ("K", C.c_int), ("alpha", C.c_float),
                ("bias", C.c_void_p), ("rowvec", C.c_void_p), ("ldv", C.c_longlong), ("rows_per_vec", C.c_int),
                ("residual", C.c_void_p), ("ldr", C.c_longlong), ("slab", C.c_void_p), ("k_per_split", C.c_int),
                ("ga", ConvGeom), ("gb", ConvGeom),
                ("A2", C.c_void_p), ("lda2", C.c_longlong), ("B2", C.c_void_p), ("ldb2", C.c_longlong),
                ("K1", C.c_int), ("K2", C.c_int),
                ("batch", C.c_int), ("bdiv", C.c_int), ("sa0", C.c_longlong), ("sa1", C.c_longlong),
                ("sb0", C.c_longlong), ("sb1", C.c_longlong), ("sc0", C.c_longlong), ("sc1", C.c_longlong),
                ("colsum", C.c_void_p), ("colsum_f32", C.c_int), ("colsum_acc", C.c_int), ("colsum_slab", C.c_void_p),
                ("D", C.c_void_p), ("ldd", C.c_longlong), ("T", C.c_void_p), ("ldt", C.c_longlong),
                ("lora_r", C.c_int), ("lora_pw", C.c_int)]


class AdamwGroup(C.Structure):
    _fields_ = [("begin", C.c_longlong), ("end", C.c_longlong), ("wd_factor", C.c_float),
                ("one_minus_beta1", C.c_float), ("beta2", C.c_float), ("one_minus_beta2", C.c_float),
                ("bc2_sqrt", C.c_float), ("eps", C.c_float), ("neg_step_size", C.c_float), ("pad", C.c_float)]


class NormChunk(C.Structure):
    _fields_ = [("begin", C.c_longlong), ("end", C.c_longlong), ("tensor", C.c_int), ("pad", C.c_int)]


class LoraShadowEntry(C.Structure):
    _fields_ = [("src", C.c_longlong), ("dst", C.c_longlong), ("rows", C.c_int), ("cols", C.c_int),
                ("dst_ld", C.c_int), ("scale", C.c_float), ("transpose", C.c_int), ("pad", C.c_int)]


class AttnArgs(C.Structure):
    _fields_ = [("q", C.c_void_p), ("k", C.c_void_p), ("v", C.c_void_p), ("o", C.c_void_p), ("lse", C.c_void_p),
                ("dout", C.c_void_p), ("delta", C.c_void_p), ("dq", C.c_void_p), ("dk", C.c_void_p),
                ("dv", C.c_void_p), ("dk32", C.c_void_p), ("dv32", C.c_void_p),
                ("ldq", C.c_longlong), ("ldk", C.c_longlong), ("ldv", C.c_longlong), ("ldo", C.c_longlong),
                ("lddo", C.c_longlong), ("lddq", C.c_longlong), ("lddk", C.c_longlong), ("lddv", C.c_longlong),
                ("bsq", C.c_longlong), ("bsk", C.c_longlong), ("bsv", C.c_longlong), ("bso", C.c_longlong),
                ("bsdo", C.c_longlong), ("bsdq", C.c_longlong), ("bsdk", C.c_longlong), ("bsdv", C.c_longlong),
                ("B", C.c_int), ("H", C.c_int), ("Nq", C.c_int), ("Nk", C.c_int), ("Dv", C.c_int),
                ("scale", C.c_float), ("qsplit", C.c_int), ("pad_", C.c_int)]


class QKRopeArgs(C.Structure):
    _fields_ = [("x", C.c_void_p), ("ldx", C.c_longlong), ("qoff", C.c_int), ("koff", C.c_int),
                ("y", C.c_void_p), ("ldy", C.c_longlong), ("yqoff", C.c_int), ("ykoff", C.c_int),
                ("dy", C.c_void_p), ("lddy", C.c_longlong), ("dyqoff", C.c_int), ("dykoff", C.c_int),
                ("wq", C.c_void_p), ("wk", C.c_void_p), ("wq_ctx", C.c_void_p), ("wk_ctx", C.c_void_p),
                ("cs", C.c_void_p), ("sn", C.c_void_p), ("dw_part", C.c_void_p),
                ("rows", C.c_int), ("B", C.c_int), ("H", C.c_int), ("L", C.c_int), ("eps", C.c_float),
                ("pad_", C.c_int)]


VP, I, LL, F, D = C.c_void_p, C.c_int, C.c_longlong, C.c_float, C.c_double
U64 = C.c_ulonglong

# symbol -> argtypes (restype int).  Mirrors include/otamd.h one-for-one.
SIGNATURES: dict[str, list] = {
    "otamd_gemm_args_size": [],
    "otamd_conv_geom_size": [],
    "otamd_gemm": [C.POINTER(GemmArgs), I, VP, LL, VP],
    "otamd_gemm_plan": [C.POINTER(GemmArgs), I, C.POINTER(C.c_int)],
    "otamd_gemm_explicit": [C.POINTER(GemmArgs), I, I, VP, LL, VP],
    "otamd_gemm_plan_tile": [C.POINTER(GemmArgs), I],
    "otamd_gemm_ws_bytes": [C.POINTER(GemmArgs), I],
    "otamd_adamw_bf16": [VP, VP, VP, VP, LL, C.POINTER(AdamwGroup), I, VP, I, C.c_ulonglong, VP],
    "otamd_adamw_bf16_range": [VP, VP, VP, VP, LL, LL, C.POINTER(AdamwGroup), I, VP, I, C.c_ulonglong, VP],
    "otamd_adamw_f32": [VP, VP, VP, VP, LL, C.POINTER(AdamwGroup), I, VP, VP],
    "otamd_adamw_master_range": [VP, VP, VP, VP, VP, LL, LL, C.POINTER(AdamwGroup), I, VP, VP],
    "otamd_grad_clip_coef": [VP, I, VP, I, VP, VP, I, F, VP, VP],
    "otamd_grad_sqnorm_chunks": [VP, I, VP, I, I, VP, VP],
    "otamd_grad_clip_finalize": [VP, I, VP, VP, I, F, I, VP, VP],
    "otamd_scale_bf16_by_device_scalar": [VP, LL, VP, VP],
    # norm.hip
    "otamd_groupnorm_fwd": [VP, LL, VP, LL, I, I, I, I, F, VP, VP, I, VP, VP, VP, VP, VP, VP],
    "otamd_groupnorm_bwd": [VP, LL, VP, LL, VP, LL, I, I, I, I, VP, I, VP, VP, VP, VP, VP, VP, I, I, VP, I, VP],
    "otamd_groupnorm_bwd_res": [VP, LL, VP, LL, VP, LL, VP, LL, I, I, I, I, VP, I, VP, VP, VP, VP, VP, VP, I, I, VP, VP],
    "otamd_groupnorm_ws_floats": [I, I, I],
    "otamd_layernorm_fwd": [VP, LL, VP, LL, I, I, F, VP, VP, VP, VP, VP],
    "otamd_layernorm_bwd": [VP, LL, VP, LL, VP, LL, I, I, VP, VP, VP, VP, VP, I, I, VP, I, VP],
    "otamd_layernorm_param_grad": [VP, LL, VP, LL, I, I, VP, VP, VP, VP, I, I, VP, VP],
    "otamd_layernorm_defer_begin": [VP, VP, LL],
    "otamd_layernorm_defer_flush": [VP],
    "otamd_layernorm_defer_end": [VP],
    "otamd_layernorm_defer_end_on": [VP, VP],
    "otamd_layernorm_defer_stats": [VP, VP],
    "otamd_layernorm_bwd_res": [VP, LL, VP, LL, VP, LL, VP, LL, I, I, VP, VP, VP, VP],
    # attention.hip
    "otamd_attn_args_size": [],
    "otamd_attn_fwd": [C.POINTER(AttnArgs), VP],
    "otamd_attn_bwd": [C.POINTER(AttnArgs), VP, LL, VP],
    "otamd_attn_bwd_ws_bytes": [C.POINTER(AttnArgs)],
    "otamd_attn_bwd_slab_bytes": [C.POINTER(AttnArgs)],
    "otamd_attn_bwd_ex": [C.POINTER(AttnArgs), VP, LL, VP, LL, VP, VP],
    # softmax.hip (materialized attention for heads > 128)
    "otamd_softmax_rows_fwd": [VP, LL, VP, LL, VP, LL, I, I, F, VP],
    "otamd_softmax_rows_bwd": [VP, LL, VP, LL, VP, LL, LL, I, I, F, VP],
    # elementwise.hip
    "otamd_geglu_fwd": [VP, LL, VP, LL, I, I, VP],
    "otamd_embed_tokens": [VP, LL, I, VP, VP, VP, I, I, VP],
    "otamd_act_fwd": [VP, LL, VP, LL, LL, I, I, VP],
    "otamd_gated_act_fwd": [VP, LL, VP, LL, LL, I, I, VP],
    "otamd_rmsnorm_fwd": [VP, LL, VP, LL, LL, I, F, VP, VP],
    "otamd_softmax_masked_fwd": [VP, LL, VP, LL, LL, I, I, F, I, I, I, VP, LL, LL, LL, VP],
    "otamd_geglu_bwd": [VP, LL, VP, LL, VP, LL, I, I, VP],
    "otamd_silu_fwd": [VP, VP, LL, VP],
    "otamd_silu_bwd": [VP, VP, VP, LL, VP],
    "otamd_concat_channels": [VP, LL, I, VP, LL, I, VP, LL, VP],
    "otamd_upsample2x_bwd": [VP, VP, I, I, I, I, I, VP],
    "otamd_colsum": [VP, LL, I, I, I, VP, I, I, VP, LL, VP],
    "otamd_colsum_ws_floats": [I, I, I],
    "otamd_conv_weight_transpose": [VP, VP, I, I, I, VP],
    "otamd_cast_f32": [VP, VP, LL, I, I, VP],
    "otamd_lora_shadow": [VP, VP, VP, I, VP],
    "otamd_lora_shadow_entry_size": [],
    "otamd_timestep_embedding": [VP, I, I, VP, LL, VP],
    "otamd_add": [VP, VP, VP, LL, VP],
    "otamd_dp_emulate": [VP, LL, VP, LL, LL, I, LL, VP],
    "otamd_gemm_defer_begin": [VP, VP, LL, VP, LL],
    "otamd_gemm_defer_flush": [VP],
    "otamd_gemm_defer_end": [VP],
    "otamd_gemm_defer_pending": [VP],
    "otamd_gemm_defer_stats": [VP],
    "otamd_image_to_nhwc": [VP, I, I, I, I, F, F, VP, I, VP],
    # flux.hip
    "otamd_adaln_fwd": [VP, LL, VP, LL, I, I, F, VP, LL, I, I, I, VP, VP, VP],
    "otamd_adaln_bwd": [VP, LL, VP, LL, VP, LL, I, I, VP, LL, I, I, I, VP, VP, VP, VP, VP],
    "otamd_adaln_bwd_res": [VP, LL, VP, LL, VP, LL, VP, LL, I, I, VP, LL, I, I, I, VP, VP, VP, VP, VP],
    "otamd_adaln_dmod": [VP, LL, VP, LL, I, I, LL, I, I, I, VP, VP, VP, VP, VP],
    "otamd_mod_part_floats": [I, I, I],
    "otamd_gated_add_fwd": [VP, LL, VP, LL, VP, LL, I, I, VP, LL, I, I, VP],
    "otamd_gated_add_bwd": [VP, LL, VP, LL, VP, LL, I, I, VP, LL, I, I, VP, VP, VP],
    "otamd_qk_rope_args_size": [],
    "otamd_qknorm_rope_fwd": [C.POINTER(QKRopeArgs), VP],
    "otamd_qknorm_rope_bwd": [C.POINTER(QKRopeArgs), VP, VP, VP, VP, I, I, VP, VP],
    "otamd_gelu_tanh_fwd": [VP, LL, VP, LL, I, I, VP],
    "otamd_gelu_tanh_bwd": [VP, LL, VP, LL, VP, LL, I, I, VP],
    "otamd_flux_pack": [VP, VP, I, I, I, I, I, I, VP],
    # diffusion.hip
    "otamd_noise": [VP, I, LL, LL, U64, VP],
    "otamd_noise_ex": [VP, I, LL, LL, U64, I, LL, F, F, VP],
    "otamd_noise_stream": [VP, I, LL, LL, U64, I, VP],
    "otamd_timesteps": [VP, I, LL, U64, I, I, I, I, F, F, F, VP, VP],
    "otamd_ddpm_prologue": [VP, VP, I, VP, VP, VP, VP, F, I, LL, I, I, VP, VP, I, VP, VP],
    "otamd_flow_prologue": [VP, VP, I, VP, F, F, I, I, LL, I, I, VP, VP, VP],
    "otamd_mse_loss": [VP, I, VP, I, I, LL, I, F, F, VP, VP, VP, VP, I, F, I, I, F, VP, LL, VP, VP, VP, VP],
    "otamd_mse_grad": [VP, I, VP, I, I, LL, I, VP, VP, VP, VP],
}

_lib = None


def lib():
    """Load libotamd.so once.  Raises if it is absent: there is no fallback path."""
    global _lib
    if _lib is None:
        path = LIB_PATH
        alt = os.environ.get("OTAMD_LIB_ALT")   # A/B measurements: another build of this library (tools/ab_lib.sh)
        if alt:
            path = LIB_PATH.with_name(f"libotamd_{alt}.so")
        if not path.exists():
            raise RuntimeError(f"onetrainer_amd HIP library not built: {path} missing "
                               "(run `python -m onetrainer_amd.build`); there is no CPU fallback")
        L = C.CDLL(str(path), mode=os.RTLD_NOW | os.RTLD_GLOBAL)
        for name, args in SIGNATURES.items():
            if alt and not hasattr(L, name):
                continue
            fn = getattr(L, name)
            fn.argtypes = args
            fn.restype = C.c_longlong if name.endswith(("_ws_floats", "_ws_bytes", "_slab_bytes", "_plan", "_part_floats")) else C.c_int
        if L.otamd_gemm_args_size() != C.sizeof(GemmArgs):   # an older build (or OTAMD_LIB_ALT revision) with another
            # GemmArgs layout would read the struct short and silently drop fields (e.g. the fused LoRA operands)
            raise RuntimeError(f"{path.name}: GemmArgs is {L.otamd_gemm_args_size()} bytes, this package's is "
                               f"{C.sizeof(GemmArgs)}: rebuild it (python -m onetrainer_amd.build)")
        _lib = L
    return _lib


def check(rc: int, what: str):
    if rc != OTAMD_OK:
        raise RuntimeError(f"{what}: {_ERR.get(rc, 'error')} (status {rc})")


def check_layouts():
    L = lib()
    assert L.otamd_gemm_args_size() == C.sizeof(GemmArgs), (L.otamd_gemm_args_size(), C.sizeof(GemmArgs))
    assert L.otamd_conv_geom_size() == C.sizeof(ConvGeom)
    assert L.otamd_attn_args_size() == C.sizeof(AttnArgs), (L.otamd_attn_args_size(), C.sizeof(AttnArgs))
    assert L.otamd_lora_shadow_entry_size() == C.sizeof(LoraShadowEntry)
    assert L.otamd_qk_rope_args_size() == C.sizeof(QKRopeArgs), (L.otamd_qk_rope_args_size(), C.sizeof(QKRopeArgs))
