"""The compute / storage dtype policy: what the reference decides from a config, and what this build does.

Reference (read from the config):
  * the network's compute dtype is `train_dtype` -- create_autocast_context (modules/util/dtype_util.py:28-49)
    returns it whether autocast is on (weights of several dtypes, or one that differs) or off (one weight dtype
    equal to train_dtype); the setups call it with the UNet / prior, text-encoder, VAE and LoRA weight dtypes
    (BaseStableDiffusionXLSetup.py:54-61, BaseFluxSetup.py:58-65);
  * per-part storage dtypes: `TrainConfig.weight_dtypes()` (TrainConfig.py:627-647), the part's own
    `weight_dtype` unless it is NONE, else the top-level `weight_dtype`; LoRA adapters `lora_weight_dtype`;
  * a GradScaler when train_dtype is FLOAT_16 and every trainable parameter is fp32
    (dtype_util.py:18-20, GenericTrainer.py:579);
  * defaults (TrainConfig.py:782, 816-817): weight FLOAT_32, train FLOAT_16, fallback BFLOAT_16.

This build's kernels compute in bf16 (MFMA bf16 inputs, fp32 accumulation; norms, softmax and the loss in
fp32) and store the trained network in bf16 (full fine-tune, bf16 weights), in fp32 master weights behind a bf16
working copy (full fine-tune, FLOAT_32 weights: module/param_store.py `master`, csrc/adamw.hip
adamw_master_kernel), or keep a frozen bf16 base plus fp32 adapters (LoRA).  `dtype_plan(cfg)` maps a config
onto that:
  * the same decision as the reference -> taken;
  * a decision that only changes precision in a direction the build supports -> taken with an OVERRIDE
    record (field, reference value, build value, reason), logged once by the trainer and kept on the model
    (`model.dtype_plan`): FLOAT_16 compute -> BFLOAT_16 (SURVEY.md §8(d) C3 prescribes exactly this); a frozen
    base in FLOAT_16 / FLOAT_32 / a quantized format -> stored BFLOAT_16 (autocast casts frozen weights to the
    compute dtype anyway; NF4 / int8 need bitsandbytes, CUDA-only); bf16 / fp16 adapters -> kept fp32; the
    reference's GradScaler -> not needed with bf16 compute;
  * a decision the build cannot honour -> ValueError before any weight is allocated: fp32 / tf32 compute, a
    trained network in a quantized format.
fp32 master weights for a full fine-tune (TrainConfig.default_values() and the SD 1.5 preset) are honoured: the
reference holds fp32 weights and autocast casts them to bf16 (round to nearest) for every GEMM, and their
gradients are those bf16 GEMM results cast to fp32; the build keeps fp32 p / m / v, bf16 gradients and a bf16
working copy rewritten by the optimizer launch.  One deviation is recorded: norm-layer gradients, which autocast
computes in fp32 (group_norm / layer_norm run in fp32), are rounded to bf16 by the shared gradient store.
"""
from __future__ import annotations

from dataclasses import dataclass, field

from .config.plain import plain

QUANTIZED = ("NFLOAT_4", "INT_8", "FLOAT_8")
BF16 = "BFLOAT_16"


def _flux(cfg) -> bool:
    return str(cfg.model_type).startswith("FLUX")


def _part(cfg, name):
    try:
        return getattr(cfg, name)
    except AttributeError:
        return None


def resolved_weight_dtypes(cfg) -> dict:
    """TrainConfig.weight_dtypes() (TrainConfig.py:627-647) for the parts the hot path has"""
    cfg = plain(cfg)
    top = cfg.weight_dtype
    out = {}
    for name in ("unet", "prior", "text_encoder", "text_encoder_2", "vae"):
        p = _part(cfg, name)
        wd = getattr(p, "weight_dtype", "NONE") if p is not None else "NONE"
        out[name] = top if wd in ("NONE", None) else wd
    lw = getattr(cfg, "lora_weight_dtype", "NONE")
    out["lora"] = top if lw in ("NONE", None) else lw
    return out


def reference_decision(cfg) -> dict:
    """what the reference runs the network in for this config: {compute, autocast, grad_scaler, network,
    adapters} (dtype_util.create_autocast_context / enable_grad_scaling as the setups call them)"""
    cfg = plain(cfg)
    w = resolved_weight_dtypes(cfg)
    lora = cfg.training_method == "LORA"
    net = w["prior"] if _flux(cfg) else w["unet"]
    listed = [net, w["text_encoder"], w["text_encoder_2"], w["vae"]] + ([w["lora"]] if lora else [])
    listed = {d for d in listed if d not in ("NONE", None)}
    autocast = not (len(listed) == 1 and cfg.train_dtype in listed)
    trainable = w["lora"] if lora else net
    return {"compute": cfg.train_dtype, "autocast": autocast,
            "grad_scaler": cfg.train_dtype == "FLOAT_16" and trainable == "FLOAT_32",
            "network": net, "adapters": w["lora"] if lora else None}


@dataclass
class DtypePlan:
    compute: str = BF16
    network: str = BF16            # trained (fine-tune) or frozen (LoRA) network storage
    adapters: str | None = None    # LoRA adapter storage
    master: bool = False           # fp32 master weights behind a bf16 working copy (full fine-tune, FLOAT_32)
    overrides: list = field(default_factory=list)   # [{field, reference, build, reason}]

    def summary(self) -> str:
        if not self.overrides:
            return "dtypes as configured (bf16 compute)"
        return "; ".join(f"{o['field']} {o['reference']} -> {o['build']} ({o['reason']})" for o in self.overrides)


def dtype_plan(cfg) -> DtypePlan:
    """the build's dtypes for this config, with every deviation from the reference recorded; ValueError for a
    config this build cannot train as configured"""
    cfg = plain(cfg)
    ref = reference_decision(cfg)
    lora = cfg.training_method == "LORA"
    net_field = ("prior" if _flux(cfg) else "unet") + ".weight_dtype"
    plan = DtypePlan(adapters="FLOAT_32" if lora else None)

    c = ref["compute"]
    if c in ("FLOAT_32", "TFLOAT_32"):
        raise ValueError(f"train_dtype {c}: this build computes the network in bf16 MFMA kernels, fp32 compute is not "
                         f"built; set train_dtype to BFLOAT_16")
    if c == "FLOAT_16":
        plan.overrides.append({"field": "train_dtype", "reference": c, "build": BF16,
                               "reason": "bf16 MFMA kernels, same rate as fp16, fp32 exponent range (SURVEY.md §8(d) C3)"})
    elif c != BF16:
        raise ValueError(f"train_dtype {c} is not a compute dtype this build supports (BFLOAT_16, or FLOAT_16 -> bf16)")

    n = ref["network"]
    if not lora:
        if n == "FLOAT_32":
            plan.network, plan.master = "FLOAT_32", True
            plan.overrides.append({"field": "norm gradients", "reference": "FLOAT_32", "build": BF16,
                                   "reason": "fp32 master weights; GroupNorm / LayerNorm weight gradients pass through "
                                             "the bf16 gradient store (every GEMM gradient is bf16-exact anyway)"})
        elif n in QUANTIZED:
            raise ValueError(f"{net_field} {n}: a quantized network cannot be fine-tuned")
        elif n == "FLOAT_16":
            plan.overrides.append({"field": net_field, "reference": n, "build": BF16,
                                   "reason": "bf16 storage of the trained network (no fp16 kernels)"})
        elif n != BF16:
            raise ValueError(f"{net_field} {n} is not supported")
    elif n != BF16:
        why = ("quantized base formats need bitsandbytes (CUDA-only, out of scope)" if n in QUANTIZED else
               "frozen base stored in the bf16 compute dtype (autocast casts it to the compute dtype anyway)")
        plan.overrides.append({"field": net_field, "reference": n, "build": BF16, "reason": why})

    if lora and ref["adapters"] != "FLOAT_32":
        plan.overrides.append({"field": "lora_weight_dtype", "reference": ref["adapters"], "build": "FLOAT_32",
                               "reason": "adapters kept in fp32 (fp32 AdamW state, bf16 shadow for the GEMMs)"})
    if ref["grad_scaler"]:
        plan.overrides.append({"field": "grad_scaler", "reference": "on", "build": "off",
                               "reason": "bf16 compute needs no loss scaling"})
    return plan
