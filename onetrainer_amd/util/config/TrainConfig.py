"""TrainConfig subset consumed by the hot path, loadable from the reference's own JSON.

Mirrors modules/util/config/TrainConfig.py (defaults at 759-995, optimizer part 114-195) for
exactly the fields the train step reads; unknown keys of a reference config /
training preset are kept in `extra` and ignored, so `training_presets/#sdxl 1.0.json` and a
reference `config.json` load unchanged.  New build-only knobs (data-parallel, bench) live in
their own fields with defaults that keep the reference behaviour.
"""
from __future__ import annotations

import json
from dataclasses import dataclass, field, fields


@dataclass
class OptimizerConfig:
    optimizer: str = "ADAMW"
    beta1: float | None = None
    beta2: float | None = None
    eps: float | None = None
    weight_decay: float | None = None
    stochastic_rounding: bool = True
    fused_back_pass: bool = False
    foreach: bool | None = False
    fused: bool | None = False


@dataclass
class ModelPartConfig:
    train: bool = True
    learning_rate: float | None = None
    weight_dtype: str = "NONE"
    dropout_probability: float = 0.0
    guidance_scale: float = 1.0          # prior (Flux) only: TrainConfig.py:228
    attention_mask: bool = False


@dataclass
class TrainConfig:
    model_type: str = "STABLE_DIFFUSION_XL_10_BASE"
    training_method: str = "FINE_TUNE"
    train_device: str = "cuda"
    temp_device: str = "cpu"
    # the build trains bf16 (util/dtype_util.py); the reference's defaults are FLOAT_16 / FLOAT_32
    # (TrainConfig.py:782,816), which util/dtype_util.dtype_plan overrides or refuses with a recorded reason
    train_dtype: str = "BFLOAT_16"
    fallback_train_dtype: str = "BFLOAT_16"
    enable_autocast_cache: bool = True
    weight_dtype: str = "BFLOAT_16"
    resolution: str = "1024"
    batch_size: int = 1
    aspect_ratio_bucketing: bool = True       # TrainConfig.py:795
    latent_caching: bool = True
    cache_dir: str = "workspace-cache/run"
    gradient_accumulation_steps: int = 1
    epochs: int = 100
    learning_rate: float = 3e-6
    learning_rate_scheduler: str = "CONSTANT"
    learning_rate_warmup_steps: float = 200.0
    learning_rate_cycles: float = 1.0
    learning_rate_min_factor: float = 0.0
    learning_rate_scaler: str = "NONE"
    clip_grad_norm: float | None = 1.0
    # noise / timesteps (ModelSetupNoiseMixin)
    offset_noise_weight: float = 0.0
    perturbation_noise_weight: float = 0.0
    timestep_distribution: str = "UNIFORM"
    min_noising_strength: float = 0.0
    max_noising_strength: float = 1.0
    noising_weight: float = 0.0
    noising_bias: float = 0.0
    timestep_shift: float = 1.0
    dynamic_timestep_shifting: bool = False
    # loss (ModelSetupDiffusionLossMixin)
    mse_strength: float = 1.0
    mae_strength: float = 0.0
    log_cosh_strength: float = 0.0
    vb_loss_strength: float = 1.0
    loss_weight_fn: str = "CONSTANT"
    loss_weight_strength: float = 5.0
    loss_scaler: str = "NONE"
    masked_training: bool = False
    # LoRA
    lora_rank: int = 16
    lora_alpha: float = 1.0
    lora_weight_dtype: str = "FLOAT_32"
    lora_layers: str = ""
    lora_layer_preset: str | None = None
    lora_decompose: bool = False
    peft_type: str = "LORA"
    dropout_probability: float = 0.0          # LoRA dropout (TrainConfig.py:828)
    # parts
    optimizer: OptimizerConfig = field(default_factory=OptimizerConfig)
    unet: ModelPartConfig = field(default_factory=ModelPartConfig)
    text_encoder: ModelPartConfig = field(default_factory=lambda: ModelPartConfig(train=False))
    text_encoder_2: ModelPartConfig = field(default_factory=lambda: ModelPartConfig(train=False))
    vae: ModelPartConfig = field(default_factory=lambda: ModelPartConfig(train=False))
    prior: ModelPartConfig = field(default_factory=ModelPartConfig)
    # model names, output, backups (TrainConfig.py base_model_name / output_* / backup fields)
    base_model_name: str = ""
    vae_model_name: str = ""
    lora_model_name: str = ""
    output_model_destination: str = "models/model.safetensors"   # TrainConfig.py:783-785
    output_model_format: str = "SAFETENSORS"
    output_dtype: str = "FLOAT_32"
    workspace_dir: str = "workspace/run"
    continue_last_backup: bool = False
    # periodic backups / saves (TrainConfig.py:981-989)
    backup_after: float = 30
    backup_after_unit: str = "MINUTE"
    rolling_backup: bool = False
    rolling_backup_count: int = 3
    backup_before_save: bool = True
    save_every: int = 0
    save_every_unit: str = "NEVER"
    save_skip_first: int = 0
    save_filename_prefix: str = ""
    # concepts (TrainConfig.py:793-794): inline list of ConceptConfig dicts, else the concept file
    concepts: list | None = None
    concept_file_name: str = "training_concepts/concepts.json"
    # build-only (not in the reference): data parallel gradient bucket size / fp32 reduction
    dp_bucket_mb: int = 256
    dp_reduce_fp32: bool = False
    extra: dict = field(default_factory=dict)

    @staticmethod
    def default_values() -> "TrainConfig":
        """the build's defaults: bf16 weights and bf16 compute (what SURVEY.md §8(d)'s C2-C5 configure)"""
        return TrainConfig()

    @staticmethod
    def reference_defaults() -> "TrainConfig":
        """the reference's TrainConfig.default_values() for the fields where the build's defaults differ
        (TrainConfig.py:782,816-817: weight_dtype FLOAT_32, train_dtype FLOAT_16): the starting point of a
        reference JSON config (scripts/train.py), so a preset that leaves a dtype unset gets the reference's
        value and util/dtype_util.dtype_plan records or refuses what the build does with it"""
        c = TrainConfig()
        c.weight_dtype, c.train_dtype, c.fallback_train_dtype = "FLOAT_32", "FLOAT_16", "BFLOAT_16"
        return c

    def from_dict(self, d: dict) -> "TrainConfig":
        names = {f.name: f for f in fields(self)}
        for k, v in d.items():
            if k in names and k != "extra":
                cur = getattr(self, k)
                if isinstance(cur, (OptimizerConfig, ModelPartConfig)) and isinstance(v, dict):
                    for kk, vv in v.items():
                        if hasattr(cur, kk):
                            setattr(cur, kk, vv)
                else:
                    setattr(self, k, v)
            else:
                self.extra[k] = v
        return self

    @staticmethod
    def load(path: str) -> "TrainConfig":
        with open(path) as f:
            return TrainConfig().from_dict(json.load(f))

    def model_names(self):
        from ..ModelNames import ModelNames
        return ModelNames(base_model=self.base_model_name, vae_model=self.vae_model_name, lora=self.lora_model_name)

    def get_last_backup_path(self) -> str | None:
        """newest directory under <workspace>/backup by name (TrainConfig.py:704-717)."""
        import os
        root = os.path.join(self.workspace_dir, "backup")
        if os.path.exists(root):
            dirs = sorted((d for d in os.listdir(root) if os.path.isdir(os.path.join(root, d))), reverse=True)
            if dirs:
                return os.path.join(root, dirs[0])
        return None

    def to_settings_dict(self) -> dict:
        from dataclasses import asdict
        d = asdict(self)
        d.update(d.pop("extra"))
        return d

    def resolution_hw(self) -> tuple[int, int]:
        r = str(self.resolution)
        if "x" in r:
            h, w = r.split("x")
            return int(h), int(w)
        return int(r), int(r)
