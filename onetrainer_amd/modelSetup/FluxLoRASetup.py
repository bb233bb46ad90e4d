"""FLUX.1 LoRA plugin (mirrors modules/modelSetup/FluxLoRASetup.py): frozen bf16 transformer, fp32
adapters on every Linear matching `lora_layers` (presets FluxLoRASetup.py:12-16), parameter group
"transformer" (prior.learning_rate), fused fp32 AdamW over the adapter store, bf16 shadow refreshed
after each update."""
from __future__ import annotations

import torch

from ..util.dtype_util import dtype_plan
from ..module.lora import LoRAWrapper
from ..util.NamedParameterGroup import NamedParameterGroup, NamedParameterGroupCollection
from ..util.optimizer.adamw_fused import FusedAdamW
from ..util.optimizer_util import restore_training_state
from .BaseFluxSetup import BaseFluxSetup
from ..util.config.plain import plain

PRESETS = {"attn-mlp": ["attn", "ff.net"], "attn-only": ["attn"], "full": []}


class FluxLoRASetup(BaseFluxSetup):
    @staticmethod
    def layer_filter(config):
        config = plain(config)
        if config.lora_layers:
            return config.lora_layers.split(",")
        return PRESETS.get(config.lora_layer_preset or "full", [])

    def create_parameters(self, model, config) -> NamedParameterGroupCollection:
        config = plain(config)
        pgc = NamedParameterGroupCollection()
        if config.text_encoder.train or config.text_encoder_2.train:
            raise NotImplementedError("text-encoder LoRA is outside this build's hot path (text is cached)")
        if config.prior.train:
            pgc.add_group(NamedParameterGroup("transformer", model.transformer_lora.parameters(),
                                              config.prior.learning_rate))
        return pgc

    def setup_optimizations(self, model, config):
        config = plain(config)
        model.dtype_plan = dtype_plan(config)   # util/dtype_util.py: the config's dtypes honoured, overridden or refused
        model.train_dtype = torch.bfloat16

    def setup_model(self, model, config):
        config = plain(config)
        if getattr(config, "lora_decompose", False) or config.peft_type != "LORA":
            raise NotImplementedError("DoRA / LoHa are not on this build's hot path")
        if config.dropout_probability and config.dropout_probability > 0:
            raise NotImplementedError("LoRA dropout > 0 is not on this build's hot path")
        if model.transformer.store.trainable:
            raise ValueError("LoRA training needs a frozen base transformer (create_model(..., training_method='LORA'))")
        self.setup_optimizations(model, config)
        if model.transformer_lora is None:
            model.transformer_lora = LoRAWrapper(model.transformer, rank=config.lora_rank, alpha=config.lora_alpha,
                                                 module_filter=self.layer_filter(config), prefix="lora_transformer",
                                                 seed=0)
        if getattr(model, "lora_state_dict", None) is not None:   # LoRA file / backup (LoRALoaderMixin)
            model.transformer_lora.load_state_dict(model.lora_state_dict)
            model.lora_state_dict = None
        model.transformer.lora = model.transformer_lora
        params = self.create_parameters(model, config)
        model.parameters = params
        oc = config.optimizer
        if oc.optimizer != "ADAMW":
            raise NotImplementedError(f"optimizer {oc.optimizer}: only ADAMW is on the hot path")
        model.optimizer = FusedAdamW(model.transformer_lora.store, params.parameters_for_optimizer(config),
                                     lr=config.learning_rate,
                                     betas=(oc.beta1 if oc.beta1 is not None else 0.9,
                                            oc.beta2 if oc.beta2 is not None else 0.999),
                                     eps=oc.eps if oc.eps is not None else 1e-8,
                                     weight_decay=oc.weight_decay if oc.weight_decay is not None else 1e-2,
                                     stochastic_rounding=oc.stochastic_rounding)
        model.param_group_mapping = params.unique_name_mapping()
        restore_training_state(model, config)

    def setup_train_device(self, model, config):
        config = plain(config)
        pass

    def after_optimizer_step(self, model, config, train_progress):
        config = plain(config)
        model.transformer_lora.refresh()
