"""FLUX.1 full fine-tune plugin (mirrors modules/modelSetup/FluxFineTuneSetup.py): every transformer
parameter trainable (bf16), fused AdamW(+SR) over the transformer's flat store."""
from __future__ import annotations

import torch

from ..util.dtype_util import dtype_plan
from ..util.NamedParameterGroup import NamedParameterGroup, NamedParameterGroupCollection
from ..util.optimizer.adamw_fused import FusedAdamW
from ..util.optimizer_util import restore_training_state
from .BaseFluxSetup import BaseFluxSetup
from ..util.config.plain import plain


class FluxFineTuneSetup(BaseFluxSetup):
    def create_parameters(self, model, config) -> NamedParameterGroupCollection:
        config = plain(config)
        pgc = NamedParameterGroupCollection()
        if config.text_encoder.train or config.text_encoder_2.train:
            raise NotImplementedError("text-encoder training is outside this build's hot path (text is cached)")
        if config.prior.train:
            pgc.add_group(NamedParameterGroup("transformer", model.transformer.parameters(),
                                              config.prior.learning_rate))
        return pgc

    def setup_optimizations(self, model, config):
        config = plain(config)
        model.dtype_plan = dtype_plan(config)   # util/dtype_util.py: the config's dtypes honoured, overridden or refused
        model.train_dtype = torch.bfloat16

    def setup_model(self, model, config):
        config = plain(config)
        self.setup_optimizations(model, config)
        params = self.create_parameters(model, config)
        model.parameters = params
        oc = config.optimizer
        if oc.optimizer != "ADAMW":
            raise NotImplementedError(f"optimizer {oc.optimizer}: only ADAMW is on the hot path")
        model.optimizer = FusedAdamW(model.transformer.store, params.parameters_for_optimizer(config),
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
        pass
