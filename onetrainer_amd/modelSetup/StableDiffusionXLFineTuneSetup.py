"""Full fine-tune plugin (mirrors modules/modelSetup/StableDiffusionXLFineTuneSetup.py:26-164):
parameter groups, optimizer creation (create.py:509-534 -> FusedAdamW), device placement."""
from __future__ import annotations

import torch

from ..util.dtype_util import dtype_plan
from ..util.NamedParameterGroup import NamedParameterGroup, NamedParameterGroupCollection
from ..util.optimizer.adamw_fused import FusedAdamW
from ..util.optimizer_util import restore_training_state
from .BaseStableDiffusionXLSetup import BaseStableDiffusionXLSetup
from ..util.config.plain import plain


class StableDiffusionXLFineTuneSetup(BaseStableDiffusionXLSetup):
    def create_parameters(self, model, config) -> NamedParameterGroupCollection:
        config = plain(config)
        pgc = NamedParameterGroupCollection()
        if config.unet.train:
            pgc.add_group(NamedParameterGroup("unet", model.unet.parameters(), config.unet.learning_rate))
        if config.text_encoder.train or config.text_encoder_2.train:
            raise NotImplementedError("text-encoder training is outside this build's hot path (text is cached)")
        return pgc

    def setup_optimizations(self, model, config):
        # no gradient checkpointing: 288 GB HBM holds every activation;
        # no autocast: the kernels fix the compute dtype (bf16 GEMMs, fp32 norms/softmax/loss)
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
        model.optimizer = FusedAdamW(model.unet.store, params.parameters_for_optimizer(config),
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
        pass   # model and data are created on the train device

    def after_optimizer_step(self, model, config, train_progress):
        config = plain(config)
        pass
