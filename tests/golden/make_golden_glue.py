"""Golden fixtures from the reference's own setup / trainer / LoRA code (container only).

    python tests/golden/make_golden_glue.py      -> tests/golden/glue_fixtures.pt

Runs, through the stub harness of SURVEY.md Appendix A (tests/golden/ref_harness.py):
  #5  StableDiffusionXLFineTuneSetup.predict + calculate_loss (epsilon, v_prediction) and
      FluxLoRASetup.predict + calculate_loss (LOGIT_NORMAL) with recording stand-in networks
      (modules/modelSetup/BaseStableDiffusionXLSetup.py:179-373, BaseFluxSetup.py:193-390);
  #6  GenericTrainer.train() for 3 steps (modules/trainer/GenericTrainer.py:568-764) with the
      oracle UNet restatement (oracle/unet.py, tiny config, fp32) as model.unet;
  LoRA: LoRAModuleWrapper (modules/module/LoRAModule.py:283-323,427-587) on a tiny Linear +
      Conv2d net: forward outputs and adapter gradients.
Only data is stored (inputs are regenerated from seeds by the functions below); no reference
source.  The fixtures pin oracle/ (tests/test_oracle_glue.py) and the HIP glue
(tests/test_glue_fixtures_gpu.py).
"""
from __future__ import annotations

import sys
from pathlib import Path

import torch

HERE = Path(__file__).resolve().parent
ROOT = HERE.parents[1]
OUT = HERE / "glue_fixtures.pt"


# ---------------------------------------------------------------------------------------------
# inputs, regenerated identically by the tests
def sdxl_batch(B=2, h=16, w=16, te1=768, te2=1280, res=128):
    g = torch.Generator().manual_seed(11)
    lat = torch.randn(B, 4, h, w, generator=g) / 0.13025
    hw = lambda v: torch.full((B,), v, dtype=torch.int64)  # noqa: E731
    return {"latent_image": lat,
            "text_encoder_1_hidden_state": torch.randn(B, 77, te1, generator=g).bfloat16(),
            "text_encoder_2_hidden_state": torch.randn(B, 77, te2, generator=g).bfloat16(),
            "text_encoder_2_pooled_state": torch.randn(B, te2, generator=g).bfloat16(),
            "original_resolution": (hw(res + 64), hw(res)), "crop_offset": (hw(8), hw(0)),
            "crop_resolution": (hw(res), hw(res)), "loss_weight": torch.tensor([1.0, 0.75])[:B],
            "tokens_1": torch.zeros(B, 77, dtype=torch.int64), "tokens_2": torch.zeros(B, 77, dtype=torch.int64),
            "concept_type": ["STANDARD"] * B}


def flux_batch(B=2, h=16, w=16):
    g = torch.Generator().manual_seed(12)
    return {"latent_image": torch.randn(B, 16, h, w, generator=g),
            "text_encoder_1_pooled_state": torch.randn(B, 768, generator=g).bfloat16(),
            "text_encoder_2_hidden_state": torch.randn(B, 77, 256, generator=g).bfloat16(),
            "loss_weight": torch.tensor([1.0, 2.0])[:B], "concept_type": ["STANDARD"] * B}


def stand_in_out(x: torch.Tensor) -> torch.Tensor:
    """the recording networks' output: elementwise, exactly reproducible in bf16 on any device."""
    return x * 0.5 + 0.25


def lora_net():
    torch.manual_seed(21)
    net = torch.nn.Module()
    net.lin = torch.nn.Linear(16, 24)
    net.conv = torch.nn.Conv2d(8, 12, 3, padding=1)
    net.down = torch.nn.Conv2d(12, 6, 3, stride=2, padding=1)
    return net


def lora_inputs():
    g = torch.Generator().manual_seed(22)
    return torch.randn(3, 16, generator=g), torch.randn(2, 8, 10, 10, generator=g)


def lora_forward(net, x_lin, x_conv):
    return net.lin(x_lin), net.down(net.conv(x_conv))


def tiny_trainer_unet():
    sys.path.insert(0, str(ROOT))
    from oracle import unet as OU
    torch.manual_seed(5)
    cfg = OU.tiny_sdxl_config()
    m = OU.UNet2DConditionModel(cfg)
    with torch.no_grad():
        for p in m.parameters():
            p.copy_(torch.randn(p.shape) * 0.05)
    return m, cfg


def trainer_batches(n=3, B=2, res=128):
    out = []
    for i in range(n):
        g = torch.Generator().manual_seed(100 + i)
        hw = lambda v: torch.full((B,), v, dtype=torch.int64)  # noqa: E731
        out.append({"latent_image": torch.randn(B, 4, res // 8, res // 8, generator=g) / 0.13025,
                    "text_encoder_1_hidden_state": torch.randn(B, 77, 48, generator=g),
                    "text_encoder_2_hidden_state": torch.randn(B, 77, 48, generator=g),
                    "text_encoder_2_pooled_state": torch.randn(B, 64, generator=g),
                    "original_resolution": (hw(res), hw(res)), "crop_offset": (hw(0), hw(0)),
                    "crop_resolution": (hw(res), hw(res)), "loss_weight": torch.ones(B),
                    "tokens_1": torch.zeros(B, 77, dtype=torch.int64),
                    "tokens_2": torch.zeros(B, 77, dtype=torch.int64), "concept_type": ["STANDARD"] * B})
    return out


# ---------------------------------------------------------------------------------------------
def main():
    sys.path.insert(0, str(HERE))
    import ref_harness
    ref_harness.install()
    from types import SimpleNamespace

    from modules.model.FluxModel import FluxModel
    from modules.model.StableDiffusionXLModel import StableDiffusionXLModel
    from modules.modelSetup.FluxLoRASetup import FluxLoRASetup
    from modules.modelSetup.StableDiffusionXLFineTuneSetup import StableDiffusionXLFineTuneSetup
    from modules.module.LoRAModule import LoRAModuleWrapper
    from modules.util.config.TrainConfig import TrainConfig
    from modules.util.enum.DataType import DataType
    from modules.util.enum.ModelType import ModelType
    from modules.util.enum.TimestepDistribution import TimestepDistribution
    from modules.util.TrainProgress import TrainProgress

    class AttrDict(dict):
        __getattr__ = dict.__getitem__

    betas = torch.linspace(0.00085 ** 0.5, 0.012 ** 0.5, 1000, dtype=torch.float32) ** 2
    acp = torch.cumprod(1 - betas, 0)

    class DDIM:
        def __init__(self, ptype):
            self.config = AttrDict(num_train_timesteps=1000, prediction_type=ptype)
            self.betas, self.alphas_cumprod = betas, acp

        def get_velocity(self, sample, noise, timesteps):   # diffusers DDIMScheduler.get_velocity
            a = self.alphas_cumprod.to(dtype=sample.dtype)
            sa = (a[timesteps] ** 0.5).flatten()
            sb = ((1 - a[timesteps]) ** 0.5).flatten()
            while sa.dim() < sample.dim():
                sa, sb = sa.unsqueeze(-1), sb.unsqueeze(-1)
            return sa * noise - sb * sample

    rec: dict = {}
    from modules.util.DiffusionScheduleCoefficients import DiffusionScheduleCoefficients
    co = DiffusionScheduleCoefficients.from_betas(betas)   # the tables _add_noise_discrete / get_velocity index
    rec["ddpm_tables"] = {"alphas_cumprod": co.alphas_cumprod, "sqrt_alphas_cumprod": co.sqrt_alphas_cumprod,
                          "sqrt_one_minus_alphas_cumprod": co.sqrt_one_minus_alphas_cumprod}
    assert torch.equal(co.alphas_cumprod, acp)

    # ---- #5 SDXL predict + loss ------------------------------------------------------------------
    class RecUNet(torch.nn.Module):
        def forward(self, sample, timestep, encoder_hidden_states, added_cond_kwargs):
            self.seen = {"sample": sample.detach().clone(), "timestep": timestep.detach().clone(),
                         "ehs": encoder_hidden_states.detach().clone(),
                         "text_embeds": added_cond_kwargs["text_embeds"].detach().clone(),
                         "time_ids": added_cond_kwargs["time_ids"].detach().clone()}
            return SimpleNamespace(sample=stand_in_out(sample))

    for ptype in ("epsilon", "v_prediction"):
        for step in (0, 7):
            model = StableDiffusionXLModel(ModelType.STABLE_DIFFUSION_XL_10_BASE)
            model.vae = torch.nn.Module()
            model.vae.config = {"scaling_factor": 0.13025}
            model.text_encoder_1, model.text_encoder_2 = torch.nn.Module(), torch.nn.Module()
            model.train_dtype = DataType.BFLOAT_16
            model.unet = RecUNet()
            model.noise_scheduler = DDIM(ptype)
            cfg = TrainConfig.default_values()
            cfg.train_device = cfg.temp_device = "cpu"
            cfg.model_type = ModelType.STABLE_DIFFUSION_XL_10_BASE
            cfg.text_encoder.train = cfg.text_encoder_2.train = False
            setup = StableDiffusionXLFineTuneSetup(torch.device("cpu"), torch.device("cpu"), False)
            tp = TrainProgress()
            tp.global_step = step
            batch = sdxl_batch()
            out = setup.predict(model, batch, cfg, tp)
            loss = setup.calculate_loss(model, batch, out, cfg)
            g = torch.Generator().manual_seed(step)       # the draw _create_noise made first
            noise = torch.randn(batch["latent_image"].shape, generator=g, dtype=batch["latent_image"].dtype)
            if ptype == "epsilon":
                assert torch.equal(noise, out["target"])
            s = model.unet.seen
            e = s["ehs"].double()
            rec[f"sdxl_{ptype}_{step}"] = {
                "noise": noise, "timestep": out["timestep"], "sample": s["sample"], "unet_timestep": s["timestep"],
                "ehs_dtype": str(s["ehs"].dtype), "ehs_shape": tuple(s["ehs"].shape),
                "ehs_sum": e.sum(), "ehs_sumsq": (e * e).sum(), "text_embeds": s["text_embeds"],
                "time_ids": s["time_ids"], "predicted": out["predicted"].detach(), "target": out["target"],
                "prediction_type": out["prediction_type"], "loss": loss.detach()}

    # ---- #5 Flux LoRA predict + loss ------------------------------------------------------------
    class RecFlux(torch.nn.Module):
        config = SimpleNamespace(guidance_embeds=True)

        def forward(self, hidden_states, timestep, guidance, pooled_projections, encoder_hidden_states, txt_ids,
                    img_ids, joint_attention_kwargs=None, return_dict=True):
            self.seen = {"hidden_states": hidden_states.detach().clone(), "model_timestep": timestep.detach().clone(),
                         "guidance": guidance.detach().clone(), "pooled": pooled_projections.detach().clone(),
                         "ehs_sum": encoder_hidden_states.double().sum(), "txt_ids": txt_ids.detach().clone(),
                         "img_ids": img_ids.detach().clone()}
            return SimpleNamespace(sample=stand_in_out(hidden_states))

    for step in (0, 3):
        model = FluxModel(ModelType.FLUX_DEV_1)
        model.vae = torch.nn.Module()
        model.vae.config = {"scaling_factor": 0.3611, "shift_factor": 0.1159}
        model.text_encoder_1, model.text_encoder_2 = torch.nn.Module(), torch.nn.Module()
        model.train_dtype = DataType.BFLOAT_16
        model.transformer = RecFlux()
        model.noise_scheduler = SimpleNamespace(config=AttrDict(num_train_timesteps=1000),
                                                timesteps=torch.arange(1000), sigmas=torch.zeros(1000))
        cfg = TrainConfig.default_values()
        cfg.train_device = cfg.temp_device = "cpu"
        cfg.model_type = ModelType.FLUX_DEV_1
        cfg.timestep_distribution = TimestepDistribution.LOGIT_NORMAL
        cfg.text_encoder.train = cfg.text_encoder_2.train = False
        setup = FluxLoRASetup(torch.device("cpu"), torch.device("cpu"), False)
        tp = TrainProgress()
        tp.global_step = step
        batch = flux_batch()
        out = setup.predict(model, batch, cfg, tp)
        loss = setup.calculate_loss(model, batch, out, cfg)
        g = torch.Generator().manual_seed(step)
        noise = torch.randn(batch["latent_image"].shape, generator=g)
        rec[f"flux_{step}"] = {"noise": noise, "timestep": out["timestep"], **model.transformer.seen,
                               "predicted": out["predicted"].detach(), "target": out["target"],
                               "loss": loss.detach()}

    # ---- LoRA wrapper -----------------------------------------------------------------------------
    net = lora_net()
    c = TrainConfig.default_values()
    c.lora_rank, c.lora_alpha = 4, 2.0
    torch.manual_seed(23)
    w = LoRAModuleWrapper(net, "lora_unet", c)
    with torch.no_grad():
        for k, p in w.state_dict().items():
            if k.endswith("lora_up.weight"):
                for m in w.lora_modules.values():
                    if m.prefix + "lora_up.weight" == k:
                        m.lora_up.weight.copy_(torch.randn(m.lora_up.weight.shape) * 0.1)
    w.hook_to_module()
    x_lin, x_conv = lora_inputs()
    y_lin, y_conv = lora_forward(net, x_lin, x_conv)
    (y_lin.square().sum() + y_conv.square().sum()).backward()
    rec["lora"] = {"state_dict": {k: v.detach().clone() for k, v in w.state_dict().items()},
                   "y_lin": y_lin.detach(), "y_conv": y_conv.detach(),
                   "grads": {m.prefix + n: p.grad.detach().clone() for m in w.lora_modules.values()
                             for n, p in (("lora_down.weight", m.lora_down.weight), ("lora_up.weight", m.lora_up.weight))}}

    # ---- #6 GenericTrainer.train() trajectory ------------------------------------------------------
    from modules.trainer.GenericTrainer import GenericTrainer
    from modules.util.callbacks.TrainCallbacks import TrainCallbacks
    from modules.util.commands.TrainCommands import TrainCommands
    from modules.util.enum.TimeUnit import TimeUnit
    from modules.util.NamedParameterGroup import NamedParameterGroup, NamedParameterGroupCollection
    from modules.util.optimizer_util import init_model_parameters

    om, ocfg = tiny_trainer_unet()

    class UNetAdapter(torch.nn.Module):
        """diffusers call signature over the oracle UNet; records what the trainer fed it."""

        def __init__(self, m):
            super().__init__()
            self.m = m
            self.calls = []

        def forward(self, sample, timestep, encoder_hidden_states, added_cond_kwargs):
            self.calls.append({"timestep": timestep.detach().clone()})
            y = self.m(sample.float(), timestep.long(), encoder_hidden_states.float(),
                       added_cond_kwargs["text_embeds"].float(), added_cond_kwargs["time_ids"].float())
            return SimpleNamespace(sample=y)

    cfg = TrainConfig.default_values()
    cfg.train_device = cfg.temp_device = "cpu"
    cfg.model_type = ModelType.STABLE_DIFFUSION_XL_10_BASE
    cfg.train_dtype = DataType.FLOAT_32
    cfg.weight_dtype = DataType.FLOAT_32
    cfg.text_encoder.train = cfg.text_encoder_2.train = False
    cfg.learning_rate = 1e-4
    cfg.learning_rate_warmup_steps = 0
    cfg.batch_size = 2
    cfg.epochs = 1
    cfg.tensorboard = False
    import tempfile
    cfg.workspace_dir = tempfile.mkdtemp(prefix="otamd_glue_")
    cfg.cache_dir = cfg.workspace_dir + "/cache"
    for unit in ("sample_after_unit", "backup_after_unit", "save_every_unit"):
        if hasattr(cfg, unit):
            setattr(cfg, unit, TimeUnit.NEVER)
    model = StableDiffusionXLModel(ModelType.STABLE_DIFFUSION_XL_10_BASE)
    model.vae = torch.nn.Module()
    model.vae.config = {"scaling_factor": 0.13025}
    model.text_encoder_1, model.text_encoder_2 = torch.nn.Module(), torch.nn.Module()
    model.train_dtype = DataType.FLOAT_32
    model.unet = UNetAdapter(om)
    model.noise_scheduler = DDIM("epsilon")
    params = NamedParameterGroupCollection()
    params.add_group(NamedParameterGroup("unet", list(om.parameters()), cfg.learning_rate))
    model.train_config = cfg
    init_model_parameters(model, params, torch.device("cpu"))
    setup = StableDiffusionXLFineTuneSetup(torch.device("cpu"), torch.device("cpu"), False)
    losses = []
    orig_loss = setup.calculate_loss

    def rec_loss(*a, **k):
        lv = orig_loss(*a, **k)
        losses.append(lv.detach().clone())
        return lv
    setup.calculate_loss = rec_loss
    batches = trainer_batches()

    class FakeDataSet:
        def start_next_epoch(self):
            pass

        def approximate_length(self):
            return len(batches)

    class FakeLoader:
        def get_data_set(self):
            return FakeDataSet()

        def get_data_loader(self):
            return iter(batches)

    tr = GenericTrainer(cfg, TrainCallbacks(), TrainCommands())
    tr.model, tr.model_setup, tr.data_loader = model, setup, FakeLoader()
    tr.parameters = list(om.parameters())
    tr.sample_queue = []
    tr.train()
    rec["trainer"] = {"losses": torch.stack(losses), "timesteps": [c["timestep"] for c in model.unet.calls],
                      "noise": [torch.randn(b["latent_image"].shape, generator=torch.Generator().manual_seed(i))
                                for i, b in enumerate(batches)],
                      "param_sum": {n: p.detach().double().sum() for n, p in om.named_parameters()},
                      "param_sumsq": {n: p.detach().double().square().sum() for n, p in om.named_parameters()},
                      "lr": cfg.learning_rate}
    torch.save(rec, OUT)
    print("wrote", OUT, sorted(rec))


if __name__ == "__main__":
    main()
