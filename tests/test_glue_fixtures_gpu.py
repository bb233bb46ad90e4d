"""The HIP plugin's predict / calculate_loss against the reference's own recorded runs
(tests/golden/glue_fixtures.pt, SURVEY.md §8(c) fixture #5; made by
tests/golden/make_golden_glue.py from StableDiffusionXLFineTuneSetup / FluxLoRASetup with
recording stand-in networks).

This build's predict() runs with the reference's noise and timesteps injected (the reference drew
them from torch's CPU generator) and the same elementwise stand-in network; everything between --
latent scaling, DDPM / flow noising, v target, time_ids, text concat, Flux 2x2 packing, t / 1000,
guidance, unpacking, the loss kernel -- is the product path.  Bit-exact for the network inputs and
targets, rtol 1e-6 for the loss.
"""
import sys
from pathlib import Path
from types import SimpleNamespace

import pytest
import torch

from onetrainer_amd.modelSetup.FluxLoRASetup import FluxLoRASetup
from onetrainer_amd.modelSetup.StableDiffusionXLFineTuneSetup import StableDiffusionXLFineTuneSetup
from onetrainer_amd.model.FluxModel import FluxModel
from onetrainer_amd.model.StableDiffusionXLModel import NoiseScheduler, StableDiffusionXLModel
from onetrainer_amd.util.config.TrainConfig import TrainConfig
from onetrainer_amd.util.TrainProgress import TrainProgress

pytestmark = pytest.mark.gpu
GOLD = Path(__file__).parent / "golden"
sys.path.insert(0, str(GOLD))
import make_golden_glue as MG  # noqa: E402

FIX = torch.load(GOLD / "glue_fixtures.pt", weights_only=True)


def _to(batch, dev):
    out = {}
    for k, v in batch.items():
        if isinstance(v, tuple):
            out[k] = tuple(t.to(dev) for t in v)
        elif isinstance(v, torch.Tensor):
            out[k] = v.to(dev)
        else:
            out[k] = v
    return out


class RecUNet:
    """this build's UNet call signature (unet_in NHWC bf16 padded, timestep, ehs, pooled, time_ids)."""
    cfg = SimpleNamespace(addition_embed=True)

    def __call__(self, x, timestep, ehs, pooled, time_ids):
        self.seen = dict(x=x.detach().clone(), timestep=timestep.clone(), ehs=ehs.clone(), pooled=pooled.clone(),
                         time_ids=time_ids.clone())
        return MG.stand_in_out(x)


class RecFlux:
    config = {"guidance_embeds": True}

    def __call__(self, tokens, t, guidance, pooled, ehs, h, w):
        self.seen = dict(tokens=tokens.detach().clone(), t=t.clone(), guidance=guidance.clone(), pooled=pooled.clone(),
                         ehs=ehs.clone())
        return MG.stand_in_out(tokens)


@pytest.mark.parametrize("key", ["sdxl_epsilon_0", "sdxl_epsilon_7", "sdxl_v_prediction_0", "sdxl_v_prediction_7"])
def test_sdxl_predict_and_loss_match_reference(dev, key):
    f = FIX[key]
    model = StableDiffusionXLModel(RecUNet(), NoiseScheduler(dev, prediction_type=f["prediction_type"]), 0.13025,
                                   model_type="STABLE_DIFFUSION_XL_10_BASE")
    # the reference's own coefficient tables: torch's CPU linspace / cumprod may round differently on
    # another host CPU, and the test is about the kernels, not about the host's table build
    tb = FIX["ddpm_tables"]
    model.noise_scheduler.coeffs = tuple(tb[k].to(dev) for k in ("alphas_cumprod", "sqrt_alphas_cumprod",
                                                                  "sqrt_one_minus_alphas_cumprod"))
    setup = StableDiffusionXLFineTuneSetup(dev)
    setup.graph_inputs = (f["noise"].permute(0, 2, 3, 1).contiguous().to(dev), f["timestep"].to(dev, torch.int32))
    cfg = TrainConfig.default_values()
    batch = _to(MG.sdxl_batch(), dev)
    out = setup.predict(model, batch, cfg, TrainProgress())
    loss = setup.calculate_loss(model, batch, out, cfg)
    s = model.unet.seen
    assert torch.equal(s["x"][..., :4].permute(0, 3, 1, 2).cpu(), f["sample"])
    assert torch.count_nonzero(s["x"][..., 4:]) == 0
    assert torch.equal(s["timestep"].cpu(), f["timestep"])
    assert torch.equal(s["time_ids"].cpu(), f["time_ids"])
    e = s["ehs"].double().cpu()
    assert tuple(s["ehs"].shape) == tuple(f["ehs_shape"]) and str(s["ehs"].dtype) == f["ehs_dtype"]
    assert e.sum().item() == f["ehs_sum"].item() and (e * e).sum().item() == f["ehs_sumsq"].item()
    assert torch.equal(s["pooled"].float().cpu(), f["text_embeds"].float())
    assert tuple(out["predicted"].shape) == (2, 4, 16, 16) and tuple(out["target"].shape) == (2, 4, 16, 16)
    assert torch.equal(out["target"].cpu(), f["target"])
    assert torch.equal(out["predicted"].cpu(), f["predicted"])
    assert out["prediction_type"] == f["prediction_type"]
    torch.testing.assert_close(loss.cpu(), f["loss"], rtol=1e-6, atol=0)


@pytest.mark.parametrize("key", ["flux_0", "flux_3"])
def test_flux_predict_and_loss_match_reference(dev, key):
    f = FIX[key]
    model = FluxModel(RecFlux())
    setup = FluxLoRASetup(dev)
    setup.graph_inputs = (f["noise"].permute(0, 2, 3, 1).contiguous().to(dev), f["timestep"].to(dev, torch.int32))
    cfg = TrainConfig.default_values()
    cfg.model_type, cfg.training_method, cfg.timestep_distribution = "FLUX_DEV_1", "LORA", "LOGIT_NORMAL"
    batch = _to(MG.flux_batch(), dev)
    out = setup.predict(model, batch, cfg, TrainProgress())
    loss = setup.calculate_loss(model, batch, out, cfg)
    s = model.transformer.seen
    B, N = 2, 64
    tok = s["tokens"].view(N, B, 64).permute(1, 0, 2).cpu()      # rows t*B + b -> [B, N, 64]
    assert torch.equal(tok, f["hidden_states"])
    assert torch.equal(s["t"].cpu(), f["model_timestep"])
    assert torch.equal(s["guidance"].to(torch.bfloat16).cpu(), f["guidance"])
    assert torch.equal(s["pooled"].cpu(), f["pooled"])
    assert s["ehs"].double().sum().item() == f["ehs_sum"].item()
    assert torch.equal(out["target"].cpu(), f["target"])
    assert torch.equal(out["predicted"].cpu(), f["predicted"])
    torch.testing.assert_close(loss.cpu(), f["loss"], rtol=1e-6, atol=0)
