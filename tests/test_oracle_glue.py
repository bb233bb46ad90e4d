"""Pin the oracle's glue, loop and LoRA against the reference's own runs (CPU).

tests/golden/glue_fixtures.pt holds what the reference's own code produced through the stub
harness (tests/golden/make_golden_glue.py, SURVEY.md §8(c) fixtures #5 / #6 + LoRA):
  * #5 StableDiffusionXLFineTuneSetup.predict/calculate_loss (eps, v) and FluxLoRASetup.predict/
    calculate_loss: the oracle's composition (scale -> add-noise -> network input, time_ids,
    text concat, target, loss; Flux pack / img_ids / t/1000 / guidance) reproduces the recorded
    tensors bit-exactly and the loss to 1e-6;
  * #6 GenericTrainer.train(): the oracle loop (oracle UNet fp32, oracle noise / loss, global clip,
    the reference-pinned fp32 AdamW restatement, constant LR) reproduces the 3-step loss trajectory
    and the final parameters of the reference loop;
  * LoRAModuleWrapper: oracle/lora.py gives the reference's forward outputs and adapter gradients.
"""
import sys
from pathlib import Path

import numpy as np
import pytest
import torch

from oracle import adamw as OA
from oracle import diffusion as OD
from oracle import flux as OF
from oracle import lora as OL

GOLD = Path(__file__).parent / "golden"
sys.path.insert(0, str(GOLD))
import make_golden_glue as MG  # noqa: E402

FIX = torch.load(GOLD / "glue_fixtures.pt", weights_only=True)


@pytest.mark.parametrize("key", ["sdxl_epsilon_0", "sdxl_epsilon_7", "sdxl_v_prediction_0", "sdxl_v_prediction_7"])
def test_sdxl_predict_glue(key):
    f = FIX[key]
    b = MG.sdxl_batch()
    betas = OD.scaled_linear_betas()
    x0 = b["latent_image"] * 0.13025
    xt = OD.add_noise_ddpm(x0, f["noise"], f["timestep"].long(), betas)
    assert torch.equal(xt.bfloat16(), f["sample"])
    assert torch.equal(f["unet_timestep"], f["timestep"])
    tid = torch.stack([b["original_resolution"][0], b["original_resolution"][1], b["crop_offset"][0],
                       b["crop_offset"][1], b["crop_resolution"][0], b["crop_resolution"][1]], 1).float()
    assert torch.equal(tid, f["time_ids"])
    ehs = torch.cat([b["text_encoder_1_hidden_state"], b["text_encoder_2_hidden_state"]], -1).double()
    assert ehs.sum().item() == f["ehs_sum"].item() and (ehs * ehs).sum().item() == f["ehs_sumsq"].item()
    assert torch.equal(b["text_encoder_2_pooled_state"].float(), f["text_embeds"].float())
    v = f["prediction_type"] == "v_prediction"
    target = OD.get_velocity(x0, f["noise"], f["timestep"].long(), betas) if v else f["noise"]
    assert torch.equal(target, f["target"])
    pred = MG.stand_in_out(f["sample"])
    assert torch.equal(pred, f["predicted"])
    loss = OD.diffusion_losses(pred, target, b["loss_weight"]).mean()
    torch.testing.assert_close(loss, f["loss"], rtol=1e-6, atol=0)


@pytest.mark.parametrize("key", ["flux_0", "flux_3"])
def test_flux_predict_glue(key):
    f = FIX[key]
    b = MG.flux_batch()
    x0 = (b["latent_image"] - 0.1159) * 0.3611
    xt, _ = OD.add_noise_flow(x0, f["noise"], f["timestep"].long())
    assert torch.equal(OF.pack_latents(xt).bfloat16(), f["hidden_states"])
    assert torch.equal((f["timestep"] / 1000), f["model_timestep"])
    assert torch.equal(f["guidance"], torch.ones(2, dtype=torch.bfloat16))
    assert torch.equal(OF.prepare_latent_image_ids(16, 16).bfloat16(), f["img_ids"])
    assert torch.count_nonzero(f["txt_ids"]) == 0 and tuple(f["txt_ids"].shape) == (77, 3)
    assert torch.equal(b["text_encoder_1_pooled_state"], f["pooled"])
    assert torch.equal(f["noise"] - x0, f["target"])
    pred = OF.unpack_latents(MG.stand_in_out(f["hidden_states"]), 16, 16)
    assert torch.equal(pred, f["predicted"])
    loss = OD.flow_matching_losses(pred, f["target"], b["loss_weight"]).mean()
    torch.testing.assert_close(loss, f["loss"], rtol=1e-6, atol=0)


def test_lora_wrapper_matches_reference():
    f = FIX["lora"]
    net = MG.lora_net()
    ol = OL.OracleLoRA(net, rank=4, alpha=2.0, prefix="lora_unet")
    ol.load_state_dict(f["state_dict"])
    x_lin, x_conv = MG.lora_inputs()
    y_lin, y_conv = MG.lora_forward(net, x_lin, x_conv)
    torch.testing.assert_close(y_lin, f["y_lin"], rtol=1e-6, atol=1e-6)
    torch.testing.assert_close(y_conv, f["y_conv"], rtol=1e-6, atol=1e-6)
    (y_lin.square().sum() + y_conv.square().sum()).backward()
    for k, g in f["grads"].items():
        torch.testing.assert_close(ol.params[k].grad, g, rtol=1e-5, atol=1e-6)


def test_trainer_trajectory_matches_reference_loop():
    f = FIX["trainer"]
    om, _ = MG.tiny_trainer_unet()
    params = list(om.parameters())
    m = [torch.zeros_like(p) for p in params]
    v = [torch.zeros_like(p) for p in params]
    betas = OD.scaled_linear_betas()
    losses = []
    for i, b in enumerate(MG.trainer_batches()):
        t = f["timesteps"][i].long()
        x0 = b["latent_image"] * 0.13025
        xt = OD.add_noise_ddpm(x0, f["noise"][i], t, betas)
        ehs = torch.cat([b["text_encoder_1_hidden_state"], b["text_encoder_2_hidden_state"]], -1)
        tid = torch.tensor([[128.0, 128.0, 0.0, 0.0, 128.0, 128.0]] * 2)
        pred = om(xt, t, ehs, b["text_encoder_2_pooled_state"], tid)
        loss = OD.diffusion_losses(pred, f["noise"][i], b["loss_weight"]).mean()
        losses.append(loss.detach())
        om.zero_grad(set_to_none=True)
        loss.backward()
        torch.nn.utils.clip_grad_norm_(params, 1.0)
        with torch.no_grad():
            for k, p in enumerate(params):
                pn, m[k], v[k] = (torch.from_numpy(a) for a in OA.adamw_step_f32(
                    p.numpy(), p.grad.numpy(), m[k].numpy(), v[k].numpy(), i + 1, f["lr"]))
                p.copy_(pn.view_as(p))
    torch.testing.assert_close(torch.stack(losses), f["losses"], rtol=1e-6, atol=0)
    for n, p in om.named_parameters():
        scale = (p.numel() * f["param_sumsq"][n].item()) ** 0.5      # ~ sum |p|: the sum cancels
        np.testing.assert_allclose(p.detach().double().sum().item(), f["param_sum"][n].item(), rtol=0,
                                   atol=1e-6 * scale)
        np.testing.assert_allclose(p.detach().double().square().sum().item(), f["param_sumsq"][n].item(), rtol=1e-6)
