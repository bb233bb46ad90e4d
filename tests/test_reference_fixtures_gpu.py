"""The reference's own recorded inputs/outputs (tests/golden/reference_math.npz, made by
tests/golden/make_golden.py from ModelSetupNoiseMixin / ModelSetupDiffusionMixin /
ModelSetupFlowMatchingMixin / ModelSetupDiffusionLossMixin) fed straight into the HIP kernels.

  * timestep transform: the reference's torch.rand / torch.normal draws through the kernel's
    injected-draw path -> bit-exact int timesteps (ModelSetupNoiseMixin.py:91-118,155);
  * DDPM / flow add-noise: bit-exact (the kernel's UNet input is bf16: bf16 latents compare
    bit-for-bit, fp32 latents compare against bf16(reference fp32 output));
  * per-sample losses for CONSTANT / MIN_SNR_GAMMA / DEBIASED_ESTIMATION / P2 (eps and v) and flow
    CONSTANT / SIGMA: rtol 1e-6 (fp32; only the summation order of the per-sample mean differs).
"""
from pathlib import Path

import numpy as np
import pytest
import torch

from onetrainer_amd import kernels as K

pytestmark = pytest.mark.gpu
G = np.load(Path(__file__).parent / "golden" / "reference_math.npz")
BF = torch.bfloat16


def bf16_from_bits(a, dev):
    return torch.from_numpy(a.astype(np.int16)).view(BF).to(dev)


TSINJ = {"uniform": 0, "uniform_shift3": 0, "uniform_range": 0, "logitnormal": 1, "logitnormal_b": 1,
         "logitnormal_shift": 1}


@pytest.mark.parametrize("name", list(TSINJ))
def test_timestep_kernel_on_reference_draws(dev, name):
    mn, mx, shift, bias, w = (float(v) for v in G[f"tsinj_{name}_cfg"])
    draws = torch.from_numpy(G[f"tsinj_{name}_draws"]).to(dev)
    t = K.timesteps(draws.numel(), seed=0, dist=TSINJ[name], min_s=mn, max_s=mx, shift=shift, bias=bias, weight=w,
                    device=dev, draws=draws)
    ref = torch.from_numpy(G[f"tsinj_{name}_t"])
    mism = (t.cpu() != ref).sum().item()
    assert mism == 0, f"{mism} of {ref.numel()} timesteps differ"


def _coeffs(dev):
    betas = torch.from_numpy(G["betas"])
    acp = torch.cumprod(1 - betas, 0)
    return acp.to(dev), acp.sqrt().to(dev), (1 - acp).sqrt().to(dev)


def _nhwc(a, dev):
    return torch.from_numpy(a).permute(0, 2, 3, 1).contiguous().to(dev)


@pytest.mark.parametrize("lat_dtype", ["f32", "bf16"])
def test_ddpm_add_noise_matches_reference(dev, lat_dtype):
    x0, eps = _nhwc(G["an_x0"], dev), _nhwc(G["an_eps"], dev)
    t = torch.from_numpy(G["an_t"]).to(dev, torch.int32)
    if lat_dtype == "bf16":
        x0, eps = x0.to(BF), eps.to(BF)
        ref = bf16_from_bits(G["an_ddpm_bf16"], dev).permute(0, 2, 3, 1)
    else:
        ref = torch.from_numpy(G["an_ddpm_f32"]).to(dev).permute(0, 2, 3, 1).to(BF)
    unet_in, target, _ = K.ddpm_prologue(x0, eps, t, _coeffs(dev), 1.0, 0, cpad=8)
    assert torch.equal(unet_in[..., :4], ref)
    assert torch.equal(target, eps)


@pytest.mark.parametrize("lat_dtype", ["f32", "bf16"])
def test_flow_add_noise_matches_reference(dev, lat_dtype):
    x0, eps = _nhwc(G["an_x0"], dev), _nhwc(G["an_eps"], dev)
    t = torch.from_numpy(G["an_t"]).to(dev, torch.int32)
    if lat_dtype == "bf16":
        x0, eps = x0.to(BF), eps.to(BF)
        ref = bf16_from_bits(G["an_flow_bf16"], dev).permute(0, 2, 3, 1)
    else:
        ref = torch.from_numpy(G["an_flow_f32"]).to(dev).permute(0, 2, 3, 1).to(BF)
    model_in, target = K.flow_prologue(x0, eps, t, 1.0, 0.0, 1000, cpad=4)
    assert torch.equal(model_in, ref)
    assert torch.equal(target, eps - x0)


def _loss_inputs(dev):
    pred = bf16_from_bits(G["loss_pred"], dev).permute(0, 2, 3, 1)
    pred = torch.nn.functional.pad(pred, (0, 4)).contiguous()         # 4 zero pad channels (cpad 8)
    target = _nhwc(G["loss_target"], dev)
    lw = torch.from_numpy(G["loss_lw"]).to(dev)
    t = torch.from_numpy(G["an_t"]).to(dev, torch.int32)
    return pred, target, lw, t


@pytest.mark.parametrize("fn", ["CONSTANT", "MIN_SNR_GAMMA", "DEBIASED_ESTIMATION", "P2"])
@pytest.mark.parametrize("vp", [0, 1])
def test_diffusion_loss_weights_match_reference(dev, fn, vp):
    pred, target, lw, t = _loss_inputs(dev)
    loss, coef, losses = K.mse_loss(pred, target, lw, loss_fn=K.LOSS_FN[fn], gamma=5.0, v_pred=bool(vp),
                                    timestep=t, coeffs=_coeffs(dev))
    ref = torch.from_numpy(G[f"loss_{fn}_{vp}"])
    torch.testing.assert_close(losses.cpu(), ref, rtol=1e-6, atol=0)
    torch.testing.assert_close(loss.cpu()[0], ref.mean(), rtol=1e-6, atol=0)


@pytest.mark.parametrize("fn", ["CONSTANT", "SIGMA"])
def test_flow_loss_weights_match_reference(dev, fn):
    pred, target, lw, t = _loss_inputs(dev)
    loss, coef, losses = K.mse_loss(pred, target, lw, loss_fn=K.LOSS_FN[fn], timestep=t, num_t=1000)
    ref = torch.from_numpy(G[f"flowloss_{fn}"])
    torch.testing.assert_close(losses.cpu(), ref, rtol=1e-6, atol=0)
    # gradient: d mean(losses) / d pred = 2 (p - t) w_b / (per * B), checked against autograd on the fixture
    pr = pred[..., :4].float().requires_grad_(True)
    w = lw.clone()
    if fn == "SIGMA":
        w = w * (t.float() + 1) / 1000
    ((pr - target).pow(2).mean((1, 2, 3)) * w).mean().backward()
    g = K.mse_grad(pred, target, coef)
    torch.testing.assert_close(g[..., :4].float(), pr.grad, rtol=1e-2, atol=1e-6)
