"""Pin oracle/ against the reference's own outputs (tests/golden/reference_math.npz). CPU only."""
from pathlib import Path

import numpy as np
import pytest
import torch

from oracle import adamw as OA
from oracle import diffusion as OD

G = np.load(Path(__file__).parent / "golden" / "reference_math.npz")

DISTS = {"UNIFORM": {}, "LOGIT_NORMAL": {"distribution": "LOGIT_NORMAL"},
         "UNIFORM_SHIFT3": {"shift": 3.0},
         "LOGIT_NORMAL_B": {"distribution": "LOGIT_NORMAL", "noising_bias": 0.5, "noising_weight": 0.3}}


@pytest.mark.parametrize("seed", [0, 7])
@pytest.mark.parametrize("dist", list(DISTS))
def test_noise_and_timesteps(seed, dist):
    g = torch.Generator().manual_seed(seed)
    noise = OD.create_noise((4, 4, 8, 8), g)
    t = OD.timestep_discrete(1000, 4, g, **DISTS[dist])
    assert np.array_equal(noise.numpy(), G[f"noise_{dist}_{seed}"])
    assert np.array_equal(t.numpy(), G[f"timestep_{dist}_{seed}"])
    g2 = torch.Generator().manual_seed(seed)
    assert np.array_equal(OD.timestep_continuous(4, g2, **DISTS[dist]).numpy(), G[f"tcont_{dist}_{seed}"])


@pytest.mark.parametrize("wname", ["off", "pert", "both"])
@pytest.mark.parametrize("dname", ["f32", "bf16"])
def test_offset_perturbation_noise(wname, dname):
    """oracle create_noise (-> compose_noise, which the GPU test pins the fused kernel to) equals the
    reference's _create_noise with offset / perturbation weights, bit for bit"""
    ow, pw = (float(x) for x in G[f"noisex_{wname}_w"])
    dt = torch.float32 if dname == "f32" else torch.bfloat16
    g = torch.Generator().manual_seed(11)
    noise = OD.create_noise((3, 4, 8, 8), g, dtype=dt, offset_noise_weight=ow, perturbation_noise_weight=pw)
    got = noise.numpy() if dname == "f32" else noise.view(torch.int16).numpy().astype(np.uint16)
    assert np.array_equal(got, G[f"noisex_{wname}_{dname}"])


def test_deterministic_timestep():
    assert np.array_equal(OD.timestep_discrete(1000, 4, None, deterministic=True).numpy(), G["timestep_deterministic"])


def test_betas_and_add_noise():
    betas = OD.scaled_linear_betas()
    assert np.array_equal(betas.numpy(), G["betas"])
    x0, eps, t = torch.from_numpy(G["an_x0"]), torch.from_numpy(G["an_eps"]), torch.from_numpy(G["an_t"])
    assert np.array_equal(OD.add_noise_ddpm(x0, eps, t, betas).numpy(), G["an_ddpm_f32"])
    xb = OD.add_noise_ddpm(x0.bfloat16(), eps.bfloat16(), t, betas)
    assert np.array_equal(xb.view(torch.int16).numpy().astype(np.uint16), G["an_ddpm_bf16"])
    xt, sig = OD.add_noise_flow(x0, eps, t)
    assert np.array_equal(xt.numpy(), G["an_flow_f32"]) and np.array_equal(sig.numpy(), G["an_flow_sigma"])
    xb, _ = OD.add_noise_flow(x0.bfloat16(), eps.bfloat16(), t)
    assert np.array_equal(xb.view(torch.int16).numpy().astype(np.uint16), G["an_flow_bf16"])


@pytest.mark.parametrize("fn", ["CONSTANT", "MIN_SNR_GAMMA", "DEBIASED_ESTIMATION", "P2"])
@pytest.mark.parametrize("vp", [0, 1])
def test_diffusion_losses(fn, vp):
    pred = torch.from_numpy(OA.bf16_to_f32(G["loss_pred"])).bfloat16()
    tgt, lw = torch.from_numpy(G["loss_target"]), torch.from_numpy(G["loss_lw"])
    t = torch.from_numpy(G["an_t"]).long()
    got = OD.diffusion_losses(pred, tgt, lw, t, OD.scaled_linear_betas(), fn, 5.0, bool(vp))
    np.testing.assert_allclose(got.numpy(), G[f"loss_{fn}_{vp}"], rtol=1e-6)


@pytest.mark.parametrize("fn", ["CONSTANT", "SIGMA"])
def test_flow_losses(fn):
    pred = torch.from_numpy(OA.bf16_to_f32(G["loss_pred"])).bfloat16()
    tgt, lw = torch.from_numpy(G["loss_target"]), torch.from_numpy(G["loss_lw"])
    t = torch.from_numpy(G["an_t"]).long()
    np.testing.assert_allclose(OD.flow_matching_losses(pred, tgt, lw, t, fn).numpy(), G[f"flowloss_{fn}"], rtol=1e-6)


@pytest.mark.parametrize("sr", [0, 1])
def test_adamw_bf16_bitexact(sr):
    p, m, v = G["adamw_p0"], np.zeros_like(G["adamw_p0"]), np.zeros_like(G["adamw_p0"])
    n = p.size
    for k in range(3):
        rand = None
        if sr:
            torch.manual_seed(1000 + k)
            rand = torch.randint_like(torch.zeros(n), dtype=torch.int32, low=0, high=1 << 16).numpy()
        p, m, v = OA.adamw_step_bf16(p, G[f"adamw_g{k}"], m, v, k + 1, 1e-3, rand16=rand)
        assert np.array_equal(m, G[f"adamw_sr{sr}_m{k}"]), f"m step {k}"
        assert np.array_equal(v, G[f"adamw_sr{sr}_v{k}"]), f"v step {k}"
        assert np.array_equal(p, G[f"adamw_sr{sr}_p{k}"]), f"p step {k}"


def test_adamw_f32():
    p = G["adamwf_init"]
    m = np.zeros_like(p)
    v = np.zeros_like(p)
    for k in range(3):
        p, m, v = OA.adamw_step_f32(p, G[f"adamwf_g{k}"], m, v, k + 1, 3e-4)
        np.testing.assert_allclose(p, G[f"adamwf_p{k}"], rtol=0, atol=2e-9)


def test_clip_grad_norm():
    grads = [G[f"clip_g{i}"] for i in range(3)]
    out, total, coef = OA.clip_grad_norm_bf16(grads, 1.0)
    assert total == G["clip_total"][0]
    for i in range(3):
        assert np.array_equal(out[i], G[f"clip_out{i}"])


def _sr_bits_py(seed, idx):
    m = 0xFFFFFFFF
    k = (seed ^ (seed >> 32)) & m
    x = ((idx & m) * 0x9E3779B1 + k) & m
    x ^= ((idx >> 32) * 0x85EBCA77) & m
    x ^= x >> 16
    x = (x * 0x21F0AAAD) & m
    x ^= x >> 15
    x = (x * 0x735A2D97) & m
    x ^= x >> 15
    return x >> 16


def test_sr_bits_uniform():
    b = OA.sr_bits(42, np.arange(1 << 16))
    assert b.min() >= 0 and b.max() < (1 << 16)
    assert abs(b.mean() - 32767.5) < 300
    bits = (b[:, None] >> np.arange(16)) & 1
    assert np.all(np.abs(bits.mean(0) - 0.5) < 0.01)
    # a different step seed gives an uncorrelated stream
    b2 = OA.sr_bits(0x5851F42D4C957F2D, np.arange(1 << 16))
    assert abs(np.corrcoef(b.astype(np.float64), b2.astype(np.float64))[0, 1]) < 0.02
    # numpy restatement == scalar restatement, including indices past 2^32
    idx = np.array([0, 1, 12345, (1 << 32) - 1, 1 << 32, (1 << 33) + 7], dtype=np.int64)
    for seed in (0, 42, 0xFFFFFFFFFFFFFFFF):
        got = OA.sr_bits(seed, idx)
        assert [int(v) for v in got] == [_sr_bits_py(seed, int(i)) for i in idx]


TSINJ = {"uniform": "UNIFORM", "uniform_shift3": "UNIFORM", "uniform_range": "UNIFORM", "logitnormal": "LOGIT_NORMAL",
         "logitnormal_b": "LOGIT_NORMAL", "logitnormal_shift": "LOGIT_NORMAL"}


@pytest.mark.parametrize("name", list(TSINJ))
def test_timestep_transform_on_draws(name):
    """oracle.timestep_from_draws on the reference's own draws == the reference's timesteps (bit-exact)."""
    mn, mx, shift, _bias, _w = G[f"tsinj_{name}_cfg"]
    t = OD.timestep_from_draws(torch.from_numpy(G[f"tsinj_{name}_draws"]), TSINJ[name], 1000, float(mn), float(mx),
                               float(shift))
    assert np.array_equal(t.numpy(), G[f"tsinj_{name}_t"])
