"""Train-step parity: the HIP step (predict -> loss -> backward -> clip -> fused AdamW) vs the
oracle step (fp32 CPU restatement of the reference step) on a tiny SDXL-shaped UNet, with the
same weights and the same (injected) noise / timesteps."""
import pytest
import torch

from onetrainer_amd import kernels as K
from onetrainer_amd.dataLoader.SyntheticDataLoader import synthetic_sdxl_batch
from onetrainer_amd.module import unet as U
from onetrainer_amd.trainer.GenericTrainer import GenericTrainer
from onetrainer_amd.util import create
from onetrainer_amd.util.config.TrainConfig import TrainConfig
from oracle import diffusion as OD
from oracle import unet as OU

from _oracle_opt import OracleBF16AdamW, OracleMasterAdamW

pytestmark = pytest.mark.gpu


def _oracle_cfg(cfg):
    return OU.UNetConfig(**{k: getattr(cfg, k) for k in OU.UNetConfig.__dataclass_fields__})


@pytest.mark.parametrize("ptype", ["epsilon", "v_prediction"])
def test_train_step_matches_oracle(dev, ptype):
    torch.manual_seed(0)
    ucfg = U.tiny_sdxl_config()
    cfg = TrainConfig.default_values()
    cfg.batch_size = 2
    cfg.learning_rate = 1e-4
    cfg.learning_rate_warmup_steps = 0
    cfg.optimizer.stochastic_rounding = False
    model = create.create_model(cfg, dev, seed=3, unet_config=ucfg, prediction_type=ptype)
    om = OU.UNet2DConditionModel(_oracle_cfg(ucfg))
    om.load_state_dict({k: v.float().cpu() for k, v in model.unet.state_dict().items()})
    tr = GenericTrainer(cfg, model=model)
    tr.start()
    res = 128
    batch = synthetic_sdxl_batch(2, res, res, dev, seed=1, te1_dim=48, te2_dim=48, pooled_dim=64)
    opt = OracleBF16AdamW(om.parameters(), lr=1e-4, weight_decay=1e-2)   # bf16 p/m/v like the reference
    betas = OD.scaled_linear_betas()
    lat = batch["latent_image"].cpu().float()
    ehs = torch.cat([batch["text_encoder_1_hidden_state"], batch["text_encoder_2_hidden_state"]], -1).float().cpu()
    te = batch["text_encoder_2_pooled_state"].float().cpu()
    tid = torch.tensor([[res, res, 0, 0, res, res]] * 2, dtype=torch.float32)
    ours, ref, cos = [], [], []
    cap = {}
    orig = tr.model_setup.predict

    def capture(*a, **k):
        out = orig(*a, **k)
        cap["pred"] = out["predicted"].detach().float().cpu()
        return out

    tr.model_setup.predict = capture
    for step in range(3):
        gs = model.train_progress.global_step
        noise = K.noise((2, res // 8, res // 8, 4), seed=gs, dtype=torch.float32, device=dev)
        t = K.timesteps(2, seed=gs, device=dev)
        ours.append(tr.train_step(batch).item())
        # oracle: same noise / timestep (the reference draws them from torch's generator)
        eps = noise.cpu().permute(0, 3, 1, 2)
        tc = t.cpu().long()
        x0 = lat * 0.13025
        xt = OD.add_noise_ddpm(x0, eps, tc, betas)
        pred = om(xt.bfloat16().float(), tc, ehs, te, tid)
        target = eps if ptype == "epsilon" else OD.get_velocity(x0, eps, tc, betas)
        per_sample = OD.diffusion_losses(pred, target, torch.ones(2))
        loss = per_sample.mean()
        loss.backward()
        opt.step()                                   # bf16 clip_grad_norm_ + patched AdamW (pinned oracle)
        ref.append(loss.item())
        # element by element, not only the scalar: the bf16 network's prediction against the fp32 oracle's,
        # and each sample's loss (a batch mean can hide per-sample differences that cancel)
        hp = cap["pred"]
        cos.append(torch.nn.functional.cosine_similarity(hp.flatten(), pred.detach().flatten(), dim=0).item())
        hs = OD.diffusion_losses(hp, target, torch.ones(2))
        assert torch.allclose(hs, per_sample.detach(), rtol=1e-3, atol=0), (step, hs, per_sample)
        assert 0 < (hp - pred.detach()).abs().max() < 0.05, step      # bf16-sized, and not the oracle's own values
    print("losses hip", ours, "oracle", ref, "prediction cosine", cos)
    for a, b in zip(ours, ref):                      # north star: loss within rtol 1e-3 of the reference
        assert abs(a - b) <= 1e-3 * abs(b), (ours, ref)
    assert min(cos) > 0.999, cos


@pytest.mark.parametrize("weight_dtype", ["BFLOAT_16", "FLOAT_32"])
def test_sd15_train_step_matches_oracle(dev, weight_dtype):
    """SD 1.5 plugin (BaseStableDiffusionSetup.py:135-330): one text encoder, no add-embedding,
    80-wide (flash) and 160-wide (materialized) heads.  FLOAT_32: the reference's default weight dtype (C1's preset),
    fp32 master weights behind the bf16 working copy (util/dtype_util.py), against the fp32 oracle optimizer."""
    torch.manual_seed(0)
    ucfg = U.tiny_sd15_config()
    cfg = TrainConfig.default_values()
    cfg.weight_dtype = weight_dtype
    cfg.model_type = "STABLE_DIFFUSION_15"
    cfg.batch_size = 2
    cfg.learning_rate = 1e-4
    cfg.learning_rate_warmup_steps = 0
    cfg.optimizer.stochastic_rounding = False
    model = create.create_model(cfg, dev, seed=3, unet_config=ucfg)
    assert model.vae.config["scaling_factor"] == 0.18215
    om = OU.UNet2DConditionModel(_oracle_cfg(ucfg))
    om.load_state_dict({k: v.float().cpu() for k, v in model.unet.state_dict().items()})
    tr = GenericTrainer(cfg, model=model)
    tr.start()
    assert type(tr.model_setup).__name__ == "StableDiffusionFineTuneSetup"
    res = 128
    batch = synthetic_sdxl_batch(2, res, res, dev, seed=1, te1_dim=96, sdxl=False, scaling_factor=0.18215)
    master = weight_dtype == "FLOAT_32"
    assert (model.unet.store.master is not None) == master
    opt = (OracleMasterAdamW if master else OracleBF16AdamW)(om.parameters(), lr=1e-4, weight_decay=1e-2)
    betas = OD.scaled_linear_betas()
    lat = batch["latent_image"].cpu().float()
    ehs = batch["text_encoder_hidden_state"].float().cpu()
    ours, ref = [], []
    for step in range(2):
        gs = model.train_progress.global_step
        noise = K.noise((2, res // 8, res // 8, 4), seed=gs, dtype=torch.float32, device=dev)
        t = K.timesteps(2, seed=gs, device=dev)
        ours.append(tr.train_step(batch).item())
        eps = noise.cpu().permute(0, 3, 1, 2)
        tc = t.cpu().long()
        xt = OD.add_noise_ddpm(lat * 0.18215, eps, tc, betas)
        pred = om(xt.bfloat16().float(), tc, ehs)
        loss = OD.diffusion_losses(pred, eps, torch.ones(2)).mean()
        loss.backward()
        opt.step()
        ref.append(loss.item())
    print("sd15", weight_dtype, "losses hip", ours, "oracle", ref)
    for a, b in zip(ours, ref):
        assert abs(a - b) <= 1e-3 * abs(b), (ours, ref)
    if master:   # the masters carry the update below bf16 resolution; the working copy is their rne cast
        st = model.unet.store
        assert torch.equal(st.data, st.master.to(torch.bfloat16))
        assert not torch.equal(st.master, st.data.float())
        for k, v in model.unet.state_dict().items():   # the trained masters against the oracle's fp32 weights
            o = dict(om.named_parameters())[k].detach()
            assert torch.allclose(v.cpu(), o, rtol=0, atol=1e-3), k   # 2 steps of <= ~2 lr each


def test_dp_noise_slices_match_global(dev):
    """rank r's predict() draws exactly samples [r*b, (r+1)*b) of the global batch's noise."""
    from onetrainer_amd.modelSetup.BaseStableDiffusionXLSetup import BaseStableDiffusionXLSetup
    g = K.noise((4, 16, 16, 4), seed=9, dtype=torch.float32, device=dev)
    s1 = BaseStableDiffusionXLSetup(dev, dp_rank=1, dp_world=2)
    off = s1.dp_rank * 2 * 16 * 16 * 4
    assert torch.equal(K.noise((2, 16, 16, 4), seed=9, offset=off, dtype=torch.float32, device=dev), g[2:])


def test_offset_perturbation_noise_step(dev):
    """with offset / perturbation noise on (ModelSetupNoiseMixin.py:31-46) predict() draws the fused noise_ex
    noise (pinned to the reference's composition in test_kernels_gpu) and the step trains"""
    cfg = TrainConfig.default_values()
    cfg.batch_size = 2
    cfg.offset_noise_weight, cfg.perturbation_noise_weight = 0.1, 0.05
    model = create.create_model(cfg, dev, seed=3, unet_config=U.tiny_sdxl_config())
    tr = GenericTrainer(cfg, model=model)
    tr.start()
    batch = synthetic_sdxl_batch(2, 128, 128, dev, seed=1, te1_dim=48, te2_dim=48, pooled_dim=64)
    gs = model.train_progress.global_step
    noise, _ = tr.model_setup.step_inputs(model, batch, cfg, model.train_progress)
    shape = tuple(noise.shape)
    assert torch.equal(noise, K.noise_ex(shape, seed=gs, offset_weight=0.1, perturbation_weight=0.05, dtype=noise.dtype,
                                         device=dev))
    assert not torch.equal(noise, K.noise(shape, seed=gs, dtype=noise.dtype, device=dev))
    losses = [tr.train_step(batch).item() for _ in range(2)]
    assert all(l == l and abs(l) < 1e4 for l in losses), losses


def test_step_graph_matches_eager(dev, monkeypatch):
    """the captured + replayed step (trainer/step_graph.py) is bit-identical to the eager step:
    losses, every parameter and the AdamW moments over 4 steps, with a second batch shape in the
    middle (its own capture, sharing the graph memory pool)."""
    ucfg = U.tiny_sdxl_config()

    def run(graphs: bool):
        monkeypatch.setenv("OTAMD_STEP_GRAPH", "1" if graphs else "0")   # opt-in
        cfg = TrainConfig.default_values()
        cfg.batch_size = 2
        cfg.learning_rate = 1e-4
        cfg.learning_rate_warmup_steps = 0
        model = create.create_model(cfg, dev, seed=3, unet_config=ucfg)
        tr = GenericTrainer(cfg, model=model)
        tr.start()
        assert (tr.graphs is not None) == graphs
        a = synthetic_sdxl_batch(2, 128, 128, dev, seed=1, te1_dim=48, te2_dim=48, pooled_dim=64)
        b = synthetic_sdxl_batch(2, 96, 160, dev, seed=2, te1_dim=48, te2_dim=48, pooled_dim=64)
        a2 = {k: (v.clone() if torch.is_tensor(v) else v) for k, v in a.items()}   # same shape, other buffers
        losses = [tr.train_step(x).clone() for x in (a, a, b, b, a2, b, a)]
        torch.cuda.synchronize()
        opt = model.optimizer
        return (torch.stack(losses).cpu(), model.unet.store.data.clone(),
                torch.cat([opt.exp_avg.float(), opt.exp_avg_sq.float()]), tr)

    l0, p0, s0, _ = run(False)
    l1, p1, s1, tr1 = run(True)
    assert len(tr1.graphs.entries) == 2
    assert torch.equal(l0, l1), (l0, l1)
    assert torch.equal(p0, p1)
    assert torch.equal(s0, s1)


def test_full_sdxl_steps_bitwise_repeatable(dev):
    """The step is deterministic under its real concurrency (weight-gradient stream, split-K slabs, the one-pass
    cross-attention backward's LDS hand-offs, the optimizer's overlapped chunks): the full SDXL UNet at 512^2 b=2,
    three steps from the same seed, run twice, gives bit-identical parameters, moments and losses.  A missing
    LDS-write fence before a barrier showed up exactly here (run-to-run loss drift), not in the per-kernel tests."""
    def run():
        cfg = TrainConfig.default_values()
        cfg.batch_size = 2
        cfg.learning_rate = 1e-4
        cfg.learning_rate_warmup_steps = 0
        tr = GenericTrainer(cfg, seed=0)
        tr.start()
        batch = synthetic_sdxl_batch(2, 512, 512, dev, seed=1)
        losses = [tr.train_step(batch).float() for _ in range(3)]
        st = tr.model.train_store
        st.wait_params()
        torch.cuda.synchronize()
        out = (torch.stack(losses).cpu(), st.data.clone(), tr.model.optimizer.exp_avg.clone())
        del tr
        torch.cuda.empty_cache()
        return out

    a, b = run(), run()
    assert torch.equal(a[0], b[0]), (a[0], b[0])
    assert torch.equal(a[1], b[1]) and torch.equal(a[2], b[2])
