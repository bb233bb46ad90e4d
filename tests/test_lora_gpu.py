"""LoRA on the GPU: the fused second-K-segment GEMMs vs fp32 torch, and a frozen-base LoRA UNet
forward/backward vs the oracle UNet with the reference LoRA hooks (oracle/lora.py)."""
import pytest
import torch
import torch.nn.functional as F

from onetrainer_amd import kernels as K
from onetrainer_amd.module import unet as U
from onetrainer_amd.module.lora import LoRAUNetWrapper
from oracle import unet as OU
from oracle.lora import OracleLoRA

pytestmark = pytest.mark.gpu
BF = torch.bfloat16


def rnd(*s, dev, scale=1.0):
    return (torch.randn(*s, device=dev) * scale).to(BF)


def close(out, ref, tol=2e-2):
    err = (out.float() - ref).abs().max().item()
    scale = ref.abs().max().item() + 1e-6
    assert err / scale < tol, f"max err {err} vs scale {scale}"


@pytest.mark.parametrize("M,K_,N,r", [(300, 640, 320, 32), (257, 72, 128, 32), (1024, 1280, 3840, 96)])
def test_linear_lora_segment(dev, M, K_, N, r):
    torch.manual_seed(0)
    x, w, b = rnd(M, K_, dev=dev), rnd(N, K_, dev=dev, scale=0.05), rnd(N, dev=dev)
    res = rnd(M, N, dev=dev)
    a, up = rnd(r, K_, dev=dev, scale=0.05), rnd(N, r, dev=dev, scale=0.05)
    t = K.linear(x, a)
    y = K.linear(x, w, bias=b, residual=res, lora=(t, up))
    ref = x.float() @ w.float().t() + b.float() + res.float() + t.float() @ up.float().t()
    close(y, ref)
    # dgrad with the adapter's second segment: dx = dy W + u A
    dy = rnd(M, N, dev=dev)
    u = K.linear_dgrad(dy, up)
    close(u, dy.float() @ up.float())
    dx = K.linear_dgrad(dy, w, lora=(u, a))
    close(dx, dy.float() @ w.float() + u.float() @ a.float())


@pytest.mark.parametrize("N_,H,W,Cin,Cout,stride,up2x", [(2, 16, 16, 64, 128, 1, False), (2, 16, 16, 64, 64, 2, False),
                                                         (1, 8, 8, 128, 64, 1, True), (2, 16, 16, 8, 64, 1, False)])
def test_conv_lora_segment(dev, N_, H, W, Cin, Cout, stride, up2x):
    torch.manual_seed(1)
    r = 32
    x = rnd(N_, H, W, Cin, dev=dev)
    w, b = rnd(Cout, 3, 3, Cin, dev=dev, scale=0.05), rnd(Cout, dev=dev)
    d, upw = rnd(r, 3, 3, Cin, dev=dev, scale=0.05), rnd(Cout, r, dev=dev, scale=0.05)
    t = K.conv2d(x, d, stride=stride, upsample=up2x)
    y = K.conv2d(x, w, bias=b, stride=stride, upsample=up2x, lora=(t, upw))
    xr = x.permute(0, 3, 1, 2).float()
    if up2x:
        xr = F.interpolate(xr, scale_factor=2.0, mode="nearest")
    ref = F.conv2d(xr, w.permute(0, 3, 1, 2).float(), b.float(), stride=stride, padding=1)
    ref = ref + F.conv2d(t.permute(0, 3, 1, 2).float(), upw.float()[:, :, None, None])
    close(y, ref.permute(0, 2, 3, 1))


def _cos(a, b):
    a, b = a.flatten().double(), b.flatten().double()
    return (a @ b / (a.norm() * b.norm() + 1e-30)).item()


def test_lora_unet_matches_oracle(dev):
    torch.manual_seed(0)
    cfg = U.tiny_sdxl_config()
    m = U.UNet2DConditionModel(cfg, dev, seed=1, trainable=False)
    om = OU.UNet2DConditionModel(OU.UNetConfig(**{k: getattr(cfg, k) for k in OU.UNetConfig.__dataclass_fields__}))
    om.load_state_dict({k: v.float().cpu() for k, v in m.state_dict().items()})
    om.requires_grad_(False)
    lw = LoRAUNetWrapper(m, rank=8, alpha=4.0, seed=0)
    m.lora = lw
    ol = OracleLoRA(om, 8, 4.0)
    g = torch.Generator().manual_seed(3)
    sd = {k: (torch.randn(v.shape, generator=g) * 0.1 if not k.endswith(".alpha") else v)
          for k, v in lw.state_dict().items()}
    lw.load_state_dict(sd)
    ol.load_state_dict({k: v for k, v in lw.state_dict().items() if not k.endswith(".alpha")})
    B, H, W = 2, 16, 16
    x = torch.randn(B, 4, H, W)
    t = torch.tensor([10, 700], dtype=torch.int32)
    ehs = torch.randn(B, 77, cfg.cross_attention_dim)
    te = torch.randn(B, cfg.projection_class_embeddings_input_dim - 6 * cfg.addition_time_embed_dim)
    tid = torch.tensor([[128., 128., 0., 0., 128., 128.]] * B)
    xin = torch.zeros(B, H, W, 8, dtype=BF, device=dev)
    xin[..., :4] = x.permute(0, 2, 3, 1).to(dev).bfloat16()
    out = m(xin, t.to(dev), ehs.to(dev).bfloat16(), te.to(dev).bfloat16(), tid.to(dev))
    ref = om(x.bfloat16().float(), t, ehs.bfloat16().float(), te.bfloat16().float(), tid)
    o4 = out[..., :4].float().cpu()
    r4 = ref.permute(0, 2, 3, 1)
    assert _cos(o4, r4.detach()) > 0.999
    wgt = torch.randn(B, H, W, 4)
    lw.store.begin_backward()
    (out[..., :4].float() * wgt.to(dev)).sum().backward()
    lw.store.finish_backward()
    (r4 * wgt).sum().backward()
    gs = lw.state_dict(grads=True)
    worst = []
    for k, p in ol.params.items():
        c = _cos(gs[k].float().cpu().reshape(p.shape), p.grad)
        worst.append((c, k))
    worst.sort()
    print("worst LoRA grad cosines:", worst[:5])
    assert worst[0][0] > 0.99, worst[:5]
    assert m.store.grad is None     # frozen base: no base gradient buffer at all


def test_lora_train_steps(dev):
    from onetrainer_amd.dataLoader.SyntheticDataLoader import synthetic_sdxl_batch
    from onetrainer_amd.trainer.GenericTrainer import GenericTrainer
    from onetrainer_amd.util import create
    from onetrainer_amd.util.config.TrainConfig import TrainConfig

    ucfg = U.tiny_sdxl_config()
    cfg = TrainConfig.default_values()
    cfg.training_method = "LORA"
    cfg.batch_size = 2
    cfg.learning_rate = 3e-4
    cfg.learning_rate_warmup_steps = 0
    cfg.lora_rank, cfg.lora_alpha = 8, 8.0
    model = create.create_model(cfg, dev, seed=3, unet_config=ucfg)
    tr = GenericTrainer(cfg, model=model)
    tr.start()
    base0 = model.unet.store.data.clone()
    lora0 = model.unet_lora.store.data.clone()
    batch = synthetic_sdxl_batch(2, 128, 128, dev, seed=1, te1_dim=48, te2_dim=48, pooled_dim=64)
    losses = [tr.train_step(batch).item() for _ in range(2)]
    assert all(torch.isfinite(torch.tensor(losses)))
    assert torch.equal(model.unet.store.data, base0)                      # frozen base untouched
    ups = [n for n in model.unet_lora.store.order if n.endswith("lora_up.weight")]
    s = model.unet_lora.store.slots[ups[0]]
    assert torch.count_nonzero(model.unet_lora.store.data[s.offset:s.offset + s.numel]) > 0
    assert not torch.equal(model.unet_lora.store.data, lora0)


def test_sdxl_lora_trajectory_matches_oracle(dev):
    """C4's path at test size: 3 SDXL LoRA train steps (frozen bf16 base, fp32 r8 adapters on every
    Linear / Conv2d, fp32 AdamW) against the oracle UNet with the reference LoRA hooks
    (LoRAModule.py:283-323) and the pinned fp32 AdamW restatement (adamw_extensions.py:17-150), on the
    same weights, noise and timesteps: every step's loss at rtol 1e-3 (the adapters' up weights start
    at zero, so steps 2 and 3 carry the trained adapters)."""
    from _oracle_opt import OracleF32AdamW
    from onetrainer_amd.dataLoader.SyntheticDataLoader import synthetic_sdxl_batch
    from onetrainer_amd.trainer.GenericTrainer import GenericTrainer
    from onetrainer_amd.util import create
    from onetrainer_amd.util.config.TrainConfig import TrainConfig
    from oracle import diffusion as OD

    ucfg = U.tiny_sdxl_config()
    cfg = TrainConfig.default_values()
    cfg.training_method = "LORA"
    cfg.batch_size = 2
    cfg.learning_rate = 3e-4
    cfg.learning_rate_warmup_steps = 0
    cfg.lora_rank, cfg.lora_alpha = 8, 8.0
    cfg.optimizer.stochastic_rounding = False
    model = create.create_model(cfg, dev, seed=3, unet_config=ucfg)
    tr = GenericTrainer(cfg, model=model)
    tr.start()
    om = OU.UNet2DConditionModel(OU.UNetConfig(**{k: getattr(ucfg, k) for k in OU.UNetConfig.__dataclass_fields__}))
    om.load_state_dict({k: v.float().cpu() for k, v in model.unet.state_dict().items()})
    om.requires_grad_(False)
    ol = OracleLoRA(om, 8, 8.0)
    ol.load_state_dict({k: v.float().cpu() for k, v in model.unet_lora.state_dict().items() if not k.endswith(".alpha")})
    assert len(ol.params) == len([k for k in model.unet_lora.state_dict() if not k.endswith(".alpha")])
    opt = OracleF32AdamW(ol.parameters(), lr=3e-4, weight_decay=1e-2)
    res = 128
    batch = synthetic_sdxl_batch(2, res, res, dev, seed=1, te1_dim=48, te2_dim=48, pooled_dim=64)
    betas = OD.scaled_linear_betas()
    lat = batch["latent_image"].cpu().float()
    ehs = torch.cat([batch["text_encoder_1_hidden_state"], batch["text_encoder_2_hidden_state"]], -1).float().cpu()
    te = batch["text_encoder_2_pooled_state"].float().cpu()
    tid = torch.tensor([[res, res, 0, 0, res, res]] * 2, dtype=torch.float32)
    base0 = model.unet.store.data.clone()
    ours, ref = [], []
    for step in range(3):
        gs = model.train_progress.global_step
        noise = K.noise((2, res // 8, res // 8, 4), seed=gs, dtype=torch.float32, device=dev)
        t = K.timesteps(2, seed=gs, device=dev)
        ours.append(tr.train_step(batch).item())
        eps = noise.cpu().permute(0, 3, 1, 2)
        tc = t.cpu().long()
        xt = OD.add_noise_ddpm(lat * 0.13025, eps, tc, betas)
        pred = om(xt.bfloat16().float(), tc, ehs, te, tid)
        loss = OD.diffusion_losses(pred, eps, torch.ones(2)).mean()
        loss.backward()
        opt.step()
        ref.append(loss.item())
    print("sdxl lora losses hip", ours, "oracle", ref)
    for a, b in zip(ours, ref):
        assert abs(a - b) <= 1e-3 * abs(b), (ours, ref)
    assert ref[1] != ref[0] and ours[2] != ours[1]
    assert torch.equal(model.unet.store.data, base0)
