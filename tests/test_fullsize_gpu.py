"""The real architectures and the BASELINE configs C1-C5 on the GPU.

Oracle comparisons at full width (oracle/unet.py, oracle/flux.py on the host CPU, fp32, same
weights, same bf16-rounded inputs, same injected noise / timesteps):
  * SDXL `sdxl_config()` (320/640/1280, depth [0,2,10], ctx 2048) at 512^2 b=1 and at C3's own resolution,
    1024^2 b=1 (level-1 self-attention over 4096 tokens, the step's hottest attention shape);
  * SD 1.5 `sd15_config()` (8 heads of 40/80/160, ctx 768) at 512^2 b=1 -- C1's shape;
  * FLUX.1 at full width (D = 3072, 24 x 128 heads, T5 ctx 4096) with 1 double + 1 single block at
    768^2 b=1 (2304 image tokens + 77 text tokens).
  * the SDXL UNet with C4's rank-32 LoRA on every Linear / Conv2d (oracle/lora.py hooks) at 512^2 b=1, and the
    full-width FLUX blocks with C5's rank-16 LoRA on every Linear at 768^2 b=1.
  Each checks the diffusion loss to rtol 1e-3 (north star), the prediction's element-wise cosine and every
  parameter (adapter) gradient's cosine.

Full-size property steps at the BASELINE workloads (too large for a CPU oracle):
  * C2 SD 1.5 FT 512^2 b=16, C3 SDXL FT 1024^2 b=4 (per-rank batch of the DP-8 config),
    C4 SDXL LoRA r32 over two aspect buckets (1024^2, 1152x896), C5 FLUX.1 LoRA r16 768^2 b=4:
  finite loss in a sane range, finite gradients, a second step moves the trained parameters, and
  for LoRA the frozen base is bit-for-bit untouched.
"""
import math

import pytest
import torch

from onetrainer_amd import kernels as K
from onetrainer_amd.dataLoader.SyntheticDataLoader import synthetic_flux_batch, synthetic_sdxl_batch
from onetrainer_amd.module import flux as FX
from onetrainer_amd.module import unet as U
from onetrainer_amd.trainer.GenericTrainer import GenericTrainer
from onetrainer_amd.util import create
from onetrainer_amd.util.config.TrainConfig import TrainConfig
from oracle import diffusion as OD
from oracle import flux as OF
from oracle import unet as OU

pytestmark = pytest.mark.gpu


def _cos(a, b):
    a, b = a.flatten().double(), b.flatten().double()
    return (a @ b / (a.norm() * b.norm() + 1e-30)).item()


def _oracle_unet(cfg, hip):
    with torch.device("meta"):
        om = OU.UNet2DConditionModel(OU.UNetConfig(**{k: getattr(cfg, k) for k in OU.UNetConfig.__dataclass_fields__}))
    om = om.to_empty(device="cpu")
    om.load_state_dict({k: v.float().cpu() for k, v in hip.state_dict().items()})
    return om


def _free():
    import gc
    gc.collect()
    torch.cuda.empty_cache()


@pytest.mark.parametrize("name,res", [("sdxl", 512), ("sd15", 512), ("sdxl", 1024)])
def test_full_unet_matches_oracle(dev, name, res):
    torch.set_num_threads(max(1, min(16, torch.get_num_threads())))
    cfg = U.sdxl_config() if name == "sdxl" else U.sd15_config()
    m = U.UNet2DConditionModel(cfg, dev, seed=1)
    om = _oracle_unet(cfg, m)
    g = torch.Generator().manual_seed(0)
    B, h = 1, res // 8
    x0 = torch.randn(B, 4, h, h, generator=g)
    eps = torch.randn(B, 4, h, h, generator=g)
    t = torch.tensor([517], dtype=torch.int32)
    ehs = torch.randn(B, 77, cfg.cross_attention_dim, generator=g).bfloat16()
    if cfg.addition_embed:
        te = torch.randn(B, 1280, generator=g).bfloat16()
        tid = torch.tensor([[float(res), float(res), 0., 0., float(res), float(res)]])
    else:
        te = tid = None
    xt = OD.add_noise_ddpm(x0, eps, t.long(), OD.scaled_linear_betas()).bfloat16()
    xin = torch.zeros(B, h, h, 8, dtype=torch.bfloat16)
    xin[..., :4] = xt.permute(0, 2, 3, 1)
    out = m(xin.to(dev), t.to(dev), ehs.to(dev), None if te is None else te.to(dev),
            None if tid is None else tid.to(dev))
    loss, coef, _ = K.mse_loss(out, eps.permute(0, 2, 3, 1).contiguous().to(dev))
    ref = om(xt.float(), t.long(), ehs.float(), None if te is None else te.float(), tid)
    ref_loss = OD.diffusion_losses(ref, eps, torch.ones(B)).mean()
    pred = out[..., :4].float().cpu().permute(0, 3, 1, 2)
    pcos = _cos(pred, ref.detach())
    print(f"{name} {res}^2 loss hip {loss.item():.6f} oracle {ref_loss.item():.6f} prediction cosine {pcos:.6f}")
    assert abs(loss.item() - ref_loss.item()) <= 1e-3 * abs(ref_loss.item())
    assert pcos > 0.999, pcos
    m.store.begin_backward()
    out.backward(K.mse_grad(out, eps.permute(0, 2, 3, 1).contiguous().to(dev), coef))
    m.store.finish_backward()
    ref_loss.backward()
    gh = m.state_dict(grads=True)
    cos = sorted((_cos(gh[n].float().cpu(), p.grad), n) for n, p in om.named_parameters())
    print("worst grad cosines:", cos[:4])
    assert cos[0][0] > 0.98, cos[:4]
    assert sum(c for c, _ in cos) / len(cos) > 0.999
    del m, om
    _free()


def test_full_width_sdxl_lora_r32_matches_oracle(dev):
    """C4's adapter set at full width: the SDXL UNet (frozen bf16 base) with rank-32 LoRA on every Linear / Conv2d
    (module/lora.py: fused down / block-diagonal up, second-K-segment GEMMs, deferred split-K weight-gradient reduces)
    against the oracle UNet with the reference LoRA hooks (oracle/lora.py; LoRAModule.py:283-323) at 512^2 b=1:
    diffusion loss to rtol 1e-3, the prediction's cosine, and every adapter gradient's cosine."""
    from onetrainer_amd.module.lora import LoRAUNetWrapper
    from oracle.lora import OracleLoRA
    torch.set_num_threads(max(1, min(16, torch.get_num_threads())))
    cfg = U.sdxl_config()
    m = U.UNet2DConditionModel(cfg, dev, seed=1, trainable=False)
    om = _oracle_unet(cfg, m)
    om.requires_grad_(False)
    rank, alpha = 32, 16.0
    lw = LoRAUNetWrapper(m, rank=rank, alpha=alpha, seed=0)
    m.lora = lw
    ol = OracleLoRA(om, rank, alpha)
    g = torch.Generator().manual_seed(3)
    # random up weights too (the reference initialises them to zero): every adapter then shapes the output and
    # receives a gradient through both of its factors
    sd = {k: (torch.randn(v.shape, generator=g) * (0.02 if "lora_up" in k else 0.05) if not k.endswith(".alpha") else v)
          for k, v in lw.state_dict().items()}
    lw.load_state_dict(sd)
    ol.load_state_dict({k: v for k, v in lw.state_dict().items() if not k.endswith(".alpha")})
    B, h, res = 1, 64, 512
    x0 = torch.randn(B, 4, h, h, generator=g)
    eps = torch.randn(B, 4, h, h, generator=g)
    t = torch.tensor([311], dtype=torch.int32)
    ehs = torch.randn(B, 77, cfg.cross_attention_dim, generator=g).bfloat16()
    te = torch.randn(B, 1280, generator=g).bfloat16()
    tid = torch.tensor([[float(res), float(res), 0., 0., float(res), float(res)]])
    xt = OD.add_noise_ddpm(x0, eps, t.long(), OD.scaled_linear_betas()).bfloat16()
    xin = torch.zeros(B, h, h, 8, dtype=torch.bfloat16)
    xin[..., :4] = xt.permute(0, 2, 3, 1)
    out = m(xin.to(dev), t.to(dev), ehs.to(dev), te.to(dev), tid.to(dev))
    loss, coef, _ = K.mse_loss(out, eps.permute(0, 2, 3, 1).contiguous().to(dev))
    ref = om(xt.float(), t.long(), ehs.float(), te.float(), tid)
    ref_loss = OD.diffusion_losses(ref, eps, torch.ones(B)).mean()
    pcos = _cos(out[..., :4].float().cpu().permute(0, 3, 1, 2), ref.detach())
    print(f"sdxl lora r32 512^2 loss hip {loss.item():.6f} oracle {ref_loss.item():.6f} prediction cosine {pcos:.6f}")
    assert abs(loss.item() - ref_loss.item()) <= 1e-3 * abs(ref_loss.item())
    assert pcos > 0.999, pcos
    lw.store.begin_backward()
    out.backward(K.mse_grad(out, eps.permute(0, 2, 3, 1).contiguous().to(dev), coef))
    lw.store.finish_backward()
    ref_loss.backward()
    gs = lw.state_dict(grads=True)
    cos = sorted((_cos(gs[k].float().cpu().reshape(p.shape), p.grad), k) for k, p in ol.params.items())
    print(f"{len(cos)} adapter tensors; worst grad cosines:", cos[:4])
    assert len(cos) > 1500
    assert cos[0][0] > 0.98, cos[:4]
    assert sum(c for c, _ in cos) / len(cos) > 0.999
    assert m.store.grad is None
    del m, om, lw, ol
    _free()


def test_full_width_flux_blocks_768_match_oracle(dev):
    cfg = FX.FluxConfig(num_layers=1, num_single_layers=1)
    ocfg = OF.FluxConfig(num_layers=1, num_single_layers=1)
    m = FX.FluxTransformer2DModel(cfg, dev, seed=1, trainable=True)
    with torch.device("meta"):
        om = OF.FluxTransformer2DModel(ocfg)
    om = om.to_empty(device="cpu")
    om.load_state_dict({k: v.float().cpu() for k, v in m.state_dict().items()})
    g = torch.Generator().manual_seed(0)
    B, h = 1, 96
    lat = torch.randn(B, 16, h, h, generator=g)
    eps = torch.randn(B, 16, h, h, generator=g)
    t = torch.tensor([611], dtype=torch.int32)
    pooled = torch.randn(B, 768, generator=g).bfloat16()
    ehs = torch.randn(B, 77, 4096, generator=g).bfloat16()
    x0 = (lat - 0.1159) * 0.3611
    xt, _ = OD.add_noise_flow(x0, eps, t.long())
    xin = xt.bfloat16().permute(0, 2, 3, 1).contiguous().to(dev)
    tok = K.flux_pack(xin)
    out_tok = m(tok, t.float().to(dev) / 1000, torch.ones(B, device=dev), pooled.to(dev), ehs.to(dev), h, h)
    out = K.flux_unpack(out_tok.contiguous(), B, h, h, 16)
    target = (eps - x0).permute(0, 2, 3, 1).contiguous().to(dev)
    loss, coef, _ = K.mse_loss(out, target)
    ref = om(OF.pack_latents(xt.bfloat16().float()), t.float() / 1000, torch.ones(B), pooled.float(), ehs.float(),
             torch.zeros(77, 3), OF.prepare_latent_image_ids(h, h))
    ref = OF.unpack_latents(ref, h, h)
    ref_loss = OD.flow_matching_losses(ref, eps - x0, torch.ones(B)).mean()
    print(f"flux D=3072 1+1 blocks 768^2 loss hip {loss.item():.6f} oracle {ref_loss.item():.6f}")
    assert abs(loss.item() - ref_loss.item()) <= 1e-3 * abs(ref_loss.item())
    m.store.begin_backward()
    d = K.mse_grad(out, target, coef)
    out_tok.backward(K.flux_pack(d))
    m.store.finish_backward()
    ref_loss.backward()
    gh = m.state_dict(grads=True)
    cos = sorted((_cos(gh[n].float().cpu(), p.grad), n) for n, p in om.named_parameters() if p.grad is not None)
    print("worst grad cosines:", cos[:4])
    assert cos[0][0] > 0.98, cos[:4]
    del m, om
    _free()


def test_full_width_flux_lora_blocks_768_match_oracle(dev):
    """C5's adapter set at full width: FLUX (D = 3072, 1 double + 1 single block, frozen bf16 base) with rank-16 LoRA on
    every Linear (module/lora.py: fused q|k|v(|mlp) downs, block-diagonal ups, second-K-segment GEMMs, the transposed
    text / image row segments) against the oracle transformer with the reference LoRA hooks (oracle/lora.py,
    LoRAModule.py:283-323) at 768^2 b=1: flow-matching loss to rtol 1e-3 and every adapter gradient's cosine."""
    from onetrainer_amd.module.lora import LoRAWrapper
    from oracle.lora import OracleLoRA
    torch.set_num_threads(max(1, min(16, torch.get_num_threads())))
    cfg = FX.FluxConfig(num_layers=1, num_single_layers=1)
    ocfg = OF.FluxConfig(num_layers=1, num_single_layers=1)
    m = FX.FluxTransformer2DModel(cfg, dev, seed=1, trainable=False)
    with torch.device("meta"):
        om = OF.FluxTransformer2DModel(ocfg)
    om = om.to_empty(device="cpu")
    om.load_state_dict({k: v.float().cpu() for k, v in m.state_dict().items()})
    om.requires_grad_(False)
    rank, alpha = 16, 16.0
    lw = LoRAWrapper(m, rank=rank, alpha=alpha, prefix="lora_transformer", seed=0)
    m.lora = lw
    ol = OracleLoRA(om, rank, alpha, prefix="lora_transformer")
    g = torch.Generator().manual_seed(5)
    sd = {k: (torch.randn(v.shape, generator=g) * (0.01 if "lora_up" in k else 0.02) if not k.endswith(".alpha") else v)
          for k, v in lw.state_dict().items()}
    lw.load_state_dict(sd)
    ol.load_state_dict({k: v for k, v in lw.state_dict().items() if not k.endswith(".alpha")})
    B, h = 1, 96
    lat = torch.randn(B, 16, h, h, generator=g)
    eps = torch.randn(B, 16, h, h, generator=g)
    t = torch.tensor([611], dtype=torch.int32)
    pooled = torch.randn(B, 768, generator=g).bfloat16()
    ehs = torch.randn(B, 77, 4096, generator=g).bfloat16()
    x0 = (lat - 0.1159) * 0.3611
    xt, _ = OD.add_noise_flow(x0, eps, t.long())
    xin = xt.bfloat16().permute(0, 2, 3, 1).contiguous().to(dev)
    tok = K.flux_pack(xin)
    out_tok = m(tok, t.float().to(dev) / 1000, torch.ones(B, device=dev), pooled.to(dev), ehs.to(dev), h, h)
    out = K.flux_unpack(out_tok.contiguous(), B, h, h, 16)
    target = (eps - x0).permute(0, 2, 3, 1).contiguous().to(dev)
    loss, coef, _ = K.mse_loss(out, target)
    ref = om(OF.pack_latents(xt.bfloat16().float()), t.float() / 1000, torch.ones(B), pooled.float(), ehs.float(),
             torch.zeros(77, 3), OF.prepare_latent_image_ids(h, h))
    ref = OF.unpack_latents(ref, h, h)
    ref_loss = OD.flow_matching_losses(ref, eps - x0, torch.ones(B)).mean()
    print(f"flux lora r16 1+1 blocks 768^2 loss hip {loss.item():.6f} oracle {ref_loss.item():.6f}")
    assert abs(loss.item() - ref_loss.item()) <= 1e-3 * abs(ref_loss.item())
    lw.store.begin_backward()
    d = K.mse_grad(out, target, coef)
    out_tok.backward(K.flux_pack(d))
    lw.store.finish_backward()
    ref_loss.backward()
    gs = lw.state_dict(grads=True)
    assert set(gs) >= set(ol.params), sorted(set(ol.params) - set(gs))[:5]
    cos = sorted((_cos(gs[k].float().cpu().reshape(p.shape), p.grad), k) for k, p in ol.params.items())
    print(f"{len(cos)} adapter tensors; worst grad cosines:", cos[:4])
    assert cos[0][0] > 0.98, cos[:4]
    assert sum(c for c, _ in cos) / len(cos) > 0.999
    del m, om, lw, ol
    _free()


# ---- full-size property steps (C2-C5) ---------------------------------------------------------
def _steps(tr, batches, store):
    losses, snaps = [], []
    for i, b in enumerate(batches):
        losses.append(tr.train_step(b).float().item())
        if i == 0:
            assert bool(torch.isfinite(store.grad).all().item()), "non-finite gradients"
        store.wait_params()                  # the optimizer update runs on its own stream (adamw_fused.py)
        snaps.append(store.data.clone() if store.numel < 3_000_000_000 else None)
    return losses, snaps


@pytest.mark.parametrize("name,res,b", [("sd15", 512, 16), ("sd15", 512, 1), ("sdxl", 1024, 4)])
def test_full_finetune_property_steps(dev, name, res, b):
    """C2 (SD 1.5 512^2 b=16), C1's shape on the GPU (SD 1.5 512^2 b=1), C3 per rank (SDXL 1024^2 b=4)."""
    cfg = TrainConfig.default_values()
    cfg.model_type = "STABLE_DIFFUSION_15" if name == "sd15" else "STABLE_DIFFUSION_XL_10_BASE"
    cfg.batch_size = b
    cfg.learning_rate = 1e-4
    cfg.learning_rate_warmup_steps = 0
    tr = GenericTrainer(cfg, seed=0)
    tr.start()
    batch = synthetic_sdxl_batch(b, res, res, dev, seed=1, sdxl=name == "sdxl",
                                 scaling_factor=0.18215 if name == "sd15" else 0.13025)
    st = tr.model.train_store
    losses, snaps = _steps(tr, [batch, batch], st)
    print(f"{name} {res}^2 b={b} losses {losses}")
    assert all(math.isfinite(v) and 0.05 < v < 20 for v in losses), losses
    assert not torch.equal(snaps[0], snaps[1]), "second step did not move the parameters"
    del tr, snaps
    _free()


def test_sdxl_lora_r32_aspect_buckets(dev):
    """C4: SDXL LoRA rank 32 (every Linear / Conv2d), fp32 adapters, two aspect buckets."""
    cfg = TrainConfig.default_values()
    cfg.training_method, cfg.lora_rank, cfg.lora_alpha = "LORA", 32, 1.0
    cfg.batch_size = 4
    cfg.learning_rate = 3e-4
    cfg.learning_rate_warmup_steps = 0
    tr = GenericTrainer(cfg, seed=0)
    tr.start()
    base0 = tr.model.unet.store.data.clone()
    batches = [synthetic_sdxl_batch(4, hh, ww, dev, seed=i) for i, (hh, ww) in enumerate([(1024, 1024), (1152, 896)])]
    st = tr.model.train_store
    n = sum(p.numel() for p in tr.model.unet_lora.parameters())
    assert abs(n - 98_825_472) / 98_825_472 < 0.02, n     # r32 over every Linear/Conv2d
    losses, snaps = _steps(tr, batches + batches, st)
    print("sdxl lora r32 ARB losses", losses)
    assert all(math.isfinite(v) and 0.05 < v < 20 for v in losses), losses
    assert not torch.equal(snaps[1], snaps[3])
    assert torch.equal(tr.model.unet.store.data, base0), "frozen base changed"
    del tr, snaps, base0
    _free()


def test_flux_lora_768_b4(dev):
    """C5: FLUX.1-dev LoRA r16 (19 double + 38 single blocks, bf16 base), flow matching, 768^2 b=4."""
    cfg = TrainConfig.default_values()
    cfg.model_type, cfg.training_method, cfg.timestep_distribution = "FLUX_DEV_1", "LORA", "LOGIT_NORMAL"
    cfg.batch_size = 4
    cfg.learning_rate = 3e-4
    cfg.learning_rate_warmup_steps = 0
    tr = GenericTrainer(cfg, seed=0)
    tr.start()
    base0 = tr.model.transformer.store.data[::4096].clone()     # strided sample of the 11.9 B base
    batch = synthetic_flux_batch(4, 768, 768, dev, seed=1)
    st = tr.model.train_store
    losses, snaps = _steps(tr, [batch, batch], st)
    print("flux lora 768 losses", losses)
    assert all(math.isfinite(v) and 0.05 < v < 20 for v in losses), losses
    assert not torch.equal(snaps[0], snaps[1])
    assert torch.equal(tr.model.transformer.store.data[::4096], base0), "frozen base changed"
    del tr, snaps
    _free()
