"""Deferred grouped split-K reduces on the weight-gradient stream (otamd_gemm_defer_*, module/streams.defer_*).

The LoRA adapter gradients are split-K GEMMs (rank-wide outputs, K = tokens); deferring their reduces and launching
them grouped must not change a bit: each output is still summed in split order.  Checked on whole backward passes
(overwrite and gradient-accumulation micro-steps) of the tiny SDXL LoRA and the full-width SDXL LoRA r32 at 512^2,
b=1 (the C4 bench configuration), plus the flush-before-read guard on a direct GEMM chain.  The LayerNorm parameter reduces (otamd_layernorm_defer_*) are
deferred the same way on the main stream: checked on full fine-tune steps of the tiny SDXL UNet and at SDXL 512^2.
"""
import copy

import pytest
import torch

from onetrainer_amd import kernels as K
from onetrainer_amd.dataLoader.SyntheticDataLoader import synthetic_sdxl_batch
from onetrainer_amd.module import streams as S
from onetrainer_amd.module import unet as U
from onetrainer_amd.trainer.GenericTrainer import GenericTrainer
from onetrainer_amd.util import create
from onetrainer_amd.util.config.TrainConfig import TrainConfig

pytestmark = pytest.mark.gpu


def _lora_trainer(dev, ucfg, rank):
    cfg = TrainConfig.default_values()
    cfg.batch_size = 1
    cfg.learning_rate_warmup_steps = 0
    cfg.gradient_accumulation_steps = 1000   # no optimizer update: every micro-step sees the same weights
    cfg.training_method, cfg.lora_rank = "LORA", rank
    model = create.create_model(cfg, dev, seed=5, unet_config=ucfg)
    tr = GenericTrainer(cfg, model=model)
    tr.start()
    return tr


def _two_microsteps(tr, batch, defer, monkeypatch):
    """an overwrite micro-step and an accumulating one from the same progress state; the grads after each"""
    monkeypatch.setattr(S, "_DEFER", defer)
    model = tr.model
    tp0 = copy.deepcopy(model.train_progress)
    store = model.train_store
    store.accumulating = False
    out = []
    for _ in range(2):
        loss = tr.train_step(batch)
        torch.cuda.synchronize()
        out.append((loss.clone(), store.grad.clone()))
    model.train_progress = tp0
    store.accumulating = False
    return out


@pytest.mark.parametrize("which", ["tiny_r8", "sdxl_r32_512"])
def test_deferred_reduces_bit_identical(dev, which, monkeypatch):
    if which == "tiny_r8":
        tr = _lora_trainer(dev, U.tiny_sdxl_config(), 8)
        batch = synthetic_sdxl_batch(1, 256, 256, dev, seed=0, te1_dim=48, te2_dim=48, pooled_dim=64)
    else:
        tr = _lora_trainer(dev, None, 32)
        batch = synthetic_sdxl_batch(1, 512, 512, dev, seed=0)
    assert S.side_stream() is not None
    tr.train_step(batch)   # plan / workspace warm-up
    torch.cuda.synchronize()
    tr.model.train_store.accumulating = False
    ref = _two_microsteps(tr, batch, False, monkeypatch)
    g0, l0 = K.defer_reduces_stats()
    got = _two_microsteps(tr, batch, True, monkeypatch)
    g1, l1 = K.defer_reduces_stats()
    deferred, launches = g1 - g0, l1 - l0
    if which != "tiny_r8":   # the tiny UNet's few-token GEMMs mostly run unsplit
        assert deferred > 0 and launches > 0, (deferred, launches)
        assert launches * 4 <= deferred, (deferred, launches)   # grouped: many reduces per launch
    for (la, ga), (lb, gb) in zip(ref, got):
        assert torch.equal(la, lb)
        assert torch.equal(ga, gb), (ga.float() - gb.float()).abs().max().item()
    assert ref[0][1].abs().sum().item() > 0
    assert not torch.equal(ref[0][1], ref[1][1])   # the second micro-step accumulated
    assert K.defer_reduces_pending(S.side_stream()) == 0
    print(f"{which}: {deferred // 2} deferred reduces in {launches // 2} grouped launches per backward")


def test_defer_flushes_before_dependent_gemm(dev):
    """a GEMM that reads a pending output as its operand flushes the pending reduces first; a GEMM whose output
    lies outside the registered gradient range is not deferred"""
    side = S.side_stream()
    g = torch.Generator(device=dev).manual_seed(1)
    BF = torch.bfloat16
    x = torch.randn(8192, 256, device=dev, generator=g).to(BF)
    dy = torch.randn(8192, 32, device=dev, generator=g).to(BF)
    grads = torch.zeros(32 * 256 + 64 * 256, device=dev, dtype=BF)
    w1 = grads[:32 * 256].view(32, 256)
    y2 = torch.randn(64, 32, device=dev, generator=g).to(BF)
    ref1 = K.linear_wgrad(dy, x)
    torch.cuda.synchronize()
    with torch.cuda.stream(side):
        K.defer_reduces_begin(side, grads)
        K.linear_wgrad(dy, x, out=w1)                     # split-K over 8192 tokens: deferred
        assert K.defer_reduces_pending(side) == 1
        z = K.linear_dgrad(y2, w1)                        # reads w1: must see the reduced value
        assert K.defer_reduces_pending(side) == 0
        outside = K.linear_wgrad(dy, x)                   # not in the gradient buffer: immediate reduce
        assert K.defer_reduces_pending(side) == 0
        K.defer_reduces_end(side)
    torch.cuda.synchronize()
    assert torch.equal(w1, ref1) and torch.equal(outside, ref1)
    assert torch.equal(z, K.linear_dgrad(y2, ref1))


def _ft_trainer(dev, ucfg):
    cfg = TrainConfig.default_values()
    cfg.batch_size = 1
    cfg.learning_rate_warmup_steps = 0
    cfg.gradient_accumulation_steps = 1000
    model = create.create_model(cfg, dev, seed=5, unet_config=ucfg)
    tr = GenericTrainer(cfg, model=model)
    tr.start()
    return tr


@pytest.mark.parametrize("which", ["tiny", "sdxl_512"])
def test_deferred_layernorm_param_reduces_bit_identical(dev, which, monkeypatch):
    if which == "tiny":
        tr = _ft_trainer(dev, U.tiny_sdxl_config())
        batch = synthetic_sdxl_batch(1, 256, 256, dev, seed=0, te1_dim=48, te2_dim=48, pooled_dim=64)
    else:
        tr = _ft_trainer(dev, None)
        batch = synthetic_sdxl_batch(1, 512, 512, dev, seed=0)
    tr.train_step(batch)
    torch.cuda.synchronize()
    tr.model.train_store.accumulating = False
    monkeypatch.setattr(S, "_LN_DEFER", False)
    ref = _two_microsteps(tr, batch, True, monkeypatch)
    monkeypatch.setattr(S, "_LN_DEFER", True)
    main = torch.cuda.current_stream()
    n0, l0, _ = K.ln_defer_stats(main)
    got = _two_microsteps(tr, batch, True, monkeypatch)
    n1, l1, pending = K.ln_defer_stats(main)
    assert pending == 0
    deferred, launches = n1 - n0, l1 - l0
    assert deferred > 0 and launches > 0 and launches * 2 <= deferred, (deferred, launches)
    for (la, ga), (lb, gb) in zip(ref, got):
        assert torch.equal(la, lb)
        assert torch.equal(ga, gb), (ga.float() - gb.float()).abs().max().item()
    assert not torch.equal(ref[0][1], ref[1][1])
    print(f"{which}: {deferred // 2} LayerNorm parameter reduces in {launches // 2} grouped launches per backward")


def test_layernorm_defer_flush_order(dev):
    """a pending reduce into the same dgamma is flushed before the next one is recorded (accumulation stays ordered);
    flush / end leave nothing pending and the sums equal the immediate path's"""
    g = torch.Generator(device=dev).manual_seed(3)
    BF = torch.bfloat16
    x = torch.randn(4096, 1280, device=dev, generator=g).to(BF)
    dy = torch.randn(4096, 1280, device=dev, generator=g).to(BF)
    gamma = torch.ones(1280, device=dev, dtype=BF)
    beta = torch.zeros(1280, device=dev, dtype=BF)
    _, stats = K.layernorm_fwd(x, gamma, beta, 1e-5)
    dg0, db0 = torch.zeros(1280, device=dev), torch.zeros(1280, device=dev)
    K.layernorm_param_grad(x, dy, stats, dg0, db0)
    K.layernorm_param_grad(x, dy, stats, dg0, db0, param_acc=True)
    main = torch.cuda.current_stream()
    dg, db = torch.zeros(1280, device=dev), torch.zeros(1280, device=dev)
    K.ln_defer_begin(main)
    K.layernorm_param_grad(x, dy, stats, dg, db)
    assert K.ln_defer_stats(main)[2] == 1
    K.layernorm_param_grad(x, dy, stats, dg, db, param_acc=True)   # same destination: the first is flushed
    assert K.ln_defer_stats(main)[2] == 1
    K.ln_defer_flush(main)
    assert K.ln_defer_stats(main)[2] == 0
    K.ln_defer_end(main)
    torch.cuda.synchronize()
    assert torch.equal(dg, dg0) and torch.equal(db, db0)
