"""INTERNAL backup / resume: a run backed up after step 2 and resumed in a fresh
trainer (continue_last_backup, GenericTrainer.py:94-108) takes step 3 bit-identically to the
uninterrupted run -- weights, optimizer moments, step counts, LR schedule position, the
global_step-seeded noise and the stochastic-rounding stream all restored.  Fine-tune and LoRA."""
import os

import pytest
import torch

from onetrainer_amd.dataLoader.SyntheticDataLoader import synthetic_sdxl_batch
from onetrainer_amd.module import unet as U
from onetrainer_amd.trainer.GenericTrainer import GenericTrainer
from onetrainer_amd.util import create
from onetrainer_amd.util.config.TrainConfig import TrainConfig

pytestmark = pytest.mark.gpu


def _cfg(tmp, lora):
    cfg = TrainConfig.default_values()
    cfg.batch_size = 2
    cfg.learning_rate = 1e-4
    cfg.learning_rate_warmup_steps = 4        # exercises the LR schedule position on resume
    cfg.workspace_dir = str(tmp)
    if lora:
        cfg.training_method = "LORA"
        cfg.lora_rank, cfg.lora_alpha = 8, 8.0
    return cfg


def _trainer(cfg, dev, seed):
    model = create.create_model(cfg, dev, seed=seed, unet_config=U.tiny_sdxl_config())
    tr = GenericTrainer(cfg, model=model)
    tr.start()
    return tr


def _store(tr):
    return tr.model.train_store.data.clone()


@pytest.mark.parametrize("lora", [False, True])
def test_backup_resume_bit_exact(dev, tmp_path, lora):
    torch.manual_seed(0)
    batch = synthetic_sdxl_batch(2, 128, 128, dev, seed=1, te1_dim=48, te2_dim=48, pooled_dim=64)
    cfg = _cfg(tmp_path, lora)
    a = _trainer(cfg, dev, seed=3)
    for _ in range(2):
        a.train_step(batch)
    path = a.backup()
    assert path and os.path.isfile(os.path.join(path, "meta.json"))
    assert os.path.isfile(os.path.join(path, "optimizer", "optimizer.pt"))
    assert os.path.isfile(os.path.join(path, "lora", "lora.safetensors") if lora else
                          os.path.join(path, "unet", "diffusion_pytorch_model.safetensors"))
    assert os.path.isfile(os.path.join(path, "onetrainer_config", "args.json"))
    loss_a = a.train_step(batch).item()
    w_a = _store(a)

    cfg_b = _cfg(tmp_path, lora)
    cfg_b.continue_last_backup = True
    # LoRA: the (frozen) base is not part of a LoRA backup; the run's base weights come from its seed
    b = _trainer(cfg_b, dev, seed=3 if lora else 7)
    assert b.model.train_progress.global_step == 2
    loss_b = b.train_step(batch).item()
    assert loss_a == loss_b, (loss_a, loss_b)
    assert torch.equal(w_a, _store(b))
    assert b.lr_scheduler.get_last_lr() == a.lr_scheduler.get_last_lr()


def test_rolling_backup_prunes(dev, tmp_path):
    cfg = _cfg(tmp_path, False)
    cfg.rolling_backup, cfg.rolling_backup_count = True, 2
    tr = _trainer(cfg, dev, seed=3)
    batch = synthetic_sdxl_batch(2, 128, 128, dev, seed=1, te1_dim=48, te2_dim=48, pooled_dim=64)
    paths = []
    for _ in range(3):
        tr.train_step(batch)
        paths.append(tr.backup())
    left = sorted(os.listdir(os.path.join(tmp_path, "backup")))
    assert len(left) == 2 and os.path.basename(paths[-1]) in left
