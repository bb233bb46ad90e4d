"""scripts/train.py (the reference's scripts/train.py:15-43 on this build): a reference-format
JSON config -> GenericTrainer(config, callbacks, commands).start() / train() / end(), reading a
latent cache written by LatentCacheWriter (SD 1.5 full UNet, random init, 128^2 images in two
aspect buckets)."""
import json

import pytest
import torch

pytestmark = pytest.mark.gpu


def test_train_script_runs_reference_config(dev, tmp_path):
    import importlib.util
    from pathlib import Path

    from onetrainer_amd.dataLoader.aspect_bucketing import AspectBucketing
    from onetrainer_amd.dataLoader.latent_cache import LatentCacheWriter
    from onetrainer_amd.module import vae as V
    torch.manual_seed(0)
    enc = V.AutoencoderKLEncoder(V.tiny_vae_config(), dev, seed=1)
    shapes = [(128, 128), (128, 128), (128, 192), (128, 192)]   # SD 1.5 latents: multiples of 8
    samples = [{"image": torch.rand(3, h, w), "text": {"text_encoder_hidden_state": torch.randn(77, 768).bfloat16()}}
               for h, w in shapes]
    cache = tmp_path / "cache"
    LatentCacheWriter(lambda im: enc.encode(im), str(cache), AspectBucketing(128, 64), dev, encode_batch=2).write(samples)
    cfg = {"__version": 6, "model_type": "STABLE_DIFFUSION_15", "training_method": "FINE_TUNE",
           "cache_dir": str(cache), "batch_size": 2, "epochs": 1, "learning_rate": 1e-5,
           "learning_rate_warmup_steps": 0, "workspace_dir": str(tmp_path / "ws"), "train_dtype": "BFLOAT_16",
           "optimizer": {"optimizer": "ADAMW", "stochastic_rounding": True},
           "unet": {"train": True}, "text_encoder": {"train": False}}
    path = tmp_path / "config.json"
    path.write_text(json.dumps(cfg))
    spec = importlib.util.spec_from_file_location("train_script", Path(__file__).parents[1] / "scripts" / "train.py")
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    mod.main(["--config-path", str(path)])
