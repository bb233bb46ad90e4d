"""scripts/train.py (the reference's scripts/train.py:15-43 on this build): a reference-format
JSON config -> GenericTrainer(config, callbacks, commands).start() / train() / end(), reading a
latent cache written by LatentCacheWriter (SD 1.5 full UNet, random init, 128^2 images in two
aspect buckets), then the loop's external behaviour: periodic backups (backup_after 1 STEP, rolling 2)
and end()'s backup-before-save + final model, reloaded through the model loader."""
import json

import pytest
import torch

pytestmark = pytest.mark.gpu


def test_train_script_runs_reference_config(dev, tmp_path):
    import importlib.util
    from pathlib import Path

    from onetrainer_amd.dataLoader.aspect_bucketing import AspectBucketing
    from onetrainer_amd.dataLoader.latent_cache import LatentCacheWriter
    from onetrainer_amd.modelLoader.StableDiffusionModelLoader import StableDiffusionXLModelLoader
    from onetrainer_amd.modelSaver import StableDiffusionXLModelSaver
    from onetrainer_amd.module import unet as U
    from onetrainer_amd.module import vae as V
    from onetrainer_amd.util import create
    from onetrainer_amd.util.ModelNames import ModelNames
    from onetrainer_amd.util.config.TrainConfig import TrainConfig
    torch.manual_seed(0)
    # the base model: a tiny SD 1.5-shaped UNet in diffusers layout (its unet/config.json sets the architecture)
    base_cfg = TrainConfig.default_values()
    base_cfg.model_type = "STABLE_DIFFUSION_15"
    base = create.create_model(base_cfg, dev, seed=5, unet_config=U.tiny_sd15_config())
    StableDiffusionXLModelSaver().save(base, None, "DIFFUSERS", str(tmp_path / "base"))
    enc = V.AutoencoderKLEncoder(V.tiny_vae_config(), dev, seed=1)
    shapes = [(128, 128), (128, 128), (128, 192), (128, 192)]   # SD 1.5 latents: multiples of 8
    samples = [{"image": torch.rand(3, h, w), "text": {"text_encoder_hidden_state": torch.randn(77, 96).bfloat16()}}
               for h, w in shapes]
    cache = tmp_path / "cache"
    LatentCacheWriter(lambda im: enc.encode(im), str(cache), AspectBucketing(128, 64), dev, encode_batch=2).write(samples)
    cfg = {"__version": 6, "model_type": "STABLE_DIFFUSION_15", "training_method": "FINE_TUNE",
           "cache_dir": str(cache), "batch_size": 2, "epochs": 1, "learning_rate": 1e-5,
           "learning_rate_warmup_steps": 0, "workspace_dir": str(tmp_path / "ws"), "train_dtype": "BFLOAT_16",
           "weight_dtype": "BFLOAT_16",
           "optimizer": {"optimizer": "ADAMW", "stochastic_rounding": True},
           "unet": {"train": True}, "text_encoder": {"train": False}, "base_model_name": str(tmp_path / "base"),
           "output_model_destination": str(tmp_path / "out" / "model.safetensors"), "output_model_format": "SAFETENSORS",
           "output_dtype": "FLOAT_32", "backup_after": 1, "backup_after_unit": "STEP", "rolling_backup": True,
           "rolling_backup_count": 2}
    path = tmp_path / "config.json"
    path.write_text(json.dumps(cfg))
    spec = importlib.util.spec_from_file_location("train_script", Path(__file__).parents[1] / "scripts" / "train.py")
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    tr = mod.main(["--config-path", str(path)])
    tp = tr.model.train_progress
    assert tp.global_step == 2 and tr.model.unet.cfg == U.tiny_sd15_config()
    # backups before steps 0 and 1 and before the final save; the rolling window keeps the newest 2
    backups = sorted((tmp_path / "ws" / "backup").iterdir())
    assert len(backups) == 2, backups
    steps = sorted(json.loads((b / "meta.json").read_text())["train_progress"]["global_step"] for b in backups)
    assert steps == [1, 2], steps
    # the final model reloads through the model loader with the trained weights (bf16 -> fp32 -> bf16 is exact)
    out = tmp_path / "out" / "model.safetensors"
    assert out.is_file()
    fresh = create.create_model(base_cfg, dev, seed=11, unet_config=U.tiny_sd15_config())
    StableDiffusionXLModelLoader().load(fresh, ModelNames(base_model=str(out)))
    trained, loaded = tr.model.unet.state_dict(), fresh.unet.state_dict()
    assert trained.keys() == loaded.keys()
    for k in trained:
        assert torch.equal(trained[k], loaded[k]), k
    base_sd = base.unet.state_dict()
    moved = sum(not torch.equal(trained[k], base_sd[k]) for k in trained)
    assert moved > 0.5 * len(trained)      # the saved weights are the trained ones, not the base


# training_presets/#sd 1.5.json of the reference (C1's preset), field for field; it sets no weight_dtype or
# train_dtype, so the reference's defaults apply: FLOAT_32 weights (fp32 master weights here) and FLOAT_16 compute
SD15_PRESET = {"base_model_name": "stable-diffusion-v1-5/stable-diffusion-v1-5", "batch_size": 4,
               "model_type": "STABLE_DIFFUSION_15", "output_model_destination": "models/model.safetensors",
               "output_model_format": "SAFETENSORS", "resolution": "512", "training_method": "FINE_TUNE",
               "unet": {"train": True}, "vae": {"weight_dtype": "FLOAT_32"}}


def test_train_script_runs_sd15_preset(dev, tmp_path):
    """the SD 1.5 preset as it stands (fp32 master weights, round 6) through scripts/train.py: trains, keeps fp32
    masters behind the bf16 working copy, and saves the fp32 masters (a tiny SD 1.5-shaped base and a latent cache
    stand in for the hub model and the dataset, which this box cannot fetch)"""
    import importlib.util
    from pathlib import Path

    from onetrainer_amd.dataLoader.aspect_bucketing import AspectBucketing
    from onetrainer_amd.dataLoader.latent_cache import LatentCacheWriter
    from onetrainer_amd.modelSaver import StableDiffusionXLModelSaver
    from onetrainer_amd.module import unet as U
    from onetrainer_amd.module import vae as V
    from onetrainer_amd.util import create
    from onetrainer_amd.util.config.TrainConfig import TrainConfig
    from safetensors.torch import load_file
    torch.manual_seed(1)
    base_cfg = TrainConfig.default_values()
    base_cfg.model_type = "STABLE_DIFFUSION_15"
    base = create.create_model(base_cfg, dev, seed=5, unet_config=U.tiny_sd15_config())
    StableDiffusionXLModelSaver().save(base, None, "DIFFUSERS", str(tmp_path / "base"))
    enc = V.AutoencoderKLEncoder(V.tiny_vae_config(), dev, seed=1)
    samples = [{"image": torch.rand(3, 128, 128), "text": {"text_encoder_hidden_state": torch.randn(77, 96).bfloat16()}}
               for _ in range(8)]
    cache = tmp_path / "cache"
    LatentCacheWriter(lambda im: enc.encode(im), str(cache), AspectBucketing(128, 64), dev, encode_batch=4).write(samples)
    cfg = dict(SD15_PRESET)
    cfg.update({"base_model_name": str(tmp_path / "base"), "cache_dir": str(cache), "epochs": 1,
                "workspace_dir": str(tmp_path / "ws"), "learning_rate_warmup_steps": 0,
                "output_model_destination": str(tmp_path / "out" / "model.safetensors"), "output_dtype": "FLOAT_32"})
    path = tmp_path / "config.json"
    path.write_text(json.dumps(cfg))
    spec = importlib.util.spec_from_file_location("train_script", Path(__file__).parents[1] / "scripts" / "train.py")
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    tr = mod.main(["--config-path", str(path)])
    assert tr.config.weight_dtype == "FLOAT_32" and tr.config.train_dtype == "FLOAT_16"
    assert tr.model.dtype_plan.master
    st = tr.model.unet.store
    assert st.master is not None and tr.model.train_progress.global_step == 2
    assert torch.equal(st.data, st.master.to(torch.bfloat16))
    assert tr.model.optimizer.exp_avg.dtype == torch.float32
    saved = load_file(str(tmp_path / "out" / "model.safetensors"))
    sd = tr.model.unet.state_dict()
    assert all(v.dtype == torch.float32 for v in sd.values())
    # the LDM-layout file holds the fp32 masters: below-bf16 detail survives the save
    below = sum(not torch.equal(v, v.bfloat16().float()) for v in sd.values())
    assert below > 0.5 * len(sd), below
    unet_saved = [v for k, v in saved.items() if k.startswith("model.diffusion_model.") and v.is_floating_point()]
    below_saved = sum(not torch.equal(v.float(), v.bfloat16().float()) for v in unet_saved)
    assert below_saved > 0.5 * len(unet_saved), (below_saved, len(unet_saved))
    base_sd = base.unet.state_dict()
    moved = sum(not torch.equal(sd[k], base_sd[k].float()) for k in sd)
    assert moved > 0.5 * len(sd)
