"""VAE-encode latent caching: HIP AutoencoderKL encoder (bf16, NHWC) vs the
oracle (fp32 CPU restatement of diffusers AutoencoderKL.encode(...).latent_dist.mean), same
weights and images.  Tolerance: bf16 activations with fp32 accumulation vs fp32 -> max abs error
<= 3e-2 of the latent range, cosine >= 0.9995 (parity unpinned: diffusers is not in the image)."""
import pytest
import torch

from onetrainer_amd import kernels as K
from onetrainer_amd.module import vae as V
from oracle import vae as OV

pytestmark = pytest.mark.gpu


def _cos(a, b):
    a, b = a.flatten().double(), b.flatten().double()
    return (a @ b / (a.norm() * b.norm() + 1e-30)).item()


@pytest.mark.parametrize("cfgname,B,H,W", [("tiny", 2, 64, 96), ("sdxl", 1, 256, 256), ("tiny16", 2, 64, 96),
                                          ("flux", 1, 256, 256)])
def test_vae_encode_matches_oracle(dev, cfgname, B, H, W):
    """SDXL / SD 1.5 (4 latent channels + quant_conv) and FLUX.1 (16 latent channels, no quant_conv)"""
    torch.manual_seed(0)
    cfg = {"tiny": V.tiny_vae_config, "sdxl": V.sdxl_vae_config, "flux": V.flux_vae_config,
           "tiny16": lambda: V.tiny_vae_config(16, False)}[cfgname]()
    enc = V.AutoencoderKLEncoder(cfg, dev, seed=1)
    om = OV.AutoencoderKLEncoder(cfg)
    om.load_state_dict({k: v.float().cpu() for k, v in enc.state_dict().items()})
    img = torch.rand(B, 3, H, W)
    lat = enc.encode(img.to(dev))
    assert lat.shape == (B, H // 2 ** (len(cfg.block_out_channels) - 1), W // 2 ** (len(cfg.block_out_channels) - 1),
                         cfg.latent_channels) and lat.dtype == torch.float32
    with torch.no_grad():
        # the oracle sees the same bf16-rounded rescaled input
        ref = om.moments((img * 2 - 1).bfloat16().float())[:, :cfg.latent_channels]
    ref = ref.permute(0, 2, 3, 1)
    err = (lat.cpu() - ref).abs().max() / ref.abs().max()
    assert err < 3e-2, f"rel err {err}"
    assert _cos(lat.cpu(), ref) > 0.9995


def test_image_to_nhwc(dev):
    img = torch.rand(2, 3, 8, 16, device=dev)
    x = K.image_to_nhwc(img)
    assert x.shape == (2, 8, 16, 8)
    ref = (img * 2 - 1).permute(0, 2, 3, 1).bfloat16()
    assert torch.equal(x[..., :3], ref) and torch.count_nonzero(x[..., 3:]) == 0


def test_downsample_conv_one_sided_padding(dev):
    """F.pad(x, (0,1,0,1)) + 3x3 stride-2 conv == the conv gather with pad 0 and out_hw = H/2."""
    torch.manual_seed(1)
    x = torch.randn(2, 16, 24, 64, device=dev).bfloat16()
    w = (torch.randn(64, 64, 3, 3, device=dev) * 0.05)
    b = torch.randn(64, device=dev) * 0.1
    y = K.conv2d(x, w.permute(0, 2, 3, 1).contiguous().bfloat16(), bias=b.bfloat16(), stride=2, pad=0, out_hw=(8, 12))
    ref = torch.nn.functional.conv2d(torch.nn.functional.pad(x.permute(0, 3, 1, 2).float(), (0, 1, 0, 1)),
                                     w.bfloat16().float(), b.bfloat16().float(), stride=2)
    assert ((y.permute(0, 3, 1, 2).float() - ref).abs().max() / ref.abs().max()).item() < 1e-2


def test_cache_then_train_on_buckets(dev, tmp_path):
    """images -> ARB buckets -> HIP VAE latent cache -> reader -> SD 1.5 train steps (mixed shapes)."""
    from onetrainer_amd.dataLoader.aspect_bucketing import AspectBucketing
    from onetrainer_amd.dataLoader.latent_cache import LatentCacheDataLoader, LatentCacheWriter
    from onetrainer_amd.module import unet as U
    from onetrainer_amd.trainer.GenericTrainer import GenericTrainer
    from onetrainer_amd.util import create
    from onetrainer_amd.util.config.TrainConfig import TrainConfig
    torch.manual_seed(0)
    enc = V.AutoencoderKLEncoder(V.tiny_vae_config(), dev, seed=1)
    ab = AspectBucketing(128, 64)
    shapes = [(128, 128), (120, 130), (100, 170), (170, 100), (128, 200), (200, 128), (96, 96), (140, 140)]
    samples = [{"image": torch.rand(3, h, w), "text": {"text_encoder_hidden_state": torch.randn(77, 96).bfloat16()}}
               for h, w in shapes]
    LatentCacheWriter(lambda im: enc.encode(im), str(tmp_path), ab, dev, encode_batch=4).write(samples)
    cfg = TrainConfig.default_values()
    cfg.model_type = "STABLE_DIFFUSION_15"
    cfg.batch_size = 2
    cfg.learning_rate_warmup_steps = 0
    model = create.create_model(cfg, dev, seed=3, unet_config=U.tiny_sd15_config())
    dl = LatentCacheDataLoader(str(tmp_path), batch_size=2, device=dev, seed=0)
    tr = GenericTrainer(cfg, model=model, data_loader=dl)
    tr.start()
    dl.get_data_set().start_next_epoch()
    shapes_seen = set()
    for batch in dl.get_data_loader():
        loss = tr.train_step(batch)
        assert torch.isfinite(loss).item()
        shapes_seen.add(tuple(batch["latent_image"].shape))
    assert len(shapes_seen) >= 2


def test_flux_cache_then_train(dev, tmp_path):
    """C5's latent caching (FluxBaseDataLoader.py:70-71): images -> the 16-channel FLUX VAE encoder (no quant_conv)
    -> latent cache (16 channels) -> reader -> FLUX.1 LoRA train steps, whose prologue applies
    (latent - shift_factor) * scaling_factor (BaseFluxSetup.py:229-230)."""
    from onetrainer_amd.dataLoader.aspect_bucketing import AspectBucketing
    from onetrainer_amd.dataLoader.latent_cache import LatentCacheDataLoader, LatentCacheWriter
    from onetrainer_amd.module import flux as FX
    from onetrainer_amd.trainer.GenericTrainer import GenericTrainer
    from onetrainer_amd.util import create
    from onetrainer_amd.util.config.TrainConfig import TrainConfig
    torch.manual_seed(0)
    enc = V.AutoencoderKLEncoder(V.tiny_vae_config(16, False), dev, seed=1)
    fcfg = FX.tiny_flux_config()
    ab = AspectBucketing(128, 64)
    shapes = [(128, 128), (120, 130), (128, 128), (130, 120)]
    samples = [{"image": torch.rand(3, h, w),
                "text": {"text_encoder_1_pooled_state": torch.randn(fcfg.pooled_projection_dim).bfloat16(),
                         "text_encoder_2_hidden_state": torch.randn(77, fcfg.joint_attention_dim).bfloat16()}}
               for h, w in shapes]
    LatentCacheWriter(lambda im: enc.encode(im), str(tmp_path), ab, dev, encode_batch=2).write(samples)
    cfg = TrainConfig.default_values()
    cfg.model_type, cfg.training_method, cfg.timestep_distribution = "FLUX_DEV_1", "LORA", "LOGIT_NORMAL"
    cfg.batch_size = 2
    cfg.learning_rate_warmup_steps = 0
    model = create.create_model(cfg, dev, seed=3, flux_config=fcfg)
    dl = LatentCacheDataLoader(str(tmp_path), batch_size=2, device=dev, seed=0)
    tr = GenericTrainer(cfg, model=model, data_loader=dl)
    tr.start()
    dl.get_data_set().start_next_epoch()
    n = 0
    for batch in dl.get_data_loader():
        assert batch["latent_image"].shape[1] == 16
        loss = tr.train_step(batch)
        assert torch.isfinite(loss).item()
        n += 1
    assert n >= 1
