"""Host logic of the data path (CPU): aspect-ratio buckets, same-resolution global batches, DP
slicing and the latent-cache write/read round trip (a stub encoder stands in for the HIP VAE,
which tests/test_vae_gpu.py covers).  mgds is not in the image: bucket lists are PARITY UNPINNED."""
import random

import torch

from onetrainer_amd.dataLoader.aspect_bucketing import (AspectBucketing, SingleAspectCalculation, aspect_batches,
                                                        crop_offset, quantization_for, rank_slice)
from onetrainer_amd.dataLoader.latent_cache import LatentCacheDataLoader, LatentCacheWriter


def test_buckets_sdxl():
    ab = AspectBucketing(1024, quantization_for("STABLE_DIFFUSION_XL_10_BASE"))
    assert (1024, 1024) in ab.resolutions and (896, 1152) in ab.resolutions and (1152, 896) in ab.resolutions
    for h, w in ab.resolutions:
        assert h % 64 == 0 and w % 64 == 0
        assert 0.8 < h * w / 1024 ** 2 < 1.15
    assert len(set(ab.resolutions)) == len(ab.resolutions)
    assert quantization_for("STABLE_DIFFUSION_15") == 8


def test_bucket_choice_covers_crop():
    ab = AspectBucketing(1024, 64)
    rng = random.Random(0)
    for _ in range(200):
        h, w = rng.randint(300, 4000), rng.randint(300, 4000)
        scale, crop = ab.bucket_for(h, w)
        assert scale[0] >= crop[0] and scale[1] >= crop[1]
        assert abs(scale[0] / scale[1] - h / w) < 0.02 * (h / w) + 2.0 / min(scale)
        best = min(abs(a - h / w) for a in ab.aspects)
        assert abs(crop[0] / crop[1] - h / w) == best
        y0, x0 = crop_offset(scale, crop)
        assert 0 <= y0 <= scale[0] - crop[0] and 0 <= x0 <= scale[1] - crop[1]
    s = SingleAspectCalculation(512)
    assert s.bucket_for(600, 400) == ((768, 512), (512, 512))


def test_aspect_batches_uniform_deterministic_and_sliced():
    rng = random.Random(1)
    res = [rng.choice([(1024, 1024), (896, 1152), (1152, 896)]) for _ in range(101)]
    b1 = aspect_batches(res, 8, seed=3, epoch=0)
    assert b1 == aspect_batches(res, 8, seed=3, epoch=0)
    assert b1 != aspect_batches(res, 8, seed=3, epoch=1)
    seen = set()
    for b in b1:
        assert len(b) == 8 and len({res[i] for i in b}) == 1
        seen.update(b)
    assert len(seen) == 8 * len(b1)
    parts = [rank_slice(b1[0], r, 4) for r in range(4)]
    assert sum(parts, []) == b1[0]


def _stub_encode(imgs):
    # [B,3,H,W] -> [B,H/8,W/8,4]: 8x8 mean pool + a zero channel (stands in for the HIP VAE)
    p = torch.nn.functional.avg_pool2d(imgs * 2 - 1, 8)
    return torch.cat([p, torch.zeros_like(p[:, :1])], 1).permute(0, 2, 3, 1)


def test_latent_cache_round_trip(tmp_path):
    torch.manual_seed(0)
    ab = AspectBucketing(128, 64)
    shapes = [(128, 128), (100, 160), (160, 100), (130, 128), (96, 192), (128, 140)]
    samples = [{"image": torch.rand(3, h, w), "text": {"text_encoder_hidden_state": torch.randn(77, 16)}}
               for h, w in shapes]
    n = LatentCacheWriter(_stub_encode, str(tmp_path), ab, "cpu", encode_batch=2).write(samples)
    assert n == len(shapes)
    dl = LatentCacheDataLoader(str(tmp_path), batch_size=1, device="cpu", seed=0, prefetch=True)
    dl.get_data_set().start_next_epoch()
    got = 0
    for batch in dl.get_data_loader():
        lat = batch["latent_image"]
        ch, cw = batch["crop_resolution"][0][0].item(), batch["crop_resolution"][1][0].item()
        assert lat.shape == (1, 4, ch // 8, cw // 8) and lat.dtype == torch.float32
        assert lat.permute(0, 2, 3, 1).is_contiguous()       # NCHW view of channels-last storage
        assert batch["text_encoder_hidden_state"].shape == (1, 77, 16)
        assert torch.count_nonzero(lat[:, 3]) == 0
        got += 1
    assert got == len(shapes)
    # two ranks of a global batch of 2 read disjoint halves of the same batches
    r0 = LatentCacheDataLoader(str(tmp_path), 1, "cpu", seed=0, rank=0, world=2, prefetch=False)
    r1 = LatentCacheDataLoader(str(tmp_path), 1, "cpu", seed=0, rank=1, world=2, prefetch=False)
    for b0, b1 in zip(r0.get_data_loader(), r1.get_data_loader()):
        assert b0["latent_image"].shape == b1["latent_image"].shape
