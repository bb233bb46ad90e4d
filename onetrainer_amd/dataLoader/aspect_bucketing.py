"""Aspect-ratio bucketing and same-resolution batch sorting.

The reference wires mgds AspectBucketing / SingleAspectCalculation / AspectBatchSorting at
modules/dataLoader/mixin/DataLoaderText2ImageMixin.py:139-172 (quantization 64 for SDXL,
StableDiffusionXLBaseDataLoader; 8 for SD) and :278-281 (batch sorting).  mgds@11ff4aa is not in
this image, so the algorithm is restated from its published behaviour and is PARITY UNPINNED:
  * buckets: for each base aspect h:w in ASPECTS (and its transpose) scale to the target pixel
    area, round each side to the quantization; duplicates removed;
  * an image (h, w) goes to the bucket with the nearest aspect h/w; it is scaled to cover the
    bucket (scale_resolution) and cropped to it (crop_resolution);
  * batch sorting: per epoch, the sample indices of every bucket are shuffled and cut into whole
    batches of the GLOBAL batch size (remainders dropped), then the batch order is shuffled --
    every batch has one resolution, so all data-parallel ranks see the same shape (§8(e)).
Host-side integer work: it runs once per epoch on the CPU, off the step's critical path.
"""
from __future__ import annotations

import math
import random

ASPECTS = [(1.0, 1.0), (1.0, 1.25), (1.0, 1.5), (1.0, 1.75), (1.0, 2.0), (1.0, 2.5), (1.0, 3.0), (1.0, 3.5),
           (1.0, 4.0)]


def quantization_for(model_type: str) -> int:
    """StableDiffusionXLBaseDataLoader passes 64, the SD 1.5 loader 8."""
    return 64 if model_type.startswith("STABLE_DIFFUSION_XL") else 8


class AspectBucketing:
    def __init__(self, target_resolution: int, quantization: int = 64, aspects=ASPECTS):
        self.target_resolution = target_resolution
        self.quantization = quantization
        res = []
        for h, w in aspects:
            s = math.sqrt(target_resolution * target_resolution / (h * w))
            rh = round(h * s / quantization) * quantization
            rw = round(w * s / quantization) * quantization
            for r in ((rh, rw), (rw, rh)):
                if r not in res:
                    res.append(r)
        self.resolutions = res
        self.aspects = [h / w for h, w in res]

    def bucket_for(self, height: int, width: int):
        """-> (scale_resolution, crop_resolution) of an image of size height x width."""
        a = height / width
        i = min(range(len(self.aspects)), key=lambda j: abs(self.aspects[j] - a))
        th, tw = self.resolutions[i]
        if a > th / tw:   # relatively taller than the bucket: match widths, crop height
            scale = (round(height * tw / width), tw)
        else:
            scale = (th, round(width * th / height))
        return scale, (th, tw)


class SingleAspectCalculation:
    """aspect_ratio_bucketing off: every image scaled to cover and cropped to the target square."""

    def __init__(self, target_resolution: int):
        self.target_resolution = target_resolution

    def bucket_for(self, height: int, width: int):
        t = self.target_resolution
        if height > width:
            return (round(height * t / width), t), (t, t)
        return (t, round(width * t / height)), (t, t)


def crop_offset(scale_res, crop_res, jitter: bool = False, rng: random.Random | None = None):
    """top-left of the crop (centre crop, or uniform jitter like ScaleCropImage's enable_crop_jitter)."""
    dy, dx = scale_res[0] - crop_res[0], scale_res[1] - crop_res[1]
    if jitter and rng is not None:
        return rng.randint(0, max(dy, 0)), rng.randint(0, max(dx, 0))
    return dy // 2, dx // 2


def aspect_batches(resolutions, batch_size: int, seed: int, epoch: int = 0):
    """AspectBatchSorting: list of global batches (lists of sample indices), each of one
    resolution.  Deterministic in (seed, epoch): every DP rank computes the same list."""
    rng = random.Random(seed * 1_000_003 + epoch)
    groups: dict = {}
    for i, r in enumerate(resolutions):
        groups.setdefault(tuple(r), []).append(i)
    batches = []
    for r in sorted(groups):
        idx = groups[r][:]
        rng.shuffle(idx)
        for k in range(0, len(idx) - batch_size + 1, batch_size):
            batches.append(idx[k:k + batch_size])
    rng.shuffle(batches)
    return batches


def rank_slice(batch, rank: int, world: int):
    """data parallel: rank r takes samples [r*b, (r+1)*b) of a global batch of world*b."""
    if len(batch) % world:
        raise ValueError(f"global batch {len(batch)} does not split over {world} ranks")
    b = len(batch) // world
    return batch[rank * b:(rank + 1) * b]
