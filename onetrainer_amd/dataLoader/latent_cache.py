"""Latent cache writer / reader with aspect-ratio buckets.

Replaces what the reference's mgds pipeline does before and around the steps
(modules/dataLoader/StableDiffusionXLBaseDataLoader.py:65-209 + DataLoaderText2ImageMixin.py:139-294):
  CalcAspect -> AspectBucketing -> ScaleCropImage -> RescaleImageChannels -> EncodeVAE ->
  SampleVAEDistribution(mean) -> DiskCache -> AspectBatchSorting -> OutputPipelineModule.
The mgds on-disk cache format is not pinned (mgds is not in this image); this build's format:
  <cache_dir>/index.json            {"version": 1, "samples": [{"file", "crop_resolution"}, ...]}
  <cache_dir>/<i:08d>.safetensors   latent_image [h, w, C] fp32 NHWC (VAE latent_dist.mean, unscaled; C = 4, FLUX.1 16),
                                    original_resolution / crop_offset / crop_resolution int64 [2],
                                    optional cached text states (text_encoder_*_hidden_state, pooled).
Images are scaled / cropped on the host (data-loader work, as in mgds' worker threads), encoded on
the GPU by the HIP VAE in same-resolution batches, and written by rank 0 only.
The reader yields the reference batch contract (DataLoaderText2ImageMixin._output_modules_from_out_names),
one resolution per GLOBAL batch, each DP rank taking its slice (aspect_bucketing.rank_slice),
with one batch prefetched on a host thread into pinned memory.
"""
from __future__ import annotations

import json
import os
import queue
import threading

import torch
import torch.nn.functional as F
from safetensors.torch import load_file, save_file

from .aspect_bucketing import AspectBucketing, aspect_batches, crop_offset, rank_slice

INDEX = "index.json"


def _to_chw01(img) -> torch.Tensor:
    """PIL image / HWC uint8 tensor / CHW float in [0, 1] -> CHW float32 [0, 1]."""
    if hasattr(img, "convert"):   # PIL
        import numpy as np
        img = torch.from_numpy(np.asarray(img.convert("RGB")).copy())
    if img.dtype == torch.uint8:
        img = img.permute(2, 0, 1).float() / 255.0 if img.shape[-1] == 3 else img.float() / 255.0
    return img.float().contiguous()


def scale_crop(img: torch.Tensor, scale_res, crop_res, offset):
    """mgds ScaleCropImage: bilinear (antialiased) resize to scale_res, then crop crop_res at offset."""
    x = F.interpolate(img[None], size=tuple(scale_res), mode="bilinear", antialias=True, align_corners=False)[0]
    y0, x0 = offset
    return x[:, y0:y0 + crop_res[0], x0:x0 + crop_res[1]].clamp(0.0, 1.0).contiguous()


class LatentCacheWriter:
    def __init__(self, encode_fn, cache_dir: str, bucketing, device, encode_batch: int = 8, rank: int = 0,
                 text_fn=None):
        """encode_fn: [B, 3, H, W] fp32 [0, 1] on `device` -> latent NHWC fp32 [B, H/8, W/8, C]
        (module.vae.AutoencoderKLEncoder.encode).  text_fn (optional): {name: int64 token ids [B, T]}
        on `device` -> {cache key: [B, ...]} (module.text_encoder.encode_sdxl_text & co.), applied to
        samples that carry "tokens" -- the reference's text-encoder caching step."""
        self.encode_fn, self.cache_dir, self.bucketing = encode_fn, cache_dir, bucketing
        self.device, self.encode_batch, self.rank = torch.device(device), encode_batch, rank
        self.text_fn = text_fn

    def write(self, samples):
        """samples: iterable of dicts {"image": PIL / tensor, optional "text": {name: tensor}}.
        Returns the number of cached samples."""
        os.makedirs(self.cache_dir, exist_ok=True)
        prepared = []
        for i, s in enumerate(samples):
            img = _to_chw01(s["image"])
            h, w = img.shape[1], img.shape[2]
            scale_res, crop_res = self.bucketing.bucket_for(h, w)
            off = crop_offset(scale_res, crop_res)
            prepared.append((i, img, (h, w), scale_res, crop_res, off, dict(s.get("text") or {}), s.get("tokens")))
        by_res: dict = {}
        for p in prepared:
            by_res.setdefault(tuple(p[4]), []).append(p)
        index = [None] * len(prepared)
        for res in sorted(by_res):
            group = by_res[res]
            for k in range(0, len(group), self.encode_batch):
                chunk = group[k:k + self.encode_batch]
                imgs = torch.stack([scale_crop(p[1], p[3], p[4], p[5]) for p in chunk]).to(self.device)
                lat = self.encode_fn(imgs).float().cpu()
                tok = [p for p in chunk if p[7] is not None]
                if tok and self.text_fn is not None:
                    names = list(tok[0][7])
                    states = self.text_fn({n: torch.stack([torch.as_tensor(p[7][n], dtype=torch.int64)
                                                           for p in tok]).to(self.device) for n in names})
                    for j, p in enumerate(tok):
                        p[6].update({k2: v[j].to(torch.bfloat16) for k2, v in states.items()})
                for p, l_ in zip(chunk, lat):
                    i = p[0]
                    rec = {"latent_image": l_.contiguous(),
                           "original_resolution": torch.tensor(p[2], dtype=torch.int64),
                           "crop_offset": torch.tensor(p[5], dtype=torch.int64),
                           "crop_resolution": torch.tensor(p[4], dtype=torch.int64)}
                    rec.update({k2: v.detach().cpu().contiguous() for k2, v in p[6].items()})
                    fn = f"{i:08d}.safetensors"
                    if self.rank == 0:
                        save_file(rec, os.path.join(self.cache_dir, fn))
                    index[i] = {"file": fn, "crop_resolution": list(p[4])}
        if self.rank == 0:
            with open(os.path.join(self.cache_dir, INDEX), "w") as f:
                json.dump({"version": 1, "samples": index}, f)
        return len(index)


class LatentCacheDataLoader:
    """Reader in the reference's BaseDataLoader shape: get_data_set().start_next_epoch() /
    approximate_length(), get_data_loader() iterable of batches on `device`."""

    def __init__(self, cache_dir: str, batch_size: int, device, seed: int = 0, rank: int = 0, world: int = 1,
                 text_defaults: dict | None = None, prefetch: bool = True):
        with open(os.path.join(cache_dir, INDEX)) as f:
            self.index = json.load(f)["samples"]
        self.cache_dir, self.batch_size, self.device = cache_dir, batch_size, torch.device(device)
        self.seed, self.rank, self.world, self.epoch = seed, rank, world, -1
        self.text_defaults = text_defaults or {}
        self.prefetch = prefetch
        self._batches = []

    # BaseDataLoader.get_data_set() -> MGDS-like
    def get_data_set(self):
        return self

    def start_next_epoch(self):
        self.epoch += 1
        res = [tuple(s["crop_resolution"]) for s in self.index]
        self._batches = aspect_batches(res, self.batch_size * self.world, self.seed, self.epoch)

    def approximate_length(self):
        if not self._batches:
            res = [tuple(s["crop_resolution"]) for s in self.index]
            return len(aspect_batches(res, self.batch_size * self.world, self.seed, 0))
        return len(self._batches)

    def _load(self, idx):
        recs = [load_file(os.path.join(self.cache_dir, self.index[i]["file"])) for i in idx]
        b = len(recs)
        out = {"latent_image": torch.stack([r["latent_image"] for r in recs])}
        for k in ("original_resolution", "crop_offset", "crop_resolution"):
            v = torch.stack([r[k] for r in recs])
            out[k] = (v[:, 0], v[:, 1])
        text_keys = {k for r in recs for k in r if k.startswith("text_encoder")}
        for k in text_keys:
            out[k] = torch.stack([r[k] for r in recs])
        for k, v in self.text_defaults.items():
            if k not in out:
                out[k] = v.expand(b, *v.shape).contiguous()
        out["loss_weight"] = torch.ones(b)
        if torch.cuda.is_available():
            for k, v in list(out.items()):
                if isinstance(v, torch.Tensor):
                    out[k] = v.pin_memory()
        return out

    def _to_device(self, host):
        dev = {}
        for k, v in host.items():
            if isinstance(v, tuple):
                dev[k] = tuple(t.to(self.device, non_blocking=True) for t in v)
            else:
                dev[k] = v.to(self.device, non_blocking=True)
        # the reference's [B, C, h, w] contract, as a view of the cached channels-last (NHWC) storage
        dev["latent_image"] = dev["latent_image"].permute(0, 3, 1, 2)
        dev["concept_type"] = ["STANDARD"] * dev["latent_image"].shape[0]
        return dev

    def get_data_loader(self):
        if not self._batches:
            self.start_next_epoch()
        mine = [rank_slice(b, self.rank, self.world) for b in self._batches]
        if not self.prefetch:
            for idx in mine:
                yield self._to_device(self._load(idx))
            return
        q: queue.Queue = queue.Queue(maxsize=2)

        def worker():
            for idx in mine:
                q.put(self._load(idx))
            q.put(None)

        t = threading.Thread(target=worker, daemon=True)
        t.start()
        while True:
            host = q.get()
            if host is None:
                break
            yield self._to_device(host)
        t.join()


def default_bucketing(config):
    from .aspect_bucketing import SingleAspectCalculation, quantization_for
    target = config.resolution_hw()[0]
    if getattr(config, "aspect_ratio_bucketing", True):
        return AspectBucketing(target, quantization_for(config.model_type))
    return SingleAspectCalculation(target)
