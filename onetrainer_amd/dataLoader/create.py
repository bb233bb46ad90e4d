"""create_data_loader: what modules/util/create.py:391-431 + the family data loaders
(StableDiffusionXLBaseDataLoader.py:33-288, DataLoaderText2ImageMixin.py:139-294) do for the
trainer, on this build's latent cache (dataLoader/latent_cache.py).

  * <cache_dir>/index.json present -> read it (LatentCacheDataLoader, ARB batches, rank slices);
  * otherwise enumerate the concepts' images (config.concepts, else the concept_file_name JSON),
    captions from the sample's .txt next to the image (prompt_source 'sample'), the concept's
    prompt file ('concept') or the file name ('filename'); tokenize with the checkpoint's own
    tokenizers (<base_model>/tokenizer[_2], transformers); encode images with the HIP VAE encoder and
    text with the HIP text encoders the model carries (attach_cache_encoders, loaded by the model
    loader with the base weights), write the cache on rank 0, then read it.
mgds itself is not in this image: enumeration and captions follow the reference's
ConceptConfig fields; the bucket list is dataLoader/aspect_bucketing.py (parity unpinned).
"""
from __future__ import annotations

import json
import os

import torch

from ..util.config.plain import plain
from .latent_cache import INDEX, LatentCacheDataLoader, LatentCacheWriter, default_bucketing

IMAGE_EXT = (".png", ".jpg", ".jpeg", ".webp", ".bmp", ".tif", ".tiff")


def cache_ready(config) -> bool:
    return os.path.isfile(os.path.join(plain(config).cache_dir, INDEX))


def has_concepts(config) -> bool:
    cfg = plain(config)
    return bool(cfg.concepts) or bool(cfg.concept_file_name and os.path.isfile(cfg.concept_file_name))


def _family(model_type: str) -> str:
    if model_type.startswith("FLUX"):
        return "flux"
    if model_type.startswith("STABLE_DIFFUSION_XL"):
        return "sdxl"
    return "sd15"


def attach_cache_encoders(model, config, device) -> None:
    """VAE encoder + caching text encoders on the model, before the model loader runs (it fills
    model.vae_encoder / text_encoder_1 / text_encoder_2 from the base checkpoint)."""
    from ..module import text_encoder as TE
    from ..module import vae as V
    cfg = plain(config)
    fam = _family(cfg.model_type)
    vcfg = {"sdxl": V.sdxl_vae_config, "sd15": V.sd15_vae_config, "flux": V.flux_vae_config}[fam]
    model.vae_encoder = V.AutoencoderKLEncoder(vcfg(), device, seed=0)
    model.text_encoder_1 = TE.CLIPTextEncoder(TE.clip_l_config(), device)
    if fam == "sdxl":
        model.text_encoder_2 = TE.CLIPTextEncoder(TE.clip_bigg_config(), device)
    elif fam == "flux":
        model.text_encoder_2 = TE.T5TextEncoder(TE.t5_xxl_config(), device)


def _concepts(cfg) -> list:
    concepts = cfg.concepts
    if not concepts:
        path = cfg.concept_file_name
        if not path or not os.path.isfile(path):
            raise FileNotFoundError(f"no concepts: config.concepts is empty and concept file {path!r} is missing")
        with open(path) as f:
            concepts = json.load(f)
    out = []
    for c in concepts:
        c = c.to_dict() if hasattr(c, "to_dict") else dict(c)
        if c.get("enabled", True):
            out.append(c)
    return out


def _caption(img_path: str, concept: dict) -> str:
    text = concept.get("text") or {}
    src = text.get("prompt_source", "sample")
    if src == "filename":
        return os.path.splitext(os.path.basename(img_path))[0]
    if src == "concept":
        p = text.get("prompt_path", "")
        if p and os.path.isfile(p):
            with open(p) as f:
                return f.readline().strip()
        return ""
    txt = os.path.splitext(img_path)[0] + ".txt"
    if os.path.isfile(txt):
        with open(txt) as f:
            return f.readline().strip()
    return ""


def enumerate_samples(config) -> list[tuple[str, str]]:
    """(image path, caption) for every enabled concept (mgds CollectPaths + caption loading)."""
    cfg = plain(config)
    out = []
    for c in _concepts(cfg):
        root = c["path"]
        walk = os.walk(root) if c.get("include_subdirectories", False) else [(root, [], os.listdir(root))]
        for d, _, files in walk:
            for fn in sorted(files):
                if fn.lower().endswith(IMAGE_EXT) and not fn.lower().endswith("-masklabel.png"):
                    p = os.path.join(d, fn)
                    out.append((p, _caption(p, c)))
    return out


def _tokenizers(cfg):
    from transformers import CLIPTokenizer
    base = cfg.base_model_name
    fam = _family(cfg.model_type)
    toks = [CLIPTokenizer.from_pretrained(os.path.join(base, "tokenizer"))]
    if fam == "sdxl":
        toks.append(CLIPTokenizer.from_pretrained(os.path.join(base, "tokenizer_2")))
    elif fam == "flux":
        from transformers import AutoTokenizer   # T5TokenizerFast (tokenizer.json) or the sentencepiece T5Tokenizer
        toks.append(AutoTokenizer.from_pretrained(os.path.join(base, "tokenizer_2")))
    return toks


def build_cache(config, model, device, rank: int = 0) -> int:
    from PIL import Image

    from ..module import text_encoder as TE
    cfg = plain(config)
    fam = _family(cfg.model_type)
    samples = enumerate_samples(cfg)
    if not samples:
        raise FileNotFoundError("no training images found in the configured concepts")
    toks = _tokenizers(cfg)

    def ids(tok, caption):
        return tok(caption, padding="max_length", max_length=77, truncation=True, return_tensors="pt").input_ids[0]

    if fam in ("sdxl", "flux"):
        enc_text = TE.encode_sdxl_text if fam == "sdxl" else TE.encode_flux_text
        text_fn = lambda t: enc_text(model.text_encoder_1, model.text_encoder_2,  # noqa: E731
                                     t["tokens_1"], t["tokens_2"])
        rows = ({"image": Image.open(p), "tokens": {"tokens_1": ids(toks[0], c), "tokens_2": ids(toks[1], c)}}
                for p, c in samples)
    else:
        text_fn = lambda t: TE.encode_sd15_text(model.text_encoder_1, t["tokens_1"])  # noqa: E731
        rows = ({"image": Image.open(p), "tokens": {"tokens_1": ids(toks[0], c)}} for p, c in samples)
    # a generator: each file is opened (and, once decoded, closed) inside the writer's loop, so a concept
    # folder larger than the open-file limit caches
    writer = LatentCacheWriter(lambda im: model.vae_encoder.encode(im), cfg.cache_dir, default_bucketing(cfg),
                               device, rank=rank, text_fn=text_fn)
    return writer.write(rows)


def create_data_loader(config, model, device, rank: int = 0, world: int = 1):
    cfg = plain(config)
    if not cache_ready(cfg):
        if getattr(model, "vae_encoder", None) is None:
            raise RuntimeError("no latent cache at cache_dir and no VAE encoder on the model "
                               "(GenericTrainer.start attaches one when the cache must be built)")
        build_cache(cfg, model, device, rank)
        if world > 1:
            torch.distributed.barrier()
        for attr in ("vae_encoder", "text_encoder_1", "text_encoder_2"):   # caching done: free the encoders
            if hasattr(model, attr):
                setattr(model, attr, None)
        if torch.cuda.is_available():
            torch.cuda.empty_cache()
    return LatentCacheDataLoader(cfg.cache_dir, cfg.batch_size, device, seed=0, rank=rank, world=world)
