"""Text-encoder caching path on the GPU vs the oracle restatement
(oracle/text_encoder.py, itself pinned to transformers in test_text_encoder.py), same weights.
bf16 GEMMs / norms against fp32: max error within 3e-2 of the output scale.  Covers the tiny
configs, one layer at the real CLIP-L / bigG / T5-XXL widths, the per-family selections
(SDXL penultimate states + bigG text_embeds, SD 1.5 final-normed state, Flux CLIP pooled + T5),
and the latent-cache writer's token -> text-state hook."""
import pytest
import torch

from onetrainer_amd.module import text_encoder as TE
from oracle import text_encoder as OT

pytestmark = pytest.mark.gpu


def close(out, ref, tol=3e-2):
    out, ref = out.float().cpu(), ref.float()
    err = (out - ref).abs().max().item()
    scale = ref.abs().max().item() + 1e-6
    assert err / scale < tol, f"max err {err} vs scale {scale}"


def _ids(B, T, vocab, seed=0):
    g = torch.Generator().manual_seed(seed)
    ids = torch.randint(1, vocab - 2, (B, T), generator=g)
    ids[:, 0] = vocab - 2
    for b in range(B):
        e = 5 + 11 * b
        ids[b, e] = vocab - 1
        ids[b, e + 1:] = 0
    return ids


def _sd(enc):
    return {k: v.float().cpu() for k, v in enc.state_dict().items()}


@pytest.mark.parametrize("cfg", [TE.tiny_clip_config(False), TE.tiny_clip_config(True),
                                 TE.CLIPTextConfig(num_hidden_layers=2),
                                 TE.CLIPTextConfig(hidden_size=1280, intermediate_size=5120, num_hidden_layers=2,
                                                   num_attention_heads=20, hidden_act="gelu", projection_dim=1280)])
def test_clip_encoder(dev, cfg):
    enc = TE.CLIPTextEncoder(cfg, dev, seed=1)
    ids = _ids(3, 77, cfg.vocab_size)
    sd = _sd(enc)
    hs, last, pooled, embeds = OT.clip_forward(sd, ids, cfg.num_attention_heads, cfg.hidden_act)
    got_hs, got_last = enc.forward(ids.to(dev), set(range(cfg.num_hidden_layers + 1)))
    for i, h in got_hs.items():
        close(h, hs[i])
    close(got_last.view(3, 77, -1), last)
    p = enc.pooled(ids.to(dev), got_last)
    close(p, embeds if cfg.projection_dim else pooled)
    # encode_clip selections (SDXL: -2 no norm; SD 1.5: -1 + norm; clip skip 1)
    for dl, skip, ln in ((-2, 0, False), (-1, 0, True), (-1, 1, True)):
        out, _ = enc.encode(ids.to(dev), default_layer=dl, layer_skip=skip, add_layer_norm=ln)
        ref, _ = OT.encode_clip(sd, ids, cfg.num_attention_heads, cfg.hidden_act, dl, skip, ln)
        close(out, ref)


@pytest.mark.parametrize("cfg", [TE.tiny_t5_config(), TE.T5Config(num_layers=1)])
def test_t5_encoder(dev, cfg):
    enc = TE.T5TextEncoder(cfg, dev, seed=2)
    ids = _ids(2, 77, cfg.vocab_size, seed=3)
    hs = OT.t5_forward(_sd(enc), ids, cfg.num_heads)
    got, last = enc.forward(ids.to(dev), set(range(cfg.num_layers + 1)))
    for i, h in got.items():
        close(h, hs[i])
    close(enc.encode(ids.to(dev)), hs[-1])


def test_family_encodes_and_cache_hook(dev, tmp_path):
    te1 = TE.CLIPTextEncoder(TE.tiny_clip_config(False), dev, seed=4)
    te2 = TE.CLIPTextEncoder(TE.tiny_clip_config(True), dev, seed=5)
    ids1, ids2 = _ids(2, 77, 1000, 6), _ids(2, 77, 1000, 7)
    out = TE.encode_sdxl_text(te1, te2, ids1.to(dev), ids2.to(dev))
    h1, _ = OT.encode_clip(_sd(te1), ids1, 2, "quick_gelu", -2, 0, False)
    h2, pooled = OT.encode_clip(_sd(te2), ids2, 2, "gelu", -2, 0, False)
    close(out["text_encoder_1_hidden_state"], h1)
    close(out["text_encoder_2_hidden_state"], h2)
    close(out["text_encoder_2_pooled_state"], pooled)
    t5 = TE.T5TextEncoder(TE.tiny_t5_config(), dev, seed=8)
    fl = TE.encode_flux_text(te1, t5, ids1.to(dev), ids2.to(dev))
    _, last, pooled1, _ = OT.clip_forward(_sd(te1), ids1, 2, "quick_gelu")
    close(fl["text_encoder_1_pooled_state"], pooled1)
    close(fl["text_encoder_2_hidden_state"], OT.t5_forward(_sd(t5), ids2, 8)[-1])

    from onetrainer_amd.dataLoader.aspect_bucketing import AspectBucketing
    from onetrainer_amd.dataLoader.latent_cache import LatentCacheDataLoader, LatentCacheWriter
    from onetrainer_amd.module import vae as V
    vae = V.AutoencoderKLEncoder(V.tiny_vae_config(), dev, seed=0)
    w = LatentCacheWriter(vae.encode, str(tmp_path), AspectBucketing(64, 8), dev,
                          text_fn=lambda t: TE.encode_sdxl_text(te1, te2, t["tokens_1"], t["tokens_2"]))
    samples = [{"image": torch.rand(3, 64, 64), "tokens": {"tokens_1": ids1[i], "tokens_2": ids2[i]}} for i in range(2)]
    assert w.write(samples) == 2
    dl = LatentCacheDataLoader(str(tmp_path), 2, dev, prefetch=False)
    batch = next(iter(dl.get_data_loader()))
    close(batch["text_encoder_2_pooled_state"], pooled)
    assert batch["text_encoder_1_hidden_state"].shape == (2, 77, 64)
