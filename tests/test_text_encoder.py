"""Text-encoder oracle pinned to transformers (the reference's own dependency for CLIP / T5, imported
here with random weights -- no checkpoint, no network), plus the build's parameter layout and T5
bucket table on CPU.  The GPU path is checked against this oracle in test_text_encoder_gpu.py."""
import numpy as np
import pytest
import torch

from onetrainer_amd.module import text_encoder as TE
from oracle import text_encoder as OT

transformers = pytest.importorskip("transformers")


def _clip_hf(cfg: TE.CLIPTextConfig, projection: bool):
    c = transformers.CLIPTextConfig(vocab_size=cfg.vocab_size, hidden_size=cfg.hidden_size,
                                    intermediate_size=cfg.intermediate_size, num_hidden_layers=cfg.num_hidden_layers,
                                    num_attention_heads=cfg.num_attention_heads,
                                    max_position_embeddings=cfg.max_position_embeddings, hidden_act=cfg.hidden_act,
                                    projection_dim=cfg.projection_dim or cfg.hidden_size,
                                    bos_token_id=cfg.vocab_size - 2, eos_token_id=2, pad_token_id=1)
    torch.manual_seed(0)
    m = transformers.CLIPTextModelWithProjection(c) if projection else transformers.CLIPTextModel(c)
    return m.eval()


def _ids(B, T, vocab, seed=0):
    g = torch.Generator().manual_seed(seed)
    ids = torch.randint(1, vocab - 2, (B, T), generator=g)
    ids[:, 0] = vocab - 2                     # BOS
    for b in range(B):                        # EOS (the largest id) then padding, at varying positions
        e = 5 + 7 * b
        ids[b, e] = vocab - 1
        ids[b, e + 1:] = 0
    return ids


@pytest.mark.parametrize("projection", [False, True])
def test_clip_oracle_matches_transformers(projection):
    cfg = TE.tiny_clip_config(projection)
    m = _clip_hf(cfg, projection)
    # checkpoint / transformers-4.x names: CLIPTextModel's own keys lack the "text_model." prefix in 5.x
    sd = {(k if k.startswith(("text_model.", "text_projection")) else "text_model." + k): v
          for k, v in m.state_dict().items()}
    names = {n for n, _ in TE.clip_specs(cfg)}
    assert names <= set(sd), sorted(names - set(sd))[:5]        # build layout = transformers names
    ids = _ids(2, 77, cfg.vocab_size)
    with torch.no_grad():
        ref = m(ids, output_hidden_states=True, return_dict=True)
        hs, last, pooled, embeds = OT.clip_forward(sd, ids, cfg.num_attention_heads, cfg.hidden_act)
    assert len(hs) == len(ref.hidden_states)
    for a, b in zip(hs, ref.hidden_states):
        torch.testing.assert_close(a, b, rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(last, ref.last_hidden_state, rtol=1e-4, atol=1e-5)
    if projection:
        torch.testing.assert_close(embeds, ref.text_embeds, rtol=1e-4, atol=1e-5)
    else:
        torch.testing.assert_close(pooled, ref.pooler_output, rtol=1e-4, atol=1e-5)


def test_t5_oracle_matches_transformers():
    cfg = TE.tiny_t5_config()
    c = transformers.T5Config(vocab_size=cfg.vocab_size, d_model=cfg.d_model, d_kv=cfg.d_kv, d_ff=cfg.d_ff,
                              num_layers=cfg.num_layers, num_heads=cfg.num_heads, feed_forward_proj="gated-gelu",
                              relative_attention_num_buckets=cfg.relative_attention_num_buckets,
                              relative_attention_max_distance=cfg.relative_attention_max_distance,
                              dropout_rate=0.0, is_encoder_decoder=False, use_cache=False)
    torch.manual_seed(0)
    m = transformers.T5EncoderModel(c).eval()
    sd = m.state_dict()
    names = {n for n, _ in TE.t5_specs(cfg)}
    assert names <= set(sd), sorted(names - set(sd))[:5]
    ids = _ids(2, 77, cfg.vocab_size, seed=1)
    with torch.no_grad():
        ref = m(ids, output_hidden_states=True, return_dict=True)
        hs = OT.t5_forward(sd, ids, cfg.num_heads)
    assert len(hs) == len(ref.hidden_states)
    for a, b in zip(hs, ref.hidden_states):
        torch.testing.assert_close(a, b, rtol=1e-4, atol=1e-4)


def test_t5_bucket_table_matches_oracle():
    for T in (7, 77, 300):
        pos = torch.arange(T)
        ref = OT.t5_bucket(pos[None, :] - pos[:, None])
        got = TE.t5_relative_buckets(T, 32, 128)
        assert np.array_equal(got, ref.numpy())


def test_text_encoder_weights_from_transformers_dir(tmp_path):
    """a transformers-saved text_encoder/ directory (5.x key names) loads into the build's encoder."""
    from onetrainer_amd.modelLoader.StableDiffusionModelLoader import load_text_encoder
    cfg = TE.tiny_clip_config(True)
    m = _clip_hf(cfg, True)
    m.save_pretrained(str(tmp_path / "text_encoder_2"))
    enc = TE.CLIPTextEncoder(cfg, torch.device("cpu"), seed=9)
    load_text_encoder(enc, str(tmp_path), "text_encoder_2")
    ref = {(k if k.startswith(("text_model.", "text_projection")) else "text_model." + k): v
           for k, v in m.state_dict().items()}
    for n, _ in TE.clip_specs(cfg):
        assert torch.equal(enc.state_dict()[n], ref[n].to(torch.bfloat16)), n
