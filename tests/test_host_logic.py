"""Host-side logic on CPU: LR schedule vs the reference's own values, config loading, flat store,
UNet parameter graph vs the oracle and the known SD/SDXL sizes, FLOP counter."""
import math
from pathlib import Path

import numpy as np
import pytest
import torch

from onetrainer_amd.module import unet as U
from onetrainer_amd.module.param_store import FlatParamStore
from onetrainer_amd.util import lr_scheduler_util as L
from onetrainer_amd.util.config.TrainConfig import TrainConfig
from oracle import unet as OU

G = np.load(Path(__file__).parent / "golden" / "reference_math.npz")


@pytest.mark.parametrize("name,fn", [
    ("constant", L.lr_lambda_warmup(200, L.lr_lambda_constant())),
    ("cosine", L.lr_lambda_warmup(50, L.lr_lambda_cosine(300))),
    ("linear", L.lr_lambda_warmup(10, L.lr_lambda_linear(390)))])
def test_lr_lambdas_match_reference(name, fn):
    got = np.array([fn(s) for s in range(400)], dtype=np.float64)
    np.testing.assert_array_equal(got, G[f"lr_{name}"])


def test_lambda_lr_drives_param_groups():
    p = torch.nn.Parameter(torch.zeros(4))
    opt = torch.optim.SGD([p], lr=1.0)
    sch = L.create_lr_scheduler(opt, "CONSTANT", warmup_steps=4, approximate_epoch_length=10, num_epochs=1)
    lrs = []
    for _ in range(6):
        lrs.append(opt.param_groups[0]["lr"])
        opt.step()
        sch.step()
    assert lrs == [0.0, 0.25, 0.5, 0.75, 1.0, 1.0]


def test_reference_presets_load():
    ref = Path("/root/reference/training_presets")
    if not ref.exists():
        pytest.skip("reference presets not present on this host")
    c = TrainConfig.load(str(ref / "#sdxl 1.0.json"))
    assert c.model_type == "STABLE_DIFFUSION_XL_10_BASE" and c.weight_dtype == "BFLOAT_16"
    assert c.vae.weight_dtype == "FLOAT_32" and c.text_encoder.train is False
    c = TrainConfig.load(str(ref / "#sdxl 1.0 LoRA.json"))
    assert c.training_method == "LORA"


def test_flat_store_layout_and_fused_views():
    st = FlatParamStore([("a", (3, 5), "g"), ("q", (8, 8), "g"), ("k", (8, 8), "g"), ("v", (8, 8), "g"),
                         ("b", (7,), "h")], torch.bfloat16, "cpu")
    for n, s in st.slots.items():
        assert s.offset % 8 == 0
    qkv = st.view(["q", "k", "v"], (24, 8))
    qkv.fill_(2.0)
    assert float(st.params["k"].sum()) == 128.0
    assert st.params["q"].grad.data_ptr() == st.view(["q"], grad=True).data_ptr()
    with pytest.raises(ValueError):
        st.view(["a", "k"])
    assert st.group_ranges()["h"][0] == st.slots["b"].offset


def test_unet_specs_match_reference_sizes():
    n_sdxl = sum(math.prod(s) for _, s, _, _ in U.unet_specs(U.sdxl_config()))
    n_sd15 = sum(math.prod(s) for _, s, _, _ in U.unet_specs(U.sd15_config()))
    assert n_sdxl == 2_567_463_684 and len(U.unet_specs(U.sdxl_config())) == 1680
    assert n_sd15 == 859_520_964 and len(U.unet_specs(U.sd15_config())) == 686


@pytest.mark.parametrize("cfgfn", [U.sdxl_config, U.sd15_config, U.tiny_sdxl_config])
def test_unet_names_and_shapes_match_oracle(cfgfn):
    cfg = cfgfn()
    with torch.device("meta"):
        om = OU.UNet2DConditionModel(OU.UNetConfig(**{k: getattr(cfg, k) for k in OU.UNetConfig.__dataclass_fields__}))
    ours = {n: tuple(s) for n, s, _, _ in U.unet_specs(cfg)}
    theirs = {n: tuple(p.shape) for n, p in om.named_parameters()}
    assert ours == theirs


def test_state_dict_roundtrip_cpu():
    m = U.UNet2DConditionModel(U.tiny_sdxl_config(), "cpu", seed=3)
    sd = m.state_dict()
    m2 = U.UNet2DConditionModel(U.tiny_sdxl_config(), "cpu", seed=None)
    m2.load_state_dict({k: v.float() for k, v in sd.items()})
    assert torch.equal(m2.store.data, m.store.data)
    assert torch.count_nonzero(m.store.params["conv_in.weight"][..., 4:]) == 0


def test_flop_counter_matches_survey():
    assert abs(U.flops_per_image(U.sdxl_config(), 128, 128) / 1e12 - 6.761) < 1e-3
    assert abs(U.flops_per_image(U.sdxl_config(), 64, 64) / 1e12 - 1.589) < 1e-3
    assert abs(U.flops_per_image(U.sd15_config(), 64, 64) / 1e12 - 0.803) < 1e-3


def test_vae_encoder_spec_and_flops():
    """VAE encoder 1.12 TF @512, 4.88 TF @1024; 34.16M params, names equal
    to the oracle's (diffusers AutoencoderKL encoder + quant_conv)."""
    from onetrainer_amd.module import vae as V
    from oracle import vae as OV
    cfg = V.sdxl_vae_config()
    assert abs(V.flops_per_image(cfg, 1024, 1024) / 1e12 - 4.88) < 5e-3
    assert abs(V.flops_per_image(cfg, 512, 512) / 1e12 - 1.12) < 5e-3
    specs = V.vae_encoder_specs(cfg)
    om = OV.AutoencoderKLEncoder(cfg)
    assert {n for n, *_ in specs} == set(om.state_dict())
    assert sum(math.prod(s) for _, s, _, _ in specs) == sum(p.numel() for p in om.parameters()) == 34_163_664
    # FLUX.1's encoder: 16 latent channels (conv_out 512 -> 32), no quant_conv
    fcfg = V.flux_vae_config()
    fspecs = V.vae_encoder_specs(fcfg)
    fom = OV.AutoencoderKLEncoder(fcfg)
    assert {n for n, *_ in fspecs} == set(fom.state_dict()) and not any(n.startswith("quant_conv") for n, *_ in fspecs)
    n_flux = 34_163_664 - (8 * 8 + 8) - (512 * 8 * 9 + 8) + (512 * 32 * 9 + 32)
    assert sum(math.prod(s) for _, s, _, _ in fspecs) == sum(p.numel() for p in fom.parameters()) == n_flux


def test_flux_spec_and_flops():
    """FLUX@768 34.71 TF, @1024 66.07 TF forward; FLUX.1-dev 11.9 B params;
    parameter names equal the oracle's (diffusers FluxTransformer2DModel); RoPE tables match."""
    import numpy as np
    import torch
    from onetrainer_amd.module import flux as FX
    from oracle import flux as OF
    c = FX.flux_dev_config()
    assert abs(FX.flops_per_image(c, 2304) / 1e12 - 34.71) < 5e-3
    assert abs(FX.flops_per_image(c, 4096) / 1e12 - 66.07) < 1e-2
    assert sum(math.prod(s) for _, s, _, _ in FX.flux_specs(c)) == 11_901_408_320
    t = FX.tiny_flux_config()
    om = OF.FluxTransformer2DModel(OF.tiny_flux_config())
    assert {n for n, *_ in FX.flux_specs(t)} == set(om.state_dict())
    cs, sn = FX.rope_tables(5, 8, 6, t)
    c2, s2 = OF.rope_tables(torch.cat([torch.zeros(5, 3), OF.prepare_latent_image_ids(8, 6)]), t.axes_dims_rope)
    assert np.abs(cs - c2.numpy()).max() < 1e-6 and np.abs(sn - s2.numpy()).max() < 1e-6


def test_flux_lora_groups():
    """LoRA fusion groups of the Flux transformer (module/lora.py): q|k|v, add_q|k|v, single-block
    q|k|v|proj_mlp, norm1|norm1_context; 'attn-mlp' adapts q|k|v but not proj_mlp (zero rows)."""
    import torch
    from onetrainer_amd.module import flux as FX
    from onetrainer_amd.module.lora import LoRAWrapper
    m = FX.FluxTransformer2DModel(FX.tiny_flux_config(), "cpu", seed=None)
    w = LoRAWrapper(m, rank=4, module_filter=["attn", "ff.net"], prefix="lora_transformer", seed=None)
    s = w.site_of["single_transformer_blocks.0.proj_mlp"]
    assert s.modules == ["single_transformer_blocks.0.attn.to_q", "single_transformer_blocks.0.attn.to_k",
                         "single_transformer_blocks.0.attn.to_v"]
    assert s.n_total == 7 * 256 and s.ranges[2] == (512, 768)
    assert "transformer_blocks.0.ff_context.net.0.proj" not in w.site_of
    assert w.site_for(["transformer_blocks.1.attn.add_q_proj", "transformer_blocks.1.attn.add_k_proj",
                       "transformer_blocks.1.attn.add_v_proj"]) is not None
    full = LoRAWrapper(m, rank=4, prefix="lora_transformer", seed=None)
    assert full.site_of["transformer_blocks.0.norm1.linear"].group == (
        "transformer_blocks.0.norm1.linear", "transformer_blocks.0.norm1_context.linear")
    del torch


def test_gemm_plan_table_wellformed():
    """the committed measured plan table (onetrainer_amd/gemm_plans_mi355x.json): every row a full
    signature key with a valid (tile, split-K) plan; loaded by kernels._plan_table."""
    import json
    from onetrainer_amd import kernels as K
    with open(K._TABLE_PATH) as f:
        rows = json.load(f)["plans"]
    assert len(rows) > 100
    for r in rows:
        assert len(r["key"]) == 16 and r["key"][2] > 0 and r["key"][3] > 0 and r["key"][4] > 0
        assert -1 <= r["tile"] <= 8 and r["splits"] >= 1
        if r["key"][1] == 5 or r["key"][5]:   # conv-weight B / second K segment: v2 tiles only
            assert r["tile"] >= 0
    assert len(K._plan_table()) == len({tuple(r["key"]) for r in rows})


def test_lora_down_projection_split_rule():
    """kernels._skinny_split: only K-mode-A rows on the skinny tiles (5 / 6) without split-K, N <= 128, that fill
    under 128 workgroups with >= 8 K-steps get split-K (up to ~256 workgroups, at most 8 splits)."""
    from onetrainer_amd import kernels as K
    z = (0,) * 11
    t = {(0, 0, 4032, 32, 1280) + z: (6, 1),     # LoRA down-projection: 63 tiles, 20 K-steps -> 4 splits
         (0, 1, 16128, 32, 640) + z: (5, 1),     # 127 tiles, 10 K-steps -> 2 splits
         (0, 0, 4096, 96, 1280) + z: (6, 1),     # fused q|k|v ranks
         (0, 0, 4096, 320, 1280) + z: (6, 1),    # N > 128: untouched
         (1, 1, 32, 1280, 16384) + z: (6, 8),    # weight gradient (MN-mode A): untouched
         (0, 0, 4096, 32, 320) + z: (6, 1),      # 5 K-steps: untouched
         (0, 0, 4032, 32, 1280, 1) + (0,) * 10: (4, 1)}   # another tile: untouched
    before = dict(t)
    K._skinny_split(t)
    assert t[(0, 0, 4032, 32, 1280) + z] == (6, 4)
    assert t[(0, 1, 16128, 32, 640) + z] == (5, 2)
    assert t[(0, 0, 4096, 96, 1280) + z] == (6, 4)
    for k in list(before)[3:]:
        assert t[k] == before[k], k


def test_overlapped_norm_buckets_skip_empty_tensors():
    """OverlappedGradNorm bucket chunk ranges: a tensor with no norm chunks (numel 0) must not stretch a
    bucket's range back to chunk 0 (every earlier tensor's chunks would be summed twice into the norm)."""
    from types import SimpleNamespace

    from onetrainer_amd.util.optimizer.adamw_fused import OverlappedGradNorm
    numels = {"a": 70000, "b": 0, "c": 1000, "d": 0, "e": 5}
    order = list(numels)
    chunk_tensor = []
    for ti, n in enumerate(order):
        chunk_tensor += [ti] * ((numels[n] + (1 << 16) - 1) >> 16)
    store = SimpleNamespace(order=order, slots={n: SimpleNamespace(numel=v) for n, v in numels.items()},
                            grad=torch.zeros(1, dtype=torch.bfloat16), ready_hooks=[])
    opt = SimpleNamespace(store=store, _chunk_tensor=chunk_tensor)
    for bucket_bytes in (2, 20, 1 << 30):   # 20 B: e and the empty d share a bucket
        ov = OverlappedGradNorm(opt, bucket_bytes=bucket_bytes)
        covered = []
        for c0, c1, names in ov.buckets:
            if c0 is None:
                assert all(numels[n] == 0 for n in names)
                continue
            want = [ci for ci, ti in enumerate(chunk_tensor) if order[ti] in names]
            assert list(range(c0, c1)) == want, (c0, c1, names)
            covered += want
        assert sorted(covered) == list(range(len(chunk_tensor)))
