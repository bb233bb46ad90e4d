"""LoRA adapter structure on CPU (no kernels): module set, names, counts, state-dict layout,
presets -- against the oracle's diffusers module tree and the reference's LoRAModuleWrapper rules
(modules/module/LoRAModule.py:427-587, StableDiffusionXLLoRASetup.py:12-16)."""
import torch

from onetrainer_amd.module import unet as U
from onetrainer_amd.module.lora import LoRAUNetWrapper, PRESETS
from oracle import unet as OU
from oracle.lora import OracleLoRA


def _oracle(cfg):
    return OU.UNet2DConditionModel(OU.UNetConfig(**{k: getattr(cfg, k) for k in OU.UNetConfig.__dataclass_fields__}))


def test_module_set_matches_reference_tree():
    cfg = U.tiny_sdxl_config()
    u = U.UNet2DConditionModel(cfg, "cpu", seed=0, trainable=False)
    w = LoRAUNetWrapper(u, rank=8, alpha=4.0)
    om = _oracle(cfg)
    ref = OracleLoRA(om, 8, 4.0)
    sd = w.state_dict()
    assert {k for k in sd if not k.endswith(".alpha")} == set(ref.params)
    for k, p in ref.params.items():
        assert tuple(sd[k].shape) == tuple(p.shape), k
    assert all(float(sd[k]) == 4.0 for k in sd if k.endswith(".alpha"))
    # fused projections are grouped the way the base GEMMs run
    assert any(len(s.modules) == 3 and s.modules[0].endswith("attn1.to_q") for s in w.sites)
    assert any(len(s.modules) == 2 and s.modules[0].endswith("attn2.to_k") for s in w.sites)


def test_sdxl_rank32_parameter_count():
    # ~98.8 M LoRA parameters over all UNet Linear/Conv2d at r = 32
    n = 0
    for name, shape, kind, _ in U.unet_specs(U.sdxl_config()):
        if name.endswith(".weight") and kind in ("linear", "conv"):
            n += 32 * (shape[1] * (shape[2] * shape[3] if kind == "conv" else 1) + shape[0])
    assert n == 98_825_472


def test_presets_and_filter():
    cfg = U.tiny_sdxl_config()
    u = U.UNet2DConditionModel(cfg, "cpu", seed=0, trainable=False)
    w = LoRAUNetWrapper(u, rank=4, module_filter=PRESETS["attn-only"])
    mods = [m for s in w.sites for m in s.modules]
    assert mods and all("attn" in m for m in mods)
    ref = OracleLoRA(_oracle(cfg), 4, 1.0, PRESETS["attn-only"])
    assert {f"lora_unet.{m}.lora_down.weight" for m in mods} == {k for k in ref.params if k.endswith("down.weight")}


def test_state_dict_round_trip_and_init():
    cfg = U.tiny_sdxl_config()
    u = U.UNet2DConditionModel(cfg, "cpu", seed=0, trainable=False)
    w = LoRAUNetWrapper(u, rank=8, alpha=8.0, seed=1)
    sd = w.state_dict()
    # reference init: down ~ U(+-1/sqrt(fan_in)), up = 0
    for k, v in sd.items():
        if k.endswith("lora_up.weight"):
            assert torch.count_nonzero(v) == 0
        elif k.endswith("lora_down.weight"):
            fan_in = v[0].numel()
            assert v.abs().max() <= 1.0 / fan_in ** 0.5 + 1e-7
    g = torch.Generator().manual_seed(5)
    rnd = {k: (torch.randn(v.shape, generator=g) if not k.endswith(".alpha") else v) for k, v in sd.items()}
    w.load_state_dict(rnd)
    back = w.state_dict()
    for k in rnd:
        assert torch.equal(back[k], rnd[k].float()), k
    assert not u.store.trainable and u.store.grad is None
