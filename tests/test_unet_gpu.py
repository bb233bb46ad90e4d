"""Whole-network parity: HIP UNet (bf16, NHWC) vs the oracle UNet (fp32, CPU), same weights."""
import pytest
import torch

from onetrainer_amd.module import unet as U
from oracle import unet as OU

pytestmark = pytest.mark.gpu


def _oracle_cfg(cfg):
    return OU.UNetConfig(**{k: getattr(cfg, k) for k in OU.UNetConfig.__dataclass_fields__})


def _cos(a, b):
    a, b = a.flatten().double(), b.flatten().double()
    return (a @ b / (a.norm() * b.norm() + 1e-30)).item()


@pytest.mark.parametrize("cfgname", ["tiny_sdxl", "tiny_sd15"])
def test_unet_forward_backward_matches_oracle(dev, cfgname):
    torch.manual_seed(0)
    cfg = getattr(U, cfgname + "_config")()
    m = U.UNet2DConditionModel(cfg, dev, seed=1)
    om = OU.UNet2DConditionModel(_oracle_cfg(cfg))
    om.load_state_dict({k: v.float().cpu() for k, v in m.state_dict().items()})
    B, H, W = 2, 16, 16
    x = torch.randn(B, 4, H, W)
    t = torch.tensor([10, 700], dtype=torch.int32)
    ehs = torch.randn(B, 77, cfg.cross_attention_dim)
    te = torch.randn(B, cfg.projection_class_embeddings_input_dim - 6 * cfg.addition_time_embed_dim)
    tid = torch.tensor([[128., 128., 0., 0., 128., 128.]] * B)
    if not cfg.addition_embed:   # SD 1.5: no pooled text / time_ids conditioning
        te = tid = None
    xin = torch.zeros(B, H, W, 8, dtype=torch.bfloat16, device=dev)
    xin[..., :4] = x.permute(0, 2, 3, 1).to(dev).bfloat16()
    dv = (lambda v: None if v is None else v.to(dev))
    out = m(xin, t.to(dev), ehs.to(dev).bfloat16(), None if te is None else te.to(dev).bfloat16(), dv(tid))
    # oracle sees the same bf16-rounded inputs
    ref = om(x.bfloat16().float(), t, ehs.bfloat16().float(), None if te is None else te.bfloat16().float(), tid)
    o4 = out[..., :4].float().cpu()
    r4 = ref.permute(0, 2, 3, 1)
    err = (o4 - r4.detach()).abs().max() / r4.detach().abs().max()
    assert err < 3e-2, f"forward rel err {err}"
    assert _cos(o4, r4.detach()) > 0.9995
    assert torch.count_nonzero(out[..., 4:]) == 0

    w = torch.randn(B, H, W, 4)
    m.store.begin_backward()
    (out[..., :4].float() * w.to(dev)).sum().backward()
    m.store.finish_backward()
    (r4 * w).sum().backward()
    g = m.state_dict(grads=True)
    worst = []
    for name, p in om.named_parameters():
        gg = g[name].float().cpu()
        c = _cos(gg, p.grad)
        worst.append((c, name))
        assert c > 0.995, f"{name}: cosine {c}"
    worst.sort()
    print("worst grad cosines:", worst[:5])
