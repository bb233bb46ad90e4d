"""LoRA forward with the down-projection fused into the base GEMM (GemmArgs.D, gemm2_tiles_e.hip) against the
two-launch form it replaces (t = x A^T, then the base GEMM with t as its second K segment), on the GPU.

With the two-launch form's GEMMs at one split, t and y are bit-identical: t is summed over K in the same 64-deep steps
and 16x16x32 MFMAs in both, rounded to bf16 the same way, and the second segment adds t (sB)^T to the same accumulators
after the base K loop.  Reference op: LoRAModule.forward (modules/module/LoRAModule.py:318-322)."""
import pytest
import torch
import torch.nn.functional as F

from onetrainer_amd import kernels as K

pytestmark = pytest.mark.gpu

BF = torch.bfloat16


def rnd(*s, dev, scale=1.0):
    return (torch.randn(*s, device=dev) * scale).to(BF)


def block_up(P, pw, r, dev, scale=0.05):
    """the fused group's up operand: block-diagonal [P*pw, P*r] (module/lora.py LoraSite.up2)"""
    up = torch.zeros(P * pw, P * r, device=dev)
    for p in range(P):
        up[p * pw:(p + 1) * pw, p * r:(p + 1) * r] = torch.randn(pw, r, device=dev) * scale
    return up.to(BF)


BN = {1: 128, 4: 128, 7: 160, 8: 160}   # tile widths of the fused instances (parts must not straddle tiles)


def two_launch_split1(monkeypatch, fn):
    with monkeypatch.context() as m:
        m.setattr(K, "_gemm_forced_splits", 1)   # every GEMM of the reference at one split (ctypes path)
        return fn()


@pytest.mark.parametrize("tile", [1, 4, 7, 8])
@pytest.mark.parametrize("M,Kd,P,pw,epi", [(1000, 640, 1, 640, True), (4096, 1280, 3, 1280, False),
                                           (300, 1280, 2, 1280, True)])
def test_linear_lora_fused_bitwise(dev, monkeypatch, tile, M, Kd, P, pw, epi):
    if pw % BN[tile]:
        pytest.skip("adapter part narrower than a tile multiple: the launcher refuses (two-launch form)")
    torch.manual_seed(21)
    r = 32
    x, w = rnd(M, Kd, dev=dev), rnd(P * pw, Kd, dev=dev, scale=0.05)
    down, up2 = rnd(P * r, Kd, dev=dev, scale=0.05), block_up(P, pw, r, dev)
    b = rnd(P * pw, dev=dev) if epi else None
    res = rnd(M, P * pw, dev=dev) if epi else None
    t = torch.full((M, P * r), float("nan"), device=dev, dtype=BF)
    y = K.linear_lora(x, w, b, res, down, up2, t, r, pw, tile=tile)

    def ref():
        t_ref = K.linear(x, down)
        return t_ref, K.linear(x, w, bias=b, residual=res, lora=(t_ref, up2))
    t_ref, y_ref = two_launch_split1(monkeypatch, ref)
    assert torch.equal(t, t_ref), (t.float() - t_ref.float()).abs().max().item()
    assert torch.equal(y, y_ref), (y.float() - y_ref.float()).abs().max().item()
    # and the fp32 product it stands for
    want = x.float() @ w.float().t() + t_ref.float() @ up2.float().t()
    if epi:
        want = want + b.float() + res.float()
    err = (y.float() - want).abs().max().item() / want.abs().max().item()
    assert err < 2e-2, err


@pytest.mark.parametrize("tile", [4, 7])
@pytest.mark.parametrize("N,H,W,Cin,Cout,stride,up", [(2, 32, 32, 320, 640, 1, False), (1, 16, 24, 640, 320, 2, False),
                                                      (2, 8, 8, 320, 320, 1, True), (1, 16, 16, 640, 1280, 1, True)])
def test_conv_lora_fused_bitwise(dev, monkeypatch, tile, N, H, W, Cin, Cout, stride, up):
    if Cout % BN[tile]:
        pytest.skip("output channels not a tile multiple: the launcher refuses (two-launch form)")
    torch.manual_seed(22)
    r = 32
    x = rnd(N, H, W, Cin, dev=dev)
    w, down = rnd(Cout, 3, 3, Cin, dev=dev, scale=0.05), rnd(r, 3, 3, Cin, dev=dev, scale=0.05)
    up2, b = rnd(Cout, r, dev=dev, scale=0.05), rnd(Cout, dev=dev)
    P, Q = K.conv_out_hw(H, W, 3, stride, 1, up)
    rowvec = rnd(N, Cout, dev=dev)
    t = torch.empty((N, P, Q, r), device=dev, dtype=BF)
    y = K.conv2d_lora(x, w, b, stride, 1, up, None, rowvec, down, up2, t, r, tile=tile)

    def ref():
        t_ref = K.conv2d(x, down, stride=stride, pad=1, upsample=up)
        return t_ref, K.conv2d(x, w, bias=b, stride=stride, pad=1, upsample=up, rowvec=rowvec, lora=(t_ref, up2))
    t_ref, y_ref = two_launch_split1(monkeypatch, ref)
    assert torch.equal(t, t_ref), (t.float() - t_ref.float()).abs().max().item()
    assert torch.equal(y, y_ref), (y.float() - y_ref.float()).abs().max().item()
    xin = F.interpolate(x.permute(0, 3, 1, 2).float(), scale_factor=2.0, mode="nearest") if up else \
        x.permute(0, 3, 1, 2).float()
    base = F.conv2d(xin, w.permute(0, 3, 1, 2).float(), b.float(), stride=stride, padding=1).permute(0, 2, 3, 1)
    want = base + rowvec.float()[:, None, None, :] + t_ref.float() @ up2.float().t()
    err = (y.float() - want).abs().max().item() / want.abs().max().item()
    assert err < 2e-2, err


def test_linear_lora_dispatch(dev):
    """the planned path (native host layer): the SDXL level-2 attention shape with a one-split table plan runs fused,
    and the two-launch fallback (set_lora_fuse(False)) gives the same product to bf16 rounding."""
    torch.manual_seed(23)
    M, Kd, r = 4096, 1280, 32
    x, w = rnd(M, Kd, dev=dev), rnd(Kd, Kd, dev=dev, scale=0.05)
    down, up2, b = rnd(r, Kd, dev=dev, scale=0.05), rnd(Kd, r, dev=dev, scale=0.05), rnd(Kd, dev=dev)
    t = torch.empty((M, r), device=dev, dtype=BF)
    f0 = K.lora_fused_counts()
    y = K.linear_lora(x, w, b, None, down, up2, t, r, Kd)
    f1 = K.lora_fused_counts()
    if K.host_layer() == "native":
        assert f1[0] == f0[0] + 1, (f0, f1)
    t2 = torch.empty_like(t)
    K.set_lora_fuse(False)
    try:
        y2 = K.linear_lora(x, w, b, None, down, up2, t2, r, Kd)
    finally:
        K.set_lora_fuse(True)
    assert (t.float() - t2.float()).abs().max().item() <= 2 ** -7 * t2.float().abs().max().item()
    err = (y.float() - y2.float()).abs().max().item() / y2.float().abs().max().item()
    assert err < 1e-2, err
    want = x.float() @ w.float().t() + b.float() + t.float() @ up2.float().t()
    assert (y.float() - want).abs().max().item() / want.abs().max().item() < 2e-2


# ---- backward input gradient with u = dy (sB) inside the dgrad GEMM (kernels.linear_dgrad_lora) ----
@pytest.mark.parametrize("tile", [1, 4, 7, 8])
@pytest.mark.parametrize("M,Nout,Kin", [(1000, 1280, 1280), (4096, 10240, 1280), (4096, 1280, 5120), (300, 640, 640)])
def test_linear_dgrad_lora_fused_bitwise(dev, monkeypatch, tile, M, Nout, Kin):
    """dx = dy W + u A and u = dy (sB), one launch, against the two-launch form at one split: bit-identical (u sums
    over the same 64-deep K steps and 16x16x32 MFMAs as the u GEMM; the second segment adds the same bf16 u)."""
    if Kin % BN[tile]:
        pytest.skip("input width not a tile multiple: the launcher refuses (two-launch form)")
    torch.manual_seed(24)
    r = 32
    dy, w = rnd(M, Nout, dev=dev), rnd(Nout, Kin, dev=dev, scale=0.05)
    up2, down = rnd(Nout, r, dev=dev, scale=0.05), rnd(r, Kin, dev=dev, scale=0.05)
    upT, downT = up2.t().contiguous(), down.t().contiguous()
    u = torch.full((M, r), float("nan"), device=dev, dtype=BF)
    dx = K.linear_dgrad_lora(dy, w, up2, down, upT, downT, u, tile=tile)

    def ref():
        u_ref = K.linear_dgrad(dy, up2)
        return u_ref, K.linear_dgrad(dy, w, lora=(u_ref, down))
    u_ref, dx_ref = two_launch_split1(monkeypatch, ref)
    assert torch.equal(u, u_ref), (u.float() - u_ref.float()).abs().max().item()
    assert torch.equal(dx, dx_ref), (dx.float() - dx_ref.float()).abs().max().item()
    want = dy.float() @ w.float() + u_ref.float() @ down.float()
    err = (dx.float() - want).abs().max().item() / want.abs().max().item()
    assert err < 2e-2, err


def test_linear_dgrad_lora_dispatch(dev):
    """the planned path (native host layer) at an SDXL level-2 shape runs fused when its plan is one split, and the
    two-launch fallback (set_lora_fuse(False)) gives the same u and dx bits at one split / the same product."""
    torch.manual_seed(25)
    M, Nout, Kin, r = 4096, 1280, 1280, 32
    dy, w = rnd(M, Nout, dev=dev), rnd(Nout, Kin, dev=dev, scale=0.05)
    up2, down = rnd(Nout, r, dev=dev, scale=0.05), rnd(r, Kin, dev=dev, scale=0.05)
    upT, downT = up2.t().contiguous(), down.t().contiguous()
    u = torch.empty((M, r), device=dev, dtype=BF)
    f0 = K.lora_dgrad_fused_counts()
    dx = K.linear_dgrad_lora(dy, w, up2, down, upT, downT, u)
    f1 = K.lora_dgrad_fused_counts()
    if K.host_layer() == "native":
        assert f1[0] + f1[1] == f0[0] + f0[1] + 1, (f0, f1)
    u2 = torch.empty_like(u)
    K.set_lora_fuse(False)
    try:
        dx2 = K.linear_dgrad_lora(dy, w, up2, down, upT, downT, u2)
    finally:
        K.set_lora_fuse(True)
    assert (u.float() - u2.float()).abs().max().item() <= 2 ** -7 * u2.float().abs().max().item()
    err = (dx.float() - dx2.float()).abs().max().item() / dx2.float().abs().max().item()
    assert err < 1e-2, err


def test_lora_shadow_transposes(dev):
    """the transposed shadows of single-module linear sites (r = 32) hold exactly up2^T and down^T"""
    from onetrainer_amd.module import unet as U
    from onetrainer_amd.module.lora import LoRAUNetWrapper
    m = U.UNet2DConditionModel(U.tiny_sdxl_config(), dev, seed=1, trainable=False)
    lw = LoRAUNetWrapper(m, rank=32, alpha=8.0, seed=0)
    g = torch.Generator(device=dev).manual_seed(5)
    lw.store.data.copy_(torch.randn(lw.store.data.shape, generator=g, device=dev) * 0.1)
    lw.refresh()
    n = 0
    nq = 0
    for s in lw.sites:
        if s.upT is None:
            assert s.kind != "linear" or len(s.group) not in (1, 3), s.key
            continue
        P, r = len(s.modules), 32
        n += 1
        nq += P == 3
        want = torch.cat([s.up2[p * s.part_width:(p + 1) * s.part_width, p * r:(p + 1) * r].t() for p in range(P)], 1)
        assert torch.equal(s.upT, want), s.key
        assert torch.equal(s.downT, s.down.t()), s.key
    assert n > 0 and nq > 0


@pytest.mark.parametrize("tile", [1, 4, 7, 8])
@pytest.mark.parametrize("M,pw,Kin", [(4096, 1280, 1280), (1000, 640, 640)])
def test_linear_dgrad_lora_fused_qkv_bitwise(dev, monkeypatch, tile, M, pw, Kin):
    """the fused q|k|v site's input gradient: three adapter parts along the dgrad's K (u_p sums over part p's rows,
    rotating accumulators), against the two-launch form with the block-diagonal up at one split: bit-identical."""
    if Kin % BN[tile]:
        pytest.skip("input width not a tile multiple: the launcher refuses (two-launch form)")
    torch.manual_seed(26)
    r, P = 32, 3
    dy, w = rnd(M, P * pw, dev=dev), rnd(P * pw, Kin, dev=dev, scale=0.05)
    up2, down = block_up(P, pw, r, dev), rnd(P * r, Kin, dev=dev, scale=0.05)
    upT = torch.cat([up2[p * pw:(p + 1) * pw, p * r:(p + 1) * r].t() for p in range(P)], dim=1).contiguous()
    downT = down.t().contiguous()
    u = torch.full((M, P * r), float("nan"), device=dev, dtype=BF)
    dx = K.linear_dgrad_lora(dy, w, up2, down, upT, downT, u, tile=tile)

    def ref():
        u_ref = K.linear_dgrad(dy, up2)
        return u_ref, K.linear_dgrad(dy, w, lora=(u_ref, down))
    u_ref, dx_ref = two_launch_split1(monkeypatch, ref)
    assert torch.equal(u, u_ref), (u.float() - u_ref.float()).abs().max().item()
    assert torch.equal(dx, dx_ref), (dx.float() - dx_ref.float()).abs().max().item()
