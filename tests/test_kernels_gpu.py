"""HIP kernel parity vs plain PyTorch fp32 references of the same op (GPU)."""
import math

import pytest
import torch
import torch.nn.functional as F

from onetrainer_amd import kernels as K

pytestmark = pytest.mark.gpu
BF = torch.bfloat16


def rnd(*s, dev, scale=1.0, shift=0.0):
    return (torch.randn(*s, device=dev) * scale + shift).to(BF)


def rel_err(out, ref):
    return ((out.float() - ref.float()).abs().max() / (ref.float().abs().max() + 1e-6)).item()


@pytest.mark.parametrize("N,H,W,C,G,silu,eps", [(2, 16, 16, 320, 32, True, 1e-5), (2, 8, 8, 1280, 32, False, 1e-6),
                                                (1, 32, 32, 960, 32, True, 1e-5), (3, 4, 4, 2560, 32, True, 1e-5),
                                                (4, 64, 64, 640, 32, True, 1e-6)])
def test_groupnorm(dev, N, H, W, C, G, silu, eps):
    torch.manual_seed(0)
    x = rnd(N, H, W, C, dev=dev, scale=2.0, shift=0.5)
    gamma, beta = rnd(C, dev=dev, scale=0.5, shift=1.0), rnd(C, dev=dev, scale=0.5)
    y, stats = K.groupnorm_fwd(x, gamma, beta, G, eps, silu)
    xr = x.permute(0, 3, 1, 2).float().requires_grad_(True)
    gr, br = gamma.float().requires_grad_(True), beta.float().requires_grad_(True)
    ref = F.group_norm(xr, G, gr, br, eps)
    if silu:
        ref = F.silu(ref)
    assert rel_err(y, ref.permute(0, 2, 3, 1)) < 1e-2
    dy = rnd(N, H, W, C, dev=dev)
    ref.backward(dy.permute(0, 3, 1, 2).float())
    dx, dg, db = K.groupnorm_bwd(x, dy, gamma, G, silu, stats)
    assert rel_err(dx, xr.grad.permute(0, 2, 3, 1)) < 2e-2
    assert rel_err(dg, gr.grad) < 1e-2
    assert rel_err(db, br.grad) < 1e-2
    # the input's residual-use gradient added in the apply pass (ResnetBlock2D shortcut): the same dx + dres,
    # rounded once (vs the separate pass + bf16 add: within one bf16 rounding of each other)
    dres = rnd(N, H, W, C, dev=dev, scale=0.7)
    dx2, _, _ = K.groupnorm_bwd(x, dy, gamma, G, silu, stats, dres=dres)
    ref2 = xr.grad.permute(0, 2, 3, 1) + dres.float()
    assert rel_err(dx2, ref2) < 2e-2
    assert (dx2.float() - (dx.float() + dres.float())).abs().max().item() <= 2 ** -7 * ref2.abs().max().item()


@pytest.mark.parametrize("rows,C", [(4096, 640),(1000, 1280), (77, 320), (16384, 640), (4096, 1280), (31, 1280),
                                    (2381, 1536)])
def test_layernorm(dev, rows, C):
    torch.manual_seed(1)
    x = rnd(rows, C, dev=dev, scale=3.0, shift=1.0)
    g, b = rnd(C, dev=dev, shift=1.0), rnd(C, dev=dev)
    y, st = K.layernorm_fwd(x, g, b, 1e-5)
    xr, gr, br = x.float().requires_grad_(True), g.float().requires_grad_(True), b.float().requires_grad_(True)
    ref = F.layer_norm(xr, (C,), gr, br, 1e-5)
    assert rel_err(y, ref) < 1e-2
    dy = rnd(rows, C, dev=dev)
    ref.backward(dy.float())
    dx, dg, db = K.layernorm_bwd(x, dy, g, st)
    assert rel_err(dx, xr.grad) < 2e-2
    assert rel_err(dg, gr.grad) < 1e-2
    assert rel_err(db, br.grad) < 1e-2
    # the parameter-gradient half alone (side-stream form), bf16 destinations, then accumulated
    dx2, none_g, _ = K.layernorm_bwd(x, dy, g, st, need_param_grads=False)
    assert none_g is None and torch.equal(dx2, dx)
    pg, pb = torch.zeros(C, dtype=BF, device=dev), torch.zeros(C, dtype=BF, device=dev)
    K.layernorm_param_grad(x, dy, st, pg, pb)
    assert rel_err(pg, gr.grad) < 1e-2 and rel_err(pb, br.grad) < 1e-2
    K.layernorm_param_grad(x, dy, st, pg, pb, param_acc=True)
    assert rel_err(pg, 2 * gr.grad) < 1e-2 and rel_err(pb, 2 * br.grad) < 1e-2
    # input gradient + the residual branch's gradient in one pass
    dres = rnd(rows, C, dev=dev)
    dxr = K.layernorm_bwd_res(x, dy, dres, g, st)
    assert rel_err(dxr, xr.grad + dres.float()) < 2e-2


def sdpa_ref(q, k, v, heads):
    B, Nq, Cq = q.shape
    D = Cq // heads
    qh = q.float().view(B, Nq, heads, D).transpose(1, 2)
    kh = k.float().view(B, -1, heads, D).transpose(1, 2)
    vh = v.float().view(B, -1, heads, D).transpose(1, 2)
    return qh, kh, vh


@pytest.mark.parametrize("B,Nq,Nk,H,D", [(2, 256, 256, 2, 64), (1, 4096, 77, 10, 64), (2, 300, 300, 3, 64),
                                         (1, 1024, 1024, 4, 64), (1, 256, 256, 2, 128), (2, 200, 77, 4, 40),
                                         (2, 2048, 2048, 4, 64), (1, 333, 1000, 2, 128), (1, 128, 50, 2, 64),
                                         (1, 192, 64, 2, 64), (1, 256, 128, 2, 64), (1, 200, 190, 2, 128),
                                         (1, 160, 3, 2, 64), (2, 1024, 96, 20, 64), (1, 100, 77, 3, 64),
                                         (1, 1024, 97, 2, 64),
                                         # the step's own shapes: SDXL 1024^2 b=4 level-1 self (the hottest) and
                                         # cross, level-2 self and cross; FLUX.1 768^2 b=4 joint attention
                                         (4, 4096, 4096, 10, 64), (4, 4096, 77, 10, 64), (4, 1024, 1024, 20, 64),
                                         (4, 1024, 77, 20, 64), (4, 2381, 2381, 24, 128)])
def test_attention(dev, B, Nq, Nk, H, D):
    torch.manual_seed(2)
    q, k, v = rnd(B, Nq, H * D, dev=dev), rnd(B, Nk, H * D, dev=dev), rnd(B, Nk, H * D, dev=dev)
    o, lse = K.attn_fwd(q, k, v, H)
    qh, kh, vh = sdpa_ref(q, k, v, H)
    qh.requires_grad_(True); kh.requires_grad_(True); vh.requires_grad_(True)
    ref = F.scaled_dot_product_attention(qh, kh, vh)
    assert rel_err(o, ref.transpose(1, 2).reshape(B, Nq, H * D)) < 2e-2
    lse_ref = torch.logsumexp((qh @ kh.transpose(-1, -2)) * D ** -0.5, dim=-1) / math.log(2.0)
    assert (lse - lse_ref).abs().max().item() < 2e-2
    do = rnd(B, Nq, H * D, dev=dev)
    ref.backward(do.float().view(B, Nq, H, D).transpose(1, 2))
    dq, dk, dv = K.attn_bwd(q, k, v, o, lse, do, H)
    for got, want in ((dq, qh.grad), (dk, kh.grad), (dv, vh.grad)):
        assert rel_err(got, want.transpose(1, 2).reshape(got.shape)) < 3e-2


@pytest.mark.parametrize("B,Nq,Nk,H,D", [(4, 4096, 77, 10, 64), (4, 1024, 77, 20, 64), (2, 300, 77, 4, 40)])
def test_attention_cross_cast_stream(dev, B, Nq, Nk, H, D):
    """otamd_attn_bwd_ex: the cross-attention dK / dV chunk sum on another stream (after an event) gives the same
    bits as the one-stream call; dq is untouched by the move."""
    torch.manual_seed(6)
    q, kv = rnd(B, Nq, H * D, dev=dev), rnd(B, Nk, 2 * H * D, dev=dev)
    k, v = kv[..., :H * D], kv[..., H * D:]
    o, lse = K.attn_fwd(q, k, v, H)
    do = rnd(B, Nq, H * D, dev=dev)
    dq0, dk0, dv0 = K.attn_bwd(q, k, v, o, lse, do, H)
    side = torch.cuda.Stream(device=dev)
    for _ in range(3):
        dkv = torch.full_like(kv, float("nan"))
        dq, dk, dv = K.attn_bwd(q, k, v, o, lse, do, H, dk=dkv[..., :H * D], dv=dkv[..., H * D:], cast_stream=side)
        torch.cuda.current_stream().wait_stream(side)
        assert torch.equal(dq, dq0) and torch.equal(dk, dk0) and torch.equal(dv, dv0)


@pytest.mark.parametrize("B,Nq,Nk,H,D,fused", [(2, 256, 256, 8, 160, True), (2, 256, 77, 8, 160, False),
                                               (1, 1024, 1024, 1, 512, False), (3, 64, 64, 2, 160, True),
                                               (2, 300, 77, 8, 80, False)])
def test_attention_wide_heads(dev, B, Nq, Nk, H, D, fused):
    """heads > 128 (SD 1.5 level-2 160-wide heads, VAE 512-wide single head): materialized path
    (batched MFMA GEMMs + row softmax kernels); D = 80 stays on the flash kernels."""
    torch.manual_seed(4)
    C = H * D
    if fused:
        qkv = rnd(B, Nq, 3 * C, dev=dev)
        q, k, v = qkv[..., :C], qkv[..., C:2 * C], qkv[..., 2 * C:]
    else:
        q, k, v = rnd(B, Nq, C, dev=dev), rnd(B, Nk, C, dev=dev), rnd(B, Nk, C, dev=dev)
    o, aux = K.attn_fwd(q, k, v, H)
    qh, kh, vh = sdpa_ref(q, k, v, H)
    qh.requires_grad_(True); kh.requires_grad_(True); vh.requires_grad_(True)
    ref = F.scaled_dot_product_attention(qh, kh, vh)
    assert rel_err(o, ref.transpose(1, 2).reshape(B, Nq, C)) < 2e-2
    do = rnd(B, Nq, C, dev=dev)
    ref.backward(do.float().view(B, Nq, H, D).transpose(1, 2))
    dq, dk, dv = K.attn_bwd(q, k, v, o, aux, do, H)
    for got, want in ((dq, qh.grad), (dk, kh.grad), (dv, vh.grad)):
        assert rel_err(got, want.transpose(1, 2).reshape(got.shape)) < 3e-2


def test_gemm_batched_heads(dev):
    # C_z = A_z B_z^T over (image, head) pairs of [B, N, H*D] operands, fp32 out
    torch.manual_seed(5)
    B, H, M, N, D = 3, 4, 136, 96, 48
    a, b = rnd(B, M, H * D, dev=dev), rnd(B, N, H * D, dev=dev)
    c = torch.empty(B * H, M, N, device=dev)
    K.gemm_batched(a, H * D, K.OPM_K, b, H * D, K.OPM_K, c, N, M, N, D, B * H, H, (M * H * D, D), (N * H * D, D),
                   (H * M * N, M * N))
    ref = torch.einsum("bmhd,bnhd->bhmn", a.float().view(B, M, H, D), b.float().view(B, N, H, D)).reshape(B * H, M, N)
    assert rel_err(c, ref) < 1e-2
    with pytest.raises(ValueError, match="out of bounds"):
        K.gemm_batched(a, H * D, K.OPM_K, b, H * D, K.OPM_K, c, N, M, N, D, B * H + 1, H, (M * H * D, D),
                       (N * H * D, D), (H * M * N, M * N))


def test_attention_strided_qkv(dev):
    # q/k/v as column slices of one fused projection output (token stride 3*C)
    torch.manual_seed(3)
    B, N, H, D = 2, 512, 5, 64
    qkv = rnd(B, N, 3 * H * D, dev=dev)
    q, k, v = qkv[..., :H * D], qkv[..., H * D:2 * H * D], qkv[..., 2 * H * D:]
    o, lse = K.attn_fwd(q, k, v, H)
    qh, kh, vh = sdpa_ref(q, k, v, H)
    ref = F.scaled_dot_product_attention(qh, kh, vh).transpose(1, 2).reshape(B, N, H * D)
    assert rel_err(o, ref) < 2e-2


def test_geglu(dev):
    torch.manual_seed(4)
    h = rnd(300, 2 * 2560, dev=dev)
    y = K.geglu_fwd(h)
    hr = h.float().requires_grad_(True)
    a, g = hr.chunk(2, dim=-1)
    ref = a * F.gelu(g)
    assert rel_err(y, ref) < 1e-2
    do = rnd(300, 2560, dev=dev)
    ref.backward(do.float())
    assert rel_err(K.geglu_bwd(h, do), hr.grad) < 1e-2
    # GELU's erf is the Abramowitz-Stegun 7.1.26 form (common.h, |erf error| <= 1.5e-7): gates over the whole range,
    # both tails and 0, element-wise against fp64 erf within bf16 rounding of the outputs + 1e-6 absolute (the
    # negative tail, where torch's own fp32 0.5 (1 + erf) loses its relative accuracy too)
    g = torch.linspace(-12, 12, 2560 * 8, device=dev).view(8, 2560)
    h2 = torch.cat([torch.ones_like(g), g], dim=-1).to(BF)
    gq = h2[:, 2560:].double()
    gelu = 0.5 * gq * (1 + torch.erf(gq / math.sqrt(2)))
    dgelu = 0.5 * (1 + torch.erf(gq / math.sqrt(2))) + gq * torch.exp(-0.5 * gq * gq) / math.sqrt(2 * math.pi)
    y2 = K.geglu_fwd(h2).double()
    assert ((y2 - gelu).abs() <= 2 ** -8 * gelu.abs() + 1e-6).all()
    d2 = K.geglu_bwd(h2, torch.ones(8, 2560, device=dev, dtype=BF)).double()
    assert ((d2[:, :2560] - gelu).abs() <= 2 ** -8 * gelu.abs() + 1e-6).all()
    assert ((d2[:, 2560:] - dgelu).abs() <= 2 ** -8 * dgelu.abs() + 1e-6).all()


def test_silu_concat_pool_colsum(dev):
    torch.manual_seed(5)
    x = rnd(4, 1280, dev=dev)
    assert rel_err(K.silu_fwd(x), F.silu(x.float())) < 1e-2
    dy = rnd(4, 1280, dev=dev)
    xr = x.float().requires_grad_(True)
    F.silu(xr).backward(dy.float())
    assert rel_err(K.silu_bwd(x, dy), xr.grad) < 1e-2
    a, b = rnd(2, 8, 8, 320, dev=dev), rnd(2, 8, 8, 640, dev=dev)
    assert torch.equal(K.concat_channels(a, b), torch.cat([a, b], dim=-1))
    up = rnd(2, 16, 16, 64, dev=dev)
    ref = up.float().view(2, 8, 2, 8, 2, 64).sum(dim=(2, 4))
    assert rel_err(K.upsample2x_bwd(up), ref) < 1e-2
    m = rnd(2 * 4096, 320, dev=dev)
    cs = K.colsum(m, 4096)
    assert rel_err(cs, m.float().view(2, 4096, 320).sum(1)) < 1e-3
    m = rnd(4 * 16384, 320, dev=dev)   # SDXL level-1 per-image drow shape
    assert rel_err(K.colsum(m, 16384), m.float().view(4, 16384, 320).sum(1)) < 1e-3
    # ragged row counts (unroll tail), wide rows, a strided column slice, fp32 accumulate
    for rows, cols in ((1, 8), (9, 24), (77, 2048), (16384 + 40, 640), (3005, 1280), (4096 * 3 + 7, 10240)):
        m = rnd(rows, cols, dev=dev)
        assert rel_err(K.colsum(m), m.float().sum(0, keepdim=True)) < 1e-3, (rows, cols)
    big = rnd(5000, 1920, dev=dev)
    sl = big[:, 640:1280]
    out = torch.ones(1, 640, device=dev)
    K.colsum(sl, out=out, accumulate=True)
    assert rel_err(out, 1.0 + sl.float().sum(0, keepdim=True)) < 1e-3


def test_conv_weight_transpose_cast_embed(dev):
    w = rnd(64, 3, 3, 32, dev=dev)
    assert torch.equal(K.conv_weight_transpose(w), w.permute(3, 1, 2, 0).contiguous())
    x = torch.randn(1000, device=dev)
    assert torch.equal(K.cast_f32_bf16(x), x.to(BF))
    t = torch.tensor([0.0, 1.0, 999.0, 1024.0], device=dev)
    emb = K.timestep_embedding(t, 320)
    half = 160
    ex = torch.exp(-math.log(10000) * torch.arange(half, dtype=torch.float32, device=dev) / half)
    a = t[:, None] * ex[None]
    ref = torch.cat([torch.cos(a), torch.sin(a)], -1)
    assert (emb.float() - ref).abs().max().item() < 1e-2


def test_noise_and_timesteps(dev):
    n = K.noise((4, 64, 64, 4), seed=7, dtype=torch.float32, device=dev)
    assert abs(n.mean().item()) < 0.02 and abs(n.std().item() - 1) < 0.02
    # counter-based: the slice of a global draw equals the rank-local draw
    g = K.noise((8, 16, 16, 4), seed=3, dtype=torch.float32, device=dev)
    loc = K.noise((4, 16, 16, 4), seed=3, offset=4 * 16 * 16 * 4, dtype=torch.float32, device=dev)
    assert torch.equal(g[4:], loc)
    t = K.timesteps(4096, seed=11, device=dev)
    assert t.min().item() >= 0 and t.max().item() <= 999
    assert abs(t.float().mean().item() - 499.5) < 15
    tg = K.timesteps(8, seed=5, device=dev)
    assert torch.equal(tg[4:], K.timesteps(4, seed=5, sample0=4, device=dev))


@pytest.mark.parametrize("dtype", [torch.float32, BF])
@pytest.mark.parametrize("ow,pw", [(0.0, 0.0), (0.1, 0.0), (0.0, 0.2), (0.35, 0.05)])
def test_noise_offset_perturbation(dev, dtype, ow, pw):
    """offset / perturbation noise (ModelSetupNoiseMixin.py:31-46): the fused kernel equals the oracle's
    composition of the raw Philox streams (1 noise, 4 offset per sample and channel, 5 perturbation) in the
    reference's op order, bit for bit, for a rank-local slice of a global batch"""
    from oracle.diffusion import compose_noise
    B, H, W, C = 3, 8, 12, 4
    seed, s0 = 21, 2
    n, off = B * H * W * C, s0 * H * W * C
    got = K.noise_ex((B, H, W, C), seed=seed, offset=off, offset_weight=ow, perturbation_weight=pw, dtype=dtype,
                     device=dev)
    base = K.noise_stream(n, seed, 1, offset=off, dtype=dtype, device=dev).view(B, H, W, C)
    assert torch.equal(base, K.noise((B, H, W, C), seed=seed, offset=off, dtype=dtype, device=dev))
    o = K.noise_stream((s0 + B) * C, seed, 4, dtype=dtype, device=dev)[s0 * C:].view(B, 1, 1, C)
    p = K.noise_stream(n, seed, 5, offset=off, dtype=dtype, device=dev).view(B, H, W, C)
    ref = compose_noise(base.cpu(), o.cpu(), p.cpu(), ow, pw)
    assert torch.equal(got.cpu(), ref)


def _coeffs(dev):
    betas = torch.linspace(0.00085 ** 0.5, 0.012 ** 0.5, 1000, dtype=torch.float32) ** 2
    acp = torch.cumprod(1 - betas, 0)
    return acp.to(dev), acp.sqrt().to(dev), (1 - acp).sqrt().to(dev)


@pytest.mark.parametrize("lat_dtype", [torch.float32, BF])
@pytest.mark.parametrize("kind", [0, 1])
def test_ddpm_prologue_and_loss(dev, lat_dtype, kind):
    torch.manual_seed(6)
    B, H, W = 3, 32, 32
    lat = torch.randn(B, H, W, 4, device=dev).to(lat_dtype)
    eps = torch.randn(B, H, W, 4, device=dev).to(lat_dtype)
    t = torch.tensor([0, 500, 999], dtype=torch.int32, device=dev)
    co = _coeffs(dev)
    unet_in, target, scaled = K.ddpm_prologue(lat, eps, t, co, 0.13025, kind)
    x0 = lat * 0.13025
    a = co[1][t.long()].view(B, 1, 1, 1)
    s = co[2][t.long()].view(B, 1, 1, 1)
    xt = (x0.float() * a + eps.float() * s).to(lat_dtype)
    assert torch.equal(unet_in[..., :4], xt.to(BF))
    assert torch.count_nonzero(unet_in[..., 4:]) == 0
    if kind == 0:
        assert torch.equal(target, eps)
    else:
        acp = co[0].to(lat_dtype)[t.long()].view(B, 1, 1, 1)
        v = acp ** 0.5 * eps - (1 - acp) ** 0.5 * x0
        assert torch.equal(target, v)
    pred = rnd(B, H, W, 8, dev=dev)
    lw = torch.tensor([1.0, 0.5, 2.0], device=dev)
    loss, coef, losses = K.mse_loss(pred, target, lw)
    pr = pred[..., :4].float().requires_grad_(True)
    ref_l = (F.mse_loss(pr, target.float(), reduction="none").mean((1, 2, 3)) * lw).mean()
    assert abs(loss.item() - ref_l.item()) <= 1e-5 * abs(ref_l.item())
    ref_l.backward()
    g = K.mse_grad(pred, target, coef)
    assert rel_err(g[..., :4], pr.grad) < 1e-2
    assert torch.count_nonzero(g[..., 4:]) == 0


def test_flow_prologue(dev):
    torch.manual_seed(7)
    lat = torch.randn(2, 16, 16, 16, device=dev)
    eps = torch.randn(2, 16, 16, 16, device=dev)
    t = torch.tensor([10, 900], dtype=torch.int32, device=dev)
    mi, tgt = K.flow_prologue(lat, eps, t, 0.3611, 0.1159)
    x0 = (lat - 0.1159) * 0.3611
    sig = ((t + 1).float() / 1000).view(2, 1, 1, 1)
    assert torch.equal(mi, (eps * sig + x0 * (1 - sig)).to(BF))
    assert torch.equal(tgt, eps - x0)
