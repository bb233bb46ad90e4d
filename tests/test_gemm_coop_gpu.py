"""Cooperative split-K GEMM (plan tile 5, gemm2.hip gemm2_sk_kernel) vs a plain PyTorch fp32
reference of the same op, through otamd_gemm_explicit(tile=5, splits=P workgroups).

Covers every operand form the kernel is instantiated for (linear fwd + bias + residual, dgrad,
wgrad with fp32 accumulate, conv fwd / dgrad with the stored weight / wgrad, the LoRA second K
segment), 8- and 4-wide combines (N % 8 != 0), ragged tiles, 1..many workgroups per tile, bitwise
run-to-run determinism, concurrent launches on two streams, and that no launch's bounded peer wait
ever gave up (otamd_gemm_sk_errors)."""
import ctypes as C

import pytest
import torch
import torch.nn.functional as F

from onetrainer_amd import kernels as K

pytestmark = pytest.mark.gpu

BF = torch.bfloat16


def rnd(*s, dev, scale=1.0):
    return (torch.randn(*s, device=dev) * scale).to(BF)


def close(out, ref, tol=2e-2):
    out = out.float()
    err = (out - ref).abs().max().item()
    scale = ref.abs().max().item() + 1e-6
    assert err / scale < tol, f"max err {err} vs scale {scale}"


def nhwc(x):
    return x.permute(0, 3, 1, 2).float()


def to_nhwc(x):
    return x.permute(0, 2, 3, 1)


@pytest.fixture
def coop(monkeypatch):
    """route every engine GEMM through the coop kernel with P workgroups (P = 1: one per CU)."""
    P = {"v": 1}

    def explicit(a, s_, device):
        K.check(K.lib().otamd_gemm_explicit(C.byref(a), 5, P["v"], None, 0, K.stream_handle()), "coop gemm")

    monkeypatch.setattr(K, "_gemm", explicit)
    yield P
    assert K.lib().otamd_gemm_sk_errors() == 0, "a coop launch's peer wait timed out"


@pytest.mark.parametrize("P", [1, 8, 37, 100])
def test_coop_linear_forms(dev, coop, P):
    torch.manual_seed(3)
    coop["v"] = P
    x, w, b = rnd(1000, 2048, dev=dev), rnd(328, 2048, dev=dev, scale=0.05), rnd(328, dev=dev)
    r = rnd(1000, 328, dev=dev)
    close(K.linear(x, w, bias=b, residual=r), x.float() @ w.float().t() + b.float() + r.float())
    w4 = rnd(300, 2048, dev=dev, scale=0.05)          # N % 8 != 0: 4-wide combine
    close(K.linear(x, w4), x.float() @ w4.float().t())
    dy = rnd(1000, 328, dev=dev)
    close(K.linear_dgrad(dy, w), dy.float() @ w.float())
    dy2, xt = rnd(4096, 328, dev=dev), rnd(4096, 264, dev=dev)
    acc0 = torch.randn(328, 264, device=dev)
    out = acc0.clone()
    K.linear_wgrad(dy2, xt, out=out, accumulate=True)
    close(out, acc0 + dy2.float().t() @ xt.float(), tol=1e-2)


def test_coop_sdxl_shapes_and_determinism(dev, coop):
    """the SDXL level-2 shapes (coop candidates when opted in); two runs give the same bits."""
    torch.manual_seed(4)
    x, w = rnd(4096, 1280, dev=dev), rnd(1280, 1280, dev=dev, scale=0.03)
    b = rnd(1280, dev=dev)
    y1 = K.linear(x, w, bias=b)
    y2 = K.linear(x, w, bias=b)
    close(y1, x.float() @ w.float().t() + b.float())
    assert torch.equal(y1, y2)
    dy = rnd(4096, 1280, dev=dev)
    close(K.linear_dgrad(dy, w), dy.float() @ w.float())
    wq = rnd(3840, 1280, dev=dev, scale=0.03)
    dq = rnd(4096, 3840, dev=dev)
    close(K.linear_dgrad(dq, wq), dq.float() @ wq.float())
    dw = K.linear_wgrad(dy, x, out=torch.empty(1280, 1280, device=dev), accumulate=False)
    close(dw, dy.float().t() @ x.float(), tol=1e-2)


@pytest.mark.parametrize("P", [1, 19])
def test_coop_conv_forms(dev, coop, P):
    torch.manual_seed(5)
    coop["v"] = P
    xc = rnd(2, 24, 20, 64, dev=dev)
    wc = rnd(96, 3, 3, 64, dev=dev, scale=0.05)
    yc = K.conv2d(xc, wc, pad=1)
    close(yc, to_nhwc(F.conv2d(nhwc(xc), wc.permute(0, 3, 1, 2).float(), padding=1)))
    dxc = K.conv2d_dgrad(yc, wc, (24, 20), 1, 1)
    refd = torch.nn.grad.conv2d_input(nhwc(xc).shape, wc.permute(0, 3, 1, 2).float(), nhwc(yc), padding=1)
    close(dxc, to_nhwc(refd))
    dwc = K.conv2d_wgrad(yc, xc, 3, 1, 1, out=torch.empty(96, 3, 3, 64, device=dev))
    refw = torch.nn.grad.conv2d_weight(nhwc(xc), (96, 64, 3, 3), nhwc(yc), padding=1)
    close(dwc, refw.permute(0, 2, 3, 1), tol=1e-2)


def test_coop_lora_segment(dev, coop):
    torch.manual_seed(6)
    x, w = rnd(2048, 1280, dev=dev), rnd(640, 1280, dev=dev, scale=0.03)
    t, b2 = rnd(2048, 32, dev=dev), rnd(640, 32, dev=dev, scale=0.1)
    close(K.linear(x, w, lora=(t, b2)), x.float() @ w.float().t() + t.float() @ b2.float().t())
    dy, a2 = rnd(2048, 640, dev=dev), rnd(32, 1280, dev=dev, scale=0.1)
    close(K.linear_dgrad(dy, w, lora=(t, a2)), dy.float() @ w.float() + t.float() @ a2.float())


def test_coop_two_streams(dev, coop):
    """coop grids of two streams in flight together (per-stream slabs and barrier words)."""
    torch.manual_seed(7)
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    xs = [rnd(4096, 1280, dev=dev) for _ in range(2)]
    w = rnd(1280, 1280, dev=dev, scale=0.03)
    torch.cuda.synchronize()
    outs = [[], []]
    for it in range(8):
        for k, st in enumerate((s1, s2)):
            with torch.cuda.stream(st):
                outs[k].append(K.linear(xs[k], w))
    torch.cuda.synchronize()
    for k in range(2):
        ref = xs[k].float() @ w.float().t()
        for y in outs[k]:
            close(y, ref)
        assert all(torch.equal(outs[k][0], y) for y in outs[k][1:])


def test_plan_leaves_coop_opt_in(dev):
    """coop is opt-in (OTAMD_GEMM_SK=1): the automatic plan keeps the 128x128 tile for 4096x1280x1280."""
    import os
    if os.environ.get("OTAMD_GEMM_SK") == "1":
        pytest.skip("coop opted in")
    a = K._new_args()
    x, w = rnd(4096, 1280, dev=dev), rnd(1280, 1280, dev=dev)
    a.A, a.lda, a.amode = K._p(x), 1280, 0
    a.B, a.ldb, a.bmode = K._p(w), 1280, 0
    a.M, a.N, a.K = 4096, 1280, 1280
    assert K.lib().otamd_gemm_plan_tile(C.byref(a), 0) != 5
