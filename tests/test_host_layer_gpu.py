"""The native host layer (csrc/host/ops_host.cpp) against the ctypes host path of kernels.py: the same launches
(same kernels, same plans, same split-K order), so every output must be bit-identical."""
import pytest
import torch

from onetrainer_amd import kernels as K

pytestmark = pytest.mark.gpu
BF = torch.bfloat16


def rnd(*s, dev, scale=1.0):
    return (torch.randn(*s, device=dev) * scale).to(BF)


def both(fn):
    """fn() through the native layer, then through the ctypes path (tensors out, cloned)."""
    assert K.host_layer() == "native"
    a = fn()
    torch.cuda.synchronize()
    with K.python_host():
        b = fn()
    torch.cuda.synchronize()
    return a, b


def same(a, b):
    if isinstance(a, (tuple, list)):
        assert len(a) == len(b)
        for x, y in zip(a, b):
            same(x, y)
        return
    if a is None:
        assert b is None
        return
    assert a.shape == b.shape and a.dtype == b.dtype
    assert torch.equal(a, b)


def test_linear_family(dev):
    torch.manual_seed(0)
    x, w, b = rnd(4096, 1280, dev=dev), rnd(3840, 1280, dev=dev, scale=0.05), rnd(3840, dev=dev)
    res = rnd(4096, 3840, dev=dev)
    same(*both(lambda: K.linear(x, w, bias=b, residual=res)))
    rv = rnd(4, 3840, dev=dev)
    same(*both(lambda: K.linear(x, w, rowvec=rv, rows_per_vec=1024)))
    t, b2 = rnd(4096, 32, dev=dev), rnd(3840, 32, dev=dev, scale=0.1)
    same(*both(lambda: K.linear(x, w, lora=(t, b2))))
    o1, o2 = torch.zeros(4096, 3840, device=dev), torch.zeros(4096, 3840, device=dev)
    K.linear(x, w, out=o1, accumulate=True, alpha=0.5)
    with K.python_host():
        K.linear(x, w, out=o2, accumulate=True, alpha=0.5)
    same(o1, o2)
    dy = rnd(4096, 3840, dev=dev)
    same(*both(lambda: K.linear_dgrad(dy, w)))
    u, a2 = rnd(4096, 32, dev=dev), rnd(32, 1280, dev=dev)
    same(*both(lambda: K.linear_dgrad(dy, w, residual=x, lora=(u, a2))))
    bg1, bg2 = torch.zeros(3840, device=dev), torch.zeros(3840, device=dev)
    g1 = K.linear_wgrad(dy, x, bias_grad=bg1)
    with K.python_host():
        g2 = K.linear_wgrad(dy, x, bias_grad=bg2)
    same(g1, g2)
    same(bg1, bg2)


def test_conv_family(dev):
    torch.manual_seed(1)
    x = rnd(2, 64, 64, 320, dev=dev)
    w, b = rnd(640, 3, 3, 320, dev=dev, scale=0.03), rnd(640, dev=dev)
    rv = rnd(2, 640, dev=dev)
    same(*both(lambda: K.conv2d(x, w, b, rowvec=rv)))
    same(*both(lambda: K.conv2d(x, w, b, stride=2)))
    same(*both(lambda: K.conv2d(x, w, b, upsample=True)))
    res = rnd(2, 64, 64, 640, dev=dev)
    same(*both(lambda: K.conv2d(x, w, b, residual=res)))
    dy = rnd(2, 64, 64, 640, dev=dev)
    same(*both(lambda: K.conv2d_dgrad(dy, w, (64, 64))))
    same(*both(lambda: K.conv2d_wgrad(dy, x)))
    bg1, bg2 = torch.zeros(640, dtype=BF, device=dev), torch.zeros(640, dtype=BF, device=dev)
    g1 = K.conv2d_wgrad(dy, x, bias_grad=bg1)
    with K.python_host():
        g2 = K.conv2d_wgrad(dy, x, bias_grad=bg2)
    same(g1, g2)
    same(bg1, bg2)


def test_norm_family(dev):
    torch.manual_seed(2)
    x = rnd(4096, 1280, dev=dev, scale=2.0)
    g, b = rnd(1280, dev=dev), rnd(1280, dev=dev)
    (y1, st1), (y2, st2) = both(lambda: K.layernorm_fwd(x, g, b, 1e-5))
    same(y1, y2)
    same(st1, st2)
    dy, dres = rnd(4096, 1280, dev=dev), rnd(4096, 1280, dev=dev)
    same(*both(lambda: K.layernorm_bwd_res(x, dy, dres, g, st1)))
    dg1, db1 = torch.zeros(1280, device=dev), torch.zeros(1280, device=dev)
    dg2, db2 = torch.zeros(1280, device=dev), torch.zeros(1280, device=dev)
    K.layernorm_param_grad(x, dy, st1, dg1, db1)
    with K.python_host():
        K.layernorm_param_grad(x, dy, st1, dg2, db2)
    same((dg1, db1), (dg2, db2))
    xg = rnd(2, 32, 32, 640, dev=dev, scale=2.0)
    gg, bb = rnd(640, dev=dev), rnd(640, dev=dev)
    for silu in (False, True):
        (yg1, sg1), (yg2, sg2) = both(lambda: K.groupnorm_fwd(xg, gg, bb, 32, 1e-5, silu))
        same(yg1, yg2)
        same(sg1, sg2)
        dyg, dr = rnd(2, 32, 32, 640, dev=dev), rnd(2, 32, 32, 640, dev=dev)
        same(*both(lambda: K.groupnorm_bwd(xg, dyg, gg, 32, silu, sg1)))
        same(*both(lambda: K.groupnorm_bwd(xg, dyg, gg, 32, silu, sg1, dres=dr)))


@pytest.mark.parametrize("Nq,Nk,heads,D", [(1024, 1024, 20, 64), (1024, 77, 20, 64), (2381, 2381, 4, 128)])
def test_attention_and_geglu(dev, Nq, Nk, heads, D):
    torch.manual_seed(3)
    q, k, v = rnd(2, Nq, heads * D, dev=dev), rnd(2, Nk, heads * D, dev=dev), rnd(2, Nk, heads * D, dev=dev)
    (o1, l1), (o2, l2) = both(lambda: K.attn_fwd(q, k, v, heads))
    same(o1, o2)
    same(l1, l2)
    do = rnd(2, Nq, heads * D, dev=dev)
    same(*both(lambda: K.attn_bwd(q, k, v, o1, l1, do, heads)))
    h = rnd(1024, 2 * 1280, dev=dev)
    same(*both(lambda: K.geglu_fwd(h)))
    dgo = rnd(1024, 1280, dev=dev)
    same(*both(lambda: K.geglu_bwd(h, dgo)))


def test_train_step_native_equals_ctypes(dev):
    """a whole tiny SDXL train step (forward, backward on both streams, clip, AdamW) gives bit-identical losses
    and parameters through either host path."""
    from onetrainer_amd.dataLoader.SyntheticDataLoader import synthetic_sdxl_batch
    from onetrainer_amd.module import unet as U
    from onetrainer_amd.trainer.GenericTrainer import GenericTrainer
    from onetrainer_amd.util import create
    from onetrainer_amd.util.config.TrainConfig import TrainConfig

    def run():
        cfg = TrainConfig.default_values()
        cfg.batch_size = 2
        cfg.learning_rate_warmup_steps = 0
        model = create.create_model(cfg, dev, seed=5, unet_config=U.tiny_sdxl_config())
        tr = GenericTrainer(cfg, model=model)
        tr.start()
        batch = synthetic_sdxl_batch(2, 128, 128, dev, seed=2, te1_dim=48, te2_dim=48, pooled_dim=64)
        losses = [tr.train_step(batch).float().item() for _ in range(2)]
        torch.cuda.synchronize()
        return losses, model.train_store.data.clone()

    l1, p1 = run()
    with K.python_host():
        l2, p2 = run()
    assert l1 == l2, (l1, l2)
    assert torch.equal(p1, p2)

