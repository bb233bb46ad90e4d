"""Fused AdamW(+SR) and global clip on the GPU vs the oracle restatement (pinned to the reference)."""
import numpy as np
import pytest
import torch

from onetrainer_amd.module.param_store import FlatParamStore
from onetrainer_amd.util.optimizer.adamw_fused import FusedAdamW
from oracle import adamw as OA

pytestmark = pytest.mark.gpu

SHAPES = [("a", (1000,)), ("b", (37,)), ("c", (64, 70)), ("d", (5,))]


def bits(t):
    return t.detach().cpu().contiguous().view(torch.int16).numpy().astype(np.uint16)


@pytest.mark.parametrize("sr", [False, True])
@pytest.mark.parametrize("clip", [False, True])
def test_fused_adamw_bitexact(dev, sr, clip):
    torch.manual_seed(0)
    st = FlatParamStore([(n, s, "g") for n, s in SHAPES], torch.bfloat16, dev)
    for n, s in SHAPES:
        st.params[n].data.copy_(torch.randn(s) * 0.05)
    opt = FusedAdamW(st, [{"params": [st.params[n] for n, _ in SHAPES]}], lr=1e-3, weight_decay=1e-2,
                     stochastic_rounding=sr, seed=123)
    ref = {n: (bits(st.params[n]).reshape(-1), np.zeros(np.prod(s), np.uint16), np.zeros(np.prod(s), np.uint16))
           for n, s in SHAPES}
    for step in range(1, 4):
        for n, s in SHAPES:
            st.params[n].grad.copy_(torch.randn(s) * 10 ** (-2 + step) * (3 if clip else 1))
        coef = None
        if clip:
            total = opt.clip_grad_norm_(1.0)
            gl = [bits(st.params[n].grad).reshape(-1) for n, _ in SHAPES]
            _, tot_ref, coef = OA.clip_grad_norm_bf16(gl, 1.0)
            assert abs(total.item() - tot_ref) <= 1e-2 * tot_ref
            assert opt.clip_out[0].item() == coef
        seed_before = opt.seed
        opt.step()
        seed = (seed_before * 6364136223846793005 + 1442695040888963407) & 0xFFFFFFFFFFFFFFFF
        for n, s in SHAPES:
            p, m, v = ref[n]
            slot = st.slots[n]
            rand = OA.sr_bits(seed, np.arange(slot.offset, slot.offset + slot.numel)) if sr else None
            p, m, v = OA.adamw_step_bf16(p, bits(st.params[n].grad).reshape(-1), m, v, step, 1e-3, rand16=rand,
                                         clip_coef=coef)
            ref[n] = (p, m, v)
            assert np.array_equal(bits(opt.exp_avg[slot.offset:slot.offset + slot.numel]), m), (n, step, "m")
            assert np.array_equal(bits(opt.exp_avg_sq[slot.offset:slot.offset + slot.numel]), v), (n, step, "v")
            assert np.array_equal(bits(st.params[n]).reshape(-1), p), (n, step, "p")


def test_fused_adamw_f32(dev):
    torch.manual_seed(1)
    st = FlatParamStore([(n, s, "g") for n, s in SHAPES], torch.float32, dev)
    for n, s in SHAPES:
        st.params[n].data.copy_(torch.randn(s) * 0.05)
    opt = FusedAdamW(st, [{"params": [st.params[n] for n, _ in SHAPES]}], lr=3e-4)
    ref = {n: (st.params[n].detach().cpu().numpy().reshape(-1).copy(), np.zeros(np.prod(s), np.float32),
               np.zeros(np.prod(s), np.float32)) for n, s in SHAPES}
    for step in range(1, 4):
        for n, s in SHAPES:
            st.params[n].grad.copy_(torch.randn(s) * 10 ** (-2 + step))
        opt.step()
        for n, s in SHAPES:
            p, m, v = OA.adamw_step_f32(*ref[n][:1], st.params[n].grad.cpu().numpy().reshape(-1), *ref[n][1:], step,
                                        3e-4)
            ref[n] = (p, m, v)
            np.testing.assert_allclose(st.params[n].detach().cpu().numpy().reshape(-1), p, rtol=0, atol=1e-8)


@pytest.mark.parametrize("clip", [False, True])
def test_fused_adamw_master_bitexact(dev, clip):
    """fp32 master weights (weight_dtype FLOAT_32 full fine-tune): fp32 p / m / v and the bf16 working copy against
    oracle.adamw.adamw_step_master bit for bit over 3 steps, with the fp32 clip (norms and coefficient in fp32 from bf16
    gradients) against oracle.adamw.clip_grad_norm_f32"""
    torch.manual_seed(2)
    st = FlatParamStore([(n, s, "g") for n, s in SHAPES], torch.bfloat16, dev, master=True)
    for n, s in SHAPES:
        st.write(n, torch.randn(s) * 0.05)
    assert torch.equal(st.data, st.master.to(torch.bfloat16))
    opt = FusedAdamW(st, [{"params": [st.params[n] for n, _ in SHAPES]}], lr=3e-4, weight_decay=1e-2, seed=5)
    assert opt.exp_avg.dtype == torch.float32
    ref = {n: (st.value(n).cpu().numpy().reshape(-1).copy(), np.zeros(np.prod(s), np.float32),
               np.zeros(np.prod(s), np.float32)) for n, s in SHAPES}
    for step in range(1, 4):
        for n, s in SHAPES:
            st.params[n].grad.copy_(torch.randn(s) * 10 ** (-2 + step) * (3 if clip else 1))
        coef = None
        if clip:
            total = opt.clip_grad_norm_(1.0).item()
            gl = [OA.bf16_to_f32(bits(st.params[n].grad).reshape(-1)) for n, _ in SHAPES]
            tot_ref, coef_ref = OA.clip_grad_norm_f32(gl, 1.0)
            assert abs(total - tot_ref) <= 1e-6 * tot_ref
            coef = np.float32(opt.clip_out[0].item())   # the device coefficient (its fp32 sum order) drives both
            assert abs(coef - coef_ref) <= 1e-6 * coef_ref
        seed_before = opt.seed
        opt.step()
        assert opt.seed == seed_before   # no stochastic rounding on fp32 parameters (adamw_extensions.py:144)
        for n, s in SHAPES:
            p, m, v = ref[n]
            slot = st.slots[n]
            sl = slice(slot.offset, slot.offset + slot.numel)
            p, m, v, w = OA.adamw_step_master(p, bits(st.params[n].grad).reshape(-1), m, v, step, 3e-4, clip_coef=coef)
            ref[n] = (p, m, v)
            assert np.array_equal(opt.exp_avg[sl].cpu().numpy(), m), (n, step, "m")
            assert np.array_equal(opt.exp_avg_sq[sl].cpu().numpy(), v), (n, step, "v")
            assert np.array_equal(st.value(n).cpu().numpy().reshape(-1), p), (n, step, "p")
            assert np.array_equal(bits(st.params[n]).reshape(-1), w), (n, step, "working copy")
    sd = opt.state_dict()
    assert sd["state"][0]["exp_avg"].dtype == torch.float32


def test_state_dict_roundtrip(dev):
    st = FlatParamStore([(n, s, "g") for n, s in SHAPES], torch.bfloat16, dev)
    opt = FusedAdamW(st, [{"params": [st.params[n] for n, _ in SHAPES]}], lr=1e-3)
    for n, s in SHAPES:
        st.params[n].grad.copy_(torch.randn(s))
    opt.step()
    sd = opt.state_dict()
    assert sd["state"][0]["exp_avg"].shape == (1000,) and float(sd["state"][2]["step"]) == 1.0
    opt2 = FusedAdamW(st, [{"params": [st.params[n] for n, _ in SHAPES]}], lr=1e-3)
    opt2.load_state_dict(sd)
    assert torch.equal(opt2.exp_avg, opt.exp_avg) and opt2.steps == [1]
    sched = torch.optim.lr_scheduler.LambdaLR(opt, lambda s: min(1.0, (s + 1) / 10))
    opt.step()
    sched.step()
    assert abs(opt.param_groups[0]["lr"] - 2e-4) < 1e-12


@pytest.mark.parametrize("sr,clip", [(True, False), (False, True)])
def test_adamw_lut_matches_computed_path(dev, sr, clip, monkeypatch):
    """The LDS denominator-table kernel (stores >= 4M elements) is bit-identical to the computed
    path (oracle-pinned above) over every bf16 exp_avg_sq magnitude, -0.0 state and two groups."""
    from onetrainer_amd import _lib, kernels as K
    n = (1 << 22) + 4096
    g0 = torch.Generator().manual_seed(7)
    # grads over ~30 binades (incl. exact zeros), states spanning the bf16 range, -0.0 in v
    g = (torch.randn(n, generator=g0) * torch.exp2(torch.randint(-30, 4, (n,), generator=g0).float()))
    g[::97] = 0.0
    m = torch.randn(n, generator=g0) * 1e-3
    v = torch.exp2(torch.randint(-120, 10, (n,), generator=g0).float()) * torch.rand(n, generator=g0)
    v[::89] = -0.0
    v[::101] = 0.0
    p = torch.randn(n, generator=g0) * 0.05
    bufs = [t.to(torch.bfloat16).to(dev) for t in (p, g, m, v)]
    split = n // 2 + 8 * 37
    common = dict(one_minus_beta1=0.1, beta2=0.999, one_minus_beta2=1e-3, bc2_sqrt=0.0447, eps=1e-8, pad=0.0)
    groups = [_lib.AdamwGroup(begin=0, end=split, wd_factor=1 - 1e-5, neg_step_size=-1e-3, **common),
              _lib.AdamwGroup(begin=split, end=n, wd_factor=1.0, neg_step_size=-3e-4, **common)]
    coef = torch.tensor([0.37], device=dev) if clip else None
    outs = []
    for mode in ("0", "1", "2"):
        monkeypatch.setenv("OTAMD_ADAMW_LUT", mode)
        pp, gg, mm, vv = (t.clone() for t in bufs)
        K.adamw_bf16(pp, gg, mm, vv, groups, clip_coef=coef, stochastic_rounding=sr, seed=99)
        torch.cuda.synchronize()
        outs.append([t.view(torch.int16).cpu() for t in (pp, mm, vv)])
    for o in outs[1:]:
        for a, b, name in zip(outs[0], o, "pmv"):
            assert torch.equal(a, b), (name, int((a != b).sum()))


def test_overlapped_chunked_adamw_matches_single_launch(dev, monkeypatch):
    """util/optimizer/adamw_fused.py overlap: 16 range chunks on the optimizer stream (events per chunk,
    FlatParamStore.wait_params) give the bits of the one-launch update, SR on, clip on."""
    shapes = [(f"t{i}", (4_500_000 + 8 * i,)) for i in range(16)]       # 72 M elements >= the 64 M threshold
    runs = []
    for overlap in ("0", "1"):
        monkeypatch.setenv("OTAMD_OPT_OVERLAP", overlap)
        torch.manual_seed(0)
        st = FlatParamStore([(n, s, "g") for n, s in shapes], torch.bfloat16, dev)
        st.data.copy_((torch.randn(st.numel, device=dev) * 0.05).to(torch.bfloat16))
        opt = FusedAdamW(st, [{"params": [st.params[n] for n, _ in shapes]}], lr=1e-3, stochastic_rounding=True,
                         seed=7)
        assert opt.overlap == (overlap == "1")
        for step in range(2):
            st.wait_params()      # what store.begin_backward does before gradients are rewritten
            g = torch.Generator(device=dev).manual_seed(100 + step)
            st.grad.copy_((torch.randn(st.numel, device=dev, generator=g) * 0.5).to(torch.bfloat16))
            opt.clip_grad_norm_(1.0)
            opt.step()
            if overlap == "1":
                assert st.update_events is not None and len(st.update_events) == len(opt._opt_chunks) >= 8
        st.wait_params()
        torch.cuda.synchronize()
        runs.append((st.data.clone(), opt.exp_avg.clone(), opt.exp_avg_sq.clone()))
    for a, b in zip(*runs):
        assert torch.equal(a, b)


def test_grad_norm_during_backward_matches_end_of_step(dev):
    """clip_grad_norm_'s norm pass spread over the backward (OverlappedGradNorm, per-bucket sums on the
    weight-gradient stream) gives the same clip coefficient, total norm and updated parameters as the
    end-of-step pass over the whole gradient buffer."""
    from onetrainer_amd.dataLoader.SyntheticDataLoader import synthetic_sdxl_batch
    from onetrainer_amd.module import unet as U
    from onetrainer_amd.trainer.GenericTrainer import GenericTrainer
    from onetrainer_amd.util import create
    from onetrainer_amd.util.config.TrainConfig import TrainConfig

    def run(overlap):
        cfg = TrainConfig.default_values()
        cfg.batch_size = 2
        cfg.learning_rate_warmup_steps = 0
        cfg.clip_grad_norm = 0.05   # small enough that clipping is active
        model = create.create_model(cfg, dev, seed=7, unet_config=U.tiny_sdxl_config())
        tr = GenericTrainer(cfg, model=model)
        tr.start()
        opt = model.optimizer
        assert opt.norm_overlap is not None
        if not overlap:
            opt.norm_overlap = None
        batch = synthetic_sdxl_batch(2, 128, 128, dev, seed=3, te1_dim=48, te2_dim=48, pooled_dim=64)
        clips = []
        for _ in range(2):
            tr.train_step(batch)
            clips.append(opt.clip_out.clone())
        torch.cuda.synchronize()
        return clips, model.train_store.data.clone()

    c1, p1 = run(True)
    c2, p2 = run(False)
    for a, b in zip(c1, c2):
        assert a[0].item() < 1.0                      # clipping active
        assert a[0].item() == b[0].item()             # coefficient (bf16 value) identical
        assert a[1].item() == b[1].item()             # per-chunk slots summed in chunk order either way
    assert torch.equal(p1, p2)


def test_grad_norm_deterministic(dev):
    """The per-tensor squared norms come from one slot per chunk summed in chunk order (no atomics): repeated
    clip_grad_norm_ over tensors of many chunks gives the same float64 bits every time, and they match a float64
    sum of the bf16 gradients."""
    shapes = [("big", (3000, 2048)), ("mid", (700, 1000)), ("small", (33,))]
    st = FlatParamStore([(n, s, "g") for n, s in shapes], torch.bfloat16, dev)
    opt = FusedAdamW(st, [{"params": [st.params[n] for n, _ in shapes]}], lr=1e-3)
    g = torch.Generator(device="cpu").manual_seed(5)
    for n, s in shapes:
        st.params[n].grad.copy_(torch.randn(s, generator=g) * 0.01)
    assert opt._n_chunks > 50
    runs = []
    for _ in range(8):
        opt.clip_grad_norm_(1.0)
        runs.append((opt._tensor_sq.clone(), opt.clip_out.clone()))
    for t, c in runs[1:]:
        assert torch.equal(t, runs[0][0]) and torch.equal(c, runs[0][1])
    want = torch.stack([st.params[n].grad.double().square().sum() for n, _ in shapes])
    assert torch.allclose(runs[0][0], want, rtol=1e-6, atol=0)   # 8-element fp32 partials, fp64 beyond


def test_grad_norm_overlap_with_untouched_tensors(dev):
    """OverlappedGradNorm when a step's backward leaves some tensors without a gradient: their buckets are summed in
    finish() after finish_backward zeroed them, so the chunk slots of the previous step (poisoned here) never reach
    the clip coefficient, which equals the end-of-step pass over the same gradients."""
    from onetrainer_amd.util.optimizer.adamw_fused import OverlappedGradNorm
    shapes = [(f"t{i}", (300 + 37 * i, 500)) for i in range(12)]
    st = FlatParamStore([(n, s, "g") for n, s in shapes], torch.bfloat16, dev)
    opt = FusedAdamW(st, [{"params": [st.params[n] for n, _ in shapes]}], lr=1e-3)
    norm = OverlappedGradNorm(opt, bucket_bytes=1 << 20)
    assert len(norm.buckets) > 4
    g = torch.Generator(device="cpu").manual_seed(9)
    touched = [n for i, (n, _) in enumerate(shapes) if i % 3 != 1]
    opt._chunk_sq.fill_(1e9)                     # what a previous step left behind
    norm.arm(True)
    st.begin_backward()
    for n, s in shapes:
        if n in touched:
            st.params[n].grad.copy_(torch.randn(s, generator=g) * 0.02)
            st.mark_ready([n])
    st.finish_backward()                        # zeroes the untouched tensors' gradients
    norm.finish()
    opt.norm_overlap = norm
    total = opt.clip_grad_norm_(0.5).item()
    coef = opt.clip_out[0].item()
    opt.norm_overlap = None
    total_ref = opt.clip_grad_norm_(0.5).item()
    assert coef == opt.clip_out[0].item() and total == total_ref, (coef, total, total_ref)
    want = torch.stack([st.params[n].grad.double().square().sum() for n, _ in shapes]).sum().sqrt().item()
    assert abs(total - want) <= 1e-3 * want and total < 1e4
