"""Data-parallel equivalence: two ranks at b=1 each == one rank at b=2, and four
ranks at b=1 with gradient accumulation 2 == one rank at b=4 with GA 2.

The ranks are fresh child processes on the one GPU of the test box (torch.distributed 'gloo'
with HIP tensors: RCCL cannot put two ranks on one device), each running
tests/workers/dp_step.py; the world-1 reference runs the whole global batch.  Compared after one
step (GenericTrainer.train_step: predict -> loss -> backward + bucketed all-reduce -> clip ->
AdamW, stochastic rounding off):
  * loss: mean over ranks vs the world-1 loss, rtol 1e-5 (fp32; summation order only);
  * clip total norm: rtol 2e-3;
  * reduced gradients: global cosine >= 0.9999 and relative L2 error <= 1e-2 -- the bf16 bucket
    reduction rounds each rank's partial and the sum (world-1 rounds the fp32 wgrad once); the fp32
    staging reduction (dp_reduce_fp32) is held to the same bound and reported next to it;
  * post-step bf16 parameters: <= 1e-2 of the elements differ, each by at most 2 lr (AdamW's first
    step moves every element by ~lr * g / (|g| + eps); the per-rank partial sums move a gradient by
    ~1 bf16 ulp, which flips the rounding of some updated parameters (<= 1 ulp of the parameter) or
    the sign of a near-zero g (<= 2 lr)).
"""
import os
import socket
import subprocess
import sys
from pathlib import Path

import pytest
import torch

pytestmark = pytest.mark.gpu
WORKER = Path(__file__).parent / "workers" / "dp_step.py"


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(tmp, world, fp32=False, global_batch=2, ga=1, norm_overlap=True):
    env = dict(os.environ)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    outs, procs = [], []
    port = _port()
    for r in range(world):
        e = dict(env)
        if world > 1:
            e.update(RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1",
                     MASTER_PORT=str(port), OTAMD_DIST_BACKEND="gloo")
        out = tmp / f"w{world}_{int(fp32)}_{global_batch}_{ga}_{int(norm_overlap)}_r{r}.pt"
        cmd = [sys.executable, str(WORKER), "--global-batch", str(global_batch), "--out", str(out), "--ga", str(ga),
               "--steps", str(ga)] + (["--fp32-reduce"] if fp32 else []) + ([] if norm_overlap else ["--no-norm-overlap"])
        procs.append(subprocess.Popen(cmd, env=e))
        outs.append(out)
    for p in procs:
        assert p.wait(timeout=240) == 0
    return [torch.load(o, weights_only=True) for o in outs]


def _compare(ranks, ref, fp32, label):
    r0 = ranks[0]
    loss_dp = sum(r["loss"] for r in ranks) / len(ranks)
    torch.testing.assert_close(loss_dp, ref["loss"], rtol=1e-5, atol=0)
    torch.testing.assert_close(r0["norm"][-1], ref["norm"][-1], rtol=2e-3, atol=0)
    for r in ranks[1:]:    # replicas identical
        assert torch.equal(r0["grad"], r["grad"]) and torch.equal(r0["param"], r["param"])
    g, gr = r0["grad"], ref["grad"]
    cos = torch.nn.functional.cosine_similarity(g, gr, dim=0).item()
    rel = ((g - gr).norm() / gr.norm()).item()
    diff = (r0["param"] != ref["param"]).float().mean().item()
    pa, pr = r0["param"].float(), ref["param"].float()
    ulp = torch.exp2(torch.floor(torch.log2(pr.abs().clamp_min(1e-30))) - 7)      # bf16 spacing at |p|
    excess = ((pa - pr).abs() - (2 * 1e-4 + ulp)).max().item()
    dmax = (pa - pr).abs().max().item()
    print(f"{label} ({'fp32' if fp32 else 'bf16'} reduce): grad cos {cos:.7f} rel-L2 {rel:.3e} "
          f"params differing {diff:.2e} (max {dmax:.2e}) loss {loss_dp.tolist()} vs {ref['loss'].tolist()}")
    assert cos >= 0.9999 and rel <= 1e-2
    assert diff <= 1e-2 and excess <= 0
    return rel


@pytest.mark.parametrize("fp32", [False, True])
def test_dp2_equals_single_rank_global_batch(tmp_path, fp32):
    ref = _run(tmp_path, 1)[0]
    _compare(_run(tmp_path, 2, fp32), ref, fp32, "dp2 vs dp1")


def test_dp4_ga2_bf16_vs_fp32_reduce(tmp_path):
    """four ranks (b=1 each, gradient accumulation 2: the reducer armed on the update micro-step only,
    over the accumulated sum) against one rank at global batch 4 with GA 2; the bf16 in-place bucket
    reduction and the fp32 staging (dp_reduce_fp32) side by side at 4 partials -- the data behind the
    dp_reduce_fp32 default."""
    ref = _run(tmp_path, 1, global_batch=4, ga=2)[0]
    rel_bf16 = _compare(_run(tmp_path, 4, False, global_batch=4, ga=2), ref, False, "dp4 ga2 vs dp1 ga2")
    rel_fp32 = _compare(_run(tmp_path, 4, True, global_batch=4, ga=2), ref, True, "dp4 ga2 vs dp1 ga2")
    print(f"dp4 reduction error vs world 1: bf16 {rel_bf16:.3e}, fp32 staging {rel_fp32:.3e}")


def test_dp8_bf16_vs_fp32_reduce(tmp_path):
    """eight ranks at b=1 (the node's rank count; gloo on the one GPU) against one rank at global batch 8: at world 8 the
    bf16 in-place ring sum rounds up to 7 times per element, the fp32 staging (dp_reduce_fp32) once -- both held to
    the same bounds as world 2 / 4, the two errors printed side by side"""
    ref = _run(tmp_path, 1, global_batch=8)[0]
    rel_bf16 = _compare(_run(tmp_path, 8, False, global_batch=8), ref, False, "dp8 vs dp1")
    rel_fp32 = _compare(_run(tmp_path, 8, True, global_batch=8), ref, True, "dp8 vs dp1")
    print(f"dp8 reduction error vs world 1: bf16 {rel_bf16:.3e}, fp32 staging {rel_fp32:.3e}")


@pytest.mark.parametrize("fp32", [False, True])
def test_dp2_overlapped_norm_equals_end_of_step(tmp_path, fp32):
    """under data parallel the clip norm's squared sums run per bucket on the reducer's post stream as each all-reduce
    completes (trainer/ddp.py reduced_hooks, OverlappedGradNorm(reducer=...)); the coefficient and the step must be
    the end-of-step pass's bit for bit (same chunks, same fixed summation order), GA 2 included"""
    for ga in (1, 2):
        on = _run(tmp_path, 2, fp32, global_batch=2 * ga, ga=ga)
        off = _run(tmp_path, 2, fp32, global_batch=2 * ga, ga=ga, norm_overlap=False)
        for a, b in zip(on, off):
            assert torch.equal(a["norm"], b["norm"]), (a["norm"], b["norm"])
            assert torch.equal(a["grad"], b["grad"]) and torch.equal(a["param"], b["param"])


def test_rccl_reducer_world1(tmp_path):
    """RCCL itself (torch.distributed 'nccl') under the bucketed reducer: a one-rank group on the box's GPU, the
    all-reduces issued from inside backward on the issue stream; a one-rank sum is the identity, so the step must
    be bit-identical to the plain step, in bf16 in place and through the fp32 staging copy
    (tests/workers/rccl_world1.py)."""
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_port()))
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "OTAMD_DIST_BACKEND"):
        env.pop(k, None)
    out = tmp_path / "rccl.pt"
    p = subprocess.run([sys.executable, str(Path(__file__).parent / "workers" / "rccl_world1.py"), "--out", str(out)],
                       env=env, timeout=240)
    assert p.returncode == 0
    r = torch.load(out, weights_only=True)
    assert r["buckets"] > 3 and r["nonzero"]
    assert r["grad_equal"] and r["param_equal"], r
    assert r["grad_equal_fp32"] and r["param_equal_fp32"], r
    assert r["norm_overlap_equal"], r
