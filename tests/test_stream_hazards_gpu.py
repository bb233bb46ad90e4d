"""Stream ordering of the two-stream step (module/streams.py) and of its captured HIP graph (trainer/step_graph.py).

* module/stream_hazards.StreamHazardCheck finds no access of the main stream that races with the weight-gradient
  stream in the SDXL (full UNet) and tiny-LoRA steps: no main-stream write into memory the side stream may still
  read or write, no main-stream read of memory it may still write, and every tensor the side stream uses is
  record_stream()ed -- checked at the aten layer and at every kernels.py entry point;
* the checker is sensitive: races planted on purpose are reported;
* the step graph captured from the same code has one root and one sink, so a replay completes only when the
  weight-gradient branch has (the join into store.finish_backward is an edge), and every fork of the side
  branch hangs off the main chain.
"""
import re

import pytest
import torch

from onetrainer_amd import kernels as K
from onetrainer_amd.dataLoader.SyntheticDataLoader import synthetic_sdxl_batch
from onetrainer_amd.module import streams as S
from onetrainer_amd.module import unet as U
from onetrainer_amd.module.stream_hazards import StreamHazardCheck
from onetrainer_amd.trainer.GenericTrainer import GenericTrainer
from onetrainer_amd.util import create
from onetrainer_amd.util.config.TrainConfig import TrainConfig

pytestmark = pytest.mark.gpu


def _trainer(dev, ucfg=None, lora=False):
    cfg = TrainConfig.default_values()
    cfg.batch_size = 1
    cfg.learning_rate_warmup_steps = 0
    if lora:
        cfg.training_method, cfg.lora_rank = "LORA", 8
    model = create.create_model(cfg, dev, seed=3, unet_config=ucfg)
    tr = GenericTrainer(cfg, model=model)
    tr.start()
    return tr


@pytest.mark.parametrize("which", ["sdxl_512", "tiny_lora"])
def test_step_has_no_stream_races(dev, which):
    if which == "sdxl_512":
        tr, batch = _trainer(dev), None
        batch = synthetic_sdxl_batch(1, 512, 512, dev, seed=0)
    else:
        tr = _trainer(dev, U.tiny_sdxl_config(), lora=True)
        batch = synthetic_sdxl_batch(1, 128, 128, dev, seed=0, te1_dim=48, te2_dim=48, pooled_dim=64)
    tr.train_step(batch)
    torch.cuda.synchronize()
    with StreamHazardCheck() as chk:
        tr.train_step(batch)
    torch.cuda.synchronize()
    assert chk.regions > 10 and chk.kernel_calls > 100 and chk.checked > 100, chk.report()
    assert not chk.hazards, chk.report()


def test_hazard_checker_reports_planted_races(dev):
    assert S.side_stream() is not None
    x = torch.randn(256, 128, device=dev).bfloat16()
    dy = torch.randn(256, 64, device=dev).bfloat16()
    gw = torch.empty(64, 128, device=dev, dtype=torch.bfloat16)
    with StreamHazardCheck() as chk:
        with S.wgrad_region((dy, x)):
            K.linear_wgrad(dy, x, out=gw)
        dy.add_(1.0)                          # aten in-place write on the main stream: WAR on dy
        K.linear(x, gw)                       # main-stream read of the side stream's output: RAW on gw
        K.cast_f32_bf16(torch.ones(256, 128, device=dev), out=x)   # kernel write into x: WAR
        u = torch.randn(256, 64, device=dev).bfloat16()
        with S.wgrad_region(()):              # u not handed over: the allocator may recycle it early
            K.linear_wgrad(u, x, out=gw)
        S.join()
    kinds = {(h[0], h[1], h[3]) for h in chk.hazards}
    assert any(k[0].startswith("aten.add_") and k[1:] == ("writes", "read") for k in kinds), chk.report()
    assert any(k[0] == "K.linear" and k[1] == "reads" and k[2] == "write" for k in kinds), chk.report()
    assert any(k[0] == "K.cast_f32_bf16" and k[1] == "writes" for k in kinds), chk.report()
    assert any(k[1] == "uses on the side stream" for k in kinds), chk.report()
    torch.cuda.synchronize()


def test_step_graph_single_sink(dev, tmp_path, monkeypatch):
    """the captured forward + backward (tiny SDXL) as hipGraphDebugDotPrint writes it: one root, one leaf, every node
    on a path between them, and one fork per weight-gradient region"""
    import sys
    from pathlib import Path
    sys.path.insert(0, str(Path(__file__).parents[1] / "tools"))
    from graph_dump import structure
    from onetrainer_amd.trainer.step_graph import StepGraphs
    monkeypatch.setenv("OTAMD_STEP_GRAPH", "1")
    tr = _trainer(dev, U.tiny_sdxl_config())
    assert tr.graphs is not None
    dot = tmp_path / "step.dot"
    monkeypatch.setattr(StepGraphs, "debug_dot", str(dot))
    batch = synthetic_sdxl_batch(1, 128, 128, dev, seed=1, te1_dim=48, te2_dim=48, pooled_dim=64)
    tr.train_step(batch)
    with StreamHazardCheck(kernels=False) as chk:   # counts the side regions of one capture (aten layer only)
        tr.train_step(batch)                        # the capture
    torch.cuda.synchronize()
    s = structure(str(dot))
    raw = dot.read_text(errors="replace")

    def kernel_of(n):   # the node's kernel symbol from its DOT record (for the failure message)
        i = raw.find(f'"{n}"[')
        m = re.search(r"ID \| \d+ \| (\S+)", raw[i:i + 600]) if i >= 0 else None
        return m.group(1)[:80] if m else "?"
    assert s["nodes"] > 100 and len(s["roots"]) == 1 and len(s["leaves"]) == 1, \
        (s["nodes"], [(n, kernel_of(n)) for n in s["roots"]], [(n, kernel_of(n)) for n in s["leaves"]])
    # every side region forks the side chain off the main chain (a node with two successors); a region whose
    # fork was missing would start a second root instead
    assert s["forks"] >= 0.5 * chk.regions, (s["forks"], chk.regions)
    # and the replay of the captured step still trains
    losses = [tr.train_step(batch).item() for _ in range(2)]
    assert all(l == l for l in losses)
