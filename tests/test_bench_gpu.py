"""bench.py's contract (the driver parses its one JSON line): a short run of the default workload at a small
resolution must print a well-formed line with the roofline and timing fields."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_json_line():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "2", "--warmup", "1", "--res", "256",
                        "--batch", "1", "--no-cpu-baseline", "--no-vae"], capture_output=True, text=True, timeout=280,
                       cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip().startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    d = json.loads(lines[0])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"):
        assert k in d, k
    assert d["value"] > 0 and d["ms_per_step"] > 0 and d["n_gpus"] == 1 and d["steps"] == 2
    rf = d["roofline"]
    assert rf["achieved"] > 0 and 0 < rf["frac"] < 1 and rf["peak"] > 0 and rf["isolated_frac"] > 0
    assert d["config"]["parallelism"] == "dp1"


def test_bench_two_ranks_json_line():
    """bench.py's multi-rank leg (launch_ranks + the world > 1 paths: barrier, max-over-ranks time, loss mean)
    run before the driver's multi-GPU node does: two child ranks on the test box's one GPU over gloo (RCCL
    cannot put two ranks on one device; the RCCL reducer itself is covered by test_rccl_reducer_world1).  The
    tiny SDXL-shaped UNet (--tiny): the leg under test is the bench's, not the network's, and the full SDXL
    pushes 5.1 GB of gradients per step through host memory over gloo."""
    env = dict(os.environ, OTAMD_DIST_BACKEND="gloo")
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "3", "--warmup", "1",
                        "--res", "128", "--batch", "2", "--tiny"], capture_output=True, text=True, timeout=170, cwd=ROOT,
                       env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip().startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]       # rank 0 only
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["config"]["global_batch"] == 4 and d["config"]["parallelism"] == "dp2"
    assert d["value"] > 0 and d["ms_per_step"] > 0 and d["steps"] == 3
    assert "tiny" in d["config"]["model"]
    import math
    assert math.isfinite(d["loss"]) and d["loss"] > 0
    assert d["cpu_baseline"] is None                 # N > 1: no CPU leg
