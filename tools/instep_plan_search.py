"""In-step GEMM plan search (not a test): the measured plan table was tuned with every candidate timed alone
on an idle chip; inside the train step the dgrad chain's GEMMs share the CUs with the weight-gradient stream,
so the fastest isolated plan need not give the fastest step.  This probe ranks the step's GEMM shapes by their
in-step time on each stream, then for the top shapes tries each candidate (tile, split-K) as an override of
that shape alone and keeps it when the median step time improves by more than --min-gain ms (greedy,
accumulating).  Prints the accepted overrides as plan-table rows (key fields as kernels._tune_key).

usage: python tools/instep_plan_search.py [--top 10] [--steps 9] [--model sdxl]
"""
import argparse
import collections
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from onetrainer_amd import kernels as K  # noqa: E402
from onetrainer_amd.dataLoader.SyntheticDataLoader import synthetic_sdxl_batch  # noqa: E402
from onetrainer_amd.module import streams  # noqa: E402
from onetrainer_amd.trainer.GenericTrainer import GenericTrainer  # noqa: E402
from onetrainer_amd.util import create  # noqa: E402
from onetrainer_amd.util.config.TrainConfig import TrainConfig  # noqa: E402

MODES = {0: "K", 1: "MN", 2: "CONVF", 3: "CONVD", 4: "CONVW", 5: "WT"}


def step_ms(tr, batch, n):
    tr.train_step(batch)   # warm-up: first launches of a new plan (LDS opt-in, workspace growth)
    ts = []
    for _ in range(n):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record()
        tr.train_step(batch)
        e1.record()
        e1.synchronize()
        ts.append(e0.elapsed_time(e1))
    ts.sort()
    return ts[len(ts) // 2]


def census(tr, batch):
    """in-step time per (amode, bmode, M, N, K) on each stream, with the plan each one runs."""
    K._HOST["off"] = True
    recs = []
    orig = K._gemm

    def timed(a, splits, device):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        orig(a, splits, device)
        e1.record()
        side = streams.side_stream()
        on_side = side is not None and torch.cuda.current_stream().cuda_stream == side.cuda_stream
        key = K._tune_key(a)
        recs.append(((a.amode, a.bmode, a.M, a.N, a.K), key, splits, on_side, e0, e1))

    K._gemm = timed
    try:
        tr.train_step(batch)
        torch.cuda.synchronize()
    finally:
        K._gemm = orig
    agg = collections.defaultdict(lambda: [0.0, 0, set(), None])
    for shape, key, splits, on_side, e0, e1 in recs:
        g = agg[(shape, on_side)]
        g[0] += e0.elapsed_time(e1)
        g[1] += 1
        g[2].add(key)
        g[3] = splits
    return agg


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--top", type=int, default=10)
    ap.add_argument("--steps", type=int, default=9)
    ap.add_argument("--min-gain", type=float, default=0.25)
    ap.add_argument("--tiles", default="0,1,2,4,7,8")
    ap.add_argument("--side", action="store_true", help="search the weight-gradient stream's shapes too")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    K._HOST["off"] = True   # overrides run through the ctypes path: baseline and candidates share it
    cfg = TrainConfig.default_values()
    cfg.batch_size = 4
    model = create.create_model(cfg, dev, seed=0)
    tr = GenericTrainer(cfg, model=model)
    tr.start()
    batch = synthetic_sdxl_batch(4, 1024, 1024, dev, seed=0)
    for _ in range(4):
        tr.train_step(batch)
    agg = census(tr, batch)
    ranked = sorted(((v[0], k) for k, v in agg.items() if args.side or not k[1]), reverse=True)[:args.top]
    table = K._plan_table()
    base = step_ms(tr, batch, args.steps)
    print(json.dumps({"baseline_ms": round(base, 3)}), flush=True)
    accepted = {}
    tiles = [int(t) for t in args.tiles.split(",")]
    for tot, (shape, on_side) in ranked:
        keys = agg[(shape, on_side)][2]
        cur = [table.get(k) for k in keys]
        cur_splits = {c[1] for c in cur if c} or {1}
        best = (base, None)
        tried = []
        for t in tiles:
            for sp in sorted(cur_splits | {1}):
                K._PLAN_OVERRIDES = dict(accepted)
                K._PLAN_OVERRIDES[shape] = (t, sp)
                try:
                    ms = step_ms(tr, batch, args.steps)
                except RuntimeError:
                    continue   # the candidate does not launch for this shape
                tried.append((t, sp, round(ms, 3)))
                if ms < best[0] - args.min_gain:
                    best = (ms, (t, sp))
        if best[1] is not None:
            accepted[shape] = best[1]
            base = best[0]
        print(json.dumps({"shape": [MODES[shape[0]], MODES[shape[1]], *shape[2:]], "side": on_side,
                          "instep_ms": round(tot, 3), "launches": agg[(shape, on_side)][1],
                          "table_plans": sorted({c for c in cur if c}), "tried": tried,
                          "accepted": best[1], "step_ms": round(base, 3)}), flush=True)
    K._PLAN_OVERRIDES = dict(accepted)
    final = step_ms(tr, batch, 2 * args.steps)
    K._PLAN_OVERRIDES = {}
    again = step_ms(tr, batch, 2 * args.steps)
    rows = []
    for shape, (t, sp) in accepted.items():
        for k in agg[(shape, False)][2] | agg[(shape, True)][2]:
            rows.append({"key": [int(x) for x in k], "tile": t, "splits": sp})
    print(json.dumps({"final_ms": round(final, 3), "table_ms": round(again, 3), "rows": rows}), flush=True)


if __name__ == "__main__":
    main()
