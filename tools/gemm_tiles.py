"""Tile / split-K probe over the real GEMM launches of one SDXL step (not a test).

Captures every GEMM's arguments from one eager train step, keeps the signatures with the largest
planned time, and times each (tile, splits) candidate with otamd_gemm_explicit into scratch
outputs (median of reps), next to the analytic plan.  Also checks that every candidate's output
equals the planned output to bf16 rounding (split-K changes only the fp32 summation order).

usage: python tools/gemm_tiles.py [--top 14] [--lora 0]
"""
import argparse
import collections
import ctypes as C
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from onetrainer_amd import _lib, kernels as K  # noqa: E402
from onetrainer_amd.dataLoader.SyntheticDataLoader import synthetic_sdxl_batch  # noqa: E402
from onetrainer_amd.trainer.GenericTrainer import GenericTrainer  # noqa: E402
from onetrainer_amd.util import create  # noqa: E402
from onetrainer_amd.util.config.TrainConfig import TrainConfig  # noqa: E402

MODES = {0: "K", 1: "MN", 2: "CONVF", 3: "CONVD", 4: "CONVW", 5: "WT"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--top", type=int, default=14)
    ap.add_argument("--lora", type=int, default=0)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--tiles", default="0,1,2,4,7,8", help="candidate tile codes (otamd_gemm_explicit)")
    ap.add_argument("--skip", type=int, default=0, help="skip the first N signatures (by step time)")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    cfg = TrainConfig.default_values()
    cfg.batch_size = 4
    if args.lora:
        cfg.training_method, cfg.lora_rank = "LORA", args.lora
    model = create.create_model(cfg, dev, seed=0)
    tr = GenericTrainer(cfg, model=model)
    tr.start()
    batch = synthetic_sdxl_batch(4, 1024, 1024, dev, seed=0)
    tr.train_step(batch)
    torch.cuda.synchronize()
    caps = collections.OrderedDict()
    K._HOST["off"] = True   # launch through the ctypes path, whose _gemm is wrapped below
    orig = K._gemm

    def grab(a, splits, device):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        orig(a, splits, device)
        e1.record()
        key = K._tune_key(a)
        if key not in caps:
            caps[key] = [K.GemmArgs.from_buffer_copy(a), 0, []]
        caps[key][1] += 1
        caps[key][2].append((e0, e1))

    from onetrainer_amd.module import streams
    streams.set_enabled(False)
    K._gemm = grab
    tr.train_step(batch)
    torch.cuda.synchronize()
    K._gemm = orig
    rows = []
    for key, (a, n, evs) in caps.items():
        rows.append((sum(e0.elapsed_time(e1) for e0, e1 in evs), key, a, n))
    rows.sort(key=lambda r: -r[0])
    lib = _lib.lib()
    tiles = tuple(int(t) for t in args.tiles.split(","))
    for tot, key, a0, n in rows[args.skip:args.skip + args.top]:
        a = K.GemmArgs.from_buffer_copy(a0)
        a.accumulate = 0
        esz = 4 if a.c_f32 else 2
        scratch = torch.zeros(((a.M - 1) * max(a.ldc, a.N) + a.N) * esz + 256, dtype=torch.uint8, device=dev)
        a.C = scratch.data_ptr()
        s_out = C.c_int(0)
        lib.otamd_gemm_plan(C.byref(a), 0, C.byref(s_out))
        plan = (lib.otamd_gemm_plan_tile(C.byref(a), 0), s_out.value)
        res = {}
        ref = None
        for s in (1, 2, 3, 4, 5, 6, 8, 12, 16):
            kps = ((a.K + s - 1) // s + 63) // 64 * 64
            se = (a.K + kps - 1) // kps
            if (s > 1 and kps < 256) or (se, 0) in [(x[1], 0) for x in res]:
                continue
            ws_bytes = se * a.M * a.N * 4 if se > 1 else 0
            ws = torch.empty(max(ws_bytes, 16), dtype=torch.uint8, device=dev)
            for t in tiles:
                rc = lib.otamd_gemm_explicit(C.byref(a), t, se, ws.data_ptr(), ws_bytes, K.stream_handle())
                if rc != 0:
                    continue
                torch.cuda.synchronize()
                out = scratch.clone()
                if ref is None:
                    ref = out
                ok = True
                if not a.c_f32:
                    x = out[:((a.M - 1) * max(a.ldc, a.N) + a.N) * 2].view(torch.bfloat16).float()
                    y = ref[:((a.M - 1) * max(a.ldc, a.N) + a.N) * 2].view(torch.bfloat16).float()
                    ok = bool(((x - y).abs().max() <= 0.02 * y.abs().max() + 1e-3).item())
                ev = [torch.cuda.Event(enable_timing=True) for _ in range(args.reps + 1)]
                ev[0].record()
                for i in range(args.reps):
                    lib.otamd_gemm_explicit(C.byref(a), t, se, ws.data_ptr(), ws_bytes, K.stream_handle())
                    ev[i + 1].record()
                torch.cuda.synchronize()
                ts = sorted(ev[i].elapsed_time(ev[i + 1]) for i in range(args.reps))
                res[(t, se)] = (ts[len(ts) // 2] * 1e3, ok)
                if not ok:
                    print(f"  mismatch {MODES[a.amode]},{MODES[a.bmode]} {a.M}x{a.N}x{a.K} tile {t} splits {se}: "
                          f"max err {(x - y).abs().max().item():.4g} ref max {y.abs().max().item():.4g}", file=sys.stderr)
        best = min(res.items(), key=lambda kv: kv[1][0])
        print(json.dumps({"a": MODES[a.amode], "b": MODES[a.bmode], "M": a.M, "N": a.N, "K": a.K, "calls": n,
                          "step_ms": round(tot, 3), "plan": plan,
                          "plan_us": round(res.get(plan, (float("nan"),))[0], 1),
                          "best": best[0], "best_us": round(best[1][0], 1),
                          "t4_us": {str(k[1]): round(v[0], 1) for k, v in res.items() if k[0] == 4},
                          "all_ok": all(v[1] for v in res.values()),
                          "cands": {f"{k[0]}/{k[1]}": round(v[0], 1) for k, v in sorted(res.items())}}), flush=True)


if __name__ == "__main__":
    main()
