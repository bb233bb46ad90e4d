"""Which kernels make one C4 aspect bucket's step slower than another's (not a test): run the SDXL LoRA (C4) step on
bucket A three times, then bucket B three times, under `rocprofv3 --kernel-trace`, and compare the third step of each
by kernel name (total microseconds per step, both streams).

usage: rocprofv3 --kernel-trace -d DIR -o run -- python tools/bucket_kernel_diff.py run --a 896x1152 --b 832x1280
       python tools/bucket_kernel_diff.py report DIR
"""
import argparse
import collections
import glob
import os
import sqlite3
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def run(a, b):
    import torch
    from onetrainer_amd.dataLoader.SyntheticDataLoader import synthetic_sdxl_batch
    from onetrainer_amd.trainer.GenericTrainer import GenericTrainer
    from onetrainer_amd.util.config.TrainConfig import TrainConfig
    cfg = TrainConfig.default_values()
    cfg.training_method, cfg.lora_rank, cfg.batch_size = "LORA", 32, 4
    tr = GenericTrainer(cfg, seed=0)
    tr.start()
    dev = tr.device
    for res in (a, b):
        h, w = (int(v) for v in res.split("x"))
        batch = synthetic_sdxl_batch(4, h, w, dev, seed=0)
        for _ in range(3):
            tr.train_step(batch)
        torch.cuda.synchronize()


def report(d):
    db = sorted(glob.glob(os.path.join(d, "**", "*.db"), recursive=True))[-1]
    c = sqlite3.connect(db)
    rows = c.execute("select name, start, end from kernels order by start").fetchall()
    marks = [r[1] for r in rows if "adamw_f32" in r[0]]
    # six steps: marks[k] is step k's optimizer; step 2 = (marks[1], marks[2]], step 5 = (marks[4], marks[5]]
    def step(i):
        t0, t1 = marks[i - 1], marks[i]
        agg = collections.Counter()
        for n, s, e in rows:
            if t0 < s <= t1:
                agg[n.split("(")[0]] += (e - s) / 1e3
        return agg, (t1 - t0) / 1e6
    A, ta = step(2)
    B, tb = step(5)
    print(f"step A {ta:.2f} ms, step B {tb:.2f} ms (optimizer to optimizer)")
    keys = sorted(set(A) | set(B), key=lambda k: -(B.get(k, 0) - A.get(k, 0)))
    for k in keys[:25] + ["..."] + keys[-12:]:
        if k == "...":
            print("   ...")
            continue
        print(f"{B.get(k, 0) - A.get(k, 0):9.1f} us   A {A.get(k, 0):9.1f}   B {B.get(k, 0):9.1f}   {k[:110]}")


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("cmd")
    ap.add_argument("dir", nargs="?")
    ap.add_argument("--a", default="896x1152")
    ap.add_argument("--b", default="832x1280")
    args = ap.parse_args()
    run(args.a, args.b) if args.cmd == "run" else report(args.dir)
