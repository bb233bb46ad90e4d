"""Per-step timeline statistics from a rocprofv3 kernel-trace DB: for the last timed train step
(between fused-AdamW launches) the busy time of each stream, the union of busy time (GPU
occupied by >= 1 kernel), the idle gaps, and the per-stream top kernels.

usage: python tools/timeline.py gpurun_out/prof/run_results.db [--marker adamw_bf16_kernel]
"""
import argparse
import collections
import sqlite3


CATS = [("gemm2_kernel", "gemm"), ("gemm_kernel", "gemm"), ("splitk", "splitk"), ("attn_", "attention"),
        ("colsum", "colsum"), ("ln_", "layernorm"), ("gn_", "groupnorm"), ("geglu", "geglu"), ("adamw", "adamw"),
        ("sqnorm", "gradnorm"), ("at::native", "torch"), ("silu", "elementwise"), ("concat", "elementwise"),
        ("upsample", "elementwise"), ("ddpm", "diffusion"), ("mse", "diffusion"), ("noise", "diffusion")]


def category(name: str) -> str:
    for key, c in CATS:
        if key in name:
            return c
    return "other"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--marker", default="adamw_bf16")
    ap.add_argument("--top", type=int, default=12)
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    rows = c.execute("select name, stream_id, queue_id, start, end from kernels order by start").fetchall()
    marks = [r[3] for r in rows if a.marker in r[0]]
    t0, t1 = marks[-4], marks[-3]   # the last timed step (bench.py runs two roofline steps after it)
    step = [r for r in rows if t0 < r[3] <= t1]
    span = (t1 - t0) / 1e6
    print(f"step span {span:.2f} ms, {len(step)} kernels")
    by_stream = collections.defaultdict(list)
    for r in step:
        by_stream[(r[1], r[2])].append(r)
    for k, v in by_stream.items():
        busy = sum(r[4] - r[3] for r in v) / 1e6
        print(f"  stream {k}: {len(v)} kernels, busy {busy:.2f} ms")
    iv = sorted((r[3], r[4]) for r in step)
    union, cs, ce = 0, iv[0][0], iv[0][1]
    gaps = []
    for s, e in iv[1:]:
        if s > ce:
            union += ce - cs
            gaps.append(s - ce)
            cs, ce = s, e
        else:
            ce = max(ce, e)
    union += ce - cs
    print(f"  union busy {union / 1e6:.2f} ms; idle {span - union / 1e6:.2f} ms in {len(gaps)} gaps "
          f"(>10us: {sum(1 for g in gaps if g > 10000)}, total {sum(g for g in gaps if g > 10000) / 1e6:.2f} ms)")
    # the backward's tail: main-stream idle between its last kernel before the grad-norm (the join) and
    # the grad-norm launch, i.e. time the main stream waits for the weight-gradient side stream
    gn = [r for r in step if "grad_sqnorm" in r[0]]
    if gn:
        g0 = gn[0][3]
        main_key = max(by_stream, key=lambda k: len(by_stream[k]))
        before = [r for r in by_stream[main_key] if r[4] <= g0 and r is not gn[0]]
        side = [r for k, v in by_stream.items() if k != main_key for r in v if r[4] <= g0]
        if before and side:
            print(f"  join: main idle {(g0 - max(r[4] for r in before)) / 1e6:.2f} ms before the grad norm; "
                  f"side stream ends {(max(r[4] for r in side) - max(r[4] for r in before)) / 1e6:.2f} ms after main's last kernel")
    for k, v in by_stream.items():
        cat = collections.Counter()
        for r in v:
            cat[category(r[0])] += r[4] - r[3]
        print(f"  stream {k} by category: " + ", ".join(f"{n} {d / 1e6:.2f}" for n, d in cat.most_common()))
    for k, v in by_stream.items():
        agg = collections.Counter()
        for r in v:
            agg[r[0][:90]] += r[4] - r[3]
        print(f"  stream {k} top:")
        for n, d in agg.most_common(a.top):
            print(f"    {d / 1e6:7.3f} ms  {n}")


if __name__ == "__main__":
    main()
