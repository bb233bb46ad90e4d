"""Main-stream idle gaps of one timed train step, classified by cause (not a test).

Input: a rocprofv3 rocpd database with kernel dispatches and the HIP runtime API (`rocprofv3 --kernel-trace
--hip-runtime-trace`).  For every gap on the main (busiest) stream between two of its kernels, the launch call of
the kernel after the gap is found through the correlation id:
  * host:  the launch call returned after the previous kernel had ended -- the host had not issued it yet;
  * wait:  the kernel was issued before the previous one ended but started late -- a cross-stream event wait
           (the weight-gradient stream, the optimizer's update stream), a barrier packet or the dispatcher;
  * alloc: a hipMalloc / hipFree call overlaps the gap (the caching allocator growing or releasing).
Prints the totals per cause and the largest gaps with the kernels around them.

usage: python tools/gap_causes.py <results.db> [--marker adamw_bf16] [--min-us 5] [--top 25]
"""
import argparse
import collections
import sqlite3


def cols(c, view):
    return [r[1] for r in c.execute(f"pragma table_info({view})").fetchall()]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--marker", default="adamw_bf16")
    ap.add_argument("--min-us", type=float, default=5.0)
    ap.add_argument("--top", type=int, default=25)
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    kc, rc = cols(c, "kernels"), cols(c, "regions")
    # the column linking a dispatch to its launch call differs between rocpd versions: take the candidate whose
    # kernels start shortly after their launch call (median lag between 0 and 100 ms)
    key, best = None, None
    for k in ("corr_id", "stack_id", "event_id", "correlation_id"):
        if k not in kc or k not in rc:
            continue
        ls = dict(c.execute(f"select {k}, start from regions where name like '%aunch%'").fetchall())
        lag = sorted(ks - ls[i] for i, ks in c.execute(f"select {k}, start from kernels").fetchall() if i in ls)
        if not lag:
            continue
        med = lag[len(lag) // 2] / 1e6
        print(f"candidate {k}: {len(lag)} matched, median kernel-after-launch lag {med:.3f} ms")
        if 0 <= med < 100 and (best is None or len(lag) > best):
            key, best = k, len(lag)
    if key is None:
        print("kernels columns:", kc)
        print("regions columns:", rc)
        raise SystemExit("no plausible correlation column")
    print(f"join column: {key}; kernels columns: {kc}; regions columns: {rc}")
    ks = c.execute(f"select name, stream_id, start, end, {key} from kernels order by start").fetchall()
    marks = [r[2] for r in ks if a.marker in r[0]]
    t0, t1 = marks[-4], marks[-3]     # the last timed step (bench.py runs two roofline steps after it)
    step = [r for r in ks if t0 < r[2] <= t1]
    launch = {}
    allocs = []
    for name, s, e, k in c.execute(f"select name, start, end, {key} from regions").fetchall():
        if "Launch" in name or "launch" in name:
            launch[k] = (s, e)
        elif name.startswith(("hipMalloc", "hipFree", "hipExtMalloc")):
            if t0 - 1e9 < s < t1:
                allocs.append((s, e, name))
    lags = sorted((r[2] - launch[r[4]][0]) / 1e3 for r in step if r[4] in launch)
    if lags:
        print(f"kernel start - launch call start (us): n {len(lags)}, min {lags[0]:.1f}, median {lags[len(lags) // 2]:.1f}, "
              f"max {lags[-1]:.1f}; kernels without a launch record: {sum(1 for r in step if r[4] not in launch)}")
    names = collections.Counter(n for n, *_ in c.execute("select name from regions").fetchall())
    print("region names:", names.most_common(12))
    by = collections.defaultdict(list)
    for r in step:
        by[r[1]].append(r)
    main_stream = max(by, key=lambda s: len(by[s]))
    mk = sorted(by[main_stream], key=lambda r: r[2])
    tot = collections.Counter()
    cnt = collections.Counter()
    gaps = []
    for prev, nxt in zip(mk, mk[1:]):
        g = nxt[2] - prev[3]
        if g < a.min_us * 1e3:
            continue
        api = launch.get(nxt[4])
        if any(s < nxt[2] and e > prev[3] for s, e, _ in allocs):
            why = "alloc"
        elif api is not None and api[1] > prev[3]:
            why = "host"
        elif api is None:
            why = "unknown"
        else:
            why = "wait"
        tot[why] += g
        cnt[why] += 1
        gaps.append((g, why, prev[0], nxt[0], (api[1] - prev[3]) / 1e3 if api else None))
    span = (t1 - t0) / 1e6
    busy = sum(r[3] - r[2] for r in mk) / 1e6
    print(f"step span {span:.2f} ms; main stream {main_stream}: {len(mk)} kernels, busy {busy:.2f} ms, "
          f"idle {span - busy:.2f} ms")
    print(f"gaps >= {a.min_us:g} us by cause: " + ", ".join(f"{k} {tot[k] / 1e6:.2f} ms ({cnt[k]})" for k in tot))
    pairs = collections.Counter()
    for g, why, p, n, _ in gaps:
        pairs[(why, p.split("(")[0][:40], n.split("(")[0][:40])] += g
    print("largest (cause, kernel before -> kernel after) totals:")
    for (why, p, n), g in pairs.most_common(a.top):
        print(f"  {g / 1e3:9.1f} us  {why:5s}  {p} -> {n}")
    print("largest single gaps:")
    for g, why, p, n, lag in sorted(gaps, reverse=True)[:a.top]:
        lg = f"launch returned {lag:+.1f} us after the previous kernel ended" if lag is not None else "launch unknown"
        print(f"  {g / 1e3:8.1f} us  {why:5s}  {p.split('(')[0][:50]} -> {n.split('(')[0][:50]}  ({lg})")


if __name__ == "__main__":
    main()
