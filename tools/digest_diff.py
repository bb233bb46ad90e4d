"""Compare tools/lora_grad_digest.py outputs (not a test): for each run, the first step and the first tensor in
backward order whose digest differs from run 1.  usage: python tools/digest_diff.py FILE..."""
import sys


def load(p):
    d, order = {}, {}
    for line in open(p):
        f = line.split()
        if len(f) == 3 and f[0].isdigit():
            k = (int(f[0]), f[1])
            d[k] = f[2]
            order.setdefault(int(f[0]), []).append(f[1])
    return d, order


def main():
    files = sys.argv[1:]
    base, order = load(files[0])
    for p in files[1:]:
        d, _ = load(p)
        diff = [k for k in base if base[k] != d.get(k)]
        if not diff:
            print(p, "same")
            continue
        st = min(k[0] for k in diff)
        names = [n for n in order[st] if (st, n) in diff]
        last = max(order[st].index(n) for n in names)
        print(p, "step", st, "ndiff", len(names), "first-in-backward", order[st][last])


if __name__ == "__main__":
    main()
