"""Capture the train step as a HIP graph (trainer/step_graph.py) in debug mode, dump its DOT and print its
structure: nodes, edges, roots, leaves (a replayed graph is complete only when every leaf is), joins.

    python tools/graph_dump.py [--res 128] [--full] [--out gpurun_out/step_graph.dot]
"""
import argparse
import collections
import os
import re
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def parse_dot(path):
    """(nodes {id: label}, edges [(a, b)]) of a graph DOT file"""
    nodes, edges = {}, []
    ident = r'"?([A-Za-z0-9_]+)"?'
    for line in open(path, errors="replace"):
        m = re.match(r'\s*' + ident + r'\s*->\s*' + ident, line)
        if m:
            edges.append((m.group(1), m.group(2)))
            continue
        m = re.match(r'\s*' + ident + r'\s*\[(.*)', line)
        if m and m.group(1) not in ("graph", "node", "edge", "digraph", "subgraph"):
            lab = re.search(r'label\s*=\s*"(.*?)"', m.group(2)) or re.search(r'label\s*=\s*<(.*?)>', m.group(2))
            nodes[m.group(1)] = lab.group(1) if lab else ""
    return nodes, edges


def structure(path):
    nodes, edges = parse_dot(path)
    for a, b in edges:
        nodes.setdefault(a, "")
        nodes.setdefault(b, "")
    out_d, in_d = collections.Counter(a for a, _ in edges), collections.Counter(b for _, b in edges)
    leaves = [n for n in nodes if out_d[n] == 0]
    roots = [n for n in nodes if in_d[n] == 0]
    joins = [n for n in nodes if in_d[n] > 1]
    forks = [n for n in nodes if out_d[n] > 1]
    return {"nodes": len(nodes), "edges": len(edges), "roots": roots, "leaves": leaves, "joins": len(joins),
            "forks": len(forks), "labels": nodes}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--res", type=int, default=128)
    ap.add_argument("--full", action="store_true", help="the SDXL UNet (default: the tiny test config)")
    ap.add_argument("--out", default="gpurun_out/step_graph.dot")
    a = ap.parse_args()
    os.environ["OTAMD_STEP_GRAPH"] = "1"
    import torch
    from onetrainer_amd.dataLoader.SyntheticDataLoader import synthetic_sdxl_batch
    from onetrainer_amd.module import unet as U
    from onetrainer_amd.trainer.GenericTrainer import GenericTrainer
    from onetrainer_amd.trainer.step_graph import StepGraphs
    from onetrainer_amd.util import create
    from onetrainer_amd.util.config.TrainConfig import TrainConfig
    dev = torch.device("cuda:0")
    cfg = TrainConfig.default_values()
    cfg.batch_size = 2
    cfg.learning_rate_warmup_steps = 0
    model = create.create_model(cfg, dev, seed=3, unet_config=None if a.full else U.tiny_sdxl_config())
    tr = GenericTrainer(cfg, model=model)
    tr.start()
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    StepGraphs.debug_dot = a.out
    kw = {} if a.full else dict(te1_dim=48, te2_dim=48, pooled_dim=64)
    batch = synthetic_sdxl_batch(2, a.res, a.res, dev, seed=1, **kw)
    for _ in range(3):
        tr.train_step(batch)
    torch.cuda.synchronize()
    s = structure(a.out)
    print(f"{a.out}: {s['nodes']} nodes, {s['edges']} edges, {len(s['roots'])} roots, {len(s['leaves'])} leaves, "
          f"{s['joins']} joins, {s['forks']} forks")
    raw = open(a.out, errors="replace").read().splitlines()
    for n in s["leaves"][:10]:
        print("  leaf", n, s["labels"][n][:160])
        for line in raw:   # the node's own DOT lines (kernel name / node type) and its incoming edges
            if re.search(r'\b%s\b' % n, line):
                print("     ", line.strip()[:300])
    return 0


if __name__ == "__main__":
    sys.exit(main())
