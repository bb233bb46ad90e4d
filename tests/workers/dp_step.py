"""One SDXL-shaped train step under data parallelism, for tests/test_dp_gpu.py (run as a child process).

    WORLD_SIZE=2 RANK=r LOCAL_RANK=r MASTER_ADDR=127.0.0.1 MASTER_PORT=p OTAMD_DIST_BACKEND=gloo \\
        python tests/workers/dp_step.py --global-batch 2 --out out_r.pt [--fp32-reduce]
    python tests/workers/dp_step.py --global-batch 2 --out ref.pt      # world 1, the whole batch

Every rank builds the same seeded model and the same global synthetic batch, keeps its slice
[r*b, (r+1)*b), runs GenericTrainer.train_step (predict -> loss -> backward with the bucketed
all-reduce -> clip -> fused AdamW) and saves: its local loss, the reduced flat gradient, the clip
total norm and the post-step flat parameters.
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--global-batch", type=int, default=2)
    ap.add_argument("--res", type=int, default=128)
    ap.add_argument("--out", required=True)
    ap.add_argument("--fp32-reduce", action="store_true")
    ap.add_argument("--steps", type=int, default=1)
    ap.add_argument("--ga", type=int, default=1, help="gradient accumulation steps (run --steps = ga for one update)")
    ap.add_argument("--no-norm-overlap", action="store_true", help="clip norm after the step instead of per bucket")
    args = ap.parse_args()
    if args.no_norm_overlap:
        os.environ["OTAMD_NORM_OVERLAP"] = "0"
    import torch

    from onetrainer_amd.dataLoader.SyntheticDataLoader import synthetic_sdxl_batch
    from onetrainer_amd.module import unet as U
    from onetrainer_amd.trainer.GenericTrainer import GenericTrainer
    from onetrainer_amd.util import create
    from onetrainer_amd.util.config.TrainConfig import TrainConfig

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    b = args.global_batch // world
    cfg = TrainConfig.default_values()
    cfg.batch_size = b
    cfg.learning_rate = 1e-4
    cfg.learning_rate_warmup_steps = 0
    cfg.optimizer.stochastic_rounding = False
    cfg.dp_reduce_fp32 = args.fp32_reduce
    cfg.dp_bucket_mb = 1            # many buckets: exercises the progressive launch
    cfg.gradient_accumulation_steps = args.ga
    model = create.create_model(cfg, dev, seed=3, unet_config=U.tiny_sdxl_config())
    tr = GenericTrainer(cfg, model=model)
    tr.start()
    assert tr.world == world and tr.rank == rank
    overlap = model.optimizer.norm_overlap is not None
    assert overlap == (not args.no_norm_overlap), overlap
    assert not overlap or model.optimizer.norm_overlap.dp == (world > 1)
    full = synthetic_sdxl_batch(args.global_batch, args.res, args.res, dev, seed=1, te1_dim=48, te2_dim=48,
                                pooled_dim=64)
    mine = {}
    for k, v in full.items():
        if isinstance(v, tuple):
            mine[k] = tuple(t[rank * b:(rank + 1) * b] for t in v)
        elif isinstance(v, list):
            mine[k] = v[rank * b:(rank + 1) * b]
        else:
            mine[k] = v[rank * b:(rank + 1) * b].contiguous()
    losses, norms = [], []
    for _ in range(args.steps):
        losses.append(tr.train_step(mine).float().cpu())
        norms.append(model.optimizer.clip_out[1].float().cpu())
    torch.cuda.synchronize()
    st = model.train_store
    torch.save({"loss": torch.stack(losses), "norm": torch.stack(norms), "grad": st.grad.float().cpu(),
                "param": st.data.cpu(), "world": world, "rank": rank, "norm_overlap": overlap}, args.out)
    if world > 1:
        torch.distributed.barrier()
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
