"""The bucketed gradient all-reduce over RCCL (torch.distributed 'nccl'), for tests/test_dp_gpu.py (child process).

A one-rank RCCL group on the box's one GPU (RCCL cannot put two ranks on one device): the same tiny SDXL train step
runs twice from the same seed, once plain and once with a GradBucketReducer on the RCCL group attached to the
trainer -- every bucket's all-reduce is issued from inside backward on the reducer's issue stream, waits on both
compute streams, and is joined by finish() before clip + AdamW.  A one-rank SUM is the identity, so the two steps
must end with bit-identical gradients and parameters; bf16 in place and the fp32 staging path both run.

    MASTER_ADDR=127.0.0.1 MASTER_PORT=p python tests/workers/rccl_world1.py --out res.pt
"""
import argparse
import datetime
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", required=True)
    args = ap.parse_args()
    import torch
    import torch.distributed as dist

    from onetrainer_amd.dataLoader.SyntheticDataLoader import synthetic_sdxl_batch
    from onetrainer_amd.module import unet as U
    from onetrainer_amd.trainer.ddp import GradBucketReducer
    from onetrainer_amd.trainer.GenericTrainer import GenericTrainer
    from onetrainer_amd.util import create
    from onetrainer_amd.util.config.TrainConfig import TrainConfig

    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=0, world_size=1, timeout=datetime.timedelta(seconds=120))
    assert dist.get_backend() == "nccl"

    def run(reducer_kind, norm_overlap=False):
        cfg = TrainConfig.default_values()
        cfg.batch_size = 2
        cfg.learning_rate = 1e-4
        cfg.learning_rate_warmup_steps = 0
        model = create.create_model(cfg, dev, seed=3, unet_config=U.tiny_sdxl_config())
        tr = GenericTrainer(cfg, model=model)
        tr.start()
        model.optimizer.norm_overlap = None   # as under data parallel: the norm is taken of the reduced gradients
        nb = 0
        if reducer_kind is not None:
            tr.reducer = GradBucketReducer(model.train_store, bucket_bytes=1 << 20, reduce_fp32=reducer_kind == "fp32")
            nb = len(tr.reducer.buckets)
            if norm_overlap:   # the clip norm's sums per bucket on the reducer's post stream, after each RCCL reduce
                from onetrainer_amd.util.optimizer.adamw_fused import OverlappedGradNorm
                model.optimizer.norm_overlap = OverlappedGradNorm(model.optimizer, reducer=tr.reducer)
        batch = synthetic_sdxl_batch(2, 128, 128, dev, seed=1, te1_dim=48, te2_dim=48, pooled_dim=64)
        for _ in range(2):
            tr.train_step(batch)
        torch.cuda.synchronize()
        st = model.train_store
        return st.grad.float().cpu(), st.data.cpu(), nb, model.optimizer.clip_out.cpu()

    g0, p0, _, c0 = run(None)
    g1, p1, nb, _ = run("bf16")
    g2, p2, _, _ = run("fp32")
    g3, p3, _, c3 = run("bf16", norm_overlap=True)
    torch.save({"grad_equal": bool(torch.equal(g0, g1)), "param_equal": bool(torch.equal(p0, p1)),
                "grad_equal_fp32": bool(torch.equal(g0, g2)), "param_equal_fp32": bool(torch.equal(p0, p2)),
                "norm_overlap_equal": bool(torch.equal(g0, g3) and torch.equal(p0, p3) and torch.equal(c0, c3)),
                "buckets": nb, "nonzero": bool(g0.abs().sum() > 0)}, args.out)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
