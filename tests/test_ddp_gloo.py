"""Data-parallel gradient reduction (trainer/ddp.py) with world_size 2 over gloo on CPU:
buckets launch as their parameters become ready (in reverse layout order, as backward produces
them) and the result equals the sum over ranks (the 1/world factor lives in the loss gradient)."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from onetrainer_amd.module.param_store import FlatParamStore
from onetrainer_amd.trainer.ddp import GradBucketReducer

SPECS = [(f"p{i}", (37 * (i + 1) % 300 + 8,), "g") for i in range(40)]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        st = FlatParamStore(SPECS, torch.float32, "cpu")
        red = GradBucketReducer(st, bucket_bytes=2048)
        assert len(red.buckets) > 3
        launched = []
        for step in range(2):
            for i, (n, s, _) in enumerate(SPECS):
                st.params[n].grad.fill_(rank + 1 + i + 100 * step)
            for n in reversed(st.order):         # backward finishes parameters in reverse order
                st.mark_ready([n])
                launched.append(len(red.works))
            red.finish()
            for i, (n, s, _) in enumerate(SPECS):
                exp = sum(r + 1 + i + 100 * step for r in range(world))
                assert torch.all(st.params[n].grad == exp), (n, st.params[n].grad[:3], exp)
        # buckets were issued progressively during "backward", not all at the end
        assert launched[len(launched) // 4] > 0
        q.put((rank, "ok"))
    except Exception as e:  # pragma: no cover
        q.put((rank, repr(e)))
    finally:
        dist.destroy_process_group()


def test_bucket_allreduce_gloo_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    assert res == {0: "ok", 1: "ok"}, res


def _worker_ga(rank, world, port, q, reduce_fp32):
    """gradient accumulation 2 (trainer/GenericTrainer.train_step): the reducer is armed only for the
    update step's backward; the first micro-step accumulates locally, no bucket is reduced twice."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        st = FlatParamStore(SPECS, torch.bfloat16 if reduce_fp32 else torch.float32, "cpu")
        red = GradBucketReducer(st, bucket_bytes=2048, reduce_fp32=reduce_fp32)
        for window in range(2):
            for micro in range(2):
                red.arm(micro == 1)
                for i, (n, s, _) in enumerate(SPECS):
                    g = st.params[n].grad
                    v = float(rank + 1 + i % 8 + 10 * micro + 20 * window)   # sums stay exact in bf16
                    if micro == 0:
                        g.fill_(v)
                    else:
                        g.add_(v)
                for n in reversed(st.order):
                    st.mark_ready([n])
                if micro == 0:
                    assert not red.works, "a GA micro-step launched an all-reduce"
            red.finish()
            for i, (n, s, _) in enumerate(SPECS):
                exp = sum(2 * (r + 1 + i % 8 + 20 * window) + 10 for r in range(world))
                assert torch.all(st.params[n].grad.float() == exp), (n, st.params[n].grad[:3], exp)
        q.put((rank, "ok"))
    except Exception as e:  # pragma: no cover
        q.put((rank, repr(e)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("reduce_fp32", [False, True])
def test_bucket_allreduce_grad_accumulation_gloo_world2(reduce_fp32):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_ga, args=(r, 2, port, q, reduce_fp32)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    assert res == {0: "ok", 1: "ok"}, res


def _worker_norm(rank, world, port, q):
    """the clip norm under data parallel (util/optimizer/adamw_fused.OverlappedGradNorm(reducer=...)): its ranges are
    the reducer's buckets and each is summed from the reducer's completion hook -- every norm chunk exactly once per
    update step, after its bucket holds the global sum, never on a GA micro-step (CPU: the hooks run in finish(); on
    the GPU on the reducer's post stream, tests/test_dp_gpu.py)"""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from onetrainer_amd.util.optimizer.adamw_fused import FusedAdamW, OverlappedGradNorm
        specs = SPECS + [("big", (70000,), "g")]   # one tensor of two norm chunks (64 K elements each)
        st = FlatParamStore(specs, torch.bfloat16, torch.device("cpu"))
        red = GradBucketReducer(st, bucket_bytes=2048)
        opt = FusedAdamW(st, [{"params": [st.params[n] for n, *_ in specs]}])
        norm = OverlappedGradNorm(opt, reducer=red)
        assert norm.dp and len(norm.buckets) == len(red.buckets)
        chunks = [(b, e) for b, e, _ in (tuple(x) for x in _chunk_table(opt))]
        hits = []

        def fake_launch(bi, side):   # the chunk kernel's arithmetic: fp64 sum of squares per chunk slot
            norm.launched[bi] = True
            c0, c1, _ = norm.buckets[bi]
            for c in range(c0, c1):
                b, e = chunks[c]
                opt._chunk_sq[c] = (st.grad[b:e].double() ** 2).sum()
                hits.append(c)
        norm._launch = fake_launch
        for window in range(2):
            for micro in range(2):
                update = micro == 1
                red.arm(update)
                norm.arm(update)
                for i, (n, *_) in enumerate(specs):
                    v = float(rank + 1 + i % 8 + 10 * micro + 20 * window)
                    g = st.params[n].grad
                    g.fill_(v) if micro == 0 else g.add_(v)
                for n in reversed(st.order):
                    st.mark_ready([n])
                if not update:
                    assert not hits, "a GA micro-step summed norm chunks"
            red.finish()
            norm.finish()
            assert sorted(hits) == list(range(len(chunks))), "every chunk exactly once"
            hits.clear()
            assert norm.take()
            want = torch.tensor([(st.grad[b:e].double() ** 2).sum().item() for b, e in chunks], dtype=torch.float64)
            assert torch.equal(opt._chunk_sq[:len(chunks)], want)   # sums of the all-reduced gradients
        q.put((rank, "ok"))
    except Exception as e:  # pragma: no cover
        import traceback
        q.put((rank, traceback.format_exc()))
    finally:
        dist.destroy_process_group()


def _chunk_table(opt):
    from onetrainer_amd import _lib
    arr = (_lib.NormChunk * opt._n_chunks).from_buffer_copy(opt._chunks.cpu().numpy().tobytes())
    return [(c.begin, c.end, c.tensor) for c in arr]


def test_overlapped_norm_follows_the_reduce_gloo_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_norm, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    assert res == {0: "ok", 1: "ok"}, res


def test_bucket_partition_is_contiguous_and_complete():
    st = FlatParamStore(SPECS, torch.bfloat16, "cpu")
    if not dist.is_available():
        pytest.skip("torch.distributed unavailable")
    red = GradBucketReducer.__new__(GradBucketReducer)
    GradBucketReducer.__init__(red, st, bucket_bytes=1024)
    names = [n for b in red.buckets for n in b[2]]
    assert sorted(names) == sorted(st.order)
    prev_begin = None
    for b, e, ns in red.buckets:
        assert b < e and b == st.slots[ns[-1]].offset
        if prev_begin is not None:
            assert e <= prev_begin + 8
        prev_begin = b


def _worker_dead_peer(rank, world, port, q):
    """rank 1 dies before the collective; rank 0's all-reduce must time out (ddp.init_from_env's
    group timeout) and the trainer's abort path must let it exit, not block forever."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(world), RANK=str(rank),
                      LOCAL_RANK=str(rank), OTAMD_DIST_BACKEND="gloo")
    import time
    from types import SimpleNamespace

    from onetrainer_amd.trainer import ddp
    from onetrainer_amd.trainer.GenericTrainer import GenericTrainer
    from onetrainer_amd.util.config.TrainConfig import TrainConfig
    from onetrainer_amd.util.TrainProgress import TrainProgress
    ddp.init_from_env(timeout_s=5)
    if rank == 1:
        os._exit(0)          # dies without a word
    cfg = TrainConfig.default_values()
    cfg.backup_after_unit = "NEVER"
    cfg.workspace_dir = os.path.join(os.environ.get("TMPDIR", "/tmp"), f"otamd_dead_peer_{os.getpid()}")
    tp = TrainProgress()
    loader = SimpleNamespace(get_data_set=lambda: SimpleNamespace(start_next_epoch=lambda: None),
                             get_data_loader=lambda: iter(range(3)))
    tr = GenericTrainer(cfg, model=SimpleNamespace(train_progress=tp), data_loader=loader)
    tr.rank, tr.world = rank, world

    def step(batch):          # the gradient all-reduce of a DP step
        dist.all_reduce(torch.ones(4))
        tp.next_step(1)
        return torch.zeros(())

    tr.train_step = step
    t0 = time.time()
    try:
        tr.train(log_every=0)
        q.put((rank, "no error"))
    except Exception as e:
        q.put((rank, f"raised after {time.time() - t0:.0f}s, group initialized: {dist.is_initialized()}"))


def test_dead_peer_times_out_and_aborts():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_dead_peer, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    rank, msg = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
    assert rank == 0 and msg.startswith("raised") and msg.endswith("group initialized: False"), msg
    assert all(p.exitcode is not None for p in procs)


def _worker_wallclock(rank, world, port, q):
    """a MINUTE backup timer under data parallel: rank 0's wall clock fires, rank 1's does not; both ranks
    back up together, and the ranks meet on the host only every `agree_every` update steps (no per-step
    rendezvous-store traffic, no keys left behind).  A STEP save timer beside it saves at its exact steps (it
    fires on every rank alike and does not wait for an agreement point), and the command rank 0 raised after
    the last agreement point runs at the end of train() instead of being dropped."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(world), RANK=str(rank),
                      LOCAL_RANK=str(rank), OTAMD_DIST_BACKEND="gloo")
    from types import SimpleNamespace

    import onetrainer_amd.util.TimedActionMixin as TM
    from onetrainer_amd.trainer import ddp
    from onetrainer_amd.trainer.GenericTrainer import GenericTrainer
    from onetrainer_amd.util.config.TrainConfig import TrainConfig
    from onetrainer_amd.util.TrainProgress import TrainProgress
    try:
        ddp.init_from_env(timeout_s=60)
        now = [1000.0]
        TM.time.time = lambda: now[0]
        cfg = TrainConfig.default_values()
        cfg.backup_after, cfg.backup_after_unit = 1, "MINUTE"
        cfg.save_every, cfg.save_every_unit = 10, "STEP"
        cfg.workspace_dir = os.path.join(os.environ.get("TMPDIR", "/tmp"), f"otamd_wallclock_{os.getpid()}")
        tp = TrainProgress()
        loader = SimpleNamespace(get_data_set=lambda: SimpleNamespace(start_next_epoch=lambda: None),
                                 get_data_loader=lambda: iter(range(40)))
        tr = GenericTrainer(cfg, model=SimpleNamespace(train_progress=tp), data_loader=loader)
        tr.rank, tr.world = rank, world
        backups = []
        tr.backup = lambda t=None: backups.append(tp.global_step)
        saves = []
        tr.save = lambda t=None: saves.append(tp.global_step)
        store = dist.distributed_c10d._get_default_store()
        keys = {}

        def step(batch):
            if tp.global_step == 17:   # after the control group's one-time rendezvous and two agreements
                keys[17] = store.num_keys()
            if rank == 0:
                now[0] += 61.0          # only rank 0's clock moves
            dist.all_reduce(torch.ones(4))
            tp.next_step(1)
            return torch.zeros(())

        tr.train_step = step
        tr.train(log_every=0, max_steps=40)
        assert tr.agreements == 4, tr.agreements          # update steps 0, 16, 32 and the end of train()
        assert backups == [16, 32, 40], backups
        assert saves == [9, 19, 29, 39], saves         # the STEP timer's own steps (TimedActionMixin, pinned)
        assert store.num_keys() == keys[17], (store.num_keys(), keys)   # nothing written per step
        q.put((rank, "ok"))
    except Exception as e:  # pragma: no cover
        q.put((rank, repr(e)))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


def test_wallclock_backup_agreement_gloo_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_wallclock, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    assert res == {0: "ok", 1: "ok"}, res
