#!/usr/bin/env python3
"""Benchmark: SDXL 1.0 UNet full fine-tune train step, 1024^2 (128^2 latents), bf16, b=4 per GPU.

BASELINE.json metric "train images/sec (whole node) + step-time p50, SDXL 1024^2 bf16 at 1/2/4/8 GPU";
workload = configs[2] (SDXL full-finetune 1024^2, global batch 32 = 8 x 4) run per GPU at b=4
(weak scaling: per-GPU work fixed).  A step is the reference's GenericTrainer step body
(GenericTrainer.py:672-749): predict (noise, timesteps, DDPM noising, UNet fwd) -> MSE loss ->
backward -> [DP all-reduce] -> clip_grad_norm(1.0) -> AdamW(+bf16 SR) -> LR step.  Inputs are
synthetic cached latents/text states resident in HBM; weights random (no network here).

    python bench.py [--gpus N --steps K --warmup W]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N   (driver, N > 1)
"""
from __future__ import annotations

import argparse
import gc
import json
import math
import os
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

PEAK_BF16_TFLOPS = 2500.0      # MI355X dense bf16 MFMA (MI355X_MICROARCH.md)
PEAK_HBM_GBS = 8000.0


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(res=512, sd15=False, warmup=1, timed=3):
    """the oracle (test infrastructure: the CPU fp32 restatement of the reference
    step -- diffusers-architecture UNet fwd+bwd, DDPM noise + timesteps seeded per step, MSE,
    clip_grad_norm 1.0, torch AdamW) on this host's cores at batch 1: `warmup` untimed steps, then
    `timed` steps.  Returns (step seconds list, threads)."""
    from oracle import unet as OU
    from oracle import diffusion as OD
    threads = len(os.sched_getaffinity(0))
    threads = min(threads, int(os.environ.get("OMP_NUM_THREADS", threads)))
    torch.set_num_threads(threads)
    cfg = OU.sd15_config() if sd15 else OU.sdxl_config()
    torch.manual_seed(0)
    with torch.device("meta"):
        m = OU.UNet2DConditionModel(cfg)
    m = m.to_empty(device="cpu")
    with torch.no_grad():
        for p in m.parameters():
            p.uniform_(-0.02, 0.02)
    opt = torch.optim.AdamW(m.parameters(), lr=3e-6, weight_decay=1e-2, foreach=True)
    betas = OD.scaled_linear_betas()
    h = res // 8
    x0 = torch.randn(1, 4, h, h)   # the scaled latent: N(0,1)/scaling_factor cached, times scaling_factor
    ehs = torch.randn(1, 77, cfg.cross_attention_dim)
    te = None if sd15 else torch.randn(1, 1280)
    tid = None if sd15 else torch.tensor([[float(res), float(res), 0., 0., float(res), float(res)]])

    def step(i):
        g = torch.Generator().manual_seed(i)
        eps = OD.create_noise(x0.shape, g)
        t = OD.timestep_discrete(1000, 1, g)
        xt = OD.add_noise_ddpm(x0, eps, t, betas)
        pred = m(xt, t, ehs, te, tid)
        loss = OD.diffusion_losses(pred, eps, torch.ones(1)).mean()
        loss.backward()
        torch.nn.utils.clip_grad_norm_(m.parameters(), 1.0)
        opt.step()
        opt.zero_grad(set_to_none=True)

    times = []
    for i in range(warmup + timed):
        t0 = time.perf_counter()
        step(i)
        dt = time.perf_counter() - t0
        log(f"[bench] cpu baseline {'SD1.5' if sd15 else 'SDXL'} {res}^2 step {i} {dt:.2f}s"
            f"{' (warm-up)' if i < warmup else ''}")
        if i >= warmup:
            times.append(dt)
    del m, opt
    return times, threads


def gemm_roofline(tr, batch, in_step: bool = True):
    """Dominant kernel family (bf16 MFMA GEMM / implicit-GEMM conv: gemm2_kernel<*>, gemm_kernel,
    splitk_reduce): one extra, untimed train step with a HIP event pair around every GEMM launch on
    the stream it is launched on.  achieved = sum(2 M N K) / sum(launch durations).

    in_step=True: the step exactly as timed (weight-gradient GEMMs on the side stream, concurrent with the
    dgrad chain), so the durations are the in-step ones a rocprofv3 kernel trace of the timed steps
    reports (profiles/r3_kstats_*.csv); in_step=False: side stream off, every GEMM alone on the chip."""
    from onetrainer_amd import kernels as K
    recs = []
    orig = K._gemm

    def timed(a, splits, device):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        orig(a, splits, device)
        e1.record()
        recs.append((2.0 * a.M * a.N * a.K, e0, e1, 2.0 * (a.M * a.K + a.K * a.N + a.M * a.N)))

    from onetrainer_amd.module import streams
    was = streams.enabled()
    if not in_step:
        streams.set_enabled(False)
    graphs, tr.graphs = tr.graphs, None   # an eager step: every GEMM launched (and timed) from the host
    K._gemm = timed
    try:
        # through the ctypes host path, whose _gemm the timer wraps: the same kernels with the same plans as the
        # native host layer (bit-identical, tests/test_host_layer_gpu.py), only the host side of the launch differs
        with K.python_host():
            tr.train_step(batch)
        torch.cuda.synchronize()
    finally:
        K._gemm = orig
        streams.set_enabled(was)
        tr.graphs = graphs
    flops = sum(r[0] for r in recs)
    ms = sum(r[1].elapsed_time(r[2]) for r in recs)
    gemm_roofline.algo_bytes = sum(r[3] for r in recs)   # GEMM-form operand bytes (conv A as im2col)
    return flops, ms, len(recs)


TRAFFIC_FILES = {"sdxl": "pmc_traffic_sdxl1024_b4.json", "sd15": "pmc_traffic_sd15.json",
                 "sdxl-lora": "pmc_traffic_sdxl-lora.json", "flux": "pmc_traffic_flux.json"}


def pmc_traffic(model: str):
    """GEMM-family memory-side traffic per step of this config from its committed PMC passes
    (tools/gpu_counters.sh -> tools/gpu_pmc.sh: rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE in separate runs of
    this bench at its default shape, FETCH_SIZE doubled for gfx950).  (path, data) or (path, None)."""
    path = os.path.join(ROOT, "profiles", TRAFFIC_FILES[model])
    if not os.path.exists(path):
        return path, None
    with open(path) as f:
        return path, json.load(f)


def _die_with_parent():
    """child side of launch_ranks, before exec: SIGTERM when the launcher dies (a launcher killed by a timeout
    must not leave ranks running on the GPU)"""
    import ctypes
    import signal
    ctypes.CDLL(None).prctl(1, int(signal.SIGTERM))   # PR_SET_PDEATHSIG


def launch_ranks(n: int) -> int:
    """`bench.py --gpus N` without a torchrun environment: start N fresh child ranks (one per GPU,
    RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* in their env) before this process touches the GPU, wait
    for all of them and return the worst exit code.  Rank 0 prints the JSON line."""
    import socket
    import subprocess
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env,
                                      preexec_fn=_die_with_parent))
    import time
    while True:   # a rank that fails ends the others (its peers would otherwise block in their next collective)
        rcs = [p.poll() for p in procs]
        bad = [rc for rc in rcs if rc not in (None, 0)]
        if bad:
            for p in procs:
                if p.poll() is None:
                    p.terminate()
            for p in procs:
                try:
                    p.wait(timeout=30)
                except subprocess.TimeoutExpired:
                    p.kill()
                    p.wait()
            print(f"bench.py: a rank exited with {bad[0]}; the other ranks were stopped", file=sys.stderr)
            return bad[0]
        if all(rc == 0 for rc in rcs):
            return 0
        time.sleep(0.2)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=None, help="per-GPU batch (default 4 sdxl / 16 sd15)")
    ap.add_argument("--res", type=int, default=None, help="default 1024 (sdxl) / 512 (sd15)")
    ap.add_argument("--model", choices=["sdxl", "sd15", "flux", "sdxl-lora"], default="sdxl",
                    help="sdxl: configs[2] per GPU (metric workload); sd15: configs[1] (SD 1.5 512^2 b=16); "
                         "flux: configs[4] per GPU (FLUX.1 LoRA r16, 768^2, b=4); sdxl-lora: configs[3] per GPU "
                         "(SDXL LoRA r32, aspect-ratio buckets drawn per step, b=4)")
    ap.add_argument("--tiny", action="store_true",
                    help="(tests of the bench's own legs, e.g. launch_ranks) the tiny SDXL-shaped test UNet instead of "
                         "the full network; never a metric line")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-vae", action="store_true", help="skip the VAE-encode (latent caching) side measurement")
    ap.add_argument("--autotune", action="store_true",
                    help="time (tile, split-K) candidates per GEMM signature in warm-up instead of the measured plan "
                         "table / analytic plan")
    ap.add_argument("--dump-plans", default=None,
                    help="with --autotune: merge the tuned plans into this plan-table JSON (kernels.dump_plan_table)")
    args = ap.parse_args()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args.gpus))
    if "WORLD_SIZE" in os.environ and int(os.environ["WORLD_SIZE"]) != args.gpus:
        log(f"[bench] note: --gpus {args.gpus} but WORLD_SIZE={os.environ['WORLD_SIZE']}; n_gpus reports the world size")

    from onetrainer_amd.dataLoader.SyntheticDataLoader import synthetic_sdxl_batch
    from onetrainer_amd.module.unet import flops_per_image, sd15_config, sdxl_config
    from onetrainer_amd.trainer.GenericTrainer import GenericTrainer
    from onetrainer_amd.util.config.TrainConfig import TrainConfig

    sd15 = args.model == "sd15"
    flux = args.model == "flux"
    sdxl_lora = args.model == "sdxl-lora"
    if args.res is None:
        args.res = 512 if sd15 else (768 if flux else 1024)
    if args.batch is None:
        args.batch = 16 if sd15 else 4
    ucfg = sd15_config() if sd15 else sdxl_config()
    cfg = TrainConfig.default_values()
    if sd15:
        cfg.model_type = "STABLE_DIFFUSION_15"
    if flux:   # training_presets/#flux LoRA.json: LORA, LOGIT_NORMAL, lr 3e-4 (base bf16: NF4 is CUDA-only)
        cfg.model_type, cfg.training_method = "FLUX_DEV_1", "LORA"
        cfg.timestep_distribution = "LOGIT_NORMAL"
        args.no_vae = True
    if sdxl_lora:   # training_presets/#sdxl 1.0 LoRA.json (lr 3e-4) + lora_rank 32, fp32 adapters, ARB on
        cfg.training_method = "LORA"
        cfg.lora_rank = 32
        args.no_vae = True
    cfg.batch_size = args.batch
    cfg.learning_rate = 3e-4 if sdxl_lora else 3e-6
    cfg.learning_rate_warmup_steps = 0
    cfg.resolution = str(args.res)

    from onetrainer_amd import kernels as K
    K.set_gemm_autotune(args.autotune)   # plans are tuned inside the untimed warm-up steps
    tiny_kw = {}
    if args.tiny:
        from onetrainer_amd.module.unet import tiny_sdxl_config
        from onetrainer_amd.util import create
        if sd15 or flux or sdxl_lora:
            raise SystemExit("--tiny: the sdxl workload only")
        ucfg = tiny_sdxl_config()
        tiny_kw = dict(te1_dim=48, te2_dim=48, pooled_dim=64)
        args.no_cpu_baseline = args.no_vae = True
        from onetrainer_amd.trainer import ddp
        ddp.init_from_env()   # the model goes to this rank's device
        tr = GenericTrainer(cfg, model=create.create_model(cfg, torch.device(f"cuda:{torch.cuda.current_device()}"),
                                                            seed=0, unet_config=ucfg))
    else:
        tr = GenericTrainer(cfg)
    t0 = time.time()
    tr.start()
    rank, world = tr.rank, tr.world
    dev = tr.device
    net = tr.model.transformer if flux else tr.model.unet
    log(f"[bench] rank {rank}/{world} model ready in {time.time() - t0:.1f}s "
        f"({net.num_parameters() / 1e9:.3f} B params)")
    if flux:
        from onetrainer_amd.dataLoader.SyntheticDataLoader import synthetic_flux_batch
        batch = synthetic_flux_batch(args.batch, args.res, args.res, dev, seed=rank)
    elif sdxl_lora:
        # every step draws ONE bucket for the whole global batch (seeded, identical
        # on all ranks, §8(e)); buckets of the restated mgds AspectBucketing, aspects up to 1:1.75
        import random
        from onetrainer_amd.dataLoader.aspect_bucketing import ASPECTS, AspectBucketing
        buckets = AspectBucketing(args.res, 64, ASPECTS[:4]).resolutions
        arb = {r: synthetic_sdxl_batch(args.batch, r[0], r[1], dev, seed=rank) for r in buckets}
        order = [random.Random(1000 + i).choice(buckets) for i in range(args.warmup + args.steps + 1)]
    else:
        batch = synthetic_sdxl_batch(args.batch, args.res, args.res, dev, seed=rank, sdxl=not sd15,
                                     scaling_factor=0.18215 if sd15 else 0.13025, **tiny_kw)
    if sdxl_lora:
        for r in buckets:   # every bucket shape once (plans, workspaces), untimed
            tr.train_step(arb[r])
        batch = arb[buckets[0]]

    for i in range(args.warmup):
        tr.train_step(arb[order[i]] if sdxl_lora else batch)
        if i == 0:
            torch.cuda.synchronize()
            log(f"[bench] first step done, mem {torch.cuda.max_memory_allocated() / 2**30:.1f} GiB")
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    stream = torch.cuda.current_stream()
    evs = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps + 1)]
    # no cyclic-GC pauses on the issuing host thread inside the timed steps (autograd graphs are freed by
    # reference counting; GenericTrainer.train does the same between its collection points)
    gc.collect()
    gc.freeze()
    gc.disable()
    ms0 = torch.cuda.memory_stats(dev)
    t_start = time.perf_counter()
    evs[0].record(stream)
    losses = []
    trace_alloc = os.environ.get("OTAMD_BENCH_ALLOC_TRACE") == "1"   # diagnostic: which timed steps grow the pool
    for i in range(args.steps):
        losses.append(tr.train_step(arb[order[args.warmup + i]] if sdxl_lora else batch))
        evs[i + 1].record(stream)
        if trace_alloc:
            log(f"[bench] timed step {i}: device allocs so far "
                f"{torch.cuda.memory_stats(dev).get('num_device_alloc', 0) - ms0.get('num_device_alloc', 0)}")
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t_start
    gc.enable()
    ms1 = torch.cuda.memory_stats(dev)
    alloc = {k: ms1.get(k, 0) - ms0.get(k, 0) for k in ("num_device_alloc", "num_device_free", "num_alloc_retries",
                                                          "num_sync_all_streams")}
    step_ms_seq = [evs[i].elapsed_time(evs[i + 1]) for i in range(args.steps)]
    step_ms = sorted(step_ms_seq)
    p50 = step_ms[len(step_ms) // 2]
    p90 = step_ms[min(len(step_ms) - 1, int(0.9 * len(step_ms)))]
    loss_last = torch.stack(losses).float().mean()
    if world > 1:
        t = torch.tensor([elapsed], device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = t.item()
        dist.all_reduce(loss_last)
        loss_last /= world
    loss_val = loss_last.item()
    if not math.isfinite(loss_val):
        raise RuntimeError(f"non-finite loss {loss_val}")

    g_flops, g_ms, g_n = gemm_roofline(tr, batch, in_step=True)
    i_flops, i_ms, _ = gemm_roofline(tr, batch, in_step=False)
    vae = None
    if not args.no_vae:   # latent caching, reported beside the step, not part of `value`
        from tools.bench_vae import run as vae_run
        vae = vae_run(args.res, args.batch, iters=5, warmup=1, device=str(dev))
    g_achieved = g_flops / (g_ms * 1e-3) / 1e12
    i_achieved = i_flops / (i_ms * 1e-3) / 1e12
    pmc_path, pmc = pmc_traffic(args.model)
    default_shape = (args.batch, args.res) == {"sdxl": (4, 1024), "sd15": (16, 512), "sdxl-lora": (4, 1024),
                                               "flux": (4, 768)}[args.model]

    imgs = args.batch * world * args.steps
    value = imgs / elapsed
    ms = 1000.0 * elapsed / args.steps
    if flux:   # LoRA: 2 x base forward (fwd + dgrad, frozen base) + 3 x LoRA branch
        from onetrainer_amd.module import flux as FX
        n_img = (args.res // 16) ** 2
        fwd_tf = FX.flops_per_image(net.cfg, n_img, 77) / 1e12
        lora_tf = 2.0 * FX.lora_macs_per_image(tr.model.transformer_lora, 77, n_img) / 1e12
        train_tf_img = 2.0 * fwd_tf + 3.0 * lora_tf
        basis = f"{train_tf_img:.3f} TFLOP/image algorithmic (2 x {fwd_tf:.3f} base fwd + 3 x {lora_tf:.3f} LoRA)"
    elif sdxl_lora:   # 2 x base forward (fwd + dgrad; frozen base) averaged over the drawn buckets
        steps_b = order[args.warmup:args.warmup + args.steps]
        fwd_tf = sum(flops_per_image(ucfg, h // 8, w // 8) for h, w in steps_b) / len(steps_b) / 1e12
        train_tf_img = 2.0 * fwd_tf
        basis = (f"{train_tf_img:.3f} TFLOP/image algorithmic (2 x {fwd_tf:.3f} base fwd averaged over the drawn "
                 f"buckets; the LoRA branch GEMMs are not counted: conservative)")
    else:
        fwd_tf = flops_per_image(ucfg, args.res // 8, args.res // 8) / 1e12
        train_tf_img = 3.0 * fwd_tf                       # fwd + dgrad + wgrad
        basis = f"{train_tf_img:.3f} TFLOP/image algorithmic (3 x {fwd_tf:.3f} fwd)"
    achieved = train_tf_img * args.batch / (ms / 1000.0)   # per GPU, TFLOP/s
    mname = "SD 1.5 UNet (859.5M params)" if sd15 else "SDXL 1.0 UNet (2.567B params)"
    if args.tiny:
        mname = f"tiny SDXL-shaped test UNet ({net.num_parameters() / 1e6:.2f}M params; bench-leg test, not a metric)"
    label = "SD1.5 512^2 bf16" if sd15 else "SDXL 1024^2 bf16"
    wl = f"{'SD 1.5' if sd15 else 'SDXL 1.0'} UNet full fine-tune train step {args.res}^2 (latent {args.res // 8}^2), " \
         f"b={args.batch}/GPU, AdamW+bf16 SR, clip 1.0"
    if sdxl_lora:
        mname = "SDXL 1.0 UNet (2.567B params, bf16 frozen base) + LoRA r32 (every Linear/Conv2d, fp32)"
        label = "SDXL LoRA r32 ARB ~1024^2 bf16"
        wl = f"SDXL 1.0 LoRA rank 32 train step, aspect-ratio buckets {buckets} (one per step, seeded), " \
             f"b={args.batch}/GPU, fp32 AdamW, clip 1.0"
    if flux:
        mname = "FLUX.1-dev transformer (11.9B params, bf16 base) + LoRA r16 (all Linear)"
        label = f"FLUX.1 LoRA {args.res}^2 bf16"
        wl = f"FLUX.1 LoRA rank {cfg.lora_rank} train step {args.res}^2 (latent {args.res // 8}^2 -> {(args.res // 16) ** 2} " \
             f"tokens + 77 text), b={args.batch}/GPU, flow matching LOGIT_NORMAL, fp32 AdamW, clip 1.0"
    out = {
        "metric": "train images/sec (whole node) + step-time p50, " + label,
        "value": round(value, 3),
        "unit": "images/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms, 2),
        "step_ms_p50": round(p50, 2),
        "step_ms_p90": round(p90, 2),
        "step_ms_max": round(step_ms[-1], 2),
        "step_ms_each": [round(t, 2) for t in step_ms_seq],   # timed steps in order
        "step_buckets": [list(b) for b in order[args.warmup:args.warmup + args.steps]] if sdxl_lora else None,
        "allocator_in_timed_steps": alloc,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "bf16",
        "data": "synthetic (random cached latents/text states, random-init weights)",
        "config": {"workload": wl,
                   "model": mname, "global_batch": args.batch * world,
                   "seq_len": (args.res // 8) ** 2, "parallelism": f"dp{world}"},
        "loss": round(loss_val, 5),
        "loss_exact": loss_val,
        "losses_exact": [float(v) for v in torch.stack(losses).float().cpu()],
        "lora_forwards_fused_vs_two_launch": list(K.lora_fused_counts()),
        "roofline": {"bound": "mfma", "achieved": round(g_achieved, 1), "peak": PEAK_BF16_TFLOPS, "unit": "TFLOP/s",
                     "frac": round(g_achieved / PEAK_BF16_TFLOPS, 4),
                     "traffic": (pmc["gemm_total_gb"] if pmc and default_shape else None),
                     "traffic_unit": "GB per step, GEMM family (FETCH_SIZE x 2 + WRITE_SIZE, memory-side L2 counters: "
                                     f"Infinity-Cache hits included), from profiles/{os.path.basename(pmc_path)} "
                                     "(PMC passes of this config's bench at its default shape)",
                     "algorithmic_gb": round(gemm_roofline.algo_bytes / 1e9, 2),
                     "kernel": "bf16 MFMA GEMM / implicit-GEMM conv (gemm2_kernel<*>, gemm_kernel, splitk_reduce_kernel)",
                     "basis": f"sum(2*M*N*K) over the {g_n} GEMM/conv launches of one step / sum of their in-step "
                              f"HIP-event durations ({g_ms:.2f} ms of GEMM kernel time per step, summed over the main "
                              f"and the weight-gradient stream, which run concurrently)",
                     "isolated_achieved": round(i_achieved, 1), "isolated_frac": round(i_achieved / PEAK_BF16_TFLOPS, 4),
                     "isolated_basis": f"the same launches with the side stream off, each GEMM alone on the chip "
                                       f"({i_ms:.2f} ms per step)",
                     "step_achieved": round(achieved, 1), "step_frac": round(achieved / PEAK_BF16_TFLOPS, 4),
                     "step_basis": basis + " x per-GPU images / step time"},
        "cpu_baseline": None,
        "vae_encode": vae,
        "gemm_plans": "autotuned in warm-up (%d signatures)" % len(K.gemm_autotune_cache()) if args.autotune
        else K.plan_source(),
        "step_graph": (f"forward+backward replayed as HIP graphs ({len(tr.graphs.entries)} captured shapes); "
                       f"noise/timesteps and the optimizer update eager") if tr.graphs is not None else "eager",
    }
    if args.autotune and args.dump_plans and rank == 0:
        n = K.dump_plan_table(args.dump_plans)
        print(f"plan table: {n} signatures -> {args.dump_plans}", file=sys.stderr)
    if rank == 0 and world == 1 and not args.no_cpu_baseline and not flux and not sdxl_lora:
        del tr
        torch.cuda.empty_cache()
        try:
            # C1 (SD 1.5 preset, 512^2, b=1): 1 warm-up + 3 timed, p50; then the bench workload's own
            # network at its resolution, b=1 (SDXL 1024^2: 1 warm-up + 3 timed, p50) -> `value`
            c1, threads = cpu_baseline(512, sd15=True, warmup=1, timed=3)
            c1_p50 = sorted(c1)[len(c1) // 2]
            if sd15 and args.res == 512:
                big, big_p50 = c1, c1_p50
            else:
                big, _ = cpu_baseline(args.res, sd15=sd15, warmup=1, timed=3)   # >= 3 timed
                big_p50 = sorted(big)[len(big) // 2]
            out["cpu_baseline"] = {
                "value": round(1.0 / big_p50, 5), "unit": "images/s", "cores": threads, "kind": "port",
                "cpu_model": cpu_model(), "threads": threads,
                "sample": (f"oracle (CPU fp32 restatement of the reference step: UNet fwd+bwd, DDPM noise, MSE, clip, "
                           f"torch AdamW) on {threads} threads of {cpu_model()}: "
                           f"{'SD 1.5' if sd15 else 'SDXL 1.0'} {args.res}^2 b=1, 1 warm-up + {len(big)} timed step(s), "
                           f"p50 {big_p50:.2f} s -> value; C1 SD 1.5 512^2 b=1 1 warm-up + 3 timed p50 "
                           f"{c1_p50:.2f} s ({1.0 / c1_p50:.4f} images/s)"),
                "c1_sd15_512_b1": {"step_s": [round(x, 3) for x in c1], "p50_s": round(c1_p50, 3),
                                   "images_per_s": round(1.0 / c1_p50, 5)},
                "workload_b1": {"step_s": [round(x, 3) for x in big], "p50_s": round(big_p50, 3)},
            }
        except Exception as e:   # the baseline must not sink the GPU measurement
            out["cpu_baseline"] = {"value": None, "unit": "images/s", "cores": None, "kind": "port",
                                   "sample": f"failed: {e!r}"}
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
