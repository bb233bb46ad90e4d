"""LR lambdas (restated from modules/util/lr_scheduler_util.py:5-104; pinned by
tests/golden/reference_math.npz lr_* via tests/test_host_logic.py) and the LambdaLR factory
of modules/util/create.py:1114-1232."""
from __future__ import annotations

import math

import torch


def lr_lambda_warmup(warmup_steps, lr_lambda):
    def warmup(current_step: int):
        if current_step < warmup_steps:
            return float(current_step) / float(warmup_steps)
        return lr_lambda(current_step - warmup_steps)
    return warmup


def lr_lambda_constant():
    return lambda current_step: 1


def apply_min_factor(factor, min_factor):
    return min_factor + (1 - min_factor) * factor


def lr_lambda_linear(scheduler_steps, min_factor=1.0):
    def f(current_step):
        lin = max(0.0, float(scheduler_steps - current_step) / float(scheduler_steps))
        return apply_min_factor(lin, min_factor)
    return f


def lr_lambda_cosine(scheduler_steps, min_factor=1.0):
    def f(current_step):
        progress = float(current_step) / float(scheduler_steps)
        return apply_min_factor(max(0.0, 0.5 * (1.0 + math.cos(progress * math.pi))), min_factor)
    return f


def lr_lambda_cosine_with_restarts(scheduler_steps, num_cycles, min_factor=1.0):
    def f(current_step):
        progress = float(min(current_step, scheduler_steps - 1)) / float(scheduler_steps)
        return apply_min_factor(max(0.0, 0.5 * (1.0 + math.cos(progress * 2.0 * math.pi * num_cycles))), min_factor)
    return f


def lr_lambda_cosine_with_hard_restarts(scheduler_steps, num_cycles, min_factor=1.0):
    def f(current_step):
        progress = float(min(current_step, scheduler_steps - 1)) / float(scheduler_steps)
        return apply_min_factor(max(0.0, 0.5 * (1.0 + math.cos(((progress * num_cycles) % 1.0) * math.pi))), min_factor)
    return f


def lr_lambda_rex(scheduler_steps, min_factor=1.0):
    def f(current_step):
        if current_step < scheduler_steps:
            progress = current_step / scheduler_steps
            val = (1 - progress) / ((1 - 0.9) + 0.9 * (1 - progress))
        else:
            val = 0
        return apply_min_factor(val, min_factor)
    return f


def create_lr_scheduler(optimizer, learning_rate_scheduler="CONSTANT", warmup_steps=200, num_cycles=1.0,
                        min_factor=0.0, num_epochs=1, approximate_epoch_length=1, gradient_accumulation_steps=1,
                        global_step=0):
    total_steps = int(approximate_epoch_length * num_epochs / gradient_accumulation_steps)
    if warmup_steps > 1:
        warmup_steps = int(warmup_steps / gradient_accumulation_steps)
    elif 0 < warmup_steps <= 1:
        warmup_steps = int(warmup_steps * total_steps)
    else:
        warmup_steps = 0
    scheduler_steps = total_steps - warmup_steps
    if learning_rate_scheduler == "CONSTANT":
        fn = lr_lambda_constant()
    elif learning_rate_scheduler == "LINEAR":
        fn = lr_lambda_linear(scheduler_steps, min_factor)
    elif learning_rate_scheduler == "COSINE":
        fn = lr_lambda_cosine(scheduler_steps, min_factor)
    elif learning_rate_scheduler == "COSINE_WITH_RESTARTS":
        fn = lr_lambda_cosine_with_restarts(scheduler_steps, num_cycles, min_factor)
    elif learning_rate_scheduler == "COSINE_WITH_HARD_RESTARTS":
        fn = lr_lambda_cosine_with_hard_restarts(scheduler_steps, num_cycles, min_factor)
    elif learning_rate_scheduler == "REX":
        fn = lr_lambda_rex(scheduler_steps, min_factor)
    else:
        fn = lr_lambda_constant()
    if warmup_steps > 0:
        fn = lr_lambda_warmup(warmup_steps, fn)
    return torch.optim.lr_scheduler.LambdaLR(optimizer, lr_lambda=fn,
                                             last_epoch=int(global_step / gradient_accumulation_steps) - 1)
