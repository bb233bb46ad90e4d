"""Oracle optimizer steps for the train-step parity tests (test infrastructure).

The reference steps bf16 parameters with bf16 grads, moments and the patched AdamW
(adamw_extensions.py:17-150; pinned bit-exact by tests/test_oracle_golden.py), after a global
clip_grad_norm_ on the bf16 grads (GenericTrainer.py:712-713).  OracleBF16AdamW reproduces that on
an fp32 oracle network whose parameters hold bf16 values: grads are rounded to bf16 (the param
dtype), clipped with the bf16 clip restatement and stepped with oracle.adamw.adamw_step_bf16.
OracleF32AdamW is the fp32 (LoRA adapter) case with adamw_step_f32.  OracleMasterAdamW is a full fine-tune with
fp32 weights under a bf16 autocast (weight_dtype FLOAT_32, TrainConfig.py:782): each weight gradient is a bf16 GEMM
result cast to fp32 (rounded to bf16 here, as the build's gradient store holds it), clip_grad_norm_ in fp32 (torch's
own), adamw_step_f32.
"""
import numpy as np
import torch

from oracle import adamw as OA


def _bits(t):
    return t.detach().cpu().contiguous().to(torch.bfloat16).view(torch.int16).numpy().astype(np.uint16).reshape(-1)


class OracleBF16AdamW:
    def __init__(self, params, lr, weight_decay=1e-2, betas=(0.9, 0.999), eps=1e-8, max_norm=1.0):
        self.params = [p for p in params]
        self.lr, self.wd, self.betas, self.eps, self.max_norm = lr, weight_decay, betas, eps, max_norm
        with torch.no_grad():
            for p in self.params:
                p.copy_(p.bfloat16().float())
        self.m = [np.zeros(p.numel(), np.uint16) for p in self.params]
        self.v = [np.zeros(p.numel(), np.uint16) for p in self.params]
        self.t = 0

    @torch.no_grad()
    def step(self):
        self.t += 1
        gb = [_bits(p.grad if p.grad is not None else torch.zeros_like(p)) for p in self.params]
        coef = None
        if self.max_norm is not None:
            _, total, coef = OA.clip_grad_norm_bf16(gb, self.max_norm)
            self.total_norm = total
        for k, p in enumerate(self.params):
            pb, self.m[k], self.v[k] = OA.adamw_step_bf16(_bits(p), gb[k], self.m[k], self.v[k], self.t, self.lr,
                                                          self.betas[0], self.betas[1], self.eps, self.wd,
                                                          clip_coef=coef)
            p.copy_(torch.from_numpy(OA.bf16_to_f32(pb)).view_as(p))
            p.grad = None


class OracleF32AdamW:
    def __init__(self, params, lr, weight_decay=1e-2, betas=(0.9, 0.999), eps=1e-8, max_norm=1.0):
        self.params = [p for p in params]
        self.lr, self.wd, self.betas, self.eps, self.max_norm = lr, weight_decay, betas, eps, max_norm
        self.m = [np.zeros(p.numel(), np.float32) for p in self.params]
        self.v = [np.zeros(p.numel(), np.float32) for p in self.params]
        self.t = 0

    @torch.no_grad()
    def step(self):
        self.t += 1
        coef = None
        if self.max_norm is not None:
            coef = torch.nn.utils.clip_grad_norm_(self.params, self.max_norm)   # fp32 grads: torch's own
            coef = None   # clip_grad_norm_ already scaled the grads in place
        for k, p in enumerate(self.params):
            g = p.grad.detach().cpu().numpy().reshape(-1) if p.grad is not None else np.zeros(p.numel(), np.float32)
            pn, self.m[k], self.v[k] = OA.adamw_step_f32(p.detach().cpu().numpy().reshape(-1), g, self.m[k], self.v[k],
                                                         self.t, self.lr, self.betas[0], self.betas[1], self.eps,
                                                         self.wd, clip_coef=coef)
            p.copy_(torch.from_numpy(pn).view_as(p))
            p.grad = None


class OracleMasterAdamW(OracleF32AdamW):
    @torch.no_grad()
    def step(self):
        for p in self.params:
            if p.grad is not None:
                p.grad.copy_(p.grad.bfloat16().float())
        super().step()
