"""LoRA restatement for the oracle UNet (test infrastructure only).

modules/module/LoRAModule.py:318-322: y = orig_forward(x) + lora_up(dropout(lora_down(x))) * (alpha / rank),
lora_down = Linear(in, r) / Conv2d(in, r, k, stride, padding), lora_up = Linear(r, out) / Conv2d(r, out, 1)
(:125-155), hooked on every Linear/Conv2d whose name contains one of the filter strings (:462-470).
Implemented as forward hooks on the oracle's nn.Modules, fp32.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F


class OracleLoRA:
    def __init__(self, model: torch.nn.Module, rank: int, alpha: float, module_filter=None, prefix="lora_unet"):
        self.rank, self.alpha, self.prefix = rank, float(alpha), prefix
        self.scale = self.alpha / rank
        filt = [x for x in (module_filter or []) if x]
        self.params = {}
        self.handles = []
        for name, m in model.named_modules():
            if not isinstance(m, (torch.nn.Linear, torch.nn.Conv2d)):
                continue
            if filt and not any(f in name for f in filt):
                continue
            if isinstance(m, torch.nn.Linear):
                down = torch.zeros(rank, m.in_features)
                up = torch.zeros(m.out_features, rank)
            else:
                down = torch.zeros(rank, m.in_channels, *m.kernel_size)
                up = torch.zeros(m.out_channels, rank, 1, 1)
            d = torch.nn.Parameter(down)
            u = torch.nn.Parameter(up)
            self.params[f"{prefix}.{name}.lora_down.weight"] = d
            self.params[f"{prefix}.{name}.lora_up.weight"] = u
            self.handles.append(m.register_forward_hook(self._hook(m, d, u)))

    def _hook(self, m, d, u):
        def fn(mod, inp, out):
            x = inp[0]
            if isinstance(mod, torch.nn.Linear):
                return out + F.linear(F.linear(x, d), u) * self.scale
            t = F.conv2d(x, d, stride=mod.stride, padding=mod.padding)
            return out + F.conv2d(t, u) * self.scale
        return fn

    def load_state_dict(self, sd):
        with torch.no_grad():
            for k, p in self.params.items():
                p.copy_(sd[k].reshape(p.shape).float())

    def parameters(self):
        return list(self.params.values())
