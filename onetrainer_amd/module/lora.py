"""LoRA adapters for the HIP UNet (SDXL / SD1.5 LoRA training).

Semantics of modules/module/LoRAModule.py:283-323 (LoRAModule) and :427-587 (LoRAModuleWrapper):
every Linear / Conv2d of the UNet whose name matches the layer filter gets
    y = orig(x) + up(down(x)) * (alpha / rank)
with `down` a Linear in->r (Conv2d: the base kernel/stride/padding, in->r), `up` a Linear r->out
(Conv2d: 1x1 r->out), down ~ kaiming_uniform(a=sqrt(5)) = U(+-1/sqrt(fan_in)), up = 0,
dropout p = 0, adapter weights fp32 (TrainConfig lora_weight_dtype), computed in bf16.
Names / state-dict keys follow the reference: "lora_unet.<module>.lora_down.weight",
".lora_up.weight" (diffusers NCHW layouts for conv) and ".alpha".

MI355X layout (not a translation):
  * one fp32 FlatParamStore holds every adapter (fused optimizer, grad-norm and DP buckets run
    over it exactly as over the full fine-tune store); the base UNet store is frozen;
  * a bf16 shadow of all adapters is refreshed by ONE kernel per step (otamd_lora_shadow),
    with alpha/rank folded into `up`;
  * adapters of weights the base runs as one GEMM (to_q|to_k|to_v, to_k|to_v) are fused the
    same way: their downs are one [P*r, in] operand, their ups one block-diagonal [sum out, P*r];
  * the up projection is the second K segment of the base GEMM (y = [x | t] [W | s B]^T), so a
    LoRA forward costs one skinny GEMM (t = x A^T) plus K + r instead of K in the base GEMM.
"""
from __future__ import annotations

import ctypes as C
import math
from dataclasses import dataclass, field

import torch

from .. import _lib
from .. import kernels as K
from .param_store import FlatParamStore

PRESETS = {"attn-mlp": ["attentions"], "attn-only": ["attn"], "full": []}   # StableDiffusionXLLoRASetup.py:12-16


@dataclass
class LoraSite:
    """adapters of one base GEMM: P parts (P > 1 for a fused q|k|v or k|v projection)."""
    key: str
    modules: list            # reference module names, one per part
    kind: str                # "linear" | "conv"
    cin: int                 # base input channels (store layout; conv_in padded)
    couts: list              # per-part base output channels (store layout; conv_out padded)
    k: int                   # conv kernel size (1 for linear)
    cin_ref: int = 0         # diffusers input channels (unpadded)
    conv1x1: bool = False    # a 1x1 Conv2d held as a linear (diffusers NCHW [out, in, 1, 1] on export)
    couts_ref: list = field(default_factory=list)
    down: torch.Tensor | None = None     # bf16 shadow [P*r, cin] or [r, k, k, cin]
    up2: torch.Tensor | None = None      # bf16 shadow [sum(couts), P*r] (block-diagonal for P > 1), x alpha/r
    g_down: torch.Tensor | None = None   # fp32 grad view, shape of `down`
    g_up: list = field(default_factory=list)   # fp32 grad views [cout_p, r]
    store: FlatParamStore | None = None
    names: list = field(default_factory=list)   # store slot names (for mark_ready / acc)
    scale: float = 1.0
    rank: int = 0
    params: tuple = ()

    def acc(self) -> bool:
        return self.store.accumulate_into(self.names)

    def done(self):
        self.store.mark_ready(self.names)


def _module_list(unet):
    """(module name, kind, cin, cout, k, cin_ref, cout_ref) for every Linear/Conv2d of the UNet, in
    forward order, from the base parameter specs (diffusers shapes) and the store layout."""
    out = []
    for name, shape, kind, _ in unet.specs:
        if not name.endswith(".weight") or kind not in ("linear", "conv"):
            continue
        mod = name[:-len(".weight")]
        st = unet.store.slots[name].shape
        if kind == "linear":
            out.append((mod, "linear", st[1], st[0], 1, shape[1], shape[0]))
        elif len(st) == 2:           # 1x1 conv, held as a linear
            out.append((mod, "linear1x1", st[1], st[0], 1, shape[1], shape[0]))
        else:
            out.append((mod, "conv", st[3], st[0], st[1], shape[1], shape[0]))
    return out


class LoRAUNetWrapper:
    """LoRAModuleWrapper(unet, "lora_unet", config, module_filter) for the HIP UNet."""

    def __init__(self, unet, rank: int = 16, alpha: float = 1.0, module_filter=None, prefix: str = "lora_unet",
                 seed: int = 0, dtype=torch.float32):
        self.unet = unet
        self.rank, self.alpha, self.prefix = rank, float(alpha), prefix
        self.scale = self.alpha / rank
        filt = [x.strip() for x in (module_filter or []) if x.strip()]
        mods = [m for m in _module_list(unet) if not filt or any(f in m[0] for f in filt)]
        by_name = {m[0]: m for m in mods}
        # group fused projections exactly as the base UNet runs them
        sites, used = [], set()
        for m in mods:
            name = m[0]
            if name in used:
                continue
            group = [name]
            if name.endswith(".attn1.to_q"):
                b = name[:-len("to_q")]
                if b + "to_k" in by_name and b + "to_v" in by_name:
                    group = [b + "to_q", b + "to_k", b + "to_v"]
            elif name.endswith(".attn2.to_k"):
                b = name[:-len("to_k")]
                if b + "to_v" in by_name:
                    group = [b + "to_k", b + "to_v"]
            parts = [by_name[g] for g in group]
            used.update(group)
            kind = "conv" if m[1] == "conv" else "linear"
            key = group[0] if len(group) == 1 else (group[0].rsplit(".", 1)[0] + "." + "|".join(
                g.rsplit(".", 1)[1] for g in group))
            sites.append(LoraSite(key=key, modules=group, kind=kind, cin=m[2], couts=[p[3] for p in parts], k=m[4],
                                  cin_ref=m[5], couts_ref=[p[6] for p in parts], scale=self.scale, rank=rank,
                                  conv1x1=m[1] == "linear1x1"))
        self.sites = sites
        self.site_of = {}
        for s in sites:
            for mname in s.modules:
                self.site_of[mname] = s
            self.site_of[s.key] = s
        # fp32 store: per site, downs adjacent (fused operand), then ups
        specs = []
        for s in sites:
            for mname in s.modules:
                dshape = (rank, s.cin) if s.kind == "linear" else (rank, s.k, s.k, s.cin)
                specs.append((f"{prefix}.{mname}.lora_down.weight", dshape, "unet_lora"))
            for mname, co in zip(s.modules, s.couts):
                specs.append((f"{prefix}.{mname}.lora_up.weight", (co, rank), "unet_lora"))
        self.store = FlatParamStore(specs, dtype, torch.device(unet.device))
        # bf16 shadow: per site the fused down then the block-diagonal up
        total = 0
        layout = []
        for s in sites:
            P = len(s.modules)
            dn = P * rank * s.cin * s.k * s.k
            un = sum(s.couts) * P * rank
            doff = (total + 7) // 8 * 8
            uoff = (doff + dn + 7) // 8 * 8
            total = uoff + un
            layout.append((doff, uoff))
        self.shadow = torch.zeros(total + 8, dtype=torch.bfloat16, device=unet.device)
        entries = []
        for s, (doff, uoff) in zip(sites, layout):
            P = len(s.modules)
            dshape = (P * rank, s.cin) if s.kind == "linear" else (rank, s.k, s.k, s.cin)
            s.down = self.shadow[doff:doff + math.prod(dshape)].view(dshape)
            s.up2 = self.shadow[uoff:uoff + sum(s.couts) * P * rank].view(sum(s.couts), P * rank)
            s.store = self.store
            s.names = [f"{prefix}.{m}.lora_down.weight" for m in s.modules] + \
                      [f"{prefix}.{m}.lora_up.weight" for m in s.modules]
            s.g_down = self.store.view(s.names[:P], dshape, grad=True)
            s.g_up = [self.store.view(n, grad=True) for n in s.names[P:]]
            s.params = tuple(self.store.params[n] for n in s.names)
            dslot = self.store.slots[s.names[0]]
            entries.append((dslot.offset, doff, P * rank, dslot.numel // rank, dslot.numel // rank, 1.0))
            row0 = 0
            for p in range(P):
                us = self.store.slots[s.names[P + p]]
                entries.append((us.offset, uoff + row0 * P * rank + p * rank, s.couts[p], rank, P * rank, self.scale))
                row0 += s.couts[p]
        arr = (_lib.LoraShadowEntry * len(entries))()
        for i, (src, dst, rows, cols, ld, sc) in enumerate(entries):
            arr[i].src, arr[i].dst, arr[i].rows, arr[i].cols, arr[i].dst_ld, arr[i].scale = src, dst, rows, cols, ld, sc
        self._table = torch.frombuffer(bytearray(bytes(arr)), dtype=torch.uint8).to(unet.device)
        self._n_entries = len(entries)
        if seed is not None:
            self.init_weights(seed)
        self.refresh()

    # ----- parameters ----------------------------------------------------------------------------
    def init_weights(self, seed: int):
        """LoRAModule.initialize_weights (LoRAModule.py:305-309): kaiming_uniform(a=sqrt(5)) on down
        = U(+-1/sqrt(fan_in)), zeros on up.  Padded input channels (conv_in) stay zero."""
        g = torch.Generator(device=self.unet.device).manual_seed(seed)
        with torch.no_grad():
            for s in self.sites:
                for m in s.modules:
                    p = self.store.params[f"{self.prefix}.{m}.lora_down.weight"]
                    fan_in = s.cin_ref * s.k * s.k
                    bound = 1.0 / math.sqrt(fan_in)
                    v = (torch.rand(p.shape, generator=g, device=p.device) * 2 - 1) * bound
                    if s.cin != s.cin_ref:
                        v[..., s.cin_ref:] = 0
                    p.copy_(v)
                    self.store.params[f"{self.prefix}.{m}.lora_up.weight"].zero_()

    def refresh(self):
        """fp32 adapters -> bf16 shadow (x alpha/rank on up): one launch; call after every update."""
        if self.store.device.type != "cuda":
            return   # structure-only use on a CPU host (tests); the kernels need the GPU
        K.lora_shadow(self.store.data, self.shadow, self._table, self._n_entries)

    def parameters(self):
        return [p for _, p in self.store.named_parameters()]

    def num_parameters(self, reference_shapes: bool = True) -> int:
        n = 0
        for s in self.sites:
            for cin_l, co in zip([s.cin_ref if reference_shapes else s.cin] * len(s.modules),
                                 s.couts_ref if reference_shapes else s.couts):
                n += self.rank * cin_l * s.k * s.k + co * self.rank
        return n

    def state_dict(self, grads: bool = False) -> dict:
        """reference key layout (LoRAModuleWrapper.state_dict): NCHW conv weights, unpadded, + alpha."""
        out = {}
        for s in self.sites:
            for m, co_ref in zip(s.modules, s.couts_ref):
                d = self.store.params[f"{self.prefix}.{m}.lora_down.weight"]
                u = self.store.params[f"{self.prefix}.{m}.lora_up.weight"]
                d = d.grad if grads else d.detach()
                u = u.grad if grads else u.detach()
                if s.kind == "conv":
                    d = d[..., :s.cin_ref].permute(0, 3, 1, 2)
                    u = u[:co_ref].reshape(co_ref, self.rank, 1, 1)
                elif s.conv1x1:
                    d = d.reshape(self.rank, s.cin_ref, 1, 1)
                    u = u.reshape(co_ref, self.rank, 1, 1)
                out[f"{self.prefix}.{m}.lora_down.weight"] = d.contiguous()
                out[f"{self.prefix}.{m}.lora_up.weight"] = u.contiguous()
                out[f"{self.prefix}.{m}.alpha"] = torch.tensor(self.alpha)
        return out

    def load_state_dict(self, sd: dict):
        with torch.no_grad():
            for s in self.sites:
                for m, co_ref in zip(s.modules, s.couts_ref):
                    dk, uk = f"{self.prefix}.{m}.lora_down.weight", f"{self.prefix}.{m}.lora_up.weight"
                    if dk not in sd:
                        continue   # LoRAModuleWrapper.load_state_dict: missing keys keep their init
                    d = sd[dk].to(self.store.device, torch.float32)
                    u = sd[uk].to(self.store.device, torch.float32)
                    pd, pu = self.store.params[dk], self.store.params[uk]
                    if d.dim() == 4 and d.shape[2] > 1:
                        pd.zero_()
                        pd[..., :s.cin_ref].copy_(d.permute(0, 2, 3, 1))
                    else:
                        pd.copy_(d.reshape(pd.shape))
                    pu.zero_()
                    pu[:co_ref].copy_(u.reshape(co_ref, self.rank))
        self.refresh()
