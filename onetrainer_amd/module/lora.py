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
    """adapters of one base GEMM (a fused group: q|k|v, k|v, q|k|v|mlp ... or a single module).
    Only the modules matching the layer filter carry adapters; the others are zero rows of `up2`."""
    key: str
    modules: list            # adapted module names (reference names), in fused order
    kind: str                # "linear" | "conv"
    cin: int                 # base input channels (store layout; conv_in padded)
    couts: list              # per adapted module, base output channels (store layout)
    k: int                   # conv kernel size (1 for linear)
    cin_ref: int = 0         # diffusers input channels (unpadded)
    conv1x1: bool = False    # a 1x1 Conv2d held as a linear (diffusers NCHW [out, in, 1, 1] on export)
    couts_ref: list = field(default_factory=list)
    ranges: list = field(default_factory=list)   # per adapted module, (n0, n1) output columns in the fused GEMM
    n_total: int = 0         # fused GEMM output width
    down: torch.Tensor | None = None     # bf16 shadow [P*r, cin] or [r, k, k, cin]
    up2: torch.Tensor | None = None      # bf16 shadow [n_total, P*r] (block-diagonal, zero rows elsewhere), x alpha/r
    upT: torch.Tensor | None = None      # bf16 shadow [r, n_total] = the parts' (s up_p)^T side by side, and downT
    downT: torch.Tensor | None = None    # [cin, P r] = down^T: the operands of the fused backward input gradient
    #                                      (kernels.linear_dgrad_lora); linear sites at r = 32 with one module or a
    #                                      fully adapted q|k|v group (the instances), else None
    g_down: torch.Tensor | None = None   # fp32 grad view, shape of `down`
    g_up: list = field(default_factory=list)   # fp32 grad views [cout_p, r]
    store: FlatParamStore | None = None
    names: list = field(default_factory=list)   # store slot names (for mark_ready / acc)
    scale: float = 1.0
    rank: int = 0
    params: tuple = ()
    group: tuple = ()        # all modules of the base GEMM (adapted or not)

    @property
    def part_width(self) -> int:
        """output columns per adapted part when the parts tile the fused GEMM's columns evenly (every module of the
        group adapted, equal widths): the down-projection can then run inside the base GEMM (kernels.linear_lora);
        0 otherwise."""
        P = len(self.modules)
        if P == 0 or self.n_total % P:
            return 0
        pw = self.n_total // P
        return pw if list(self.ranges) == [(p * pw, (p + 1) * pw) for p in range(P)] else 0

    def acc(self) -> bool:
        return self.store.accumulate_into(self.names)

    def done(self):
        self.store.mark_ready(self.names)


def module_list(model):
    """(module name, kind, cin, cout, k, cin_ref, cout_ref) for every Linear/Conv2d of a model with
    `specs` (name, diffusers shape, kind, fan_in) and a FlatParamStore `store`, in forward order."""
    out = []
    for name, shape, kind, _ in model.specs:
        if not name.endswith(".weight") or kind not in ("linear", "conv"):
            continue
        mod = name[:-len(".weight")]
        st = model.store.slots[name].shape
        if kind == "linear":
            out.append((mod, "linear", st[1], st[0], 1, shape[1], shape[0]))
        elif len(st) == 2:           # 1x1 conv, held as a linear
            out.append((mod, "linear1x1", st[1], st[0], 1, shape[1], shape[0]))
        else:
            out.append((mod, "conv", st[3], st[0], st[1], shape[1], shape[0]))
    return out


def unet_fused_group(name, by_name):
    """the base GEMM a UNet module runs in (module/unet.py): attn1 q|k|v and attn2 k|v are fused."""
    for suf in (".attn1.to_q", ".attn1.to_k", ".attn1.to_v"):
        if name.endswith(suf):
            b = name[:-len(suf)] + ".attn1."
            return [b + "to_q", b + "to_k", b + "to_v"]
    for suf in (".attn2.to_k", ".attn2.to_v"):
        if name.endswith(suf):
            b = name[:-len(suf)] + ".attn2."
            return [b + "to_k", b + "to_v"]
    return [name]


class LoRAWrapper:
    """LoRAModuleWrapper(model, prefix, config, module_filter) for a HIP model (UNet or Flux
    transformer): the model supplies `specs`, `store`, `device` and optionally `fused_group(name, by_name)`."""

    def __init__(self, model, rank: int = 16, alpha: float = 1.0, module_filter=None, prefix: str = "lora_unet",
                 seed: int = 0, dtype=torch.float32):
        self.model = self.unet = model
        self.rank, self.alpha, self.prefix = rank, float(alpha), prefix
        self.scale = self.alpha / rank
        filt = [x.strip() for x in (module_filter or []) if x.strip()]
        allmods = module_list(model)
        by_name = {m[0]: m for m in allmods}
        adapted = {m[0] for m in allmods if not filt or any(f in m[0] for f in filt)}
        group_of = getattr(model, "fused_group", unet_fused_group)
        sites, seen = [], set()
        for m in allmods:
            if m[0] in seen:
                continue
            group = [g for g in group_of(m[0], by_name) if g in by_name]
            seen.update(group)
            mods = [g for g in group if g in adapted]
            if not mods:
                continue
            n0, ranges = 0, {}
            for g in group:
                ranges[g] = (n0, n0 + by_name[g][3])
                n0 += by_name[g][3]
            kind = "conv" if m[1] == "conv" else "linear"
            key = group[0] if len(group) == 1 else (group[0].rsplit(".", 1)[0] + "." + "|".join(
                g.rsplit(".", 1)[1] for g in group))
            sites.append(LoraSite(key=key, modules=mods, kind=kind, cin=m[2], couts=[by_name[g][3] for g in mods],
                                  k=m[4], cin_ref=m[5], couts_ref=[by_name[g][6] for g in mods], scale=self.scale,
                                  rank=rank, conv1x1=m[1] == "linear1x1", ranges=[ranges[g] for g in mods],
                                  n_total=n0, group=tuple(group)))
        self.sites = sites
        self.site_of = {}
        for s in sites:
            for mname in s.group:
                self.site_of[mname] = s
            self.site_of[s.key] = s
        # fp32 store: per site, downs adjacent (fused operand), then ups
        specs = []
        for s in sites:
            for mname in s.modules:
                dshape = (rank, s.cin) if s.kind == "linear" else (rank, s.k, s.k, s.cin)
                specs.append((f"{prefix}.{mname}.lora_down.weight", dshape, prefix))
            for mname, co in zip(s.modules, s.couts):
                specs.append((f"{prefix}.{mname}.lora_up.weight", (co, rank), prefix))
        self.store = FlatParamStore(specs, dtype, torch.device(model.device))
        # bf16 shadow: per site the fused down then the block-diagonal up (+ their transposes for the fused backward
        # input gradient on single-module linear sites)
        total = 0
        layout = []
        for s in sites:
            P = len(s.modules)
            dn = P * rank * s.cin * s.k * s.k
            un = s.n_total * P * rank
            doff = (total + 7) // 8 * 8
            uoff = (doff + dn + 7) // 8 * 8
            total = uoff + un
            toff = None
            if s.kind == "linear" and rank == 32 and ((P == 1 and len(s.group) == 1) or
                                                      (P == 3 and len(s.group) == 3 and s.part_width > 0)):
                toff = (total + 7) // 8 * 8                  # upT [r, n_total], then downT [cin, P r]
                total = toff + rank * s.n_total + s.cin * P * rank
            layout.append((doff, uoff, toff))
        self.shadow = torch.zeros(total + 8, dtype=torch.bfloat16, device=model.device)
        entries = []
        for s, (doff, uoff, toff) in zip(sites, layout):
            P = len(s.modules)
            dshape = (P * rank, s.cin) if s.kind == "linear" else (rank, s.k, s.k, s.cin)
            s.down = self.shadow[doff:doff + math.prod(dshape)].view(dshape)
            s.up2 = self.shadow[uoff:uoff + s.n_total * P * rank].view(s.n_total, P * rank)
            s.store = self.store
            s.names = [f"{prefix}.{m}.lora_down.weight" for m in s.modules] + \
                      [f"{prefix}.{m}.lora_up.weight" for m in s.modules]
            s.g_down = self.store.view(s.names[:P], dshape, grad=True)
            s.g_up = [self.store.view(n, grad=True) for n in s.names[P:]]
            s.params = tuple(self.store.params[n] for n in s.names)
            dslot = self.store.slots[s.names[0]]
            entries.append((dslot.offset, doff, P * rank, dslot.numel // rank, dslot.numel // rank, 1.0))
            for p in range(P):
                us = self.store.slots[s.names[P + p]]
                entries.append((us.offset, uoff + s.ranges[p][0] * P * rank + p * rank, s.couts[p], rank, P * rank,
                                self.scale))
            if toff is not None:   # upT = [(s up_0)^T | (s up_1)^T | ...] along the output, downT = [down_0; ...]^T
                s.upT = self.shadow[toff:toff + rank * s.n_total].view(rank, s.n_total)
                e0 = toff + rank * s.n_total
                s.downT = self.shadow[e0:e0 + s.cin * P * rank].view(s.cin, P * rank)
                for p in range(P):
                    us = self.store.slots[s.names[P + p]]
                    entries.append((us.offset, toff + s.ranges[p][0], s.couts[p], rank, s.n_total, self.scale, 1))
                entries.append((dslot.offset, e0, P * rank, s.cin, P * rank, 1.0, 1))
        arr = (_lib.LoraShadowEntry * len(entries))()
        for i, (src, dst, rows, cols, ld, sc, *tr) in enumerate(entries):
            arr[i].src, arr[i].dst, arr[i].rows, arr[i].cols, arr[i].dst_ld, arr[i].scale = src, dst, rows, cols, ld, sc
            arr[i].transpose = tr[0] if tr else 0
        self._table = torch.frombuffer(bytearray(bytes(arr)), dtype=torch.uint8).to(model.device)
        self._n_entries = len(entries)
        if seed is not None:
            self.init_weights(seed)
        self.refresh()

    def site_for(self, modules):
        """site of the base GEMM running `modules` (None when none of them carries an adapter)."""
        s = self.site_of.get(modules[0])
        if s is not None and tuple(modules) != s.group:
            raise NotImplementedError(f"base GEMM {modules} does not match the LoRA fusion group {s.group}")
        return s

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


LoRAUNetWrapper = LoRAWrapper   # the UNet form (prefix "lora_unet")
