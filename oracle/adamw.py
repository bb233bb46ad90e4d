"""numpy restatement of the reference optimizer step (test infrastructure only).

Follows:
  step_adamw_parameter   modules/util/optimizer/adamw_extensions.py:17-150 (non-capturable branch 125-148)
  addcdiv_stochastic_    modules/util/bf16_stochastic_rounding.py:48-61
  copy_stochastic_       modules/util/bf16_stochastic_rounding.py:5-30
  clip_grad_norm_        torch.nn.utils, as called at modules/trainer/GenericTrainer.py:712-713
Each torch op of the bf16 path rounds its result to bf16 (round-to-nearest-even); lerp_ and
addcmul_ are fused multiply-adds in torch's CPU kernels (pinned by the golden fixtures).
"""
from __future__ import annotations

import math

import numpy as np

U64 = np.uint64


def bf16_to_f32(bits: np.ndarray) -> np.ndarray:
    return (bits.astype(np.uint32) << 16).view(np.float32)


def f32_to_bf16_bits(x: np.ndarray) -> np.ndarray:
    u = np.asarray(x, dtype=np.float32).view(np.uint32).astype(np.uint64)
    nan = (u & 0x7FFFFFFF) > 0x7F800000
    r = ((u + 0x7FFF + ((u >> 16) & 1)) >> 16).astype(np.uint16)
    return np.where(nan, np.uint16(0x7FC0), r)


def rbf(x: np.ndarray) -> np.ndarray:
    return bf16_to_f32(f32_to_bf16_bits(x))


def fma32(a, b, c) -> np.ndarray:
    """float32 fused multiply-add via float64 (the float32 product is exact in float64)."""
    return (np.asarray(a, np.float64) * np.asarray(b, np.float64) + np.asarray(c, np.float64)).astype(np.float32)


def sr_bits(seed: int, idx: np.ndarray) -> np.ndarray:
    """The HIP kernel's SR dither (onetrainer_amd/csrc/adamw.hip sr_bits): a 32-bit
    multiply-xorshift hash of (element index, step seed); the dither is its high 16 bits.
    (The reference draws torch.randint per step, bf16_stochastic_rounding.py:17-24; the
    stream itself is not reproducible across implementations, only its distribution.)"""
    U32 = np.uint32
    idx = idx.astype(np.uint64)
    k = U32((seed ^ (seed >> 32)) & 0xFFFFFFFF)
    with np.errstate(over="ignore"):
        x = (idx & np.uint64(0xFFFFFFFF)).astype(U32) * U32(0x9E3779B1) + k
        x ^= (idx >> np.uint64(32)).astype(U32) * U32(0x85EBCA77)
        x ^= x >> U32(16)
        x *= U32(0x21F0AAAD)
        x ^= x >> U32(15)
        x *= U32(0x735A2D97)
        x ^= x >> U32(15)
    return (x >> U32(16)).astype(np.uint32)


def copy_stochastic(source_f32: np.ndarray, rand16: np.ndarray) -> np.ndarray:
    """bf16 bits of SR(source): add the 16-bit dither to the int32 view, mask 0xFFFF0000."""
    u = source_f32.astype(np.float32).view(np.int32).astype(np.int64)
    u = (u + rand16.astype(np.int64)) & 0xFFFF0000
    return ((u.astype(np.uint64) & 0xFFFFFFFF) >> 16).astype(np.uint16)


def adamw_step_bf16(p, g, m, v, step, lr, beta1=0.9, beta2=0.999, eps=1e-8, weight_decay=1e-2,
                    rand16=None, clip_coef=None):
    """One step on bf16 bit arrays p, g, m, v (uint16).  rand16: SR dither (None = SR off).
    Returns new (p, m, v) bf16 bits."""
    pf, gf, mf, vf = bf16_to_f32(p), bf16_to_f32(g), bf16_to_f32(m), bf16_to_f32(v)
    if clip_coef is not None:
        gf = rbf(gf * np.float32(clip_coef))
    pf = rbf(pf * np.float32(1 - lr * weight_decay))
    mf = rbf(fma32(np.float32(1 - beta1), gf - mf, mf))
    vf = rbf(vf * np.float32(beta2))
    vf = rbf(fma32(np.float32(1 - beta2) * gf, gf, vf))
    bc1 = 1 - beta1 ** step
    bc2 = 1 - beta2 ** step
    step_size = lr / bc1
    d = rbf(np.sqrt(vf))
    d = rbf(d / np.float32(math.sqrt(bc2)))
    d = rbf(d + np.float32(eps))
    r = pf + (np.float32(-step_size) * mf) / d
    pb = copy_stochastic(r, rand16) if rand16 is not None else f32_to_bf16_bits(r)
    return pb, f32_to_bf16_bits(mf), f32_to_bf16_bits(vf)


def adamw_step_f32(p, g, m, v, step, lr, beta1=0.9, beta2=0.999, eps=1e-8, weight_decay=1e-2, clip_coef=None):
    p, g, m, v = (np.asarray(a, np.float32) for a in (p, g, m, v))
    if clip_coef is not None:
        g = g * np.float32(clip_coef)
    p = p * np.float32(1 - lr * weight_decay)
    m = fma32(np.float32(1 - beta1), g - m, m)
    v = v * np.float32(beta2)
    v = fma32(np.float32(1 - beta2) * g, g, v)
    bc1 = 1 - beta1 ** step
    bc2 = 1 - beta2 ** step
    d = np.sqrt(v) / np.float32(math.sqrt(bc2)) + np.float32(eps)
    p = p + (np.float32(-lr / bc1) * m) / d
    return p.astype(np.float32), m.astype(np.float32), v.astype(np.float32)


def adamw_step_master(p, g_bits, m, v, step, lr, beta1=0.9, beta2=0.999, eps=1e-8, weight_decay=1e-2, clip_coef=None):
    """fp32 master weights under a bf16 autocast (weight_dtype FLOAT_32, TrainConfig.py:782): the fp32 step on the
    fp32 value of a bf16 gradient; returns (p, m, v) fp32 and the bits of the bf16 working copy rne(p) (autocast's
    cast of the weight at the next forward)."""
    p, m, v = adamw_step_f32(p, bf16_to_f32(g_bits), m, v, step, lr, beta1, beta2, eps, weight_decay, clip_coef)
    return p, m, v, f32_to_bf16_bits(p)


def clip_grad_norm_f32(grads: list[np.ndarray], max_norm=1.0):
    """torch clip_grad_norm_ on fp32 grads: per-tensor fp32 norms, their fp32 2-norm, coef = max_norm / (total + 1e-6)
    clamped to 1, in fp32.  (torch sums in fp32 with its own order; the sums here are fp64, rounded once.)"""
    norms = np.array([np.float32(np.sqrt(np.sum(np.asarray(g, np.float64) ** 2))) for g in grads], np.float32)
    total = np.float32(np.sqrt(np.sum(norms.astype(np.float64) ** 2)))
    coef = np.float32(min(np.float32(max_norm) / (total + np.float32(1e-6)), np.float32(1.0)))
    return float(total), coef


def clip_grad_norm_bf16(grads_bits: list[np.ndarray], max_norm=1.0):
    """torch clip_grad_norm_ on bf16 grads: per-tensor norms (bf16), total (bf16), coef (bf16).
    Returns (clipped grads bits, total norm, coef)."""
    norms = [rbf(np.float32(np.sqrt(np.sum(bf16_to_f32(g).astype(np.float64) ** 2)))) for g in grads_bits]
    total = rbf(np.float32(np.sqrt(np.sum(np.array(norms, np.float64) ** 2))))
    coef = rbf(np.float32(max_norm) / rbf(total + np.float32(1e-6)))
    coef = np.float32(min(coef, 1.0))
    out = [f32_to_bf16_bits(bf16_to_f32(g) * coef) for g in grads_bits]
    return out, float(total), float(coef)
