"""Thin torch-tensor front end over the C-ABI launchers (include/otamd.h).

Every function validates shapes/strides/dtypes on the host BEFORE launching (a bad
launch on the GPU box can fault the device), extracts raw device pointers, and
launches on torch's current HIP stream.  No function here has a fallback: a missing
library raises (onetrainer_amd/_lib.py).
"""
from __future__ import annotations

import ctypes as C

import torch

from . import _lib
from ._lib import ConvGeom, GemmArgs, check, lib

BF16 = torch.bfloat16
F32 = torch.float32

OPM_K, OPM_MN, OPM_CONV_FWD, OPM_CONV_DGRAD, OPM_CONV_WGRAD = 0, 1, 2, 3, 4


def stream_handle() -> int:
    return torch.cuda.current_stream().cuda_stream


def _p(t: torch.Tensor | None) -> int | None:
    return None if t is None else t.data_ptr()


def _req(cond: bool, msg: str):
    if not cond:
        raise ValueError(msg)


# ------------------------------------------------------------------------------------------
# workspace (split-K slabs etc.): one growing buffer per device, stream-ordered reuse
_WS: dict[int, torch.Tensor] = {}


def workspace(nbytes: int, device: torch.device) -> torch.Tensor:
    idx = device.index if device.index is not None else torch.cuda.current_device()
    ws = _WS.get(idx)
    if ws is None or ws.numel() < nbytes:
        ws = torch.empty(max(nbytes, 64 << 20), dtype=torch.uint8, device=device)
        _WS[idx] = ws
    return ws


def _gemm(a: GemmArgs, splits: int, device) -> None:
    ws_bytes = splits * a.M * a.N * 4 if splits > 1 else 0
    ws = workspace(ws_bytes, device) if splits > 1 else None
    check(lib().otamd_gemm(C.byref(a), splits, _p(ws), ws_bytes, stream_handle()), "otamd_gemm")


def _new_args() -> GemmArgs:
    a = GemmArgs()
    a.alpha = 1.0
    a.rows_per_vec = 1
    return a


def _ld_rows(t: torch.Tensor) -> int:
    _req(t.dim() == 2 and t.stride(1) == 1, "2-D row-major tensor with unit inner stride required")
    _req(t.stride(0) % 8 == 0 or t.shape[0] == 1, "row stride must be a multiple of 8 elements")
    return t.stride(0) if t.shape[0] > 1 else t.shape[1]


def _aligned(t: torch.Tensor) -> bool:
    return t.data_ptr() % 16 == 0


def pick_splits(M: int, N: int, K: int, min_k: int = 512) -> int:
    tiles = ((M + 127) // 128) * ((N + 127) // 128)
    if tiles >= 256 or K < 2 * min_k:
        return 1
    s = 1
    while tiles * s < 512 and K // (2 * s) >= min_k:
        s *= 2
    return s


def _epilogue(a: GemmArgs, bias, rowvec, rows_per_vec, residual, M, N):
    if bias is not None:
        _req(bias.dtype == BF16 and bias.numel() == N and bias.is_contiguous(), "bias: bf16 [N]")
        a.bias = _p(bias)
    if rowvec is not None:
        _req(rowvec.dtype == BF16 and rowvec.dim() == 2 and rowvec.shape[1] == N and rowvec.stride(1) == 1,
             "rowvec: bf16 [groups, N]")
        _req(rows_per_vec > 0 and (M + rows_per_vec - 1) // rows_per_vec <= rowvec.shape[0], "rowvec rows")
        a.rowvec, a.ldv, a.rows_per_vec = _p(rowvec), rowvec.stride(0), rows_per_vec
    if residual is not None:
        _req(residual.dtype == BF16 and residual.shape == (M, N) and residual.stride(1) == 1, "residual: bf16 [M,N]")
        a.residual, a.ldr = _p(residual), residual.stride(0)


def _out(out, M, N, dtype, device):
    if out is None:
        out = torch.empty((M, N), dtype=dtype, device=device)
    _req(out.shape == (M, N) and out.stride(1) == 1 and out.dtype in (BF16, F32), "out: [M,N] bf16/f32")
    _req(out.stride(0) % 4 == 0 or M == 1, "out row stride must be a multiple of 4")
    return out


def linear(x: torch.Tensor, w: torch.Tensor, bias=None, residual=None, rowvec=None, rows_per_vec=0,
           out=None, out_dtype=BF16, alpha=1.0, accumulate=False) -> torch.Tensor:
    """y[M,N] = alpha * x[M,K] @ w[N,K]^T (+bias[N]) (+rowvec[m//rows_per_vec]) (+residual)."""
    _req(x.dtype == BF16 and w.dtype == BF16 and x.is_cuda, "linear: bf16 cuda tensors")
    M, K = x.shape
    N, K2 = w.shape
    _req(K == K2 and K % 8 == 0 and N % 4 == 0, f"linear shapes {tuple(x.shape)} x {tuple(w.shape)}")
    _req(_aligned(x) and _aligned(w), "16-byte aligned operands required")
    out = _out(out, M, N, out_dtype, x.device)
    a = _new_args()
    a.A, a.lda, a.amode = _p(x), _ld_rows(x), OPM_K
    a.B, a.ldb, a.bmode = _p(w), _ld_rows(w), OPM_K
    a.C, a.ldc, a.c_f32, a.accumulate = _p(out), out.stride(0) if M > 1 else N, int(out.dtype == F32), int(accumulate)
    a.M, a.N, a.K, a.alpha = M, N, K, alpha
    _epilogue(a, bias, rowvec, rows_per_vec, residual, M, N)
    _gemm(a, 1, x.device)
    return out


def linear_dgrad(dy: torch.Tensor, w: torch.Tensor, out=None, residual=None, accumulate=False) -> torch.Tensor:
    """dx[M,K] = dy[M,N] @ w[N,K]."""
    _req(dy.dtype == BF16 and w.dtype == BF16, "linear_dgrad: bf16")
    M, N = dy.shape
    N2, K = w.shape
    _req(N == N2 and N % 8 == 0 and K % 8 == 0, "linear_dgrad shapes")
    out = _out(out, M, K, BF16 if out is None else out.dtype, dy.device)
    a = _new_args()
    a.A, a.lda, a.amode = _p(dy), _ld_rows(dy), OPM_K
    a.B, a.ldb, a.bmode = _p(w), _ld_rows(w), OPM_MN
    a.C, a.ldc, a.c_f32, a.accumulate = _p(out), out.stride(0) if M > 1 else K, int(out.dtype == F32), int(accumulate)
    a.M, a.N, a.K = M, K, N
    _epilogue(a, None, None, 0, residual, M, K)
    _gemm(a, 1, dy.device)
    return out


def linear_wgrad(dy: torch.Tensor, x: torch.Tensor, out=None, accumulate=False, splits=None) -> torch.Tensor:
    """dw[N,K] = dy[T,N]^T @ x[T,K]  (split-K over tokens T, deterministic slab reduce)."""
    _req(dy.dtype == BF16 and x.dtype == BF16, "linear_wgrad: bf16")
    T, N = dy.shape
    T2, K = x.shape
    _req(T == T2 and N % 8 == 0 and K % 8 == 0, "linear_wgrad shapes")
    out = _out(out, N, K, BF16 if out is None else out.dtype, dy.device)
    a = _new_args()
    a.A, a.lda, a.amode = _p(dy), _ld_rows(dy), OPM_MN
    a.B, a.ldb, a.bmode = _p(x), _ld_rows(x), OPM_MN
    a.C, a.ldc, a.c_f32, a.accumulate = _p(out), out.stride(0), int(out.dtype == F32), int(accumulate)
    a.M, a.N, a.K = N, K, T
    _gemm(a, splits or pick_splits(N, K, T), dy.device)
    return out


# ------------------------------------------------------------------------------------------
# convolutions, NHWC activations, weights [Cout][KH][KW][Cin]
def _geom(N, SH, SW, SC, RH, RW, KH, KW, stride, pad, upsample, ld) -> ConvGeom:
    g = ConvGeom()
    g.N, g.SH, g.SW, g.SC, g.RH, g.RW = N, SH, SW, SC, RH, RW
    g.KH, g.KW, g.stride, g.pad, g.upsample, g.ld = KH, KW, stride, pad, int(upsample), ld
    return g


def conv_out_hw(H, W, k, stride, pad, upsample=False):
    if upsample:
        H, W = 2 * H, 2 * W
    return (H + 2 * pad - k) // stride + 1, (W + 2 * pad - k) // stride + 1


def _nhwc(x: torch.Tensor):
    _req(x.dim() == 4 and x.dtype == BF16 and x.stride(3) == 1, "NHWC bf16 activation required")
    N, H, W, Cc = x.shape
    _req(x.stride(2) == x.stride(3) * Cc or x.stride(2) % 8 == 0, "pixel stride")
    _req(x.stride(1) == x.stride(2) * W and x.stride(0) == x.stride(1) * H, "NHWC pixels must be uniformly strided")
    _req(Cc % 8 == 0 and x.stride(2) % 8 == 0, "channels and pixel stride must be multiples of 8")
    return N, H, W, Cc, x.stride(2)


def conv2d(x: torch.Tensor, w: torch.Tensor, bias=None, stride=1, pad=1, upsample=False, residual=None,
           rowvec=None, out=None) -> torch.Tensor:
    """NHWC conv: y[n,p,q,co] = sum w[co,r,s,ci] * x[n, p*st+r-pad, q*st+s-pad, ci] (+bias, +rowvec[n], +residual).
    upsample=True reads x through a nearest-2x upsample (diffusers Upsample2D)."""
    N, H, W, Cin, ldx = _nhwc(x)
    Cout, KH, KW, Cin2 = w.shape
    _req(Cin2 == Cin and w.dtype == BF16 and w.is_contiguous() and Cout % 8 == 0, "conv weight [Cout,KH,KW,Cin]")
    _req(_aligned(x) and _aligned(w), "aligned operands")
    P, Q = conv_out_hw(H, W, KH, stride, pad, upsample)
    M = N * P * Q
    if out is None:
        out = torch.empty((N, P, Q, Cout), dtype=BF16, device=x.device)
    _req(out.shape == (N, P, Q, Cout) and out.is_contiguous(), "conv out")
    a = _new_args()
    a.A, a.lda, a.amode = _p(x), 8, OPM_CONV_FWD
    a.ga = _geom(N, H, W, Cin, P, Q, KH, KW, stride, pad, upsample, ldx)
    a.B, a.ldb, a.bmode = _p(w), KH * KW * Cin, OPM_K
    a.C, a.ldc = _p(out), Cout
    a.M, a.N, a.K = M, Cout, KH * KW * Cin
    res2 = residual.reshape(M, Cout) if residual is not None else None
    _epilogue(a, bias, rowvec, P * Q if rowvec is not None else 0, res2, M, Cout)
    _gemm(a, 1, x.device)
    return out


def conv2d_dgrad(dy: torch.Tensor, w_t: torch.Tensor, in_hw, stride=1, pad=1, out=None) -> torch.Tensor:
    """dx of conv2d (no upsample): dx[n,h,w,ci] = sum_{r,s,co} dy[n,(h+pad-r)/st,(w+pad-s)/st,co] * w[co,r,s,ci].
    w_t is the weight transposed to [Cin][KH][KW][Cout] (conv_weight_transpose)."""
    N, P, Q, Cout, ldy = _nhwc(dy)
    Cin, KH, KW, Cout2 = w_t.shape
    _req(Cout2 == Cout and w_t.is_contiguous() and Cin % 8 == 0, "w_t [Cin,KH,KW,Cout]")
    H, W = in_hw
    _req(conv_out_hw(H, W, KH, stride, pad) == (P, Q), "dgrad geometry")
    if out is None:
        out = torch.empty((N, H, W, Cin), dtype=BF16, device=dy.device)
    a = _new_args()
    a.A, a.lda, a.amode = _p(dy), 8, OPM_CONV_DGRAD
    a.ga = _geom(N, P, Q, Cout, H, W, KH, KW, stride, pad, False, ldy)
    a.B, a.ldb, a.bmode = _p(w_t), KH * KW * Cout, OPM_K
    a.C, a.ldc = _p(out), Cin
    a.M, a.N, a.K = N * H * W, Cin, KH * KW * Cout
    _gemm(a, 1, dy.device)
    return out


def conv2d_wgrad(dy: torch.Tensor, x: torch.Tensor, ksize=3, stride=1, pad=1, upsample=False, out=None,
                 accumulate=False, splits=None) -> torch.Tensor:
    """dw[co,r,s,ci] = sum_{n,p,q} dy[n,p,q,co] * x[n, p*st+r-pad, q*st+s-pad, ci]."""
    N, P, Q, Cout, ldy = _nhwc(dy)
    N2, H, W, Cin, ldx = _nhwc(x)
    _req(N == N2 and conv_out_hw(H, W, ksize, stride, pad, upsample) == (P, Q), "wgrad geometry")
    _req(ldy == Cout, "dy must be dense NHWC")
    if out is None:
        out = torch.empty((Cout, ksize, ksize, Cin), dtype=BF16, device=dy.device)
    _req(out.shape == (Cout, ksize, ksize, Cin) and out.is_contiguous(), "wgrad out")
    a = _new_args()
    a.A, a.lda, a.amode = _p(dy), Cout, OPM_MN
    a.B, a.ldb, a.bmode = _p(x), 8, OPM_CONV_WGRAD
    a.gb = _geom(N, H, W, Cin, P, Q, ksize, ksize, stride, pad, upsample, ldx)
    a.C, a.ldc, a.c_f32, a.accumulate = _p(out), ksize * ksize * Cin, int(out.dtype == F32), int(accumulate)
    Kg = N * P * Q
    a.M, a.N, a.K = Cout, ksize * ksize * Cin, Kg
    _gemm(a, splits or pick_splits(Cout, ksize * ksize * Cin, Kg), dy.device)
    return out


# ------------------------------------------------------------------------------------------
# optimizer
def adamw_bf16(p, g, m, v, groups, clip_coef=None, stochastic_rounding=True, seed=0):
    n = p.numel()
    for t in (p, g, m, v):
        _req(t.dtype == BF16 and t.is_contiguous() and t.numel() == n and _aligned(t), "adamw flat bf16 buffers")
    arr = (_lib.AdamwGroup * len(groups))(*groups)
    check(lib().otamd_adamw_bf16(_p(p), _p(g), _p(m), _p(v), n, arr, len(groups), _p(clip_coef),
                                 int(stochastic_rounding), seed & 0xFFFFFFFFFFFFFFFF, stream_handle()),
          "otamd_adamw_bf16")


def adamw_f32(p, g, m, v, groups, clip_coef=None):
    n = p.numel()
    for t in (p, g, m, v):
        _req(t.dtype == F32 and t.is_contiguous() and t.numel() == n and _aligned(t), "adamw flat f32 buffers")
    arr = (_lib.AdamwGroup * len(groups))(*groups)
    check(lib().otamd_adamw_f32(_p(p), _p(g), _p(m), _p(v), n, arr, len(groups), _p(clip_coef), stream_handle()),
          "otamd_adamw_f32")


def grad_clip_coef(grads, chunks_dev, n_chunks, tensor_sq, n_tensors, max_norm, out):
    _req(grads.dtype in (BF16, F32) and grads.is_contiguous(), "grads flat")
    _req(tensor_sq.dtype == torch.float64 and tensor_sq.numel() >= n_tensors, "tensor_sq f64")
    _req(out.dtype == F32 and out.numel() >= 2, "out f32[2]")
    check(lib().otamd_grad_clip_coef(_p(grads), 0 if grads.dtype == BF16 else 1, _p(chunks_dev), n_chunks,
                                     _p(tensor_sq), n_tensors, float(max_norm), _p(out), stream_handle()),
          "otamd_grad_clip_coef")
