"""Train-mode Conv1d(k=1) + BatchNorm1d [+ ReLU] blocks on the HIP kernels of
include/ndnet_train.h (csrc/train_kernels.hip), as torch autograd Functions.

The reference's training step (tools/train.py:67-81) runs every per-point
block of NDTNetSegmentation -- ndnet/models/ndtnet.py:48-50 (TNet convs),
:148-152 (NDTNet convs), :233-239 (segmentation head) -- as torch
Conv1d -> BatchNorm1d (batch statistics) -> ReLU, and autograd runs their
backward.  ``conv_bn_act`` is that block with the same arguments, results
(fp32, within summation order) and side effects (running statistics updated
with the module's momentum and the unbiased variance, ``num_batches_tracked``
incremented), computed by:

  forward   ndnet_tr_gemm (y = W x + b)  ->  ndnet_tr_bn_fwd
  backward  ndnet_tr_bn_bwd (ReLU mask, BN backward, conv bias gradient)
            -> ndnet_tr_gemm (dx = W^T dy)  +  ndnet_tr_gemm (split-K partials
            of dW = sum dy x^T)  ->  ndnet_tr_sum_parts

Everything launches on torch's current stream and allocates through torch,
so a training step that uses these blocks is capturable as one HIP graph
(ndnet.training.GraphedTrainStep).  No fallback: the library must load.
"""
from __future__ import annotations

from typing import Optional

import torch

from .. import _lib

# split-K of the weight gradient: aim for this many workgroups per launch, with
# at most this many partial products (the partials are written, then re-read
# by ndnet_tr_sum_parts: round 3 measured 1024 / 256+ parts at 130 MB a step)
_DW_TARGET_WGS = 1024
_DW_MAX_PARTS = 32
_KSTEP = 16  # the GEMM's k-step


def _ptr(t: Optional[torch.Tensor]):
    return None if t is None else t.data_ptr()


def _stream() -> int:
    return torch.cuda.current_stream().cuda_stream


def _batches_tracked(bn) -> Optional[torch.Tensor]:
    """The module's num_batches_tracked when the BatchNorm kernel can increment
    it in its own launch (a one-element int64 device tensor), else None."""
    t = getattr(bn, "num_batches_tracked", None)
    if t is not None and t.is_cuda and t.dtype == torch.int64 and t.numel() == 1 and t.is_contiguous():
        return t
    return None


def _check_f32(*ts: torch.Tensor) -> None:
    for t in ts:
        if t.dtype != torch.float32 or not t.is_cuda or not t.is_contiguous():
            raise ValueError("train kernels take contiguous float32 cuda tensors")


def gemm(A, B, C, bias, M, N, K, lda, ldb, ldc, sAz, sBz, sCz, batch, a_kmajor, b_kmajor,
         nchunks: int = 1, kchunk: Optional[int] = None, sbias: int = 0, clouds_per_part: int = 1) -> None:
    """ndnet_tr_gemm (include/ndnet_train.h): C[z] = sum over the part's clouds
    of A[c] B[c] (+ bias)."""
    rc = _lib.lib().ndnet_tr_gemm(_ptr(A), _ptr(B), _ptr(C), _ptr(bias), sbias, M, N, K, lda, ldb, ldc, sAz, sBz, sCz,
                                  batch, clouds_per_part, int(a_kmajor), int(b_kmajor), nchunks,
                                  K if kchunk is None else kchunk, _stream())
    _lib.check(rc, "ndnet_tr_gemm")


def conv_forward(x: torch.Tensor, w: torch.Tensor, b: Optional[torch.Tensor],
                 per_cloud_bias: bool = False) -> torch.Tensor:
    """y[b] = W x[b] + bias (bias [Cout], or [B,Cout] per cloud): x [B,Cin,N],
    W [Cout,Cin] -> [B,Cout,N]."""
    Bn, Cin, N = x.shape
    Cout = w.shape[0]
    y = torch.empty(Bn, Cout, N, device=x.device, dtype=torch.float32)
    gemm(w, x, y, b, Cout, N, Cin, Cin, N, N, 0, Cin * N, Cout * N, Bn, True, False,
         sbias=Cout if per_cloud_bias else 0)
    return y


def conv_input_grad(dy: torch.Tensor, w: torch.Tensor) -> torch.Tensor:
    """dx[b] = W^T dy[b]: dy [B,Cout,N] -> [B,Cin,N]."""
    Bn, Cout, N = dy.shape
    Cin = w.shape[1]
    dx = torch.empty(Bn, Cin, N, device=dy.device, dtype=torch.float32)
    gemm(w, dy, dx, None, Cin, N, Cout, Cin, N, N, 0, Cout * N, Cin * N, Bn, False, False)
    return dx


def dw_split(Bn: int, Cout: int, Cin: int, N: int):
    """(clouds_per_part, nchunks, kchunk) of the weight gradient's split-K:
    about _DW_TARGET_WGS workgroups but at most _DW_MAX_PARTS partial
    products (each part then sums >= 1/32 of the batch's points) -- several
    clouds per part when the output has many tiles, several point chunks per
    cloud when it has few."""
    tiles = -(-Cout // 64) * -(-Cin // 64)
    parts = max(1, min(_DW_MAX_PARTS, -(-_DW_TARGET_WGS // tiles), Bn * -(-N // 64)))
    if parts <= Bn:
        return -(-Bn // parts), 1, N
    want = max(1, parts // Bn)  # point chunks per cloud: B * want <= parts
    kchunk = -(-N // want)
    kchunk = -(-kchunk // _KSTEP) * _KSTEP
    return 1, -(-N // kchunk), kchunk


def conv_weight_grad(dy: torch.Tensor, x: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """dW = sum over clouds and points of dy x^T: [Cout,Cin], into ``out``
    when given (a [Cout,Cin] view with unit column stride: rows of any stride,
    e.g. the first columns of a wider weight's gradient)."""
    Bn, Cout, N = dy.shape
    Cin = x.shape[1]
    cpz, nch, kchunk = dw_split(Bn, Cout, Cin, N)
    parts = -(-Bn // cpz) * nch
    dw = torch.empty(Cout, Cin, device=dy.device, dtype=torch.float32) if out is None else out
    if dw.shape != (Cout, Cin) or dw.stride(1) != 1:
        raise ValueError("conv_weight_grad: out must be [Cout, Cin] with unit column stride")
    ldo = dw.stride(0)
    if parts == 1:
        gemm(dy, x, dw, None, Cout, Cin, N, N, N, ldo, Cout * N, Cin * N, Cout * ldo, Bn, True, True, nch, kchunk,
             clouds_per_part=cpz)
        return dw
    tmp = torch.empty(parts, Cout, Cin, device=dy.device, dtype=torch.float32)
    gemm(dy, x, tmp, None, Cout, Cin, N, N, N, Cin, Cout * N, Cin * N, Cout * Cin, Bn, True, True, nch, kchunk,
         clouds_per_part=cpz)
    _lib.check(_lib.lib().ndnet_tr_sum_parts_2d(tmp.data_ptr(), dw.data_ptr(), Cout, Cin, ldo, parts, _stream()),
               "ndnet_tr_sum_parts_2d")
    return dw


def row_sum(x: torch.Tensor) -> torch.Tensor:
    """[B,C,N] -> [B,C]: the sum over points (a per-cloud bias gradient)."""
    Bn, C, N = x.shape
    out = torch.empty(Bn, C, device=x.device, dtype=torch.float32)
    _lib.check(_lib.lib().ndnet_tr_row_sum(x.data_ptr(), out.data_ptr(), Bn * C, N, _stream()), "ndnet_tr_row_sum")
    return out


def chan_sum(x: torch.Tensor) -> torch.Tensor:
    Bn, C, N = x.shape
    out = torch.empty(C, device=x.device, dtype=torch.float32)
    _lib.check(_lib.lib().ndnet_tr_chan_sum(x.data_ptr(), out.data_ptr(), Bn, C, N, _stream()), "ndnet_tr_chan_sum")
    return out


class _ConvBNAct(torch.autograd.Function):
    """Conv1d(k=1) [-> BatchNorm1d (batch statistics)] [-> ReLU]; the bias is
    either the conv's ``b`` [Cout] or a per-cloud ``cb`` [B,Cout]."""

    @staticmethod
    def forward(ctx, x, w, b, cb, gamma, beta, run_mean, run_var, eps, momentum, relu, nbt=None):
        x = x.contiguous()
        w2 = w.detach().reshape(w.shape[0], -1).contiguous()
        _check_f32(x, w2)
        Bn, Cin, N = x.shape
        if w2.shape[1] != Cin:
            raise ValueError(f"conv expects {w2.shape[1]} input channels, got {Cin}")
        if cb is not None:
            if b is not None or tuple(cb.shape) != (Bn, w2.shape[0]):
                raise ValueError("a per-cloud bias [B,Cout] replaces the conv bias")
            bias = cb.detach().contiguous()
        else:
            bias = None if b is None else b.detach().contiguous()
        y = conv_forward(x, w2, bias, per_cloud_bias=cb is not None)
        ctx.w_shape, ctx.has_bias, ctx.bn, ctx.relu = w.shape, b is not None, gamma is not None, bool(relu)
        ctx.has_cb = cb is not None
        if gamma is None:
            if relu:
                raise ValueError("ReLU without BatchNorm is not a block of this model")
            ctx.save_for_backward(x, w2)
            return y
        C = y.shape[1]
        z = torch.empty_like(y)
        mean = torch.empty(C, device=y.device, dtype=torch.float32)
        invstd = torch.empty_like(mean)
        g, bt = gamma.detach().contiguous(), beta.detach().contiguous()
        rc = _lib.lib().ndnet_tr_bn_fwd(y.data_ptr(), z.data_ptr(), mean.data_ptr(), invstd.data_ptr(),
                                        _ptr(run_mean), _ptr(run_var), g.data_ptr(), bt.data_ptr(), Bn, C, N,
                                        float(eps), float(momentum), int(relu), None, None, _ptr(nbt), _stream())
        _lib.check(rc, "ndnet_tr_bn_fwd")
        ctx.save_for_backward(x, w2, y, mean, invstd, g, bt)
        return z

    @staticmethod
    def backward(ctx, dz):
        dz = dz.contiguous()
        need = ctx.needs_input_grad
        dgamma = dbeta = None
        if ctx.bn:
            x, w2, y, mean, invstd, g, bt = ctx.saved_tensors
            Bn, C, N = y.shape
            dy = torch.empty_like(y)
            dgamma = torch.empty(C, device=y.device, dtype=torch.float32)
            dbeta = torch.empty_like(dgamma)
            dbias = torch.empty_like(dgamma)
            rc = _lib.lib().ndnet_tr_bn_bwd(dz.data_ptr(), y.data_ptr(), mean.data_ptr(), invstd.data_ptr(),
                                            g.data_ptr(), bt.data_ptr(), dy.data_ptr(), dgamma.data_ptr(),
                                            dbeta.data_ptr(), dbias.data_ptr(), Bn, C, N, int(ctx.relu), None,
                                            _stream())
            _lib.check(rc, "ndnet_tr_bn_bwd")
        else:
            x, w2 = ctx.saved_tensors
            dy = dz
            dbias = chan_sum(dy) if ctx.has_bias and need[2] else None
        if ctx.bn and not ctx.has_bias:
            dbias = None
        dx = conv_input_grad(dy, w2) if need[0] else None
        dw = conv_weight_grad(dy, x).view(ctx.w_shape) if need[1] else None
        dcb = row_sum(dy) if ctx.has_cb and need[3] else None
        return (dx, dw, dbias if ctx.has_bias and need[2] else None, dcb,
                dgamma if need[4] else None, dbeta if need[5] else None, None, None, None, None, None, None)


def conv_bn_act(conv: torch.nn.Conv1d, bn: Optional[torch.nn.BatchNorm1d], x: torch.Tensor,
                relu: bool, weight: Optional[torch.Tensor] = None,
                cloud_bias: Optional[torch.Tensor] = None) -> torch.Tensor:
    """``relu(bn(conv(x)))`` (or without relu / bn) in training mode on the HIP
    kernels; x [B,Cin,N] float32 on the GPU.  ``weight`` (a view of
    conv.weight, e.g. its first Cin input channels) and ``cloud_bias`` [B,Cout]
    (replacing conv.bias) run the block on part of a concatenated input whose
    rest is constant over the points (the segmentation head)."""
    if conv.kernel_size != (1,) or conv.groups != 1 or conv.stride != (1,) or conv.padding != (0,):
        raise ValueError("only pointwise Conv1d(k=1) blocks run on the train kernels")
    w = conv.weight if weight is None else weight
    b = conv.bias if cloud_bias is None else None
    if bn is None:
        return _ConvBNAct.apply(x, w, b, cloud_bias, None, None, None, None, 0.0, 0.0, False)
    if not bn.affine or bn.momentum is None:
        raise ValueError("the train kernels take affine BatchNorm1d with a fixed momentum (the model's defaults)")
    track = bn.track_running_stats and bn.running_mean is not None
    nbt = _batches_tracked(bn) if track else None
    out = _ConvBNAct.apply(x, w, b, cloud_bias, bn.weight, bn.bias,
                           bn.running_mean if track else None, bn.running_var if track else None,
                           bn.eps, bn.momentum, relu, nbt)
    if track and nbt is None:
        bn.num_batches_tracked.add_(1)
    return out


def _seg_fc_ok(g: torch.Tensor, W: torch.Tensor, c: int) -> bool:
    """The seg head's per-cloud bias GEMMs fit the FC kernels (ndnet_tr_fc_*,
    include/ndnet_train.h): <= 16 clouds, F % 4 == 0, g staged whole in LDS,
    16-byte aligned rows of W[:, c:] (row stride Ct) and g."""
    Bn, F = g.shape
    Ct = W.shape[1]
    return (Bn <= FC_MAX_ROWS and F % 4 == 0 and Bn * F <= 16384 and Ct % 4 == 0 and c % 4 == 0
            and W.stride(1) == 1 and W.stride(0) == Ct and W.data_ptr() % 16 == 0
            and g.is_contiguous() and g.data_ptr() % 16 == 0)


def _seg_bias(g: torch.Tensor, W: torch.Tensor, b: torch.Tensor, c: int) -> torch.Tensor:
    """cb = b + g W[:, c:]^T [B,Cout]: one FC-kernel launch reading the weight's
    columns c.. in place (torch's addmm on the strided slice: ~8 us)."""
    if not _seg_fc_ok(g, W, c):
        return torch.addmm(b, g, W[:, c:].t())
    Bn, F = g.shape
    Cout, Ct = W.shape
    cb = torch.empty(Bn, Cout, device=g.device, dtype=torch.float32)
    b = b.contiguous()
    rc = _lib.lib().ndnet_tr_fc_fwd(g.data_ptr(), W[:, c:].data_ptr(), b.data_ptr(), None, cb.data_ptr(), None, None,
                                    None, None, None, None, Bn, F, Cout, Ct, 0.0, 0.0, 0, 0, None, _stream())
    _lib.check(rc, "ndnet_tr_fc_fwd (seg bias)")
    return cb


class _SegConv1(torch.autograd.Function):
    """The segmentation head's first block (ndtnet.py:230-234): relu(bn(conv1(
    cat(x_t2, g broadcast over the points)))) as a conv over x_t2's c channels
    with the per-cloud bias cb = b + W[:, c:] g.  The whole weight W [Cout,
    c + F, 1] is one operand: the conv reads its first c columns in place (row
    stride c + F) and the backward returns the whole dW, so no slice of the
    weight is copied forward and no zero-filled gradient is summed backward."""

    @staticmethod
    def forward(ctx, x, g, w, b, gamma, beta, run_mean, run_var, eps, momentum, nbt):
        x, g = x.contiguous(), g.contiguous()
        W = w.detach().reshape(w.shape[0], -1)
        _check_f32(x, g, W)
        Bn, c, N = x.shape
        Cout, Ct = W.shape
        if Ct != c + g.shape[1]:
            raise ValueError(f"conv1 expects {Ct} input channels, got {c} + {g.shape[1]}")
        cb = _seg_bias(g, W, b.detach(), c)                         # [B,Cout]: b + W[:, c:] g
        y = torch.empty(Bn, Cout, N, device=x.device, dtype=torch.float32)
        gemm(W, x, y, cb, Cout, N, c, Ct, N, N, 0, c * N, Cout * N, Bn, True, False, sbias=Cout)
        z = torch.empty_like(y)
        mean = torch.empty(Cout, device=y.device, dtype=torch.float32)
        invstd = torch.empty_like(mean)
        gm, bt = gamma.detach().contiguous(), beta.detach().contiguous()
        rc = _lib.lib().ndnet_tr_bn_fwd(y.data_ptr(), z.data_ptr(), mean.data_ptr(), invstd.data_ptr(),
                                        _ptr(run_mean), _ptr(run_var), gm.data_ptr(), bt.data_ptr(), Bn, Cout, N,
                                        float(eps), float(momentum), 1, None, None, _ptr(nbt), _stream())
        _lib.check(rc, "ndnet_tr_bn_fwd")
        ctx.w_shape = w.shape
        ctx.save_for_backward(x, g, W, y, mean, invstd, gm, bt)
        return z

    @staticmethod
    def backward(ctx, dz):
        x, g, W, y, mean, invstd, gm, bt = ctx.saved_tensors
        dz = dz.contiguous()
        need = ctx.needs_input_grad
        Bn, Cout, N = y.shape
        c, Ct = x.shape[1], W.shape[1]
        dy = torch.empty_like(y)
        dgamma = torch.empty(Cout, device=y.device, dtype=torch.float32)
        dbeta, dbias = torch.empty_like(dgamma), torch.empty_like(dgamma)
        rc = _lib.lib().ndnet_tr_bn_bwd(dz.data_ptr(), y.data_ptr(), mean.data_ptr(), invstd.data_ptr(),
                                        gm.data_ptr(), bt.data_ptr(), dy.data_ptr(), dgamma.data_ptr(),
                                        dbeta.data_ptr(), dbias.data_ptr(), Bn, Cout, N, 1, None, _stream())
        _lib.check(rc, "ndnet_tr_bn_bwd")
        dx = None
        if need[0]:  # W[:, :c]^T dy, the weight read in place
            dx = torch.empty(Bn, c, N, device=dy.device, dtype=torch.float32)
            gemm(W, dy, dx, None, c, N, Cout, Ct, N, N, 0, Cout * N, c * N, Bn, False, False)
        dcb = row_sum(dy)                                            # [B,Cout]: the per-cloud bias gradient
        dW = None
        fc = _seg_fc_ok(g, W, c)
        if need[2]:
            dW = torch.empty(Cout, Ct, device=dy.device, dtype=torch.float32)
            conv_weight_grad(dy, x, out=dW[:, :c])
            if fc:  # dW[:, c:] = dcb^T g on the FC kernel, rows of stride Ct written in place
                rc = _lib.lib().ndnet_tr_fc_bwd_w(dcb.data_ptr(), g.data_ptr(), None, None, None, None, None, None,
                                                  dW[:, c:].data_ptr(), None, None, None, Bn, Ct - c, Cout, Ct, 0,
                                                  _stream())
                _lib.check(rc, "ndnet_tr_fc_bwd_w (seg bias)")
            else:
                torch.mm(dcb.t(), g, out=dW[:, c:])
            dW = dW.view(ctx.w_shape)
        db = dbias if need[3] else None  # sum over clouds and points of dy (bn_bwd's conv-bias output)
        dg = None
        if need[1]:
            if fc:  # dg = dcb W[:, c:], the weight read in place
                F = Ct - c
                dg = torch.empty(Bn, F, device=dy.device, dtype=torch.float32)
                ns = _fc_splits(Cout)
                part = torch.empty(ns, Bn, F, device=dy.device, dtype=torch.float32) if ns > 1 else None
                rc = _lib.lib().ndnet_tr_fc_bwd_x(dcb.data_ptr(), W[:, c:].data_ptr(), dg.data_ptr(), _ptr(part), Bn,
                                                  F, Cout, Ct, ns, _stream())
                _lib.check(rc, "ndnet_tr_fc_bwd_x (seg bias)")
            else:
                dg = torch.mm(dcb, W[:, c:])
        return (dx, dg, dW, db, dgamma if need[4] else None, dbeta if need[5] else None,
                None, None, None, None, None)


def seg_conv1(conv: torch.nn.Conv1d, bn: torch.nn.BatchNorm1d, x_t2: torch.Tensor, g: torch.Tensor) -> torch.Tensor:
    """``relu(bn(conv(cat(x_t2, g[:, :, None].expand(-1, -1, N)))))`` in
    training mode (the segmentation head's first block, ndtnet.py:230-234):
    x_t2 [B,c,N], the pooled global feature g [B,F]."""
    if conv.kernel_size != (1,) or conv.groups != 1 or conv.bias is None or not bn.affine or bn.momentum is None:
        raise ValueError("seg_conv1 takes the model's pointwise conv1 with bias and affine bn1")
    track = bn.track_running_stats and bn.running_mean is not None
    nbt = _batches_tracked(bn) if track else None
    out = _SegConv1.apply(x_t2, g, conv.weight, conv.bias, bn.weight, bn.bias,
                          bn.running_mean if track else None, bn.running_var if track else None,
                          bn.eps, bn.momentum, nbt)
    if track and nbt is None:
        bn.num_batches_tracked.add_(1)
    return out


class _ConvBNPool(torch.autograd.Function):
    """``amax(relu(bn(conv(x))), dim=2)`` -> [B,C] without the [B,C,N]
    activation: the BatchNorm kernel's pool mode keeps each cloud's first
    maximum and its point; the backward sends the pooled gradient to that
    point only.  That is the index routing of the reference's
    ``torch.max(x, 2)`` (ndtnet.py:50, :224), not the even split of this
    package's torch composition (``amax``): distinct points whose activations
    round to the same fp32 maximum get different weight gradients from the
    two (identical points give the same gradients either way)."""

    @staticmethod
    def forward(ctx, x, w, b, gamma, beta, run_mean, run_var, eps, momentum, relu, nbt=None):
        x = x.contiguous()
        w2 = w.detach().reshape(w.shape[0], -1).contiguous()
        _check_f32(x, w2)
        Bn, Cin, N = x.shape
        if w2.shape[1] != Cin:
            raise ValueError(f"conv expects {w2.shape[1]} input channels, got {Cin}")
        y = conv_forward(x, w2, b.detach().contiguous())
        C = y.shape[1]
        pool = torch.empty(Bn, C, device=y.device, dtype=torch.float32)
        idx = torch.empty(Bn, C, device=y.device, dtype=torch.int32)
        mean = torch.empty(C, device=y.device, dtype=torch.float32)
        invstd = torch.empty_like(mean)
        g, bt = gamma.detach().contiguous(), beta.detach().contiguous()
        rc = _lib.lib().ndnet_tr_bn_fwd(y.data_ptr(), None, mean.data_ptr(), invstd.data_ptr(),
                                        _ptr(run_mean), _ptr(run_var), g.data_ptr(), bt.data_ptr(), Bn, C, N,
                                        float(eps), float(momentum), int(relu), pool.data_ptr(), idx.data_ptr(),
                                        _ptr(nbt), _stream())
        _lib.check(rc, "ndnet_tr_bn_fwd (pool)")
        ctx.relu, ctx.w_shape = bool(relu), w.shape
        ctx.save_for_backward(x, w2, y, mean, invstd, g, bt, idx)
        return pool

    @staticmethod
    def backward(ctx, dpool):
        dpool = dpool.contiguous()
        need = ctx.needs_input_grad
        x, w2, y, mean, invstd, g, bt, idx = ctx.saved_tensors
        Bn, C, N = y.shape
        dy = torch.empty_like(y)
        dgamma = torch.empty(C, device=y.device, dtype=torch.float32)
        dbeta = torch.empty_like(dgamma)
        dbias = torch.empty_like(dgamma)
        rc = _lib.lib().ndnet_tr_bn_bwd(dpool.data_ptr(), y.data_ptr(), mean.data_ptr(), invstd.data_ptr(),
                                        g.data_ptr(), bt.data_ptr(), dy.data_ptr(), dgamma.data_ptr(),
                                        dbeta.data_ptr(), dbias.data_ptr(), Bn, C, N, int(ctx.relu), idx.data_ptr(),
                                        _stream())
        _lib.check(rc, "ndnet_tr_bn_bwd (pool)")
        dx = conv_input_grad(dy, w2) if need[0] else None
        dw = conv_weight_grad(dy, x).view(ctx.w_shape) if need[1] else None
        return (dx, dw, dbias if need[2] else None, dgamma if need[3] else None, dbeta if need[4] else None,
                None, None, None, None, None, None)


def conv_bn_act_pool(conv: torch.nn.Conv1d, bn: torch.nn.BatchNorm1d, x: torch.Tensor,
                     relu: bool) -> torch.Tensor:
    """``relu(bn(conv(x))).amax(dim=2)`` in training mode on the HIP kernels:
    x [B,Cin,N] -> [B,Cout] (B <= 64 clouds)."""
    if conv.kernel_size != (1,) or conv.groups != 1 or conv.stride != (1,) or conv.padding != (0,):
        raise ValueError("only pointwise Conv1d(k=1) blocks run on the train kernels")
    if conv.bias is None or not bn.affine or bn.momentum is None:
        raise ValueError("the pooled block takes a biased conv and affine BatchNorm1d with a fixed momentum")
    track = bn.track_running_stats and bn.running_mean is not None
    nbt = _batches_tracked(bn) if track else None
    out = _ConvBNPool.apply(x, conv.weight, conv.bias, bn.weight, bn.bias,
                            bn.running_mean if track else None, bn.running_var if track else None,
                            bn.eps, bn.momentum, relu, nbt)
    if track and nbt is None:
        bn.num_batches_tracked.add_(1)
    return out



# ---- TNet FC heads (ndtnet.py:53-60) and the x^T t2 product (:153-155) ----

FC_MAX_ROWS = 16  # clouds per batch the FC kernels take (include/ndnet_train.h ndnet_tr_fc_fwd)


def _fc_splits(N: int) -> int:
    """Channel splits of the input-gradient kernel: about 128 workgroups over
    the k blocks, at most 256 channels (the kernel's LDS stage) per split."""
    return max(-(-N // 256), min(N, 32))


class _FcBNAct(torch.autograd.Function):
    """Linear [-> BatchNorm1d over the batch rows -> ReLU] (or + identity, fc3),
    on x [B,K] with B <= 16 (ndnet_tr_fc_fwd / _bwd_w / _bwd_x)."""

    @staticmethod
    def forward(ctx, x, w, b, gamma, beta, run_mean, run_var, eps, momentum, relu, eye, nbt=None):
        x = x.contiguous()
        w2 = w.detach().contiguous()
        _check_f32(x, w2)
        Bn, K = x.shape
        N = w2.shape[0]
        z = torch.empty(Bn, N, device=x.device, dtype=torch.float32)
        bn = gamma is not None
        y = torch.empty_like(z) if bn else None
        mean = torch.empty(N, device=x.device, dtype=torch.float32) if bn else None
        invstd = torch.empty_like(mean) if bn else None
        g = gamma.detach().contiguous() if bn else None
        bt = beta.detach().contiguous() if bn else None
        rc = _lib.lib().ndnet_tr_fc_fwd(x.data_ptr(), w2.data_ptr(), b.detach().contiguous().data_ptr(), _ptr(y),
                                        z.data_ptr(), _ptr(mean), _ptr(invstd), _ptr(run_mean), _ptr(run_var),
                                        _ptr(g), _ptr(bt), Bn, K, N, 0, float(eps), float(momentum), int(relu),
                                        int(eye), _ptr(nbt), _stream())
        _lib.check(rc, "ndnet_tr_fc_fwd")
        ctx.relu, ctx.bn = bool(relu), bn
        ctx.save_for_backward(x, w2, y, mean, invstd, g, bt)
        return z

    @staticmethod
    def backward(ctx, dz):
        dz = dz.contiguous()
        need = ctx.needs_input_grad
        x, w2, y, mean, invstd, g, bt = ctx.saved_tensors
        Bn, K = x.shape
        N = w2.shape[0]
        dev = x.device
        dpre = torch.empty(Bn, N, device=dev, dtype=torch.float32)
        dw = torch.empty(N, K, device=dev, dtype=torch.float32) if need[1] else None
        db = torch.empty(N, device=dev, dtype=torch.float32) if need[2] else None
        dgamma = torch.empty(N, device=dev, dtype=torch.float32) if ctx.bn and need[3] else None
        dbeta = torch.empty(N, device=dev, dtype=torch.float32) if ctx.bn and need[4] else None
        rc = _lib.lib().ndnet_tr_fc_bwd_w(dz.data_ptr(), x.data_ptr(), _ptr(y), _ptr(mean), _ptr(invstd), _ptr(g),
                                          _ptr(bt), dpre.data_ptr(), _ptr(dw), _ptr(db), _ptr(dgamma), _ptr(dbeta),
                                          Bn, K, N, 0, int(ctx.relu), _stream())
        _lib.check(rc, "ndnet_tr_fc_bwd_w")
        dx = None
        if need[0]:
            dx = torch.empty(Bn, K, device=dev, dtype=torch.float32)
            ns = _fc_splits(N)
            part = torch.empty(ns, Bn, K, device=dev, dtype=torch.float32) if ns > 1 else None
            rc = _lib.lib().ndnet_tr_fc_bwd_x(dpre.data_ptr(), w2.data_ptr(), dx.data_ptr(), _ptr(part), Bn, K, N, 0,
                                              ns, _stream())
            _lib.check(rc, "ndnet_tr_fc_bwd_x")
        return dx, dw, db, dgamma, dbeta, None, None, None, None, None, None, None


def fc_bn_act(fc: torch.nn.Linear, bn: Optional[torch.nn.BatchNorm1d], x: torch.Tensor, relu: bool,
              eye: int = 0) -> torch.Tensor:
    """``relu(bn(fc(x)))`` in training mode on the HIP kernels (x [B,K], B <= 16;
    the TNet heads' fc1 / fc2), or ``fc(x) + eye(eye).flatten()`` without
    ``bn`` (fc3, ndtnet.py:57-59).  Same results (fp32, within summation
    order) and side effects (running statistics, num_batches_tracked) as the
    torch modules."""
    if bn is None:
        return _FcBNAct.apply(x, fc.weight, fc.bias, None, None, None, None, 0.0, 0.0, False, eye)
    if not bn.affine or bn.momentum is None:
        raise ValueError("the FC kernels take affine BatchNorm1d with a fixed momentum (the model's defaults)")
    track = bn.track_running_stats and bn.running_mean is not None
    nbt = _batches_tracked(bn) if track else None
    out = _FcBNAct.apply(x, fc.weight, fc.bias, bn.weight, bn.bias, bn.running_mean if track else None,
                         bn.running_var if track else None, bn.eps, bn.momentum, relu, 0, nbt)
    if track and nbt is None:
        bn.num_batches_tracked.add_(1)
    return out


class _TransformT(torch.autograd.Function):
    """x_t2 = (x^T t2)^T per cloud (ndtnet.py:153-155) on ndnet_tr_gemm: x
    [B,C,N] (NCL), t [B,C,C] -> [B,C,N] with x_t2[b] = t[b]^T x[b]."""

    @staticmethod
    def forward(ctx, x, t):
        x, t = x.contiguous(), t.contiguous()
        _check_f32(x, t)
        Bn, C, N = x.shape
        y = torch.empty_like(x)
        # A(m, k) = t[b][k][m] (not k-major, lda C), B(k, n) = x[b][k][n]
        gemm(t, x, y, None, C, N, C, C, N, N, C * C, C * N, C * N, Bn, False, False)
        ctx.save_for_backward(x, t)
        return y

    @staticmethod
    def backward(ctx, dy):
        dy = dy.contiguous()
        x, t = ctx.saved_tensors
        Bn, C, N = x.shape
        dx = dt = None
        if ctx.needs_input_grad[0]:
            dx = torch.empty_like(x)  # dx[b] = t[b] dy[b]: A(m, k) = t[b][m][k] (k-major)
            gemm(t, dy, dx, None, C, N, C, C, N, N, C * C, C * N, C * N, Bn, True, False)
        if ctx.needs_input_grad[1]:
            # dt[b][i][j] = sum_p x[b][i][p] dy[b][j][p]: A = x[b] (k-major, lda N), B(k, n) = dy[b][n][k] (k-major)
            dt = torch.empty_like(t)
            gemm(x, dy, dt, None, C, C, N, N, N, C, C * N, C * N, C * C, Bn, True, True)
        return dx, dt


def transform_t(x: torch.Tensor, t: torch.Tensor) -> torch.Tensor:
    """``torch.bmm(x.transpose(1, 2), t).transpose(1, 2)`` for x [B,C,N], t [B,C,C]."""
    return _TransformT.apply(x, t)


class _PointTransform(torch.autograd.Function):
    """x [B,12,N] = (t . p, t . C) of the point transform t1 (ndtnet.py:141-147);
    the gradient reaches t only (ndnet_tr_point_transform / _bwd)."""

    @staticmethod
    def forward(ctx, t, points, extra):
        t = t.contiguous()
        points, extra = _rows(points), _rows(extra)  # views of the NDT's [B,N,12] rows are read in place
        _check_f32(t)
        Bn, N, _ = points.shape
        x = torch.empty((Bn, 12, N), device=points.device, dtype=torch.float32)
        _lib.check(_lib.lib().ndnet_tr_point_transform(t.data_ptr(), points.data_ptr(), points.stride(1),
                                                       extra.data_ptr(), extra.stride(1), x.data_ptr(), Bn, N,
                                                       _stream()), "ndnet_tr_point_transform")
        ctx.save_for_backward(points, extra)
        return x

    @staticmethod
    def backward(ctx, dx):
        points, extra = ctx.saved_tensors
        dx = dx.contiguous()
        Bn, N, _ = points.shape
        dt = torch.empty((Bn, 3, 3), device=points.device, dtype=torch.float32)
        _lib.check(_lib.lib().ndnet_tr_point_transform_bwd(dx.data_ptr(), points.data_ptr(), points.stride(1),
                                                           extra.data_ptr(), extra.stride(1), dt.data_ptr(), Bn, N,
                                                           _stream()), "ndnet_tr_point_transform_bwd")
        return dt, None, None


def _rows(a: torch.Tensor) -> torch.Tensor:
    """a [B,N,w] as the point-transform kernels read it: rows of stride
    a.stride(1) >= w floats, clouds N rows apart, unit column stride (a column
    slice of a contiguous [B,N,W] block qualifies); otherwise a contiguous copy."""
    if not (a.dtype == torch.float32 and a.is_cuda):
        raise ValueError("train kernels take float32 cuda tensors")
    Bn, N, w = a.shape
    if a.stride(2) == 1 and a.stride(1) >= w and a.stride(0) == N * a.stride(1):
        return a
    return a.contiguous()


def point_transform(t: torch.Tensor, points: torch.Tensor, extra: torch.Tensor) -> torch.Tensor:
    """The first conv's input [B,12,N] = cat(t . p, t . C) for t [B,3,3], points
    [B,N,3], extra [B,N,9] (fp32, cuda; points and extra without gradient):
    one launch each way instead of two cats, a permute and a batched GEMM."""
    assert not points.requires_grad and not extra.requires_grad
    return _PointTransform.apply(t, points, extra)


class _LogSoftmaxC(torch.autograd.Function):
    """log_softmax over dim 1 of [B,C,N] (ndtnet.py:241; ndnet_tr_log_softmax_c)."""

    @staticmethod
    def forward(ctx, x):
        x = x.contiguous()
        _check_f32(x)
        Bn, C, N = x.shape
        y = torch.empty_like(x)
        _lib.check(_lib.lib().ndnet_tr_log_softmax_c(x.data_ptr(), y.data_ptr(), Bn, C, N, _stream()),
                   "ndnet_tr_log_softmax_c")
        ctx.save_for_backward(y)
        return y

    @staticmethod
    def backward(ctx, dy):
        (y,) = ctx.saved_tensors
        dy = dy.contiguous()
        Bn, C, N = y.shape
        dx = torch.empty_like(y)
        _lib.check(_lib.lib().ndnet_tr_log_softmax_c_bwd(y.data_ptr(), dy.data_ptr(), dx.data_ptr(), Bn, C, N,
                                                         _stream()), "ndnet_tr_log_softmax_c_bwd")
        return dx


def log_softmax_c(x: torch.Tensor) -> torch.Tensor:
    """``torch.nn.functional.log_softmax(x, dim=1)`` for x [B,C,N] (fp32, cuda)
    on the HIP kernels: one launch each way instead of torch's spatial softmax."""
    return _LogSoftmaxC.apply(x)


class _NllOneHot(torch.autograd.Function):
    """-(gt * logp^T).sum(-1).mean() for logp [B,C,N] and one-hot gt [B,N,C]."""

    @staticmethod
    def forward(ctx, logp, gt):
        logp, gt = logp.contiguous(), gt.contiguous()
        _check_f32(logp, gt)
        Bn, C, N = logp.shape
        part = torch.empty(-(-(Bn * N) // 64), device=logp.device, dtype=torch.float64)
        loss = torch.empty((), device=logp.device, dtype=torch.float32)
        _lib.check(_lib.lib().ndnet_tr_nll_onehot(logp.data_ptr(), gt.data_ptr(), part.data_ptr(), loss.data_ptr(),
                                                  Bn, C, N, _stream()), "ndnet_tr_nll_onehot")
        ctx.save_for_backward(gt)
        ctx.shape = logp.shape
        return loss

    @staticmethod
    def backward(ctx, dloss):
        (gt,) = ctx.saved_tensors
        Bn, C, N = ctx.shape
        dl = dloss.contiguous().float().reshape(1)
        dlogp = torch.empty(Bn, C, N, device=gt.device, dtype=torch.float32)
        _lib.check(_lib.lib().ndnet_tr_nll_onehot_bwd(gt.data_ptr(), dl.data_ptr(), dlogp.data_ptr(), Bn, C, N,
                                                      _stream()), "ndnet_tr_nll_onehot_bwd")
        return dlogp, None


def nll_onehot(logp: torch.Tensor, gt: torch.Tensor) -> torch.Tensor:
    """The training loss of ndnet.training.segmentation_loss on the HIP kernels:
    logp [B,C,N] (the model's log-softmax before its transpose), gt [B,N,C]."""
    return _NllOneHot.apply(logp, gt)

