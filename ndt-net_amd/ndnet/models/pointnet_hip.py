"""Eval-mode NDTNetSegmentation forward on the HIP point-MLP kernel.

The reference forward (ndnet/models/ndtnet.py:112-164, 218-243) is rewritten
as four fused point-MLP chains (``ndnet_pn_chain_run``, csrc/pointnet_kernels.hip)
with small per-cloud steps between them:

  A  TNet(3):   p -> 64 -> 128 -> 1024, max over points          -> g1
     FC head (1024 -> 512 -> 256 -> 9) + I                       -> t1
  B  conv1 with t1 folded in (x' = [t1 p, t1 C] is linear in x), then
     TNet(64):  -> 64 -> 64 -> 128 -> 1024, max                  -> g2
     FC head (1024 -> 512 -> 256 -> 4096) + I                    -> t2
  C  conv2 with t2^T folded in (x_t2 = t2^T x1), conv3, max      -> g3 [F]
  D  seg conv1 split: W[:, :64] t2^T x1 per point + (W[:, 64:] g3 + b) per
     cloud (the reference concatenates the broadcast g3 to every point:
     ndtnet.py:227-230), -> 512 -> 256 -> 128 -> C+1, log_softmax

Every BatchNorm (running statistics) is folded into the preceding 1x1 conv /
linear layer.  Per-point GEMMs run in FP32 on MFMA; the per-cloud steps
(FC heads, weight folding) are batched torch ops on the same stream.
"""
from __future__ import annotations

import ctypes

import torch

from .. import _lib

MAX_LAYERS = 5


class _Layer(ctypes.Structure):
    _fields_ = [("wT", ctypes.c_void_p), ("w_cloud_stride", ctypes.c_int64), ("bias", ctypes.c_void_p),
                ("bias_cloud_stride", ctypes.c_int64), ("K", ctypes.c_int32), ("N", ctypes.c_int32),
                ("relu", ctypes.c_int32), ("ldw", ctypes.c_int32)]


class _Chain(ctypes.Structure):
    _fields_ = [("x", ctypes.c_void_p), ("x_ld", ctypes.c_int32), ("in_cols", ctypes.c_int32),
                ("num_points", ctypes.c_int32), ("num_layers", ctypes.c_int32), ("L", _Layer * MAX_LAYERS),
                ("mode", ctypes.c_int32), ("out_cols", ctypes.c_int32), ("gmax", ctypes.c_void_p),
                ("gmax_ld", ctypes.c_int32), ("max_width", ctypes.c_int32), ("max_width2", ctypes.c_int32),
                ("out", ctypes.c_void_p)]


_lib.POINTNET_EXPORTS["ndnet_pn_chain_run"] = (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p])


def available() -> bool:
    try:
        return torch.cuda.is_available() and hasattr(_lib.lib(), "ndnet_pn_chain_run")
    except RuntimeError:
        return False


def _pad(n: int, m: int) -> int:
    return (n + m - 1) // m * m


def _bn_fold(w: torch.Tensor, b: torch.Tensor, bn: torch.nn.BatchNorm1d):
    """y = bn(W x + b) -> W' x + b' (eval statistics)."""
    s = bn.weight / torch.sqrt(bn.running_var + bn.eps)
    return w * s[:, None], (b - bn.running_mean) * s + bn.bias


def _wT(w: torch.Tensor, kpad: int, npad: int) -> torch.Tensor:
    """[N][K] weight -> zero-padded transposed [Kpad][Npad] fp32, contiguous."""
    n, k = w.shape
    out = torch.zeros((kpad, npad), dtype=torch.float32, device=w.device)
    out[:k, :n] = w.t()
    return out


def _bpad(b: torch.Tensor, npad: int) -> torch.Tensor:
    out = torch.zeros(npad, dtype=torch.float32, device=b.device)
    out[: b.shape[0]] = b
    return out


class _Folded:
    """BN-folded, transposed, padded weights of one model (on its device)."""

    def __init__(self, m) -> None:
        fe = m.feature_extractor
        with torch.no_grad():
            def conv(c, bn):
                return _bn_fold(c.weight[:, :, 0].float(), c.bias.float(), bn)

            def tnet(t):
                w1, b1 = conv(t.conv1, t.bn1)
                w2, b2 = conv(t.conv2, t.bn2)
                w3, b3 = conv(t.conv3, t.bn3)
                f1, c1 = _bn_fold(t.fc1.weight.float(), t.fc1.bias.float(), t.bn4)
                f2, c2 = _bn_fold(t.fc2.weight.float(), t.fc2.bias.float(), t.bn5)
                return dict(w1=w1, b1=b1, w2=w2, b2=b2, w3=w3, b3=b3, f1=f1, c1=c1, f2=f2, c2=c2,
                            f3=t.fc3.weight.float(), c3=t.fc3.bias.float())

            self.t1 = tnet(fe.t1)
            self.t2 = tnet(fe.t2)
            self.c1w, self.c1b = conv(fe.conv1, fe.bn1)   # [64, 12]
            self.c2w, self.c2b = conv(fe.conv2, fe.bn2)   # [128, 64]
            self.c3w, self.c3b = conv(fe.conv3, fe.bn3)   # [F, 128]
            self.s1w, self.s1b = conv(m.conv1, m.bn1)     # [512, 64 + F]
            self.s2w, self.s2b = conv(m.conv2, m.bn2)
            self.s3w, self.s3b = conv(m.conv3, m.bn3)
            self.s4w, self.s4b = m.conv4.weight[:, :, 0].float(), m.conv4.bias.float()
            F = m.feature_dim
            self.F, self.C1 = F, m.num_classes + 1
            # shared per-point layers, W^T padded
            t1, t2 = self.t1, self.t2
            self.A = [(_wT(t1["w1"], 4, 64), t1["b1"]), (_wT(t1["w2"], 64, 128), t1["b2"]),
                      (_wT(t1["w3"], 128, 1024), t1["b3"])]
            self.B_tail = [(_wT(t2["w1"], 64, 64), t2["b1"]), (_wT(t2["w2"], 64, 128), t2["b2"]),
                           (_wT(t2["w3"], 128, 1024), t2["b3"])]
            self.C_tail = (_wT(self.c3w, 128, _pad(F, 32)), _bpad(self.c3b, _pad(F, 32)))
            self.s1a = self.s1w[:, :64].contiguous()      # acts on x_t2
            self.s1bT = self.s1w[:, 64:].t().contiguous()  # [F, 512], acts on g3
            self.D_tail = [(_wT(self.s2w, 512, 256), self.s2b), (_wT(self.s3w, 256, 128), self.s3b),
                           (_wT(self.s4w, 128, _pad(self.C1, 32)), _bpad(self.s4b, _pad(self.C1, 32)))]
            self.c1wT = self.c1w.t().contiguous()         # [12, 64]
            self.c2wT = self.c2w.t().contiguous()         # [64, 128]
            self.s1aT = self.s1a.t().contiguous()         # [64, 512]
            # x_t2 = t2^T x1 feeds conv2 and the seg head: one bmm t2 @ [W2^T | Ws1a^T]
            self.t2_rhs = torch.cat((self.c2wT, self.s1aT), dim=1).contiguous()  # [64, 640]
            # conv1 of the t1-transformed input: (W1 M(t1))^T = sum_ac t1[a,c] E_ac^T W1^T,
            # M(t1) = blockdiag(t1, kron(t1, I3)) (p' = t1 p, C' = t1 C)
            dev = self.c1wT.device
            E = torch.zeros((9, 12, 12), device=dev)
            for a in range(3):
                for c in range(3):
                    E[3 * a + c, a, c] = 1.0
                    for j in range(3):
                        E[3 * a + c, 3 + 3 * a + j, 3 + 3 * c + j] = 1.0
            self.t1_basis = torch.matmul(E.transpose(1, 2), self.c1wT).reshape(9, 12 * 64).contiguous()
            # the identity the TNet heads add (ndtnet.py:59), folded into fc3's bias
            self.t1["c3"] = self.t1["c3"] + torch.eye(3, device=dev).reshape(-1)
            self.t2["c3"] = self.t2["c3"] + torch.eye(64, device=dev).reshape(-1)


def _signature(m) -> tuple:
    return tuple((t.data_ptr(), t._version) for t in list(m.parameters()) + list(m.buffers()))


def _fc_head(g: torch.Tensor, t: dict, dim: int) -> torch.Tensor:
    """TNet FC head (ndtnet.py:53-60); the identity is folded into t["c3"]."""
    h = torch.addmm(t["c1"], g, t["f1"].t()).relu_()
    h = torch.addmm(t["c2"], h, t["f2"].t()).relu_()
    return torch.addmm(t["c3"], h, t["f3"].t()).view(-1, dim, dim)


def _chain_gpu(x: torch.Tensor, n: int, in_cols: int, layers, relus, mode: int, gmax=None, out=None, out_cols=0,
               per_cloud=()) -> None:
    ch = _Chain()
    ch.x = x.data_ptr()
    ch.x_ld = x.stride(1)
    ch.in_cols = in_cols
    ch.num_points = n
    ch.num_layers = len(layers)
    widths = [layers[0][0].shape[-2], 4]  # LDS regions: layer l reads l & 1, writes (l + 1) & 1
    for i, (w, b) in enumerate(layers):
        L = ch.L[i]
        L.wT = w.data_ptr()
        L.K, L.N = w.shape[-2], w.shape[-1]
        L.ldw = w.stride(-2)
        L.w_cloud_stride = w.stride(0) if (i in per_cloud and w.dim() == 3) else 0
        L.bias = b.data_ptr()
        L.bias_cloud_stride = b.stride(0) if b.dim() == 2 else 0
        L.relu = relus[i]
        if i + 1 < len(layers) or mode == 1:
            widths[(i + 1) & 1] = max(widths[(i + 1) & 1], L.N)
    ch.mode = mode
    ch.out_cols = out_cols
    ch.gmax = gmax.data_ptr() if gmax is not None else None
    ch.gmax_ld = gmax.stride(0) if gmax is not None else 0
    ch.max_width, ch.max_width2 = widths
    ch.out = out.data_ptr() if out is not None else None
    rc = _lib.lib().ndnet_pn_chain_run(ctypes.byref(ch), x.shape[0], _lib.stream_ptr(x.device))
    _lib.check(rc, "ndnet_pn_chain_run")


def _chain_torch(x: torch.Tensor, n: int, in_cols: int, layers, relus, mode: int, gmax=None, out=None,
                 out_cols=0, per_cloud=()) -> None:
    """What one ``ndnet_pn_chain_run`` computes, in torch ops (tests: checks the
    folding algebra on CPU and the kernel against it on the GPU)."""
    h = x[..., :in_cols].float()
    k0 = layers[0][0].shape[-2]
    h = torch.nn.functional.pad(h, (0, k0 - in_cols))
    for i, (w, b) in enumerate(layers):
        h = torch.matmul(h, w[..., : h.shape[-1], :]) + (b[:, None, :] if b.dim() == 2 else b)
        if relus[i]:
            h = torch.relu(h)
    if mode == 0:
        gmax.copy_(torch.maximum(gmax, h.amax(dim=1)))
    else:
        out.copy_(torch.log_softmax(h[..., :out_cols], dim=2))


def segmentation_forward(model, points: torch.Tensor, covariances: torch.Tensor, chain=None) -> torch.Tensor:
    """model(points [B,N,3], covariances [B,N,9]) -> log-probs [B,N,C+1], eval mode."""
    _chain = chain or _chain_gpu
    sig = _signature(model)
    if model._hip is None or model._hip[0] != sig:
        model._hip = (sig, _Folded(model))
    W = model._hip[1]
    B, N, _ = points.shape
    dev = points.device
    # one [B,N,12] block; ndt_preprocessing already returns views of one
    base = points
    if (points.stride() == (N * 12, 12, 1) and covariances.stride() == (N * 12, 12, 1)
            and covariances.data_ptr() == points.data_ptr() + 12 and points.dtype == torch.float32):
        x = points.as_strided((B, N, 12), (N * 12, 12, 1))
    else:
        x = torch.cat((points, covariances), dim=2).float().contiguous()
    del base
    # the three max-pooled vectors, -inf before the atomic maxima (ReLU'd maxima are >= 0)
    Fp = W.C_tail[0].shape[1]
    gbuf = torch.full((B, 2048 + Fp), float("-inf"), dtype=torch.float32, device=dev)
    g1, g2, g3 = gbuf[:, :1024], gbuf[:, 1024:2048], gbuf[:, 2048:]
    # A: TNet(3)
    _chain(x, N, 3, W.A, (1, 1, 1), 0, gmax=g1)
    t1 = _fc_head(g1, W.t1, 3)                                        # [B,3,3]
    w1T = torch.matmul(t1.reshape(B, 9), W.t1_basis).view(B, 12, 64)  # (W1 M(t1))^T
    # B: conv1 (+t1) then TNet(64)
    _chain(x, N, 12, [(w1T, W.c1b)] + W.B_tail, (0, 1, 1, 1), 0, gmax=g2, per_cloud=(0,))
    t2 = _fc_head(g2, W.t2, 64)                                       # [B,64,64]
    t2w = torch.matmul(t2, W.t2_rhs)                                  # [B,64,640]
    w2T, sT = t2w[:, :, :128], t2w[:, :, 128:]                        # conv2, seg conv1[:, :64]; t2 folded
    # C: conv2, conv3, max over points
    _chain(x, N, 12, [(w1T, W.c1b), (w2T, W.c2b), W.C_tail], (0, 0, 0), 0, gmax=g3, per_cloud=(0, 1))
    # D: seg head; the broadcast global feature enters as a per-cloud bias
    cvec = torch.addmm(W.s1b, g3[:, : W.F], W.s1bT)                   # [B,512]
    out = torch.empty((B, N, W.C1), dtype=torch.float32, device=dev)
    _chain(x, N, 12, [(w1T, W.c1b), (sT, cvec)] + W.D_tail, (0, 1, 1, 1, 0), 1, out=out, out_cols=W.C1,
           per_cloud=(0, 1))
    return out
