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
linear layer.  The per-point GEMMs run on the matrix cores: eleven layers
(the three 128 -> 1024 / F max-pooled convs, the t2-folded conv2, the seg
head's 64 -> 512, 512 -> 256, 256 -> 128 and 128 -> C+1, and the TNets'
64 -> 64 / 64 -> 128; ``X6_NARROW``) as fp32-accurate split-bf16 products
(``SPLIT_BF16`` below), the K = 16 first layers on the fp32 MFMA.  The
per-cloud steps (TNet FC heads and the seg head's global-feature bias on the
fp32 MFMA, ``ndnet_pn_fc_mfma_run``; the t1 / t2 weight folds) are HIP
kernels on the same stream (``_glue_hip``); ``_glue_torch`` is their torch
restatement for the tests.
"""
from __future__ import annotations

import ctypes
import os

import torch

from .. import _lib

MAX_LAYERS = 5
CHAIN_NAMES = ("A: TNet(3) 3-64-128-1024 + max", "B: conv1(t1) + TNet(64) 64-64-128-1024 + max",
               "C: conv1, conv2(t2), conv3 + max", "D: seg head 64-512-256-128-(C+1) + log_softmax")

# set to a list to collect (chain index, start event, end event) per chain launch
chain_timing = None

# The three wide max-pooled layers (TNet(3) / TNet(64) conv3, NDTNet conv3:
# 128 -> 1024 / 768, 90% of chains A-C's FLOPs) and the seg head's 512 -> 256
# (fed chunk by chunk from the fused 64 -> 512), the 64 -> 512 itself, 256 -> 128
# and NDTNet's t2-folded conv2 run as split-bf16 "x6" GEMMs
# (include/ndnet_pointnet.h prec = 1): fp32-accurate (operands split into
# three bf16, six exact partial products accumulated in fp32) on the bf16
# matrix cores.  NDNET_PN_PRECISION: "x6" (default), or "fp32" to keep every
# layer on the fp32 MFMA.  (Round 2's "x6f" -- fp32 weights split in
# registers, measured 20-25% slower per layer -- was removed in round 3: its
# code paths alone cost the kernel registers and scratch,
# profiles/r03l_stamps_depth.txt.)
PRECISION = SPLIT_BF16 = X6_PREC = None


def set_precision(mode: str) -> None:
    """"x6" or "fp32" for models folded from now on (a model re-folds when its
    ``_hip`` cache is cleared)."""
    global PRECISION, SPLIT_BF16, X6_PREC
    if mode not in ("x6", "fp32"):
        raise ValueError(f"unknown PointNet precision mode {mode!r}")
    PRECISION = mode
    SPLIT_BF16 = mode != "fp32"
    X6_PREC = 1


set_precision(os.environ.get("NDNET_PN_PRECISION", "x6"))
# split-bf16 also on the narrower per-point layers with K >= 64 (TNet(3)'s
# 64 -> 128, TNet(64)'s 64 -> 64 and 64 -> 128, the seg head's 128 -> C+1):
# default on, measured -5 us per forward (chains A / B / D 3 / 2 / 1.5 us
# faster); "0" keeps them on the fp32 MFMA.  Only the K = 16 first layers stay fp32.
X6_NARROW = os.environ.get("NDNET_PN_X6_NARROW", "1") == "1"


class _Layer(ctypes.Structure):
    _fields_ = [("w", ctypes.c_void_p), ("w_cloud_stride", ctypes.c_int64), ("bias", ctypes.c_void_p),
                ("bias_cloud_stride", ctypes.c_int64), ("K", ctypes.c_int32), ("N", ctypes.c_int32),
                ("relu", ctypes.c_int32), ("prec", ctypes.c_int32), ("fuse_next", ctypes.c_int32)]


class _Chain(ctypes.Structure):
    _fields_ = [("x", ctypes.c_void_p), ("x_ld", ctypes.c_int32), ("in_cols", ctypes.c_int32),
                ("num_points", ctypes.c_int32), ("num_layers", ctypes.c_int32), ("L", _Layer * MAX_LAYERS),
                ("mode", ctypes.c_int32), ("out_cols", ctypes.c_int32), ("gmax", ctypes.c_void_p),
                ("gmax_ld", ctypes.c_int32), ("max_width", ctypes.c_int32), ("max_width2", ctypes.c_int32),
                ("out", ctypes.c_void_p), ("clear", ctypes.c_void_p), ("clear_count", ctypes.c_int64),
                ("head_h2", ctypes.c_void_p), ("head_ld", ctypes.c_int32), ("head_K", ctypes.c_int32),
                ("head_w3", ctypes.c_void_p), ("head_b3", ctypes.c_void_p), ("head_basis", ctypes.c_void_p),
                ("head_kin", ctypes.c_int32), ("head_nout", ctypes.c_int32), ("head_t1", ctypes.c_void_p),
                ("fold_t2", ctypes.c_void_p), ("fold_ld", ctypes.c_int32), ("fold_out_w", ctypes.c_void_p),
                ("fold_out_b", ctypes.c_void_p)]


class _FoldJob(ctypes.Structure):  # ndnet_pn_fold_job (include/ndnet_pointnet.h)
    _fields_ = [("w", ctypes.c_void_p), ("bias", ctypes.c_void_p), ("gamma", ctypes.c_void_p),
                ("beta", ctypes.c_void_p), ("mean", ctypes.c_void_p), ("var", ctypes.c_void_p),
                ("out", ctypes.c_void_p), ("kind", ctypes.c_int32), ("N", ctypes.c_int32), ("K", ctypes.c_int32),
                ("ld", ctypes.c_int32), ("k0", ctypes.c_int32), ("Kp", ctypes.c_int32), ("Np", ctypes.c_int32),
                ("eye", ctypes.c_int32), ("eps", ctypes.c_float), ("reserved", ctypes.c_int32),
                ("block0", ctypes.c_int64)]



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


def _frag(wT: torch.Tensor) -> torch.Tensor:
    """Plain W^T [..., K, N] (K % 16 == 0, N % 16 == 0) -> the fragment-major
    layout of include/ndnet_pointnet.h, flattened: [cb][kg][kq][cl][s] with
    k = 16 kg + 4 kq + s, n = 16 cb + cl."""
    *lead, K, N = wT.shape
    v = wT.reshape(*lead, K // 16, 4, 4, N // 16, 16)
    nl = len(lead)
    perm = list(range(nl)) + [nl + 3, nl + 0, nl + 1, nl + 4, nl + 2]
    return v.permute(*perm).reshape(*lead, K * N).contiguous()


def _npad(n: int) -> int:
    """Output width the chain kernel splits evenly: 32, or a multiple of 64."""
    return 32 if n <= 32 else _pad(n, 64)


def _frag_x6(wT: torch.Tensor) -> torch.Tensor:
    """Plain W^T [K, N] (K % 32 == 0, N % 16 == 0) -> the split-bf16 layout of
    include/ndnet_pointnet.h (prec 1), flattened bf16: W^T = h + m + l
    (h = bf16(w), m = bf16(w - h), l = bf16(w - h - m), residuals exact in
    fp32), [cb][kg][plane][kq][cl][j] with k = 32 kg + 8 kq + j, n = 16 cb + cl."""
    K, N = wT.shape
    w = wT.float()
    h = w.to(torch.bfloat16)
    r = w - h.float()
    m = r.to(torch.bfloat16)
    lo = (r - m.float()).to(torch.bfloat16)
    planes = torch.stack([h, m, lo])                                  # [3, K, N]
    v = planes.reshape(3, K // 32, 4, 8, N // 16, 16)                 # plane, kg, kq, j, cb, cl
    return v.permute(4, 1, 0, 2, 5, 3).reshape(-1).contiguous()        # cb, kg, plane, kq, cl, j


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
            self.A = [(_wT(t1["w1"], 16, 64), t1["b1"]), (_wT(t1["w2"], 64, 128), t1["b2"]),
                      (_wT(t1["w3"], 128, 1024), t1["b3"])]
            self.B_tail = [(_wT(t2["w1"], 64, 64), t2["b1"]), (_wT(t2["w2"], 64, 128), t2["b2"]),
                           (_wT(t2["w3"], 128, 1024), t2["b3"])]
            self.C_tail = (_wT(self.c3w, 128, _npad(F)), _bpad(self.c3b, _npad(F)))
            self.s1a = self.s1w[:, :64].contiguous()      # acts on x_t2
            self.s1bT = self.s1w[:, 64:].t().contiguous()  # [F, 512], acts on g3
            self.s1g = self.s1w[:, 64:].contiguous()       # [512, F] row-major for ndnet_pn_fc_run
            self.D_tail = [(_wT(self.s2w, 512, 256), self.s2b), (_wT(self.s3w, 256, 128), self.s3b),
                           (_wT(self.s4w, 128, _npad(self.C1)), _bpad(self.s4b, _npad(self.C1)))]
            self.c1wT = self.c1w.t().contiguous()         # [12, 64]
            # x_t2 = t2^T x1 (ndtnet.py:152-157) feeds conv2 and the seg head's
            # conv1a; t2 is folded into chains C / D's layer 0 (their prologue,
            # ndnet_pn_chain.fold_t2), so both layers keep shared weights
            self.C_mid = (_wT(self.c2w, 64, 128), self.c2b)          # conv2 W^T [64, 128]
            self.s1aT = _wT(self.s1a, 64, 512)                        # seg conv1a W^T [64, 512]
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
            # fragment-major copies of the shared per-point layers (the HIP chains)
            self.frag = {id(w): _frag(w) for w, _ in
                         self.A + self.B_tail + [self.C_mid, self.C_tail, (self.s1aT, None)] + self.D_tail}
            # the wide pooled layers, conv2 and the seg head's conv1a in split-bf16 form
            self.wide = [self.A[2][0], self.B_tail[2][0], self.C_tail[0], self.D_tail[0][0], self.D_tail[1][0],
                         self.C_mid[0], self.s1aT]
            if X6_NARROW:  # the K >= 64 fp32-MFMA layers too (64 -> 128 of TNet(3) / TNet(64), 64 -> 64, 128 -> C+1)
                self.wide += [self.A[1][0], self.B_tail[0][0], self.B_tail[1][0], self.D_tail[2][0]]
            self.frag6 = {id(w): _frag_x6(w) for w in self.wide}
            # the FC layers of the TNet heads and the seg head's global-feature
            # bias, W^T fragment-major for the MFMA GEMV (ndnet_pn_fc_mfma_run)
            self.fcf = {id(w): _frag(w.t().contiguous()) for w in
                        (self.t1["f1"], self.t1["f2"], self.t2["f1"], self.t2["f2"], self.t2["f3"], self.s1g)}
            # the identity the TNet heads add (ndtnet.py:59), folded into fc3's bias
            self.t1["c3"] = self.t1["c3"] + torch.eye(3, device=dev).reshape(-1)
            self.t2["c3"] = self.t2["c3"] + torch.eye(64, device=dev).reshape(-1)
        self.tensors = _tensors(m)
        self.prec = (SPLIT_BF16, X6_NARROW)
        self.jobs = self._fold_jobs(m)
        self._dev_jobs, self._blocks = None, 0

    def _fold_jobs(self, m) -> list:
        """The recipe of every tensor above as ndnet_pn_fold_job fields (kind,
        out, layer, BatchNorm, k0, K, Kp, Np, eye): what ``refold`` re-runs in
        place.  Aliases of parameters (fc3 / conv4 weights, conv4 bias) need
        none.  Only for fp32, contiguous parameters (else None: a re-fold
        rebuilds)."""
        if not all(t.dtype == torch.float32 and t.is_contiguous() for t in m.parameters()):
            return None
        fe = m.feature_extractor
        jobs, src = [], {}

        def add(kind, out, layer, bn, k0=0, K=None, Kp=0, Np=0, eye=0):
            ld = layer.weight.shape[1]
            K = ld - k0 if K is None else K
            jobs.append((kind, out, layer, bn, k0, K, Kp, Np, eye))
            src[id(out)] = (layer, bn, k0, K)

        def rows(out, layer, bn, k0=0, K=None):
            add(3, out, layer, bn, k0, K)

        def wt(out, layer, bn, k0=0, K=None):
            add(0, out, layer, bn, k0, K, out.shape[0], out.shape[1])

        def bias(out, layer, bn, eye=0):
            add(5, out, layer, bn, Np=out.shape[0], eye=eye)

        for t, tm, d in ((self.t1, fe.t1, 3), (self.t2, fe.t2, 64)):
            for i in (1, 2, 3):
                conv, bn = getattr(tm, f"conv{i}"), getattr(tm, f"bn{i}")
                rows(t[f"w{i}"], conv, bn)
                bias(t[f"b{i}"], conv, bn)
            rows(t["f1"], tm.fc1, tm.bn4)
            bias(t["c1"], tm.fc1, tm.bn4)
            rows(t["f2"], tm.fc2, tm.bn5)
            bias(t["c2"], tm.fc2, tm.bn5)
            bias(t["c3"], tm.fc3, None, eye=d)
            src[id(t["f3"])] = (tm.fc3, None, 0, tm.fc3.weight.shape[1])  # the parameter itself
        for (w, b), conv, bn in (((self.c1w, self.c1b), fe.conv1, fe.bn1), ((self.c2w, self.c2b), fe.conv2, fe.bn2),
                                 ((self.c3w, self.c3b), fe.conv3, fe.bn3), ((self.s1w, self.s1b), m.conv1, m.bn1),
                                 ((self.s2w, self.s2b), m.conv2, m.bn2), ((self.s3w, self.s3b), m.conv3, m.bn3)):
            rows(w, conv, bn)
            bias(b, conv, bn)
        rows(self.s1a, m.conv1, m.bn1, 0, 64)
        rows(self.s1g, m.conv1, m.bn1, 64, self.F)
        wt(self.s1bT, m.conv1, m.bn1, 64, self.F)
        for layers, tm in ((self.A, fe.t1), (self.B_tail, fe.t2)):
            for i, (w, _) in enumerate(layers, 1):
                wt(w, getattr(tm, f"conv{i}"), getattr(tm, f"bn{i}"))
        wt(self.C_tail[0], fe.conv3, fe.bn3)
        bias(self.C_tail[1], fe.conv3, fe.bn3)
        wt(self.D_tail[0][0], m.conv2, m.bn2)
        wt(self.D_tail[1][0], m.conv3, m.bn3)
        wt(self.D_tail[2][0], m.conv4, None)
        bias(self.D_tail[2][1], m.conv4, None)
        wt(self.c1wT, fe.conv1, fe.bn1)
        wt(self.C_mid[0], fe.conv2, fe.bn2)
        wt(self.s1aT, m.conv1, m.bn1, 0, 64)
        add(4, self.t1_basis, fe.conv1, fe.bn1)
        wts = {id(w): w for w, _ in self.A + self.B_tail + [self.C_mid, self.C_tail, (self.s1aT, None)] + self.D_tail}
        for key, out in self.frag.items():
            layer, bn, k0, K = src[key]
            add(1, out, layer, bn, k0, K, *wts[key].shape)
        for w in self.wide:
            layer, bn, k0, K = src[id(w)]
            add(2, self.frag6[id(w)], layer, bn, k0, K, *w.shape)
        fcs = (self.t1["f1"], self.t1["f2"], self.t2["f1"], self.t2["f2"], self.t2["f3"], self.s1g)
        for w in fcs:
            layer, bn, k0, K = src[id(w)]
            add(1, self.fcf[id(w)], layer, bn, k0, K, w.shape[1], w.shape[0])
        return jobs

    def can_refold(self, tensors) -> bool:
        """In place: the same parameter / buffer tensors, on a GPU, at the same precision."""
        return (self.jobs is not None and self.prec == (SPLIT_BF16, X6_NARROW) and self.c1wT.is_cuda
                and len(tensors) == len(self.tensors) and all(a is b for a, b in zip(tensors, self.tensors))
                and all(t.is_contiguous() and t.dtype == torch.float32 for t in tensors if t.is_floating_point()))

    def refold(self) -> None:
        """Every fold above again, from the current weights and running
        statistics, into the same tensors: one ``ndnet_pn_fold_run`` launch on
        the current stream (the workspaces and prebuilt chain argument blocks
        that point at these tensors stay valid)."""
        dev = self.c1wT.device
        if self._dev_jobs is None:
            arr = (_FoldJob * len(self.jobs))()
            for J, (kind, out, layer, bn, k0, K, Kp, Np, eye) in zip(arr, self.jobs):
                J.kind, J.out, J.N, J.K, J.ld, J.k0 = kind, out.data_ptr(), layer.weight.shape[0], K, \
                    layer.weight.shape[1], k0
                J.Kp, J.Np, J.eye = Kp, Np, eye
                if kind == 5:
                    J.bias = layer.bias.data_ptr()
                else:
                    J.w = layer.weight.data_ptr()
                if bn is not None:
                    J.gamma, J.beta = bn.weight.data_ptr(), bn.bias.data_ptr()
                    J.mean, J.var, J.eps = bn.running_mean.data_ptr(), bn.running_var.data_ptr(), bn.eps
            blocks = ctypes.c_int64()
            _lib.check(_lib.lib().ndnet_pn_fold_prepare(arr, len(arr), ctypes.byref(blocks)), "ndnet_pn_fold_prepare")
            self._dev_jobs = torch.frombuffer(bytearray(bytes(arr)), dtype=torch.uint8).to(dev)
            self._blocks = blocks.value
        rc = _lib.lib().ndnet_pn_fold_run(self._dev_jobs.data_ptr(), len(self.jobs), self._blocks,
                                          _lib.stream_ptr(dev))
        _lib.check(rc, "ndnet_pn_fold_run")


def _tensors(m) -> list:
    return list(m.parameters()) + list(m.buffers())


def _signature(tensors) -> tuple:
    """Storage and in-place version of every weight: a change re-folds."""
    return tuple((t.data_ptr(), t._version) for t in tensors)


def _fc_head(g: torch.Tensor, t: dict, dim: int, h1: torch.Tensor, h2: torch.Tensor, out: torch.Tensor):
    """TNet FC head (ndtnet.py:53-60) into preallocated buffers; the identity is
    folded into t["c3"]."""
    torch.addmm(t["c1"], g, t["f1"].t(), out=h1).relu_()
    torch.addmm(t["c2"], h1, t["f2"].t(), out=h2).relu_()
    torch.addmm(t["c3"], h2, t["f3"].t(), out=out)
    return out.view(-1, dim, dim)


def _build_chain(n: int, in_cols: int, layers, relus, mode: int, gmax=None, out_cols=0, fuse=()) -> "_Chain":
    """ctypes argument block of one ``ndnet_pn_chain_run`` (x / out set per call).
    ``layers``: (fragment-major weights, per-cloud stride in floats or 0, bias,
    K, N[, prec]) per layer.  Layers in ``fuse`` are produced in 64-column chunks
    straight into the next layer (include/ndnet_pointnet.h)."""
    ch = _Chain()
    ch.x_ld = 12
    ch.in_cols = in_cols
    ch.num_points = n
    ch.num_layers = len(layers)
    # LDS regions: layer l reads l & 1, writes (l + 1) & 1; the input tile is
    # zero-filled to the first layer's K; a fused layer's output has no region
    widths = [layers[0][3], 8]
    for i, (w, stride, b, K, N, *prec) in enumerate(layers):
        L = ch.L[i]
        L.prec = prec[0] if prec else 0
        L.w = w.data_ptr()
        L.w_cloud_stride = stride
        L.K, L.N = K, N
        L.bias = b.data_ptr()
        L.bias_cloud_stride = b.stride(0) if b.dim() == 2 else 0
        L.relu = relus[i]
        L.fuse_next = 1 if i in fuse else 0
        if i in fuse:
            continue
        if i + 1 < len(layers) or mode == 1:
            widths[(i + 1) & 1] = max(widths[(i + 1) & 1], N)
    ch.mode = mode
    ch.out_cols = out_cols
    ch.gmax = gmax.data_ptr() if gmax is not None else None
    ch.gmax_ld = gmax.stride(0) if gmax is not None else 0
    ch.max_width, ch.max_width2 = widths
    return ch


# 32-point tiles (ndnet_pn_chain_run_t32) when 64-point tiles would fill at
# most half the CUs (C5's 500-point level: 16 x 8 tiles on 256 CUs); "0" off.
# Always taking them (8-wave workgroups, two per CU, beside other forwards'
# kernels) measured 71-74k against 81k clouds/s (profiles/r03af_t32_ab.txt).
TILE32 = os.environ.get("NDNET_PN_TILE32", "1") == "1"
_cus = {}


def _use_t32(B: int, n: int, device) -> bool:
    if not TILE32:
        return False
    if device not in _cus:
        _cus[device] = torch.cuda.get_device_properties(device).multi_processor_count
    return 2 * B * ((n + 63) // 64) <= _cus[device]


def _run_chain(ch: "_Chain", x: torch.Tensor, out=None) -> None:
    assert x.stride(1) == 12 and x.stride(2) == 1 and x.dtype == torch.float32
    ch.x = x.data_ptr()
    ch.out = out.data_ptr() if out is not None else None
    if _use_t32(x.shape[0], x.shape[1], x.device):
        rc = _lib.lib().ndnet_pn_chain_run_t32(ctypes.byref(ch), x.shape[0], _lib.stream_ptr(x.device))
        _lib.check(rc, "ndnet_pn_chain_run_t32")
        return
    rc = _lib.lib().ndnet_pn_chain_run(ctypes.byref(ch), x.shape[0], _lib.stream_ptr(x.device))
    _lib.check(rc, "ndnet_pn_chain_run")


def _chain_torch(x: torch.Tensor, n: int, in_cols: int, layers, relus, mode: int, gmax=None, out=None,
                 out_cols=0, fuse=()) -> None:
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


class _Workspace:
    """Per-(batch, points) intermediates and prebuilt chain argument blocks, so
    an eval forward does no allocation but its output and no struct building."""

    def __init__(self, W: _Folded, B: int, N: int, dev) -> None:
        self.W = W
        f32 = dict(dtype=torch.float32, device=dev)
        Fp = W.C_tail[0].shape[1]
        # the three max-pooled vectors, -inf before the atomic maxima (ReLU'd maxima are >= 0)
        # -inf before the first forward; chain D re-arms it for the next one
        self.gbuf = torch.full((B, 2048 + Fp), float("-inf"), **f32)
        self.g1, self.g2, self.g3 = self.gbuf[:, :1024], self.gbuf[:, 1024:2048], self.gbuf[:, 2048:]
        self.h1, self.h2 = torch.empty((B, 512), **f32), torch.empty((B, 256), **f32)
        self.t1, self.t2 = torch.empty((B, 9), **f32), torch.empty((B, 4096), **f32)
        self.cvec = torch.empty((B, 512), **f32)        # per-cloud bias of the seg head
        # per-cloud folded weights: plain W^T for the torch emulation ...
        self.w1T = torch.empty((B, 12, 64), **f32)      # (W1 M(t1))^T per cloud
        self.w1t2 = torch.empty((B, 12, 64), **f32)     # (W1 M(t1))^T t2: layer 0 of chains C / D
        self.b1t2 = torch.empty((B, 64), **f32)         # b1^T t2
        # ... and fragment-major for the HIP chains (K of conv1 padded 12 -> 16);
        # the HIP chains C / D fold t2 in their prologue (fold_t2)
        self.w1f = torch.empty((B, 16 * 64), **f32)
        self.w1t2f = torch.zeros((B, 16 * 64), **f32)   # chain C publishes (W1 M(t1))^T t2 here for chain D
        self.specs = [  # torch emulation: (in_cols, [(W^T, bias)], relus, mode, kwargs)
            (3, W.A, (1, 1, 1), 0, dict(gmax=self.g1)),
            (12, [(self.w1T, W.c1b)] + W.B_tail, (0, 1, 1, 1), 0, dict(gmax=self.g2)),
            (12, [(self.w1t2, self.b1t2), W.C_mid, W.C_tail], (0, 0, 0), 0, dict(gmax=self.g3)),
            # the 512-wide seg conv1 output feeds conv2 chunk by chunk (never stored whole)
            (12, [(self.w1t2, self.b1t2), (W.s1aT, self.cvec)] + W.D_tail, (0, 1, 1, 1, 0), 1,
             dict(out_cols=W.C1, fuse=(1,))),
        ]

        def shared(wb):
            w, b = wb
            if SPLIT_BF16 and id(w) in W.frag6:
                return (W.frag6[id(w)], 0, b, w.shape[0], w.shape[1], X6_PREC)
            return (W.frag[id(w)], 0, b, w.shape[0], w.shape[1])

        L1 = (self.w1f, self.w1f.stride(0), W.c1b, 16, 64)
        # chain C's layer 0: conv1 with t1 and t2 folded (ndnet_pn_fold_t2_run), or
        # with t1 only and t2 folded in its prologue (NDNET_PN_FOLD_T2=chain)
        LC = (self.w1t2f, self.w1t2f.stride(0), self.b1t2, 16, 64) if FOLD_T2_KERNEL else L1
        self.hip_layers = [
            [shared(x) for x in W.A],
            [L1] + [shared(x) for x in W.B_tail],
            [LC, shared(W.C_mid), shared(W.C_tail)],
            [(self.w1t2f, self.w1t2f.stride(0), self.b1t2, 16, 64), shared((W.s1aT, self.cvec))] +
            [shared(x) for x in W.D_tail],
        ]
        self.N = N
        self.structs = None

    def chain(self, i: int, x: torch.Tensor, chain_fn=None, out=None) -> None:
        in_cols, layers, relus, mode, kw = self.specs[i]
        if chain_fn is not None:
            kw = dict(kw)
            if out is not None:
                kw["out"] = out
            chain_fn(x, self.N, in_cols, layers, relus, mode, **kw)
            return
        if self.structs is None:
            self.structs = [_build_chain(self.N, s[0], hl, s[2], s[3], **s[4])
                            for s, hl in zip(self.specs, self.hip_layers)]
            # the last chain re-arms the max-pool buffer (-inf) for the next forward
            self.structs[3].clear = self.gbuf.data_ptr()
            self.structs[3].clear_count = self.gbuf.numel()
            if HEAD3_IN_CHAIN:  # chain B computes t1 and its conv1 weights itself
                W, cb = self.W, self.structs[1]
                cb.head_h2, cb.head_ld, cb.head_K = self.h2.data_ptr(), self.h2.stride(0), self.h2.shape[1]
                cb.head_w3, cb.head_b3 = W.t1["f3"].data_ptr(), W.t1["c3"].data_ptr()
                cb.head_basis, cb.head_kin, cb.head_nout = W.t1_basis.data_ptr(), 12, 64
                cb.head_t1 = self.t1.data_ptr()
            if not FOLD_T2_KERNEL:  # chain C: t2 through layer 0 (prologue fold), published for chain D
                cc = self.structs[2]
                cc.fold_t2, cc.fold_ld = self.t2.data_ptr(), self.t2.stride(0)
                cc.fold_out_w, cc.fold_out_b = self.w1t2f.data_ptr(), self.b1t2.data_ptr()
        if chain_timing is not None:  # torch events on the launch stream (bench.py)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            _run_chain(self.structs[i], x, out)
            e1.record()
            chain_timing.append((i, e0, e1))
        else:
            _run_chain(self.structs[i], x, out)


def _folded(model):
    """The model's folded weights, re-folded when any weight changed."""
    cache = model._hip
    if cache is None:
        tensors = _tensors(model)
        cache = model._hip = {"tensors": tensors, "sig": None, "stale": False}
    sig = _signature(cache["tensors"])
    cur = _tensors(model)  # a parameter or buffer replaced by another tensor is a change too
    replaced = len(cur) != len(cache["tensors"]) or any(a is not b for a, b in zip(cur, cache["tensors"]))
    if replaced or cache["sig"] != sig or cache["stale"]:
        # stale: the model was in train mode since the last fold, where a
        # replayed training graph updates the weights without bumping their
        # versions (ndnet.training.GraphedTrainStep)
        W = cache.get("W")
        if W is not None and W.can_refold(_tensors(model)):
            W.refold()  # one launch, in place: workspaces and argument blocks stay valid
        else:
            cache.update(tensors=_tensors(model), W=_Folded(model), ws={})
            sig = _signature(cache["tensors"])
        cache.update(sig=sig, stale=False)
    return cache


# TNet(64)'s transform through conv1 (layer 0 of chains C and D): "kernel"
# (default, round 5) once per cloud by ndnet_pn_fold_t2_run after fc3; "chain"
# in chain C's prologue, every workgroup (fold_t2), published for chain D
FOLD_T2_KERNEL = os.environ.get("NDNET_PN_FOLD_T2", "kernel") == "kernel"
# TNet(3)'s tail (fc3 + the t1 fold of conv1): "chain" (default) computes it in
# chain B's prologue, per workgroup (ndnet_pn_chain.head_*: one launch and one
# boundary fewer); "kernel" runs ndnet_pn_head3_run before chain B
HEAD3_IN_CHAIN = os.environ.get("NDNET_PN_HEAD3", "chain") == "chain"

# TNet / seg-bias FC layers: "mfma" (default: ndnet_pn_fc_mfma_run, 16-row
# fp32-MFMA GEMM over fragment-major weights) or "gemv" (ndnet_pn_fc_run,
# VALU dot products over row-major weights).  Round 3 also tried a TNet head's
# 2-3 layers in ONE launch handing off through an in-memory counter (stage
# workgroups polling, sc1 stores / loads): the forward's non-chain time rose
# from 46 to 63 us (profiles/r03z_fc_ab.txt), so every layer stays a launch.
FC_MFMA = os.environ.get("NDNET_PN_FC", "mfma") == "mfma"


def _fc(x: torch.Tensor, w: torch.Tensor, b: torch.Tensor, out: torch.Tensor, relu: bool, wf=None) -> None:
    """out = act(x @ w^T + b) on a HIP kernel (chunks of 16 clouds); wf: W^T
    fragment-major (the MFMA kernel), else the GEMV kernel on w."""
    B = x.shape[0]
    st = _lib.stream_ptr(x.device)
    for c0 in range(0, B, 16):
        n = min(16, B - c0)
        if FC_MFMA and wf is not None:
            rc = _lib.lib().ndnet_pn_fc_mfma_run(x[c0].data_ptr(), x.stride(0), wf.data_ptr(), b.data_ptr(),
                                                 out[c0].data_ptr(), out.stride(0), n, w.shape[1], w.shape[0],
                                                 1 if relu else 0, st)
            _lib.check(rc, "ndnet_pn_fc_mfma_run")
        else:
            rc = _lib.lib().ndnet_pn_fc_run(x[c0].data_ptr(), x.stride(0), w.data_ptr(), b.data_ptr(),
                                            out[c0].data_ptr(), out.stride(0), n, w.shape[1], w.shape[0],
                                            1 if relu else 0, st)
            _lib.check(rc, "ndnet_pn_fc_run")


def _glue_hip(W, ws, B: int):
    """The per-cloud steps as HIP kernels: TNet heads (fc1, fc2, fc3 + I) and the
    weight folds (t1 into conv1, t2 into conv2 / seg conv1)."""
    st = lambda: _lib.stream_ptr(ws.gbuf.device)  # noqa: E731

    def fc(x, w, b, out, relu):  # with the layer's fragment-major weights (the MFMA kernel)
        _fc(x, w, b, out, relu, W.fcf.get(id(w)))

    def head_a():
        t = W.t1
        fc(ws.g1, t["f1"], t["c1"], ws.h1, True)
        fc(ws.h1, t["f2"], t["c2"], ws.h2, True)
        if HEAD3_IN_CHAIN:  # fc3 and the t1 fold run in chain B's prologue
            return
        for c0 in range(0, B, 16):
            n = min(16, B - c0)
            rc = _lib.lib().ndnet_pn_head3_run(ws.h2[c0].data_ptr(), ws.h2.stride(0), t["f3"].data_ptr(),
                                               t["c3"].data_ptr(), W.t1_basis.data_ptr(), ws.t1[c0].data_ptr(),
                                               ws.w1f[c0].data_ptr(), n, 256, 12, 64, st())
            _lib.check(rc, "ndnet_pn_head3_run")

    def head_b():
        t = W.t2
        fc(ws.g2, t["f1"], t["c1"], ws.h1, True)
        fc(ws.h1, t["f2"], t["c2"], ws.h2, True)
        fc(ws.h2, t["f3"], t["c3"], ws.t2, False)  # t2
        if FOLD_T2_KERNEL:  # t2 through conv1: chains C / D's layer 0, once per cloud
            rc = _lib.lib().ndnet_pn_fold_t2_run(ws.w1f.data_ptr(), ws.w1f.stride(0), W.c1b.data_ptr(),
                                                 ws.t2.data_ptr(), ws.t2.stride(0), ws.w1t2f.data_ptr(),
                                                 ws.b1t2.data_ptr(), B, st())
            _lib.check(rc, "ndnet_pn_fold_t2_run")

    def seg_bias():
        fc(ws.g3[:, : W.F], W.s1g, W.s1b, ws.cvec, False)

    return head_a, head_b, seg_bias


def _glue_torch(W, ws, B: int):
    """The same steps as torch ops (the emulation path of the tests)."""
    def head_a():
        t1 = _fc_head(ws.g1, W.t1, 3, ws.h1, ws.h2, ws.t1)
        torch.matmul(t1.reshape(B, 9), W.t1_basis, out=ws.w1T.view(B, 12 * 64))

    def head_b():
        t2 = _fc_head(ws.g2, W.t2, 64, ws.h1, ws.h2, ws.t2)
        torch.matmul(ws.w1T, t2, out=ws.w1t2)
        torch.matmul(W.c1b[None, None, :], t2, out=ws.b1t2.view(B, 1, 64))

    def seg_bias():
        torch.addmm(W.s1b, ws.g3[:, : W.F], W.s1bT, out=ws.cvec)

    return head_a, head_b, seg_bias


# Workspace slot of the forwards launched from now on (``workspace_slot``).
_slot = 0


class workspace_slot:
    """``with workspace_slot(i):`` -- forwards launched inside use workspace
    slot ``i`` of their shape.  A forward's workspace (the max-pool buffer
    that chain D re-arms, the FC-head intermediates, the per-cloud folded
    weights and the prebuilt argument blocks) is cached per (batch, points,
    device, slot) and is written by every forward of that key, so forwards
    that may run CONCURRENTLY -- launched on different streams with no order
    between them, e.g. two halves of a batch captured on two streams of one
    graph -- must use different slots; forwards in stream order may share one
    (the default slot 0).  This was the hazard behind round 2's crashed
    two-stream capture: both halves shared one slot, so one half's chain D
    re-armed the max-pool buffer the other half was still reducing into."""

    def __init__(self, slot: int) -> None:
        self.slot, self.prev = int(slot), None

    def __enter__(self):
        global _slot
        self.prev, _slot = _slot, self.slot
        return self

    def __exit__(self, *exc):
        global _slot
        _slot = self.prev
        return False


def segmentation_forward(model, points: torch.Tensor, covariances: torch.Tensor, chain=None) -> torch.Tensor:
    """model(points [B,N,3], covariances [B,N,9]) -> log-probs [B,N,C+1], eval mode.

    ``chain``: None runs every step on the HIP kernels; a chain emulator
    (``_chain_torch``) runs the chains and the per-cloud steps as torch ops.
    Concurrent forwards (different streams, no order) need different
    ``workspace_slot``s."""
    cache = _folded(model)
    W = cache["W"]
    B, N, _ = points.shape
    dev = points.device
    key = (B, N, dev, _slot)
    ws = cache["ws"].get(key)
    if ws is None:
        ws = cache["ws"][key] = _Workspace(W, B, N, dev)
    # one [B,N,12] block; ndt_preprocessing already returns views of one
    if (points.stride() == (N * 12, 12, 1) and covariances.stride() == (N * 12, 12, 1)
            and covariances.data_ptr() == points.data_ptr() + 12 and points.dtype == torch.float32):
        x = points.as_strided((B, N, 12), (N * 12, 12, 1))
    else:
        x = torch.cat((points, covariances), dim=2).float().contiguous()
    head_a, head_b, seg_bias = (_glue_hip if chain is None else _glue_torch)(W, ws, B)
    if chain is not None:
        ws.gbuf.fill_(float("-inf"))
    ws.chain(0, x, chain)   # A: TNet(3) -> g1
    head_a()                # t1, (W1 M(t1))^T
    ws.chain(1, x, chain)   # B: conv1 (+t1) then TNet(64) -> g2
    head_b()                # t2, t2 @ [W2^T | Ws1a^T]
    ws.chain(2, x, chain)   # C: conv2, conv3, max over points -> g3
    seg_bias()              # the broadcast global feature as a per-cloud bias of the seg head
    out = torch.empty((B, N, W.C1), dtype=torch.float32, device=dev)
    ws.chain(3, x, chain, out=out)
    if chain is not None:
        ws.gbuf.fill_(float("-inf"))  # the HIP path expects it armed (chain D re-arms it there)
    return out
