"""NDTNet: PointNet over 12-D normal distributions (mean | flattened covariance).

Module tree and parameter names follow the reference
(ndnet/models/ndtnet.py:7-243) so its ``state_dict`` checkpoints
(tools/train.py:186-194) load unchanged:

    NDTNetSegmentation
      feature_extractor: NDTNet
        conv1/conv2/conv3 (+bn1..3), t1: TNet(3), t2: TNet(64)
      conv1..conv4, bn1..bn3

Two forward paths:
  * eval mode on a gfx950 GPU with no autograd wanted (``torch.no_grad()``,
    or nothing requires grad) -> the fused HIP kernels of
    lib/libndnet_amd.so (``ndnet.models.pointnet_hip``): BatchNorm folded into
    the 1x1 convolutions, MFMA GEMMs over (points x channels), global
    max-pool fused into the producing GEMM.
  * train mode on the GPU -> every Conv1d(k=1) + BatchNorm1d (batch
    statistics) [+ ReLU] block forward and backward on the train kernels of
    lib/libndnet_amd.so (``ndnet.models.train_hip``, include/ndnet_train.h);
    the TNet FC heads (Linear + BatchNorm1d + ReLU fused per layer), the
    point transform t1, x^T t2, the seg head's conv1 over cat(x_t2, g), the
    log-softmax over the class dim and the loss also run on HIP kernels
    (round 5); what torch still runs per step is listed in DESIGN.md §3.
    ``NDNET_TRAIN_PATH=torch`` selects the torch composition instead (A/B).
  * anything else (eval-mode autograd, CPU) -> the PyTorch composition below,
    which is also the fp32 reference the kernels are tested against.
"""
from __future__ import annotations

import os
from enum import Enum

import torch
from torch import nn

_TRAIN_TORCH = os.environ.get("NDNET_TRAIN_PATH", "hip").lower() == "torch"


def _conv(cin: int, cout: int) -> nn.Conv1d:
    return nn.Conv1d(cin, cout, 1)


def _hip_train(conv: nn.Conv1d, bn, x: torch.Tensor) -> bool:
    """The HIP train kernels compute in fp32: any other input or weight dtype,
    or an autocast region (which would have torch's convs run narrower), takes
    the torch composition."""
    return (x.is_cuda and conv.training and (bn is None or bn.training) and not _TRAIN_TORCH
            and x.dtype == torch.float32 and conv.weight.dtype == torch.float32
            and not torch.is_autocast_enabled("cuda"))


def _hip_fc(t: "TNet", g: torch.Tensor) -> bool:
    """The TNet head on the HIP FC kernels: train mode, fp32 on the GPU, at most
    16 clouds (train_hip.FC_MAX_ROWS), every layer's input width a multiple of
    4 and its rows small enough for the kernels' LDS stage (B * K <= 16384),
    and what ndnet_tr_fc_fwd / _bwd_w read with 16-byte loads 16-byte aligned
    and contiguous (a weight viewed at an odd offset into a flat buffer, or a
    layer without a bias, takes the torch path)."""
    def aligned(x):
        return x is not None and x.is_contiguous() and x.data_ptr() % 16 == 0
    return (_hip_train(t.conv1, t.bn1, g) and t.fc1.training and t.bn4.training and t.bn5.training
            and 2 <= g.shape[0] <= 16 and g.dim() == 2 and g.is_contiguous() and g.data_ptr() % 16 == 0
            and all(fc.weight.dtype == torch.float32 and fc.in_features % 4 == 0
                    and g.shape[0] * fc.in_features <= 16384 and fc.bias is not None
                    and aligned(fc.weight) and aligned(fc.bias)
                    and (fc.weight.grad is None or aligned(fc.weight.grad))
                    for fc in (t.fc1, t.fc2, t.fc3)))


def _block_pool(conv: nn.Conv1d, bn, x: torch.Tensor, relu: bool) -> torch.Tensor:
    """``_block(...).amax(dim=2)``: on the HIP train path one fused block that
    never materialises the [B,C,N] activation (train_hip.conv_bn_act_pool)."""
    if _hip_train(conv, bn, x) and x.shape[0] <= 64:
        from . import train_hip
        return train_hip.conv_bn_act_pool(conv, bn, x, relu)
    return _block(conv, bn, x, relu).amax(dim=2)


def _block(conv: nn.Conv1d, bn, x: torch.Tensor, relu: bool) -> torch.Tensor:
    """``relu(bn(conv(x)))`` (bn / relu optional): on the HIP train kernels in
    train mode on the GPU (ndnet.models.train_hip), else torch ops."""
    if _hip_train(conv, bn, x):
        from . import train_hip
        return train_hip.conv_bn_act(conv, bn, x, relu)
    x = conv(x)
    if bn is not None:
        x = bn(x)
    return torch.relu(x) if relu else x


class TNet(nn.Module):
    """Predicts a ``in_dim x in_dim`` transform (reference ndtnet.py:7-62)."""

    def __init__(self, in_dim: int = 64) -> None:
        super().__init__()
        self.in_dim = in_dim
        self.conv1, self.conv2, self.conv3 = _conv(in_dim, 64), _conv(64, 128), _conv(128, 1024)
        self.fc1, self.fc2, self.fc3 = nn.Linear(1024, 512), nn.Linear(512, 256), nn.Linear(256, in_dim * in_dim)
        self.relu = nn.ReLU()
        self.bn1, self.bn2, self.bn3 = nn.BatchNorm1d(64), nn.BatchNorm1d(128), nn.BatchNorm1d(1024)
        self.bn4, self.bn5 = nn.BatchNorm1d(512), nn.BatchNorm1d(256)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        # pointwise MLP with BN+ReLU, max over points, FC head, + identity
        x = _block(self.conv1, self.bn1, x, True)
        x = _block(self.conv2, self.bn2, x, True)
        g = _block_pool(self.conv3, self.bn3, x, True)
        if _hip_fc(self, g):
            # the FC head on the HIP train kernels (train_hip.fc_bn_act): one launch
            # per layer forward, Linear + BatchNorm's batch statistics + ReLU fused
            from . import train_hip
            g = train_hip.fc_bn_act(self.fc1, self.bn4, g, True)
            g = train_hip.fc_bn_act(self.fc2, self.bn5, g, True)
            t = train_hip.fc_bn_act(self.fc3, None, g, False, eye=self.in_dim)
            return t.view(-1, self.in_dim, self.in_dim)
        g = self.relu(self.bn4(self.fc1(g)))
        g = self.relu(self.bn5(self.fc2(g)))
        t = self.fc3(g) + torch.eye(self.in_dim, device=g.device, dtype=g.dtype).reshape(1, -1)
        return t.view(-1, self.in_dim, self.in_dim)


class NDTNet(nn.Module):
    """Feature extractor (reference ndtnet.py:65-164)."""

    class AdditionalFeatures(Enum):
        NONE = "none"
        COVARIANCES = "covariances"
        FEATURE_VECTOR = "feature_vector"

    def __init__(self, point_dim: int = 3, feature_dim: int = 768,
                 extra_type: "NDTNet.AdditionalFeatures" = AdditionalFeatures.COVARIANCES) -> None:
        super().__init__()
        self.point_dim = point_dim
        self.feature_dim = feature_dim
        extra = {
            NDTNet.AdditionalFeatures.COVARIANCES: point_dim ** 2,
            NDTNet.AdditionalFeatures.FEATURE_VECTOR: feature_dim + point_dim ** 2,
            NDTNet.AdditionalFeatures.NONE: 0,
        }
        self.extra_dim = extra.get(extra_type, 0)
        self.conv1 = _conv(point_dim + self.extra_dim, 64)
        self.conv2 = _conv(64, 128)
        self.conv3 = _conv(128, feature_dim)
        self.bn1, self.bn2, self.bn3 = nn.BatchNorm1d(64), nn.BatchNorm1d(128), nn.BatchNorm1d(feature_dim)
        self.t1 = TNet(in_dim=point_dim)
        self.t2 = TNet(in_dim=64)

    def forward(self, points: torch.Tensor, extra: torch.Tensor, pooled: bool = False):
        """points [B,N,3], extra [B,N,9] -> (features [B,F,N], x_t2 [B,64,N]);
        ``pooled``: (features.amax(dim=2) [B,F], x_t2) -- what the heads use."""
        B, N, _ = points.shape
        d = self.point_dim
        xyz = points.transpose(1, 2)                      # [B,3,N]
        t = self.t1(xyz)                                  # [B,3,3]
        if (extra.shape[-1] == d * d and d == 3 and _hip_train(self.conv1, self.bn1, points)
                and not points.requires_grad and not extra.requires_grad):
            # (HIP train path; the torch composition below stays the reference's op for op)
            from . import train_hip
            x = train_hip.point_transform(t, points, extra)   # t . p and t . C, one launch each way
        elif extra.shape[-1] == d * d and _hip_train(self.conv1, self.bn1, points):
            # t . p and t . C (left only, ndtnet.py:141-147) as ONE bmm per cloud: each point
            # contributes 4 columns (p, C[:, 0], C[:, 1], C[:, 2]) of a [3, 4N] matrix -- torch's
            # batched matmul of 16000 3x3 products costs ~85 us each way on this GPU
            X = torch.cat((points.unsqueeze(-1), extra.reshape(B, N, d, d)), dim=3)  # [B,N,j,4]
            Y = torch.bmm(t, X.permute(0, 2, 1, 3).reshape(B, d, N * (d + 1))).reshape(B, d, N, d + 1)
            x = torch.cat((Y[..., 0], Y[..., 1:].permute(0, 1, 3, 2).reshape(B, d * d, N)), dim=1)  # [B,12,N]
        else:
            xyz = torch.bmm(t, xyz)                           # t . p
            cov = torch.matmul(t.unsqueeze(1), extra.reshape(B, N, d, d)).reshape(B, N, d * d)  # t . C (left only)
            x = torch.cat((xyz.transpose(1, 2), cov), dim=2).transpose(1, 2)  # [B,12,N]
        x = _block(self.conv1, self.bn1, x, False)        # no ReLU (reference ndtnet.py:149)
        t2 = self.t2(x)                                   # [B,64,64]
        if _hip_train(self.conv2, self.bn2, x):
            from . import train_hip
            x = train_hip.transform_t(x, t2)              # x^T t2 on the HIP GEMM (ndtnet.py:153-155)
        else:
            x = torch.bmm(x.transpose(1, 2), t2).transpose(1, 2)  # x^T t2
        x_t2 = x
        x = _block(self.conv2, self.bn2, x, False)
        if pooled:
            return _block_pool(self.conv3, self.bn3, x, False), x_t2
        x = _block(self.conv3, self.bn3, x, False)
        return x, x_t2


class NDTNetClassification(nn.Module):
    """Global classifier head (reference ndtnet.py:166-196)."""

    def __init__(self, point_dim: int = 3, num_classes: int = 512, feature_dim: int = 768) -> None:
        super().__init__()
        self.point_dim, self.num_classes, self.feature_dim = point_dim, num_classes, feature_dim
        self.feature_extractor = NDTNet(point_dim, feature_dim=feature_dim)
        self.conv1, self.conv2, self.conv3 = _conv(feature_dim, 512), _conv(512, 256), _conv(256, num_classes)

    def forward(self, points: torch.Tensor, covariances: torch.Tensor) -> torch.Tensor:
        x, _ = self.feature_extractor(points, covariances)
        x = x.amax(dim=2, keepdim=True)
        x = torch.relu(self.conv1(x))
        x = torch.relu(self.conv2(x))
        return torch.softmax(self.conv3(x), dim=1)


class NDTNetSegmentation(nn.Module):
    """Per-ND segmentation (reference ndtnet.py:198-243): log-probs [B,N,C+1]."""

    def __init__(self, point_dim: int = 3, num_classes: int = 16, feature_dim: int = 1024) -> None:
        super().__init__()
        self.point_dim, self.num_classes, self.feature_dim = point_dim, num_classes, feature_dim
        self.feature_extractor = NDTNet(point_dim, feature_dim=feature_dim)
        self.conv1 = _conv(feature_dim + 64, 512)
        self.conv2 = _conv(512, 256)
        self.conv3 = _conv(256, 128)
        self.conv4 = _conv(128, num_classes + 1)
        self.bn1, self.bn2, self.bn3 = nn.BatchNorm1d(512), nn.BatchNorm1d(256), nn.BatchNorm1d(128)
        self._hip = None  # folded-weight cache of the HIP path

    def forward_torch(self, points: torch.Tensor, covariances: torch.Tensor) -> torch.Tensor:
        hip = _hip_train(self.conv1, self.bn1, points)
        x, x_t2 = self.feature_extractor(points, covariances, pooled=hip)
        blocks = ((self.conv1, self.bn1), (self.conv2, self.bn2), (self.conv3, self.bn3))
        if hip:
            # conv1 over cat(x_t2, g broadcast over the points) (ndtnet.py:230-234) as a 64-channel
            # conv with the global feature's term a per-cloud bias: W[:, 64:] g + b -- 1/13 of the
            # layer's FLOPs forward and backward; the gradient reaches g through the bias
            from . import train_hip
            x = train_hip.seg_conv1(self.conv1, self.bn1, x_t2, x)  # x: the pooled global feature [B,F]
            blocks = blocks[1:]
        else:
            g = x.amax(dim=2, keepdim=True).expand(-1, -1, x_t2.shape[2])
            x = torch.cat((x_t2, g), dim=1)
        for conv, bn in blocks:
            x = _block(conv, bn, x, True)
        x = _block(self.conv4, None, x, False)
        if hip and x.shape[1] <= 32:  # one HIP launch each way (torch's spatial softmax: ~20 us each)
            from . import train_hip
            x = train_hip.log_softmax_c(x)
        else:
            x = torch.nn.functional.log_softmax(x, dim=1)
        return x.transpose(2, 1)

    def _needs_autograd(self, points: torch.Tensor, covariances: torch.Tensor) -> bool:
        """The reference forward is differentiable in eval mode too (frozen-BN
        fine-tuning, saliency): with grad enabled and anything requiring grad,
        the autograd composition runs, not the inference kernels."""
        if not torch.is_grad_enabled():
            return False
        return points.requires_grad or covariances.requires_grad or any(p.requires_grad for p in self.parameters())

    def forward(self, points: torch.Tensor, covariances: torch.Tensor) -> torch.Tensor:
        if (not self.training and points.is_cuda and self.point_dim == 3
                and not self._needs_autograd(points, covariances)):
            # a cuda eval forward IS the HIP path: a missing library raises
            # (ndnet._lib.lib()) instead of silently running the torch composition
            from . import pointnet_hip
            return pointnet_hip.segmentation_forward(self, points, covariances)
        return self.forward_torch(points, covariances)

    def train(self, mode: bool = True):
        # a mode change: weights may change (also inside a replayed training
        # graph, which bumps no tensor versions), so the next eval forward
        # re-folds -- in place, one ndnet_pn_fold_run launch
        # (pointnet_hip._folded); a redundant eval() keeps the fold
        if bool(mode) != self.training and self._hip is not None:
            self._hip["stale"] = True
        return super().train(mode)
