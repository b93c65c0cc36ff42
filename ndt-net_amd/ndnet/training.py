"""The training step of tools/train.py, on the HIP path.

Reference: tools/train.py:16-92 (run_one_epoch) and :95-208 (driver).  Per
batch: ndt_preprocessing with labels (the labelled NDT path: per-voxel class
histogram + first-max argmax, one-hot of num_classes + 1) -> NDTNetSegmentation
forward in train mode (BatchNorm batch statistics, torch autograd) -> loss ->
backward -> Adam step.  With more than one process the model is wrapped in
DistributedDataParallel: one process per GPU, gradients all-reduced over RCCL
(backend "nccl") in buckets that overlap the backward pass; BatchNorm stays
per-rank (the reference has no SyncBN).  Gradients are 3.37 M fp32 = 13.5 MB
per step at F = 768: ``bucket_cap_mb`` 4 gives four all-reduces, the first
starting while the seg head's backward still runs.

The reference's defects on this path are fixed, not reproduced:
  * the loss: train.py:72 calls cross_entropy(pred [B,N,C+1], gt) -- dim 1
    (points) taken as the class dim -- on log-probabilities; here the NLL of
    the one-hot target over the class dim of the model's log-softmax output;
  * backward/step ran in val/test too (train.py:74-81): only in train mode;
  * loss.item() on a float (train.py:77-78) raised; the LR decay
    ``epoch+1 % 20`` was dead code (train.py:54): halved every 20 epochs.
"""
from __future__ import annotations

from typing import Optional, Tuple

import torch


def segmentation_loss(pred: torch.Tensor, gt: torch.Tensor) -> torch.Tensor:
    """Mean NLL of one-hot ``gt`` [B,N,C+1] under log-probs ``pred`` [B,N,C+1]
    (= cross_entropy over the class dim of the pre-log-softmax logits)."""
    return -(gt * pred).sum(dim=-1).mean()


def accuracy(pred: torch.Tensor, gt: torch.Tensor) -> float:
    """Fraction of NDs whose argmax class matches (train.py:84-87)."""
    return (pred.argmax(dim=-1) == gt.argmax(dim=-1)).float().mean().item()


def lr_for_epoch(base_lr: float, epoch: int) -> float:
    """The intended schedule of train.py:53-57: halve every 20 epochs."""
    return base_lr * 0.5 ** ((epoch + 1) // 20)


class Trainer:
    """One model + Adam (+ DDP when a process group is active)."""

    def __init__(self, model: torch.nn.Module, lr: float, num_nds: int, num_classes: int,
                 device: torch.device, ddp: Optional[bool] = None, bucket_cap_mb: float = 4.0) -> None:
        import torch.distributed as dist
        self.model = model.to(device)
        self.device = device
        self.num_nds, self.num_classes = int(num_nds), int(num_classes)
        self.base_lr = float(lr)
        if ddp is None:
            ddp = dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1
        if ddp:
            from torch.nn.parallel import DistributedDataParallel as DDP
            ids = [device.index if device.index is not None else torch.cuda.current_device()] \
                if device.type == "cuda" else None
            self.net = DDP(self.model, device_ids=ids, bucket_cap_mb=bucket_cap_mb, gradient_as_bucket_view=True)
        else:
            self.net = self.model
        self.opt = torch.optim.Adam(self.model.parameters(), lr=self.base_lr)

    def set_epoch(self, epoch: int) -> None:
        for g in self.opt.param_groups:
            g["lr"] = lr_for_epoch(self.base_lr, epoch)

    def step_on_nds(self, pcl: torch.Tensor, covs: torch.Tensor, gt: torch.Tensor,
                    train: bool = True) -> Tuple[float, float]:
        """Forward (+ backward + Adam step when ``train``) on preprocessed NDs:
        ``pcl`` [B,k,3], ``covs`` [B,k,9], one-hot ``gt`` [B,k,C+1]."""
        if train:
            self.model.train()
            pred = self.net(pcl, covs)
            loss = segmentation_loss(pred, gt)
            self.opt.zero_grad(set_to_none=True)
            loss.backward()
            self.opt.step()
        else:
            self.model.eval()
            with torch.no_grad():
                pred = self.model(pcl, covs)
                loss = segmentation_loss(pred, gt)
        return loss.item(), accuracy(pred.detach(), gt)

    def step(self, points: torch.Tensor, gt_points: torch.Tensor, train: bool = True) -> Tuple[float, float]:
        """One batch of raw clouds: ``points`` [B,n,3], one-hot ``gt_points``
        [B,n,C+1] -> the labelled NDT path on the GPU -> step_on_nds."""
        from .preprocessing.ndtnet_preprocessing import ndt_preprocessing
        pcl, covs, gt = ndt_preprocessing(self.num_nds, points.to(self.device), gt_points.to(self.device),
                                          self.num_classes)
        return self.step_on_nds(pcl, covs, gt, train)
