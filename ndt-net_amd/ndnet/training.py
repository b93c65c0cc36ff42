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
    (= cross_entropy over the class dim of the pre-log-softmax logits).  On the
    GPU, for the model's output (the transposed view of a [B,C+1,N] tensor),
    one HIP reduction and one HIP gradient launch (train_hip.nll_onehot)
    instead of torch's ~8 elementwise / reduce launches."""
    if (pred.is_cuda and gt.is_cuda and pred.dtype == torch.float32 and gt.dtype == torch.float32
            and pred.dim() == 3 and pred.shape == gt.shape and pred.shape[-1] <= 32
            and pred.transpose(1, 2).is_contiguous()
            and gt.is_contiguous()):
        from .models import train_hip
        return train_hip.nll_onehot(pred.transpose(1, 2), gt)
    return -(gt * pred).sum(dim=-1).mean()


class HipAdam(torch.optim.Adam):
    """``torch.optim.Adam(..., capturable=True, fused=True)`` -- the graphed
    step's optimizer -- with the update of every parameter on one HIP launch
    per 32 tensors (``ndnet_tr_adam``, include/ndnet_train.h: torch's fused
    order of operations, the step counts and moments kept in torch's state
    layout, so ``state_dict`` round-trips).  torch's fused kernel took two
    ~46 us launches per step on the 3.37 M parameters (r05p trace).  Falls
    back to torch's own step for anything the kernel does not cover (amsgrad,
    maximize, non-float32 or sparse gradients, a closure)."""

    def __init__(self, params, lr, betas=(0.9, 0.999), eps: float = 1e-8, weight_decay: float = 0.0) -> None:
        super().__init__(params, lr=lr, betas=betas, eps=eps, weight_decay=weight_decay, capturable=True, fused=True)

    @staticmethod
    def _covered(group, ps) -> bool:
        lr = group["lr"]
        return (not group.get("amsgrad") and not group.get("maximize") and not group.get("differentiable")
                and not group.get("decoupled_weight_decay", False)
                and torch.is_tensor(lr) and lr.is_cuda and lr.dtype == torch.float32 and lr.numel() == 1
                and all(p.is_cuda and p.dtype == torch.float32 and p.is_contiguous() and not p.grad.is_sparse
                        and p.grad.dtype == torch.float32 and p.grad.is_contiguous() for p in ps))

    @torch.no_grad()
    def step(self, closure=None):
        if closure is not None:
            return super().step(closure)
        groups = [(g, [p for p in g["params"] if p.grad is not None]) for g in self.param_groups]
        if not all(self._covered(g, ps) for g, ps in groups):
            return super().step()
        import ctypes
        from . import _lib
        for group, ps in groups:
            if not ps:
                continue
            for p in ps:
                st = self.state[p]
                if len(st) == 0:  # torch's capturable fused initial state
                    st["step"] = torch.zeros((), dtype=torch.float32, device=p.device)
                    st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                    st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
            n = len(ps)
            arr = lambda ts: (ctypes.c_void_p * n)(*[t.data_ptr() for t in ts])  # noqa: E731
            b1, b2 = group["betas"]
            rc = _lib.lib().ndnet_tr_adam(
                n, arr(ps), arr([p.grad for p in ps]), arr([self.state[p]["exp_avg"] for p in ps]),
                arr([self.state[p]["exp_avg_sq"] for p in ps]), arr([self.state[p]["step"] for p in ps]),
                (ctypes.c_int64 * n)(*[p.numel() for p in ps]), group["lr"].data_ptr(), float(b1), float(b2),
                float(group["eps"]), float(group["weight_decay"]), torch.cuda.current_stream(ps[0].device).cuda_stream)
            _lib.check(rc, "ndnet_tr_adam")
        return None


def accuracy_tensor(pred: torch.Tensor, gt: torch.Tensor) -> torch.Tensor:
    """Fraction of NDs whose argmax class matches (train.py:84-87), as a 0-d
    tensor on pred's device (no host sync).  On the GPU one HIP kernel
    (ndnet_tr_argmax_match: torch's reduction kernels took ~83 us per argmax)."""
    if (pred.is_cuda and gt.is_cuda and pred.shape == gt.shape and pred.numel() > 0
            and pred.dtype == torch.float32 and gt.dtype == torch.float32):
        # the kernel indexes gt with pred's rows and columns: only for equal shapes
        from . import _lib
        g = gt.contiguous()
        cols = pred.shape[-1]
        rows = pred.numel() // cols
        st = torch.cuda.current_stream().cuda_stream
        if pred.dim() == 3 and cols <= 32 and not pred.is_contiguous() and pred.transpose(1, 2).is_contiguous():
            # the model's [B,N,C] view of its [B,C,N] log-probs: read in place, the
            # fraction written by the kernel's last workgroup
            Bn, N, C = pred.shape
            ctr = torch.zeros(2, device=pred.device, dtype=torch.int32)
            acc = torch.empty((), device=pred.device, dtype=torch.float32)
            _lib.check(_lib.lib().ndnet_tr_argmax_match_cm(pred.data_ptr(), g.data_ptr(), Bn, C, N, ctr.data_ptr(),
                                                           acc.data_ptr(), st), "ndnet_tr_argmax_match_cm")
            return acc
        else:
            cnt = torch.zeros((), device=pred.device, dtype=torch.int32)
            p = pred.contiguous()
            _lib.check(_lib.lib().ndnet_tr_argmax_match(p.data_ptr(), g.data_ptr(), rows, cols, cnt.data_ptr(), st),
                       "ndnet_tr_argmax_match")
        return cnt.float() / rows
    return (pred.argmax(dim=-1) == gt.argmax(dim=-1)).float().mean()


def accuracy(pred: torch.Tensor, gt: torch.Tensor) -> float:
    """Fraction of NDs whose argmax class matches (train.py:84-87)."""
    return accuracy_tensor(pred, gt).item()


def lr_for_epoch(base_lr: float, epoch: int) -> float:
    """The intended schedule of train.py:53-57: halve every 20 epochs."""
    return base_lr * 0.5 ** ((epoch + 1) // 20)


class Trainer:
    """One model + Adam (+ DDP when a process group is active).

    ``graphs=True`` (one GPU, no DDP): ``step`` replays the whole training step
    -- labelled NDT, train forward, loss, backward, Adam -- as one HIP graph per
    input shape (``GraphedTrainStep``).  The optimizer is then Adam's fused,
    capturable form (``HipAdam``: its update on the HIP kernel) with the
    learning rate in a device tensor, so ``set_epoch`` still takes effect
    inside the graph."""

    def __init__(self, model: torch.nn.Module, lr: float, num_nds: int, num_classes: int,
                 device: torch.device, ddp: Optional[bool] = None, bucket_cap_mb: float = 4.0,
                 graphs: bool = False) -> None:
        import torch.distributed as dist
        self.model = model.to(device)
        self.device = device
        self.num_nds, self.num_classes = int(num_nds), int(num_classes)
        self.base_lr = float(lr)
        if ddp is None:
            ddp = dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1
        if graphs and (ddp or device.type != "cuda"):
            raise ValueError("graphs=True needs one GPU and no DDP (the gradient all-reduce is not captured)")
        self.graphs = bool(graphs)
        self._graphed: dict = {}
        if ddp:
            from torch.nn.parallel import DistributedDataParallel as DDP
            ids = [device.index if device.index is not None else torch.cuda.current_device()] \
                if device.type == "cuda" else None
            self.net = DDP(self.model, device_ids=ids, bucket_cap_mb=bucket_cap_mb, gradient_as_bucket_view=True)
        else:
            self.net = self.model
        if self.graphs:
            self.opt = HipAdam(self.model.parameters(), lr=torch.tensor(self.base_lr, device=device))
        else:
            self.opt = torch.optim.Adam(self.model.parameters(), lr=self.base_lr)

    def set_epoch(self, epoch: int) -> None:
        for g in self.opt.param_groups:
            if torch.is_tensor(g["lr"]):
                g["lr"].fill_(lr_for_epoch(self.base_lr, epoch))  # the captured step reads it
            else:
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
        [B,n,C+1] -> the labelled NDT path on the GPU -> step_on_nds (or, with
        ``graphs``, a replay of the captured step)."""
        if train and self.graphs:
            loss, acc = self.step_graphed(points, gt_points)
            return loss.item(), acc.item()
        from .preprocessing.ndtnet_preprocessing import ndt_preprocessing
        pcl, covs, gt = ndt_preprocessing(self.num_nds, points.to(self.device), gt_points.to(self.device),
                                          self.num_classes)
        return self.step_on_nds(pcl, covs, gt, train)

    def _graph_for(self, points_shape, gt_shape) -> "GraphedTrainStep":
        key = (tuple(points_shape), tuple(gt_shape))
        g = self._graphed.get(key)
        if g is None:
            g = self._graphed[key] = GraphedTrainStep(self, points_shape, gt_shape[-1])
        return g

    def step_graphed(self, points: torch.Tensor, gt_points: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
        """A training step as a graph replay; returns (loss, accuracy) as device
        scalars, without synchronising.  Passing the graph's own input buffers
        (``graph_inputs``) skips the copies into them."""
        return self._graph_for(points.shape, gt_points.shape)(points, gt_points)

    def graph_inputs(self, points_shape, gt_shape) -> Tuple[torch.Tensor, torch.Tensor]:
        """The static (points, one-hot gt) buffers the captured step of this
        shape reads: a loader can fill them in place (e.g. a pinned-host copy)
        and pass them to ``step_graphed`` with no device-to-device copy."""
        g = self._graph_for(points_shape, gt_shape)
        return g.s_points, g.s_gt


class GraphedTrainStep:
    """tools/train.py:67-81 for one input shape, captured once and replayed:
    ndt_preprocessing with labels (HIP) -> train-mode forward -> NLL loss ->
    backward -> fused Adam, with the inputs copied into static buffers.

    Capture needs the step's lazy state to exist (cuBLAS-style handles,
    MIOpen's algorithm choices, the gradients and Adam's moments), so a few
    steps run eagerly on a side stream first; the parameters, buffers and
    optimizer state are snapshotted before them and restored after the
    capture, so the first replay is the trainer's first step."""

    def __init__(self, trainer: Trainer, points_shape, gt_width: int, warmup: int = 3) -> None:
        tr = self.tr = trainer
        dev = tr.device
        self.s_points = torch.zeros(tuple(points_shape), dtype=torch.float32, device=dev)
        self.s_gt = torch.zeros(tuple(points_shape[:2]) + (int(gt_width),), dtype=torch.float32, device=dev)
        # a non-degenerate cloud for the warm-up steps (zeros would be one voxel)
        gen = torch.Generator(device=dev).manual_seed(0)
        self.s_points.copy_(torch.rand(self.s_points.shape, device=dev, generator=gen) * 20 - 10)
        self.s_gt[..., 0] = 1.0
        model, opt = tr.model, tr.opt
        with torch.no_grad():
            params = [p.detach().clone() for p in model.parameters()]
            bufs = [b.detach().clone() for b in model.buffers()]
            saved = {p: {k: v.clone() for k, v in st.items() if torch.is_tensor(v)} for p, st in opt.state.items()}
        side = torch.cuda.Stream(dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(side):
            for _ in range(max(1, int(warmup))):
                opt.zero_grad(set_to_none=True)
                self._body()
        torch.cuda.current_stream(dev).wait_stream(side)
        torch.cuda.synchronize(dev)
        opt.zero_grad(set_to_none=True)
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph):
            self.loss, self.acc = self._body()
        with torch.no_grad():
            for p, s in zip(model.parameters(), params):
                p.copy_(s)
            for b, s in zip(model.buffers(), bufs):
                b.copy_(s)
            for p, st in opt.state.items():
                before = saved.get(p, {})
                for k, v in st.items():
                    if torch.is_tensor(v):
                        if k in before:
                            v.copy_(before[k])
                        else:
                            v.zero_()  # a fresh moment / step count
        torch.cuda.synchronize(dev)

    def _body(self):
        from .preprocessing.ndtnet_preprocessing import ndt_preprocessing
        tr = self.tr
        pcl, covs, gt = ndt_preprocessing(tr.num_nds, self.s_points, self.s_gt, tr.num_classes)
        tr.model.train()
        pred = tr.net(pcl, covs)
        loss = segmentation_loss(pred, gt)
        loss.backward()
        tr.opt.step()
        acc = accuracy_tensor(pred.detach(), gt)
        return loss.detach(), acc

    def __call__(self, points: torch.Tensor, gt_points: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
        # the replay does not run Python: flip the mode here, so an eval forward
        # after it re-folds the updated weights (NDTNetSegmentation.train)
        self.tr.model.train()
        if points.data_ptr() != self.s_points.data_ptr():
            self.s_points.copy_(points, non_blocking=True)
        if gt_points.data_ptr() != self.s_gt.data_ptr():
            self.s_gt.copy_(gt_points, non_blocking=True)
        self.graph.replay()
        return self.loss, self.acc
