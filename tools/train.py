#!/usr/bin/env python3
"""Counterpart of the reference's tools/train.py (segmentation task) on the
HIP path, one process per GPU:

    python tools/train.py --epochs 2 --steps-per-epoch 4
    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 \\
        tools/train.py --epochs 2                      # DDP over RCCL

The CARLA PLY dataset (ndnet/datasets/CARLA_Seg.py) is not available here,
so batches are labelled synthetic L clouds (ndnet.synthetic), a different
seed per rank and step.  Arguments keep the reference's names and defaults
(train.py:97-111) where they apply; the step itself is ndnet.training.Trainer
(its docstring lists the reference defects fixed on the way).  Checkpoints are
saved under the reference's file names (train.py:191-193).
"""
import argparse
import datetime
import os
import sys
import time

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "ndt-net_amd"))

from ndnet import distributed as D  # noqa: E402
from ndnet.models.ndtnet import NDTNetSegmentation  # noqa: E402
from ndnet.synthetic import make_labelled_batch  # noqa: E402
from ndnet.training import Trainer  # noqa: E402


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--task", default="segmentation")
    ap.add_argument("--n_desired_nds", type=int, default=2080)
    ap.add_argument("--n_samples", type=int, default=70000)
    ap.add_argument("--out_path", default="out")
    ap.add_argument("--epochs", type=int, default=200)
    ap.add_argument("--save_every", type=int, default=2)
    ap.add_argument("--batch_size", type=int, default=16)
    ap.add_argument("--learning_rate", type=float, default=0.034)
    ap.add_argument("--n_classes", type=int, default=28)
    ap.add_argument("--feature_dim", type=int, default=768)
    ap.add_argument("--train_path", default=None, help="CARLA PLY scans (ndnet.datasets.CARLA_Seg); synthetic if absent")
    ap.add_argument("--val_path", default=None)
    ap.add_argument("--num_workers", type=int, default=4)
    ap.add_argument("--steps-per-epoch", type=int, default=8, help="synthetic batches per epoch and rank")
    ap.add_argument("--val-steps", type=int, default=2)
    ap.add_argument("--no-save", action="store_true")
    ap.add_argument("--graphs", action="store_true",
                    help="one GPU: replay each training step from a captured HIP graph (Trainer(graphs=True))")
    args = ap.parse_args()
    if args.task != "segmentation":
        raise NotImplementedError("only the segmentation task is on the hot path (train.py:122-123)")

    rank, local, world = D.world_from_env()
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    D.init("nccl", dev)
    torch.manual_seed(0)  # identical initial weights on every rank (DDP also broadcasts rank 0's)
    model = NDTNetSegmentation(3, args.n_classes, args.feature_dim)
    if args.graphs and world > 1:
        raise SystemExit("--graphs runs on one GPU (the DDP all-reduce is not captured)")
    tr = Trainer(model, args.learning_rate, args.n_desired_nds, args.n_classes, dev, graphs=args.graphs)
    path = os.path.join(args.out_path, datetime.datetime.now().strftime("%Y%m%d_%H%M%S"))

    loaders = {}
    if args.train_path:
        from ndnet.datasets.carla_seg import CARLA_Seg, loader
        from torch.utils.data.distributed import DistributedSampler
        for mode, pth in (("train", args.train_path), ("val", args.val_path or args.train_path)):
            ds = CARLA_Seg(args.n_classes, args.n_samples, pth)
            sampler = DistributedSampler(ds, world, rank) if world > 1 else None
            loaders[mode] = torch.utils.data.DataLoader(
                ds, batch_size=args.batch_size, shuffle=sampler is None, sampler=sampler, pin_memory=True,
                num_workers=args.num_workers, drop_last=True) if world > 1 else loader(ds, args.batch_size,
                                                                                     num_workers=args.num_workers)

    def batches(epoch: int, mode: str, steps: int):
        if mode in loaders:  # scans from disk, parsed ahead by the loader's workers
            for pcl, gt in loaders[mode]:
                if pcl.shape[0] > 1:  # train.py:49-51 skips single-cloud batches
                    yield pcl.to(dev, non_blocking=True), gt.to(dev, non_blocking=True)
            return
        for s in range(steps):
            seed = ((epoch * 1000 + s) * world + rank) * args.batch_size + (0 if mode == "train" else 10 ** 7)
            pts, gt = make_labelled_batch(args.batch_size, args.n_samples, args.n_classes, seed0=seed)
            yield torch.from_numpy(pts), torch.from_numpy(gt)

    def run(epoch: int, mode: str, steps: int):
        tot_loss = tot_acc = 0.0
        t0 = time.perf_counter()
        s = -1
        for s, (pts, gt) in enumerate(batches(epoch, mode, steps)):
            loss, acc = tr.step(pts, gt, train=mode == "train")
            tot_loss += loss
            tot_acc += acc
            if rank == 0:
                print(f"{mode} epoch {epoch + 1} step {s + 1}/{steps}: loss {loss:.4f} acc {acc:.3f}", flush=True)
        torch.cuda.synchronize()
        dt = D.max_over_ranks(time.perf_counter() - t0)
        n = max(s + 1, 1)
        return tot_loss / n, tot_acc / n, dt, n

    for epoch in range(args.epochs):
        tr.set_epoch(epoch)
        for ld in loaders.values():
            if isinstance(getattr(ld, "sampler", None), torch.utils.data.distributed.DistributedSampler):
                ld.sampler.set_epoch(epoch)
        loss, acc, dt, nb = run(epoch, "train", args.steps_per_epoch)
        if rank == 0:
            print(f"--- epoch {epoch + 1}/{args.epochs}: train loss {loss:.4f} acc {acc:.3f}, "
                  f"{world * args.batch_size * nb / dt:.1f} clouds/s over {world} rank(s)")
        vloss, vacc, _, _ = run(epoch, "val", args.val_steps)
        if rank == 0:
            print(f"--- epoch {epoch + 1}: val loss {vloss:.4f} acc {vacc:.3f}")
        if rank == 0 and not args.no_save and (epoch + 1) % args.save_every == 0:
            os.makedirs(path, exist_ok=True)
            torch.save(model.state_dict(), f"{path}/ndtnet_{args.task}_full_{epoch + 1}.pth")
            torch.save(model.feature_extractor.state_dict(), f"{path}/ndtnet_{args.task}_backbone_{epoch + 1}.pth")
    if torch.distributed.is_initialized():
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
