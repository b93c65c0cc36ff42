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
    ap.add_argument("--steps-per-epoch", type=int, default=8, help="synthetic batches per epoch and rank")
    ap.add_argument("--val-steps", type=int, default=2)
    ap.add_argument("--no-save", action="store_true")
    args = ap.parse_args()
    if args.task != "segmentation":
        raise NotImplementedError("only the segmentation task is on the hot path (train.py:122-123)")

    rank, local, world = D.world_from_env()
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    D.init("nccl", dev)
    torch.manual_seed(0)  # identical initial weights on every rank (DDP also broadcasts rank 0's)
    model = NDTNetSegmentation(3, args.n_classes, args.feature_dim)
    tr = Trainer(model, args.learning_rate, args.n_desired_nds, args.n_classes, dev)
    path = os.path.join(args.out_path, datetime.datetime.now().strftime("%Y%m%d_%H%M%S"))

    def run(epoch: int, mode: str, steps: int):
        tot_loss = tot_acc = 0.0
        t0 = time.perf_counter()
        for s in range(steps):
            seed = ((epoch * 1000 + s) * world + rank) * args.batch_size + (0 if mode == "train" else 10 ** 7)
            pts, gt = make_labelled_batch(args.batch_size, args.n_samples, args.n_classes, seed0=seed)
            loss, acc = tr.step(torch.from_numpy(pts), torch.from_numpy(gt), train=mode == "train")
            tot_loss += loss
            tot_acc += acc
            if rank == 0:
                print(f"{mode} epoch {epoch + 1} step {s + 1}/{steps}: loss {loss:.4f} acc {acc:.3f}", flush=True)
        torch.cuda.synchronize()
        dt = D.max_over_ranks(time.perf_counter() - t0)
        return tot_loss / steps, tot_acc / steps, dt

    for epoch in range(args.epochs):
        tr.set_epoch(epoch)
        loss, acc, dt = run(epoch, "train", args.steps_per_epoch)
        if rank == 0:
            print(f"--- epoch {epoch + 1}/{args.epochs}: train loss {loss:.4f} acc {acc:.3f}, "
                  f"{world * args.batch_size * args.steps_per_epoch / dt:.1f} clouds/s over {world} rank(s)")
        vloss, vacc, _ = run(epoch, "val", args.val_steps)
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
