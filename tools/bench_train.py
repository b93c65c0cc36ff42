#!/usr/bin/env python3
"""The training step of tools/train.py:67-81, timed by stage
on one GPU: labelled NDT on HIP (16 x 100k points -> 1000 NDs, 28 classes,
one-hot) -> NDTNetSegmentation train-mode forward (BatchNorm batch
statistics) -> NLL loss -> backward -> Adam.  The conv blocks' forward and
backward run on the HIP train kernels (include/ndnet_train.h, autograd
Functions of ndnet.models.train_hip); NDNET_TRAIN_PATH=torch runs the torch
composition (MIOpen / hipBLASLt) instead, for the A/B.  The eval forward of
the same batch on the HIP chains is timed beside them.

    python tools/bench_train.py [--steps 20] [--warmup 5] [--batch 16]

Prints one JSON line: ms per stage (HIP events on the step's stream) and
clouds/s of the whole step.
"""
import argparse
import json
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "ndt-net_amd"))
from ndnet.models import pointnet_hip  # noqa: E402
from ndnet.models.ndtnet import NDTNetSegmentation  # noqa: E402
from ndnet.preprocessing.ndtnet_preprocessing import ndt_preprocessing  # noqa: E402
from ndnet.synthetic import make_labelled_batch  # noqa: E402
from ndnet.training import Trainer, segmentation_loss  # noqa: E402

# which train-mode blocks run: the HIP kernels (default) or the torch composition
TRAIN_PATH = "torch" if os.environ.get("NDNET_TRAIN_PATH", "hip").lower() == "torch" else "hip"


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--points", type=int, default=100_000)
    ap.add_argument("--nds", type=int, default=1000)
    ap.add_argument("--classes", type=int, default=28)
    ap.add_argument("--feature-dim", type=int, default=768)
    ap.add_argument("--graph", action="store_true",
                    help="time Trainer(graphs=True): the whole step as one HIP graph replay")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    pts, gt = make_labelled_batch(a.batch, a.points, a.classes, seed0=0)
    pts, gt = torch.from_numpy(pts).to(dev), torch.from_numpy(gt).to(dev)
    model = NDTNetSegmentation(3, a.classes, a.feature_dim)
    if a.graph:
        tr = Trainer(model, 1e-3, a.nds, a.classes, dev, ddp=False, graphs=True)
        # the batch resident in the captured step's own input buffers (as the
        # inference bench's inputs are resident before its timed region): the
        # steps replay without a device-to-device copy of the 204 MB batch
        s_pts, s_gt = tr.graph_inputs(pts.shape, gt.shape)
        s_pts.copy_(pts)
        s_gt.copy_(gt)
        pts, gt = s_pts, s_gt
        for _ in range(a.warmup):
            loss, _ = tr.step_graphed(pts, gt)
        torch.cuda.synchronize()
        st = torch.cuda.current_stream(dev)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(a.steps):
            loss, acc = tr.step_graphed(pts, gt)
        e1.record(st)
        torch.cuda.synchronize()
        step = e0.elapsed_time(e1) / a.steps
        # an eval forward right after a replayed step: re-fold (in place, one launch) + the HIP forward
        pcl, covs, _ = ndt_preprocessing(a.nds, pts, gt, a.classes)
        after = []
        for _ in range(5):
            tr.step_graphed(pts, gt)
            model.eval()
            e2, e3 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e2.record(st)
            with torch.no_grad():
                model(pcl, covs)
            e3.record(st)
            torch.cuda.synchronize()
            after.append(e2.elapsed_time(e3))
        print(json.dumps({"what": "training step (tools/train.py:67-81) as one HIP graph: HIP labelled NDT + "
                                  "train forward/backward + fused capturable Adam", "train_path": TRAIN_PATH,
                          "batch": a.batch,
                          "points": a.points, "nds": a.nds, "classes": a.classes, "F": a.feature_dim,
                          "steps": a.steps, "step_ms": round(step, 4),
                          "clouds_per_s": round(a.batch / step * 1e3, 1), "loss": round(loss.item(), 5),
                          "eval_forward_after_step_ms": round(sorted(after)[len(after) // 2], 4)}))
        return
    tr = Trainer(model, 1e-3, a.nds, a.classes, dev, ddp=False)
    names = ("ndt_labelled", "forward_train", "loss", "backward", "adam", "refold", "forward_eval_hip")
    tot = {n: 0.0 for n in names}
    st = torch.cuda.current_stream(dev)
    for it in range(a.warmup + a.steps):
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(len(names) + 1)]
        ev[0].record(st)
        pcl, covs, g1 = ndt_preprocessing(a.nds, pts, gt, a.classes)
        ev[1].record(st)
        model.train()
        pred = tr.net(pcl, covs)
        ev[2].record(st)
        loss = segmentation_loss(pred, g1)
        ev[3].record(st)
        tr.opt.zero_grad(set_to_none=True)
        loss.backward()
        ev[4].record(st)
        tr.opt.step()
        ev[5].record(st)
        model.eval()
        pointnet_hip._folded(model)  # the re-fold of the updated weights (ndnet_pn_fold_run), else inside the forward
        ev[6].record(st)
        with torch.no_grad():
            model(pcl, covs)
        ev[7].record(st)
        torch.cuda.synchronize()
        if it >= a.warmup:
            for i, n in enumerate(names):
                tot[n] += ev[i].elapsed_time(ev[i + 1])
    ms = {n: round(v / a.steps, 4) for n, v in tot.items()}
    step = sum(v for n, v in ms.items() if n not in ("refold", "forward_eval_hip"))
    print(json.dumps({"what": "training step (tools/train.py:67-81): HIP labelled NDT + train "
                              "forward/backward + Adam", "train_path": TRAIN_PATH, "batch": a.batch,
                      "points": a.points, "nds": a.nds,
                      "classes": a.classes, "F": a.feature_dim, "steps": a.steps, "ms": ms,
                      "step_ms": round(step, 4), "clouds_per_s": round(a.batch / step * 1e3, 1),
                      "train_forward_vs_hip_eval": round(ms["forward_train"] / ms["forward_eval_hip"], 2)}))


if __name__ == "__main__":
    main()
