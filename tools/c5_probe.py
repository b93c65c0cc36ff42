#!/usr/bin/env python3
"""Why the C5 pipeline runs slower as bench.py's --levels main line than as
the default run's config line: times the multiscale pipeline built first,
then after a k = 1000 pipeline, in one process.

    python tools/c5_probe.py [--steps 50] [--order c5,u,c5]
"""
import argparse
import os
import sys
import time

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "ndt-net_amd"))
from ndnet.models.ndtnet import NDTNetSegmentation  # noqa: E402
from ndnet.pipeline import PipelinedSegmentation  # noqa: E402
from ndnet.synthetic import make_batch  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--steps", type=int, default=50)
ap.add_argument("--order", default="c5,u,c5new,c5")
a = ap.parse_args()
dev = torch.device("cuda", 0)
B, n = 16, 100_000
pts = torch.from_numpy(make_batch("U", B, n)).to(dev)
torch.manual_seed(1234)
model = NDTNetSegmentation(3, 28, 768).to(dev).eval()
with torch.no_grad():
    for m in model.modules():
        if isinstance(m, torch.nn.BatchNorm1d):
            m.running_mean.uniform_(-0.2, 0.2)
            m.running_var.uniform_(0.5, 1.5)


def timed(p, steps):
    with torch.no_grad():
        t = time.perf_counter()
        while time.perf_counter() - t < 0.2:
            p.replay_steps(12)
            torch.cuda.synchronize()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        p.replay_steps(steps)
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / steps * 1e3


pipes = {}
for name in a.order.split(","):
    if name == "c5new" or name not in pipes:
        key = "c5" if name.startswith("c5") else "u"
        levels = (2000, 1000, 500) if key == "c5" else None
        k = 2000 if key == "c5" else 1000
        p = PipelinedSegmentation(model, k, B, n, device=dev, levels=levels)
        p.load_resident(pts)
        pipes[name] = p
        if name == "c5new":
            pipes["c5"] = p
    p = pipes["c5" if name.startswith("c5") else name]
    print(f"{name:6s} {timed(p, a.steps):.4f} ms/step", flush=True)
