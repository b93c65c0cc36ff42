#!/usr/bin/env python3
"""Run only the NDTNetSegmentation eval forward (the four k_pn_chain launches
and their per-cloud glue) on synthetic 12-D NDs -- a small driver for
rocprofv3 counter passes on the point-MLP kernel.

    python tools/pn_forward.py [--batch 16 --nds 1000 --reps 5]
"""
import argparse
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "ndt-net_amd"))

from ndnet.models.ndtnet import NDTNetSegmentation  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--batch", type=int, default=16)
ap.add_argument("--nds", type=int, default=1000)
ap.add_argument("--feature-dim", type=int, default=768)
ap.add_argument("--classes", type=int, default=28)
ap.add_argument("--reps", type=int, default=5)
a = ap.parse_args()
dev = torch.device("cuda", 0)
torch.manual_seed(0)
m = NDTNetSegmentation(3, a.classes, a.feature_dim).to(dev).eval()
x = torch.randn(a.batch, a.nds, 12, device=dev)
with torch.no_grad():
    for _ in range(a.reps):
        out = m(x[..., :3], x[..., 3:])
torch.cuda.synchronize()
print("ok", tuple(out.shape), float(out.float().abs().mean()))
