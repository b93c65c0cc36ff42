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

# per-chain HIP-event times (bench.py's roofline figures) over a few more reps
from ndnet.models import pointnet_hip  # noqa: E402
import numpy as np  # noqa: E402
sys.path.insert(0, REPO)
from bench import chain_flops_per_point  # noqa: E402
pointnet_hip.chain_timing = []
with torch.no_grad():
    for _ in range(a.reps):
        m(x[..., :3], x[..., 3:])
torch.cuda.synchronize()
ms = np.zeros(4)
for i, e0, e1 in pointnet_hip.chain_timing:
    ms[i] += e0.elapsed_time(e1) / a.reps
fl = np.array(chain_flops_per_point(a.feature_dim, a.classes)) * a.nds * a.batch
for i in range(4):
    print(f"chain {pointnet_hip.CHAIN_NAMES[i][:40]:40s} {ms[i] * 1e3:7.1f} us  {fl[i] / (ms[i] * 1e-3) / 1e12:6.1f} TFLOP/s")
