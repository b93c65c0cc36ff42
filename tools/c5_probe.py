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
ap.add_argument("--stages", action="store_true", help="also time each stage graph alone")
ap.add_argument("--prewarm", action="store_true", help="eager forwards of every level size in every workspace slot first")
ap.add_argument("--pre-plans", type=int, default=0, help="NdtPlans of the C5 shape created (and kept) before the pipelines")
ap.add_argument("--pre-graph", action="store_true", help="capture and replay a trivial graph before the pipelines")
ap.add_argument("--pre-alloc-mb", type=int, default=0, help="a device buffer allocated (and kept) before the pipelines")
ap.add_argument("--pre-streams", type=int, default=0, help="torch streams taken from the pool before the pipelines")
ap.add_argument("--order", default="c5,u,c5new,c5:old,c5b,c5b:old")
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
        torch.arange(7, device=dev).flip(0)  # a marker kernel between windows (tools/trace_windows.py)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        p.replay_steps(steps)
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / steps * 1e3


pre = [torch.cuda.Stream(device=dev) for _ in range(a.pre_streams)]
pre_buf = torch.empty(a.pre_alloc_mb << 20, dtype=torch.uint8, device=dev) if a.pre_alloc_mb else None
if a.pre_graph:
    xg = torch.zeros(16, device=dev)
    sg = torch.cuda.Stream(device=dev)
    sg.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(sg):
        xg.add_(1)
    torch.cuda.synchronize()
    g0 = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g0, stream=sg):
        xg.add_(1)
    g0.replay()
    torch.cuda.synchronize()
from ndnet.preprocessing.ndtnet_preprocessing import NdtPlan  # noqa: E402
pre_plans = [NdtPlan(B, n, 2000, -1, device=dev) for _ in range(a.pre_plans)]
if a.prewarm:
    from ndnet.models import pointnet_hip
    with torch.no_grad():
        for slot in range(3):
            for kk in (2000, 1000, 500):
                r = torch.randn(B, kk, 12, device=dev) * 0.1
                with pointnet_hip.workspace_slot(slot):
                    model(r[..., :3], r[..., 3:])
    torch.cuda.synchronize()
pipes = {}  # by name: c5 / c5new build a multiscale pipeline, u a k = 1000 one; "name:old" re-times one built earlier
for name in a.order.split(","):
    if name.endswith(":old"):
        p = pipes[name[:-4]]
    else:
        key = "c5" if name.startswith("c5") else "u"
        levels = (2000, 1000, 500) if key == "c5" else None
        p = PipelinedSegmentation(model, 2000 if key == "c5" else 1000, B, n, device=dev, levels=levels)
        p.load_resident(pts)
        pipes[name] = p
    print(f"{name:8s} {timed(p, a.steps):.4f} ms/step", flush=True)
    if a.stages:  # each stage's graph alone, back to back on its stream
        for kind, gs, sts in (("ndt", p.g_ndt, p.s_ndts), ("fwd", p.g_fwd, p.s_fwds)):
            st = sts[0]
            st.wait_stream(torch.cuda.current_stream(dev))
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            with torch.cuda.stream(st):
                for _ in range(a.steps):
                    gs[0].replay()
            torch.cuda.synchronize()
            print(f"   {kind} graph alone {(time.perf_counter() - t0) / a.steps * 1e3:.4f} ms", flush=True)
