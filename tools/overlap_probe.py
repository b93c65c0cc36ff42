#!/usr/bin/env python3
"""How much of the NDT stage and the PointNet forward can run concurrently:
NDT of batch i+1 on one stream while the forward of batch i runs on another
(both from HIP graphs), against the same work back to back.

    python tools/overlap_probe.py [--reps 20]
"""
import argparse
import os
import sys
import time

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "ndt-net_amd"))
from ndnet.models.ndtnet import NDTNetSegmentation  # noqa: E402
from ndnet.preprocessing.ndtnet_preprocessing import ndt_preprocessing  # noqa: E402
from ndnet.synthetic import make_batch  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--reps", type=int, default=20)
a = ap.parse_args()
dev = torch.device("cuda", 0)
B, n, k = 16, 100_000, 1000
pts = torch.from_numpy(make_batch("U", B, n)).to(dev)
torch.manual_seed(0)
model = NDTNetSegmentation(3, 28, 768).to(dev).eval()
s1, s2 = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
with torch.no_grad():
    p, c, _ = ndt_preprocessing(k, pts)
    rows = torch.cat((p, c), dim=2).contiguous()  # a finished batch for the forward
    for _ in range(2):
        ndt_preprocessing(k, pts)
        model(rows[..., :3], rows[..., 3:])
    torch.cuda.synchronize()
    g_ndt, g_pn = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
    with torch.cuda.stream(s1):
        with torch.cuda.graph(g_ndt, stream=s1):
            ndt_preprocessing(k, pts)
    with torch.cuda.stream(s2):
        with torch.cuda.graph(g_pn, stream=s2):
            model(rows[..., :3], rows[..., 3:])
    torch.cuda.synchronize()

    def timeit(fn):
        fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.reps):
            fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / a.reps * 1e6

    def ndt_only():
        with torch.cuda.stream(s1):
            g_ndt.replay()

    def pn_only():
        with torch.cuda.stream(s2):
            g_pn.replay()

    def serial():
        with torch.cuda.stream(s1):
            g_ndt.replay()
            g_pn.replay()

    def overlapped():
        with torch.cuda.stream(s1):
            g_ndt.replay()
        with torch.cuda.stream(s2):
            g_pn.replay()
        s1.synchronize()
        s2.synchronize()

    t = {f.__name__: timeit(f) for f in (ndt_only, pn_only, serial, overlapped)}
print(" ".join(f"{k_}={v:.1f}us" for k_, v in t.items()))
print(f"overlap gain {t['serial'] / t['overlapped']:.3f}x")
