#!/usr/bin/env python3
"""Where a k_pn_chain launch spends its time, layer by layer, from in-kernel
s_memrealtime stamps (a -DNDNET_PN_STAMPS build: NDNET_AMD_LIB=.../libndnet_amd_stamps.so).

Runs each of the four chains of a C3 forward (16 x 1000 points) alone, after
a warm-up forward, and prints per chain: the spread of the workgroups' start
times (dispatch), the median and max per-phase time over workgroups, and the
launch span (first start to last end).

    NDNET_AMD_LIB=ndt-net_amd/lib/variants/libndnet_amd_stamps.so python tools/pn_stamps.py
"""
import argparse
import ctypes
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "ndt-net_amd"))
from ndnet import _lib  # noqa: E402
from ndnet.models import pointnet_hip as ph  # noqa: E402
from ndnet.models.ndtnet import NDTNetSegmentation  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--batch", type=int, default=16)
ap.add_argument("--points", type=int, default=1000)
ap.add_argument("--reps", type=int, default=5)
ap.add_argument("--cold", action="store_true", help="evict L2 (a 64 MB write) before each timed launch")
a = ap.parse_args()
dev = torch.device("cuda", 0)
B, n = a.batch, a.points
torch.manual_seed(0)
model = NDTNetSegmentation(3, 28, 768).to(dev).eval()
x = torch.randn(B, n, 12, device=dev)
with torch.no_grad():
    model(x[..., :3], x[..., 3:])
    torch.cuda.synchronize()
cache = ph._folded(model)
ws = cache["ws"][(B, n, dev, 0)]
tiles = (n + 63) // 64
wgs = B * tiles
buf = np.zeros((wgs, 16), np.uint64)
junk = torch.empty(16 << 20, device=dev)
for i, name in enumerate(ph.CHAIN_NAMES):
    spans, phases = [], []
    for _ in range(a.reps):
        if a.cold:
            junk.fill_(1.0)
        torch.cuda.synchronize()
        buf[:] = 0
        _lib.lib().ndnet_pn_debug_stamps_clear()
        out = torch.empty((B, n, 29), device=dev) if i == 3 else None
        with torch.no_grad():
            ws.chain(i, x, out=out)
        torch.cuda.synchronize()
        rc = _lib.lib().ndnet_pn_debug_stamps(buf.ctypes.data, wgs)
        if rc != 0:
            sys.exit(f"ndnet_pn_debug_stamps rc {rc}: run with a -DNDNET_PN_STAMPS build (NDNET_AMD_LIB)")
        s = buf.astype(np.int64)
        t0 = s[:, 0].min()
        spans.append((s[:, 15].max() - t0) * 10e-3)
        idx = [j for j in range(16) if (s[:, j] > 0).all()]  # stamps this launch wrote
        phases.append((idx, s[:, idx] - t0))
    idx, rel = phases[-1]
    print(f"chain {name}: launch span median {np.median(spans):.2f} us (first start -> last end, reps {a.reps})")
    st = rel[:, 0] * 10e-3
    print(f"  start skew: median {np.median(st):.2f} us, max {st.max():.2f} us")
    labels = {0: "start", 1: "t2 fold" if name.startswith("C") else "head prologue", 2: "input tile", 15: "end"}
    for p, q in zip(idx, idx[1:]):
        d = (rel[:, idx.index(q)] - rel[:, idx.index(p)]) * 10e-3
        lab = labels.get(q, f"layer {q - 3}")
        print(f"  {lab:14s} median {np.median(d):7.2f} us  max {d.max():7.2f} us")
