#!/usr/bin/env python3
"""Per-phase time inside k_front (limits, bisection passes, dense ids,
binning) from workgroup 0's s_memrealtime stamps (timing level 2).

    python tools/front_phases.py [--batch 16 --points 100000 --nds 1000 --kind U]
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
from ndnet.preprocessing.ndtnet_preprocessing import ndt_preprocessing, get_plan  # noqa: E402
from ndnet.synthetic import make_batch  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--batch", type=int, default=16)
ap.add_argument("--points", type=int, default=100_000)
ap.add_argument("--nds", type=int, default=1000)
ap.add_argument("--kind", default="U")
ap.add_argument("--reps", type=int, default=5)
ap.add_argument("--share", type=int, default=1, help="CU share of the NDT stage (the pipeline's is 2)")
a = ap.parse_args()
dev = torch.device("cuda", 0)
pts = torch.from_numpy(make_batch(a.kind, a.batch, a.points, seed0=0)).to(dev)
ndt_preprocessing(a.nds, pts)
plan = get_plan(a.batch, a.points, a.nds, -1, dev)
if a.share > 1:
    from ndnet.pipeline import PIPE_WQ_SHARE  # noqa: E402
    plan.set_cu_share(a.share, PIPE_WQ_SHARE)
    ndt_preprocessing(a.nds, pts)
_lib.check(_lib.lib().ndnet_ndt_set_timing(plan.handle, 2), "set_timing")
names = {0: "start", 1: "limits in", 2: "limits out", 20: "accepted", 21: "dense ids", 22: "point NDs",
         23: "offsets in", 24: "offsets out", 25: "offsets", 26: "scattered"}
names.update({19: "p1 grid (thread 0)", 27: "p1 loop top", 28: "p1 keys", 29: "p1 atomics", 30: "p1 sum", 31: "p1 counts read"})
if os.environ.get("NDNET_FRONT_BINMARKS"):
    names.update({27: "ranks done (wave 0)", 28: "ranks barrier", 29: "nd prefix done"})
    for i in (30, 31):
        names.pop(i)
for p in range(8):
    names[3 + 2 * p] = f"pass {p} in"
    names[4 + 2 * p] = f"pass {p} out"
acc = np.zeros(32)
for _ in range(a.reps):
    ndt_preprocessing(a.nds, pts)
    m = np.zeros(a.batch * 32, np.uint64)
    _lib.check(_lib.lib().ndnet_ndt_debug_front_marks(plan.handle, m.ctypes.data), "front_marks")
    m = m.reshape(a.batch, 32).astype(np.float64)
    valid = m > 0
    rel = (m - m[:, :1]) * 0.01  # 100 MHz ticks -> us
    acc += np.where(valid, rel, np.nan).mean(axis=0)
G = ctypes.c_int(0)
wgm = np.zeros(a.batch * 256 * 2, np.uint64)
_lib.check(_lib.lib().ndnet_ndt_debug_front_wg_marks(plan.handle, wgm.ctypes.data, ctypes.byref(G)), "wg_marks")
_lib.lib().ndnet_ndt_set_timing(plan.handle, 0)
acc /= a.reps
wg = wgm[: a.batch * G.value * 2].reshape(a.batch * G.value, 2).astype(np.float64)
t0 = wg[:, 0].min()
print(f"k_front workgroups ({a.batch} x {G.value}, last run): start skew {(wg[:, 0].max() - t0) * 0.01:.2f} us, "
      f"first end {(wg[:, 1].min() - t0) * 0.01:.2f} us, last end {(wg[:, 1].max() - t0) * 0.01:.2f} us "
      f"(from the first workgroup's start)")
prev = 0.0
for i in sorted(names, key=lambda i: acc[i] if np.isfinite(acc[i]) else 1e9):
    if np.isfinite(acc[i]):
        print(f"  {i:2d} {names[i]:12s} {acc[i]:8.2f} us  (+{acc[i] - prev:6.2f})")
        prev = acc[i]

