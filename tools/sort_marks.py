#!/usr/bin/env python3
"""Per-level stamps of k_kl_sort (timing level 2): thread 0's level end
(marks 20 + 2 l) and the level's barrier (21 + 2 l), from the sort's start
(12) and its staging (16).

    python tools/sort_marks.py [--kind L]
"""
import argparse
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
ap.add_argument("--kind", default="L")
ap.add_argument("--reps", type=int, default=5)
a = ap.parse_args()
dev = torch.device("cuda", 0)
B, n, k = 16, 100_000, 1000
pts = torch.from_numpy(make_batch(a.kind, B, n, seed0=0)).to(dev)
ndt_preprocessing(k, pts)
plan = get_plan(B, n, k, -1, dev)
_lib.check(_lib.lib().ndnet_ndt_debug_set_list_sort(plan.handle, 1), "set_list_sort")  # k_kl_sort at any share
_lib.check(_lib.lib().ndnet_ndt_set_timing(plan.handle, 2), "set_timing")
acc = []
for _ in range(a.reps):
    ndt_preprocessing(k, pts)
    m = np.zeros(B * 32, np.uint64)
    _lib.check(_lib.lib().ndnet_ndt_debug_kl_marks(plan.handle, m.ctypes.data), "kl_marks")
    acc.append(m.reshape(B, 32).astype(np.float64))
m = np.mean(acc, axis=0)
prev = m[:, 16]
print(f"  staging {((m[:, 16] - m[:, 12]) * 0.01).mean():7.2f} us")
for l in range(6):
    e, bar = m[:, 20 + 2 * l], m[:, 21 + 2 * l]
    if not e.any():
        break
    print(f"  level {l}: thread 0 done {((e - prev) * 0.01).mean():6.2f} us, barrier {((bar - e) * 0.01).mean():6.2f} us")
    prev = bar
print(f"  NaN merge + writes {((m[:, 13] - prev) * 0.01).mean():7.2f} us")
