#!/usr/bin/env python3
"""Per-phase time inside k_kl (the one-workgroup-per-cloud insertion-order /
prune / emit kernel) from its s_memrealtime stamps (timing level 2).

    python tools/kl_phases.py [--batch 16 --points 100000 --nds 1000 --kind U]
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

# (from mark, to mark, phase); the event order itself is built before k_kl by
# k_kl_rank_chunks / k_kl_merge (time those with rocprofv3 --kernel-trace)
PHASES = [(0, 1, "zero outputs"), (1, 2, "event count"), (2, 5, "list init"), (5, 6, "first occurrences"),
          (6, 7, "walk scan"), (7, 8, "kills"), (8, 9, "shift"), (9, 10, "rows emitted"), (10, 11, "end")]

ap = argparse.ArgumentParser()
ap.add_argument("--batch", type=int, default=16)
ap.add_argument("--points", type=int, default=100_000)
ap.add_argument("--nds", type=int, default=1000)
ap.add_argument("--kind", default="U")
ap.add_argument("--reps", type=int, default=5)
ap.add_argument("--list-sort", type=int, default=-1, help="ndnet_ndt_debug_set_list_sort form (default: the plan's)")
a = ap.parse_args()
dev = torch.device("cuda", 0)
pts = torch.from_numpy(make_batch(a.kind, a.batch, a.points, seed0=0)).to(dev)
ndt_preprocessing(a.nds, pts)
plan = get_plan(a.batch, a.points, a.nds, -1, dev)
if a.list_sort >= 0:
    _lib.check(_lib.lib().ndnet_ndt_debug_set_list_sort(plan.handle, a.list_sort), "set_list_sort")
_lib.check(_lib.lib().ndnet_ndt_set_timing(plan.handle, 2), "set_timing")
# k_kl_rank_chunks, chunk 0 of each cloud (marks 3, 4, 15); k_kl_merge, workgroup 0 of each cloud
# (marks 12-14): staging, searches; then the gap to k_kl
MPHASES = [(3, 4, "rank: chunk 0 scores"), (4, 15, "rank: scans, rank, writes"), (4, 18, "rank: chunk 0 scores -> last chunk end"), (18, 12, "last rank end -> merge start"),
           (12, 16, "merge: stage runs"), (16, 17, "merge: NaN bases"), (17, 13, "merge: NaN keys"), (13, 14, "merge: searches+writes"), (14, 19, "merge wg 0 end -> last merge end"), (19, 0, "last merge end -> k_kl start")]
if _lib.lib().ndnet_ndt_debug_get_list_sort(plan.handle) == 1:  # k_kl_sort (round 6): its own marks
    MPHASES = MPHASES[:4] + [(12, 16, "sort: load + place runs"), (16, 17, "sort: score-run levels"),
                             (17, 13, "sort: NaN merge + list writes"), (13, 0, "sort end -> prune start")]
acc = np.zeros(len(PHASES))
macc = np.zeros(len(MPHASES))
for _ in range(a.reps):
    ndt_preprocessing(a.nds, pts)
    m = np.zeros(a.batch * 32, np.uint64)
    _lib.check(_lib.lib().ndnet_ndt_debug_kl_marks(plan.handle, m.ctypes.data), "kl_marks")
    m = m.reshape(a.batch, 32).astype(np.float64)
    acc += np.array([((m[:, j] - m[:, i]) * 0.01).mean() for i, j, _ in PHASES])  # 100 MHz ticks -> us
    macc += np.array([((m[:, j] - m[:, i]) * 0.01).mean() for i, j, _ in MPHASES])
_lib.lib().ndnet_ndt_set_timing(plan.handle, 0)
acc /= a.reps
for (_, _, nm), v in zip(PHASES, acc):
    print(f"  {nm:20s} {v:8.2f} us")
print(f"  {'total':20s} {acc.sum():8.2f} us (mean over clouds)")
for (_, _, nm), v in zip(MPHASES, macc / a.reps):
    print(f"  {nm:24s} {v:8.2f} us")
# the event census behind the stages: events, NaN scores, chunks per cloud
st = plan.host_stats()
ev = np.array([s.num_events for s in st])
nds = np.array([s.num_nds for s in st])
nan = []
for b in range(a.batch):
    ne = int(st[b].num_events)  # the dump writes the physical list (num_events entries)
    v = np.zeros(max(ne, 1))
    z = lambda n, t=np.uint32: np.zeros(max(n, 1), t)  # noqa: E731
    p = lambda x: x.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
    n = int(nds[b])
    bufs = [z(n), z(3 * n, np.float64), z(9 * n, np.float64), z(9 * n, np.float64), z(n), v, z(ne), z(ne),
            np.zeros(16), z(16), None, z(n, np.uint8)]
    it = ctypes.c_uint32(0)
    args = [p(x) if x is not None else ctypes.byref(it) for x in bufs]
    _lib.check(_lib.lib().ndnet_ndt_debug_dump(plan.handle, b, *args), "dump")
    nan.append(int(np.isnan(v[:int(st[b].num_kl)]).sum()))
print(f"  events per cloud: mean {ev.mean():.0f} max {ev.max()}; NDs mean {nds.mean():.0f}; "
      f"chunks {int(np.ceil(6 * nds.max() / 256))}; NaN scores in the retained lists: mean {np.mean(nan):.1f} max {max(nan)}")
