"""Two processes, one GPU, each with its own full-chip NDT plan (VERDICT r5
item 6).

The front lanes (csrc/ndt_kernels.hip front_launch) order the k_front
launches of ONE process.  Two processes on one card do not see each other's
lanes, so their share-1 k_front grids (16 x 16 workgroups: the whole chip
each) run at once.  k_front deals a launch's clouds cloud-major within each
XCD (csrc/ndt_front.h), so at any moment at most one cloud per launch and XCD
has only part of its workgroups resident, and two launches leave at most
2 x 15 of an XCD's 32 CUs waiting: every barrier completes.

Each child builds an ``NdtPlan(16, 100k, 1000)`` at CU share 1, warms it,
waits for the parent's go, then enqueues ``RUNS`` back-to-back runs of the C2
batch (U in one child, L in the other) and checks: no barrier timeout
(NDNET_ERR_SYNC, -22) on any run, every cloud rc 0, and the last run's rows
hash-equal the oracle's (tests/golden/fullsize_rows.npz).  The parent checks
that the two children's run windows overlapped, so the case was exercised.
"""
import json
import os
import subprocess
import sys
import time

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
RUNS = 200

CHILD = r"""
import hashlib, json, os, sys, time
import numpy as np
import torch
sys.path.insert(0, os.path.join(sys.argv[1], "ndt-net_amd"))
from ndnet.preprocessing.ndtnet_preprocessing import NdtPlan
from ndnet.synthetic import make_batch
kind, go, ready, runs = sys.argv[2], sys.argv[3], sys.argv[4], int(sys.argv[5])
z = np.load(os.path.join(sys.argv[1], "tests", "golden", "fullsize_rows.npz"))
B, n, k = int(z["batch"]), int(z["points"]), int(z["levels_C2"][0])
plan = NdtPlan(B, n, k, -1)
assert plan.path == 2 and plan.front_lanes[1] == 4, plan.front_lanes   # CU share 1: the whole chip
pts = torch.from_numpy(make_batch(kind, B, n)).cuda()
out = torch.zeros((B, k, 12), dtype=torch.float32, device="cuda")
plan.run(pts, None, out, None)
torch.cuda.synchronize()
open(ready, "w").close()
t_end = time.time() + 600
while not os.path.exists(go):
    assert time.time() < t_end, "no go from the parent"
    time.sleep(0.001)
t0 = time.time()
fails = 0
for i in range(runs):
    plan.run(pts, None, out, None)
    if i % 10 == 9:   # 10 runs in flight at a time; a timeout is flagged in mapped host memory
        torch.cuda.synchronize()
        try:
            plan.raise_sync_failures()
        except Exception:
            fails += 1
            break     # a timed-out barrier costs ~2 s per run: stop at the first
torch.cuda.synchronize()
t1 = time.time()
rcs = [st.rc for st in plan.host_stats()]
rows = out.cpu().numpy()
sha = z[f"C2_{kind}_sha"]
bad = [b for b in range(B) if hashlib.sha256(np.ascontiguousarray(rows[b]).tobytes()).digest() != sha[b, 0].tobytes()]
print(json.dumps({"kind": kind, "t0": t0, "t1": t1, "rcs": rcs, "sync_fails": fails, "bad_clouds": bad}))
"""


@pytest.mark.gpu
def test_two_processes_share_one_gpu(tmp_path):
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    go = str(tmp_path / "go")
    procs = []
    for kind in ("U", "L"):
        ready = str(tmp_path / f"ready_{kind}")
        procs.append((ready, subprocess.Popen([sys.executable, "-c", CHILD, REPO, kind, go, ready, str(RUNS)],
                                              stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, env=env)))
    t_end = time.time() + 300
    while not all(os.path.exists(r) for r, _ in procs):
        for _, p in procs:
            assert p.poll() is None, p.communicate()
        assert time.time() < t_end, "children not ready"
        time.sleep(0.01)
    open(go, "w").close()
    res = []
    for _, p in procs:
        out, err = p.communicate(timeout=300)
        assert p.returncode == 0, err[-3000:]
        res.append(json.loads(out.strip().splitlines()[-1]))
    for r in res:
        assert r["sync_fails"] == 0 and r["rcs"] == [0] * 16, r
        assert r["bad_clouds"] == [], r
    (a0, a1), (b0, b1) = ((r["t0"], r["t1"]) for r in res)
    overlap = min(a1, b1) - max(a0, b0)
    print(f"run windows {a1 - a0:.4f} s / {b1 - b0:.4f} s, overlap {overlap:.4f} s")
    assert overlap > 0.25 * min(a1 - a0, b1 - b0), (a0, a1, b0, b1)
