#!/usr/bin/env python3
"""Per-item timing inside k_welford_q (timing level 2 stamps): heavy items
(a whole wave per long ND, wq_heavy) and light items (64 NDs one per lane,
wq_light64; --light-nds 16 for a build with the round-4 lane quads),
cycles per sample of each, the epilogue (neighbours, LU chain, classes), and
which items end last.

    python tools/wq_items.py [--kind L --batch 16 --points 100000 --nds 1000 --heavy 256]
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
from ndnet.preprocessing.ndtnet_preprocessing import NdtPlan  # noqa: E402
from ndnet.synthetic import make_batch  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--batch", type=int, default=16)
ap.add_argument("--points", type=int, default=100_000)
ap.add_argument("--nds", type=int, default=1000)
ap.add_argument("--kind", default="L")
ap.add_argument("--heavy", type=int, default=256)
ap.add_argument("--reps", type=int, default=5)
ap.add_argument("--light-nds", type=int, default=64)
ap.add_argument("--classes", type=int, default=-1, help="labelled run with this many classes (random labels)")
a = ap.parse_args()
dev = torch.device("cuda", 0)
B, n, k = a.batch, a.points, a.nds
pts = torch.from_numpy(make_batch(a.kind, B, n, seed0=0)).to(dev)
plan = NdtPlan(B, n, k, a.classes)
plan.set_heavy_threshold(a.heavy)
out = torch.empty((B, k, 12), dtype=torch.float32, device=dev)
lbl = ocls = None
if a.classes > 0:
    lbl = torch.randint(0, a.classes + 1, (B, n), dtype=torch.int32, device=dev)
    ocls = torch.empty((B, k, a.classes + 1), dtype=torch.float32, device=dev)
plan.run(pts, lbl, out, ocls)
_lib.check(_lib.lib().ndnet_ndt_set_timing(plan.handle, 2), "set_timing")
cap = B * (int(1.2 * k) + 1 + (int(1.2 * k) + 1 + 15) // 16)  # the plan's item capacity (16-ND quads' bound)
m = np.zeros(cap * 8, np.uint64)
items = ctypes.c_uint32(0)
per_sample_h, per_sample_l, epi_h, epi_l, spans, phases, pro_l, loop_l, lbl_l = [], [], [], [], [], [], [], [], []
for r in range(a.reps):
    plan.run(pts, lbl, out, ocls)
    torch.cuda.synchronize()
    st = plan.host_stats()
    L = a.light_nds
    light = sum((s.num_nds + L - 1) // L for s in st if s.rc == 0 or s.num_nds)
    _lib.check(_lib.lib().ndnet_ndt_debug_wq_marks(plan.handle, m.ctypes.data, ctypes.byref(items)), "wq_marks")
    w = m.reshape(-1, 8)
    heavy = int((w[:, 4] >> np.uint64(63)).astype(bool)[: cap].sum())
    # the run's items: heavy first, then light; stale entries past them are ignored
    hv = (w[:, 4] >> np.uint64(63)).astype(bool)
    cnt = ((w[:, 4] >> np.uint64(32)) & np.uint64(0xFFFFFF)).astype(np.int64)
    hwid = (w[:, 4] & np.uint64(0xFFFFFFFF)).astype(np.int64)
    xcc = ((w[:, 4] >> np.uint64(56)) & np.uint64(15)).astype(np.int64)
    rt0 = w[:, 0].astype(np.float64)
    t0, t1, t2 = (w[:, i].astype(np.int64) for i in (1, 2, 3))
    H = int(hv[: cap].sum())
    run = slice(0, H + light)
    hv, cnt, rt0, t0, t1, t2 = hv[run], cnt[run], rt0[run], t0[run], t1[run], t2[run]
    hwid, xcc = hwid[run], xcc[run]
    start = rt0.min()
    end_rt = rt0 + (t2 - t0) / 2.1e9 * 1e8  # approximate: shader clock ~2.1 GHz -> 100 MHz ticks
    spans.append((end_rt.max() - start) * 0.01)
    per_sample_h += list((t1 - t0)[hv] / np.maximum(cnt[hv], 1))
    ph = w[run, 5:8].astype(np.float64)[hv] / np.maximum(cnt[hv], 1)[:, None]
    phases.append(ph)
    per_sample_l += list((t1 - t0)[~hv] / np.maximum(cnt[~hv], 1))
    epi_h += list((t2 - t1)[hv])
    epi_l += list((t2 - t1)[~hv])
    pro_l += list(w[run, 5].astype(np.int64)[~hv])
    loop_l += list(((t1 - t0) - w[run, 5].astype(np.int64))[~hv] / np.maximum(cnt[~hv], 1))
    lbl_l += list(w[run, 6].astype(np.int64)[~hv])
    if r == a.reps - 1:
        order = np.argsort(-(end_rt - start))[:8]
        print(f"items: {H} heavy + {light} light; span ~{spans[-1]:.1f} us (end stamps from the shader clock at 2.1 GHz)")
        print("last-ending items: (heavy, samples of the longest ND, start us, moments cycles, epilogue cycles)")
        for i in order:
            print(f"  {'H' if hv[i] else 'L'} {cnt[i]:5d}  start {(rt0[i] - start) * 0.01:7.2f}  "
                  f"moments {t1[i] - t0[i]:7d}  epilogue {t2[i] - t1[i]:6d}")
        # placement (HW_ID: simd 5:4, cu 11:8, sh 12, se 15:13, tg 19:16; + XCC)
        simd = (hwid >> 4) & 3
        cu_key = (xcc << 8) | (((hwid >> 13) & 7) << 5) | (((hwid >> 12) & 1) << 4) | ((hwid >> 8) & 15)
        simd_key = cu_key * 4 + simd
        tg = (hwid >> 16) & 15
        ncu = len(np.unique(cu_key))
        wgs = {}
        for ck, g in zip(cu_key, tg):
            wgs.setdefault(int(ck), set()).add(int(g))
        per = np.bincount([len(v) for v in wgs.values()])
        print(f"placement: {ncu} CUs used; workgroups per CU histogram {list(per)}")
        end_m = rt0 + (t1 - t0) / 2.1e9 * 1e8
        end_all = end_rt
        share = []
        for i in np.nonzero(hv)[0]:
            same = (simd_key == simd_key[i])
            same[i] = False
            ov = np.clip(np.minimum(end_m[i], end_all[same]) - np.maximum(rt0[i], rt0[same]), 0, None)
            share.append(ov.sum() / max(end_m[i] - rt0[i], 1e-9))
        share = np.array(share) if share else np.zeros(1)
        cps = ((t1 - t0)[hv] / np.maximum(cnt[hv], 1))
        print("heavy items: mean other waves on the same SIMD during the moments: median %.2f p90 %.2f max %.2f"
              % (np.median(share), np.percentile(share, 90), share.max()))
        for lo_, hi_ in ((0, 0.05), (0.05, 0.5), (0.5, 1.0), (1.0, 9.0)):
            sel = (share >= lo_) & (share < hi_)
            if sel.any() and hv.any():
                print(f"  sharing {lo_:.2f}-{hi_:.2f}: {sel.sum():4d} heavy items, cycles/sample median {np.median(cps[sel]):.1f}")
        top = np.argsort(-cnt * hv)[: min(8, int(hv.sum()))]
        for i in top:
            j = list(np.nonzero(hv)[0]).index(i)
            print(f"  heaviest: {cnt[i]:5d} samples, simd {simd[i]}, cu {cu_key[i]:4d}, cycles/sample {(t1[i] - t0[i]) / cnt[i]:.1f}, "
                  f"other waves on SIMD {share[j]:.2f}")
        # CUs still holding a k_welford_q wave over time (a workgroup's CU is
        # released when its last wave ends; items of one wave run back to back)
        cu_end = {}
        for ck, e in zip(cu_key, end_rt):
            cu_end[int(ck)] = max(cu_end.get(int(ck), 0.0), float(e))
        ends = np.array(sorted(cu_end.values()))
        held = [(t_us, int((ends - start > t_us * 100).sum())) for t_us in (20, 30, 40, 50, 60)]
        print("CUs still held after t us: " + ", ".join(f"{t}: {h}" for t, h in held))
        hc = np.sort(cnt[hv])[::-1][:5]
        print(f"heaviest heavy NDs: {list(hc)}; heaviest light group: {cnt[~hv].max() if (~hv).any() else 0}")
_lib.lib().ndnet_ndt_set_timing(plan.handle, 0)
q = lambda v: f"median {np.median(v):.1f} p90 {np.percentile(v, 90):.1f} max {np.max(v):.1f}" if len(v) else "-"  # noqa: E731
print(f"cycles per sample, heavy items: {q(per_sample_h)}")
print(f"cycles per sample (of the group's longest ND), light items: {q(per_sample_l)}")
if pro_l:
    print(f"light items: prologue cycles (item start -> first block) {q(pro_l)}; loop cycles per sample {q(loop_l)}")
    print(f"light items: class histogram cycles (labelled runs) {q(lbl_l)}")
if phases and len(np.concatenate(phases)):
    P = np.concatenate(phases)
    print("heavy items, cycles per sample by phase (median): 0+2 loads/products %.1f, 1 mean recurrence + "
          "ordered sums %.1f" % tuple(np.median(P, axis=0))[:2])
print(f"epilogue cycles, heavy: {q(epi_h)}; light: {q(epi_l)}")
print(f"span us over reps: {[round(s, 1) for s in spans]}")
