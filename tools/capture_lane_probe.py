#!/usr/bin/env python3
"""Which form of k_front's front-lane admission survives HIP stream capture
(csrc/ndt_kernels.hip front_launch, NDNET_LANE_CAPTURE 0..4)?  Each mode runs
in a subprocess (a crash in one does not end the probe): capture one plan's
run on a side stream, replay it, compare with the eager run, then two share-1
plans captured on two streams and replayed concurrently (stats rc 0 = no
barrier timeout).

    python tools/capture_lane_probe.py            # every mode
    python tools/capture_lane_probe.py --mode 3   # one mode, in-process
"""
import argparse
import os
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def one(mode: int) -> None:
    os.environ["NDNET_LANE_CAPTURE"] = str(mode)
    sys.path.insert(0, os.path.join(REPO, "ndt-net_amd"))
    import torch
    from ndnet.preprocessing.ndtnet_preprocessing import NdtPlan
    from ndnet.synthetic import make_batch
    B, n, k = 16, 100_000, 1000
    plans, ins, outs, refs = [], [], [], []
    for kind in ("U", "L"):
        p = NdtPlan(B, n, k, -1)
        x = torch.from_numpy(make_batch(kind, B, n)).cuda()
        o = torch.zeros((B, k, 12), device="cuda")
        p.run(x, None, o, None)
        torch.cuda.synchronize()
        plans.append(p), ins.append(x), outs.append(o), refs.append(o.clone())
    import ctypes
    import numpy as np
    from ndnet import _lib
    for p in plans:  # per-workgroup k_front stamps: do the two launches overlap in time?
        _lib.lib().ndnet_ndt_set_timing(p.handle, 2)

    def span(p):
        G = ctypes.c_int(0)
        m = np.zeros(B * 256 * 2, np.uint64)
        _lib.lib().ndnet_ndt_debug_front_wg_marks(p.handle, m.ctypes.data, ctypes.byref(G))
        m = m[: B * G.value * 2].reshape(B, G.value, 2).astype(np.int64)
        return int(m[..., 0].min()), int(m[..., 1].max())

    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    for s in streams:
        s.wait_stream(torch.cuda.current_stream())
    gs = []
    t0 = time.time()
    for i in range(2):
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=streams[i]):
            plans[i].run(ins[i], None, outs[i], None)
        gs.append(g)
    torch.cuda.synchronize()
    print(f"mode {mode}: captured ({time.time() - t0:.2f} s)", flush=True)
    for rnd in range(3):
        for o in outs:
            o.zero_()
        torch.cuda.synchronize()
        t0 = time.time()
        for _ in range(2):
            for i in range(2):
                with torch.cuda.stream(streams[i]):
                    gs[i].replay()
        torch.cuda.synchronize()
        dt = time.time() - t0
        ok = [torch.equal(outs[i], refs[i]) for i in range(2)]
        rcs = [sorted({s.rc for s in p.host_stats()}) for p in plans]
        (a0, a1), (b0, b1) = span(plans[0]), span(plans[1])
        overlap = max(0, min(a1, b1) - max(a0, b0)) * 0.01  # 100 MHz ticks -> us
        print(f"mode {mode}: round {rnd}: {dt * 1e3:.1f} ms, rows equal {ok}, rcs {rcs}, "
              f"k_front spans {(a1 - a0) * 0.01:.1f} / {(b1 - b0) * 0.01:.1f} us, overlap {overlap:.1f} us", flush=True)


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--mode", type=int, default=None)
    ap.add_argument("--modes", type=int, nargs="*", default=None)
    a = ap.parse_args()
    if a.mode is not None:
        one(a.mode)
        return
    for mode in (a.modes or (3, 1, 2, 4, 0)):  # 0 (no admission) last: concurrent share-1 replays may wait out the barrier timeout
        r = subprocess.run([sys.executable, "-u", __file__, "--mode", str(mode)], capture_output=True, text=True,
                           timeout=120)
        tail = (r.stdout + r.stderr).strip().splitlines()[-6:]
        print(f"== mode {mode}: exit {r.returncode}")
        for ln in tail:
            print("   " + ln[:200])


if __name__ == "__main__":
    main()
