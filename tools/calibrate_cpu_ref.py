#!/usr/bin/env python3
"""Calibrates the reference-structured CPU baseline (oracle/cpu_ref.c) against
the reference's own compiled estimate stage (oracle/_ref: the unmodified
normal_distributions.c / voxel.c / pointclouds.c, -O0, 8 pthreads), build
container only (the reference never travels to the GPU box).

For C2 clouds (U and L, 100k points, k = 1000) it times the 8-thread
estimate at every bisection pass the search runs (the ~60% of the
reference's ndt_downsample that can be compiled here: SURVEY §3.2) through
both, and the whole cpu_ref downsample.  The KL stage has no compilable
reference (GSL absent); cpu_ref restates its call and heap structure.

    python tools/calibrate_cpu_ref.py [--clouds 6] > profiles/r02_cpu_ref_calibration.txt
"""
import argparse
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "oracle"))
sys.path.insert(0, os.path.join(REPO, "ndt-net_amd"))
import oracle as O  # noqa: E402
from ndnet.synthetic import make_batch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--clouds", type=int, default=6)
    a = ap.parse_args()
    assert O.ref_lib() is not None, "oracle/_ref is not built (needs /root/reference)"
    print(f"host: {os.cpu_count()} CPUs; {a.clouds} clouds per kind, 100k points -> 1000 NDs")
    for kind in "UL":
        pts = make_batch(kind, a.clouds, 100_000)
        tr = tc = tw = tor = 0.0
        for b in range(a.clouds):
            p = pts[b].astype(np.float64)
            r = O.run(p, 1000)
            s = r.search
            for g in s.guesses:
                ln = [int(np.ceil((s.lim[i] - s.lim[3 + i]) / g)) for i in range(3)]
                off = s.lim[3:]
                t = time.perf_counter()
                O.ref_estimate(p, g, ln, off, threads=True)
                tr += time.perf_counter() - t
                t = time.perf_counter()
                O.cref_estimate_only(p, g, ln, off)
                tc += time.perf_counter() - t
            t = time.perf_counter()
            _, _, rc = O.cref_downsample(p, 1000)
            tw += time.perf_counter() - t
            assert rc == 0
            t = time.perf_counter()
            O.run(p, 1000)
            tor += time.perf_counter() - t
        m = 1e3 / a.clouds
        print(f"{kind}: search passes (8-thread estimate): reference {tr * m:.1f} ms/cloud, cpu_ref {tc * m:.1f} "
              f"ms/cloud, ratio cpu_ref/reference {tc / tr:.3f}")
        print(f"{kind}: cpu_ref whole ndt_downsample {tw * m:.1f} ms/cloud; oracle (-O2, 1 thread) {tor * m:.1f} "
              f"ms/cloud")


if __name__ == "__main__":
    main()
