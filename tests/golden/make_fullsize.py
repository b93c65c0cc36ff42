#!/usr/bin/env python3
"""Full-size parity fixtures (build container; oracle only, no reference code).

For configs C2 (16 x 100k -> 1000), C5 (16 x 100k -> 2000 -> 1000 -> 500)
and C4 (128 x 100k -> 1000: the 8 rank shards of 16 clouds bench.py --gpus 8
runs, seeds 0..127), U and L clouds (SURVEY §8d generators, cloud i = seed i),
the CPU oracle is run
through the reference ABI sequence NDT_Sampler drives (ndt_legacy.py:111-240)
in three arithmetic variants:

  canonical  portable (correctly rounded) log + GSL 2.7.1 LU_invert -- what
             the HIP kernels compute, bit for bit;
  glibc      glibc's log (what the reference calls, kullback_leibler.c:115)
             + GSL LU_invert;
  columns    portable log + the column-solve inverse (round 1's variant).

Stored per (config, kind, cloud, level): the SHA-256 of the float32 rows
ndt_preprocessing returns ([k,12] after nan_to_num) for the canonical variant,
and for each other variant the number of NDs its kept set has that the
canonical one lacks (rows are compared as sets of float64 means, which are
unique per voxel).  tests/test_ndt_gpu.py::test_fullsize_fixture checks the
HIP rows against the canonical digests; DESIGN.md §4 tabulates the variant
mismatch counts.

Run:  python tests/golden/make_fullsize.py
"""
from __future__ import annotations

import hashlib
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "oracle"))
sys.path.insert(0, os.path.join(REPO, "ndt-net_amd"))

import oracle as O  # noqa: E402
from ndnet.synthetic import make_batch  # noqa: E402

# config -> (NDs per level, clouds)
CONFIGS = {"C2": ((1000,), 16), "C5": ((2000, 1000, 500), 16), "C4": ((1000,), 128)}
VARIANTS = {"canonical": (True, True), "glibc": (False, True), "columns": (True, False)}
N = 100_000


def rows_f32(pc, cov):
    k = pc.shape[0]
    r = np.zeros((k, 12), np.float32)
    r[:, :3] = np.nan_to_num(pc.astype(np.float32), nan=0.0, posinf=0.0, neginf=0.0)
    r[:, 3:] = np.nan_to_num(cov.astype(np.float32), nan=0.0, posinf=0.0, neginf=0.0)
    return r


def chain(pts, levels, portable, gsl):
    O.set_gsl_invert(gsl)
    ch = O.LegacyChain(pts, portable_log=portable)
    out = [ch.downsample(levels[0])]
    assert ch.rc == 0
    out += [ch.prune(k) for k in levels[1:]]
    ch.cleanup()
    O.set_gsl_invert(True)
    return out


def main():
    data = {}
    for cfg, (levels, B) in CONFIGS.items():
        for kind in ("U", "L"):
            pts = make_batch(kind, B, N)
            sha = np.zeros((B, len(levels), 32), np.uint8)
            extra = {v: np.zeros((B, len(levels)), np.int32) for v in VARIANTS if v != "canonical"}
            for b in range(B):
                p64 = pts[b].astype(np.float64)
                res = {v: chain(p64, levels, *VARIANTS[v]) for v in VARIANTS}
                for lv in range(len(levels)):
                    pc, cov = res["canonical"][lv]
                    sha[b, lv] = np.frombuffer(hashlib.sha256(rows_f32(pc, cov).tobytes()).digest(), np.uint8)
                    keep = {tuple(m) for m in pc}
                    for v in extra:
                        extra[v][b, lv] = sum(tuple(m) not in keep for m in res[v][lv][0])
            data[f"{cfg}_{kind}_sha"] = sha
            for v, a in extra.items():
                data[f"{cfg}_{kind}_{v}_extra"] = a
                print(f"{cfg} {kind} {v:8s}: clouds with a different kept set per level "
                      f"{[int((a[:, lv] > 0).sum()) for lv in range(len(levels))]}, "
                      f"NDs differing per level {[int(a[:, lv].sum()) for lv in range(len(levels))]} "
                      f"of {[B * k for k in levels]}")
    np.savez_compressed(os.path.join(HERE, "fullsize_rows.npz"), **data, batch=CONFIGS["C2"][1], points=N,
                        batch_C4=CONFIGS["C4"][1],
                        **{f"levels_{c}": np.array(lv) for c, (lv, _) in CONFIGS.items()})
    print("wrote fullsize_rows.npz")


if __name__ == "__main__":
    main()
