#!/usr/bin/env python3
"""Generate tests/golden/ingest_carla_seg.npz from the reference's own
CARLA_Seg.get_data_pcl (ndnet/datasets/CARLA_Seg.py:97-175), build container
only.

The reference module is imported from /root/reference (nothing is copied).
Its top-level ``import open3d as o3d`` (CARLA_Seg.py:4) is bound to an empty
module: open3d is absent here and get_data_pcl never calls it (its only use is
inside a string literal, :150-166).  Its ``from ndnet.preprocessing.ndt_legacy
import NDT_Sampler`` resolves to the reference's own module, whose hard-coded
libndnet.so load is redirected to an inert stand-in (make_golden.py's
load_reference): the dataset never calls it either.

Inputs: synthetic scans in the CARLA PLY layout written by
tests/test_ingest.py's _write_scan (deterministic, so the test rewrites the
same files); outputs: the points and the class of every one-hot row the
reference returns for ``np.random.seed(s)`` before each __getitem__.

Run:  python tests/golden/make_ingest_golden.py
"""
from __future__ import annotations

import importlib.util
import os
import sys
import tempfile
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(REPO, "tests"))

from make_golden import REF_ROOT, load_reference  # noqa: E402
from test_ingest import _write_scan  # noqa: E402

# (points in the scan, seed of the scan, n_samples, np.random seed), 28 classes
SCANS = [(3000, 40, 1024, 7), (2500, 41, 2500, 8), (4097, 42, 1000, 9)]
N_CLASSES = 28


def reference_carla_seg():
    sys.modules.setdefault("open3d", types.ModuleType("open3d"))  # imported, unused on the path
    load_reference()  # refndnet, libndnet.so load inert
    saved = {k: sys.modules.get(k) for k in ("ndnet", "ndnet.preprocessing", "ndnet.preprocessing.ndt_legacy")}
    sys.modules["ndnet"] = sys.modules["refndnet"]
    sys.modules["ndnet.preprocessing"] = sys.modules["refndnet.preprocessing"]
    sys.modules["ndnet.preprocessing.ndt_legacy"] = sys.modules["refndnet.preprocessing.ndt_legacy"]
    try:
        spec = importlib.util.spec_from_file_location("ref_carla_seg", f"{REF_ROOT}/ndnet/datasets/CARLA_Seg.py")
        mod = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(mod)
    finally:
        for k, v in saved.items():
            if v is None:
                sys.modules.pop(k, None)
            else:
                sys.modules[k] = v
    return mod.CARLA_Seg


def main() -> None:
    CARLA_Seg = reference_carla_seg()
    out = {}
    with tempfile.TemporaryDirectory() as d:
        for i, (n, seed, ns, rs) in enumerate(SCANS):
            sub = os.path.join(d, f"s{i}")
            os.mkdir(sub)
            _write_scan(os.path.join(sub, "0000.ply"), n, N_CLASSES, seed)
            ds = CARLA_Seg(N_CLASSES, ns, sub)
            np.random.seed(rs)
            pts, gt = ds[0]
            g = gt.numpy()
            assert (g.sum(axis=1) == 1).all()
            out[f"points_{i}"] = pts.numpy()
            out[f"classes_{i}"] = g.argmax(axis=1).astype(np.uint16)
    out["scans"] = np.array(SCANS, np.int64)
    out["n_classes"] = np.array(N_CLASSES)
    np.savez_compressed(os.path.join(HERE, "ingest_carla_seg.npz"), **out)
    print("wrote ingest_carla_seg.npz", {k: v.shape for k, v in out.items()})


if __name__ == "__main__":
    main()
