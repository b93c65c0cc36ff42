"""Ingest: the native ASCII-PLY reader and the CARLA_Seg
drop-in against the reference's get_data_pcl restated in oracle/ingest_oracle.py
(CARLA_Seg.py:97-175), on synthetic scans in the CARLA PLY layout (10 header
lines; x y z, extra columns, class tag last).  Host code: runs on the CPU."""
import os

import numpy as np
import pytest
import torch

HEADER = """ply
format ascii 1.0
element vertex {n}
property float32 x
property float32 y
property float32 z
property float32 CosAngle
property uint32 ObjIdx
property uint32 ObjTag
end_header
"""


def _write_scan(path, n, n_classes, seed, fmt="{:.6f}"):
    rng = np.random.default_rng(seed)
    xyz = rng.uniform(-80, 80, (n, 3))
    cos = rng.uniform(-1, 1, n)
    obj = rng.integers(0, 5000, n)
    tag = rng.integers(0, n_classes + 1, n)
    with open(path, "w") as f:
        f.write(HEADER.format(n=n))
        for i in range(n):
            f.write(" ".join(fmt.format(float(v)) for v in xyz[i]) + f" {cos[i]:.6f} {obj[i]} {tag[i]}\n")
    return xyz, tag


def test_native_reader_matches_python_parse(tmp_path):
    from ndnet.datasets.carla_seg import read_ply
    p = tmp_path / "scan.ply"
    _write_scan(p, 20_000, 28, seed=1, fmt="{!r}")  # full double precision tokens
    xyz, cls = read_ply(str(p), 28, threads=4)
    lines = open(p).read().splitlines()[10:]
    ref = np.array([[float(t) for t in ln.split()[:3]] for ln in lines])
    tags = np.array([int(ln.split()[-1]) for ln in lines], np.uint16)
    assert np.array_equal(xyz, ref) and np.array_equal(cls, tags)
    for th in (1, 3, 8):  # range splitting changes nothing
        x2, c2 = read_ply(str(p), 28, threads=th)
        assert np.array_equal(x2, xyz) and np.array_equal(c2, cls)


def test_carla_seg_matches_reference_get_data_pcl(tmp_path):
    import ingest_oracle as O
    from ndnet.datasets import CARLA_Seg
    d = tmp_path / "scans"
    d.mkdir()
    for i in range(3):
        _write_scan(d / f"{i:04d}.ply", 5000 + 97 * i, 28, seed=10 + i)
    ds = CARLA_Seg(28, 4096, str(d))
    assert len(ds) == 3
    for i in range(3):
        np.random.seed(123 + i)
        pts, gt = ds[i]
        np.random.seed(123 + i)
        rp, rg = O.get_data_pcl(os.path.join(str(d), ds.filenames[i]), 28, 4096)
        assert pts.dtype == torch.float32 and gt.shape == (4096, 29)
        assert np.array_equal(pts.numpy(), rp) and np.array_equal(gt.numpy(), rg)
    assert ds.color_to_class(ds.class_to_color(0x12ab34)) == 0x12ab34


def test_reader_errors(tmp_path):
    from ndnet.datasets.carla_seg import read_ply
    p = tmp_path / "bad.ply"
    _write_scan(p, 100, 28, seed=2)
    with pytest.raises(ValueError, match="Class tag"):
        read_ply(str(p), 5)  # tags up to 28 > 5 (CARLA_Seg.py:126-127)
    with open(p, "a") as f:
        f.write("1.0 2.0 abc 0.5 3 4\n")
    with pytest.raises(ValueError, match="Malformed"):
        read_ply(str(p), 28)
    with pytest.raises(FileNotFoundError):
        read_ply(str(tmp_path / "missing.ply"), 28)


def test_carla_seg_matches_reference_run_fixture(tmp_path):
    """ndnet.datasets.CARLA_Seg and the restatement in oracle/ingest_oracle.py
    against the reference's own CARLA_Seg.get_data_pcl, run in the build
    container (tests/golden/make_ingest_golden.py -> ingest_carla_seg.npz):
    identical float32 points and one-hot classes for the same scans and
    np.random seeds, including n_samples == the scan's size (a permutation)."""
    import ingest_oracle as O
    from conftest import golden
    from ndnet.datasets import CARLA_Seg
    z = golden("ingest_carla_seg.npz")
    nc = int(z["n_classes"])
    for i, (n, seed, ns, rs) in enumerate(z["scans"]):
        d = tmp_path / f"s{i}"
        d.mkdir()
        _write_scan(d / "0000.ply", int(n), nc, int(seed))
        ds = CARLA_Seg(nc, int(ns), str(d))
        np.random.seed(int(rs))
        pts, gt = ds[0]
        assert np.array_equal(pts.numpy(), z[f"points_{i}"])
        g = gt.numpy()
        assert g.shape == (int(ns), nc + 1) and (g.sum(axis=1) == 1).all()
        assert np.array_equal(g.argmax(axis=1), z[f"classes_{i}"])
        np.random.seed(int(rs))
        rp, rg = O.get_data_pcl(str(d / "0000.ply"), nc, int(ns))
        assert np.array_equal(rp, z[f"points_{i}"]) and np.array_equal(rg.argmax(axis=1), z[f"classes_{i}"])
