"""CARLA semantic-segmentation scans (ingest), drop-in for
the reference's ndnet/datasets/CARLA_Seg.py:9-175 without open3d.

``get_data_pcl`` parses the ASCII PLY with the native multi-threaded reader
(``ndnet_ply_read``, include/ndnet_ingest.h) instead of readlines + split +
float() per token, then does what the reference does: a random subsample of
``n_samples`` points without replacement on numpy's global RNG
(``np.random.choice``, CARLA_Seg.py:137-138, unseeded there too), float32
points, and a one-hot ``[n_samples, n_classes + 1]`` ground truth.  For the
same RNG state it returns the reference's tensors exactly
(tests/test_ingest.py against oracle/ingest_oracle.py).

``loader()`` pipelines ingest with the GPU: DataLoader worker processes parse
scans while the GPU runs the previous batch, into pinned host memory
(train.py:134-137 uses 4 workers + pin_memory), and the H2D copy is
non-blocking.
"""
from __future__ import annotations

import ctypes
import os
from typing import List, Tuple

import numpy as np
import torch
from torch.utils.data import Dataset

from .. import _lib


def read_ply(path: str, num_classes: int, num_header_lines: int = 10, threads: int = 0) -> Tuple[np.ndarray, np.ndarray]:
    """(xyz [n, 3] float64, class tags [n] uint16) of an ASCII PLY scan."""
    lib = _lib.lib()
    bpath = os.fsencode(path)
    n = ctypes.c_uint64(0)
    rc = lib.ndnet_ply_count(bpath, num_header_lines, ctypes.byref(n))
    if rc == -30:
        raise FileNotFoundError(path)
    _lib.check(rc, "ndnet_ply_count")
    xyz = np.empty((n.value, 3), np.float64)
    cls = np.empty(n.value, np.uint16)
    rc = lib.ndnet_ply_read(bpath, num_header_lines, int(num_classes), xyz.ctypes.data, cls.ctypes.data,
                            n.value, ctypes.byref(n), int(threads))
    if rc == -32:
        raise ValueError(f"Class tag out of bounds on data line {n.value} of {path}")
    if rc == -31:
        raise ValueError(f"Malformed data line {n.value} of {path}")
    _lib.check(rc, "ndnet_ply_read")
    return xyz, cls


class CARLA_Seg(Dataset):
    """Same constructor, methods and outputs as the reference's CARLA_Seg."""

    def __init__(self, n_classes: int, n_samples: int, path: str) -> None:
        super().__init__()
        self.n_classes: int = n_classes
        self.n_samples = n_samples
        self.path: str = path
        if not os.path.exists(self.path):
            raise FileNotFoundError(f"Dataset not found at {self.path}")
        self.filenames: List[str] = sorted(os.listdir(self.path))

    def __len__(self) -> int:
        return len(self.filenames)

    def __getitem__(self, idx: int) -> Tuple[torch.Tensor, torch.Tensor]:
        if idx < 0 or idx >= len(self.filenames):
            raise IndexError(f"Index {idx} out of bounds")
        return self.get_data_pcl(os.path.join(self.path, self.filenames[idx]))

    def color_to_class(self, color: np.ndarray) -> int:
        """RGB in [0, 1] -> 24-bit tag (CARLA_Seg.py:58-74)."""
        c = (np.asarray(color) * 255).astype(np.uint8)
        return int(c[0]) << 16 | int(c[1]) << 8 | int(c[2])

    def class_to_color(self, class_tag: int) -> np.ndarray:
        """24-bit tag -> RGB in [0, 1] (CARLA_Seg.py:76-94)."""
        return np.array([(class_tag >> 16) & 0xff, (class_tag >> 8) & 0xff, class_tag & 0xff], np.float32) / 255.0

    def get_data_pcl(self, pcl_filename: str, num_header_lines: int = 10, threads: int = 0):
        xyz, cls = read_ply(pcl_filename, self.n_classes, num_header_lines, threads)
        idx = np.random.choice(xyz.shape[0], self.n_samples, replace=False)  # CARLA_Seg.py:137-138
        points = torch.from_numpy(xyz[idx]).float()
        gt = torch.zeros((self.n_samples, self.n_classes + 1), dtype=torch.float32)
        gt[torch.arange(self.n_samples), torch.from_numpy(cls[idx].astype(np.int64))] = 1.0
        return points, gt


def loader(dataset: Dataset, batch_size: int, shuffle: bool = True, num_workers: int = 4):
    """DataLoader as train.py:134-137 builds it: worker processes parse ahead
    of the GPU, batches land in pinned memory for non-blocking H2D copies."""
    return torch.utils.data.DataLoader(dataset, batch_size=batch_size, shuffle=shuffle, pin_memory=True,
                                       num_workers=num_workers, persistent_workers=num_workers > 0)
