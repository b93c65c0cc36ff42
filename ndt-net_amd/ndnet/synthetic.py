"""Synthetic point clouds of SURVEY §8(d).

The reference trains on CARLA PLY scans (ndnet/datasets/CARLA_Seg.py), which
are not available here; benchmarks and parity fixtures use these two seeded
generators instead.  Canonical clouds are float32, as CARLA_Seg yields
(CARLA_Seg.py:168); the NDT core consumes float64(float32)
(ndtnet_preprocessing.py:30).
"""
from __future__ import annotations

import numpy as np


def uniform_cloud(n: int, seed: int) -> np.ndarray:
    """U: uniform cube [-10, 10)^3."""
    rng = np.random.default_rng(seed=seed)
    return rng.uniform(-10.0, 10.0, (n, 3)).astype(np.float32)


def lidar_cloud(n: int, seed: int) -> np.ndarray:
    """L: a flat ground patch plus 20 vertical object clusters."""
    rng = np.random.default_rng(seed=seed)
    ng = int(0.6 * n)
    ground = np.c_[rng.uniform(-40, 40, ng), rng.uniform(-40, 40, ng), rng.normal(-1.7, 0.05, ng)]
    c = rng.uniform(-35, 35, (20, 2))
    idx = rng.integers(0, 20, n - ng)
    objects = np.c_[c[idx] + rng.normal(0, 1.0, (n - ng, 2)), rng.uniform(-1.7, 1.5, n - ng)]
    return np.r_[ground, objects].astype(np.float32)


def make_batch(kind: str, batch: int, n: int, seed0: int = 0) -> np.ndarray:
    """[batch, n, 3] float32; cloud i uses seed seed0 + i."""
    gen = {"U": uniform_cloud, "L": lidar_cloud}[kind]
    return np.stack([gen(n, seed0 + i) for i in range(batch)])


def lidar_cloud_labelled(n: int, seed: int, num_classes: int):
    """L cloud plus per-point labels in [0, num_classes]: 0 for the ground,
    1 + (cluster % num_classes) for the object clusters.  Returns
    (points [n, 3] float32, one-hot [n, num_classes + 1] float32) -- the pair
    CARLA_Seg yields (CARLA_Seg.py:39-56) -- for the training step."""
    if num_classes < 1:
        raise ValueError("num_classes must be >= 1")
    rng = np.random.default_rng(seed=seed)
    ng = int(0.6 * n)
    ground = np.c_[rng.uniform(-40, 40, ng), rng.uniform(-40, 40, ng), rng.normal(-1.7, 0.05, ng)]
    c = rng.uniform(-35, 35, (20, 2))
    idx = rng.integers(0, 20, n - ng)
    objects = np.c_[c[idx] + rng.normal(0, 1.0, (n - ng, 2)), rng.uniform(-1.7, 1.5, n - ng)]
    pts = np.r_[ground, objects].astype(np.float32)
    lbl = np.r_[np.zeros(ng, np.int64), 1 + idx % num_classes]
    onehot = np.zeros((n, num_classes + 1), np.float32)
    onehot[np.arange(n), lbl] = 1.0
    return pts, onehot


def make_labelled_batch(batch: int, n: int, num_classes: int, seed0: int = 0):
    """([batch, n, 3], [batch, n, num_classes + 1]) float32; cloud i uses seed seed0 + i."""
    pairs = [lidar_cloud_labelled(n, seed0 + i, num_classes) for i in range(batch)]
    return np.stack([p for p, _ in pairs]), np.stack([g for _, g in pairs])
