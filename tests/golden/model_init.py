"""Closed-form deterministic NDTNet weights for the model fixtures.

Every tensor of a state_dict is filled from a Philox stream keyed by the CRC32
of its name, so the fixture generator (reference model, build container) and
the GPU tests (our model, GPU box) rebuild identical weights without shipping
a 13 MB checkpoint.
"""
from __future__ import annotations

import zlib

import numpy as np
import torch


def deterministic_state(sd: dict) -> dict:
    out = {}
    for name, t in sd.items():
        rng = np.random.Generator(np.random.Philox(zlib.crc32(name.encode())))
        shape = tuple(t.shape)
        if name.endswith("num_batches_tracked"):
            out[name] = torch.zeros_like(t)
            continue
        if name.endswith("running_mean"):
            v = rng.uniform(-0.2, 0.2, shape)
        elif name.endswith("running_var"):
            v = rng.uniform(0.5, 1.5, shape)
        elif ".bn" in name or name.startswith("bn"):
            v = rng.uniform(0.5, 1.5, shape) if name.endswith("weight") else rng.uniform(-0.1, 0.1, shape)
        else:
            fan_in = int(np.prod(shape[1:])) if len(shape) > 1 else shape[0]
            bound = 1.0 / np.sqrt(max(fan_in, 1))
            v = rng.uniform(-bound, bound, shape)
        out[name] = torch.from_numpy(v.astype(np.float32))
    return out
