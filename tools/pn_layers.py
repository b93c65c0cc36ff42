#!/usr/bin/env python3
"""Time single-layer (and fused-pair) k_pn_chain launches per layer shape on
16 x 1000 points: where the chain kernel's time goes, layer by layer.

    python tools/pn_layers.py [--batch 16 --points 1000 --reps 20]
"""
import argparse
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "ndt-net_amd"))
from ndnet.models import pointnet_hip as ph  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--batch", type=int, default=16)
ap.add_argument("--points", type=int, default=1000)
ap.add_argument("--reps", type=int, default=20)
a = ap.parse_args()
dev = torch.device("cuda", 0)
B, n = a.batch, a.points
x = torch.randn(B, n, 12, device=dev)
# a 1024-wide input region (the chain reads its input tile from x, so a layer
# with K > 16 is timed behind a 16 -> K producer layer, reported separately)
shapes = [(16, 64), (64, 64), (64, 128), (128, 1024), (128, 768), (256, 128), (128, 32), (512, 256)]


def layer(K, N):
    w = torch.randn(K, N, device=dev) * 0.05
    return (ph._frag(w), 0, torch.zeros(N, device=dev), K, N)


def time_chain(layers, relus, mode, gmax=None, out=None, out_cols=0, fuse=()):
    ch = ph._build_chain(n, 12, layers, relus, mode, gmax=gmax, out_cols=out_cols, fuse=fuse)
    for _ in range(3):
        ph._run_chain(ch, x, out)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.reps):
        ph._run_chain(ch, x, out)
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / a.reps * 1e3


gmax = torch.full((B, 1024), float("-inf"), device=dev)
base = {}
for K, N in shapes:
    flops = 2.0 * B * n * K * N
    if K == 16:
        us = time_chain([layer(16, N)], (1,), 0, gmax=gmax)
        print(f"{K:4d} -> {N:4d} (max-pool)            {us:7.1f} us  {flops / (us * 1e-6) / 1e12:6.1f} TFLOP/s")
        continue
    if K not in base:
        base[K] = time_chain([layer(16, K)], (1,), 0, gmax=gmax)
    us_pool = time_chain([layer(16, K), layer(K, N)], (1, 1), 0, gmax=gmax) - base[K]
    print(f"{K:4d} -> {N:4d} (max-pool, minus producer) {us_pool:7.1f} us  {flops / (us_pool * 1e-6) / 1e12:6.1f} TFLOP/s")
# the seg head's fused pair 64 -> 512 -> 256, then 256 -> 128 -> 32 + log_softmax
out = torch.empty(B, n, 29, device=dev)
flops = 2.0 * B * n * (64 * 512 + 512 * 256)
us = time_chain([layer(16, 64), layer(64, 512), layer(512, 256)], (1, 1, 1), 0, gmax=gmax, fuse=(1,)) - base[64]
print(f"  64 -> 512 -> 256 fused (minus producer) {us:7.1f} us  {flops / (us * 1e-6) / 1e12:6.1f} TFLOP/s")


# split-bf16 (prec 1) layers: bf16-MFMA utilisation (6 bf16 products per fp32 FLOP)
def layer_x6(K, N):
    w = torch.randn(K, N, device=dev) * 0.05
    return (ph._frag_x6(w), 0, torch.zeros(N, device=dev), K, N, 1)




BF16_PEAK = 2.5e15
for K, N in [(128, 1024), (128, 768), (128, 512), (128, 256), (64, 1024), (256, 1024)]:
    flops = 2.0 * B * n * K * N
    if K not in base:
        base[K] = time_chain([layer(16, K)], (1,), 0, gmax=gmax)
    for tag, fn in (("x6 ", layer_x6),):
        us = time_chain([layer(16, K), fn(K, N)], (1, 1), 0, gmax=gmax) - base[K]
        print(f"{tag} {K:4d} -> {N:4d} (max-pool, minus producer) {us:7.1f} us  {flops / (us * 1e-6) / 1e12:6.1f} "
              f"TFLOP/s fp32-eq, bf16 MFMA {6 * flops / (us * 1e-6) / BF16_PEAK * 100:5.1f}% of peak   "
              f"(producer {base[K]:.1f} us)")

# the seg head's fused pair in split-bf16 (64 -> 512 -> 256, as chain D runs it) and the whole D tail
if "--no-d" not in sys.argv:
    flops = 2.0 * B * n * (64 * 512 + 512 * 256)
    us = time_chain([layer(16, 64), layer_x6(64, 512), layer_x6(512, 256)], (1, 1, 1), 0, gmax=gmax, fuse=(1,)) \
        - base[64]
    print(f"x6  64 -> 512 -> 256 fused (minus producer) {us:7.1f} us  {flops / (us * 1e-6) / 1e12:6.1f} TFLOP/s "
          f"fp32-eq, bf16 MFMA {6 * flops / (us * 1e-6) / BF16_PEAK * 100:5.1f}% of peak")
    flops = 2.0 * B * n * (64 * 512 + 512 * 256 + 256 * 128 + 128 * 32)
    us = time_chain([layer(16, 64), layer_x6(64, 512), layer_x6(512, 256), layer_x6(256, 128), layer(128, 32)],
                    (1, 1, 1, 1, 0), 1, out=out, out_cols=29, fuse=(1,)) - base[64]
    print(f"D tail 64 -> 512 -> 256 -> 128 -> 32 + log_softmax (minus producer) {us:7.1f} us  "
          f"{flops / (us * 1e-6) / 1e12:6.1f} TFLOP/s fp32-eq")

