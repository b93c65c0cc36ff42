#!/usr/bin/env python3
"""fp32 GEMM rates of the training step's conv1x1 shapes: the HIP train GEMM
(ndnet_tr_gemm through train_hip) against torch.matmul (rocBLAS / hipBLASLt),
NCL layouts as the train path holds them (B = 16, N = 1000).

    python tools/gemm_probe.py
"""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "ndt-net_amd"))

dev = torch.device("cuda", 0)
torch.backends.cuda.matmul.allow_tf32 = False
B, N = 16, 1000
shapes = [(128, 1024), (64, 128), (64, 64), (1088, 512), (512, 256), (256, 128), (128, 768)]


def timed(fn, reps=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3  # us


for cin, cout in shapes:
    W = torch.randn(cout, cin, device=dev)
    x = torch.randn(B, cin, N, device=dev)
    dy = torch.randn(B, cout, N, device=dev)
    fl = 2.0 * cin * cout * B * N
    t_fwd = timed(lambda: torch.matmul(W, x))
    t_dx = timed(lambda: torch.matmul(W.t(), dy))
    t_dw = timed(lambda: torch.matmul(dy, x.transpose(1, 2)).sum(0))
    x2 = x.permute(1, 0, 2).reshape(cin, B * N).contiguous()
    dy2 = dy.permute(1, 0, 2).reshape(cout, B * N).contiguous()
    t_dw2 = timed(lambda: torch.matmul(dy2, x2.t()))
    print(f"{cin:5d}->{cout:5d}: fwd {t_fwd:7.1f} us ({fl / t_fwd / 1e6:6.1f} TF)  dX {t_dx:7.1f} us  "
          f"dW bmm+sum {t_dw:7.1f} us  dW one GEMM (CN layout) {t_dw2:7.1f} us ({fl / t_dw2 / 1e6:6.1f} TF)")
