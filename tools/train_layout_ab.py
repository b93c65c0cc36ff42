#!/usr/bin/env python3
"""A/B of the train-mode forward + backward layouts on one GPU (B = 16,
k = 1000, F = 768, 28 classes):

  module   NDTNetSegmentation.forward_torch ([B, C, N] Conv1d / BatchNorm1d:
           MIOpen convolutions with NCHW <-> NHWC transposes)
  cl       points-major [B, N, C]: every 1x1 convolution one GEMM
           (F.linear over B*N rows), BatchNorm over the rows (same batch
           statistics and running-stat updates)
  cl_nomi  cl with MIOpen off (torch's own BatchNorm kernels)
  cl_split cl, and the seg head's first layer split as x_t2 W_a + (g W_b)
           per cloud (no [B, N, 64 + F] concat, 768 of its 832 input
           channels computed once per cloud)

Prints ms per forward + backward and the largest loss / gradient deviation
from ``module``.
"""
import json
import os
import sys

import torch
import torch.nn.functional as Fn

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "ndt-net_amd"))
from ndnet.models.ndtnet import NDTNetSegmentation  # noqa: E402
from ndnet.training import segmentation_loss  # noqa: E402


def lin(conv, x):
    return Fn.linear(x, conv.weight.squeeze(-1), conv.bias)


def bn(m, x):
    if m.training and m.track_running_stats:
        m.num_batches_tracked.add_(1)
    y = Fn.batch_norm(x.reshape(-1, x.shape[-1]), m.running_mean, m.running_var, m.weight, m.bias,
                      m.training, m.momentum, m.eps)
    return y.view(x.shape)


def tnet(t, x):
    for c, b in ((t.conv1, t.bn1), (t.conv2, t.bn2), (t.conv3, t.bn3)):
        x = torch.relu(bn(b, lin(c, x)))
    g = x.amax(dim=1)
    g = torch.relu(t.bn4(t.fc1(g)))
    g = torch.relu(t.bn5(t.fc2(g)))
    tt = t.fc3(g) + torch.eye(t.in_dim, device=g.device, dtype=g.dtype).reshape(1, -1)
    return tt.view(-1, t.in_dim, t.in_dim)


def forward_cl(m, points, extra, split=False):
    fe = m.feature_extractor
    B, N, _ = points.shape
    t = tnet(fe.t1, points)
    xyz = torch.bmm(points, t.transpose(1, 2))
    cov = torch.matmul(t.unsqueeze(1), extra.reshape(B, N, 3, 3)).reshape(B, N, 9)
    x = torch.cat((xyz, cov), dim=2)
    x = bn(fe.bn1, lin(fe.conv1, x))
    t2 = tnet(fe.t2, x)
    x = torch.bmm(x, t2)
    x_t2 = x
    x = bn(fe.bn2, lin(fe.conv2, x))
    x = bn(fe.bn3, lin(fe.conv3, x))
    g = x.amax(dim=1)  # [B, F]
    w = m.conv1.weight.squeeze(-1)
    if split:
        y = Fn.linear(x_t2, w[:, :64]) + Fn.linear(g, w[:, 64:], m.conv1.bias).unsqueeze(1)
    else:
        y = lin(m.conv1, torch.cat((x_t2, g.unsqueeze(1).expand(-1, N, -1)), dim=2))
    x = torch.relu(bn(m.bn1, y))
    x = torch.relu(bn(m.bn2, lin(m.conv2, x)))
    x = torch.relu(bn(m.bn3, lin(m.conv3, x)))
    return Fn.log_softmax(lin(m.conv4, x), dim=-1)


def main():
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    B, N, C, F = 16, 1000, 28, 768
    pts = torch.rand(B, N, 3, device=dev) * 20 - 10
    cov = torch.randn(B, N, 9, device=dev) * 0.1
    lbl = torch.randint(0, C + 1, (B, N), device=dev)
    gt = Fn.one_hot(lbl, C + 1).float()
    base = NDTNetSegmentation(3, C, F).to(dev).train()
    state = {k: v.clone() for k, v in base.state_dict().items()}
    variants = {
        "module": lambda m: m.forward_torch(pts, cov),
        "cl": lambda m: forward_cl(m, pts, cov),
        "cl_split": lambda m: forward_cl(m, pts, cov, split=True),
    }
    res, ref = {}, None
    for name, fwd in list(variants.items()) + [("cl_nomi", None)]:
        m = base
        m.load_state_dict(state)
        f = fwd if fwd is not None else variants["cl"]
        ctx = torch.backends.cudnn.flags(enabled=False) if name == "cl_nomi" else torch.backends.cudnn.flags(enabled=True)
        with ctx:
            def step():
                for p in m.parameters():
                    p.grad = None
                loss = segmentation_loss(f(m), gt)
                loss.backward()
                return loss
            for _ in range(3):
                step()
            m.load_state_dict(state)
            loss = step()
            grads = [p.grad.clone() for p in m.parameters()]
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(20):
                step()
            e1.record()
            torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / 20
        if ref is None:
            ref = (loss.item(), grads)
            dl, dg = 0.0, 0.0
        else:
            dl = abs(loss.item() - ref[0])
            scale = max(g.abs().max().item() for g in ref[1])
            dg = max((a - b).abs().max().item() for a, b in zip(grads, ref[1])) / scale
        res[name] = {"ms_fwd_bwd": round(ms, 4), "d_loss": dl, "d_grad_rel": dg}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
