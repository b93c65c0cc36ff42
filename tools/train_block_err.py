#!/usr/bin/env python3
"""Per-block fp32 error of the train-mode blocks (HIP vs torch) against float64,
each block fed the same input (the one the HIP forward produced)."""
import copy, os, sys
import torch
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "ndt-net_amd"))
from ndnet.models import ndtnet, train_hip  # noqa: E402

torch.manual_seed(3)
model = ndtnet.NDTNetSegmentation(num_classes=28, feature_dim=768).cuda().train()
g = torch.Generator(device="cuda").manual_seed(11)
pts = torch.randn(4, 1000, 3, device="cuda", generator=g) * 5
a = torch.randn(4, 1000, 3, 3, device="cuda", generator=g) * 0.3
cov = (a @ a.transpose(-1, -2)).reshape(4, 1000, 9)
rec = []
real = train_hip.conv_bn_act
def spy(conv, bn, x, relu, **kw):
    if kw:  # the segmentation head's folded conv1: not recorded
        return real(conv, bn, x, relu, **kw)
    c2, b2 = copy.deepcopy(conv), copy.deepcopy(bn)
    rec.append((c2, b2, x.detach().clone(), relu))
    return real(conv, bn, x, relu)
train_hip.conv_bn_act = spy
with torch.no_grad():
    model(pts, cov)
for i, (c, b, x, relu) in enumerate(rec):
    def tr(c, b, x):
        y = c(x)
        if b is not None: y = b(y)
        return torch.relu(y) if relu else y
    with torch.no_grad():
        h = real(copy.deepcopy(c), copy.deepcopy(b), x, relu)
        t = tr(copy.deepcopy(c), copy.deepcopy(b), x)
        f = tr(copy.deepcopy(c).double(), None if b is None else copy.deepcopy(b).double(), x.double())
    eh = (h.double() - f).abs().max().item(); et = (t.double() - f).abs().max().item()
    ratio = None
    if b is not None:
        y = c.double()(x.double())
        m = y.mean((0, 2)); s = y.std((0, 2))
        ratio = (m.abs() / s).max().item()
    print(f"block {i:2d} {tuple(c.weight.shape[:2])} bn={b is not None} relu={relu}: HIP {eh:.3e} torch {et:.3e}"
          f"  max|mean|/std {ratio}")
