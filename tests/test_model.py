"""NDTNetSegmentation: the reference module tree and numerics (CPU), and the
HIP MFMA forward against torch fp32 (GPU).

Tolerance: |log-prob difference| <= 1e-4 absolute (SURVEY §8d, FP32 mode);
the kernels compute in fp32 with a different summation order and with the
BatchNorms and the t1/t2 transforms folded into the weights."""
import numpy as np
import pytest
import torch

from conftest import golden
from model_init import deterministic_state

TOL = 1e-4


def _model(F, C, device="cpu"):
    from ndnet.models.ndtnet import NDTNetSegmentation
    m = NDTNetSegmentation(3, C, F)
    m.load_state_dict(deterministic_state(m.state_dict()))
    return m.to(device).eval()


@pytest.mark.parametrize("name", ["ndtnet_seg_F768_C28.npz", "ndtnet_seg_F64_C5.npz"])
def test_torch_forward_matches_reference_fixture(name):
    z = golden(name)
    m = _model(int(z["feature_dim"]), int(z["num_classes"]))
    p, c = torch.from_numpy(z["points"]), torch.from_numpy(z["covs"])
    with torch.no_grad():
        assert np.array_equal(m(p, c).numpy(), z["out_eval"])       # CPU -> torch path
        m.train()
        assert np.array_equal(m(p, c).numpy(), z["out_train"])      # batch-statistics BN


def test_torch_train_forward_matches_reference_b16_fixture():
    """The 16-cloud train-mode fixture (make_golden.model_train_fixture): this
    package's torch composition on the CPU reproduces the reference's output
    bit for bit."""
    z = golden("ndtnet_seg_train_F768_C28_B16.npz")
    m = _model(int(z["feature_dim"]), int(z["num_classes"])).train()
    with torch.no_grad():
        out = m(torch.from_numpy(z["points"]), torch.from_numpy(z["covs"])).numpy()
    assert np.array_equal(out, z["out_train"])


def test_state_dict_keys_match_reference_layout():
    m = _model(768, 28)
    keys = set(m.state_dict())
    for k in ["feature_extractor.t1.conv1.weight", "feature_extractor.t2.fc3.bias", "feature_extractor.bn3.running_var",
              "conv4.weight", "bn3.num_batches_tracked"]:
        assert k in keys
    assert sum(p.numel() for p in m.parameters()) == 3_366_822  # reference NDTNetSegmentation(3, 28, 768)


@pytest.mark.parametrize("name", ["ndtnet_seg_F768_C28.npz", "ndtnet_seg_F64_C5.npz"])
def test_folded_algebra_cpu(name):
    """The HIP path's folding (BN, t1, t2, split seg head), evaluated with torch ops."""
    from ndnet.models import pointnet_hip as ph
    z = golden(name)
    m = _model(int(z["feature_dim"]), int(z["num_classes"]))
    with torch.no_grad():
        out = ph.segmentation_forward(m, torch.from_numpy(z["points"]), torch.from_numpy(z["covs"]),
                                      chain=ph._chain_torch)
    assert np.abs(out.numpy() - z["out_eval"]).max() < TOL


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["ndtnet_seg_F768_C28.npz", "ndtnet_seg_F64_C5.npz"])
def test_hip_forward_matches_reference_fixture(name):
    from ndnet.models import pointnet_hip as ph
    assert ph.available(), "the HIP forward must be built (no silent fallback)"
    z = golden(name)
    m = _model(int(z["feature_dim"]), int(z["num_classes"]), "cuda")
    with torch.no_grad():
        out = m(torch.from_numpy(z["points"]).cuda(), torch.from_numpy(z["covs"]).cuda()).cpu().numpy()
    assert np.abs(out - z["out_eval"]).max() < TOL


@pytest.mark.gpu
@pytest.mark.parametrize("B,N", [(16, 1000), (3, 77), (1, 31)])
def test_hip_forward_matches_torch_fp32(B, N):
    """Full-size C3 shape plus ragged point counts (tails of the 32-point tiles)."""
    from ndnet.models import pointnet_hip as ph
    m = _model(768, 28, "cuda")
    g = torch.Generator(device="cuda").manual_seed(B * 1000 + N)
    p = torch.rand((B, N, 3), device="cuda", generator=g) * 20 - 10
    c = torch.randn((B, N, 9), device="cuda", generator=g)
    with torch.no_grad():
        out = m(p, c)
        ref = m.forward_torch(p, c)
        emu = ph.segmentation_forward(m, p, c, chain=ph._chain_torch)
    assert out.shape == (B, N, 29)
    assert (out - ref).abs().max().item() < TOL
    assert (out - emu).abs().max().item() < TOL
    # the predicted class agrees wherever the reference's top two classes are
    # further apart than the two forwards can differ (a flip inside 2 TOL is a
    # tie at fp32 rounding, which the abs bound above already covers)
    top2 = ref.topk(2, dim=-1).values
    clear = (top2[..., 0] - top2[..., 1]) > 2 * TOL
    assert torch.equal(out.argmax(-1)[clear], ref.argmax(-1)[clear])


@pytest.mark.gpu
def test_hip_forward_on_ndt_rows():
    """End to end: ndt_preprocessing rows (views of one [B,k,12] block) into the model."""
    from ndnet.preprocessing.ndtnet_preprocessing import ndt_preprocessing
    from ndnet.synthetic import make_batch
    m = _model(768, 28, "cuda")
    pts = torch.from_numpy(make_batch("L", 4, 20_000)).cuda()
    p, c, _ = ndt_preprocessing(500, pts)
    with torch.no_grad():
        out = m(p, c)
        ref = m.forward_torch(p.contiguous(), c.contiguous())
    assert (out - ref).abs().max().item() < TOL


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["U", "L"])
def test_hip_forward_on_c2_rows(kind):
    """Config C3 on the rows the NDT stage actually emits: the C2 batch (16 x
    100k -> 1000, seeds 0..15) through ndt_preprocessing, its rows (means and
    the post-KL covariances: asymmetric LU iterates with negative diagonals,
    magnitudes up to ~65) into the model.  Log-probs within
    1e-4 of torch fp32, the predicted class equal wherever the reference's top
    two are further apart than 2e-4."""
    from ndnet.preprocessing.ndtnet_preprocessing import ndt_preprocessing
    from ndnet.synthetic import make_batch
    m = _model(768, 28, "cuda")
    pts = torch.from_numpy(make_batch(kind, 16, 100_000)).cuda()
    p, c, _ = ndt_preprocessing(1000, pts, check=True)
    assert c.abs().max().item() > 1.0  # the LU-mutated covariances, not unit-scale noise
    with torch.no_grad():
        out = m(p, c)
        ref = m.forward_torch(p.contiguous(), c.contiguous())
    assert out.shape == (16, 1000, 29)
    assert (out - ref).abs().max().item() < TOL
    top2 = ref.topk(2, dim=-1).values
    clear = (top2[..., 0] - top2[..., 1]) > 2 * TOL
    assert torch.equal(out.argmax(-1)[clear], ref.argmax(-1)[clear])


@pytest.mark.parametrize("F,C", [(768, 28), (64, 5)])
def test_fold_jobs_cover_every_folded_tensor(F, C):
    """The re-fold's job list (ndnet_pn_fold_job per output, the kernel's
    launch on the GPU): each job writes exactly its output tensor's elements,
    and every tensor the forward reads is either re-folded or a parameter."""
    from ndnet.models import pointnet_hip as ph
    m = _model(F, C)
    W = ph._Folded(m)
    size = {0: lambda K, N, Kp, Np: Kp * Np, 1: lambda K, N, Kp, Np: Kp * Np, 2: lambda K, N, Kp, Np: 3 * Kp * Np,
            3: lambda K, N, Kp, Np: N * K, 4: lambda K, N, Kp, Np: 9 * K * N, 5: lambda K, N, Kp, Np: Np}
    outs = set()
    for kind, out, layer, bn, k0, K, Kp, Np, eye in W.jobs:
        N = layer.weight.shape[0]
        assert out.is_contiguous() and out.numel() == size[kind](K, N, Kp, Np)
        assert out.dtype == (torch.bfloat16 if kind == 2 else torch.float32)
        assert k0 + K <= layer.weight.shape[1] and (bn is None or bn.num_features == N)
        outs.add(id(out))
    params = {id(t) for t in m.parameters()}
    read = [w for w, _ in W.A + W.B_tail + [W.C_mid, W.C_tail] + W.D_tail] + [W.s1aT, W.t1_basis]
    read += [b for _, b in W.A + W.B_tail + [W.C_mid, W.C_tail] + W.D_tail] + [W.c1b, W.s1b, W.s1g]
    read += list(W.frag.values()) + list(W.frag6.values()) + list(W.fcf.values())
    for t in (W.t1, W.t2):
        read += [t[k] for k in ("f1", "c1", "f2", "c2", "c3")]
    for t in read:
        assert id(t) in outs or id(t) in params
    assert len(outs) == len(W.jobs)


def _perturb(m, seed, versions=True, params=True):
    """Scales every parameter (``params``) and moves every BatchNorm's running
    statistics; ``versions=False`` writes through ``.data`` (no version bump:
    what a replayed training graph does to the weights)."""
    g = torch.Generator(device="cuda").manual_seed(seed)
    with torch.no_grad():
        for t in (list(m.parameters()) if params else []) + [b for b in m.buffers() if b.is_floating_point()]:
            d = t if versions else t.data
            d.mul_(1.0 + 0.05 * torch.randn(t.shape, device="cuda", generator=g))
            if t.dim() == 1:
                d.add_(0.01 * torch.rand(t.shape, device="cuda", generator=g))  # running_var stays > 0


@pytest.mark.gpu
@pytest.mark.parametrize("F,C", [(768, 28), (64, 5)])
def test_refold_in_place_equals_fresh_fold(F, C):
    """ndnet_pn_fold_run (one launch) re-folds changed weights and running
    statistics into the SAME tensors; every one of them equals what a fresh
    torch fold writes, bit for bit (fp32 operations in torch's order, bf16
    rounding to nearest even), and the forward follows the new weights."""
    from ndnet.models import pointnet_hip as ph
    m = _model(F, C, "cuda")
    g = torch.Generator(device="cuda").manual_seed(F + C)
    p = torch.rand((3, 200, 3), device="cuda", generator=g) * 20 - 10
    c = torch.randn((3, 200, 9), device="cuda", generator=g) * 0.1
    with torch.no_grad():
        m(p, c)
    cache = m._hip
    W, ws = cache["W"], dict(cache["ws"])
    assert W.jobs is not None and len(W.jobs) > 60
    _perturb(m, 1)
    with torch.no_grad():
        out = m(p, c)
    assert m._hip is cache and cache["W"] is W and cache["ws"] == ws, "re-fold must be in place"
    fresh = ph._Folded(m)
    bad = []
    for j, f in zip(W.jobs, fresh.jobs):
        a, b = j[1], f[1]
        assert a.shape == b.shape and a.dtype == b.dtype and j[0] == f[0]
        if not torch.equal(a, b):
            bad.append((j[0], tuple(a.shape), (a.float() - b.float()).abs().max().item()))
    assert not bad, bad
    with torch.no_grad():
        ref = m.forward_torch(p, c)
    assert (out - ref).abs().max().item() < TOL


@pytest.mark.gpu
def test_mode_switch_refolds_weights_changed_without_versions():
    """A replayed training graph changes weights without bumping versions:
    the mode switch (train() -> eval()) marks the fold stale, so the next eval
    forward re-folds; without a mode switch the fold is kept."""
    m = _model(64, 5, "cuda")
    p = torch.rand((2, 100, 3), device="cuda") * 20 - 10
    c = torch.randn((2, 100, 9), device="cuda") * 0.1
    with torch.no_grad():
        first = m(p, c).clone()
        m.train()
        _perturb(m, 2, versions=False)
        m.eval()
        out = m(p, c)
        ref = m.forward_torch(p, c)
    assert (out - ref).abs().max().item() < TOL and (out - first).abs().max().item() > 1e-3
    with torch.no_grad():
        # running statistics only: the fc3 / conv4 weights the forward reads
        # unfolded (pointnet_hip._Folded aliases them) would change it anyway
        _perturb(m, 3, versions=False, params=False)
        kept = m(p, c)   # no mode switch, no version bump: the previous fold
    assert torch.equal(kept, out)


def test_fragment_layout_matches_mfma_operands():
    """_frag puts W^T[k][n] where k-group kg, column block cb, lane 16 kq + cl,
    element s of the float4 with k = 16 kg + 4 kq + s, n = 16 cb + cl
    (include/ndnet_pointnet.h; the kernel's B operand of MFMA step s)."""
    from ndnet.models import pointnet_hip as ph
    K, N = 48, 96
    wT = torch.arange(K * N, dtype=torch.float32).reshape(K, N)
    f = ph._frag(wT).numpy()
    KG = K // 16
    for cb in range(N // 16):
        for kg in range(KG):
            for lane in range(64):
                kq, cl = lane >> 4, lane & 15
                for s in range(4):
                    idx = ((cb * KG + kg) * 64 + lane) * 4 + s
                    assert f[idx] == wT[16 * kg + 4 * kq + s, 16 * cb + cl]
    # per-cloud leading dims are kept
    f3 = ph._frag(torch.stack([wT, 2 * wT]))
    assert f3.shape == (2, K * N) and torch.equal(f3[1], 2 * f3[0])


def test_split_bf16_fragment_layout():
    """_frag_x6: three bf16 planes summing to W^T exactly where representable,
    at [cb][kg][plane][lane][j] with k = 32 kg + 8 (lane >> 4) + j,
    n = 16 cb + (lane & 15) (the 16x16x32 bf16 MFMA B operand)."""
    from ndnet.models import pointnet_hip as ph
    K, N = 64, 32
    g = torch.Generator().manual_seed(0)
    wT = torch.randn((K, N), generator=g)
    f = ph._frag_x6(wT).float().reshape(N // 16, K // 32, 3, 64, 8)
    rec = torch.zeros((K, N))
    for cb in range(N // 16):
        for kg in range(K // 32):
            for lane in range(64):
                for j in range(8):
                    k, n = 32 * kg + 8 * (lane >> 4) + j, 16 * cb + (lane & 15)
                    rec[k, n] = f[cb, kg, 0, lane, j] + f[cb, kg, 1, lane, j] + f[cb, kg, 2, lane, j]
    # h + m + l carries 24 significant bits: equal to the fp32 weight
    assert torch.equal(rec, wT)




@pytest.mark.gpu
def test_split_bf16_layers_are_fp32_accurate():
    """The split-bf16 ("x6") wide layers against a float64 evaluation of the
    same model: their error is at the level of the all-fp32 MFMA path and of
    torch's own fp32 forward (not at bf16's 2^-8)."""
    import copy
    from ndnet.models import pointnet_hip as ph
    m = _model(768, 28, "cuda")
    g = torch.Generator(device="cuda").manual_seed(5)
    p = torch.rand((16, 1000, 3), device="cuda", generator=g) * 20 - 10
    c = torch.randn((16, 1000, 9), device="cuda", generator=g)
    with torch.no_grad():
        ref64 = copy.deepcopy(m).double().forward_torch(p.double(), c.double())
        saved = ph.PRECISION
        outs = {}
        try:
            for mode in ("x6", "fp32"):
                ph.set_precision(mode)
                m._hip = None
                outs[mode] = m(p, c).double()
        finally:
            ph.set_precision(saved)
            m._hip = None
        out_x6, out_32 = outs["x6"], outs["fp32"]
        out_t32 = m.forward_torch(p, c).double()
    e_x6 = (out_x6 - ref64).abs().max().item()
    e_32 = (out_32 - ref64).abs().max().item()
    e_t32 = (out_t32 - ref64).abs().max().item()
    print(f"max |err| vs fp64: x6 {e_x6:.3e}, fp32 MFMA {e_32:.3e}, torch fp32 {e_t32:.3e}")
    assert e_x6 <= 2.0 * max(e_32, e_t32) + 1e-6


@pytest.mark.gpu
@pytest.mark.parametrize("B,K,N,relu", [(16, 1024, 512, True), (5, 768, 512, False), (3, 256, 4096, False)])
def test_fc_mfma_matches_torch(B, K, N, relu):
    """ndnet_pn_fc_mfma_run (16-row fp32-MFMA GEMM over fragment-major W^T)
    against torch fp32 addmm, row stride past K (the max-pool buffer's)."""
    from ndnet.models import pointnet_hip as ph
    g = torch.Generator().manual_seed(B * K + N)
    xfull = torch.randn(B, K + 64, generator=g).cuda()
    x = xfull[:, :K]
    w = (torch.randn(N, K, generator=g) / K ** 0.5).cuda()
    b = torch.randn(N, generator=g).cuda()
    out = torch.empty(B, N, device="cuda")
    ph._fc(x, w, b, out, relu, ph._frag(w.t().contiguous()))
    ref = torch.addmm(b, x, w.t())
    if relu:
        ref = ref.relu()
    torch.cuda.synchronize()
    assert (out - ref).abs().max().item() < 1e-5


@pytest.mark.gpu
@pytest.mark.parametrize("B,relu", [(16, False), (7, True)])
def test_fc_mfma_column_blocks_are_bit_identical(B, relu):
    """A 256 -> 4096 layer (TNet(64)'s fc3) runs as four-column-block
    workgroups (k_pn_fc_mfma<4>); the same layer issued as eight 512-column
    slices runs one block per workgroup (k_pn_fc_mfma<1>: 32 blocks per
    slice).  Same per-column sums in the same order: bit-identical."""
    from ndnet import _lib
    from ndnet.models import pointnet_hip as ph
    K, N = 256, 4096
    g = torch.Generator().manual_seed(40 + B)
    x = torch.randn(B, K, generator=g).cuda()
    w = (torch.randn(N, K, generator=g) / K ** 0.5).cuda()
    b = torch.randn(N, generator=g).cuda()
    wf = ph._frag(w.t().contiguous())
    wide = torch.empty(B, N, device="cuda")
    ph._fc(x, w, b, wide, relu, wf)
    sliced = torch.empty(B, N, device="cuda")
    st = _lib.stream_ptr(x.device)
    per = K * 512                                     # fragment-major floats per 512 columns
    for s in range(N // 512):
        rc = _lib.lib().ndnet_pn_fc_mfma_run(x.data_ptr(), K, wf.data_ptr() + 4 * per * s, b.data_ptr() + 4 * 512 * s,
                                             sliced.data_ptr() + 4 * 512 * s, N, B, K, 512, 1 if relu else 0, st)
        _lib.check(rc, "ndnet_pn_fc_mfma_run")
    torch.cuda.synchronize()
    assert torch.equal(wide, sliced)
    ref = torch.addmm(b, x, w.t())
    assert ((wide - (ref.relu() if relu else ref)).abs().max().item()) < 1e-5


@pytest.mark.gpu
def test_head3_in_chain_equals_head3_kernel(monkeypatch):
    """TNet(3)'s fc3 + t1 fold in chain B's prologue (default) against the
    separate k_pn_head3 launch: same log-probs within fp32 reduction order."""
    from ndnet.models import pointnet_hip as ph
    torch.manual_seed(7)
    pts, cov = torch.randn(4, 300, 3).cuda(), torch.randn(4, 300, 9).cuda() * 0.1
    outs = []
    for flag in (True, False):
        monkeypatch.setattr(ph, "HEAD3_IN_CHAIN", flag)
        m = _model(768, 28, "cuda")
        with torch.no_grad():
            outs.append(m(pts, cov))
    assert (outs[0] - outs[1]).abs().max().item() < 1e-5


@pytest.mark.gpu
@pytest.mark.parametrize("B,N", [(16, 500), (4, 77), (2, 1000)])
def test_chain_t32_equals_t64(monkeypatch, B, N):
    """The 32-point-tile chain build (ndnet_pn_chain_run_t32: 8 waves, two row
    blocks) against the 64-point build on the same model and input: log-probs
    within fp32 summation order, and both within the torch fp32 tolerance."""
    from ndnet.models import pointnet_hip as ph
    torch.manual_seed(11)
    pts, cov = torch.randn(B, N, 3).cuda(), torch.randn(B, N, 9).cuda() * 0.1
    outs = []
    for force in (True, False):
        monkeypatch.setattr(ph, "_use_t32", lambda b, n, d, f=force: f)
        m = _model(768, 28, "cuda")
        with torch.no_grad():
            outs.append(m(pts, cov))
    ref = m.forward_torch(pts, cov)
    assert (outs[0] - outs[1]).abs().max().item() < 1e-5
    assert (outs[0] - ref).abs().max().item() < TOL
