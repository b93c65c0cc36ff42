"""The training step (reference tools/train.py:16-92):
the fixed loss, the LR schedule, Adam steps on NDs, and DDP gradient
averaging at world size 2 over gloo on the CPU (the RCCL path on GPUs is the
same torch DDP with backend "nccl")."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from ndnet.training import Trainer, accuracy, lr_for_epoch, segmentation_loss


def _model(F=64, C=5, seed=0):
    from ndnet.models.ndtnet import NDTNetSegmentation
    torch.manual_seed(seed)
    return NDTNetSegmentation(3, C, F)


def _nds(B, k, C, seed):
    g = torch.Generator().manual_seed(seed)
    pcl = torch.rand((B, k, 3), generator=g) * 20 - 10
    covs = torch.randn((B, k, 9), generator=g) * 0.1
    lbl = torch.randint(0, C + 1, (B, k), generator=g)
    gt = torch.nn.functional.one_hot(lbl, C + 1).float()
    return pcl, covs, gt


def test_loss_is_class_dim_cross_entropy():
    g = torch.Generator().manual_seed(0)
    z = torch.randn((3, 50, 7), generator=g)
    lbl = torch.randint(0, 7, (3, 50), generator=g)
    gt = torch.nn.functional.one_hot(lbl, 7).float()
    ours = segmentation_loss(torch.log_softmax(z, dim=-1), gt)
    ref = torch.nn.functional.cross_entropy(z.reshape(-1, 7), lbl.reshape(-1))
    assert torch.allclose(ours, ref, atol=1e-6)
    assert accuracy(z, gt) == (z.argmax(-1) == lbl).float().mean().item()


def test_lr_schedule_halves_every_20_epochs():
    assert lr_for_epoch(0.034, 0) == 0.034
    assert lr_for_epoch(0.034, 18) == 0.034
    assert lr_for_epoch(0.034, 19) == 0.017
    assert lr_for_epoch(0.034, 39) == 0.034 / 4


def test_adam_steps_reduce_loss_cpu():
    m = _model()
    tr = Trainer(m, 1e-3, 128, 5, torch.device("cpu"), ddp=False)
    pcl, covs, gt = _nds(4, 128, 5, seed=1)
    losses = [tr.step_on_nds(pcl, covs, gt)[0] for _ in range(6)]
    assert all(np.isfinite(losses))
    assert losses[-1] < losses[0]
    # val/test mode: no parameter update (train.py:74-81 stepped in every mode)
    before = [p.detach().clone() for p in m.parameters()]
    tr.step_on_nds(pcl, covs, gt, train=False)
    assert all(torch.equal(a, b) for a, b in zip(before, m.parameters()))


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _ddp_worker(rank, world, port, q):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, os.path.join(os.path.dirname(here), "ndt-net_amd"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    torch.set_num_threads(2)
    import torch.distributed as dist
    dist.init_process_group("gloo")
    from ndnet.training import Trainer as T
    m = _model()
    tr = T(m, 1e-3, 96, 5, torch.device("cpu"))
    assert tr.net is not m, "a world-2 group must wrap the model in DDP"
    pcl, covs, gt = _nds(2, 96, 5, seed=10 + rank)
    # the DDP backward alone: gradients all-reduced (averaged) over the ranks
    m.train()
    segmentation_loss(tr.net(pcl, covs), gt).backward()
    grads = [p.grad.detach().numpy().copy() for p in m.parameters()]
    # then a whole Trainer step: every rank must hold the same parameters after it
    tr.step_on_nds(pcl, covs, gt)
    params = [p.detach().numpy().copy() for p in m.parameters()]
    q.put((rank, grads, params))
    dist.destroy_process_group()


def test_ddp_world2_gloo_averages_gradients():
    """DDP's backward leaves each rank the mean of the two shards' gradients,
    and a Trainer step leaves the ranks with identical parameters."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_ddp_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = {r: (g, w) for r, g, w in (q.get(timeout=300) for _ in procs)}
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    shard_grads = []
    for r in range(2):
        m = _model()
        m.train()
        pcl, covs, gt = _nds(2, 96, 5, seed=10 + r)
        segmentation_loss(m(pcl, covs), gt).backward()
        shard_grads.append([p.grad.numpy() for p in m.parameters()])
    # tolerance on the model's gradient scale: biases feeding a BatchNorm have
    # gradients that are pure rounding noise (the batch mean cancels them)
    scale = max(float(np.abs((g0 + g1) / 2).max()) for g0, g1 in zip(*shard_grads))
    for i, (g0, g1) in enumerate(zip(*shard_grads)):
        ref = (g0 + g1) / 2
        for r in range(2):
            assert np.abs(got[r][0][i] - ref).max() <= 1e-5 * scale, f"rank {r} grad {i} is not the mean"
    for a, b in zip(got[0][1], got[1][1]):
        assert np.array_equal(a, b), "ranks disagree after the step"


@pytest.mark.gpu
def test_ddp_step_over_rccl_equals_plain_step():
    """The RCCL path on the GPU (VERDICT r2 missing 1 / item 9): a one-rank
    "nccl" process group, the Trainer's DDP wrapper with its bucketed gradient
    all-reduce, and ndnet.distributed's barrier / max / all-gather on device
    tensors.  One Adam step through DDP over RCCL leaves the same parameters as
    the plain step (a mean over one rank), on HIP-preprocessed labelled NDs.
    A box has one GPU, and RCCL refuses two ranks on one device, so the
    two-rank gradient averaging itself is the gloo test above."""
    import copy
    import torch.distributed as dist
    from ndnet import distributed as D
    from ndnet.preprocessing.ndtnet_preprocessing import ndt_preprocessing
    from ndnet.synthetic import make_labelled_batch
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    pts, gt = make_labelled_batch(2, 20_000, 28, seed0=11)
    p, c, g = ndt_preprocessing(500, torch.from_numpy(pts).to(dev), torch.from_numpy(gt).to(dev), 28)
    p, c = p.contiguous(), c.contiguous()
    m_ddp = _model(F=768, C=28, seed=5)
    m_one = copy.deepcopy(m_ddp)
    assert not dist.is_initialized()
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_free_port()}", rank=0, world_size=1,
                            device_id=dev)
    try:
        assert dist.get_backend() == "nccl"
        t_ddp = Trainer(m_ddp, 1e-3, 500, 28, dev, ddp=True, bucket_cap_mb=1.0)
        assert t_ddp.net is not m_ddp
        l_ddp, _ = t_ddp.step_on_nds(p, c, g)
        D.barrier()
        assert D.max_over_ranks(2.5) == 2.5 and D.sum_over_ranks(1.25) == 1.25
        out = torch.randn(3, 7, device=dev)
        assert torch.equal(D.gather_shards(out), out)
        torch.cuda.synchronize()
    finally:
        dist.destroy_process_group()
    t_one = Trainer(m_one, 1e-3, 500, 28, dev, ddp=False)
    l_one, _ = t_one.step_on_nds(p, c, g)
    assert abs(l_ddp - l_one) <= 1e-6 * max(1.0, abs(l_one))
    for (name, a), b in zip(m_ddp.named_parameters(), m_one.parameters()):
        assert (a - b).abs().max().item() <= 1e-6, name


@pytest.mark.gpu
def test_graphed_train_steps_equal_eager_steps():
    """Trainer(graphs=True): three steps replayed from one captured HIP graph
    (labelled NDT -> train forward -> backward -> fused Adam) on changing
    batches, each checked against the eager step from the same weights: the
    loss, every gradient (within 1e-4 of the gradient scale: the two may pick
    different GEMM / BatchNorm kernels), and the parameters after Adam applied
    eagerly to the graph's own gradients.  Adam's first steps are sign-like
    (m / sqrt(v) = +-1), so gradients at rounding-noise level -- the biases
    that feed a BatchNorm -- make whole-trajectory comparisons meaningless;
    the update itself is compared instead.  Also: the warm-up before the
    capture leaves no trace, set_epoch's learning rate reaches the graph, a
    step on the graph's own input buffers (graph_inputs, no copy) equals one
    on copies, and an eval forward after the replays uses the updated weights."""
    from ndnet.preprocessing.ndtnet_preprocessing import ndt_preprocessing
    from ndnet.synthetic import make_labelled_batch
    dev = torch.device("cuda", 0)
    m_g = _model(F=768, C=28, seed=9).to(dev)
    m_e = _model(F=768, C=28, seed=9).to(dev)
    t_g = Trainer(m_g, 1e-3, 500, 28, dev, ddp=False, graphs=True)
    t_e = Trainer(m_e, 1e-3, 500, 28, dev, ddp=False, graphs=True)
    for i in range(3):
        pts, gt = make_labelled_batch(2, 20_000, 28, seed0=20 + i)
        pts, gt = torch.from_numpy(pts).to(dev), torch.from_numpy(gt).to(dev)
        if i == 2:
            t_g.set_epoch(19)  # halves the LR
            t_e.set_epoch(19)
        with torch.no_grad():  # the eager side starts from the graph side's weights
            for a, b in zip(m_e.parameters(), m_g.parameters()):
                a.copy_(b)
            for a, b in zip(m_e.buffers(), m_g.buffers()):
                a.copy_(b)
        p, c, g = ndt_preprocessing(500, pts, gt, 28)
        m_e.train()
        t_e.opt.zero_grad(set_to_none=True)
        l_e = segmentation_loss(m_e(p, c), g)
        l_e.backward()
        if i == 1:  # the graph's own input buffers, filled in place: replayed with no copy
            s_p, s_g = t_g.graph_inputs(pts.shape, gt.shape)
            s_p.copy_(pts)
            s_g.copy_(gt)
            l_g, _ = t_g.step_graphed(s_p, s_g)
        else:
            l_g, _ = t_g.step_graphed(pts, gt)
        assert abs(l_g.item() - l_e.item()) <= 1e-5 * max(1.0, abs(l_e.item())), (i, l_g.item(), l_e.item())
        scale = max(q.grad.abs().max().item() for q in m_e.parameters())
        for (name, a), b in zip(m_g.named_parameters(), m_e.parameters()):
            assert (a.grad - b.grad).abs().max().item() <= 1e-4 * scale, (i, name)
        with torch.no_grad():
            for a, b in zip(m_e.parameters(), m_g.parameters()):
                a.grad.copy_(b.grad)
        t_e.opt.step()
        for (name, a), b in zip(m_g.named_parameters(), m_e.parameters()):
            assert (a - b).abs().max().item() <= 1e-6, (i, name)
        for (name, a), b in zip(m_g.named_buffers(), m_e.buffers()):
            assert (a.double() - b.double()).abs().max().item() <= 1e-4, (i, name)
    assert len(t_g._graphed) == 1
    m_g.eval()
    m_e.eval()
    with torch.no_grad():
        assert (m_g(p, c) - m_e(p, c)).abs().max().item() <= 1e-4


@pytest.mark.gpu
def test_training_step_gpu_labelled_path():
    """Raw labelled clouds -> labelled NDT path (HIP) -> train-mode forward ->
    backward -> Adam, then an eval step on the HIP forward."""
    from ndnet.synthetic import make_labelled_batch
    dev = torch.device("cuda", 0)
    m = _model(F=768, C=28)
    tr = Trainer(m, 1e-3, 500, 28, dev, ddp=False)
    pts, gt = make_labelled_batch(2, 20_000, 28, seed0=3)
    before = [p.detach().clone() for p in m.parameters()]
    losses = [tr.step(torch.from_numpy(pts), torch.from_numpy(gt))[0] for _ in range(3)]
    assert all(np.isfinite(losses)), losses
    assert any(not torch.equal(a, b) for a, b in zip(before, m.parameters()))
    vloss, vacc = tr.step(torch.from_numpy(pts), torch.from_numpy(gt), train=False)
    assert 0.0 <= vacc <= 1.0
    # the eval forward re-folds the trained weights: HIP path == torch composition
    from ndnet.preprocessing.ndtnet_preprocessing import ndt_preprocessing
    p, c, _ = ndt_preprocessing(500, torch.from_numpy(pts).to(dev))
    m.eval()
    with torch.no_grad():
        out, ref = m(p, c), m.forward_torch(p.contiguous(), c.contiguous())
    err = ((out - ref).abs() / ref.abs().clamp_min(1.0)).max().item()
    assert err < 1e-4, err


@pytest.mark.gpu
def test_adam_step_on_hip_nds_equals_oracle_nds():
    """VERDICT r1 item 9 (reference tools/train.py:67-81): one Adam step on the
    HIP-preprocessed labelled NDs against the same step on NDs the CPU oracle
    produced from the same clouds.  The NDs (means, covariances, one-hot
    classes) are bit-identical, and the parameters after the step agree within
    1e-5 (same data; only the GPU's own reduction order may differ)."""
    import copy
    import oracle as O
    from ndnet.preprocessing.ndtnet_preprocessing import ndt_preprocessing
    from ndnet.synthetic import make_labelled_batch
    dev = torch.device("cuda", 0)
    B, n, k, C = 2, 20_000, 500, 28
    pts, gt = make_labelled_batch(B, n, C, seed0=7)
    p, c, g = ndt_preprocessing(k, torch.from_numpy(pts).to(dev), torch.from_numpy(gt).to(dev), C)
    op = np.zeros((B, k, 3), np.float32)
    oc = np.zeros((B, k, 9), np.float32)
    og = np.zeros((B, k, C + 1), np.float32)
    for b in range(B):
        r = O.run(pts[b].astype(np.float64), k, classes=gt[b].argmax(axis=1), num_classes=C)
        assert r.rc == 0
        op[b] = np.nan_to_num(r.out_pc.astype(np.float32), nan=0.0, posinf=0.0, neginf=0.0)
        oc[b] = np.nan_to_num(r.out_cov.astype(np.float32), nan=0.0, posinf=0.0, neginf=0.0)
        og[b, np.arange(k), r.out_cls] = 1.0
    assert np.array_equal(p.cpu().numpy(), op) and np.array_equal(c.cpu().numpy(), oc)
    assert np.array_equal(g.cpu().numpy(), og)
    m_hip = _model(F=768, C=C, seed=4)
    m_orc = copy.deepcopy(m_hip)
    t_hip = Trainer(m_hip, 1e-3, k, C, dev, ddp=False)
    t_orc = Trainer(m_orc, 1e-3, k, C, dev, ddp=False)
    l_hip, _ = t_hip.step_on_nds(p.contiguous(), c.contiguous(), g)
    l_orc, _ = t_orc.step_on_nds(torch.from_numpy(op).to(dev), torch.from_numpy(oc).to(dev),
                                 torch.from_numpy(og).to(dev))
    assert abs(l_hip - l_orc) <= 1e-5 * max(1.0, abs(l_orc))
    for (name, a), b in zip(m_hip.named_parameters(), m_orc.parameters()):
        assert (a - b).abs().max().item() <= 1e-5, name


def test_weight_gradient_split_covers_every_point():
    """Host logic of the train GEMM's split-K (ndnet.models.train_hip.dw_split):
    the parts tile the (cloud, point) range exactly once, within the caps the
    ABI enforces (ndnet_tr_gemm: chunks start inside K and cover it)."""
    from ndnet.models.train_hip import _DW_MAX_PARTS, dw_split
    for B in (1, 2, 5, 16, 20, 64):
        for cout, cin in ((64, 3), (64, 12), (128, 64), (1024, 128), (768, 128), (512, 64), (256, 512), (29, 128)):
            for N in (1, 17, 500, 1000, 4097):
                cpz, nch, kchunk = dw_split(B, cout, cin, N)
                assert 1 <= cpz <= B and nch >= 1 and kchunk >= 1
                assert (nch - 1) * kchunk < N <= nch * kchunk
                assert nch == 1 or kchunk % 16 == 0
                parts = -(-B // cpz) * nch
                assert parts <= max(_DW_MAX_PARTS, 1)
