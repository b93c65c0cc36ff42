"""The graph-captured pipeline and the device-side stamp-epoch wrap.

* ``GraphedSegmentation`` replays exactly the eager kernels, so its output is
  bit-identical to ``model(*ndt_preprocessing(k, points)[:2])``.
* The NDT plan's voxel stamps carry a 26-bit run epoch; when it wraps the
  device clears the stale stamps itself (k_reset / k_limits), so results stay
  identical across the wrap with no host bookkeeping (graph replays never run
  host code).  The cloud is wide and sparse so the bisection's grids exceed
  the bitmap capacity and run in stamp mode.
"""
import ctypes

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _model(F=64, C=5, seed=3):
    import torch
    from ndnet.models.ndtnet import NDTNetSegmentation
    torch.manual_seed(seed)
    m = NDTNetSegmentation(3, C, F).cuda().eval()
    with torch.no_grad():
        for mod in m.modules():
            if isinstance(mod, torch.nn.BatchNorm1d):
                mod.running_mean.uniform_(-0.2, 0.2)
                mod.running_var.uniform_(0.5, 1.5)
    return m


def test_graph_replay_matches_eager():
    import torch
    from ndnet.synthetic import make_batch
    from ndnet.pipeline import GraphedSegmentation
    from ndnet.preprocessing.ndtnet_preprocessing import ndt_preprocessing
    B, n, k = 4, 20000, 256
    m = _model()
    pts = torch.from_numpy(make_batch("L", B, n, seed0=11)).cuda()
    with torch.no_grad():
        p, c, _ = ndt_preprocessing(k, pts)
        eager = m(p, c).clone()
    g = GraphedSegmentation(m, k, B, n)
    out = g(pts).clone()
    torch.cuda.synchronize()
    assert torch.equal(out, eager)
    assert all(s.rc == 0 and s.prune_rc == 0 for s in g.stats())
    # new input through the same graph
    pts2 = torch.from_numpy(make_batch("U", B, n, seed0=23)).cuda()
    with torch.no_grad():
        p, c, _ = ndt_preprocessing(k, pts2)
        eager2 = m(p, c).clone()
    out2 = g(pts2).clone()
    torch.cuda.synchronize()
    assert torch.equal(out2, eager2)
    assert not torch.equal(out2, out)


def test_epoch_wrap_clears_stamps():
    import torch
    from ndnet import _lib
    from ndnet.preprocessing.ndtnet_preprocessing import ndt_preprocessing, get_plan
    rng = np.random.default_rng(5)
    B, n, k = 2, 20000, 500
    # 60 clusters in an 800^3 box: ~500 occupied voxels on grids of ~10^5 voxels
    # (oracle: 4 bisection passes, accepted grids 49x49x48 and 49x48x46)
    centers = rng.uniform(0, 800, (B, 60, 3))
    pick = rng.integers(0, 60, (B, n))
    pts = (np.take_along_axis(centers, pick[..., None], 1) + rng.normal(0, 4.0, (B, n, 3))).astype(np.float32)
    t = torch.from_numpy(pts).cuda()
    p0, c0, _ = ndt_preprocessing(k, t)
    first = torch.cat((p0, c0), 2).clone()
    plan = get_plan(B, n, k, -1, t.device)
    st0 = plan.host_stats()
    assert all(s.rc == 0 for s in st0)
    assert any(s.len[0] * s.len[1] * s.len[2] > 32768 for s in st0)  # stamp-mode grids
    rc = _lib.lib().ndnet_ndt_debug_set_epoch(plan.handle, ctypes.c_uint32((1 << 26) - 2))
    assert rc == 0
    for _ in range(3):  # epochs 2^26 - 1, then the wrap to 1 (stale stamps of epoch 1 exist), then 2
        p, c, _ = ndt_preprocessing(k, t)
        assert torch.equal(torch.cat((p, c), 2), first)
        st = plan.host_stats()
        assert [s.iters for s in st] == [s.iters for s in st0]


def test_pipelined_steps_equal_sequential_batches():
    """PipelinedSegmentation: step i's forward output is the log-probs of the
    batch fed at step i - 1, equal to the one-graph-per-step path's."""
    import torch
    from ndnet.models.ndtnet import NDTNetSegmentation
    from ndnet.pipeline import GraphedSegmentation, PipelinedSegmentation
    from ndnet.synthetic import make_batch
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    m = NDTNetSegmentation(3, 28, 768).to(dev).eval()
    batches = [torch.from_numpy(make_batch("L", 4, 20_000, seed0=10 * i)).to(dev) for i in range(3)]
    ref = GraphedSegmentation(m, 400, 4, 20_000, device=dev)
    expect = [ref(b).clone() for b in batches]
    pipe = PipelinedSegmentation(m, 400, 4, 20_000, device=dev)
    outs = []
    for b in batches + [batches[-1]]:
        pipe.points.copy_(b)
        outs.append(pipe.replay().clone())
    torch.cuda.synchronize()
    for i in range(3):
        assert torch.equal(outs[i + 1], expect[i]), f"batch {i}"


@pytest.mark.parametrize("fwd_streams,ndt_streams", [(1, 1), (2, 1), (3, 2)])
def test_pipelined_free_running_steps_equal_sequential_batches(fwd_streams, ndt_streams):
    """replay_steps: the stage streams ordered by events only (the NDT stream
    up to a step ahead, no per-step join; with several forward streams
    consecutive forwards overlap in separate workspace slots, with 2 NDT
    streams consecutive NDT stages on separate plans) give every step the forward
    of the batch before it, bit-equal to the one-graph-per-step path;
    single-step replays before it keep the ring position."""
    import torch
    from ndnet.models.ndtnet import NDTNetSegmentation
    from ndnet.pipeline import GraphedSegmentation, PipelinedSegmentation
    from ndnet.synthetic import make_batch
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    m = NDTNetSegmentation(3, 28, 768).to(dev).eval()
    pipe = PipelinedSegmentation(m, 400, 4, 20_000, device=dev, fwd_streams=fwd_streams, ndt_streams=ndt_streams)
    R = pipe.R
    assert R >= fwd_streams + ndt_streams + 1 and R % fwd_streams == 0 and R % ndt_streams == 0
    batches = [torch.from_numpy(make_batch("L", 4, 20_000, seed0=10 * i + 1)).to(dev) for i in range(R)]
    ref = GraphedSegmentation(m, 400, 4, 20_000, device=dev)
    expect = [ref(b).clone() for b in batches]
    for j, b in enumerate(batches):  # step s reads input s % R
        pipe.inputs[j].copy_(b)
    for _ in range(R):
        pipe.replay()                        # steps 0 .. R - 1
    for rnd in range(2):
        last = pipe.replay_steps(R + R * rnd)  # then R, then 2 R steps
        torch.cuda.synchronize()
        for j in range(R):  # slot j's last step s = j mod R: the forward of batch (s - 1) % R
            assert torch.equal(pipe.out[j], expect[(j - 1) % R]), f"round {rnd} slot {j}"
        assert last.data_ptr() == pipe.out[R - 1].data_ptr()
    out = pipe.replay()                      # slot 0
    torch.cuda.synchronize()
    assert torch.equal(out, expect[R - 1])


def test_two_ndt_streams_keep_k_front_resident():
    """Two NDT streams run two k_front launches at once; asked for CU share 1
    (each launch would span the chip, their workgroups waiting on each other at
    the cloud barriers) the pipeline takes share 2 instead, and every step's
    clouds complete (no barrier timeout) with the one-graph-per-step path's
    output, at the full C2 shape."""
    import torch
    from ndnet.models.ndtnet import NDTNetSegmentation
    from ndnet.pipeline import GraphedSegmentation, PipelinedSegmentation
    from ndnet.synthetic import make_batch
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    m = NDTNetSegmentation(3, 28, 768).to(dev).eval()
    pipe = PipelinedSegmentation(m, 1000, 16, 100_000, device=dev, cu_share=1, ndt_streams=2)
    assert pipe.front_share == [2, 2]
    R = pipe.R
    batches = [torch.from_numpy(make_batch("L" if j % 2 else "U", 16, 100_000, seed0=100 * j)).to(dev)
               for j in range(R)]
    ref = GraphedSegmentation(m, 1000, 16, 100_000, device=dev)
    expect = [ref(b).clone() for b in batches]
    for j, b in enumerate(batches):
        pipe.inputs[j].copy_(b)
    for _ in range(R):
        pipe.replay()
    pipe.replay_steps(2 * R)
    torch.cuda.synchronize()
    for plan in pipe.plans:
        assert all(st.rc == 0 for st in plan.host_stats())
    for j in range(R):
        assert torch.equal(pipe.out[j], expect[(j - 1) % R]), f"slot {j}"


def test_pipelined_levels_equal_graphed_levels():
    """C5-shaped pipeline (downsample + two prune levels, a forward per level):
    every step's per-level outputs, single-step and free-running, bit-equal the
    one-graph multiscale path on the batch before it."""
    import torch
    from ndnet.models.ndtnet import NDTNetSegmentation
    from ndnet.pipeline import GraphedSegmentation, PipelinedSegmentation
    from ndnet.synthetic import make_batch
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    m = NDTNetSegmentation(3, 28, 768).to(dev).eval()
    levels = (400, 200, 100)
    pipe = PipelinedSegmentation(m, levels[0], 4, 20_000, device=dev, levels=levels)
    R = pipe.R
    batches = [torch.from_numpy(make_batch("L", 4, 20_000, seed0=7 * i + 2)).to(dev) for i in range(R)]
    ref = GraphedSegmentation(m, levels[0], 4, 20_000, device=dev, levels=levels)
    expect = [[o.clone() for o in ref(b)] for b in batches]
    for j, b in enumerate(batches):
        pipe.inputs[j].copy_(b)
    outs = [[o.clone() for o in pipe.replay()] for _ in range(R)]   # steps 0 .. R - 1
    pipe.replay_steps(R)                                              # steps R .. 2 R - 1, free-running
    torch.cuda.synchronize()
    for s in range(1, R):
        for lv in range(3):
            assert torch.equal(outs[s][lv], expect[s - 1][lv]), f"step {s} level {lv}"
    for j in range(R):  # step R + j (slot j): batch (j - 1) % R
        for lv in range(3):
            assert torch.equal(pipe.out[j][lv], expect[(j - 1) % R][lv]), f"slot {j} level {lv}"


def test_pipelined_streamed_host_batches():
    """replay_streamed: host batches copied on a copy stream one step ahead
    (double-buffered inputs) give the same outputs as the one-graph path."""
    import torch
    from ndnet.models.ndtnet import NDTNetSegmentation
    from ndnet.pipeline import GraphedSegmentation, PipelinedSegmentation
    from ndnet.synthetic import make_batch
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    m = NDTNetSegmentation(3, 28, 768).to(dev).eval()
    host = [torch.from_numpy(make_batch("L", 4, 20_000, seed0=10 * i)).pin_memory() for i in range(4)]
    ref = GraphedSegmentation(m, 400, 4, 20_000, device=dev)
    expect = [ref(b.to(dev)).clone() for b in host]
    pipe = PipelinedSegmentation(m, 400, 4, 20_000, device=dev)
    pipe.points.copy_(host[0])
    outs = []
    # replay i runs batch i and streams batch i + 1; its forward is batch i - 1's
    for i in range(len(host)):
        outs.append(pipe.replay_streamed(host[min(i + 1, len(host) - 1)]).clone())
    outs.append(pipe.replay().clone())
    torch.cuda.synchronize()
    for i in range(len(host)):
        assert torch.equal(outs[i + 1], expect[i]), f"batch {i}"


def test_graph_keeps_captured_fold_alive():
    """a captured graph reads the model's folded weights and
    workspace through raw pointers.  A redundant eval() or an eager forward
    after capture must not free them.  ADVICE r4: the replays follow an
    in-place weight change (re-folded before the replay: equal to the eager
    forward with the new weights); a replaced parameter is refused."""
    import torch
    from ndnet.synthetic import make_batch
    from ndnet.pipeline import GraphedSegmentation
    B, n, k = 2, 8000, 200
    m = _model()
    pts = torch.from_numpy(make_batch("U", B, n, seed0=3)).cuda()
    g = GraphedSegmentation(m, k, B, n)
    first = g(pts).clone()
    m.eval()                       # redundant: keeps the fold
    m.train()                      # marks the fold stale
    m.eval()
    with torch.no_grad():
        from ndnet.preprocessing.ndtnet_preprocessing import ndt_preprocessing
        p, c, _ = ndt_preprocessing(k, pts)
        eager = m(p, c).clone()   # re-folds in place: the same values into the graph's buffers
        junk = [torch.randn(1 << 20, device="cuda") for _ in range(8)]  # reuse freed blocks, if any
    again = g(pts).clone()
    torch.cuda.synchronize()
    del junk
    assert torch.equal(again, first) and torch.equal(eager, first)
    with torch.no_grad():
        m.conv4.bias.add_(1.0)
    followed = g(pts).clone()        # no eager forward in between: the replay re-folds itself
    with torch.no_grad():
        eager2 = m(p, c).clone()
    torch.cuda.synchronize()
    assert torch.equal(followed, eager2) and not torch.equal(followed, first)
    m.conv4.bias = torch.nn.Parameter(m.conv4.bias.detach().clone())  # a new tensor: no in-place fold
    with pytest.raises(RuntimeError, match="build a new graph"):
        g(pts)


def test_eval_mode_autograd_uses_differentiable_path():
    """the reference forward is differentiable in eval mode; with
    grad enabled the model must not return a grad-less kernel output."""
    import torch
    m = _model()
    p = torch.rand((2, 64, 3), device="cuda")
    c = torch.randn((2, 64, 9), device="cuda", requires_grad=True)
    out = m(p, c)
    assert out.grad_fn is not None
    out.sum().backward()
    assert c.grad is not None and torch.isfinite(c.grad).all()
    assert m.conv4.weight.grad is not None
    with torch.no_grad():
        hip = m(p, c)
    assert hip.grad_fn is None and (hip - out.detach()).abs().max().item() < 1e-4


def test_legacy_entry_points_run_concurrently():
    """the reference ABI is called from several DataLoader workers
    at once; its plans use the multi-launch path (no grid barrier), so
    concurrent callers all succeed."""
    import threading
    import oracle as O
    from ndnet.preprocessing.ndt_legacy import NDT_Sampler
    from ndnet.synthetic import lidar_cloud, uniform_cloud
    clouds = [uniform_cloud(40_000, s).astype(np.float64) for s in range(2)] + \
             [lidar_cloud(40_000, s).astype(np.float64) for s in range(2)]
    res = [None] * len(clouds)

    def work(i):
        s = NDT_Sampler(clouds[i])
        res[i] = s.downsample(500)
        s.cleanup()

    th = [threading.Thread(target=work, args=(i,)) for i in range(len(clouds))]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=60)
    for i, cl in enumerate(clouds):
        assert res[i] is not None, f"worker {i} did not finish"
        ref = O.LegacyChain(cl)
        pc, cov = ref.downsample(500)
        assert np.array_equal(res[i][0], pc) and np.array_equal(res[i][1], cov, equal_nan=True)
        ref.cleanup()


def test_two_stream_forward_capture_matches_eager():
    """two forwards captured on two streams of one graph
    (the two halves of a batch, forked from and joined back into the capture
    stream), each in its own workspace slot, replay to exactly the eager
    forwards of the halves.  Concurrent forwards in ONE slot share the
    max-pool buffer, FC-head intermediates and folded weights (the round-2
    crash): pointnet_hip.workspace_slot keeps them apart."""
    import torch
    from ndnet.models import pointnet_hip
    from ndnet.preprocessing.ndtnet_preprocessing import ndt_preprocessing
    from ndnet.synthetic import make_batch
    dev = torch.device("cuda", 0)
    torch.manual_seed(1)
    m = _model(F=768, C=28, seed=5)
    B, n, k = 8, 20_000, 400
    with torch.no_grad():
        p, c, _ = ndt_preprocessing(k, torch.from_numpy(make_batch("L", B, n, seed0=3)).to(dev))
        rows = torch.cat((p, c), 2).contiguous()
        halves = [rows[: B // 2].contiguous(), rows[B // 2:].contiguous()]
        eager = [m(h[..., :3], h[..., 3:]).clone() for h in halves]
    streams = [torch.cuda.Stream(device=dev), torch.cuda.Stream(device=dev)]

    def step():
        cur = torch.cuda.current_stream(dev)
        outs = []
        for i, (h, s) in enumerate(zip(halves, streams)):
            s.wait_stream(cur)
            with torch.cuda.stream(s), pointnet_hip.workspace_slot(i):
                outs.append(m(h[..., :3], h[..., 3:]))
        for s in streams:
            cur.wait_stream(s)
        return outs

    side = torch.cuda.Stream(device=dev)
    side.wait_stream(torch.cuda.current_stream(dev))
    with torch.no_grad(), torch.cuda.stream(side):
        for _ in range(2):  # warm-up: both slots' workspaces exist before capture
            step()
    torch.cuda.current_stream(dev).wait_stream(side)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.no_grad(), torch.cuda.graph(g):
        outs = step()
    for _ in range(3):
        g.replay()
        torch.cuda.synchronize()
        for o, e in zip(outs, eager):
            assert torch.equal(o, e)


def test_two_unrolled_pipelined_steps_in_one_graph():
    """Round-3 DESIGN recorded a host segfault in hipStreamEndCapture for one
    graph holding several unrolled pipelined steps.  Round 4 re-ran that
    capture (tools/capture_probe.py, profiles/r04_capture_probe.txt): the
    pipeline's own pattern -- NDT and forward streams forked from the capture
    stream by events, every cross-stream order an event recorded inside the
    capture, every side stream joined back before the capture ends -- captures
    and replays correctly; an unjoined stream fails cleanly
    (hipErrorStreamCaptureUnjoined) and replaying a graph inside a capture is
    refused by torch, neither crashes.  Two unrolled steps in one graph,
    replayed, equal the eager steps."""
    import torch
    from ndnet.pipeline import PipelinedSegmentation
    from ndnet.synthetic import make_batch
    dev = torch.device("cuda", 0)
    B, n, k = 4, 20000, 200
    m = _model(F=768, C=28)
    pipe = PipelinedSegmentation(m, k, B, n, device=dev)
    for j in range(pipe.R):
        pipe.inputs[j].copy_(torch.from_numpy(make_batch("U" if j % 2 else "L", B, n, seed0=10 * j)).to(dev))
    F = pipe.F
    with torch.no_grad():
        for j in (0, 1, 2):
            pipe._ndt(j)
        ref = [pipe._fwd(j).clone() for j in (1, 2)]
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    cap = torch.cuda.Stream(device=dev)
    cap.wait_stream(torch.cuda.current_stream(dev))
    ev = [torch.cuda.Event() for _ in range(8)]
    outs = []
    s_ndt = pipe.s_ndts[0]
    with torch.no_grad(), torch.cuda.graph(g, stream=cap):
        ev[0].record(cap)
        s_ndt.wait_event(ev[0])
        for s in pipe.s_fwds:
            s.wait_event(ev[0])
        for i, j in enumerate((1, 2)):
            with torch.cuda.stream(s_ndt):
                pipe._ndt(j)
            ev[1 + i].record(s_ndt)
            s_f = pipe.s_fwds[j % F]
            s_f.wait_event(ev[1 + i])
            with torch.cuda.stream(s_f):
                outs.append(pipe._fwd(j))
            ev[4 + i].record(s_f)
        for i in range(2):
            cap.wait_event(ev[4 + i])
        ev[7].record(s_ndt)
        cap.wait_event(ev[7])
        for s in pipe.s_fwds:  # streams without work in this capture join too
            e = torch.cuda.Event()
            e.record(s)
            cap.wait_event(e)
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    for a, b in zip(outs, ref):
        assert torch.equal(a, b)
